# round 3: sharded-path tests + re-pointed parity tests, then the per-job host overhead probe with and
# without graph segments.  Usage: bash scripts/gpu_r3b.sh TAG
set -o pipefail
TAG=${1:-r3b}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/$TAG/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest died ($rc)"; exit $rc; fi
for S in 0 100 50 0 100 25; do
  PETDIFF_GRAPH_SEG=$S timeout -k 10 200 python scripts/probe/job_overhead.py > gpurun_out/$TAG/probe_seg$S.json 2>&1 || exit 1
  echo "seg $S $(cat gpurun_out/$TAG/probe_seg$S.json)"
done
echo EXIT 0
