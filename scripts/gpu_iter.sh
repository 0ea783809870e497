# One build->measure iteration on the GPU box: fused-layer micro breakdown, the GPU parity tests, the bench.
# Usage: bash scripts/gpu_iter.sh TAG   (PYTEST_FILES / NO_MICRO / NO_BENCH to trim)
set -o pipefail
TAG=${1:-iter}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
if [ -z "$NO_MICRO" ]; then bash scripts/micro/fused_breakdown.sh run $TAG > /dev/null || exit $?; fi
timeout -k 10 400 python -u -m pytest ${PYTEST_FILES:-tests/test_gpu_parity.py tests/test_gpu_parity16.py} -x -q -m gpu \
  -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/$TAG/pytest.log
[ $rc -ne 0 ] && { tail -30 gpurun_out/$TAG/pytest.log; exit $rc; }
[ -n "$NO_BENCH" ] && { echo EXIT 0; exit 0; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
echo EXIT 0
