# MH GPU round-trip: MH parity tests + a short MH bench probe.  Usage: bash scripts/gpu_mh.sh TAG
set -o pipefail
TAG=${1:-mh}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
make -C oracle > gpurun_out/$TAG/make.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests/test_gpu_mh.py -q -p no:cacheprovider > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/$TAG/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest died ($rc)"; exit $rc; fi
timeout -k 10 300 python bench.py --workload mh ${MH_ARGS:---mh-chains 10000 --mh-iters 100} > gpurun_out/$TAG/bench_mh.json 2> gpurun_out/$TAG/bench_mh.err
echo EXIT $?
