# GPU round-trip: parity tests, bench, rocprofv3 kernel stats.  Usage: bash scripts/gpu_test_bench.sh TAG
set -o pipefail
TAG=${1:-run}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
if [ -n "$MICRO" ]; then MODES="$MICRO" TAG=$TAG bash scripts/micro/run.sh > /dev/null || exit $?; fi
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/$TAG/pytest.log
# 1 = ordinary test failures; anything else (abort, segfault, timeout) ends the call here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest died ($rc)"; exit $rc; fi
[ -n "$NO_BENCH" ] && { echo EXIT 0; exit 0; }
timeout -k 10 400 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline --no-extras > gpurun_out/$TAG/bench_prof.log 2>&1
echo EXIT $?
