# Training-step GPU round: tests, bench (--workload train), rocprofv3 kernel stats.
set -o pipefail
TAG=${1:-train}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests/test_gpu_train.py -q -p no:cacheprovider > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/$TAG/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest died ($rc)"; exit $rc; fi
timeout -k 10 400 python bench.py --workload train --steps ${STEPS:-20} --warmup 3 > gpurun_out/$TAG/bench_train.json 2> gpurun_out/$TAG/bench_train.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --workload train --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/prof.log 2>&1
echo EXIT $?
