# Tests + iDDPM bench + rocprof stats + a short MH bench.  Usage: bash scripts/gpu_all.sh TAG
set -o pipefail
TAG=${1:-all}
cd $GRAFT_REPO_ROOT
make -C oracle > /dev/null 2>&1 || exit 1
bash scripts/gpu_test_bench.sh $TAG || exit $?
timeout -k 10 300 python bench.py --workload mh ${MH_ARGS:---mh-chains 10000 --mh-iters 200 --mh-tune 100 --no-cpu-baseline} > gpurun_out/$TAG/bench_mh.json 2> gpurun_out/$TAG/bench_mh.err
echo EXIT $?
