# Secondary workloads in one GPU call: same-GPU iDDPM vs MCMC comparison, MH bench (config 3),
# fp16 bench (config 5), training bench.  Usage: bash scripts/gpu_secondary.sh TAG
set -o pipefail
TAG=${1:-sec}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python scripts/compare_mcmc.py gpurun_out/$TAG/compare_mcmc.json > gpurun_out/$TAG/compare.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --dtype float16 > gpurun_out/$TAG/bench_f16.json 2> gpurun_out/$TAG/bench_f16.err || exit $?
timeout -k 10 400 python bench.py --workload mh > gpurun_out/$TAG/bench_mh.json 2> gpurun_out/$TAG/bench_mh.err || exit $?
timeout -k 10 300 python bench.py --workload train > gpurun_out/$TAG/bench_train.json 2> gpurun_out/$TAG/bench_train.err || exit $?
echo EXIT 0
