# BASELINE configs[3] per-rank shard on one GPU (32 TACs x 8192 samples, chunks of 65536 per launch),
# plus the default config at 8192 samples per launch.  Usage: bash scripts/gpu_cfg4.sh TAG
set -o pipefail
TAG=${1:-cfg4}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python bench.py --batch 8192 --tacs 1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/b8192.json 2> gpurun_out/$TAG/b8192.err || exit $?
timeout -k 10 600 python bench.py --config4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/cfg4.json 2> gpurun_out/$TAG/cfg4.err || exit $?
echo EXIT 0
