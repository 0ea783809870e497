# Rehearse bench.py's N>1 code path on a 1-GPU box: 2 ranks share the GPU, collectives over gloo
# (RCCL refuses two ranks on one device).  Usage: bash scripts/gpu_dist2.sh TAG
set -o pipefail
TAG=${1:-dist2}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
export PETDIFF_BENCH_BACKEND=gloo
RUN="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 300 $RUN --master-port 29511 bench.py --gpus 2 --steps 1 --warmup 1 > gpurun_out/$TAG/iddpm.json 2> gpurun_out/$TAG/iddpm.err || exit $?
timeout -k 10 300 $RUN --master-port 29512 bench.py --gpus 2 --workload mh --mh-chains 1024 --mh-iters 200 --mh-tune 200 > gpurun_out/$TAG/mh.json 2> gpurun_out/$TAG/mh.err || exit $?
timeout -k 10 300 $RUN --master-port 29513 bench.py --gpus 2 --workload train --steps 2 > gpurun_out/$TAG/train.json 2> gpurun_out/$TAG/train.err || exit $?
echo EXIT 0
