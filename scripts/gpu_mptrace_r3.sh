# round 3: kernel traces of (a) two processes sharing the GPU (gloo ranks, B = 1024 each) and (b) one process
# with two streams (PETDIFF_SPLIT=2), to see whether kernels of the two loops overlap in time.
# torch.distributed.run starts rocprofv3 as each rank's program (--no-python), so the launcher itself never
# touches the GPU.  Usage: bash scripts/gpu_mptrace_r3.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-mptrace}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
B="--steps 2 --warmup 1 --reverse-steps 200 --no-cpu-baseline --no-kernel-timing --no-extras"
PETDIFF_BENCH_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 --no-python \
  rocprofv3 --kernel-trace -d $OUT/two_%pid% -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --gpus 2 $B \
  > $OUT/two.log 2>&1 || exit 1
PETDIFF_SPLIT=2 timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/split -o run --output-format csv -- \
  python $GRAFT_REPO_ROOT/bench.py $B > $OUT/split.log 2>&1 || exit 1
echo EXIT 0
