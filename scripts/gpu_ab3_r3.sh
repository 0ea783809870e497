# A/B of the current build against scripts/micro/alt/{xcd3,prev}.so in one call: the per-XCD tile block
# (CONV_XCD_MAP=3) and the session-start build (8526eb3), bf16 and bf16x3.  Usage: bash scripts/gpu_ab3_r3.sh TAG
set -o pipefail
TAG=${1:-ab3}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
ALT=xcd3.so REPS=3 bash scripts/ab_bench.sh $TAG/xcd3 || exit 1
ALT=prev.so REPS=3 bash scripts/ab_bench.sh $TAG/prev_bf16 || exit 1
ALT=prev.so REPS=2 ARGS="--steps 2 --dtype bf16x3" bash scripts/ab_bench.sh $TAG/prev_x3 || exit 1
echo EXIT 0
