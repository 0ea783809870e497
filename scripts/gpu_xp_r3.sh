# bf16x3 with down2 / down3 on the three-pass chunks (CONV_X3_PAIRED_PM=0, scripts/micro/alt/xp0.so) against
# the product (paired): bench A/B pairs (bf16x3), rocprofv3 of both.  Usage: bash scripts/gpu_xp_r3.sh TAG
set -o pipefail
TAG=${1:-xp}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
ALT=xp0.so REPS=3 ARGS="--steps 2 --dtype bf16x3" bash scripts/ab_bench.sh $TAG/ab_x3 || exit 1
ALT=xp0.so ARGS="--dtype bf16x3" bash scripts/gpu_prof2_r3.sh $TAG/prof || exit 1
echo EXIT 0
