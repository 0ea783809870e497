# bf16 vs fp16 network: per-kernel busy cycles (GRBM_GUI_ACTIVE, SQ_BUSY_CYCLES) next to the
# kernel durations, to separate instruction count from clock.  Usage: bash scripts/gpu_clock_ab.sh TAG
set -o pipefail
TAG=${1:-clk}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for DT in bfloat16 float16; do
  APP="python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --reverse-steps 300 --dtype $DT --no-cpu-baseline --no-kernel-timing"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES -d $OUT/$DT -o run --output-format csv -- $APP > $OUT/$DT.log 2>&1 || { echo "pass $DT failed"; exit 1; }
done
echo EXIT 0
