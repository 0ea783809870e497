# rocprofv3 PMC passes (separate passes per counter group, MI355X_MICROARCH.md HBM/rocprofv3 section).
# Usage: bash scripts/gpu_pmc.sh TAG
set -o pipefail
TAG=${1:-pmc}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
# BENCH_EXTRA: more bench.py flags, e.g. "--dtype bf16x3"
APP="python $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --reverse-steps 20 --no-cpu-baseline --no-kernel-timing ${BENCH_EXTRA}"
i=0
for CTR in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $CTR -d $OUT/p$i -o run --output-format csv -- $APP > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo EXIT 0
