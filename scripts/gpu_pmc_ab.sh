# PMC counters of the product build and of scripts/micro/alt/$ALT side by side (diagnosis of an
# A/B result).  Usage: ALT=<name>.so bash scripts/gpu_pmc_ab.sh TAG
set -o pipefail
TAG=${1:-pmcab}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT/a $OUT/b
APP="python $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --reverse-steps 20 --no-cpu-baseline --no-kernel-timing"
for v in a b; do
  i=0
  for CTR in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM" "SQC_ICACHE_MISSES SQC_ICACHE_HITS"; do
    i=$((i+1))
    if [ $v = b ]; then export PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/$ALT; fi
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CTR -d $OUT/$v/p$i -o run --output-format csv -- $APP > $OUT/$v/p$i.log 2>&1 || echo "pass $v$i failed ($?)"
  done
done
python scripts/pmc_summary.py $OUT/a $OUT/a/pmc.json > $OUT/a/summary.txt 2>&1
python scripts/pmc_summary.py $OUT/b $OUT/b/pmc.json > $OUT/b/summary.txt 2>&1
echo EXIT 0
