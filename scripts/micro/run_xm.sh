# A/B of two prebuilt conv_micro builds (xm_old_m<mode>, xm_new_m<mode>) on the bf16x3 (x) and bf16 (f) step layers
set -o pipefail
cd $GRAFT_REPO_ROOT/scripts/micro
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-xm}
mkdir -p $OUT
for sel in ${SELS:-x f}; do
  for m in ${MODES:-0 128}; do
    for v in ${VARIANTS:-old new}; do
      echo "== $v mode $m sel $sel" >> $OUT/micro.txt
      timeout -k 10 120 ./xm_${v}_m$m 1024 $sel >> $OUT/micro.txt 2>&1 || { echo "micro $v $m $sel failed"; exit 1; }
    done
  done
done
grep -E "==|mode|loop cycles|null" $OUT/micro.txt
