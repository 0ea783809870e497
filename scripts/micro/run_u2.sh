# The final level alone (bf16 u2, bf16x3 u2x) in conv_micro builds shipped in scripts/micro/ship/: product
# (m0) and stamp (m128) modes of the working tree and of a _base variant, alternating, REPS times.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-u2}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT/scripts/micro/ship
for r in $(seq 1 ${REPS:-2}); do
  for b in ${BINS:-m0 m0_base m128 m128_base}; do
    for sel in u2 u2x; do
      echo "== $b $sel r$r" >> $OUT/micro.txt
      timeout -k 10 60 ./conv_micro_$b 1024 $sel >> $OUT/micro.txt 2>&1 || { echo "micro $b $sel failed"; exit 1; }
    done
  done
done
grep -E "==|us:|epilogue us|loop cycles|mode" $OUT/micro.txt
echo EXIT 0
