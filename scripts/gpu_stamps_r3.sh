# Stamped per-layer breakdown of the current step kernels (conv_micro mode 128; 192 = no LDS fragment reads).
set -o pipefail
cd $GRAFT_REPO_ROOT/scripts/micro
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-stamps}
mkdir -p $OUT
for b in fb_m128 fb_m192; do
  echo "== $b" >> $OUT/micro.txt
  timeout -k 10 90 ./$b 1024 f >> $OUT/micro.txt 2>&1 || exit $?
done
echo EXIT 0
