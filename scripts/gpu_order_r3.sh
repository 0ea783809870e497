# MFMA issue order (CONV_MFMA_ORDER=1, B-major) against the product (A-major): conv_micro per layer, bitwise
# of the product library, bench A/B.  Usage: bash scripts/gpu_order_r3.sh TAG
set -o pipefail
TAG=${1:-order}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
for b in fb_o0 fb_o1 fb_o0 fb_o1; do
  echo "== $b" >> $OUT/micro.txt
  timeout -k 10 60 scripts/micro/$b 1024 f >> $OUT/micro.txt 2>&1 || exit $?
done
( export PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/o1.so; timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/o1.npz ) > $OUT/bitwise.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/o0.npz >> $OUT/bitwise.txt 2>&1 || exit 1
python scripts/lib_bitwise.py compare $OUT/o0.npz $OUT/o1.npz >> $OUT/bitwise.txt 2>&1
tail -1 $OUT/bitwise.txt
rm -f $OUT/*.npz
ALT=o1.so REPS=3 bash scripts/ab_bench.sh $TAG/ab || exit 1
echo EXIT 0
