# up0 zero-skip with cached A fragments (CONV_UP0_ZS_CACHE=1, scripts/micro/alt/zc1.so) against the product:
# bitwise, up0 stamps in isolation, bench A/B (bf16, bf16x3).  Usage: bash scripts/gpu_zc_r3.sh TAG
set -o pipefail
TAG=${1:-zc}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
( export PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/zc1.so; timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/zc1.npz ) > $OUT/bitwise.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/cur.npz >> $OUT/bitwise.txt 2>&1 || exit 1
python scripts/lib_bitwise.py compare $OUT/cur.npz $OUT/zc1.npz >> $OUT/bitwise.txt 2>&1
tail -1 $OUT/bitwise.txt
rm -f $OUT/*.npz
for b in fb_zs128 fb_zc128 fb_zs128 fb_zc128; do
  echo "== $b" >> $OUT/micro.txt
  timeout -k 10 60 scripts/micro/$b 1024 u0 >> $OUT/micro.txt 2>&1 || exit $?
done
ALT=zc1.so REPS=3 bash scripts/ab_bench.sh $TAG/ab || exit 1
ALT=zc1.so REPS=2 ARGS="--steps 2 --dtype bf16x3" bash scripts/ab_bench.sh $TAG/ab_x3 || exit 1
echo EXIT 0
