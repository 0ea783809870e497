# up1 with keyed A-fragment cache (CONV_UP1_CACHE=1, scripts/micro/alt/uc1.so) against the product:
# bitwise, step layers in isolation, bench A/B (bf16, bf16x3).  Usage: bash scripts/gpu_uc_r3.sh TAG
set -o pipefail
TAG=${1:-zc}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
( export PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/uc1.so; timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/uc1.npz ) > $OUT/bitwise.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/cur.npz >> $OUT/bitwise.txt 2>&1 || exit 1
python scripts/lib_bitwise.py compare $OUT/cur.npz $OUT/uc1.npz >> $OUT/bitwise.txt 2>&1
tail -1 $OUT/bitwise.txt
rm -f $OUT/*.npz
for b in fb_u0c fb_u1c fb_u0c fb_u1c; do
  echo "== $b" >> $OUT/micro.txt
  timeout -k 10 60 scripts/micro/$b 1024 f >> $OUT/micro.txt 2>&1 || exit $?
done
ALT=uc1.so REPS=3 bash scripts/ab_bench.sh $TAG/ab || exit 1
ALT=uc1.so REPS=2 ARGS="--steps 2 --dtype bf16x3" bash scripts/ab_bench.sh $TAG/ab_x3 || exit 1
echo EXIT 0
