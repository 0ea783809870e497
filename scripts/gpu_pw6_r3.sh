# position-major down layers with 6 fragments per wave (CONV_PM_W6=1, scripts/micro/alt/pw6.so) against the product:
# bitwise, step layers in isolation, bench A/B (bf16, bf16x3).  Usage: bash scripts/gpu_pw6_r3.sh TAG
set -o pipefail
TAG=${1:-zc}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
( export PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/pw6.so; timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/pw6.npz ) > $OUT/bitwise.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/cur.npz >> $OUT/bitwise.txt 2>&1 || exit 1
python scripts/lib_bitwise.py compare $OUT/cur.npz $OUT/pw6.npz >> $OUT/bitwise.txt 2>&1
tail -1 $OUT/bitwise.txt
rm -f $OUT/*.npz
for b in fb_q0 fb_q6 fb_q0 fb_q6; do
  echo "== $b" >> $OUT/micro.txt
  timeout -k 10 60 scripts/micro/$b 1024 f >> $OUT/micro.txt 2>&1 || exit $?
done
ALT=pw6.so REPS=3 bash scripts/ab_bench.sh $TAG/ab || exit 1
ALT=pw6.so REPS=2 ARGS="--steps 2 --dtype bf16x3" bash scripts/ab_bench.sh $TAG/ab_x3 || exit 1
echo EXIT 0
