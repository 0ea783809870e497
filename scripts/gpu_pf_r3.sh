# L2 prefetch of the next launch's chunk 0 (CONV_PREFETCH=1, scripts/micro/alt/pf1.so) against the product:
# bitwise, bench A/B (bf16, bf16x3), rocprofv3 of both.  Usage: bash scripts/gpu_pf_r3.sh TAG
set -o pipefail
TAG=${1:-pf}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
( export PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/pf1.so; timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/pf1.npz ) > $OUT/bitwise.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/cur.npz >> $OUT/bitwise.txt 2>&1 || exit 1
python scripts/lib_bitwise.py compare $OUT/cur.npz $OUT/pf1.npz >> $OUT/bitwise.txt 2>&1
tail -1 $OUT/bitwise.txt
rm -f $OUT/*.npz
ALT=pf1.so REPS=3 bash scripts/ab_bench.sh $TAG/ab || exit 1
ALT=pf1.so REPS=2 ARGS="--steps 2 --dtype bf16x3" bash scripts/ab_bench.sh $TAG/ab_x3 || exit 1
ALT=pf1.so ARGS="" bash scripts/gpu_prof2_r3.sh $TAG/prof || exit 1
echo EXIT 0
