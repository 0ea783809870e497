# final-level map rows issued mid-loop (scripts/micro/alt/fm.so)
# against the product: bitwise, bench A/B (bf16, bf16x3).  Usage: bash scripts/gpu_fm_r3.sh TAG
set -o pipefail
TAG=${1:-fm}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
( export PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/fm.so; timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/fm.npz ) > $OUT/bitwise.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/cur.npz >> $OUT/bitwise.txt 2>&1 || exit 1
python scripts/lib_bitwise.py compare $OUT/cur.npz $OUT/fm.npz >> $OUT/bitwise.txt 2>&1
tail -1 $OUT/bitwise.txt
rm -f $OUT/*.npz
ALT=fm.so REPS=4 bash scripts/ab_bench.sh $TAG/ab || exit 1
ALT=fm.so REPS=2 ARGS="--steps 2 --dtype bf16x3" bash scripts/ab_bench.sh $TAG/ab_x3 || exit 1
echo EXIT 0
