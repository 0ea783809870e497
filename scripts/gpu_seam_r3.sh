# round 3: down2 -> down3 in one launch (PETDIFF_SEAM23) -- bitwise against the separate launches and the
# previous build, in-process A/B per dtype, rocprofv3 kernel stats of both.  Usage: bash scripts/gpu_seam_r3.sh TAG
set -o pipefail
TAG=${1:-seam}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider -k "seam23" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/head.so timeout -k 10 200 python scripts/lib_bitwise.py dump $OUT/head.npz > $OUT/bitwise.log 2>&1 || exit 1
timeout -k 10 200 python scripts/lib_bitwise.py dump $OUT/new.npz >> $OUT/bitwise.log 2>&1 || exit 1
PETDIFF_SEAM23=1 timeout -k 10 200 python scripts/lib_bitwise.py dump $OUT/seam.npz >> $OUT/bitwise.log 2>&1 || exit 1
python scripts/lib_bitwise.py compare $OUT/head.npz $OUT/new.npz >> $OUT/bitwise.log 2>&1
python scripts/lib_bitwise.py compare $OUT/new.npz $OUT/seam.npz >> $OUT/bitwise.log 2>&1
grep -E "BITWISE|differ|max" $OUT/bitwise.log | head
AB_VAR=PETDIFF_SEAM23 timeout -k 10 300 python scripts/ab_fd1.py $OUT/ab.jsonl bfloat16 bf16x3 || exit 1
PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/head.so AB_VAR=PETDIFF_SEAM23 timeout -k 10 300 python scripts/ab_fd1.py $OUT/ab_head.jsonl bfloat16 || exit 1
for S in 0 1; do
  PETDIFF_SEAM23=$S timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof$S -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline --no-extras > $OUT/prof$S.log 2>&1 || exit 1
done
echo EXIT 0
