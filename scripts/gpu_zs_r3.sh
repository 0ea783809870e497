# up0 zero-skip (CONV_UP0_ZS) validation: bitwise against the previous build (scripts/micro/alt/head.so),
# the GPU test suite, then bench A/B pairs for bf16 and bf16x3.  Usage: bash scripts/gpu_zs_r3.sh TAG
set -o pipefail
TAG=${1:-zs}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
( export PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/head.so; timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/head.npz ) > $OUT/bitwise.txt 2>&1 || { echo "dump head failed"; exit 1; }
timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/zs.npz >> $OUT/bitwise.txt 2>&1 || { echo "dump zs failed"; exit 1; }
python scripts/lib_bitwise.py compare $OUT/head.npz $OUT/zs.npz >> $OUT/bitwise.txt 2>&1
tail -3 $OUT/bitwise.txt
rm -f $OUT/*.npz
timeout -k 10 700 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  > $OUT/pytest.log 2>&1
rc=$?
echo "pytest exit $rc" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest died ($rc)"; exit $rc; fi
ALT=head.so REPS=3 bash scripts/ab_bench.sh $TAG/ab_bf16 || exit 1
ALT=head.so REPS=2 ARGS="--steps 2 --dtype bf16x3" bash scripts/ab_bench.sh $TAG/ab_x3 || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline --no-extras > $OUT/bench_prof.log 2>&1 || exit 1
echo EXIT 0
