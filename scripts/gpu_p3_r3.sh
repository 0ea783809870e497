# Paired bf16x3 chunks (CONV_X3_PAIRED): bf16 bitwise against the previous build (scripts/micro/alt/zs.so)
# -- only bf16x3 may change --, the GPU test suite, then bench A/B pairs for bf16x3 and bf16.
# Usage: bash scripts/gpu_p3_r3.sh TAG
set -o pipefail
TAG=${1:-p3}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
( export PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/zs.so; timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/prev.npz ) > $OUT/bitwise.txt 2>&1 || { echo "dump prev failed"; exit 1; }
timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/new.npz >> $OUT/bitwise.txt 2>&1 || { echo "dump new failed"; exit 1; }
python scripts/lib_bitwise.py compare $OUT/prev.npz $OUT/new.npz >> $OUT/bitwise.txt 2>&1
tail -4 $OUT/bitwise.txt
rm -f $OUT/*.npz
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16x3.py tests/test_gpu_golden.py -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > $OUT/pytest_x3.log 2>&1
rc=$?
echo "pytest exit $rc" >> $OUT/pytest_x3.log
tail -3 $OUT/pytest_x3.log
if [ $rc -ne 0 ]; then echo "bf16x3 tests failed ($rc)"; exit $rc; fi
ALT=zs.so REPS=3 ARGS="--steps 2 --dtype bf16x3" bash scripts/ab_bench.sh $TAG/ab_x3 || exit 1
timeout -k 10 700 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  > $OUT/pytest.log 2>&1
rc=$?
echo "pytest exit $rc" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --dtype bf16x3 --no-cpu-baseline --no-extras > $OUT/bench_prof.log 2>&1 || exit 1
echo EXIT 0
