# round 3: final-epilogue changes (final kernel loaded at kernel start; maps + ReLU formed while the C tile
# is staged).  Bitwise against the previous build (scripts/micro/alt/wf0.so), micro stamps of the final
# level, alternating bench A/B per dtype, parity tests.  Usage: bash scripts/gpu_fin_r3.sh TAG
set -o pipefail
TAG=${1:-fin}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
OLD=$GRAFT_REPO_ROOT/scripts/micro/alt/wf0.so
PETDIFF_LIB=$OLD timeout -k 10 200 python scripts/lib_bitwise.py dump $OUT/old.npz > $OUT/bitwise.log 2>&1 || exit 1
timeout -k 10 200 python scripts/lib_bitwise.py dump $OUT/new.npz >> $OUT/bitwise.log 2>&1 || exit 1
python scripts/lib_bitwise.py compare $OUT/old.npz $OUT/new.npz >> $OUT/bitwise.log 2>&1
grep -E "BITWISE|differ" $OUT/bitwise.log | head -3
( cd scripts/micro && for r in 1 2; do for b in fb_m0 fb_m0ms0 fb_m128 fb_ms0; do echo "== $b" >> ../../$OUT/micro.txt; \
  timeout -k 10 60 ./$b 1024 u2 nod1 >> ../../$OUT/micro.txt 2>&1 || exit 1; done; done ) || exit 1
grep -E "==|us:|up2" $OUT/micro.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_parity16.py -q -x \
  --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_envab_r3.sh ${TAG}_ab "PETDIFF_LIB=$OLD" || exit 1
BENCH_EXTRA="--dtype bf16x3" bash scripts/gpu_envab_r3.sh ${TAG}_ab3 "PETDIFF_LIB=$OLD" || exit 1
echo EXIT 0
