# round 3: fused down1 with the LDS-staged 16-B output stores -- bitwise tests, in-process A/B per dtype,
# micro phase stamps.  Usage: bash scripts/gpu_fd1b_r3.sh TAG
set -o pipefail
TAG=${1:-fd1b}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider \
  -k "down1 or down0 or tac_major or chunked" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest exit $rc" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then echo "pytest failed ($rc)"; exit $rc; fi
timeout -k 10 300 python scripts/ab_fd1.py $OUT/ab.jsonl bfloat16 bf16x3 float16 || exit 1
cd scripts/micro
for b in fb_m128 fb_m128r; do
  for d in nod1 d1; do
    echo "== $b $d" >> ../../$OUT/times.txt
    timeout -k 10 60 ./$b 1024 u2 $d >> ../../$OUT/times.txt 2>&1 || exit $?
  done
done
cat ../../$OUT/times.txt | grep -E "==|final epilogue|up2.fused"
echo EXIT 0
