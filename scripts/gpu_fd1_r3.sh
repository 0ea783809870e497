# round 3: fused next-step down1 for fp16 / bf16x3 / multi-condition tiles, LDS-DMA B ring (FD1_LDS) --
# bitwise tests, in-process A/B (fused vs standalone down1) per dtype for the in-tree library and the
# register-ring build, and an 8-TAC batch.  Usage: bash scripts/gpu_fd1_r3.sh TAG
set -o pipefail
TAG=${1:-fd1}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16x3.py -q -m gpu -p no:cacheprovider \
  -k "down1 or down0 or bf16x3 or tac_major or chunked" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest exit $rc" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest died ($rc)"; exit $rc; fi
timeout -k 10 300 python scripts/ab_fd1.py $OUT/ab.jsonl bfloat16 bf16x3 float16 || exit 1
PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/fd1reg.so timeout -k 10 300 python scripts/ab_fd1.py $OUT/ab.jsonl bfloat16 bf16x3 || exit 1
for F in 0 1; do
  PETDIFF_FUSE_DOWN1=$F timeout -k 10 300 python bench.py --batch 65536 --tacs 8 --steps 2 --warmup 1 --no-cpu-baseline \
    --no-extras --no-kernel-timing > $OUT/bench_tac8_f$F.json 2> $OUT/bench_tac8_f$F.err || exit 1
  python -c "import json;d=json.load(open('$OUT/bench_tac8_f$F.json'));print('8 TACs x 8192','fuse_d1=$F',d['value'])"
done
echo EXIT 0
