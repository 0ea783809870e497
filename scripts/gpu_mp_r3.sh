# round 3: do two processes on one GPU overlap their graph loops where two streams of one process do not?
# Same box, alternating: one process (B = 1024), two processes sharing the GPU (gloo ranks, B = 512 each and
# B = 1024 each), one process with PETDIFF_SPLIT=2 (two streams).  Usage: bash scripts/gpu_mp_r3.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-mp}
OUT=gpurun_out/$TAG
mkdir -p $OUT
B="--steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-kernel-timing --no-extras"
RUN="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
for i in ${TRIALS:-1 2}; do
  timeout -k 10 120 python bench.py $B > $OUT/one_$i.json 2> $OUT/one_$i.err || exit 1
  PETDIFF_BENCH_BACKEND=gloo timeout -k 10 180 $RUN --master-port 2952$i bench.py --gpus 2 --batch 512 $B > $OUT/two512_$i.json 2> $OUT/two512_$i.err || exit 1
  PETDIFF_BENCH_BACKEND=gloo timeout -k 10 180 $RUN --master-port 2953$i bench.py --gpus 2 $B > $OUT/two1024_$i.json 2> $OUT/two1024_$i.err || exit 1
  PETDIFF_SPLIT=2 timeout -k 10 120 python bench.py $B > $OUT/split_$i.json 2> $OUT/split_$i.err || exit 1
  python - <<EOF
import json
def v(f):
    l = [x for x in open('$OUT/' + f).read().splitlines() if x.startswith('{')][-1]
    return json.loads(l)['value']
print($i, 'one', v('one_$i.json'), '| two x512', v('two512_$i.json'), '| two x1024', v('two1024_$i.json'), '| split2', v('split_$i.json'))
EOF
done
echo EXIT 0
