# round 3: the secondary bench workloads on the final build -- configs[3] per-rank shard (32 TACs x 8192),
# the fp16 network (configs[4] dtype), MH configs[2], the training step -- plus the new MH op test.
# Usage: bash scripts/gpu_secondary_r3.sh TAG
set -o pipefail
TAG=${1:-secondary}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_mh.py -q -x -k "create_tac or srtm2" --timeout 120 --timeout-method thread \
  > $OUT/pytest_mh_op.log 2>&1; rc=$?; tail -2 $OUT/pytest_mh_op.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --no-extras"
timeout -k 10 300 python bench.py --config4 --steps 1 --warmup 1 $B > $OUT/bench_config4.json 2> $OUT/bench_config4.err || exit 1
timeout -k 10 200 python bench.py --dtype float16 --steps 10 --warmup 3 $B > $OUT/bench_f16.json 2> $OUT/bench_f16.err || exit 1
timeout -k 10 200 python bench.py --workload mh --steps 1 --warmup 1 > $OUT/bench_mh.json 2> $OUT/bench_mh.err || exit 1
timeout -k 10 200 python bench.py --workload train --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_train.json 2> $OUT/bench_train.err || exit 1
for f in config4 f16 mh train; do head -c 400 $OUT/bench_$f.json; echo; done
echo EXIT 0
