# rocprofv3 kernel stats of the bf16x3 and fp16 networks on the current build (bench.py --dtype ...).
set -o pipefail
TAG=${1:-profdt}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for dt in bf16x3 float16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/$dt -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --dtype $dt --no-cpu-baseline --no-extras > $OUT/$dt.log 2>&1 || exit 1
done
echo EXIT 0
