# rocprofv3 kernel stats of the current build and of scripts/micro/alt/$ALT on one box (bench.py ARGS).
# Usage: ALT=prev.so ARGS="--dtype bf16x3" bash scripts/gpu_prof2_r3.sh TAG
set -o pipefail
TAG=${1:-prof2}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in cur alt cur2; do
  ( if [ $v = alt ]; then export PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/$ALT; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/$v -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 $ARGS --no-cpu-baseline --no-extras > $OUT/$v.log 2>&1 ) || exit 1
done
echo EXIT 0
