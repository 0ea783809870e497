# Kernel-trace stats of bench.py for the product build and each ALTS library, one GPU call.
# Usage: ALTS="fin1.so fin2.so" bash scripts/prof_multi.sh TAG
set -o pipefail
TAG=${1:-profm}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/base -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline --no-kernel-timing > gpurun_out/$TAG/base.log 2>&1 || exit $?
for A in $ALTS; do
  ( export PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/$A
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/${A%.so} -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline --no-kernel-timing > gpurun_out/$TAG/${A%.so}.log 2>&1 ) || exit $?
done
echo EXIT 0
