# Kernel-trace stats of bench.py as built (a) and with ENVB set (b), one GPU call.
# Usage: ENVB="PETDIFF_FUSE_DOWN0=0" | ALT=<scripts/micro/alt lib> bash scripts/prof_ab.sh TAG
set -o pipefail
TAG=${1:-profab}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/a -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline > gpurun_out/$TAG/a.log 2>&1 || exit $?
( if [ -n "$ALT" ]; then export PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/$ALT; fi
  if [ -n "$ENVB" ]; then export $ENVB; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/b -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline > gpurun_out/$TAG/b.log 2>&1 ) || exit $?
echo EXIT 0
