# A/B the product library in one GPU call: bench.py alternately as built (a) and as the
# variant (b).  The variant is an alternative build (ALT=scripts/micro/alt/<name>.so) or an
# environment switch (ENVB="PETDIFF_FUSE_DOWN0=0").  Usage: ALT=... | ENVB=... bash scripts/ab_bench.sh TAG
set -o pipefail
TAG=${1:-ab}
REPS=${REPS:-2}
ARGS=${ARGS:---steps 3}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
for rep in $(seq 1 $REPS); do
  timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline --no-kernel-timing > gpurun_out/$TAG/a$rep.json 2>/dev/null || exit $?
  ( if [ -n "$ALT" ]; then export PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/$ALT; fi
    if [ -n "$ENVB" ]; then export $ENVB; fi
    timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline --no-kernel-timing > gpurun_out/$TAG/b$rep.json 2>/dev/null ) || exit $?
done
echo EXIT 0
