# A/B the product library against an alternative build (scripts/micro/alt/$ALT) in one GPU call:
# bench.py alternately with each library.  Usage: ALT=libpetdiff_nt.so bash scripts/ab_bench.sh TAG
set -o pipefail
TAG=${1:-ab}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-kernel-timing > gpurun_out/$TAG/a$rep.json 2>/dev/null || exit $?
  PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/$ALT timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-kernel-timing > gpurun_out/$TAG/b$rep.json 2>/dev/null || exit $?
done
echo EXIT 0
