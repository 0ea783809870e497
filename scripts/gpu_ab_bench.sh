# A/B of the product build against scripts/micro/alt/$ALT (bench.py, REPS pairs), then the default
# bench line.  Usage: ALT=<name>.so bash scripts/gpu_ab_bench.sh TAG
set -o pipefail
TAG=${1:-abb}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
REPS=${REPS:-3} bash scripts/ab_bench.sh ${TAG}_ab || exit $?
timeout -k 10 400 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
echo EXIT $?
