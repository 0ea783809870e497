# Round-3 final build: full validation (tests, smoke, PMC passes, driver bench, rocprof) then the secondary
# workloads.  Usage: bash scripts/gpu_final_r3.sh TAG
set -o pipefail
TAG=${1:-final}
cd $GRAFT_REPO_ROOT
bash scripts/gpu_full_r3.sh $TAG || exit 1
bash scripts/gpu_secondary_r3.sh ${TAG}_sec || exit 1
echo EXIT 0
