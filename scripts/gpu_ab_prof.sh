# Parity tests, A/B of the product build vs scripts/micro/alt/$ALT, and kernel stats of both.
# Usage: ALT=<name>.so bash scripts/gpu_ab_prof.sh TAG
set -o pipefail
TAG=${1:-abp}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
REPS=${REPS:-3} bash scripts/ab_bench.sh ${TAG}_ab || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_a -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline > gpurun_out/$TAG/prof_a.log 2>&1 && \
PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/$ALT timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_b -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline > gpurun_out/$TAG/prof_b.log 2>&1
echo EXIT $?
