# A/B: standalone down1 (a, default) vs PETDIFF_FUSE_DOWN1=1 (b); rocprofv3 stats and the bitwise
# tests with the fusion on.  Usage: bash scripts/gpu_fd1_ab2.sh TAG
set -o pipefail
TAG=${1:-fd1e}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/$TAG
ENVB="PETDIFF_FUSE_DOWN1=1" ARGS="--steps 3 --no-extras" REPS=${REPS:-3} bash scripts/ab_bench.sh $TAG || exit $?
PETDIFF_FUSE_DOWN1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline --no-extras --no-kernel-timing > gpurun_out/$TAG/prof.log 2>&1 || exit $?
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -k "down1_bitwise or down0_bitwise" -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
echo EXIT $?
