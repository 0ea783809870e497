# Uniform-position prologue for the position-major layers: parity, bitwise vs the down2 PM build,
# A/B vs the previous build and vs down2 PM, kernel stats.  Usage: bash scripts/gpu_pm_prologue.sh TAG
set -o pipefail
TAG=${1:-pmpro}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
timeout -k 10 200 python scripts/lib_bitwise.py dump gpurun_out/$TAG/a.npz > /dev/null && \
PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/down2_pm.so timeout -k 10 200 python scripts/lib_bitwise.py dump gpurun_out/$TAG/b.npz > /dev/null && \
python scripts/lib_bitwise.py compare gpurun_out/$TAG/a.npz gpurun_out/$TAG/b.npz > gpurun_out/$TAG/bitwise.txt; tail -1 gpurun_out/$TAG/bitwise.txt
rm -f gpurun_out/$TAG/*.npz
ALT=head.so REPS=3 bash scripts/ab_bench.sh ${TAG}_ab_head || exit $?
ALT=down2_pm.so REPS=3 bash scripts/ab_bench.sh ${TAG}_ab_d2pm || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline > gpurun_out/$TAG/prof.log 2>&1 && \
PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/down2_pm.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_d2pm -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline > gpurun_out/$TAG/prof_d2pm.log 2>&1
echo EXIT $?
