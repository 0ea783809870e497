# Fused next-step down1 (PETDIFF_FUSE_DOWN1, default on) vs the standalone down1 launch:
# bitwise dump compare, the GPU suite, REPS bench pairs (a = fused, b = PETDIFF_FUSE_DOWN1=0),
# rocprofv3 kernel stats of the fused build.  Usage: bash scripts/gpu_fd1_ab.sh TAG
set -o pipefail
TAG=${1:-fd1}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 200 python scripts/lib_bitwise.py dump gpurun_out/$TAG/a.npz > gpurun_out/$TAG/bitwise.log 2>&1 || exit $?
PETDIFF_FUSE_DOWN1=0 timeout -k 10 200 python scripts/lib_bitwise.py dump gpurun_out/$TAG/b.npz >> gpurun_out/$TAG/bitwise.log 2>&1 || exit $?
python scripts/lib_bitwise.py compare gpurun_out/$TAG/a.npz gpurun_out/$TAG/b.npz >> gpurun_out/$TAG/bitwise.log 2>&1
rm -f gpurun_out/$TAG/a.npz gpurun_out/$TAG/b.npz
tail -3 gpurun_out/$TAG/bitwise.log
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/$TAG/pytest.log; tail -2 gpurun_out/$TAG/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest died ($rc)"; exit $rc; fi
ENVB="PETDIFF_FUSE_DOWN1=0" ARGS="--steps 3 --no-extras" REPS=${REPS:-3} bash scripts/ab_bench.sh $TAG || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline --no-extras > gpurun_out/$TAG/prof.log 2>&1
echo EXIT $?
