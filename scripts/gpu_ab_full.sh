# One GPU call: bitwise check of the working-tree build against scripts/micro/alt/$ALT, the GPU parity
# tests, then REPS bench pairs (a = working tree, b = ALT).  Usage: ALT=base.so bash scripts/gpu_ab_full.sh TAG
set -o pipefail
TAG=${1:-abf}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 200 python scripts/lib_bitwise.py dump gpurun_out/$TAG/a.npz > gpurun_out/$TAG/bitwise.log 2>&1 || exit $?
PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/$ALT timeout -k 10 200 python scripts/lib_bitwise.py dump gpurun_out/$TAG/b.npz >> gpurun_out/$TAG/bitwise.log 2>&1 || exit $?
python scripts/lib_bitwise.py compare gpurun_out/$TAG/a.npz gpurun_out/$TAG/b.npz >> gpurun_out/$TAG/bitwise.log 2>&1
rm -f gpurun_out/$TAG/a.npz gpurun_out/$TAG/b.npz
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest ${PYTEST_FILES:-tests/test_gpu_parity.py tests/test_gpu_parity16.py} -x -q -m gpu \
    -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
fi
REPS=${REPS:-3} bash scripts/ab_bench.sh $TAG || exit $?
echo EXIT 0
