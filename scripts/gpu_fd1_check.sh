# Default build vs scripts/micro/alt/base.so (bitwise) and the fused-down1 bitwise test.
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/fd1c
timeout -k 10 200 python scripts/lib_bitwise.py dump gpurun_out/fd1c/a.npz > gpurun_out/fd1c/bitwise.log 2>&1 || exit $?
PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/base.so timeout -k 10 200 python scripts/lib_bitwise.py dump gpurun_out/fd1c/b.npz >> gpurun_out/fd1c/bitwise.log 2>&1 || exit $?
python scripts/lib_bitwise.py compare gpurun_out/fd1c/a.npz gpurun_out/fd1c/b.npz >> gpurun_out/fd1c/bitwise.log 2>&1
rm -f gpurun_out/fd1c/*.npz; tail -1 gpurun_out/fd1c/bitwise.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/fd1c/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/fd1c/pytest.log; echo EXIT $rc
