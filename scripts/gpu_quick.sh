# Quick GPU check: conv micro-benchmark + U-Net parity tests.  Usage: bash scripts/gpu_quick.sh TAG
set -o pipefail
TAG=${1:-quick}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
MODES="${MODES:-0 128}" TAG=$TAG bash scripts/micro/run.sh > /dev/null || exit $?
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/$TAG/pytest.log
echo EXIT $rc
