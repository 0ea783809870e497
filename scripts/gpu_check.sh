# Focused GPU check: selected tests (-k EXPR), then optionally an A/B bench (ENVB / ALT as ab_bench.sh).
# Usage: K="fused_up" TAG=x [AB=1 ENVB="PETDIFF_FUSE_UP=0"] bash scripts/gpu_check.sh
set -o pipefail
TAG=${TAG:-check}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu -k "$K" > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/$TAG/pytest.log
tail -5 gpurun_out/$TAG/pytest.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$AB" ]; then bash scripts/ab_bench.sh ${TAG}_ab || exit $?; fi
echo EXIT 0
