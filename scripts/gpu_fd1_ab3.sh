# fused down1 A/B (scripts/gpu_fd1_ab2.sh) + the whole GPU suite with PETDIFF_FUSE_DOWN1=1
set -o pipefail
TAG=${1:-fd1g}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
bash scripts/gpu_fd1_ab2.sh $TAG || exit $?
PETDIFF_FUSE_DOWN1=1 timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest_all_fused.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/pytest_all_fused.log; echo EXIT $rc
