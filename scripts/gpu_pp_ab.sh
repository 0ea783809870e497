# down1 pair-position-major (CONV_DOWN1_PP) vs sample-major rows (scripts/micro/alt/$ALT):
# bitwise dump compare, the 16-bit parity tests, REPS bench pairs, PMC passes of both builds.
# Usage: ALT=base.so bash scripts/gpu_pp_ab.sh TAG
set -o pipefail
TAG=${1:-ppab}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ARGS="--steps 3 --no-extras" REPS=${REPS:-3} PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_parity16.py tests/test_gpu_bf16x3.py" \
  bash scripts/gpu_ab_full.sh $TAG || exit $?
bash scripts/gpu_pmc_ab.sh ${TAG}_pmc || exit $?
echo EXIT 0
