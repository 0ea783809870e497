# Re-entry check of a freshly rebuilt tree: GPU test suite, smoke, one bench line.
# Usage: bash scripts/gpu_check_r3.sh TAG
set -o pipefail
TAG=${1:-check}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  > $OUT/pytest.log 2>&1
rc=$?
echo "pytest exit $rc" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then echo "pytest failed ($rc)"; exit $rc; fi
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
head -c 400 $OUT/bench.json; echo
echo EXIT 0
