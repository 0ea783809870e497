# Full validation of the current build (round 3): the GPU test suite, the driver's bench command, a
# rocprofv3 kernel-stats pass, and PMC passes over the bf16 and bf16x3 networks whose summaries stamp
# profiles/pmc_traffic.json with this build's kernel code-object hash (copied back under gpurun_out/TAG).
# Usage: bash scripts/gpu_full_r3.sh TAG
set -o pipefail
TAG=${1:-full}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  > $OUT/pytest.log 2>&1
rc=$?
echo "pytest exit $rc" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest died ($rc)"; exit $rc; fi
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
bash scripts/gpu_pmc.sh ${TAG}_pmc || exit 1
python scripts/pmc_summary.py gpurun_out/${TAG}_pmc gpurun_out/${TAG}_pmc/pmc.json --traffic > gpurun_out/${TAG}_pmc/summary.txt 2>&1 || exit 1
BENCH_EXTRA="--dtype bf16x3" bash scripts/gpu_pmc.sh ${TAG}_pmc_x3 || exit 1
python scripts/pmc_summary.py gpurun_out/${TAG}_pmc_x3 gpurun_out/${TAG}_pmc_x3/pmc.json --traffic --dtype=bf16x3 > gpurun_out/${TAG}_pmc_x3/summary.txt 2>&1 || exit 1
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
head -c 600 $OUT/bench.json; echo
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline --no-extras > $OUT/bench_prof.log 2>&1 || exit 1
echo EXIT 0
