# Full GPU round-trip: parity tests, iDDPM bench + rocprofv3 stats, PMC passes, MH bench (config 3).
# Usage: bash scripts/gpu_round.sh TAG
set -o pipefail
TAG=${1:-round}
cd $GRAFT_REPO_ROOT
bash scripts/gpu_test_bench.sh $TAG || exit $?
grep -q "pytest exit 0" gpurun_out/$TAG/pytest.log || { echo "tests failed"; exit 1; }
bash scripts/gpu_pmc.sh ${TAG}_pmc || exit $?
python scripts/pmc_summary.py gpurun_out/${TAG}_pmc gpurun_out/${TAG}_pmc/pmc.json --traffic > gpurun_out/${TAG}_pmc/summary.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload mh > gpurun_out/$TAG/bench_mh.json 2> gpurun_out/$TAG/bench_mh.err
echo EXIT $?
