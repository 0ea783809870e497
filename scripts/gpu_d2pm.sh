set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/d2pm
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/d2pm/pytest.log 2>&1 || { echo "pytest failed $?"; tail -30 gpurun_out/d2pm/pytest.log; exit 1; }
tail -2 gpurun_out/d2pm/pytest.log
timeout -k 10 200 python scripts/lib_bitwise.py dump gpurun_out/d2pm/a.npz && \
PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/down2_sm.so timeout -k 10 200 python scripts/lib_bitwise.py dump gpurun_out/d2pm/b.npz && \
python scripts/lib_bitwise.py compare gpurun_out/d2pm/a.npz gpurun_out/d2pm/b.npz > gpurun_out/d2pm/bitwise.txt; cat gpurun_out/d2pm/bitwise.txt | tail -3
rm -f gpurun_out/d2pm/*.npz
ALT=down2_sm.so REPS=3 bash scripts/ab_bench.sh d2pm_ab && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/d2pm/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline > gpurun_out/d2pm/prof.log 2>&1
echo EXIT $?
