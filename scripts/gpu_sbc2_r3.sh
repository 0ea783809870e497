# round 3: MH calibration variants -- the textbook element-wise ratio, and PyMC's with twice the chain length
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
timeout -k 10 500 python -u scripts/mcmc_calibration.py gpurun_out/r3c/sbc_textbook.json --tacs 32 --textbook > gpurun_out/r3c/sbc_textbook.log 2>&1 || exit 1
tail -1 gpurun_out/r3c/sbc_textbook.log | cut -c1-600
timeout -k 10 700 python -u scripts/mcmc_calibration.py gpurun_out/r3c/sbc_long.json --tacs 32 --draws 40000 --tune 80000 > gpurun_out/r3c/sbc_long.log 2>&1 || exit 1
tail -1 gpurun_out/r3c/sbc_long.log | cut -c1-600
echo EXIT 0
