# round 3: MH simulation-based calibration on the reference prior (32 TACs, reference protocol).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
timeout -k 10 1000 python -u scripts/mcmc_calibration.py gpurun_out/r3c/sbc.json --tacs 32 > gpurun_out/r3c/sbc.log 2>&1
echo EXIT $?
