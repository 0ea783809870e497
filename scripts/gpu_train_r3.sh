# round 3: the reference's training protocol on the reference prior (prior_stats_nROI48), then the
# posterior of 8 held-out TACs scored against the MH baseline (reference protocol, with R-hat).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3train
timeout -k 10 1120 python -u scripts/train_protocol.py gpurun_out/r3train --epochs 500 --eval-tacs 8 --period 100000 --mh-textbook \
  --time-budget 880 > gpurun_out/r3train/train_log.txt 2>&1
echo EXIT $?
