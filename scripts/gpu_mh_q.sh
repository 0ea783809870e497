#!/bin/bash
set -e
mkdir -p gpurun_out/micro
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mh.py > gpurun_out/pytest_mh.txt 2>&1
rm -f gpurun_out/micro/mhq.txt
cd scripts/micro
for b in mh_micro_pair mh_micro_single mh_micro_pair; do
  PETMH_KERNEL=batched timeout -k 10 120 ./$b mh_problem.bin >> $GRAFT_REPO_ROOT/gpurun_out/micro/mhq.txt 2>&1
done
cd ../..
timeout -k 10 300 python -u scripts/mh_ab.py > gpurun_out/mh_ab3.jsonl
cat gpurun_out/micro/mhq.txt gpurun_out/mh_ab3.jsonl; tail -2 gpurun_out/pytest_mh.txt
