#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mh.py > gpurun_out/pytest_mh.txt 2>&1
rm -f gpurun_out/mh_sweep.jsonl
PETMH_KERNEL=wave timeout -k 10 200 python -u scripts/mh_sweep.py >> gpurun_out/mh_sweep.jsonl
for w in 0 4 12; do
  if [ $w = 0 ]; then unset PETMH_WPC; else export PETMH_WPC=$w; fi
  PETMH_KERNEL=batched timeout -k 10 200 python -u scripts/mh_sweep.py >> gpurun_out/mh_sweep.jsonl
done
unset PETMH_WPC
timeout -k 10 300 python -u scripts/mh_ab.py > gpurun_out/mh_ab2.jsonl
cat gpurun_out/mh_sweep.jsonl gpurun_out/mh_ab2.jsonl
tail -2 gpurun_out/pytest_mh.txt
