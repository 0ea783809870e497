#!/bin/bash
# MH: GPU tests + A/B of the batched-proposal kernel vs the one-update-at-a-time kernel (same call)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mh.py > gpurun_out/pytest_mh.txt 2>&1
for k in batched wave batched; do
  if [ "$k" = wave ]; then export PETMH_KERNEL=wave; else unset PETMH_KERNEL; fi
  timeout -k 10 300 python -u scripts/mh_ab.py >> gpurun_out/mh_ab.jsonl
done
cat gpurun_out/mh_ab.jsonl
tail -3 gpurun_out/pytest_mh.txt
