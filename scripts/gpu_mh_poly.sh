#!/bin/bash
set -e
mkdir -p gpurun_out/micro
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mh.py > gpurun_out/pytest_mh.txt 2>&1
rm -f gpurun_out/micro/mhpoly.txt
cd scripts/micro
for k in wave; do for b in mh_micro_fexp mh_micro_oexp mh_micro_fexp; do
  echo "kernel=$k" >> $GRAFT_REPO_ROOT/gpurun_out/micro/mhpoly.txt
  PETMH_KERNEL=$k timeout -k 10 120 ./$b mh_problem.bin >> $GRAFT_REPO_ROOT/gpurun_out/micro/mhpoly.txt 2>&1
done; done
cd ../..
timeout -k 10 300 python -u scripts/mh_ab.py > gpurun_out/mh_ab4.jsonl
cat gpurun_out/micro/mhpoly.txt gpurun_out/mh_ab4.jsonl; tail -2 gpurun_out/pytest_mh.txt
