#!/bin/bash
# A/B of several alternative builds against the product build, interleaved, with per-layer times.
# Usage: ALTS="a.so b.so" REPS=2 bash scripts/gpu_ab_multi.sh TAG
set -o pipefail
TAG=${1:-abm}
REPS=${REPS:-2}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
for rep in $(seq 1 $REPS); do
  timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-extras > gpurun_out/$TAG/base_$rep.json 2>/dev/null || exit $?
  for alt in $ALTS; do
    PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/$alt timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-extras > gpurun_out/$TAG/${alt%.so}_$rep.json 2>/dev/null || exit $?
  done
done
python - <<PY
import json,glob
for f in sorted(glob.glob('gpurun_out/$TAG/*.json')):
    d=json.load(open(f)); print(f.split('/')[-1], d['value'], {k:v for k,v in d['layer_us'].items() if v})
PY
