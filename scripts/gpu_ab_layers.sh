#!/bin/bash
# A/B with per-layer times: bench.py as built (a) vs PETDIFF_LIB=scripts/micro/alt/$ALT (b), REPS pairs.
set -o pipefail
TAG=${1:-abl}
REPS=${REPS:-2}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
for rep in $(seq 1 $REPS); do
  timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-extras > gpurun_out/$TAG/a$rep.json 2>/dev/null || exit $?
  PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/$ALT timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-extras > gpurun_out/$TAG/b$rep.json 2>/dev/null || exit $?
done
python - <<PY
import json,glob
for f in sorted(glob.glob('gpurun_out/$TAG/*.json')):
    d=json.load(open(f)); print(f.split('/')[-1], d['value'], {k:v for k,v in d['layer_us'].items() if v})
PY
