# round 3: A/B of HIP runtime environment switches on the bf16 bench (separate processes, alternating),
# e.g. kernel arguments in device memory, or PETDIFF_LIB=<another build>; BENCH_EXTRA: more bench flags.  Usage: bash scripts/gpu_envab_r3.sh TAG "VAR=VAL [VAR2=VAL2]"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-envab}
ENVB=${2:-HIP_FORCE_DEV_KERNARG=1}
mkdir -p gpurun_out/$TAG
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing --no-extras $BENCH_EXTRA \
    > gpurun_out/$TAG/a$i.json 2> gpurun_out/$TAG/a$i.err || exit 1
  timeout -k 10 120 env $ENVB python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing --no-extras $BENCH_EXTRA \
    > gpurun_out/$TAG/b$i.json 2> gpurun_out/$TAG/b$i.err || exit 1
  python -c "import json,sys; a=json.load(open('gpurun_out/$TAG/a$i.json')); b=json.load(open('gpurun_out/$TAG/b$i.json')); print('$i default', a['value'], '| $ENVB', b['value'])"
done
echo EXIT 0
