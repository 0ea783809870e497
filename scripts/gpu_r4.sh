#!/bin/bash
# Round-4 GPU check of the working tree.  Stages (STAGES, default "bitwise tests bench"):
#   bitwise  scripts/lib_bitwise.py dumps of every ALT build (scripts/micro/alt/<name>.so) and of this
#            build, compared array by array (bf16 / fp16 / bf16x3 forwards + 20-step loops)
#   tests    the GPU test suite;  smoke  __graft_entry__.smoke()
#   micro    conv_micro step layers in isolation + stamps (prebuilt binaries)
#   pmc      rocprofv3 PMC passes (bf16, bf16x3) -> $OUT/pmc_traffic.json (bench.py's per-kernel counters)
#   cores    scripts/micro/coresident.sh (down1 co-residency experiment, prebuilt binaries)
#   ldspmc   one rocprofv3 PMC pass of the LDS counters per network (bank conflicts per kernel)
#   bench    the driver's bench command (1 GPU) and a rocprofv3 kernel-stats pass
#   ab       REPS interleaved bench pairs: this build vs each ALT build and each ALTENVS setting (VAR=value)
# Usage: ALTS="pre_prune.so" STAGES="bitwise tests" [PYTEST_K="expr"] bash scripts/gpu_r4.sh TAG
set -o pipefail
TAG=${1:-r4}
STAGES=${STAGES:-"bitwise tests bench"}
REPS=${REPS:-2}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
has() { [[ " $STAGES " == *" $1 "* ]]; }
if has bitwise; then
  timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/cur.npz > $OUT/bitwise.txt 2>&1 || { echo "dump failed"; exit 1; }
  for alt in $ALTS; do
    PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/$alt timeout -k 10 300 python scripts/lib_bitwise.py dump $OUT/${alt%.so}.npz >> $OUT/bitwise.txt 2>&1 || { echo "dump $alt failed"; exit 1; }
    echo "== $alt vs this build" >> $OUT/bitwise.txt
    python scripts/lib_bitwise.py compare $OUT/${alt%.so}.npz $OUT/cur.npz >> $OUT/bitwise.txt 2>&1
  done
  grep -E "==|ALL|differ" $OUT/bitwise.txt
fi
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_ARGS} > $OUT/pytest.log 2>&1
  rc=$?
  echo "pytest exit $rc" >> $OUT/pytest.log
  tail -4 $OUT/pytest.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest died ($rc)"; exit $rc; fi
fi
if has smoke; then
  timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
  tail -1 $OUT/smoke.log
fi
if has cores; then
  timeout -k 10 300 bash scripts/micro/coresident.sh > $OUT/coresident.txt 2>&1 || { echo "coresident failed"; tail $OUT/coresident.txt; exit 1; }
  grep -E "==|down1|checksum" $OUT/coresident.txt | head -40
fi
if has micro; then
  # conv_micro (prebuilt: MODES="0 128" bash scripts/micro/build.sh): the 16-bit step layers in isolation, with
  # per-workgroup s_memrealtime stamps in mode 128 (prologue / loop / epilogue; the final level's epilogue parts)
  # MICRO_MODES: the prebuilt modes to run (default "0 128")
  : > $OUT/micro.txt
  for sel in f x; do
    for m in ${MICRO_MODES:-0 128}; do
      (cd scripts/micro && timeout -k 10 120 ./conv_micro_m$m 1024 $sel) >> $OUT/micro.txt 2>&1 || { echo "micro failed"; tail $OUT/micro.txt; exit 1; }
    done
  done
  grep -E "us|mode" $OUT/micro.txt | head -40
fi
if has pmc; then
  # PMC passes over the bf16 and bf16x3 networks; the summaries stamp profiles/pmc_traffic.json with this
  # build's kernel code hash (copied back under gpurun_out/TAG)
  bash scripts/gpu_pmc.sh ${TAG}_pmc || exit 1
  python scripts/pmc_summary.py gpurun_out/${TAG}_pmc gpurun_out/${TAG}_pmc/pmc.json --traffic > gpurun_out/${TAG}_pmc/summary.txt 2>&1 || exit 1
  BENCH_EXTRA="--dtype bf16x3" bash scripts/gpu_pmc.sh ${TAG}_pmc_x3 || exit 1
  python scripts/pmc_summary.py gpurun_out/${TAG}_pmc_x3 gpurun_out/${TAG}_pmc_x3/pmc.json --traffic --dtype=bf16x3 > gpurun_out/${TAG}_pmc_x3/summary.txt 2>&1 || exit 1
  cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
fi
if has ldspmc; then
  # one PMC pass (LDS counters) per network: a quick bank-conflict check without the full pmc stage
  for d in bfloat16 bf16x3; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL \
      -d $GRAFT_REPO_ROOT/$OUT/lds_$d/p1 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 \
      --reverse-steps 20 --no-cpu-baseline --no-kernel-timing --dtype $d > $OUT/lds_$d.log 2>&1 || { echo "lds pmc failed"; exit 1; }
    python scripts/pmc_summary.py $OUT/lds_$d > $OUT/lds_$d.txt 2>&1 || exit 1
    grep -E "^(down|up)" $OUT/lds_$d.txt
  done
fi
if has mhpmc; then
  # configs[2]'s chain kernel (10k chains, mh_chain_kernel) on a short run: its time unprofiled, then one
  # rocprofv3 PMC pass per counter group (instruction mix, issue / wait cycles, LDS, fetched bytes)
  MHAPP="python $GRAFT_REPO_ROOT/bench.py --workload mh --mh-iters 300 --mh-tune 300 --no-cpu-baseline"
  timeout -k 10 120 $MHAPP > $OUT/mh_short.json 2> $OUT/mh_short.err || { echo "mh short failed"; exit 1; }
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/mhpmc/kt -o run --output-format csv -- $MHAPP > $OUT/mhpmc_kt.log 2>&1 || { echo "mh kt failed"; exit 1; }
  i=0
  for CTR in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INST_CYCLES_SALU" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CTR -d $GRAFT_REPO_ROOT/$OUT/mhpmc/p$i -o run --output-format csv -- $MHAPP > $OUT/mhpmc_p$i.log 2>&1 || { echo "mh pmc pass $i failed"; tail -5 $OUT/mhpmc_p$i.log; exit 1; }
  done
  python scripts/mh_pmc_summary.py $OUT/mhpmc 10000 600 $OUT/mh_pmc.json > /dev/null || { echo "mh pmc summary failed"; exit 1; }
  cp $OUT/mh_pmc.json profiles/mh_pmc.json   # (the bench stage below reads it)
  head -c 300 $OUT/mh_short.json; echo
fi
if has bench; then
  timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_EXTRA} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
  head -c 400 $OUT/bench.json; echo
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline --no-extras ${BENCH_EXTRA} > $OUT/bench_prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof_x3 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline --no-extras --dtype bf16x3 > $OUT/bench_prof_x3.log 2>&1 || { echo "rocprof x3 failed"; exit 1; }
fi
if has ab; then
  for rep in $(seq 1 $REPS); do
    for d in bfloat16 bf16x3; do
      timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-extras --dtype $d > $OUT/ab_cur_${d}_$rep.json 2>/dev/null || exit 1
      for alt in $ALTS; do
        PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/$alt timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-extras --dtype $d > $OUT/ab_${alt%.so}_${d}_$rep.json 2>/dev/null || exit 1
      done
      for ev in $ALTENVS; do
        env $ev timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-extras --dtype $d > $OUT/ab_env_${ev//[=]/_}_${d}_$rep.json 2>/dev/null || exit 1
      done
    done
  done
  python - <<PY
import json, glob
for f in sorted(glob.glob('$OUT/ab_*.json')):
    d = json.load(open(f)); print(f.split('/')[-1], round(d['value'], 1), {k: round(v, 2) for k, v in d.get('layer_us', {}).items() if v})
PY
fi
echo EXIT 0
