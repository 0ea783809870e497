# Per-layer times of the product's 16-bit step kernels in isolation (random bf16 data, B = 1024):
# mode 0 (product), 16 (return after the prologue), 4 (no epilogue), 128 (stamps: prologue / loop / epilogue),
# and the final-level epilogue parts (FIN_EXP 1: no fused down0, 4: no row loop, 8: fp32 Box-Muller).
# Build here (CPU): bash scripts/micro/fused_breakdown.sh build;  run on the GPU box: bash scripts/micro/fused_breakdown.sh run TAG
set -o pipefail
cd "$(dirname "$0")"
if [ "$1" = build ]; then
  for v in m0:-DCONV_EXP_MODE=0 m16:-DCONV_EXP_MODE=16 m4:-DCONV_EXP_MODE=4 m128:-DCONV_EXP_MODE=128 \
           f1:-DFIN_EXP=1 f4:-DFIN_EXP=4 f8:-DFIN_EXP=8 f5:-DFIN_EXP=5; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 ${v#*:} conv_micro.hip -o fb_${v%%:*} &
  done
  wait
  exit 0
fi
TAG=${2:-fb}
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/micro
for b in fb_m0 fb_m16 fb_m4 fb_m128 fb_f1 fb_f4 fb_f8 fb_f5; do
  echo "== $b" >> $GRAFT_REPO_ROOT/gpurun_out/micro/$TAG.txt
  timeout -k 10 60 ./$b 1024 f >> $GRAFT_REPO_ROOT/gpurun_out/micro/$TAG.txt 2>&1 || exit $?
done
echo EXIT 0
