#!/bin/bash
# Co-residency experiment: down1 as built (3-stage ring of 64-B
# chunks, loader waves, ~150 KB LDS: one workgroup per CU) against CONV_DOWN1_CORES=1 (2-stage ring of 32-B
# chunks, 4 waves, C tile staged in two row blocks: ~62 KB of LDS, 186 VGPRs, so two workgroups share a
# CU).  B = 1024 launches 256 workgroups (one per CU either way); B = 2048 and 4096 launch 512 / 1024, which
# the small variant can run two at a time per CU.  Mode 128: per-workgroup s_memrealtime stamps.
# Build: for v in 0 1; do for m in 0 128; do hipcc -O3 -std=c++17 --offload-arch=gfx950 -DCONV_EXP_MODE=$m \
#          -DCONV_DOWN1_CORES=$v conv_micro.hip -o coresident_m${m}_c$v; done; done
set -o pipefail
cd "$(dirname "$0")"
for B in 1024 2048 4096; do
  for v in 0 1; do
    echo "== B=$B variant c$v"
    timeout -k 10 60 ./coresident_m0_c$v $B d1 || exit 1
    timeout -k 10 60 ./coresident_m128_c$v $B d1 || exit 1
  done
done
