# Builds the conv micro-benchmark in its experiment modes (0 = product code).
set -e
cd "$(dirname "$0")"
for m in ${MODES:-0 1 2 3 4}; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -DCONV_EXP_MODE=$m $EXTRA conv_micro.hip -o conv_micro_m$m$SUFFIX &
done
wait
