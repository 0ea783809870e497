# up0.fused in isolation (conv_micro, B = 1024, stamps): which part of the K loop sets the clock.
# 128 product, 129 no in-loop DMA, 130 no MFMAs, 131 neither, 192 no LDS fragment reads, 193 MFMAs only.
set -o pipefail
cd $GRAFT_REPO_ROOT/scripts/micro
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-power}
mkdir -p $OUT
for b in fb_zs128 fb_zs129 fb_zs130 fb_zs131 fb_zs192 fb_zs193 fb_zs128; do
  echo "== $b" >> $OUT/micro.txt
  timeout -k 10 60 ./$b 1024 u0 >> $OUT/micro.txt 2>&1 || exit $?
done
echo EXIT 0
