# up0.fused in isolation (conv_micro, B = 1024): zero-skip vs tap-reuse builds, product mode and
# stamps (128), with the in-loop DMA issue removed (129) or the MFMAs removed (130).
set -o pipefail
cd $GRAFT_REPO_ROOT/scripts/micro
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-zsmicro}
mkdir -p $OUT
for b in fb_zs0 fb_rs0 fb_zs128 fb_rs128 fb_zs129 fb_zs130 fb_zs0 fb_rs0; do
  echo "== $b" >> $OUT/micro.txt
  timeout -k 10 60 ./$b 1024 u0 >> $OUT/micro.txt 2>&1 || exit $?
done
echo EXIT 0
