# Where the fused down1's time goes (FD1_LDS path): stamps (K loop vs epilogue + drain) of builds with parts
# removed (FD1_DIAG 2: no MFMAs, 4: no B DMA, 8: no staging / stores, 14: none of them).
# Run on the GPU box: bash scripts/micro/fd1_diag.sh TAG   (binaries fb_s* built here with hipcc, see DESIGN)
set -o pipefail
cd "$(dirname "$0")"
OUT=$GRAFT_REPO_ROOT/gpurun_out/micro/${1:-fd1diag}
mkdir -p $OUT
for b in fb_sd0 fb_sd2 fb_sd4 fb_sd8 fb_sd14 fb_sd0; do
  echo "== $b" >> $OUT/times.txt
  timeout -k 10 60 ./$b 1024 u2 d1 >> $OUT/times.txt 2>&1 || exit $?
done
grep -E "==|final epilogue|up2.fused" $OUT/times.txt
echo EXIT 0
