# Where the final level's time (up2.fused + final conv + p_sample + next-step down0 + down1) goes, and
# which phase owns its LDS bank conflicts: micro builds of the product kernel with parts removed
# (FIN_EXP 1: no down0, 4: no row loop; d1: the fused down1 on), stamps (mode 128), and one
# rocprofv3 PMC pass (LDS bank conflicts) per build.
# Build here (CPU): bash scripts/micro/up2_phases.sh build;  run on the GPU box: bash scripts/micro/up2_phases.sh run TAG
set -o pipefail
cd "$(dirname "$0")"
VARIANTS="m0:-DCONV_EXP_MODE=0 m0r:-DFD1_LDS=0 m128:-DCONV_EXP_MODE=128 m128r:-DCONV_EXP_MODE=128@-DFD1_LDS=0 f1:-DFIN_EXP=1 f4:-DFIN_EXP=4"
if [ "$1" = build ]; then
  for v in $VARIANTS; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 $(echo ${v#*:} | tr @ " ") conv_micro.hip -o fb_${v%%:*} &
  done
  wait
  exit 0
fi
TAG=${2:-u2}
OUT=$GRAFT_REPO_ROOT/gpurun_out/micro/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in $VARIANTS; do
  b=fb_${v%%:*}
  for d in nod1 d1; do
    echo "== $b $d" >> $OUT/times.txt
    timeout -k 10 60 ./$b 1024 u2 $d >> $OUT/times.txt 2>&1 || exit $?
  done
done
for v in m0 m0r f1 f4; do
  for d in nod1 d1; do
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES \
      -d $OUT/pmc_${v}_$d -o run --output-format csv -- ./fb_$v 1024 u2 $d > $OUT/pmc_${v}_$d.log 2>&1 || exit $?
  done
done
echo EXIT 0
