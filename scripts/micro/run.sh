set -o pipefail
cd $GRAFT_REPO_ROOT/scripts/micro
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/micro
for m in ${MODES:-0 1 2 3 4 5 6}; do
  timeout -k 10 60 ./conv_micro_m$m ${B:-1024} >> $GRAFT_REPO_ROOT/gpurun_out/micro/${TAG:-m}.txt 2>&1 || exit $?
done
echo EXIT 0
