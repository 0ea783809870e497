set -o pipefail
cd $GRAFT_REPO_ROOT/scripts/micro
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/micro
for b in mh_micro_*; do
  [ -x "$b" ] || continue
  timeout -k 10 120 ./$b mh_problem.bin >> $GRAFT_REPO_ROOT/gpurun_out/micro/${TAG:-mh}.txt 2>&1 || exit $?
done
echo EXIT 0
