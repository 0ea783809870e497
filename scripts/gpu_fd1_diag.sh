cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/fd1d
for v in prod diag1 diag2; do
  if [ $v != prod ]; then export PETDIFF_LIB=$GRAFT_REPO_ROOT/scripts/micro/alt/fd1$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/fd1d/$v -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --no-cpu-baseline --no-extras --no-kernel-timing > gpurun_out/fd1d/$v.log 2>&1 || exit $?
done
echo EXIT 0
