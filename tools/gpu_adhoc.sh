export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for r in 1 2 3; do
  for lib in product abtest/libofdm_h2mul.so; do
    if [ $lib = product ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=$GRAFT_REPO_ROOT/$lib; fi
    echo -n "$lib "; timeout -k 10 120 python3 tools/ab_step.py || exit 1
  done
done
