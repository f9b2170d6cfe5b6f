#!/bin/bash
# rx stagger experiment: the CU's second rx workgroup started late (abtest/
# variants) vs the product, bench.py's step per kernel (tools/ab_step.py), 3 rounds
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/r04p_rx_stagger.jsonl; : > $OUT
for round in 1 2 3; do
  for lib in product abtest/libofdm_stag8.so abtest/libofdm_stag16.so abtest/libofdm_stag24.so; do
    if [ "$lib" = product ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=$R/$lib; fi
    timeout -k 10 120 python tools/ab_step.py >> $OUT 2>/dev/null || { echo "failed $lib"; exit 1; }
  done
done
unset OFDM_MI355X_LIB
cat $OUT
