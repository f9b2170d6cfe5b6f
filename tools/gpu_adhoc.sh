#!/bin/bash
# scratch slot for one-off GPU commands (overwritten per experiment)
# current: tx grid sweep at 4 workgroups per CU (abtest/libofdm_txgrid.so, OFDM_EXP_TX_GRID)
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/txgrid4.txt
: > $O
for rep in 1 2; do
  timeout -k 10 120 python tools/ab_step.py 2>/dev/null | sed "s/^/product /" >> $O || exit 1
  for g in 1024 2048 3072 5120 8192 16384; do
    OFDM_MI355X_LIB=abtest/libofdm_txgrid.so OFDM_EXP_TX_GRID=$g timeout -k 10 120 python tools/ab_step.py 2>/dev/null | sed "s/^/grid $g /" >> $O || exit 1
  done
done
cat $O
