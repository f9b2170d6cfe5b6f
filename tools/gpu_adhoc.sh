#!/bin/bash
# scratch slot for one-off GPU commands (overwritten per experiment)
# current: tx dynamic symbol queue (product build) vs HEAD (abtest/libofdm_head.so),
# and a static tx grid-size sweep (abtest/libofdm_txgrid.so, OFDM_EXP_TX_GRID;
# negative = that many workgroups per CU)
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/txq.txt
: > $O
for rep in 1 2 3; do
  OFDM_MI355X_LIB=abtest/libofdm_head.so timeout -k 10 120 python tools/ab_step.py 2>/dev/null | sed "s/^/head /" >> $O || exit 1
  timeout -k 10 120 python tools/ab_step.py 2>/dev/null | sed "s/^/queue /" >> $O || exit 1
done
for g in -3 -6 8192 65536; do
  OFDM_MI355X_LIB=abtest/libofdm_txgrid.so OFDM_EXP_TX_GRID=$g timeout -k 10 120 python tools/ab_step.py 2>/dev/null | sed "s/^/grid $g /" >> $O || exit 1
done
cat $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "tx or loopback or parity or bench or dropin" > gpurun_out/txq_tests.log 2>&1; tail -3 gpurun_out/txq_tests.log
