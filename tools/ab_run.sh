#!/bin/bash
# A/B of the product library and every abtest/ variant on bench.py's step, twice
# each in alternation (same box); output gpurun_out/ab_<tag>.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-run}
OUT=gpurun_out/ab_$TAG.jsonl
: > $OUT
for r in 1 2; do
  timeout -k 10 120 python tools/ab_step.py >> $OUT 2>/dev/null || exit 1
  for v in abtest/libofdm_*.so; do
    OFDM_MI355X_LIB=$PWD/$v timeout -k 10 120 python tools/ab_step.py >> $OUT 2>/dev/null || exit 1
  done
done
