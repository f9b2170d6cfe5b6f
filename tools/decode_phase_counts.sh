#!/bin/bash
# Executed instructions per segment of the fused stream decode
# (stream_decode_kernel, N = 512): the diagnostics instantiation ends every
# wave at stop point k (OFDM_DECODE_STOP=k; 1 = after pilot_freq_sinh,
# 2 = after the rest of the sync stage and the ramp table, 3 = after the
# message transforms, 4 = after the channel line, phys and the gains,
# 5 = after the emit), the product kernel is the full count. One SQ pass per
# stop point over one stream_bench call; the per-segment numbers are the
# differences (tools/decode_phase_summary.py). Args: extra stream_bench args.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
TAG=${TAG:-dp}
for k in 1 2 3 4 5 0; do
  D=$R/gpurun_out/${TAG}_stop$k; rm -rf $D
  if [ $k = 0 ]; then unset OFDM_DECODE_STOP; else export OFDM_DECODE_STOP=$k; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU \
      --output-format csv -d $D -o run -- python3 tools/stream_bench.py --reps 1 --warmup 1 "$@" > $D.log 2>&1 || { tail $D.log; exit 1; }
done
unset OFDM_DECODE_STOP
python3 tools/decode_phase_summary.py $R/gpurun_out/${TAG}
