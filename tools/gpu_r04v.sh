#!/bin/bash
# round 4 (v): SQ counters of the stream kernels after the per-format
# instantiation (D f64, D int16, B f64, B int16)
export TMPDIR=/tmp
mkdir -p gpurun_out
for args in "" "--i16" "--config B --frames 4096" "--config B --frames 4096 --i16"; do
  tag=$(echo "D $args" | tr -d ' -' | sed 's/configB/B/; s/frames4096//')
  bash tools/sq_stream.sh $args || { echo "sq_stream failed for '$args'"; tail gpurun_out/ss1.log gpurun_out/ss2.log; exit 1; }
  cp gpurun_out/sq_stream.txt gpurun_out/r04v_sq_$tag.txt
  echo "== $tag"; grep -E "SQ_INSTS_VALU|SQ_WAVES |SQ_ACTIVE_INST_VALU|GRBM_GUI_ACTIVE|SQ_BUSY_CYCLES" gpurun_out/sq_stream.txt | grep -v compact
done
