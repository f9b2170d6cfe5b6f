#!/bin/bash
# The stream's HBM traffic per call (separate FETCH_SIZE / WRITE_SIZE passes,
# tools/pmc_stream.sh) for the three bench workloads, summarised in the form
# bench.py reads (tools/pmc_stream_summary.py): gpurun_out/pmc_stream_${TAG}_{f64,int16,B}.json
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r05}
mkdir -p $R/gpurun_out
for spec in "f64:--frames 16384" "int16:--frames 16384 --i16" "B:--config B --frames 4096"; do
  mode=${spec%%:*}; a=${spec#*:}
  SUF=_$mode bash tools/pmc_stream.sh $a || exit 1
  line=$(grep '^{' gpurun_out/pmcs_fetch_$mode.log | tail -1)
  w=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['workload'])" "$line")
  alg=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['roofline']['algorithmic_bytes'])" "$line")
  python3 tools/pmc_stream_summary.py gpurun_out/pmc_stream_$mode.json $w $alg gpurun_out/pmc_stream_${TAG}_$mode.json > /dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/pmc_stream_${TAG}_$mode.json'))
print('$mode', d['workload'], 'traffic/alg', round(d['traffic_over_algorithmic'],3), {k: round((v['read_bytes']+v['write_bytes'])/1e9,3) for k,v in d['kernels'].items()})"
done
