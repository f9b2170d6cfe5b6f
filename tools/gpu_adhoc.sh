export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/gpu_profile_round.sh || exit 1
bash tools/pmc_stream.sh || exit 1
SUF=_i16 bash tools/pmc_stream.sh --i16 || exit 1
for suf in "" _i16; do
  alg=$(grep -h "^{" gpurun_out/pmcs_fetch$suf.log | tail -1 | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['roofline']['algorithmic_bytes'])")
  wl=$(grep -h "^{" gpurun_out/pmcs_fetch$suf.log | tail -1 | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['workload'])")
  python3 tools/pmc_stream_summary.py gpurun_out/pmc_stream$suf.json $wl $alg gpurun_out/pmc_stream_r03$suf.json
  grep traffic_over gpurun_out/pmc_stream_r03$suf.json
done
python3 -c "
import json;d=json.load(open('gpurun_out/bench.json'))
print('value', d['value']/1e9, 'rx frac', d['roofline']['frac'], 'traffic', d['roofline']['traffic'], 'stream', d['stream']['value']/1e9, d['stream_int16']['value']/1e9)"
cat gpurun_out/pmc_rx.json | head -20
