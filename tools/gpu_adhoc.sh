# Scratch slot for one-off GPU commands (`gpurun -- bash tools/gpu_adhoc.sh`);
# its content changes with the experiment at hand and is not part of any flow.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/gpu_stream_check.sh r03p || exit 1
bash tools/pmc_stream.sh || exit 1
SUF=_i16 bash tools/pmc_stream.sh --i16 || exit 1
for suf in "" _i16; do
  alg=$(grep -h "^{" gpurun_out/pmcs_fetch$suf.log | tail -1 | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['roofline']['algorithmic_bytes'])")
  wl=$(grep -h "^{" gpurun_out/pmcs_fetch$suf.log | tail -1 | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['workload'])")
  python3 tools/pmc_stream_summary.py gpurun_out/pmc_stream$suf.json $wl $alg gpurun_out/pmc_stream_r03b$suf.json
  grep -o '"traffic_over_algorithmic": [0-9.]*' gpurun_out/pmc_stream_r03b$suf.json
done
timeout -k 10 900 python bench.py --gpus 4 --backend gloo --steps 3 --warmup 1 --no-cpu-baseline --stream-reps 3 --stream-warmup 2 --no-config3 > gpurun_out/gloo4.json 2> gpurun_out/gloo4.err || exit 1
python3 -c "
import json;d=json.load(open('gpurun_out/gloo4.json'))
for k in ('stream','stream_int16'):
    s=d[k]; print(k, s['n_gpus'], s['frames_found'], s['rewalks_per_call'])"
