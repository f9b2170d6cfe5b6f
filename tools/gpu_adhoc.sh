export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python bench.py --gpus 4 --backend gloo --steps 5 --warmup 2 --no-cpu-baseline --stream-reps 3 --stream-warmup 2 --no-config3 > gpurun_out/gloo4.json 2> gpurun_out/gloo4.err; rc=$?
wc -l gpurun_out/gloo4.json
python3 -c "
import json;d=json.load(open('gpurun_out/gloo4.json'))
print('n_gpus', d['n_gpus'], 'value', d['value']/1e9, 'ms', d['ms_per_step'], 'ber', d.get('ber'))
for k in ('stream','stream_int16'):
    s=d[k]; print(k, s['value']/1e9, s['frames_found'], s['frames_error_free'], s['rewalks_per_call'], s.get('exchange_ms_per_call'))
"
exit $rc
