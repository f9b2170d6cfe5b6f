#!/bin/bash
# Full GPU pass: every -m gpu test, smoke(), the default bench line. Output: gpurun_out/${TAG}_*
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-full}
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 1; }
grep smoke gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/${TAG}_bench.json'))
print('value', d['value']/1e9, 'ms', d['ms_per_step'], 'rx frac', d['roofline']['frac'], 'rx ms', d['roofline']['avg_launch_ms'], 'tx ms', d['tx_avg_launch_ms'])
for k in ('stream','stream_int16'):
    s=d[k]; print(k, s['value']/1e9, s['ms_per_call'], s['roofline']['frac'], s['frames_found'], s['frames_error_free'], s['rewalks_per_call'], (s['cpu_baseline'] or {}).get('value'))
    print('  compute frac', s['compute']['frac'], s['compute']['kernels_us'])
b=d.get('stream_B')
if b: print('stream_B', b['value']/1e9, b['ms_per_call'], b['frames_found'], b['frames_error_free'], 'staged', b['staged']['value']/1e9, b['staged']['ms_per_call'], 'speedup', b['staged']['fused_speedup_per_sample'])
g=d.get('stream_ingest')
if g: print('stream_ingest', g.get('value', 0)/1e9, g.get('ms_per_stream'), 'pcie', g.get('pcie_h2d'), 'frac', g.get('frac_of_pcie_ceiling'), 'equal', g.get('outputs_equal_device_resident_call'))
c=d['config3']; print('config3', c['value']/1e9, c['roofline']['frac'])
"
