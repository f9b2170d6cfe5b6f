#!/bin/bash
# SQ counter passes over the config-4 stream bench, one rocprofv3 --pmc run per
# counter group, summarised per stream kernel into gpurun_out/sq_stream.txt.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
A="python3 tools/stream_bench.py --reps 1 $*"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/ss1 -o run -- $A > $R/gpurun_out/ss1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/ss2 -o run -- $A > $R/gpurun_out/ss2.log 2>&1
python3 - <<'PY' > $R/gpurun_out/sq_stream.txt
import csv, glob, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/ss*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        for key in ('stream_walk_kernel', 'stream_decode_wide_kernel', 'stream_params_kernel', 'rx_kernel', 'cfo_kernel', 'stream_decode_kernel', 'stream_sync_kernel', 'rx_stream2_kernel', 'compact_kernel'):
            if key in k:
                tmpl = k[k.find(key):k.find('>') + 1]
                acc[(tmpl, r['Counter_Name'])].append(float(r['Counter_Value']))
for (kern, ctr), vals in sorted(acc.items()):
    print(f"{kern:40s} {ctr:28s} n={len(vals)} mean={sum(vals)/len(vals):.5g}")
PY
