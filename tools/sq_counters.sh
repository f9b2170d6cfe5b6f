#!/bin/bash
# SQ counter passes over kbench (config ${SQ_CONFIG:-B}), one rocprofv3 --pmc
# run per counter group (no more than 8 SQ_ counters per pass), summarised per
# kernel into gpurun_out/sq_summary.txt.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
C=${SQ_CONFIG:-B}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/sq1 -o run -- python3 tools/kbench.py --configs $C --reps 2 > $R/gpurun_out/sq1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/sq2 -o run -- python3 tools/kbench.py --configs $C --reps 2 > $R/gpurun_out/sq2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD --output-format csv -d $R/gpurun_out/sq3 -o run -- python3 tools/kbench.py --configs $C --reps 2 > $R/gpurun_out/sq3.log 2>&1
python3 - <<'PY' > $R/gpurun_out/sq_summary.txt
import csv, glob, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/sq*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        for key in ('tx_kernel', 'rx_kernel'):
            if key in k:
                tmpl = k[k.find(key):k.find('>') + 1]
                acc[(tmpl, r['Counter_Name'])].append(float(r['Counter_Value']))
# sum over dimensions per dispatch is done by rocprofv3 rows (one row per dispatch x counter)
for (kern, ctr), vals in sorted(acc.items()):
    print(f"{kern:40s} {ctr:28s} n={len(vals)} mean={sum(vals)/len(vals):.5g}")
PY
