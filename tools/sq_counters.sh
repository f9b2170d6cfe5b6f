# SQ counter passes on the rx kernel (one rocprofv3 --pmc pass per group, --kernel-trace-free).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/sq
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY" \
           "SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/sq/p$i -o run -- python3 tools/rx_only.py 8192 2 > $R/gpurun_out/sq/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $R/gpurun_out/sq/p$i.log; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/sq/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        for kn in ("rx_kernel", "tx_kernel"):
            if kn in r["Kernel_Name"] and int(r["Grid_Size"]) > 100000:
                acc[(kn, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (kn, k), v in sorted(acc.items()):
    print(f"{kn:10s} {k:28s} n={len(v)} mean={sum(v)/len(v):.6g}")
PY
