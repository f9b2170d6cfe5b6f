# SQ counter passes on the rx kernel (one rocprofv3 --pmc pass per group, --kernel-trace-free).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/sq
rocprofv3 --list-avail > $R/gpurun_out/sq/avail.txt 2>&1 || true
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
        if "rx_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(f"{k:28s} n={len(v)} mean={sum(v)/len(v):.6g}")
PY
