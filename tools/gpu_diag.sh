# diagnostic GPU pass: kernel micro-bench + counter inventory + SQ counters on kbench (config B)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python tools/kbench.py --configs B,C,D > gpurun_out/kbench.jsonl 2> gpurun_out/kbench.err && \
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/prof_sq1 -o run -- python3 tools/kbench.py --configs B --reps 2 > gpurun_out/prof_sq1.log 2>&1 ; \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/prof_sq2 -o run -- python3 tools/kbench.py --configs B --reps 2 > gpurun_out/prof_sq2.log 2>&1
