# One GPU pass producing the round's measurement artefacts (copied into profiles/ afterwards):
#   gpurun_out/prof_stats   rocprofv3 --kernel-trace --stats of bench.py (headline leg only: default steps/warmup)
#   gpurun_out/trace_timed.json  the same trace's rx/tx averages over the 20 timed launches
#   gpurun_out/prof_fetch   --pmc FETCH_SIZE   (separate pass, as MI355X_MICROARCH.md prescribes)
#   gpurun_out/prof_write   --pmc WRITE_SIZE
#   gpurun_out/pmc_rx.json  HBM bytes per rx launch (tools/pmc_traffic.py)
#   gpurun_out/bench.json   the bench line
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
W=config2_B_N2048_D1024_P32_cp512_QPSK_8192frames_x8sym_per_gpu
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stats -o run -- python3 bench.py --no-cpu-baseline --no-stream --no-config3 > gpurun_out/prof_stats.log 2>&1 && \
python3 tools/trace_timed.py gpurun_out/prof_stats/run_kernel_trace.csv 20 gpurun_out/trace_timed.json > /dev/null && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stream --no-config3 > gpurun_out/prof_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stream --no-config3 > gpurun_out/prof_write.log 2>&1 && \
python3 tools/pmc_traffic.py gpurun_out/prof_fetch/run_counter_collection.csv gpurun_out/prof_write/run_counter_collection.csv "rx_kernel<11" $W gpurun_out/pmc_rx.json 3238002688 > /dev/null && \
python3 tools/pmc_traffic.py gpurun_out/prof_fetch/run_counter_collection.csv gpurun_out/prof_write/run_counter_collection.csv "tx_kernel<11" $W gpurun_out/pmc_tx.json 2700083200 > /dev/null && \
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
