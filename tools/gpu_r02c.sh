#!/bin/bash
# round 2 checkpoint: full GPU suite + smoke on the current code, then the
# measurement artefacts (kernel trace/stats of the bench, rx/tx PMC traffic,
# stream PMC traffic, rx SQ counters) and the default bench line.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
W=config2_B_N2048_D1024_P32_cp512_QPSK_8192frames_x8sym_per_gpu
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02c_gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02c_smoke.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stats -o run -- python3 bench.py --no-cpu-baseline --no-stream > gpurun_out/prof_stats.log 2>&1 || exit 1
python3 tools/trace_timed.py gpurun_out/prof_stats/run_kernel_trace.csv 20 gpurun_out/trace_timed.json > /dev/null || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stream > gpurun_out/prof_fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stream > gpurun_out/prof_write.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/prof_fetch/run_counter_collection.csv gpurun_out/prof_write/run_counter_collection.csv "rx_kernel<11" $W gpurun_out/pmc_rx.json 3238002688 > /dev/null || exit 1
python3 tools/pmc_traffic.py gpurun_out/prof_fetch/run_counter_collection.csv gpurun_out/prof_write/run_counter_collection.csv "tx_kernel<11" $W gpurun_out/pmc_tx.json 2700083200 > /dev/null || exit 1
bash tools/pmc_stream.sh || exit 1
SQ_CONFIG=B bash tools/sq_counters.sh || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r02c_bench.json 2> gpurun_out/r02c_bench.err
