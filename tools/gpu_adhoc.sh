export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/stt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config3 --stream-pipeline 1 > gpurun_out/stt.log 2>&1 || { tail gpurun_out/stt.log; exit 1; }
python3 tools/stream_trace_calls.py gpurun_out/stt/run_kernel_trace.csv 10
