# Development GPU pass: gpu parity tests, kernel micro-bench (configs B,C incl.
# alternating tx->rx pairs) and the driver bench without the CPU baseline.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
timeout -k 10 200 python tools/kbench.py --configs ${KB_CONFIGS:-B,C} --alt > gpurun_out/kbench.jsonl 2> gpurun_out/kbench.err || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
