export TMPDIR=/tmp
mkdir -p gpurun_out
OFDM_MI355X_LIB=$PWD/abtest/libofdm_rprof.so timeout -k 10 200 python tools/rx_prof.py > gpurun_out/r02_rx_prof.json 2> gpurun_out/r02_rx_prof.err || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_decision_boundary.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_parity.log 2>&1 || exit 1
bash tools/ab_run.sh emit
