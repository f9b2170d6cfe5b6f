export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dropin_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03e_dropin.log 2>&1; tail -15 gpurun_out/r03e_dropin.log
timeout -k 10 300 python tools/dropin_rx_timing.py --frames 200 > gpurun_out/r03e_dropin_timing.json 2> gpurun_out/r03e_dropin_timing.err; cat gpurun_out/r03e_dropin_timing.json; tail -3 gpurun_out/r03e_dropin_timing.err
LIBS="abtest/libofdm_base.so product" TAG=r03e bash tools/stream_ab.sh
