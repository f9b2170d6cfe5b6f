export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sync.py tests/test_dropin_gpu.py > gpurun_out/adhoc_tests.log 2>&1; rc=$?; tail -3 gpurun_out/adhoc_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u tools/dropin_rx_timing.py --frames 200 > gpurun_out/adhoc_dropin.log 2>&1; rc=$?; tail -c 600 gpurun_out/adhoc_dropin.log; exit $rc
