export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "demod_read or copy_kernel" > gpurun_out/adhoc_tests.log 2>&1; rc=$?; tail -15 gpurun_out/adhoc_tests.log; exit $rc
