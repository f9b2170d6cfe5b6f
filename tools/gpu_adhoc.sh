# Scratch slot for one-off GPU commands (`gpurun -- bash tools/gpu_adhoc.sh`);
# its content changes with the experiment at hand and is not part of any flow.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sync.py tests/test_dropin_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/wide_tests.log 2>&1 || { tail -60 gpurun_out/wide_tests.log; exit 1; }
tail -3 gpurun_out/wide_tests.log
timeout -k 10 300 python tools/chain_bench.py > gpurun_out/chain_bench.json 2> gpurun_out/chain_bench.err || { tail gpurun_out/chain_bench.err; exit 1; }
cat gpurun_out/chain_bench.json
timeout -k 10 300 python tools/dropin_rx_timing.py --frames 200 > gpurun_out/wide_dropin.json 2> gpurun_out/wide_dropin.err || { tail gpurun_out/wide_dropin.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/wide_dropin.json')); print(d['median_us'], d['frames_payload_exact'], d['stage_median_us'])"
