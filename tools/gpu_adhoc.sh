#!/bin/bash
# scratch slot for one-off GPU commands (overwritten per experiment)
# current: ingest + bench-record tests, then the two-context overlap trace
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
TAG=${1:-r06c}
timeout -k 10 900 python -u -m pytest tests/test_gpu_stream_ingest.py tests/test_gpu_multigpu_app.py tests/test_bench_gpu.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/${TAG}_tests.log | tail -20
bash tools/gpu_stream_overlap.sh && cp gpurun_out/stream_overlap.json gpurun_out/${TAG}_stream_overlap.json
