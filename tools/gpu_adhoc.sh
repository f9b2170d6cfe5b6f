#!/bin/bash
# scratch slot for one-off GPU commands (overwritten per experiment)
# current: walker int16 prefetch: stream parity, same-box A/B against the
# previous build, ingest chunk sweep
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
TAG=${1:-r06e}
timeout -k 10 900 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_stream_full.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
TAG=$TAG LIBS="product abtest/libofdm_nopf.so" bash tools/stream_ab.sh || exit 1
timeout -k 10 300 python3 tools/ingest_bench.py > gpurun_out/${TAG}_ingest.jsonl 2> gpurun_out/${TAG}_ingest.err || { tail gpurun_out/${TAG}_ingest.err; exit 1; }
cat gpurun_out/${TAG}_ingest.jsonl
