#!/bin/bash
# stream tests, head/new A/B of the stream bench, then the phase-clock build
export TMPDIR=/tmp
bash tools/stream_ab.sh || exit 1
OFDM_MI355X_LIB=exp/libofdm_wprof.so timeout -k 10 200 python tools/walk_prof.py > gpurun_out/wprof.txt 2>&1
