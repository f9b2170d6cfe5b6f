#!/bin/bash
# Build an experiment variant of the modem library with extra compile flags:
#   tools/build_variant.sh NAME "-DOFDM_RX_NOFFT ..."  ->  abtest/libofdm_NAME.so
# (timing experiments only; the product is c-ofdm_amd/lib/libofdm_mi355x.so).
# abtest/ travels to the GPU box (git-ignored); delete it after an experiment.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
FLAGS="$*"
SRC=${SRC:-$R}  # source tree (e.g. an exported older commit)
B=$R/abtest/build_$NAME
mkdir -p $B $R/abtest
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -munsafe-fp-atomics -I$SRC/include $FLAGS"
$H -c $SRC/c-ofdm_amd/csrc/ofdm_kernels.hip -o $B/k.o &
$H -c $SRC/c-ofdm_amd/csrc/ofdm_sync.hip -o $B/s.o &
[ -f $SRC/c-ofdm_amd/csrc/ofdm_stream_wide.hip ] && $H -c $SRC/c-ofdm_amd/csrc/ofdm_stream_wide.hip -o $B/w.o &
$H -x hip -c $SRC/c-ofdm_amd/csrc/ofdm_capi.cpp -o $B/c.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $R/abtest/libofdm_$NAME.so $B/*.o
rm -rf $B
echo built abtest/libofdm_$NAME.so
