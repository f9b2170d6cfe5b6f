#!/bin/bash
# VGPR / SGPR / LDS / scratch of every kernel in a source file (gfx950), from
# the compiler's own metadata: tools/kernel_resources.sh c-ofdm_amd/csrc/ofdm_sync.hip [regex]
set -e
SRC=$(realpath "$1"); PAT=${2:-.}
D=$(mktemp -d)
cd "$D" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics \
    -I"$(dirname "$SRC")/../../include" --cuda-device-only -S -o k.s "$SRC" 2>/dev/null
python3 - "$PAT" <<'PY'
import re, sys
s = open("k.s").read()
for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", s, re.S):
    name, body = m.group(1), m.group(2)
    if not re.search(sys.argv[1], name):
        continue
    g = lambda k: (re.search(r"\." + k + r"\s+(\d+)", body) or [None, "?"])[1]
    print(f"{name[:90]:90s} vgpr_next={g('amdhsa_next_free_vgpr')} agpr_off={g('amdhsa_accum_offset')} "
          f"sgpr_next={g('amdhsa_next_free_sgpr')} lds={g('amdhsa_group_segment_fixed_size')} "
          f"scratch={g('amdhsa_private_segment_fixed_size')}")
PY
rm -rf "$D"
