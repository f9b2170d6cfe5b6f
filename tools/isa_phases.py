#!/usr/bin/env python3
"""Annotated-ISA instruction count per phase of a kernel.

Compiles a source with -DOFDM_PHASE_MARKS (OFDM_PHASE(name) emits an
assembler comment where each phase starts, ofdm_fft.hpp), takes the kernel's
gfx950 assembly and counts its instructions per phase and class (VALU, of
which FP64 / packed FP32 / SGPR-spill lane moves; SALU; LDS; VMEM; branches),
split by loop depth (the compiler's "Loop: Header ... Depth=d" block notes).
Straight-line code (unrolled symbols, transforms) counts what a wave
executes; code at depth > 0 runs once per trip of its loop.

  python3 tools/isa_phases.py c-ofdm_amd/csrc/ofdm_sync.hip stream_decode_kernelILb0E [--json out]
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def compile_asm(src: str) -> str:
    d = tempfile.mkdtemp()
    out = os.path.join(d, "k.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                    "-munsafe-fp-atomics", "-DOFDM_PHASE_MARKS", "-I" + os.path.join(ROOT, "include"),
                    "--cuda-device-only", "-S", "-o", out, src], check=True, stderr=subprocess.DEVNULL)
    return open(out).read()


def classify(op: str) -> list:
    c = []
    if op.startswith("v_"):
        c.append("valu")
        if "f64" in op:
            c.append("valu_f64")
        if op.startswith("v_pk_"):
            c.append("valu_pk")
        if op in ("v_readlane_b32", "v_writelane_b32"):
            c.append("valu_lane")
        if op.startswith(("v_sin", "v_cos", "v_rcp", "v_rsq", "v_sqrt", "v_log", "v_exp", "v_div", "v_frexp",
                          "v_ldexp", "v_trig", "v_fract")):
            c.append("valu_transc")
    elif op.startswith("s_"):
        c.append("branch" if op.startswith(("s_cbranch", "s_branch")) else "salu")
    elif op.startswith("ds_"):
        c.append("lds")
    elif op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        c.append("vmem")
    else:
        c.append("other")
    return c


def phases(asm: str, kernel_substr: str) -> dict:
    m = re.search(r"^(\w*" + re.escape(kernel_substr) + r"\w*):", asm, re.M)
    if not m:
        raise SystemExit(f"kernel matching {kernel_substr!r} not found")
    name = m.group(1)
    i = m.end()
    j = asm.find(".Lfunc_end", i)
    phase, depth = "prologue", 0
    acc = collections.defaultdict(collections.Counter)
    order = []
    for ln in asm[i:j].splitlines():
        s = ln.strip()
        pm = re.search(r"OFDM_PHASE (\w+)", s)
        if pm:
            phase = pm.group(1)
            continue
        bm = re.match(r"^\.LBB\d+_\d+:(.*)", s)
        if bm:
            dm = re.search(r"Depth=(\d+)", bm.group(1))
            depth = int(dm.group(1)) if dm else 0
            continue
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            continue
        op = s.split()[0]
        key = f"{phase}@d{depth}"
        if key not in acc:
            order.append(key)
        acc[key]["all"] += 1
        for c in classify(op):
            acc[key][c] += 1
    return {"kernel": name, "phases": [{"phase": k, **dict(acc[k])} for k in order]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("kernel")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    res = phases(compile_asm(os.path.abspath(a.src)), a.kernel)
    cols = ("all", "valu", "valu_f64", "valu_pk", "valu_transc", "valu_lane", "salu", "lds", "vmem", "branch")
    print(res["kernel"])
    print(f"{'phase@loopdepth':32s}" + "".join(f"{c:>12s}" for c in cols))
    tot = collections.Counter()
    for p in res["phases"]:
        print(f"{p['phase']:32s}" + "".join(f"{p.get(c, 0):12d}" for c in cols))
        for c in cols:
            tot[c] += p.get(c, 0)
    print(f"{'TOTAL (static)':32s}" + "".join(f"{tot[c]:12d}" for c in cols))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    sys.exit(main())
