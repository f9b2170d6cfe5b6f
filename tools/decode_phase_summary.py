#!/usr/bin/env python3
"""Per-segment executed instructions of the fused stream decode from the SQ
passes of tools/decode_phase_counts.sh (<prefix>_stop{1..5,0}/run_counter_collection.csv):
counts per located frame and per wave, each segment the difference of two
consecutive stop points (stop 0 = the product kernel, the full decode)."""
import csv
import json
import sys
from collections import defaultdict

SEGMENTS = [(1, "pilot_freq_sinh (5 x 128-point transforms, radix-5 combine, window argmax)"),
            (2, "rest of the sync stage: preamble ramp + transform + phase, unwrap, LS line (wave 0) | "
                "message CP sums (wave 1); ramp table"),
            (3, "8 message symbols: ramp start, loads, ramp, 512-point transform, pilot / carrier gathers"),
            (4, "channel line (sincos), phys, gains"),
            (5, "emit: gain and channel products, constellation store, decisions"),
            (0, "byte packing (to the full kernel)")]


def load(prefix: str, k: int) -> dict:
    acc = defaultdict(float)
    n = 0
    for r in csv.DictReader(open(f"{prefix}_stop{k}/run_counter_collection.csv")):
        if "stream_decode_kernel" not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        n += 1
    return dict(acc)


def main():
    prefix = sys.argv[1]
    stops = {k: load(prefix, k) for k, _ in SEGMENTS}
    full = stops[0]
    waves = full["SQ_WAVES"]
    frames = waves / 2  # one 2-wave workgroup per located frame
    out = {"frames_per_call": frames, "segments": []}
    prev = {}
    for k, name in SEGMENTS:
        cur = stops[k]
        seg = {c: (cur.get(c, 0.0) - prev.get(c, 0.0)) for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
                                                                   "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR")}
        out["segments"].append({"stop": k, "segment": name,
                                **{c.replace("SQ_INSTS_", "").lower() + "_per_wave_per_frame": round(v / waves, 1)
                                   for c, v in seg.items()}})
        prev = cur
    out["total_valu_per_wave_per_frame"] = round(full["SQ_INSTS_VALU"] / waves, 1)
    out["valu_busy_of_wave_cycles"] = full["SQ_ACTIVE_INST_VALU"] / full["SQ_WAVE_CYCLES"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
