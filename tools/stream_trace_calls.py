#!/usr/bin/env python3
"""stream_trace_calls.py — per-call kernel times of bench.py's stream legs
from a rocprofv3 --kernel-trace CSV of bench.py --stream-pipeline 1: for
each call (walker, compaction, decode), the kernels' durations and the launch
gaps; means over the last N calls of each leg (f64, int16).

  python tools/stream_trace_calls.py run_kernel_trace.csv [N] > out.json
"""
import csv
import json
import sys


def main():
    path, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10
    rows = [r for r in csv.DictReader(open(path))
            if any(k in r["Kernel_Name"] for k in ("stream_walk_kernel", "compact_kernel", "resolve_kernel",
                                                   "stream_decode_kernel", "stream_decode_wide_kernel"))]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    calls = []
    for i in range(len(rows) - 2):
        a, b, c = rows[i:i + 3]
        if "stream_walk" in a["Kernel_Name"] and ("compact" in b["Kernel_Name"] or "resolve" in b["Kernel_Name"]) \
                and "decode" in c["Kernel_Name"]:
            t = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in (a, b, c)]
            wide = "wide" in c["Kernel_Name"]
            i16 = ("<true>" in c["Kernel_Name"]) or ("true>" in c["Kernel_Name"].split("(")[0])
            calls.append({"i16": i16, "leg": ("B" if wide else "") + ("int16" if i16 else "f64"),
                          "walk_us": (t[0][1] - t[0][0]) / 1e3,
                          "compact_us": (t[1][1] - t[1][0]) / 1e3, "decode_us": (t[2][1] - t[2][0]) / 1e3,
                          "gap1_us": (t[1][0] - t[0][1]) / 1e3, "gap2_us": (t[2][0] - t[1][1]) / 1e3,
                          "span_us": (t[2][1] - t[0][0]) / 1e3, "walk_start": t[0][0], "decode_end": t[2][1]})
    for c0, c1 in zip(calls, calls[1:]):  # decode end -> next call's walk start (host between calls)
        c0["gap_next_us"] = (c1["walk_start"] - c0["decode_end"]) / 1e3
    out = {"source": path, "note": "trace of bench.py --stream-pipeline 1 (serial calls); mean over each "
                                   "leg's last n calls"}
    for leg in ("f64", "int16", "Bf64", "Bint16"):
        cs = [c for c in calls if c["leg"] == leg and c["gap1_us"] >= 0 and c["gap2_us"] >= 0]
        cs = [c for c in cs if "gap_next_us" in c and 0 <= c["gap_next_us"] < 5000][-n:]
        if not cs:
            continue
        m = lambda k: round(sum(c[k] for c in cs) / len(cs), 1)
        out[leg] = {"calls": len(cs), **{k: m(k) for k in ("walk_us", "compact_us", "decode_us", "gap1_us",
                                                          "gap2_us", "span_us", "gap_next_us")},
                    "walk_plus_decode_us": round(m("walk_us") + m("decode_us"), 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
