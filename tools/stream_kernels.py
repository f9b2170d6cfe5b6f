#!/usr/bin/env python3
"""stream_kernels.py — per-kernel mean durations of the stream pipeline, one
workload per rocprofv3 --kernel-trace CSV of tools/stream_bench.py, over the
last N launches of each kernel (warm clocks). Writes the JSON bench.py reads
(load_stream_kernels: the decode's own time for its compute record).

  python tools/stream_kernels.py out.json N workload=run_kernel_trace.csv [...]
"""
import csv
import json
import sys

KINDS = {"walker_us": ("stream_walk_kernel",), "resolve_us": ("resolve_kernel", "compact_kernel"),
         "decode_us": ("stream_decode_kernel", "stream_decode_wide_kernel")}


def summarise(path, n):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    out = {}
    for key, names in KINDS.items():
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
             if any(k in r["Kernel_Name"] for k in names)]
        if d:
            d = d[-n:]
            out[key] = round(sum(d) / len(d), 2)
            out[key.replace("_us", "_launches")] = len(d)
    walks = [r for r in rows if "stream_walk_kernel" in r["Kernel_Name"]]
    decs = [r for r in rows if any(k in r["Kernel_Name"] for k in KINDS["decode_us"])]
    if len(walks) >= 2 and len(decs) >= 2:  # call span: walker start -> decode end, last n calls
        spans = [(int(dd["End_Timestamp"]) - int(w["Start_Timestamp"])) / 1e3 for w, dd in zip(walks, decs)][-n:]
        out["call_span_us"] = round(sum(spans) / len(spans), 2)
    out["trace"] = path
    return out


def main():
    dst, n = sys.argv[1], int(sys.argv[2])
    res = {"note": "mean kernel durations over the last N launches of each stream kernel (rocprofv3 "
                   "--kernel-trace of tools/stream_bench.py, one workload per trace)", "N": n, "workloads": {}}
    for arg in sys.argv[3:]:
        w, path = arg.split("=", 1)
        res["workloads"][w] = summarise(path, n)
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
