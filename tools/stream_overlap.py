#!/usr/bin/env python3
"""stream_overlap.py — how the stream kernels of concurrent calls overlap,
from a rocprofv3 --kernel-trace CSV (e.g. of bench.py --stream-pipeline 2):
for every walker and decode kernel, its duration and the share of it that
ran beside a kernel of the other kind; means split by overlapped / alone.

  python tools/stream_overlap.py run_kernel_trace.csv [last N kernels of each kind] > out.json
"""
import csv
import json
import sys

import numpy as np


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows = list(csv.DictReader(open(path)))
    kinds = {"walk": "stream_walk_kernel", "decode": "stream_decode", "resolve": "resolve_kernel"}
    ks = {k: sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in rows
                     if v in r["Kernel_Name"]), key=lambda x: x[0]) for k, v in kinds.items()}

    def overlap(a, others):
        s, e = a[0], a[1]
        return sum(max(0, min(e, o[1]) - max(s, o[0])) for o in others) / max(e - s, 1)

    out = {"source": path}
    for k, other in (("walk", "decode"), ("decode", "walk")):
        xs = ks[k][-n:]
        d = np.array([(x[1] - x[0]) / 1e3 for x in xs])
        ov = np.array([overlap(x, ks[other]) for x in xs])
        out[k] = {"n": len(xs), "mean_us": round(float(d.mean()), 1) if len(d) else None,
                  "mean_us_overlapped": round(float(d[ov > 0.5].mean()), 1) if (ov > 0.5).any() else None,
                  "mean_us_alone": round(float(d[ov < 0.1].mean()), 1) if (ov < 0.1).any() else None,
                  "overlap_share_mean": round(float(ov.mean()), 3) if len(ov) else None}
    ev = sorted([x for k in ("walk", "decode", "resolve") for x in ks[k][-n:]])
    if ev:
        span = (max(x[1] for x in ev) - min(x[0] for x in ev)) / 1e3
        out["span_us_last_kernels"] = round(span, 1)
        out["calls_in_span"] = len(ks["walk"][-n:])
        out["us_per_call"] = round(span / max(len(ks["walk"][-n:]), 1), 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
