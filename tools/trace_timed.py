#!/usr/bin/env python3
"""trace_timed.py — per-kernel launch durations from a rocprofv3 kernel trace,
split into the warmup launches and the last K (the bench's timed steps), so the
profile can be compared with bench.py's live HIP-event averages.

  python tools/trace_timed.py run_kernel_trace.csv STEPS out.json
"""
import csv
import json
import sys


def main():
    path, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    rows = list(csv.DictReader(open(path)))
    res = {"source": path, "timed_launches": steps, "kernels": {}}
    for key in ("rx_kernel", "tx_kernel"):
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows
             if key in r["Kernel_Name"] and int(r["Grid_Size_X"]) > 1024]
        if not d:
            continue
        timed = d[-steps:]
        res["kernels"][key] = {
            "name": next(r["Kernel_Name"] for r in rows if key in r["Kernel_Name"] and int(r["Grid_Size_X"]) > 1024),
            "launches": len(d),
            "avg_all_ms": sum(d) / len(d),
            "avg_timed_ms": sum(timed) / len(timed),
            "first_ms": d[0], "last_ms": d[-1],
        }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
