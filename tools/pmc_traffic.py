#!/usr/bin/env python3
"""pmc_traffic.py — HBM bytes per launch of one kernel from two separate
rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE), corrected as
MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE (KiB) reports half the bytes
of a wide coalesced streaming read on gfx950 -> x2; WRITE_SIZE (KiB) is exact
for 16-B-per-lane streaming stores. Only dispatches with the kernel's largest
grid are used (skips e.g. the 1-symbol preamble synthesis at ctx creation).

  python tools/pmc_traffic.py FETCH.csv WRITE.csv KERNEL_SUBSTR WORKLOAD OUT.json [ALG_BYTES]
"""
import csv
import json
import sys


def per_launch(path, kernel, counter):
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    if not rows:
        raise SystemExit(f"no {counter} rows for {kernel} in {path}")
    gmax = max(int(r["Grid_Size"]) for r in rows)
    vals = [float(r["Counter_Value"]) for r in rows if int(r["Grid_Size"]) == gmax]
    return sum(vals) / len(vals), len(vals)


def main():
    fetch_csv, write_csv, kernel, workload, out = sys.argv[1:6]
    alg = float(sys.argv[6]) if len(sys.argv) > 6 else None
    f_kib, nf = per_launch(fetch_csv, kernel, "FETCH_SIZE")
    w_kib, nw = per_launch(write_csv, kernel, "WRITE_SIZE")
    read_b = 2.0 * f_kib * 1024
    write_b = w_kib * 1024
    d = {"workload": workload, "kernel": kernel, "dispatches": [nf, nw],
         "fetch_size_kib": f_kib, "write_size_kib": w_kib,
         "hbm_read_bytes_per_launch": read_b, "hbm_write_bytes_per_launch": write_b,
         "hbm_bytes_per_launch": read_b + write_b,
         "correction": "read = 2 x FETCH_SIZE (gfx950 16-B streaming reads), write = WRITE_SIZE"}
    if alg:
        d["algorithmic_bytes_per_launch"] = alg
        d["traffic_over_algorithmic"] = (read_b + write_b) / alg
    with open(out, "w") as fh:
        json.dump(d, fh, indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
