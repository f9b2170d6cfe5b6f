#!/usr/bin/env python3
"""pmc_stream_summary.py — HBM bytes per config-4 stream call from the per-kernel
FETCH_SIZE / WRITE_SIZE means that tools/pmc_stream.sh collects (separate
rocprofv3 --pmc passes), in the form bench.py's stream leg reads
(profiles/pmc_stream_*.json: workload + hbm_bytes_per_call). Reads are taken
at 2 x FETCH_SIZE (the MI355X_MICROARCH.md gfx950 correction for 16-B
streaming reads; the rx kernel's exact algorithmic read confirms it), writes
at WRITE_SIZE.

  python tools/pmc_stream_summary.py gpurun_out/pmc_stream.json WORKLOAD ALG_BYTES OUT.json
"""
import json
import sys


def main():
    src, workload, alg, out = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
    d = json.load(open(src))
    per = {}
    tot = 0.0
    for k, v in d.items():
        if not isinstance(v, dict):
            continue
        r = 2.0 * v.get("FETCH_SIZE_kib", 0.0) * 1024
        w = v.get("WRITE_SIZE_kib", 0.0) * 1024
        per[k] = {"read_bytes": r, "write_bytes": w}
        tot += r + w
    res = {"workload": workload, "source": src, "kernels": per, "hbm_bytes_per_call": tot,
           "algorithmic_bytes_per_call": alg, "traffic_over_algorithmic": tot / alg,
           "correction": "read = 2 x FETCH_SIZE (gfx950 16-B streaming reads), write = WRITE_SIZE; "
                         "per-kernel means over the run's dispatches"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
