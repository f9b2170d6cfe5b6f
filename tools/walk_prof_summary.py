#!/usr/bin/env python3
"""walk_prof_summary.py — per-call summary of the stream walker timelines that
OFDM_WALK_PROF=<file> writes (one JSON line per ofdm_rx_stream* call; per
chunk: start, first frame past the core end, end in wall_clock64 ticks of
100 MHz, frames past the core end, look-back polls that waited, workgroup,
XCC, frames located).

  python tools/walk_prof_summary.py prof.jsonl [calls to skip] > summary.json
"""
import json
import sys

import numpy as np

TICK_US = 0.01  # wall_clock64: 100 MHz


def summarise(d):
    a = np.array(d["chunks"], dtype=np.int64)
    t0, tc, te, ext, waits, blk, xcc, nrec = a.T[:8]
    base = t0.min()
    start, end = (t0 - base) * TICK_US, (te - base) * TICK_US
    dur = end - start
    core = np.where(tc > 0, (tc - t0) * TICK_US, dur)
    span = end.max()
    late = np.argsort(end)[-8:][::-1]
    q = lambda v: [round(float(x), 1) for x in np.percentile(v, [0, 10, 50, 90, 99, 100])]
    out = {
        "nchunks": d["nchunks"], "chunk": d["chunk"], "lookback": d["lookback"], "grid": d["grid"],
        "kernel_span_us": round(float(span), 1),
        "walker_us_pct_0_10_50_90_99_100": q(dur), "walker_mean_us": round(float(dur.mean()), 1),
        "start_us_pct": q(start), "core_us_pct": q(core),
        "ext_frames_hist": {int(k): int(v) for k, v in zip(*np.unique(ext, return_counts=True))},
        "waits_total": int(waits.sum()), "chunks_that_waited": int((waits > 0).sum()),
        "nrec_mean": round(float(nrec.mean()), 2),
        "tail_chunks": [{"chunk": int(c), "start_us": round(float(start[c]), 1), "end_us": round(float(end[c]), 1),
                         "core_us": round(float(core[c]), 1), "ext_frames": int(ext[c]), "waits": int(waits[c]),
                         "nrec": int(nrec[c]), "xcc": int(xcc[c]), "block": int(blk[c])} for c in late],
        "end_by_xcc_max_us": {int(x): round(float(end[xcc == x].max()), 1) for x in np.unique(xcc)},
    }
    if a.shape[1] >= 13:  # phase split: T2 scans, preamble searches (ticks), scan steps, FP64 evaluations, searches
        t2, pre, steps, f64, nsearch = a.T[8:13]
        nf = max(int(nsearch.sum()), 1)
        out["phases"] = {
            "t2_scan_us_per_walker": round(float(t2.mean()) * TICK_US, 1),
            "preamble_us_per_walker": round(float(pre.mean()) * TICK_US, 1),
            "other_us_per_walker": round(float(dur.mean() - (t2.mean() + pre.mean()) * TICK_US), 1),
            "t2_scan_us_per_search": round(float(t2.sum()) * TICK_US / nf, 2),
            "preamble_us_per_search": round(float(pre.sum()) * TICK_US / nf, 2),
            "scan_steps_per_search": round(float(steps.sum()) / nf, 2),
            "fp64_evals_per_search": round(float(f64.sum()) / nf, 3),
            "searches_per_walker": round(float(nsearch.mean()), 2),
        }
    return out


def main():
    path = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    rows = [json.loads(l) for l in open(path) if l.strip()]
    out = [summarise(d) for d in rows[skip:]]
    print(json.dumps({"source": path, "calls": out}, indent=1))


if __name__ == "__main__":
    main()
