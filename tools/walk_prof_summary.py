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
    if a.shape[1] >= 14:  # HW_ID: the CU each walker ran on; per CU, its walkers' work against its finish
        hw = a[:, 13]
        cu = (xcc << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)
        keys, inv = np.unique(cu, return_inverse=True)
        fin = np.zeros(len(keys))
        busy = np.zeros(len(keys))
        first = np.full(len(keys), 1e30)
        cnt = np.zeros(len(keys), np.int64)
        np.maximum.at(fin, inv, end)
        np.minimum.at(first, inv, end)
        np.add.at(busy, inv, dur)
        np.add.at(cnt, inv, 1)
        simd = (hw >> 4) & 3
        out["cus"] = {
            "count": int(len(keys)), "walkers_per_cu": {int(k): int(v) for k, v in zip(*np.unique(cnt, return_counts=True))},
            "finish_us_pct": q(fin), "first_walker_end_us_pct": q(first),
            "walker_us_sum_per_cu_pct": q(busy),
            "walkers_per_simd": {int(k): int(v) for k, v in zip(*np.unique(simd, return_counts=True))},
            # how much of the span the CU had all its walkers running: mean end / finish
            "mean_end_over_finish": round(float(np.mean([end[inv == i].mean() / fin[i] for i in range(len(keys))])), 3),
            "corr_finish_vs_frames": round(float(np.corrcoef(fin, np.bincount(inv, weights=nrec))[0, 1]), 3),
        }
        # walker duration by its dispatch rank on its CU (block order)
        rank = np.zeros(len(a), np.int64)
        for i in range(len(keys)):
            m = np.nonzero(inv == i)[0]
            rank[m[np.argsort(blk[m])]] = np.arange(len(m))
        out["cus"]["walker_us_by_dispatch_rank"] = [round(float(dur[rank == r].mean()), 1) for r in range(int(rank.max()) + 1)]
    return out


def main():
    path = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    rows = [json.loads(l) for l in open(path) if l.strip()]
    out = [summarise(d) for d in rows[skip:]]
    print(json.dumps({"source": path, "calls": out}, indent=1))


if __name__ == "__main__":
    main()
