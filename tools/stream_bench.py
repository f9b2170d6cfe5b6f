#!/usr/bin/env python3
"""stream_bench.py — throughput of the streaming receiver.

The stream is bench.py's own (c-ofdm_amd/python/ofdm_synth.py StreamLayout +
stream_slice: full frames with counter-based payloads, 0..4096-sample gaps,
per-frame CFO U(-0.004, 0.004) cycles/sample, random phase, AWGN 20 dB), so
the two tools measure one workload. Two figures:
  - G_stream_samples_per_s / ms: calls enqueued back to back (the host
    returns once the walk is resolved and issues the next call while the
    decode drains), exactly bench.py's stream records;
  - isolated_call_ms: one call between two device synchronisations (latency,
    including launch and host round trips).
Stream samples consumed per second is the figure (~21.6 B per
stream sample algorithmic, ~370 G samples/s HBM roofline).

  python tools/stream_bench.py [--frames 16384] [--reps 10] [--i16] [--config B]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "c-ofdm_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402  (config dicts and geometry only)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16384)
    ap.add_argument("--config", choices=("D", "B", "C"), default="D",
                    help="frame geometry: D (config.txt, the fused decode), B (2048 carriers) or C (4096)")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=10, help="untimed calls first (clock ramp)")
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--i16", action="store_true", help="wire-format complex<int16> stream (x mult)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="contexts alternating on their own HIP streams (call k+1's walk overlaps call k's decode)")
    ap.add_argument("--walk-tuning", default="",
                    help="ofdm_set_walk_tuning fields, e.g. 'chunks_per_slot=2,halo_milli=1500,lookback=0'")
    ap.add_argument("--cpu-seconds", type=float, default=0.0,
                    help="also time the oracle's walk + decode on a prefix of the stream (~this many s)")
    args = ap.parse_args()
    import torch
    import ofdm_mi355x as M
    import ofdm_synth as Y
    from ofdm_synth import payload_bytes

    cfg = dict({"D": O.DEFAULT, "B": O.CONFIG_B, "C": O.CONFIG_C}[args.config])
    g = O.geometry(cfg)
    m = M.Modem(cfg, 0)
    tuning = {}
    if args.walk_tuning:
        kv = dict(item.split("=") for item in args.walk_tuning.split(","))
        tuning = {k: (float(v) if k == "t2_margin" else int(v)) for k, v in kv.items()}
        m.walk_tuning(**tuning)
    nf = args.frames
    dev = torch.device("cuda", 0)
    layout = Y.StreamLayout(cfg, nf)
    n = layout.n
    x = Y.stream_slice(m, layout, 0, n, dev, i16=args.i16)
    out = torch.empty((nf * g["bytes_per_frame"],), dtype=torch.uint8, device="cuda")
    cons = torch.empty((nf * g["npts"],), dtype=torch.complex128, device="cuda")
    pbs = torch.empty((nf,), dtype=torch.int64, device="cuda")
    P = max(1, args.pipeline)
    mods = [m] + [M.Modem(cfg, 0) for _ in range(P - 1)]
    for mm in mods[1:]:
        if tuning:
            mm.walk_tuning(**tuning)
    sts = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(P - 1)]
    outs = [(pbs, out, cons)] + [(torch.empty_like(pbs), torch.empty_like(out), torch.empty_like(cons))
                                 for _ in range(P - 1)]

    def call(i):
        mm = mods[i % P]
        rx = mm.rx_stream_i16 if args.i16 else mm.rx_stream
        o = outs[i % P]
        return rx(x, n, nf, pb_out=o[0], bytes_out=o[1], constell_out=o[2], chunk=args.chunk, stream=sts[i % P])

    for i in range(max(P, args.warmup)):
        found = call(i)
    # back to back (bench.py's timing): one timed region over reps * P calls
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.reps * P):
        found = call(i)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / (args.reps * P) * 1e3
    # isolated calls (latency)
    iso = []
    for r in range(args.reps):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        found = call(0)
        torch.cuda.synchronize()
        iso.append(time.perf_counter() - t1)
    # located frames decode to the payload of the frame placed there
    k = min(found, nf)
    ok = 0
    if k:
        pk = pbs[:k].cpu().numpy()
        where = np.searchsorted(layout.starts, pk, side="right") - 1
        fa, fb = int(where.min()), int(where.max()) + 1
        sent = payload_bytes(fa * layout.bpf, (fb - fa) * layout.bpf).reshape(fb - fa, layout.bpf)
        ok = int((out.reshape(nf, -1)[:k].cpu().numpy() == sent[where - fa]).all(axis=1).sum())
    # SURVEY §8d config 4 algorithmic bytes: the stream read once, plus each
    # located frame's constellation and payload bytes written
    esz = 4 if args.i16 else 16
    alg = n * esz + found * (16 * g["npts"] + g["bytes_per_frame"])
    res = {"workload": "config4_stream_%s_frames_gaps0-4096_cfo0.004_awgn20dB%s"
                       % (args.config, "_int16" if args.i16 else ""),
           "stream_samples": n, "frames_sent": nf, "frames_found": found, "frames_error_free": ok,
           "ms": round(ms, 4), "G_stream_samples_per_s": round(n / ms / 1e6, 2),
           "isolated_call_ms": round(float(np.median(iso)) * 1e3, 4),
           "frames_per_s": round(found / ms * 1e3), "stream_GB": round(n * esz / 1e9, 3),
           "chunk": args.chunk, "pipeline": P, "walk_tuning": args.walk_tuning,
           "roofline": {"bound": "hbm", "algorithmic_bytes": alg, "achieved": round(alg / ms / 1e6, 1),
                        "peak": 8000.0, "unit": "GB/s", "frac": round(alg / ms / 1e6 / 8000.0, 4),
                        "note": "whole stream pipeline (walk + resolve + decode), back-to-back calls, against "
                                "the bytes it must move once"}}
    if args.cpu_seconds > 0 and not args.i16:
        res["cpu_baseline"] = cpu_stream_baseline(cfg, x, args.cpu_seconds)
    print(json.dumps(res), flush=True)
    for mm in mods:
        mm.close()


def cpu_stream_baseline(cfg, x, budget_s):
    """The oracle's rx.cpp walk + main.cpp:60-80 decode, single-threaded as the
    reference runs, over a prefix of the same stream sized to ~budget_s."""
    g = O.geometry(cfg)
    span = g["preamble_len"] + g["message_len"]
    n = 1 << 18
    while True:
        h = x[:n].cpu().numpy()
        t0 = time.perf_counter()
        pbs = O.stream_walk_ring(cfg, h)[0]
        for pb in pbs:
            if pb + span <= len(h):
                O.decode_frame(cfg, h[pb:pb + span])
        dt = time.perf_counter() - t0
        if dt > budget_s / 4 or n >= len(x):
            break
        n = min(len(x), n * 2)
    return {"value": n / dt, "unit": "stream samples/s", "cores": 1, "kind": "port",
            "sample": f"oracle orc_stream_walk_ring + orc_decode_frame (own FFT; FFTW absent) over the first "
                      f"{n} samples ({len(pbs)} frames) of the same stream, {dt:.1f} s, 1 thread"}


if __name__ == "__main__":
    main()
