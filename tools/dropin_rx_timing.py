#!/usr/bin/env python3
"""Per-frame time of the reference's OWN rx.cpp loop running on the drop-in
layer (oracle/_ref/rx: rx.cpp compiled unchanged against c-ofdm_amd/compat),
from the LOG.txt its TIME_TRACE macros write (rx.cpp:31-43,240-244), next to
the reference's committed LOG.txt (its authors' CPU/FFTW run).

The reference's tx.cpp (oracle/_ref/tx, also on the drop-in layer) frames a
payload file into data/tx.bin-layout int16 IQ through the SDR stand-in; rx
then reads that capture through the stand-in (OFDM_SDR_RX_FILE) with the
radio's refill pacing. An iteration that decoded a frame (SEQ field) and did
not refill the ring (no SDR field) is one frame's processing: find_t2sin,
find_preamble, the sync chain, FFT, equalise, demod, MAC.

  python tools/dropin_rx_timing.py [--frames 200] > profiles/<name>.json
"""
import argparse
import json
import os
import re
import statistics
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "c-ofdm_amd", "python")]
REF_BIN = os.path.join(ROOT, "oracle", "_ref")


STAGES = ("T2SIN", "PILOT_SINH", "FREQ_PHASE_SINH", "PFC", "MAC")


def parse_log(text):
    frames, refills, stages = [], [], {k: [] for k in STAGES}
    for line in text.splitlines():
        kv = dict(re.findall(r"(\w+):(\S+)", line))
        if "TIME" not in kv:
            continue
        if "SEQ" in kv and "SDR" not in kv:
            frames.append(float(kv["TIME"]))
            for k in STAGES:
                if k in kv:
                    stages[k].append(float(kv[k]))
        elif "SDR" in kv:
            refills.append(float(kv.get("CONVERT", "nan")))
    return frames, refills, stages


def gapped_capture(txf, frame_len, seed=4, gap_max=3000):
    """The tx app's back-to-back frames with random 0..gap_max-sample silences
    between them (the air between bursts, as the config-4 stream has): rx.cpp
    tests T2 blocks on a 256-sample grid from the end of the previous frame's
    message, so back-to-back frames put every other marker across two blocks."""
    import numpy as np
    iq = np.fromfile(txf, np.int16).reshape(-1, frame_len, 2)
    rng = np.random.default_rng(seed)
    parts = []
    for f in iq:
        parts += [np.zeros((int(rng.integers(0, gap_max + 1)), 2), np.int16), f]
    parts.append(np.zeros((frame_len, 2), np.int16))
    np.concatenate(parts).tofile(txf)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--trace", action="store_true",
                    help="OFDM_COMPAT_TRACE=1: median wall time of each compat member call (diagnostics)")
    args = ap.parse_args()
    from test_dropin_gpu import D, O, write_config
    g = O.geometry(D)
    with tempfile.TemporaryDirectory() as d:
        write_config(d, D, iterations=args.frames + 40)
        pay = g["bytes_per_frame"] - 8
        # per-frame distinct payloads (frame f's bytes shift by 249 f mod 256)
        body = bytes((i * 131 + 7 + (i // pay) * 17) & 0xFF for i in range(args.frames * pay))
        with open(os.path.join(d, "FlyMeToTheMoon_mono.wav"), "wb") as f:
            f.write(body)
        txf = os.path.join(d, "tx.bin")
        env = dict(os.environ, OFDM_SDR_TX_FILE=txf)
        r = subprocess.run([os.path.join(REF_BIN, "tx")], cwd=d, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        gapped_capture(txf, g["frame_len"])
        env = dict(os.environ, OFDM_SDR_RX_FILE=txf)
        if args.trace:
            env["OFDM_COMPAT_TRACE"] = "1"
        r = subprocess.run([os.path.join(REF_BIN, "rx")], cwd=d, env=env, capture_output=True, text=True, timeout=300)
        calls = {}
        for ln in r.stderr.splitlines():
            m = re.match(r"\[compat\] (\S+) ([0-9.]+)$", ln)
            if m:
                calls.setdefault(m.group(1), []).append(float(m.group(2)))
        assert r.returncode == 0, r.stderr[-2000:]
        with open(os.path.join(d, "LOG.txt")) as f:
            ours, refills, stages = parse_log(f.read())
        with open(os.path.join(d, "Res.wav"), "rb") as f:
            res = f.read()
    chunks = {body[i * pay:(i + 1) * pay] for i in range(args.frames)}
    index = {body[i * pay:(i + 1) * pay]: i for i in range(args.frames)}
    idx = [index.get(res[i * pay:(i + 1) * pay], -1) for i in range(len(res) // pay)]
    order_ok = -1 not in idx and idx == sorted(idx) and len(set(idx)) == len(idx)
    out = {"frames_sent": args.frames, "what": "rx.cpp per-frame iteration time (LOG.txt TIME of iterations that decoded a frame without a "
                   "ring refill), reference rx.cpp compiled unchanged on the drop-in layer",
           "config": "D (config/config.txt)", "frames_decoded": len(ours),
           "frames_written": len(res) // pay,
           "frames_payload_exact": sum(res[i * pay:(i + 1) * pay] in chunks for i in range(len(res) // pay)),
           "frames_in_order": order_ok,
           "median_us": statistics.median(ours) * 1e6 if ours else None,
           "p10_us": sorted(ours)[len(ours) // 10] * 1e6 if ours else None,
           "p90_us": sorted(ours)[9 * len(ours) // 10] * 1e6 if ours else None,
           "refill_convert_median_us": statistics.median(refills) * 1e6 if refills else None,
           "stage_median_us": {k: statistics.median(v) * 1e6 for k, v in stages.items() if v},
           "compat_call_median_us": {k: [len(v), statistics.median(v)] for k, v in calls.items()} if args.trace else None,
           # parse_log over the reference's committed LOG.txt (9 430 frame iterations; its
           # authors' machine, FFTW on the CPU), evaluated in the build container
           "reference_LOG_txt_median_us": 238.42,
           "reference_LOG_txt_stage_median_us": {"T2SIN": 17.2, "PILOT_SINH": 57.2, "FREQ_PHASE_SINH": 84.2, "PFC": 27.2,
                                                 "MAC": 3.3},
           "reference_note": "the reference's committed LOG.txt (its authors' machine, FFTW, CPU)"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
