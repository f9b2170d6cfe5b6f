#!/usr/bin/env python3
"""txrx_gap_probe.py — why rx takes longer inside the bench step (right after
tx) than alone. Config B, 8192 frames, as bench.py. Prints one JSON line with:
  step: tx then rx back to back (bench.py's step), per-kernel ms
  rx_alone: rx repeated with no tx in between
  rx_after_gap: tx, an idle GPU gap (torch.cuda._sleep), rx
  sub_N: the batch as N sub-batches, tx(sub) then rx(sub) each (a timing
         experiment on cache residency; not the bench's definition)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "c-ofdm_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402


def main():
    import torch
    import ofdm_mi355x as M
    p = dict(O.CONFIG_B)
    m = M.Modem(p, 0)
    geo = m.geo
    nf = 8192
    msg, bpf = geo.message_len, geo.bytes_per_frame
    npts = p["num_data_subc"] * p["num_symb"]
    g = torch.Generator(device="cuda").manual_seed(1)
    data = torch.randint(0, 256, (nf * bpf,), dtype=torch.uint8, device="cuda", generator=g)
    iq = torch.empty((nf * msg,), dtype=torch.complex128, device="cuda")
    cons = torch.empty((nf * npts,), dtype=torch.complex128, device="cuda")
    out = torch.empty((nf * bpf,), dtype=torch.uint8, device="cuda")
    noise = float(np.sqrt(2.0 / 10.0))
    st = torch.cuda.current_stream()

    def tx(f0=0, n=nf):
        m.tx(data[f0 * bpf:(f0 + n) * bpf], n, iq[f0 * msg:(f0 + n) * msg], noise_std=noise, seed=1,
             sample_offset=f0 * msg, stream=st)

    def rx(f0=0, n=nf):
        m.rx(iq[f0 * msg:(f0 + n) * msg], n, constell_out=cons[f0 * npts:(f0 + n) * npts],
             bytes_out=out[f0 * bpf:(f0 + n) * bpf], stream=st)

    def timed(fn, reps=20, warm=10):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize()
        evs = []
        for _ in range(reps):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            e[0].record(st)
            fn()
            e[1].record(st)
            evs.append(e)
        torch.cuda.synchronize()
        return float(np.mean([a.elapsed_time(b) for a, b in evs]))

    res = {}
    # bench step with per-kernel events
    for _ in range(10):
        tx(); rx()
    torch.cuda.synchronize()
    ev = []
    for _ in range(20):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record(st); tx(); e[1].record(st); rx(); e[2].record(st)
        ev.append(e)
    torch.cuda.synchronize()
    res["step_tx_ms"] = float(np.mean([a.elapsed_time(b) for a, b, _ in ev]))
    res["step_rx_ms"] = float(np.mean([b.elapsed_time(c) for _, b, c in ev]))
    res["step_ms"] = float(np.mean([a.elapsed_time(c) for a, _, c in ev]))
    res["rx_alone_ms"] = timed(rx)
    res["tx_alone_ms"] = timed(tx)
    # tx, idle gap, rx
    ev = []
    for i in range(30):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        tx()
        torch.cuda._sleep(2_000_000)  # ~1 ms of GPU idle-spin on one wave
        e[0].record(st); rx(); e[1].record(st)
        if i >= 10:
            ev.append(e)
    torch.cuda.synchronize()
    res["rx_after_gap_ms"] = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    for nb in (2, 4, 8, 16, 32):
        sub = nf // nb

        def piped():
            for k in range(nb):
                tx(k * sub, sub)
                rx(k * sub, sub)
        res[f"sub{nb}_step_ms"] = timed(piped)
    print(json.dumps({k: round(v, 4) for k, v in res.items()}), flush=True)
    m.close()


if __name__ == "__main__":
    main()
