#!/usr/bin/env python3
"""overlap_probe.py — can tx and rx kernels share the GPU? Times tx(half A) and
rx(half B) run back to back on one stream against the same pair issued on two
streams (no dependency between them), config B. Design probe, not a bench."""
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
    p = O.CONFIG_B
    g = O.geometry(p)
    m = M.Modem(p, 0)
    nf = 8192
    data = torch.randint(0, 256, (nf * g["bytes_per_frame"],), dtype=torch.uint8, device="cuda")
    iq = torch.empty((nf * g["message_len"],), dtype=torch.complex128, device="cuda")
    cons = torch.empty((nf * g["npts"],), dtype=torch.complex128, device="cuda")
    out = torch.empty_like(data)
    m.tx(data, nf, iq, noise_std=0.4, seed=1)
    h = nf // 2
    bpf, ml, npt = g["bytes_per_frame"], g["message_len"], g["npts"]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def tx_a(st):
        m.tx(data[:h * bpf], h, iq[:h * ml], noise_std=0.4, seed=1, stream=st)

    def rx_b(st):
        m.rx(iq[h * ml:], nf - h, constell_out=cons[h * npt:], bytes_out=out[h * bpf:], stream=st)

    def timeit(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            e0.record()
            fn()
            torch.cuda.synchronize()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts))

    cur = torch.cuda.current_stream()

    def seq():
        tx_a(cur.cuda_stream)
        rx_b(cur.cuda_stream)

    def par():
        ev = torch.cuda.Event()
        ev.record(cur)
        s1.wait_event(ev)
        s2.wait_event(ev)
        tx_a(s1.cuda_stream)
        rx_b(s2.cuda_stream)
        e1, e2 = torch.cuda.Event(), torch.cuda.Event()
        e1.record(s1)
        e2.record(s2)
        cur.wait_event(e1)
        cur.wait_event(e2)

    res = {"tx_half_ms": timeit(lambda: tx_a(cur.cuda_stream)),
           "rx_half_ms": timeit(lambda: rx_b(cur.cuda_stream)),
           "sequential_ms": timeit(seq), "two_streams_ms": timeit(par)}
    # co-residency: cap the persistent grids (workgroups per CU) so that both
    # kernels fit the CUs at once (OFDM_RX_WGS_PER_CU / OFDM_TX_WGS_PER_CU)
    for rxw, txw in ((1, 1), (1, 2), (2, 1)):
        os.environ["OFDM_RX_WGS_PER_CU"] = str(rxw)
        os.environ["OFDM_TX_WGS_PER_CU"] = str(txw)
        res[f"two_streams_rx{rxw}_tx{txw}_ms"] = timeit(par)
        res[f"sequential_rx{rxw}_tx{txw}_ms"] = timeit(seq)
    os.environ.pop("OFDM_RX_WGS_PER_CU")
    os.environ.pop("OFDM_TX_WGS_PER_CU")
    print(json.dumps({k: round(v, 4) for k, v in res.items()}))


if __name__ == "__main__":
    main()
