#!/usr/bin/env python3
"""rx_prof.py — per-workgroup phase clocks of rx_kernel (timing experiment;
needs a -DOFDM_RX_PROF build: tools/build_variant.sh rprof -DOFDM_RX_PROF,
selected with OFDM_MI355X_LIB). Runs bench.py's step (config B, 8192 frames,
tx with AWGN then rx) a few times, then prints where rx's wave 0 of each
workgroup spent its cycles per frame: waiting for symbol 0's LDS-DMA, waiting
for the next symbols' register prefetch, FFT + carrier extraction, and the
epilogue (gains, equalise, decide, stores, packing)."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "c-ofdm_amd", "python"))
sys.path.insert(0, ROOT)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--noref", action="store_true", help="rx without the bit-error count (no ref bytes)")
    args = ap.parse_args()
    import torch
    import bench
    import ofdm_mi355x as M
    p = dict(bench.CONFIG_B)
    m = M.Modem(p, 0)
    g = m.geo
    nf = 8192
    data = torch.from_numpy(bench.payload_bytes(0, nf * g.bytes_per_frame)).cuda()
    iq = torch.empty((nf * g.message_len,), dtype=torch.complex128, device="cuda")
    cons = torch.empty((nf * p["num_data_subc"] * 8,), dtype=torch.complex128, device="cuda")
    out = torch.empty_like(data)
    errs = torch.zeros((1,), dtype=torch.int64, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    times = []
    for _ in range(12):
        ev[0].record()
        m.tx(data, nf, iq, noise_std=0.447, seed=1)
        ev[1].record()
        if args.noref:
            m.rx(iq, nf, constell_out=cons, bytes_out=out)
        else:
            m.rx(iq, nf, constell_out=cons, bytes_out=out, ref=data, bit_errors=errs)
        ev[2].record()
        torch.cuda.synchronize()
        times.append((ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])))
    buf = np.zeros(2 * 4096 * 8, dtype=np.uint64)
    assert M.lib().ofdm_rx_prof(buf.ctypes.data_as(C.c_void_p)) == 0
    q = buf[:4096 * 8].reshape(4096, 8).astype(np.float64)
    u = buf[4096 * 8:].reshape(4096, 8).astype(np.float64)
    live = q[:, 4] > 0
    q, u = q[live], u[live]
    s0, pf, fft, epi, nfr, tot, w0, w1 = q.T
    F = nfr.sum()
    res = {"workgroups": len(q), "frames_per_wg": float(nfr.mean()),
           "tx_ms": float(np.median([t[0] for t in times[2:]])), "rx_ms": float(np.median([t[1] for t in times[2:]])),
           "cyc_per_frame": float(tot.sum() / F),
           "s0_wait_per_frame": float(s0.sum() / F), "pf_wait_per_frame": float(pf.sum() / F),
           "fft_per_frame": float(fft.sum() / F), "epilogue_per_frame": float(epi.sum() / F),
           "fft_per_symbol": float(fft.sum() / F / 8), "pf_wait_per_symbol": float(pf.sum() / F / 7),
           "wall_us_mean": float(((w1 - w0) / 100.0).mean()), "wall_us_max": float(((w1 - w0) / 100.0).max()),
           "start_spread_us": float((w0.max() - w0.min()) / 100.0),
           "epi_gain_per_frame": float(u[:, 0].sum() / F), "epi_emit_per_frame": float(u[:, 1].sum() / F),
           "epi_pack_per_frame": float(u[:, 2].sum() / F), "ref": not args.noref}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
