#!/usr/bin/env python3
"""ber_sweep.py — SURVEY §8d config 3: bit-error rate of the modem over AWGN.

Config C (N=4096, D=2048, P=64, cp=1024, 16-QAM, 8 symbols per frame); Es/N0
from 0 to 30 dB in 2 dB steps; >= 1e7 bits per point; counter-based
Box-Muller noise (the same definition as the oracle's orc_awgn), seed =
1000 + SNR. Es/N0 = Es / sigma^2 with sigma^2 the complex noise variance per
time sample (the unnormalised forward FFT scales signal and noise alike), Es
the mean energy of the reference's 16-QAM table (modulation.cpp:4-36).
One JSON line per SNR: BER, bits, errors, GPU time of tx+AWGN+rx.

  python tools/ber_sweep.py [--snr 0:30:2] [--bits 1e7]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "c-ofdm_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402  (config dict, geometry, constellation table)


def noise_std_for(cfg, snr_db: float) -> float:
    es = float(np.mean(np.abs(O.constellation(cfg["mod_type"])) ** 2))
    return float(np.sqrt(es / 10 ** (snr_db / 10)))


def sweep(m, cfg, snrs, bits, torch):
    g = O.geometry(cfg)
    bpf = g["bytes_per_frame"]
    nf = int(np.ceil(bits / (8 * bpf)))
    gen = torch.Generator(device="cuda").manual_seed(3)
    data = torch.randint(0, 256, (nf * bpf,), dtype=torch.uint8, device="cuda", generator=gen)
    iq = torch.empty((nf * g["message_len"],), dtype=torch.complex128, device="cuda")
    out = torch.empty_like(data)
    errs = torch.zeros((1,), dtype=torch.int64, device="cuda")
    rows = []
    for snr in snrs:
        std = noise_std_for(cfg, snr)
        errs.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        m.tx(data, nf, iq, noise_std=std, seed=1000 + int(snr))
        m.rx(iq, nf, bytes_out=out, ref=data, bit_errors=errs)
        e1.record()
        torch.cuda.synchronize()
        nbits = 8 * nf * bpf
        ne = int(errs.item())
        rows.append({"config": "config3_C_N4096_D2048_P64_cp1024_16QAM", "es_n0_db": snr, "noise_std": std,
                     "seed": 1000 + int(snr), "frames": nf, "bits": nbits, "bit_errors": ne, "ber": ne / nbits,
                     "gpu_ms": round(e0.elapsed_time(e1), 3)})
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--snr", default="0:30:2", help="start:stop:step in dB (inclusive)")
    ap.add_argument("--bits", type=float, default=1e7)
    args = ap.parse_args()
    import torch
    import ofdm_mi355x as M

    a, b, c = (float(v) for v in args.snr.split(":"))
    snrs = list(np.arange(a, b + c / 2, c))
    cfg = dict(O.CONFIG_C)
    m = M.Modem(cfg, 0)
    for row in sweep(m, cfg, snrs, args.bits, torch):
        print(json.dumps(row), flush=True)
    m.close()


if __name__ == "__main__":
    main()
