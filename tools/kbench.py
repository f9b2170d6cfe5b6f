#!/usr/bin/env python3
"""kbench.py — per-kernel timing of the HIP modem kernels (HIP events on the
launch stream), for design work and DESIGN.md tables. Not the driver bench.

  python tools/kbench.py [--configs B,C,D] [--reps 20]
Prints one JSON line per (config, variant) with ms/launch and algorithmic GB/s
(SURVEY §8d bytes: rx 16N+16D+Dk/8 per symbol, tx Dk/8+16(N+cp) per symbol).
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "c-ofdm_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402  (config dicts only)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="B,C,D")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--samples", type=float, default=1.68e8, help="target IQ samples per launch")
    ap.add_argument("--alt", action="store_true", help="also time tx->rx alternating pairs")
    args = ap.parse_args()
    import torch
    import ofdm_mi355x as M

    cfgs = {"B": O.CONFIG_B, "C": O.CONFIG_C, "D": O.DEFAULT, "G": O.GOLDEN}
    st = torch.cuda.current_stream()
    for name in args.configs.split(","):
        p = cfgs[name]
        m = M.Modem(p, 0)
        g = O.geometry(p)
        nf = int(args.samples // g["message_len"])
        S, N, D, k, cp = p["num_symb"], p["fft_size"], p["num_data_subc"], p["mod_type"], p["cp_size"]
        data = torch.randint(0, 256, (nf * g["bytes_per_frame"],), dtype=torch.uint8, device="cuda")
        iq = torch.empty((nf * g["message_len"],), dtype=torch.complex128, device="cuda")
        iq16 = torch.empty((2 * nf * g["message_len"],), dtype=torch.int16, device="cuda")
        cons = torch.empty((nf * g["npts"],), dtype=torch.complex128, device="cuda")
        out = torch.empty_like(data)
        errs = torch.zeros((1,), dtype=torch.int64, device="cuda")
        rx_b = nf * S * (16 * N + 16 * D + D * k // 8)
        tx_b = nf * S * (D * k // 8 + 16 * (N + cp))
        variants = {
            "tx": (lambda: m.tx(data, nf, iq), tx_b),
            "tx+awgn": (lambda: m.tx(data, nf, iq, noise_std=0.4, seed=1), tx_b),
            "tx+int16": (lambda: m.tx(data, nf, iq, iq16_out=iq16), tx_b + nf * S * 4 * (N + cp)),
            "rx(constell+bytes+ber)": (lambda: m.rx(iq, nf, constell_out=cons, bytes_out=out, ref=data,
                                                   bit_errors=errs), rx_b + nf * S * D * k // 8),
            "rx(bytes)": (lambda: m.rx(iq, nf, bytes_out=out), nf * S * (16 * N + D * k // 8)),
            # achievable-bandwidth reference: a torch device copy of the constellation's size
            "torch copy (ref)": (lambda: cons.copy_(iq[:cons.numel()]), 2 * 16 * cons.numel()),
            "rx_i16(constell+bytes+ber)": (lambda: m.rx_i16(iq16, nf, constell_out=cons, bytes_out=out, ref=data,
                                                           bit_errors=errs),
                                          nf * S * (4 * N + 16 * D + D * k // 8) + nf * S * D * k // 8),
        }
        # alternating tx -> rx (the bench step): time each kernel of the pair
        def alt(noise):
            ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.reps)]
            for _ in range(3):
                m.tx(data, nf, iq, noise_std=noise, seed=1)
                m.rx(iq, nf, constell_out=cons, bytes_out=out, ref=data, bit_errors=errs)
            for e in ev:
                e[0].record(st)
                m.tx(data, nf, iq, noise_std=noise, seed=1)
                e[1].record(st)
                m.rx(iq, nf, constell_out=cons, bytes_out=out, ref=data, bit_errors=errs)
                e[2].record(st)
            torch.cuda.synchronize()
            return (float(np.median([e[0].elapsed_time(e[1]) for e in ev])),
                    float(np.median([e[1].elapsed_time(e[2]) for e in ev])))
        if args.alt:
            for noise in (0.0, 0.4):
                txm, rxm = alt(noise)
                print(json.dumps({"config": name, "variant": f"alt tx{'+awgn' if noise else ''} -> rx",
                                  "tx_ms": round(txm, 4), "rx_ms": round(rxm, 4)}), flush=True)
            # rx after a plain 2.7 GB device write (dirty-line write-back cost seen by the next kernel)
            junk = torch.empty_like(iq)
            ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.reps)]
            for e in ev:
                e[0].record(st)
                junk.fill_(1.0)
                e[1].record(st)
                m.rx(iq, nf, constell_out=cons, bytes_out=out, ref=data, bit_errors=errs)
                e[2].record(st)
            torch.cuda.synchronize()
            print(json.dumps({"config": name, "variant": "alt fill -> rx",
                              "fill_ms": round(float(np.median([e[0].elapsed_time(e[1]) for e in ev])), 4),
                              "rx_ms": round(float(np.median([e[1].elapsed_time(e[2]) for e in ev])), 4)}), flush=True)
            del junk
        for vname, (fn, nbytes) in variants.items():
            for _ in range(3):
                fn()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(args.reps)]
            for e0, e1 in evs:
                e0.record(st)
                fn()
                e1.record(st)
            torch.cuda.synchronize()
            ms = float(np.median([a.elapsed_time(b) for a, b in evs]))
            print(json.dumps({"config": name, "variant": vname, "frames": nf, "ms": round(ms, 4),
                              "GBps": round(nbytes / ms / 1e6, 1),
                              "Gsamples_per_s": round(nf * g["message_len"] / ms / 1e6, 2)}), flush=True)
        m.close()


if __name__ == "__main__":
    main()
