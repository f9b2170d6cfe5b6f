#!/usr/bin/env python3
"""Experiment: the bench step (config B, 8192 frames: tx+AWGN then rx) with
the frames in C chunks, tx of chunk k+1 on one HIP stream beside rx of chunk k
on another (event per chunk); TXRX_SEQ=1: tx(k), rx(k) in turn on one stream.
Prints ms per step and bit errors per C."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "c-ofdm_amd", "python")]
import torch  # noqa: E402

import ofdm_mi355x as M  # noqa: E402
from bench import CONFIG_B  # noqa: E402
from ofdm_synth import payload_bytes  # noqa: E402

dev = torch.device("cuda:0")
p = dict(CONFIG_B)
modem = M.Modem(p, 0)
geo = modem.geo
nf = 8192
msg, bpf = geo.message_len, geo.bytes_per_frame
npts = p["num_data_subc"] * p["num_symb"]
data = torch.from_numpy(payload_bytes(0, nf * bpf)).to(dev)
iq = torch.empty((nf * msg,), dtype=torch.complex128, device=dev)
cons = torch.empty((nf * npts,), dtype=torch.complex128, device=dev)
out = torch.empty((nf * bpf,), dtype=torch.uint8, device=dev)
errs = torch.zeros((1,), dtype=torch.int64, device=dev)
noise_std = float(np.sqrt(2.0 / 10 ** 1.0))
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


SEQ = os.environ.get("TXRX_SEQ") == "1"  # one stream: tx(k), rx(k), tx(k+1), ...


def step(C):
    per = (nf + C - 1) // C
    if SEQ:
        for k in range(C):
            f0, n = k * per, min(per, nf - k * per)
            if n <= 0:
                break
            modem.tx(data[f0 * bpf:], n, iq[f0 * msg:], noise_std=noise_std, seed=1, sample_offset=f0 * msg, stream=sa)
            modem.rx(iq[f0 * msg:], n, constell_out=cons[f0 * npts:], bytes_out=out[f0 * bpf:], ref=data[f0 * bpf:],
                     bit_errors=errs, stream=sa)
        return
    evs = []
    for k in range(C):
        f0, n = k * per, min(per, nf - k * per)
        if n <= 0:
            break
        modem.tx(data[f0 * bpf:], n, iq[f0 * msg:], noise_std=noise_std, seed=1, sample_offset=f0 * msg, stream=sa)
        e = torch.cuda.Event()
        e.record(sa)
        evs.append((e, f0, n))
    for e, f0, n in evs:
        sb.wait_event(e)
        modem.rx(iq[f0 * msg:], n, constell_out=cons[f0 * npts:], bytes_out=out[f0 * bpf:], ref=data[f0 * bpf:],
                 bit_errors=errs, stream=sb)
    # the next step's tx rewrites iq: wait for this step's rx
    done = torch.cuda.Event()
    done.record(sb)
    sa.wait_event(done)


for C in [int(c) for c in (sys.argv[1:] or ["1", "2", "4", "8", "16"])]:
    for _ in range(10):
        step(C)
    torch.cuda.synchronize()
    errs.zero_()
    t0 = time.perf_counter()
    for _ in range(20):
        step(C)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 20 * 1e3
    if SEQ:
        print("seq", end=" ")
    print(f"C={C:3d} {ms:.4f} ms/step {nf * msg / ms / 1e6:.1f} G IQ/s errs/step {int(errs.item()) // 20}", flush=True)
