#!/usr/bin/env python3
"""ab_step.py — bench.py's step (config B, 8192 frames: tx with AWGN, then rx
with constellation, bytes and bit errors) timed with HIP events per kernel,
for A/B of library variants (OFDM_MI355X_LIB). Prints one JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "c-ofdm_amd", "python"))
sys.path.insert(0, ROOT)


def main():
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
    steps = int(os.environ.get("AB_STEPS", "60"))
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    # back to back, as bench.py times them (no host sync between steps: the
    # clocks stay up); the first third is warmup
    for e in ev:
        e[0].record()
        m.tx(data, nf, iq, noise_std=0.447, seed=1)
        e[1].record()
        m.rx(iq, nf, constell_out=cons, bytes_out=out, ref=data, bit_errors=errs)
        e[2].record()
    torch.cuda.synchronize()
    times = [(e[0].elapsed_time(e[1]), e[1].elapsed_time(e[2])) for e in ev]
    t = np.array(times[steps // 3:])
    print(json.dumps({"lib": os.path.basename(os.environ.get("OFDM_MI355X_LIB", "product")),
                      "tx_ms": float(np.median(t[:, 0])), "rx_ms": float(np.median(t[:, 1])),
                      "rx_min_ms": float(t[:, 1].min()), "step_ms": float(np.median(t.sum(1)))}), flush=True)


if __name__ == "__main__":
    main()
