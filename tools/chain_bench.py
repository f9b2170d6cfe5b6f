#!/usr/bin/env python3
"""Latency of one drop-in sync chain launch (config D form, one frame): the
chain kernel with its stage copies to page-locked host memory, to device
memory and without copies; chan estimate; rx_demod_read. HIP-event timed,
median of --reps launches each synchronised (the drop-in's use)."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "c-ofdm_amd", "python")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    import numpy as np
    import torch
    import ofdm_mi355x as M
    import oracle as O
    from common import D
    g = O.geometry(D)
    n = g["preamble_len"] + g["message_len"]
    nsym = D["num_pr_symb"] + D["num_symb"]
    m = M.Modem(D, 0)
    rng = np.random.default_rng(1)
    x0 = torch.from_numpy(rng.standard_normal(n) + 1j * rng.standard_normal(n)).cuda()
    cfo = torch.full((1,), 1e-4, dtype=torch.float64, device="cuda")
    x = x0.clone()

    def timed(fn):
        ts = []
        for _ in range(args.reps):
            x.copy_(x0)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        return statistics.median(ts)

    hp = [torch.zeros((n,), dtype=torch.complex128, pin_memory=True) for _ in range(3)]
    dv = [torch.zeros((n,), dtype=torch.complex128, device="cuda") for _ in range(3)]
    chan = torch.zeros((D["num_data_subc"],), dtype=torch.complex128, device="cuda")
    npts = g["npts"]
    hr = torch.zeros((npts,), dtype=torch.complex128, pin_memory=True)
    he = torch.zeros((npts,), dtype=torch.complex128, pin_memory=True)
    hb = torch.zeros((g["bytes_per_frame"],), dtype=torch.uint8, pin_memory=True)
    msg = x[g["preamble_len"]:]
    out = {
        "chain_pinned_us": timed(lambda: m.sync_chain(x, 1, n, n, nsym, cfo, *hp)),
        "chain_device_us": timed(lambda: m.sync_chain(x, 1, n, n, nsym, cfo, *dv)),
        "chain_nocopy_us": timed(lambda: m.sync_chain(x, 1, n, n, nsym, cfo)),
        "three_stages_us": timed(lambda: (m.freq_shift(x, 1, n, n, cfo), m.cp_sync(x, 1, n, nsym),
                                          m.phase_sync(x, 1, n, n))),
        "chan_us": timed(lambda: m.chan_estimate(x, 1, n, chan)),
        "rx_read_pinned_us": timed(lambda: m.rx_read(msg, 1, chan=chan, read_out=hr, constell_out=he,
                                                     bytes_out=hb)),
        "cfo_us": timed(lambda: m.cfo_estimate(x, 1, n, D["num_pr_symb"], cfo)),
        "empty_us": timed(lambda: None),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
