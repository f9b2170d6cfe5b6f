#!/usr/bin/env python3
"""rx_only.py — run the tx (with AWGN) and rx kernels a few times each at the
bench workload (config B, 8192 frames), for rocprofv3 counter passes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "c-ofdm_amd", "python"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import ofdm_mi355x as M
    from bench import CONFIG_B, payload_bytes
    nf = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    m = M.Modem(dict(CONFIG_B), 0)
    g = m.geo
    data = torch.from_numpy(payload_bytes(0, nf * g.bytes_per_frame)).cuda()
    iq = torch.empty((nf * g.message_len,), dtype=torch.complex128, device="cuda")
    cons = torch.empty((nf * CONFIG_B["num_data_subc"] * CONFIG_B["num_symb"],), dtype=torch.complex128, device="cuda")
    out = torch.empty_like(data)
    errs = torch.zeros((1,), dtype=torch.int64, device="cuda")
    for _ in range(reps):
        m.tx(data, nf, iq, noise_std=0.447, seed=1)
    for _ in range(reps):
        m.rx(iq, nf, constell_out=cons, bytes_out=out, ref=data, bit_errors=errs)
    torch.cuda.synchronize()
    print("bit_errors", int(errs.item()))
    m.close()


if __name__ == "__main__":
    main()
