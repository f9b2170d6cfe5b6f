#!/usr/bin/env python3
"""walk_debug.py — where a GPU stream walk departs from the oracle's on a
tx.cpp-style capture (exact-zero silences): per ring mode, chunking and walk
tuning, the frames missing / extra, and for the first missing frame the
oracle's step that located it (T2 hit, preamble lag)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("tests", "oracle", "c-ofdm_amd/python")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ofdm_mi355x as M  # noqa: E402
import oracle as O  # noqa: E402
from common import D, capture_stream  # noqa: E402


def main():
    g = O.geometry(D)
    x, x16 = capture_stream(D, 120, seed=4)
    m = M.Modem(D, 0)
    dx = torch.from_numpy(x).cuda()
    first_missing = None
    for ring in (None, 0):
        want = O.stream_walk_ring(D, x, ring=ring)[0]
        old = m.stream_ring(ring) if ring is not None else None
        for tun in (dict(), dict(t2_f32=0), dict(exact_search=1), dict(t2_f32=0, exact_search=1)):
            m.walk_tuning(**tun)
            for chunk in (0, 2000000):
                pb = torch.full((256,), -1, dtype=torch.int64, device="cuda")
                nf = m.rx_stream(dx, len(x), 256, pb_out=pb, chunk=chunk)
                torch.cuda.synchronize()
                got = pb[:min(nf, 256)].cpu().numpy()
                ok = np.array_equal(got, want)
                miss = sorted(set(want) - set(got))
                extra = sorted(set(got) - set(want))
                print(f"ring={ring} tuning={tun} chunk={chunk}: nf {nf} want {len(want)} equal {ok} "
                      f"missing {miss[:8]} extra {extra[:8]}", flush=True)
                if miss and first_missing is None:
                    first_missing = (ring, miss[0], want)
        m.walk_tuning()
        if old is not None:
            m.stream_ring(old)
    if first_missing:
        ring, pbm, want = first_missing
        k = list(want).index(pbm)
        prev = want[k - 1] if k else None
        pos = prev + g["message_len"] if prev is not None else 0
        hit = O.find_t2sin(D, x, pos)
        print(f"first missing pb {pbm} (ring {ring}); previous pb {prev}, walk pos {pos}, "
              f"oracle find_t2sin(pos) = {hit}", flush=True)
        if hit >= 0:
            print("  find_preamble(hit) =", O.find_preamble(D, x, hit), flush=True)
        nz = np.nonzero(x[pos:pbm + 10])[0]
        print(f"  nonzero samples between pos and pb: first {pos + nz[0] if nz.size else None}", flush=True)


if __name__ == "__main__":
    main()
