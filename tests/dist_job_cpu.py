"""One rank of a CPU rehearsal of bench.py's multi-rank job (gloo), started by
ofdm_dist.launch_ranks — the launcher bench.py uses for `--gpus N`. Each rank
takes its contiguous frame shard (ofdm_dist.shard), runs the loopback on it
with the ORACLE (this is test infrastructure: on MI355X bench.py runs the HIP
modem in the same place), and the job reduces {bit errors, bits, samples,
frames} with ofdm_dist.reduce_counters; rank 0 prints one JSON line.
Not collected by pytest (no test_ prefix)."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "c-ofdm_amd", "python"), HERE]

import numpy as np  # noqa: E402

import ofdm_dist  # noqa: E402
import oracle as O  # noqa: E402
from common import D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=10)
    args = ap.parse_args()
    import torch
    world, rank, local = ofdm_dist.env_world()
    dist, dev = ofdm_dist.init("gloo", local, use_gpu=False)
    g = O.geometry(D)
    L, bpf = g["message_len"], g["bytes_per_frame"]
    data = np.random.default_rng(5).integers(0, 256, args.frames * bpf, dtype=np.uint8)
    b, c = ofdm_dist.shard(args.frames, world, rank)
    d = data[b * bpf:(b + c) * bpf]
    iq = O.awgn(O.tx_batch(D, d, c), 0.45, seed=7, sample_offset=b * L)
    _, out, errs = O.rx_batch(D, iq, c, L, ref=d)
    counters = torch.tensor([errs, c * bpf * 8, c * L, c], dtype=torch.int64)
    ofdm_dist.reduce_counters(counters, dist)
    elapsed = ofdm_dist.max_over_ranks(float(rank + 1), dev, dist)
    seen = [None] * world
    if dist:
        dist.all_gather_object(seen, (rank, int(os.environ["WORLD_SIZE"]), b, c, out.tobytes().hex()))
    else:
        seen = [(rank, world, b, c, out.tobytes().hex())]
    if rank == 0:
        print(json.dumps({"n_gpus": world, "grouped": dist is not None, "totals": counters.tolist(), "max_elapsed": elapsed,
                          "ranks": [[r, w, b, c] for r, w, b, c, _ in seen],
                          "bytes_hex": "".join(h for *_, h in sorted(seen))}), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
