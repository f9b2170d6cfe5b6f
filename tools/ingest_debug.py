"""Debug helper: the chunked ingest (ofdm_ingest.StreamIngest) call by call on a small stream."""
import sys, os
sys.path[:0] = ["c-ofdm_amd/python", "oracle", "tests"]
import torch, numpy as np
import ofdm_mi355x as M, ofdm_ingest as I, ofdm_synth as Y
from common import D
m = M.Modem(D, 0)
lay = Y.StreamLayout(D, 64)
x16 = Y.stream_slice(m, lay, 0, lay.n, torch.device("cuda", 0), i16=True)
torch.cuda.synchronize()
cap = 80
def outs():
    return {"pb_out": torch.full((cap,), -7, dtype=torch.int64, device="cuda"),
            "bytes_out": torch.zeros((cap * 1024,), dtype=torch.uint8, device="cuda"),
            "constell_out": torch.zeros((cap * 2048,), dtype=torch.complex128, device="cuda"),
            "cfo_out": torch.zeros((cap,), dtype=torch.float64, device="cuda")}
ref = outs()
print("n", lay.n, "ref", m.rx_stream_i16(x16, lay.n, cap, **ref), "init", m.initial_state(), "ring", m.stream_ring())
ch = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
ing = I.StreamIngest(m, D, I.host_pinned_i16(x16), lay.n, ch, outs(), torch.device("cuda", 0), cap)
print("slices", ing.slices()[:3], "halo", ing.halo, "tail", ing.tail)
orig = m.rx_stream_shard
def spy(*a, **k):
    print("call n", a[1], "start", a[2], "own", a[3], a[4], flush=True)
    r = orig(*a, **k); print("   ->", r[0], r[3], flush=True); return r
m.rx_stream_shard = spy
print(ing.run())
