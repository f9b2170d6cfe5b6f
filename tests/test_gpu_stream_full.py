"""GPU parity of the streaming receiver at the config-4 bench size (SURVEY §8d
config 4; tools/stream_bench.py's stream: 16 384 D-config frames, 0-4096
gaps, CFO +-0.004, random phase, 20 dB AWGN; 132 M samples). The GPU's
chunk-parallel walk must equal the oracle's sequential rx.cpp:94-198 walk
over the whole stream, with rx.cpp's SDR ring (the default; the oracle's ring
walk is checked against rx.cpp's loop replayed on a real ring buffer here
too) and without it, and every located frame must decode as the oracle's
main.cpp:60-80 chain does (CFO exact, constellation to 1e-9, every decision
equal). The per-run summaries go to gpurun_out/stream_full_summary.jsonl.
The oracle walk and the OpenMP decode of all ~16 000 frames take a few
seconds of CPU."""
import json
import os

import numpy as np
import pytest

import oracle as O
from common import check_stream_frames

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import ofdm_mi355x as M  # noqa: E402


def build_stream(cfg, nf, seed=4):
    """The stream of tools/stream_bench.py, built on the GPU."""
    g = O.geometry(cfg)
    m = M.Modem(cfg, 0)
    flen = g["frame_len"]
    gen = torch.Generator(device="cuda").manual_seed(seed)
    data = torch.randint(0, 256, (nf * g["bytes_per_frame"],), dtype=torch.uint8, device="cuda", generator=gen)
    frames = torch.empty((nf * flen,), dtype=torch.complex128, device="cuda")
    m.tx_frames(data, nf, frames)
    gaps = torch.randint(0, 4097, (nf + 1,), device="cuda", generator=gen)
    starts = torch.cumsum(gaps[:-1] + flen, 0) - flen
    n = int(starts[-1].item()) + flen + int(gaps[-1].item())
    x = torch.zeros((n,), dtype=torch.complex128, device="cuda")
    idx = (starts[:, None] + torch.arange(flen, device="cuda")[None, :]).reshape(-1)
    cfo = (torch.rand((nf, 1), dtype=torch.float64, device="cuda", generator=gen) * 2 - 1) * 0.004
    ph = (torch.rand((nf, 1), dtype=torch.float64, device="cuda", generator=gen) * 2 - 1) * np.pi
    ramp = torch.arange(flen, dtype=torch.float64, device="cuda")[None, :]
    rot = torch.polar(torch.ones_like(cfo * ramp), 2 * np.pi * cfo * ramp + ph).reshape(-1)
    x[idx] = frames * rot
    sig = 10 ** (-20.0 / 20) / np.sqrt(2)
    x += torch.complex(torch.randn(n, dtype=torch.float64, device="cuda", generator=gen) * sig,
                       torch.randn(n, dtype=torch.float64, device="cuda", generator=gen) * sig)
    return m, x, n


def run_full(m, x, n, nf, i16):
    cfg = dict(O.DEFAULT)
    g = O.geometry(cfg)
    pbs = torch.full((nf,), -1, dtype=torch.int64, device="cuda")
    out = torch.zeros((nf * g["bytes_per_frame"],), dtype=torch.uint8, device="cuda")
    cons = torch.zeros((nf * g["npts"],), dtype=torch.complex128, device="cuda")
    cfo = torch.zeros((nf,), dtype=torch.float64, device="cuda")
    fn = m.rx_stream_i16 if i16 else m.rx_stream
    found = fn(x, n, nf, pb_out=pbs, bytes_out=out, constell_out=cons, cfo_out=cfo)
    torch.cuda.synchronize()
    k = min(found, nf)
    return (found, pbs.cpu().numpy()[:k], out.cpu().numpy().reshape(nf, -1)[:k],
            cons.cpu().numpy().reshape(nf, -1)[:k], cfo.cpu().numpy()[:k])


@pytest.mark.parametrize("i16,ring", [(False, True), (True, True), (False, False)],
                         ids=["f64", "int16", "f64-continuous"])
def test_stream_bench_size_every_frame_matches_oracle(i16, ring):
    """The config-4 bench stream (16 384 frames, 132 M samples), f64 and the
    int16 wire format: the walk equals the oracle's sequential walk, and EVERY
    located frame decodes as the oracle's main.cpp:60-80 chain on the same
    samples (CFO exact, constellation 1e-9, every decision equal; see
    common.check_stream_frames)."""
    cfg = dict(O.DEFAULT)
    nf = 16384
    m, x, n = build_stream(cfg, nf, seed=5 if i16 else 4)
    if not ring:
        m.stream_ring(0)
    if i16:
        # the SDR wire format: the GPU reads complex<int16>, the oracle their exact doubles
        x16 = (torch.view_as_real(x) * float(cfg["mult"])).round().clamp(-32768, 32767).to(torch.int16).reshape(-1)
        del x
        h16 = x16.cpu().numpy().reshape(-1, 2).astype(np.float64)
        h = h16[:, 0] + 1j * h16[:, 1]
        found, pbs, out, cons, cfo = run_full(m, x16, n, nf, True)
    else:
        h = x.cpu().numpy()
        found, pbs, out, cons, cfo = run_full(m, x, n, nf, False)
    if ring:
        want = O.stream_walk_ring(cfg, h)[0]
        assert np.array_equal(want, O.rx_app_walk(cfg, h))  # rx.cpp's loop on a real ring buffer
    else:
        want = O.stream_walk(cfg, h)
    assert found == len(want) and found > 0.95 * nf
    assert np.array_equal(pbs, want[:len(pbs)])
    summary = check_stream_frames(cfg, h, pbs, out, cons, cfo)
    assert summary["frames"] == found and summary["decision_flips"] == 0
    summary.update(stream="int16" if i16 else "f64", ring=int(m.stream_ring()), samples=int(n),
                   frames_sent=nf)
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "stream_full_summary.jsonl"), "a") as f:
        f.write(json.dumps(summary) + "\n")
    m.close()
