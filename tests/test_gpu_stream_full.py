"""GPU parity of the streaming receiver at the config-4 bench size (SURVEY §8d
config 4; tools/stream_bench.py's stream: 16 384 D-config frames, 0-4096
gaps, CFO +-0.004, random phase, 20 dB AWGN; 132 M samples). The GPU's
chunk-parallel walk must equal the oracle's sequential rx.cpp:125-221 walk
over the whole stream, and a sample of the located frames must decode as
the oracle's main.cpp:60-80 chain does (CFO exact, bytes exact,
constellation to 1e-9). The oracle walk over the full stream takes a few
seconds of CPU."""
import numpy as np
import pytest

import oracle as O

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


def test_stream_bench_size_walk_and_decode_match_oracle():
    cfg = dict(O.DEFAULT)
    g = O.geometry(cfg)
    nf = 16384
    m, x, n = build_stream(cfg, nf)
    pbs = torch.full((nf,), -1, dtype=torch.int64, device="cuda")
    out = torch.zeros((nf * g["bytes_per_frame"],), dtype=torch.uint8, device="cuda")
    cons = torch.zeros((nf * g["npts"],), dtype=torch.complex128, device="cuda")
    cfo = torch.zeros((nf,), dtype=torch.float64, device="cuda")
    found = m.rx_stream(x, n, nf, pb_out=pbs, bytes_out=out, constell_out=cons, cfo_out=cfo)
    torch.cuda.synchronize()
    h = x.cpu().numpy()
    want = O.stream_walk(cfg, h)
    assert found == len(want) and found > 0.95 * nf
    k = min(found, nf)
    got = pbs.cpu().numpy()[:k]
    assert np.array_equal(got, want[:k])
    # decode parity on a sample of the located frames (first, last, random)
    span = g["preamble_len"] + g["message_len"]
    pick = np.unique(np.concatenate([[0, k - 1], np.random.default_rng(7).integers(0, k, 62)]))
    h_out = out.cpu().numpy().reshape(nf, -1)
    h_cons = cons.cpu().numpy().reshape(nf, -1)
    h_cfo = cfo.cpu().numpy()
    for f in pick:
        c, oc, ob = O.decode_frame(cfg, h[want[f]: want[f] + span])
        assert h_cfo[f] == c
        assert np.array_equal(h_out[f], ob)
        assert np.abs(h_cons[f] - oc).max() / np.abs(oc).max() < 1e-9
    m.close()


def test_stream_bench_size_int16_walk_matches_oracle():
    # the SDR wire format (stream_bench.py --i16): the walk over the
    # complex<int16> samples equals the oracle's walk over their exact doubles
    cfg = dict(O.DEFAULT)
    g = O.geometry(cfg)
    nf = 16384
    m, x, n = build_stream(cfg, nf, seed=5)
    x16 = (torch.view_as_real(x) * float(cfg["mult"])).round().clamp(-32768, 32767).to(torch.int16).reshape(-1)
    del x
    pbs = torch.full((nf,), -1, dtype=torch.int64, device="cuda")
    out = torch.zeros((nf * g["bytes_per_frame"],), dtype=torch.uint8, device="cuda")
    found = m.rx_stream_i16(x16, n, nf, pb_out=pbs, bytes_out=out)
    torch.cuda.synchronize()
    h16 = x16.cpu().numpy().reshape(-1, 2).astype(np.float64)
    h = h16[:, 0] + 1j * h16[:, 1]
    want = O.stream_walk(cfg, h)
    assert found == len(want) and found > 0.95 * nf
    k = min(found, nf)
    assert np.array_equal(pbs.cpu().numpy()[:k], want[:k])
    span = g["preamble_len"] + g["message_len"]
    h_out = out.cpu().numpy().reshape(nf, -1)
    for f in np.unique(np.random.default_rng(8).integers(0, k, 32)):
        _, _, ob = O.decode_frame(cfg, h[want[f]: want[f] + span])
        assert np.array_equal(h_out[f], ob)
    m.close()
