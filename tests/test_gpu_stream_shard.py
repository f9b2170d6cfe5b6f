"""Streaming rx sharded over ranks on the GPU (ofdm_stream.py +
ofdm_rx_stream_shard): the stream is split into 2..8 sample shards, each with
its walk-in halo and tail, each run on its OWN ofdm_ctx (as one rank per GPU
would run it; here all on the box's one MI355X), with the report / plan /
re-walk protocol between them (ofdm_stream.run_local). The union of the owned
frames must equal the oracle's one sequential rx.cpp:94-198 walk with its SDR
ring over the whole stream (indices exact; orc_stream_walk_ring), and the owned frames decode as the oracle's
main.cpp:60-80 chain (CFO exact, bytes exact, constellation to 1e-9); at the
bench size (config 4, 132 M samples) too."""
import numpy as np
import pytest

import oracle as O
from common import D, check_stream_frames, impaired_stream, rel_err

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import ofdm_mi355x as M  # noqa: E402
import ofdm_stream as SS  # noqa: E402
import ofdm_synth as Y  # noqa: E402


def run_sharded(cfg, x, n, world, halo=None, i16=False, max_frames=None):
    """x: the whole stream on the GPU (complex128 (n,), or int16 (2n,)).
    Returns (pbs, bytes, constellation, cfo) of the owned frames in stream
    order (host arrays), and the re-walk count."""
    g = O.geometry(cfg)
    rxs, walks, outs, mods = [], [], [], []
    for r in range(world):
        m = M.Modem(cfg, 0)
        rx = SS.ShardedStreamRx(cfg, n, world, r, halo=halo, ring=m.stream_ring(), initial=m.initial_state())
        xs = x[2 * rx.slice_lo:2 * rx.slice_hi] if i16 else x[rx.slice_lo:rx.slice_hi]
        cap = max_frames or (rx.slice_hi - rx.slice_lo) // g["message_len"] + 8
        o = {"pb_out": torch.full((cap,), -1, dtype=torch.int64, device="cuda"),
             "bytes_out": torch.zeros((cap * g["bytes_per_frame"],), dtype=torch.uint8, device="cuda"),
             "constell_out": torch.zeros((cap * g["npts"],), dtype=torch.complex128, device="cuda"),
             "cfo_out": torch.zeros((cap,), dtype=torch.float64, device="cuda")}
        walks.append(SS.hip_walker(m, xs, rx.slice_hi - rx.slice_lo, rx.own_lo - rx.slice_lo,
                                   rx.own_hi - rx.slice_lo, cap, o, i16=i16, report_cap=rx.cap))
        rxs.append(rx)
        outs.append((o, cap))
        mods.append(m)
    counts = SS.run_local(rxs, walks)
    torch.cuda.synchronize()
    pbs, byt, cons, cfo = [], [], [], []
    for rx, (o, cap), k in zip(rxs, outs, counts):
        k = min(k, cap)
        pbs.append(o["pb_out"][:k].cpu().numpy() + rx.slice_lo)
        byt.append(o["bytes_out"].cpu().numpy().reshape(cap, -1)[:k])
        cons.append(o["constell_out"].cpu().numpy().reshape(cap, -1)[:k])
        cfo.append(o["cfo_out"].cpu().numpy()[:k])
    for m in mods:
        m.close()
    return (np.concatenate(pbs), np.concatenate(byt), np.concatenate(cons), np.concatenate(cfo),
            sum(rx.rewalks for rx in rxs))


def check_frames(cfg, h, want, got, pick=None):
    pbs, byt, cons, cfo, _ = got
    assert np.array_equal(pbs, want)
    g = O.geometry(cfg)
    span = g["preamble_len"] + g["message_len"]
    for f in (range(len(want)) if pick is None else pick):
        c, oc, ob = O.decode_frame(cfg, h[want[f]: want[f] + span])
        assert cfo[f] == c
        assert np.array_equal(byt[f], ob)
        assert rel_err(cons[f], oc) < 1e-9


@pytest.fixture(scope="module")
def small():
    x, _ = impaired_stream(D, 90, seed=4)  # ~3 ring ends of the config's 40-frame ring
    return x, O.stream_walk_ring(D, x)[0]


@pytest.mark.parametrize("world", [2, 3, 5, 8])
def test_sharded_stream_equals_sequential_walk(small, world):
    x, want = small
    got = run_sharded(D, torch.from_numpy(x).cuda(), len(x), world)
    check_frames(D, x, want, got)


@pytest.mark.parametrize("halo", [0, 700, 4000])
def test_sharded_stream_short_halos_rewalk_exactly(small, halo):
    x, want = small
    got = run_sharded(D, torch.from_numpy(x).cuda(), len(x), 4, halo=halo)
    check_frames(D, x, want, got)
    if halo == 0:
        assert got[4] > 0  # no walk-in: later shards re-walk from their predecessor's exit state


def test_sharded_stream_int16_equals_f64(small):
    x, _ = small
    x16 = O.get_int16(x, D["mult"]).reshape(-1)
    h = x16.reshape(-1, 2).astype(np.float64)
    h = h[:, 0] + 1j * h[:, 1]
    want = O.stream_walk_ring(D, h)[0]
    got = run_sharded(D, torch.from_numpy(np.ascontiguousarray(x16)).cuda(), len(x), 3, i16=True)
    check_frames(D, h, want, got)


RB3 = dict(D, rx_buf_size=3)


@pytest.mark.parametrize("world,halo", [(3, None), (5, 0), (4, 2500)])
def test_sharded_stream_small_ring(world, halo):
    # a ring end every ~2.4 frames: shards start speculatively in ring
    # states, exit states carry the ring end, re-walks resume from them
    x, _ = impaired_stream(RB3, 40, seed=4)
    want = O.stream_walk_ring(RB3, x)[0]
    got = run_sharded(RB3, torch.from_numpy(x).cuda(), len(x), world, halo=halo)
    check_frames(RB3, x, want, got)


def test_sharded_stream_more_shards_than_frames():
    x, _ = impaired_stream(D, 3, seed=11)
    want = O.stream_walk_ring(D, x)[0]
    got = run_sharded(D, torch.from_numpy(x).cuda(), len(x), 8)
    check_frames(D, x, want, got)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_stream_bench_size_matches_oracle(world):
    """The bench's config-4 stream (ofdm_synth, 16 384 frames, ~132 M samples)
    split over 2/4/8 contexts: every owned index equals the oracle's sequential
    walk over the whole stream; every owned frame decodes as the oracle's
    main.cpp:60-80 chain (common.check_stream_frames)."""
    cfg = dict(O.DEFAULT)
    lay = Y.StreamLayout(cfg, 16384)
    m = M.Modem(cfg, 0)
    x = Y.stream_slice(m, lay, 0, lay.n, torch.device("cuda", 0))
    m.close()
    h = x.cpu().numpy()
    want = _bench_walk(h)
    got = run_sharded(cfg, x, lay.n, world, max_frames=None)
    k = len(want)
    assert k > 0.95 * 16384
    pbs, byt, cons, cfo, _ = got
    assert np.array_equal(pbs, want)
    summary = check_stream_frames(cfg, h, pbs, byt, cons, cfo)
    print(f"{world} shards: {summary}")


_WALK = {}


def _bench_walk(h):
    key = (len(h), float(h[12345].real))
    if key not in _WALK:
        _WALK.clear()
        _WALK[key] = O.stream_walk_ring(dict(O.DEFAULT), h)[0]
    return _WALK[key]
