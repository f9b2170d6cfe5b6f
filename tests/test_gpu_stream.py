"""GPU parity of the streaming receiver (rx.cpp:94-221):
ofdm_rx_stream's chunk-parallel walk must locate exactly the frames of
rx.cpp's sequential walk over its SDR ring (oracle orc_stream_walk_ring,
itself pinned to rx.cpp's loop replayed on a real ring buffer in
tests/test_stream_shard.py), or of the continuous walk with the ring off
(orc_stream_walk), and decode each as main.cpp:60-80 (oracle
orc_decode_frame) — on the reference capture data/data.bin and on synthetic
impaired streams, for any chunking of the walk and any ring size."""
import ctypes as C

import numpy as np
import pytest

import oracle as O
from common import CC, B, D, G, capture_stream, golden, impaired_stream, payload, rel_err

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import ofdm_mi355x as M  # noqa: E402

_m = {}


def modem(cfg):
    key = repr(sorted(cfg.items()))
    if key not in _m:
        _m[key] = M.Modem(cfg, 0)
    return _m[key]


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


GD = golden()


def run_stream(cfg, x, max_frames=4096, chunk=0, tuning=None, ring=None):
    m = modem(cfg)
    if tuning:
        old = m.walk_tuning(**tuning)
        try:
            return run_stream(cfg, x, max_frames, chunk, ring=ring)
        finally:
            m.walk_tuning(**old)
    if ring is not None:
        old = m.stream_ring(ring)
        try:
            return run_stream(cfg, x, max_frames, chunk)
        finally:
            m.stream_ring(old)
    g = O.geometry(cfg)
    dx = dev(x)
    pbs = torch.full((max_frames,), -1, dtype=torch.int64, device="cuda")
    out = torch.zeros((max_frames * g["bytes_per_frame"],), dtype=torch.uint8, device="cuda")
    cons = torch.zeros((max_frames * g["npts"],), dtype=torch.complex128, device="cuda")
    cfo = torch.zeros((max_frames,), dtype=torch.float64, device="cuda")
    nf = m.rx_stream(dx, len(x), max_frames, pb_out=pbs, bytes_out=out, constell_out=cons, cfo_out=cfo,
                     chunk=chunk)
    k = min(nf, max_frames)
    assert torch.equal(dx, dev(x))  # the input stream is not modified
    return (nf, host(pbs)[:k], host(out).reshape(max_frames, -1)[:k], host(cons).reshape(max_frames, -1)[:k],
            host(cfo)[:k])


def want_walk(cfg, x, ring=None):
    """The oracle's walk: rx.cpp's ring (ring None: the config's R), or the
    continuous walk (ring 0)."""
    return O.stream_walk_ring(cfg, x, ring=ring)[0]


def frame_at(x, pb, span):
    """Samples [pb, pb + span) of the stream, zero before sample 0 (rx.cpp's
    ring header, rx.cpp:105-114) and past its end."""
    out = np.zeros(span, np.complex128)
    lo, hi = max(pb, 0), min(pb + span, len(x))
    if hi > lo:
        out[lo - pb:hi - pb] = x[lo:hi]
    return out


def check_against_oracle(cfg, x, got, ring=None):
    nf, pbs, out, cons, cfo = got
    want = want_walk(cfg, x, ring)
    assert nf == len(want)
    assert np.array_equal(pbs, want)
    g = O.geometry(cfg)
    span = g["preamble_len"] + g["message_len"]
    for f, pb in enumerate(want):
        c, oc, ob = O.decode_frame(cfg, frame_at(x, pb, span))
        assert cfo[f] == c
        assert rel_err(cons[f], oc) < 1e-9
        assert np.array_equal(out[f], ob)
    return want


def test_stream_replay_of_reference_capture():
    nf, pbs, out, cons, cfo = run_stream(G, GD["data"])
    assert nf == 2 and list(pbs) == list(GD["preamble_begin"])        # rx.cpp walk over data.bin
    assert np.array_equal(out[0], GD["payload"]) and np.array_equal(out[1], GD["payload"])
    assert cfo[0] == GD["cfo_frame1"]
    assert np.abs(cons[0] - GD["constell"]).max() / np.abs(GD["constell"]).max() < 1e-9  # constell.bin


@pytest.mark.parametrize("chunk", [0, 5000, 9000, 20000, 64000])
def test_stream_config4_matches_sequential_walk(chunk):
    x, data = impaired_stream(D, 40, seed=4)
    want = check_against_oracle(D, x, run_stream(D, x, chunk=chunk))
    assert len(want) >= 20  # the grid-relative T2 search misses some frames, as the reference does


def test_stream_continuous_walk_matches_oracle():
    # ring 0: the continuous walk over the stream held whole (orc_stream_walk)
    x, data = impaired_stream(D, 40, seed=4)
    for chunk in (0, 9000):
        got = run_stream(D, x, chunk=chunk, ring=0)
        want = check_against_oracle(D, x, got, ring=0)
        assert np.array_equal(want, O.stream_walk(D, x))


# rx.cpp's ring with 1-, 2- and 3-frame refills: a ring end every ~1-2 frames
# of the stream, so most steps meet a refill (misses that restart the grid,
# carries; rx_buf_size = 1, R = output_size, is the smallest ring a config makes)
RING_CFGS = [dict(D, rx_buf_size=2), dict(D, rx_buf_size=3), dict(D, rx_buf_size=1)]


@pytest.mark.parametrize("rcfg", RING_CFGS, ids=["rb2", "rb3", "rb1"])
@pytest.mark.parametrize("chunk", [0, 5000, 9000, 20000])
def test_stream_ring_walk_matches_rx_cpp_loop(rcfg, chunk):
    x, data = impaired_stream(rcfg, 40, seed=4)
    want = check_against_oracle(rcfg, x, run_stream(rcfg, x, chunk=chunk))
    assert np.array_equal(want, O.rx_app_walk(rcfg, x))  # rx.cpp's loop on a real ring buffer


@pytest.mark.parametrize("ring", [None, 0], ids=["ring", "continuous"])
@pytest.mark.parametrize("chunk", [0, 20000, 2000000])
def test_stream_wire_capture_with_exact_zero_gaps(ring, chunk):
    """A capture as tx.cpp writes it (int16 scaling, exact-zero silences, no
    noise): every zero T2 block is uncertain for the FP32 screen and goes to
    the FP64 evaluation, back to back with the screen's steps (the slot
    protocol of the T2 first hit is exercised on every step). f64 and int16
    input, whole-walker and chunked."""
    x, x16 = capture_stream(D, 120, seed=4)
    want = check_against_oracle(D, x, run_stream(D, x, chunk=chunk, max_frames=256, ring=ring), ring=ring)
    assert len(want) >= 110
    m = modem(D)
    old = m.stream_ring(ring) if ring is not None else None
    try:
        got = run_stream_i16(D, x16, max_frames=256, chunk=chunk)
    finally:
        if old is not None:
            m.stream_ring(old)
    assert got[0] == len(want) and np.array_equal(got[1], want)


@pytest.mark.parametrize("lookback", [0, 1], ids=["host_stitch", "lookback"])
@pytest.mark.parametrize("halo,ext", [(0, 0), (250, 0), (100, 2000)])
@pytest.mark.parametrize("chunk", [5000, 20000])
def test_stream_ring_short_halo_rewalks(halo, ext, chunk, lookback):
    # host stitching: re-walks from ring states (position and ring end) stay
    # exact; look-back: walks joined on ring states (the record's lag bit)
    rcfg = RING_CFGS[1]
    x, data = impaired_stream(rcfg, 40, seed=6, gap_max=6000)
    check_against_oracle(rcfg, x, run_stream(rcfg, x, chunk=chunk,
                                             tuning=dict(halo_milli=halo, ext_milli=ext, lookback=lookback)))


def test_stream_ring_validation_and_state():
    m = modem(D)
    g = O.geometry(D)
    assert m.stream_ring() == 40 * g["frame_len"] == O.ring_len(D)  # rx_buf_size * output_size
    assert m.initial_state() == (-g["frame_len"], 40 * g["frame_len"])
    for bad in (-1, g["frame_len"] - 1):
        with pytest.raises(M.OfdmError):
            m.stream_ring(bad)
    old = m.stream_ring(g["frame_len"])  # R = output_size (rx_buf_size = 1) is accepted
    m.stream_ring(old)
    old = m.stream_ring(0)
    assert m.initial_state() == (0, 0)
    m.stream_ring(old)


@pytest.mark.parametrize("lookback", [0, 1], ids=["host_stitch", "lookback"])
@pytest.mark.parametrize("halo,ext", [(0, 0), (100, 0), (250, 0), (500, 0), (100, 2000), (1500, 2000)])
@pytest.mark.parametrize("chunk", [0, 9000, 20000])
def test_stream_short_halo_rewalks_match_sequential_walk(halo, ext, chunk, lookback):
    # host stitching: walk-in halos (in 1/1000 frames) too short to meet the
    # true walk force re-walks from the previous chunk's hand-over state (with
    # or without the walk-on past the core end); look-back: any halo, the
    # walks join on the device. Still exact
    x, data = impaired_stream(D, 40, seed=4)
    check_against_oracle(D, x, run_stream(D, x, chunk=chunk,
                                          tuning=dict(halo_milli=halo, ext_milli=ext, lookback=lookback)))


@pytest.mark.parametrize("ring", [None, 0], ids=["ring", "continuous"])
@pytest.mark.parametrize("nf,chunk,halo", [(40, 1500, 0), (40, 2500, 0), (40, 6000, 0), (40, 13000, 0),
                                           (120, 300, 100)])
def test_stream_lookback_chain_across_chunks(nf, chunk, halo, ring):
    # look-back with chunks shorter than a frame (5 760 samples): most cores
    # hold no frame start, a walk joins a chunk several cores ahead, and the
    # chain resolution passes over chunks no walk joins (non-anchor chunks).
    # 120 frames in 300-sample chunks: more chunks than resident walkers, so
    # walkers wait on chunks taken from the queue after theirs. Every frame
    # against the oracle's walk
    x, data = impaired_stream(D, nf, seed=7, gap_max=6000)
    got = run_stream(D, x, chunk=chunk, ring=ring, tuning=dict(halo_milli=halo))
    check_against_oracle(D, x, got, ring=ring)


@pytest.mark.parametrize("ring", [None, 0], ids=["ring", "continuous"])
@pytest.mark.parametrize("cap,chunk", [(1, 9000), (2, 20000), (1, 20000)])
def test_stream_lookback_overflow_falls_back_to_halo_walk(cap, chunk, ring, monkeypatch, capfd):
    """A look-back walker whose records overflow (the test hook max_rec_cap
    shrinks its record buffer) makes the resolve kernel flag RESOLVE_OVERFLOW,
    write no list and a zero count (the speculative decode behind it then
    does nothing), and the host re-runs the call as the halo walk: every
    output equals the oracle's and the host-stitched run's. The next call
    with the normal bound runs on the same (now stale) walk scratch."""
    x, data = impaired_stream(D, 40, seed=5, gap_max=6000)
    monkeypatch.setenv("OFDM_STREAM_DEBUG", "1")
    got = run_stream(D, x, chunk=chunk, ring=ring, tuning=dict(max_rec_cap=cap))
    assert "look-back overflow" in capfd.readouterr().err  # the fallback branch ran
    check_against_oracle(D, x, got, ring=ring)
    halo = run_stream(D, x, chunk=chunk, ring=ring, tuning=dict(lookback=0))
    assert got[0] == halo[0]
    for a, b in zip(got[1:], halo[1:]):
        assert np.array_equal(a, b)
    again = run_stream(D, x, chunk=chunk, ring=ring)
    assert "look-back overflow" not in capfd.readouterr().err
    for a, b in zip(got, again):
        assert np.array_equal(a, b)


def test_stream_walk_certified_search_equals_serial_recurrence():
    # the walker's parallel preamble search (window sums + error bound) against
    # the reference's serial running-energy recurrence (ofdm_walk_tuning)
    x, data = impaired_stream(D, 40, seed=4)
    fast = run_stream(D, x, chunk=9000)
    exact = run_stream(D, x, chunk=9000, tuning=dict(exact_search=1))
    assert fast[0] == exact[0]
    for a, b in zip(fast[1:], exact[1:]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("tuning", [dict(t2_margin=1.0), dict(t2_f32=0), dict(t2_margin=0.0, allow_uncertified=1)])
def test_stream_walk_fp32_t2_screen_equals_fp64(tuning):
    # the walker's certified FP32 T2 screen against FP64 only: margin 1 makes
    # every block uncertain (each scan step re-evaluated by the FP64 path),
    # t2_f32 = 0 is the FP64 scan, margin 0 trusts the raw FP32 ratios
    # (still equal on this stream: no block within 1e-5 of the level)
    for cfg, nf, seed in ((D, 40, 4), (dict(D, fft_size=256, num_data_subc=128, num_pilot_subc=8, cp_size=64), 30, 6)):
        x, data = impaired_stream(cfg, nf, seed=seed)
        screened = run_stream(cfg, x, chunk=9000)
        other = run_stream(cfg, x, chunk=9000, tuning=tuning)
        assert screened[0] == other[0]
        for a, b in zip(screened[1:], other[1:]):
            assert np.array_equal(a, b)
        check_against_oracle(cfg, x, screened)


@pytest.mark.parametrize("ring", [None, 0], ids=["ring", "continuous"])
def test_stream_walk_fp32_preamble_tier_equals_fp64(ring):
    # the FFT preamble search's certified FP32 tier (pre_f32, the default)
    # against the FP64 search alone: the same walk and outputs, on impaired
    # streams and on a tx.cpp-style capture with exact-zero silences (windows
    # of tiny energy, where the FP32 bound leaves lags uncertain and the FP64
    # pass decides them)
    for cfg, x in ((D, impaired_stream(D, 40, seed=4)[0]), (D, capture_stream(D, 60, seed=5)[0])):
        tiered = run_stream(cfg, x, chunk=9000, ring=ring)
        fp64 = run_stream(cfg, x, chunk=9000, ring=ring, tuning=dict(pre_f32=0))
        assert tiered[0] == fp64[0]
        for a, b in zip(tiered[1:], fp64[1:]):
            assert np.array_equal(a, b)
        check_against_oracle(cfg, x, tiered, ring=ring)


def test_stream_calls_on_alternating_streams_one_context():
    # one ctx, stream calls issued on two HIP streams in turn without host
    # syncs between them: each call waits (on the device) for the previous
    # call's decode before rewriting the ctx's scratch, so every call's
    # outputs equal the serial call's (include/ofdm_mi355x.h stream rules)
    x, data = impaired_stream(D, 400, seed=11)
    mf = 512
    ref = run_stream(D, x, max_frames=mf)
    m = modem(D)
    g = O.geometry(D)
    dx = dev(x)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    bufs = [(torch.full((mf,), -1, dtype=torch.int64, device="cuda"),
             torch.zeros((mf * g["bytes_per_frame"],), dtype=torch.uint8, device="cuda"),
             torch.zeros((mf * g["npts"],), dtype=torch.complex128, device="cuda"),
             torch.zeros((mf,), dtype=torch.float64, device="cuda")) for _ in range(6)]
    torch.cuda.synchronize()  # input and zeroed outputs ready before either stream reads them
    outs = []
    for k, (pbs, out, cons, cfo) in enumerate(bufs):  # no host sync between the calls
        nf = m.rx_stream(dx, len(x), mf, pb_out=pbs, bytes_out=out, constell_out=cons, cfo_out=cfo,
                         stream=streams[k % 2])
        outs.append((nf, pbs, out, cons, cfo))
    torch.cuda.synchronize()
    for nf, pbs, out, cons, cfo in outs:
        k = min(nf, mf)
        assert nf == ref[0]
        assert np.array_equal(host(pbs)[:k], ref[1])
        assert np.array_equal(host(out).reshape(mf, -1)[:k], ref[2])
        assert np.array_equal(host(cons).reshape(mf, -1)[:k], ref[3])
        assert np.array_equal(host(cfo)[:k], ref[4])


def test_stream_two_contexts_concurrent_lookback_walks():
    # two contexts receiving on two HIP streams in turn, no host sync between
    # calls: one call's look-back walk runs beside the other context's decode,
    # so walkers of a grid are not all resident at once; a walker waits only on
    # chunks whose walker has started (WALK_PUB_STARTED), and every call's
    # outputs equal the serial call's
    x, _ = impaired_stream(D, 1200, seed=13)
    mf = 1536
    for chunk in (0, 6000):
        ref = run_stream(D, x, max_frames=mf, chunk=chunk)
        mods = [modem(D), M.Modem(D, 0)]
        g = O.geometry(D)
        dx = dev(x)
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        bufs = [(torch.full((mf,), -1, dtype=torch.int64, device="cuda"),
                 torch.zeros((mf * g["bytes_per_frame"],), dtype=torch.uint8, device="cuda"),
                 torch.zeros((mf * g["npts"],), dtype=torch.complex128, device="cuda")) for _ in range(6)]
        torch.cuda.synchronize()
        outs = []
        for k, (pbs, out, cons) in enumerate(bufs):
            nf = mods[k % 2].rx_stream(dx, len(x), mf, pb_out=pbs, bytes_out=out, constell_out=cons, chunk=chunk,
                                       stream=streams[k % 2])
            outs.append((nf, pbs, out, cons))
        torch.cuda.synchronize()
        mods[1].close()
        for nf, pbs, out, cons in outs:
            k = min(nf, mf)
            assert nf == ref[0]
            assert np.array_equal(host(pbs)[:k], ref[1])
            assert np.array_equal(host(out).reshape(mf, -1)[:k], ref[2])
            assert np.array_equal(host(cons).reshape(mf, -1)[:k], ref[3])


def test_stream_unfused_decode_path():
    # num_symb = 12 exceeds the rx register window, so the located frames take
    # the gather + staged sync chain + staged rx path instead of the fused decode
    cfg = dict(D, num_symb=12)
    x, data = impaired_stream(cfg, 12, seed=5)
    want = check_against_oracle(cfg, x, run_stream(cfg, x, chunk=20000))
    assert len(want) >= 6


def test_stream_config_b_and_payload_roundtrip():
    x, data = impaired_stream(B, 12, seed=9, snr_db=30.0, cfo_max=0.001)
    nf, pbs, out, cons, cfo = got = run_stream(B, x, chunk=30000)
    check_against_oracle(B, x, got)
    g = O.geometry(B)
    frames = data.reshape(12, g["bytes_per_frame"])
    assert nf >= 6 and all(any(np.array_equal(o, fr) for fr in frames) for o in out)


@pytest.mark.parametrize("name", ["B", "C"])
def test_stream_wide_fused_decode_matches_oracle_and_staged(name):
    # configs B / C (N = 2048 / 4096, cp = N/4): the located frames decode
    # through the fused wide kernel (ofdm_stream_wide.hip); staged_decode = 1
    # takes the cfo -> params -> rx kernels. Both against the oracle, every
    # frame (CFO and bytes exact, constellation 1e-9, no decision flips)
    cfg = {"B": B, "C": CC}[name]
    x, data = impaired_stream(cfg, 10, seed=21)
    fused = run_stream(cfg, x, chunk=40000)
    want = check_against_oracle(cfg, x, fused)
    staged = run_stream(cfg, x, chunk=40000, tuning=dict(staged_decode=1))
    check_against_oracle(cfg, x, staged)
    assert len(want) >= 5
    assert np.array_equal(fused[2], staged[2]) and np.array_equal(fused[4], staged[4])
    assert rel_err(fused[3], staged[3]) < 1e-9


WIDE_VARIANTS = {
    # N = 1024, cp = N/4: 1280-point CFO form of 5 x 256 (two CFO transforms
    # per wave, a dummy one on the third wave's spare lanes)
    "N1024": dict(B, fft_size=1024, num_data_subc=512, num_pilot_subc=16, cp_size=256),
    "N1024_qam16_s5": dict(B, fft_size=1024, num_data_subc=512, num_pilot_subc=16, cp_size=256, mod_type=4,
                           num_symb=5),
    "B_s3": dict(B, num_symb=3),                                   # odd S: group 1 idle in the last step
    "B_s5_qam16": dict(B, num_symb=5, mod_type=4),
    "B_d512_p16": dict(B, num_data_subc=512, num_pilot_subc=16),  # D < 4T, half = T
    "B_p64_s1": dict(B, num_pilot_subc=64, num_symb=1),           # one symbol, P = T/4
}


@pytest.mark.parametrize("name", list(WIDE_VARIANTS))
def test_stream_wide_fused_decode_geometry_variants(name):
    # the wide kernel's geometry bounds (S <= 8 with idle group steps, D <= 4T,
    # P <= T) on impaired streams, every frame against the oracle and the
    # staged kernels
    cfg = WIDE_VARIANTS[name]
    x, data = impaired_stream(cfg, 8, seed=23)
    fused = run_stream(cfg, x, chunk=40000)
    want = check_against_oracle(cfg, x, fused)
    staged = run_stream(cfg, x, chunk=40000, tuning=dict(staged_decode=1))
    assert len(want) >= 4
    assert np.array_equal(fused[1], staged[1]) and np.array_equal(fused[2], staged[2])
    assert np.array_equal(fused[4], staged[4]) and rel_err(fused[3], staged[3]) < 1e-9


@pytest.mark.parametrize("name,cfg", [("B_cp0", dict(B, cp_size=0)), ("D_cp0", dict(D, cp_size=0)),
                                      ("N1024_cp0", dict(B, fft_size=1024, num_data_subc=512, num_pilot_subc=16,
                                                         cp_size=0))])
def test_stream_cp_not_quarter_matches_oracle(name, cfg):
    # cp != N/4: a 2^a-point CFO form (no radix-5 combine), decoded by the
    # staged cfo -> params -> rx kernels; every located frame against the
    # oracle (CFO and bytes exact, constellation 1e-9, no decision flips)
    x, data = impaired_stream(cfg, 8, seed=25)
    want = check_against_oracle(cfg, x, run_stream(cfg, x, chunk=40000))
    assert len(want) >= 4


def test_stream_wide_fused_decode_i16_equals_f64():
    x, _ = impaired_stream(B, 10, seed=22)
    x16 = to_i16(x * 200.0)
    xd = x16[0::2].astype(np.float64) + 1j * x16[1::2].astype(np.float64)
    got = run_stream_i16(B, x16, chunk=40000)
    ref = run_stream(B, xd, chunk=40000)
    assert got[0] == ref[0] and got[0] >= 5
    for a, b in zip(got[1:], ref[1:4]):
        assert np.array_equal(a, b)
    check_against_oracle(B, xd, ref)


def test_stream_edges():
    g = O.geometry(D)
    # no frames: noise only, and a stream shorter than one T2 block
    noise = O.awgn(np.zeros(50000, np.complex128), 0.1, seed=1)
    assert run_stream(D, noise)[0] == 0
    assert run_stream(D, noise[:100])[0] == 0
    # max_frames truncates outputs but reports every frame found
    x, _ = impaired_stream(D, 10, seed=21)
    want = want_walk(D, x)
    nf, pbs, out, _, _ = run_stream(D, x, max_frames=3)
    assert nf == len(want) and np.array_equal(pbs, want[:3])
    # a stream cut inside the last frame drops it, as the walk stops there
    cut = want[-1] + g["preamble_len"] + g["message_len"] - 1
    nf2, pbs2, *_ = run_stream(D, x[:cut])
    assert np.array_equal(pbs2, want_walk(D, x[:cut])) and nf2 == len(want) - 1



@pytest.mark.parametrize("lookback", [1, 0], ids=["lookback", "host_stitch"])
@pytest.mark.parametrize("cut0", [3000, 700, 300, 120, 64, 1, 0, -1, -64, -200, -700, -3000])
def test_stream_capture_starting_inside_a_frame(cut0, lookback):
    # ring mode: a capture that starts cut0 samples before the first frame's
    # preamble start (inside its T2 marker for 0 < cut0 <= T2sin_size; inside
    # its preamble or message for cut0 < 0). rx.cpp walks from its ring's
    # zero header (rx.cpp:105-114), and a preamble search (rx.cpp:158-168)
    # that finds none moves on by a message; one that finds a preamble in the
    # header region (pb < 0) decodes that frame from the zeros. The stream API
    # locates the frames rx.cpp's loop replayed on a real ring buffer locates
    # (orc_rx_app_walk), and decodes each as the oracle does on the same
    # samples (zero before sample 0)
    x, _ = impaired_stream(D, 10, seed=21)
    first = int(want_walk(D, x)[0])
    y = x[max(0, first - cut0):]
    w = want_walk(D, y)
    assert np.array_equal(w, O.rx_app_walk(D, y))  # the state form is rx.cpp's loop
    check_against_oracle(D, y, run_stream(D, y, tuning=dict(lookback=lookback)))


def to_i16(x):
    """complex<double> -> interleaved complex<int16> (values already integral or rounded here)."""
    r = np.empty(2 * len(x), np.int16)
    r[0::2] = np.clip(np.round(x.real), -32768, 32767)
    r[1::2] = np.clip(np.round(x.imag), -32768, 32767)
    return r


def run_stream_i16(cfg, x16, max_frames=4096, chunk=0):
    m = modem(cfg)
    g = O.geometry(cfg)
    n = len(x16) // 2
    pbs = torch.full((max_frames,), -1, dtype=torch.int64, device="cuda")
    out = torch.zeros((max_frames * g["bytes_per_frame"],), dtype=torch.uint8, device="cuda")
    cons = torch.zeros((max_frames * g["npts"],), dtype=torch.complex128, device="cuda")
    nf = m.rx_stream_i16(dev(x16), n, max_frames, pb_out=pbs, bytes_out=out, constell_out=cons, chunk=chunk)
    k = min(nf, max_frames)
    return nf, host(pbs)[:k], host(out).reshape(max_frames, -1)[:k], host(cons).reshape(max_frames, -1)[:k]


def test_stream_i16_replays_reference_wire_capture():
    """data.bin as the SDR delivered it (complex<int16>): rx_stream_i16 fuses
    form_int16_to_double and equals the f64 path bit for bit."""
    nf, pbs, out, cons = run_stream_i16(G, GD["data_i16"])
    nf2, pbs2, out2, cons2, _ = run_stream(G, GD["data"])
    assert nf == nf2 == 2 and np.array_equal(pbs, pbs2) and list(pbs) == list(GD["preamble_begin"])
    assert np.array_equal(out, out2) and np.array_equal(cons, cons2)
    assert np.array_equal(out[0], GD["payload"])


def test_stream_i16_synthetic_equals_f64_path():
    x, _ = impaired_stream(D, 20, seed=8)
    x16 = to_i16(x * 200.0)  # the wire scaling of FRAME_FORM::get_int16 (mult)
    xd = x16[0::2].astype(np.float64) + 1j * x16[1::2].astype(np.float64)
    got = run_stream_i16(D, x16, chunk=7000)
    ref = run_stream(D, xd, chunk=7000)
    assert got[0] == ref[0] and got[0] >= 10
    for a, b in zip(got[1:], ref[1:4]):
        assert np.array_equal(a, b)
    check_against_oracle(D, xd, ref)


@pytest.mark.parametrize("name,cfg", [
    ("N1024", WIDE_VARIANTS["N1024"]),                    # the wide fused decode, N = 1024
    ("B_cp0", dict(B, cp_size=0)),                        # staged decode (ramp table), N = 2048
    ("D_cp0", dict(D, cp_size=0)),                        # staged decode, N = 512 (rx_stream2)
])
def test_stream_i16_equals_f64_path_other_geometries(name, cfg):
    # complex<int16> wire input through the decode kernels of the other
    # geometries (each instantiated per stream format): bit-identical to the
    # f64 path on the converted samples, which matches the oracle
    x, _ = impaired_stream(cfg, 8, seed=29)
    x16 = to_i16(x * 200.0)
    xd = x16[0::2].astype(np.float64) + 1j * x16[1::2].astype(np.float64)
    got = run_stream_i16(cfg, x16, chunk=40000)
    ref = run_stream(cfg, xd, chunk=40000)
    assert got[0] == ref[0] and got[0] >= 4
    for a, b in zip(got[1:], ref[1:4]):
        assert np.array_equal(a, b)
    check_against_oracle(cfg, xd, ref)


@pytest.mark.parametrize("name,cfg", [("B", B), ("D", D)])
def test_rx_i16_equals_rx_on_converted_samples(name, cfg):
    m = modem(cfg)
    g = O.geometry(cfg)
    nf = 64
    data = payload(nf * g["bytes_per_frame"], seed=5)
    d = dev(data)
    iq = torch.empty((nf * g["message_len"],), dtype=torch.complex128, device="cuda")
    iq16 = torch.empty((2 * nf * g["message_len"],), dtype=torch.int16, device="cuda")
    m.tx(d, nf, iq, iq16_out=iq16)  # FRAME_FORM::get_int16 wire samples
    conv = torch.complex(iq16[0::2].double(), iq16[1::2].double())
    outs = []
    for fn, src in ((m.rx_i16, iq16), (m.rx, conv)):
        cons = torch.zeros((nf * g["npts"],), dtype=torch.complex128, device="cuda")
        out = torch.zeros((nf * g["bytes_per_frame"],), dtype=torch.uint8, device="cuda")
        errs = torch.zeros((1,), dtype=torch.int64, device="cuda")
        fn(src, nf, constell_out=cons, bytes_out=out, ref=d, bit_errors=errs)
        outs.append((host(cons), host(out), int(host(errs)[0])))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    assert outs[0][2] == 0 and np.array_equal(outs[0][1], data)
    ocons, oout, _ = O.rx_batch(cfg, host(conv), nf, g["message_len"])
    assert rel_err(outs[0][0], ocons) < 1e-9 and np.array_equal(outs[0][1], oout)


def test_walk_tuning_defaults_and_validation():
    m = modem(D)
    t = M.WalkTuning()
    M.check(M.lib().ofdm_get_walk_tuning(m.h, C.byref(t)))
    assert (t.chunks_per_slot, t.halo_milli, t.ext_milli, t.exact_search, t.t2_f32) == (1, -1, 0, 0, 1)
    assert t.t2_margin == 4e-5 and t.lookback == 1
    with pytest.raises(M.OfdmError):
        m.walk_tuning(lookback=2)
    with pytest.raises(M.OfdmError):
        m.walk_tuning(halo_milli=-2)
    with pytest.raises(M.OfdmError):
        m.walk_tuning(chunks_per_slot=0)
    with pytest.raises(M.OfdmError):
        m.walk_tuning(t2_margin=-1.0)
    with pytest.raises(M.OfdmError, match="certified"):
        m.walk_tuning(t2_margin=1e-5)  # below the certified margin: refused in production
    m.walk_tuning(t2_margin=1e-5, allow_uncertified=1)  # the test-only switch
    assert t.staged_decode == 0
    with pytest.raises(M.OfdmError):
        m.walk_tuning(staged_decode=2)
    assert t.max_rec_cap == 0 and t.pre_f32 == 1
    with pytest.raises(M.OfdmError):
        m.walk_tuning(max_rec_cap=-1)
    with pytest.raises(M.OfdmError):
        m.walk_tuning(pre_f32=2)
    m.walk_tuning()  # back to the defaults


def test_stream_shard_margins_cover_python_sharding():
    # the Python shard planner (ofdm_stream.stream_halo/stream_tail) holds at
    # least what the library says a shard needs
    import ofdm_stream as SS
    for cfg in (D, B, G):
        halo, tail = modem(cfg).shard_margins()
        assert SS.stream_halo(cfg) >= halo
        assert SS.stream_tail(cfg) >= tail
