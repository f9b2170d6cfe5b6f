"""Pin the oracle (oracle/ofdm_oracle.c) to the reference's golden files.

Fixtures: tests/golden/ (made by tests/golden/make_golden.py from the
reference's data/*.bin + data.txt: one BPSK main.cpp run, main.cpp:74-78,106-108).
"""
import numpy as np

import oracle as O
from common import G, golden, impaired_stream, rel_err

GD = golden()


def test_preamble_bytes_match_reference_run():
    # PREAMBLE_FORM ctor, Frame.cpp:269-272 (mt19937(42) + uniform_int_distribution<int>(0,255))
    assert list(O.preamble_bytes(G)) == GD["preamble_bytes"]


def test_tx_frame_regenerates_source_bin_bit_exact():
    # FRAME_FORM::write + get_int16 (Frame.cpp:235-256) of the golden payload == data/source.bin
    fr = O.frame_write(G, GD["payload"])
    i16 = O.get_int16(fr, G["mult"])
    assert np.array_equal(i16, GD["source"])


def test_t2_corr_matches_reference():
    corr = O.t2_corr(G, GD["data"])  # T2SIN_FORM::corr, Frame.hpp:96-147
    assert corr.shape == GD["t2_corr"].shape
    assert np.abs(corr - GD["t2_corr"]).max() < 1e-12
    assert list(np.nonzero(corr)[0]) == GD["t2_blocks"]


def _sync_chain(x, pos):
    """main.cpp:51-71 replay: t2 find, preamble find(+1), copy, sync, equalise."""
    t2 = O.find_t2sin(G, x, pos)
    pre, modp, templ = O.preamble_setup(G)
    pr = O.find_preamble(G, x, t2, templ) + 1
    g = O.geometry(G)
    frame = x[pr - G["t2sin_size"]: pr - G["t2sin_size"] + g["frame_len"]].copy()
    mwp = frame[G["t2sin_size"]:]
    cfo = O.pilot_freq_sinh(G, mwp[: g["preamble_len"]])
    mwp = O.freq_shift(mwp, cfo)
    mwp = O.cp_freq_sinh(G, mwp)
    mwp = O.pr_phase_sinh(mwp, pre)
    chan = O.chan_char_lq(G, mwp[: g["preamble_len"]], modp)
    cons = O.ofdm_fft(G, mwp[g["preamble_len"]:]) / np.tile(chan, G["num_symb"])
    return t2, pr, cfo, chan, cons


def test_rx_chain_frame1_matches_goldens():
    t2, pr, cfo, chan, cons = _sync_chain(GD["data"], 0)
    assert t2 == GD["t2_first_block_start"]
    assert pr == GD["preamble_begin"][0]
    assert cfo == GD["cfo_frame1"]
    assert np.abs(chan - GD["phases"]).max() < 1e-12                  # data/phases.bin
    assert rel_err(cons, GD["constell"]) < 1e-12                       # data/constell.bin
    assert np.abs(cons - GD["constell"]).max() / np.abs(GD["constell"]).min() < 1e-12
    b, _ = O.demod(1, cons)
    assert np.array_equal(b, GD["payload"])                             # data.txt + MAC header


def test_rx_chain_frame2_decodes():
    # second frame of the capture (rx.cpp streaming continues after the first)
    _, pr1, *_ = _sync_chain(GD["data"], 0)
    g = O.geometry(G)
    t2, pr, cfo, chan, cons = _sync_chain(GD["data"], pr1 + g["message_len"])
    assert pr == GD["preamble_begin"][1]
    b, _ = O.demod(1, cons)
    assert np.array_equal(b, GD["payload"])


def test_fft_is_the_dft_definition():
    rng = np.random.default_rng(1)
    for n in (8, 64, 256, 512, 640, 2048, 2560, 12, 17):
        x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
        assert rel_err(O.fft(x, -1), np.fft.fft(x)) < 1e-13
        assert rel_err(O.fft(x, +1), np.fft.ifft(x) * n) < 1e-13


def test_stream_walk_and_decode_match_reference_capture():
    """The rx.cpp:125-221 walk over data/data.bin finds both frames at the
    reference's preamble starts; the located-frame decode (main.cpp:60-80)
    reproduces cfo, constell.bin and data.txt."""
    pbs = O.stream_walk(G, GD["data"])
    assert list(pbs) == list(GD["preamble_begin"])
    g = O.geometry(G)
    span = g["preamble_len"] + g["message_len"]
    cfo, cons, out = O.decode_frame(G, GD["data"][pbs[0]: pbs[0] + span])
    assert cfo == GD["cfo_frame1"]
    assert rel_err(cons, GD["constell"]) < 1e-12
    assert np.array_equal(out, GD["payload"])
    _, _, out2 = O.decode_frame(G, GD["data"][pbs[1]: pbs[1] + span])
    assert np.array_equal(out2, GD["payload"])
    # a stream cut inside frame 2 yields frame 1 only; before frame 1's end, none
    assert list(O.stream_walk(G, GD["data"][: pbs[1] + span - 1])) == [pbs[0]]
    assert list(O.stream_walk(G, GD["data"][: pbs[0] + span - 1])) == []
    # rx.cpp's own loop over data.bin as its SDR stream (ring buffer, zero
    # header, 40-frame refills) and the ring walk's state form find the same two
    assert list(O.rx_app_walk(G, GD["data"])) == list(GD["preamble_begin"])
    assert list(O.stream_walk_ring(G, GD["data"])[0]) == list(GD["preamble_begin"])


def test_awgn_is_counter_based_and_thread_independent():
    x = np.zeros(100003, np.complex128)
    a = O.awgn(x, 0.5, seed=17, sample_offset=(1 << 32) - 50000)
    b = O.awgn(x, 0.5, seed=17, sample_offset=(1 << 32) - 50000, threads=4)
    assert np.array_equal(a, b)
    # a sub-range at its global offset is the same noise
    c = O.awgn(x[:1000], 0.5, seed=17, sample_offset=(1 << 32) - 50000 + 777)
    assert np.array_equal(c, a[777:1777])
    assert abs(np.mean(np.abs(a) ** 2) - 0.25) < 0.01


def test_decode_frames_batch_equals_single_frame_decode():
    # the batched (OpenMP) orc_decode_frames used by the full-stream GPU parity
    # tests is orc_decode_frame frame by frame
    x, _ = impaired_stream(O.DEFAULT, 12, seed=11)
    pbs = O.stream_walk(O.DEFAULT, x)
    assert len(pbs) >= 8
    cfo, cons, out = O.decode_frames(O.DEFAULT, x, pbs, threads=4)
    g = O.geometry(O.DEFAULT)
    span = g["preamble_len"] + g["message_len"]
    for f, pb in enumerate(pbs):
        c1, cons1, out1 = O.decode_frame(O.DEFAULT, x[pb:pb + span])
        assert cfo[f] == c1 and np.array_equal(cons[f], cons1) and np.array_equal(out[f], out1)
