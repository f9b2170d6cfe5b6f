"""Shared test helpers: golden fixtures, configs, seeded payloads."""
import json
import os

import numpy as np

import oracle as O

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden():
    with open(os.path.join(GOLDEN_DIR, "golden.json")) as f:
        meta = json.load(f)
    g = dict(meta)
    g["source"] = np.load(os.path.join(GOLDEN_DIR, "source_bin.npy"))
    g["data_i16"] = np.load(os.path.join(GOLDEN_DIR, "data_bin_i16.npz"))["iq"]  # interleaved complex<int16>
    d = g["data_i16"].astype(np.float64)
    g["data"] = d[0::2] + 1j * d[1::2]
    g["t2_corr"] = np.load(os.path.join(GOLDEN_DIR, "t2_sin_corr.npy"))
    g["phases"] = np.load(os.path.join(GOLDEN_DIR, "phases.npy"))
    g["constell"] = np.load(os.path.join(GOLDEN_DIR, "constell.npy"))
    with open(os.path.join(GOLDEN_DIR, "data_txt.bin"), "rb") as f:
        g["payload_text"] = np.frombuffer(f.read(), np.uint8)
    g["payload"] = np.concatenate([np.array(meta["mac_header"], np.uint8), g["payload_text"]])
    return g


def payload(nbytes: int, seed: int) -> np.ndarray:
    return np.random.default_rng(seed).integers(0, 256, nbytes, dtype=np.uint8)


def cfg(base: dict, **kw) -> dict:
    d = dict(base)
    d.update(kw)
    return d


# Configs used across tests (D default, G golden, B 2048/QPSK, C 4096/16-QAM)
D = O.DEFAULT
G = O.GOLDEN
B = O.CONFIG_B
CC = O.CONFIG_C
EXTRA = {
    "D_qam64": cfg(O.DEFAULT, mod_type=6),
    "D_qam256": cfg(O.DEFAULT, mod_type=8),
    "D_qpsk": cfg(O.DEFAULT, mod_type=2),
    "N1024_k4": cfg(O.DEFAULT, fft_size=1024, num_data_subc=512, num_pilot_subc=16, cp_size=256),
    "N256_k2": cfg(O.DEFAULT, fft_size=256, num_data_subc=128, num_pilot_subc=8, cp_size=64, mod_type=2),
    "N128_k4_s3": cfg(O.DEFAULT, fft_size=128, num_data_subc=64, num_pilot_subc=4, cp_size=16, num_symb=3),
    "N64_k1": cfg(O.DEFAULT, fft_size=64, num_data_subc=32, num_pilot_subc=4, cp_size=16, mod_type=1,
                  num_symb=2, pr_sin_len=64, t2sin_size=64, t2_sin_f1=5, t2_sin_f2=20, smooth=2),
    "D_s12_staged": cfg(O.DEFAULT, num_symb=12),
    "D_s1": cfg(O.DEFAULT, num_symb=1),
    "D_p2": cfg(O.DEFAULT, num_pilot_subc=2),
    "D_cp0": cfg(O.DEFAULT, cp_size=0),
    "D_p16": cfg(O.DEFAULT, num_pilot_subc=16),  # S*P = 128 > 64: rx_wide_kernel's phys broadcast
}
ALL_CONFIGS = {"D": D, "G": G, "B": B, "C": CC, **EXTRA}


def rel_err(a, b) -> float:
    a = np.asarray(a)
    b = np.asarray(b)
    if a.size == 0:
        return 0.0
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def impaired_stream(cfg, nf, seed, snr_db=20.0, cfo_max=0.004, gap_max=4096):
    """Config-4 stream: full frames (T2+preamble+message) with random 0..gap_max
    zero gaps, per-frame CFO U(-cfo_max, cfo_max) and phase, AWGN over all."""
    g = O.geometry(cfg)
    rng = np.random.default_rng(seed)
    data = payload(nf * g["bytes_per_frame"], seed)
    parts = [np.zeros(int(rng.integers(0, gap_max + 1)), np.complex128)]
    for f in range(nf):
        fr = O.frame_write(cfg, data[f * g["bytes_per_frame"]:(f + 1) * g["bytes_per_frame"]])
        n = np.arange(len(fr))
        fr = fr * np.exp(2j * np.pi * rng.uniform(-cfo_max, cfo_max) * n + 1j * rng.uniform(-np.pi, np.pi))
        parts += [fr, np.zeros(int(rng.integers(0, gap_max + 1)), np.complex128)]
    x = np.concatenate(parts)
    return O.awgn(x, 10 ** (-snr_db / 20), seed=seed), data


def capture_stream(cfg, nf, seed, gap_max=3000):
    """A wire capture as tx.cpp + the SDR stand-in make it (data/tx.bin
    layout): full frames in FRAME_FORM::get_int16 scaling (x mult), exact-zero
    silences of 0..gap_max samples between them (no noise), one frame_len of
    zeros at the end. Returns (complex128 samples, interleaved int16)."""
    g = O.geometry(cfg)
    rng = np.random.default_rng(seed)
    data = payload(nf * g["bytes_per_frame"], seed)
    parts = []
    for f in range(nf):
        fr = O.frame_write(cfg, data[f * g["bytes_per_frame"]:(f + 1) * g["bytes_per_frame"]])
        parts += [np.zeros((int(rng.integers(0, gap_max + 1)), 2), np.int16),
                  O.get_int16(fr, cfg["mult"]).reshape(-1, 2)]
    parts.append(np.zeros((g["frame_len"], 2), np.int16))
    x16 = np.ascontiguousarray(np.concatenate(parts).reshape(-1))
    w = x16.astype(np.float64)
    return w[0::2] + 1j * w[1::2], x16


def decision_thresholds(k):
    """Modulation::demod's cell edges on each axis (modulation.cpp:53-87)."""
    m = 1 << (k // 2)
    s1 = (m - 1) / 2.0
    return np.array([(j - 0.5) / s1 - 1.0 for j in range(1, m)])


def distance_to_threshold(k, pts):
    """Distance of each equalised point from the decision edge nearest to it
    (BPSK: the line re + im = 0; QAM: the clamped re / im cell edges)."""
    if k == 1:
        return np.abs(pts.real + pts.imag)
    th = decision_thresholds(k)
    dre = np.min(np.abs(np.clip(pts.real, -1, 1)[..., None] - th), axis=-1)
    dim = np.min(np.abs(np.clip(pts.imag, -1, 1)[..., None] - th), axis=-1)
    return np.minimum(dre, dim)


def check_stream_frames(cfg, x, pbs, got_bytes, got_cons, got_cfo=None, tol=1e-9, allow_flips=False):
    """Every located frame of a stream against the oracle's main.cpp:60-80
    chain on the same samples (orc_decode_frames): CFO exact, constellation
    within `tol` relative per frame, and every byte equal, except that a
    decision may differ where the oracle's own point lies within the rounding
    band of its threshold (twice the largest GPU-oracle point difference of
    the whole stream: the sync chain's transcendentals and the FFT round
    differently). With allow_flips False (the default) no
    decision may differ at all: north_star's bit-exact decisions. Returns a
    summary dict."""
    k = cfg["mod_type"]
    g = O.geometry(cfg)
    nf = len(pbs)
    ocfo, ocons, obytes = O.decode_frames(cfg, x, pbs)
    if got_cfo is not None:
        bad = np.nonzero(got_cfo != ocfo)[0]
        assert bad.size == 0, f"CFO differs on {bad.size} frames, first {bad[:8]}"
    scale = np.abs(ocons).max(axis=1)
    err = np.abs(got_cons - ocons).max(axis=1) / np.maximum(scale, 1e-300)
    assert err.max() < tol, f"constellation rel err {err.max():.2e} on frame {int(err.argmax())}"
    band = 2.0 * float(np.abs(got_cons - ocons).max())
    diff_frames = np.nonzero(np.any(got_bytes != obytes, axis=1))[0]
    flips, worst = 0, 0.0
    for f in diff_frames:
        bg = np.unpackbits(got_bytes[f])[:g["npts"] * k].reshape(-1, k)
        bo = np.unpackbits(obytes[f])[:g["npts"] * k].reshape(-1, k)
        pts = np.nonzero(np.any(bg != bo, axis=1))[0]
        d = distance_to_threshold(k, ocons[f][pts])
        flips += len(pts)
        worst = max(worst, float(d.max()))
        assert np.all(d <= band), (f"frame {f}: {len(pts)} decisions differ, farthest {d.max():.3e} "
                                   f"from its threshold (band {band:.3e})")
    assert allow_flips or flips == 0, f"{flips} decisions differ from the oracle on {diff_frames.size} frames"
    return {"frames": nf, "max_constellation_rel_err": float(err.max()), "band": band,
            "frames_with_flips": int(diff_frames.size), "decision_flips": flips,
            "farthest_flip_from_threshold": worst}
