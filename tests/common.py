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
