"""oracle.py — TEST INFRASTRUCTURE ONLY.

ctypes view of oracle/liboracle.so (the C restatement, ofdm_oracle.c) and of
oracle/_ref/libref.so (the reference's own modulation.cpp + parser.cpp, built
in this container only). Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module, and only as the checker / CPU baseline.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libref.so")

PARAM_FIELDS = [
    "fft_size", "num_data_subc", "num_pilot_subc", "cp_size", "num_symb", "num_pr_symb",
    "pr_sin_len", "pr_seed", "pr_level", "t2sin_size", "t2_sin_f1", "t2_sin_f2",
    "t2_sin_level", "smooth", "mod_type", "pilot_ampl", "mult", "rx_buf_size", "iterations",
]


class Params(C.Structure):
    _fields_ = [(f, C.c_long) for f in PARAM_FIELDS]

    @classmethod
    def make(cls, **kw) -> "Params":
        p = cls()
        for f in PARAM_FIELDS:
            setattr(p, f, int(kw.get(f, 0)))
        return p

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f in PARAM_FIELDS}


# config/config.txt as committed (reference config/config.txt:1-32)
DEFAULT = dict(fft_size=512, num_data_subc=256, num_pilot_subc=8, cp_size=128, num_symb=8,
               num_pr_symb=1, pr_sin_len=128, pr_seed=42, pr_level=500, t2sin_size=256,
               t2_sin_f1=17, t2_sin_f2=51, t2_sin_level=800, smooth=5, mod_type=4,
               pilot_ampl=2500, mult=200, rx_buf_size=40, iterations=10000)
GOLDEN = dict(DEFAULT, mod_type=1)           # the BPSK run that wrote data/*.bin
CONFIG_B = dict(DEFAULT, fft_size=2048, num_data_subc=1024, num_pilot_subc=32, cp_size=512,
                mod_type=2)
CONFIG_C = dict(DEFAULT, fft_size=4096, num_data_subc=2048, num_pilot_subc=64, cp_size=1024,
                mod_type=4)


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None
_ref = None

P_d = C.POINTER(C.c_double)
P_u8 = C.POINTER(C.c_uint8)
P_i16 = C.POINTER(C.c_int16)
P_int = C.POINTER(C.c_int)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        sz, i, d, l, v, u64 = C.c_size_t, C.c_int, C.c_double, C.c_long, None, C.c_ulonglong
        PP = C.POINTER(Params)
        sig = {
            "orc_constellation": (i, [i, P_d]),
            "orc_bit_convert": (sz, [i, i, P_u8, sz, P_u8]),
            "orc_mod": (sz, [i, P_u8, sz, P_d]),
            "orc_demod": (sz, [i, P_d, sz, P_u8]),
            "orc_layout": (v, [i, i, i, P_int, P_int]),
            "orc_fft": (v, [P_d, i, i]),
            "orc_fft_write": (v, [i, i, i, i, d, P_d, P_d]),
            "orc_fft_read": (v, [i, i, i, i, d, P_d, P_d]),
            "orc_ofdm_write": (v, [PP, i, i, P_u8, P_d]),
            "orc_ofdm_fft": (v, [PP, i, P_d, P_d]),
            "orc_ofdm_read": (sz, [PP, i, i, P_d, P_u8]),
            "orc_pilot_freq_sinh": (d, [PP, i, P_d]),
            "orc_freq_shift": (v, [P_d, l, d]),
            "orc_cp_freq_sinh": (v, [PP, i, P_d]),
            "orc_pr_phase_sinh": (v, [P_d, l, P_d, l]),
            "orc_t2_symbol": (v, [PP, P_d]),
            "orc_t2_mask": (v, [PP, P_d]),
            "orc_t2_corr": (v, [PP, P_d, l, P_d]),
            "orc_find_t2sin": (l, [PP, P_d, l, l]),
            "orc_preamble_bytes": (v, [PP, P_u8]),
            "orc_preamble_setup": (v, [PP, P_d, P_d, P_d]),
            "orc_find_preamble": (l, [PP, P_d, P_d, l, l]),
            "orc_chan_char_lq": (v, [PP, P_d, P_d, P_d]),
            "orc_frame_write": (v, [PP, P_u8, P_d]),
            "orc_get_int16": (v, [P_d, l, l, P_i16]),
            "orc_awgn": (v, [P_d, l, d, u64, u64]),
            "orc_awgn_mt": (v, [P_d, l, d, u64, u64, i]),
            "orc_rx_batch": (u64, [PP, P_d, l, l, P_d, P_u8, P_u8, i]),
            "orc_tx_batch": (v, [PP, P_u8, l, P_d, l, i]),
            "orc_decode_frame": (d, [PP, P_d, P_d, P_u8]),
            "orc_decode_frames": (v, [PP, P_d, C.POINTER(C.c_long), l, P_d, P_d, P_u8, i]),
            "orc_stream_walk": (l, [PP, P_d, l, C.POINTER(C.c_long), l]),
            "orc_stream_walk_ring": (l, [PP, P_d, l, l, l, l, l, C.POINTER(C.c_long), P_u8, l,
                                         C.POINTER(C.c_long), C.POINTER(C.c_long)]),
            "orc_rx_app_walk": (l, [PP, P_d, l, l, i, C.POINTER(C.c_long), l]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def ref_available() -> bool:
    return os.path.exists(REF_PATH)


def ref():
    """The reference's own modulation.cpp/parser.cpp (this container only)."""
    global _ref
    if _ref is None:
        if not ref_available():
            build()
        R = C.CDLL(REF_PATH)
        sz, i = C.c_size_t, C.c_int
        R.ref_constellation.restype = i
        R.ref_constellation.argtypes = [i, P_d]
        R.ref_mod.restype = sz
        R.ref_mod.argtypes = [i, P_u8, sz, P_d]
        R.ref_demod.restype = sz
        R.ref_demod.argtypes = [i, P_d, sz, P_u8]
        R.ref_bit_convert.restype = sz
        R.ref_bit_convert.argtypes = [i, i, P_u8, sz, P_u8]
        R.ref_parse_config.restype = i
        R.ref_parse_config.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_long)]
        R.ref_std_preamble_bytes.restype = None
        R.ref_std_preamble_bytes.argtypes = [C.c_long, C.c_long, P_u8]
        _ref = R
    return _ref


# ---------------------------------------------------------------- helpers
def _d(a: np.ndarray):
    assert a.flags.c_contiguous
    return a.ctypes.data_as(P_d)


def _u8(a: np.ndarray):
    assert a.flags.c_contiguous and a.dtype == np.uint8
    return a.ctypes.data_as(P_u8)


def P(params) -> Params:
    return params if isinstance(params, Params) else Params.make(**params)


def geometry(params) -> dict:
    p = P(params)
    N, cp, S = p.fft_size, p.cp_size, p.num_symb
    L = N + cp
    return dict(symbol_len=L, message_len=L * S, preamble_len=L * p.num_pr_symb,
                frame_len=p.t2sin_size + L * p.num_pr_symb + L * S,
                data_per_frame=p.num_data_subc * S,
                bytes_per_frame=p.num_data_subc * S * p.mod_type // 8,
                npts=(p.num_data_subc // p.num_pilot_subc) * p.num_pilot_subc * S)


def constellation(k: int) -> np.ndarray:
    out = np.zeros(1 << k, np.complex128)
    lib().orc_constellation(k, _d(out))
    return out


def bit_convert(out_bits: int, in_bits: int, data: np.ndarray) -> np.ndarray:
    data = np.ascontiguousarray(data, np.uint8)
    n = (len(data) * in_bits + out_bits - 1) // out_bits
    out = np.zeros(max(n, 1), np.uint8)
    m = lib().orc_bit_convert(out_bits, in_bits, _u8(data), len(data), _u8(out))
    return out[:m]


def mod(k: int, data: np.ndarray) -> np.ndarray:
    data = np.ascontiguousarray(data, np.uint8)
    n = (len(data) * 8 + k - 1) // k
    out = np.zeros(max(n, 1), np.complex128)
    m = lib().orc_mod(k, _u8(data), len(data), _d(out))
    return out[:m]


def demod(k: int, pts: np.ndarray):
    """Returns (bytes, clamped points) — demod clamps in place like the reference."""
    pts = np.array(pts, np.complex128, copy=True)
    out = np.zeros(max((len(pts) * k + 7) // 8, 1), np.uint8)
    m = lib().orc_demod(k, _d(pts), len(pts), _u8(out))
    return out[:m], pts


def fft(x: np.ndarray, sign: int = -1) -> np.ndarray:
    x = np.array(x, np.complex128, copy=True)
    lib().orc_fft(_d(x), len(x), sign)
    return x


def layout(N: int, D: int, P_: int):
    pil = np.zeros(P_, np.int32)
    seg = np.zeros(P_, np.int32)
    lib().orc_layout(N, D, P_, pil.ctypes.data_as(P_int), seg.ctypes.data_as(P_int))
    return pil, seg


def ofdm_write(params, data: np.ndarray, S: int | None = None, k: int | None = None):
    p = P(params)
    S = p.num_symb if S is None else S
    k = p.mod_type if k is None else k
    out = np.zeros((p.fft_size + p.cp_size) * S, np.complex128)
    data = np.ascontiguousarray(data, np.uint8)
    assert len(data) >= p.num_data_subc * S * k // 8
    lib().orc_ofdm_write(C.byref(p), S, k, _u8(data), _d(out))
    return out


def ofdm_fft(params, x: np.ndarray, S: int | None = None):
    p = P(params)
    S = p.num_symb if S is None else S
    x = np.ascontiguousarray(x, np.complex128)
    assert len(x) >= (p.fft_size + p.cp_size) * S
    out = np.zeros((p.num_data_subc // p.num_pilot_subc) * p.num_pilot_subc * S, np.complex128)
    lib().orc_ofdm_fft(C.byref(p), S, _d(x), _d(out))
    return out


def ofdm_read(params, x: np.ndarray, S: int | None = None, k: int | None = None):
    pts = ofdm_fft(params, x, S)
    p = P(params)
    return demod(p.mod_type if k is None else k, pts)[0]


def t2_symbol(params):
    p = P(params)
    out = np.zeros(p.t2sin_size, np.complex128)
    lib().orc_t2_symbol(C.byref(p), _d(out))
    return out


def t2_corr(params, x: np.ndarray):
    p = P(params)
    x = np.ascontiguousarray(x, np.complex128)
    out = np.zeros(len(x) // p.t2sin_size, np.float64)
    lib().orc_t2_corr(C.byref(p), _d(x), len(x), _d(out))
    return out


def find_t2sin(params, x: np.ndarray, start: int = 0) -> int:
    p = P(params)
    x = np.ascontiguousarray(x, np.complex128)
    return lib().orc_find_t2sin(C.byref(p), _d(x), len(x), start)


def preamble_bytes(params) -> np.ndarray:
    p = P(params)
    out = np.zeros(p.num_data_subc * p.num_pr_symb // 8, np.uint8)
    lib().orc_preamble_bytes(C.byref(p), _u8(out))
    return out


def preamble_setup(params):
    p = P(params)
    g = geometry(p)
    pre = np.zeros(g["preamble_len"], np.complex128)
    modp = np.zeros(p.num_data_subc * p.num_pr_symb, np.complex128)
    templ = np.zeros(p.pr_sin_len, np.complex128)
    lib().orc_preamble_setup(C.byref(p), _d(pre), _d(modp), _d(templ))
    return pre, modp, templ


def find_preamble(params, x: np.ndarray, start: int, templ=None) -> int:
    p = P(params)
    if templ is None:
        templ = preamble_setup(p)[2]
    x = np.ascontiguousarray(x, np.complex128)
    return lib().orc_find_preamble(C.byref(p), _d(templ), _d(x), len(x), start)


def pilot_freq_sinh(params, x: np.ndarray) -> float:
    p = P(params)
    x = np.ascontiguousarray(x, np.complex128)
    return lib().orc_pilot_freq_sinh(C.byref(p), p.num_pr_symb, _d(x))


def freq_shift(x: np.ndarray, shift: float) -> np.ndarray:
    x = np.array(x, np.complex128, copy=True)
    lib().orc_freq_shift(_d(x), len(x), shift)
    return x


def cp_freq_sinh(params, x: np.ndarray, S: int | None = None) -> np.ndarray:
    p = P(params)
    S = p.num_symb + p.num_pr_symb if S is None else S
    x = np.array(x, np.complex128, copy=True)
    lib().orc_cp_freq_sinh(C.byref(p), S, _d(x))
    return x


def pr_phase_sinh(x: np.ndarray, pr: np.ndarray) -> np.ndarray:
    x = np.array(x, np.complex128, copy=True)
    pr = np.ascontiguousarray(pr, np.complex128)
    lib().orc_pr_phase_sinh(_d(x), len(x), _d(pr), len(pr))
    return x


def chan_char_lq(params, pre_region: np.ndarray, mod_preamble=None) -> np.ndarray:
    p = P(params)
    if mod_preamble is None:
        mod_preamble = preamble_setup(p)[1]
    x = np.array(pre_region, np.complex128, copy=True)
    out = np.zeros(p.num_data_subc, np.complex128)
    lib().orc_chan_char_lq(C.byref(p), _d(x), _d(np.ascontiguousarray(mod_preamble)), _d(out))
    return out


def frame_write(params, data: np.ndarray) -> np.ndarray:
    p = P(params)
    out = np.zeros(geometry(p)["frame_len"], np.complex128)
    data = np.ascontiguousarray(data, np.uint8)
    lib().orc_frame_write(C.byref(p), _u8(data), _d(out))
    return out


def get_int16(x: np.ndarray, mult: int) -> np.ndarray:
    x = np.ascontiguousarray(x, np.complex128)
    out = np.zeros(2 * len(x), np.int16)
    lib().orc_get_int16(_d(x), len(x), mult, out.ctypes.data_as(P_i16))
    return out


def awgn(x: np.ndarray, noise_std: float, seed: int, sample_offset: int = 0, threads: int = 1) -> np.ndarray:
    x = np.array(x, np.complex128, copy=True)
    lib().orc_awgn_mt(_d(x), len(x), noise_std, seed, sample_offset, threads)
    return x


def rx_batch(params, iq: np.ndarray, nframes: int, frame_stride: int, ref=None, threads=1,
             want_constell=True):
    p = P(params)
    g = geometry(p)
    iq = np.ascontiguousarray(iq, np.complex128)
    assert len(iq) >= (nframes - 1) * frame_stride + g["message_len"]
    cons = np.zeros(nframes * g["npts"], np.complex128) if want_constell else None
    out = np.zeros(nframes * g["bytes_per_frame"], np.uint8)
    refp = _u8(np.ascontiguousarray(ref, np.uint8)) if ref is not None else None
    errs = lib().orc_rx_batch(C.byref(p), _d(iq), nframes, frame_stride,
                              _d(cons) if cons is not None else None, _u8(out), refp, threads)
    return cons, out, int(errs)


def tx_batch(params, data: np.ndarray, nframes: int, frame_stride: int | None = None, threads=1):
    p = P(params)
    g = geometry(p)
    stride = g["message_len"] if frame_stride is None else frame_stride
    out = np.zeros((nframes - 1) * stride + g["message_len"], np.complex128)
    data = np.ascontiguousarray(data, np.uint8)
    assert len(data) >= nframes * g["bytes_per_frame"]
    lib().orc_tx_batch(C.byref(p), _u8(data), nframes, _d(out), stride, threads)
    return out


def decode_frame(params, region: np.ndarray):
    """main.cpp:60-80 on one [preamble | message] region -> (cfo, constell, bytes)."""
    p = P(params)
    g = geometry(p)
    region = np.ascontiguousarray(region, np.complex128)
    assert len(region) >= g["preamble_len"] + g["message_len"]
    cons = np.zeros(g["npts"], np.complex128)
    out = np.zeros(g["bytes_per_frame"], np.uint8)
    cfo = lib().orc_decode_frame(C.byref(p), _d(region), _d(cons), _u8(out))
    return cfo, cons, out


def decode_frames(params, x: np.ndarray, pbs, threads: int = 0):
    """decode_frame on every located frame x[pbs[f]:...] (OpenMP over frames;
    threads 0 = os.cpu_count()) -> (cfo (nf,), constell (nf, npts), bytes (nf, bpf))."""
    import os
    p = P(params)
    g = geometry(p)
    x = np.ascontiguousarray(x, np.complex128)
    pbs = np.ascontiguousarray(pbs, np.int64)
    nf = len(pbs)
    assert nf == 0 or (pbs.min() >= 0 and pbs.max() + g["preamble_len"] + g["message_len"] <= len(x))
    cfo = np.zeros(nf, np.float64)
    cons = np.zeros((nf, g["npts"]), np.complex128)
    out = np.zeros((nf, g["bytes_per_frame"]), np.uint8)
    lib().orc_decode_frames(C.byref(p), _d(x), pbs.ctypes.data_as(C.POINTER(C.c_long)), nf, _d(cfo), _d(cons),
                            _u8(out), threads or os.cpu_count() or 1)
    return cfo, cons, out


def stream_walk(params, x: np.ndarray, max_frames: int = 1 << 20) -> np.ndarray:
    """rx.cpp:125-221 detection walk over a contiguous stream -> preamble starts."""
    p = P(params)
    x = np.ascontiguousarray(x, np.complex128)
    out = np.zeros(max_frames, np.int64)
    nf = lib().orc_stream_walk(C.byref(p), _d(x), len(x), out.ctypes.data_as(C.POINTER(C.c_long)), max_frames)
    return out[:nf].copy()


def ring_len(params) -> int:
    """rx.cpp's SDR refill size R = rx_buf_size * output_size (sdr.hpp:141,
    rx.cpp:53): 0 when rx_buf_size is 0 (no ring: the continuous walk)."""
    p = P(params)
    return p.rx_buf_size * geometry(p)["frame_len"]


def stream_walk_ring(params, x: np.ndarray, ring: int | None = None, start: int | None = None,
                     ring_end: int | None = None, own_hi: int | None = None, max_frames: int = 1 << 20,
                     with_lags: bool = False):
    """rx.cpp's detection walk WITH its SDR ring, in stream coordinates
    (orc_stream_walk_ring): ring = R (None: the config's; 0: the continuous
    walk), start state (start, ring_end) (None: rx.cpp's initial state
    (-output_size, R)), stop at the first state at or past own_hi (None: the
    stream end). Returns (pbs, (exit_pos, exit_ring_end)), or (pbs, lags,
    exit) with_lags."""
    p = P(params)
    R = ring_len(p) if ring is None else ring
    out_len = geometry(p)["frame_len"]
    if start is None:
        start = -out_len if R else 0
    if ring_end is None:
        ring_end = R
    x = np.ascontiguousarray(x, np.complex128)
    n = len(x)
    out = np.zeros(max_frames, np.int64)
    lag = np.zeros(max_frames, np.uint8)
    ex, exr = C.c_long(), C.c_long()
    nf = lib().orc_stream_walk_ring(C.byref(p), _d(x), n, R, start, ring_end, n if own_hi is None else own_hi,
                                    out.ctypes.data_as(C.POINTER(C.c_long)), _u8(lag), max_frames, C.byref(ex),
                                    C.byref(exr))
    m = min(nf, max_frames)
    if with_lags:
        return out[:m].copy(), lag[:m].copy(), (ex.value, exr.value)
    return out[:m].copy(), (ex.value, exr.value)


def rx_app_walk(params, x: np.ndarray, iterations: int = 0, stop_at_end: bool = True,
                max_frames: int = 1 << 20) -> np.ndarray:
    """rx.cpp:94-198 replayed on a real ring buffer (orc_rx_app_walk): the
    frames its loop locates in `iterations` iterations (0: until the capture
    is used up) from the SDR stream x (zeros past its end), as stream
    positions."""
    p = P(params)
    x = np.ascontiguousarray(x, np.complex128)
    out = np.zeros(max_frames, np.int64)
    nf = lib().orc_rx_app_walk(C.byref(p), _d(x), len(x), iterations, int(stop_at_end),
                               out.ctypes.data_as(C.POINTER(C.c_long)), max_frames)
    return out[:min(nf, max_frames)].copy()
