"""ofdm_mi355x — Python view of the C-ABI in include/ofdm_mi355x.h.

Thin ctypes binding over c-ofdm_amd/lib/libofdm_mi355x.so for tests and
bench.py. Device buffers are torch tensors on cuda (PyTorch is plumbing here:
HBM allocation, streams, events, torch.distributed); every compute call goes
through the HIP kernels of the shared library. There is no CPU fallback: if
the library is missing, import of `lib()` raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
# OFDM_MI355X_LIB: an alternative build of the same library (kernel A/B experiments)
LIB_PATH = os.environ.get("OFDM_MI355X_LIB") or os.path.join(PKG, "lib", "libofdm_mi355x.so")
HEADER = os.path.join(os.path.dirname(PKG), "include", "ofdm_mi355x.h")

PARAM_FIELDS = [
    "fft_size", "num_data_subc", "num_pilot_subc", "cp_size", "num_symb", "num_pr_symb",
    "pr_sin_len", "pr_seed", "pr_level", "t2sin_size", "t2_sin_f1", "t2_sin_f2",
    "t2_sin_level", "smooth", "mod_type", "pilot_ampl", "mult", "rx_buf_size", "iterations",
]

OFDM_OK = 0
ERRORS = {-1: "INVALID", -2: "UNSUPPORTED", -3: "HIP", -4: "IO", -5: "NOMEM", -6: "PARSE"}
SYNC_CFO, SYNC_FREQ_SHIFT, SYNC_CP, SYNC_PHASE, SYNC_CHAN, SYNC_ALL = 1, 2, 4, 8, 16, 31


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


class Geometry(C.Structure):
    _fields_ = [("symbol_len", C.c_long), ("message_len", C.c_long), ("preamble_len", C.c_long),
                ("frame_len", C.c_long), ("ring_len", C.c_long), ("data_per_frame", C.c_long),
                ("bytes_per_frame", C.c_long), ("segment_size", C.c_long),
                ("pilot_bin", C.c_long * 256), ("segment_bin", C.c_long * 256)]


class Channel(C.Structure):
    _fields_ = [("noise_std", C.c_double), ("seed", C.c_ulonglong), ("sample_offset", C.c_ulonglong)]


class WalkTuning(C.Structure):
    """ofdm_walk_tuning: per-context stream walker settings (tests, experiments)."""
    _fields_ = [("chunks_per_slot", C.c_long), ("halo_milli", C.c_long), ("ext_milli", C.c_long),
                ("exact_search", C.c_int), ("t2_f32", C.c_int), ("t2_margin", C.c_double),
                ("allow_uncertified", C.c_int), ("staged_decode", C.c_int), ("lookback", C.c_int),
                ("max_rec_cap", C.c_int), ("pre_f32", C.c_int)]


class WalkState(C.Structure):
    """ofdm_walk_state: (pos, ring_end) of the stream walk."""
    _fields_ = [("pos", C.c_long), ("ring_end", C.c_long)]


class OfdmError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ofdm error {code} ({ERRORS.get(code, '?')}): {msg}")
        self.code = code


# Every symbol include/ofdm_mi355x.h declares, with its ctypes signature.
_V, _I, _L, _SZ, _D = C.c_void_p, C.c_int, C.c_long, C.c_size_t, C.c_double
_PP = C.POINTER(Params)
SIGNATURES = {
    "ofdm_last_error": (C.c_char_p, []),
    "ofdm_abi_version": (_I, []),
    "ofdm_params_default": (_I, [_PP]),
    "ofdm_params_from_config": (_I, [C.c_char_p, _PP]),
    "ofdm_config_lookup": (_I, [C.c_char_p, C.c_char_p, C.POINTER(C.c_long)]),
    "ofdm_create": (_I, [_PP, _I, C.POINTER(_V)]),
    "ofdm_destroy": (_I, [_V]),
    "ofdm_get_geometry": (_I, [_V, C.POINTER(Geometry)]),
    "ofdm_get_t2_symbol": (_I, [_V, _V]),
    "ofdm_get_preamble": (_I, [_V, _V, _V, _V, _V]),
    "ofdm_device_alloc": (_I, [_V, _SZ, C.POINTER(_V)]),
    "ofdm_device_free": (_I, [_V, _V]),
    "ofdm_memcpy_h2d": (_I, [_V, _V, _V, _SZ, _V]),
    "ofdm_memcpy_d2h": (_I, [_V, _V, _V, _SZ, _V]),
    "ofdm_copy": (_I, [_V, _V, _V, _SZ, _V]),
    "ofdm_rx_demod_read": (_I, [_V, _V, _SZ, _SZ, _V, _SZ, _V, _V, _V, _V]),
    "ofdm_memset_device": (_I, [_V, _V, _I, _SZ, _V]),
    "ofdm_stream_synchronize": (_I, [_V, _V]),
    "ofdm_tx_modulate": (_I, [_V, _V, _SZ, _V, _SZ, _V, C.POINTER(Channel), _V]),
    "ofdm_tx_frames": (_I, [_V, _V, _SZ, _V, _V, _V]),
    "ofdm_rx_demod": (_I, [_V, _V, _SZ, _SZ, _V, _SZ, _V, _V, _V, _V, _V]),
    "ofdm_rx_demod_i16": (_I, [_V, _V, _SZ, _SZ, _V, _SZ, _V, _V, _V, _V, _V]),
    "ofdm_demap": (_I, [_V, _V, _SZ, _V, _V]),
    "ofdm_map": (_I, [_V, _V, _SZ, _V, _V]),
    "ofdm_fft_write": (_I, [_V, _V, _SZ, _V, _V]),
    "ofdm_fft_read": (_I, [_V, _V, _SZ, _V, _V]),
    "ofdm_bit_convert": (_I, [_V, _V, _SZ, _I, _I, _V, C.POINTER(_SZ), _V]),
    "ofdm_int16_to_double": (_I, [_V, _V, _SZ, _V, _V]),
    "ofdm_double_to_int16": (_I, [_V, _V, _SZ, _V, _V]),
    "ofdm_preamble_corr": (_I, [_V, _V, _SZ, _L, _V, _V]),
    "ofdm_t2_scan": (_I, [_V, _V, _SZ, _L, _V, _V, _V]),
    "ofdm_find_preamble": (_I, [_V, _V, _SZ, _V, _SZ, _V, _V]),
    "ofdm_cfo_estimate": (_I, [_V, _V, _SZ, _SZ, _I, _V, _V]),
    "ofdm_freq_shift": (_I, [_V, _V, _SZ, _SZ, _SZ, _V, _V]),
    "ofdm_cp_sync": (_I, [_V, _V, _SZ, _SZ, _I, _V]),
    "ofdm_phase_sync": (_I, [_V, _V, _SZ, _SZ, _SZ, _V, _SZ, _V]),
    "ofdm_sync_chain": (_I, [_V, _V, _SZ, _SZ, _SZ, _I, _V, _V, _V, _V, _SZ, _V]),
    "ofdm_chan_estimate": (_I, [_V, _V, _SZ, _SZ, _V, _SZ, _V]),
    "ofdm_sync_frames": (_I, [_V, _V, _SZ, _SZ, _I, _V, _V, _V, _V]),
    "ofdm_rx_stream": (_I, [_V, _V, _SZ, _SZ, _L, _V, _V, _V, _V, C.POINTER(_SZ), _V]),
    "ofdm_rx_stream_i16": (_I, [_V, _V, _SZ, _SZ, _L, _V, _V, _V, _V, C.POINTER(_SZ), _V]),
    "ofdm_rx_stream_shard": (_I, [_V, _V, _V, _SZ, C.POINTER(WalkState), _L, _L, _SZ, _L, _V, _V, _V, _V,
                                  C.POINTER(_SZ), _V, _V, _SZ, C.POINTER(_SZ), C.POINTER(WalkState), _V]),
    "ofdm_stream_initial_state": (_I, [_V, C.POINTER(WalkState)]),
    "ofdm_set_stream_ring": (_I, [_V, _L]),
    "ofdm_get_stream_ring": (_I, [_V, C.POINTER(_L)]),
    "ofdm_set_stream_timing": (_I, [_V, _I]),
    "ofdm_get_stream_timing": (_I, [_V, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    "ofdm_stream_shard_margins": (_I, [_V, C.POINTER(_L), C.POINTER(_L)]),
    "ofdm_host_alloc": (_I, [_V, _SZ, C.POINTER(_V)]),
    "ofdm_host_free": (_I, [_V, _V]),
    "ofdm_stream_create": (_I, [_V, C.POINTER(_V)]),
    "ofdm_stream_destroy": (_I, [_V, _V]),
    "ofdm_memcpy_d2d": (_I, [_V, _V, _V, _SZ, _V]),
    "ofdm_event_create": (_I, [_V, C.POINTER(_V)]),
    "ofdm_event_record": (_I, [_V, _V, _V]),
    "ofdm_event_synchronize": (_I, [_V, _V]),
    "ofdm_event_destroy": (_I, [_V, _V]),
    "ofdm_walk_tuning_default": (_I, [C.POINTER(WalkTuning)]),
    "ofdm_get_walk_tuning": (_I, [_V, C.POINTER(WalkTuning)]),
    "ofdm_set_walk_tuning": (_I, [_V, C.POINTER(WalkTuning)]),
    "ofdm_shard_range": (_I, [_SZ, _I, _I, C.POINTER(_SZ), C.POINTER(_SZ)]),
    "ofdm_stream_shard_plan": (_I, [_PP, _SZ, _I, _I, C.POINTER(_L), C.POINTER(_L), C.POINTER(_L), C.POINTER(_L)]),
    "ofdm_reduce_counters": (_I, [_V, _V, _SZ, _V, _V]),
    "ofdm_device_count": (_I, [C.POINTER(_I)]),
    "ofdm_stream_report_pack": (_I, [_I, _L, _L, _L, _V, _V, _SZ, C.POINTER(WalkState), _I, _SZ, _V]),
    "ofdm_stream_stitch_plan": (_I, [_V, _I, _SZ, _L, C.POINTER(_I), C.POINTER(WalkState)]),
}

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", PKG, "-j8"], check=True)


def lib():
    """Load the HIP shared library (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} missing: run `make -C c-ofdm_amd` (no CPU fallback exists)")
        L = C.CDLL(LIB_PATH)
        variant = "OFDM_MI355X_LIB" in os.environ  # an A/B build of an older tree may lack newer entries
        for name, (res, args) in SIGNATURES.items():
            if variant and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != OFDM_OK:
        raise OfdmError(rc, lib().ofdm_last_error().decode())


def params_default() -> Params:
    p = Params()
    check(lib().ofdm_params_default(C.byref(p)))
    return p


def params_from_config(path: str) -> Params:
    p = Params()
    check(lib().ofdm_params_from_config(path.encode(), C.byref(p)))
    return p


def config_lookup(path: str, key: str) -> int:
    v = C.c_long()
    check(lib().ofdm_config_lookup(path.encode(), key.encode(), C.byref(v)))
    return v.value


def _ptr(t):
    """Device (or host numpy) pointer of a tensor/array, or None."""
    if t is None:
        return None
    if hasattr(t, "data_ptr"):
        return t.data_ptr()
    return t.ctypes.data


def _stream(stream):
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    return stream if isinstance(stream, int) else stream.cuda_stream


class Modem:
    """One ofdm_ctx: the FRAME_FORM constants for a config on one GPU."""

    def __init__(self, params, device: int = 0):
        if isinstance(params, dict):
            params = Params.make(**params)
        self.params = params
        self.device = device
        h = C.c_void_p()
        check(lib().ofdm_create(C.byref(params), device, C.byref(h)))
        self.h = h
        g = Geometry()
        check(lib().ofdm_get_geometry(h, C.byref(g)))
        self.geo = g

    def close(self):
        if getattr(self, "h", None):
            lib().ofdm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- constants
    def t2_symbol(self):
        import numpy as np
        out = np.zeros(self.params.t2sin_size, np.complex128)
        check(lib().ofdm_get_t2_symbol(self.h, out.ctypes.data))
        return out

    def preamble(self):
        import numpy as np
        p = self.params
        b = np.zeros(p.num_data_subc * p.num_pr_symb // 8, np.uint8)
        pre = np.zeros(self.geo.preamble_len, np.complex128)
        modp = np.zeros(p.num_data_subc * p.num_pr_symb, np.complex128)
        tpl = np.zeros(p.pr_sin_len, np.complex128)
        check(lib().ofdm_get_preamble(self.h, b.ctypes.data, pre.ctypes.data, modp.ctypes.data,
                                      tpl.ctypes.data))
        return b, pre, modp, tpl

    # ---- compute (device tensors)
    def tx(self, data, nframes: int, iq_out, frame_stride: int | None = None, iq16_out=None,
           noise_std: float = 0.0, seed: int = 0, sample_offset: int = 0, stream=None):
        stride = self.geo.message_len if frame_stride is None else frame_stride
        ch = Channel(noise_std, seed, sample_offset) if noise_std > 0 else None
        check(lib().ofdm_tx_modulate(self.h, _ptr(data), nframes, _ptr(iq_out), stride,
                                     _ptr(iq16_out), C.byref(ch) if ch else None, _stream(stream)))

    def tx_frames(self, data, nframes: int, frames_out, frames16_out=None, stream=None):
        check(lib().ofdm_tx_frames(self.h, _ptr(data), nframes, _ptr(frames_out), _ptr(frames16_out),
                                   _stream(stream)))

    def rx(self, iq, nframes: int, frame_stride: int | None = None, chan=None, chan_stride: int = 0,
           constell_out=None, bytes_out=None, ref=None, bit_errors=None, stream=None):
        stride = self.geo.message_len if frame_stride is None else frame_stride
        check(lib().ofdm_rx_demod(self.h, _ptr(iq), nframes, stride, _ptr(chan), chan_stride,
                                  _ptr(constell_out), _ptr(bytes_out), _ptr(ref), _ptr(bit_errors),
                                  _stream(stream)))

    def rx_read(self, iq, nframes: int, chan, read_out, frame_stride: int | None = None, chan_stride: int = 0,
                constell_out=None, bytes_out=None, stream=None):
        """ofdm_rx_demod_read: rx with a channel divisor that also writes
        FFT_FORM::read's points before the division."""
        stride = self.geo.message_len if frame_stride is None else frame_stride
        check(lib().ofdm_rx_demod_read(self.h, _ptr(iq), nframes, stride, _ptr(chan), chan_stride, _ptr(read_out),
                                       _ptr(constell_out), _ptr(bytes_out), _stream(stream)))

    def copy(self, dst, src, nbytes: int, stream=None):
        """ofdm_copy: a kernel copy on the stream (device or page-locked memory)."""
        check(lib().ofdm_copy(self.h, _ptr(dst), _ptr(src), nbytes, _stream(stream)))

    def rx_i16(self, iq16, nframes: int, frame_stride: int | None = None, chan=None, chan_stride: int = 0,
               constell_out=None, bytes_out=None, ref=None, bit_errors=None, stream=None):
        """rx on complex<int16> wire samples (frame_stride in complex samples)."""
        stride = self.geo.message_len if frame_stride is None else frame_stride
        check(lib().ofdm_rx_demod_i16(self.h, _ptr(iq16), nframes, stride, _ptr(chan), chan_stride,
                                      _ptr(constell_out), _ptr(bytes_out), _ptr(ref), _ptr(bit_errors),
                                      _stream(stream)))

    def demap(self, points, n: int, bytes_out, stream=None):
        check(lib().ofdm_demap(self.h, _ptr(points), n, _ptr(bytes_out), _stream(stream)))

    def map(self, data, nbytes: int, points_out, stream=None):
        check(lib().ofdm_map(self.h, _ptr(data), nbytes, _ptr(points_out), _stream(stream)))

    def fft_write(self, points, nframes: int, fft_buf, stream=None):
        check(lib().ofdm_fft_write(self.h, _ptr(points), nframes, _ptr(fft_buf), _stream(stream)))

    def fft_read(self, fft_buf, nframes: int, restored, stream=None):
        check(lib().ofdm_fft_read(self.h, _ptr(fft_buf), nframes, _ptr(restored), _stream(stream)))

    def bit_convert(self, data, n: int, in_bits: int, out_bits: int, out, stream=None) -> int:
        m = C.c_size_t()
        check(lib().ofdm_bit_convert(self.h, _ptr(data), n, in_bits, out_bits, _ptr(out), C.byref(m),
                                     _stream(stream)))
        return m.value

    def int16_to_double(self, iq16, n: int, out, stream=None):
        check(lib().ofdm_int16_to_double(self.h, _ptr(iq16), n, _ptr(out), _stream(stream)))

    def double_to_int16(self, iq, n: int, out16, stream=None):
        check(lib().ofdm_double_to_int16(self.h, _ptr(iq), n, _ptr(out16), _stream(stream)))

    def preamble_corr(self, iq, n: int, start: int, cor_out, stream=None):
        check(lib().ofdm_preamble_corr(self.h, _ptr(iq), n, start, _ptr(cor_out), _stream(stream)))

    def t2_scan(self, iq, n: int, start: int, rel_out=None, first_out=None, stream=None):
        check(lib().ofdm_t2_scan(self.h, _ptr(iq), n, start, _ptr(rel_out), _ptr(first_out),
                                 _stream(stream)))

    def find_preamble(self, iq, n: int, starts, nstarts: int, idx_out, stream=None):
        check(lib().ofdm_find_preamble(self.h, _ptr(iq), n, _ptr(starts), nstarts, _ptr(idx_out),
                                       _stream(stream)))

    def cfo_estimate(self, x, nframes: int, frame_stride: int, nsym: int, cfo_out, stream=None):
        check(lib().ofdm_cfo_estimate(self.h, _ptr(x), nframes, frame_stride, nsym, _ptr(cfo_out),
                                      _stream(stream)))

    def freq_shift(self, x, nframes: int, frame_stride: int, nsamples: int, cfo, stream=None):
        check(lib().ofdm_freq_shift(self.h, _ptr(x), nframes, frame_stride, nsamples, _ptr(cfo),
                                    _stream(stream)))

    def cp_sync(self, x, nframes: int, frame_stride: int, nsym: int, stream=None):
        check(lib().ofdm_cp_sync(self.h, _ptr(x), nframes, frame_stride, nsym, _stream(stream)))

    def phase_sync(self, x, nframes: int, frame_stride: int, nsamples: int, pr=None, pr_len: int = 0,
                   stream=None):
        check(lib().ofdm_phase_sync(self.h, _ptr(x), nframes, frame_stride, nsamples, _ptr(pr), pr_len,
                                    _stream(stream)))

    def sync_chain(self, x, nframes: int, frame_stride: int, nsamples: int, nsym: int, cfo,
                   shift_out=None, cp_out=None, phase_out=None, out_stride: int = 0, stream=None):
        """freq_shift + cp_sync + phase_sync(context preamble) in one launch, each
        stage's state optionally copied out."""
        check(lib().ofdm_sync_chain(self.h, _ptr(x), nframes, frame_stride, nsamples, nsym, _ptr(cfo),
                                    _ptr(shift_out), _ptr(cp_out), _ptr(phase_out), out_stride,
                                    _stream(stream)))

    def chan_estimate(self, x, nframes: int, frame_stride: int, chan_out, chan_stride: int | None = None,
                      stream=None):
        cs = self.params.num_data_subc if chan_stride is None else chan_stride
        check(lib().ofdm_chan_estimate(self.h, _ptr(x), nframes, frame_stride, _ptr(chan_out), cs,
                                       _stream(stream)))

    def rx_stream(self, iq, n: int, max_frames: int, pb_out=None, bytes_out=None, constell_out=None,
                  cfo_out=None, chunk: int = 0, stream=None) -> int:
        """rx.cpp:94-221 (with its SDR ring, ofdm_set_stream_ring) over a
        device-resident stream; returns the frames found."""
        m = C.c_size_t()
        check(lib().ofdm_rx_stream(self.h, _ptr(iq), n, max_frames, chunk, _ptr(pb_out), _ptr(bytes_out),
                                   _ptr(constell_out), _ptr(cfo_out), C.byref(m), _stream(stream)))
        return m.value

    def rx_stream_i16(self, iq16, n: int, max_frames: int, pb_out=None, bytes_out=None, constell_out=None,
                      cfo_out=None, chunk: int = 0, stream=None) -> int:
        """rx_stream on n complex<int16> wire samples."""
        m = C.c_size_t()
        check(lib().ofdm_rx_stream_i16(self.h, _ptr(iq16), n, max_frames, chunk, _ptr(pb_out), _ptr(bytes_out),
                                       _ptr(constell_out), _ptr(cfo_out), C.byref(m), _stream(stream)))
        return m.value

    def walk_tuning(self, **changes) -> dict:
        """ofdm_set_walk_tuning: start from the defaults, apply `changes`
        (WalkTuning field names); returns the previous settings as a dict."""
        old = WalkTuning()
        check(lib().ofdm_get_walk_tuning(self.h, C.byref(old)))
        t = WalkTuning()
        check(lib().ofdm_walk_tuning_default(C.byref(t)))
        for k, v in changes.items():
            if not hasattr(t, k):
                raise KeyError(k)
            setattr(t, k, v)
        check(lib().ofdm_set_walk_tuning(self.h, C.byref(t)))
        return {f: getattr(old, f) for f, _ in WalkTuning._fields_}

    def shard_margins(self) -> tuple[int, int]:
        """ofdm_stream_shard_margins: (halo, tail) samples a stream shard needs."""
        h, t = C.c_long(), C.c_long()
        check(lib().ofdm_stream_shard_margins(self.h, C.byref(h), C.byref(t)))
        return h.value, t.value

    def stream_ring(self, ring: int | None = None) -> int:
        """ofdm_get/set_stream_ring: rx.cpp's SDR ring R of the stream walk (0:
        the continuous walk). With `ring` set, changes it; returns the old R."""
        old = C.c_long()
        check(lib().ofdm_get_stream_ring(self.h, C.byref(old)))
        if ring is not None:
            check(lib().ofdm_set_stream_ring(self.h, ring))
        return old.value

    def stream_timing(self, on: bool) -> None:
        """ofdm_set_stream_timing: per-phase HIP events in later stream calls."""
        check(lib().ofdm_set_stream_timing(self.h, 1 if on else 0))

    def last_stream_times(self) -> dict:
        """ofdm_get_stream_timing: the last timed stream call's device times
        (ms) of its walk, resolve and decode."""
        w, r, d = C.c_float(), C.c_float(), C.c_float()
        check(lib().ofdm_get_stream_timing(self.h, C.byref(w), C.byref(r), C.byref(d)))
        return {"walk_ms": w.value, "resolve_ms": r.value, "decode_ms": d.value}

    def initial_state(self) -> tuple[int, int]:
        """ofdm_stream_initial_state: rx.cpp's first walk state (pos, ring_end)."""
        st = WalkState()
        check(lib().ofdm_stream_initial_state(self.h, C.byref(st)))
        return st.pos, st.ring_end

    def rx_stream_shard(self, iq, n: int, start, own_lo: int, own_hi: int, max_frames: int, pb_out=None,
                        bytes_out=None, constell_out=None, cfo_out=None, chunk: int = 0, i16: bool = False,
                        located_cap: int = 4096, stream=None):
        """ofdm_rx_stream_shard: the walk from state `start` = (pos, ring_end)
        over this shard's n samples, frames with pb in [own_lo, own_hi)
        decoded. Returns (frames decoded, located pbs (numpy int64, relative),
        their ring lags (numpy uint8), exit state (pos, ring_end)); when the
        walk located more than located_cap frames, the located arrays hold
        the first located_cap - located_cap // 2 and the last located_cap // 2
        of them (located_cap = 0: no list, empty arrays)."""
        import numpy as np
        m, nl, ex = C.c_size_t(), C.c_size_t(), WalkState()
        cap = max(1, located_cap)
        if getattr(self, "_located", None) is None or len(self._located) < cap:
            self._located = np.empty(cap, dtype=np.int64)
            self._located_lag = np.empty(cap, dtype=np.uint8)
        loc, lag = self._located, self._located_lag
        st = WalkState(*start)
        want = located_cap > 0
        check(lib().ofdm_rx_stream_shard(self.h, None if i16 else _ptr(iq), _ptr(iq) if i16 else None, n,
                                         C.byref(st), own_lo, own_hi, max_frames, chunk, _ptr(pb_out),
                                         _ptr(bytes_out), _ptr(constell_out), _ptr(cfo_out), C.byref(m),
                                         loc.ctypes.data if want else None, lag.ctypes.data if want else None,
                                         located_cap, C.byref(nl), C.byref(ex), _stream(stream)))
        k = min(nl.value, located_cap)
        return m.value, loc[:k].copy(), lag[:k].copy(), (ex.pos, ex.ring_end)

    def sync_frames(self, frames, nframes: int, frame_stride: int, stages: int = SYNC_ALL,
                    cfo_in=None, cfo_out=None, chan_out=None, stream=None):
        check(lib().ofdm_sync_frames(self.h, _ptr(frames), nframes, frame_stride, stages, _ptr(cfo_in),
                                     _ptr(cfo_out), _ptr(chan_out), _stream(stream)))
