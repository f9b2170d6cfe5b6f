"""The walker's FP32 T2 screen (ofdm_sync.hip stream_walk_kernel, ofdm_fft32.hpp)
decides a block from FP32 only when its detector ratio clears the level by
t2_margin = 4e-5 (the derived bound is ~2.1e-5). Here the size of
the FP32 error is checked empirically on the blocks the walker sees: numpy's
FP32 FFT against FP64 on noise, on the T2 symbol's tones and on partial
overlaps of the two (the decision-relevant case), at the stream's amplitude
scales. CPU only; no GPU code runs."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle as O  # noqa: E402

MARGIN = 4e-5


def ratio(x, mask, dtype):
    X = np.fft.fft(x.astype(dtype))
    e = (X.real.astype(X.real.dtype) ** 2 + X.imag ** 2)
    return float(np.sum(e * mask, dtype=e.dtype) / np.sum(e, dtype=e.dtype))


def test_fp32_ratio_error_is_far_below_the_margin():
    p = dict(O.DEFAULT)
    n, f1, f2, sm = p["t2sin_size"], p["t2_sin_f1"], p["t2_sin_f2"], p["smooth"]
    k = np.arange(n)
    mask = (((k >= f1 - sm) & (k <= f1 + sm)) | ((k >= f2 - sm) & (k <= f2 + sm))).astype(np.float64)
    t2 = O.t2_symbol(p)
    rng = np.random.default_rng(7)
    worst = 0.0
    for trial in range(400):
        scale = 10.0 ** rng.uniform(-2, 4)
        noise = (rng.standard_normal(n) + 1j * rng.standard_normal(n)) * scale * rng.uniform(0.01, 1.0)
        shift = int(rng.integers(0, n))
        block = noise.copy()
        block[shift:] += np.asarray(t2)[: n - shift] * scale  # a block that overlaps the T2 symbol partly
        r64 = ratio(block, mask, np.complex128)
        r32 = ratio(block, mask.astype(np.float32), np.complex64)
        worst = max(worst, abs(r32 - r64))
    assert worst < MARGIN / 20, worst
