"""Pin the oracle's Modulation restatement bit-exactly to the reference's own
OFDM/modulation.cpp (compiled unmodified into oracle/_ref/libref.so, this
container only; skipped where the reference is absent, e.g. the GPU box)."""
import ctypes as C

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built (reference absent)")

KS = [1, 2, 4, 6, 8]


@pytest.mark.parametrize("k", KS)
def test_constellation(k):
    a = np.zeros(1 << k, np.complex128)
    n = O.ref().ref_constellation(k, O._d(a))
    assert n == 1 << k
    assert np.array_equal(O.constellation(k).view(np.uint64), a.view(np.uint64))


@pytest.mark.parametrize("k", KS)
@pytest.mark.parametrize("nbytes", [0, 1, 3, 7, 32, 257])
def test_mod(k, nbytes):
    data = np.random.default_rng(nbytes * 10 + k).integers(0, 256, nbytes, dtype=np.uint8)
    n = (nbytes * 8 + k - 1) // k
    r = np.zeros(max(n, 1), np.complex128)
    m = O.ref().ref_mod(k, O._u8(data) if nbytes else None, nbytes, O._d(r))
    o = O.mod(k, data)
    assert m == len(o)
    assert np.array_equal(o.view(np.uint64), r[:m].view(np.uint64))


@pytest.mark.parametrize("k", KS)
@pytest.mark.parametrize("n", [1, 5, 8, 100, 2048])
def test_demod(k, n):
    rng = np.random.default_rng(n + 100 * k)
    pts = (rng.standard_normal(n) + 1j * rng.standard_normal(n)) * 0.9
    # exact decision boundaries and out-of-range values too
    m = 1 << (k // 2)
    edges = np.linspace(-1, 1, m)[:-1] + 1.0 / max(m - 1, 1)
    pts[: min(n, len(edges))] = edges[: min(n, len(edges))] + 1j * edges[: min(n, len(edges))]
    if n > 4:
        pts[-1] = 3.0 - 2.5j
        pts[-2] = 0.0
    rp = pts.copy()
    nb = (n * k + 7) // 8
    rout = np.zeros(nb, np.uint8)
    rm = O.ref().ref_demod(k, O._d(rp), n, O._u8(rout))
    ob, op = O.demod(k, pts)
    assert rm == len(ob)
    assert np.array_equal(ob, rout[:rm])
    assert np.array_equal(op.view(np.uint64), rp.view(np.uint64))  # in-place clamp identical


@pytest.mark.parametrize("ob,ib", [(1, 8), (2, 8), (4, 8), (6, 8), (8, 8), (8, 1), (8, 2), (8, 4), (8, 6),
                                   (3, 5), (5, 3), (7, 2)])
def test_bit_stream_converter(ob, ib):
    rng = np.random.default_rng(ob * 31 + ib)
    for n in (1, 2, 9, 33):
        data = rng.integers(0, 1 << ib, n, dtype=np.uint8)
        out = np.zeros(n * 8, np.uint8)
        m = O.ref().ref_bit_convert(ob, ib, O._u8(data), n, O._u8(out))
        o = O.bit_convert(ob, ib, data)
        assert np.array_equal(o, out[:m])


def test_std_preamble_bytes():
    for seed, n in ((42, 32), (0, 100), (12345, 256)):
        r = np.zeros(n, np.uint8)
        O.ref().ref_std_preamble_bytes(seed, n, O._u8(r))
        p = O.Params.make(**dict(O.DEFAULT, pr_seed=seed, num_data_subc=n * 8 // 1, num_pr_symb=1))
        assert np.array_equal(O.preamble_bytes(p), r)
