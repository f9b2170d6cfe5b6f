"""GPU parity of the chunked ingest of a stream that keeps arriving
(c-ofdm_amd/python/ofdm_ingest.py; rx.cpp:58-91's reader thread and buf[2]
as two HIP streams and two device buffers): the int16 wire samples cross
from page-locked host memory chunk by chunk, each chunk's walk starting from
the previous chunk's exit state, and the frames received, in order, with
their bytes, constellations and CFOs, must equal one device-resident call of
ofdm_rx_stream_i16 over the whole stream (itself held to the oracle frame by
frame in test_gpu_stream_full.py). Chunk cores from a few frames (many
chunk boundaries, exit states inside the next slice's halo) to millions of
samples; ring mode (rx.cpp's SDR ring, the default) and the continuous walk."""
import numpy as np
import pytest

from common import D

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import ofdm_mi355x as M  # noqa: E402
import ofdm_ingest as I  # noqa: E402
import ofdm_synth as Y  # noqa: E402

NF = 1024


@pytest.fixture(scope="module")
def stream():
    m = M.Modem(D, 0)
    lay = Y.StreamLayout(D, NF)
    x16 = Y.stream_slice(m, lay, 0, lay.n, torch.device("cuda", 0), i16=True)
    torch.cuda.synchronize()
    return m, lay, x16


def outputs(cap):
    g = {"bpf": D["num_data_subc"] * D["num_symb"] * D["mod_type"] // 8, "npts": D["num_data_subc"] * D["num_symb"]}
    return {"pb_out": torch.full((cap,), -7, dtype=torch.int64, device="cuda"),
            "bytes_out": torch.zeros((cap * g["bpf"],), dtype=torch.uint8, device="cuda"),
            "constell_out": torch.zeros((cap * g["npts"],), dtype=torch.complex128, device="cuda"),
            "cfo_out": torch.zeros((cap,), dtype=torch.float64, device="cuda")}


@pytest.mark.parametrize("ring", [None, 0], ids=["ring", "continuous"])
@pytest.mark.parametrize("chunk", [20_000, 250_000, 3_000_000])
def test_chunked_ingest_equals_device_resident_call(stream, chunk, ring):
    m, lay, x16 = stream
    old = m.stream_ring(ring) if ring is not None else None
    try:
        cap = NF + 16
        ref = outputs(cap)
        nref = m.rx_stream_i16(x16, lay.n, cap, **ref)
        torch.cuda.synchronize()
        assert nref >= 0.95 * NF
        host = I.host_pinned_i16(x16)
        got = outputs(cap)
        ing = I.StreamIngest(m, D, host, lay.n, chunk, got, torch.device("cuda", 0), cap)
        res = ing.run()
        torch.cuda.synchronize()
        assert res["calls"] == -(-lay.n // chunk)
        assert res["frames"] == nref
        for k in ("pb_out", "bytes_out", "constell_out", "cfo_out"):
            assert torch.equal(got[k], ref[k]), k
    finally:
        if old is not None:
            m.stream_ring(old)
