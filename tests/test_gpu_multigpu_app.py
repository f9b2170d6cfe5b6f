"""The multi-GPU job from C++ over the C-ABI alone (apps/ofdm_multigpu.cpp;
SURVEY §8e, BASELINE configs[4]): one thread and one ofdm_ctx per GPU,
contiguous frame shards (ofdm_shard_range), the tx -> rx loopback, and the
RCCL SUM all-reduce of the counters (ofdm_reduce_counters). On this one-GPU
box the job runs with one rank (a one-rank RCCL communicator); its counters
must equal the Python binding's run of the same frames, payload and noise
(bench.py's counter-based definitions), so they do not depend on the GPU
count."""
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import ofdm_mi355x as M  # noqa: E402
import oracle as O  # noqa: E402
from ofdm_synth import payload_bytes  # noqa: E402

APP = os.path.join(os.path.dirname(M.HEADER), "..", "c-ofdm_amd", "bin", "ofdm_multigpu")


def run_app(*args):
    out = subprocess.run([APP, *args], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def bit_errors(nf, f0=0, snr_db=10.0):
    """The Python binding's tx (fused AWGN, seed 1) -> rx over frames [f0, f0 + nf)."""
    p = dict(O.CONFIG_B)
    g = O.geometry(p)
    m = M.Modem(p, 0)
    data = torch.from_numpy(payload_bytes(f0 * g["bytes_per_frame"], nf * g["bytes_per_frame"])).cuda()
    iq = torch.empty((nf * g["message_len"],), dtype=torch.complex128, device="cuda")
    errs = torch.zeros((1,), dtype=torch.int64, device="cuda")
    std = float(np.sqrt(2.0 / 10 ** (snr_db / 10)))
    m.tx(data, nf, iq, noise_std=std, seed=1, sample_offset=f0 * g["message_len"])
    m.rx(iq, nf, ref=data, bit_errors=errs)
    torch.cuda.synchronize()
    e = int(errs.cpu().numpy()[0])
    m.close()
    return e, g


@pytest.mark.skipif(not os.path.exists(APP), reason="ofdm_multigpu not built")
def test_multigpu_app_one_rank_counters_equal_python_run():
    d = run_app("--gpus", "1", "--frames", "512", "--steps", "3", "--warmup", "1")
    e, g = bit_errors(512)
    assert d["n_gpus"] == 1 and d["frames"] == 3 * 512 and d["scaling"] == "weak"
    assert d["bits"] == 3 * 512 * g["bytes_per_frame"] * 8
    assert d["bit_errors"] == 3 * e > 0
    assert d["value"] > 1e10  # whole-job IQ samples/s


@pytest.mark.skipif(not os.path.exists(APP), reason="ofdm_multigpu not built")
def test_multigpu_app_strong_scaling_shard():
    # --total-frames: the one rank takes every frame (ofdm_shard_range)
    d = run_app("--gpus", "1", "--total-frames", "1001", "--steps", "2", "--warmup", "1")
    e, _ = bit_errors(1001)
    assert d["frames"] == 2 * 1001 and d["scaling"] == "strong" and d["bit_errors"] == 2 * e


@pytest.fixture(scope="module")
def wire_stream(tmp_path_factory):
    """bench.py's config-4 stream (2048 D-config frames, gaps, CFO, 20 dB) as
    the SDR's complex<int16> wire samples in a file, and the oracle's
    sequential rx.cpp walk over it (its SDR ring, the library default)."""
    import ofdm_synth as Y
    p = dict(O.DEFAULT)
    m = M.Modem(p, 0)
    lay = Y.StreamLayout(p, 2048)
    x16 = Y.stream_slice(m, lay, 0, lay.n, torch.device("cuda", 0), i16=True).cpu().numpy()
    m.close()
    path = tmp_path_factory.mktemp("stream") / "stream_i16.bin"
    x16.tofile(path)
    w = x16.astype(np.float64)
    want = O.stream_walk_ring(p, w[0::2] + 1j * w[1::2])[0]
    return str(path), lay.n, np.asarray(want, dtype=np.int64)


@pytest.mark.skipif(not os.path.exists(APP), reason="ofdm_multigpu not built")
@pytest.mark.parametrize("shards", [1, 2, 3, 8])
def test_multigpu_app_sharded_stream_owns_the_sequential_walks_frames(wire_stream, shards, tmp_path):
    # the C++ host's sharded stream receive (ofdm_stream_report_pack /
    # ofdm_stream_stitch_plan, rows all-gathered through host memory: the
    # ranks share the one GPU here; one rank per GPU uses ncclAllGather):
    # the union of the owned frames, in stream order, is the oracle's walk
    path, n, want = wire_stream
    out = tmp_path / "pbs.bin"
    d = run_app("--stream", path, "--shards", str(shards), "--gpus", "1", "--pbs-out", str(out), "--reps", "2")
    got = np.fromfile(out, dtype=np.int64)
    assert d["ranks"] == shards and d["stream_samples"] == n and d["frames"] == len(got)
    assert d["exchange"].startswith("host memory") or shards == 1
    assert np.array_equal(got, want)
    assert d["value"] > 0


@pytest.mark.skipif(not os.path.exists(APP), reason="ofdm_multigpu not built")
def test_multigpu_app_sharded_stream_rewalks_stay_exact(wire_stream, tmp_path):
    # a report cap of 1 frame: the ranks' reports carry only their first and
    # last located frames, so speculative walks are rarely accepted and the
    # plan makes ranks re-walk from their predecessor's exit state: still the
    # oracle's walk
    path, n, want = wire_stream
    out = tmp_path / "pbs.bin"
    d = run_app("--stream", path, "--shards", "6", "--gpus", "1", "--report-cap", "1", "--pbs-out", str(out))
    assert np.array_equal(np.fromfile(out, dtype=np.int64), want)
    assert d["rewalks"] >= 1  # the re-walk path ran
