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
