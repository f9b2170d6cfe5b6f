"""SURVEY §8d config 5 (BASELINE configs[4]) on the box's one MI355X: the 10 GB
strong-scaling workload, `bench.py --total-frames 30517` (30 517 config-B
frames = 625 M IQ samples = 10 GB of complex f64), through the launched RCCL
path (`torch.distributed.run --nproc-per-node 1`, backend nccl: the rank joins
the process group, so the SUM/MAX all-reduces and the stream report
all-gather run over RCCL) and as a two-rank gloo split sharing the GPU. The
job's reduced counters agree between the two, and frames at the start, at the
shard boundary and at the end decode byte-identically to the oracle
(main.cpp's rx chain, oracle/ofdm_oracle.c) on the same noisy IQ. The 1/2/4/8
GPU curve itself is the driver's 8-GPU run."""
import glob
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle as O
from common import rel_err
from ofdm_dist import free_port
from ofdm_synth import payload_bytes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

TOTAL = 30517
# start, around the two-rank boundary (15259 | 15258), the end
CHECK = [0, 1, 15257, 15258, 15259, 15260, TOTAL - 2, TOTAL - 1]


def _env():
    return {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}


def _json_line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout[-3000:]
    return json.loads(lines[0])


def _check_dumps(outdir, rec):
    p = dict(O.CONFIG_B)
    g = O.geometry(p)
    msg = g["message_len"]
    seen = set()
    for path in sorted(glob.glob(os.path.join(outdir, "rank*.npz"))):
        d = np.load(path)
        for gf in d["frames"]:
            gf = int(gf)
            seen.add(gf)
            iq = d[f"iq_{gf}"]
            # the tx side: the oracle's tx + counter-based AWGN of the same
            # global frame / sample index (bench.py's payload definition)
            data = payload_bytes(gf * g["bytes_per_frame"], g["bytes_per_frame"])
            clean = O.tx_batch(p, data, 1)
            ref_iq = O.awgn(clean, rec["check"]["noise_std"], seed=rec["check"]["seed"], sample_offset=gf * msg)
            # the channel model's tolerance, on the noise component (the fused
            # AWGN draws on the FP32 transcendental units), as every AWGN check
            assert rel_err(iq - clean, ref_iq - clean) < 1e-6, gf
            # the rx side, bit-exact on the GPU's own noisy IQ
            cons, out, _ = O.rx_batch(p, iq, 1, msg)
            assert np.array_equal(d[f"bytes_{gf}"], out), gf
            assert rel_err(d[f"constell_{gf}"], cons) < 1e-9, gf
    assert seen == set(CHECK)


@pytest.mark.timeout(900)
def test_config5_10gb_rccl_one_rank_and_gloo_two_ranks(tmp_path):
    common = ["--total-frames", str(TOTAL), "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-config3",
              "--check-frames", ",".join(map(str, CHECK))]
    # one launched rank over RCCL, with a one-call stream leg (the report
    # all-gather of ofdm_stream over RCCL)
    d1 = str(tmp_path / "nccl")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "bench.py"), *common,
           "--backend", "nccl", "--check-out", d1, "--stream-frames", "2048", "--stream-reps", "1",
           "--stream-warmup", "1", "--stream-pipeline", "1"]
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    one = _json_line(r.stdout)
    assert one["n_gpus"] == 1 and one["scaling"] == "strong"
    assert one["config"]["backend"] == "nccl" and one["config"]["total_frames"] == TOTAL
    assert one["frames"] == 2 * TOTAL  # frames counted over the 2 timed steps
    assert one["config"]["samples_per_step_per_gpu"] * 16 > 0.999e10  # the 10 GB workload on one GPU
    assert one["bit_errors"] > 0
    for key in ("stream", "stream_int16"):
        s = one[key]
        assert s["n_gpus"] == 1 and s["frames_found"] >= 0.95 * s["frames_sent"]
        assert s["frames_error_free"] > 0.5 * s["frames_found"]  # 16-QAM at 20 dB: most frames error-free
    _check_dumps(d1, one)

    # two gloo ranks sharing the GPU: the same global frames, shard boundary
    # at frame 15259
    d2 = str(tmp_path / "gloo")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", *common,
                        "--no-stream", "--check-out", d2], env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    two = _json_line(r.stdout)
    assert two["n_gpus"] == 2 and two["config"]["total_frames"] == TOTAL
    assert two["frames"] == one["frames"]
    assert two["bit_errors"] == one["bit_errors"]
    _check_dumps(d2, two)
    # each rank dumped the frames of its own shard
    r0 = set(np.load(os.path.join(d2, "rank0.npz"))["frames"].tolist())
    r1 = set(np.load(os.path.join(d2, "rank1.npz"))["frames"].tolist())
    assert max(r0) < min(r1) and r0 | r1 == set(CHECK)
