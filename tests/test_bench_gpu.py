"""bench.py's multi-rank path on the GPU: `--gpus 2 --backend gloo` starts two
ranks itself (ofdm_dist.launch_ranks) that share the box's one MI355X, each
running the HIP modem on its frame shard; the job's reduced counters equal a
single-rank run over the same global frames (the payload and the AWGN are
counter-based functions of the global byte / sample index). RCCL itself needs
one GPU per rank, so the nccl backend runs only on the driver's 8-GPU node."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _bench(*argv, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], env=env, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_two_ranks_equal_one_rank_over_the_same_frames():
    common = ["--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-stream", "--no-config3"]
    one = _bench("--frames", "128", *common)
    two = _bench("--gpus", "2", "--backend", "gloo", "--frames", "64", *common)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["total_frames"] == 128 and two["config"]["backend"] == "gloo"
    assert two["frames"] == one["frames"] == 2 * 128
    assert two["bit_errors"] == one["bit_errors"] > 0
    assert two["value"] > 0 and two["roofline"]["frac"] > 0


def test_bench_strong_scaling_shards_total_frames():
    common = ["--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-stream", "--no-config3"]
    one = _bench("--total-frames", "101", *common)
    three = _bench("--gpus", "3", "--backend", "gloo", "--total-frames", "101", *common)
    assert three["scaling"] == "strong" and three["n_gpus"] == 3
    assert three["frames"] == one["frames"] == 101
    assert three["bit_errors"] == one["bit_errors"]


def test_bench_config3_record():
    # SURVEY §8d config 3 in the driver's bench line: the config-C loopback
    # step and the AWGN BER sweep (0..30 dB, >= 1e7 bits per point)
    r = _bench("--steps", "2", "--warmup", "1", "--frames", "64", "--no-cpu-baseline", "--no-stream",
               "--config3-frames", "160")
    c3 = r["config3"]
    assert c3["n_gpus"] == 1 and c3["value"] > 0 and 0 < c3["roofline"]["frac"] < 1
    pts = c3["ber_sweep"]["points"]
    assert [p["es_n0_db"] for p in pts] == list(range(0, 31, 2))
    assert all(p["bits"] >= 10_000_000 for p in pts)
    bers = [p["ber"] for p in pts]
    assert 0.25 < bers[0] < 0.4 and bers[-1] == 0.0  # 16-QAM: ~1/3 at 0 dB, error-free at 30 dB
    assert all(b1 <= b0 + 1e-3 for b0, b1 in zip(bers, bers[1:]))


def test_bench_stream_records():
    # SURVEY §8d config 4 in the driver's bench line (small stream): the serial
    # per-call record with its per-phase times measured in the run, the
    # config-B frames' wide fused decode beside the staged kernels, and the
    # host-ingest record (outputs equal to the device-resident call); the
    # two-context figure is off by default (one context per GPU)
    r = _bench("--steps", "1", "--warmup", "1", "--frames", "64", "--no-cpu-baseline", "--no-config3",
               "--stream-frames", "512", "--stream-reps", "2", "--stream-warmup", "1", "--stream-b-frames", "96",
               "--ingest-chunk", "300000", "--ingest-reps", "1")
    for key in ("stream", "stream_int16"):
        s = r[key]
        assert s["value"] > 0 and s["frames_found"] >= 0.95 * s["frames_sent"]
        assert "pipelined" not in s and s["walk_halo"] == 0 and s["slice_halo"] == 0
        assert s["compute"]["bound"] == "valu" and 0 < s["compute"]["frac"] < 1
        ku = s["compute"]["kernels_us"]
        assert ku["walk_us"] > 0 and ku["decode_us"] > 0 and "this run" in ku["source"]
    b = r["stream_B"]
    assert b["workload"].startswith("config4_stream_B") and b["frames_found"] >= 0.95 * b["frames_sent"]
    assert b["frames_error_free"] >= 0.95 * b["frames_found"] and "pipelined" not in b
    assert b["staged"]["value"] > 0 and b["staged"]["fused_speedup_per_sample"] > 0
    g = r["stream_ingest"]
    assert g["outputs_equal_device_resident_call"] is True and g["frames_found"] >= 0.95 * 512
    assert g["calls_per_stream"] > 1 and 0 < g["frac_of_pcie_ceiling"] < 2


def test_bench_two_context_stream_figure_on_request():
    # --stream-pipeline 2: two contexts on two HIP streams taking calls in
    # turn (an experiment, off by default); outputs equal the serial calls'
    r = _bench("--steps", "1", "--warmup", "1", "--frames", "64", "--no-cpu-baseline", "--no-config3",
               "--stream-frames", "512", "--stream-reps", "2", "--stream-warmup", "1", "--stream-b-frames", "0",
               "--no-ingest", "--stream-pipeline", "2")
    for key in ("stream", "stream_int16"):
        pp = r[key]["pipelined"]
        assert pp["contexts"] == 2 and pp["calls"] == 4 and pp["outputs_match_serial"] is True and pp["value"] > 0
