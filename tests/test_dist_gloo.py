"""Multi-rank driver logic on CPU (gloo, world_size 2): frame sharding covers
the batch exactly once, the per-rank results concatenate to the single-rank
result, and the one SUM all-reduce of the counters equals the serial totals.
The per-rank compute here is the oracle (CPU checker); on MI355X bench.py runs
the HIP kernels with the same sharding and reduction (c-ofdm_amd/python/ofdm_dist.py)."""
import os
import socket

import numpy as np
import pytest

import ofdm_dist
import oracle as O
from common import D

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def test_shard_partitions_exactly():
    for n in (0, 1, 7, 8, 30517, 65536):
        for w in (1, 2, 3, 4, 8):
            seen = []
            for r in range(w):
                b, c = ofdm_dist.shard(n, w, r)
                seen.extend(range(b, b + c))
            assert seen == list(range(n))
            counts = [ofdm_dist.shard(n, w, r)[1] for r in range(w)]
            assert max(counts) - min(counts) <= 1


NF = 10


def _dataset():
    g = O.geometry(D)
    data = np.random.default_rng(5).integers(0, 256, NF * g["bytes_per_frame"], dtype=np.uint8)
    iq = O.awgn(O.tx_batch(D, data, NF), 0.45, seed=7)
    return g, data, iq


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g, data, iq = _dataset()
    b, c = ofdm_dist.shard(NF, world, rank)
    L, bpf = g["message_len"], g["bytes_per_frame"]
    _, out, errs = O.rx_batch(D, iq[b * L:(b + c) * L], c, L, ref=data[b * bpf:(b + c) * bpf])
    counters = torch.tensor([errs, c * bpf * 8, c * L, c], dtype=torch.int64)
    ofdm_dist.reduce_counters(counters, dist)
    parts = [None] * world
    dist.all_gather_object(parts, (b, out))
    if rank == 0:
        q.put((counters.tolist(), parts))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_shard_and_reduce_equals_single_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    counters, parts = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g, data, iq = _dataset()
    _, out, errs = O.rx_batch(D, iq, NF, g["message_len"], ref=data)
    assert counters == [errs, NF * g["bytes_per_frame"] * 8, NF * g["message_len"], NF]
    joined = np.concatenate([o for _, o in sorted(parts, key=lambda t: t[0])])
    assert np.array_equal(joined, out)


def test_launcher_starts_ranks_and_reduction_equals_single_rank():
    """ofdm_dist.launch_ranks (bench.py --gpus N) spawns 2 ranks under
    torch.distributed.run; each sees WORLD_SIZE=2, the shards tile the batch,
    the reduced counters and the joined bytes equal the single-rank run, and
    rank 0 reports n_gpus=2 and the max over ranks of the elapsed time."""
    import json
    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_job_cpu.py")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    os.environ.pop("WORLD_SIZE", None)
    assert ofdm_dist.needs_launch(2) and not ofdm_dist.needs_launch(1)
    rc, out = ofdm_dist.launch_ranks(2, script, ["--frames", str(NF)], env=env, capture=True)
    assert rc == 0, out
    line = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(line) == 1, out  # rank 0 only
    res = json.loads(line[0])
    assert res["n_gpus"] == 2
    assert [w for _, w, _, _ in res["ranks"]] == [2, 2]
    assert [(b, c) for _, _, b, c in res["ranks"]] == [ofdm_dist.shard(NF, 2, r) for r in range(2)]
    assert res["max_elapsed"] == 2.0
    g = O.geometry(D)
    data = np.random.default_rng(5).integers(0, 256, NF * g["bytes_per_frame"], dtype=np.uint8)
    iq = O.awgn(O.tx_batch(D, data, NF), 0.45, seed=7)
    _, out1, errs = O.rx_batch(D, iq, NF, g["message_len"], ref=data)
    assert res["totals"] == [errs, NF * g["bytes_per_frame"] * 8, NF * g["message_len"], NF]
    assert bytes.fromhex(res["bytes_hex"]) == out1.tobytes()


def test_launched_single_rank_joins_the_group():
    """Under torch.distributed.run at one rank (WORLD_SIZE=1 in the
    environment) the rank still joins the process group, so the reduction
    path (RCCL on the GPU box) runs; the totals equal the unlaunched run's."""
    import json
    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_job_cpu.py")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    rc, out = ofdm_dist.launch_ranks(1, script, ["--frames", str(NF)], env=env, capture=True)
    assert rc == 0, out
    res = json.loads([ln for ln in out.splitlines() if ln.startswith("{")][0])
    assert res["n_gpus"] == 1 and res["grouped"] and res["max_elapsed"] == 1.0
    g = O.geometry(D)
    data = np.random.default_rng(5).integers(0, 256, NF * g["bytes_per_frame"], dtype=np.uint8)
    iq = O.awgn(O.tx_batch(D, data, NF), 0.45, seed=7)
    _, out1, errs = O.rx_batch(D, iq, NF, g["message_len"], ref=data)
    assert res["totals"] == [errs, NF * g["bytes_per_frame"] * 8, NF * g["message_len"], NF]


def test_bench_gpus_flag_launches_ranks(monkeypatch):
    """bench.py --gpus 4 without a launcher environment hands off to
    ofdm_dist.launch_ranks with its own path and argv (before any GPU call)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(ofdm_dist, "launch_ranks", lambda n, script, argv: calls.append((n, script, argv)) or 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    assert calls == [(4, os.path.join(root, "bench.py"), ["--gpus", "4", "--steps", "3"])]
