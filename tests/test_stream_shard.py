"""Streaming rx sharded over ranks (c-ofdm_amd/python/ofdm_stream.py)
on the CPU: the report / plan / re-walk protocol with the ORACLE's walk as each
rank's walker (the sequential rx.cpp:125-221 walk, restarted at a given state
and stopped at the first state at or past the core end). The union of the
owned frames must equal the single sequential walk over the whole stream, for
any rank count and halo (short halos force re-walks), in one process and over
gloo with two real ranks. tests/test_gpu_stream_shard.py runs the same
protocol on the HIP walker."""
import os

import numpy as np
import pytest

import ofdm_dist
import ofdm_stream as S
import oracle as O
from common import D, impaired_stream

torch = pytest.importorskip("torch")


def oracle_shard_walk(p, xs, start, own_lo, own_hi):
    """The reference walk over the slice xs from state `start`: (owned count,
    located pbs, exit state). Exit = the first state at or past own_hi: a
    position after a frame or a no-preamble step, the equivalent first T2 grid
    position past own_hi when the scan passes it without a hit, or the start of
    the step that located the first frame past own_hi; -1 if the samples ran
    out first."""
    g = S.geometry(p)
    t2, msg, pre = g["t2"], g["msg"], g["pre"]
    n = len(xs)
    pos, located = start, []
    while True:
        if pos >= own_hi:
            ex = pos
            break
        hit = O.find_t2sin(p, xs, pos)
        grid = pos + -(-(own_hi - pos) // t2) * t2  # first scan block at or past own_hi
        if hit < 0 or hit >= own_hi:
            ex = grid if (hit >= 0 or grid + t2 <= n) else -1
            break
        pb = O.find_preamble(p, xs, hit) + 1
        if pb < -2:
            pos = hit + msg
            continue
        if pb + pre + msg > n:
            ex = -1
            break
        located.append(pb)
        if pb >= own_hi:
            ex = pos
            break
        pos = pb + msg
    owned = [pb for pb in located if own_lo <= pb < own_hi]
    return len(owned), np.array(located, np.int64), ex


def _walkers(p, x, world, halo=None):
    rxs, walks = [], []
    for r in range(world):
        rx = S.ShardedStreamRx(p, len(x), world, r, halo=halo)
        xs = x[rx.slice_lo:rx.slice_hi]
        lo, hi = rx.own_lo - rx.slice_lo, rx.own_hi - rx.slice_lo
        rxs.append(rx)
        walks.append(lambda s, xs=xs, lo=lo, hi=hi: oracle_shard_walk(p, xs, s, lo, hi))
    return rxs, walks




@pytest.fixture(scope="module")
def stream():
    x, _ = impaired_stream(D, 24, seed=4)
    return x, O.stream_walk(D, x)


def _run_local(p, x, world, halo=None):
    rxs, walks = _walkers(p, x, world, halo)
    owned_lists = {}

    def recording(r, w):
        def walk(s):
            n, loc, ex = w(s)
            rx = rxs[r]
            owned_lists[r] = [int(v) + rx.slice_lo for v in loc if rx.own_lo <= v + rx.slice_lo < rx.own_hi]
            return n, loc, ex
        return walk

    counts = S.run_local(rxs, [recording(r, w) for r, w in enumerate(walks)])
    for r, rx in enumerate(rxs):
        if counts[r] == 0:
            owned_lists[r] = []
    return counts, [owned_lists[r] for r in range(world)], sum(rx.rewalks for rx in rxs)


def test_shard_stream_tiles_the_stream():
    halo, tail = S.stream_halo(D), S.stream_tail(D)
    g = O.geometry(D)
    assert halo >= g["frame_len"] + 2 * D["t2sin_size"] + D["pr_sin_len"]  # SURVEY §8e minimum
    for n in (0, 5, 100_000, 1_000_003):
        for w in (1, 2, 3, 8):
            cores = [S.shard_stream(n, w, r, halo, tail) for r in range(w)]
            assert [c[2] for c in cores] == [ofdm_dist.shard(n, w, r)[0] for r in range(w)]
            assert cores[0][2] == 0 and cores[-1][3] == n
            for a, b in zip(cores, cores[1:]):
                assert a[3] == b[2]
            for lo, hi, olo, ohi in cores:
                assert lo == max(0, olo - halo) and hi == min(n, ohi + tail)


@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
def test_sharded_walk_equals_sequential_walk(stream, world):
    x, want = stream
    counts, owned, _ = _run_local(D, x, world)
    assert sum(counts) == len(want)
    assert np.array_equal(np.concatenate([np.array(o, np.int64) for o in owned]), want)


@pytest.mark.parametrize("halo", [0, 700, 3000, 9000])
def test_short_halos_force_rewalks_and_stay_exact(stream, halo):
    x, want = stream
    counts, owned, rewalks = _run_local(D, x, 4, halo=halo)
    assert np.array_equal(np.concatenate([np.array(o, np.int64) for o in owned]), want)
    if halo == 0:
        assert rewalks > 0  # no walk-in: no common frame, every later rank re-walks


def test_stitch_plan_rules():
    t2 = 256
    r0 = S.ShardReport(0, 0, 0, 1000, [10, 500, 990, 1200], 1300, True)
    ok = S.ShardReport(1, 700, 1000, 2000, [720, 990, 1200, 1900], 2100, False)
    assert S.stitch_plan([r0, ok], t2) is None
    late = S.ShardReport(1, 700, 1000, 2000, [730, 1250], 2100, False)  # 1200 missed, 1250 spurious
    assert S.stitch_plan([r0, late], t2) == (1, 1300)
    # an exit state before the slice moves forward on its T2 grid
    r0b = S.ShardReport(0, 0, 0, 1000, [10], 100, True)
    far = S.ShardReport(1, 900, 1000, 2000, [], 2100, False)
    assert S.stitch_plan([r0b, far], t2) == (1, 100 + 4 * 256)
    # the true walk ended inside rank 0's slice: rank 1 owns nothing
    r0c = S.ShardReport(0, 0, 0, 1000, [10], -1, True)
    assert S.stitch_plan([r0c, far], t2) == (1, -1)
    row = S.pack_report(ok, 2)
    back = S.unpack_report(row, 2)
    assert (back.rank, back.slice_lo, back.own_lo, back.own_hi, back.exit, back.true_start) == (1, 700, 1000, 2000,
                                                                                               2100, False)
    assert back.located == [720, 990, 1200, 1900]


def _gloo_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x, _ = impaired_stream(D, 24, seed=4)
    rx = S.ShardedStreamRx(D, len(x), world, rank, halo=2000)
    xs = x[rx.slice_lo:rx.slice_hi]
    lo, hi = rx.own_lo - rx.slice_lo, rx.own_hi - rx.slice_lo
    last = {}

    def walk(s):
        n, loc, ex = oracle_shard_walk(D, xs, s, lo, hi)
        last["owned"] = [int(v) + rx.slice_lo for v in loc if lo <= v < hi]
        return n, loc, ex

    n_owned = rx.run(walk, S.torch_exchange(dist, torch.device("cpu")))
    owned = last["owned"] if n_owned else []
    parts = [None] * world
    dist.all_gather_object(parts, (rank, owned, rx.rewalks))
    if rank == 0:
        q.put(parts)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_two_ranks_sharded_walk_equals_sequential_walk(stream, world):
    import torch.multiprocessing as mp
    x, want = stream
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = ofdm_dist.free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    parts = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    owned = np.concatenate([np.array(o, np.int64) for _, o, _ in sorted(parts, key=lambda t: t[0])])
    assert np.array_equal(owned, want)
