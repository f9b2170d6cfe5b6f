"""Streaming rx sharded over ranks (c-ofdm_amd/python/ofdm_stream.py)
on the CPU: the report / plan / re-walk protocol with the ORACLE's walk as each
rank's walker (the sequential rx.cpp:94-198 walk with or without its SDR ring,
restarted at a given state and stopped at the first state at or past the core
end). Also pins that state form of the ring walk to rx.cpp's loop replayed on
a real ring buffer. The union of the
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


def oracle_shard_walk(p, xs, start, own_lo, own_hi, ring=0):
    """The reference walk over the slice xs from state `start` = (pos,
    ring_end) (orc_stream_walk_ring; ring = 0: the continuous walk): (owned
    count, located pbs, their ring lags, exit state). Exit = the first state
    at or past own_hi: a state after a step, the first scan block at or past
    own_hi when the scan passes it, or the start of the step that located the
    first frame past own_hi; pos -1 if the walk ended first."""
    pbs, lags, ex = O.stream_walk_ring(p, xs, ring=ring, start=start[0], ring_end=start[1], own_hi=own_hi,
                                       with_lags=True)
    owned = [pb for pb in pbs if own_lo <= pb < own_hi]
    return len(owned), pbs, lags, ex


def _walkers(p, x, world, halo=None, ring=0):
    rxs, walks = [], []
    init = (-O.geometry(p)["frame_len"], ring) if ring else (0, 0)
    for r in range(world):
        rx = S.ShardedStreamRx(p, len(x), world, r, halo=halo, ring=ring, initial=init)
        xs = x[rx.slice_lo:rx.slice_hi]
        lo, hi = rx.own_lo - rx.slice_lo, rx.own_hi - rx.slice_lo
        rxs.append(rx)
        walks.append(lambda s, xs=xs, lo=lo, hi=hi: oracle_shard_walk(p, xs, s, lo, hi, ring))
    return rxs, walks


# walk modes: the continuous walk, rx.cpp's ring with 3-frame refills (a ring
# end every ~2.4 frames of this stream) and the config's 40-frame ring
MODES = {
    "continuous": (D, 0, 24),
    "ring3": (dict(D, rx_buf_size=3), None, 24),
    "ring40": (D, None, 90),
}


@pytest.fixture(scope="module", params=list(MODES))
def stream(request):
    cfg, ring, nf = MODES[request.param]
    R = O.ring_len(cfg) if ring is None else ring
    x, _ = impaired_stream(cfg, nf, seed=4)
    want = O.stream_walk_ring(cfg, x, ring=R)[0]
    return cfg, R, x, want


def _run_local(p, x, world, halo=None, ring=0):
    rxs, walks = _walkers(p, x, world, halo, ring)
    owned_lists = {}

    def recording(r, w):
        def walk(s):
            n, loc, lag, ex = w(s)
            rx = rxs[r]
            owned_lists[r] = [int(v) + rx.slice_lo for v in loc if rx.own_lo <= v + rx.slice_lo < rx.own_hi]
            return n, loc, lag, ex
        return walk

    counts = S.run_local(rxs, [recording(r, w) for r, w in enumerate(walks)])
    for r, rx in enumerate(rxs):
        if counts[r] == 0:
            owned_lists[r] = []
    return counts, [owned_lists[r] for r in range(world)], sum(rx.rewalks for rx in rxs)


def test_ring_walk_is_rx_cpp_loop():
    """The state form of the ring walk (orc_stream_walk_ring: the product's
    semantics) equals rx.cpp's loop replayed on a real ring buffer
    (orc_rx_app_walk: buffer copies, carries, refills) on streams crossing
    many ring ends, and differs from the continuous walk where a marker
    straddles a refill."""
    differs = 0
    for seed, nf, gap in [(4, 24, 4096), (5, 60, 3000), (7, 40, 0), (8, 40, 12000)]:
        x, _ = impaired_stream(D, nf, seed=seed, gap_max=gap)
        for rb in (1, 2, 3, 5, 40):
            cfg = dict(D, rx_buf_size=rb)
            a = O.stream_walk_ring(cfg, x)[0]
            b = O.rx_app_walk(cfg, x)
            assert np.array_equal(a, b), (seed, rb)
            differs += not np.array_equal(a, O.stream_walk(cfg, x))
        # the loop's iteration cap (config["iterations"]) cuts the walk short
        cfg = dict(D, rx_buf_size=3)
        full = O.rx_app_walk(cfg, x)
        assert np.array_equal(O.rx_app_walk(cfg, x, iterations=10), full[:len(O.rx_app_walk(cfg, x, iterations=10))])
    assert differs > 0  # the ring loses frames the continuous walk finds


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
    cfg, R, x, want = stream
    counts, owned, _ = _run_local(cfg, x, world, ring=R)
    assert sum(counts) == len(want)
    assert np.array_equal(np.concatenate([np.array(o, np.int64) for o in owned]), want)


@pytest.mark.parametrize("halo", [0, 700, 3000, 9000])
def test_short_halos_force_rewalks_and_stay_exact(stream, halo):
    cfg, R, x, want = stream
    counts, owned, rewalks = _run_local(cfg, x, 4, halo=halo, ring=R)
    assert np.array_equal(np.concatenate([np.array(o, np.int64) for o in owned]), want)
    if halo == 0:
        assert rewalks > 0  # no walk-in: no common frame, every later rank re-walks


def test_stitch_plan_rules():
    t2 = 256
    r0 = S.ShardReport(0, 0, 0, 1000, [(10, 0), (500, 0), (990, 0), (1200, 0)], (1300, 0), True)
    ok = S.ShardReport(1, 700, 1000, 2000, [(720, 0), (990, 0), (1200, 0), (1900, 0)], (2100, 0), False)
    assert S.stitch_plan([r0, ok], t2) is None
    late = S.ShardReport(1, 700, 1000, 2000, [(730, 0), (1250, 0)], (2100, 0), False)  # 1200 missed, 1250 spurious
    assert S.stitch_plan([r0, late], t2) == (1, (1300, 0))
    # the same frame in another ring state is not a common frame
    lag = S.ShardReport(1, 700, 1000, 2000, [(990, 1), (1200, 1), (1900, 0)], (2100, 0), False)
    assert S.stitch_plan([r0, lag], t2) == (1, (1300, 0))
    # an exit state before the slice moves forward on its T2 grid, in its ring
    r0b = S.ShardReport(0, 0, 0, 1000, [(10, 0)], (100, 5000), True)
    far = S.ShardReport(1, 900, 1000, 2000, [], (2100, 5000), False)
    assert S.stitch_plan([r0b, far], t2) == (1, (100 + 4 * 256, 5000))
    # the true walk ended inside rank 0's slice: rank 1 owns nothing
    r0c = S.ShardReport(0, 0, 0, 1000, [(10, 0)], (-1, 0), True)
    assert S.stitch_plan([r0c, far], t2) == (1, (-1, 0))
    row = S.pack_report(lag, 2)
    back = S.unpack_report(row, 2)
    assert (back.rank, back.slice_lo, back.own_lo, back.own_hi, back.exit, back.true_start) == (1, 700, 1000, 2000,
                                                                                               (2100, 0), False)
    assert back.located == [(990, 1), (1200, 1), (1900, 0)]


def _gloo_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg, ring, nf = MODES["ring3"]
    R = O.ring_len(cfg)
    x, _ = impaired_stream(cfg, nf, seed=4)
    rx = S.ShardedStreamRx(cfg, len(x), world, rank, halo=2000, ring=R, initial=(-O.geometry(cfg)["frame_len"], R))
    xs = x[rx.slice_lo:rx.slice_hi]
    lo, hi = rx.own_lo - rx.slice_lo, rx.own_hi - rx.slice_lo
    last = {}

    def walk(s):
        n, loc, lag, ex = oracle_shard_walk(cfg, xs, s, lo, hi, R)
        last["owned"] = [int(v) + rx.slice_lo for v in loc if lo <= v < hi]
        return n, loc, lag, ex

    n_owned = rx.run(walk, S.torch_exchange(dist, torch.device("cpu")))
    owned = last["owned"] if n_owned else []
    parts = [None] * world
    dist.all_gather_object(parts, (rank, owned, rx.rewalks))
    if rank == 0:
        q.put(parts)
    dist.destroy_process_group()


def test_gloo_two_ranks_sharded_ring_walk_equals_sequential_walk():
    import torch.multiprocessing as mp
    cfg, ring, nf = MODES["ring3"]
    x, _ = impaired_stream(cfg, nf, seed=4)
    want = O.stream_walk_ring(cfg, x)[0]
    world = 2
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


def test_walker_report_cap_must_match_the_receiver_cap():
    # the library truncates the located list to the walk's first and last
    # report_cap frames, pack_report to the receiver's cap: one value for both
    rx = S.ShardedStreamRx(D, 100000, 2, 1, cap=64)

    def walk(start_rel):
        return 0, [], [], (-1, 0)
    walk.report_cap = 32
    with pytest.raises(ValueError, match="report_cap"):
        rx.first_walk(walk)
    walk.report_cap = 64
    rx.first_walk(walk)
