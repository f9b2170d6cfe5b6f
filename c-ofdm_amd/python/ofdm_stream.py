"""ofdm_stream — streaming rx sharded over ranks (multi-GPU config 4).

The reference's detection walk (rx.cpp:125-221) is sequential: each step's
T2 search starts where the previous frame left it (pos = pb + message_len,
rx.cpp:192), and rx.cpp carries the last frame of one ring into the next
(rx.cpp:145-156). A stream therefore shards by SAMPLES the same way one GPU
shards it over its walkers (ofdm_rx_stream's chunk stitching), one level up:

* rank r owns the core [own_lo, own_hi) of the stream (ofdm_dist.shard over
  samples) and holds the slice [own_lo - halo, own_hi + tail): a walk-in halo
  (stream_halo: 3 frames, > output_size + 2*T2sin_size + pr_sin_len, SURVEY
  §8e) and a tail long enough for the step that crosses own_hi to locate and
  decode its frame (stream_tail);
* every rank walks its slice from the slice start (rank 0: from the true
  initial state), decodes the frames whose preamble start lies in its core
  (ofdm_rx_stream_shard, the HIP walker + fused decode) and reports the
  frames its walk located and its exit state — the first walk state at or
  past own_hi;
* the reports (a few dozen integers per rank) are exchanged; rank r's walk is
  the true walk if it and rank r-1's (already accepted) walk located a common
  frame no later than r's first owned frame — from a common frame on, the two
  walks are the same computation on the same samples. Otherwise rank r walks
  again from r-1's exit state (exact), and the check moves on. Every rank
  evaluates the same plan from the same reports, so the only collective is
  the small all-gather of reports (plus the end-of-job counter reduction).

With rx.cpp's SDR ring (the default, ofdm_set_stream_ring) a walk state is
(pos, ring_end) and a located frame is keyed by its preamble start and the
ring "lag" of the state after it (the library's located_lag): two walks that
located the same key are in the same state from there on. Rank 0 starts from
rx.cpp's initial state (ofdm_stream_initial_state), the others speculatively
at their slice start with the first ring end after it (ring ends lie on
multiples of R in stream coordinates).

The union of the owned frames equals the single-walk result for any number of
ranks; tests/test_stream_shard.py (gloo, oracle walker) and
tests/test_gpu_stream_shard.py (HIP, 2/4/8 shards) check it.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

# Samples one walker T2 scan step covers at most (ofdm_sync.hpp WALK_SCAN_MAX:
# the FP32 screen's 2 x 128 threads x 8 samples). The library states what a
# shard needs (ofdm_stream_shard_margins); tests/test_gpu_stream.py checks
# stream_halo / stream_tail against it.
WALK_SCAN = 2048


def geometry(params: dict) -> dict:
    N, cp = params["fft_size"], params["cp_size"]
    L = N + cp
    pre, msg = L * params["num_pr_symb"], L * params["num_symb"]
    t2 = params["t2sin_size"]
    return {"t2": t2, "pre": pre, "msg": msg, "frame_len": t2 + pre + msg,
            "window": 2 * t2 + params["pr_sin_len"]}


def stream_halo(params: dict) -> int:
    """Walk-in before a rank's core: 3 frames (the walker's chunk halo), which
    exceeds SURVEY §8e's minimum of one output_size + 2*T2sin_size + pr_sin_len."""
    g = geometry(params)
    return max(3 * g["frame_len"], g["frame_len"] + g["window"] + g["t2"])


def stream_tail(params: dict) -> int:
    """Samples past own_hi a rank must hold: a step starting before own_hi
    scans at most one more walker scan step, then the preamble window, then
    its frame (preamble + message) must fit."""
    g = geometry(params)
    return WALK_SCAN + g["t2"] + g["window"] + g["pre"] + g["msg"] + 1


def shard_stream(n: int, world: int, rank: int, halo: int, tail: int) -> tuple[int, int, int, int]:
    """(slice_lo, slice_hi, own_lo, own_hi) of `rank`: the core is a contiguous
    sample range (remainder to the low ranks), the slice adds the halo before
    and the tail after it, clipped to the stream."""
    base, rem = divmod(n, world)
    own_lo = rank * base + min(rank, rem)
    own_hi = own_lo + base + (1 if rank < rem else 0)
    return max(0, own_lo - halo), min(n, own_hi + tail), own_lo, own_hi


State = tuple  # (pos, ring_end): ring_end 0 without a ring


def first_ring_end(pos: int, ring: int) -> int:
    """The first ring end after stream position pos (ring ends at k * ring)."""
    return (pos // ring + 1) * ring if ring else 0


@dataclass
class ShardReport:
    """What one rank's walk of its slice tells the others (absolute positions).
    located: keys (pb, lag) of every frame the walk located, in walk order."""
    rank: int
    slice_lo: int
    own_lo: int
    own_hi: int
    located: list = field(default_factory=list)   # (pb, lag) keys
    exit: State = (-1, 0)                          # first walk state >= own_hi; pos -1: samples ran out
    true_start: bool = False                       # walked from a state of the true walk

    def first_owned(self) -> float:
        own = [pb for pb, _ in self.located if self.own_lo <= pb < self.own_hi]
        return min(own) if own else float("inf")


def rewalk_start(exit_prev: State, slice_lo: int, t2: int) -> State:
    """Start state for re-walking a rank from its predecessor's exit state. An
    exit state before the slice (a step that started early and located a frame
    past own_hi) moves forward on its own T2 grid: the blocks it skips lie
    before that step's first T2 hit, inside its ring, so the walk from the
    moved state is the same computation (the halo exceeds the preamble window,
    so it stays before the hit)."""
    pos, ring_end = exit_prev
    if pos >= slice_lo:
        return exit_prev
    return pos + -(-(slice_lo - pos) // t2) * t2, ring_end


def stitch_plan(reports: list[ShardReport], t2: int):
    """The first rank whose walk is not yet known to be the true walk, with the
    absolute state to re-walk it from, or None when every rank is accepted.
    Rank 0 walks from the true initial state; rank r is accepted when it was
    walked from a true state, or when it and the accepted rank r-1 located a
    common frame (same key) no later than r's first owned frame."""
    for r in range(1, len(reports)):
        cur, prev = reports[r], reports[r - 1]
        if cur.true_start:
            continue
        first = cur.first_owned()
        common = set(prev.located).intersection(cur.located)
        if any(pb <= first for pb, _ in common):
            continue
        if prev.exit[0] < 0:
            # the true walk ran out of samples inside rank r-1's slice (its
            # slice reaches the stream end): rank r and the ranks after it own
            # no frame
            return r, (-1, 0)
        return r, rewalk_start(prev.exit, cur.slice_lo, t2)
    return None


HEADER = 7


def pack_report(rep: ShardReport, cap: int) -> np.ndarray:
    """Fixed-size int64 row for an all-gather: a header and the walk's first
    and last `cap` located frames, each as 2*pb + lag (a check reads only the
    frames near the two core ends: the walk-in and first owned frames, the
    last owned and past ones; cap exceeds the frames a halo or tail can hold)."""
    loc = [2 * pb + lag for pb, lag in rep.located]
    head = loc[:cap]
    tail = loc[-cap:] if len(loc) > cap else []
    out = np.full(HEADER + 2 * cap, -1, dtype=np.int64)
    out[:HEADER] = [rep.rank, rep.slice_lo, rep.own_lo, rep.own_hi, rep.exit[0], rep.exit[1], int(rep.true_start)]
    out[HEADER:HEADER + len(head)] = head
    out[HEADER + cap:HEADER + cap + len(tail)] = tail
    return out


def unpack_report(a: np.ndarray, cap: int) -> ShardReport:
    head = [int(v) for v in a[HEADER:HEADER + cap] if v >= 0]
    tail = [int(v) for v in a[HEADER + cap:HEADER + 2 * cap] if v >= 0]
    loc = [(v >> 1, v & 1) for v in sorted(set(head) | set(tail))]
    return ShardReport(int(a[0]), int(a[1]), int(a[2]), int(a[3]), loc, (int(a[4]), int(a[5])), bool(a[6]))


class ShardedStreamRx:
    """Runs one rank's part of a sharded stream receive.

    walk(start_rel) -> (n_owned, located_rel, lags, exit_rel) walks this
    rank's slice from a slice-relative state (pos, ring_end) and decodes its
    owned frames (ofdm_rx_stream_shard on the GPU). exchange(rows) all-gathers
    one int64 row per rank and returns the rows of every rank (RCCL/gloo, or an
    in-process list when several shards run in one process). ring: rx.cpp's
    SDR ring R (0: the continuous walk); initial: the stream's first walk
    state (ofdm_stream_initial_state)."""

    def __init__(self, params: dict, n: int, world: int, rank: int, halo: int | None = None,
                 tail: int | None = None, cap: int = 64, ring: int = 0, initial: State = (0, 0)):
        self.params = params
        self.t2 = params["t2sin_size"]
        self.halo = stream_halo(params) if halo is None else halo
        self.tail = stream_tail(params) if tail is None else tail
        self.world, self.rank, self.cap = world, rank, cap
        self.ring, self.initial = ring, tuple(initial)
        self.slice_lo, self.slice_hi, self.own_lo, self.own_hi = shard_stream(n, world, rank, self.halo, self.tail)
        self.rewalks = 0

    def _rel(self, st: State) -> State:
        return st[0] - self.slice_lo, (st[1] - self.slice_lo if self.ring else 0)

    def speculative_start(self) -> State:
        """Rank 0: the true initial state; others: the slice start, with the
        first ring end after it."""
        if self.rank == 0:
            return self.initial
        return self.slice_lo, first_ring_end(self.slice_lo, self.ring)

    def _walk(self, walk, start: State):
        if start[0] < 0 and self.rank > 0:  # the true walk ended before this core: nothing owned
            self.n_owned = 0
            return self._report([], [], (-1, 0), True)
        n_own, loc, lag, ex = walk(self._rel(start))
        self.n_owned = n_own
        return self._report(loc, lag, ex, True)

    def _check_cap(self, walk) -> None:
        # the library's head/tail truncation of the located list and
        # pack_report's windows must be the same frames: one cap sets both
        wc = getattr(walk, "report_cap", self.cap)
        if wc != self.cap:
            raise ValueError(f"walker report_cap {wc} != ShardedStreamRx.cap {self.cap}")

    def first_walk(self, walk) -> ShardReport:
        self._check_cap(walk)
        n_own, loc, lag, ex = walk(self._rel(self.speculative_start()))
        self.n_owned = n_own
        return self._report(loc, lag, ex, self.rank == 0)

    def _report(self, loc, lag, ex, true_start) -> ShardReport:
        # only the frames near the core ends matter to a check (pack_report)
        loc = np.asarray(loc, dtype=np.int64)
        lag = np.asarray(lag, dtype=np.int64) if len(lag) else np.zeros(len(loc), np.int64)
        if len(loc) > 2 * self.cap:
            loc = np.concatenate([loc[:self.cap], loc[-self.cap:]])
            lag = np.concatenate([lag[:self.cap], lag[-self.cap:]])
        keys = [(int(p) + self.slice_lo, int(g)) for p, g in zip(loc, lag)]
        exit_abs = (-1, 0) if ex[0] < 0 else (ex[0] + self.slice_lo, ex[1] + self.slice_lo if self.ring else 0)
        return ShardReport(self.rank, self.slice_lo, self.own_lo, self.own_hi, keys, exit_abs, true_start)

    def run(self, walk, exchange) -> int:
        """The walk, the report exchange and any re-walks; returns this rank's
        owned frame count (its outputs hold them, in stream order)."""
        if self.world == 1:  # the walk from the stream's initial state is the true walk: no report
            quiet = getattr(walk, "no_report", None)
            if quiet is not None:
                self.n_owned = quiet(self._rel(self.initial))
                return self.n_owned
            self.first_walk(walk)
            return self.n_owned
        rep = self.first_walk(walk)
        while True:
            rows = exchange(pack_report(rep, self.cap))
            reps = [unpack_report(np.asarray(r), self.cap) for r in rows]
            plan = stitch_plan(reps, self.t2)
            if plan is None:
                return self.n_owned
            r, start = plan
            if r == self.rank:
                self.rewalks += 1
                rep = self._walk(walk, start)


def run_local(rxs: list[ShardedStreamRx], walks: list) -> list[int]:
    """Every rank of a sharded receive in one process (several contexts on one
    GPU, or a CPU walker in tests): the reports, plan and re-walks of
    ShardedStreamRx.run with the all-gather replaced by a list. Returns each
    rank's owned frame count."""
    reps = [rx.first_walk(w) for rx, w in zip(rxs, walks)]
    t2 = rxs[0].t2
    while True:
        rows = [pack_report(rep, rx.cap) for rep, rx in zip(reps, rxs)]
        plan = stitch_plan([unpack_report(row, rx.cap) for row, rx in zip(rows, rxs)], t2)
        if plan is None:
            return [rx.n_owned for rx in rxs]
        r, start = plan
        rxs[r].rewalks += 1
        reps[r] = rxs[r]._walk(walks[r], start)


def torch_exchange(dist, device):
    """all-gather of one int64 row per rank over the job's process group (RCCL
    over xGMI with the rows on the GPU, gloo on the host). On the GPU the
    rows travel on a side stream of their own: an RCCL collective waits for
    the issuing stream's pending work, and on the receiver's stream that is
    the speculative decode of this very call, which the exchange should run
    beside, not after."""
    import contextlib

    import torch
    side = torch.cuda.Stream(device) if device.type == "cuda" else None

    def exchange(row):
        if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
            return [row]
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            t = torch.from_numpy(np.ascontiguousarray(row)).to(device)
            out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
            dist.all_gather(out, t)
            return [o.cpu().numpy() for o in out]
    return exchange


def hip_walker(modem, x_slice, n_slice: int, own_lo_rel: int, own_hi_rel: int, max_frames: int, outputs: dict,
               i16: bool = False, chunk: int = 0, stream=None, report_cap: int = 64):
    """walk(start_rel) over one rank's device-resident slice through
    ofdm_rx_stream_shard; outputs: pb_out / bytes_out / constell_out / cfo_out
    device tensors for max_frames frames (pb relative to the slice). The
    located list holds the walk's first and last report_cap frames (all a
    report packs, pack_report): pass the ShardedStreamRx's cap (its runs
    refuse a walker whose report_cap differs); walk.no_report(start_rel)
    skips the list (one rank)."""
    def walk(start_rel):
        return modem.rx_stream_shard(x_slice, n_slice, start_rel, own_lo_rel, own_hi_rel, max_frames,
                                     chunk=chunk, i16=i16, located_cap=2 * report_cap, stream=stream, **outputs)

    def no_report(start_rel):  # one rank: the owned frames only, no located list
        return modem.rx_stream_shard(x_slice, n_slice, start_rel, own_lo_rel, own_hi_rel, max_frames,
                                     chunk=chunk, i16=i16, located_cap=0, stream=stream, **outputs)[0]
    walk.no_report = no_report
    walk.report_cap = report_cap
    return walk
