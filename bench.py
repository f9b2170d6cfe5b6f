#!/usr/bin/env python3
"""bench.py — IQ-samples/s of the MI355X OFDM modem hot path (BASELINE.json).

Workload (BASELINE.json configs[1]): per GPU a batch of
65 536 OFDM symbols = 8 192 frames x 8 symbols, N=2048, D=1024 data + 32
pilots, cp=512, QPSK. One step = tx (map + pilot comb + IFFT + CP, fused
counter-based AWGN at Es/N0 = 10 dB) then rx (CP strip + FFT + pilot
normalise/equalise + demap + bit-error count) over the whole batch, inputs
resident in HBM. value = IQ samples through the tx->rx loopback per second,
whole job (all ranks). Multi-GPU: frames shard across ranks (weak scaling, no
data-path collective); one RCCL all-reduce of {bit errors, bits, samples,
frames} and a MAX of the elapsed time at the end.

Run: python bench.py [--gpus N --steps K --warmup W]; N>1 via
torch.distributed.run (one process per GPU, RCCL over xGMI).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "c-ofdm_amd", "python"))
from ofdm_synth import payload_bytes  # noqa: E402  (counter-based job payload)

METRIC = "IQ-samples/sec (tx IFFT+CP and rx FFT+equalise), 2048-subcarrier frames, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s spec
CONFIG_B = dict(fft_size=2048, num_data_subc=1024, num_pilot_subc=32, cp_size=512, num_symb=8,
                num_pr_symb=1, pr_sin_len=128, pr_seed=42, pr_level=500, t2sin_size=256, t2_sin_f1=17,
                t2_sin_f2=51, t2_sin_level=800, smooth=5, mod_type=2, pilot_ampl=2500, mult=200,
                rx_buf_size=40, iterations=10000)
# config/config.txt (the D config of SURVEY §8): the config-4 stream's frames
CONFIG_D = dict(CONFIG_B, fft_size=512, num_data_subc=256, num_pilot_subc=8, cp_size=128, mod_type=4)
STREAM_WORKLOAD = "config4_stream_D_frames_gaps0-4096_cfo0.004_awgn20dB"
STREAM_WORKLOAD_B = "config4_stream_B_frames_gaps0-4096_cfo0.004_awgn20dB"


def rx_bytes_per_symbol(p) -> int:
    """rx reads 16*N (CP not read), writes 16*D constellation + D*k/8 bytes."""
    N, D, k = p["fft_size"], p["num_data_subc"], p["mod_type"]
    return 16 * N + 16 * D + D * k // 8


def tx_bytes_per_symbol(p) -> int:
    """tx reads D*k/8 bytes, writes 16*(N+cp)."""
    return p["num_data_subc"] * p["mod_type"] // 8 + 16 * (p["fft_size"] + p["cp_size"])


def load_pmc(workload: str):
    """HBM traffic per rx launch from a committed rocprofv3 PMC summary
    (profiles/pmc_rx_*.json, made by tools/pmc_traffic.py), or None."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_rx_*.json"))):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload:
            best = d
    return best


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def granted_cpus() -> dict:
    """CPUs this process may use: the affinity mask, capped by a cgroup v2
    CPU quota and by OMP_NUM_THREADS, which the GPU lease sets to its CPU
    share (a lease sees every core of the host and is granted a share)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    omp = int(omp) if omp.isdigit() and int(omp) > 0 else None  # the lease's stated CPU share
    granted = min(v for v in (aff, quota, omp) if v)
    return {"cpu_count": os.cpu_count(), "affinity": aff, "cgroup_quota": quota, "omp_num_threads": omp,
            "granted": granted}


def cpu_baseline(p, data_host: np.ndarray, noise_std: float, budget_s: float, threads: int):
    """Oracle (plain-C restatement) tx+AWGN+rx loopback on host cores over a
    bounded sample of the same workload: single-threaded (one frame at a time,
    as the reference runs) and OpenMP over `threads` cores (one frame per
    thread). Reported beside the GPU number; `value` is the all-cores rate."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    g = O.geometry(p)
    bpf, msg = g["bytes_per_frame"], g["message_len"]
    nf_avail = len(data_host) // bpf

    def run(nthreads, batch, budget):
        done, f0 = 0, 0
        t0 = time.perf_counter()
        while True:
            nb = min(batch, nf_avail - f0)
            d = data_host[f0 * bpf:(f0 + nb) * bpf]
            iq = O.tx_batch(p, d, nb, threads=nthreads)
            iq = O.awgn(iq, noise_std, seed=1, sample_offset=f0 * msg, threads=nthreads)
            O.rx_batch(p, iq, nb, msg, ref=d, threads=nthreads, want_constell=True)
            done += nb
            f0 = (f0 + nb) % max(1, nf_avail - batch)
            el = time.perf_counter() - t0
            if el >= budget:
                return done * msg / el, done, el

    st, st_frames, st_s = run(1, 4, budget_s / 2)
    mt, mt_frames, mt_s = run(threads, 4 * threads, budget_s / 2)
    return {"value": mt, "unit": "IQ-samples/s", "cores": threads, "kind": "port",
            "single_thread_value": st,
            "sample": (f"config-B tx+AWGN+rx loopback (oracle/ofdm_oracle.c, own radix-4/2 FFT; FFTW absent) "
                       f"on {_cpu_model()} (os.cpu_count()={os.cpu_count()}): {mt_frames} frames on {threads} "
                       f"OpenMP threads in {mt_s:.1f} s; {st_frames} frames single-threaded in {st_s:.1f} s")}


def load_pmc_stream(workload: str):
    """HBM traffic per stream call from a committed PMC summary
    (profiles/pmc_stream_*.json), or None."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_stream_*.json"))):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload:
            best = d
    return best


def cpu_stream_baseline(p, x_host: np.ndarray, budget_s: float, i16: bool = False):
    """The oracle's rx.cpp walk + main.cpp:60-80 decode, single-threaded as the
    reference's rx runs, over a prefix of the same stream sized to ~budget_s.
    i16: x_host is the interleaved complex<int16> wire stream, converted to
    complex<double> inside the timed region (FRAME_FORM::form_int16_to_double,
    rx.cpp:81-90), as the reference's receiver does before its walk."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    g = O.geometry(p)
    span = g["preamble_len"] + g["message_len"]
    n = 1 << 18
    total = len(x_host) // 2 if i16 else len(x_host)
    while True:
        t0 = time.perf_counter()
        if i16:
            w = x_host[:2 * n].astype(np.float64)
            h = w[0::2] + 1j * w[1::2]
        else:
            h = x_host[:n]
        pbs = O.stream_walk_ring(p, h)[0]  # rx.cpp's walk with its SDR ring
        for pb in pbs:
            if pb + span <= len(h):
                O.decode_frame(p, h[pb:pb + span])
        dt = time.perf_counter() - t0
        if dt > budget_s / 3 or n >= total:
            break
        n = min(total, n * 4)
    conv = "int16 -> f64 conversion + " if i16 else ""
    return {"value": n / dt, "unit": "stream samples/s", "cores": 1, "kind": "port",
            "sample": f"{conv}oracle orc_stream_walk_ring + orc_decode_frame (own FFT; FFTW absent) over the first {n} "
                      f"samples ({len(pbs)} frames) of the same stream in {dt:.1f} s, 1 thread "
                      f"(rx.cpp's loop is single-threaded) on {_cpu_model()}"}


def stream_leg(args, dist, dev, world, rank, M, i16: bool, p=None, frames_per_gpu=0, workload=STREAM_WORKLOAD,
               pipeline=True, staged_ab=False, deferred=None):
    """SURVEY §8d config 4 (BASELINE configs[3]): the streaming receiver (T2
    detection walk + preamble sync + CFO/CP/phase/channel sync + demod,
    ofdm_rx_stream_shard) over a synthetic continuous stream of D-config
    frames. Weak scaling: the job's stream holds stream_frames frames per GPU;
    each rank holds its core plus halo/tail (ofdm_stream.shard_stream), walks
    and decodes it, and the ranks exchange their walk reports (ofdm_stream:
    one small all-gather; a rank whose walk-in did not meet the true walk
    walks again from its predecessor's exit state). One call = the whole
    stream; value = stream samples / s."""
    import torch
    import ofdm_dist
    import ofdm_stream as SS
    import ofdm_synth as Y
    # p: another frame geometry (config B's: the wide fused decode); staged_ab:
    # the same calls again through the staged decode kernels (walk tuning
    # staged_decode = 1), reported beside the fused figure
    p = dict(CONFIG_D if p is None else p)
    modem = M.Modem(p, dev.index)
    layout = Y.StreamLayout(p, (frames_per_gpu or args.stream_frames) * world)
    # rx.cpp's SDR ring (the config's rx_buf_size, the library's default) and initial state
    rx = SS.ShardedStreamRx(p, layout.n, world, rank, ring=modem.stream_ring(), initial=modem.initial_state())
    nsl = rx.slice_hi - rx.slice_lo
    x = Y.stream_slice(modem, layout, rx.slice_lo, rx.slice_hi, dev, i16=i16)
    f0, f1 = layout.frames_overlapping(rx.slice_lo, rx.slice_hi)
    cap = f1 - f0 + 16
    npts = p["num_data_subc"] * p["num_symb"]
    outs = {"pb_out": torch.full((cap,), -1, dtype=torch.int64, device=dev),
            "bytes_out": torch.zeros((cap * layout.bpf,), dtype=torch.uint8, device=dev),
            "constell_out": torch.zeros((cap * npts,), dtype=torch.complex128, device=dev),
            "cfo_out": torch.zeros((cap,), dtype=torch.float64, device=dev)}
    stream = torch.cuda.current_stream(dev)
    walk = SS.hip_walker(modem, x, nsl, rx.own_lo - rx.slice_lo, rx.own_hi - rx.slice_lo, cap, outs, i16=i16,
                         stream=stream, report_cap=rx.cap)
    exchange0 = SS.torch_exchange(dist, ofdm_dist.collective_device(dist, dev))
    xt = [0.0]  # host seconds inside the report all-gathers (the one collective of a call)

    def exchange(row):
        t = time.perf_counter()
        r = exchange0(row)
        xt[0] += time.perf_counter() - t
        return r
    for _ in range(args.stream_warmup):
        rx.run(walk, exchange)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    rx.rewalks = 0
    xt[0] = 0.0
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.stream_reps):
        n_owned = rx.run(walk, exchange)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = ofdm_dist.max_over_ranks(time.perf_counter() - t0, dev, dist)
    exchange_ms = ofdm_dist.max_over_ranks(xt[0], dev, dist) / args.stream_reps * 1e3
    call_ms = ev0.elapsed_time(ev1) / args.stream_reps  # this rank, its stream
    # located frames decode to the payload of the frame placed there
    k = min(n_owned, cap)
    pbs = outs["pb_out"][:k].cpu().numpy() + rx.slice_lo
    where = np.searchsorted(layout.starts, pbs, side="right") - 1
    ok = 0
    if k:
        got = outs["bytes_out"][:k * layout.bpf].view(k, layout.bpf).cpu().numpy()
        fa, fb = int(where.min()), int(where.max()) + 1
        sent = payload_bytes(fa * layout.bpf, (fb - fa) * layout.bpf).reshape(fb - fa, layout.bpf)
        ok = int((got == sent[where - fa]).all(axis=1).sum())
    cdev = ofdm_dist.collective_device(dist, dev)
    tot = torch.tensor([n_owned, ok, rx.rewalks], dtype=torch.int64, device=cdev)
    ofdm_dist.reduce_counters(tot, dist)
    tot = tot.cpu().numpy()
    # per-phase device times, measured in this run: a few more calls (outside
    # the timed region) with HIP events around the walk, resolve and decode
    # (the events cost launch gaps, so the timed calls run without them)
    phases = []
    modem.stream_timing(True)
    try:
        # every rank makes all three calls (each holds the report
        # all-gather): a call without timed phases is skipped, not the rest
        for _ in range(3):
            rx.run(walk, exchange)
            try:
                phases.append(modem.last_stream_times())
            except M.OfdmError:
                pass  # no timed decode (e.g. a shard whose call took the halo walk)
    finally:
        modem.stream_timing(False)
    torch.cuda.synchronize(dev)
    staged = None
    if staged_ab:
        modem.walk_tuning(staged_decode=1)
        for _ in range(2):
            rx.run(walk, exchange)
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        t1 = time.perf_counter()
        for _ in range(args.stream_reps):
            rx.run(walk, exchange)
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        el_st = ofdm_dist.max_over_ranks(time.perf_counter() - t1, dev, dist)
        modem.walk_tuning()
        staged = {"value": layout.n * args.stream_reps / el_st, "unit": "stream samples/s",
                  "ms_per_call": el_st / args.stream_reps * 1e3, "fused_speedup_per_sample": el_st / elapsed,
                  "note": "same stream and calls, the located frames decoded by the staged cfo -> params -> rx "
                          "kernels (walk tuning staged_decode = 1) instead of the fused decode kernel"}
    esz = 4 if i16 else 16
    core = rx.own_hi - rx.own_lo
    alg_rank = core * esz + n_owned * (16 * npts + layout.bpf)  # stream once + outputs
    workload = workload + ("_int16" if i16 else "")
    pmc = load_pmc_stream(workload) if world == 1 else None
    res = {"metric": "stream samples/s (T2 walk + preamble sync + CFO/CP/phase/chan sync + demod), "
                     "config-4 stream", "workload": workload, "value": layout.n * args.stream_reps / elapsed,
           "unit": "stream samples/s", "dtype": "f64" + (" (int16 wire input)" if i16 else ""),
           "n_gpus": world, "scaling": "weak", "reps": args.stream_reps, "warmup": args.stream_warmup,
           "ms_per_call": elapsed / args.stream_reps * 1e3, "stream_samples": layout.n,
           "stream_GB": layout.n * esz / 1e9, "frames_sent": layout.total_frames, "frames_found": int(tot[0]),
           "frames_error_free": int(tot[1]), "rewalks_per_call": int(tot[2]) / args.stream_reps,
           "walk_halo": 0, "slice_halo": rx.own_lo - rx.slice_lo, "slice_tail": rx.slice_hi - rx.own_hi,
           "exchange_ms_per_call": exchange_ms,
           "roofline": {"bound": "hbm", "kernel": "whole stream pipeline (walker + compaction + fused decode, "
                                                  "host stitching overlapped)",
                        "achieved": alg_rank / (call_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": alg_rank / (call_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                        "algorithmic_bytes_per_call": alg_rank, "avg_call_ms": call_ms,
                        "traffic": (pmc or {}).get("hbm_bytes_per_call")},
           "cpu_baseline": None}
    res["compute"] = decode_compute(p, n_owned, call_ms, phases)
    if staged is not None:
        res["staged"] = staged
    if pipeline and world == 1 and args.stream_pipeline > 1:
        res["pipelined"] = stream_pipelined(args, p, M, dev, modem, layout, rx, walk, outs, x, nsl, cap, i16,
                                            n_owned, exchange, SS)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the CPU baseline runs after every GPU measurement (deferred: the GPU
        # would idle meanwhile); its sample of the stream is copied out now
        xh = x[:(2 << 27) if i16 else (1 << 27)].cpu().numpy()

        def cpu_leg():
            try:
                res["cpu_baseline"] = cpu_stream_baseline(p, xh, args.stream_cpu_budget, i16=i16)
            except Exception as e:  # reported, not fatal
                res["cpu_baseline"] = {"error": repr(e)}
        deferred.append(cpu_leg)
    modem.close()
    return res


FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X_MICROARCH.md: FP64 vector


def decode_flops_per_frame(p) -> int:
    """Useful FP64 flops of one located frame's decode (main.cpp:60-80 on the
    frame): the radix-5 x 2^m pilot_freq_sinh transform, the preamble body
    and the message FFTs at 5 N log2 N each, the per-sample phase ramps (one
    complex product each), the CP correlations, and per data point the
    equalisation and channel products and the decision. Transcendentals and
    reductions are left out (a lower bound of the work)."""
    import math
    N, cp, D, S = p["fft_size"], p["cp_size"], p["num_data_subc"], p["num_symb"]
    L = N + cp
    m = L // 5
    cfo = 5 * (5 * m * math.log2(m)) + m * 44 if L % 5 == 0 and m & (m - 1) == 0 else 5 * L * math.log2(L)
    ffts = (S + 1) * 5 * N * math.log2(N)
    ramps = 6 * N * S + 6 * L
    cps = 8 * cp * (S + 1)
    emit = D * S * (6 + 6 + 6)
    return int(cfo + ffts + ramps + cps + emit)


def decode_compute(p, frames: int, call_ms: float, phases: list) -> dict:
    """The decode's compute side (VALU-bound: it takes about the same time
    with int16 input at a quarter of the bytes): useful FP64 flop/s over the
    decode's own device time, measured in this run (HIP events around the
    walk, resolve and decode of 3 calls after the timed ones,
    ofdm_get_stream_timing), against the FP64 vector peak; over the whole
    call time when no phase was timed (a lower bound)."""
    f = decode_flops_per_frame(p)
    if phases:
        mean = {k: float(np.mean([ph[k] for ph in phases])) * 1e3 for k in phases[0]}
        kus = {k.replace("_ms", "_us"): round(v, 1) for k, v in mean.items()}
        kus["source"] = (f"this run: HIP events around each phase of {len(phases)} calls after the timed ones "
                         "(ofdm_get_stream_timing; the events add launch gaps, so the phases sum above the "
                         "timed call)")
        t_s, basis = mean["decode_ms"] * 1e-6, f"decode phase {mean['decode_ms']:.1f} us, HIP events, this run"
    else:
        kus = None
        t_s, basis = call_ms * 1e-3, "whole call time (walk + resolve + decode): no phase timed"
    ach = f * frames / t_s / 1e12
    return {"bound": "valu", "flops_per_frame": f, "achieved": ach, "peak": FP64_VALU_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": ach / FP64_VALU_PEAK_TFLOPS, "time_basis": basis,
            "kernels_us": kus}


def stream_pipelined(args, p, M, dev, modem, layout, rx, walk, outs, x, nsl, cap, i16, n_owned, exchange, SS):
    """The same stream received by `stream_pipeline` contexts in turn, each on
    its own HIP stream with its own outputs (double-buffered receive): call
    k + 1's walk runs while call k's decode drains. Throughput of back-to-back
    calls (one timed region); every context's outputs are checked against the
    serial calls'."""
    import torch
    P = args.stream_pipeline
    mods, sts, walks, rxs, outl = [modem], [torch.cuda.current_stream(dev)], [walk], [rx], [outs]
    for _ in range(P - 1):
        m2 = M.Modem(p, dev.index)
        st2 = torch.cuda.Stream(dev)
        o2 = {k: torch.empty_like(v) for k, v in outs.items()}
        r2 = SS.ShardedStreamRx(p, layout.n, 1, 0, ring=m2.stream_ring(), initial=m2.initial_state())
        mods.append(m2)
        sts.append(st2)
        outl.append(o2)
        rxs.append(r2)
        walks.append(SS.hip_walker(m2, x, nsl, r2.own_lo - r2.slice_lo, r2.own_hi - r2.slice_lo, cap, o2, i16=i16,
                                   stream=st2, report_cap=r2.cap))
    for i in range(P):
        rxs[i].run(walks[i], exchange)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.stream_reps * P):
        rxs[k % P].run(walks[k % P], exchange)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    same = all(r.n_owned == n_owned for r in rxs[1:])
    k = min(n_owned, cap)
    for o in outl[1:]:
        same = same and bool(torch.equal(o["pb_out"][:k], outs["pb_out"][:k])) and \
            bool(torch.equal(o["bytes_out"][:k * layout.bpf], outs["bytes_out"][:k * layout.bpf]))
    for m2 in mods[1:]:
        m2.close()
    return {"contexts": P, "value": layout.n * args.stream_reps * P / el, "unit": "stream samples/s",
            "ms_per_call": el / (args.stream_reps * P) * 1e3, "calls": args.stream_reps * P,
            "outputs_match_serial": same,
            "note": "back-to-back calls on the same stream, alternating contexts/HIP streams (call k+1's walk "
                    "overlaps call k's decode); the record's value is the serial per-call figure"}


def stream_ingest_leg(args, dev, M):
    """A stream that keeps arriving (rx.cpp:58-91: the SDR reader thread and
    buf[2]): the config-4 int16 wire stream in page-locked host memory,
    received chunk by chunk (ofdm_ingest.StreamIngest: H2D of chunk k+1 on a
    copy stream while chunk k walks and decodes; each chunk's walk starts
    from the previous one's exit state). value = stream samples / s end to
    end (first copy to last decode), against the PCIe ceiling measured here
    (one pinned H2D copy of the whole stream); outputs compared with one
    device-resident call over the same stream. One GPU."""
    import torch
    import ofdm_ingest as I
    import ofdm_synth as Y
    p = dict(CONFIG_D)
    modem = M.Modem(p, dev.index)
    layout = Y.StreamLayout(p, args.stream_frames)
    x16 = Y.stream_slice(modem, layout, 0, layout.n, dev, i16=True)
    host = I.host_pinned_i16(x16)
    cap = layout.total_frames + 16
    npts = p["num_data_subc"] * p["num_symb"]

    def outs():
        return {"pb_out": torch.full((cap,), -1, dtype=torch.int64, device=dev),
                "bytes_out": torch.zeros((cap * layout.bpf,), dtype=torch.uint8, device=dev),
                "constell_out": torch.zeros((cap * npts,), dtype=torch.complex128, device=dev),
                "cfo_out": torch.zeros((cap,), dtype=torch.float64, device=dev)}
    ref = outs()
    nref = modem.rx_stream_i16(x16, layout.n, cap, **ref)
    got = outs()
    ing = I.StreamIngest(modem, p, host, layout.n, args.ingest_chunk, got, dev, cap)
    ing.run()  # warm-up (buffers, kernels)
    torch.cuda.synchronize(dev)
    reps = max(1, args.ingest_reps)
    t0 = time.perf_counter()
    for _ in range(reps):
        res = ing.run()
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / reps
    same = res["frames"] == nref and all(bool(torch.equal(got[k], ref[k])) for k in got)
    # the PCIe ceiling: one page-locked H2D copy of the whole stream
    d = torch.empty_like(x16)
    d.copy_(host, non_blocking=True)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    d.copy_(host, non_blocking=True)
    torch.cuda.synchronize(dev)
    h2d_s = time.perf_counter() - t1
    del d
    modem.close()
    return {"metric": "stream samples/s end to end from host memory (int16 wire samples H2D overlapped with "
                      "walk + decode)", "workload": STREAM_WORKLOAD + "_int16_host_ingest",
            "value": layout.n / el, "unit": "stream samples/s", "n_gpus": 1, "reps": reps,
            "ms_per_stream": el * 1e3, "chunk_samples": args.ingest_chunk, "calls_per_stream": res["calls"],
            "stream_samples": layout.n, "frames_found": res["frames"],
            "outputs_equal_device_resident_call": same,
            "pcie_h2d": {"GB_per_s": layout.n * 4 / h2d_s / 1e9, "samples_per_s": layout.n / h2d_s,
                         "note": "one page-locked H2D copy of the whole int16 stream, measured in this run"},
            "frac_of_pcie_ceiling": (layout.n / el) / (layout.n / h2d_s)}


CONFIG_C = dict(CONFIG_B, fft_size=4096, num_data_subc=2048, num_pilot_subc=64, cp_size=1024, mod_type=4)


def config3_leg(args, dist, dev, world, rank, M):
    """SURVEY §8d config 3 (BASELINE configs[2]): config C (N=4096, D=2048,
    P=64, cp=1024, 16-QAM, 8 symbols per frame). (1) The loopback step
    timed as the headline one (tx with fused AWGN at Es/N0 = 10 dB, then rx
    with constellation, bytes and bit errors; frames per GPU, weak scaling);
    (2) the AWGN BER sweep, Es/N0 0..30 dB step 2, >= 1e7 bits per point per
    GPU, seed 1000 + SNR (tools/ber_sweep.py's definition), errors and bits
    summed over the ranks."""
    import torch
    import ofdm_dist
    p = dict(CONFIG_C)
    modem = M.Modem(p, dev.index)
    geo = modem.geo
    nf, S = args.config3_frames, p["num_symb"]
    msg, bpf = geo.message_len, geo.bytes_per_frame
    f0 = rank * nf
    data = torch.from_numpy(payload_bytes(f0 * bpf, nf * bpf)).to(dev)
    iq = torch.empty((nf * msg,), dtype=torch.complex128, device=dev)
    cons = torch.empty((nf * p["num_data_subc"] * S,), dtype=torch.complex128, device=dev)
    out = torch.empty_like(data)
    errs = torch.zeros((1,), dtype=torch.int64, device=dev)
    es = 10.0 / 9.0  # mean energy of the reference's 16-QAM table (modulation.cpp:4-36): levels +-1/3, +-1 per axis
    stream = torch.cuda.current_stream(dev)

    def std_for(db):
        return float(np.sqrt(es / 10 ** (db / 10)))

    def step(events=None):
        if events:
            events[0].record(stream)
        modem.tx(data, nf, iq, noise_std=std_for(10.0), seed=1010, sample_offset=f0 * msg, stream=stream)
        if events:
            events[1].record(stream)
        modem.rx(iq, nf, constell_out=cons, bytes_out=out, ref=data, bit_errors=errs, stream=stream)
        if events:
            events[2].record(stream)

    # BER sweep on a prefix of the frames (>= 1e7 bits per point per GPU),
    # before the timed loop: its small synchronised launches would leave the
    # GPU lightly loaded right before the headline
    nb = min(nf, int(np.ceil(1e7 / (8 * bpf))))
    rows = []
    for db in range(0, 31, 2):
        errs.zero_()
        modem.tx(data, nb, iq, noise_std=std_for(db), seed=1000 + db, sample_offset=f0 * msg, stream=stream)
        modem.rx(iq, nb, bytes_out=out, ref=data, bit_errors=errs, stream=stream)
        cnt = torch.cat([errs, torch.tensor([8 * nb * bpf], dtype=torch.int64, device=dev)])
        ofdm_dist.reduce_counters(cnt, dist)
        e, b = (int(v) for v in cnt.cpu().numpy())
        rows.append({"es_n0_db": db, "bits": b, "bit_errors": e, "ber": e / b})
    for _ in range(args.config3_warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    ev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(ev[i])
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = ofdm_dist.max_over_ranks(time.perf_counter() - t0, dev, dist)
    tx_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    rx_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))
    rx_bytes = nf * S * rx_bytes_per_symbol(p)
    modem.close()
    return {"metric": "IQ-samples/sec (tx IFFT+CP and rx FFT+equalise), config C 4096-subcarrier 16-QAM frames",
            "workload": f"config3_C_N4096_D2048_P64_cp1024_16QAM_{nf}frames_x8sym_per_gpu",
            "value": world * args.steps * nf * msg / elapsed, "unit": "IQ-samples/s", "n_gpus": world,
            "scaling": "weak", "steps": args.steps, "warmup": args.config3_warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "dtype": "f64",
            "tx_avg_launch_ms": tx_ms, "rx_avg_launch_ms": rx_ms,
            "step_ms": [round(e[0].elapsed_time(e[2]), 4) for e in ev],
            "roofline": {"bound": "hbm", "kernel": "rx (CP strip+FFT+equalise+demap), config C",
                         "achieved": rx_bytes / (rx_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": rx_bytes / (rx_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "algorithmic_bytes_per_launch": rx_bytes, "avg_launch_ms": rx_ms},
            "ber_sweep": {"es_n0_db": "0..30 step 2", "seed": "1000 + Es/N0", "frames_per_gpu": nb, "points": rows}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU). Under torch.distributed.run WORLD_SIZE decides; otherwise "
                         "bench.py starts the N ranks itself (torch.distributed.run, 127.0.0.1)")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="nccl = RCCL over xGMI, one GPU per rank; gloo = host collectives, ranks may share "
                         "a GPU (rehearsal of the multi-rank path on a 1-GPU box)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10, help="untimed steps (the GPU clocks ramp over the first ~10 launches)")
    ap.add_argument("--frames", type=int, default=8192, help="frames per GPU (8 symbols each); weak scaling")
    ap.add_argument("--total-frames", type=int, default=0,
                    help="strong scaling: shard this many frames over the GPUs (config 5: 30517 = 10 GB)")
    ap.add_argument("--snr-db", type=float, default=10.0)
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline (half 1 thread, half all)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0: every CPU the lease grants)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stream", action="store_true", help="skip the config-4 stream sub-record")
    ap.add_argument("--stream-frames", type=int, default=16384, help="config-4 stream frames per GPU (weak)")
    ap.add_argument("--stream-reps", type=int, default=10)
    ap.add_argument("--stream-warmup", type=int, default=40,
                    help="untimed stream calls (the clocks ramp over ~30 ms of load; the stream legs run first)")
    ap.add_argument("--stream-cpu-budget", type=float, default=8.0)
    ap.add_argument("--stream-b-frames", type=int, default=4096,
                    help="config-B stream frames per GPU for the stream_B sub-record (0: skip)")
    ap.add_argument("--stream-pipeline", type=int, default=1,
                    help="contexts for the stream record's two-context figure (1: off, the default: one context "
                         "per GPU is the supported mode, INTEGRATION.md; one GPU only)")
    ap.add_argument("--no-ingest", action="store_true", help="skip the host-ingest stream sub-record")
    ap.add_argument("--ingest-chunk", type=int, default=1 << 24,
                    help="stream samples per ingest call (16 M: a call's walk latency, ~0.3 ms, hides behind the "
                         "next chunk's ~1.2 ms PCIe copy; profiles/r06/ingest_chunk_sweep.jsonl)")
    ap.add_argument("--ingest-reps", type=int, default=3)
    ap.add_argument("--no-config3", action="store_true", help="skip the config-3 (config C) sub-record")
    ap.add_argument("--config3-frames", type=int, default=4096, help="config C frames per GPU (weak)")
    ap.add_argument("--config3-warmup", type=int, default=30, help="untimed config-3 steps (clock ramp)")
    ap.add_argument("--check-frames", default="",
                    help="comma-separated GLOBAL frame indices: after the timed steps each rank holding one writes "
                         "its noisy IQ, decoded bytes and constellation to --check-out (parity tests)")
    ap.add_argument("--check-out", default="", help="directory for the --check-frames dumps (rank<r>.npz)")
    args = ap.parse_args()

    import ofdm_dist
    if ofdm_dist.needs_launch(args.gpus):
        # one process per GPU: the ranks are children of this process, which
        # never touches the GPU itself; rank 0 prints the JSON line
        sys.exit(ofdm_dist.launch_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:]))

    # exactly one line on stdout (rank 0's JSON): every other write to fd 1,
    # including C++ library banners (gloo's peer-connection notes), goes to
    # stderr
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    import torch
    import ofdm_mi355x as M

    world, rank, local = ofdm_dist.env_world()
    if world != args.gpus and rank == 0:
        print(f"bench.py: WORLD_SIZE={world} (launcher) overrides --gpus {args.gpus}", file=sys.stderr)
    dist, dev = ofdm_dist.init(args.backend, local)

    # Order: the headline's host-side setup (payload, buffers) first, then
    # the sub-records' GPU work (config-4 streams, config 3), then the
    # headline, then every CPU baseline. The headline is timed as the contract
    # says (W untimed warmup steps, then K timed steps) right after the
    # sub-records' last kernels: the GPU's clocks ramp over ~30 ms of sustained
    # load (step time 1.31 ms over the first 10 steps, 1.18 ms from step 30:
    # profiles/r05_ramp.txt), and a host-side gap before the headline (the
    # payload's 0.8 s) would let them fall back. CPU baselines last: the GPU
    # would idle meanwhile.
    p = dict(CONFIG_B)
    modem = M.Modem(p, dev.index)
    geo = modem.geo
    strong = args.total_frames > 0
    if strong:
        f0, nf = ofdm_dist.shard(args.total_frames, world, rank)
    else:
        f0, nf = rank * args.frames, args.frames
    S = p["num_symb"]
    msg = geo.message_len
    bpf = geo.bytes_per_frame
    npts = p["num_data_subc"] * S

    # payload: this rank's shard of the job's counter-based payload, resident in HBM
    data_host = payload_bytes(f0 * bpf, nf * bpf)
    data = torch.from_numpy(data_host).to(dev)
    iq = torch.empty((nf * msg,), dtype=torch.complex128, device=dev)
    cons = torch.empty((nf * npts,), dtype=torch.complex128, device=dev)
    out = torch.empty((nf * bpf,), dtype=torch.uint8, device=dev)
    errs = torch.zeros((1,), dtype=torch.int64, device=dev)
    es = 2.0  # QPSK constellation energy (points +-1 +-1j)
    noise_std = float(np.sqrt(es / 10 ** (args.snr_db / 10)))
    stream = torch.cuda.current_stream(dev)

    K, W = args.steps, args.warmup
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(K)]

    deferred = []
    sub = {}

    def record(name, fn):
        # a sub-record that raises is reported in its field, and the headline
        # is still measured (every rank runs the same legs, so a failure that
        # comes from the configuration fails on all of them alike)
        try:
            sub[name] = fn()
        except Exception as e:
            sub[name] = {"error": repr(e)}
            print(f"bench.py: sub-record {name} failed: {e!r}", file=sys.stderr)
        torch.cuda.empty_cache()
    if not args.no_stream:
        record("stream", lambda: stream_leg(args, dist, dev, world, rank, M, i16=False, deferred=deferred))
        record("stream_int16", lambda: stream_leg(args, dist, dev, world, rank, M, i16=True, deferred=deferred))
        if args.stream_b_frames > 0:  # the wide-geometry fused decode (config B frames) against the staged kernels
            record("stream_B", lambda: stream_leg(args, dist, dev, world, rank, M, i16=False, p=CONFIG_B,
                                                  frames_per_gpu=args.stream_b_frames, workload=STREAM_WORKLOAD_B,
                                                  pipeline=False, staged_ab=True, deferred=deferred))
        if not args.no_ingest and world == 1:  # host ingest: one GPU's PCIe link
            record("stream_ingest", lambda: stream_ingest_leg(args, dev, M))
    if not args.no_config3:
        record("config3", lambda: config3_leg(args, dist, dev, world, rank, M))

    def step(i, events=None):
        if events:
            events[0].record(stream)
        modem.tx(data, nf, iq, noise_std=noise_std, seed=1, sample_offset=f0 * msg, stream=stream)
        if events:
            events[1].record(stream)
        modem.rx(iq, nf, constell_out=cons, bytes_out=out, ref=data, bit_errors=errs, stream=stream)
        if events:
            events[2].record(stream)

    for i in range(W):
        step(i)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    errs.zero_()
    consts = torch.tensor([K * nf * bpf * 8, K * nf * msg, K * nf], dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(K):
        step(i, ev[i])
    # final BER/throughput reduction (the one collective of the path)
    totals = torch.cat([errs, consts])
    ofdm_dist.reduce_counters(totals, dist)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = ofdm_dist.max_over_ranks(time.perf_counter() - t0, dev, dist)

    tx_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    rx_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))
    tot = totals.cpu().numpy().astype(np.int64)
    samples = int(tot[2])
    value = samples / elapsed

    rx_bytes = nf * S * rx_bytes_per_symbol(p)
    tx_bytes = nf * S * tx_bytes_per_symbol(p)
    achieved = rx_bytes / (rx_ms * 1e-3) / 1e9
    workload = (f"config5_B_N2048_D1024_P32_cp512_QPSK_{args.total_frames}frames_sharded" if strong else
                f"config2_B_N2048_D1024_P32_cp512_QPSK_{nf}frames_x8sym_per_gpu")
    pmc = load_pmc(workload)

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "IQ-samples/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic: seeded random payload per rank, counter-based AWGN Es/N0={args.snr_db:g} dB",
        "config": {
            "workload": workload,
            "fft_size": p["fft_size"], "num_data_subc": p["num_data_subc"],
            "num_pilot_subc": p["num_pilot_subc"], "cp_size": p["cp_size"], "num_symb": S,
            "mod_type": p["mod_type"], "frames_per_gpu": nf, "symbols_per_gpu": nf * S,
            "total_frames": args.total_frames if strong else world * nf,
            "samples_per_step_per_gpu": nf * msg, "parallelism": f"frame-sharded x{world}",
            "backend": args.backend if dist else None,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "rx_kernel<11> (CP strip+FFT+equalise+demap)",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "algorithmic_bytes_per_launch": rx_bytes,
            "avg_launch_ms": rx_ms,
            "traffic": (pmc or {}).get("hbm_bytes_per_launch"),
        },
        "rx_iq_samples_per_s_per_gpu": nf * msg / (rx_ms * 1e-3),
        "tx_iq_samples_per_s_per_gpu": nf * msg / (tx_ms * 1e-3),
        "tx_achieved_gbs": tx_bytes / (tx_ms * 1e-3) / 1e9,
        "tx_avg_launch_ms": tx_ms,
        "step_ms": [round(e[0].elapsed_time(e[2]), 4) for e in ev],  # device time per timed step (tx start -> rx end)
        "ber": float(tot[0]) / max(float(tot[1]), 1.0),
        "bit_errors": int(tot[0]),
        "frames": int(tot[3]),
        "cpu_baseline": None,
    }
    if args.check_frames:
        # outside the timed region: the last step's noisy IQ (tx is a pure
        # function of the global frame / sample index) and its rx outputs
        torch.cuda.synchronize(dev)
        want = sorted({int(v) for v in args.check_frames.split(",") if v.strip()})
        mine = [g for g in want if f0 <= g < f0 + nf]
        dump = {"frames": np.array(mine, dtype=np.int64)}
        for g in mine:
            lf = g - f0
            dump[f"iq_{g}"] = iq[lf * msg:(lf + 1) * msg].cpu().numpy()
            dump[f"bytes_{g}"] = out[lf * bpf:(lf + 1) * bpf].cpu().numpy()
            dump[f"constell_{g}"] = cons[lf * npts:(lf + 1) * npts].cpu().numpy()
        os.makedirs(args.check_out, exist_ok=True)
        np.savez(os.path.join(args.check_out, f"rank{rank}.npz"), **dump)
        result["check"] = {"frames": want, "noise_std": noise_std, "seed": 1, "message_len": msg}
    modem.close()
    del iq, cons, out, data

    def headline_cpu():
        try:
            cpus = granted_cpus()
            thr = args.cpu_threads or cpus["granted"]
            result["cpu_baseline"] = cpu_baseline(p, data_host, noise_std, args.cpu_budget, thr)
            result["cpu_baseline"]["host_cpus"] = cpus
        except Exception as e:  # reported, not fatal: the GPU number stands alone
            result["cpu_baseline"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        deferred.insert(0, headline_cpu)
    result.update(sub)
    for fn in deferred:  # every CPU baseline, after the GPU measurements
        fn()
    if rank == 0:
        print(json.dumps(result), file=json_out, flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
