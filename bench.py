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

METRIC = "IQ-samples/sec (tx IFFT+CP and rx FFT+equalise), 2048-subcarrier frames, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s spec
CONFIG_B = dict(fft_size=2048, num_data_subc=1024, num_pilot_subc=32, cp_size=512, num_symb=8,
                num_pr_symb=1, pr_sin_len=128, pr_seed=42, pr_level=500, t2sin_size=256, t2_sin_f1=17,
                t2_sin_f2=51, t2_sin_level=800, smooth=5, mod_type=2, pilot_ampl=2500, mult=200,
                rx_buf_size=40, iterations=10000)


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


def payload_bytes(begin: int, count: int, seed: int = 0x5EED) -> np.ndarray:
    """Counter-based synthetic payload: byte i of the whole job = splitmix64(seed + i) & 0xFF,
    so every rank generates exactly its shard and the job is independent of the GPU count."""
    z = np.arange(begin, begin + count, dtype=np.uint64) + np.uint64(seed)
    z = z * np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    return (z & np.uint64(0xFF)).astype(np.uint8)


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10, help="untimed steps (the GPU clocks ramp over the first ~10 launches)")
    ap.add_argument("--frames", type=int, default=8192, help="frames per GPU (8 symbols each); weak scaling")
    ap.add_argument("--total-frames", type=int, default=0,
                    help="strong scaling: shard this many frames over the GPUs (config 5: 30517 = 10 GB)")
    ap.add_argument("--snr-db", type=float, default=10.0)
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline (half 1 thread, half all)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0: min(16, cpu_count))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import ofdm_dist
    import ofdm_mi355x as M

    world, rank, local = ofdm_dist.env_world()
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    p = dict(CONFIG_B)
    modem = M.Modem(p, local)
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
        "ber": float(tot[0]) / max(float(tot[1]), 1.0),
        "bit_errors": int(tot[0]),
        "frames": int(tot[3]),
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            thr = args.cpu_threads or min(16, os.cpu_count() or 1)  # the GPU box's CPU share is 16
            result["cpu_baseline"] = cpu_baseline(p, data_host, noise_std, args.cpu_budget, thr)
        except Exception as e:  # reported, not fatal: the GPU number stands alone
            result["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    modem.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
