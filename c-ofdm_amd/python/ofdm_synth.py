"""ofdm_synth — synthetic workloads of bench.py, as counter-based functions of
global indices so that every rank builds exactly its own shard and a job's
data does not depend on the number of GPUs (there is no dataset:
the reference's inputs are radio captures).

* payload_bytes: byte i of the job = splitmix64(seed + i) & 0xFF.
* config-4 stream (stream_layout / stream_slice): D-config full frames
  (T2 + preamble + message, FRAME_FORM::get, built by the HIP tx) separated by
  0..4096-sample zero gaps, per-frame CFO U(-0.004, 0.004) cycles/sample and
  phase U(-pi, pi), AWGN at 20 dB over every sample. Gap, CFO and phase of
  frame f are splitmix64 functions of f; the noise of sample i comes from the
  2^22-sample block holding i, drawn by a generator seeded with the block
  index. Built on the GPU with torch (plumbing: the data, not the path).
"""
from __future__ import annotations

import numpy as np

_M1, _M2, _M3 = np.uint64(0x9E3779B97F4A7C15), np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB)
NOISE_BLOCK = 1 << 22


def splitmix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64) * _M1
    z = (z ^ (z >> np.uint64(30))) * _M2
    z = (z ^ (z >> np.uint64(27))) * _M3
    return z ^ (z >> np.uint64(31))


def payload_bytes(begin: int, count: int, seed: int = 0x5EED) -> np.ndarray:
    """Byte i of the whole job = splitmix64(seed + i) & 0xFF."""
    z = np.arange(begin, begin + count, dtype=np.uint64) + np.uint64(seed)
    return (splitmix64(z) & np.uint64(0xFF)).astype(np.uint8)


def _uniform(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    z = splitmix64(idx.astype(np.uint64) + np.uint64((seed << 40) + (stream << 36)))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


class StreamLayout:
    """Where the frames of a synthetic config-4 stream lie."""

    def __init__(self, params: dict, total_frames: int, seed: int = 4, gap_max: int = 4096,
                 cfo_max: float = 0.004, snr_db: float = 20.0):
        N, cp = params["fft_size"], params["cp_size"]
        L = N + cp
        self.params, self.seed, self.snr_db = params, seed, snr_db
        self.flen = params["t2sin_size"] + L * (params["num_pr_symb"] + params["num_symb"])
        self.bpf = params["num_data_subc"] * params["num_symb"] * params["mod_type"] // 8
        f = np.arange(total_frames + 1)
        gaps = (splitmix64(f.astype(np.uint64) + np.uint64(seed << 44)) % np.uint64(gap_max + 1)).astype(np.int64)
        self.starts = np.cumsum(gaps[:-1] + self.flen) - self.flen  # frame f after gaps 0..f, frames 0..f-1
        self.n = int(self.starts[-1] + self.flen + gaps[-1]) if total_frames else int(gaps[-1])
        self.cfo = (_uniform(seed, 1, f[:-1]) * 2 - 1) * cfo_max
        self.phase = (_uniform(seed, 2, f[:-1]) * 2 - 1) * np.pi
        self.total_frames = total_frames

    def frames_overlapping(self, lo: int, hi: int) -> tuple[int, int]:
        """[f0, f1): the frames with a sample in [lo, hi)."""
        f0 = int(np.searchsorted(self.starts + self.flen, lo, side="right"))
        f1 = int(np.searchsorted(self.starts, hi, side="left"))
        return f0, max(f0, f1)


def stream_slice(modem, layout: StreamLayout, lo: int, hi: int, device, i16: bool = False):
    """Samples [lo, hi) of the stream as a device tensor: complex128 (n,), or
    with i16 the SDR wire format complex<int16> of x*mult as int16 (2n,)."""
    import torch
    p = layout.params
    n = hi - lo
    x = torch.zeros((n,), dtype=torch.complex128, device=device)
    f0, f1 = layout.frames_overlapping(lo, hi)
    flen = layout.flen
    step = 4096  # frames per tx batch
    for a in range(f0, f1, step):
        b = min(f1, a + step)
        nf = b - a
        data = torch.from_numpy(payload_bytes(a * layout.bpf, nf * layout.bpf)).to(device)
        fr = torch.empty((nf * flen,), dtype=torch.complex128, device=device)
        modem.tx_frames(data, nf, fr)
        ramp = torch.arange(flen, dtype=torch.float64, device=device)[None, :]
        cfo = torch.from_numpy(layout.cfo[a:b, None]).to(device)
        ph = torch.from_numpy(layout.phase[a:b, None]).to(device)
        fr = fr.view(nf, flen) * torch.polar(torch.ones_like(cfo * ramp), 2 * np.pi * cfo * ramp + ph)
        idx = torch.from_numpy(layout.starts[a:b, None] - lo).to(device) + ramp.long()
        ok = (idx >= 0) & (idx < n)
        x[idx[ok]] = fr[ok]
        del fr, idx, ok
    sig = 10 ** (-layout.snr_db / 20) / np.sqrt(2)
    for blk in range(lo // NOISE_BLOCK, (hi - 1) // NOISE_BLOCK + 1 if n else 0):
        g = torch.Generator(device=device).manual_seed((layout.seed << 32) + blk)
        z = torch.randn((NOISE_BLOCK, 2), dtype=torch.float64, device=device, generator=g) * sig
        b0 = blk * NOISE_BLOCK
        s0, s1 = max(lo, b0), min(hi, b0 + NOISE_BLOCK)
        x[s0 - lo:s1 - lo] += torch.view_as_complex(z[s0 - b0:s1 - b0].contiguous())
        del z
    if i16:
        x = (torch.view_as_real(x) * float(p["mult"])).round().clamp(-32768, 32767).to(torch.int16).reshape(-1)
    return x
