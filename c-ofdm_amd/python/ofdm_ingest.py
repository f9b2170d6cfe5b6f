"""ofdm_ingest — a stream that keeps arriving: host-to-device ingest of the
SDR's int16 wire samples overlapped with the walk + decode (SURVEY §2.2's
mapping of rx.cpp's reader thread, rx.cpp:58-91, onto HIP streams).

rx.cpp runs a reader thread that fills one SDR buffer while the DSP loop
walks the other (buf[2], two semaphores). Here the samples sit in page-locked
host memory (standing in for the SDR's DMA target) and reach the GPU in
chunks through two device buffers:

* chunk k owns the samples [k*C, (k+1)*C) and its device buffer holds the
  slice [own_lo - halo, own_hi + tail) of the stream (the halo covers the
  previous call's exit state, the tail the frame crossing own_hi:
  ofdm_stream.stream_halo / stream_tail, the shard margins);
* the copy of chunk k+1 runs on a copy stream while chunk k's walk and
  decode (ofdm_rx_stream_shard on the compute stream) run; a buffer is
  refilled only after the decode that read it (events both ways);
* chunk k's walk starts from chunk k-1's exit state, so the chunked receive
  is rx.cpp's one sequential walk (the ring state travels with it) and its
  frames, in order, equal one device-resident call over the whole stream.
"""
from __future__ import annotations

import numpy as np

import ofdm_stream as SS


class StreamIngest:
    """Chunked receive of a host-resident int16 wire stream on one context.

    host16: page-locked torch int16 tensor (2n values: complex<int16> pairs);
    chunk: core samples per call; outputs: device tensors pb_out / bytes_out /
    constell_out / cfo_out sized for every frame of the stream (filled in
    stream order)."""

    def __init__(self, modem, params: dict, host16, n: int, chunk: int, outputs: dict, device, max_frames: int):
        import torch
        self.modem, self.n, self.chunk = modem, n, chunk
        self.halo, self.tail = SS.stream_halo(params), SS.stream_tail(params)
        self.host16, self.outputs, self.device, self.max_frames = host16, outputs, device, max_frames
        self.npts = params["num_data_subc"] * params["num_symb"]
        self.bpf = params["num_data_subc"] * params["num_symb"] * params["mod_type"] // 8
        span = chunk + self.halo + self.tail
        self.bufs = [torch.empty((2 * span,), dtype=torch.int16, device=device) for _ in range(2)]
        self.copy_stream = torch.cuda.Stream(device)
        self.compute_stream = torch.cuda.Stream(device)
        self.copied = [torch.cuda.Event() for _ in range(2)]
        self.consumed = [torch.cuda.Event() for _ in range(2)]
        self.ring = modem.stream_ring()

    def slices(self):
        """(own_lo, own_hi, slice_lo, slice_hi) per chunk."""
        out = []
        for lo in range(0, self.n, self.chunk):
            hi = min(self.n, lo + self.chunk)
            out.append((lo, hi, max(0, lo - self.halo), min(self.n, hi + self.tail)))
        return out

    def _copy(self, k: int, sl) -> None:
        import torch
        _, _, s0, s1 = sl
        b = self.bufs[k % 2]
        with torch.cuda.stream(self.copy_stream):
            if k >= 2:
                self.copy_stream.wait_event(self.consumed[k % 2])  # the decode that read this buffer is done
            b[:2 * (s1 - s0)].copy_(self.host16[2 * s0:2 * s1], non_blocking=True)
            self.copied[k % 2].record(self.copy_stream)

    def run(self) -> dict:
        """Every chunk in turn; returns {frames, exit, calls}. The decodes may
        still run on the compute stream when it returns (synchronise it)."""
        sls = self.slices()
        if not sls:
            return {"frames": 0, "calls": 0, "exit": self.modem.initial_state()}
        # rx.cpp's first walk state (absolute; ring mode: in the zero header
        # before sample 0, pos < 0); None once the walk has ended
        state = self.modem.initial_state()
        done = 0
        self._copy(0, sls[0])
        for k, sl in enumerate(sls):
            own_lo, own_hi, s0, s1 = sl
            if k + 1 < len(sls):
                self._copy(k + 1, sls[k + 1])  # the next chunk crosses PCIe while this one is received
            if state is None:  # the walk ended (samples ran out): nothing more is owned
                break
            if k > 0 and state[0] < s0:
                raise RuntimeError(f"exit state {state} before chunk {k}'s slice start {s0}: halo too short")
            self.compute_stream.wait_event(self.copied[k % 2])
            rel = (state[0] - s0, (state[1] - s0) if self.ring else 0)
            o = self.outputs
            cap = self.max_frames - done
            nf, _, _, ex = self.modem.rx_stream_shard(
                self.bufs[k % 2], s1 - s0, rel, own_lo - s0, own_hi - s0, cap,
                pb_out=o["pb_out"][done:], bytes_out=o["bytes_out"][done * self.bpf:],
                constell_out=o["constell_out"][done * self.npts:], cfo_out=o["cfo_out"][done:],
                i16=True, located_cap=0, stream=self.compute_stream)
            self.consumed[k % 2].record(self.compute_stream)
            # pb_out is slice-relative: shift this call's entries to stream coordinates
            got = min(nf, cap)
            if got and s0:
                import torch
                with torch.cuda.stream(self.compute_stream):
                    o["pb_out"][done:done + got] += s0
            done += got
            state = None if ex[0] < 0 else (ex[0] + s0, (ex[1] + s0) if self.ring else 0)
        return {"frames": done, "calls": len(sls), "exit": state if state is not None else (-1, 0)}


def host_pinned_i16(x16_dev):
    """A page-locked host copy of a device int16 stream (the SDR's DMA target)."""
    import torch
    h = torch.empty(x16_dev.shape, dtype=torch.int16, pin_memory=True)
    h.copy_(x16_dev)
    return h
