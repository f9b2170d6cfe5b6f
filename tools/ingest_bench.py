#!/usr/bin/env python3
"""Host-ingest stream throughput (ofdm_ingest.StreamIngest) against chunk
size: bench.py's config-4 int16 wire stream in page-locked host memory,
received chunk by chunk; prints one JSON line per chunk size with the end-to-end
samples/s, the PCIe H2D ceiling measured on the same stream, and whether the
outputs equal one device-resident call."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "c-ofdm_amd", "python")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16384)
    ap.add_argument("--chunks", default="1048576,4194304,16777216")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    import bench
    import ofdm_mi355x as M
    for ch in (int(v) for v in a.chunks.split(",")):
        args = argparse.Namespace(stream_frames=a.frames, ingest_chunk=ch, ingest_reps=a.reps)
        r = bench.stream_ingest_leg(args, torch.device("cuda", 0), M)
        print(json.dumps({k: r[k] for k in ("chunk_samples", "calls_per_stream", "value", "ms_per_stream",
                                             "frac_of_pcie_ceiling", "outputs_equal_device_resident_call")}
                         | {"pcie_samples_per_s": r["pcie_h2d"]["samples_per_s"]}), flush=True)
        torch.cuda.empty_cache()
    time.sleep(0)


if __name__ == "__main__":
    main()
