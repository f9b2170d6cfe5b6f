#!/usr/bin/env python3
"""walk_prof.py — per-walker phase clocks of stream_walk_kernel (timing
experiment; needs the exp/libofdm_wprof.so build: tools/build_variant.sh wprof
-DOFDM_WALK_PROF, selected with OFDM_MI355X_LIB). Runs tools/stream_bench.py
once, then prints where the walkers spent their cycles."""
import ctypes as C
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "c-ofdm_amd", "python"))
import stream_bench  # noqa: E402
import ofdm_mi355x as M  # noqa: E402

sys.argv = [sys.argv[0], "--reps", "1"] + sys.argv[1:]
stream_bench.main()
lib = M.lib()
buf = np.zeros(2 * 8192 * 8 + 16, dtype=np.uint64)
fb = np.zeros(1, dtype=np.uint64)
assert lib.ofdm_walk_prof(buf.ctypes.data_as(C.c_void_p), fb.ctypes.data_as(C.c_void_p)) == 0
q = buf[:8192 * 8].reshape(8192, 8).astype(np.float64)
sub = buf[8192 * 8:2 * 8192 * 8].reshape(8192, 8).astype(np.float64)
live = q[:, 5] > 0
q = q[live]
sub = sub[live]
tot, t2, n2, pre, npre, steps, w0, w1 = q.T
wall_us = (w1 - w0) / 100.0  # wall_clock64: 100 MHz
res = {
    "walkers": int(live.sum()),
    "steps_mean": steps.mean(), "t2_iters_mean": n2.mean(), "pre_mean": npre.mean(),
    "cyc_total_mean": tot.mean(), "cyc_t2_frac": t2.sum() / tot.sum(), "cyc_pre_frac": pre.sum() / tot.sum(),
    "cyc_per_t2_iter": t2.sum() / n2.sum(), "cyc_per_pre": pre.sum() / max(npre.sum(), 1),
    "wall_us_mean": wall_us.mean(), "wall_us_max": wall_us.max(), "wall_us_min": wall_us.min(),
    "start_spread_us": (w0.max() - w0.min()) / 100.0,
    "end_spread_us": (w1.max() - w1.min()) / 100.0,
    "fallbacks": int(fb[0]),
    # preamble search: load+fwd FFT, prefix+spectrum product, inverse FFT, decisions (cycles per search)
    "pre_sub": [round(float(x), 1) for x in sub[:, :4].sum(0) / npre.sum()],
    # T2 iteration: load + FFT, reduce + decision (cycles per iteration)
    "t2_sub": [round(float(x), 1) for x in sub[:, 4:6].sum(0) / n2.sum()],
    "corr_wall_steps": float(np.corrcoef(wall_us, steps)[0, 1]),
    "corr_wall_t2iters": float(np.corrcoef(wall_us, n2)[0, 1]),
    "corr_wall_cycles": float(np.corrcoef(wall_us, tot)[0, 1]),
    # stream_params_kernel phases, cycles per frame (thread 0): CP sums, symbol phases,
    # preamble correction, FFT, pilot/bin phases (4: incl. unwrap), sums, channel, ramps
    "params_phases": [round(float(x) / max(float(buf[-16 + 8]), 1.0), 1) for x in buf[-16:-8]],
    "cyc_per_us_min_max": [float((tot / wall_us).min()), float((tot / wall_us).max())],
}
np.savez(os.path.join("gpurun_out", "wprof%s.npz" % ("_i16" if "--i16" in sys.argv else "")), q=q, sub=sub)
print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}))
