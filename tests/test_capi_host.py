"""C-ABI host-side checks (no GPU compute): the library loads, exports every
entry point include/ofdm_mi355x.h declares, and its config parser behaves like
the reference's parse_config (config/parser.cpp:4-33)."""
import ctypes as C
import os
import re

import pytest

import ofdm_mi355x as M
import oracle as O


def header_functions():
    with open(M.HEADER) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ofdm_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    L = M.lib()
    declared = header_functions()
    assert len(declared) >= 20
    missing = [n for n in declared if not hasattr(L, n)]
    assert missing == []
    assert set(declared) == set(M.SIGNATURES), "python binding out of sync with the header"
    assert L.ofdm_abi_version() == 5


def test_params_default_is_committed_config():
    p = M.params_default()
    assert p.as_dict() == O.DEFAULT


CFG_TEXT = """# comment line
fft_size        = 2048
  num_data_subc = 1024
num_pilot_subc=32
cp_size = 5 12
modType = 2
not a key value line
T2_sin_f1 = -17
"""


def _ref_lookup(path, key):
    v = C.c_long()
    rc = O.ref().ref_parse_config(path.encode(), key.encode(), C.byref(v))
    return rc, v.value


@pytest.mark.skipif(not O.ref_available(), reason="reference parser not built here")
def test_config_parser_matches_reference(tmp_path):
    path = str(tmp_path / "cfg.txt")
    with open(path, "w") as f:
        f.write(CFG_TEXT)
    p = M.params_from_config(path)
    for key, field in (("fft_size", "fft_size"), ("num_data_subc", "num_data_subc"),
                       ("num_pilot_subc", "num_pilot_subc"), ("cp_size", "cp_size"),
                       ("modType", "mod_type"), ("T2_sin_f1", "t2_sin_f1"), ("num_symb", "num_symb")):
        rc, v = _ref_lookup(path, key)
        assert rc == 0
        assert getattr(p, field) == v, key
        assert M.config_lookup(path, key) == v
    # the reference's committed config/config.txt
    ref_cfg = "/root/reference/config/config.txt"
    if os.path.exists(ref_cfg):
        assert M.params_from_config(ref_cfg).as_dict() == O.DEFAULT


def test_config_errors(tmp_path):
    with pytest.raises(M.OfdmError) as e:
        M.params_from_config(str(tmp_path / "missing.txt"))
    assert e.value.code == -4 and "Cannot open config file" in str(e.value)
    bad = tmp_path / "bad.txt"
    bad.write_text("fft_size = abc\n")
    with pytest.raises(M.OfdmError) as e:
        M.params_from_config(str(bad))
    assert e.value.code == -6
    if O.ref_available():
        assert _ref_lookup(str(bad), "fft_size")[0] == -6
        assert _ref_lookup(str(tmp_path / "missing.txt"), "x")[0] == -4


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(M.OfdmError) as e:
        M.Modem(O.DEFAULT)
    assert e.value.code in (-3,)


def test_reference_apps_build_unchanged_against_compat_headers():
    """main.cpp / tx.cpp / rx.cpp of the reference compile and link against
    c-ofdm_amd/compat/include + the MI355X library (oracle/Makefile `dropin`)."""
    import subprocess
    if not os.path.exists("/root/reference/main.cpp"):
        pytest.skip("reference absent")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["make", "-s", "-C", os.path.join(root, "c-ofdm_amd")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    r = subprocess.run(["make", "-s", "-C", os.path.join(root, "oracle"), "dropin"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    for app in ("main", "tx", "rx"):
        path = os.path.join(root, "oracle", "_ref", app)
        assert os.access(path, os.X_OK)
        ldd = subprocess.run(["ldd", path], capture_output=True, text=True).stdout
        assert "libofdm_compat.so" in ldd and "not found" not in ldd


def test_shard_range_and_stream_plan_match_python_sharding():
    """The multi-GPU C-ABI (ofdm_shard_range, ofdm_stream_shard_plan) gives
    the frame and stream shards the Python launcher uses (ofdm_dist.shard,
    ofdm_stream.shard_stream with its halo / tail): no GPU needed."""
    import ofdm_dist
    import ofdm_stream as SS
    L = M.lib()
    first, count = C.c_size_t(), C.c_size_t()
    for total in (0, 1, 7, 8192, 30517, 10 ** 9 + 3):
        for world in (1, 2, 3, 4, 8):
            got = []
            for r in range(world):
                assert L.ofdm_shard_range(total, world, r, C.byref(first), C.byref(count)) == 0
                assert (first.value, count.value) == ofdm_dist.shard(total, world, r)
                got.append((first.value, count.value))
            assert sum(c for _, c in got) == total
    assert L.ofdm_shard_range(10, 2, 2, C.byref(first), C.byref(count)) != 0  # rank out of range
    for name, cfg in (("D", O.DEFAULT), ("B", O.CONFIG_B)):
        p = M.Params.make(**cfg)
        halo, tail = SS.stream_halo(cfg), SS.stream_tail(cfg)
        v = [C.c_long() for _ in range(4)]
        for n in (10 ** 6, 132_314_816):
            for world in (1, 2, 4, 8):
                for r in range(world):
                    assert L.ofdm_stream_shard_plan(C.byref(p), n, world, r, *[C.byref(x) for x in v]) == 0
                    assert tuple(x.value for x in v) == SS.shard_stream(n, world, r, halo, tail), (name, n, world, r)


def test_multigpu_app_plan_only():
    """apps/ofdm_multigpu.cpp --plan-only: the C++ job's shard plan without a GPU."""
    import json
    import subprocess
    import ofdm_dist
    app = os.path.join(os.path.dirname(M.HEADER), "..", "c-ofdm_amd", "bin", "ofdm_multigpu")
    if not os.path.exists(app):
        pytest.skip("ofdm_multigpu not built")
    out = subprocess.run([app, "--plan-only", "--gpus", "8", "--total-frames", "30517"], capture_output=True,
                         text=True, timeout=60, check=True).stdout
    d = json.loads(out)
    assert d["world"] == 8 and len(d["ranks"]) == 8
    for r in d["ranks"]:
        assert (r["first"], r["count"]) == ofdm_dist.shard(30517, 8, r["rank"])


def test_stream_report_pack_and_stitch_plan_match_python_protocol():
    # the C-ABI's report row and stitch plan (ofdm_stream_report_pack /
    # ofdm_stream_stitch_plan, for C/C++ hosts) against ofdm_stream.py's
    # pack_report / unpack_report / stitch_plan on random reports: accepted
    # ranks, re-walks from the predecessor's exit state (before the slice:
    # moved forward on the T2 grid), walks that ran out, long located lists
    import numpy as np
    import ofdm_stream as SS
    L = M.lib()
    rng = np.random.default_rng(7)
    t2 = 256
    for trial in range(300):
        world = int(rng.integers(1, 6))
        cap = int(rng.integers(1, 9))
        reps, rows_c = [], []
        base = 0
        for r in range(world):
            own_lo = base
            own_hi = own_lo + int(rng.integers(10000, 60000))
            slice_lo = max(0, own_lo - int(rng.integers(0, 20000)))
            base = own_hi
            nloc = int(rng.integers(0, 3 * cap + 2))
            pbs = np.sort(rng.choice(np.arange(slice_lo, own_hi + 8000, 97), size=nloc, replace=False))
            if r > 0 and reps and reps[-1].located and rng.random() < 0.5:  # share a frame with the predecessor
                shared = reps[-1].located[int(rng.integers(0, len(reps[-1].located)))][0]
                pbs = np.sort(np.unique(np.append(pbs, shared)))
            lags = rng.integers(0, 2, size=len(pbs)).astype(np.uint8)
            ex = (-1, 0) if rng.random() < 0.1 else (int(own_hi - rng.integers(-3000, 6000)), int(rng.integers(0, 10**6)))
            true_start = r == 0 or rng.random() < 0.2
            rep = SS.ShardReport(r, slice_lo, own_lo, own_hi, [(int(p), int(g)) for p, g in zip(pbs, lags)], ex,
                                 true_start)
            reps.append(rep)
            row_py = SS.pack_report(rep, cap)
            row = np.empty(SS.HEADER + 2 * cap, dtype=np.int64)
            la = np.ascontiguousarray(pbs, dtype=np.int64)
            M.check(L.ofdm_stream_report_pack(r, slice_lo, own_lo, own_hi, la.ctypes.data, lags.ctypes.data, len(pbs),
                                              C.byref(M.WalkState(*ex)), int(true_start), cap, row.ctypes.data))
            assert np.array_equal(row, row_py), (trial, r)
            rows_c.append(row)
        plan_py = SS.stitch_plan([SS.unpack_report(rw, cap) for rw in rows_c], t2)
        allr = np.ascontiguousarray(np.stack(rows_c))
        rk, st = C.c_int(), M.WalkState()
        M.check(L.ofdm_stream_stitch_plan(allr.ctypes.data, world, cap, t2, C.byref(rk), C.byref(st)))
        if plan_py is None:
            assert rk.value == -1
        else:
            assert (rk.value, (st.pos, st.ring_end)) == (plan_py[0], tuple(plan_py[1])), trial
