"""Drop-in runs on the GPU: the class-surface compatibility layer
(c-ofdm_amd/compat) driving the HIP modem, through (1) this repo's own
main.cpp-style loopback app and (2) the reference's OWN main/tx/rx apps built
unchanged against the compat headers (oracle/_ref/, built in the build
container by `make -C oracle dropin`; skipped where absent). The SDR is the
file/loopback stand-in (compat/include/sdr/sdr.hpp)."""
import os
import subprocess

import numpy as np
import pytest

import oracle as O
from common import D, G, golden

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LOOPBACK = os.path.join(ROOT, "c-ofdm_amd", "bin", "ofdm_loopback")
REF_BIN = os.path.join(ROOT, "oracle", "_ref")
GD = golden()

KEYS = {"fft_size": "fft_size", "num_data_subc": "num_data_subc", "num_pilot_subc": "num_pilot_subc",
        "cp_size": "cp_size", "num_symb": "num_symb", "num_pr_symb": "num_pr_symb", "pr_sin_len": "pr_sin_len",
        "pr_seed": "pr_seed", "pr_level": "pr_level", "t2sin_size": "T2sin_size", "t2_sin_f1": "T2_sin_f1",
        "t2_sin_f2": "T2_sin_f2", "t2_sin_level": "T2_sin_level", "smooth": "smooth", "mod_type": "modType",
        "pilot_ampl": "pilot_ampl", "mult": "mult", "rx_buf_size": "rx_buf_size", "iterations": "iterations"}


def write_config(d, cfg, **extra):
    os.makedirs(os.path.join(d, "config"), exist_ok=True)
    path = os.path.join(d, "config", "config.txt")
    with open(path, "w") as f:
        f.write("# written by tests/test_dropin_gpu.py\n")
        for k, v in dict(cfg, **extra).items():
            f.write(f"{KEYS.get(k, k)} = {v}\n")
        f.write("bw_hz = 10000000\nfs_hz = 5000000\nlo_hz = 2800000000\nhardwaregain = 50\n"
                "tx_cycle_buf = 0\ntx_time_int = 0\n")
    return path


def run(cmd, cwd, env=None, timeout=180):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run(cmd, cwd=cwd, env=e, capture_output=True, text=True, timeout=timeout)


def test_loopback_app_default_config(tmp_path):
    cfg = write_config(tmp_path, D)
    r = run([LOOPBACK, cfg, "", str(tmp_path / "data")], tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ACCURACY: 1" in r.stdout
    cons = np.fromfile(tmp_path / "data" / "constell.bin", np.float64)
    assert cons.size == 2 * D["num_data_subc"] * D["num_symb"]


def test_loopback_app_golden_config_regenerates_source_bin(tmp_path):
    """Golden BPSK config + the golden payload text through the drop-in layer:
    the tx frame dumped to data/source.bin equals the reference's file."""
    cfg = write_config(tmp_path, G)
    pay = tmp_path / "payload.bin"
    pay.write_bytes(GD["payload_text"].tobytes())
    r = run([LOOPBACK, cfg, str(pay), str(tmp_path / "data")], tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    src = np.fromfile(tmp_path / "data" / "source.bin", np.int16)
    assert np.array_equal(src, GD["source"])


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_BIN, "rx")), reason="drop-in reference apps not built")
def test_reference_rx_app_decodes_golden_capture(tmp_path):
    """The reference's own rx.cpp (unchanged) streams the golden capture
    (data/data.bin) through the SDR stand-in, detects and decodes the frame and
    writes its payload to Res.wav. rx.cpp tests the T2 marker only on its
    256-sample block grid (Frame.hpp:164) after a one-frame carry region, so the
    capture starts 128 samples earlier to put frame 1 on that grid."""
    write_config(tmp_path, G, iterations=12)
    cap = tmp_path / "capture_f64.bin"
    x = np.concatenate([np.zeros(128, np.complex128), GD["data"]])
    np.stack([x.real, x.imag], 1).astype(np.float64).tofile(cap)
    r = run([os.path.join(REF_BIN, "rx")], tmp_path, {"OFDM_SDR_RX_FILE": str(cap), "OFDM_SDR_RX_FORMAT": "f64"})
    assert r.returncode == 0, (sorted(os.listdir(tmp_path)), r.stderr[-3000:])
    res = (tmp_path / "Res.wav").read_bytes()
    want = GD["payload_text"].tobytes()
    assert len(res) >= len(want) and len(res) % len(want) == 0
    assert res[: len(want)] == want
    assert "SEQ:0" in r.stdout and (tmp_path / "LOG.txt").exists()


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_BIN, "main")), reason="drop-in reference apps not built")
def test_reference_main_app_loopback(tmp_path):
    """The reference's own main.cpp (unchanged): MAC-framed text -> tx -> SDR
    stand-in -> full sync chain -> demod -> ACCURACY 1, data/*.bin written."""
    write_config(tmp_path, D)
    os.makedirs(tmp_path / "data")
    text = (GD["payload_text"].tobytes() * 8)
    (tmp_path / "WARANDPEACE.txt").write_bytes(text)
    r = run([os.path.join(REF_BIN, "main")], tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "ACCURACY: 1\n" in r.stdout and "Bit-level ACCURACY: 1\n" in r.stdout, r.stdout
    assert "FRAME FROM 1 TO 0 SEQ 0" in r.stdout
    g = O.geometry(D)
    assert np.fromfile(tmp_path / "data" / "source.bin", np.int16).size == 2 * g["frame_len"]
    assert (tmp_path / "data.txt").read_bytes() == text[: g["bytes_per_frame"] - 8]


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_BIN, "tx")), reason="drop-in reference apps not built")
def test_reference_tx_app_frames_decode(tmp_path):
    """The reference's own tx.cpp (unchanged) frames a file into int16 IQ via
    the SDR stand-in (data/tx.bin layout); the GPU rx decodes every frame."""
    torch = pytest.importorskip("torch")
    import ofdm_mi355x as M
    write_config(tmp_path, D)
    g = O.geometry(D)
    pay = g["bytes_per_frame"] - 8
    body = np.random.default_rng(3).integers(0, 256, 3 * pay, dtype=np.uint8).tobytes()
    (tmp_path / "FlyMeToTheMoon_mono.wav").write_bytes(body)
    txf = tmp_path / "tx.bin"
    r = run([os.path.join(REF_BIN, "tx")], tmp_path, {"OFDM_SDR_TX_FILE": str(txf)})
    assert r.returncode == 0, r.stderr[-3000:]
    iq16 = np.fromfile(txf, np.int16)
    nfr = iq16.size // (2 * g["frame_len"])
    assert nfr == 3
    m = M.Modem(D, 0)
    d16 = torch.from_numpy(iq16).cuda()
    x = torch.zeros((iq16.size // 2,), dtype=torch.complex128, device="cuda")
    m.int16_to_double(d16, iq16.size // 2, x)
    out = torch.zeros((nfr * g["bytes_per_frame"],), dtype=torch.uint8, device="cuda")
    hdr = D["t2sin_size"] + g["preamble_len"]
    m.rx(x[hdr:], nfr, frame_stride=g["frame_len"], bytes_out=out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(nfr, -1)[:, 8:].tobytes()
    assert got == body
    m.close()


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_BIN, "main")), reason="drop-in reference apps not built")
def test_reference_main_writes_python_code_file_contract(tmp_path):
    """The files the reference's main.cpp:74-78 writes for python_code/ofdm.py
    (and graph.py), from the reference's own main on the golden G config and
    payload: data/source.bin equals the reference's committed capture bit for
    bit; data.bin, t2_sin_corr.bin, phases.bin and constell.bin have the flat
    f64 layouts ofdm.py:9-54 reads (x[::2] + 1j*x[1::2] for complex), and
    their contents equal the oracle's computation on the written data.bin
    (T2 correlation, the main.cpp:52-71 sync chain and equalised points)."""
    write_config(tmp_path, G)
    os.makedirs(tmp_path / "data")
    (tmp_path / "WARANDPEACE.txt").write_bytes(GD["payload_text"].tobytes() * 4)
    r = run([os.path.join(REF_BIN, "main")], tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "ACCURACY: 1\n" in r.stdout, r.stdout
    g = O.geometry(G)
    d = tmp_path / "data"
    assert np.array_equal(np.fromfile(d / "source.bin", np.int16), GD["source"])
    # python_code/ofdm.py's readers
    raw = np.fromfile(d / "data.bin", dtype=np.float64)
    x = raw[::2] + 1j * raw[1::2]
    ring_len = g["frame_len"] * (G["rx_buf_size"] + 1)  # FRAME_FORM::from_sdr_buf (Frame.cpp:229)
    assert x.size == ring_len
    corr = np.fromfile(d / "t2_sin_corr.bin", dtype=np.float64)
    assert corr.size == ring_len // G["t2sin_size"]
    assert np.abs(corr - O.t2_corr(G, x)).max() < 1e-12
    ph = np.fromfile(d / "phases.bin", dtype=np.float64)
    ph = ph[::2] + 1j * ph[1::2]
    assert ph.size == G["num_data_subc"]
    assert np.abs(np.abs(ph) - 1).max() < 1e-12
    cons = np.fromfile(d / "constell.bin", dtype=np.float64)
    cons = cons[::2] + 1j * cons[1::2]
    assert cons.size == g["npts"]
    hit = O.find_t2sin(G, x, 0)
    pb = O.find_preamble(G, x, hit) + 1
    _, ocons, obytes = O.decode_frame(G, x[pb: pb + g["preamble_len"] + g["message_len"]])
    assert np.abs(cons - ocons).max() / np.abs(ocons).max() < 1e-9
    assert obytes.tobytes() == GD["payload"].tobytes()


SELFTEST = os.path.join(ROOT, "c-ofdm_amd", "bin", "compat_selftest")


def gapped_capture(txf, frame_len):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from dropin_rx_timing import gapped_capture as gc
    gc(txf, frame_len)


@pytest.mark.parametrize("name", ["D", "G"])
def test_compat_device_mirrors_equal_staged_path(tmp_path, name):
    """c-ofdm_amd/apps/compat_selftest: a FRAME_FORM's device-mirrored buffers
    (the forms move only what the host changed, copy back what they change in
    place) give bit-identical results to the same members on a plain vector
    (staged through the pinned arena): fresh frames, the same frame copied in
    again after the in-place members, partial host writes between members,
    the int16 ring and direct host writes to from_sdr_buf; and
    PREAMBLE_FORM::chan_char equals Frame.hpp:375-385 on fft()'s output."""
    cfg = write_config(tmp_path, {"D": D, "G": G}[name])
    r = run([SELFTEST, cfg, "12"], tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "SELFTEST OK" in r.stdout


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_BIN, "rx")), reason="drop-in reference apps not built")
def test_reference_tx_rx_apps_stream_120_frames(tmp_path):
    """The reference's own tx.cpp frames a 120-frame payload file into the SDR
    stand-in's int16 capture (data/tx.bin layout); its own rx.cpp streams the
    capture (with 0-3000-sample silences between the bursts) through its
    ring buffer, the detection walk and the per-frame sync chain on the
    device-mirrored FRAME_FORM, and writes every payload it decodes to
    Res.wav. The written payloads must be exactly, in order, those of the
    frames rx.cpp's loop locates when replayed by the oracle on a real ring
    buffer (orc_rx_app_walk: the zero header, 40-frame refills, the refill
    without carry on a T2 miss, the carries, the iteration cap), each decoded
    by the oracle's main.cpp:60-80 chain; and the stream API in ring mode
    locates the same frames."""
    nfr = 120
    iters = nfr + 60
    write_config(tmp_path, D, iterations=iters)
    g = O.geometry(D)
    pay = g["bytes_per_frame"] - 8
    # per-frame distinct payloads (frame f's bytes shift by 249 f mod 256: 256 distinct frames)
    body = bytes((i * 131 + 7 + (i // pay) * 17) & 0xFF for i in range(nfr * pay))
    (tmp_path / "FlyMeToTheMoon_mono.wav").write_bytes(body)
    txf = tmp_path / "tx.bin"
    r = run([os.path.join(REF_BIN, "tx")], tmp_path, {"OFDM_SDR_TX_FILE": str(txf)})
    assert r.returncode == 0, r.stderr[-3000:]
    assert np.fromfile(txf, np.int16).size == 2 * nfr * g["frame_len"]
    gapped_capture(txf, g["frame_len"])  # silences between the bursts, as on air
    r = run([os.path.join(REF_BIN, "rx")], tmp_path, {"OFDM_SDR_RX_FILE": str(txf)}, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = (tmp_path / "Res.wav").read_bytes()
    assert len(res) % pay == 0
    got = [res[i * pay:(i + 1) * pay] for i in range(len(res) // pay)]
    chunks = [body[i * pay:(i + 1) * pay] for i in range(nfr)]
    # the oracle's replay of rx.cpp's loop over the same SDR samples
    w = np.fromfile(txf, np.int16).astype(np.float64)
    x = w[0::2] + 1j * w[1::2]
    pbs = O.rx_app_walk(D, x, iterations=iters, stop_at_end=False)
    span = g["preamble_len"] + g["message_len"]
    xz = np.concatenate([x, np.zeros(span, np.complex128)])  # the stand-in's zeros past the capture
    want = [O.decode_frame(D, xz[pb:pb + span])[2][8:].tobytes() for pb in pbs]
    assert len(got) == len(want), f"rx wrote {len(got)} payloads, its loop locates {len(want)} frames"
    assert got == want
    idx = [chunks.index(c) if c in chunks else -1 for c in got]
    assert -1 not in idx and idx == sorted(idx) and len(set(idx)) == len(idx)
    assert len(got) >= 0.9 * nfr
    # the stream API (ring mode, the config's R) locates the same frames
    import torch
    import ofdm_mi355x as M
    m = M.Modem(D, 0)
    inside = [pb for pb in pbs if pb + span <= len(x)]
    pb_out = torch.full((nfr + 8,), -1, dtype=torch.int64, device="cuda")
    nf = m.rx_stream(torch.from_numpy(x).cuda(), len(x), nfr + 8, pb_out=pb_out)
    torch.cuda.synchronize()
    assert nf == len(inside) and list(pb_out[:nf].cpu().numpy()) == inside
    m.close()
