"""One context per host thread (include/ofdm_mi355x.h: "One ofdm_ctx per
thread"): two threads, each with its own context and HIP stream, create their
contexts and run tx + rx at the same time on one GPU. The launch helpers'
process-wide state (the per-(kernel, device) LDS opt-in, the walker slot
cache) is shared between them; each thread's bytes and constellation must
equal the oracle's, as when run alone."""
import threading

import numpy as np
import pytest

import oracle as O
from common import ALL_CONFIGS, payload, rel_err

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import ofdm_mi355x as M  # noqa: E402


def _job(name, seed, reps, out, barrier):
    try:
        cfg = ALL_CONFIGS[name]
        g = O.geometry(cfg)
        nf = 3
        data = payload(nf * g["bytes_per_frame"], seed=seed)
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            d_data = torch.from_numpy(data).cuda()
            iq = torch.zeros((nf * g["message_len"],), dtype=torch.complex128, device="cuda")
            cons = torch.zeros((nf * g["npts"],), dtype=torch.complex128, device="cuda")
            got = torch.zeros((nf * g["bytes_per_frame"],), dtype=torch.uint8, device="cuda")
            barrier.wait()  # contexts created and launches issued concurrently
            m = M.Modem(cfg, 0)
            for _ in range(reps):
                m.tx(d_data, nf, iq)
                m.rx(iq, nf, constell_out=cons, bytes_out=got)
            st.synchronize()
            out[name] = (data, iq.cpu().numpy(), cons.cpu().numpy(), got.cpu().numpy())
    except BaseException as e:  # reported by the main thread
        out[name] = e


def test_two_threads_two_contexts_match_oracle():
    names = ["D", "B"]
    out, barrier = {}, threading.Barrier(len(names))
    ths = [threading.Thread(target=_job, args=(n, 11 + i, 20, out, barrier)) for i, n in enumerate(names)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=100)
    for n in names:
        r = out.get(n)
        assert r is not None, f"thread {n} did not finish"
        if isinstance(r, BaseException):
            raise r
        data, iq, cons, got = r
        cfg = ALL_CONFIGS[n]
        g = O.geometry(cfg)
        assert rel_err(iq, O.tx_batch(cfg, data, 3)) < 1e-10
        ocons, obytes, _ = O.rx_batch(cfg, iq, 3, g["message_len"])
        assert rel_err(cons, ocons) < 1e-10
        assert np.array_equal(got, obytes) and np.array_equal(got, data)
