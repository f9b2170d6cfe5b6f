"""Regenerate tests/golden/ from the reference's own data files.

Run in the build container only (needs /root/reference). The fixtures are
DATA: the outputs of the reference's one BPSK main.cpp run (reference
data/*.bin, data.txt), re-encoded compactly. No reference source is copied.

  reference file            -> fixture
  data/source.bin  (int16)  -> source_bin.npy        (6016 x {re,im} int16, verbatim)
  data/data.bin    (f64)    -> data_bin_i16.npz      (integer-valued, stored losslessly as int16)
  data/t2_sin_corr.bin      -> t2_sin_corr.npy       (963 f64)
  data/phases.bin           -> phases.npy            (256 complex128)
  data/constell.bin         -> constell.npy          (2048 complex128)
  data/row.bin              -> row.npy               (5760 complex128, verbatim: a preamble+message region,
                                                      BASELINE config 4's named input)
  data.txt                  -> data_txt.bin          (248-B decoded payload)
  derived (verified by tests/test_oracle_golden.py): golden.json
"""
import json
import os

import numpy as np

REF = os.environ.get("OFDM_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    src = np.fromfile(os.path.join(REF, "data/source.bin"), np.int16)
    np.save(os.path.join(HERE, "source_bin.npy"), src)
    d = np.fromfile(os.path.join(REF, "data/data.bin"), np.float64)
    assert np.all(d == np.round(d)) and np.abs(d).max() < 32768
    np.savez_compressed(os.path.join(HERE, "data_bin_i16.npz"), iq=d.astype(np.int16))
    np.save(os.path.join(HERE, "t2_sin_corr.npy"), np.fromfile(os.path.join(REF, "data/t2_sin_corr.bin")))
    np.save(os.path.join(HERE, "phases.npy"), np.fromfile(os.path.join(REF, "data/phases.bin")).view(np.complex128))
    np.save(os.path.join(HERE, "constell.npy"),
            np.fromfile(os.path.join(REF, "data/constell.bin")).view(np.complex128))
    np.save(os.path.join(HERE, "row.npy"), np.fromfile(os.path.join(REF, "data/row.bin")).view(np.complex128))
    with open(os.path.join(REF, "data.txt"), "rb") as f:
        payload = f.read()
    with open(os.path.join(HERE, "data_txt.bin"), "wb") as f:
        f.write(payload)
    meta = {
        "config": {  # config/config.txt with modType=1: the run that wrote data/*.bin
            "fft_size": 512, "num_data_subc": 256, "num_pilot_subc": 8, "cp_size": 128,
            "num_symb": 8, "num_pr_symb": 1, "pr_sin_len": 128, "pr_seed": 42, "pr_level": 500,
            "t2sin_size": 256, "t2_sin_f1": 17, "t2_sin_f2": 51, "t2_sin_level": 800, "smooth": 5,
            "mod_type": 1, "pilot_ampl": 2500, "mult": 200, "rx_buf_size": 40, "iterations": 10000},
        # MAC header of the golden frame: tx_id=1, rx_id=0, seq=0, cs=0x577E (LE), SURVEY §2.1 row 10
        "mac_header": [1, 0, 0, 0, 0, 0, 0x7E, 0x57],
        "preamble_bytes": [95, 203, 243, 46, 187, 199, 153, 152, 39, 114, 39, 25, 14, 117, 221, 85,
                           153, 36, 181, 166, 5, 14, 248, 184, 213, 240, 54, 0, 46, 254, 46, 158],
        "t2_first_block_start": 10752,
        "t2_blocks": [42, 74],
        "preamble_begin": [11040, 19302],
        "cfo_frame1": -0.0037109375,
    }
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
