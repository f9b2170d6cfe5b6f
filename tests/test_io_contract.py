"""The compat io/io.hpp free functions against the readers in the
reference's python_code (reference io/io.hpp:15-144):
* send_data -> /tmp/row_input, read as real_time_graph.py:24-33 does
  (int16 pairs, x[::2] + 1j*x[1::2]); the writer opens O_NONBLOCK and
  silently skips when no reader has the FIFO open (io.hpp:82-87);
* write_complex_to_pipe -> /tmp/fifo_frame, /tmp/fifo_constell, read as
  frame_pipe.py:25-43 does (flat f64 pairs until EOF);
* write_complex_to_file / write_double_to_file / read_complex_from_file:
  the flat data/*.bin layouts ofdm.py:9-54 reads.
A small host program compiled here against c-ofdm_amd/compat/include writes
them; no GPU is involved (the functions are header-only host code)."""
import os
import select
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMPAT = os.path.join(ROOT, "c-ofdm_amd", "compat", "include")

PROG = r'''
#include <complex>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
#include "io/io.hpp"
int main(int argc, char** argv) {
    const int n = 1000;
    std::vector<std::complex<int16_t>> s16(n);
    std::vector<std::complex<double>> s64(n);
    std::vector<double> d(n);
    for (int i = 0; i < n; ++i) {
        s16[i] = std::complex<int16_t>((int16_t)(i * 37 - 18000), (int16_t)(-i * 29 + 12345));
        s64[i] = std::complex<double>(i * 0.25 - 3.0, 1.0 / (i + 1));
        d[i] = i * 1e-3 - 0.5;
    }
    const std::string mode = argv[1];
    if (mode == "pipes") {
        send_data(argv[2], s16);
        write_complex_to_pipe(s64.begin(), s64.end(), argv[3]);
    } else if (mode == "nopipe") {
        send_data(argv[2], s16);  // no reader: returns without blocking or failing
    } else {
        const std::string dir = argv[2];
        write_complex_to_file(dir + "/c64.bin", s64);
        write_complex_to_file(dir + "/c16.bin", s16);
        write_double_to_file(dir + "/d.bin", d);
        std::vector<std::complex<double>> back(n);
        read_complex_from_file(dir + "/c64.bin", back.begin());
        for (int i = 0; i < n; ++i)
            if (back[i] != s64[i]) return 3;
    }
    return 0;
}
'''


@pytest.fixture(scope="module")
def prog(tmp_path_factory):
    d = tmp_path_factory.mktemp("io")
    src = d / "io_prog.cpp"
    src.write_text(PROG)
    exe = d / "io_prog"
    r = subprocess.run(["g++", "-O1", "-std=c++17", f"-I{COMPAT}", str(src), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return str(exe)


def _want(n=1000):
    i = np.arange(n)
    s16 = np.stack([(i * 37 - 18000).astype(np.int16), (-i * 29 + 12345).astype(np.int16)], 1).reshape(-1)
    s64 = (i * 0.25 - 3.0) + 1j / (i + 1)
    return s16, s64, i * 1e-3 - 0.5


def test_fifo_writers_match_python_code_readers(prog, tmp_path):
    row, frame = str(tmp_path / "row_input"), str(tmp_path / "fifo_frame")
    os.mkfifo(row)
    os.mkfifo(frame)
    fd_row = os.open(row, os.O_RDONLY | os.O_NONBLOCK)
    fd_frame = os.open(frame, os.O_RDONLY | os.O_NONBLOCK)
    p = subprocess.Popen([prog, "pipes", row, frame])
    bufs = {row: [], frame: []}
    open_fds = {fd_row: row, fd_frame: frame}
    seen_writer = set()
    while open_fds:
        r, _, _ = select.select(list(open_fds), [], [], 10)
        assert r, "FIFO reader timed out"
        for fd in r:
            b = os.read(fd, 1 << 16)
            if b:
                bufs[open_fds[fd]].append(b)
                seen_writer.add(fd)
            elif fd in seen_writer or p.poll() is not None:
                os.close(fd)
                del open_fds[fd]
    assert p.wait(timeout=30) == 0
    s16, s64, _ = _want()
    data = np.frombuffer(b"".join(bufs[row]), dtype=np.int16)  # real_time_graph.py
    assert np.array_equal(data, s16)
    cd = data[::2] + 1j * data[1::2]
    assert cd.size == 1000
    fr = np.frombuffer(b"".join(bufs[frame]), dtype=np.float64)  # frame_pipe.py
    assert np.array_equal(fr[::2] + 1j * fr[1::2], s64)


def test_send_data_without_reader_returns(prog, tmp_path):
    row = str(tmp_path / "row_input")
    os.mkfifo(row)
    assert subprocess.run([prog, "nopipe", row], timeout=30).returncode == 0


def test_file_writers_flat_layout(prog, tmp_path):
    assert subprocess.run([prog, "files", str(tmp_path)], timeout=30).returncode == 0
    s16, s64, d = _want()
    c = np.fromfile(tmp_path / "c64.bin", dtype=np.float64)  # ofdm.py:9-11
    assert np.array_equal(c[::2] + 1j * c[1::2], s64)
    assert np.array_equal(np.fromfile(tmp_path / "c16.bin", dtype=np.int16), s16)  # source.bin / tx.bin
    assert np.array_equal(np.fromfile(tmp_path / "d.bin", dtype=np.float64), d)  # t2_sin_corr.bin
