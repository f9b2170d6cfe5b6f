// io/io.hpp — drop-in for the reference's io/io.hpp:15-144: the data/*.bin
// writers/readers (interleaved re/im of the element type), the int16 FIFO
// and f64 pipe writers read by python_code/, and bench_us. Host I/O only.
#pragma once
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <unistd.h>

#include <chrono>
#include <complex>
#include <cstdint>
#include <fstream>
#include <iostream>
#include <iterator>
#include <stdexcept>
#include <string>
#include <vector>

template <typename Iter>
void write_complex_to_file(const std::string& filename, Iter begin, Iter end)
{
    using T = typename std::iterator_traits<Iter>::value_type::value_type;
    std::ofstream out(filename, std::ios::binary);
    if (!out) throw std::runtime_error("Cannot open file");
    for (Iter it = begin; it != end; ++it) {
        const T v[2] = {it->real(), it->imag()};
        out.write(reinterpret_cast<const char*>(v), sizeof v);
    }
}

template <typename T>
void write_complex_to_file(const std::string& filename, const std::vector<std::complex<T>>& data)
{
    write_complex_to_file(filename, data.begin(), data.end());
}

template <typename Iter>
void read_complex_from_file(const std::string& filename, Iter out)
{
    using T = typename std::iterator_traits<Iter>::value_type::value_type;
    std::ifstream in(filename, std::ios::binary);
    if (!in) throw std::runtime_error("Cannot open file");
    T v[2];
    while (in.read(reinterpret_cast<char*>(&v[0]), sizeof(T))) {
        if (!in.read(reinterpret_cast<char*>(&v[1]), sizeof(T)))
            throw std::runtime_error("File corrupted: incomplete complex number");
        *out++ = std::complex<T>(v[0], v[1]);
    }
}

inline void write_double_to_file(const std::string& filename, const std::vector<double>& data)
{
    std::ofstream out(filename, std::ios::binary);
    if (!out) throw std::runtime_error("Cannot open file");
    out.write(reinterpret_cast<const char*>(data.data()), data.size() * sizeof(double));
}

// int16 IQ into a FIFO (real_time_graph.py), non-blocking; samples dropped when full.
inline void send_data(const char* pipe, const std::vector<std::complex<int16_t>>& buf)
{
    const int fd = open(pipe, O_WRONLY | O_NONBLOCK);
    if (fd < 0) return;
    for (const auto& s : buf) {
        const int16_t v[2] = {s.real(), s.imag()};
        if (write(fd, v, sizeof v) < 0 && errno != EAGAIN && errno != EWOULDBLOCK) {
            perror("write pipe");
            break;
        }
    }
    close(fd);
}

// complex f64 samples into a pipe (frame_pipe.py)
template <typename Iter>
void write_complex_to_pipe(Iter begin, Iter end, const char* pipe_name)
{
    std::ofstream out(pipe_name, std::ios::binary);
    for (Iter it = begin; it != end; ++it) {
        const double v[2] = {(double)it->real(), (double)it->imag()};
        out.write(reinterpret_cast<const char*>(v), sizeof v);
    }
}

template <typename F>
long long bench_us(F&& f, int warmup = 5, int iters = 10000)
{
    for (int i = 0; i < warmup; ++i) f();
    long long total = 0;
    for (int i = 0; i < iters; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        f();
        const auto t1 = std::chrono::steady_clock::now();
        total += std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0).count();
    }
    return total / iters;
}

inline void print_vector(std::vector<uint8_t>& v)
{
    for (auto& c : v) std::cout << c;
    std::cout << "\n\n";
}
