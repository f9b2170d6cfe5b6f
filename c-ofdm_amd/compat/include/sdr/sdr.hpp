// sdr/sdr.hpp — stand-in for the reference's libiio ADALM-Pluto driver
// (sdr/sdr.hpp:25-276; radio hardware is out of scope), so
// main.cpp / tx.cpp / rx.cpp link and run on a GPU box without radios.
// Same class name, constructor and member surface (rx_buf_size, send, recv);
// the "air" is file- or process-backed:
//   send(buf)  appends the first sdr_buffer_capacity samples to an in-process
//              loopback air, and to $OFDM_SDR_TX_FILE if set (int16 IQ
//              interleaved = data/tx.bin, read by python_code/channel.py).
//   recv(buf)  fills rx_buf_size = capacity * config["rx_buf_size"] samples
//              from $OFDM_SDR_RX_FILE if set (int16 IQ, or f64 IQ when
//              $OFDM_SDR_RX_FORMAT=f64, e.g. the reference's data/data.bin),
//              consumed sequentially, zeros after the end; otherwise from the
//              loopback air preceded by $OFDM_SDR_GAP (default 1000) zero
//              samples. The real driver scales tx by 16 for the 12-bit DAC
//              (sdr.hpp:217-218); the loopback does not (pilot normalisation
//              makes rx scale-free).
//   Pacing: like iio_buffer_refill, recv takes rx_buf_size / fs_hz seconds
//   (fill first, then wait; $OFDM_SDR_REALTIME=0 disables). rx.cpp relies on
//   that: its reader thread is never stopped and main frees the two buffers
//   it writes into (rx.cpp:58-66,246-247), which only works while a refill
//   outlasts main's shutdown.
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <complex>
#include <deque>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "config/parser.hpp"

class SDR {
private:
    ConfigMap config;
    int16_t mult;
    size_t sdr_buffer_capacity;
    FILE* rx_file = nullptr;
    bool rx_f64 = false;

    struct Air {
        std::mutex mu;
        std::deque<std::complex<int16_t>> q;
        bool primed = false;
    };
    static Air& air()
    {
        static Air a;
        return a;
    }

    // fill n samples (zeros once the source is exhausted), then pace like the radio
    void fill(std::complex<int16_t>* out, size_t n)
    {
        size_t got = 0;
        if (rx_file) {
            if (rx_f64) {
                std::vector<double> v(2 * n);
                got = std::fread(v.data(), 2 * sizeof(double), n, rx_file);
                for (size_t i = 0; i < got; ++i) out[i] = std::complex<int16_t>((int16_t)v[2 * i], (int16_t)v[2 * i + 1]);
            } else {
                got = std::fread(out, sizeof(std::complex<int16_t>), n, rx_file);
            }
        } else {
            Air& a = air();
            std::lock_guard<std::mutex> lock(a.mu);
            got = std::min(n, a.q.size());
            std::copy(a.q.begin(), a.q.begin() + got, out);
            a.q.erase(a.q.begin(), a.q.begin() + got);
        }
        for (size_t i = got; i < n; ++i) out[i] = std::complex<int16_t>(0, 0);
        const char* rt = std::getenv("OFDM_SDR_REALTIME");
        const double fs = (double)config["fs_hz"];
        if (fs > 0 && !(rt && std::string(rt) == "0"))
            std::this_thread::sleep_for(std::chrono::duration<double>((double)n / fs));
    }

public:
    size_t rx_buf_size;

    SDR(int device_num, size_t sdr_buffer_capacity, const std::string& CONFIGNAME)
        : config(parse_config(CONFIGNAME)),
          mult((int16_t)config["mult"]),
          sdr_buffer_capacity(sdr_buffer_capacity),
          rx_buf_size(sdr_buffer_capacity * config["rx_buf_size"])
    {
        (void)device_num;
        if (const char* f = std::getenv("OFDM_SDR_RX_FILE")) {
            rx_file = std::fopen(f, "rb");
            const char* fmt = std::getenv("OFDM_SDR_RX_FORMAT");
            rx_f64 = fmt && std::string(fmt) == "f64";
        }
    }

    ~SDR()
    {
        if (rx_file) std::fclose(rx_file);
    }

    void send(std::vector<std::complex<int16_t>>& buf)
    {
        const size_t n = std::min(sdr_buffer_capacity, buf.size());
        Air& a = air();
        {
            std::lock_guard<std::mutex> lock(a.mu);
            if (!a.primed) {
                const char* g = std::getenv("OFDM_SDR_GAP");
                a.q.insert(a.q.end(), g ? std::strtoul(g, nullptr, 10) : 1000, std::complex<int16_t>(0, 0));
                a.primed = true;
            }
            a.q.insert(a.q.end(), buf.begin(), buf.begin() + n);
        }
        if (const char* f = std::getenv("OFDM_SDR_TX_FILE")) {
            if (FILE* fp = std::fopen(f, "ab")) {
                std::fwrite(buf.data(), sizeof(std::complex<int16_t>), n, fp);
                std::fclose(fp);
            }
        }
    }

    void recv(std::vector<std::complex<int16_t>>& buf) { fill(buf.data(), std::min(rx_buf_size, buf.size())); }

    void recv(std::complex<int16_t>* buf) { fill(buf, rx_buf_size); }
};
