// oracle/ref_wrap.cpp — TEST INFRASTRUCTURE ONLY.
//
// extern "C" shim over the reference's OWN sources, compiled unmodified from
// /root/reference by oracle/Makefile into oracle/_ref/libref.so (never copied
// into this repo, never shipped). Used only by tests/ to pin the C
// restatement (oracle/ofdm_oracle.c) and the product's config parser:
//   OFDM/modulation.cpp  (Modulation, psk/qam, bit_stream_converter)
//   config/parser.cpp    (parse_config)
// Frame.cpp is NOT built: it needs <fftw3.h>/libfftw3, absent from this image.
#include <cstring>
#include <random>
#include <stdexcept>
#include "modulation.hpp"
#include "parser.hpp"

extern "C" {

int ref_constellation(int k, double* out) {
    Modulation m(static_cast<mod_type>(k));
    std::memcpy(out, m.constell.data(), m.constell.size() * sizeof(complex_double));
    return (int)m.constell.size();
}

size_t ref_mod(int k, const uint8_t* in, size_t n, double* out) {
    Modulation m(static_cast<mod_type>(k));
    std::vector<uint8_t> v(in, in + n);
    complex_vector o = m.mod(v);
    std::memcpy(out, o.data(), o.size() * sizeof(complex_double));
    return o.size();
}

// demod clamps its argument in place (modulation.cpp:70-75): copy it back.
size_t ref_demod(int k, double* pts, size_t n, uint8_t* out) {
    Modulation m(static_cast<mod_type>(k));
    complex_vector v(n);
    std::memcpy(v.data(), pts, n * sizeof(complex_double));
    std::vector<uint8_t> o = m.demod(v);
    std::memcpy(pts, v.data(), n * sizeof(complex_double));
    std::memcpy(out, o.data(), o.size());
    return o.size();
}

size_t ref_bit_convert(int out_bits, int in_bits, const uint8_t* in, size_t n, uint8_t* out) {
    Modulation m(qam16);
    std::vector<uint8_t> v(in, in + n);
    std::vector<uint8_t> o = m.bit_stream_converter(out_bits, in_bits, v);
    std::memcpy(out, o.data(), o.size());
    return o.size();
}

// 0 ok, -4 cannot open (runtime_error), -6 std::stol threw.
int ref_parse_config(const char* path, const char* key, long* value) {
    try {
        ConfigMap c = parse_config(path);
        *value = c[key];
        return 0;
    } catch (const std::invalid_argument&) {
        return -6;
    } catch (const std::out_of_range&) {
        return -6;
    } catch (const std::runtime_error&) {
        return -4;
    }
}

// The host libstdc++'s std::mt19937 + uniform_int_distribution<int>(0,255),
// i.e. what PREAMBLE_FORM's ctor calls (Frame.cpp:269-272).
void ref_std_preamble_bytes(long seed, long n, uint8_t* out) {
    std::mt19937 rng(seed);
    std::uniform_int_distribution<int> dist(0, 255);
    for (long i = 0; i < n; i++) out[i] = (uint8_t)dist(rng);
}
}
