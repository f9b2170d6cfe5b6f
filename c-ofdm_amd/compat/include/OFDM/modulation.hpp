// OFDM/modulation.hpp — drop-in for the reference's OFDM/modulation.hpp
// (mod_type, the complex/bit vector aliases, psk/qam, class Modulation).
// mod / demod / bit_stream_converter run as HIP kernels through the C-ABI
// (include/ofdm_mi355x.h: ofdm_map, ofdm_demap, ofdm_bit_convert).
#pragma once
#include <math.h>
#include <stdlib.h>

#include <algorithm>
#include <complex>
#include <cstdint>
#include <memory>
#include <utility>
#include <vector>

enum mod_type { bpsk = 1, qam4 = 2, qam16 = 4, qam64 = 6, qam256 = 8 };

using complex_double = std::complex<double>;
using complex_vector = std::vector<std::complex<double>>;
using complex16_vector = std::vector<std::complex<int16_t>>;
using bit_vector = std::vector<uint8_t>;

complex_double psk(uint8_t input, double angle, int deg);
complex_double qam(uint8_t input, int deg);

namespace ofdm_compat {
struct Context;
}

class Modulation {
public:
    mod_type modulation;
    std::vector<complex_double> constell;
    size_t mod_index;

    Modulation(mod_type mod);

    complex_vector mod(std::vector<uint8_t>& bin_input);
    std::vector<uint8_t> demod(complex_vector& input);  // clamps `input` in place, as the reference
    std::vector<uint8_t> bit_stream_converter(size_t output_block_size, size_t input_block_size,
                                              std::vector<uint8_t>& input);

private:
    std::shared_ptr<ofdm_compat::Context> ctx_;
};
