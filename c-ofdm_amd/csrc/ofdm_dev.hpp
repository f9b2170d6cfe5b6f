// ofdm_dev.hpp — device helpers shared by the rx kernels (ofdm_kernels.hip)
// and the fused stream decode (ofdm_sync.hip): the demod decision, output
// byte packing and non-temporal 16-B accesses.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <mutex>
#include <set>
#include <utility>

#include "ofdm_fft.hpp"

namespace ofdm {

// Host side: opt a kernel into `bytes` of dynamic LDS once per (kernel,
// device). The launch helpers run on any host thread (one context per thread,
// or two contexts on two streams) and on any device of the process.
inline void lds_opt_in(const void* fn, int bytes)
{
    static std::mutex mu;
    static std::set<std::pair<const void*, int>> done;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    std::lock_guard<std::mutex> g(mu);
    if (done.insert({fn, dev}).second)
        (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// Modulation::demod decision for one point (modulation.cpp:62-84): BPSK
// re+im > 0; QAM clamp to [-1,1] then uint8((v+1)*str_size_1 + 0.5) per axis,
// idx = re | im*str_size. Separate roundings (no FMA) as on x86-64.
// The clamp is v_max/v_min: equal to the reference's compare chain for every
// non-NaN value; a NaN (degenerate all-zero pilots) decides 0 either way
// (chain: cvt(NaN) = 0; min/max: clamps to -1, then uint8(0.5) = 0).
// decide() as a select (no branch on k): the same value for every k.
__device__ __forceinline__ int decide_select(double2 z, int k, double s1, int m)
{
    const double re = __builtin_fmin(__builtin_fmax(z.x, -1.0), 1.0);
    const double im = __builtin_fmin(__builtin_fmax(z.y, -1.0), 1.0);
    const int ire = (uint8_t)(int)add_rn(mul_rn(add_rn(re, 1.0), s1), 0.5);
    const int iim = (uint8_t)(int)add_rn(mul_rn(add_rn(im, 1.0), s1), 0.5);
    const int qam = (ire | (iim * m)) & 0xff;
    const int bpsk = (z.x + z.y) > 0.0;
    return k == 1 ? bpsk : qam;
}

// Four output bytes (one little-endian word) from 32/K consecutive K-bit
// decisions held one per byte in LDS (MSB-first within each byte, as
// bit_stream_converter(8, K, ...), modulation.cpp:90-125).
template <int K>
__device__ __forceinline__ uint32_t pack_word(const uint8_t* __restrict__ dec)
{
    constexpr int PER = 8 / K;  // decisions per output byte
    constexpr int NW = 8 / K;   // 32-bit LDS words holding the 32/K decisions (dec is 32/K-byte aligned)
    uint32_t d[NW];
    const uint32_t* d32 = reinterpret_cast<const uint32_t*>(dec);
#pragma unroll
    for (int i = 0; i < NW; ++i) d[i] = d32[i];
    uint32_t word = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        uint32_t byte = 0;
#pragma unroll
        for (int r = 0; r < PER; ++r) {
            const int idx = b * PER + r;
            byte = (byte << K) | ((d[idx >> 2] >> (8 * (idx & 3))) & 0xffu);
        }
        word |= byte << (8 * b);
    }
    return word;
}

// Streams touched once (tx output, rx input, constellation output): non-temporal
// 16-B accesses, so a launch neither evicts the caches for nothing nor leaves
// gigabytes of dirty lines for the next launch to write back.
typedef double nt_double2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void store_nt(double2* p, double2 v)
{
    nt_double2 w = {v.x, v.y};
    __builtin_nontemporal_store(w, reinterpret_cast<nt_double2*>(p));
}

__device__ __forceinline__ double2 load_nt(const double2* p)
{
    const nt_double2 w = __builtin_nontemporal_load(reinterpret_cast<const nt_double2*>(p));
    return make_double2(w.x, w.y);
}

}  // namespace ofdm
