// ofdm_syncdev.hpp — device helpers of the rx sync front end shared by
// ofdm_sync.hip and ofdm_stream_wide.hip: g++-rounded complex products and
// sums, workgroup sums, chan_char_lq's parallel unwrap and the stream sample
// load (f64 or complex<int16>). Every body carries its own
// `fp contract(off)`: the sync arithmetic mirrors the reference's x86-64
// build (no FMA) wherever the header is included.
#pragma once
#include <hip/hip_runtime.h>

#include "ofdm_fft.hpp"

namespace ofdm {
namespace {

__device__ __forceinline__ double2 cconj_mul(double2 a, double2 b)  // conj(a) * b, as g++ (no FMA)
{
    return cmul_exact(make_double2(a.x, -a.y), b);
}

__device__ __forceinline__ double2 cadd_rn(double2 a, double2 b)
{
    return make_double2(add_rn(a.x, b.x), add_rn(a.y, b.y));
}

// Block-wide complex / double sums (NT threads, multiple of 64 or < 64).
template <int NT>
__device__ __forceinline__ double2 block_sum2(double2 v, double2* red)
{
#pragma clang fp contract(off)
    constexpr int W0 = NT >= 64 ? 32 : NT / 2;
#pragma unroll
    for (int o = W0; o > 0; o >>= 1) {
        v.x += __shfl_xor(v.x, o);
        v.y += __shfl_xor(v.y, o);
    }
    constexpr int NW = (NT + 63) / 64;
    if constexpr (NW == 1) {
        return v;
    } else {
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        __syncthreads();
        if (lane == 0) red[w] = v;
        __syncthreads();
        double2 s = make_double2(0.0, 0.0);
#pragma unroll
        for (int i = 0; i < NW; ++i) s = cadd(s, red[i]);
        return s;
    }
}

// ---------------------------------------------------------------- unwrap
// chan_char_lq's one-pass unwrap (Frame.hpp:407-414: a phase moves by -/+2 pi
// when it differs from the already-adjusted previous one by more than pi) as
// a parallel scan. Entry i's rule maps the previous entry's adjustment
// k in {-1, 0, +1} (state k+1) to its own, so each entry is a map on 3
// states, 2 bits per state; maps compose associatively. Per state the same
// FP64 operations as the serial loop run, so the result is bit-identical.
constexpr unsigned UMAP_ID = 0u | (1u << 2) | (2u << 4);

__device__ __forceinline__ unsigned umap_then(unsigned f, unsigned g)  // f, then g
{
    unsigned h = 0;
#pragma unroll
    for (int s = 0; s < 3; ++s) h |= ((g >> (2 * ((f >> (2 * s)) & 3))) & 3) << (2 * s);
    return h;
}

// ph[0..n) raw phases in LDS (visible to every thread); on return they are
// unwrapped and visible. All NT threads call it; scr: NT/64 words of LDS.
// n - 1 <= 4 * NT (chan_char_lq: n = D/2 <= N/2 = 4 * NT).
template <int NT, bool WAVE = false>
__device__ void unwrap_scan(double* ph, int n, unsigned* scr)
{
#pragma clang fp contract(off)
    static_assert(!WAVE || NT == 64, "a wave-local scan is one wave");
    const int t = threadIdx.x, lane = t & 63;
    const int R = (n - 1 + NT - 1) / NT;  // entries 1..n-1, R consecutive per thread
    const int i0 = 1 + t * R;
    unsigned m[4];
    double raw[4];
    unsigned loc = UMAP_ID;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = i0 + r;
        m[r] = UMAP_ID;
        raw[r] = 0.0;
        if (r < R && i < n) {
            const double x = ph[i], prev = ph[i - 1];
            raw[r] = x;
            unsigned mr = 0;
#pragma unroll
            for (int st = 0; st < 3; ++st) {
                const double pa = st == 1 ? prev : (st == 0 ? prev - 2 * M_PI : prev + 2 * M_PI);
                const double d = x - pa;
                mr |= (d > M_PI ? 0u : (d < -M_PI ? 2u : 1u)) << (2 * st);
            }
            m[r] = mr;
            loc = umap_then(loc, mr);
        }
    }
    // exclusive scan of the per-thread maps (wave shuffles, then wave totals)
    unsigned inc = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned y = __shfl_up(inc, o);
        if (lane >= o) inc = umap_then(y, inc);
    }
    unsigned ex = __shfl_up(inc, 1);
    if (lane == 0) ex = UMAP_ID;
    if constexpr (NT > 64) {
        if (lane == 63) scr[t >> 6] = inc;
        __syncthreads();
        unsigned pre = UMAP_ID;
        for (int w = 0; w < (t >> 6); ++w) pre = umap_then(pre, scr[w]);
        ex = umap_then(pre, ex);
    }
    if constexpr (WAVE)
        wave_lds_sync();
    else
        __syncthreads();  // every raw phase has been read
    int st = (ex >> 2) & 3;  // entry 0 is never adjusted (state 1)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = i0 + r;
        if (r < R && i < n) {
            st = (m[r] >> (2 * st)) & 3;
            ph[i] = st == 1 ? raw[r] : (st == 0 ? raw[r] - 2 * M_PI : raw[r] + 2 * M_PI);
        }
    }
    if constexpr (WAVE)
        wave_lds_sync();
    else
        __syncthreads();
}

// One stream sample as complex<double> (f64 stream, or complex<int16>
// converted exactly: FRAME_FORM::form_int16_to_double, Frame.hpp:472-481).
__device__ __forceinline__ double2 src_sample(const double2* iq, const short2* iq16, long j)
{
    if (iq16) {
        const short2 w = iq16[j];
        return make_double2((double)w.x, (double)w.y);
    }
    return iq[j];
}

// src_sample with the stream's format fixed at compile time (kernels
// instantiated per format): no per-sample branch between the loads, so an
// unrolled loop issues its loads back to back.
template <bool I16>
__device__ __forceinline__ double2 src_sample_t(const double2* iq, const short2* iq16, long j)
{
    if constexpr (I16) {
        const short2 w = iq16[j];
        return make_double2((double)w.x, (double)w.y);
    } else {
        return iq[j];
    }
}

}  // namespace
}  // namespace ofdm
