// ofdm_fft32.hpp — FP32 Stockham FFT within one wave, for the stream
// walker's T2 detector screen (ofdm_sync.hip stream_walk_kernel).
//
// The T2 decision (Frame.hpp:150-197: energy share of the detector bins >
// level) is screened in FP32 and certified: a block whose FP32 energy ratio
// clears the level by more than its error bound is decided as the FP64
// reference decides it; any other block is re-evaluated in FP64. Same shape
// and indexing as ofdm_fft.hpp's fft_regs_wave (radix-8 Stockham, thread t
// holds x[t + T*i], T = N/8 <= 64, LDS image XOR-swizzled), on float2: half
// the registers, LDS bytes and VALU cycles per block.
#pragma once
#include "ofdm_fft.hpp"

namespace ofdm {

__device__ __forceinline__ float2 fadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 fsub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 fmulc(float2 a, float2 b)
{
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

template <int SIGN>
__device__ __forceinline__ float2 fmul_j(float2 a)
{
    return SIGN > 0 ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x);
}

template <int SIGN>
__device__ __forceinline__ void fdft2(float2& a, float2& b)
{
    const float2 t = a;
    a = fadd(t, b);
    b = fsub(t, b);
}

template <int SIGN>
__device__ __forceinline__ void fdft4(float2& a0, float2& a1, float2& a2, float2& a3)
{
    const float2 t0 = fadd(a0, a2), t1 = fsub(a0, a2);
    const float2 t2 = fadd(a1, a3), t3 = fmul_j<SIGN>(fsub(a1, a3));
    a0 = fadd(t0, t2);
    a1 = fadd(t1, t3);
    a2 = fsub(t0, t2);
    a3 = fsub(t1, t3);
}

template <int SIGN>
__device__ __forceinline__ void fdft8(float2& x0, float2& x1, float2& x2, float2& x3, float2& x4, float2& x5,
                                      float2& x6, float2& x7)
{
    constexpr float C = 0.70710678118654752440f;
    fdft4<SIGN>(x0, x2, x4, x6);
    fdft4<SIGN>(x1, x3, x5, x7);
    const float2 o1 = make_float2((x3.x - SIGN * x3.y) * C, (x3.y + SIGN * x3.x) * C);
    const float2 o2 = fmul_j<SIGN>(x5);
    const float2 o3 = make_float2(-(x7.x + SIGN * x7.y) * C, (SIGN * x7.x - x7.y) * C);
    const float2 e0 = x0, e1 = x2, e2 = x4, e3 = x6, o0 = x1;
    x0 = fadd(e0, o0);
    x4 = fsub(e0, o0);
    x1 = fadd(e1, o1);
    x5 = fsub(e1, o1);
    x2 = fadd(e2, o2);
    x6 = fsub(e2, o2);
    x3 = fadd(e3, o3);
    x7 = fsub(e3, o3);
}

template <int LOGN, int R, int NS, int SIGN>
__device__ __forceinline__ void stockham_pass32(float2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                float2* __restrict__ lds, bool write)
{
    constexpr int N = 1 << LOGN, T = N / 8, B = 8 / R;
#pragma unroll
    for (int u = 0; u < B; ++u) {
        const int b = t + T * u;
        const int k = b & (NS - 1);
        if constexpr (NS > 1) {
            // the base twiddle from the FP64 table (TwLds), rounded once
            const double2 w64 = tw_get<LOGN, N / R>(lds_tw, k * (N / (NS * R)));
            float2 w1 = make_float2((float)w64.x, (float)w64.y);
            if (SIGN > 0) w1.y = -w1.y;
            float2 w = w1;
            v[u + B] = fmulc(v[u + B], w1);
#pragma unroll
            for (int r = 2; r < R; ++r) {
                w = fmulc(w, w1);
                v[u + r * B] = fmulc(v[u + r * B], w);
            }
        }
        if constexpr (R == 8)
            fdft8<SIGN>(v[u], v[u + B], v[u + 2 * B], v[u + 3 * B], v[u + 4 * B], v[u + 5 * B], v[u + 6 * B],
                        v[u + 7 * B]);
        else if constexpr (R == 4)
            fdft4<SIGN>(v[u], v[u + B], v[u + 2 * B], v[u + 3 * B]);
        else
            fdft2<SIGN>(v[u], v[u + B]);
        if (!write) continue;
        const int idxD = (b - k) * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) lds[lds_swz(idxD + r * NS)] = v[u + r * B];
    }
}

template <int LOGN, int PASS, int SIGN>
__device__ __forceinline__ void fft_regs_tail_wave32(float2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                     float2* __restrict__ lds)
{
    using S = FftShape<LOGN>;
    constexpr int T = S::T;
    constexpr int NPASS = S::NPASS8 + (S::REM ? 1 : 0);
    constexpr bool is8 = PASS < S::NPASS8;
    constexpr int R = is8 ? 8 : (1 << S::REM);
    constexpr int NS = 1 << (3 * PASS);
    constexpr bool LAST = PASS == NPASS - 1;
    wave_lds_sync();  // previous pass fully written
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = lds[lds_swz(t + T * i)];
    if constexpr (LAST) {
        stockham_pass32<LOGN, R, NS, SIGN>(v, t, lds_tw, lds, false);
    } else {
        wave_lds_sync();  // every lane has read before the image is overwritten
        stockham_pass32<LOGN, R, NS, SIGN>(v, t, lds_tw, lds, true);
        fft_regs_tail_wave32<LOGN, PASS + 1, SIGN>(v, t, lds_tw, lds);
    }
}

// On entry v[i] = x[t + T*i] (T = N/8 <= 64 threads of one wave per
// transform, lds its N-entry image, lds_tw the FP64 TwLds table); on exit
// v[i] = X[t + T*i].
template <int LOGN, int SIGN>
__device__ __forceinline__ void fft_regs_wave32(float2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                float2* __restrict__ lds)
{
    static_assert(LOGN >= 6 && LOGN <= 9, "N/8 <= one wave");
    stockham_pass32<LOGN, 8, 1, SIGN>(v, t, lds_tw, lds, true);
    fft_regs_tail_wave32<LOGN, 1, SIGN>(v, t, lds_tw, lds);
}

}  // namespace ofdm

namespace ofdm {

// ---------------------------------------------------------------- two blocks at once
// Two FP32 transforms in lockstep, element = float4 {A.re, A.im, B.re, B.im}:
// the LDS image holds 16-B elements, so ofdm_fft.hpp's swizzle (built for
// 16-B accesses) keeps every pass conflict-free, and one ds_read/ds_write_b128
// moves a value of both blocks (a float2 image with that swizzle conflicted
// 4-way on the stride-8 writes).
__device__ __forceinline__ float4 q_add(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 q_sub(float4 a, float4 b) { return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
__device__ __forceinline__ float4 q_mulw(float4 a, float2 w)  // both halves times w
{
    return make_float4(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x, a.z * w.x - a.w * w.y, a.z * w.y + a.w * w.x);
}
template <int SIGN>
__device__ __forceinline__ float4 q_mul_j(float4 a)
{
    return SIGN > 0 ? make_float4(-a.y, a.x, -a.w, a.z) : make_float4(a.y, -a.x, a.w, -a.z);
}
__device__ __forceinline__ float4 q_scale(float4 a, float c) { return make_float4(a.x * c, a.y * c, a.z * c, a.w * c); }

template <int SIGN>
__device__ __forceinline__ void qdft2(float4& a, float4& b)
{
    const float4 t = a;
    a = q_add(t, b);
    b = q_sub(t, b);
}

template <int SIGN>
__device__ __forceinline__ void qdft4(float4& a0, float4& a1, float4& a2, float4& a3)
{
    const float4 t0 = q_add(a0, a2), t1 = q_sub(a0, a2);
    const float4 t2 = q_add(a1, a3), t3 = q_mul_j<SIGN>(q_sub(a1, a3));
    a0 = q_add(t0, t2);
    a1 = q_add(t1, t3);
    a2 = q_sub(t0, t2);
    a3 = q_sub(t1, t3);
}

template <int SIGN>
__device__ __forceinline__ void qdft8(float4& x0, float4& x1, float4& x2, float4& x3, float4& x4, float4& x5,
                                      float4& x6, float4& x7)
{
    constexpr float C = 0.70710678118654752440f;
    qdft4<SIGN>(x0, x2, x4, x6);
    qdft4<SIGN>(x1, x3, x5, x7);
    // O1 *= W8, O2 *= W8^2 = SIGN*i, O3 *= W8^3
    const float4 o1 = q_scale(q_add(x3, q_mul_j<SIGN>(x3)), C);
    const float4 o2 = q_mul_j<SIGN>(x5);
    const float4 o3 = q_scale(q_sub(q_mul_j<SIGN>(x7), x7), C);
    const float4 e0 = x0, e1 = x2, e2 = x4, e3 = x6, o0 = x1;
    x0 = q_add(e0, o0);
    x4 = q_sub(e0, o0);
    x1 = q_add(e1, o1);
    x5 = q_sub(e1, o1);
    x2 = q_add(e2, o2);
    x6 = q_sub(e2, o2);
    x3 = q_add(e3, o3);
    x7 = q_sub(e3, o3);
}

template <int LOGN, int R, int NS, int SIGN>
__device__ __forceinline__ void stockham_pass32x2(float4 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                  float4* __restrict__ lds, bool write)
{
    constexpr int N = 1 << LOGN, T = N / 8, B = 8 / R;
#pragma unroll
    for (int u = 0; u < B; ++u) {
        const int b = t + T * u;
        const int k = b & (NS - 1);
        if constexpr (NS > 1) {
            const double2 w64 = tw_get<LOGN, N / R>(lds_tw, k * (N / (NS * R)));
            float2 w1 = make_float2((float)w64.x, (float)w64.y);
            if (SIGN > 0) w1.y = -w1.y;
            float2 w = w1;
            v[u + B] = q_mulw(v[u + B], w1);
#pragma unroll
            for (int r = 2; r < R; ++r) {
                w = fmulc(w, w1);
                v[u + r * B] = q_mulw(v[u + r * B], w);
            }
        }
        if constexpr (R == 8)
            qdft8<SIGN>(v[u], v[u + B], v[u + 2 * B], v[u + 3 * B], v[u + 4 * B], v[u + 5 * B], v[u + 6 * B],
                        v[u + 7 * B]);
        else if constexpr (R == 4)
            qdft4<SIGN>(v[u], v[u + B], v[u + 2 * B], v[u + 3 * B]);
        else
            qdft2<SIGN>(v[u], v[u + B]);
        if (!write) continue;
        const int idxD = (b - k) * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) lds[lds_swz(idxD + r * NS)] = v[u + r * B];
    }
}

template <int LOGN, int PASS, int SIGN>
__device__ __forceinline__ void fft_regs_tail_wave32x2(float4 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                       float4* __restrict__ lds)
{
    using S = FftShape<LOGN>;
    constexpr int T = S::T;
    constexpr int NPASS = S::NPASS8 + (S::REM ? 1 : 0);
    constexpr bool is8 = PASS < S::NPASS8;
    constexpr int R = is8 ? 8 : (1 << S::REM);
    constexpr int NS = 1 << (3 * PASS);
    constexpr bool LAST = PASS == NPASS - 1;
    wave_lds_sync();  // previous pass fully written
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = lds[lds_swz(t + T * i)];
    if constexpr (LAST) {
        stockham_pass32x2<LOGN, R, NS, SIGN>(v, t, lds_tw, lds, false);
    } else {
        wave_lds_sync();  // every lane has read before the image is overwritten
        stockham_pass32x2<LOGN, R, NS, SIGN>(v, t, lds_tw, lds, true);
        fft_regs_tail_wave32x2<LOGN, PASS + 1, SIGN>(v, t, lds_tw, lds);
    }
}

// Two N-point FP32 transforms (v[i] = {a[t + T*i], b[t + T*i]}) by T <= 64
// threads of one wave, image lds (N float4); on exit v[i] = {A, B}[t + T*i].
template <int LOGN, int SIGN>
__device__ __forceinline__ void fft_regs_wave32x2(float4 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                  float4* __restrict__ lds)
{
    static_assert(LOGN >= 6 && LOGN <= 9, "N/8 <= one wave");
    stockham_pass32x2<LOGN, 8, 1, SIGN>(v, t, lds_tw, lds, true);
    fft_regs_tail_wave32x2<LOGN, 1, SIGN>(v, t, lds_tw, lds);
}

}  // namespace ofdm
