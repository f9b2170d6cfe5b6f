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
#include <type_traits>

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

// ---------------------------------------------------------------- two blocks at once, packed
// Two FP32 transforms in lockstep, structure-of-arrays: a point is the pair
// re = {A.re, B.re}, im = {A.im, B.im} (pf2 = two packed floats), so every
// add, subtract and twiddle product of the two blocks is one gfx950 packed
// instruction (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32, the twiddle a
// broadcast operand): half the VALU issue of two unpacked transforms. The LDS
// image holds 16-B elements {A.re, B.re, A.im, B.im}, so ofdm_fft.hpp's
// swizzle (built for 16-B accesses) keeps every pass conflict-free and one
// ds_read/ds_write_b128 moves a point of both blocks.
typedef float pf2 __attribute__((ext_vector_type(2)));

struct PCx {
    pf2 re, im;
};

__device__ __forceinline__ PCx p_add(PCx a, PCx b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ PCx p_sub(PCx a, PCx b) { return {a.re - b.re, a.im - b.im}; }
// both blocks times the complex scalar w
__device__ __forceinline__ PCx p_mulw(PCx a, float2 w)
{
    const pf2 wr = {w.x, w.x}, wi = {w.y, w.y};
    return {a.re * wr - a.im * wi, a.re * wi + a.im * wr};
}
template <int SIGN>
__device__ __forceinline__ PCx p_mul_j(PCx a)  // a * (SIGN i)
{
    return SIGN > 0 ? PCx{-a.im, a.re} : PCx{a.im, -a.re};
}

template <int SIGN>
__device__ __forceinline__ void pdft2(PCx& a, PCx& b)
{
    const PCx t = a;
    a = p_add(t, b);
    b = p_sub(t, b);
}

template <int SIGN>
__device__ __forceinline__ void pdft4(PCx& a0, PCx& a1, PCx& a2, PCx& a3)
{
    const PCx t0 = p_add(a0, a2), t1 = p_sub(a0, a2);
    const PCx t2 = p_add(a1, a3), t3 = p_mul_j<SIGN>(p_sub(a1, a3));
    a0 = p_add(t0, t2);
    a1 = p_add(t1, t3);
    a2 = p_sub(t0, t2);
    a3 = p_sub(t1, t3);
}

template <int SIGN>
__device__ __forceinline__ void pdft8(PCx& x0, PCx& x1, PCx& x2, PCx& x3, PCx& x4, PCx& x5, PCx& x6, PCx& x7)
{
    constexpr float C = 0.70710678118654752440f;
    const pf2 c2 = {C, C};
    pdft4<SIGN>(x0, x2, x4, x6);
    pdft4<SIGN>(x1, x3, x5, x7);
    // O1 *= W8 = C (1 + SIGN i), O2 *= SIGN i, O3 *= W8^3 = C (-1 + SIGN i)
    const PCx o1 = SIGN > 0 ? PCx{(x3.re - x3.im) * c2, (x3.im + x3.re) * c2}
                            : PCx{(x3.re + x3.im) * c2, (x3.im - x3.re) * c2};
    const PCx o2 = p_mul_j<SIGN>(x5);
    const PCx o3 = SIGN > 0 ? PCx{-(x7.re + x7.im) * c2, (x7.re - x7.im) * c2}
                            : PCx{(x7.im - x7.re) * c2, -(x7.re + x7.im) * c2};
    const PCx e0 = x0, e1 = x2, e2 = x4, e3 = x6, o0 = x1;
    x0 = p_add(e0, o0);
    x4 = p_sub(e0, o0);
    x1 = p_add(e1, o1);
    x5 = p_sub(e1, o1);
    x2 = p_add(e2, o2);
    x6 = p_sub(e2, o2);
    x3 = p_add(e3, o3);
    x7 = p_sub(e3, o3);
}

// Sum over aligned groups of G lanes (G = 2..64, a power of two), valid in
// every lane of the group: DPP row permutations (xor 1, xor 2, the 8-lane
// half-mirror, the 16-lane mirror; each folds into the add as a DPP
// operand, no LDS) up to 16 lanes, then ds_swizzle / bpermute shuffles.
template <int G>
__device__ __forceinline__ float group_sum(float v)
{
    auto dpp = [](float x, auto ctrl) {
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), decltype(ctrl)::value, 0xf, 0xf, false));
    };
    if constexpr (G >= 2) v += dpp(v, std::integral_constant<int, 0xB1>{});   // quad_perm [1,0,3,2]
    if constexpr (G >= 4) v += dpp(v, std::integral_constant<int, 0x4E>{});   // quad_perm [2,3,0,1]
    if constexpr (G >= 8) v += dpp(v, std::integral_constant<int, 0x141>{});  // row_half_mirror
    if constexpr (G >= 16) v += dpp(v, std::integral_constant<int, 0x140>{}); // row_mirror
    if constexpr (G >= 32) v += __shfl_xor(v, 16);
    if constexpr (G >= 64) v += __shfl_xor(v, 32);
    return v;
}

__device__ __forceinline__ float4 p_pack(PCx a) { return make_float4(a.re.x, a.re.y, a.im.x, a.im.y); }
__device__ __forceinline__ PCx p_unpack(float4 v) { return {pf2{v.x, v.y}, pf2{v.z, v.w}}; }

template <int LOGN, int R, int NS, int SIGN>
__device__ __forceinline__ void stockham_pass32p(PCx (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                 float4* __restrict__ lds, bool write)
{
    constexpr int N = 1 << LOGN, T = N / 8, B = 8 / R;
#pragma unroll
    for (int u = 0; u < B; ++u) {
        const int b = t + T * u;
        const int k = b & (NS - 1);
        if constexpr (NS > 1) {
            // the base twiddle from the FP64 table (TwLds), rounded once;
            // its powers by a running product (scalar: one per butterfly)
            const double2 w64 = tw_get<LOGN, N / R>(lds_tw, k * (N / (NS * R)));
            float2 w1 = make_float2((float)w64.x, (float)w64.y);
            if (SIGN > 0) w1.y = -w1.y;
            float2 w = w1;
            v[u + B] = p_mulw(v[u + B], w1);
#pragma unroll
            for (int r = 2; r < R; ++r) {
                w = fmulc(w, w1);
                v[u + r * B] = p_mulw(v[u + r * B], w);
            }
        }
        if constexpr (R == 8)
            pdft8<SIGN>(v[u], v[u + B], v[u + 2 * B], v[u + 3 * B], v[u + 4 * B], v[u + 5 * B], v[u + 6 * B],
                        v[u + 7 * B]);
        else if constexpr (R == 4)
            pdft4<SIGN>(v[u], v[u + B], v[u + 2 * B], v[u + 3 * B]);
        else
            pdft2<SIGN>(v[u], v[u + B]);
        if (!write) continue;
        const int idxD = (b - k) * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) lds[lds_swz(idxD + r * NS)] = p_pack(v[u + r * B]);
    }
}

template <int LOGN, int PASS, int SIGN>
__device__ __forceinline__ void fft_regs_tail_wave32p(PCx (&v)[8], int t, const double2* __restrict__ lds_tw,
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
    for (int i = 0; i < 8; ++i) v[i] = p_unpack(lds[lds_swz(t + T * i)]);
    if constexpr (LAST) {
        stockham_pass32p<LOGN, R, NS, SIGN>(v, t, lds_tw, lds, false);
    } else {
        wave_lds_sync();  // every lane has read before the image is overwritten
        stockham_pass32p<LOGN, R, NS, SIGN>(v, t, lds_tw, lds, true);
        fft_regs_tail_wave32p<LOGN, PASS + 1, SIGN>(v, t, lds_tw, lds);
    }
}

// Two N-point FP32 transforms (v[i] = {a, b}[t + T*i] as packed re / im
// pairs) by T <= 64 threads of one wave, image lds (N float4); on exit
// v[i] = {A, B}[t + T*i].
template <int LOGN, int SIGN>
__device__ __forceinline__ void fft_regs_wave32p(PCx (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                 float4* __restrict__ lds)
{
    static_assert(LOGN >= 6 && LOGN <= 9, "N/8 <= one wave");
    stockham_pass32p<LOGN, 8, 1, SIGN>(v, t, lds_tw, lds, true);
    fft_regs_tail_wave32p<LOGN, 1, SIGN>(v, t, lds_tw, lds);
}

}  // namespace ofdm

namespace ofdm {

// ---------------------------------------------------------------- one transform, packed
// One FP32 transform with a point packed as {re, im} in a pf2: a complex add
// is one v_pk_add_f32, a product by a twiddle two packed instructions (the
// real part times {w.re, w.re}, then the swapped point times {-w.im, w.im}
// added by v_pk_fma_f32 with swapped operand halves). Used by the stream
// walker's FP32 tier of the FFT preamble search (ofdm_sync.hip
// walk_preamble_fft): the correlation of a 512-sample window by two such
// transforms, certified against its error bound like the FP64 form. The LDS
// image keeps ofdm_fft.hpp's 16-B slots and swizzle (the point in the low 8
// bytes): the walker is VALU-bound, not LDS-bound, and the swizzle stays
// conflict-free.
// Packed FP32 arithmetic with operand-half selection spelled out (VOP3P
// op_sel / op_sel_hi / neg modifiers): the compiler does not fold the swaps
// of shufflevector into the instruction and emitted a v_mov per swapped half
// and a v_xor per negation (~125 extra VALU per 512-point transform pair).
// On a 64-bit pair {lo, hi} of FP32, op_sel picks the source half of the lo
// result, op_sel_hi that of the hi result.
__device__ __forceinline__ pf2 c_mulw(pf2 a, pf2 w)  // a * w (complex)
{
    pf2 t, r;
    // t = {a.re w.re, a.im w.re}
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(t) : "v"(a), "v"(w));
    // r = {-a.im w.im + t.lo, a.re w.im + t.hi}
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[0,1,0]"
        : "=v"(r) : "v"(a), "v"(w), "v"(t));
    return r;
}
// x + SIGN i y
template <int SIGN>
__device__ __forceinline__ pf2 c_add_j(pf2 x, pf2 y)
{
    pf2 r;
    if constexpr (SIGN > 0)  // {x.re - y.im, x.im + y.re}
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(x), "v"(y));
    else  // {x.re + y.im, x.im - y.re}
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(x), "v"(y));
    return r;
}
// x - SIGN i y
template <int SIGN>
__device__ __forceinline__ pf2 c_sub_j(pf2 x, pf2 y)
{
    return c_add_j<-SIGN>(x, y);
}

template <int SIGN>
__device__ __forceinline__ void cdft4(pf2& a0, pf2& a1, pf2& a2, pf2& a3)
{
    const pf2 t0 = a0 + a2, t1 = a0 - a2;
    const pf2 t2 = a1 + a3, d = a1 - a3;  // t3 = SIGN i d
    a0 = t0 + t2;
    a1 = c_add_j<SIGN>(t1, d);
    a2 = t0 - t2;
    a3 = c_sub_j<SIGN>(t1, d);
}

template <int SIGN>
__device__ __forceinline__ void cdft8(pf2& x0, pf2& x1, pf2& x2, pf2& x3, pf2& x4, pf2& x5, pf2& x6, pf2& x7)
{
    constexpr float C = 0.70710678118654752440f;
    const pf2 c2 = {C, C};
    cdft4<SIGN>(x0, x2, x4, x6);
    cdft4<SIGN>(x1, x3, x5, x7);
    // O1 *= W8 = C (1 + SIGN i), O2 *= SIGN i, O3 *= W8^3 = C (-1 + SIGN i)
    const pf2 o1 = c_add_j<SIGN>(x3, x3) * c2;
    const pf2 o3 = c_sub_j<SIGN>(x7, x7) * (-c2);
    const pf2 e0 = x0, e1 = x2, e2 = x4, e3 = x6, o0 = x1, y5 = x5;
    x0 = e0 + o0;
    x4 = e0 - o0;
    x1 = e1 + o1;
    x5 = e1 - o1;
    x2 = c_add_j<SIGN>(e2, y5);  // e2 + o2, o2 = SIGN i x5
    x6 = c_sub_j<SIGN>(e2, y5);
    x3 = e3 + o3;
    x7 = e3 - o3;
}

template <int LOGN, int R, int NS, int SIGN>
__device__ __forceinline__ void stockham_pass32c(pf2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                 double2* __restrict__ lds, bool write)
{
    constexpr int N = 1 << LOGN, T = N / 8, B = 8 / R;
#pragma unroll
    for (int u = 0; u < B; ++u) {
        const int b = t + T * u;
        const int k = b & (NS - 1);
        if constexpr (NS > 1) {
            const double2 w64 = tw_get<LOGN, N / R>(lds_tw, k * (N / (NS * R)));
            const pf2 w1 = {(float)w64.x, SIGN > 0 ? -(float)w64.y : (float)w64.y};
            pf2 w = w1;
            v[u + B] = c_mulw(v[u + B], w1);
#pragma unroll
            for (int r = 2; r < R; ++r) {
                w = c_mulw(w, w1);
                v[u + r * B] = c_mulw(v[u + r * B], w);
            }
        }
        if constexpr (R == 8)
            cdft8<SIGN>(v[u], v[u + B], v[u + 2 * B], v[u + 3 * B], v[u + 4 * B], v[u + 5 * B], v[u + 6 * B],
                        v[u + 7 * B]);
        else if constexpr (R == 4)
            cdft4<SIGN>(v[u], v[u + B], v[u + 2 * B], v[u + 3 * B]);
        if (!write) continue;
        const int idxD = (b - k) * R + k;
        float* img = reinterpret_cast<float*>(lds);
#pragma unroll
        for (int r = 0; r < R; ++r)
            *reinterpret_cast<pf2*>(img + 4 * lds_swz(idxD + r * NS)) = v[u + r * B];
    }
}

template <int LOGN, int PASS, int SIGN>
__device__ __forceinline__ void fft_regs_tail_wave32c(pf2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                      double2* __restrict__ lds)
{
    using S = FftShape<LOGN>;
    constexpr int T = S::T;
    constexpr int NPASS = S::NPASS8 + (S::REM ? 1 : 0);
    constexpr bool is8 = PASS < S::NPASS8;
    constexpr int R = is8 ? 8 : (1 << S::REM);
    constexpr int NS = 1 << (3 * PASS);
    constexpr bool LAST = PASS == NPASS - 1;
    static_assert(R == 8 || R == 4, "radix-8 / radix-4 passes");
    wave_lds_sync();  // previous pass fully written
    const float* img = reinterpret_cast<const float*>(lds);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const pf2*>(img + 4 * lds_swz(t + T * i));
    if constexpr (LAST) {
        stockham_pass32c<LOGN, R, NS, SIGN>(v, t, lds_tw, lds, false);
    } else {
        wave_lds_sync();  // every lane has read before the image is overwritten
        stockham_pass32c<LOGN, R, NS, SIGN>(v, t, lds_tw, lds, true);
        fft_regs_tail_wave32c<LOGN, PASS + 1, SIGN>(v, t, lds_tw, lds);
    }
}

// One N-point FP32 transform (v[i] = x[t + T*i] as {re, im}) by the T = N/8
// <= 64 lanes of one wave, image lds (N 16-B slots); on exit v[i] = X[t + T*i].
template <int LOGN, int SIGN>
__device__ __forceinline__ void fft_regs_wave32c(pf2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                 double2* __restrict__ lds)
{
    static_assert(LOGN >= 6 && LOGN <= 9, "N/8 <= one wave");
    stockham_pass32c<LOGN, 8, 1, SIGN>(v, t, lds_tw, lds, true);
    fft_regs_tail_wave32c<LOGN, 1, SIGN>(v, t, lds_tw, lds);
}

}  // namespace ofdm
