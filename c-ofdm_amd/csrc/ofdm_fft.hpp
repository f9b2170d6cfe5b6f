// ofdm_fft.hpp — FP64 complex helpers and the workgroup-wide FFT used by the
// tx/rx kernels (gfx950 / CDNA4).
//
// Replaces the reference's FFTW plans (OFDM/Frame.cpp:16-24 batched
// forward/backward `fftw_plan_many_dft`, executed at Frame.cpp:64,74): an
// unnormalised DFT X[k] = sum_n x[n] exp(SIGN*2*pi*i*n*k/N), SIGN = -1
// (FFTW_FORWARD) or +1 (FFTW_BACKWARD), N = 2^LOGN, 64 <= N <= 4096.
//
// Shape: one workgroup of T = N/8 threads per transform. Every pass is a
// Stockham auto-sort radix-8 pass (last pass radix 2 or 4 when LOGN%3 != 0).
// Thread t always holds in[t + T*i], i = 0..7, so the first pass reads
// straight from HBM (or an LDS-DMA stage) with 16-B coalesced accesses;
// intermediate passes exchange through LDS (ds_read/ds_write_b128). The LDS
// image is XOR-swizzled, slot(e) = e ^ ((e >> 3) & 7): the stride-8 writes of
// the first pass and the unit-stride reads of every pass are both
// bank-conflict free under gfx950's ds_write_b128 (8-lane) and ds_read_b128
// (16-lane) groups, with no padding (N x 16 B per transform).
//
// Twiddles live in LDS as a two-level table W_N^j = HI[j>>6] * LO[j&63]
// (N/64 + 64 entries, ~1.5 KiB at N=2048; LO stored at (j ^ ((j>>4)&3)),
// which makes the strided LO reads of every pass conflict-free for N=64..4096): the FFT issues no global loads,
// so an LDS-DMA prefetch of the next symbol stays in flight across it, and the
// workgroup barriers are raw s_barrier + lgkmcnt(0) (a __syncthreads()
// would add vmcnt(0) and drain that prefetch).
#pragma once
#include <hip/hip_runtime.h>
#include <cfloat>

// Phase markers for the annotated-ISA instruction count (tools/isa_phases.py,
// built with -DOFDM_PHASE_MARKS): an assembler comment naming the phase that
// starts there. Empty in the product build.
#ifdef OFDM_PHASE_MARKS
#define OFDM_PHASE(name) asm volatile("; OFDM_PHASE " #name)
#else
#define OFDM_PHASE(name) ((void)0)
#endif

namespace ofdm {

// Diagnostics build of the fused stream decode (stream_decode_kernel<.., true>,
// selected by OFDM_DECODE_STOP=k): every wave ends at stop point k, so SQ
// counters of runs with k = 1, 2, ... give each segment's executed
// instructions by difference (tools/decode_phase_counts.sh). Never set in
// the product path; the product instantiation has no checks.
static __device__ int g_decode_stop = 1 << 30;
#define OFDM_STOP(PROF, k)                                                   \
    do {                                                                     \
        if constexpr (PROF) {                                                \
            if ((k) >= g_decode_stop) __builtin_amdgcn_endpgm();             \
        }                                                                    \
    } while (0)

// ---------------------------------------------------------------- complex
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }

// Complex product. FFT-internal: contraction allowed.
__device__ __forceinline__ double2 cmul(double2 a, double2 b)
{
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

// Separately rounded FP64 operations, as the reference's x86-64 build (no
// FMA) computes them. HIP's __dmul_rn/__dadd_rn are plain operators that the
// default -ffp-contract=fast-honor-pragmas would fuse into v_fma_f64; the
// pragma drops the `contract` flag on these operations, even after inlining.
__device__ __forceinline__ double mul_rn(double a, double b)
{
#pragma clang fp contract(off)
    return a * b;
}
__device__ __forceinline__ double add_rn(double a, double b)
{
#pragma clang fp contract(off)
    return a + b;
}
__device__ __forceinline__ double sub_rn(double a, double b)
{
#pragma clang fp contract(off)
    return a - b;
}

// Complex product with the fused form spelled out (no choice left to the
// compiler's contraction: two instantiations of one kernel round alike).
__device__ __forceinline__ double2 cmul_fma(double2 a, double2 b)
{
    return make_double2(__builtin_fma(a.x, b.x, -mul_rn(a.y, b.y)), __builtin_fma(a.x, b.y, mul_rn(a.y, b.x)));
}

// Complex product with the exact rounding of g++'s inline _Complex multiply
// on x86-64 (no FMA): used where the reference's own arithmetic is mirrored.
__device__ __forceinline__ double2 cmul_exact(double2 a, double2 b)
{
    return make_double2(sub_rn(mul_rn(a.x, b.x), mul_rn(a.y, b.y)),
                        add_rn(mul_rn(a.x, b.y), mul_rn(a.y, b.x)));
}

// atan2 for the stream decode's phases (carg of a complex sum: cp_freq_sinh,
// pr_phase_sinh, chan_char_lq's per-carrier angles; Frame.hpp:238-274,
// 397-405), within 3 ulp of the correctly rounded value (the stream's 1e-9
// parity bar; measured 2.5 ulp worst over 2e5 random arguments against a
// 50-digit atan2), branch-free, about 45 VALU instructions against the math
// library's ~105. Octant reduction to |u| <= tan(pi/8) with one division
// (u = n/d, or (n - d)/(n + d) and pi/4 added), then atan(u) = u + u z P(z),
// z = u^2, P of degree 10 (a Chebyshev-node fit with 2e-18 absolute error
// on [0, tan^2(pi/8)]). IEEE special cases by selects: zeros (+-0 or +-pi
// by the signs), infinities (multiples of pi/4), NaN.
__device__ __forceinline__ double atan2_fast(double y, double x)
{
    double ax = fabs(x), ay = fabs(y);
    const bool ix = ax > DBL_MAX, iy = ay > DBL_MAX;  // infinite (NaN compares false)
    if (ix || iy) {  // the direction of the infinite argument(s)
        ax = ix ? 1.0 : 0.0;
        ay = iy ? 1.0 : 0.0;
    }
    const bool sw = ay > ax;
    const double n = sw ? ax : ay, d0 = sw ? ay : ax;  // n <= d
    const double d = d0 > 0.0 ? d0 : 1.0;              // both zero: u = 0
    const bool hi = n > d * 0.41421356237309503;       // tan(pi/8)
    const double u = hi ? (n - d) / (n + d) : n / d;
    const double z = u * u;
    double p = -0.01917688711906226;
    p = __builtin_fma(p, z, 0.03923165829558719);
    p = __builtin_fma(p, z, -0.0508544973794026);
    p = __builtin_fma(p, z, 0.0585814891280221);
    p = __builtin_fma(p, z, -0.06664511447381948);
    p = __builtin_fma(p, z, 0.07692183190826087);
    p = __builtin_fma(p, z, -0.09090904578123903);
    p = __builtin_fma(p, z, 0.11111111015256361);
    p = __builtin_fma(p, z, -0.14285714284666542);
    p = __builtin_fma(p, z, 0.1999999999999552);
    p = __builtin_fma(p, z, -0.3333333333333333);
    double r = __builtin_fma(u * z, p, u);
    if (hi) r += 0.78539816339744830962;  // pi/4
    if (sw) r = 1.5707963267948966192 - r;
    if (__builtin_signbit(x)) r = 3.1415926535897932385 - r;
    r = copysign(r, y);
    return (x != x || y != y) ? x + y : r;
}

// cp_freq_sinh's symbol phase carg(sum_j conj(x_j) x_{j+N}) over the
// freq-shifted samples (Frame.hpp:238-263), from the sum acc over the raw
// samples times the shift's phasor rot. The reference's sum starts at +0, so
// an empty or all-zero one (cp = 0) has phase 0, where the signed zeros of
// acc * rot would give atan2(+-0, -0) = +-pi.
__device__ __forceinline__ double cp_phase(double2 acc, double2 rot)
{
    if (acc.x == 0.0 && acc.y == 0.0) return 0.0;
    const double2 r = cmul_exact(acc, rot);
    return atan2_fast(r.y, r.x);
}

// libgcc __divdc3 (Smith's algorithm) for finite operands — what the
// reference's std::complex<double> operator/ compiles to.
__device__ __forceinline__ double2 cdiv_exact(double2 n, double2 d)
{
    const double a = n.x, b = n.y, c = d.x, e = d.y;
    double x, y;
    if (fabs(c) < fabs(e)) {
        const double ratio = c / e;
        const double denom = add_rn(mul_rn(c, ratio), e);
        x = add_rn(mul_rn(a, ratio), b) / denom;
        y = sub_rn(mul_rn(b, ratio), a) / denom;
    } else {
        const double ratio = e / c;
        const double denom = add_rn(mul_rn(e, ratio), c);
        x = add_rn(mul_rn(b, ratio), a) / denom;
        y = sub_rn(b, mul_rn(a, ratio)) / denom;
    }
    return make_double2(x, y);
}

// a * (SIGN * i)
template <int SIGN>
__device__ __forceinline__ double2 mul_j(double2 a)
{
    return SIGN > 0 ? make_double2(-a.y, a.x) : make_double2(a.y, -a.x);
}

__device__ __forceinline__ int lds_swz(int e) { return e ^ ((e >> 3) & 7); }

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// operations, not for its vector-memory queue (so stores and LDS-DMA issued
// earlier stay in flight).
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// ---------------------------------------------------------------- twiddles
template <int LOGN>
struct TwLds {
    static constexpr int N = 1 << LOGN;
    static constexpr int NHI = N / 64;          // >= 1 for N >= 64
    static constexpr int SIZE = NHI + 64;       // double2 entries in LDS
};

// Fill the two-level table from the context's global W_N^j table.
template <int LOGN>
__device__ __forceinline__ void load_twiddles(const double2* __restrict__ tw, double2* __restrict__ lds_tw, int t,
                                              int nthreads)
{
    constexpr int NHI = TwLds<LOGN>::NHI;
    for (int i = t; i < NHI + 64; i += nthreads) {  // branch-free body: loads are not serialised
        const int j = i - NHI;
        const bool hi = i < NHI;
        const double2 w = tw[hi ? i * 64 : j];
        lds_tw[hi ? i : NHI + (j ^ ((j >> 4) & 3))] = w;
    }
}

// Split fill for kernels that must not wait on their own prefetch: fetch one
// table entry per thread unconditionally (clamped), store it later. Needs
// T >= TwLds::SIZE (N >= 1024); smaller N use load_twiddles.
template <int LOGN>
struct TwPiece {
    double2 w;
    int dst;
};

template <int LOGN>
__device__ __forceinline__ TwPiece<LOGN> tw_fetch(const double2* __restrict__ tw, int t)
{
    constexpr int NHI = TwLds<LOGN>::NHI;
    const int i = t < NHI + 64 ? t : 0;
    const int j = i - NHI;
    const bool hi = i < NHI;
    return {tw[hi ? i * 64 : j], hi ? i : NHI + (j ^ ((j >> 4) & 3))};
}

// Unconditional: threads past the table rewrite entry 0 with the identical
// value (a guarded store would let the compiler sink the load into the guard
// and wait on every load issued before it).
template <int LOGN>
__device__ __forceinline__ void tw_store(const TwPiece<LOGN>& p, double2* __restrict__ lds_tw)
{
    lds_tw[p.dst] = p.w;
}

// W_N^j (forward sign) from the LDS table, for 0 <= j < JMAX. When JMAX <= 64
// (every base twiddle of a radix-R pass with N/R <= 64, e.g. all radix-8
// passes of N <= 512) the HI factor is HI[0] = (1, -0), whose product leaves
// LO bit for bit: it is skipped.
template <int LOGN, int JMAX = (1 << LOGN)>
__device__ __forceinline__ double2 tw_get(const double2* __restrict__ lds_tw, int j)
{
    constexpr int NHI = TwLds<LOGN>::NHI;
    const int lo = j & 63;
    const double2 wlo = lds_tw[NHI + (lo ^ ((lo >> 4) & 3))];
    if constexpr (NHI == 1 || JMAX <= 64) return wlo;
    return cmul(lds_tw[j >> 6], wlo);
}

// ---------------------------------------------------------------- DFTs
template <int SIGN>
__device__ __forceinline__ void dft2(double2& a, double2& b)
{
    const double2 t = a;
    a = cadd(t, b);
    b = csub(t, b);
}

template <int SIGN>
__device__ __forceinline__ void dft4(double2& a0, double2& a1, double2& a2, double2& a3)
{
    const double2 t0 = cadd(a0, a2), t1 = csub(a0, a2);
    const double2 t2 = cadd(a1, a3), t3 = mul_j<SIGN>(csub(a1, a3));
    a0 = cadd(t0, t2);
    a1 = cadd(t1, t3);
    a2 = csub(t0, t2);
    a3 = csub(t1, t3);
}

template <int SIGN>
__device__ __forceinline__ void dft8(double2& x0, double2& x1, double2& x2, double2& x3,
                                     double2& x4, double2& x5, double2& x6, double2& x7)
{
    constexpr double C = 0.70710678118654752440084436210484903928483593768847;
    dft4<SIGN>(x0, x2, x4, x6);  // E0..E3
    dft4<SIGN>(x1, x3, x5, x7);  // O0..O3
    // O1 *= W8, O2 *= W8^2 = SIGN*i, O3 *= W8^3
    const double2 o1 = make_double2((x3.x - SIGN * x3.y) * C, (x3.y + SIGN * x3.x) * C);
    const double2 o2 = mul_j<SIGN>(x5);
    const double2 o3 = make_double2(-(x7.x + SIGN * x7.y) * C, (SIGN * x7.x - x7.y) * C);
    const double2 e0 = x0, e1 = x2, e2 = x4, e3 = x6, o0 = x1;
    x0 = cadd(e0, o0);
    x4 = csub(e0, o0);
    x1 = cadd(e1, o1);
    x5 = csub(e1, o1);
    x2 = cadd(e2, o2);
    x6 = csub(e2, o2);
    x3 = cadd(e3, o3);
    x7 = csub(e3, o3);
}

// ---------------------------------------------------------------- passes
template <int LOGN>
struct FftShape {
    static constexpr int N = 1 << LOGN;
    static constexpr int T = N / 8;            // threads per transform
    static constexpr int NPASS8 = LOGN / 3;    // radix-8 passes
    static constexpr int REM = LOGN % 3;       // trailing radix-2/4 pass
    static constexpr int PADN = N;             // LDS elements per transform (swizzled, unpadded)
};

// One Stockham pass, radix R, input span NS. v[i] holds in[t + T*i].
// Twiddle powers w^r, r < R, of w = W_N^(k*N/(NS*R)) from the LDS table.
// Base twiddles w = W_N^(k*N/(NS*R)) of a pass, one per butterfly of this
// thread (B = 8/R of them). Data independent: the streaming FFT fetches them
// before the barrier that precedes the pass.
template <int LOGN, int R, int NS, int SIGN>
struct PassTw {
    double2 w[8 / R];
};

template <int LOGN, int R, int NS, int SIGN>
__device__ __forceinline__ PassTw<LOGN, R, NS, SIGN> pass_twiddles(int t, const double2* __restrict__ lds_tw)
{
    constexpr int N = 1 << LOGN, T = N / 8, B = 8 / R;
    PassTw<LOGN, R, NS, SIGN> tw;
#pragma unroll
    for (int u = 0; u < B; ++u) {
        if constexpr (NS > 1) {
            const int k = (t + T * u) & (NS - 1);
            double2 w1 = tw_get<LOGN, N / R>(lds_tw, k * (N / (NS * R)));
            if (SIGN > 0) w1.y = -w1.y;
            tw.w[u] = w1;
        }
    }
    return tw;
}

// One Stockham pass with given base twiddles (see stockham_pass).
// WRITE = false: the butterflies' results stay in v (last pass of fft_regs).
template <int LOGN, int R, int NS, int SIGN, bool WRITE = true>
__device__ __forceinline__ void stockham_apply(double2 (&v)[8], int t, const PassTw<LOGN, R, NS, SIGN>& tw,
                                               double2* __restrict__ lds)
{
    constexpr int N = 1 << LOGN, T = N / 8, B = 8 / R;
#pragma unroll
    for (int u = 0; u < B; ++u) {
        const int b = t + T * u;
        const int k = b & (NS - 1);
        if constexpr (NS > 1) {
            // running power w^r (two live twiddles: the register window of the
            // streaming kernels leaves no room for all seven)
            const double2 w1 = tw.w[u];
            double2 w = w1;
            v[u + B] = cmul(v[u + B], w1);
#pragma unroll
            for (int r = 2; r < R; ++r) {
                w = cmul(w, w1);
                v[u + r * B] = cmul(v[u + r * B], w);
            }
        }
        if constexpr (R == 8)
            dft8<SIGN>(v[u], v[u + B], v[u + 2 * B], v[u + 3 * B], v[u + 4 * B], v[u + 5 * B],
                       v[u + 6 * B], v[u + 7 * B]);
        else if constexpr (R == 4)
            dft4<SIGN>(v[u], v[u + B], v[u + 2 * B], v[u + 3 * B]);
        else
            dft2<SIGN>(v[u], v[u + B]);
        if constexpr (!WRITE) continue;
        const int idxD = (b - k) * R + k;
        if constexpr (NS % 64 == 0) {
            // r*NS has zero low 6 bits: the swizzle of idxD carries over, so one
            // base address + immediate offsets
            double2* base = lds + lds_swz(idxD);
#pragma unroll
            for (int r = 0; r < R; ++r) base[r * NS] = v[u + r * B];
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) lds[lds_swz(idxD + r * NS)] = v[u + r * B];
        }
    }
}

// One Stockham pass, radix R, input span NS. v[i] holds in[t + T*i].
// Twiddle powers w^r, r < R, of w = W_N^(k*N/(NS*R)) from the LDS table.
template <int LOGN, int R, int NS, int SIGN>
__device__ __forceinline__ void stockham_pass(double2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                              double2* __restrict__ lds)
{
    stockham_apply<LOGN, R, NS, SIGN>(v, t, pass_twiddles<LOGN, R, NS, SIGN>(t, lds_tw), lds);
}

// Last pass kept in registers (v[i] = X[t + T*i] on exit; see fft_regs).
template <int LOGN, int R, int NS, int SIGN>
__device__ __forceinline__ void stockham_pass_regs(double2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                   double2* __restrict__ lds)
{
    stockham_apply<LOGN, R, NS, SIGN, false>(v, t, pass_twiddles<LOGN, R, NS, SIGN>(t, lds_tw), lds);
}

template <int LOGN>
__device__ __forceinline__ void lds_load8(double2 (&v)[8], int t, const double2* __restrict__ lds)
{
    constexpr int T = (1 << LOGN) / 8;
    if constexpr (T % 64 == 0) {
        const double2* base = lds + lds_swz(t);  // T*i has zero low 6 bits
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = base[T * i];
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = lds[lds_swz(t + T * i)];
    }
}

// Remaining passes after the first one has been written to `lds`.
template <int LOGN, int PASS, int SIGN>
__device__ __forceinline__ void fft_tail(double2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                         double2* __restrict__ lds)
{
    using S = FftShape<LOGN>;
    constexpr int NPASS = S::NPASS8 + (S::REM ? 1 : 0);
    if constexpr (PASS < NPASS) {
        constexpr bool is8 = PASS < S::NPASS8;
        constexpr int R = is8 ? 8 : (1 << S::REM);
        constexpr int NS = 1 << (3 * PASS);
        lds_barrier();  // previous pass fully written
        lds_load8<LOGN>(v, t, lds);
        lds_barrier();  // everyone has read before the buffer is overwritten
        stockham_pass<LOGN, R, NS, SIGN>(v, t, lds_tw, lds);
        fft_tail<LOGN, PASS + 1, SIGN>(v, t, lds_tw, lds);
    }
}

// Full transform. On entry v[i] = x[t + T*i]; on exit the natural-order
// result X[0..N) is in lds (index lds_swz(k)) and the workgroup is synced.
template <int LOGN, int SIGN>
__device__ __forceinline__ void fft_block(double2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                          double2* __restrict__ lds)
{
    static_assert(LOGN >= 6 && LOGN <= 12, "N must be 64..4096");
    stockham_pass<LOGN, 8, 1, SIGN>(v, t, lds_tw, lds);
    fft_tail<LOGN, 1, SIGN>(v, t, lds_tw, lds);
    lds_barrier();
}

// ---------------------------------------------------------------- partial workgroup
// fft_block run by the first N/8 threads of a larger workgroup: `active` is
// wave-uniform (N/8 a multiple of 64); every thread takes the barriers.
template <int LOGN, int PASS, int SIGN>
__device__ __forceinline__ void fft_tail_active(double2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                double2* __restrict__ lds, bool active)
{
    using S = FftShape<LOGN>;
    constexpr int NPASS = S::NPASS8 + (S::REM ? 1 : 0);
    if constexpr (PASS < NPASS) {
        constexpr bool is8 = PASS < S::NPASS8;
        constexpr int R = is8 ? 8 : (1 << S::REM);
        constexpr int NS = 1 << (3 * PASS);
        lds_barrier();
        if (active) lds_load8<LOGN>(v, t, lds);
        lds_barrier();
        if (active) stockham_pass<LOGN, R, NS, SIGN>(v, t, lds_tw, lds);
        fft_tail_active<LOGN, PASS + 1, SIGN>(v, t, lds_tw, lds, active);
    }
}

template <int LOGN, int SIGN>
__device__ __forceinline__ void fft_block_active(double2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                 double2* __restrict__ lds, bool active)
{
    static_assert(LOGN >= 9 && LOGN <= 12, "N/8 must be whole waves");
    if (active) stockham_pass<LOGN, 8, 1, SIGN>(v, t, lds_tw, lds);
    fft_tail_active<LOGN, 1, SIGN>(v, t, lds_tw, lds, active);
    lds_barrier();
}

// ---------------------------------------------------------------- register output
// The last Stockham pass (span NS = N/R) writes butterfly b = t + T*u, output
// r to index b + r*N/R = t + T*(u + r*B): exactly the register v[u + r*B]
// that holds it. So the final pass needs no LDS write and no re-read: on exit
// v[i] = X[t + T*i] (natural order, coalesced for a direct HBM store).
// Single LDS image; the caller must barrier before `lds` is written again
// (other threads may still be reading the last pass's inputs).
template <int LOGN, int PASS, int SIGN>
__device__ __forceinline__ void fft_regs_tail(double2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                              double2* __restrict__ lds)
{
    using S = FftShape<LOGN>;
    constexpr int NPASS = S::NPASS8 + (S::REM ? 1 : 0);
    constexpr bool is8 = PASS < S::NPASS8;
    constexpr int R = is8 ? 8 : (1 << S::REM);
    constexpr int NS = 1 << (3 * PASS);
    constexpr bool LAST = PASS == NPASS - 1;
    const auto tw = pass_twiddles<LOGN, R, NS, SIGN>(t, lds_tw);  // constant table: before the barrier
    lds_barrier();  // previous pass fully written
    lds_load8<LOGN>(v, t, lds);
    if constexpr (LAST) {
        stockham_apply<LOGN, R, NS, SIGN, false>(v, t, tw, lds);
    } else {
        lds_barrier();  // everyone has read before the image is overwritten
        stockham_apply<LOGN, R, NS, SIGN>(v, t, tw, lds);
        fft_regs_tail<LOGN, PASS + 1, SIGN>(v, t, lds_tw, lds);
    }
}

template <int LOGN, int SIGN>
__device__ __forceinline__ void fft_regs(double2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                         double2* __restrict__ lds)
{
    static_assert(LOGN >= 6 && LOGN <= 12, "N must be 64..4096");
    stockham_pass<LOGN, 8, 1, SIGN>(v, t, lds_tw, lds);
    fft_regs_tail<LOGN, 1, SIGN>(v, t, lds_tw, lds);
}

// fft_regs run by the first N/8 threads of a larger workgroup (`active`
// wave-uniform); every thread takes the barriers.
template <int LOGN, int PASS, int SIGN>
__device__ __forceinline__ void fft_regs_tail_active(double2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                     double2* __restrict__ lds, bool active)
{
    using S = FftShape<LOGN>;
    constexpr int NPASS = S::NPASS8 + (S::REM ? 1 : 0);
    constexpr bool is8 = PASS < S::NPASS8;
    constexpr int R = is8 ? 8 : (1 << S::REM);
    constexpr int NS = 1 << (3 * PASS);
    constexpr bool LAST = PASS == NPASS - 1;
    lds_barrier();  // previous pass fully written
    if (active) lds_load8<LOGN>(v, t, lds);
    if constexpr (LAST) {
        if (active) stockham_pass_regs<LOGN, R, NS, SIGN>(v, t, lds_tw, lds);
    } else {
        lds_barrier();  // everyone has read before the image is overwritten
        if (active) stockham_pass<LOGN, R, NS, SIGN>(v, t, lds_tw, lds);
        fft_regs_tail_active<LOGN, PASS + 1, SIGN>(v, t, lds_tw, lds, active);
    }
}

template <int LOGN, int SIGN>
__device__ __forceinline__ void fft_regs_active(double2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                double2* __restrict__ lds, bool active)
{
    static_assert(LOGN >= 9 && LOGN <= 12, "N/8 must be whole waves");
    if (active) stockham_pass<LOGN, 8, 1, SIGN>(v, t, lds_tw, lds);
    fft_regs_tail_active<LOGN, 1, SIGN>(v, t, lds_tw, lds, active);
}

// ---------------------------------------------------------------- one wave
// fft_regs for N = 512 (T = 64) run by ONE wave of a larger workgroup. Within
// a wave an LDS hand-off needs only the wave's own LDS operations complete
// (lgkmcnt(0)), not a workgroup barrier, so the other waves stay free (they
// wait at the caller's next barrier instead of at every pass).
__device__ __forceinline__ void wave_lds_sync()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

template <int LOGN, int PASS, int SIGN>
__device__ __forceinline__ void fft_regs_tail_wave(double2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                                   double2* __restrict__ lds)
{
    using S = FftShape<LOGN>;
    constexpr int NPASS = S::NPASS8 + (S::REM ? 1 : 0);
    constexpr bool is8 = PASS < S::NPASS8;
    constexpr int R = is8 ? 8 : (1 << S::REM);
    constexpr int NS = 1 << (3 * PASS);
    constexpr bool LAST = PASS == NPASS - 1;
    const auto tw = pass_twiddles<LOGN, R, NS, SIGN>(t, lds_tw);
    wave_lds_sync();  // previous pass fully written
    lds_load8<LOGN>(v, t, lds);
    if constexpr (LAST) {
        stockham_apply<LOGN, R, NS, SIGN, false>(v, t, tw, lds);
    } else {
        wave_lds_sync();  // every lane has read before the image is overwritten
        stockham_apply<LOGN, R, NS, SIGN>(v, t, tw, lds);
        fft_regs_tail_wave<LOGN, PASS + 1, SIGN>(v, t, lds_tw, lds);
    }
}

// On entry v[i] = x[t + T*i] (T = N/8 <= 64; for N < 512 a wave holds
// 512/N transforms side by side, t the thread's index within its transform,
// lds that transform's image); on exit v[i] = X[t + T*i].
template <int LOGN, int SIGN>
__device__ __forceinline__ void fft_regs_wave(double2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                              double2* __restrict__ lds)
{
    static_assert(LOGN >= 6 && LOGN <= 9, "N/8 <= one wave");
    stockham_pass<LOGN, 8, 1, SIGN>(v, t, lds_tw, lds);
    fft_regs_tail_wave<LOGN, 1, SIGN>(v, t, lds_tw, lds);
}

// fft_block run within ONE wave (N <= 512): natural-order result X[0..N) in
// lds (index lds_swz(k)), visible to the wave on exit.
template <int LOGN, int PASS, int SIGN>
__device__ __forceinline__ void fft_tail_wave(double2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                              double2* __restrict__ lds)
{
    using S = FftShape<LOGN>;
    constexpr int NPASS = S::NPASS8 + (S::REM ? 1 : 0);
    if constexpr (PASS < NPASS) {
        constexpr bool is8 = PASS < S::NPASS8;
        constexpr int R = is8 ? 8 : (1 << S::REM);
        constexpr int NS = 1 << (3 * PASS);
        const auto tw = pass_twiddles<LOGN, R, NS, SIGN>(t, lds_tw);
        wave_lds_sync();  // previous pass fully written
        lds_load8<LOGN>(v, t, lds);
        wave_lds_sync();  // every lane has read before the image is overwritten
        stockham_apply<LOGN, R, NS, SIGN>(v, t, tw, lds);
        fft_tail_wave<LOGN, PASS + 1, SIGN>(v, t, lds_tw, lds);
    }
}

// For N < 512 a wave holds 512/N transforms side by side (t: the thread's
// index within its transform, lds: that transform's image).
template <int LOGN, int SIGN>
__device__ __forceinline__ void fft_block_wave(double2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                               double2* __restrict__ lds)
{
    static_assert(LOGN >= 6 && LOGN <= 9, "N/8 <= one wave");
    stockham_pass<LOGN, 8, 1, SIGN>(v, t, lds_tw, lds);
    fft_tail_wave<LOGN, 1, SIGN>(v, t, lds_tw, lds);
    wave_lds_sync();
}

// ---------------------------------------------------------------- ping-pong
// Same transform over two LDS images: pass p writes buf[(start + p) & 1] and
// pass p+1 reads it, so one barrier per pass suffices (a buffer is only
// rewritten two passes later, after every thread has crossed the barrier that
// follows its last read). Used by the streaming tx/rx kernels, where it halves
// the per-symbol barriers of fft_block.
template <int LOGN>
struct FftPasses {
    static constexpr int value = FftShape<LOGN>::NPASS8 + (FftShape<LOGN>::REM ? 1 : 0);
};

struct NoHook {
    __device__ __forceinline__ void operator()() const {}
};

template <int LOGN, int PASS, int SIGN, class Hook>
__device__ __forceinline__ void fft_pp_tail(double2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                            double2* __restrict__ b0, double2* __restrict__ b1, const Hook& hook)
{
    using S = FftShape<LOGN>;
    constexpr int NPASS = FftPasses<LOGN>::value;
    if constexpr (PASS < NPASS) {
        constexpr bool is8 = PASS < S::NPASS8;
        constexpr int R = is8 ? 8 : (1 << S::REM);
        constexpr int NS = 1 << (3 * PASS);
        const auto tw = pass_twiddles<LOGN, R, NS, SIGN>(t, lds_tw);  // constant table: before the barrier
        lds_barrier();  // pass PASS-1 fully written to b1
        lds_load8<LOGN>(v, t, b1);
        stockham_apply<LOGN, R, NS, SIGN>(v, t, tw, b0);
        fft_pp_tail<LOGN, PASS + 1, SIGN>(v, t, lds_tw, b1, b0, hook);
    } else {
        hook();         // e.g. publish the next symbol's LDS inputs under the same barrier
        lds_barrier();  // result (in b1) visible
    }
}

// On entry v[i] = x[t + T*i]. Pass 0 writes `first`; returns the buffer
// holding the natural-order result (index lds_swz(k)), workgroup synced. A
// caller that streams symbols passes the returned buffer as `second` (and the
// other one as `first`) on the next call, so pass 0 never overwrites a buffer
// other threads may still be reading.
template <int LOGN, int SIGN, class Hook = NoHook>
__device__ __forceinline__ double2* fft_pp(double2 (&v)[8], int t, const double2* __restrict__ lds_tw,
                                           double2* __restrict__ first, double2* __restrict__ second,
                                           const Hook& hook = Hook())
{
    static_assert(LOGN >= 6 && LOGN <= 12, "N must be 64..4096");
    stockham_pass<LOGN, 8, 1, SIGN>(v, t, lds_tw, first);
    fft_pp_tail<LOGN, 1, SIGN>(v, t, lds_tw, second, first, hook);
    return (FftPasses<LOGN>::value & 1) ? first : second;
}

}  // namespace ofdm
