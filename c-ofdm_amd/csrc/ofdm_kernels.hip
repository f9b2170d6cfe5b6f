// ofdm_kernels.hip — hand-written HIP kernels for the OFDM modem hot path on
// MI355X (gfx950). FP64 throughout (the reference computes in
// std::complex<double>); memory-bound by design (~2.4 flop/B),
// so no MFMA: the levers are coalesced 16-B HBM traffic, LDS-resident FFT
// passes and one HBM round trip per sample.
//
//   tx_kernel   : Modulation::mod (modulation.cpp:39-50) + FFT_FORM::write
//                 (Frame.cpp:54-70) + OFDM_FORM::write CP attach
//                 (Frame.cpp:185-198) [+ FRAME_FORM::get_int16, Frame.cpp:249-256]
//                 — one workgroup per OFDM symbol.
//   rx_kernel   : OFDM_FORM::fft CP strip (Frame.hpp:276-282) + FFT_FORM::read
//                 (Frame.cpp:73-96) [+ caller's chan divide, main.cpp:69-71]
//                 + Modulation::demod (modulation.cpp:53-87) + bit-error count
//                 — one workgroup per frame; the frame's data carriers stay in
//                 VGPRs until the frame-global pilot normalisation is known.
//   demap/map   : Modulation::demod / ::mod on flat point arrays.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "ofdm_dev.hpp"
#include "ofdm_fft.hpp"
#include "ofdm_internal.hpp"
#include "ofdm_rx2.hpp"

#include <type_traits>

namespace ofdm {

// ------------------------------------------------------------------ helpers

// k-bit symbol g of an MSB-first byte stream (bit_stream_converter(k, 8, ...),
// modulation.cpp:90-125; bits past the end read as the converter's zero pad).
__device__ __forceinline__ int symbol_bits(const uint8_t* __restrict__ b, long nbytes, long g, int k)
{
    const long bit = g * k;
    const long byte = bit >> 3;
    const int off = (int)(bit & 7);
    const int mask = (1 << k) - 1;
    if (off + k <= 8) return (b[byte] >> (8 - off - k)) & mask;
    const int w = ((int)b[byte] << 8) | (byte + 1 < nbytes ? (int)b[byte + 1] : 0);
    return (w >> (16 - off - k)) & mask;
}

__device__ __forceinline__ int decide(double2 z, int k, double s1, int m)
{
    if (k == 1) return (z.x + z.y) > 0.0;
    const double re = __builtin_fmin(__builtin_fmax(z.x, -1.0), 1.0);
    const double im = __builtin_fmin(__builtin_fmax(z.y, -1.0), 1.0);
    const int ire = (uint8_t)(int)add_rn(mul_rn(add_rn(re, 1.0), s1), 0.5);
    const int iim = (uint8_t)(int)add_rn(mul_rn(add_rn(im, 1.0), s1), 0.5);
    return (ire | (iim * m)) & 0xff;
}

__device__ __forceinline__ double2 clamp_point(double2 z)
{
    return make_double2(z.x < -1.0 ? -1.0 : (1.0 < z.x ? 1.0 : z.x),
                        z.y < -1.0 ? -1.0 : (1.0 < z.y ? 1.0 : z.y));
}

// 32-bit integer hash (lowbias32: two 32-bit multiplies; full 64-bit mixers
// cost ~4x more quarter-rate v_mul per sample).
__device__ __forceinline__ uint32_t lowbias32(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// Per-seed keys of the AWGN counter hash.
struct AwgnKey {
    uint32_t k0, k1;
};

__device__ __forceinline__ AwgnKey awgn_key(unsigned long long seed)
{
    const uint32_t k0 = lowbias32((uint32_t)seed ^ 0x9E3779B9u);
    return {k0, lowbias32((uint32_t)(seed >> 32) + k0)};
}

// Counter-based Box-Muller AWGN (same definition as oracle orc_awgn). A
// channel model, not modem arithmetic: sample g's two 24-bit uniforms come
// from h1 = H(lo(g) ^ K(hi(g))), K(h) = H(h ^ k1) ^ k0 (H = lowbias32), and
// h2 = h1 * 0x9E3779B9 (the pair spans h1's 2^32 values, as a second hash of
// h1 did: (u1, u2) lie on a Fibonacci rank-1 lattice; one quarter-rate
// multiply instead of two, tx 0.564 -> 0.539 ms same box); log/sqrt/sin/cos
// run on the gfx950 FP32 transcendental units (v_log_f32 = log2, v_sin/cos_f32
// take revolutions).
// Per run of samples from g0 (< 2^32 long) the two possible K values are
// computed once and selected on low-word wrap.
struct AwgnRun {
    uint32_t lo0, ka, kb;  // lo(g0), K(hi(g0)), K(hi(g0) + 1)
};

__device__ __forceinline__ AwgnRun awgn_run(AwgnKey key, unsigned long long g0)
{
    const uint32_t hi = (uint32_t)(g0 >> 32);
    return {(uint32_t)g0, lowbias32(hi ^ key.k1) ^ key.k0, lowbias32((hi + 1u) ^ key.k1) ^ key.k0};
}

__device__ __forceinline__ double2 awgn_sample(const AwgnRun& run, uint32_t j, double sc)
{
    const uint32_t lo = run.lo0 + j;
    const uint32_t h1 = lowbias32(lo ^ (lo < run.lo0 ? run.kb : run.ka));
    const uint32_t h2 = h1 * 0x9E3779B9u;  // u2: h1 times the Fibonacci multiplier
    const float u1 = (float)((h1 >> 8) + 1) * 0x1.0p-24f;  // (0, 1]
    const float u2 = (float)(h2 >> 8) * 0x1.0p-24f;        // [0, 1)
    const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));  // sqrt(-2 ln u1)
    const float c = __builtin_amdgcn_cosf(u2), s = __builtin_amdgcn_sinf(u2);                  // of 2*pi*u2
    return make_double2((double)(r * c) * sc, (double)(r * s) * sc);
}

// awgn_sample with the scale folded into the FP32 radius (one FP32 multiply
// instead of two FP64 ones per sample; the noise moves by ~1 FP32 ulp, far
// inside the channel model's 1e-5 parity against the FP64 oracle). The f64 tx
// output uses this form; the int16 wire output keeps awgn_sample's FP64
// scale, so the two outputs' noise can differ by that ulp before truncation.
__device__ __forceinline__ double2 awgn_sample_scaled(const AwgnRun& run, uint32_t j, float scf)
{
    const uint32_t lo = run.lo0 + j;
    const uint32_t h1 = lowbias32(lo ^ (lo < run.lo0 ? run.kb : run.ka));
    const uint32_t h2 = h1 * 0x9E3779B9u;
    const float u1 = (float)((h1 >> 8) + 1) * 0x1.0p-24f;
    const float u2 = (float)(h2 >> 8) * 0x1.0p-24f;
    const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1)) * scf;
    const float c = __builtin_amdgcn_cosf(u2), s = __builtin_amdgcn_sinf(u2);
    return make_double2((double)(r * c), (double)(r * s));
}

__device__ __forceinline__ int16_t to_int16(double v) { return (int16_t)(int)v; }

// A global load the compiler's wait-count pass does not track: issued and
// waited for (vmcnt(0)) inside one asm block. For rare paths (e.g. channel
// carriers that do not fit LDS) inside code that otherwise issues only
// stores: a tracked load there makes the pass put `s_waitcnt vmcnt(0)` in
// front of every later store that reuses its registers, which serialises the
// epilogue's stores behind each other and behind the next frame's prefetch.
__device__ __forceinline__ double2 load_untracked(const double2* p)
{
    double2 v;
    asm volatile("global_load_dwordx4 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}

template <int NT>
__device__ __forceinline__ double block_sum(double v, double* red)
{
#pragma unroll
    for (int o = (NT >= 64 ? 32 : NT / 2); o > 0; o >>= 1) v += __shfl_xor(v, o);
    constexpr int NW = (NT + 63) / 64;
    if constexpr (NW == 1) {
        return v;
    } else {
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        __syncthreads();
        if (lane == 0) red[w] = v;
        __syncthreads();
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < NW; ++i) s += red[i];
        return s;
    }
}

// block_sum with LDS-only barriers: leaves in-flight vector-memory loads and
// stores outstanding (a __syncthreads() would drain them).
template <int NT>
__device__ __forceinline__ double block_sum_lds(double v, double* red)
{
#pragma unroll
    for (int o = (NT >= 64 ? 32 : NT / 2); o > 0; o >>= 1) v += __shfl_xor(v, o);
    constexpr int NW = (NT + 63) / 64;
    if constexpr (NW == 1) {
        return v;
    } else {
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        if (lane == 0) red[w] = v;
        lds_barrier();
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < NW; ++i) s += red[i];
        lds_barrier();  // red is rewritten by the next reduction
        return s;
    }
}

template <int NT>
__device__ __forceinline__ unsigned long long block_sum_u64(unsigned long long v, double* red)
{
    for (int o = (NT >= 64 ? 32 : NT / 2); o > 0; o >>= 1) v += __shfl_xor(v, o);
    constexpr int NW = (NT + 63) / 64;
    if constexpr (NW == 1) {
        return v;
    } else {
        unsigned long long* r = reinterpret_cast<unsigned long long*>(red);
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        __syncthreads();
        if (lane == 0) r[w] = v;
        __syncthreads();
        unsigned long long s = 0;
        for (int i = 0; i < NW; ++i) s += r[i];
        return s;
    }
}

// ------------------------------------------------------------------ tx
// Persistent over symbols: grid-stride loop, so the twiddle table and each
// thread's bin classification are loaded once per workgroup, and the next
// symbol's payload bytes are fetched into registers while this one is
// transformed and written.
// POINTS = true: FFT_FORM::write on given constellation points (no payload bytes).
// NOISE / I16: fused AWGN and int16 wire output compiled in (a.noise_scale > 0,
// a.iq16 != nullptr), so each variant gets its own register allocation.
// Workgroups per CU the register allocation is bounded for: 4 at N = 2048
// with f64 output (128 VGPRs, ~36 dwords spilled; 3 per CU at the unbounded
// 163 VGPRs): tx 0.556 -> 0.545 ms in the bench step, same box
// (profiles/r03z_tx_occupancy.txt). Other shapes and the int16 output keep
// the compiler's choice.
constexpr int tx_min_blocks(int logn, bool i16) { return logn == 11 && !i16 ? 4 : 1; }

template <int LOGN, bool POINTS, bool NOISE, bool I16>
__global__ void __launch_bounds__((1 << LOGN) / 8, tx_min_blocks(LOGN, I16)) tx_kernel(TxArgs a)
{
    using FS = FftShape<LOGN>;
    constexpr int N = FS::N, T = FS::T;
    extern __shared__ double2 smem[];
    double2* fft = smem;
    double2* lds_tw = smem + FS::PADN;
    double2* lds_const = lds_tw + TwLds<LOGN>::SIZE;  // 2^k points, then pilot (TX_LDS_PILOT) and 0 (TX_LDS_ZERO)
    uint8_t* sbytes = reinterpret_cast<uint8_t*>(lds_const + TX_LDS_ZERO + 1);  // one symbol's payload (N bytes)
    const int t = threadIdx.x;
    load_twiddles<LOGN>(a.tab.tw, lds_tw, t, T);
    for (int i = t; i < (1 << a.k); i += T) lds_const[i] = a.tab.constell[i];
    if (t == 0) {
        lds_const[TX_LDS_PILOT] = make_double2(a.pilot_ampl, 0.0);
        lds_const[TX_LDS_ZERO] = make_double2(0.0, 0.0);
    }

    // FFT_FORM::write layout (Frame.cpp:31-44,54-62) as per-bin codes: data
    // index, payload-symbol mask, table base (ofdm_internal.hpp tx_code)
    // the per-bin codes are re-read per symbol (L1/L2-resident 4*N bytes)
    // rather than held across the symbol loop: 8 fewer VGPRs live across the
    // transform and the emit

    const long nsym = a.nframes * a.S;
    const int k = a.k;
    const int bps = a.D * k / 8;  // payload bytes per symbol (host checks D*k % 8 == 0)
    const int L = N + a.cp;
    auto sym_bytes = [&](long sym) {
        const long f = sym / a.S;
        return a.bytes + f * a.bytes_per_frame + (sym - f * a.S) * bps;
    };
    // Payload prefetch, written to LDS only after the FFT so the loads' latency
    // hides behind it: 32-bit words t and t + T when every symbol's payload is
    // word aligned (bps <= N bytes = 2T words), else bytes t + T*r. Indices are
    // clamped and the whole N-byte stage is rewritten (bytes past bps are never
    // decoded), so neither side needs per-lane guards.
    const bool by_word = (bps & 3) == 0 && (a.bytes_per_frame & 3) == 0 && ((uintptr_t)a.bytes & 3) == 0;
    const int nwords = bps >> 2;
    uint32_t nb[8];
    auto fetch = [&](long s) {
        const uint8_t* src = sym_bytes(s);
        if (by_word) {
            // word indices from an opaque copy of the thread index (not held
            // across the symbol loop)
            int tt;
            asm volatile("v_mov_b32 %0, %1" : "=v"(tt) : "v"(t));
            const int wi0 = tt < nwords ? tt : 0, wi1 = tt + T < nwords ? tt + T : 0;
            const uint32_t* w = reinterpret_cast<const uint32_t*>(src);
            nb[0] = w[wi0];
            nb[1] = w[wi1];
        } else {
#pragma unroll
            for (int r = 0; r < 8; ++r) nb[r] = src[t + T * r < bps ? t + T * r : 0];
        }
    };
    auto publish = [&]() {
        if (by_word) {
            uint32_t* w = reinterpret_cast<uint32_t*>(sbytes);
            w[t] = nb[0];
            w[t + T] = nb[1];
        } else {
#pragma unroll
            for (int r = 0; r < 8; ++r) sbytes[t + T * r] = (uint8_t)nb[r];
        }
    };

    long sym = blockIdx.x;
    if (!POINTS && sym < nsym) {
        fetch(sym);
        publish();
    }
    lds_barrier();  // twiddle table + first payload visible

    // CP samples n in [N-cp, N) are registers v[i], i >= 8 - cp/T, of the same
    // thread when cp is a multiple of T (the configs' cp = N/4 = 2T)
    const bool cp_reg = (a.cp % T) == 0;
    const int i_cp = 8 - a.cp / T;
    const int kmask = (1 << k) - 1;

    // (frame, symbol) of `sym`, advanced incrementally (no 64-bit division in the loop)
    const long gstep_f = gridDim.x / a.S;
    const int gstep_s = (int)(gridDim.x - gstep_f * a.S);
    long f = sym / a.S;
    int s = (int)(sym - f * a.S);
    for (; sym < nsym; sym += gridDim.x) {
        // Modulation::mod: k-bit symbol -> constellation point (modulation.cpp:39-50);
        // pilots = pilot_ampl, unused bins 0 (Frame.cpp:56-62)
        double2 v[8];
        int code[8];
        {
            // opaque copy of the thread index: the loads stay in the loop
            int tt;
            asm volatile("v_mov_b32 %0, %1" : "=v"(tt) : "v"(t));
            const int* ct = a.tab.tx_code + tt;
#pragma unroll
            for (int i = 0; i < 8; ++i) code[i] = ct[T * i];
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int d = code[i] & 0x1fff, m = (code[i] >> 13) & 0xff, base = code[i] >> 21;
            if constexpr (POINTS) {
                v[i] = m ? a.points[sym * a.D + d] : lds_const[base];
            } else {
                const int bit = d * k;
                const int byte = bit >> 3, off = bit & 7;
                const int w = ((int)sbytes[byte] << 8) | (int)sbytes[byte + 1];
                v[i] = lds_const[((w >> (16 - off - k)) & kmask & m) + base];
            }
        }
        const long nxt = sym + gridDim.x;
        if constexpr (!POINTS) fetch(nxt < nsym ? nxt : sym);

        // unnormalised backward DFT (Frame.cpp:64); v[i] = x[t + T*i] on exit
        fft_regs<LOGN, +1>(v, t, lds_tw, fft);
        // Publish the next payload now, before this symbol's stores: on gfx9
        // vmcnt also counts stores, so a wait on these loads placed after the
        // stores would drain them every symbol. Every thread has mapped this
        // symbol (FFT barriers since), so the single stage can be rewritten.
        if constexpr (!POINTS) publish();

        // body / sqrt(N) after a CP copy of its last cp samples (Frame.cpp:66-68,191-197)
        const long base = f * a.frame_stride + a.msg_offset + (long)s * L;
        double2* out = a.iq + base;
        int16_t* out16 = I16 ? a.iq16 + 2 * base : nullptr;
        const unsigned long long g0 = a.sample_offset + (unsigned long long)sym * L;
        const AwgnRun run = NOISE ? awgn_run(awgn_key(a.seed), g0) : AwgnRun{};
        auto emit = [&](int j, double2 z) {
            if constexpr (NOISE && !I16) {  // body / sqrt(N) + noise as one FMA per component
                const double2 w = awgn_sample_scaled(run, (uint32_t)j, (float)a.noise_scale);
                store_nt(out + j, make_double2(fma(z.x, a.inv_sqrt_n, w.x), fma(z.y, a.inv_sqrt_n, w.y)));
                return;
            }
            z.x *= a.inv_sqrt_n;
            z.y *= a.inv_sqrt_n;
            if constexpr (I16) {
                const uint32_t w = (uint16_t)to_int16(z.x * a.mult) | ((uint32_t)(uint16_t)to_int16(z.y * a.mult) << 16);
                __builtin_nontemporal_store(w, reinterpret_cast<uint32_t*>(out16 + 2 * j));
            }
            if constexpr (NOISE) {
                const double2 w = awgn_sample(run, (uint32_t)j, a.noise_scale);
                z.x += w.x;
                z.y += w.y;
            }
            store_nt(out + j, z);
        };
        if (cp_reg) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (i >= i_cp) emit(t + T * i - (N - a.cp), v[i]);
        } else {
            // general cp: the tail of the symbol through the LDS image (its
            // addresses from an opaque copy of the thread index, so they are
            // not hoisted out of the symbol loop and held live for this rare path)
            int tt;
            asm volatile("v_mov_b32 %0, %1" : "=v"(tt) : "v"(t));
            lds_barrier();  // every thread has read the last pass's inputs
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (tt + T * i >= N - a.cp) fft[lds_swz(tt + T * i)] = v[i];
            lds_barrier();
            for (int j = tt; j < a.cp; j += T) emit(j, fft[lds_swz(N - a.cp + j)]);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) emit(a.cp + t + T * i, v[i]);
        // [T2 | preamble] header of full FRAME_FORM buffers (Frame.cpp:219,228-229)
        if (a.header && s == 0) {
            double2* fr = a.iq + f * a.frame_stride;
            int16_t* fr16 = I16 ? a.iq16 + 2 * f * a.frame_stride : nullptr;
            for (int j = t; j < a.header_len; j += T) {
                const double2 z = a.header[j];
                fr[j] = z;
                if constexpr (I16) {
                    fr16[2 * j] = to_int16(z.x * a.mult);
                    fr16[2 * j + 1] = to_int16(z.y * a.mult);
                }
            }
        }
        lds_barrier();  // next payload visible; the last pass's LDS reads precede the next pass 0
        s += gstep_s;
        f += gstep_f;
        if (s >= a.S) {
            s -= a.S;
            ++f;
        }
    }
}

// ------------------------------------------------------------------ rx
// One workgroup per frame. Symbol s+1 is loaded into registers (8 x 16 B per
// thread, coalesced) while symbol s is transformed; the FFT ping-pongs
// between two LDS images (fft_pp: one barrier per pass, no input stage).
// STAGED=false: the frame's S*D equalisation inputs live in VGPRs
//   (S <= RX_SMAX, D <= RX_DPT*T), written through a wave-uniform switch on
//   the symbol index so every register index is compile-time.
// STAGED=true: any S; inputs parked in a.ystage (same-thread re-read).
// The next symbol's 8 samples per thread, held in registers across the FFT:
// complex<double> (4 VGPRs each) or, for wire-format input, complex<int16>
// (1 VGPR each, converted exactly on use: FRAME_FORM::form_int16_to_double,
// Frame.hpp:472-481, fused).
template <int LOGN, bool I16>
struct SymbolRegs;

template <int LOGN>
struct SymbolRegs<LOGN, false> {
    double2 r[8];
    __device__ __forceinline__ void load(const RxArgs& a, long off, int t)
    {
        constexpr int T = (1 << LOGN) / 8;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            r[i] = load_nt(a.iq + off + t + T * i);
    }
    __device__ __forceinline__ double2 get(int i) const { return r[i]; }
};

template <int LOGN>
struct SymbolRegs<LOGN, true> {
    int r[8];
    __device__ __forceinline__ void load(const RxArgs& a, long off, int t)
    {
        constexpr int T = (1 << LOGN) / 8;
        const int* p = reinterpret_cast<const int*>(a.iq16 + off);
#pragma unroll
        for (int i = 0; i < 8; ++i) r[i] = __builtin_nontemporal_load(p + t + T * i);
    }
    __device__ __forceinline__ double2 get(int i) const
    {
        return make_double2((double)(int)(short)(r[i] & 0xffff), (double)(r[i] >> 16));
    }
};

// Symbol 0 of a frame streams HBM -> LDS by LDS-DMA (global_load_lds_dwordx4,
// or _dword for complex<int16>), issued while the previous frame's epilogue
// runs: no registers stay live across the epilogue for it. Lane l of wave w0
// lands element w0 + T*i + l, so each thread later reads only what its own
// wave fetched (a vmcnt wait, no barrier). Inline asm (MI355X guide LDS-DMA
// recipe: M0 = wave-uniform LDS byte address): the compiler does not track
// the transfer, so the reader issues its own `s_waitcnt vmcnt(0)`.
template <int LOGN, bool I16>
__device__ __forceinline__ void dma_symbol(const RxArgs& a, long off, void* stage, int t)
{
    constexpr int T = (1 << LOGN) / 8;
    constexpr int ESZ = I16 ? 4 : 16;
    const int w0 = t & ~63;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int e0 = w0 + T * i;  // wave-uniform
        const char* g = I16 ? reinterpret_cast<const char*>(a.iq16 + off + e0 + (t & 63))
                            : reinterpret_cast<const char*>(a.iq + off + e0 + (t & 63));
        const unsigned lds = __builtin_amdgcn_readfirstlane(
            (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)((char*)stage + (size_t)e0 * ESZ));
        unsigned keep;
        if constexpr (I16)
            asm volatile(
                "s_mov_b32 %0, m0\n\t"
                "s_mov_b32 m0, %2\n\t"
                "s_nop 0\n\t"
                "global_load_lds_dword %1, off nt\n\t"
                "s_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(g), "s"(lds)
                : "memory");
        else
            asm volatile(
                "s_mov_b32 %0, m0\n\t"
                "s_mov_b32 m0, %2\n\t"
                "s_nop 0\n\t"
                "global_load_lds_dwordx4 %1, off nt\n\t"
                "s_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(g), "s"(lds)
                : "memory");
    }
}

// LDS-DMA of a frame's D channel carriers (complex<double>) to chl: RX_DPT
// 16-B transfers per lane at most, lanes past D masked off. Issued before the
// next frame's symbol-0 DMA, so (returns are in order) they land first.
template <int LOGN>
__device__ __forceinline__ void dma_chan(const double2* chan, int D, double2* chl, int t)
{
    constexpr int T = (1 << LOGN) / 8;
    const int w0 = t & ~63;
#pragma unroll
    for (int i = 0; i < RX_DPT; ++i) {
        const int e0 = w0 + T * i;  // wave-uniform
        if (e0 + (t & 63) < D) {
            const char* g = reinterpret_cast<const char*>(chan + e0 + (t & 63));
            const unsigned lds = __builtin_amdgcn_readfirstlane(
                (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)((char*)chl + (size_t)e0 * 16));
            unsigned keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\t"
                "s_mov_b32 m0, %2\n\t"
                "s_nop 0\n\t"
                "global_load_lds_dwordx4 %1, off\n\t"
                "s_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(g), "s"(lds)
                : "memory");
        }
    }
}

template <int LOGN, bool I16>
__device__ __forceinline__ double2 stage_get(const void* stage, int e)
{
    if constexpr (I16) {
        const int r = reinterpret_cast<const int*>(stage)[e];
        return make_double2((double)(int)(short)(r & 0xffff), (double)(r >> 16));
    } else {
        return reinterpret_cast<const double2*>(stage)[e];
    }
}

template <int LOGN, bool STAGED, bool I16, bool SYNC>
__global__ void __launch_bounds__((1 << LOGN) / 8, 2) rx_kernel(RxArgs a)
{
    using FS = FftShape<LOGN>;
    constexpr int N = FS::N, T = FS::T;
    constexpr int SW = STAGED ? 1 : RX_SMAX;  // register window (symbols)
    extern __shared__ double2 smem[];
    const int S0 = a.S, P0 = a.P;
    double2* bufA = smem;                   // FFT ping-pong images
    double2* bufB = bufA + N;
    double2* lds_tw = bufB + FS::PADN;      // TwLds::SIZE
    double2* pil = lds_tw + TwLds<LOGN>::SIZE;  // S*P raw pilots
    double2* gain = pil + S0 * P0;          // S*P equaliser gains
    double* red = reinterpret_cast<double*>(gain + S0 * P0);
    uint8_t* dec = reinterpret_cast<uint8_t*>(bufA);  // aliases the FFT images after the transforms

    const int t0 = threadIdx.x;
    const int L = N + a.cp;
    const long fstep = gridDim.x;
    // frames to process: a.nframes, or fewer when the count is device-side
    // (speculative stream decode); uniform early exit before any prefetch
    // stream mode: a first frame whose preamble starts before the stream's
    // first sample is the host's (gather path, zeros before sample 0): the
    // frames taken here are fbase, fbase + 1, ...
    const long fbase = (SYNC && a.nframes > 0 && (!a.count || *a.count > 0) && a.starts[0] < 0) ? 1 : 0;
    const long nfr = (a.count ? min(*a.count, a.nframes) : a.nframes) - fbase;
    // Dynamic frames (a.queue): a workgroup's first frame is its blockIdx,
    // later ones come from a counter, so workgroups that run faster (CU and
    // memory-channel placement make them differ by ~15%) take more frames and
    // the kernel ends with the mean workgroup, not the slowest. The last
    // workgroup to leave zeroes the counters for the next launch.
    auto leave = [&]() {
        if (a.queue && threadIdx.x == 0) {
            __threadfence();
            if (atomicAdd(a.queue + 1, 1) == (int)gridDim.x - 1) {
                a.queue[0] = 0;
                a.queue[1] = 0;
            }
        }
    };
    if ((long)blockIdx.x >= nfr) {
        leave();
        return;
    }
    int* qslot = reinterpret_cast<int*>(red + 16);  // the next frame from the queue (red[0..7]: reductions)

    // table loads first, then symbol 0 of the first frame: every prologue wait
    // below is a counted vmcnt that leaves the symbol prefetch in flight
    constexpr bool kTwSplit = T >= TwLds<LOGN>::SIZE;
    TwPiece<LOGN> twp{};
    if constexpr (kTwSplit)
        twp = tw_fetch<LOGN>(a.tab.tw, t0);
    else
        load_twiddles<LOGN>(a.tab.tw, lds_tw, t0, T);
    // data carrier d = t0 + T*i: swizzled LDS slot of its FFT bin (low 16 bits)
    // | pilot slot (high 16); host tables are zero-padded, so no guards here
    int pk[RX_DPT];
#pragma unroll
    for (int i = 0; i < RX_DPT; ++i) pk[i] = a.tab.rx_pack[t0 + T * i];
    const int pbin = a.tab.pilot_swz[t0];
    long fl = blockIdx.x;  // this workgroup's frame
    auto frame_of = [&](long l) { return l + fbase; };
    SymbolRegs<LOGN, I16> pf;
    // sample offset of frame g's first message body (CP strip, Frame.hpp:278-279)
    auto body0 = [&](long g) { return SYNC ? a.starts[g] + a.start_off : g * a.frame_stride + a.cp; };
    dma_symbol<LOGN, I16>(a, body0(frame_of(fl)), bufB, t0);  // grid <= nframes
    if constexpr (kTwSplit) tw_store<LOGN>(twp, lds_tw);
    lds_barrier();  // twiddle table visible: fft_pp reads a pass's twiddles before its barrier

    unsigned long long errs = 0;

    // Persistent over frames (grid <= 2 workgroups per CU): the next frame's
    // symbol 0 is fetched (LDS-DMA into bufB) while this frame's epilogue
    // runs, so HBM reads do not stop between frames, and the tables are
    // loaded once per workgroup.
#pragma unroll 1
    for (long fnext; fl < nfr; fl = fnext) {
        const long f = frame_of(fl);
        // Opaque per-frame copies of the thread index, the carrier tables and
        // the geometry: everything derived from them is recomputed per frame
        // instead of being hoisted out of the frame loop and held live beside
        // the register window (which spills).
        int t;
        asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"(t0));
#pragma unroll
        for (int i = 0; i < RX_DPT; ++i) asm volatile("" : "+v"(pk[i]));
        int S = a.S, D = a.D, P = a.P;
        asm volatile("" : "+s"(S), "+s"(D), "+s"(P));
        const long x0 = body0(f);
        const int m = 1 << (a.k / 2);
        const double s1 = a.k == 1 ? 0.0 : 1.0 / (2.0 / (m - 1));
        const bool whole_frame_dec = (long)S * D <= (long)FS::PADN * 16;
        const long bpf = a.bytes_per_frame;
        // word-wise packing: k in {1,2,4,8}, whole words, 4-byte aligned outputs
        const bool by_word = (a.k == 1 || a.k == 2 || a.k == 4 || a.k == 8) && (bpf & 3) == 0 &&
                             ((uintptr_t)a.bytes & 3) == 0 && ((uintptr_t)a.ref & 3) == 0;
        double2 y[SW][RX_DPT];
        // symbol 0 is read from bufB, so pass 0 writes bufA (free: the
        // previous epilogue ended with a barrier)
        double2* first = bufA;
        double2* second = bufB;
#pragma unroll 1
        for (int s = 0; s < S; ++s) {
            double2 v[8];
            if (s == 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of symbol 0 landed
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = stage_get<LOGN, I16>(bufB, t + T * i);
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = pf.get(i);
            }
            // SYNC: the phase ramp is applied before the next symbol's
            // prefetch is issued, so its sincos temporaries are not live
            // beside the 8 prefetch registers (which spilled at N = 512)
            if (!SYNC && s + 1 < S) pf.load(a, x0 + (long)(s + 1) * L, t);
            if constexpr (SYNC) {
                // sample m = t + T*i of the body: *= e^{i(A + B m)}, by a
                // running product from e^{i(A + B t)} in steps of e^{i B T};
                // e^{i(A + B t)} from the table (uniform loads), the bits of t
                // selecting its powers (x (1, 0) is exact)
                // (the bit tests on a per-symbol opaque copy of t: hoisted
                // out of the loop, their lane masks filled the SGPRs and spilled)
                const double2* rt = a.corr + (f * S + s) * CORR_PER_SYM;
                int tr;
                asm volatile("v_mov_b32 %0, %1" : "=v"(tr) : "v"(t));
                double2 c = rt[0];
#pragma unroll
                for (int j = 0; j < LOGN - 3; ++j) c = cmul_exact(c, (tr >> j) & 1 ? rt[1 + j] : make_double2(1.0, 0.0));
                const double2 w = rt[CORR_PER_SYM - 1];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    v[i] = cmul(v[i], c);
                    if (i < 7) c = cmul(c, w);
                }
                asm volatile("" ::: "memory");  // keep the prefetch below the ramp
                if (s + 1 < S) pf.load(a, x0 + (long)(s + 1) * L, t);
            }
            // opaque copy of t: the per-pass LDS addresses are recomputed each
            // symbol instead of being hoisted out of the loop and held live
            // beside the register window
            int tl;
            asm volatile("v_mov_b32 %0, %1" : "=v"(tl) : "v"(t));
            double2* res = fft_pp<LOGN, -1>(v, tl, lds_tw, first, second);
            first = res == bufA ? bufB : bufA;
            second = res;
            if (t < P) pil[s * P + t] = res[pbin];
            if constexpr (STAGED) {
#pragma unroll
                for (int i = 0; i < RX_DPT; ++i) {
                    const int d = t + T * i;
                    if (d < D) a.ystage[(f * S + s) * D + d] = res[pk[i] & 0xffff];
                }
            } else {
                switch (s) {
#define OFDM_RX_PUT(W)                                                                    \
    case W:                                                                               \
        if constexpr (W < SW) {                                                           \
            _Pragma("unroll") for (int i = 0; i < RX_DPT; ++i) y[W][i] = res[pk[i] & 0xffff]; \
        }                                                                                 \
        break;
                    OFDM_RX_PUT(0) OFDM_RX_PUT(1) OFDM_RX_PUT(2) OFDM_RX_PUT(3)
                    OFDM_RX_PUT(4) OFDM_RX_PUT(5) OFDM_RX_PUT(6) OFDM_RX_PUT(7)
#undef OFDM_RX_PUT
                    default: break;
                }
            }
        }
        lds_barrier();  // pilots of the last symbol visible; every thread is done reading bufB
        // The channel carriers go to LDS (bufA past the decisions) by DMA
        // issued ahead of the next frame's symbol 0: read per point from HBM
        // behind that DMA (in-order returns), they cost the stream rx ~18%.
        const double2* chan = a.chan ? a.chan + f * a.chan_stride : nullptr;
        const int dec_b = (S * D + 15) & ~15;
        double2* chl = reinterpret_cast<double2*>(reinterpret_cast<char*>(bufA) + dec_b);
        const bool chan_lds = chan && dec_b + D * 16 <= N * 16;  // uniform
        if (chan_lds) dma_chan<LOGN>(chan, D, chl, t);
        // Static frame order (no queue; the stream decode): the next frame's
        // symbol 0 streams into bufB (free since the pilot barrier) from here,
        // behind the channel carriers, so it overlaps the gains as well.
        // With the queue the next frame is asked for now, its answer awaited
        // after the gains (the register holding it is live across the gains
        // only), and its DMA issued after them.
        const bool early = !a.queue;  // uniform
        if (early) {
            fnext = fl + fstep;
            if (fnext < nfr) dma_symbol<LOGN, I16>(a, body0(frame_of(fnext)), bufB, t);
        }
        int qv = 0;
        if (a.queue && t == 0) qv = atomicAdd(a.queue, 1);

        // phys_pilot_ampl = sum |pilot| / (P*S*pilot_ampl)   (Frame.cpp:76-80)
        double acc = 0.0;
        for (int i = t; i < S * P; i += T) acc += hypot(pil[i].x, pil[i].y);
        acc = block_sum_lds<T>(acc, red);
        const double phys = acc / ((double)(P * S) * a.pilot_ampl);

        // out = (F/phys) / ((F[s,p]/phys) / (F[0,p]/phys)) = F * gain[s][j]   (Frame.cpp:82-93)
        for (int i = t; i < S * P; i += T) {
            const int j = i % P;
            const double2 c0 = make_double2(pil[j].x / phys, pil[j].y / phys);
            const double2 cs = make_double2(pil[i].x / phys, pil[i].y / phys);
            const double2 coef = cdiv_exact(cs, c0);
            const double2 g = cdiv_exact(make_double2(1.0, 0.0), coef);
            gain[i] = make_double2(g.x / phys, g.y / phys);
        }
        if (chan_lds) {  // the channel DMA landed (the 8 symbol-0 transfers issued after it may still fly)
            if (early && fnext < nfr)
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (a.queue && t == 0) *qslot = qv;
        lds_barrier();
        if (!early) {
            // symbol 0 of the next frame streams into bufB behind the emit and
            // the packing
            fnext = fstep + __builtin_amdgcn_readfirstlane(*qslot);  // uniform: an SGPR
            if (fnext < nfr) dma_symbol<LOGN, I16>(a, body0(frame_of(fnext)), bufB, t);
        }

        // One symbol's RX_DPT points of the register window. Without a
        // channel (the common case) the group's gain loads are issued first
        // and the points then computed, stored and decided; the uniform
        // branches are taken once per group, so the points' LDS latencies
        // overlap. With a channel, one point at a time (register pressure).
        auto emit_point = [&](int s, int i, double2 yv) {
            // opaque: the per-point addresses are computed here, not hoisted
            // out of the emit loop and held (32 of them) across it
            int d = t + T * i, gi = s * P + (pk[i] >> 16);
            asm volatile("" : "+v"(d), "+v"(gi));
            double2 o = cmul_exact(yv, gain[gi]);
            if (a.read_out) store_nt(a.read_out + (f * S + s) * D + d, o);
            const double2 cv = chan_lds ? chl[d] : load_untracked(chan + d);
            o = a.chan_recip ? cmul_exact(o, cv) : cdiv_exact(o, cv);
            if (a.constell) store_nt(a.constell + (f * S + s) * D + d, o);
            dec[whole_frame_dec ? s * D + d : d] = (uint8_t)decide(o, a.k, s1, m);
        };
        // Without a channel (the common case) a group is straight-line code:
        // the output branch is taken once per group and the decision is
        // branch-free, so the scheduler can overlap the points' LDS reads.
        auto emit_plain = [&](int s, const double2 (&yw)[RX_DPT], auto with_store) {
            double2* cbase = a.constell + (f * S + s) * D;
#pragma unroll
            for (int i = 0; i < RX_DPT; ++i) {
                int d = t + T * i, gi = s * P + (pk[i] >> 16);
                asm volatile("" : "+v"(d), "+v"(gi));  // opaque: not hoisted and held
                if (d < D) {
                    const double2 o = cmul_exact(yw[i], gain[gi]);
                    if constexpr (decltype(with_store)::value) store_nt(cbase + d, o);
                    dec[whole_frame_dec ? s * D + d : d] = (uint8_t)decide_select(o, a.k, s1, m);
                }
            }
        };
        auto emit_group = [&](int s, const double2 (&yw)[RX_DPT]) {
            if (SYNC || chan) {  // the stream decode always has its channel
#pragma unroll
                for (int i = 0; i < RX_DPT; ++i)
                    if (t + T * i < D) emit_point(s, i, yw[i]);
            } else if (a.constell) {
                emit_plain(s, yw, std::true_type{});
            } else {
                emit_plain(s, yw, std::false_type{});
            }
        };

        auto pack = [&](long jb0, long jb1, long dbase) {
            for (long jb = jb0 + t; jb < jb1; jb += T) {
                int byte = 0;
                if (a.k == 1 || a.k == 2 || a.k == 4 || a.k == 8) {
                    const int per = 8 / a.k;
                    const long p0 = (jb - jb0) * per + dbase;
                    for (int r = 0; r < per; ++r) byte = (byte << a.k) | dec[p0 + r];
                } else {
                    for (int b = 0; b < 8; ++b) {
                        const long bit = (jb - jb0) * 8 + b;
                        const long g = bit / a.k + dbase;
                        const int within = (int)(bit % a.k);
                        byte = (byte << 1) | ((dec[g] >> (a.k - 1 - within)) & 1);
                    }
                }
                if (a.bytes) a.bytes[f * bpf + jb] = (uint8_t)byte;
                if (a.ref) errs += __popc((unsigned)(byte ^ a.ref[f * bpf + jb]));
            }
        };

        auto pack_words = [&]() {
            const int per_word = 32 / a.k;  // decisions per output word
            for (long w = t; w < bpf / 4; w += T) {
                const uint8_t* dw = dec + w * per_word;
                uint32_t word;
                switch (a.k) {
                    case 1: word = pack_word<1>(dw); break;
                    case 2: word = pack_word<2>(dw); break;
                    case 4: word = pack_word<4>(dw); break;
                    default: word = pack_word<8>(dw); break;
                }
                if (a.bytes) reinterpret_cast<uint32_t*>(a.bytes + f * bpf)[w] = word;
                if (a.ref) errs += __popc(word ^ reinterpret_cast<const uint32_t*>(a.ref + f * bpf)[w]);
            }
        };

        if constexpr (!STAGED) {
            // one symbol per (non-unrolled) iteration: a case's register
            // indices are compile-time, and the scheduler cannot interleave
            // symbols (the next frame's symbol 0 is live in registers here)
#pragma unroll 1
            for (int w = 0; w < S; ++w) {
                switch (w) {
#define OFDM_RX_EMIT(W)                 \
    case W:                             \
        if constexpr (W < SW) {         \
            emit_group(w, y[W]);        \
        }                               \
        break;
                    OFDM_RX_EMIT(0) OFDM_RX_EMIT(1) OFDM_RX_EMIT(2) OFDM_RX_EMIT(3)
                    OFDM_RX_EMIT(4) OFDM_RX_EMIT(5) OFDM_RX_EMIT(6) OFDM_RX_EMIT(7)
#undef OFDM_RX_EMIT
                    default: break;
                }
            }
            lds_barrier();
            if (by_word)
                pack_words();
            else
                pack(0, bpf, 0);
        } else {
            const long bps = (long)D * a.k / 8;  // bytes per symbol (host checks D*k % 8 == 0)
            for (int s = 0; s < S; ++s) {
                double2 yst[RX_DPT];
#pragma unroll
                for (int i = 0; i < RX_DPT; ++i)
                    yst[i] = t + T * i < D ? a.ystage[(f * S + s) * D + t + T * i] : make_double2(0.0, 0.0);
                emit_group(s, yst);
                lds_barrier();
                if (!whole_frame_dec) {
                    pack(s * bps, (s + 1) * bps, 0);
                    lds_barrier();
                }
            }
            if (whole_frame_dec) pack(0, bpf, 0);
        }
        lds_barrier();  // dec / pil / gain / red are rewritten by the next frame
    }
    if (a.bit_errors) {
        errs = block_sum_u64<T>(errs, red);
        if (t0 == 0 && errs) atomicAdd(a.bit_errors, errs);
    }
    leave();
}

// ------------------------------------------------------------------ rx for a few frames
// rx_kernel spends one wave per frame and runs the frame's S transforms one
// after another: right for thousands of frames, slow for the drop-in's one
// frame per call (rx.cpp:211-220), whose latency is what counts there. Here a
// workgroup holds one frame and a group of T threads per symbol (whole waves,
// N >= 512), so the S transforms run side by side and the epilogue is spread
// over S*T threads. Every point, gain and decision is computed by rx_kernel's
// formulas and phys is reduced by the first T threads in rx_kernel's order,
// so the outputs equal rx_kernel's bit for bit.
template <int LOGN>
__global__ void __launch_bounds__(1024) rx_wide_kernel(RxArgs a)
{
    using FS = FftShape<LOGN>;
    constexpr int N = FS::N, T = FS::T;
    extern __shared__ double2 smem[];
    const int S = a.S, D = a.D, P = a.P;
    double2* lds_tw = smem;                                  // TwLds::SIZE
    double2* bufs = lds_tw + TwLds<LOGN>::SIZE;              // S ping-pong pairs (N + PADN)
    double2* pil = bufs + (size_t)S * (N + FS::PADN);        // S*P raw pilots
    double2* gain = pil + S * P;                             // S*P equaliser gains
    double* red = reinterpret_cast<double*>(gain + S * P);   // 16 wave sums
    uint8_t* dec = reinterpret_cast<uint8_t*>(red + 16);     // S*D decisions
    const int WT = S * T, tid = threadIdx.x, s = tid / T, t = tid - s * T;
    const long f = blockIdx.x;
    const int L = N + a.cp;
    double2 v[8];
    const double2* src = a.iq + f * a.frame_stride + a.cp + (long)s * L;  // CP strip (Frame.hpp:278-279)
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = load_nt(src + t + T * i);
    load_twiddles<LOGN>(a.tab.tw, lds_tw, tid, WT);
    int pk[RX_DPT];
#pragma unroll
    for (int i = 0; i < RX_DPT; ++i) pk[i] = a.tab.rx_pack[t + T * i];
    const int pbin = a.tab.pilot_swz[t];
    lds_barrier();
    double2* b0 = bufs + (size_t)s * (N + FS::PADN);
    const double2* res = fft_pp<LOGN, -1>(v, t, lds_tw, b0, b0 + N);
    if (t < P) pil[s * P + t] = res[pbin];
    double2 y[RX_DPT];
#pragma unroll
    for (int i = 0; i < RX_DPT; ++i) y[i] = res[pk[i] & 0xffff];
    lds_barrier();
    // phys_pilot_ampl (Frame.cpp:76-80): group 0's sum, rx_kernel's order
    double acc = 0.0;
    if (s == 0)
        for (int i = t; i < S * P; i += T) acc += hypot(pil[i].x, pil[i].y);
    acc = block_sum_lds<T>(acc, red);  // group 0's sum in group 0's threads
    // broadcast it: at T = 64 block_sum_lds is the wave's own shuffle sum, so
    // the other groups (tid >= T) hold their own zero sums
    if (tid == 0) red[15] = acc;
    lds_barrier();
    acc = red[15];
    const double phys = acc / ((double)(P * S) * a.pilot_ampl);
    for (int i = tid; i < S * P; i += WT) {  // Frame.cpp:82-93
        const int j = i % P;
        const double2 c0 = make_double2(pil[j].x / phys, pil[j].y / phys);
        const double2 cs = make_double2(pil[i].x / phys, pil[i].y / phys);
        const double2 coef = cdiv_exact(cs, c0);
        const double2 g = cdiv_exact(make_double2(1.0, 0.0), coef);
        gain[i] = make_double2(g.x / phys, g.y / phys);
    }
    lds_barrier();
    const int m = 1 << (a.k / 2);
    const double s1 = a.k == 1 ? 0.0 : 1.0 / (2.0 / (m - 1));
    const double2* chan = a.chan ? a.chan + f * a.chan_stride : nullptr;
#pragma unroll
    for (int i = 0; i < RX_DPT; ++i) {
        const int d = t + T * i;
        if (d >= D) continue;
        double2 o = cmul_exact(y[i], gain[s * P + (pk[i] >> 16)]);
        int dv;
        if (chan) {
            if (a.read_out) store_nt(a.read_out + (f * S + s) * D + d, o);
            const double2 cv = load_untracked(chan + d);
            o = a.chan_recip ? cmul_exact(o, cv) : cdiv_exact(o, cv);
            dv = decide(o, a.k, s1, m);
        } else {
            dv = decide_select(o, a.k, s1, m);
        }
        if (a.constell) store_nt(a.constell + (f * S + s) * D + d, o);
        dec[s * D + d] = (uint8_t)dv;
    }
    lds_barrier();
    const long bpf = a.bytes_per_frame;
    const bool by_word = (a.k == 1 || a.k == 2 || a.k == 4 || a.k == 8) && (bpf & 3) == 0 &&
                         ((uintptr_t)a.bytes & 3) == 0 && ((uintptr_t)a.ref & 3) == 0;
    unsigned long long errs = 0;
    if (by_word) {
        const int per_word = 32 / a.k;
        for (long w = tid; w < bpf / 4; w += WT) {
            const uint8_t* dw = dec + w * per_word;
            uint32_t word;
            switch (a.k) {
                case 1: word = pack_word<1>(dw); break;
                case 2: word = pack_word<2>(dw); break;
                case 4: word = pack_word<4>(dw); break;
                default: word = pack_word<8>(dw); break;
            }
            if (a.bytes) reinterpret_cast<uint32_t*>(a.bytes + f * bpf)[w] = word;
            if (a.ref) errs += __popc(word ^ reinterpret_cast<const uint32_t*>(a.ref + f * bpf)[w]);
        }
    } else {
        for (long jb = tid; jb < bpf; jb += WT) {
            int byte = 0;
            for (int b = 0; b < 8; ++b) {
                const long bit = jb * 8 + b;
                byte = (byte << 1) | ((dec[bit / a.k] >> (a.k - 1 - (int)(bit % a.k))) & 1);
            }
            if (a.bytes) a.bytes[f * bpf + jb] = (uint8_t)byte;
            if (a.ref) errs += __popc((unsigned)(byte ^ a.ref[f * bpf + jb]));
        }
    }
    if (a.bit_errors) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) errs += __shfl_xor(errs, o);
        if ((tid & 63) == 0 && errs) atomicAdd(a.bit_errors, errs);
    }
}

template <int LOGN>
static size_t rx_wide_shm(const RxArgs& a)
{
    using FS = FftShape<LOGN>;
    return sizeof(double2) * (TwLds<LOGN>::SIZE + (size_t)a.S * (FS::N + FS::PADN) + 2 * (size_t)a.S * a.P) +
           16 * sizeof(double) + (size_t)a.S * a.D;
}

static int num_cus();

// The few-frames form: f64 input, register-window shapes, whole-wave symbol
// groups, and fewer frames than half the compute units (beyond that the
// persistent rx_kernel's throughput wins). It takes no frames from a.queue,
// whose counters stay zero.
template <int LOGN>
static bool rx_wide_ok(const RxArgs& a)
{
    constexpr int T = FftShape<LOGN>::T;
    return LOGN >= 9 && !a.iq16 && !a.starts && !a.count && !a.ystage && a.S >= 1 &&
           (long)a.S * T <= 1024 && a.nframes <= num_cus() / 2 && rx_wide_shm<LOGN>(a) <= 160 * 1024;
}

// ------------------------------------------------------------------ stream rx, two waves per frame
// rx_kernel's stream mode (SYNC) for N = 512 (one transform = one wave),
// persistent over the located frames: each frame's channel reciprocals to
// LDS, then rx2_frame (ofdm_rx2.hpp: two waves per frame, 3 waves/SIMD).
template <bool I16>
__global__ void __launch_bounds__(128, 3) rx_stream2_kernel(RxArgs a)
{
    constexpr int LOGN = 9, N = 512, T = 64;
    extern __shared__ double2 smem[];
    const int S = a.S, D = a.D, P = a.P;
    Rx2Lds L;
    L.img = smem;                                            // 2 * N
    L.tw = smem + 2 * N;                                     // TwLds::SIZE
    L.pil = L.tw + TwLds<LOGN>::SIZE;                        // S*P raw pilots
    L.gain = L.pil + S * P;                                  // S*P equaliser gains
    L.chl = L.gain + S * P;                                  // D channel reciprocals
    L.red = reinterpret_cast<double*>(L.chl + D);            // phys
    const int tid = threadIdx.x, lane0 = tid & 63;
    const long nfr = a.count ? min(*a.count, a.nframes) : a.nframes;
    if ((long)blockIdx.x >= nfr) return;  // uniform
    load_twiddles<LOGN>(a.tab.tw, L.tw, tid, 128);
    int pk[RX_DPT];
#pragma unroll
    for (int i = 0; i < RX_DPT; ++i) pk[i] = a.tab.rx_pack[lane0 + T * i];
    const int pbin = a.tab.pilot_swz[lane0];
#pragma unroll 1
    for (long f = blockIdx.x; f < nfr; f += gridDim.x) {
        if (a.starts[f] < 0) continue;  // uniform: before the stream's first sample (the host's gather path)
        const double2* chan = a.chan + f * a.chan_stride;
        for (int d = tid; d < D; d += 128) L.chl[d] = chan[d];
        __syncthreads();  // twiddles (first frame) and the channel visible
        rx2_frame<I16>(a, f, L, reinterpret_cast<const double*>(a.corr + f * S * CORR_PER_SYM), pk, pbin);
    }
}

// ------------------------------------------------------------------ demap / map
// Modulation::demod on n points: one thread per output byte.
__global__ void demap_kernel(double2* pts, long n, int k, uint8_t* bytes, long nbytes)
{
    const long jb = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (jb >= nbytes) return;
    const int m = 1 << (k / 2);
    const double s1 = k == 1 ? 0.0 : 1.0 / (2.0 / (m - 1));
    const long g0 = (jb * 8) / k, g1 = (jb * 8 + 7) / k;
    int dv[9];
    for (long g = g0; g <= g1; ++g) {
        int dcs = 0;
        if (g < n) {
            const double2 z = pts[g];
            dcs = decide(z, k, s1, m);
            if (k != 1 && (g * k) / 8 == jb) pts[g] = clamp_point(z);
        }
        dv[g - g0] = dcs;
    }
    int byte = 0;
    for (int b = 0; b < 8; ++b) {
        const long bit = jb * 8 + b;
        const long g = bit / k;
        const int within = (int)(bit % k);
        const int bitv = g < n ? (dv[g - g0] >> (k - 1 - within)) & 1 : 0;
        byte = (byte << 1) | bitv;
    }
    bytes[jb] = (uint8_t)byte;
}

__global__ void map_kernel(const uint8_t* bytes, long nbytes, int k, const double2* table, double2* out,
                           long npts)
{
    const long g = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (g >= npts) return;
    out[g] = table[symbol_bits(bytes, nbytes, g, k)];
}

// Modulation::bit_stream_converter: output unit o = bits [o*ob, (o+1)*ob) of
// the MSB-first stream of ib-bit input units (zero past the end).
__global__ void bit_convert_kernel(const uint8_t* in, long len, int ib, int ob, uint8_t* out, long out_len)
{
    const long o = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (o >= out_len) return;
    const long total = len * ib;
    int v = 0;
    for (int b = 0; b < ob; ++b) {
        const long bit = o * ob + b;
        int x = 0;
        if (bit < total) {
            const long u = bit / ib;
            x = (in[u] >> (ib - 1 - (int)(bit - u * ib))) & 1;
        }
        v = (v << 1) | x;
    }
    out[o] = (uint8_t)v;
}

// FRAME_FORM::form_int16_to_double: element-wise int16 -> f64 (16 B out per 4 B in).
__global__ void i16_to_f64_kernel(const short2* __restrict__ in, long n, double2* __restrict__ out)
{
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const short2 v = in[i];
        out[i] = make_double2((double)v.x, (double)v.y);
    }
}

// FRAME_FORM::get_int16 on arbitrary samples: trunc(x * mult) per component.
__global__ void f64_to_i16_kernel(const double2* __restrict__ in, long n, double mult, short2* __restrict__ out)
{
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const double2 v = in[i];
        out[i] = make_short2(to_int16(v.x * mult), to_int16(v.y * mult));
    }
}

// ------------------------------------------------------------------ launchers
static int num_cus();

template <int LOGN, bool POINTS, bool NOISE, bool I16>
static hipError_t tx_launch_n(const TxArgs& a, hipStream_t st)
{
    using FS = FftShape<LOGN>;
    const size_t shm = sizeof(double2) * (FS::PADN + TwLds<LOGN>::SIZE + TX_LDS_ZERO + 1) + FS::N;  // + points + payload
    lds_opt_in((const void*)tx_kernel<LOGN, POINTS, NOISE, I16>, (int)shm);
    const long nsym = a.nframes * a.S;
    if (nsym <= 0) return hipSuccess;
    // persistent grid: enough workgroups to fill every CU several times over
    const long grid = nsym < TX_MAX_GRID ? nsym : TX_MAX_GRID;
    hipLaunchKernelGGL((tx_kernel<LOGN, POINTS, NOISE, I16>), dim3((unsigned)grid), dim3(FS::T), shm, st, a);
    return hipGetLastError();
}

template <int LOGN>
static hipError_t tx_launch_modes(const TxArgs& a, hipStream_t st)
{
    const bool noise = a.noise_scale > 0.0, i16 = a.iq16 != nullptr;
    if (a.points) {
        if (noise) return i16 ? tx_launch_n<LOGN, true, true, true>(a, st) : tx_launch_n<LOGN, true, true, false>(a, st);
        return i16 ? tx_launch_n<LOGN, true, false, true>(a, st) : tx_launch_n<LOGN, true, false, false>(a, st);
    }
    if (noise) return i16 ? tx_launch_n<LOGN, false, true, true>(a, st) : tx_launch_n<LOGN, false, true, false>(a, st);
    return i16 ? tx_launch_n<LOGN, false, false, true>(a, st) : tx_launch_n<LOGN, false, false, false>(a, st);
}

hipError_t launch_tx(int logn, const TxArgs& a, hipStream_t st)
{
    switch (logn) {
        case 6: return tx_launch_modes<6>(a, st);
        case 7: return tx_launch_modes<7>(a, st);
        case 8: return tx_launch_modes<8>(a, st);
        case 9: return tx_launch_modes<9>(a, st);
        case 10: return tx_launch_modes<10>(a, st);
        case 11: return tx_launch_modes<11>(a, st);
        case 12: return tx_launch_modes<12>(a, st);
        default: return hipErrorInvalidValue;
    }
}

// Compute units of the current device (cached per device).
static int num_cus()
{
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    if (!cache[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cache[dev] = n;
    }
    return cache[dev];
}

template <int LOGN>
static size_t rx_shm(const RxArgs& a)
{
    using FS = FftShape<LOGN>;
    return sizeof(double2) * (FS::N + FS::PADN + TwLds<LOGN>::SIZE + 2 * (size_t)a.S * a.P) + 32 * sizeof(double);
}

template <int LOGN, bool STAGED, bool I16, bool SYNC>
static hipError_t rx_launch_n(const RxArgs& a, hipStream_t st)
{
    using FS = FftShape<LOGN>;
    const size_t shm = rx_shm<LOGN>(a);
    if (shm > 160 * 1024) return hipErrorInvalidValue;
    lds_opt_in((const void*)rx_kernel<LOGN, STAGED, I16, SYNC>, 160 * 1024);
    if (a.nframes <= 0) return hipSuccess;
    // persistent: RX_WAVES_PER_CU resident waves per CU (the register
    // window's occupancy: 2 per SIMD), as far as LDS allows
    const long per_cu_w = RX_WAVES_PER_CU / (FS::T >= 64 ? FS::T / 64 : 1);
    const long per_cu_l = (long)(160 * 1024) / (long)shm;
    const long per_cu = per_cu_w < per_cu_l ? per_cu_w : per_cu_l;
    const long cap = per_cu * num_cus();
    const long grid = a.nframes < cap ? a.nframes : cap;
    hipLaunchKernelGGL((rx_kernel<LOGN, STAGED, I16, SYNC>), dim3((unsigned)grid), dim3(FS::T), shm, st, a);
    return hipGetLastError();
}

template <bool I16>
static hipError_t rx_stream2_launch(const RxArgs& a, hipStream_t st)
{
    const size_t shm = sizeof(double2) * (2 * 512 + TwLds<9>::SIZE + 2 * (size_t)a.S * a.P + a.D) + 2 * sizeof(double);
    if (shm > 160 * 1024) return hipErrorInvalidValue;
    lds_opt_in((const void*)rx_stream2_kernel<I16>, 160 * 1024);
    if (a.nframes <= 0) return hipSuccess;
    // persistent: 12 waves per CU (3 per SIMD: 155 VGPRs) = 6 workgroups, as far as LDS allows
    long per_cu = (long)(160 * 1024) / (long)shm;
    if (per_cu > 6) per_cu = 6;
    const long cap = per_cu * num_cus();
    const long grid = a.nframes < cap ? a.nframes : cap;
    hipLaunchKernelGGL(rx_stream2_kernel<I16>, dim3((unsigned)grid), dim3(128), shm, st, a);
    return hipGetLastError();
}

template <int LOGN>
static hipError_t rx_dispatch(const RxArgs& a, hipStream_t st, bool* staged)
{
    using FS = FftShape<LOGN>;
    const bool fits = a.S <= RX_SMAX && a.D <= RX_DPT * FS::T;
    if (staged) *staged = !fits;
    if (a.P > FS::T) return hipErrorInvalidValue;
    if (!fits && a.ystage == nullptr) return hipErrorInvalidValue;
    if (a.starts) {  // stream mode: register window only
        if (!fits || !a.corr) return hipErrorInvalidValue;
        if (LOGN == 9 && a.chan && a.chan_recip)
            return a.iq16 ? rx_stream2_launch<true>(a, st) : rx_stream2_launch<false>(a, st);
        return a.iq16 ? rx_launch_n<LOGN, false, true, true>(a, st) : rx_launch_n<LOGN, false, false, true>(a, st);
    }
    if (a.iq16)
        return fits ? rx_launch_n<LOGN, false, true, false>(a, st) : rx_launch_n<LOGN, true, true, false>(a, st);
    if constexpr (LOGN >= 9) {
        if (fits && a.nframes > 0 && rx_wide_ok<LOGN>(a)) {
            lds_opt_in((const void*)rx_wide_kernel<LOGN>, 160 * 1024);
            hipLaunchKernelGGL(rx_wide_kernel<LOGN>, dim3((unsigned)a.nframes), dim3(a.S * FS::T),
                               rx_wide_shm<LOGN>(a), st, a);
            return hipGetLastError();
        }
    }
    return fits ? rx_launch_n<LOGN, false, false, false>(a, st) : rx_launch_n<LOGN, true, false, false>(a, st);
}

hipError_t launch_rx(int logn, const RxArgs& a, hipStream_t st, bool* staged)
{
    switch (logn) {
        case 6: return rx_dispatch<6>(a, st, staged);
        case 7: return rx_dispatch<7>(a, st, staged);
        case 8: return rx_dispatch<8>(a, st, staged);
        case 9: return rx_dispatch<9>(a, st, staged);
        case 10: return rx_dispatch<10>(a, st, staged);
        case 11: return rx_dispatch<11>(a, st, staged);
        case 12: return rx_dispatch<12>(a, st, staged);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_demap(double2* pts, long n, int k, uint8_t* bytes, hipStream_t st)
{
    const long nbytes = (n * k + 7) / 8;
    if (nbytes <= 0) return hipSuccess;
    const int bs = 256;
    hipLaunchKernelGGL(demap_kernel, dim3((unsigned)((nbytes + bs - 1) / bs)), dim3(bs), 0, st, pts, n, k, bytes,
                       nbytes);
    return hipGetLastError();
}

hipError_t launch_map(const uint8_t* bytes, long nbytes, int k, const double2* table, double2* out, hipStream_t st)
{
    const long npts = (nbytes * 8 + k - 1) / k;
    if (npts <= 0) return hipSuccess;
    const int bs = 256;
    hipLaunchKernelGGL(map_kernel, dim3((unsigned)((npts + bs - 1) / bs)), dim3(bs), 0, st, bytes, nbytes, k, table,
                       out, npts);
    return hipGetLastError();
}

hipError_t launch_bit_convert(const uint8_t* in, long len, int ib, int ob, uint8_t* out, long out_len, hipStream_t st)
{
    if (out_len <= 0) return hipSuccess;
    const int bs = 256;
    hipLaunchKernelGGL(bit_convert_kernel, dim3((unsigned)((out_len + bs - 1) / bs)), dim3(bs), 0, st, in, len, ib, ob,
                       out, out_len);
    return hipGetLastError();
}

hipError_t launch_f64_to_i16(const double* in, long n, double mult, int16_t* out, hipStream_t st)
{
    if (n <= 0) return hipSuccess;
    long grid = (n + 255) / 256;
    if (grid > 8192) grid = 8192;
    hipLaunchKernelGGL(f64_to_i16_kernel, dim3((unsigned)grid), dim3(256), 0, st, reinterpret_cast<const double2*>(in),
                       n, mult, reinterpret_cast<short2*>(out));
    return hipGetLastError();
}

hipError_t launch_i16_to_f64(const int16_t* in, long n, double* out, hipStream_t st)
{
    if (n <= 0) return hipSuccess;
    long grid = (n + 255) / 256;
    if (grid > 8192) grid = 8192;
    hipLaunchKernelGGL(i16_to_f64_kernel, dim3((unsigned)grid), dim3(256), 0, st, reinterpret_cast<const short2*>(in), n,
                       reinterpret_cast<double2*>(out));
    return hipGetLastError();
}

// Copy by a kernel on the stream's compute queue: device memory or mapped
// page-locked host memory on either side. Small transfers between kernels
// then need no hand-off to a DMA engine and back (each such hand-off costs
// several microseconds of queue synchronisation).
__global__ void __launch_bounds__(256) copy16_kernel(uint4* dst, const uint4* src, long n16, char* dtail,
                                                     const char* stail, int ntail)
{
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n16; i += (long)gridDim.x * 256) dst[i] = src[i];
    if (blockIdx.x == 0 && threadIdx.x < ntail) dtail[threadIdx.x] = stail[threadIdx.x];
}

__global__ void __launch_bounds__(256) copy1_kernel(char* dst, const char* src, long n)
{
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) dst[i] = src[i];
}

hipError_t launch_copy(void* dst, const void* src, size_t n, hipStream_t st)
{
    if (!n) return hipSuccess;
    char* d = static_cast<char*>(dst);
    const char* s = static_cast<const char*>(src);
    if ((((uintptr_t)d | (uintptr_t)s) & 15) == 0) {
        const long n16 = (long)(n / 16);
        const long grid = std::max(1L, std::min((n16 + 255) / 256, 2048L));
        hipLaunchKernelGGL(copy16_kernel, dim3((unsigned)grid), dim3(256), 0, st, reinterpret_cast<uint4*>(d),
                           reinterpret_cast<const uint4*>(s), n16, d + n16 * 16, s + n16 * 16, (int)(n % 16));
    } else {
        const long grid = std::min(((long)n + 255) / 256, 2048L);
        hipLaunchKernelGGL(copy1_kernel, dim3((unsigned)grid), dim3(256), 0, st, d, s, (long)n);
    }
    return hipGetLastError();
}

}  // namespace ofdm
