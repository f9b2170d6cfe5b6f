// ofdm_rx2.hpp — the stream rx stage for N = 512 with two waves per frame
// (rx_kernel's stream mode, main.cpp:67-71 + FFT_FORM::read Frame.cpp:73-96
// + Modulation::demod modulation.cpp:53-87 on a located frame whose
// freq_shift / cp_freq_sinh / pr_phase_sinh corrections are two ramp numbers
// per symbol). Used by rx_stream2_kernel (ofdm_kernels.hip) and by the fused
// stream decode (ofdm_sync.hip stream_decode_kernel). Included before any
// `#pragma clang fp contract(off)`: the arithmetic is rx_kernel's.
//
// The frame's message symbols are split over two waves, wave w transforming
// s = w, w + 2, ..., so each wave holds half of the frame's register window
// (RX_SMAX/2 symbols x RX_DPT carriers = 64 VGPRs): 3 waves per SIMD (rx_kernel:
// 2 at 256 VGPRs), each frame transformed by two waves at once (one LDS
// image per wave; the transforms sync within their wave). No prefetch
// registers: the other waves of the SIMD cover the load latency. The
// operations are rx_kernel's (the phase ramp, the transform, phys in wave 0's
// lane order, the channel reciprocal multiply in chan_recip mode with
// D <= 256, the decisions) with one rounding difference: the gains are
// c0*conj(cs) / (|cs|^2 phys), one division, where rx_kernel keeps the
// reference's two Smith divisions (Frame.cpp:82-93). The stream points are
// therefore not bit-identical to batch rx; they are held to the oracle at
// 1e-9 relative with bit-exact decisions (tests/common.py
// check_stream_frames), the same bar as the rest of the sync chain.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "ofdm_dev.hpp"
#include "ofdm_fft.hpp"
#include "ofdm_internal.hpp"

namespace ofdm {

struct Rx2Lds {
    double2* img;   // 2 * 512: one transform image per wave; the S*D decisions over them afterwards
    double2* tw;    // TwLds<9>
    double2* pil;   // S*P raw pilots
    double2* gain;  // S*P equaliser gains
    double2* chl;   // D channel reciprocals: filled and visible on entry, or (chan_g) staged
                    // here from global after the transforms (then over the images, past the
                    // S*D decisions)
    double* red;    // phys
};

// The fused decode's per-frame table (LDS, written by sync_frame): per
// message symbol s, RT_PER_SYM phasors {e^{i(A+Bj)}, j < 8; e^{i8B}, e^{i16B},
// e^{i32B}; e^{iBT}}, then the channel line's two 128-carrier steps {e^{i128b},
// e^{i(128b-K)}} (K = bD/2 + b*half: the upper half's offset), then {b, aa}.
// A lane's ramp start e^{i(A + B lq)} is entry lq % 8 times the powers of
// e^{i8B} the bits of lq / 8 select: one table read and three products, not a
// sincos per lane and symbol. (Uncontracted products here: the int16 and
// f64 instantiations must round alike, so no FMA choice is left to the
// compiler.)
constexpr int RT_PER_SYM = 12;
__host__ __device__ constexpr int rt_size(int S) { return RT_PER_SYM * S + 3; }  // double2 entries

// Frame f of a.starts (message body at starts[f] + start_off); corr: its S
// ramp tables of CORR_PER_SYM phasors (ofdm_internal.hpp), or (TAB) the
// table above, from which the channel reciprocals are made too; chan_g: nullptr,
// or the frame's D channel reciprocals in global memory, requested after the
// transforms and stored to L.chl after the gains (loads issued among the
// emit's stores would wait for them). Every thread of the 128-thread
// workgroup calls it; it returns after a barrier (LDS reusable).
template <bool I16, bool TAB = false, bool PROF = false>
__device__ __forceinline__ void rx2_frame(const RxArgs& a, long f, const Rx2Lds& L, const double* corr,
                                          const int (&pk0)[RX_DPT], int pbin, const double2* chan_g = nullptr)
{
    constexpr int LOGN = 9, N = 512, T = 64, SH = RX_SMAX / 2;
    const int S = a.S, D = a.D, P = a.P;
    const int tid = threadIdx.x;
    const int m = 1 << (a.k / 2);
    const double s1 = a.k == 1 ? 0.0 : 1.0 / (2.0 / (m - 1));
    const long bpf = a.bytes_per_frame;
    const bool by_word = (a.k == 1 || a.k == 2 || a.k == 4 || a.k == 8) && (bpf & 3) == 0 &&
                         ((uintptr_t)a.bytes & 3) == 0;
    const int Lf = N + a.cp;
    uint8_t* dec = reinterpret_cast<uint8_t*>(L.img);
    // opaque per-frame copies: addresses derived from them are recomputed per
    // frame, not held live beside the register window
    int lane;
    asm volatile("v_mov_b32 %0, %1" : "=v"(lane) : "v"(tid & 63));
    int pk[RX_DPT];
#pragma unroll
    for (int i = 0; i < RX_DPT; ++i) {
        pk[i] = pk0[i];
        asm volatile("" : "+v"(pk[i]));
    }
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    double2* img = L.img + w * N;
    const long x0 = a.starts[f] + a.start_off;
    double2 y[SH][RX_DPT];
    // complex<int16> input: the wave's next symbol is requested before this
    // one's transform (8 registers), so its HBM latency hides behind it
    int rnext[8];
    auto load16 = [&](int s, int l) {
        const int* p = reinterpret_cast<const int*>(a.iq16 + x0 + (long)s * Lf + l);
#pragma unroll
        for (int i = 0; i < 8; ++i) rnext[i] = __builtin_nontemporal_load(p + T * i);
    };
    if constexpr (I16) {
        if (w < S) load16(w, lane);
    }
    // the wave's symbols, unrolled (compile-time window registers); each
    // starts from an opaque lane copy and a memory fence, so nothing of one
    // symbol (loads, LDS addresses) is hoisted and held across another
#pragma unroll
    for (int q = 0; q < SH; ++q) {
        const int s = 2 * q + w;
        if (s < S) {  // uniform
            OFDM_PHASE(rx_symbol);
            asm volatile("" ::: "memory");
            int lq;
            asm volatile("v_mov_b32 %0, %1" : "=v"(lq) : "v"(lane));
            // the ramp's start phasor first (its sincos temporaries die
            // before the sample registers are allocated)
            double2 c, wr;
            if constexpr (TAB) {
                const double2* rt = reinterpret_cast<const double2*>(corr) + s * RT_PER_SYM;
                c = rt[lq & 7];
                const int hi = lq >> 3;
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double2 p = rt[8 + k];
                    c = cmul_exact(c, (hi >> k) & 1 ? p : make_double2(1.0, 0.0));  // x (1, 0): exact
                }
                wr = rt[11];
            } else {
                // the staged decode's table (CORR_PER_SYM per symbol)
                const double2* rt = reinterpret_cast<const double2*>(corr) + s * CORR_PER_SYM;
                c = rt[0];
#pragma unroll
                for (int j = 0; j < 6; ++j) c = cmul_exact(c, (lq >> j) & 1 ? rt[1 + j] : make_double2(1.0, 0.0));
                wr = rt[CORR_PER_SYM - 1];
            }
            asm volatile("" ::: "memory");
            double2 v[8];
            const long off = x0 + (long)s * Lf + lq;
            if constexpr (I16) {
                (void)off;
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    v[i] = make_double2((double)(int)(short)(rnext[i] & 0xffff), (double)(rnext[i] >> 16));
                if (s + 2 < S) load16(s + 2, lq);  // uniform
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = load_nt(a.iq + off + T * i);
            }
            // sample m = lq + T*i of the body: *= e^{i(A + B m)}, by a
            // running product from e^{i(A + B lq)} in steps of e^{i B T}
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if constexpr (TAB) {
                    v[i] = cmul_fma(v[i], c);
                    if (i < 7) c = cmul_fma(c, wr);
                } else {
                    v[i] = cmul(v[i], c);
                    if (i < 7) c = cmul(c, wr);
                }
            }
            OFDM_PHASE(rx_symbol_fft);
            fft_block_wave<LOGN, -1>(v, lq, L.tw, img);
            OFDM_PHASE(rx_symbol_gather);
            if (lq < P) L.pil[s * P + lq] = img[pbin];
#pragma unroll
            for (int i = 0; i < RX_DPT; ++i) y[q][i] = img[pk[i] & 0xffff];
            wave_lds_sync();  // read before the next transform rewrites the image
        }
    }
    __syncthreads();  // both waves' pilots visible; the images are free
    OFDM_STOP(PROF, 3);
    OFDM_PHASE(rx_chan_line);
    // two named registers, not an array (an array held across the barriers
    // below went to scratch)
    double2 chv0 = make_double2(0.0, 0.0), chv1 = make_double2(0.0, 0.0);
    if constexpr (TAB) {
        // chan_char_lq's line (Frame.hpp:397-434): carrier tid's phase as the
        // reference computes it, carrier tid + 128's by one step of the table;
        // stored as reciprocals (conjugates of the unit phasors) for the emit
        const double2* rt = reinterpret_cast<const double2*>(corr) + RT_PER_SYM * S;
        const double b = rt[2].x, aa = rt[2].y;
        const int half = D / 2;
        double th;
        if (tid < half)
            th = add_rn(mul_rn(b, (double)tid), aa);
        else
            th = add_rn(add_rn(mul_rn(-b, (double)D) / 2, mul_rn((double)(tid - half), b)), aa);
        double sn, cs;
        sincos(th, &sn, &cs);
        const double2 h = make_double2(cs, sn);
        const double2 h2 = cmul_exact(h, tid < half && tid + 128 >= half ? rt[1] : rt[0]);
        chv0 = make_double2(h.x, -h.y);
        chv1 = make_double2(h2.x, -h2.y);
    } else if (chan_g) {  // D <= 256 = 2 x 128
        chv0 = chan_g[tid < D ? tid : 0];
        chv1 = chan_g[tid + 128 < D ? tid + 128 : 0];
    }
    // phys_pilot_ampl = sum |pilot| / (P*S*pilot_ampl)   (Frame.cpp:76-80),
    // summed by wave 0 in rx_kernel's lane order
    OFDM_PHASE(rx_phys_gains);
    if (w == 0) {
        double acc = 0.0;
        for (int i = lane; i < S * P; i += T) acc += hypot(L.pil[i].x, L.pil[i].y);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if (lane == 0) L.red[0] = acc;
    }
    __syncthreads();
    const double phys = L.red[0] / ((double)(P * S) * a.pilot_ampl);
    // out = (F/phys) / ((F[s,p]/phys) / (F[0,p]/phys)) = F * gain[s][j]   (Frame.cpp:82-93)
    // with gain = F[0,p] conj(F[s,p]) / (|F[s,p]|^2 phys): the points are
    // multiplied, not divided as the reference does (within rounding: the
    // constellation to ~1e-15 relative), phys cancelling inside coef
    for (int i = tid; i < S * P; i += 128) {
        const int j = i % P;
        const double2 c0 = L.pil[j], cs = L.pil[i];
        const double2 num = cmul_exact(c0, make_double2(cs.x, -cs.y));
        const double r = 1.0 / mul_rn(add_rn(mul_rn(cs.x, cs.x), mul_rn(cs.y, cs.y)), phys);
        L.gain[i] = make_double2(num.x * r, num.y * r);
    }
    if (TAB || chan_g) {
        if (tid < D) L.chl[tid] = chv0;
        if (tid + 128 < D) L.chl[tid + 128] = chv1;
    }
    __syncthreads();
    OFDM_STOP(PROF, 4);
    OFDM_PHASE(rx_emit);
    auto emit = [&](int s, const double2 (&yw)[RX_DPT]) {
        double2* cbase = a.constell ? a.constell + (f * S + s) * D : nullptr;
#pragma unroll
        for (int i = 0; i < RX_DPT; ++i) {
            int d = lane + T * i, gi = s * P + (pk[i] >> 16);
            asm volatile("" : "+v"(d), "+v"(gi));  // opaque: not hoisted and held
            if (d < D) {
                double2 o = cmul_exact(yw[i], L.gain[gi]);
                o = cmul_exact(o, L.chl[d]);  // main.cpp:69-71's divisor, as its reciprocal
                if (cbase) store_nt(cbase + d, o);
                dec[s * D + d] = (uint8_t)decide_select(o, a.k, s1, m);
            }
        }
    };
#pragma unroll
    for (int q = 0; q < SH; ++q) {
        const int s = 2 * q + w;
        if (s < S) emit(s, y[q]);  // uniform
    }
    __syncthreads();  // decisions visible
    OFDM_STOP(PROF, 5);
    OFDM_PHASE(rx_pack);
    if (a.bytes) {
        if (by_word) {
            const int per_word = 32 / a.k;  // decisions per output word
            for (long wd = tid; wd < bpf / 4; wd += 128) {
                const uint8_t* dw = dec + wd * per_word;
                uint32_t word;
                switch (a.k) {
                    case 1: word = pack_word<1>(dw); break;
                    case 2: word = pack_word<2>(dw); break;
                    case 4: word = pack_word<4>(dw); break;
                    default: word = pack_word<8>(dw); break;
                }
                reinterpret_cast<uint32_t*>(a.bytes + f * bpf)[wd] = word;
            }
        } else {
            for (long jb = tid; jb < bpf; jb += 128) {
                int byte = 0;
                for (int b = 0; b < 8; ++b) {
                    const long bit = jb * 8 + b;
                    const long g = bit / a.k;
                    const int within = (int)(bit % a.k);
                    byte = (byte << 1) | ((dec[g] >> (a.k - 1 - within)) & 1);
                }
                a.bytes[f * bpf + jb] = (uint8_t)byte;
            }
        }
    }
    __syncthreads();  // dec / pil / gain / chl are rewritten by the next frame
    OFDM_PHASE(rx_end);
}

}  // namespace ofdm
