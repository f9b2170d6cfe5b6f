// ofdm_stream_wide.hip — the fused stream decode for the wide geometries:
// N = 1024, 2048 and 4096 with cp = N/4 (BASELINE configs B and C at 2048 /
// 4096), whose pilot_freq_sinh form is 5 x N/4 points. The N = 512 geometry (config D)
// has its own kernel (ofdm_sync.hip stream_decode_kernel), whose one-wave
// transforms do not scale to these sizes.
//
// One workgroup of two transform groups (2 x N/8 threads) per located frame:
//   sync stage   pilot_freq_sinh (Frame.hpp:285-337): the five interleaved
//                N/4-point transforms side by side, the radix-5 combine (one
//                bin per thread: 5 x N/4 / (N/4)), fftshift, the window
//                argmax; the CP correlation sums of every symbol, one wave
//                per symbol (cp_freq_sinh, Frame.hpp:238-263); on group 0 the
//                preamble chain (freq_shift + CP correction, the body FFT,
//                pr_phase_sinh by Parseval, chan_char_lq with the parallel
//                unwrap scan; Frame.hpp:265-274,340-348,389-434); then one
//                transcendental pass for the message symbols' ramp table;
//   rx stage     the message symbols split over the groups (s = g, g + 2,
//                ...: each thread holds 4 symbols x 4 carriers of the
//                equalisation inputs, 64 VGPRs), each symbol ramped on load
//                and transformed by its group (Frame.cpp:73-96), then phys,
//                gains, channel, decisions and word packing (main.cpp:67-71,
//                modulation.cpp:53-87) — ofdm_rx2.hpp's rx2_frame with
//                workgroup transforms instead of one-wave ones.
// Nothing goes through global memory between the stages, and the frame's
// samples are read from the stream once per stage (preamble, CP pairs,
// bodies). LDS: the N-point twiddles, two N-point images (the sync stage's
// arrays live in the second one's upper half), the pilots and the ramp
// table: ~75 KB at N = 2048 (2 frames per CU, 4 waves per SIMD) and ~150 KB
// at N = 4096 (1 frame per CU). The arithmetic is the N = 512 kernel's
// (same formulas and rounding choices), so the results meet the same bar
// against the oracle: CFO and bytes exact, constellation to 1e-9.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cstdint>

#include "ofdm_dev.hpp"
#include "ofdm_fft.hpp"
#include "ofdm_sync.hpp"
#include "ofdm_syncdev.hpp"

// The sync arithmetic mirrors the reference's x86-64 build (no FMA); the FFT
// (ofdm_fft.hpp) keeps its FMAs, and the rx stage spells its products out.
#pragma clang fp contract(off)

namespace ofdm {

template <int LOGN>
struct WideGeo {
    static constexpr int N = 1 << LOGN, T = N / 8, NT = 2 * T, NW = NT / 64;
    static constexpr int CP = N / 4, L = N + CP;
    static constexpr int LOGM = LOGN - 2, M = 1 << LOGM, TM = M / 8, G = 5, S5 = G * M;
    static constexpr int LT = L / T, CT = CP / T;  // preamble samples per group-0 thread; CP share
    static constexpr int NB = LOGN - 6;            // bits of lq / 8 (lq < T)
    static constexpr int RTS = 8 + NB + 1;         // ramp table entries per message symbol
    static_assert(M == NT, "one combine bin per thread");
    static_assert(TM % 64 == 0 || 64 % TM == 0, "CFO transforms of whole waves, or several per wave");
    static_assert(LT == 10 && CT == 2, "cp = N/4");
};

// The sync stage's arrays, in the upper quarter of the two-image region
// (image 1's half: free until the rx stage), after the CFO transforms
// [0, 5N/4), dat [5N/4, 3N/2) and ph [3N/2, 13N/8 + 1). At N = 1024 they run
// ~85 entries past the images: REGION is what the kernel reserves.
template <int LOGN>
struct WideSyncLds {
    using W = WideGeo<LOGN>;
    static constexpr int TWM = 7 * W::N / 4;               // TwLds<LOGM>
    static constexpr int SPIL = TWM + TwLds<W::LOGM>::SIZE; // <= T preamble pilots
    static constexpr int RED = SPIL + W::T;                 // 32: block sums, unwrap scratch
    static constexpr int CPS = RED + 32;                    // 16: 1 + S CP sums
    static constexpr int PHI = CPS + 16;                    // 64 doubles
    static constexpr int PSI = PHI + 32;                    // 64 doubles
    static constexpr int WSUM = PSI + 32;                   // T + 2 ints
    static constexpr int END = WSUM + (W::T + 2 + 3) / 4;
    static constexpr int REGION = END > 2 * W::N ? (END + 7) / 8 * 8 : 2 * W::N;  // images + sync arrays
};

template <int LOGN, bool I16>
__global__ void __launch_bounds__(WideGeo<LOGN>::NT, 4) stream_decode_wide_kernel(CfoArgs c, StreamParamsArgs a,
                                                                                  RxArgs r)
{
    using W = WideGeo<LOGN>;
    using SL = WideSyncLds<LOGN>;
    constexpr int N = W::N, T = W::T, NT = W::NT, NW = W::NW, CP = W::CP, L = W::L, LOGM = W::LOGM, M = W::M,
                  TM = W::TM, G = W::G, S5 = W::S5, LT = W::LT, CT = W::CT, NB = W::NB, RTS = W::RTS;
    constexpr int SH = RX_SMAX / 2;
    extern __shared__ double2 smem[];
    const int S = a.S, D = a.D, P = a.P, half = D / 2, Q = 1 + S;
    double2* tw = smem;
    double2* A = tw + TwLds<LOGN>::SIZE;  // 2N: the two transform images (+ the sync arrays' overhang)
    double2* pil = A + SL::REGION;        // S*P raw pilots (rx stage)
    double2* rtg = pil + S * P;           // the ramp table (sync -> rx), then the gains
    double2* misc = rtg + (S * P > RTS * S ? S * P : RTS * S);  // {b, aa}, e^{-i phi_pr}
    double2* dat = A + 5 * M;
    double* ph = reinterpret_cast<double*>(A + 3 * N / 2);
    double2* twm = A + SL::TWM;
    double2* spil = A + SL::SPIL;
    double2* red = A + SL::RED;
    double2* cps = A + SL::CPS;
    double* phi = reinterpret_cast<double*>(A + SL::PHI);
    int* wsum = reinterpret_cast<int*>(A + SL::WSUM);

    const long f = blockIdx.x;
    if (a.count && f >= *a.count) return;  // uniform: past the speculative frame count
    if (a.starts[f] < 0) return;           // before the stream's first sample: the host's gather path
    int tid;
    asm volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"((int)threadIdx.x));
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const long x0 = a.starts[f];

    // ------------------------------------------------------------ pilot_freq_sinh
    // The CFO transforms occupy the first CFO_W waves; the others meanwhile
    // sum the CP correlations (cp_freq_sinh's raw sums need no CFO: the
    // rotation by e^{-2 pi i cfo N} is applied to the sum afterwards).
    // (TM < 64: 64/TM transforms per wave, the last wave's spare lanes run a
    // dummy transform into the free LDS past the five)
    constexpr int CFO_W = (G * TM + 63) / 64;
    static_assert(CFO_W < NW, "waves left for the CP sums");
    static_assert(CFO_W * 64 / TM * M <= 3 * N / 2, "the dummy transforms stay below ph");
    __builtin_amdgcn_s_setprio(1);  // the sync stage's chains ahead of the other frame's transforms
    {
        // the combine twiddles first (in-order vector-memory returns)
        double2 twk[G - 1];
#pragma unroll
        for (int q = 1; q < G; ++q) twk[q - 1] = c.tw_full[(long)q * tid % S5];
        const double2 w1 = c.tw_full[M], w2 = c.tw_full[2 * M];
        // transform g holds x[G*n + g], n = tt + TM*i (groups of whole waves)
        const int g = tid / TM, tt = tid % TM;
        const bool act = w < CFO_W;  // wave-uniform
        double2 v[8];
        if (act) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = src_sample_t<I16>(c.x, c.x16, x0 + (long)G * (tt + TM * i) + g);
        }
        load_twiddles<LOGN>(a.tab.tw, tw, tid, NT);
        if constexpr (TM <= 64) {
            // one wave per transform (64/TM per wave at N = 1024): each CFO
            // wave writes the whole M-point table itself (the same values at
            // the same addresses), so its own LDS wait publishes it, and the
            // transforms sync within their wave
            if (act) {
                load_twiddles<LOGM>(c.tw_sub, twm, lane, 64);
                wave_lds_sync();
                fft_block_wave<LOGM, -1>(v, tt, twm, A + g * M);
            }
        } else {
            load_twiddles<LOGM>(c.tw_sub, twm, tid, NT);
            __syncthreads();  // twiddles visible
        }
        if (!act) {
            // symbol q (0: the preamble): sum_j conj(x[qL + j]) x[qL + j + N], j < cp
            for (int q = w - CFO_W; q < Q; q += NW - CFO_W) {
                double2 acc = make_double2(0.0, 0.0);
#pragma unroll 4
                for (int j = lane; j < CP; j += 64) {
                    const long i0 = x0 + (long)q * L + j;
                    acc = cadd(acc, cconj_mul(src_sample_t<I16>(a.iq, a.iq16, i0), src_sample_t<I16>(a.iq, a.iq16, i0 + N)));
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    acc.x += __shfl_xor(acc.x, o);
                    acc.y += __shfl_xor(acc.y, o);
                }
                if (lane == 0) cps[q] = acc;
            }
        }
        if constexpr (TM <= 64)
            __syncthreads();  // the transforms and the CP sums visible
        else
            fft_block_active<LOGM, -1>(v, tt, twm, A + (act ? g : 0) * M, act);
        // X[k + M r] = sum_q W_S^{q k} W_G^{q r} F_q[k], k = tid; stored
        // fftshifted: shifted[i] = spec[(i + S/2) % S] (Frame.hpp:300-305)
        double2 tq[G];
#pragma unroll
        for (int q = 0; q < G; ++q) {
            const double2 fq = A[q * M + lds_swz(tid)];
            tq[q] = q == 0 ? fq : cmul(fq, twk[q - 1]);
        }
        __syncthreads();  // every transform read: the spectrum overwrites them
        // the 5-point DFT over q by the symmetric pairs (1, 4), (2, 3) (as
        // the N = 512 kernel: W5 = (c1, n1), W5^2 = (c2, n2))
        const double c1 = w1.x, n1 = w1.y, c2 = w2.x, n2 = w2.y;
        const double2 a0 = tq[0];
        const double2 s1 = make_double2(tq[1].x + tq[4].x, tq[1].y + tq[4].y);
        const double2 d1 = make_double2(tq[1].x - tq[4].x, tq[1].y - tq[4].y);
        const double2 s2 = make_double2(tq[2].x + tq[3].x, tq[2].y + tq[3].y);
        const double2 d2 = make_double2(tq[2].x - tq[3].x, tq[2].y - tq[3].y);
        const double2 t1 = make_double2(a0.x + c1 * s1.x + c2 * s2.x, a0.y + c1 * s1.y + c2 * s2.y);
        const double2 t2 = make_double2(a0.x + c2 * s1.x + c1 * s2.x, a0.y + c2 * s1.y + c1 * s2.y);
        const double2 u1 = make_double2(n1 * d1.x + n2 * d2.x, n1 * d1.y + n2 * d2.y);
        const double2 u2 = make_double2(n2 * d1.x - n1 * d2.x, n2 * d1.y - n1 * d2.y);
        const double2 X[G] = {make_double2(a0.x + s1.x + s2.x, a0.y + s1.y + s2.y),
                              make_double2(t1.x - u1.y, t1.y + u1.x), make_double2(t2.x - u2.y, t2.y + u2.x),
                              make_double2(t2.x + u2.y, t2.y - u2.x), make_double2(t1.x + u1.y, t1.y - u1.x)};
        double2* spec = A;
#pragma unroll
        for (int q = 0; q < G; ++q) spec[(tid + M * q + S5 / 2) % S5] = X[q];
        __syncthreads();  // spectrum visible
        // first argmax of |X| = hypot in each pilot window [borders[i],
        // borders[i+1]), i != P/2 (std::max_element), decided on |X|^2 where
        // the runner-up is certainly below (the N = 512 kernel's rule)
        constexpr int AG = 8;
        constexpr double SURE = 1.0 - 64.0 * 0x1.0p-53;
        for (int g0 = 0; g0 < c.P; g0 += NT / AG) {
            if (g0 + w * (64 / AG) >= c.P) continue;  // uniform per wave
            const int gi = g0 + tid / AG, l = tid % AG;
            const int i = gi < c.P / 2 ? gi : gi + 1;
            const bool on = gi < c.P;
            int lo = 0, hi = 0;
            if (on) {
                lo = c.borders[i];
                hi = c.borders[i + 1];
            }
            double bv = -1.0, sv = -1.0;
            int bi = INT_MAX, odd = 0;
            for (int j = lo + l; j < hi; j += AG) {
                const double2 z = spec[j];
                const double e = add_rn(mul_rn(z.x, z.x), mul_rn(z.y, z.y));
                odd |= !(e <= DBL_MAX);
                if (bv < e) {
                    sv = bv;
                    bv = e;
                    bi = j;
                } else if (sv < e) {
                    sv = e;
                }
            }
#pragma unroll
            for (int o = 1; o < AG; o <<= 1) {
                const double ov = __shfl_xor(bv, o), os = __shfl_xor(sv, o);
                const int oi = __shfl_xor(bi, o);
                odd |= __shfl_xor(odd, o);
                if (ov > bv || (ov == bv && oi < bi)) {
                    sv = fmax(bv, fmax(sv, os));
                    bv = ov;
                    bi = oi;
                } else {
                    sv = fmax(sv, fmax(ov, os));
                }
            }
            bool first_nan = false;
            if (odd || !(sv < bv * SURE)) {
                bv = -1.0;
                bi = INT_MAX;
                for (int j = lo + l; j < hi; j += AG) {
                    const double h = hypot(spec[j].x, spec[j].y);
                    if (bv < h) {
                        bv = h;
                        bi = j;
                    }
                }
#pragma unroll
                for (int o = 1; o < AG; o <<= 1) {
                    const double ov = __shfl_xor(bv, o);
                    const int oi = __shfl_xor(bi, o);
                    if (ov > bv || (ov == bv && oi < bi)) {
                        bv = ov;
                        bi = oi;
                    }
                }
                first_nan = lo < hi && isnan(hypot(spec[lo].x, spec[lo].y));
            }
            if (on && l == 0) wsum[i] = lo < hi ? (first_nan ? lo : bi) : hi;
        }
        __syncthreads();  // window maxima visible
        if (tid == 0) {
            double shift = 0.0;
            for (int i = 0; i <= c.P; ++i)
                if (i != c.P / 2) shift += wsum[i];
            shift /= c.P;
            shift -= S5 / 2;
            shift /= S5;
            red[0].x = shift;
            c.cfo_out[f] = shift;
        }
        __syncthreads();  // the CFO visible
    }
    const double cfo = red[0].x;

    {
        double rs, rc;
        sincospi(-2.0 * cfo * (double)N, &rs, &rc);
        if (tid < Q) {
            const double2 acc = cadd(make_double2(0.0, 0.0), cps[tid]);
            phi[tid] = cp_phase(acc, make_double2(rc, rs));
        }
    }
    __syncthreads();  // phases visible

    // ------------------------------------------------------------ preamble (group 0)
    const bool g0 = tid < T;  // wave-uniform
    double b, aa;
    {
        const int t = tid;
        double2 z[LT], pz = make_double2(0.0, 0.0), dz[4], mpre[4], prc[CT];
        int dbin[4];
        double2 acc = make_double2(0.0, 0.0);
        if (g0) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = t + T * u;
                dbin[u] = i < D ? a.tab.data_bin[i] : 0;
                mpre[u] = i < D ? a.mod_pre[i] : make_double2(0.0, 0.0);
            }
#pragma unroll
            for (int u = 0; u < CT; ++u) prc[u] = a.pre[t + T * u];
#pragma unroll
            for (int rr = 0; rr < LT; ++rr) z[rr] = src_sample_t<I16>(a.iq, a.iq16, x0 + t + (long)T * rr);
            const double slope0 = -2.0 * M_PI * cfo - phi[0] / N;
            double sn, cs, ws, wc;
            sincos(slope0 * (double)t, &sn, &cs);
            sincos(slope0 * (double)T, &ws, &wc);
            double2 cc = make_double2(cs, sn);
            const double2 wv = make_double2(wc, ws);
#pragma unroll
            for (int rr = 0; rr < LT; ++rr) {
                z[rr] = cmul_exact(z[rr], cc);
                if (rr < CT) acc = cadd(acc, cconj_mul(prc[rr], z[rr]));
                cc = cmul(cc, wv);
            }
        } else {
#pragma unroll
            for (int rr = 0; rr < LT; ++rr) z[rr] = make_double2(0.0, 0.0);
            // group 1, while group 0 runs the preamble chain: the message
            // symbols' ramp table. Per symbol s, {e^{i(A+Bk)}, k < 8;
            // e^{i B 8 2^m}, m < NB; e^{i B T}}, one sincos per entry; theta(m)
            // = A_s + B_s m over the CP-stripped body, freq_shift + cp_freq_sinh
            // (psi_q = phi_0 + ... + phi_{q-1}, summed in the reference's
            // order). pr_phase_sinh's common e^{-i phi_pr} is left out here and
            // applied with the channel divisor (the FFT is linear, and the
            // gains F[0,p] conj(F[s,p]) / |F[s,p]|^2 do not see a common phase)
            for (int e = t - T; e < RTS * S; e += T) {
                const int s = e / RTS, kk = e % RTS, q = 1 + s;
                double psq = 0.0;
                for (int r = 0; r < q; ++r) psq += phi[r];
                const double Aq = -2.0 * M_PI * cfo * (double)((long)q * L + CP) - (psq * L + phi[q] * CP) / N;
                const double Bq = -2.0 * M_PI * cfo - phi[q] / N;
                const double th = kk < 8 ? add_rn(Aq, mul_rn(Bq, (double)kk))
                                         : mul_rn(Bq, kk < 8 + NB ? (double)(8 << (kk - 8)) : (double)T);
                double sn, cs;
                sincos(th, &sn, &cs);
                rtg[e] = make_double2(cs, sn);
            }
        }
        // body sample t + T i of the preamble is register CT + i
        double2 vv[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) vv[i] = z[CT + i];
        fft_block_active<LOGN, -1>(vv, t, tw, A, g0);  // Z (unrotated), natural order in A[0, N)
        if (g0) {
            const int pbin = a.tab.pilot_bin[t < P ? t : 0];
            pz = t < P ? A[lds_swz(pbin)] : make_double2(0.0, 0.0);
            double2 bacc = make_double2(a.pilot_ampl * pz.x, a.pilot_ampl * pz.y);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                dz[u] = t + T * u < D ? A[lds_swz(dbin[u])] : make_double2(0.0, 0.0);
                bacc = cadd(bacc, cconj_mul(mpre[u], dz[u]));
            }
            const double isn = 1.0 / sqrt((double)N);
            acc = cadd(acc, make_double2(bacc.x * isn, bacc.y * isn));
        }
        acc = block_sum2<NT>(acc, red);  // group 1 adds zeros
        const double phr = atan2_fast(acc.y, acc.x);
        // e^{-i phr} = conj(acc) / |acc| (uniform; sincos for a zero or non-finite sum)
        double2 rot;
        const double ha = hypot(acc.x, acc.y);
        if (ha > 0.0 && ha <= DBL_MAX) {
            const double ir = 1.0 / ha;
            rot = make_double2(acc.x * ir, -acc.y * ir);
        } else {
            double rs2, rc2;
            sincos(-phr, &rs2, &rc2);
            rot = make_double2(rc2, rs2);
        }
        if (t == 0) misc[1] = rot;
        if (g0) {
            if (t < P) spil[t] = cmul_exact(pz, rot);
#pragma unroll
            for (int u = 0; u < 2; ++u)
                if (t + T * u < half) dat[t + T * u] = cmul_exact(dz[u], rot);
        }
    }
    __syncthreads();  // preamble pilots and data bins visible
    {
        double acc = 0.0;
        for (int i = tid; i < P; i += NT) acc += hypot(spil[i].x, spil[i].y);
        acc = block_sum2<NT>(make_double2(acc, 0.0), red).x;
        const double phys = acc / ((double)P * a.pilot_ampl);
        // arg((F/phys)/coef/mod_pre) (Frame.hpp:397-405): for a finite
        // positive phys arg(F conj(mod_pre)) (coef is 1 to the last bit);
        // otherwise the reference's divisions verbatim
        const bool plain = phys > 0.0 && phys <= DBL_MAX;  // uniform
        if (tid < half) {  // half <= NT (D <= 4T)
            const double2 mp = a.mod_pre[tid];
            double2 q;
            if (plain) {
                q = cmul_exact(dat[tid], make_double2(mp.x, -mp.y));
            } else {
                const int j = a.tab.data_slot[tid];
                const double2 p0 = make_double2(spil[j].x / phys, spil[j].y / phys);
                const double2 coef = cdiv_exact(p0, p0);
                const double2 fs = make_double2(dat[tid].x / phys, dat[tid].y / phys);
                q = cdiv_exact(cdiv_exact(fs, coef), mp);
            }
            ph[tid] = atan2_fast(q.y, q.x);
        }
    }
    __syncthreads();
    unwrap_scan<NT>(ph, half, reinterpret_cast<unsigned*>(red + 16));  // one-pass unwrap (Frame.hpp:407-414)
    {
        double sxy = 0.0, sy = 0.0;
        for (int i = tid; i < half; i += NT) {
            sxy += ph[i] * i;
            sy += ph[i];
        }
        const double2 sums = block_sum2<NT>(make_double2(sxy, sy), red);
        const double hn = (double)half;
        const double sx = hn * (hn - 1) / 2, sx2 = (hn - 1) * hn * (2 * hn - 1) / 6;
        b = (sums.x - sx * sums.y) / (sx2 - sx * sx);
        aa = sums.y - b * sx;
    }
    if (tid == 0) misc[0] = make_double2(b, aa);
    __syncthreads();  // the table visible; the sync arrays are free
    __builtin_amdgcn_s_setprio(0);

    // ------------------------------------------------------------ rx stage
    const int grp = __builtin_amdgcn_readfirstlane(tid / T);
    int lq;
    asm volatile("v_mov_b32 %0, %1" : "=v"(lq) : "v"(tid & (T - 1)));
    int pk[RX_DPT];
#pragma unroll
    for (int i = 0; i < RX_DPT; ++i) {
        pk[i] = r.tab.rx_pack[lq + T * i];
        asm volatile("" : "+v"(pk[i]));
    }
    const int pbin = r.tab.pilot_swz[lq];
    double2* img = A + grp * N;
    const long xb = r.starts[f] + r.start_off;
    double2 y[SH][RX_DPT];
#pragma unroll
    for (int q = 0; q < SH; ++q) {
        if (2 * q >= S) break;  // uniform over the workgroup
        const int s = 2 * q + grp;
        const bool live = s < S;  // wave-uniform
        asm volatile("" ::: "memory");
        double2 v[8];
        if (live) {
            int l2;
            asm volatile("v_mov_b32 %0, %1" : "=v"(l2) : "v"(lq));
            const double2* rts = rtg + s * RTS;
            double2 cr = rts[l2 & 7];
            const int hi = l2 >> 3;
#pragma unroll
            for (int kk = 0; kk < NB; ++kk) cr = cmul_exact(cr, (hi >> kk) & 1 ? rts[8 + kk] : make_double2(1.0, 0.0));
            const double2 wr = rts[8 + NB];
            asm volatile("" ::: "memory");
            const long off = xb + (long)s * L + l2;
            if constexpr (I16) {
                const int* p = reinterpret_cast<const int*>(r.iq16 + off);
                int rw[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) rw[i] = __builtin_nontemporal_load(p + T * i);
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    v[i] = make_double2((double)(int)(short)(rw[i] & 0xffff), (double)(rw[i] >> 16));
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = load_nt(r.iq + off + T * i);
            }
            // sample m = lq + T i of the body: *= e^{i(A + B m)}, by a running
            // product from e^{i(A + B lq)} in steps of e^{i B T}
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                v[i] = cmul_fma(v[i], cr);
                if (i < 7) cr = cmul_fma(cr, wr);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = make_double2(0.0, 0.0);
        }
        // opaque per-symbol copies of the thread index and the carrier slots:
        // the transform's pass addresses and the gathers are recomputed per
        // symbol instead of being hoisted out of the loop and spilled (the
        // loop-invariant addresses went to scratch and came back on every
        // pass's critical path)
        int tl;
        asm volatile("v_mov_b32 %0, %1" : "=v"(tl) : "v"(lq));
#pragma unroll
        for (int i = 0; i < RX_DPT; ++i) asm volatile("" : "+v"(pk[i]));
        fft_block_active<LOGN, -1>(v, tl, tw, img, live);
        if (live) {
            if (tl < P) pil[s * P + tl] = img[pbin];
#pragma unroll
            for (int i = 0; i < RX_DPT; ++i) y[q][i] = img[pk[i] & 0xffff];
        }
        lds_barrier();  // read before the next transform rewrites the images
    }
    // the channel line (chan_char_lq, Frame.hpp:415-434) at carriers tid and
    // tid + NT, as the conjugates of its unit phasors (the divisor's reciprocal)
    const double2 ba = misc[0], rot = misc[1];
    double2 chv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int d = tid + NT * u;
        double th;
        if (d < half)
            th = add_rn(mul_rn(ba.x, (double)d), ba.y);
        else
            th = add_rn(add_rn(mul_rn(-ba.x, (double)D) / 2, mul_rn((double)(d - half), ba.x)), ba.y);
        double sn, cs;
        sincos(th, &sn, &cs);
        chv[u] = cmul_exact(make_double2(cs, -sn), rot);  // and pr_phase_sinh's e^{-i phi_pr}
    }
    // phys_pilot_ampl = sum |pilot| / (P*S*pilot_ampl)   (Frame.cpp:76-80)
    double pacc = 0.0;
    for (int i = tid; i < S * P; i += NT) pacc += hypot(pil[i].x, pil[i].y);
    const double phys = block_sum2<NT>(make_double2(pacc, 0.0), red).x / ((double)(P * S) * r.pilot_ampl);
    // gain = F[0,p] conj(F[s,p]) / (|F[s,p]|^2 phys)   (Frame.cpp:82-93, ofdm_rx2.hpp)
    for (int i = tid; i < S * P; i += NT) {
        const int j = i % P;
        const double2 c0 = pil[j], cs = pil[i];
        const double2 num = cmul_exact(c0, make_double2(cs.x, -cs.y));
        const double rr = 1.0 / mul_rn(add_rn(mul_rn(cs.x, cs.x), mul_rn(cs.y, cs.y)), phys);
        rtg[i] = make_double2(num.x * rr, num.y * rr);
    }
    uint8_t* dec = reinterpret_cast<uint8_t*>(A);
    double2* chl = A + ((S * D + 15) >> 4);  // over the images, past the decisions
#pragma unroll
    for (int u = 0; u < 2; ++u)
        if (tid + NT * u < D) chl[tid + NT * u] = chv[u];
    __syncthreads();  // gains and channel visible
    const int m = 1 << (r.k / 2);
    const double s1 = r.k == 1 ? 0.0 : 1.0 / (2.0 / (m - 1));
#pragma unroll
    for (int q = 0; q < SH; ++q) {
        const int s = 2 * q + grp;
        if (s >= S) continue;  // wave-uniform
        double2* cbase = r.constell ? r.constell + (f * S + s) * D : nullptr;
#pragma unroll
        for (int i = 0; i < RX_DPT; ++i) {
            int d = lq + T * i, gi = s * P + (pk[i] >> 16);
            asm volatile("" : "+v"(d), "+v"(gi));
            if (d < D) {
                double2 o = cmul_exact(y[q][i], rtg[gi]);
                o = cmul_exact(o, chl[d]);  // main.cpp:69-71's divisor, as its reciprocal
                if (cbase) store_nt(cbase + d, o);
                dec[s * D + d] = (uint8_t)decide_select(o, r.k, s1, m);
            }
        }
    }
    __syncthreads();  // decisions visible
    if (r.bytes) {
        const long bpf = r.bytes_per_frame;
        const bool by_word = (r.k == 1 || r.k == 2 || r.k == 4 || r.k == 8) && (bpf & 3) == 0 &&
                             ((uintptr_t)r.bytes & 3) == 0;
        if (by_word) {
            const int per_word = 32 / r.k;
            for (long wd = tid; wd < bpf / 4; wd += NT) {
                const uint8_t* dw = dec + wd * per_word;
                uint32_t word;
                switch (r.k) {
                    case 1: word = pack_word<1>(dw); break;
                    case 2: word = pack_word<2>(dw); break;
                    case 4: word = pack_word<4>(dw); break;
                    default: word = pack_word<8>(dw); break;
                }
                reinterpret_cast<uint32_t*>(r.bytes + f * bpf)[wd] = word;
            }
        } else {
            for (long jb = tid; jb < bpf; jb += NT) {
                int byte = 0;
                for (int bb = 0; bb < 8; ++bb) {
                    const long bit = jb * 8 + bb;
                    const long gq = bit / r.k;
                    const int within = (int)(bit % r.k);
                    byte = (byte << 1) | ((dec[gq] >> (r.k - 1 - within)) & 1);
                }
                r.bytes[f * bpf + jb] = (uint8_t)byte;
            }
        }
    }
}

template <int LOGN>
static size_t wide_shm(const StreamParamsArgs& a)
{
    using W = WideGeo<LOGN>;
    const size_t sp = (size_t)a.S * a.P, rt = (size_t)W::RTS * a.S;
    return sizeof(double2) * (TwLds<LOGN>::SIZE + (size_t)WideSyncLds<LOGN>::REGION + sp + std::max(sp, rt) + 2);
}

template <int LOGN, bool I16>
static hipError_t wide_launch(const CfoArgs& c, const StreamParamsArgs& a, const RxArgs& r, hipStream_t st)
{
    const size_t shm = wide_shm<LOGN>(a);
    if (shm > 160 * 1024) return hipErrorNotSupported;
    lds_opt_in((const void*)stream_decode_wide_kernel<LOGN, I16>, 160 * 1024);
    hipLaunchKernelGGL((stream_decode_wide_kernel<LOGN, I16>), dim3((unsigned)a.nframes), dim3(WideGeo<LOGN>::NT),
                       shm, st, c, a, r);
    return hipGetLastError();
}

bool stream_decode_wide_fits(const StreamParamsArgs& a, int logn, int logm, int g, int cfo_p)
{
    if (logn != 10 && logn != 11 && logn != 12) return false;
    const int N = 1 << logn, T = N / 8;
    return g == 5 && logm == logn - 2 && a.cp == N / 4 && a.npr == 1 && a.S >= 1 && a.S <= RX_SMAX &&
           a.D >= 2 && a.D <= RX_DPT * T && a.P >= 1 && a.P <= T && cfo_p == a.P &&
           (logn == 10 ? wide_shm<10>(a) : logn == 11 ? wide_shm<11>(a) : wide_shm<12>(a)) <= 160 * 1024;
}

hipError_t launch_stream_decode_wide(const CfoArgs& c, const StreamParamsArgs& a, const RxArgs& r, int logn,
                                     hipStream_t st)
{
    if (a.nframes <= 0) return hipSuccess;
    if (logn == 10) return r.iq16 ? wide_launch<10, true>(c, a, r, st) : wide_launch<10, false>(c, a, r, st);
    if (logn == 11) return r.iq16 ? wide_launch<11, true>(c, a, r, st) : wide_launch<11, false>(c, a, r, st);
    if (logn == 12) return r.iq16 ? wide_launch<12, true>(c, a, r, st) : wide_launch<12, false>(c, a, r, st);
    return hipErrorNotSupported;
}

}  // namespace ofdm
