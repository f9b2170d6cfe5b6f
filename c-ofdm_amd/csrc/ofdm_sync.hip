// ofdm_sync.hip — the rx synchronisation front end as HIP kernels for gfx950
// (SURVEY.md §8f rank 1). One kernel per reference member, batched over
// frames (a located frame = one workgroup or one grid row):
//
//   t2_scan_kernel        T2SIN_FORM::find_t2sin / corr   (Frame.hpp:96-197)
//   find_preamble_kernel  PREAMBLE_FORM::find_preamble    (Frame.cpp:338-378)
//   cfo_kernel            OFDM_FORM::pilot_freq_sinh      (Frame.hpp:285-337)
//   freq_shift_kernel     OFDM_FORM::freq_shift           (Frame.hpp:340-348)
//   cp_sync_kernel        OFDM_FORM::cp_freq_sinh         (Frame.hpp:238-263)
//   phase_sync_kernel     OFDM_FORM::pr_phase_sinh        (Frame.hpp:265-274)
//   chan_kernel           PREAMBLE_FORM::chan_char_lq     (Frame.hpp:389-434)
//   stream_walk_kernel    the rx.cpp:125-221 detection walk, one walker per
//                         stream chunk (find_t2sin + find_preamble per step)
//   gather_kernel         copy located frames into a batch (rx.cpp:185-189)
//
// Arithmetic notes. The reference builds its phasor ramps by recursive
// products (p *= step); here every sample's phasor is computed directly
// (sincospi / sincos of the accumulated angle), which is within ~1e-13 of the
// recursion (whose own rounding drift is of that order) and needs no serial
// chain. The preamble detector keeps the reference's serial running-energy
// recurrence and its exact j = 0..L-1 accumulation order (no FMA), so its
// threshold decisions are bit-identical.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cstdint>

#include "ofdm_dev.hpp"
#include "ofdm_fft.hpp"
#include "ofdm_fft32.hpp"
#include "ofdm_rx2.hpp"
#include "ofdm_sync.hpp"
#include "ofdm_syncdev.hpp"

// The sync chain mirrors the reference's x86-64 arithmetic (no FMA): no
// contraction in this file (the FFT in ofdm_fft.hpp keeps its FMAs).
#pragma clang fp contract(off)

namespace ofdm {

constexpr int SYNC_THREADS = 256;

// ========================================================================
// T2 detector: G transforms of N = 2^LOGN points per workgroup.
// ========================================================================
template <int LOGN>
struct T2Geo {
    static constexpr int N = 1 << LOGN;
    static constexpr int T = N / 8;
    static constexpr int G = T >= 256 ? 1 : 256 / T;  // blocks per workgroup
    static constexpr int NT = G * T;
};

template <int LOGN>
__global__ void __launch_bounds__(T2Geo<LOGN>::NT) t2_scan_kernel(T2Args a)
{
    using Geo = T2Geo<LOGN>;
    constexpr int N = Geo::N, T = Geo::T, G = Geo::G;
    extern __shared__ double2 smem[];
    double2* lds_tw = smem;
    double2* red = lds_tw + TwLds<LOGN>::SIZE;  // G * (T/64 + 1) * 2 doubles
    double2* fftb = red + 2 * G * (T / 64 + 1);
    const int tid = threadIdx.x, g = tid / T, t = tid - g * T;
    load_twiddles<LOGN>(a.tw, lds_tw, tid, Geo::NT);
    const long b = (long)blockIdx.x * G + g;
    const bool live = b < a.nblocks;
    const double2* x = a.iq + a.start + (live ? b : 0) * N;
    double2 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = live ? x[t + T * i] : make_double2(0.0, 0.0);
    __syncthreads();
    fft_block<LOGN, -1>(v, t, lds_tw, fftb + g * N);
    // energies: total = sum |X|^2, sin = sum mask*|X|^2 (Frame.hpp:172-180)
    double tot = 0.0, sine = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int k = t + T * i;
        const double2 z = fftb[g * N + lds_swz(k)];
        const double e = z.x * z.x + z.y * z.y;
        const double m = (double)((k >= a.a1 && k <= a.b1) + (k >= a.a2 && k <= a.b2));
        tot += e;
        sine += m * e;
    }
    // reduce within the group (T lanes: a wave fragment, or T/64 waves)
    constexpr int W0 = T >= 64 ? 32 : T / 2;
#pragma unroll
    for (int o = W0; o > 0; o >>= 1) {
        tot += __shfl_xor(tot, o);
        sine += __shfl_xor(sine, o);
    }
    if constexpr (T > 64) {
        constexpr int NW = T / 64;
        if ((tid & 63) == 0) red[g * NW + (t >> 6)] = make_double2(tot, sine);
        __syncthreads();
        tot = 0.0;
        sine = 0.0;
        for (int w = 0; w < NW; ++w) {
            tot += red[g * NW + w].x;
            sine += red[g * NW + w].y;
        }
    }
    if (t == 0 && live) {
        double out = 0.0;
        if (tot != 0.0) {
            const double rel = sine / tot;
            if (!isnan(rel) && rel > a.level) {
                out = rel;
                atomicMin(a.first_scratch, (int)b);
            }
        }
        if (a.rel_out) a.rel_out[b] = out;
    }
    // the last workgroup to finish turns the minimum into find_t2sin's answer
    // and leaves the scratch {INT_MAX, 0} for the next launch (one launch per
    // call: no reset or finalize launches around it)
    __syncthreads();
    if (tid == 0) {
        __threadfence();
        if (atomicAdd(a.first_scratch + 1, 1) == (int)gridDim.x - 1) {
            const int m = atomicExch(a.first_scratch, INT_MAX);
            if (a.first_out) {
                *a.first_out = m == INT_MAX ? -1 : (int)(a.start + (long)m * N);
                __threadfence_system();  // a pinned host answer is polled by the caller
            }
            atomicExch(a.first_scratch + 1, 0);
        }
    }
}

__global__ void t2_finalize_kernel(const int* scratch, int* first_out, long start, int size)
{
    const int m = *scratch;
    *first_out = m == INT_MAX ? -1 : (int)(start + (long)m * size);
    __threadfence_system();  // as t2_scan_kernel: a pinned host answer may be polled by the caller
}

template <int LOGN>
static hipError_t t2_launch_n(const T2Args& a, hipStream_t st)
{
    using Geo = T2Geo<LOGN>;
    const size_t shm = sizeof(double2) * (TwLds<LOGN>::SIZE + 2 * Geo::G * (Geo::T / 64 + 1) + Geo::G * Geo::N);
    lds_opt_in((const void*)t2_scan_kernel<LOGN>, 160 * 1024);
    const long grid = (a.nblocks + Geo::G - 1) / Geo::G;
    hipLaunchKernelGGL(t2_scan_kernel<LOGN>, dim3((unsigned)grid), dim3(Geo::NT), shm, st, a);
    return hipGetLastError();
}

hipError_t launch_t2_scan(int logn, const T2Args& a0, int* first_out, hipStream_t st)
{
    T2Args a = a0;
    a.first_out = first_out;
    hipError_t e = hipSuccess;
    if (a.nblocks > 0) {
        switch (logn) {
            case 6: e = t2_launch_n<6>(a, st); break;
            case 7: e = t2_launch_n<7>(a, st); break;
            case 8: e = t2_launch_n<8>(a, st); break;
            case 9: e = t2_launch_n<9>(a, st); break;
            case 10: e = t2_launch_n<10>(a, st); break;
            case 11: e = t2_launch_n<11>(a, st); break;
            case 12: e = t2_launch_n<12>(a, st); break;
            default: return hipErrorInvalidValue;
        }
    }
    if (e != hipSuccess) return e;
    if (first_out && a.nblocks <= 0) {  // no block to scan: -1 (the scratch holds INT_MAX)
        hipLaunchKernelGGL(t2_finalize_kernel, dim3(1), dim3(1), 0, st, a.first_scratch, first_out, a.start,
                           1 << logn);
        e = hipGetLastError();
    }
    return e;
}

// ========================================================================
// Preamble detector: per start index, ceil(C / PRE_THREADS) workgroups each
// correlate PRE_THREADS lags (one per thread); the last of them to finish
// (a per-start counter) gathers the magnitudes and runs the screen and the
// serial energy recurrence.
// ========================================================================
constexpr int PRE_THREADS = 256;
constexpr int PRE_BATCH = 16;  // serial recurrence: energies fetched 16 at a time

__global__ void __launch_bounds__(PRE_THREADS) find_preamble_kernel(PreambleArgs a)
{
    extern __shared__ double2 smem[];
    const int L = a.L, C = a.cycles, n = C + L;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const long s = a.starts[blockIdx.y];
    const int nsplit = gridDim.x, lag0 = blockIdx.x * PRE_THREADS;
    const int cnt = nsplit == 1 ? C : min(PRE_THREADS, C - lag0);  // this workgroup's lags
    int& last_block = *reinterpret_cast<int*>(smem);  // (dynamic LDS only: the opt-in takes all 160 KB)
    double* hv = reinterpret_cast<double*>(smem + 1);  // C correlation magnitudes
    {
        double2* xs = reinterpret_cast<double2*>(hv + C);  // this slice's cnt + L samples
        for (int i = t; i < cnt + L; i += PRE_THREADS) {
            const long j = s + lag0 + i;
            xs[i] = (j >= 0 && j < a.n) ? a.iq[j] : make_double2(0.0, 0.0);
        }
        __syncthreads();
        // correlation per lag, j = 0..L-1 in order (Frame.cpp:360-363), and its magnitude
        for (int i = t; i < cnt; i += PRE_THREADS) {
            double2 e = make_double2(0.0, 0.0);
            int j = 0;
            for (; j + 8 <= L; j += 8) {  // operands a batch ahead: the chain waits on its adds alone
                double2 xv[8], cv[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    xv[k] = xs[i + j + k];
                    cv[k] = a.templ[j + k];
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) e = cadd_rn(e, cmul_exact(xv[k], cv[k]));
            }
            for (; j < L; ++j) e = cadd_rn(e, cmul_exact(xs[i + j], a.templ[j]));
            const double h = hypot(e.x, e.y);
            hv[lag0 + i] = h;
            if (nsplit > 1) a.hv_scratch[blockIdx.y * (long)C + lag0 + i] = h;
        }
        if (nsplit > 1) {
            __threadfence();  // release this slice
            __syncthreads();
            if (t == 0) last_block = atomicAdd(a.done + blockIdx.y, 1u) == (unsigned)nsplit - 1;
            __syncthreads();
            if (!last_block) return;
            __threadfence();  // acquire the other slices
            for (int i = t; i < C; i += PRE_THREADS)
                if (i - lag0 < 0 || i - lag0 >= cnt) hv[i] = a.hv_scratch[blockIdx.y * (long)C + i];
            if (t == 0) a.done[blockIdx.y] = 0u;  // zero between launches
        }
    }
    double* en = hv + C;                     // C + L sample energies
    double* ps = en + n;                     // C + L + 1 prefix sums of en (ps[k] = sum en[0..k))
    double* normv = ps + n + 1;              // C + PRE_BATCH running energies
    double* wsum = normv + C + PRE_BATCH;    // PRE_THREADS / 64 wave totals
    int* best = reinterpret_cast<int*>(wsum + PRE_THREADS / 64);
    int* lastc = best + 1;
    unsigned* cand = reinterpret_cast<unsigned*>(best + 2);  // C bits: lags whose test can pass
    __syncthreads();  // the slice's samples are dead: en overlays them
    for (int i = t; i < n; i += PRE_THREADS) {
        const long j = s + i;
        const double2 v = (j >= 0 && j < a.n) ? a.iq[j] : make_double2(0.0, 0.0);
        en[i] = add_rn(mul_rn(v.x, v.x), mul_rn(v.y, v.y));  // |x|^2 as the reference rounds it
    }
    for (int i = t; i < (C + 31) / 32; i += PRE_THREADS) cand[i] = 0u;
    if (t == 0) {
        *best = INT_MAX;
        *lastc = -1;
    }
    __syncthreads();
    if (a.cor_out) {
        // find_corr: every lag's value, so the whole serial recurrence
        if (t == 0) {
            double norm = 0.0;
            for (int i = 0; i < L; ++i) norm = add_rn(norm, en[i]);
            for (int i = 0; i < C; ++i) {
                normv[i] = norm;
                norm = add_rn(norm, en[i + L]);
                norm = sub_rn(norm, en[i]);
            }
        }
        __syncthreads();
        double* cor = a.cor_out + (long)blockIdx.y * C;
        for (int i = t; i < C; i += PRE_THREADS) {
            const double norm = normv[i];
            const double r = norm > 1.0 ? hv[i] / sqrt(norm) : 0.0;
            cor[i] = r;
            if (norm > 1.0 && r > a.level) atomicMin(best, i);
        }
        __syncthreads();
        if (t == 0 && a.idx_out) a.idx_out[blockIdx.y] = *best == INT_MAX ? -10 : (int)(s + *best);
        return;
    }
    // Certified screen. The reference's running energy norm_i (Frame.cpp:346-375:
    // +|x[i+L]|^2 - |x[i]|^2 after each test) is L - 1 + 2i rounded adds /
    // subs of nonnegative energies, each erring by at most u (2^-53) of a
    // partial sum <= P[i+L]; the window sum W_i = ps[i+L] - ps[i] of the
    // parallel prefix sum (a serial run per thread, a wave scan, the wave
    // totals: fewer than n + 2 PRE_THREADS rounded adds on any path) errs by at
    // most 2 (n + 2 PRE_THREADS) u P[n] + u |W_i|. b_i is twice their sum. A
    // lag is a candidate when its test (norm > 1, |corr| / sqrt(norm) > level;
    // sqrt and division round by u each) can pass for a norm within b_i of
    // W_i; the others certainly fail. The exact serial recurrence then runs
    // only up to the first candidate that passes (or the last candidate),
    // testing the candidates alone.
    {
        const int per = (n + PRE_THREADS - 1) / PRE_THREADS, lo = min(n, t * per), hi = min(n, lo + per);
        double run = 0.0;
        for (int i = lo; i < hi; ++i) run += en[i];
        double inc = run;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const double y = __shfl_up(inc, o);
            if (lane >= o) inc += y;
        }
        if (lane == 63) wsum[w] = inc;
        __syncthreads();
        double acc = inc - run;  // exclusive within the wave (any rounding: covered by the bound)
        for (int k = 0; k < w; ++k) acc += wsum[k];
        for (int i = lo; i < hi; ++i) {
            acc += en[i];
            ps[i + 1] = acc;
        }
        if (t == 0) ps[0] = 0.0;
        __syncthreads();
        constexpr double u = 0x1.0p-53;
        const double total = ps[n];
        const double lev2 = a.level * a.level;
        for (int i = t; i < C; i += PRE_THREADS) {
            const double wi = ps[i + L] - ps[i];
            const double b = 2.0 * u * ((L + 2.0 * i + 2.0) * ps[i + L] + 2.0 * (n + 2.0 * PRE_THREADS) * total) +
                             4.0 * u * fabs(wi);
            const double hmax = hv[i] * (1.0 + 8.0 * u);
            const bool can = !isnan(hv[i]) && wi + b > 1.0 && hmax * hmax * (1.0 + 8.0 * u) > lev2 * fmax(wi - b, 1.0);
            if (can) {
                atomicOr(&cand[i >> 5], 1u << (i & 31));
                atomicMax(lastc, i);
            }
        }
    }
    __syncthreads();
    // the reference's serial recurrence, up to the first passing candidate.
    // A batch of PRE_BATCH steps is straight-line code on energies fetched
    // ahead (the chain waits on its adds alone); a batch holding candidates
    // keeps each step's norm and tests them afterwards, in order. Steps past
    // `last` read beyond the energies (into ps) and are never tested.
    if (t == 0) {
        const int last = *lastc;
        double norm = 0.0;
        int i0 = 0;
        for (; i0 + PRE_BATCH <= L; i0 += PRE_BATCH) {
            double v[PRE_BATCH];
#pragma unroll
            for (int k = 0; k < PRE_BATCH; ++k) v[k] = en[i0 + k];
#pragma unroll
            for (int k = 0; k < PRE_BATCH; ++k) norm = add_rn(norm, v[k]);
        }
        for (; i0 < L; ++i0) norm = add_rn(norm, en[i0]);
        int found = INT_MAX;
        for (int b0 = 0; b0 <= last && found == INT_MAX; b0 += PRE_BATCH) {
            double in[PRE_BATCH], out[PRE_BATCH];
#pragma unroll
            for (int k = 0; k < PRE_BATCH; ++k) {
                in[k] = en[b0 + k + L];
                out[k] = en[b0 + k];
            }
            unsigned bits = (cand[b0 >> 5] >> (b0 & 31)) & ((1u << PRE_BATCH) - 1u);  // PRE_BATCH divides 32
            if (bits) {
#pragma unroll
                for (int k = 0; k < PRE_BATCH; ++k) {
                    normv[b0 + k] = norm;
                    norm = add_rn(norm, in[k]);
                    norm = sub_rn(norm, out[k]);
                }
                for (; bits; bits &= bits - 1u) {
                    const int i = b0 + __builtin_ctz(bits);
                    const double nv = normv[i];
                    if (nv > 1.0 && hv[i] / sqrt(nv) > a.level) {
                        found = i;
                        break;
                    }
                }
            } else {
#pragma unroll
                for (int k = 0; k < PRE_BATCH; ++k) {
                    norm = add_rn(norm, in[k]);
                    norm = sub_rn(norm, out[k]);
                }
            }
        }
        *best = found;
    }
    __syncthreads();
    if (t == 0 && a.idx_out) a.idx_out[blockIdx.y] = *best == INT_MAX ? -10 : (int)(s + *best);
}

hipError_t launch_find_preamble(const PreambleArgs& a, hipStream_t st)
{
    if (a.nstarts <= 0) return hipSuccess;
    // split over workgroups when the caller provides the scratch, else one
    // workgroup per start index
    const int nsplit = a.hv_scratch && a.done ? preamble_splits(a.cycles) : 1;
    if (a.nstarts > 65535) return hipErrorInvalidValue;
    const size_t C = (size_t)a.cycles, nn = C + a.L;
    const size_t corr = sizeof(double) * C + sizeof(double2) * ((nsplit > 1 ? std::min<size_t>(C, PRE_THREADS) : C) + a.L);
    const size_t tail = sizeof(double) * (C + nn + nn + 1 + C + PRE_BATCH + PRE_THREADS / 64) + sizeof(int) * 2 +
                        sizeof(unsigned) * ((C + 31) / 32) + 64;
    const size_t shm = sizeof(double2) + std::max(corr, tail);
    if (shm > 160 * 1024) return hipErrorInvalidValue;
    lds_opt_in((const void*)find_preamble_kernel, 160 * 1024);
    hipLaunchKernelGGL(find_preamble_kernel, dim3((unsigned)nsplit, (unsigned)a.nstarts), dim3(PRE_THREADS), shm, st, a);
    return hipGetLastError();
}

int preamble_splits(int cycles) { return (cycles + PRE_THREADS - 1) / PRE_THREADS; }

// ========================================================================
// pilot_freq_sinh: FFT of the whole form (M or 5*M points, M = 2^LOGM) as G
// interleaved sub-FFTs of M points + a radix-5 combine, |.|, fftshift, first
// argmax per pilot window.
// ========================================================================
template <int LOGM, int G>
__global__ void __launch_bounds__(G * (1 << LOGM) / 8) cfo_kernel(CfoArgs a)
{
    constexpr int M = 1 << LOGM, T = M / 8, NT = G * T, S = G * M;
    extern __shared__ double2 smem[];
    double2* lds_tw = smem;
    double2* fftb = lds_tw + TwLds<LOGM>::SIZE;          // G * M
    double* amp = reinterpret_cast<double*>(fftb + S);    // S magnitudes (fftshifted)
    int* wsum = reinterpret_cast<int*>(amp + S);          // per-window argmax
    const int tid = threadIdx.x, g = tid / T, t = tid - g * T;
    const long f = blockIdx.x;
    if (a.count && f >= *a.count) return;  // uniform: past the speculative frame count
    // a stream frame whose preamble starts before the stream's first sample
    // (rx.cpp decodes it from its ring's zero header) is decoded by the
    // host's gather path, which reads those samples as zero
    if (a.starts && a.starts[f] < 0) return;
    const long x0 = a.starts ? a.starts[f] : f * a.frame_stride;
    // the combine twiddles are requested before the samples (in-order
    // vector-memory returns: issued after them they would wait behind every
    // stream load in flight on the CU; cfo 93 -> 80 us on config 4)
    constexpr int KM = (M + NT - 1) / NT;
    double2 twk[KM][G > 1 ? G - 1 : 1], twg[G > 1 ? G - 1 : 1];
    if constexpr (G > 1) {
#pragma unroll
        for (int u = 0; u < KM; ++u)
#pragma unroll
            for (int q = 1; q < G; ++q) {
                const int k = tid + NT * u;
                twk[u][q - 1] = k < M ? a.tw_full[(long)q * k % S] : make_double2(1.0, 0.0);
            }
#pragma unroll
        for (int q = 1; q < G; ++q) twg[q - 1] = a.tw_full[(long)q * M];
    }
    load_twiddles<LOGM>(a.tw_sub, lds_tw, tid, NT);
    double2 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // decimated input x[G*n + g]
        const long j = x0 + (long)G * (t + T * i) + g;
        if (a.x16) {
            const short2 w = a.x16[j];
            v[i] = make_double2((double)w.x, (double)w.y);
        } else {
            v[i] = a.x[j];
        }
    }
    __syncthreads();
    fft_block<LOGM, -1>(v, t, lds_tw, fftb + g * M);
    // X[k + M*r] = sum_q W_S^{q k} W_G^{q r} F_q[k]; amp stored fftshifted:
    // shifted[i] = spec[(i + S/2) % S]  (Frame.hpp:300-305)
    const int half = S / 2;
#pragma unroll
    for (int u = 0; u < KM; ++u) {
        const int k = tid + NT * u;
        if (k >= M) break;
        if constexpr (G == 1) {
            const double2 z = fftb[lds_swz(k)];
            amp[(k + half) % S] = hypot(z.x, z.y);
        } else {
            double2 tq[G];
#pragma unroll
            for (int q = 0; q < G; ++q) {
                const double2 fq = fftb[q * M + lds_swz(k)];
                tq[q] = q == 0 ? fq : cmul(fq, twk[u][q - 1]);
            }
#pragma unroll
            for (int r = 0; r < G; ++r) {
                double2 acc = tq[0];
#pragma unroll
                for (int q = 1; q < G; ++q)
                    acc = cadd(acc, cmul(tq[q], (q * r) % G ? twg[(q * r) % G - 1] : make_double2(1.0, 0.0)));
                const int idx = k + M * r;
                amp[(idx + half) % S] = hypot(acc.x, acc.y);
            }
        }
    }
    __syncthreads();
    // first argmax inside each pilot window [borders[i], borders[i+1]), i != P/2
    // (std::max_element: strictly-greater keeps the first maximum). A group
    // of AG lanes per window: each lane the first maximum of its strided
    // share, then a butterfly keeping the larger value, the lower index on
    // ties, which is the window's first maximum.
    constexpr int AG = 8;
    for (int i0 = 0; i0 <= a.P; i0 += NT / AG) {
        const int i = i0 + tid / AG, l = tid % AG;
        const bool act = tid < (NT / AG) * AG && i <= a.P;
        int lo = 0, hi = 0;
        if (act) {
            lo = a.borders[i];
            hi = a.borders[i + 1];
        }
        double bv = -1.0;  // below every magnitude
        int bi = INT_MAX;
        for (int j = lo + l; j < hi; j += AG)
            if (bv < amp[j]) {
                bv = amp[j];
                bi = j;
            }
#pragma unroll
        for (int o = 1; o < AG; o <<= 1) {  // AG-lane groups are aligned within a wave
            const double ov = __shfl_xor(bv, o);
            const int oi = __shfl_xor(bi, o);
            if (ov > bv || (ov == bv && oi < bi)) {
                bv = ov;
                bi = oi;
            }
        }
        // max_element of an empty range = end; a NaN first element is kept
        // (nothing compares greater than it)
        if (act && l == 0) wsum[i] = lo < hi ? (isnan(amp[lo]) ? lo : bi) : hi;
    }
    __syncthreads();
    if (tid == 0) {
        double shift = 0.0;
        for (int i = 0; i <= a.P; ++i)
            if (i != a.P / 2) shift += wsum[i];
        shift /= a.P;
        shift -= S / 2;
        shift /= S;
        a.cfo_out[f] = shift;
        if (a.host_out) __threadfence_system();  // a pinned host word its caller polls
    }
}

template <int LOGM, int G>
static hipError_t cfo_launch_n(const CfoArgs& a, hipStream_t st)
{
    constexpr int M = 1 << LOGM, NT = G * M / 8;
    static_assert(NT <= 1024, "cfo workgroup too large");
    const size_t shm = sizeof(double2) * (TwLds<LOGM>::SIZE + (size_t)G * M) + sizeof(double) * G * M +
                       sizeof(int) * (a.P + 2) + 16;
    if (shm > 160 * 1024) return hipErrorInvalidValue;
    lds_opt_in((const void*)cfo_kernel<LOGM, G>, 160 * 1024);
    hipLaunchKernelGGL((cfo_kernel<LOGM, G>), dim3((unsigned)a.nframes), dim3(NT), shm, st, a);
    return hipGetLastError();
}

hipError_t launch_cfo(int logm, int g, const CfoArgs& a, hipStream_t st)
{
    if (a.nframes <= 0) return hipSuccess;
    if (g == 1) {
        switch (logm) {
            case 6: return cfo_launch_n<6, 1>(a, st);
            case 7: return cfo_launch_n<7, 1>(a, st);
            case 8: return cfo_launch_n<8, 1>(a, st);
            case 9: return cfo_launch_n<9, 1>(a, st);
            case 10: return cfo_launch_n<10, 1>(a, st);
            case 11: return cfo_launch_n<11, 1>(a, st);
            case 12: return cfo_launch_n<12, 1>(a, st);
            default: return hipErrorInvalidValue;
        }
    }
    if (g == 5) {
        switch (logm) {
            case 6: return cfo_launch_n<6, 5>(a, st);
            case 7: return cfo_launch_n<7, 5>(a, st);
            case 8: return cfo_launch_n<8, 5>(a, st);
            case 9: return cfo_launch_n<9, 5>(a, st);
            case 10: return cfo_launch_n<10, 5>(a, st);
            default: return hipErrorInvalidValue;
        }
    }
    return hipErrorInvalidValue;
}

// ========================================================================
// freq_shift: x[n] *= exp(-2 pi i cfo n)
// ========================================================================
// The per-sample arithmetic of freq_shift / cp_freq_sinh / pr_phase_sinh,
// rounded as the reference's g++ complex<double> code (no FMA): shared by the
// three single-stage kernels and sync_chain_kernel, which equal each other
// bit for bit.
__device__ __forceinline__ double2 shift_sample(double2 v, double cfo, long n)
{
    double sn, cs;
    sincospi(-2.0 * cfo * (double)n, &sn, &cs);
    return cmul_exact(v, make_double2(cs, sn));
}

__device__ __forceinline__ double2 cp_rotate(double2 v, double psi, double phi, int L, int j, int N)
{
    const double th = -add_rn(mul_rn(psi, (double)L), mul_rn(phi, (double)j)) / N;
    double sn, cs;
    sincos(th, &sn, &cs);
    return cmul_exact(v, make_double2(cs, sn));
}

__global__ void __launch_bounds__(SYNC_THREADS) freq_shift_kernel(ShiftArgs a)
{
    const long f = blockIdx.y;
    const double cfo = a.cfo[f];
    double2* x = a.x + f * a.frame_stride;
    for (long n = blockIdx.x * (long)SYNC_THREADS + threadIdx.x; n < a.nsamples;
         n += (long)gridDim.x * SYNC_THREADS)
        x[n] = shift_sample(x[n], cfo, n);
}

hipError_t launch_freq_shift(const ShiftArgs& a, hipStream_t st)
{
    if (a.nframes <= 0 || a.nsamples <= 0) return hipSuccess;
    long gx = (a.nsamples + SYNC_THREADS * 4 - 1) / (SYNC_THREADS * 4);
    if (gx > 64) gx = 64;
    hipLaunchKernelGGL(freq_shift_kernel, dim3((unsigned)gx, (unsigned)a.nframes), dim3(SYNC_THREADS), 0, st, a);
    return hipGetLastError();
}

// ========================================================================
// cp_freq_sinh: phi_s = arg sum_{j<cp} conj(x[sL+j]) x[sL+j+N];
// sample (s, j) *= exp(-i (sum_{q<s} phi_q * L + phi_s * j) / N)
// ========================================================================
// One 1024-thread workgroup per frame: wave w correlates the CP of symbols
// w, w + 16, ... (wave-level sums, no workgroup barrier per symbol), then the
// phase prefix once, then the correction of every sample.
constexpr int CP_THREADS = 1024;

__global__ void __launch_bounds__(CP_THREADS) cp_sync_kernel(CpArgs a)
{
    __shared__ double phi[64];
    __shared__ double psi[64];
    const long f = blockIdx.x;
    double2* x = a.x + f * a.frame_stride;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, L = a.N + a.cp;
    for (int s = w; s < a.nsym; s += CP_THREADS / 64) {
        double2 acc = make_double2(0.0, 0.0);
        for (int j = lane; j < a.cp; j += 64) acc = cadd(acc, cconj_mul(x[(long)s * L + j], x[(long)s * L + j + a.N]));
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            acc.x += __shfl_xor(acc.x, o);
            acc.y += __shfl_xor(acc.y, o);
        }
        if (lane == 0) phi[s] = atan2(acc.y, acc.x);
    }
    __syncthreads();
    if (t == 0) {  // psi_s = phi_0 + ... + phi_{s-1}, in that order (Frame.hpp:257-260)
        double p = 0.0;
        for (int q = 0; q < a.nsym; ++q) {
            psi[q] = p;
            p += phi[q];
        }
    }
    __syncthreads();
    const long total = (long)a.nsym * L;
    for (long n = t; n < total; n += CP_THREADS) {
        const int s = (int)(n / L), j = (int)(n - (long)s * L);
        x[n] = cp_rotate(x[n], psi[s], phi[s], L, j, a.N);
    }
}

hipError_t launch_cp_sync(const CpArgs& a, hipStream_t st)
{
    if (a.nframes <= 0) return hipSuccess;
    if (a.nsym > 64) return hipErrorInvalidValue;
    hipLaunchKernelGGL(cp_sync_kernel, dim3((unsigned)a.nframes), dim3(CP_THREADS), 0, st, a);
    return hipGetLastError();
}

// ========================================================================
// pr_phase_sinh: phi = arg sum_i conj(pr_i) x_i; x *= exp(-i phi)
// ========================================================================
__global__ void __launch_bounds__(SYNC_THREADS) phase_sync_kernel(PhaseArgs a)
{
    __shared__ double2 red[SYNC_THREADS / 64];
    __shared__ double2 rot;
    const long f = blockIdx.x;
    double2* x = a.x + f * a.frame_stride;
    const int t = threadIdx.x;
    double2 acc = make_double2(0.0, 0.0);
    for (long i = t; i < a.pr_len; i += SYNC_THREADS) acc = cadd(acc, cconj_mul(a.pr[i], x[i]));
    acc = block_sum2<SYNC_THREADS>(acc, red);
    if (t == 0) {
        double sn, cs;
        sincos(-atan2(acc.y, acc.x), &sn, &cs);
        rot = make_double2(cs, sn);
    }
    __syncthreads();
    const double2 r = rot;
    for (long n = t; n < a.nsamples; n += SYNC_THREADS) x[n] = cmul_exact(x[n], r);
}

hipError_t launch_phase_sync(const PhaseArgs& a, hipStream_t st)
{
    if (a.nframes <= 0) return hipSuccess;
    hipLaunchKernelGGL(phase_sync_kernel, dim3((unsigned)a.nframes), dim3(SYNC_THREADS), 0, st, a);
    return hipGetLastError();
}

// ========================================================================
// The three stages above (pilot_freq_sinh's shift, cp_freq_sinh,
// pr_phase_sinh: main.cpp:61-63) in one workgroup per form, the form held in
// LDS between them. Every sample, sum and angle is computed as in
// freq_shift_kernel / cp_sync_kernel / phase_sync_kernel (the phase
// correlation by 256 threads with block_sum2's order), so x and the stage
// copies equal the three launches bit for bit.
// ========================================================================
constexpr int CHAIN_THREADS = 1024;
constexpr long CHAIN_LDS = 158 * 1024;  // dynamic part: 160 KB less the kernel's static LDS

bool sync_chain_fits(long nsamples) { return nsamples > 0 && nsamples * (long)sizeof(double2) <= CHAIN_LDS; }

// IN_LDS = false (a form beyond 158 KB): the same steps on x itself, which
// the workgroup's own barriers order (one workgroup per form).
template <bool IN_LDS>
__global__ void __launch_bounds__(CHAIN_THREADS) sync_chain_kernel(SyncChainArgs a)
{
    extern __shared__ double2 smem_chain[];
    __shared__ double phi[64];
    __shared__ double psi[64];
    __shared__ double2 red[SYNC_THREADS / 64];
    __shared__ double2 rot;
    const long f = blockIdx.x;
    double2* x = a.x + f * a.frame_stride;
    double2* xs = IN_LDS ? smem_chain : x;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, L = a.N + a.cp;
    const long ns = a.nsamples, off = f * a.out_stride;
    const double cfo = a.cfo[f];
    for (long n = t; n < ns; n += CHAIN_THREADS) {
        const double2 v = shift_sample(x[n], cfo, n);
        xs[n] = v;
        if (a.out[0]) a.out[0][off + n] = v;
    }
    __syncthreads();
    for (int s = w; s < a.nsym; s += CHAIN_THREADS / 64) {
        double2 acc = make_double2(0.0, 0.0);
        for (int j = lane; j < a.cp; j += 64) acc = cadd(acc, cconj_mul(xs[s * L + j], xs[s * L + j + a.N]));
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            acc.x += __shfl_xor(acc.x, o);
            acc.y += __shfl_xor(acc.y, o);
        }
        if (lane == 0) phi[s] = atan2(acc.y, acc.x);
    }
    __syncthreads();
    if (t == 0) {
        double p = 0.0;
        for (int q = 0; q < a.nsym; ++q) {
            psi[q] = p;
            p += phi[q];
        }
    }
    __syncthreads();
    const long total = (long)a.nsym * L;
    for (long n = t; n < ns; n += CHAIN_THREADS) {
        double2 v = xs[n];
        if (n < total) {
            const int s = (int)(n / L), j = (int)(n - (long)s * L);
            v = cp_rotate(v, psi[s], phi[s], L, j, a.N);
            xs[n] = v;
        }
        if (a.out[1]) a.out[1][off + n] = v;
    }
    __syncthreads();
    // phase_sync_kernel's correlation: threads 0..255, stride 256, then the
    // four wave sums added in wave order from 0.0 (block_sum2<256>)
    if (t < SYNC_THREADS) {
        double2 acc = make_double2(0.0, 0.0);
        for (long i = t; i < a.pr_len; i += SYNC_THREADS) acc = cadd(acc, cconj_mul(a.pr[i], xs[i]));
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            acc.x += __shfl_xor(acc.x, o);
            acc.y += __shfl_xor(acc.y, o);
        }
        if (lane == 0) red[w] = acc;
    }
    __syncthreads();
    if (t == 0) {
        double2 s = make_double2(0.0, 0.0);
#pragma unroll
        for (int i = 0; i < SYNC_THREADS / 64; ++i) s = cadd(s, red[i]);
        double sn, cs;
        sincos(-atan2(s.y, s.x), &sn, &cs);
        rot = make_double2(cs, sn);
    }
    __syncthreads();
    const double2 r = rot;
    for (long n = t; n < ns; n += CHAIN_THREADS) {
        const double2 v = cmul_exact(xs[n], r);
        x[n] = v;
        if (a.out[2]) a.out[2][off + n] = v;
    }
}

hipError_t launch_sync_chain(const SyncChainArgs& a, hipStream_t st)
{
    if (a.nframes <= 0) return hipSuccess;
    if (a.nsym > 64 || a.nsamples <= 0 || a.pr_len > a.nsamples || (long)a.nsym * (a.N + a.cp) > a.nsamples ||
        a.nframes > 0x7fffffffL)
        return hipErrorInvalidValue;
    if (sync_chain_fits(a.nsamples)) {
        lds_opt_in((const void*)sync_chain_kernel<true>, (int)CHAIN_LDS);
        hipLaunchKernelGGL(sync_chain_kernel<true>, dim3((unsigned)a.nframes), dim3(CHAIN_THREADS),
                           (size_t)a.nsamples * sizeof(double2), st, a);
    } else {
        hipLaunchKernelGGL(sync_chain_kernel<false>, dim3((unsigned)a.nframes), dim3(CHAIN_THREADS), 0, st, a);
    }
    return hipGetLastError();
}

// ========================================================================
// chan_char_lq: FFT_FORM::read of the preamble form (phys over its pilots,
// coef = F0/F0), phase of pr/mod_preamble over the first D/2 carriers,
// one-pass unwrap, least squares on raw sums, unit phasors.
// ========================================================================
template <int LOGN>
__global__ void __launch_bounds__((1 << LOGN) / 8) chan_kernel(ChanArgs a)
{
    using FS = FftShape<LOGN>;
    constexpr int N = FS::N, T = FS::T;
    extern __shared__ double2 smem[];
    double2* lds_tw = smem;
    double2* fftb = lds_tw + TwLds<LOGN>::SIZE;   // N
    double2* pil = fftb + N;                       // npr * P
    double2* dat = pil + a.npr * a.P;              // D/2 raw bins of symbol 0
    double* ph = reinterpret_cast<double*>(dat + a.D / 2 + 1);
    double* red = ph + a.D / 2 + 2;
    const int t = threadIdx.x;
    const long f = blockIdx.x;
    const double2* x = a.x + f * a.frame_stride;
    const int L = N + a.cp, half = a.D / 2;
    load_twiddles<LOGN>(a.tab.tw, lds_tw, t, T);
    __syncthreads();
    for (int s = 0; s < a.npr; ++s) {
        double2 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = x[(long)s * L + a.cp + t + T * i];
        fft_block<LOGN, -1>(v, t, lds_tw, fftb);
        for (int j = t; j < a.P; j += T) pil[s * a.P + j] = fftb[lds_swz(a.tab.pilot_bin[j])];
        if (s == 0)
            for (int i = t; i < half; i += T) dat[i] = fftb[lds_swz(a.tab.data_bin[i])];
        __syncthreads();
    }
    // phys (Frame.cpp:76-80), parallel sum
    double acc = 0.0;
    for (int i = t; i < a.npr * a.P; i += T) acc += hypot(pil[i].x, pil[i].y);
    {
        double2 r2 = block_sum2<T>(make_double2(acc, 0.0), reinterpret_cast<double2*>(red));
        acc = r2.x;
    }
    const double phys = acc / ((double)(a.P * a.npr) * a.pilot_ampl);
    // pr[i] = (F/phys) / coef, coef = (F[0,p]/phys)/(F[0,p]/phys); phase of pr/mod
    for (int i = t; i < half; i += T) {
        const int j = a.tab.data_slot[i];
        const double2 p0 = make_double2(pil[j].x / phys, pil[j].y / phys);
        const double2 coef = cdiv_exact(p0, p0);
        const double2 fs = make_double2(dat[i].x / phys, dat[i].y / phys);
        const double2 q = cdiv_exact(cdiv_exact(fs, coef), a.mod_pre[i]);
        ph[i] = atan2(q.y, q.x);
    }
    __syncthreads();
    unwrap_scan<T>(ph, half, reinterpret_cast<unsigned*>(red) + 96);  // one-pass unwrap (Frame.hpp:407-414)
    double sxy = 0.0, sy = 0.0;
    for (int i = t; i < half; i += T) {
        sxy += ph[i] * i;
        sy += ph[i];
    }
    const double2 sums = block_sum2<T>(make_double2(sxy, sy), reinterpret_cast<double2*>(red) + 16);
    // integer sums are exact in any order
    const double hn = (double)half;
    const double sx = hn * (hn - 1) / 2, sx2 = (hn - 1) * hn * (2 * hn - 1) / 6;
    const double b = (sums.x - sx * sums.y) / (sx2 - sx * sx);
    const double aa = sums.y - b * sx;
    double2* chan = a.chan_out + f * a.chan_stride;
    for (int i = t; i < a.D; i += T) {
        double th;
        if (i < half)
            th = add_rn(mul_rn(b, (double)i), aa);
        else
            th = add_rn(add_rn(mul_rn(-b, (double)a.D) / 2, mul_rn((double)(i - half), b)), aa);
        double sn, cs;
        sincos(th, &sn, &cs);
        chan[i] = make_double2(cs, sn);
    }
}

template <int LOGN>
static hipError_t chan_launch_n(const ChanArgs& a, hipStream_t st)
{
    using FS = FftShape<LOGN>;
    const size_t shm = sizeof(double2) * (TwLds<LOGN>::SIZE + FS::N + (size_t)a.npr * a.P + a.D / 2 + 1) +
                       sizeof(double) * (a.D / 2 + 2) + sizeof(double2) * 40;
    if (shm > 160 * 1024) return hipErrorInvalidValue;
    lds_opt_in((const void*)chan_kernel<LOGN>, 160 * 1024);
    hipLaunchKernelGGL(chan_kernel<LOGN>, dim3((unsigned)a.nframes), dim3(FS::T), shm, st, a);
    return hipGetLastError();
}

hipError_t launch_chan(int logn, const ChanArgs& a, hipStream_t st)
{
    if (a.nframes <= 0) return hipSuccess;
    switch (logn) {
        case 6: return chan_launch_n<6>(a, st);
        case 7: return chan_launch_n<7>(a, st);
        case 8: return chan_launch_n<8>(a, st);
        case 9: return chan_launch_n<9>(a, st);
        case 10: return chan_launch_n<10>(a, st);
        case 11: return chan_launch_n<11>(a, st);
        case 12: return chan_launch_n<12>(a, st);
        default: return hipErrorInvalidValue;
    }
}

// ========================================================================
// Fused stream decode, stage 2: main.cpp:61-65 on a located frame, read
// straight from the stream (rx.cpp:185-189 copies the frame out first; here
// nothing is copied and nothing corrected is written back).
//   freq_shift     x[n] *= e^{-2 pi i cfo n}                (Frame.hpp:340-348)
//   cp_freq_sinh   phi_q = arg sum_{j<cp} conj(y[qL+j]) y[qL+j+N] of the
//                  shifted y; sample (q, j) *= e^{-i (psi_q L + phi_q j)/N},
//                  psi_q = sum_{r<q} phi_r                  (Frame.hpp:238-263)
//   pr_phase_sinh  phi_pr = arg sum_{i<pre} conj(pr_i) z_i; x *= e^{-i phi_pr}
//                                                           (Frame.hpp:265-274)
//   chan_char_lq   on the corrected preamble                (Frame.hpp:389-434)
// conj(y_a) y_{a+N} = e^{-2 pi i cfo N} conj(x_a) x_{a+N}, so phi_q comes
// from raw samples and one rotation of the sum. Every correction is one
// phasor e^{i theta(q, j)}, theta linear in j within a symbol; the message
// symbols' (A_s, B_s) are handed to the rx kernel (stream mode).
// ========================================================================

template <int LOGN>
__global__ void __launch_bounds__((1 << LOGN) / 8, 3) stream_params_kernel(StreamParamsArgs a)
{
    // one preamble symbol (npr == 1) whose form length L is a multiple of T
    // (host-checked): thread t holds the preamble form samples t + T*r, r < L/T
    using FS = FftShape<LOGN>;
    constexpr int N = FS::N, T = FS::T, RMAX = 16;
    extern __shared__ double2 smem[];
    double2* lds_tw = smem;
    double2* fftb = lds_tw + TwLds<LOGN>::SIZE;   // N
    double2* pil = fftb + N;                       // P
    double2* dat = pil + a.P;                      // D/2 raw bins of the preamble
    constexpr int NWV = T >= 64 ? T / 64 : 1;      // waves
    const int ndat = (a.D / 2 + 1) > (1 + a.S) * NWV ? (a.D / 2 + 1) : (1 + a.S) * NWV;
    double* ph = reinterpret_cast<double*>(dat + ndat);
    double2* red = reinterpret_cast<double2*>(ph + a.D / 2 + 2);  // 32 entries
    double* phi = reinterpret_cast<double*>(red + 32);            // Q symbol phases
    double* psi = phi + 64;                                       // Q prefix sums
    double& phpr = psi[64];  // (dynamic LDS only: the 160 KiB attribute leaves no room for static)
    const int t = threadIdx.x;
    const long f = blockIdx.x;
    if (a.count && f >= *a.count) return;  // uniform: past the speculative frame count
    if (a.starts[f] < 0) return;           // before the stream's first sample: the gather path's
    const long x0 = a.starts[f];
    const double cfo = a.cfo[f];
    const int L = N + a.cp, half = a.D / 2, Q = 1 + a.S, LT = L / T, CT = a.cp / T;

    // The per-thread table entries are requested before the stream samples:
    // vector-memory returns are in order, so a table load issued later waits
    // behind every stream load in flight on the CU. (Doing the same for the
    // preamble template, through LDS, costs more occupancy than it saves:
    // params 230 -> 263 us.)
    // data carrier i = t + T*u (D <= 4T, host-checked): its bin and BPSK
    // preamble point; the slot for the first half (chan_char_lq); the CP part
    // of the preamble template (pr_phase_sinh's time-domain share)
    int dbin[4], dslot[2];
    double2 mpre[4], prc[2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = t + T * u;
        dbin[u] = i < a.D ? a.tab.data_bin[i] : 0;
        mpre[u] = i < a.D ? a.mod_pre[i] : make_double2(0.0, 0.0);
        if (u < 2) {
            dslot[u] = i < half ? a.tab.data_slot[i] : 0;
            prc[u] = u < CT ? a.pre[i] : make_double2(0.0, 0.0);  // CT <= 2 (host-checked)
        }
    }
    const int pbin = t < a.P ? a.tab.pilot_bin[t] : 0;
    // the preamble form into registers, then the message symbols' CP pairs
    double2 z[RMAX];
#pragma unroll
    for (int r = 0; r < RMAX; ++r)
        z[r] = r < LT ? src_sample(a.iq, a.iq16, x0 + t + (long)T * r) : make_double2(0.0, 0.0);
    load_twiddles<LOGN>(a.tab.tw, lds_tw, t, T);

    // cp_freq_sinh phases: per-thread partial sums of every symbol, reduced
    // per wave by shuffles, then across waves in LDS (no barrier between
    // symbols: their loads overlap)
    double2* part = dat;  // Q*NWV wave partials (dat is filled only later)
    const int lane = t & 63, wv = t >> 6;
    auto wave_part = [&](int q, double2 acc) {
        constexpr int W0 = T >= 64 ? 32 : T / 2;
#pragma unroll
        for (int o = W0; o > 0; o >>= 1) {
            acc.x += __shfl_xor(acc.x, o);
            acc.y += __shfl_xor(acc.y, o);
        }
        if (lane == 0) part[q * NWV + wv] = acc;
    };
    double rs, rc;
    sincospi(-2.0 * cfo * (double)N, &rs, &rc);
    {
        double2 acc = make_double2(0.0, 0.0);  // preamble: CP sample j = t + T*r, r < cp/T, pairs with r + N/T
#pragma unroll
        for (int r = 0; r < RMAX; ++r)
            if (r < CT && r + N / T < RMAX) acc = cadd(acc, cconj_mul(z[r], z[r + N / T]));
        wave_part(0, acc);
    }
    // two symbols per iteration, so both symbols' CP loads are in flight
    // together (the shuffles in wave_part keep the compiler from unrolling)
    for (int q = 1; q < Q; q += 2) {
        const bool two = q + 1 < Q;  // uniform
        double2 acc0 = make_double2(0.0, 0.0), acc1 = make_double2(0.0, 0.0);
#pragma unroll 2
        for (int j = t; j < a.cp; j += T) {
            const long i0 = x0 + (long)q * L + j, i1 = two ? i0 + L : i0;
            const double2 a0 = src_sample(a.iq, a.iq16, i0), b0 = src_sample(a.iq, a.iq16, i0 + N);
            const double2 a1 = src_sample(a.iq, a.iq16, i1), b1 = src_sample(a.iq, a.iq16, i1 + N);
            acc0 = cadd(acc0, cconj_mul(a0, b0));
            acc1 = cadd(acc1, cconj_mul(a1, b1));
        }
        wave_part(q, acc0);
        if (two) wave_part(q + 1, acc1);
    }
    __syncthreads();
    for (int q = t; q < Q; q += T) {
        double2 acc = make_double2(0.0, 0.0);
        for (int u = 0; u < NWV; ++u) acc = cadd(acc, part[q * NWV + u]);
        phi[q] = cp_phase(acc, make_double2(rc, rs));
    }
    __syncthreads();
    if (t == 0) {
        double acc = 0.0;
        for (int q = 0; q < Q; ++q) {
            psi[q] = acc;
            acc += phi[q];
        }
    }
    // freq_shift + cp_freq_sinh on the preamble: theta(j) = slope * j (psi_0 = 0),
    // applied as e^{i slope t} * (e^{i slope T})^r. pr_phase_sinh's sum
    // sum_{i<L} conj(pre_i) z_i is taken as its CP share in time plus its body
    // share by Parseval, sum_k conj(S_k) Z_k / sqrt(N) over the preamble's
    // nonzero bins (pre's body = IFFT(S)/sqrt(N): Frame.cpp:54-70), from the
    // unrotated FFT Z that chan_char_lq needs anyway; that FFT of the
    // e^{-i phi_pr}-rotated body is then e^{-i phi_pr} Z. The same quantities,
    // rounded differently (~1e-16 relative); the 640 template loads are gone.
    const double slope0 = -2.0 * M_PI * cfo - phi[0] / N;
    double phr;
    {
        double sn, cs, ws, wc;
        sincos(slope0 * (double)t, &sn, &cs);
        sincos(slope0 * (double)T, &ws, &wc);
        double2 c = make_double2(cs, sn);
        const double2 w = make_double2(wc, ws);
        double2 acc = make_double2(0.0, 0.0);
#pragma unroll
        for (int r = 0; r < RMAX; ++r) {
            if (r < LT) {
                z[r] = cmul_exact(z[r], c);
                if (r < 2 && r < CT) acc = cadd(acc, cconj_mul(prc[r], z[r]));
                c = cmul(c, w);
            }
        }
        // body sample cp + t + T*i is register CT + i: regrouped through LDS
        // (CT is a runtime count; a register select chain would cost more)
#pragma unroll
        for (int r = 0; r < RMAX; ++r)
            if (r >= CT && r < LT) fftb[(r - CT) * T + t] = z[r];
        lds_barrier();
        double2 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = fftb[t + T * i];
        lds_barrier();
        fft_block<LOGN, -1>(v, t, lds_tw, fftb);  // Z (unrotated)
        const double2 pz = t < a.P ? fftb[lds_swz(pbin)] : make_double2(0.0, 0.0);  // P <= T (host-checked)
        double2 dz[4];
        double2 bacc = make_double2(a.pilot_ampl * pz.x, a.pilot_ampl * pz.y);  // S = pilot_ampl (real)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            dz[u] = t + T * u < a.D ? fftb[lds_swz(dbin[u])] : make_double2(0.0, 0.0);
            bacc = cadd(bacc, cconj_mul(mpre[u], dz[u]));
        }
        const double isn = 1.0 / sqrt((double)N);
        acc = cadd(acc, make_double2(bacc.x * isn, bacc.y * isn));
        acc = block_sum2<T>(acc, red);
        if (t == 0) phpr = atan2_fast(acc.y, acc.x);
        __syncthreads();
        phr = phpr;
        double rs2, rc2;
        sincos(-phr, &rs2, &rc2);
        const double2 rot = make_double2(rc2, rs2);
        if (t < a.P) pil[t] = cmul_exact(pz, rot);
#pragma unroll
        for (int u = 0; u < 2; ++u)  // D/2 <= 2T
            if (t + T * u < half) dat[t + T * u] = cmul_exact(dz[u], rot);
    }
    __syncthreads();
    double acc = 0.0;
    for (int i = t; i < a.P; i += T) acc += hypot(pil[i].x, pil[i].y);
    acc = block_sum2<T>(make_double2(acc, 0.0), red).x;
    const double phys = acc / ((double)a.P * a.pilot_ampl);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int i = t + T * u;
        if (i < half) {
            const int j = dslot[u];
            const double2 p0 = make_double2(pil[j].x / phys, pil[j].y / phys);
            const double2 coef = cdiv_exact(p0, p0);
            const double2 fs = make_double2(dat[i].x / phys, dat[i].y / phys);
            const double2 q = cdiv_exact(cdiv_exact(fs, coef), mpre[u]);
            ph[i] = atan2_fast(q.y, q.x);
        }
    }
    __syncthreads();
    unwrap_scan<T>(ph, half, reinterpret_cast<unsigned*>(red + 24));  // one-pass unwrap (Frame.hpp:407-414)
    double sxy = 0.0, sy = 0.0;
    for (int i = t; i < half; i += T) {
        sxy += ph[i] * i;
        sy += ph[i];
    }
    const double2 sums = block_sum2<T>(make_double2(sxy, sy), red + 16);
    const double hn = (double)half;
    const double sx = hn * (hn - 1) / 2, sx2 = (hn - 1) * hn * (2 * hn - 1) / 6;
    const double b = (sums.x - sx * sums.y) / (sx2 - sx * sx);
    const double aa = sums.y - b * sx;
    double2* chan = a.chan_out + f * a.D;
    for (int i = t; i < a.D; i += T) {
        double th;
        if (i < half)
            th = add_rn(mul_rn(b, (double)i), aa);
        else
            th = add_rn(add_rn(mul_rn(-b, (double)a.D) / 2, mul_rn((double)(i - half), b)), aa);
        double sn, cs;
        sincos(th, &sn, &cs);
        // the reciprocal once per carrier (libgcc division, as the caller's
        // constell /= chan would round it) instead of a division per point
        chan[i] = a.chan_recip ? cdiv_exact(make_double2(1.0, 0.0), make_double2(cs, sn)) : make_double2(cs, sn);
    }
    // message symbols: theta(m) = A_s + B_s m over the CP-stripped body, as
    // the ramp table {e^{iA}, e^{iB 2^j} (j < CORR_BITS), e^{iBT}}; B 2^j and
    // B T are exact products (powers of two)
    for (int e = t; e < a.S * CORR_PER_SYM; e += T) {
        const int s = e / CORR_PER_SYM, j = e % CORR_PER_SYM, q = 1 + s;
        const double B = -2.0 * M_PI * cfo - phi[q] / N;
        const double th = j == 0 ? -2.0 * M_PI * cfo * (double)((long)q * L + a.cp) - (psi[q] * L + phi[q] * a.cp) / N - phr
                                 : B * (double)(j <= CORR_BITS ? 1 << (j - 1) : T);
        double sn, cs;
        sincos(th, &sn, &cs);
        a.corr_out[(f * a.S + s) * CORR_PER_SYM + j] = make_double2(cs, sn);
    }
}

template <int LOGN>
static hipError_t params_launch_n(const StreamParamsArgs& a, hipStream_t st)
{
    using FS = FftShape<LOGN>;
    const size_t ndat = std::max<size_t>(a.D / 2 + 1, (size_t)(1 + a.S) * (FS::T >= 64 ? FS::T / 64 : 1));  // bins, or CP wave partials
    const size_t shm = sizeof(double2) * (TwLds<LOGN>::SIZE + FS::N + (size_t)a.P + ndat) +
                       sizeof(double) * (a.D / 2 + 2) + sizeof(double2) * 32 + sizeof(double) * 130;
    if (shm > 160 * 1024) return hipErrorInvalidValue;
    lds_opt_in((const void*)stream_params_kernel<LOGN>, 160 * 1024);
    hipLaunchKernelGGL(stream_params_kernel<LOGN>, dim3((unsigned)a.nframes), dim3(FS::T), shm, st, a);
    return hipGetLastError();
}

hipError_t launch_stream_params(int logn, const StreamParamsArgs& a, hipStream_t st)
{
    if (a.nframes <= 0) return hipSuccess;
    // one preamble symbol, form length a multiple of T (register layout), <= 16 registers
    const int T = (1 << logn) / 8, L = (1 << logn) + a.cp;
    if (a.npr != 1 || a.S + 1 > 64 || L % T != 0 || L / T > 16 || a.cp > 2 * T || a.D > 4 * T || a.P > T)
        return hipErrorInvalidValue;
    switch (logn) {
        case 6: return params_launch_n<6>(a, st);
        case 7: return params_launch_n<7>(a, st);
        case 8: return params_launch_n<8>(a, st);
        case 9: return params_launch_n<9>(a, st);
        case 10: return params_launch_n<10>(a, st);
        case 11: return params_launch_n<11>(a, st);
        case 12: return params_launch_n<12>(a, st);
        default: return hipErrorInvalidValue;
    }
}

// ========================================================================
// Fused stream decode, stages 1 + 2 in one kernel, for N = 512 and a
// pilot_freq_sinh form of 640 = 5 x 128 points (the D geometry): two waves
// per located frame, the preamble read once for both stages.
//   wave 0: pilot_freq_sinh as cfo_kernel<7, 5> (five interleaved 128-point
//           transforms, four side by side and then one, the radix-5 combine,
//           |.|, fftshift, first argmax per window), then the preamble part
//           of stream_params_kernel (its cp_freq_sinh phase, freq_shift +
//           cp correction, the body FFT, pr_phase_sinh, chan_char_lq);
//   wave 1: meanwhile the message symbols' CP correlation sums (raw samples;
//           rotated once the CFO is known).
// Then both waves: the symbol phases, the channel reciprocals and the ramps.
// Every quantity is computed with the arithmetic of the two kernels it
// replaces (same transforms, same reduction orders), so the results are the
// same to the last bit.
// ========================================================================
// LDS of the sync stage (stream_decode_kernel).
struct SyncLds {
    double2* tw9;   // TwLds<9>
    double2* tw7;   // TwLds<7>
    double2* img;   // 640: the CFO transforms (amp over them), then the body FFT (512)
    double2* pil;   // P
    double2* dat;   // D/2 + 1 raw bins of the preamble (not over img[0, 512))
    double2* red;   // 32
    double2* cps;   // 1 + S raw CP sums
    double* amp;    // 640 magnitudes (fftshifted), over img
    double* ph;     // D/2 + 2
    double* phi;    // 64 symbol phases
    double* psi;    // 64 prefix sums
    double* scal;   // cfo, phr, b, aa
    int* wsum;      // P + 1 window maxima
};

// One located frame's sync stage (128 threads): writes cfo_out[f] and the
// frame's ramp / channel table (ofdm_rx2.hpp rt_size) to rt, in LDS over the
// stage's small arrays; returns after a barrier. load_tw: fill the twiddle
// tables here (else they are resident and visible).
template <bool I16, bool PROF = false>
__device__ __forceinline__ void sync_frame(const CfoArgs& c, const StreamParamsArgs& a, long f, const SyncLds& Ls,
                                           double2* rt, bool load_tw)
{
    // the geometry is fixed (host-checked): N = 512, cp = 128, L = 640 = 10 T
    constexpr int LOGN = 9, N = 512, T = 64, LOGM = 7, M = 128, G = 5, S5 = G * M, CP = 128, L = N + CP;
    constexpr int LT = L / T, CT = CP / T, RMAX = LT;
    double2* tw9 = Ls.tw9;
    double2* tw7 = Ls.tw7;
    double2* img = Ls.img;
    double2* pil = Ls.pil;
    double2* dat = Ls.dat;
    double2* red = Ls.red;
    double2* cps = Ls.cps;
    double* ph = Ls.ph;
    double* phi = Ls.phi;
    double* psi = Ls.psi;
    double* scal = Ls.scal;
    int* wsum = Ls.wsum;
    // opaque per-frame copy of the thread index: the per-lane table loads and
    // addresses are made here, not hoisted out of a caller's frame loop and
    // held live across it
    int tid;
    asm volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"((int)threadIdx.x));
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const long x0 = a.starts[f];
    const int half = a.D / 2, Q = 1 + a.S;
    OFDM_PHASE(cfo_transforms);
    // ---------------------------------------------------------- pilot_freq_sinh (both waves)
    // transform g holds x[G*n + g], n = tt + 16*i: g = lane/16 (0..3) on
    // wave 0, g = 4 on wave 1's lanes 0..15
    {
        const int g = w == 0 ? lane >> 4 : 4, tt = lane & 15;
        double2 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const long j = x0 + (long)G * (tt + 16 * i) + g;
            v[i] = src_sample_t<I16>(c.x, c.x16, j);
        }
        if (load_tw) {
            load_twiddles<LOGM>(c.tw_sub, tw7, tid, 128);
            load_twiddles<LOGN>(a.tab.tw, tw9, tid, 128);
        }
        __syncthreads();  // twiddles visible; the previous frame's LDS use is over
        if (w == 0 || lane < 16) fft_block_wave<LOGM, -1>(v, tt, tw7, img + g * M);
        __syncthreads();  // the five transforms visible
    }
    OFDM_PHASE(cfo_radix5);
    {
        // X[k + M*r] = sum_q W_S^{q k} W_G^{q r} F_q[k]; stored fftshifted:
        // shifted[i] = spec[(i + S/2) % S]  (Frame.hpp:300-305). The window
        // argmax below works on |X|^2 and takes hypot only where it must.
        constexpr int half5 = S5 / 2;
        double2* spec = img;
        double2 twg[G - 1];
#pragma unroll
        for (int q = 1; q < G; ++q) twg[q - 1] = c.tw_full[(long)q * M];
        {
            const int k = tid;  // M = 128 = the workgroup
            double2 twk[G - 1];
#pragma unroll
            for (int q = 1; q < G; ++q) twk[q - 1] = c.tw_full[(long)q * k % S5];
            double2 tq[G];
#pragma unroll
            for (int q = 0; q < G; ++q) {
                const double2 fq = img[q * M + lds_swz(k)];
                tq[q] = q == 0 ? fq : cmul(fq, twk[q - 1]);
            }
            __syncthreads();  // every transform read: the spectrum overwrites them
            // the 5-point DFT over q by the symmetric pairs (1, 4), (2, 3):
            // X_r, X_{5-r} = t_r +- i u_r, with W5 = twg[0] = (c1, n1), W5^2 =
            // twg[1] = (c2, n2) (44 operations instead of 20 products + sums)
            static_assert(G == 5, "radix-5 combine");
            const double c1 = twg[0].x, n1 = twg[0].y, c2 = twg[1].x, n2 = twg[1].y;
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
#pragma unroll
            for (int r = 0; r < G; ++r) spec[(k + M * r + half5) % S5] = X[r];
        }
        __syncthreads();  // spectrum visible
        // first argmax of |X| = hypot inside each pilot window [borders[i],
        // borders[i+1]), i != P/2 (std::max_element: 8-lane groups, the larger
        // value, the lower index on ties). Decided on e = |X|^2 (two products,
        // one sum: relative error <= 2u, u = 2^-53) where the runner-up e2 <
        // e1 * (1 - 64u): then every other element's hypot (error <= 4u) is
        // strictly below the winner's, so the winner is hypot's first maximum.
        // Otherwise (near-ties, or a non-finite element) the group takes
        // hypot of its window, as cfo_kernel does.
        OFDM_PHASE(cfo_argmax);
        constexpr int AG = 8;
        constexpr double SURE = 1.0 - 64.0 * 0x1.0p-53;
        // the P windows that count (window P/2 is skipped by the sum below),
        // 8 lanes each: for P <= 8 wave 0 alone, and a wave whose groups are
        // all past the last window skips the pass (a uniform branch)
        for (int g0 = 0; g0 < c.P; g0 += 128 / AG) {
            if (g0 + w * (64 / AG) >= c.P) continue;  // uniform per wave
            const int gi = g0 + tid / AG, l = tid % AG;
            const int i = gi < c.P / 2 ? gi : gi + 1;
            const bool act = gi < c.P;
            int lo = 0, hi = 0;
            if (act) {
                lo = c.borders[i];
                hi = c.borders[i + 1];
            }
            double bv = -1.0, sv = -1.0;  // best and runner-up |X|^2 (below every magnitude)
            int bi = INT_MAX, odd = 0;
            for (int j = lo + l; j < hi; j += AG) {
                const double2 z = spec[j];
                const double e = add_rn(mul_rn(z.x, z.x), mul_rn(z.y, z.y));
                odd |= !(e <= DBL_MAX);  // NaN or inf: hypot decides
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
            if (odd || !(sv < bv * SURE)) {  // uniform within the 8-lane group
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
            if (act && l == 0) wsum[i] = lo < hi ? (first_nan ? lo : bi) : hi;
        }
        __syncthreads();  // window maxima visible
        OFDM_PHASE(cfo_final);
        if (tid == 0) {
            double shift = 0.0;
            for (int i = 0; i <= c.P; ++i)
                if (i != c.P / 2) shift += wsum[i];
            shift /= c.P;
            shift -= S5 / 2;
            shift /= S5;
            scal[0] = shift;
            c.cfo_out[f] = shift;
        }
        __syncthreads();  // the CFO visible; the CFO images are free
        OFDM_STOP(PROF, 1);
    }
    if (w == 0) {
        const double cfo = scal[0];

        // ---------------------------------------------------------- preamble (stream_params_kernel)
        OFDM_PHASE(w0_pre_load);
        const int t = lane;
        int dbin[4], dslot[2];
        double2 mpre[4], prc[2];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = t + T * u;
            dbin[u] = i < a.D ? a.tab.data_bin[i] : 0;
            mpre[u] = i < a.D ? a.mod_pre[i] : make_double2(0.0, 0.0);
            if (u < 2) {
                dslot[u] = i < half ? a.tab.data_slot[i] : 0;
                prc[u] = u < CT ? a.pre[i] : make_double2(0.0, 0.0);
            }
        }
        const int pbin = t < a.P ? a.tab.pilot_bin[t] : 0;
        double2 z[RMAX];
#pragma unroll
        for (int r = 0; r < RMAX; ++r)
            z[r] = r < LT ? src_sample_t<I16>(a.iq, a.iq16, x0 + t + (long)T * r) : make_double2(0.0, 0.0);
        OFDM_PHASE(w0_pre_cpsum);
        double rs, rc;
        sincospi(-2.0 * cfo * (double)N, &rs, &rc);
        {
            // the preamble's cp_freq_sinh sum (CP sample r pairs with r + N/T)
            double2 acc = make_double2(0.0, 0.0);
#pragma unroll
            for (int r = 0; r < RMAX; ++r)
                if (r < CT && r + N / T < RMAX) acc = cadd(acc, cconj_mul(z[r], z[r + N / T]));
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                acc.x += __shfl_xor(acc.x, o);
                acc.y += __shfl_xor(acc.y, o);
            }
            acc = cadd(make_double2(0.0, 0.0), acc);
            if (t == 0) phi[0] = cp_phase(acc, make_double2(rc, rs));
        }
        wave_lds_sync();
        const double slope0 = -2.0 * M_PI * cfo - phi[0] / N;
        double phr;
        {
            // the step e^{i slope0 T} by its own sincos. (Round 3 took it as
            // lane T/2's phasor squared, a shuffle instead of a second sincos
            // pass: no change in a serial call, but two contexts receiving on
            // two streams then no longer overlapped one call's walk with the
            // other's decode: int16 stream 183 -> 162 G samples/s in a
            // same-box A/B that reverted each part of that change alone,
            // profiles/r04h_pipelined_rev.json.)
            OFDM_PHASE(w0_pre_ramp);
            double sn, cs, ws, wc;
            sincos(slope0 * (double)t, &sn, &cs);
            sincos(slope0 * (double)T, &ws, &wc);
            double2 cc = make_double2(cs, sn);
            const double2 wv = make_double2(wc, ws);
            double2 acc = make_double2(0.0, 0.0);
#pragma unroll
            for (int r = 0; r < RMAX; ++r) {
                if (r < LT) {
                    z[r] = cmul_exact(z[r], cc);
                    if (r < 2 && r < CT) acc = cadd(acc, cconj_mul(prc[r], z[r]));
                    cc = cmul(cc, wv);
                }
            }
            double2* fftb = img;  // the CFO images are free
#pragma unroll
            for (int r = 0; r < RMAX; ++r)
                if (r >= CT && r < LT) fftb[(r - CT) * T + t] = z[r];
            wave_lds_sync();
            double2 vv[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) vv[i] = fftb[t + T * i];
            wave_lds_sync();
            OFDM_PHASE(w0_pre_fft);
            fft_block_wave<LOGN, -1>(vv, t, tw9, fftb);  // Z (unrotated)
            OFDM_PHASE(w0_pre_phase);
            const double2 pz = t < a.P ? fftb[lds_swz(pbin)] : make_double2(0.0, 0.0);
            double2 dz[4];
            double2 bacc = make_double2(a.pilot_ampl * pz.x, a.pilot_ampl * pz.y);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                dz[u] = t + T * u < a.D ? fftb[lds_swz(dbin[u])] : make_double2(0.0, 0.0);
                bacc = cadd(bacc, cconj_mul(mpre[u], dz[u]));
            }
            const double isn = 1.0 / sqrt((double)N);
            acc = cadd(acc, make_double2(bacc.x * isn, bacc.y * isn));
            acc = block_sum2<T>(acc, red);
            phr = atan2_fast(acc.y, acc.x);
            // e^{-i phr} = conj(acc) / |acc| (acc is uniform: a uniform
            // branch keeps sincos for a zero or non-finite sum)
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
            if (t < a.P) pil[t] = cmul_exact(pz, rot);
#pragma unroll
            for (int u = 0; u < 2; ++u)
                if (t + T * u < half) dat[t + T * u] = cmul_exact(dz[u], rot);
        }
        wave_lds_sync();
        OFDM_PHASE(w0_pre_phys_atan);
        double acc = 0.0;
        for (int i = t; i < a.P; i += T) acc += hypot(pil[i].x, pil[i].y);
        acc = block_sum2<T>(make_double2(acc, 0.0), red).x;
        const double phys = acc / ((double)a.P * a.pilot_ampl);
        // arg((F/phys)/coef/mod_pre) (Frame.hpp:397-405 over FFT_FORM::read,
        // Frame.cpp:82-93): only the angle is used, so for a finite positive
        // phys it is arg(F conj(mod_pre)) (a positive real factor apart; coef
        // is 1 to the last bit, below); otherwise the reference's divisions
        // verbatim
        const bool plain = phys > 0.0 && phys <= DBL_MAX;  // uniform
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = t + T * u;
            if (i < half) {
                const int j = dslot[u];
                double2 q;
                if (plain) {
                    // coef = (F/phys)/(F/phys) of the one preamble symbol is 1
                    // up to its last bit (Smith's division of a number by
                    // itself): its angle, ~1e-16, is dropped with the division
                    q = cmul_exact(dat[i], make_double2(mpre[u].x, -mpre[u].y));
                } else {
                    const double2 p0 = make_double2(pil[j].x / phys, pil[j].y / phys);
                    const double2 coef = cdiv_exact(p0, p0);
                    const double2 fs = make_double2(dat[i].x / phys, dat[i].y / phys);
                    q = cdiv_exact(cdiv_exact(fs, coef), mpre[u]);
                }
                ph[i] = atan2_fast(q.y, q.x);
            }
        }
        wave_lds_sync();
        OFDM_PHASE(w0_pre_unwrap_ls);
        unwrap_scan<T, true>(ph, half, reinterpret_cast<unsigned*>(red + 24));  // one-pass unwrap (Frame.hpp:407-414)
        double sxy = 0.0, sy = 0.0;
        for (int i = t; i < half; i += T) {
            sxy += ph[i] * i;
            sy += ph[i];
        }
        const double2 sums = block_sum2<T>(make_double2(sxy, sy), red + 16);
        const double hn = (double)half;
        const double sx = hn * (hn - 1) / 2, sx2 = (hn - 1) * hn * (2 * hn - 1) / 6;
        const double b = (sums.x - sx * sums.y) / (sx2 - sx * sx);
        if (t == 0) {
            scal[1] = phr;
            scal[2] = b;
            scal[3] = sums.y - b * sx;
        }
    } else {
        // ---------------------------------------------------------- message CP sums (wave 1)
        // two symbols per iteration, so both symbols' CP loads are in flight together
        OFDM_PHASE(w1_msg_cpsums);
        const int t = lane;
        for (int q = 1; q < Q; q += 2) {
            const bool two = q + 1 < Q;  // uniform
            double2 acc0 = make_double2(0.0, 0.0), acc1 = make_double2(0.0, 0.0);
#pragma unroll 2
            for (int j = t; j < a.cp; j += T) {
                const long i0 = x0 + (long)q * L + j, i1 = two ? i0 + L : i0;
                const double2 a0 = src_sample_t<I16>(a.iq, a.iq16, i0), b0 = src_sample_t<I16>(a.iq, a.iq16, i0 + N);
                const double2 a1 = src_sample_t<I16>(a.iq, a.iq16, i1), b1 = src_sample_t<I16>(a.iq, a.iq16, i1 + N);
                acc0 = cadd(acc0, cconj_mul(a0, b0));
                acc1 = cadd(acc1, cconj_mul(a1, b1));
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                acc0.x += __shfl_xor(acc0.x, o);
                acc0.y += __shfl_xor(acc0.y, o);
                acc1.x += __shfl_xor(acc1.x, o);
                acc1.y += __shfl_xor(acc1.y, o);
            }
            if (t == 0) {
                cps[q] = acc0;
                if (two) cps[q + 1] = acc1;
            }
        }
        // the message symbols' CP phases, here rather than after the join:
        // one atan2 pass on this wave instead of one on each
        wave_lds_sync();  // cps visible
        double rs, rc;
        sincospi(-2.0 * scal[0] * (double)N, &rs, &rc);
        if (t < a.S) {
            const int q = 1 + t;
            const double2 acc = cadd(make_double2(0.0, 0.0), cps[q]);
            phi[q] = cp_phase(acc, make_double2(rc, rs));
        }
    }
    __syncthreads();  // cfo, phi[0..S], phr and the LS fit visible
    OFDM_PHASE(ramp_table);
    const double cfo = scal[0], phr = scal[1], b = scal[2], aa = scal[3];
    if (tid == 0) {
        double acc = 0.0;
        for (int q = 0; q < Q; ++q) {
            psi[q] = acc;
            acc += phi[q];
        }
    }
    __syncthreads();  // psi visible
    // the frame's table (ofdm_rx2.hpp rt_size): one transcendental pass for
    // every ramp and both channel steps. Message symbol s: theta(m) = A_s +
    // B_s m over the CP-stripped body.
    const int nt = RT_PER_SYM * a.S + 2;  // <= 128 (S <= RX_SMAX)
    double2 val = make_double2(0.0, 0.0);
    if (tid < nt) {
        double th;
        if (tid < RT_PER_SYM * a.S) {
            const int s = tid / RT_PER_SYM, k = tid % RT_PER_SYM, q = 1 + s;
            const double A = -2.0 * M_PI * cfo * (double)((long)q * L + a.cp) - (psi[q] * L + phi[q] * a.cp) / N - phr;
            const double B = -2.0 * M_PI * cfo - phi[q] / N;
            th = k < 8 ? add_rn(A, mul_rn(B, (double)k)) : mul_rn(B, k < 11 ? (double)(8 << (k - 8)) : (double)T);
        } else {
            const double step = mul_rn(128.0, b);
            th = tid == RT_PER_SYM * a.S ? step : sub_rn(step, add_rn(mul_rn(b, (double)a.D) / 2, mul_rn(b, (double)half)));
        }
        double sn, cs;
        sincos(th, &sn, &cs);
        val = make_double2(cs, sn);
    }
    __syncthreads();  // phi / psi / scal read: the table is written over them
    if (tid < nt) rt[tid] = val;
    if (tid == 0) rt[nt] = make_double2(b, aa);
    __syncthreads();  // the table visible; the stage's other LDS is free
    OFDM_STOP(PROF, 2);
    OFDM_PHASE(sync_end);
}

// ========================================================================
// The whole fused stream decode in one kernel (N = 512, 640-point CFO form):
// one workgroup per located frame runs sync_frame (pilot_freq_sinh, the CP / phase
// corrections, chan_char_lq; Frame.hpp:238-348,389-434) and then rx2_frame
// (the 8 message transforms, equalisation, channel, decisions;
// Frame.cpp:73-96, main.cpp:67-71, modulation.cpp:53-87) in the same
// two-wave workgroup, the ramps and the channel passed through LDS. Each
// frame's samples are read once from HBM (the preamble, then the CP pairs,
// then the bodies, whose CP-pair tails are fresh in the caches), and the
// latency-bound sync stage of one frame overlaps the bandwidth-bound
// transforms of the CU's other frames. LDS (~19.4 KB: 8 frames per CU at 4
// waves per SIMD): the 512-point twiddles, one 16 KB region (the sync stage's
// transforms and 128-point twiddles, then the two rx images, then the
// decisions and the channel), the ramps, and the two stages' small arrays
// over each other. The channel reciprocals go through the chan scratch (L2)
// from the sync stage to the rx stage's emit.
// ========================================================================
template <bool I16, bool PROF = false>
__global__ void __launch_bounds__(128, 4) stream_decode_kernel(CfoArgs c, StreamParamsArgs a, RxArgs r)
{
    extern __shared__ double2 smem[];
    const int S = a.S, D = a.D, P = a.P;
    double2* tw9 = smem;
    double2* A = tw9 + TwLds<9>::SIZE;        // 1024: sync transforms (+ tw7) / dat / ph, then the rx images
    double2* tw7 = A + 640;                   // over A, past the CFO transforms (dead with them)
    double2* U = A + 1024;                    // the stages' small arrays, over each other
    double2* rt = U + S * P;                  // the ramp / channel table: sync -> rx (rx's gains come after it)
    SyncLds Ls;
    Ls.tw9 = tw9;
    Ls.tw7 = tw7;
    Ls.img = A;
    Ls.amp = reinterpret_cast<double*>(A);
    Ls.dat = A + 512;
    Ls.ph = reinterpret_cast<double*>(A + 650);
    Ls.pil = U;
    Ls.red = Ls.pil + P;
    Ls.cps = Ls.red + 32;
    Ls.phi = reinterpret_cast<double*>(Ls.cps + 1 + S);
    Ls.psi = Ls.phi + 64;
    Ls.scal = Ls.psi + 64;
    Ls.wsum = reinterpret_cast<int*>(Ls.scal + 4);
    Rx2Lds Lr;
    Lr.img = A;
    Lr.tw = tw9;
    Lr.pil = U;
    Lr.gain = U + S * P;
    Lr.chl = A + ((S * D + 15) >> 4);  // over the images, past the decisions (rx2_frame stages it)
    Lr.red = reinterpret_cast<double*>(rt + std::max(S * P, rt_size(S)));
    const int lane0 = threadIdx.x & 63;
    const long f = blockIdx.x;
    if (a.count && f >= *a.count) return;  // uniform: past the speculative frame count
    if (a.starts[f] < 0) return;           // before the stream's first sample: the gather path's
    // one frame per workgroup (a persistent frame loop let the compiler hoist
    // the sync stage's math-library constants and tables out of it: spills)
    int pk[RX_DPT];
#pragma unroll
    for (int i = 0; i < RX_DPT; ++i) pk[i] = r.tab.rx_pack[lane0 + 64 * i];
    const int pbin = r.tab.pilot_swz[lane0];
    // the sync stage's dependent chains issue ahead of the transform-heavy
    // rx stage of the CU's other frames (priority 1 vs 0: 498 -> 478 us;
    // 2 and 3 gain less)
    __builtin_amdgcn_s_setprio(1);
    sync_frame<I16, PROF>(c, a, f, Ls, rt, true);
    __builtin_amdgcn_s_setprio(0);
    rx2_frame<I16, true, PROF>(r, f, Lr, reinterpret_cast<const double*>(rt), pk, pbin);
}

static bool stream_sync_geometry(const CfoArgs& c, const StreamParamsArgs& a, int logn, int logm, int g)
{
    const int L = (1 << logn) + a.cp;
    return logn == 9 && logm == 7 && g == 5 && L == 640 && a.npr == 1 && a.S + 1 <= 64 && a.S <= RX_SMAX &&
           a.cp == 128 && a.D <= 256 && a.P <= 64 && c.P == a.P;
}

template <bool I16>
static hipError_t decode_launch(const CfoArgs& c, const StreamParamsArgs& a, const RxArgs& r, hipStream_t st)
{
    const size_t rx_u = sizeof(double2) * ((size_t)a.S * a.P + std::max(a.S * a.P, rt_size(a.S))) + sizeof(double) * 2;
    const size_t sync_u = sizeof(double2) * (a.P + 32 + 1 + a.S) + sizeof(double) * 132 + sizeof(int) * (a.P + 2);
    const size_t shm = sizeof(double2) * (TwLds<9>::SIZE + 1024) + std::max(rx_u, sync_u);
    // diagnostics: OFDM_DECODE_STOP=k runs the build whose waves end at stop
    // point k (per-segment instruction counts from SQ counters)
    static const int stop = [] {
        const char* e = getenv("OFDM_DECODE_STOP");
        return e ? atoi(e) : 0;
    }();
    if (stop > 0) {
        static std::once_flag once;
        std::call_once(once, [] { (void)hipMemcpyToSymbol(HIP_SYMBOL(g_decode_stop), &stop, sizeof(int)); });
        lds_opt_in((const void*)stream_decode_kernel<I16, true>, 160 * 1024);
        hipLaunchKernelGGL((stream_decode_kernel<I16, true>), dim3((unsigned)a.nframes), dim3(128), shm, st, c, a, r);
        return hipGetLastError();
    }
    lds_opt_in((const void*)stream_decode_kernel<I16>, 160 * 1024);
    hipLaunchKernelGGL(stream_decode_kernel<I16>, dim3((unsigned)a.nframes), dim3(128), shm, st, c, a, r);
    return hipGetLastError();
}

hipError_t launch_stream_decode(const CfoArgs& c, const StreamParamsArgs& a, const RxArgs& r, int logn, int logm, int g,
                                hipStream_t st)
{
    if (a.nframes <= 0) return hipSuccess;
    if (!r.chan_recip || r.D != a.D || r.S != a.S || r.P != a.P) return hipErrorNotSupported;
    // the fused kernels are instantiated per stream format (the sample loads
    // carry no per-sample branch): every view of the stream is the same one
    const bool i16 = r.iq16 != nullptr;
    if (i16 != (a.iq16 != nullptr) || i16 != (c.x16 != nullptr) || (!i16 && (!r.iq || !a.iq || !c.x)))
        return hipErrorInvalidValue;
    // N = 2048 / 4096 with cp = N/4 (configs B, C): ofdm_stream_wide.hip
    if (stream_decode_wide_fits(a, logn, logm, g, c.P)) return launch_stream_decode_wide(c, a, r, logn, st);
    if (!stream_sync_geometry(c, a, logn, logm, g))
        return hipErrorNotSupported;  // the staged launches cover other geometries
    return r.iq16 ? decode_launch<true>(c, a, r, st) : decode_launch<false>(c, a, r, st);
}

// ========================================================================
// Streaming detection walk (rx.cpp:125-221; oracle orc_stream_walk). One
// 256-thread workgroup walks one chunk of the stream sequentially:
//   hit = first T2 block with rel > level on the grid pos + k*T2sin_size
//         (G blocks transformed per step, first hit taken);
//   pb  = find_preamble(hit) + 1;  pb < -2 -> pos = hit + message;
//   frame past the stream end -> stop;  else record pb, pos = pb + message.
// A walker starts `halo` samples before its core [c*chunk, (c+1)*chunk) (or
// at an exact state in a re-walk) and stops at the first state >= the core
// end. The host accepts a chunk when its walk shares a located frame with
// the previous chunk's (after which both walks are the same computation), and
// re-walks it from the previous chunk's exit state otherwise.
// ========================================================================
namespace {


// Walker workgroup: 128 threads (2 waves) for T2sin_size <= 1024, so that 8
// walkers share a CU (~19 KB of LDS each, 128 VGPRs = 4 waves per SIMD): the
// walk is latency-bound, and twice the walkers halve each one's chunk. One
// 256-thread transform for T2sin_size = 2048.
template <int LOGT>
struct WalkShape {
    static constexpr int T = (1 << LOGT) / 8;
    static constexpr int WT = T > 128 ? T : 128;  // threads
    static constexpr int G = WT / T;              // T2 blocks per scan step
};

// Stream format of the walker's loads: FMT_ANY tests the int16 pointer at
// run time (one kernel for both formats); FMT_I16 / FMT_F64 fix it at compile
// time (the walker is instantiated per format: no dead path's registers and
// no branch between a batch's loads and their uses).
enum { FMT_ANY = 0, FMT_I16 = 1, FMT_F64 = 2 };

template <int F, class A>
__device__ __forceinline__ bool fmt_i16(const A& a)
{
    return F == FMT_ANY ? a.iq16 != nullptr : F == FMT_I16;
}

// Stream sample j as complex<double> (int16 wire samples convert exactly, as
// FRAME_FORM::form_int16_to_double, Frame.hpp:472-481); zero outside [0, n).
template <int F = FMT_ANY, class A>
__device__ __forceinline__ double2 stream_sample(const A& a, long j)
{
    if (j < 0 || j >= a.n) return make_double2(0.0, 0.0);
    if (fmt_i16<F>(a)) {
        const short2 v = a.iq16[j];
        return make_double2((double)v.x, (double)v.y);
    }
    return a.iq[j];
}

// The same for j known to lie in [0, n) (no per-sample 64-bit bounds test).
template <int F = FMT_ANY, class A>
__device__ __forceinline__ double2 stream_sample_in(const A& a, long j)
{
    if (fmt_i16<F>(a)) {
        const short2 v = a.iq16[j];
        return make_double2((double)v.x, (double)v.y);
    }
    return a.iq[j];
}

// Eight samples x[base + lane + 64*i] (zero where lane + 64*i >= W or the
// index is outside [0, n)), all eight loads issued before any is used:
// clamped addresses and selects, no per-sample branch (a branch around each
// load, or a use inside it, makes each load wait for the one before).
template <int F = FMT_ANY, class A>
__device__ __forceinline__ void load8_window(const A& a, long base, int lane, int W, double2 (&v)[8])
{
    long j[8];
    bool ok[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const long q = base + lane + 64 * i;
        ok[i] = lane + 64 * i < W && q >= 0 && q < a.n;
        j[i] = ok[i] ? q : 0;
    }
    if (fmt_i16<F>(a)) {  // uniform
        const int* p = reinterpret_cast<const int*>(a.iq16);
        int w[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = p[j[i]];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            v[i] = ok[i] ? make_double2((double)(int)(short)(w[i] & 0xffff), (double)(w[i] >> 16))
                         : make_double2(0.0, 0.0);
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = a.iq[j[i]];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (!ok[i]) v[i] = make_double2(0.0, 0.0);
    }
}

// x[base + T*i], i < 8, all in [0, n) when `live` (else zeros), loads
// issued together (the int16 loads waited one by one behind per-sample branches).
template <int T, int F = FMT_ANY, class A>
__device__ __forceinline__ void load8_block(const A& a, long base, bool live, double2 (&v)[8])
{
    const long b0 = live ? base : 0;
    if (fmt_i16<F>(a)) {  // uniform
        const int* p = reinterpret_cast<const int*>(a.iq16) + b0;
        int w[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = p[T * i];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            v[i] = live ? make_double2((double)(int)(short)(w[i] & 0xffff), (double)(w[i] >> 16))
                        : make_double2(0.0, 0.0);
    } else {
        const double2* p = a.iq + b0;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = p[T * i];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (!live) v[i] = make_double2(0.0, 0.0);
    }
}

// x[base + T*i], i < 8, for a block that straddles the stream's ends (ring
// mode: rx.cpp's zero header before the first SDR buffer, the zeros after a
// capture): samples outside [0, n) read as zero. Rare (a walk's first and
// last blocks), so per-sample guards are fine here.
template <int T, int F = FMT_ANY, class A>
__device__ __forceinline__ void load8_block_part(const A& a, long base, double2 (&v)[8])
{
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = stream_sample<F>(a, base + T * i);
}

__device__ __forceinline__ double energy_rn(double2 v) { return add_rn(mul_rn(v.x, v.x), mul_rn(v.y, v.y)); }

// load8_block rounded to FP32 (int16 wire samples convert exactly).
template <int T, int F = FMT_ANY, class A>
__device__ __forceinline__ void load8_block32(const A& a, long base, bool live, float2 (&v)[8])
{
    const long b0 = live ? base : 0;
    if (fmt_i16<F>(a)) {  // uniform
        const int* p = reinterpret_cast<const int*>(a.iq16) + b0;
        int w[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = p[T * i];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            v[i] = live ? make_float2((float)(short)(w[i] & 0xffff), (float)(w[i] >> 16)) : make_float2(0.f, 0.f);
    } else {
        const double2* p = a.iq + b0;
        double2 d[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) d[i] = p[T * i];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = live ? make_float2((float)d[i].x, (float)d[i].y) : make_float2(0.f, 0.f);
    }
}

// PREAMBLE_FORM::find_preamble from s: first lag with norm > 1 and
// |sum_j x[s+i+j] c_j| / sqrt(norm) > level (Frame.cpp:338-378), INT_MAX if
// none. Exact form: the running energy is the reference's serial recurrence
// (+ new, then - old, separately rounded; each sample's energy as re*re+im*im
// rounded as the reference rounds it); lags are tested WT at a time with an
// early exit. xs: C + L samples, normv: C running energies (LDS).
template <int WT, int F>
__device__ int walk_preamble_exact(const WalkArgs& a, long s, double2* xs, const double2* c, double* normv,
                                   int* best, int t)
{
    const int L = a.L, C = a.cycles;
    for (int i = t; i < C + L; i += WT) xs[i] = stream_sample<F>(a, s + i);
    if (t == 0) *best = INT_MAX;
    __syncthreads();
    if (t == 0) {
        double norm = 0.0;
        for (int i = 0; i < L; ++i) norm = add_rn(norm, energy_rn(xs[i]));
        for (int i = 0; i < C; ++i) {
            normv[i] = norm;
            norm = add_rn(norm, energy_rn(xs[i + L]));
            norm = sub_rn(norm, energy_rn(xs[i]));
        }
    }
    __syncthreads();
    int found = INT_MAX;
    for (int base = 0; base < C; base += WT) {
        const int i = base + t;
        if (i < C) {
            const double norm = normv[i];
            if (norm > 1.0) {
                double2 e = make_double2(0.0, 0.0);
                for (int j = 0; j < L; ++j) e = cadd_rn(e, cmul_exact(xs[i + j], c[j]));
                if (hypot(e.x, e.y) / sqrt(norm) > a.pr_level) atomicMin(best, i);
            }
        }
        __syncthreads();
        found = *best;
        if (found != INT_MAX) break;  // uniform
    }
    __syncthreads();  // every thread has read *best before the next search resets it
    return found;
}

// Certified parallel form of the same search. Each lag's correlation e is
// computed exactly as the reference (j = 0..L-1 in order, no FMA); its energy
// is the window sum s_i = sum_{j<L} E[i+j] taken per lag instead of the
// serial recurrence n_i. The two differ by at most
//   |n_i - s_i| <= (2L + 2i + 4) u M  (u = 2^-53, M >= every partial value
// the recurrence passes through: max window sum + max sample energy), so a
// lag whose norm test and ratio test both clear their thresholds by more
// than that bound is decided exactly as the reference decides it. The first
// lag that is not a certain FAIL is the answer when it is a certain PASS;
// otherwise (margins ~1e-13, practically never) the exact serial search runs.
// xs: C + L samples, E: C + L energies, normv: C, c: the L template taps
// (all in the search scratch; c is loaded here).
template <int WT, int F>
__device__ int walk_preamble(const WalkArgs& a, long s, double2* xs, double2* c, double* E, double* normv,
                             int* best, int* unsure, double* mred, int t)
{
    constexpr double U = 0x1.0p-53;
    const int L = a.L, C = a.cycles;
    if (a.exact_only) return walk_preamble_exact<WT, F>(a, s, xs, a.templ, normv, best, t);
    for (int i = t; i < L; i += WT) c[i] = a.templ[i];
    double emax = 0.0;
    for (int i = t; i < C + L; i += WT) {
        const double2 v = stream_sample<F>(a, s + i);
        xs[i] = v;
        const double e2 = add_rn(mul_rn(v.x, v.x), mul_rn(v.y, v.y));
        E[i] = e2;
        emax = fmax(emax, e2);
    }
    if (t == 0) {
        *best = INT_MAX;
        *unsure = INT_MAX;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) emax = fmax(emax, __shfl_xor(emax, o));
    if ((t & 63) == 0) mred[WT / 64 + (t >> 6)] = emax;
    double M = 0.0;  // max window sum over every lag so far
    int found = INT_MAX;
    for (int base = 0; base < C; base += 2 * WT) {
        __syncthreads();  // xs/E visible (first batch); best/unsure reset
        // two lags per thread, interleaved (two independent accumulation chains)
        const int i0 = base + t, i1 = base + WT + t;
        const bool v0 = i0 < C, v1 = i1 < C;
        const int j0 = v0 ? i0 : 0, j1 = v1 ? i1 : 0;
        double2 e0 = make_double2(0.0, 0.0), e1 = make_double2(0.0, 0.0);
        double s0 = 0.0, s1 = 0.0;
        for (int j = 0; j < L; ++j) {
            const double2 cj = c[j];
            e0 = cadd_rn(e0, cmul_exact(xs[j0 + j], cj));
            e1 = cadd_rn(e1, cmul_exact(xs[j1 + j], cj));
            s0 = add_rn(s0, E[j0 + j]);
            s1 = add_rn(s1, E[j1 + j]);
        }
        // M over every lag so far (block max; the bound needs it for all i' <= i)
        double mloc = fmax(v0 ? s0 : 0.0, v1 ? s1 : 0.0);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mloc = fmax(mloc, __shfl_xor(mloc, o));
        if ((t & 63) == 0) mred[t >> 6] = mloc;
        __syncthreads();
        double mb = mred[0], eb = mred[WT / 64];
        for (int w = 1; w < WT / 64; ++w) {
            mb = fmax(mb, mred[w]);
            eb = fmax(eb, mred[WT / 64 + w]);
        }
        M = fmax(M, mb);
        const double Mall = M + eb;  // bounds every partial value of the recurrence
        auto decide = [&](int i, double2 e, double sn) {
            // 0 = certain FAIL, 1 = certain PASS, 2 = uncertain
            const double B = (2.0 * L + 2.0 * i + 8.0) * U * (Mall + sn) * 1.25;
            if (sn + B <= 1.0) return 0;           // n_i <= 1 for sure
            const bool norm_ok = sn - B > 1.0;     // n_i > 1 for sure
            const double r = hypot(e.x, e.y) / sqrt(sn);
            const double d = (sn - B > 0.0 ? B / (sn - B) : 1.0) * 0.5 + 16.0 * U;
            if (r * (1.0 + d) <= a.pr_level) return 0;
            if (norm_ok && r * (1.0 - d) > a.pr_level) return 1;
            return 2;
        };
        if (v0) {
            const int d0 = decide(i0, e0, s0);
            if (d0) atomicMin(best, i0);
            if (d0 == 2) atomicMin(unsure, i0);
        }
        if (v1) {
            const int d1 = decide(i1, e1, s1);
            if (d1) atomicMin(best, i1);
            if (d1 == 2) atomicMin(unsure, i1);
        }
        __syncthreads();
        found = *best;
        const int un = *unsure;
        if (found != INT_MAX) {  // uniform
            __syncthreads();     // every thread has read best/unsure
            if (un == found) return walk_preamble_exact<WT, F>(a, s, xs, c, normv, best, t);
            return found;
        }
    }
    __syncthreads();
    return found;
}

// FFT form of the certified search, run by wave 0 alone over windows of
// Q = M - L + 1 lags (M = WALK_FFT_M = 512): a window's correlations are
// e = IFFT(FFT(x) . tspec) / M over its Q + L - 1 samples (linear correlation:
// no wrap), its energies prefix sums. Lags are decided in order and the
// search stops at the window holding the first lag that is not a certain
// FAIL, so the usual step (preamble ~T2sin_size after the hit) transforms one
// window of 512 samples. The FFT result differs from the reference's in-order
// sum by at most
//   |e^ - e| <= 1024 u ||x||_2 max|tspec|   (~10x the FFT-convolution bound,
// (2 c log2 M + 1) u ||x|| ||tspec||_inf), and a window energy from two prefix
// sums from the serial recurrence by (2L + 2i + 8) u (M + s_i) + (4R + 64) u P
// (i: the lag from the search start; M >= the largest window sum plus sample
// energy of every lag so far: each window's total energy plus the largest
// sample energy), so a lag clear of both thresholds by those
// margins is decided as the reference decides it; the first lag that is not a
// certain FAIL must be a certain PASS, else the exact search runs. The other
// waves wait at the closing barrier (the transforms synchronise within the
// wave only). buf: M entries, P: M doubles (both in the search scratch).
template <int WT, int F>
__device__ int walk_preamble_fft(const WalkArgs& a, long s, double2* buf, double* P, const double2* tw_m, int* res,
                                 double2* xs, double* normv, int* best, int t)
{
    constexpr double U = 0x1.0p-53;
    constexpr int LM = WALK_FFT_LOGM, M = WALK_FFT_M, R = M / 64;
    static_assert(M == 512, "one wave: M/8 = 64 lanes");
    if (t < 64) {  // wave 0
        const int L = a.L, C = a.cycles, Q = M - L + 1;
        double mrun = 0.0, erun = 0.0;  // largest window sum / sample energy of the windows so far
        int out = INT_MAX;              // first certain PASS; -2 - lag: the first undecided lag
        constexpr double inv_m = 1.0 / M;
        const double lev2 = a.pr_level * a.pr_level;
        // One window's pass: the correlations of lags i0 .. i0 + nl - 1 by
        // the FFT in FP64 or (F32) in packed FP32, their energies from the
        // FP64 prefix sums; returns 0 when every lag is a certain FAIL, else
        // the first lag that is not, as lag + 1 (a certain PASS) or -1 - lag
        // (uncertain). The FP32 pass's transform error bound is the FP64
        // pass's with u = 2^-24 (the inputs and tspec rounded to FP32 are
        // inside its 1024 u ||x|| max|tspec| as well); its decisions are made
        // in FP64, so an uncertain lag is re-decided by the FP64 pass of the
        // same window, and only an FP64-uncertain lag goes to the exact search.
        auto pass = [&](int i0, auto f32tag) -> int {
            constexpr bool F32 = decltype(f32tag)::value;
            // opaque per-window copy of the lane: the addresses derived from
            // it are recomputed here, not hoisted out of the walk and held
            // live (spilled) across it
            int lane;
            asm volatile("v_mov_b32 %0, %1" : "=v"(lane) : "v"(t));
            const int nl = min(Q, C - i0), W = nl + L - 1;
            const long s0 = s + i0;
            double2 v[8];
            OFDM_PHASE(pre_window_load);
            load8_window<F>(a, s0, lane, W, v);
            double emax = 0.0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int k = lane + 64 * i;
                const double e2 = add_rn(mul_rn(v[i].x, v[i].x), mul_rn(v[i].y, v[i].y));
                if (k < W) P[k] = e2;
                emax = fmax(emax, e2);
            }
            wave_lds_sync();  // P visible across the wave
            // inclusive prefix sums of P: lane owns entries R*lane .. R*lane + R-1
            double ptot;
            {
                double pl[R], loc = 0.0;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int k = R * lane + r;
                    pl[r] = k < W ? P[k] : 0.0;
                    loc += pl[r];
                }
                double inc = loc;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const double y = __shfl_up(inc, o);
                    if (lane >= o) inc += y;
                }
                ptot = __shfl(inc, 63);
                double run = inc - loc;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int k = R * lane + r;
                    run += pl[r];
                    if (k < W) P[k] = run;
                }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) emax = fmax(emax, __shfl_xor(emax, o));
            OFDM_PHASE(pre_transforms);
            // Y = X . tspec (L2-resident table). The table address comes from
            // an opaque copy of the lane here: hoisted out of the walk loop,
            // the eight 64-bit addresses stayed live (and spilled) across it
            int ln;
            asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
            if constexpr (F32) {
                // the FP32 table (16 VGPRs) is requested before the forward
                // transform, so its L2 round trip hides behind it
                const float2* tp = a.tspec32 + ln;
                float2 ts[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) ts[i] = tp[64 * i];
                pf2 c[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) c[i] = pf2{(float)v[i].x, (float)v[i].y};
                fft_regs_wave32c<LM, -1>(c, lane, tw_m, buf);  // X[lane + 64 i] (its LDS syncs publish P too)
#pragma unroll
                for (int i = 0; i < 8; ++i) c[i] = c_mulw(c[i], pf2{ts[i].x, ts[i].y});
                fft_regs_wave32c<LM, +1>(c, lane, tw_m, buf);  // c[j] = M e_{i0 + lane + 64 j} (P final: synced inside)
                // parked in LDS (each lane its own entries, after its last read of the image)
#pragma unroll
                for (int j = 0; j < 8; ++j) buf[lane + 64 * j] = make_double2((double)c[j].x, (double)c[j].y);
            } else {
                fft_regs_wave<LM, -1>(v, lane, tw_m, buf);  // X[lane + 64 i] (its LDS syncs publish P too)
                const double2* tp = a.tspec + ln;
                double2 ts[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) ts[i] = tp[64 * i];
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = cmul(v[i], ts[i]);
                fft_regs_wave<LM, +1>(v, lane, tw_m, buf);  // v[j] = M e_{i0 + lane + 64 j} (P final: synced inside)
                // parked in LDS (each lane its own entries, after its last read of
                // the image), so the decisions below run as a rolled loop
#pragma unroll
                for (int j = 0; j < 8; ++j) buf[lane + 64 * j] = v[j];
            }
            OFDM_PHASE(pre_decisions);
            // every window sum of this window's lags is at most its total
            // energy (its samples lie inside the window): a bound on the
            // largest window sum without a pass over the lags
            const double mr = fmax(mrun, ptot), er = fmax(erun, emax);
            const double Mall = (mr + er) * 1.0625;
            const double scan_err = (4.0 * R + 64.0) * U * ptot;
            const double uf = F32 ? 0x1.0p-24 : U;  // the transform's unit roundoff
            const double ef = 1024.0 * uf * sqrt(ptot * 1.0625) * a.tspec_max;
            int ret = 0;
#pragma unroll 1  // rolled: it exits at the first decided lag
            for (int j = 0; j < 8; ++j) {
                const int r = lane + 64 * j, i = i0 + r;
                int d = 0;  // 0 = certain FAIL, 1 = certain PASS, 2 = uncertain
                if (r < nl) {
                    const double sn = P[r + L - 1] - (r ? P[r - 1] : 0.0);
                    const double B = (2.0 * L + 2.0 * i + 8.0) * U * (Mall + sn) * 1.25 + scan_err;
                    if (sn + B > 1.0) {  // else n_i <= 1 for sure
                        // the ratio tests squared (one sqrt, no hypot or division): the
                        // 32U / 16U slack factors cover these roundings and the
                        // reference's own (hypot, sqrt, divide)
                        const double2 e = buf[r];
                        const double ae = sqrt(e.x * e.x + e.y * e.y) * inv_m;
                        const double hi = (ae + ef) * (1.0 + 32.0 * U);
                        const double lo = fmax(ae - ef, 0.0) * (1.0 - 32.0 * U);
                        if (!(hi * hi <= lev2 * fmax(sn - B, 0x1.0p-1000) * (1.0 - 16.0 * U)))
                            d = (sn - B > 1.0 && lo * lo > lev2 * (sn + B) * (1.0 + 16.0 * U)) ? 1 : 2;
                    }
                }
                const unsigned long long hitm = __ballot(d != 0);
                if (hitm) {  // uniform: the lowest such lane is the first undecided-or-PASS lag
                    const int l0 = __ffsll((long long)hitm) - 1;
                    const int d0 = __shfl(d, l0);
                    const int lag = i0 + 64 * j + l0;
                    ret = d0 == 1 ? lag + 1 : -1 - lag;
                    break;
                }
            }
            wave_lds_sync();  // every lane is done with buf / P before the next pass overwrites them
            if (ret >= 0) {   // decided (PASS) or all FAIL: the window counts toward the bounds
                mrun = mr;
                erun = er;
            }
            return ret;
        };
        for (int i0 = 0; i0 < C && out == INT_MAX; i0 += Q) {  // uniform
            int r = a.tspec32 ? pass(i0, std::true_type{}) : -1;
            if (r < 0) r = pass(i0, std::false_type{});  // no FP32 tier, or an FP32-uncertain lag
            if (r > 0) out = r - 1;
            else if (r < 0) out = -2 - (-1 - r);
        }
        if (t == 0) *res = out;
    }
    lds_barrier();  // the answer visible to every wave
    const int found = *res;
    if (found < -1) {  // uniform: a lag within the error bounds of a threshold
        lds_barrier();  // every wave has read *res (the exact search reuses the scratch)
        return walk_preamble_exact<WT, F>(a, s, xs, a.templ, normv, best, t);
    }
    return found;
}

// Look-back (WalkArgs::lookback), thread 0 of a walker that located the frame
// with record r at pb, past its own core end and inside chunk m's core: the
// index of r in m's published records, or -1 when m's walk does not hold it
// (m published a record past pb, or finished). While m has not reached pb
// the walker waits for it, but only once m's walker has started (it marks its
// chunk WALK_PUB_STARTED: running, not merely queued or waiting for a CU
// behind another kernel's workgroups), and that walker publishes every
// record before any wait of its own, so the wait ends. Records and counts are
// stored write-through
// (sc1) by the publishing lane, which drains its stores before each count;
// every load here is an sc1 load of them.
__device__ int lookback_find(const WalkArgs& a, long pb, long r, long* prof)
{
    const long m = (pb - a.core_lo) / a.chunk;
    const long* rm = a.rec + m * a.max_rec;
    for (int spin = 0;; ++spin) {
        const int pv = __hip_atomic_load(a.pub + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // the record loads stay behind the poll
        const int cnt = min(pv & WALK_PUB_COUNT, a.max_rec);
        for (int j = 0; j < cnt; ++j) {
            const long v = __hip_atomic_load(rm + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (v == r) return j;
            if ((v < 0 ? v : (v & WALK_REC_PB)) > pb) return -1;  // m's walk passed pb without this frame
        }
        if (pv & WALK_PUB_DONE) return -1;
        if (spin >= WALK_SPIN_MAX || !(pv & WALK_PUB_STARTED))
            return -1;  // m's walker not running: walk on (always exact), and look again at the next frame
        if (prof) ++prof[4];
        __builtin_amdgcn_s_sleep(4);
    }
}

}  // namespace

// LDS of a walker: the fixed part, then the scratch (`big`) that the T2
// transforms and the preamble searches share (they run one after the other).
template <int LOGT>
struct WalkLds {
    static constexpr int WT = WalkShape<LOGT>::WT, G = WalkShape<LOGT>::G, T = WalkShape<LOGT>::T;
    static constexpr int NW = T >= 64 ? T / 64 : 1;
    static constexpr size_t FIXED = sizeof(double2) * (TwLds<LOGT>::SIZE + G * NW) + sizeof(double) * 2 * (WT / 64) +
                                    16 + sizeof(double) * 16 + sizeof(double2) * TwLds<WALK_FFT_LOGM>::SIZE;
    // scratch bytes: T2 images; FFT search (M samples + M prefix energies); exact
    // search (C + L samples + C energies); direct search (+ C + L energies + L taps)
    static size_t big(int L, int C, bool fft)
    {
        const size_t t2 = sizeof(double2) * (size_t)G * (1 << LOGT);
        const size_t fs = fft ? (sizeof(double2) + sizeof(double)) * WALK_FFT_M : 0;
        const size_t ex = sizeof(double2) * (size_t)(C + L) + sizeof(double) * C;
        const size_t di = fft ? 0 : ex + sizeof(double) * (C + L) + 16 + sizeof(double2) * L;
        return std::max(std::max(t2, fs), std::max(ex, di));
    }
};

template <int LOGT, bool I16, bool PROF = false>
__global__ void __launch_bounds__(WalkShape<LOGT>::WT, 4) stream_walk_kernel(WalkArgs a)
{
    constexpr int N = 1 << LOGT, T = N / 8, WT = WalkShape<LOGT>::WT, G = WalkShape<LOGT>::G;
    constexpr int F = I16 ? FMT_I16 : FMT_F64;
    constexpr int NW = T >= 64 ? T / 64 : 1;  // waves per transform
    // LDS: the T2 transforms and the preamble search run one after the other,
    // so their buffers alias (walk_lds_big): 4 walkers fit a CU
    extern __shared__ double2 smem[];
    double2* lds_tw = smem;
    double2* red = lds_tw + TwLds<LOGT>::SIZE;          // G * NW (tot, sine)
    double* mred = reinterpret_cast<double*>(red + G * NW);  // 2 * WT/64 maxima
    int* best = reinterpret_cast<int*>(mred + 2 * (WT / 64));
    int* bestg = best + 1;
    int* unsure = best + 2;
    double* scr = reinterpret_cast<double*>(best + 4);  // 16 scan / max scratch
    // T2 first-hit block, three slots used in turn (one barrier per scan
    // step), in scr[4..6] (the preamble search's answer is scr[2]): the
    // walker's LDS stays at 4 walkers per CU. Evaluation k collects into slot
    // k % 3 and, BEFORE its barrier, thread 0 resets slot (k + 1) % 3 for the
    // next one: every thread read that slot (evaluation k - 2's answer)
    // before evaluation k - 1's barrier, and evaluation k + 1's atomics
    // follow evaluation k's barrier. (With two slots reset after the barrier,
    // a wave running ahead into the next evaluation could post its hit before
    // a starved thread 0 reset the slot, and the hit was lost: a frame
    // skipped. Streams with exact-zero gaps, whose every zero block the FP32
    // screen sends to FP64, met it.) Every evaluation, FP64 or FP32, resets
    // both the hit and the uncertain slot of the next one: the FP64
    // re-evaluations advance the rotation too, and an uncertain slot left
    // stale by them let a later FP32 step take an uncertain (zero) block for a
    // certain T2 hit, whose failed preamble search then skipped a frame.
    int* bslot = reinterpret_cast<int*>(scr + 4);  // [0..2] first hit, [3..5] first uncertain (FP32 screen)
    double2* tw_m = reinterpret_cast<double2*>(scr + 16);  // TwLds<WALK_FFT_LOGM> (FFT search)
    double2* big = tw_m + TwLds<WALK_FFT_LOGM>::SIZE;
    double2* fftb = big;                                // G * N (T2 transforms)
    double2* xs = big;                                  // cycles + L samples (exact / direct search)
    double* normv = reinterpret_cast<double*>(xs + a.cycles + a.L);  // cycles running energies
    double* E = normv + a.cycles;                       // cycles + L energies (direct search)
    double2* ctap = reinterpret_cast<double2*>(reinterpret_cast<uintptr_t>(E + a.cycles + a.L + 1) & ~(uintptr_t)15);
    double* P = reinterpret_cast<double*>(big + WALK_FFT_M);  // a window's prefix energies (FFT search)

    int* qslot = best + 3;  // the chunk taken from the queue
    const int t0 = threadIdx.x;
    load_twiddles<LOGT>(a.t2tw, lds_tw, t0, WT);
    if (a.tspec) load_twiddles<WALK_FFT_LOGM>(a.tw_m, tw_m, t0, WT);
    if (t0 == 0) {
        *bestg = INT_MAX;
        for (int i = 0; i < 6; ++i) bslot[i] = INT_MAX;
    }
    int sl = 0;  // the slot of the next T2 evaluation (uniform; cycles 0, 1, 2)
    // chunks: the workgroup's own (its blockIdx), then from the queue until
    // it is drained (walkers that run slower on their CU take fewer); or the
    // one chunk of a re-walk launch. The first chunk takes no atomic: one
    // counter serves ~88 dequeues per us, and 2048 walkers taking their first
    // chunk from it started over ~24 us
    for (int round = 0;; ++round) {
    int c;
    if (a.queue) {
        if (round == 0) {
            c = (int)blockIdx.x;
        } else {
            if ((long)gridDim.x >= a.nchunks) break;  // uniform: no chunk left for the queue
            if (t0 == 0) *qslot = (int)gridDim.x + atomicAdd(a.queue, 1);
            __syncthreads();
            c = *qslot;
            __syncthreads();  // every thread has read the slot
        }
        if ((long)c >= a.nchunks) break;
    } else {
        if (round > 0) break;
        c = a.chunk_ids ? a.chunk_ids[blockIdx.x] : (int)blockIdx.x;
    }
    // chunk cores tile [core_lo, core_hi); chunk 0 walks in from the given
    // start state, the others from a halo before their core (look-back: none
    // by default). `end` is where the walk's exit logic applies: the chunk's
    // core end, or with look-back core_hi (a chunk walks on past its core
    // until its walk joins a later chunk's)
    const bool lb = a.lookback != 0;  // uniform
    const long core0 = a.core_lo + (long)c * a.chunk, cend = min(core0 + a.chunk, a.core_hi);
    const long end = lb ? a.core_hi : cend;
    // look-back link {chunk this walk joins, the shared frame's index here and
    // there}: none until the walk joins one
    if (lb && t0 == 0) {
        // all three words: the scratch is reused across calls of other
        // layouts, and the resolve reads them for every chunk
        a.link[3 * c] = -1;
        a.link[3 * c + 1] = 0;
        a.link[3 * c + 2] = 0;
        __hip_atomic_store(a.pub + c, WALK_PUB_STARTED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // diagnostics (a.prof): stored as they happen, nothing held in registers
#define WALK_PROF (PROF ? a.prof + (long)c * WALK_PROF_FIELDS : nullptr)
    if (long* prof = WALK_PROF; prof && t0 == 0) {
        prof[0] = (long)wall_clock64();
        prof[1] = 0;
        prof[3] = 0;
        prof[4] = 0;
        for (int i = 8; i < WALK_PROF_FIELDS; ++i) prof[i] = 0;
    }
    long pos = a.start_pos ? a.start_pos[blockIdx.x] : (c == 0 ? a.start : (core0 > a.halo ? core0 - a.halo : 0));
    const bool ring = a.ring > 0;  // uniform
    // ring mode: the first ring end after position q (the ring ends lie on
    // ring_phase + k*ring)
    auto ring_after = [&](long q) -> long {
        const long d = q - a.ring_phase;
        const long k = d >= 0 ? d / a.ring : -((-d + a.ring - 1) / a.ring);  // floor(d / ring)
        return a.ring_phase + (k + 1) * a.ring;
    };
    // the start state's ring end: given (chunk 0, re-walks), else the first
    // ring end after the halo start (a guess; the host's stitching checks it)
    long rend = 0;
    if (ring) rend = a.start_pos ? a.start_ring[blockIdx.x] : (c == 0 ? a.start_ring_end : ring_after(pos));
    int nrec = 0, ncore = 0, first_in = 0;
    long exitp = -1, exitr = 0;
    bool past = false;  // a frame at or past the core end is located
    __syncthreads();
    for (;;) {
        // opaque per-step copy of the thread index: the transforms' LDS
        // addresses are recomputed per step instead of being hoisted out of
        // the walk loop and held live (register pressure sets the walkers per CU)
        int t;
        asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"(t0));
        const int g = t / T, tt0 = t - g * T;
        // The exit state is the first walk state at or past the core end, or
        // the state whose step located the first frame past it (a re-walk of
        // the next chunk starts there). The walk goes on until it
        // has located the first frame at or past the end (within a.ext), so
        // the next chunk's first frame is in this chunk's records whenever the
        // two walks agree: a short halo then suffices to meet the true walk.
        if (pos >= end) {
            if (exitp < 0) {
                exitp = pos;
                exitr = rend;
            }
            if (past || pos >= end + a.ext) break;
        }
        OFDM_PHASE(walk_frame_top);
        const long spos = pos, srend = rend;  // this step's start state
        {
            // issue priority by the work left: walkers further from their
            // core end go first. The arbiter otherwise favours the oldest
            // resident wave, whatever its progress: equal chunks finished in
            // dispatch order (253 us for a CU's first walker, 325 us for its
            // eighth), and the CUs drained slowly (walker 386 -> 365 us)
            const long left = cend - pos, span = cend - core0 + a.halo;
            const int pr = left <= 0 ? 0 : (int)min(3L, left * 4 / max(1L, span));
            switch (__builtin_amdgcn_readfirstlane(pr)) {
                case 3: __builtin_amdgcn_s_setprio(3); break;
                case 2: __builtin_amdgcn_s_setprio(2); break;
                case 1: __builtin_amdgcn_s_setprio(1); break;
                default: __builtin_amdgcn_s_setprio(0); break;
            }
        }
        // find_t2sin(pos): blocks pos + k*N, first hit wins
        long hit = -1;
        bool stop = false;
        const long prof_t2 = PROF ? (long)wall_clock64() : 0;
        // FP64: G blocks from `base` (block g per group of T threads); the
        // first block whose ratio exceeds the level (Frame.hpp:150-197), or
        // INT_MAX. Slot sl collects the first hit; slot sl + 1 (mod 3) is reset
        // for the next evaluation before this one's barrier.
        auto t2_eval64 = [&](long base) -> int {
            // opaque per-evaluation copy of the thread's index in its group:
            // the pass addresses and bin masks are derived here, not hoisted
            // out of the scan and held live across it
            int tt;
            asm volatile("v_mov_b32 %0, %1" : "=v"(tt) : "v"(tt0));
            const long b = base + (long)g * N;
            // a block is tested when it lies in the stream (ring mode: in the
            // ring, data or zeros; blocks wholly past n are zeros and never hit)
            const bool live = ring ? (b + N <= rend && b < a.n) : b + N <= a.n;
            double2 v[8];
            if (ring && live && (b < 0 || b + N > a.n))
                load8_block_part<T, F>(a, b + tt, v);
            else
                load8_block<T, F>(a, b + tt, live, v);
            // the last pass stays in registers: v[i] = X[tt + T*i], the bins
            // this thread sums (no final LDS write, barrier and re-read); a
            // transform of T <= 64 threads lies within one wave, so its LDS
            // hand-offs need only wave-local syncs
            if constexpr (T <= 64)
                fft_regs_wave<LOGT, -1>(v, tt, lds_tw, fftb + g * N);
            else
                fft_regs<LOGT, -1>(v, tt, lds_tw, fftb + g * N);
            double tot = 0.0, sine = 0.0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int k = tt + T * i;
                const double2 z = v[i];
                const double e = z.x * z.x + z.y * z.y;
                const double m = (double)((k >= a.a1 && k <= a.b1) + (k >= a.a2 && k <= a.b2));
                tot += e;
                sine += m * e;
            }
            constexpr int W0 = T >= 64 ? 32 : T / 2;
#pragma unroll
            for (int o = W0; o > 0; o >>= 1) {
                tot += __shfl_xor(tot, o);
                sine += __shfl_xor(sine, o);
            }
            if constexpr (NW > 1) {
                if ((t & 63) == 0) red[g * NW + (tt >> 6)] = make_double2(tot, sine);
                __syncthreads();
                tot = 0.0;
                sine = 0.0;
                for (int w = 0; w < NW; ++w) {
                    tot += red[g * NW + w].x;
                    sine += red[g * NW + w].y;
                }
            }
            if (long* prof = WALK_PROF; prof && t == 0) ++prof[11];
            int* hslot = bslot + sl;
            const int nx = sl == 2 ? 0 : sl + 1;
            if (t == 0) {  // both slots of the next evaluation, whichever kind it is
                bslot[nx] = INT_MAX;
                bslot[3 + nx] = INT_MAX;
            }
            if (tt == 0 && live && tot != 0.0) {
                const double rel = sine / tot;
                if (!isnan(rel) && rel > a.t2_level) atomicMin(hslot, g);
            }
            __syncthreads();
            const int bg = *hslot;
            sl = nx;
            return bg;
        };
        // checks before a scan step from `base` (the walk state is (base, rend)):
        // 1 = stop, 2 = ring exhausted (rx.cpp:137-145: refill without carry,
        // the grid restarts at the next buffer), 0 = scan
        bool miss = false;
        auto scan_stop = [&](long base) -> int {
            // no full block left / (ring) the scan is past the capture, whose
            // zeros never hit: the walk has consumed the stream
            if (ring ? base >= a.n : base + N > a.n) return 1;
            if (base >= end) {                // scanning past the core: an equivalent state
                if (exitp < 0) {
                    exitp = base;
                    exitr = rend;
                }
                // the end fell inside a scan: walk on to the next located frame
                // (within ext_scan), so that the next chunk's walk, which
                // locates it too, syncs with this one without a re-walk
                if (base >= end + a.ext_scan) return 1;
            }
            if (ring && base + N > rend) return 2;  // find_t2sin's blocks end with the buffer
            return 0;
        };
        if constexpr (T <= 64) {
            if (a.t2_f32) {
                // FP32 screen of 2G blocks per scan step (blocks g and g + G per
                // group): half the registers and LDS of an FP64 block, so twice
                // the blocks per step at the FP64 step's cost, fewer steps per
                // frame. Certified per block: FP32 energies in the normal range
                // and a ratio clear of the level by t2_margin (>= 4x the bound
                // of the FP32 transform and sums) decide as FP64
                // does; when the first block that is not a certain FAIL is
                // uncertain, the step is evaluated again in FP64.
                float4* fftb32 = reinterpret_cast<float4*>(big);  // one image per group, both blocks
                const float lev = (float)a.t2_level, marg = (float)a.t2_margin;
                // detector-bin weights of this thread's 8 bins k = tt + T*i
                // (0, 1 or 2: Frame.hpp's mask adds the two tone ranges),
                // two bits each, built once per scan
                int mbits = 0;
                {
                    const int tm = t0 & (T - 1);
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const int k = tm + T * i;
                        mbits |= ((k >= a.a1 && k <= a.b1) + (k >= a.a2 && k <= a.b2)) << (2 * i);
                    }
                }
                for (long base = pos;; base += 2L * G * N) {
                    if (const int ss = scan_stop(base)) {
                        stop = ss == 1;
                        miss = ss == 2;
                        break;
                    }
                    int tt;  // opaque per-step copy (see t2_eval64)
                    asm volatile("v_mov_b32 %0, %1" : "=v"(tt) : "v"(tt0));
                    if (long* prof = WALK_PROF; prof && t == 0) ++prof[10];
                    OFDM_PHASE(t2_step32_load);
                    const long bA = base + (long)g * N, bB = bA + (long)G * N;
                    const bool liveA = ring ? (bA + N <= rend && bA < a.n) : bA + N <= a.n;
                    const bool liveB = ring ? (bB + N <= rend && bB < a.n) : bB + N <= a.n;
                    PCx v[8];
                    {
                        float2 va[8], vb[8];
                        if (ring && ((liveA && (bA < 0 || bA + N > a.n)) || (liveB && (bB < 0 || bB + N > a.n)))) {
                            // a block straddles the stream's ends (rare): guarded loads
                            double2 da[8], db[8];
                            load8_block_part<T, F>(a, bA + tt, da);
                            load8_block_part<T, F>(a, bB + tt, db);
#pragma unroll
                            for (int i = 0; i < 8; ++i) {
                                va[i] = liveA ? make_float2((float)da[i].x, (float)da[i].y) : make_float2(0.f, 0.f);
                                vb[i] = liveB ? make_float2((float)db[i].x, (float)db[i].y) : make_float2(0.f, 0.f);
                            }
                        } else if (F == FMT_I16 && __all(liveA && liveB)) {
                            // int16: every block of the step live (the rule), no selects
                            // (int16 walker 231 -> 228 us same box, profiles/r06/ab_walker_int16_all_live_loads.txt;
                            // the f64 instantiation spilled with it: 298 -> 303 us)
                            load8_block32<T, F>(a, bA + tt, true, va);
                            load8_block32<T, F>(a, bB + tt, true, vb);
                        } else {
                            load8_block32<T, F>(a, bA + tt, liveA, va);
                            load8_block32<T, F>(a, bB + tt, liveB, vb);
                        }
#pragma unroll
                        for (int i = 0; i < 8; ++i) v[i] = PCx{pf2{va[i].x, vb[i].x}, pf2{va[i].y, vb[i].y}};
                    }
                    OFDM_PHASE(t2_step32_fft);
                    fft_regs_wave32p<LOGT, -1>(v, tt, lds_tw, fftb32 + g * N);
                    OFDM_PHASE(t2_step32_sums);
                    // per block: total energy and detector-bin energy (packed A | B)
                    pf2 tot2 = {0.f, 0.f}, sin2 = {0.f, 0.f};
                    int mb;
                    asm volatile("v_mov_b32 %0, %1" : "=v"(mb) : "v"(mbits));
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const float m = (float)((mb >> (2 * i)) & 3);
                        const pf2 e = v[i].re * v[i].re + v[i].im * v[i].im;
                        tot2 += e;
                        sin2 += pf2{m, m} * e;
                    }
                    const float ta = group_sum<T>(tot2.x), sa = group_sum<T>(sin2.x);
                    const float tb = group_sum<T>(tot2.y), sb = group_sum<T>(sin2.y);
                    // 0 = certain FAIL, 1 = certain PASS, 2 = uncertain
                    auto screen = [&](bool live, float tot, float sine) -> int {
                        if (!live) return 0;
                        if (!(tot >= 1e-20f && tot <= 1e30f)) return 2;  // zero, tiny, huge or NaN: FP64 decides
                        const float rel = sine / tot;
                        if (rel > lev + marg) return 1;
                        if (rel <= lev - marg) return 0;
                        return 2;
                    };
                    int* hslot = bslot + sl;
                    int* uslot = bslot + 3 + sl;
                    const int nx = sl == 2 ? 0 : sl + 1;
                    if (t == 0) {
                        bslot[nx] = INT_MAX;
                        bslot[3 + nx] = INT_MAX;
                    }
                    if (tt == 0) {
                        const int da = screen(liveA, ta, sa), db = screen(liveB, tb, sb);
                        if (da) atomicMin(hslot, g);
                        if (da == 2) atomicMin(uslot, g);
                        if (db) atomicMin(hslot, g + G);
                        if (db == 2) atomicMin(uslot, g + G);
                    }
                    __syncthreads();
                    int bg = *hslot;
                    const int bu = *uslot;
                    sl = nx;
                    if (bg != INT_MAX && bu == bg) {  // uniform: this step's decision in FP64
                        bg = t2_eval64(base);
                        if (bg == INT_MAX) {
                            bg = t2_eval64(base + (long)G * N);
                            if (bg != INT_MAX) bg += G;
                        }
                    }
                    if (bg != INT_MAX) {
                        hit = base + (long)bg * N;
                        break;
                    }
                }
            }
        }
        if (!(T <= 64 && a.t2_f32)) {
            for (long base = pos;; base += (long)G * N) {
                if (const int ss = scan_stop(base)) {
                    stop = ss == 1;
                    miss = ss == 2;
                    break;
                }
                if (long* prof = WALK_PROF; prof && t == 0) ++prof[10];
                const int bg = t2_eval64(base);
                if (bg != INT_MAX) {
                    hit = base + (long)bg * N;
                    break;
                }
            }
        }
        if (long* prof = WALK_PROF; prof && t == 0) prof[8] += (long)wall_clock64() - prof_t2;
        OFDM_PHASE(walk_after_scan);
        if (stop) break;
        if (miss) {  // rx.cpp:137-145: pos = output_size of the next buffer
            pos = rend;
            rend += a.ring;
            continue;
        }
        if (ring && hit >= rend - a.out_len) rend += a.ring;  // rx.cpp:147-156: carry, next buffer
        const long prof_pre = PROF ? (long)wall_clock64() : 0;
        OFDM_PHASE(walk_preamble_call);
        const int lag = (a.tspec && !a.exact_only)
                            ? walk_preamble_fft<WT, F>(a, hit, big, P, tw_m, reinterpret_cast<int*>(scr + 2), xs, normv,
                                                    best, t)
                            : walk_preamble<WT, F>(a, hit, xs, ctap, E, normv, best, unsure, mred, t);
        if (long* prof = WALK_PROF; prof && t == 0) {
            prof[9] += (long)wall_clock64() - prof_pre;
            ++prof[12];
        }
        OFDM_PHASE(walk_record);
        // rx.cpp:160-168: find_preamble's -10 (no lag passes) moves on by a
        // message. rx.cpp tests preamble_begin < -2 in buffer coordinates,
        // where a found preamble gives >= 1; in stream coordinates a found
        // preamble may lie in the ring's zero header (pb < 0, a capture that
        // starts inside a frame), so the test is on the search result itself
        if (lag == INT_MAX) {
            pos = hit + a.msg;
            continue;
        }
        const long pb = hit + lag + 1;
        if (ring && pb >= rend - a.out_len + N) rend += a.ring;  // rx.cpp:180-189
        if (pb + a.pre + a.msg > a.n) break;  // frame not in the stream: the walk ends
        // ring mode: the state after the frame, (pb + msg, rend), is one of
        // two; the record says which (a frame before the stream's first
        // sample is kept as is: the host rejects it)
        // (rend is a ring end, so rend == ring_after(q) exactly when q lies in
        // [rend - ring, rend): no 64-bit division per frame)
        const long qn = pb + a.msg;
        const long rv = (ring && pb >= 0 && !(qn >= rend - a.ring && qn < rend)) ? (pb | WALK_REC_LAG) : pb;
        if (t == 0 && nrec < a.max_rec) {
            long* rp = a.rec + (long)c * a.max_rec + nrec;
            if (lb) {
                // published for the walkers that look back on this chunk: the
                // count of the previous record goes out now (its store landed
                // long ago: the wait is free), this record's with the next one,
                // before any look-back wait of this walker, or at the end
                if (nrec > 0) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __hip_atomic_store(a.pub + c, nrec | WALK_PUB_STARTED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                __hip_atomic_store(rp, rv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                *rp = rv;
            }
        }
        if (pb >= core0 && pb < cend) {  // in this chunk's core: one contiguous run of records
            if (ncore == 0) first_in = nrec;
            ++ncore;
        }
        if (long* prof = WALK_PROF; prof && pb >= cend && t == 0) {
            if (prof[3] == 0) prof[1] = (long)wall_clock64();
            ++prof[3];
        }
        if (lb && pb >= cend && pb < a.core_hi) {  // uniform: a frame of a later chunk's core
            if (nrec >= a.max_rec) {               // overflow: the host falls back to the halo walk
                nrec = a.max_rec + 1;
                break;
            }
            int* lbres = reinterpret_cast<int*>(scr + 8);
            if (t == 0) {
                // every record of this walk published before it waits on another
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(a.pub + c, (nrec + 1) | WALK_PUB_STARTED, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                *lbres = lookback_find(a, pb, rv, WALK_PROF);
            }
            __syncthreads();
            const int j = *lbres;
            if (j >= 0) {  // this walk joins chunk m's from this frame on: done
                if (t == 0) {
                    a.link[3 * c] = (int)((pb - a.core_lo) / a.chunk);
                    a.link[3 * c + 1] = nrec;
                    a.link[3 * c + 2] = j;
                }
                ++nrec;
                break;
            }
        }
        past = pb >= end;
        // a frame of the next core located from a state before this core's
        // end: that state is the hand-over (a re-walk from pb + msg would
        // miss the frame)
        if (past && exitp < 0) {
            exitp = spos;
            exitr = srend;
        }
        ++nrec;
        pos = pb + a.msg;  // rx.cpp:192
    }
    if (t0 == 0) {
        if (long* prof = WALK_PROF) {
            unsigned xcc, hwid;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
            prof[13] = (long)hwid;  // wave, SIMD, CU, SH, SE of this walker's first wave
            prof[2] = (long)wall_clock64();
            prof[5] = blockIdx.x;
            prof[6] = xcc & 0xf;
            prof[7] = nrec;
        }
        a.nrec[c] = nrec;
        a.exit_pos[c] = exitp;
        if (a.exit_ring) a.exit_ring[c] = exitr;
        if (a.ncore) {
            a.ncore[c] = ncore;
            a.first_in[c] = first_in;
        }
        if (lb) {
            // the walk's end: a walker still looking back on this chunk stops waiting
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(a.pub + c, min(nrec, a.max_rec) | WALK_PUB_DONE, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    }  // chunks
#undef WALK_PROF
}

__global__ void gather_kernel(GatherArgs a)
{
    const long f = blockIdx.y;
    const long s = a.starts[f];
    double2* d = a.dst + f * a.span;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < a.span; i += (long)gridDim.x * blockDim.x) {
        d[i] = stream_sample(a, s + i);
    }
}

template <int LOGT>
static size_t walk_shm(int L, int C, bool fft)
{
    return WalkLds<LOGT>::FIXED + WalkLds<LOGT>::big(L, C, fft);
}

template <int LOGT>
static hipError_t walk_launch_n(const WalkArgs& a, long nblocks, hipStream_t st)
{
    const size_t shm = walk_shm<LOGT>(a.L, a.cycles, a.tspec != nullptr);
    if (shm > 160 * 1024) return hipErrorInvalidValue;
    if ((a.iq16 != nullptr) == (a.iq != nullptr)) return hipErrorInvalidValue;  // exactly one stream format
    if constexpr (LOGT == 8) {  // the diagnostics build of the default T2 size (OFDM_WALK_PROF)
        if (a.prof) {
            const void* k = a.iq16 ? (const void*)stream_walk_kernel<LOGT, true, true>
                                   : (const void*)stream_walk_kernel<LOGT, false, true>;
            lds_opt_in(k, 160 * 1024);
            if (a.iq16)
                hipLaunchKernelGGL((stream_walk_kernel<LOGT, true, true>), dim3((unsigned)nblocks),
                                   dim3(WalkShape<LOGT>::WT), shm, st, a);
            else
                hipLaunchKernelGGL((stream_walk_kernel<LOGT, false, true>), dim3((unsigned)nblocks),
                                   dim3(WalkShape<LOGT>::WT), shm, st, a);
            return hipGetLastError();
        }
    }
    if (a.iq16) {
        lds_opt_in((const void*)stream_walk_kernel<LOGT, true>, 160 * 1024);
        hipLaunchKernelGGL((stream_walk_kernel<LOGT, true>), dim3((unsigned)nblocks), dim3(WalkShape<LOGT>::WT), shm,
                           st, a);
    } else {
        lds_opt_in((const void*)stream_walk_kernel<LOGT, false>, 160 * 1024);
        hipLaunchKernelGGL((stream_walk_kernel<LOGT, false>), dim3((unsigned)nblocks), dim3(WalkShape<LOGT>::WT), shm,
                           st, a);
    }
    return hipGetLastError();
}

template <int LOGT>
static long walk_slots_n(int L, int C, bool fft)
{
    int dev = 0, ncu = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    static std::mutex mu;           // contexts on several host threads query it
    static long cache[64][4] = {};  // device: {L, C, fft, slots} of the last query
    std::lock_guard<std::mutex> g(mu);
    long* q = cache[dev];
    if (q[3] && q[0] == L && q[1] == C && q[2] == (long)fft) return q[3];
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
    // the fewer resident walkers of the two format instantiations: the
    // chunking does not depend on the stream's format
    for (const void* k : {(const void*)stream_walk_kernel<LOGT, false>, (const void*)stream_walk_kernel<LOGT, true>}) {
        int pk = 0;
        lds_opt_in(k, 160 * 1024);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pk, k, WalkShape<LOGT>::WT, walk_shm<LOGT>(L, C, fft)) !=
                hipSuccess ||
            pk <= 0)
            pk = 1;
        per = per ? std::min(per, pk) : pk;
    }
    q[0] = L;
    q[1] = C;
    q[2] = fft;
    q[3] = (long)per * ncu;
    return q[3];
}

long stream_walk_slots(int logt, int L, int C, bool fft)
{
    switch (logt) {
        case 6: return walk_slots_n<6>(L, C, fft);
        case 7: return walk_slots_n<7>(L, C, fft);
        case 8: return walk_slots_n<8>(L, C, fft);
        case 9: return walk_slots_n<9>(L, C, fft);
        case 10: return walk_slots_n<10>(L, C, fft);
        case 11: return walk_slots_n<11>(L, C, fft);
        default: return 256;
    }
}

hipError_t launch_stream_walk(int logt, const WalkArgs& a, long nblocks, hipStream_t st)
{
    if (nblocks <= 0) return hipSuccess;
    switch (logt) {
        case 6: return walk_launch_n<6>(a, nblocks, st);
        case 7: return walk_launch_n<7>(a, nblocks, st);
        case 8: return walk_launch_n<8>(a, nblocks, st);
        case 9: return walk_launch_n<9>(a, nblocks, st);
        case 10: return walk_launch_n<10>(a, nblocks, st);
        case 11: return walk_launch_n<11>(a, nblocks, st);
        default: return hipErrorInvalidValue;
    }
}

// Blocks of 1024 x CPT chunks (CPT consecutive chunks per thread; 2048
// chunks are one block): every workgroup scans their in-core record counts
// (exclusive), then each output slot finds its chunk by binary search over the
// scan; the slots are spread over the workgroups (G per thread, gathered
// before any is stored, so the loads overlap).
__global__ void __launch_bounds__(1024) compact_kernel(CompactArgs a)
{
    constexpr int CPT = 4, G = 2, NB = 1024 * CPT;
    __shared__ int excl[NB];  // exclusive scan of the block's counts
    __shared__ int srcb[NB];  // rec index of each chunk's first in-core record
    __shared__ long wsum[16];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const long* __restrict__ rec = a.rec;
    long base = 0;
    for (long k0 = 0; k0 < a.nchunks; k0 += NB) {
        // only stored records: an overflowing walk (nrec > max_rec) kept the
        // first max_rec, the host rejects it, and nothing past them is read
        // branch-free: every thread loads its (clamped) chunks' counts
        // together (loads under a per-chunk branch were waited one by one)
        int cnt[CPT], fiv[CPT], ncv[CPT], mine = 0;
#pragma unroll
        for (int u = 0; u < CPT; ++u) {
            const long k = min(k0 + (long)t * CPT + u, a.nchunks - 1);
            fiv[u] = a.first_in[k];
            ncv[u] = a.ncore[k];
        }
#pragma unroll
        for (int u = 0; u < CPT; ++u) {
            const long k = k0 + (long)t * CPT + u;
            const bool in = k < a.nchunks;
            cnt[u] = in ? max(0, min(ncv[u], a.max_rec - fiv[u])) : 0;
            srcb[t * CPT + u] = in ? (int)(k * a.max_rec + fiv[u]) : 0;
            mine += cnt[u];
        }
        int inc = mine;  // inclusive scan: wave, then wave totals
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(inc, o);
            if (lane >= o) inc += y;
        }
        if (lane == 63) wsum[w] = inc;
        __syncthreads();
        int off = inc - mine;
        for (int u = 0; u < w; ++u) off += (int)wsum[u];
        long tot = 0;
        for (int u = 0; u < 16; ++u) tot += wsum[u];
#pragma unroll
        for (int u = 0; u < CPT; ++u) {
            excl[t * CPT + u] = off;
            off += cnt[u];
        }
        __syncthreads();
        const int nb = (int)min((long)NB, a.nchunks - k0);
        for (long i0 = (long)blockIdx.x * 1024 * G; i0 < tot; i0 += (long)gridDim.x * 1024 * G) {
            long pbv[G];
            // branch-free (a load inside a per-slot branch waits before the
            // next is issued): every slot searches and loads, clamped
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const long idx0 = i0 + g * 1024 + t;
                const int idx = (int)(idx0 < tot ? idx0 : tot - 1);
                int lo = 0, hi = nb;  // last j with excl[j] <= idx
#pragma unroll
                for (int it = 0; it < 13; ++it) {  // nb <= 4096 = 2^12: 13 halvings reach hi - lo == 1
                    const int mid = (lo + hi) >> 1;
                    const bool go = hi - lo > 1;
                    const bool le = excl[mid] <= idx;
                    lo = go && le ? mid : lo;
                    hi = go && !le ? mid : hi;
                }
                pbv[g] = rec[srcb[lo] + (idx - excl[lo])] & WALK_REC_PB;
            }
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const long idx = i0 + g * 1024 + t, out = base + idx;
                if (idx < tot && out < a.cap) {
                    a.list[out] = pbv[g];
                    if (a.list2) a.list2[out] = pbv[g];
                }
            }
        }
        base += tot;
        __syncthreads();  // excl / srcb / wsum are rewritten by the next block
    }
    if (t == 0 && blockIdx.x == 0) {
        *a.count = base;
        if (a.queue_reset) *a.queue_reset = 0;
    }
}

hipError_t launch_compact(const CompactArgs& a, hipStream_t st)
{
    // every block scans the counts; the output slots are spread over the
    // blocks (one CU's LDS was the limit: 16 binary searches per thread there)
    const long nb = std::max(1L, std::min(64L, (a.cap + 2047) / 2048));
    hipLaunchKernelGGL(compact_kernel, dim3((unsigned)nb), dim3(1024), 0, st, a);
    return hipGetLastError();
}

// Look-back resolution (ResolveArgs). Every workgroup resolves the chain in
// LDS (a few KB of links), then writes its share of the owned frames.
//  - next[c] = the chunk c's walk joined (nchunks: none). Chunk 0's walk is
//    true; a chain chunk's walk is true from its entry frame, so the chain
//    0 -> next -> next ... is the sequential walk.
//  - c is certainly on the chain when no chunk before it jumps past it
//    (prefix max of next <= c: the increasing chain cannot step over c). These
//    anchors are found by one scan; from each anchor one thread follows next
//    to the following anchor, marking the chain chunks between (usually none)
//    and setting each one's entry index from its predecessor's link.
//  - each chain chunk contributes records [entry, shared frame) (the last: to
//    its walk's end), trimmed to [own_lo, own_hi): only chunk 0 holds walk-in
//    records and only the last chain chunk records past own_hi.
__global__ void __launch_bounds__(1024) resolve_kernel(ResolveArgs a)
{
    constexpr int NT = 1024, NC = RESOLVE_MAX_CHUNKS, UP = NC / NT, G = 2, TR = 8;
    __shared__ int nxt[NC];   // the chunk c's walk joins (C: none)
    __shared__ int jx[NC];    // its entry index there; after the chain pass, the owned-count scan
    __shared__ int sege[NC];  // segment end (the shared frame; back-trimmed) | back trim << 16 | SEG_OVF
    constexpr int SEG_OVF = 1 << 30;
    __shared__ int ent[NC];   // entry index; after the trim, the first owned record
    __shared__ unsigned char anc[NC], onc[NC];
    __shared__ long wsum[NT / 64];
    __shared__ int wmax[NT / 64];
    __shared__ int sflags, sfront, sneg;
    __shared__ long sexit[2];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int C = (int)a.nchunks, MR = a.max_rec;
    auto rpb = [](long r) { return r < 0 ? r : (r & WALK_REC_PB); };
    if (t == 0) {
        sflags = 0;
        sfront = 0;
        sneg = 0;
        sexit[0] = -1;
        sexit[1] = 0;
    }
    // 1. every global read of the chain pass at once: links and counts
    // (chunks t + NT*u, coalesced), then the few records the trims need
    int lm[UP], li[UP], lj[UP], nr[UP];
#pragma unroll
    for (int u = 0; u < UP; ++u) {
        const int c = min(t + NT * u, C - 1);
        lm[u] = a.link[3 * c];
        li[u] = a.link[3 * c + 1];
        lj[u] = a.link[3 * c + 2];
        nr[u] = a.nrec[c];
    }
    __syncthreads();  // sflags / sfront initialised
#pragma unroll
    for (int u = 0; u < UP; ++u) {
        const int c = t + NT * u;
        if (c >= C) continue;
        const bool ovf = nr[u] > MR;
        // an overflowed walk joins nothing; as c + 1 it hides no later anchor
        nxt[c] = ovf ? c + 1 : (lm[u] >= 0 ? lm[u] : C);
        jx[c] = (lm[u] >= 0 && !ovf) ? lj[u] : 0;  // the link's entry index only where it joined
        onc[c] = 0;
        int e = (lm[u] >= 0 && !ovf) ? li[u] : min(nr[u], MR), bt = 0;
        const long* rc = a.rec + (long)c * MR;
        if (c == 0) {  // walk-in records before own_lo (records rise along the walk)
            long r[TR];
#pragma unroll
            for (int k = 0; k < TR; ++k) r[k] = rc[min(k, max(e - 1, 0))];
            int f = 0, ng = 0;
#pragma unroll
            for (int k = 0; k < TR; ++k) {
                f += (k < e && rpb(r[k]) < a.own_lo) ? 1 : 0;
                ng += (k < e && rpb(r[k]) >= a.own_lo && rpb(r[k]) < 0) ? 1 : 0;
            }
            sneg = ng;  // owned frames before the stream's first sample (a prefix of the list)
            if (ng) atomicOr(&sflags, RESOLVE_NEG_FRAME);
            while (f >= TR && f < e && rpb(rc[f]) < a.own_lo) ++f;  // longer walk-ins (rare)
            sfront = f;
        }
        if (lm[u] < 0 && !ovf) {  // a walk that ended: the chain's last chunk if on it; records past own_hi
            long r[TR];
#pragma unroll
            for (int k = 0; k < TR; ++k) r[k] = rc[max(e - 1 - k, 0)];
#pragma unroll
            for (int k = 0; k < TR; ++k) bt += (bt == k && k < e && rpb(r[k]) >= a.own_hi) ? 1 : 0;
            while (bt < e && bt >= TR && rpb(rc[e - 1 - bt]) >= a.own_hi) ++bt;
        }
        sege[c] = (e - bt) | (bt << 16) | (ovf ? SEG_OVF : 0);
    }
    __syncthreads();
    // 2. anchors: chunk c is on the chain when no chunk before it jumps past
    // it (exclusive prefix max of nxt <= c), contiguous chunks per thread
    const int CPT = (C + NT - 1) / NT, c0 = t * CPT;
    int tm = 0;
    for (int u = 0; u < CPT; ++u)
        if (c0 + u < C) tm = max(tm, nxt[c0 + u]);
    int inc = tm;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(inc, o);
        if (lane >= o) inc = max(inc, y);
    }
    if (lane == 63) wmax[w] = inc;
    __syncthreads();
    int pm = __shfl_up(inc, 1);
    if (lane == 0) pm = 0;
    for (int u = 0; u < w; ++u) pm = max(pm, wmax[u]);
    for (int u = 0; u < CPT; ++u) {
        const int c = c0 + u;
        if (c < C) {
            const bool an = c == 0 || pm <= c;
            anc[c] = an;
            if (an) onc[c] = 1;
            pm = max(pm, nxt[c]);
        }
    }
    if (t == 0) ent[0] = 0;
    __syncthreads();
    // 3. from each anchor, the chain to the next anchor (usually one step)
    for (int u = 0; u < CPT; ++u) {
        const int c = c0 + u;
        if (c < C && anc[c]) {
            for (int x = c;;) {
                const int y = nxt[x];
                if (y >= C) break;
                ent[y] = jx[x];
                onc[y] = 1;
                if (anc[y]) break;
                x = y;
            }
        }
    }
    __syncthreads();
    // 4. each chain chunk's owned records: [entry, shared frame) trimmed to
    // [own_lo, own_hi) (walk-in: chunk 0; past own_hi: the last chain chunk)
    long own = 0, chn = 0;
    int cnt[RESOLVE_MAX_CHUNKS / NT], fi[RESOLVE_MAX_CHUNKS / NT];
#pragma unroll
    for (int u = 0; u < UP; ++u) {
        const int c = c0 + u;
        cnt[u] = fi[u] = 0;
        if (u < CPT && c < C && onc[c]) {
            const int se = sege[c], e = se & 0xffff, bt = (se >> 16) & 0x3fff;
            if (se & SEG_OVF) atomicOr(&sflags, RESOLVE_OVERFLOW);  // its records are incomplete
            const int b0 = min(ent[c], e), b = c == 0 ? max(b0, sfront) : b0;
            cnt[u] = max(0, e - b);
            fi[u] = b;
            chn += max(0, e + bt - b0);
            if (nxt[c] >= C) {  // the chain's last chunk: its walk's exit state is the walk's
                sexit[0] = a.exit_pos[c];
                sexit[1] = a.exit_ring ? a.exit_ring[c] : 0;
            }
        }
        own += cnt[u];
    }
    // block scan of (chain records << 32 | owned) in chunk order
    const long v = (chn << 32) | own;
    long vi = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long y = __shfl_up(vi, o);
        if (lane >= o) vi += y;
    }
    if (lane == 63) wsum[w] = vi;
    __syncthreads();  // also: every thread is done with jx (reused for the scan)
    long off = vi - v, tot = 0;
    for (int u = 0; u < NT / 64; ++u) {
        if (u < w) off += wsum[u];
        tot += wsum[u];
    }
    const long tot_own = tot & 0xffffffffL, tot_chn = tot >> 32;
    long oo = off & 0xffffffffL, oc = off >> 32;
#pragma unroll
    for (int u = 0; u < UP; ++u) {
        const int c = c0 + u;
        if (u < CPT && c < C) {
            jx[c] = (int)oo;
            ent[c] = fi[u];
            if (blockIdx.x == 0 && a.chain && onc[c]) {
                // the walk's first chain_head and last chain_tail records
                // (shard reports): chain index q goes to q (head) or to
                // chain_head + q - (tot - chain_tail) (tail); only the
                // chunks holding those write
                const long* rc = a.rec + (long)c * MR;
                const int se = sege[c], kb = c == 0 ? 0 : fi[u], ke = (se & 0xffff) + ((se >> 16) & 0x3fff);
                const long tl = max(a.chain_head, tot_chn - a.chain_tail);  // first tail index
                for (int k = kb; k < ke; ++k, ++oc) {
                    if (oc < a.chain_head) a.chain[oc] = rc[k];
                    else if (oc >= tl) a.chain[a.chain_head + (oc - tl)] = rc[k];
                    else {  // skip the middle of this chunk's run
                        const long skip = min((long)(ke - k), tl - oc) - 1;
                        k += (int)skip;
                        oc += skip;
                    }
                }
            }
        }
        oo += cnt[u];
    }
    __syncthreads();
    // An overflowed chain chunk's records are incomplete: no list and a zero
    // count, so the decode enqueued behind this kernel (the host has not read
    // the flags yet) does nothing, and the host's halo walk writes every output
    const bool overflow = (sflags & RESOLVE_OVERFLOW) != 0;  // uniform (set before the scan's barrier)
    // 5. owned slots, spread over the workgroups: slot -> its chunk by binary
    // search over the scan (last chunk with scan <= slot), then the record
    const long lim = overflow ? 0 : min(tot_own, a.cap);
    for (long i0 = (long)blockIdx.x * NT * G; i0 < lim; i0 += (long)gridDim.x * NT * G) {
        long pbv[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const long idx0 = i0 + g * NT + t;
            const int idx = (int)(idx0 < lim ? idx0 : lim - 1);
            int lo = 0, hi = C;
#pragma unroll
            for (int it = 0; it < 14; ++it) {  // C <= 8192 = 2^13
                const int mid = (lo + hi) >> 1;
                const bool go = hi - lo > 1;
                const bool le = jx[mid] <= idx;
                lo = go && le ? mid : lo;
                hi = go && !le ? mid : hi;
            }
            pbv[g] = rpb(a.rec[(long)lo * MR + ent[lo] + (idx - jx[lo])]);
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const long idx = i0 + g * NT + t;
            if (idx < lim) {
                a.list[idx] = pbv[g];
                if (a.list2) a.list2[idx] = pbv[g];
            }
        }
    }
    if (blockIdx.x == 0) {
        // the walkers' publication counts and chunk counter, zero for the next call
        for (int c = t; c < C; c += NT) a.pub[c] = 0;
        if (t == 0) {
            *a.count = overflow ? 0 : tot_own;
            if (a.queue_reset) *a.queue_reset = 0;
            // page-locked status the host polls: the fields, a system-scope
            // release, then the flags word it waits on (-1 until then)
            a.status[0] = tot_own;
            a.status[2] = sexit[0];
            a.status[3] = sexit[1];
            a.status[4] = tot_chn;
            a.status[5] = sneg;
            __threadfence_system();
            __hip_atomic_store(a.status + 1, (long)sflags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __threadfence_system();
        }
    }
}

hipError_t launch_resolve(const ResolveArgs& a, hipStream_t st)
{
    if (a.nchunks < 1 || a.nchunks > RESOLVE_MAX_CHUNKS) return hipErrorInvalidValue;
    const long nb = std::max(1L, std::min(64L, (a.cap + 2047) / 2048));
    hipLaunchKernelGGL(resolve_kernel, dim3((unsigned)nb), dim3(1024), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_gather(const GatherArgs& a, hipStream_t st)
{
    if (a.nframes <= 0) return hipSuccess;
    const long per = (a.span + 255) / 256;
    const unsigned gx = (unsigned)(per < 64 ? per : 64);
    hipLaunchKernelGGL(gather_kernel, dim3(gx, (unsigned)a.nframes), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace ofdm

