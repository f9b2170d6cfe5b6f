/*
 * ofdm_oracle.c — TEST INFRASTRUCTURE ONLY (see ofdm_oracle.h).
 *
 * Plain-C restatement of the reference modem path, one function per reference
 * member, each citing the reference file:line it follows (paths relative to the
 * reference root). Arithmetic deliberately uses C99 `double complex`, whose
 * multiply/divide are GCC's __muldc3/__divdc3 — the same code the reference's
 * std::complex<double> compiles to — and the same libm calls (cabs=hypot,
 * carg=atan2, cexp). Build with -ffp-contract=off (x86-64 baseline, as the
 * reference's `g++ -O3 -m64` has no FMA).
 */
#include "ofdm_oracle.h"

#include <complex.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

typedef double complex cplx;

static int imin(int a, int b) { return a < b ? a : b; }
static int imax(int a, int b) { return a > b ? a : b; }

/* ------------------------------------------------------------------------ */
/* Modulation — OFDM/modulation.cpp                                          */
/* ------------------------------------------------------------------------ */

/* psk() modulation.cpp:4-9 with angle 5π/4, deg 2; qam() modulation.cpp:12-20;
 * table built in Modulation::Modulation modulation.cpp:23-36. */
int orc_constellation(int k, double* outd)
{
    cplx* out = (cplx*)outd;
    int n = 1 << k;
    if (k == 1) {
        double step = M_PI * 2 / (double)2;
        for (int i = 0; i < n; i++) {
            /* j*(step*complex(i) + angle) = (0, step*i + angle) */
            double a = step * (double)i + M_PI_4 * 5;
            out[i] = cexp(CMPLX(0.0, a));
        }
    } else {
        if ((k % 2) || k > 8) {
            for (int i = 0; i < n; i++) out[i] = 0;
            return n;
        }
        unsigned num = 1u << (k / 2);
        for (int i = 0; i < n; i++) {
            uint8_t in = (uint8_t)i;
            out[i] = CMPLX(2.0 / (num - 1) * (double)(in % num) - 1.0,
                           2.0 / (num - 1) * (double)(in >> (k / 2)) - 1.0);
        }
    }
    return n;
}

/* Modulation::bit_stream_converter, modulation.cpp:90-125 (MSB-first repack,
 * last output left-shifted to pad). Returns output length. */
size_t orc_bit_convert(int out_bits, int in_bits, const uint8_t* in, size_t len, uint8_t* out)
{
    size_t total = (size_t)in_bits * len;
    size_t out_len = total / out_bits + (total % out_bits > 0);
    memset(out, 0, out_len);
    if (len == 0) return out_len;
    size_t oi = 0, ii = 0;
    uint8_t mask = (uint8_t)(1u << (in_bits - 1));
    for (size_t i = 0, j = 0; i < total; i++) {
        if (j == (size_t)out_bits) {
            j = 0;
            oi++;
        }
        j++;
        out[oi] = (uint8_t)(out[oi] << 1);
        if ((mask & in[ii]) > 0) out[oi]++;
        mask >>= 1;
        if (mask == 0) {
            mask = (uint8_t)(1u << (in_bits - 1));
            ii++;
        }
    }
    if (total % out_bits > 0)
        out[out_len - 1] = (uint8_t)(out[out_len - 1] << (out_bits - total % out_bits));
    return out_len;
}

/* Modulation::mod, modulation.cpp:39-50. */
size_t orc_mod(int k, const uint8_t* bytes, size_t nbytes, double* outd)
{
    cplx* out = (cplx*)outd;
    cplx table[256];
    orc_constellation(k, (double*)table);
    size_t nsym = (nbytes * 8) / k + ((nbytes * 8) % k > 0);
    uint8_t* sym = (uint8_t*)malloc(nsym ? nsym : 1);
    orc_bit_convert(k, 8, bytes, nbytes, sym);
    for (size_t i = 0; i < nsym; i++) out[i] = table[sym[i]];
    free(sym);
    return nsym;
}

/* Modulation::demod, modulation.cpp:53-87. QAM clamps the caller's buffer in
 * place (modulation.cpp:70-75), exactly as the reference. Returns byte count. */
size_t orc_demod(int k, double* pointsd, size_t n, uint8_t* out)
{
    cplx* pts = (cplx*)pointsd;
    uint8_t* dec = (uint8_t*)malloc(n ? n : 1);
    if (k == 1) {
        for (size_t i = 0; i < n; i++) dec[i] = (uint8_t)(creal(pts[i]) + cimag(pts[i]) > 0);
    } else {
        uint8_t str_size = (uint8_t)(1u << (k / 2));
        double step = 2.0 / (str_size - 1);
        double str_size_1 = 1.0 / step;
        for (size_t i = 0; i < n; i++) {
            double re = creal(pts[i]), im = cimag(pts[i]);
            re = re < -1.0 ? -1.0 : (1.0 < re ? 1.0 : re); /* std::clamp */
            im = im < -1.0 ? -1.0 : (1.0 < im ? 1.0 : im);
            pts[i] = CMPLX(re, im);
        }
        for (size_t i = 0; i < n; i++) {
            double re = creal(pts[i]), im = cimag(pts[i]);
            int v = (uint8_t)((re + 1.0) * str_size_1 + 0.5) |
                    (uint8_t)((im + 1.0) * str_size_1 + 0.5) * str_size;
            dec[i] = (uint8_t)v;
        }
    }
    size_t nb = orc_bit_convert(8, k, dec, n, out);
    free(dec);
    return nb;
}

/* ------------------------------------------------------------------------ */
/* FFT: FFTW's unnormalised DFT definition (fftw3 doc: FFTW_FORWARD = -1,   */
/* FFTW_BACKWARD = +1 in the exponent), independent mixed-radix DIT.        */
/* ------------------------------------------------------------------------ */

typedef struct {
    int n, sign;
    cplx* w;
} tw_cache;

static __thread tw_cache g_tw[4];
static __thread int g_tw_next;
static __thread cplx* g_scratch;
static __thread int g_scratch_n;

static const cplx* twiddles(int n, int sign)
{
    for (int i = 0; i < 4; i++)
        if (g_tw[i].w && g_tw[i].n == n && g_tw[i].sign == sign) return g_tw[i].w;
    tw_cache* c = &g_tw[g_tw_next];
    g_tw_next = (g_tw_next + 1) & 3;
    free(c->w);
    c->w = (cplx*)malloc(sizeof(cplx) * n);
    c->n = n;
    c->sign = sign;
    for (int j = 0; j < n; j++) {
        double a = 2.0 * M_PI * (double)j / (double)n;
        c->w[j] = CMPLX(cos(a), sign * sin(a));
    }
    return c->w;
}

static int smallest_factor(int n)
{
    if (n % 4 == 0) return 4;
    if (n % 2 == 0) return 2;
    for (int p = 3; p * p <= n; p += 2)
        if (n % p == 0) return p;
    return n;
}

/* out[k] = sum_t in[t*is] W^{tk}; W table for size ntop. */
static void dft_rec(const cplx* in, long is, cplx* out, int n, const cplx* W, int ntop)
{
    if (n == 1) {
        out[0] = in[0];
        return;
    }
    int p = smallest_factor(n);
    int m = n / p;
    int ws = ntop / n; /* W_n^j = W[j*ws] */
    if (p == n) {      /* prime: direct DFT */
        cplx tmp[64];
        cplx* t = n <= 64 ? tmp : (cplx*)malloc(sizeof(cplx) * n);
        for (int k = 0; k < n; k++) {
            cplx acc = 0;
            for (int q = 0; q < n; q++) acc += in[q * is] * W[((long)q * k % n) * ws];
            t[k] = acc;
        }
        for (int k = 0; k < n; k++) out[k] = t[k];
        if (t != tmp) free(t);
        return;
    }
    for (int q = 0; q < p; q++) dft_rec(in + q * is, is * p, out + q * m, m, W, ntop);
    if (p == 2) {
        for (int k = 0; k < m; k++) {
            cplx t0 = out[k];
            cplx t1 = out[k + m] * W[k * ws];
            out[k] = t0 + t1;
            out[k + m] = t0 - t1;
        }
    } else if (p == 4) {
        /* W_4 = W[ntop/4] = sign*i exactly (cos(pi/2) rounding aside) */
        int sgn = cimag(W[ntop / 4]) > 0 ? 1 : -1;
        for (int k = 0; k < m; k++) {
            cplx t0 = out[k];
            cplx t1 = out[k + m] * W[k * ws];
            cplx t2 = out[k + 2 * m] * W[2 * k * ws];
            cplx t3 = out[k + 3 * m] * W[3 * k * ws];
            cplx a = t0 + t2, b = t0 - t2, c = t1 + t3, d = t1 - t3;
            cplx jd = sgn > 0 ? CMPLX(-cimag(d), creal(d)) : CMPLX(cimag(d), -creal(d));
            out[k] = a + c;
            out[k + m] = b + jd;
            out[k + 2 * m] = a - c;
            out[k + 3 * m] = b - jd;
        }
    } else {
        cplx tmp[64];
        cplx* t = p <= 64 ? tmp : (cplx*)malloc(sizeof(cplx) * p);
        for (int k = 0; k < m; k++) {
            for (int q = 0; q < p; q++) t[q] = out[k + q * m] * W[((long)q * k % n) * ws];
            for (int r = 0; r < p; r++) {
                cplx acc = 0;
                for (int q = 0; q < p; q++) acc += t[q] * W[((long)q * r % p) * (ntop / p)];
                out[k + r * m] = acc;
            }
        }
        if (t != tmp) free(t);
    }
}

void orc_fft(double* xd, int n, int sign)
{
    cplx* x = (cplx*)xd;
    if (n <= 1) return;
    if (g_scratch_n < n) {
        free(g_scratch);
        g_scratch = (cplx*)malloc(sizeof(cplx) * n);
        g_scratch_n = n;
    }
    memcpy(g_scratch, x, sizeof(cplx) * n);
    dft_rec(g_scratch, 1, x, n, twiddles(n, sign), n);
}

/* ------------------------------------------------------------------------ */
/* FFT_FORM — OFDM/Frame.cpp:4-96                                            */
/* ------------------------------------------------------------------------ */

/* Pilot / segment layout, FFT_FORM ctor Frame.cpp:31-44. */
void orc_layout(int N, int D, int P, int* pilot_bin, int* seg_start)
{
    int step = D / P + 1, seg = step - 1, half = P / 2;
    int j = 0;
    for (int pos = 1 + seg; j < half; j++, pos += step) {
        pilot_bin[j] = pos;
        seg_start[j] = pos - seg;
    }
    for (int pos = N - step * half; j < P; j++, pos += step) {
        pilot_bin[j] = pos;
        seg_start[j] = pos + 1;
    }
}

/* FFT_FORM::write, Frame.cpp:54-70: zero, pilots = pilot_ampl, scatter
 * segments, batched backward DFT, /sqrt(N). out: N*S complex. */
void orc_fft_write(int N, int D, int P, int S, double ampl, const double* ind, double* outd)
{
    const cplx* in = (const cplx*)ind;
    cplx* buf = (cplx*)outd;
    int seg = D / P;
    int* pil = (int*)malloc(sizeof(int) * P * 2);
    int* sst = pil + P;
    orc_layout(N, D, P, pil, sst);
    memset(buf, 0, sizeof(cplx) * N * S);
    for (int s = 0; s < S; s++)
        for (int j = 0; j < P; j++) buf[(long)s * N + pil[j]] = CMPLX(ampl, 0.0);
    for (long i = 0; i < (long)P * S; i++) {
        long s = i / P, j = i % P;
        memcpy(buf + s * N + sst[j], in + i * seg, sizeof(cplx) * seg);
    }
    double norm_factor = sqrt((double)N);
    for (int s = 0; s < S; s++) orc_fft((double*)(buf + (long)s * N), N, +1);
    for (long i = 0; i < (long)N * S; i++) buf[i] = buf[i] / norm_factor;
    free(pil);
}

/* FFT_FORM::read, Frame.cpp:73-96: forward DFT per symbol, global pilot
 * amplitude normalisation, per-segment equalisation vs symbol 0's pilots.
 * buf (N*S, modified in place like FFT_buf); out: (D/P)*P*S complex. */
void orc_fft_read(int N, int D, int P, int S, double ampl, double* bufd, double* outd)
{
    cplx* buf = (cplx*)bufd;
    cplx* out = (cplx*)outd;
    int seg = D / P;
    int* pil = (int*)malloc(sizeof(int) * P * 2);
    int* sst = pil + P;
    orc_layout(N, D, P, pil, sst);
    for (int s = 0; s < S; s++) orc_fft((double*)(buf + (long)s * N), N, -1);
    double phys = 0.0;
    for (int s = 0; s < S; s++)
        for (int j = 0; j < P; j++) phys += cabs(buf[(long)s * N + pil[j]]);
    phys /= (double)((size_t)P * (size_t)S) * ampl;
    for (long i = 0; i < (long)N * S; i++) buf[i] = buf[i] / phys;
    for (long i = 0; i < (long)P * S; i++) {
        long s = i / P, j = i % P;
        cplx* o = out + i * seg;
        memcpy(o, buf + s * N + sst[j], sizeof(cplx) * seg);
        cplx coef = buf[s * N + pil[j]] / buf[pil[j]];
        for (int t = 0; t < seg; t++) o[t] = o[t] / coef;
    }
    free(pil);
}

/* ------------------------------------------------------------------------ */
/* OFDM_FORM — Frame.cpp:157-208, Frame.hpp:238-348                          */
/* ------------------------------------------------------------------------ */

/* OFDM_FORM::write, Frame.cpp:185-198 (mod -> FFT_FORM::write -> body after
 * CP -> CP = last cp samples). out: S*(N+cp) complex. */
void orc_ofdm_write(const ofdm_params* p, int S, int k, const uint8_t* bytes, double* outd)
{
    int N = (int)p->fft_size, D = (int)p->num_data_subc, P = (int)p->num_pilot_subc;
    int cp = (int)p->cp_size, L = N + cp;
    size_t nbytes = (size_t)D * S * k / 8;
    size_t npts = (nbytes * 8) / k + 1;
    cplx* pts = (cplx*)calloc(npts > (size_t)D * S ? npts : (size_t)D * S, sizeof(cplx));
    orc_mod(k, bytes, nbytes, (double*)pts);
    cplx* fbuf = (cplx*)malloc(sizeof(cplx) * N * S);
    orc_fft_write(N, D, P, S, (double)p->pilot_ampl / 1000, (double*)pts, (double*)fbuf);
    cplx* out = (cplx*)outd;
    for (int s = 0; s < S; s++) {
        memcpy(out + (long)s * L + cp, fbuf + (long)s * N, sizeof(cplx) * N);
        memcpy(out + (long)s * L, out + (long)s * L + N, sizeof(cplx) * cp);
    }
    free(fbuf);
    free(pts);
}

/* OFDM_FORM::fft, Frame.hpp:276-282: CP strip then FFT_FORM::read. */
void orc_ofdm_fft(const ofdm_params* p, int S, const double* ind, double* outd)
{
    int N = (int)p->fft_size, cp = (int)p->cp_size, L = N + cp;
    const cplx* in = (const cplx*)ind;
    cplx* fbuf = (cplx*)malloc(sizeof(cplx) * N * S);
    for (int s = 0; s < S; s++) memcpy(fbuf + (long)s * N, in + (long)s * L + cp, sizeof(cplx) * N);
    orc_fft_read(N, (int)p->num_data_subc, (int)p->num_pilot_subc, S,
                 (double)p->pilot_ampl / 1000, (double*)fbuf, outd);
    free(fbuf);
}

/* OFDM_FORM::read, Frame.cpp:201-208. Returns bytes written. */
size_t orc_ofdm_read(const ofdm_params* p, int S, int k, const double* in, uint8_t* bytes)
{
    int D = (int)p->num_data_subc, P = (int)p->num_pilot_subc;
    size_t n = (size_t)(D / P) * P * S;
    double* pts = (double*)malloc(sizeof(cplx) * n);
    orc_ofdm_fft(p, S, in, pts);
    size_t nb = orc_demod(k, pts, n, bytes);
    free(pts);
    return nb;
}

/* OFDM_FORM::pilot_freq_sinh, Frame.hpp:285-337. x: the form's first sample,
 * size = (N+cp)*S samples. Coarse CFO in cycles/sample. The reference's
 * out-of-range write at Frame.hpp:322 does not affect the result and is not
 * reproduced. */
double orc_pilot_freq_sinh(const ofdm_params* p, int S, const double* xd)
{
    int N = (int)p->fft_size, D = (int)p->num_data_subc, P = (int)p->num_pilot_subc;
    int size = (N + (int)p->cp_size) * S;
    cplx* spec = (cplx*)malloc(sizeof(cplx) * size);
    double* amp = (double*)calloc(size, sizeof(double));
    memcpy(spec, xd, sizeof(cplx) * size);
    orc_fft((double*)spec, size, -1);
    int half = size / 2;
    for (int i = 0; i < half; i++) {
        amp[i] = cabs(spec[i + half]);
        amp[i + half] = cabs(spec[i]);
    }
    double rel_bw = (double)(D + P) / (N);
    double rel_pilot_w = rel_bw / P;
    int pilot_w = (int)(size * rel_pilot_w);
    int* borders = (int*)malloc(sizeof(int) * (P + 2));
    for (int i = 0, j = (int)((1.0 - rel_bw - rel_pilot_w) / 2.0 * size); i < P + 2; i++) {
        borders[i] = j;
        j += pilot_w;
    }
    borders[0] = imax(0, borders[0]);
    double shift = 0;
    for (int i = 0; i < P + 1; i++) {
        if (i == P / 2) continue;
        int lo = borders[i], hi = borders[i + 1];
        int best = hi; /* std::max_element of an empty range returns last */
        if (lo < hi) {
            best = lo;
            for (int t = lo + 1; t < hi; t++)
                if (amp[best] < amp[t]) best = t;
        }
        shift += best;
    }
    shift /= P;
    shift -= size / 2;
    shift /= size;
    free(borders);
    free(amp);
    free(spec);
    return shift;
}

/* OFDM_FORM::freq_shift, Frame.hpp:340-348 (recursive phasor). */
void orc_freq_shift(double* xd, long n, double shift)
{
    cplx* x = (cplx*)xd;
    cplx step = cexp(CMPLX(0.0, -2 * M_PI * shift));
    cplx phase = CMPLX(1.0, 0.0);
    for (long i = 0; i < n; i++) {
        x[i] *= phase;
        phase *= step;
    }
}

/* exp(-complex(0,1) * r) exactly as libstdc++ forms it: (-0.0*r, -1.0*r). */
static cplx exp_minus_j(double r) { return cexp(CMPLX(-0.0 * r, -1.0 * r)); }

/* OFDM_FORM::cp_freq_sinh, Frame.hpp:238-263 on S symbols (the
 * message_with_preamble form: num_pr_symb + num_symb). */
void orc_cp_freq_sinh(const ofdm_params* p, int S, double* xd)
{
    cplx* x = (cplx*)xd;
    int N = (int)p->fft_size, cp = (int)p->cp_size, L = N + cp;
    long size = (long)L * S;
    cplx shift = CMPLX(1.0, 0.0);
    for (long i = 0; i < size; i += L) {
        cplx phase = 0;
        cplx cur = CMPLX(1.0, 0.0);
        for (int j = 0; j < L; ++j) x[i + j] *= shift;
        for (int j = 0; j < cp; j++) phase += conj(x[i + j]) * x[i + j + N];
        cplx step = exp_minus_j(carg(phase) / N);
        for (int j = 0; j < L; ++j) {
            x[i + j] *= cur;
            cur *= step;
        }
        shift *= cur;
    }
}

/* OFDM_FORM::pr_phase_sinh, Frame.hpp:265-274. */
void orc_pr_phase_sinh(double* xd, long size, const double* prd, long pr_size)
{
    cplx* x = (cplx*)xd;
    const cplx* pr = (const cplx*)prd;
    cplx phase = 0;
    for (long i = 0; i < pr_size; i++) phase += conj(pr[i]) * x[i];
    phase = exp_minus_j(carg(phase));
    for (long i = 0; i < size; i++) x[i] *= phase;
}

/* ------------------------------------------------------------------------ */
/* T2SIN_FORM — Frame.cpp:99-154, Frame.hpp:96-197                          */
/* ------------------------------------------------------------------------ */

/* T2SIN_FORM::set, Frame.cpp:139-154: X[f1]=X[f2]=0.5, unnormalised IFFT. */
void orc_t2_symbol(const ofdm_params* p, double* outd)
{
    int size = (int)p->t2sin_size;
    cplx* out = (cplx*)outd;
    memset(out, 0, sizeof(cplx) * size);
    if (size) {
        out[p->t2_sin_f1] = CMPLX(0.5, 0);
        out[p->t2_sin_f2] = CMPLX(0.5, 0);
    }
    orc_fft(outd, size, +1);
}

/* Detector mask, T2SIN_FORM ctor Frame.cpp:120-133. */
void orc_t2_mask(const ofdm_params* p, double* mask)
{
    int size = (int)p->t2sin_size, f1 = (int)p->t2_sin_f1, f2 = (int)p->t2_sin_f2;
    int sm = (int)p->smooth;
    memset(mask, 0, sizeof(double) * size);
    int a1 = imax(0, f1 - sm), b1 = imin(size - 1, f1 + sm);
    int a2 = imax(0, f2 - sm), b2 = imin(size - 1, f2 + sm);
    for (int i = a1; i <= b1; i++) mask[i] += 1.0;
    for (int i = a2; i <= b2; i++) mask[i] += 1.0;
}

/* Energy ratio of one block; returns -1 when the reference `continue`s. */
static double t2_block_rel(int size, const double* mask, const cplx* blk, cplx* tmp)
{
    memcpy(tmp, blk, sizeof(cplx) * size);
    orc_fft((double*)tmp, size, -1);
    double total = 0.0, sin_e = 0.0;
    for (int j = 0; j < size; j++) {
        double re = creal(tmp[j]), im = cimag(tmp[j]);
        double e = re * re + im * im;
        total += e;
        sin_e += mask[j] * e;
    }
    if (total == 0) return -1.0;
    double rel = sin_e / total;
    if (isnan(rel)) return -1.0;
    return rel;
}

/* T2SIN_FORM::corr, Frame.hpp:96-147: out has n/size entries. */
void orc_t2_corr(const ofdm_params* p, const double* xd, long n, double* out)
{
    int size = (int)p->t2sin_size;
    double level = (double)p->t2_sin_level / 1000;
    long cycles = n / size;
    double* mask = (double*)malloc(sizeof(double) * size);
    cplx* tmp = (cplx*)malloc(sizeof(cplx) * size);
    orc_t2_mask(p, mask);
    const cplx* x = (const cplx*)xd;
    for (long i = 0; i < cycles; i++) {
        out[i] = 0.0;
        double rel = t2_block_rel(size, mask, x + i * size, tmp);
        if (rel > level) out[i] = rel;
    }
    free(tmp);
    free(mask);
}

/* T2SIN_FORM::find_t2sin, Frame.hpp:150-197. */
long orc_find_t2sin(const ofdm_params* p, const double* xd, long n, long start)
{
    int size = (int)p->t2sin_size;
    double level = (double)p->t2_sin_level / 1000;
    long cycles = (n - start) / size;
    double* mask = (double*)malloc(sizeof(double) * size);
    cplx* tmp = (cplx*)malloc(sizeof(cplx) * size);
    orc_t2_mask(p, mask);
    const cplx* x = (const cplx*)xd + start;
    long found = -1;
    for (long i = 0; i < cycles; i++) {
        double rel = t2_block_rel(size, mask, x + i * size, tmp);
        if (rel > level) {
            found = i * size + start;
            break;
        }
    }
    free(tmp);
    free(mask);
    return found;
}

/* ------------------------------------------------------------------------ */
/* PREAMBLE_FORM — Frame.cpp:259-378, Frame.hpp:389-434                      */
/* ------------------------------------------------------------------------ */

/* std::mt19937 (C++11 [rand.eng.mers] parameters). */
typedef struct {
    uint32_t mt[624];
    int idx;
} mt19937;

static void mt_seed(mt19937* m, uint32_t s)
{
    m->mt[0] = s;
    for (int i = 1; i < 624; i++) m->mt[i] = 1812433253u * (m->mt[i - 1] ^ (m->mt[i - 1] >> 30)) + (uint32_t)i;
    m->idx = 624;
}

static uint32_t mt_next(mt19937* m)
{
    if (m->idx >= 624) {
        for (int i = 0; i < 624; i++) {
            uint32_t y = (m->mt[i] & 0x80000000u) | (m->mt[(i + 1) % 624] & 0x7fffffffu);
            m->mt[i] = m->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        m->idx = 0;
    }
    uint32_t y = m->mt[m->idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

/* PREAMBLE_FORM ctor, Frame.cpp:269-272: std::uniform_int_distribution<int>(0,255)
 * over std::mt19937(pr_seed). libstdc++ (GCC >= 11, <bits/uniform_int_dist.h>)
 * maps a 32-bit engine with Lemire's multiply-shift: (u64)g() * 256 >> 32;
 * with range 256 the rejection threshold (-256 % 256) is 0. */
void orc_preamble_bytes(const ofdm_params* p, uint8_t* out)
{
    long n = p->num_data_subc * p->num_pr_symb * 1 / 8;
    mt19937 m;
    mt_seed(&m, (uint32_t)p->pr_seed);
    for (long i = 0; i < n; i++) out[i] = (uint8_t)(((uint64_t)mt_next(&m) * 256u) >> 32);
}

/* PREAMBLE_FORM::set, Frame.cpp:276-294 (BPSK OFDM preamble, its BPSK points,
 * and the normalised conjugate correlation template). Any output nullable. */
void orc_preamble_setup(const ofdm_params* p, double* ofdm_preamble, double* mod_preamble,
                        double* templd)
{
    int N = (int)p->fft_size, cp = (int)p->cp_size, S = (int)p->num_pr_symb;
    int D = (int)p->num_data_subc, L = (int)p->pr_sin_len;
    long size = (long)(N + cp) * S;
    long nb = (long)D * S / 8;
    uint8_t* bytes = (uint8_t*)malloc(nb ? nb : 1);
    orc_preamble_bytes(p, bytes);
    cplx* pre = (cplx*)malloc(sizeof(cplx) * size);
    orc_ofdm_write(p, S, 1, bytes, (double*)pre);
    if (ofdm_preamble) memcpy(ofdm_preamble, pre, sizeof(cplx) * size);
    if (mod_preamble) orc_mod(1, bytes, nb, mod_preamble);
    if (templd) {
        cplx* c = (cplx*)templd;
        double norm = 0.0;
        for (int i = 0; i < L; i++) {
            c[i] = conj(pre[i]);
            norm += cabs(c[i] * c[i]);
        }
        norm = sqrt(norm);
        for (int i = 0; i < L; i++) c[i] = c[i] / CMPLX(norm, 0.0);
    }
    free(pre);
    free(bytes);
}

static cplx sample_or_zero(const cplx* x, long n, long i) { return (i >= 0 && i < n) ? x[i] : 0; }

/* PREAMBLE_FORM::find_preamble, Frame.cpp:338-378 (first threshold crossing,
 * running energy updated after each test). Samples past n read as 0 (the
 * reference reads past its vector there). Returns start+lag or -10. */
static long find_preamble_lag(const ofdm_params* p, const double* templd, const double* xd, long n, long start);

long orc_find_preamble(const ofdm_params* p, const double* templd, const double* xd, long n,
                       long start)
{
    const long lag = find_preamble_lag(p, templd, xd, n, start);
    return lag < 0 ? -10 : start + lag;
}

/* The same search, returning the passing lag (>= 0) or -1: in stream
 * coordinates start + lag may be any value, -10 included. */
static long find_preamble_lag(const ofdm_params* p, const double* templd, const double* xd, long n, long start)
{
    const cplx* c = (const cplx*)templd;
    const cplx* x = (const cplx*)xd;
    int L = (int)p->pr_sin_len;
    long cycles = 2 * p->t2sin_size + L;
    double level = (double)p->pr_level / 1000;
    double norm = 0;
    for (int i = 0; i < L; i++) {
        cplx v = sample_or_zero(x, n, start + i);
        norm += creal(v) * creal(v) + cimag(v) * cimag(v);
    }
    for (long i = 0; i < cycles; i++) {
        long base = start + i;
        if (norm > 1.0) {
            cplx energy = 0;
            for (int j = 0; j < L; j++) energy += sample_or_zero(x, n, base + j) * c[j];
            if (cabs(energy) / sqrt(norm) > level) return i;
        }
        cplx a = sample_or_zero(x, n, base + L), b = sample_or_zero(x, n, base);
        norm += creal(a) * creal(a) + cimag(a) * cimag(a);
        norm -= creal(b) * creal(b) + cimag(b) * cimag(b);
    }
    return -1;
}

/* PREAMBLE_FORM::chan_char_lq, Frame.hpp:389-434: FFT of the preamble form
 * (coef == 1), phase of pr/mod_preamble over the first D/2 carriers, one-pass
 * unwrap, least squares on raw sums, unit phasors over D carriers. */
void orc_chan_char_lq(const ofdm_params* p, double* pred, const double* modd, double* chand)
{
    int D = (int)p->num_data_subc, P = (int)p->num_pilot_subc, S = (int)p->num_pr_symb;
    long n = (long)(D / P) * P * S;
    cplx* pr = (cplx*)malloc(sizeof(cplx) * (n > D ? n : D));
    orc_ofdm_fft(p, S, pred, (double*)pr);
    const cplx* mod = (const cplx*)modd;
    cplx* chan = (cplx*)chand;
    int half = D / 2;
    double* ph = (double*)malloc(sizeof(double) * (half ? half : 1));
    for (int i = 0; i < half; i++) ph[i] = carg(pr[i] / mod[i]);
    for (int i = 1; i < half; i++) {
        double d = ph[i] - ph[i - 1];
        if (d > M_PI)
            ph[i] -= 2 * M_PI;
        else if (d < -M_PI)
            ph[i] += 2 * M_PI;
    }
    double mx = 0.0, my = 0.0, mxy = 0.0, mx2 = 0.0;
    for (int i = 0; i < half; i++) {
        mxy += ph[i] * i;
        mx2 += i * i;
        mx += i;
        my += ph[i];
    }
    double b = (mxy - mx * my) / (mx2 - mx * mx);
    double a = my - b * mx;
    size_t sz = (size_t)D;
    for (int i = 0; i < (int)(sz / 2); i++) chan[i] = cexp(CMPLX(0.0, b * i + a));
    for (int i = (int)(sz / 2); i < (int)sz; i++)
        chan[i] = cexp(CMPLX(0.0, -b * sz / 2 + (double)(i - sz / 2) * b + a));
    free(ph);
    free(pr);
}

/* ------------------------------------------------------------------------ */
/* FRAME_FORM — Frame.cpp:213-256                                            */
/* ------------------------------------------------------------------------ */

/* FRAME_FORM ctor + write: [T2 | preamble | message] (output_size samples). */
void orc_frame_write(const ofdm_params* p, const uint8_t* bytes, double* framed)
{
    int N = (int)p->fft_size, cp = (int)p->cp_size;
    long t2 = p->t2sin_size, pre = (long)(N + cp) * p->num_pr_symb;
    cplx* f = (cplx*)framed;
    orc_t2_symbol(p, framed);
    orc_preamble_setup(p, (double*)(f + t2), NULL, NULL);
    orc_ofdm_write(p, (int)p->num_symb, (int)p->mod_type, bytes, (double*)(f + t2 + pre));
}

/* FRAME_FORM::get_int16, Frame.cpp:249-256: complex<int16>(x * complex(mult))
 * = per-component truncation toward zero of x*mult (low 16 bits of the int32
 * conversion, as g++ emits it). */
void orc_get_int16(const double* xd, long n, long mult, int16_t* out)
{
    const cplx* x = (const cplx*)xd;
    cplx m = CMPLX((double)mult, 0.0);
    for (long i = 0; i < n; i++) {
        cplx v = x[i] * m;
        out[2 * i] = (int16_t)(int32_t)creal(v);
        out[2 * i + 1] = (int16_t)(int32_t)cimag(v);
    }
}

/* ------------------------------------------------------------------------ */
/* Loopback channel + batched drivers (bench cpu_baseline)                   */
/* ------------------------------------------------------------------------ */

static inline uint32_t lowbias32(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

/* Counter-based Box-Muller AWGN; same definition as the HIP tx kernel
 * (ofdm_kernels.hip awgn_sample): 24-bit uniforms from a lowbias32 hash h1 of
 * the 64-bit sample counter and seed, u1 from h1 and u2 from h1 times the
 * 32-bit Fibonacci multiplier (the pair spans h1's 2^32 values either way;
 * the multiply replaces a second hash). The GPU evaluates log/sin/cos on its FP32
 * units, so the two agree to ~1e-6 of noise_std, not bitwise. A channel model
 * of this repo (the reference's channel is the radio, python_code/channel.py). */
void orc_awgn(double* xd, long n, double noise_std, unsigned long long seed,
              unsigned long long off)
{
    orc_awgn_mt(xd, n, noise_std, seed, off, 1);
}

/* orc_awgn on `threads` OpenMP threads (the noise is counter-based, so the
 * result does not depend on the thread count). */
void orc_awgn_mt(double* xd, long n, double noise_std, unsigned long long seed,
                 unsigned long long off, int threads)
{
    cplx* x = (cplx*)xd;
    double sc = noise_std * M_SQRT1_2;
    const uint32_t k0 = lowbias32((uint32_t)seed ^ 0x9E3779B9u);
    const uint32_t k1 = lowbias32((uint32_t)(seed >> 32) + k0);
    if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(static)
    for (long i = 0; i < n; i++) {
        uint64_t g = off + (uint64_t)i;
        uint32_t h1 = lowbias32((uint32_t)g ^ lowbias32((uint32_t)(g >> 32) ^ k1) ^ k0);
        uint32_t h2 = h1 * 0x9E3779B9u; /* Fibonacci multiplier: (u1, u2) on a rank-1 lattice */
        double u1 = (double)(float)((float)((h1 >> 8) + 1) * 0x1.0p-24f);
        double u2 = (double)(float)((float)(h2 >> 8) * 0x1.0p-24f);
        double r = sqrt(-2.0 * log(u1)) * sc;
        double th = 2.0 * M_PI * u2;
        x[i] += CMPLX(r * cos(th), r * sin(th));
    }
}

unsigned long long orc_rx_batch(const ofdm_params* p, const double* iq, long nframes,
                                long frame_stride, double* constell, uint8_t* bytes,
                                const uint8_t* ref, int threads)
{
    int S = (int)p->num_symb, k = (int)p->mod_type;
    int D = (int)p->num_data_subc, P = (int)p->num_pilot_subc;
    long npts = (long)(D / P) * P * S;
    long nb = (long)D * S * k / 8;
    unsigned long long errs = 0;
    if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(static) reduction(+ : errs)
    for (long f = 0; f < nframes; f++) {
        double* pts = (double*)malloc(sizeof(cplx) * npts);
        uint8_t* b = (uint8_t*)malloc(nb + 8);
        orc_ofdm_fft(p, S, iq + 2 * f * frame_stride, pts);
        if (constell) memcpy(constell + 2 * f * npts, pts, sizeof(cplx) * npts);
        orc_demod(k, pts, npts, b);
        if (bytes) memcpy(bytes + f * nb, b, nb);
        if (ref)
            for (long i = 0; i < nb; i++) errs += __builtin_popcount((unsigned)(b[i] ^ ref[f * nb + i]));
        free(b);
        free(pts);
    }
    return errs;
}

void orc_tx_batch(const ofdm_params* p, const uint8_t* bytes, long nframes, double* iq,
                  long frame_stride, int threads)
{
    int S = (int)p->num_symb, k = (int)p->mod_type;
    long nb = p->num_data_subc * S * k / 8;
    if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(static)
    for (long f = 0; f < nframes; f++) orc_ofdm_write(p, S, k, bytes + f * nb, iq + 2 * f * frame_stride);
}


/* ---- located-frame decode and the streaming walk (rx.cpp:125-221) ------ */

/* main.cpp:60-80 / rx.cpp:181-216 on one located frame. `region` is
 * [preamble | message] ((N+cp)*(npr+S) samples); it is copied first, as
 * rx.cpp:185-189 copies it into FRAME_FORM::buf. Writes D*S equalised points
 * (before demod's clamp, data/constell.bin layout) and D*S*k/8 bytes; returns
 * the pilot_freq_sinh CFO. */
double orc_decode_frame(const ofdm_params* p, const double* region, double* constell, uint8_t* bytes)
{
    int N = (int)p->fft_size, cp = (int)p->cp_size, L = N + cp;
    int npr = (int)p->num_pr_symb, S = (int)p->num_symb, D = (int)p->num_data_subc;
    int k = (int)p->mod_type;
    long pre = (long)L * npr, msg = (long)L * S;
    cplx* x = (cplx*)malloc(sizeof(cplx) * (pre + msg));
    memcpy(x, region, sizeof(cplx) * (pre + msg));
    cplx* opre = (cplx*)malloc(sizeof(cplx) * pre);
    cplx* modp = (cplx*)malloc(sizeof(cplx) * (long)D * npr);
    cplx* templ = (cplx*)malloc(sizeof(cplx) * p->pr_sin_len);
    cplx* chan = (cplx*)malloc(sizeof(cplx) * D);
    orc_preamble_setup(p, (double*)opre, (double*)modp, (double*)templ);
    double cfo = orc_pilot_freq_sinh(p, npr, (const double*)x);          /* main.cpp:60 */
    orc_freq_shift((double*)x, pre + msg, cfo);                          /* main.cpp:61 */
    orc_cp_freq_sinh(p, npr + S, (double*)x);                            /* main.cpp:62 */
    orc_pr_phase_sinh((double*)x, pre + msg, (const double*)opre, pre);  /* main.cpp:63 */
    orc_chan_char_lq(p, (double*)x, (const double*)modp, (double*)chan); /* main.cpp:65 */
    cplx* c = (cplx*)constell;
    orc_ofdm_fft(p, S, (const double*)(x + pre), constell);              /* main.cpp:66 */
    long npts = (long)D * S;
    for (long j = 0; j < npts; j++) c[j] /= chan[j % D];                 /* main.cpp:69-71 */
    cplx* tmp = (cplx*)malloc(sizeof(cplx) * npts);
    memcpy(tmp, c, sizeof(cplx) * npts);
    orc_demod(k, (double*)tmp, (size_t)npts, bytes);                     /* main.cpp:73 (clamps its copy) */
    free(tmp);
    free(chan);
    free(templ);
    free(modp);
    free(opre);
    free(x);
    return cfo;
}

/* orc_decode_frame on every located frame of a stream (frame f's region at
 * x + pbs[f]), OpenMP over the frames: the per-frame chain is independent. */
void orc_decode_frames(const ofdm_params* p, const double* x, const long* pbs, long nframes, double* cfo,
                       double* constell, uint8_t* bytes, int threads)
{
    long npts = p->num_data_subc * p->num_symb, nb = npts * p->mod_type / 8;
    if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 16)
    for (long f = 0; f < nframes; f++) {
        const double c = orc_decode_frame(p, x + 2 * pbs[f], constell + 2 * f * npts, bytes + f * nb);
        if (cfo) cfo[f] = c;
    }
}

/* The detection walk of rx.cpp:125-221 over one contiguous stream held whole,
 * WITHOUT rx.cpp's SDR ring (the continuous walk; orc_stream_walk_ring below
 * has the ring and is what rx.cpp does):
 *   pos = 0; loop { hit = find_t2sin(pos) (256-sample grid from pos);
 *   none -> stop; pb = find_preamble(hit) + 1 (rx.cpp:160);
 *   pb < -2 -> pos = hit + message.size (rx.cpp:162-168);
 *   frame [pb, pb + preamble + message) past the stream end -> stop;
 *   record pb; pos = pb + message.size (rx.cpp:192) }.
 * rx.cpp's ring differs from this at its refills (rx.cpp:137-145): a T2 miss
 * discards the ring's unscanned tail and restarts the grid on the next SDR
 * buffer, so a marker straddling a refill can be lost. Samples past n read as
 * zero in the preamble search. Returns the number of frames (at most max) and
 * their preamble starts. */
long orc_stream_walk(const ofdm_params* p, const double* x, long n, long* pb_out, long max)
{
    long ex, exr;
    return orc_stream_walk_ring(p, x, n, 0, 0, 0, n, pb_out, NULL, max, &ex, &exr);
}

/* One T2 block of T2SIN_FORM::find_t2sin (Frame.hpp:164-193) at stream
 * position b, samples outside [0, n) read as zero (rx.cpp's zero-initialised
 * ring header, FRAME_FORM ctor Frame.cpp:221, and the SDR stand-in's zeros
 * past a capture's end). */
static double t2_block_rel_at(int size, const double* mask, const cplx* x, long n, long b, cplx* blk, cplx* tmp)
{
    for (int i = 0; i < size; i++) blk[i] = sample_or_zero(x, n, b + i);
    return t2_block_rel(size, mask, blk, tmp);
}

/* rx.cpp's detection walk in stream coordinates, with its SDR ring (ring > 0)
 * or without it (ring = 0, the continuous walk).
 *
 * rx.cpp's ring (rx.cpp:94-198, buf_update :73-91): from_sdr_buf holds
 * output_size + R samples, R = rx_buf_size * output_size (the SDR's
 * rx_buf_size, sdr.hpp:141; output_size = frame_len, Frame.cpp:221-224); each
 * refill copies the next R SDR samples to offset output_size. In stream
 * coordinates (sample 0 = the SDR's first sample) the walk state is
 * (pos, ring_end), ring_end = one past the ring's last sample:
 *   start (-output_size, R): the zero header before the first buffer (:105-114);
 *   T2 search from pos over the blocks that end by ring_end (find_t2sin's
 *     cycles = (size - pos)/T2sin_size on the buffer, Frame.hpp:152);
 *   a miss -> (ring_end, ring_end + R): the refill without carry, grid
 *     restarted at output_size (:137-145);
 *   hit >= ring_end - output_size -> ring_end += R: the carry at
 *     pos >= threshold (:147-156);
 *   pb = find_preamble(hit) + 1; no preamble (-10) -> pos = hit + message.size
 *     (:160-166; a found preamble may have pb < 0 here, in the zero header);
 *   pb >= ring_end - output_size + T2sin_size -> ring_end += R (:180-189);
 *   record pb; pos = pb + message.size (:198).
 * Every sample a step reads lies in the buffer, so the decoded frames are the
 * stream's samples (orc_rx_app_walk replays the buffer itself; the tests
 * check the two agree). Samples outside [0, n) read as zero; the walk stops
 * when a scan starts at or past n (ring = 0: when no full block is left) or
 * a located frame runs past n.
 *
 * The walk starts at (start, ring_end) (ring_end ignored when ring = 0) and
 * stops at its first state at or past own_hi (own_hi = n: the whole stream):
 * *exit_out / *exit_ring_out = that state (a position after a step; the
 * first scan block at or past own_hi when the scan passes it, an equivalent
 * state; the start of the step that located the first frame past own_hi),
 * or -1 when the walk ended first. lag_out (nullable): per frame, whether
 * the state after it has the later of its two possible ring ends (a carry
 * loaded the next buffer; the library's WALK_REC_LAG). Returns the frames
 * located (at most max stored). */
/* The first ring end after q on the grid of ring end e (ring ends e + k*ring). */
static long ring_after(long q, long e, long ring)
{
    const long d = q - e;
    const long k = d >= 0 ? d / ring : -((-d + ring - 1) / ring);
    return e + (k + 1) * ring;
}

long orc_stream_walk_ring(const ofdm_params* p, const double* xd, long n, long ring, long start, long ring_end,
                          long own_hi, long* pb_out, uint8_t* lag_out, long max, long* exit_out, long* exit_ring_out)
{
    int N = (int)p->fft_size, cp = (int)p->cp_size, L = N + cp;
    const int size = (int)p->t2sin_size;
    const long pre = (long)L * p->num_pr_symb, msg = (long)L * p->num_symb, out = size + pre + msg;
    const double level = (double)p->t2_sin_level / 1000;
    const cplx* x = (const cplx*)xd;
    int D = (int)p->num_data_subc;
    cplx* opre = (cplx*)malloc(sizeof(cplx) * pre);
    cplx* modp = (cplx*)malloc(sizeof(cplx) * (long)D * p->num_pr_symb);
    cplx* templ = (cplx*)malloc(sizeof(cplx) * p->pr_sin_len);
    double* mask = (double*)malloc(sizeof(double) * size);
    cplx* blk = (cplx*)malloc(sizeof(cplx) * size);
    cplx* tmp = (cplx*)malloc(sizeof(cplx) * size);
    orc_preamble_setup(p, (double*)opre, (double*)modp, (double*)templ);
    orc_t2_mask(p, mask);
    long pos = start, rend = ring_end, nf = 0;
    *exit_out = -1;
    *exit_ring_out = 0;
    for (;;) {
        if (pos >= own_hi) {
            *exit_out = pos;
            *exit_ring_out = rend;
            break;
        }
        const long spos = pos, srend = rend;
        long hit = -1;
        int stop = 0, miss = 0, passed = 0;
        for (long b = pos;; b += size) {
            if (ring ? b >= n : b + size > n) {
                stop = 1;
                break;
            }
            if (b >= own_hi) {  /* the scan passes own_hi: an equivalent state */
                *exit_out = b;
                *exit_ring_out = rend;
                passed = 1;
                break;
            }
            if (ring && b + size > rend) {
                miss = 1;
                break;
            }
            if (t2_block_rel_at(size, mask, x, n, b, blk, tmp) > level) {
                hit = b;
                break;
            }
        }
        if (stop || passed) break;
        if (miss) {
            pos = rend;
            rend += ring;
            continue;
        }
        if (ring && hit >= rend - out) rend += ring;
        /* rx.cpp:160-168 tests preamble_begin < -2 in buffer coordinates,
         * where a found preamble gives >= 1; here a found preamble may lie in
         * the ring's zero header (pb < 0), so the test is on the search */
        const long lag = find_preamble_lag(p, (const double*)templ, xd, n, hit);
        if (lag < 0) {
            pos = hit + msg;
            continue;
        }
        const long pb = hit + lag + 1;
        if (ring && pb >= rend - out + size) rend += ring;
        if (pb + pre + msg > n) break;
        if (nf < max) {
            pb_out[nf] = pb;
            /* the state after the frame is (pb + msg, rend): rend is the first
             * ring end after pb + msg, or (after a carry) the one after it */
            if (lag_out) lag_out[nf] = ring && rend != ring_after(pb + msg, rend, ring);
        }
        nf++;
        if (pb >= own_hi) {
            *exit_out = spos;
            *exit_ring_out = srend;
            break;
        }
        pos = pb + msg;
    }
    free(tmp);
    free(blk);
    free(mask);
    free(templ);
    free(modp);
    free(opre);
    return nf;
}

/* rx.cpp's receive loop itself (rx.cpp:94-198 with buf_update :73-91), replayed
 * on a real ring buffer: from_sdr_buf = output_size + R samples (Frame.cpp:221,
 * R = rx_buf_size * output_size, sdr.hpp:141), each SDR refill written at
 * offset output_size, the carry copying the last output_size samples to the
 * front (:149-153, :182-186), the refill on a T2 miss leaving the front as
 * it was. x is the SDR's sample stream (zeros past n, as the stand-in
 * delivers). `iterations` loop iterations are run (config["iterations"],
 * :124-126); iterations <= 0 runs until a refill's buffer starts at or past
 * n. stop_at_end: stop at the first located frame running past n (the
 * stream API's rule) instead of decoding the zeros after it. Frames are
 * reported as stream positions (buffer index + the buffer's stream offset). */
long orc_rx_app_walk(const ofdm_params* p, const double* xd, long n, long iterations, int stop_at_end, long* pb_out,
                     long max)
{
    int N = (int)p->fft_size, cp = (int)p->cp_size, L = N + cp;
    const int size = (int)p->t2sin_size;
    const long pre = (long)L * p->num_pr_symb, msg = (long)L * p->num_symb, out = size + pre + msg;
    const long R = p->rx_buf_size * out, bufsize = out + R, threshold = bufsize - out;
    const cplx* x = (const cplx*)xd;
    int D = (int)p->num_data_subc;
    cplx* opre = (cplx*)malloc(sizeof(cplx) * pre);
    cplx* modp = (cplx*)malloc(sizeof(cplx) * (long)D * p->num_pr_symb);
    cplx* templ = (cplx*)malloc(sizeof(cplx) * p->pr_sin_len);
    cplx* buf = (cplx*)calloc((size_t)bufsize, sizeof(cplx));
    orc_preamble_setup(p, (double*)opre, (double*)modp, (double*)templ);
    long src = 0, base = 0, nf = 0;
    /* buf_update: the next SDR buffer to offset output_size; buf[0] is then
     * stream sample src - R - out */
#define RING_REFILL()                                                   \
    do {                                                                \
        for (long i = 0; i < R; i++) buf[out + i] = sample_or_zero(x, n, src + i); \
        src += R;                                                       \
        base = src - R - out;                                           \
    } while (0)
    RING_REFILL();
    long pos = 0;
    for (long it = 0; iterations <= 0 || it < iterations; it++) {
        pos = orc_find_t2sin(p, (const double*)buf, bufsize, pos);
        if (pos == -1) {
            pos = out;
            if (iterations <= 0 && src >= n) break; /* the next buffer would start past the capture */
            RING_REFILL();
            continue;
        }
        if (pos >= threshold) {
            pos -= threshold;
            memmove(buf, buf + threshold, sizeof(cplx) * out);
            RING_REFILL();
        }
        long preamble_begin = orc_find_preamble(p, (const double*)templ, (const double*)buf, bufsize, pos) + 1;
        if (preamble_begin < -2) {
            pos += msg;
            continue;
        }
        pos = preamble_begin;
        if (pos >= threshold + size) {
            pos -= threshold;
            memmove(buf, buf + threshold, sizeof(cplx) * out);
            RING_REFILL();
        }
        const long pb = base + pos;
        if (stop_at_end && pb + pre + msg > n) break;
        if (nf < max) pb_out[nf] = pb;
        nf++;
        pos += msg;
    }
#undef RING_REFILL
    free(buf);
    free(templ);
    free(modp);
    free(opre);
    return nf;
}
