/*
 * ofdm_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C99, FP64, C `double complex` arithmetic = the
 * libgcc __muldc3/__divdc3 semantics of the reference's std::complex<double>)
 * of the DmSM-1/C-OFDM modem path. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker / the
 * reported CPU baseline. The product (c-ofdm_amd/) never links it.
 *
 * Pinning:
 *   - Modulation / bit repacking: compared bit-exactly against the reference's
 *     own OFDM/modulation.cpp compiled unmodified into oracle/_ref/.
 *   - Frame path (FFT_FORM/OFDM_FORM/T2SIN/PREAMBLE): the reference's
 *     Frame.cpp needs FFTW (absent here) and is unbuildable; the restatement is
 *     pinned by the reference's golden files data/{source,data,t2_sin_corr,
 *     phases,constell}.bin and data.txt (tests/golden/).
 *   - FFTW itself is third-party (version unpinned, Makefile:3 `-lfftw3`): its
 *     published definition is the unnormalised DFT X[k] = sum x[n] e^{-+2πi nk/N};
 *     orc_fft computes that definition with an independent mixed-radix FFT.
 */
#ifndef OFDM_ORACLE_H
#define OFDM_ORACLE_H

#include <stddef.h>
#include <stdint.h>
#include "../include/ofdm_mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

/* All complex buffers are interleaved double {re, im}. */

/* Modulation (OFDM/modulation.cpp) */
int orc_constellation(int k, double* out);                       /* returns 2^k points */
size_t orc_bit_convert(int out_bits, int in_bits, const uint8_t* in, size_t len, uint8_t* out);
size_t orc_mod(int k, const uint8_t* bytes, size_t nbytes, double* out);
size_t orc_demod(int k, double* points /* clamped in place */, size_t n, uint8_t* out);

/* Layout + FFT (OFDM/Frame.cpp:4-96) */
void orc_layout(int N, int D, int P, int* pilot_bin, int* seg_start);
void orc_fft(double* x, int n, int sign);  /* sign -1 = FFTW_FORWARD, +1 = FFTW_BACKWARD */
void orc_fft_write(int N, int D, int P, int S, double ampl, const double* in, double* out);
void orc_fft_read(int N, int D, int P, int S, double ampl, double* buf, double* out);

/* OFDM_FORM (Frame.cpp:157-208, Frame.hpp:238-348) */
void orc_ofdm_write(const ofdm_params* p, int S, int k, const uint8_t* bytes, double* out);
void orc_ofdm_fft(const ofdm_params* p, int S, const double* in, double* out);
size_t orc_ofdm_read(const ofdm_params* p, int S, int k, const double* in, uint8_t* bytes);
double orc_pilot_freq_sinh(const ofdm_params* p, int S, const double* x);
void orc_freq_shift(double* x, long n, double shift);
void orc_cp_freq_sinh(const ofdm_params* p, int S, double* x);
void orc_pr_phase_sinh(double* x, long size, const double* pr, long pr_size);

/* T2SIN_FORM (Frame.cpp:99-154, Frame.hpp:96-197) */
void orc_t2_symbol(const ofdm_params* p, double* out);
void orc_t2_mask(const ofdm_params* p, double* mask);
void orc_t2_corr(const ofdm_params* p, const double* x, long n, double* out);
long orc_find_t2sin(const ofdm_params* p, const double* x, long n, long start);

/* PREAMBLE_FORM (Frame.cpp:259-378, Frame.hpp:389-434) */
void orc_preamble_bytes(const ofdm_params* p, uint8_t* out);      /* D*npr/8 bytes */
void orc_preamble_setup(const ofdm_params* p, double* ofdm_preamble, double* mod_preamble,
                        double* templ);
long orc_find_preamble(const ofdm_params* p, const double* templ, const double* x, long n,
                       long start);
void orc_chan_char_lq(const ofdm_params* p, double* pre /* preamble region, in/out */,
                      const double* mod_preamble, double* chan);

/* FRAME_FORM (Frame.cpp:213-256) */
void orc_frame_write(const ofdm_params* p, const uint8_t* bytes, double* frame);
void orc_get_int16(const double* x, long n, long mult, int16_t* out);

/* Loopback channel used by the bench (not in the reference): counter-based AWGN. */
void orc_awgn(double* x, long n, double noise_std, unsigned long long seed,
              unsigned long long sample_offset);
void orc_awgn_mt(double* x, long n, double noise_std, unsigned long long seed,
                 unsigned long long sample_offset, int threads);

/* Batched rx over message frames, optionally OpenMP-parallel over frames
 * (cpu_baseline leg). Returns bit errors vs ref (if ref != NULL). */
unsigned long long orc_rx_batch(const ofdm_params* p, const double* iq, long nframes,
                                long frame_stride, double* constell, uint8_t* bytes,
                                const uint8_t* ref, int threads);
void orc_tx_batch(const ofdm_params* p, const uint8_t* bytes, long nframes, double* iq,
                  long frame_stride, int threads);

/* Located-frame decode (main.cpp:60-80) and the streaming detection walk
 * (rx.cpp:125-221) over a contiguous stream. */
double orc_decode_frame(const ofdm_params* p, const double* region, double* constell, uint8_t* bytes);
void orc_decode_frames(const ofdm_params* p, const double* x, const long* pbs, long nframes, double* cfo,
                       double* constell, uint8_t* bytes, int threads);
long orc_stream_walk(const ofdm_params* p, const double* x, long n, long* pb_out, long max);
long orc_stream_walk_ring(const ofdm_params* p, const double* x, long n, long ring, long start, long ring_end,
                          long own_hi, long* pb_out, uint8_t* lag_out, long max, long* exit_out,
                          long* exit_ring_out);
long orc_rx_app_walk(const ofdm_params* p, const double* x, long n, long iterations, int stop_at_end, long* pb_out,
                     long max);

#ifdef __cplusplus
}
#endif
#endif
