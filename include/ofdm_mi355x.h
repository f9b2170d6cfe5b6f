/*
 * ofdm_mi355x.h — C-ABI of the MI355X-native OFDM modem core.
 *
 * This is the drop-in boundary for the reference's DSP layer (DmSM-1/C-OFDM,
 * OFDM/Frame.{hpp,cpp} + OFDM/modulation.{hpp,cpp} + config/parser.{hpp,cpp}).
 * The reference exposes a C++ class surface and no C ABI; each
 * entry point below names the reference member it replaces (file:line,
 * relative to the reference root). The C++ compatibility layer in
 * c-ofdm_amd/compat/ re-exposes that class surface on top of these calls.
 *
 * Conventions
 *   - Every function returns an int status: OFDM_OK (0) or a negative
 *     OFDM_ERR_* code; ofdm_last_error() gives a thread-local message.
 *   - Complex samples are interleaved FP64 {re, im} (the std::complex<double>
 *     layout of the reference and of its data/<name>.bin files).
 *   - Batched compute entry points take DEVICE pointers and an explicit HIP
 *     stream passed as void* (NULL = the legacy default stream). They are
 *     asynchronous; they never allocate, copy to the host or synchronise, so
 *     they can be captured into a hipGraph.
 *   - One ofdm_ctx per thread (or per GPU); a ctx is not re-entrant, matching
 *     the reference (one FRAME_FORM per thread).
 *   - Streams: rx launches keep their frame-queue counter per HIP stream, so
 *     one ctx may run rx / fft_read on several streams at once. The detector
 *     entry points (find_t2sin, find_preamble) and the stream receiver keep
 *     one scratch per ctx: a ctx has at most one of those calls in flight at
 *     a time (consecutive calls on one stream are always fine); overlapping
 *     them on two streams takes two contexts (measured slower than one
 *     context's back-to-back calls: INTEGRATION.md). A stream call waits (on
 *     the device) for the previous stream call's decode when it is issued on
 *     another stream.
 */
#ifndef OFDM_MI355X_H
#define OFDM_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OFDM_MI355X_ABI_VERSION 5

enum {
    OFDM_OK = 0,
    OFDM_ERR_INVALID = -1,     /* bad argument / geometry the kernels do not cover */
    OFDM_ERR_UNSUPPORTED = -2, /* valid reference config this build does not run   */
    OFDM_ERR_HIP = -3,         /* HIP runtime error (no GPU, launch failure, ...)  */
    OFDM_ERR_IO = -4,          /* config/file I/O (reference throws runtime_error) */
    OFDM_ERR_NOMEM = -5,
    OFDM_ERR_PARSE = -6        /* std::stol failure in parse_config                */
};

/*
 * Flat view of the ConfigMap keys the hot path consumes
 * (config/parser.hpp:8, consumed in OFDM/Frame.cpp:99-118,157-176,213-232,259-273).
 * Integer-coded fixed point is kept as in config.txt: pilot_ampl/1000,
 * pr_level/1000, t2_sin_level/1000. Missing keys read as 0, as with the
 * reference's ConfigMap::operator[].
 */
typedef struct ofdm_params {
    long fft_size;       /* N */
    long num_data_subc;  /* D */
    long num_pilot_subc; /* P */
    long cp_size;
    long num_symb;       /* message symbols per frame */
    long num_pr_symb;    /* preamble symbols */
    long pr_sin_len;     /* preamble correlation template length */
    long pr_seed;        /* std::mt19937 seed of the preamble bytes */
    long pr_level;       /* /1000: preamble detection threshold */
    long t2sin_size;     /* T2 marker length = detector block */
    long t2_sin_f1;
    long t2_sin_f2;
    long t2_sin_level;   /* /1000: T2 energy-ratio threshold */
    long smooth;         /* T2 mask half-width */
    long mod_type;       /* bits per symbol: 1 bpsk, 2 qam4, 4 qam16, 6 qam64, 8 qam256 */
    long pilot_ampl;     /* /1000: transmitted pilot amplitude */
    long mult;           /* int16 wire scaling (FRAME_FORM::get_int16) */
    long rx_buf_size;    /* rx ring = frame * (rx_buf_size + 1) */
    long iterations;     /* rx.cpp loop count (not used by the core) */
} ofdm_params;

/* Derived frame geometry (FRAME_FORM ctor, OFDM/Frame.cpp:213-232). */
typedef struct ofdm_geometry {
    long symbol_len;       /* N + cp (OFDM_FORM::ofdm_len)                       */
    long message_len;      /* (N+cp)*num_symb  (message.size)                   */
    long preamble_len;     /* (N+cp)*num_pr_symb (preamble.size)                */
    long frame_len;        /* T2 + preamble + message (FRAME_FORM::output_size) */
    long ring_len;         /* frame_len*(rx_buf_size+1) (from_sdr_buf.size())   */
    long data_per_frame;   /* D*num_symb constellation points (message.usefull_size) */
    long bytes_per_frame;  /* D*num_symb*k/8 (FRAME_FORM::usefull_size)         */
    long segment_size;     /* D/P data carriers between pilots                  */
    long pilot_bin[256];   /* pilot FFT bins of one symbol (first P entries)    */
    long segment_bin[256]; /* first FFT bin of each data segment                */
} ofdm_geometry;

/* Optional AWGN channel fused into the tx kernel (bench/loopback only; the
 * reference's channel is the radio, python_code/channel.py). Counter-based
 * noise: identical sample index -> identical noise on every GPU/rank. */
typedef struct ofdm_channel {
    double noise_std;        /* std of the complex noise per time sample (total power) */
    unsigned long long seed;
    unsigned long long sample_offset; /* global index of this batch's first sample */
} ofdm_channel;

typedef struct ofdm_ctx ofdm_ctx;

/* ---- errors / version -------------------------------------------------- */
const char* ofdm_last_error(void);
int ofdm_abi_version(void);

/* ---- config (config/parser.cpp:4-33, config/config.txt) ---------------- */
/* The committed config/config.txt values. */
int ofdm_params_default(ofdm_params* out);
/* parse_config(path) + the config["..."] lookups of the Frame ctors.
 * Returns OFDM_ERR_IO if the file cannot be opened ("Cannot open config
 * file"), OFDM_ERR_PARSE where std::stol would throw. Unknown keys ignored. */
int ofdm_params_from_config(const char* path, ofdm_params* out);
/* Read one raw key the way ConfigMap::operator[] would (0 when missing). */
int ofdm_config_lookup(const char* path, const char* key, long* value);

/* ---- context ----------------------------------------------------------- */
/* Builds every constant the FRAME_FORM ctor builds (Frame.cpp:213-232):
 * pilot/segment tables (Frame.cpp:31-44), T2 marker (Frame.cpp:139-154),
 * preamble bytes/symbol/template (Frame.cpp:259-294), T2 mask (Frame.cpp:120-133),
 * FFT twiddle tables; uploads them to `device`. */
int ofdm_create(const ofdm_params* params, int device, ofdm_ctx** out);
int ofdm_destroy(ofdm_ctx* ctx);
int ofdm_get_geometry(const ofdm_ctx* ctx, ofdm_geometry* out);
/* Host copies of the constant frame parts (for FRAME_FORM::buf, get(), preamble.*). */
int ofdm_get_t2_symbol(const ofdm_ctx* ctx, double* out /* t2sin_size complex */);
int ofdm_get_preamble(const ofdm_ctx* ctx,
                      uint8_t* bytes_out /* D*num_pr_symb/8, nullable */,
                      double* ofdm_preamble_out /* preamble_len complex, nullable */,
                      double* mod_preamble_out /* D*num_pr_symb complex, nullable */,
                      double* template_out /* pr_sin_len complex, nullable */);

/* ---- device memory helpers (so hosts need not link HIP) ----------------- */
int ofdm_device_alloc(ofdm_ctx* ctx, size_t bytes, void** dptr);
int ofdm_device_free(ofdm_ctx* ctx, void* dptr);
int ofdm_memcpy_h2d(ofdm_ctx* ctx, void* dst, const void* src, size_t bytes, void* stream);
int ofdm_memcpy_d2h(ofdm_ctx* ctx, void* dst, const void* src, size_t bytes, void* stream);
int ofdm_memset_device(ofdm_ctx* ctx, void* dst, int value, size_t bytes, void* stream);
int ofdm_stream_synchronize(ofdm_ctx* ctx, void* stream);
/* Page-locked host memory (DMA-able: copies from / to it are asynchronous). */
int ofdm_host_alloc(ofdm_ctx* ctx, size_t bytes, void** hptr);
int ofdm_host_free(ofdm_ctx* ctx, void* hptr);
/* A non-blocking HIP stream on the ctx's device, and its destruction. */
int ofdm_stream_create(ofdm_ctx* ctx, void** stream);
int ofdm_stream_destroy(ofdm_ctx* ctx, void* stream);
/* Device-to-device copy on a stream; HIP events (timing disabled) to wait
 * for part of a stream's work. */
int ofdm_memcpy_d2d(ofdm_ctx* ctx, void* dst, const void* src, size_t bytes, void* stream);
/* Copy by a kernel on the stream (no DMA engine): dst and src each device
 * memory or page-locked host memory from ofdm_host_alloc. For the small
 * transfers between a stream's kernels, where a DMA hand-off costs more than
 * the copy. */
int ofdm_copy(ofdm_ctx* ctx, void* dst, const void* src, size_t bytes, void* stream);
int ofdm_event_create(ofdm_ctx* ctx, void** event);
int ofdm_event_record(ofdm_ctx* ctx, void* event, void* stream);
int ofdm_event_synchronize(ofdm_ctx* ctx, void* event);
int ofdm_event_destroy(ofdm_ctx* ctx, void* event);

/* ---- tx: FRAME_FORM::write (Frame.cpp:235-237) -> OFDM_FORM::write
 *      (Frame.cpp:185-198) -> Modulation::mod (modulation.cpp:39-50) +
 *      FFT_FORM::write (Frame.cpp:54-70), batched over frames ------------- */
/* bytes: nframes * bytes_per_frame (device). iq_out: device, frame f's
 * message starts at iq_out + 2*f*frame_stride (complex samples; stride >=
 * message_len). Each symbol is [CP | body], body = IFFT(pilots+data)/sqrt(N).
 * iq16_out (nullable, device): the same samples as complex<int16>
 * trunc(x*mult) — FRAME_FORM::get_int16 (Frame.cpp:249-256), same stride.
 * ch (nullable, host struct): AWGN added to iq_out only. */
int ofdm_tx_modulate(ofdm_ctx* ctx, const uint8_t* bytes, size_t nframes,
                     double* iq_out, size_t frame_stride, int16_t* iq16_out,
                     const ofdm_channel* ch, void* stream);

/* Full FRAME_FORM buffers: [T2 | preamble | message] per frame (output_size
 * samples, contiguous frames), i.e. what FRAME_FORM::get() returns. */
int ofdm_tx_frames(ofdm_ctx* ctx, const uint8_t* bytes, size_t nframes,
                   double* frames_out, int16_t* frames16_out, void* stream);

/* ---- rx: OFDM_FORM::fft (Frame.hpp:276-282) -> FFT_FORM::read
 *      (Frame.cpp:73-96) [-> caller's constell /= chan (main.cpp:69-71)]
 *      -> Modulation::demod (modulation.cpp:53-87), batched over frames ---- */
/* iq: device, frame f's message (num_symb [CP|body] symbols) at
 * iq + 2*f*frame_stride. chan (nullable, device): per-frame D complex
 * divisors (chan_stride complex between frames; 0 = one shared vector).
 * constell_out (nullable): nframes*D*num_symb complex, equalised points
 * BEFORE demod's clamp (data/constell.bin layout). bytes_out (nullable):
 * nframes*bytes_per_frame. ref_bytes + bit_errors (both nullable, device):
 * accumulate popcount(bytes ^ ref_bytes) into *bit_errors (u64 atomic). */
int ofdm_rx_demod(ofdm_ctx* ctx, const double* iq, size_t nframes, size_t frame_stride,
                  const double* chan, size_t chan_stride,
                  double* constell_out, uint8_t* bytes_out,
                  const uint8_t* ref_bytes, unsigned long long* bit_errors,
                  void* stream);

/* ofdm_rx_demod on wire-format input: iq16 = complex<int16> samples (4-byte
 * aligned, device), same frame indexing (FRAME_FORM::from_sdr_int16_buf). The
 * int16 -> double conversion of FRAME_FORM::form_int16_to_double
 * (Frame.hpp:472-481) is exact and fused into the load, so results equal
 * ofdm_rx_demod on the converted samples bit for bit, at 4 B/sample input. */
int ofdm_rx_demod_i16(ofdm_ctx* ctx, const int16_t* iq16, size_t nframes, size_t frame_stride,
                      const double* chan, size_t chan_stride,
                      double* constell_out, uint8_t* bytes_out,
                      const uint8_t* ref_bytes, unsigned long long* bit_errors,
                      void* stream);

/* ofdm_rx_demod with a channel divisor that also writes FFT_FORM::read's
 * points before the division (read_out, npts per frame): one launch for
 * rx.cpp:211-220 (message.fft(), the host loop dividing by chan_char_lq(),
 * Modulation::demod). read_out and constell_out may be page-locked host
 * memory from ofdm_host_alloc (the kernel writes it directly). */
int ofdm_rx_demod_read(ofdm_ctx* ctx, const double* iq, size_t nframes, size_t frame_stride,
                       const double* chan, size_t chan_stride,
                       double* read_out, double* constell_out, uint8_t* bytes_out,
                       void* stream);

/* Modulation::demod alone on n points (modulation.cpp:53-87): clamps `points`
 * IN PLACE for QAM (as the reference does) and writes n*k/8 bytes (rounded up,
 * last byte left-aligned as bit_stream_converter pads). Device pointers. */
int ofdm_demap(ofdm_ctx* ctx, double* points, size_t n, uint8_t* bytes_out, void* stream);
/* Modulation::mod alone (modulation.cpp:39-50): nbytes -> nbytes*8/k points. */
int ofdm_map(ofdm_ctx* ctx, const uint8_t* bytes, size_t nbytes, double* points_out, void* stream);

/* FFT_FORM::write (Frame.cpp:54-70) on given points: per frame, D*num_symb
 * constellation points -> FFT_buf layout (num_symb bodies of N samples, no
 * CP): zero, pilots, segments, unnormalised IFFT, /sqrt(N). Device buffers. */
int ofdm_fft_write(ofdm_ctx* ctx, const double* points, size_t nframes, double* fft_buf, void* stream);
/* FFT_FORM::read (Frame.cpp:73-96) on an FFT_buf layout (num_symb bodies of
 * N samples per frame, no CP) -> restored D*num_symb points per frame. The
 * input is not modified (the reference transforms FFT_buf in place). */
int ofdm_fft_read(ofdm_ctx* ctx, const double* fft_buf, size_t nframes, double* restored, void* stream);

/* Modulation::bit_stream_converter (modulation.cpp:90-125): MSB-first repack
 * of len in_bits-wide units into ceil(len*in_bits/out_bits) out_bits-wide
 * units, last one left-aligned; *out_len receives the count. 1 <= bits <= 8. */
int ofdm_bit_convert(ofdm_ctx* ctx, const uint8_t* in, size_t len, int in_bits, int out_bits,
                     uint8_t* out, size_t* out_len, void* stream);

/* FRAME_FORM::form_int16_to_double (Frame.hpp:472-481): n complex<int16>
 * samples -> n complex<double>. Device buffers. */
int ofdm_int16_to_double(ofdm_ctx* ctx, const int16_t* in, size_t n, double* out, void* stream);

/* FRAME_FORM::get_int16 (Frame.cpp:249-256) on n given samples:
 * complex<int16>(x * complex(mult)) = per-component trunc(x*mult). Device buffers. */
int ofdm_double_to_int16(ofdm_ctx* ctx, const double* in, size_t n, int16_t* out, void* stream);

/* ---- rx sync front end ----------------------------- */
/* T2SIN_FORM::corr (Frame.hpp:96-147) over all floor((n-start)/t2sin_size)
 * blocks from `start`: rel_out[b] = energy ratio if > level else 0 (device,
 * nullable). first_out (device int, or page-locked host int from
 * ofdm_host_alloc; nullable): T2SIN_FORM::find_t2sin (Frame.hpp:150-197) =
 * start + b*size of the first block above level, or -1, written once by the
 * launch's last workgroup (system-scope fence after it: a host thread may
 * poll a pinned first_out instead of synchronising the stream). */
int ofdm_t2_scan(ofdm_ctx* ctx, const double* iq, size_t n, long start,
                 double* rel_out, int* first_out, void* stream);

/* PREAMBLE_FORM::find_preamble (Frame.cpp:338-378) for a batch of starts:
 * idx_out[i] = starts[i] + first lag whose normalised correlation with the
 * preamble template exceeds pr_level/1000 (lags 0 .. 2*T2sin_size+pr_sin_len-1,
 * running window energy updated after each test, as the reference), or -10.
 * Samples past n read as 0. Device arrays. Callers add +1 (main.cpp:53). */
int ofdm_find_preamble(ofdm_ctx* ctx, const double* iq, size_t n,
                       const int* starts, size_t nstarts, int* idx_out, void* stream);

/* PREAMBLE_FORM::find_corr (Frame.cpp:297-335): the normalised correlation
 * at every lag from `start` (cor_out[i] = |sum x[start+i+j] c_j| / sqrt(norm_i)
 * where norm_i > 1, else 0; 2*T2sin_size + pr_sin_len lags). Device arrays. */
int ofdm_preamble_corr(ofdm_ctx* ctx, const double* iq, size_t n, long start, double* cor_out,
                       void* stream);

/* ---- per-frame synchronisation, batched over located frames ------------
 * `x` points at the first sample of a form in frame 0; frame f's form starts
 * at x + 2*f*frame_stride. A "form" is nsym consecutive [CP|body] symbols
 * (OFDM_FORM: preamble form nsym = num_pr_symb, message_with_preamble form
 * nsym = num_pr_symb + num_symb). All pointers are device pointers. */

/* OFDM_FORM::pilot_freq_sinh (Frame.hpp:285-337): coarse CFO (cycles/sample)
 * of each frame's form from the pilot peaks of its (N+cp)*nsym-point FFT.
 * Needs (N+cp)*nsym = 2^a or 5*2^a. cfo_out may be pinned host memory
 * (ofdm_host_alloc): each value is written with a system-scope fence, so a
 * caller can poll it instead of synchronising the stream (as ofdm_t2_scan's
 * first_out). */
int ofdm_cfo_estimate(ofdm_ctx* ctx, const double* x, size_t nframes, size_t frame_stride,
                      int nsym, double* cfo_out, void* stream);

/* OFDM_FORM::freq_shift (Frame.hpp:340-348): x[n] *= exp(-2*pi*i*cfo[f]*n),
 * n = 0 .. nsamples-1, in place. cfo: device array of nframes values. */
int ofdm_freq_shift(ofdm_ctx* ctx, double* x, size_t nframes, size_t frame_stride,
                    size_t nsamples, const double* cfo, void* stream);

/* OFDM_FORM::cp_freq_sinh (Frame.hpp:238-263): per-symbol CP-correlation fine
 * CFO, phase-continuous across the nsym symbols of the form, in place. */
int ofdm_cp_sync(ofdm_ctx* ctx, double* x, size_t nframes, size_t frame_stride, int nsym,
                 void* stream);

/* OFDM_FORM::pr_phase_sinh (Frame.hpp:265-274): common phase vs pr[0..pr_len)
 * (device), applied to nsamples samples in place. pr = NULL uses the
 * context's own ofdm_preamble (preamble_len samples), as main.cpp:63 does. */
int ofdm_phase_sync(ofdm_ctx* ctx, double* x, size_t nframes, size_t frame_stride,
                    size_t nsamples, const double* pr, size_t pr_len, void* stream);

/* main.cpp:61-63 after the CFO estimate in one launch: ofdm_freq_shift(cfo),
 * ofdm_cp_sync(nsym), ofdm_phase_sync(pr = NULL), in place on nsamples
 * samples per frame (nsym*(N+cp) <= nsamples; a form up to 158 KB is held in
 * LDS between the stages). x equals the three calls bit for bit; shift_out,
 * cp_out, phase_out (each nullable; device or page-locked host memory from
 * ofdm_host_alloc, frame f at + 2*f*out_stride) receive the form after each
 * stage: the states OFDM_FORM's output[0] holds between the members. */
int ofdm_sync_chain(ofdm_ctx* ctx, double* x, size_t nframes, size_t frame_stride, size_t nsamples,
                    int nsym, const double* cfo, double* shift_out, double* cp_out, double* phase_out,
                    size_t out_stride, void* stream);

/* PREAMBLE_FORM::chan_char_lq (Frame.hpp:389-434): linear-phase channel
 * estimate from the preamble form at x -> chan_out[f*D .. f*D+D) unit phasors
 * (data/phases.bin layout). chan_stride: complex elements between frames. */
int ofdm_chan_estimate(ofdm_ctx* ctx, const double* x, size_t nframes, size_t frame_stride,
                       double* chan_out, size_t chan_stride, void* stream);

/* The main.cpp:60-66 chain on each frame's message_with_preamble region
 * (preamble + message, in place): cfo -> freq_shift -> cp_sync -> phase_sync
 * (context preamble) -> chan_estimate. Clear OFDM_SYNC_* bits to skip a stage
 * (cfo_in, nullable, then supplies the CFO). Outputs nullable. */
enum {
    OFDM_SYNC_CFO = 1, OFDM_SYNC_FREQ_SHIFT = 2, OFDM_SYNC_CP = 4,
    OFDM_SYNC_PHASE = 8, OFDM_SYNC_CHAN = 16, OFDM_SYNC_ALL = 31
};
int ofdm_sync_frames(ofdm_ctx* ctx, double* frames, size_t nframes, size_t frame_stride,
                     int stages, const double* cfo_in, double* cfo_out, double* chan_out,
                     void* stream);

/* ---- streaming rx (rx.cpp:94-221) --------------------------------------
 * Every frame rx.cpp's receive loop locates in a stream of n complex samples
 * (device), then the main.cpp:60-80 chain and demod on each. The walk
 * (rx.cpp:126-198) is, per step:
 *   hit = find_t2sin(pos) (blocks pos + k*T2sin_size); pb = find_preamble(hit) + 1;
 *   pb < -2 -> pos = hit + message_len; else the frame
 *   [pb, pb + preamble_len + message_len) is decoded and pos = pb + message_len.
 * rx.cpp runs it over its SDR ring (from_sdr_buf, rx.cpp:73-91,137-189): the
 * buffer holds output_size + R samples, R = rx_buf_size * output_size (one SDR
 * refill, sdr.hpp:141); find_t2sin only tests blocks that end inside the
 * buffer; a T2 miss refills WITHOUT carrying the tail and restarts the grid
 * at the new buffer, and a hit (preamble) in the buffer's last output_size
 * (+ T2sin_size) samples carries them to the front before the refill. So a
 * marker straddling a refill can be lost, and the grid's phase depends on
 * the ring. The stream API reproduces this exactly (ring mode, the default
 * when the config's rx_buf_size > 0: R from the config; ofdm_set_stream_ring
 * changes R, 0 = no ring, the continuous walk over the stream held whole).
 * In ring mode sample 0 of `iq` is the SDR's first sample and the walk starts
 * as rx.cpp does, at the zero header before it (ofdm_stream_initial_state);
 * samples past n read as zero (the walk ends once its scan passes n).
 * A frame the walk locates past the stream end stops the walk. A frame whose
 * preamble starts before sample 0 (a capture that begins inside it; rx.cpp
 * locates it in its ring's zero header, rx.cpp:105-114,158) is decoded as
 * rx.cpp decodes it, with the samples before 0 read as zero; its pb_out
 * entry is negative.
 * The walk runs as parallel chunk walkers joined into the one sequential
 * walk on the device (chunk = samples per walker, 0 = automatic; see
 * ofdm_walk_tuning). Outputs (device, nullable):
 * pb_out[f] preamble start, bytes_out (bytes_per_frame per frame),
 * constell_out (D*num_symb complex per frame), cfo_out. *nframes_out = frames
 * found; outputs hold the first max_frames. The input is not modified.
 * Returns once the walk is resolved (the host waits for a small status block);
 * the decode is enqueued on `stream` and may still be running, so order later
 * work on `stream`, or synchronise it, before reading the outputs. */
int ofdm_rx_stream(ofdm_ctx* ctx, const double* iq, size_t n, size_t max_frames, long chunk,
                   long* pb_out, uint8_t* bytes_out, double* constell_out, double* cfo_out,
                   size_t* nframes_out, void* stream);
/* ofdm_rx_stream on the SDR's wire format (rx.cpp's from_sdr_int16_buf):
 * iq16 = n complex<int16> samples (device, 4-byte aligned), converted exactly
 * on load; results equal ofdm_rx_stream on the converted stream. */
int ofdm_rx_stream_i16(ofdm_ctx* ctx, const int16_t* iq16, size_t n, size_t max_frames, long chunk,
                       long* pb_out, uint8_t* bytes_out, double* constell_out, double* cfo_out,
                       size_t* nframes_out, void* stream);

/* rx.cpp's SDR ring for the stream walk: R samples per refill (>=
 * output_size), 0 = the continuous walk. Default: rx_buf_size * output_size. */
int ofdm_set_stream_ring(ofdm_ctx* ctx, long ring);
int ofdm_get_stream_ring(const ofdm_ctx* ctx, long* ring);

/* Measurement (no reference counterpart): with on = 1, every later stream
 * call records HIP events around its walk, its resolve and its decode on the
 * call's stream, and ofdm_get_stream_timing returns the last call's three
 * device times in ms (waiting for its decode). The events sit between
 * dependent kernels and cost launch gaps, so time the calls themselves with
 * timing off. Fails when the last call had no timed decode (timing off, the
 * halo walk, or a decode that is not the speculative one). */
int ofdm_set_stream_timing(ofdm_ctx* ctx, int on);
int ofdm_get_stream_timing(ofdm_ctx* ctx, float* walk_ms, float* resolve_ms, float* decode_ms);

/* A state of the stream walk: the position of the next T2 search and, in
 * ring mode, one past the last sample of the ring buffer's current SDR
 * refill (stream coordinates; 0 without a ring). */
typedef struct ofdm_walk_state {
    long pos;
    long ring_end;
} ofdm_walk_state;
/* rx.cpp's initial state (rx.cpp:105-114): ring mode {-output_size, R} (pos 0
 * of a buffer whose zero header precedes the first SDR buffer), else {0, 0}. */
int ofdm_stream_initial_state(const ofdm_ctx* ctx, ofdm_walk_state* out);

/* One shard of a longer stream (multi-GPU streaming rx; the
 * reference's rx.cpp:145-156 carries one frame from ring to ring, this is the
 * same hand-over between GPUs). Exactly one of iq (complex f64) / iq16
 * (complex<int16>) is set; it holds the shard's n samples: its core plus a
 * walk-in halo before it and a tail after it. The walk starts at state
 * `start` (shard-relative; the whole stream's initial state, or the
 * predecessor shard's exit state, or any other state for a speculative walk
 * that the caller checks, see c-ofdm_amd/python/ofdm_stream.py; ring mode
 * also fixes the ring ends' phase: start->ring_end + k*R) and the frames
 * located with pb in [own_lo, own_hi) are decoded into the outputs exactly as
 * ofdm_rx_stream does (pb_out relative to iq). Requires 0 <= own_lo <= own_hi
 * <= n and start->pos >= 0 (ring mode: >= -output_size, start->pos - 2048 -
 * T2sin_size < start->ring_end <= start->pos + R + output_size).
 *   *exit_out: the walk's first state at or past own_hi (where the next
 *     shard's walk resumes; a state equivalent to it, or the state whose step
 *     located the first frame past own_hi), pos -1 if the samples ran out.
 *     In ring mode its pos may lie up to one T2 scan step past its ring end
 *     (a scan that crossed own_hi where the ring runs out: its next step is
 *     the refill); it is a valid start state for the next call.
 *   located (host, nullable, located_cap entries) / located_lag (host,
 *     nullable: ring mode's state after the frame has the later of its two
 *     possible ring ends) / *nlocated_out (nullable): the frames the walk
 *     located from `start` until it stopped: those before own_lo, the owned
 *     ones, and any located past own_hi; *nlocated_out counts them all, and
 *     when they are more than located_cap the arrays hold the first
 *     located_cap - located_cap/2 and the last located_cap/2 of them (what a
 *     shard-to-shard check reads: the walk-in and the frames past own_hi).
 *     Two walks that located the same frame with the same lag are in the
 *     same state from there on. located_cap = 0: no list is made.
 * ofdm_rx_stream(iq, n) is ofdm_rx_stream_shard(iq, n, initial state, 0, n). */
int ofdm_rx_stream_shard(ofdm_ctx* ctx, const double* iq, const int16_t* iq16, size_t n,
                         const ofdm_walk_state* start, long own_lo, long own_hi, size_t max_frames, long chunk,
                         long* pb_out, uint8_t* bytes_out, double* constell_out, double* cfo_out,
                         size_t* nframes_out, long* located, uint8_t* located_lag, size_t located_cap,
                         size_t* nlocated_out, ofdm_walk_state* exit_out, void* stream);

/* Samples a shard of ofdm_rx_stream_shard needs around its core
 * [own_lo, own_hi): *halo_out before own_lo for the walk-in to meet the true
 * walk without a re-walk (the walkers' chunk halo), *tail_out past own_hi for
 * the step that crosses own_hi (one scan step, a T2 block, the preamble
 * window, then the frame). Either pointer may be NULL. */
int ofdm_stream_shard_margins(const ofdm_ctx* ctx, long* halo_out, long* tail_out);

/* ---- multi-GPU (BASELINE configs[4]) -------------------------
 * One process (or thread) per GPU, one ofdm_ctx per GPU. Frames are
 * independent, so a batch shards as contiguous frame ranges with no data-path
 * collective; the job's one collective is a SUM all-reduce of its counters
 * (bit errors, bits, samples, frames) over RCCL (xGMI). A stream shards by
 * samples: each rank walks its core plus a walk-in halo and a tail, and the
 * ranks check their walks against each other with one small exchange
 * (c-ofdm_amd/python/ofdm_stream.py; ofdm_rx_stream_shard). See
 * INTEGRATION.md for the 8-GPU C++ binding (apps/ofdm_multigpu.cpp). */
/* Contiguous share of `total` units for `rank` of `world`, the remainder to
 * the low ranks: [*first, *first + *count). */
int ofdm_shard_range(size_t total, int world, int rank, size_t* first, size_t* count);
/* A stream of n samples sharded by samples: `rank`'s core [*own_lo, *own_hi)
 * and the slice [*slice_lo, *slice_hi) it must hold (the core plus a 3-frame
 * walk-in halo, at least ofdm_stream_shard_margins' halo, and the tail a walk
 * crossing own_hi reads), clipped to [0, n). The plan of ofdm_stream.py's
 * shard_stream. Pure arithmetic on the config: no GPU needed. */
int ofdm_stream_shard_plan(const ofdm_params* params, size_t n, int world, int rank, long* slice_lo,
                           long* slice_hi, long* own_lo, long* own_hi);
/* The job's one collective: SUM all-reduce, in place, of `count` int64
 * counters in device memory over an RCCL communicator (ncclComm_t passed as
 * void*; every rank calls it), enqueued on `stream`. RCCL (librccl.so) is
 * loaded at the first call; without it OFDM_ERR_UNSUPPORTED. */
int ofdm_reduce_counters(ofdm_ctx* ctx, int64_t* counters, size_t count, void* nccl_comm, void* stream);
/* Visible HIP devices (0 and OFDM_ERR_HIP without a GPU). */
int ofdm_device_count(int* count);

/* The sharded stream's report exchange (the protocol of
 * c-ofdm_amd/python/ofdm_stream.py, which these restate for C/C++ hosts).
 * Each rank walks its slice (ofdm_rx_stream_shard: rank 0 from the stream's
 * initial state, the others speculatively from their slice start with the
 * first ring end after it), packs a fixed-size report row, and the ranks
 * all-gather the rows (one ncclAllGather of int64). Every rank then runs the
 * same plan on the same rows: the first rank whose walk is not yet known to
 * be the true walk re-walks from the state the plan returns (its
 * predecessor's exit state), re-packs its row with true_start = 1, and the
 * exchange repeats until the plan accepts every rank. The union of the owned
 * frames is then exactly the one sequential walk's (rx.cpp:125-221).
 * Row length in int64: OFDM_STREAM_REPORT_HEADER + 2 * cap. */
#define OFDM_STREAM_REPORT_HEADER 7
/* Pack a report row. located / located_lag: the walk's located frames in
 * walk order (ABSOLUTE preamble starts: ofdm_rx_stream_shard's relative ones
 * plus slice_lo) and their ring lags (NULL: all 0), nlocated of them, as
 * ofdm_rx_stream_shard returns them with located_cap = 2 * cap (the walk's
 * first and last cap frames when longer); exit_state absolute (pos -1: the
 * samples ran out); true_start: the walk started from a state of the true
 * walk (rank 0, or a re-walk). row: OFDM_STREAM_REPORT_HEADER + 2 * cap. */
int ofdm_stream_report_pack(int rank, long slice_lo, long own_lo, long own_hi, const long* located,
                            const uint8_t* located_lag, size_t nlocated, const ofdm_walk_state* exit_state,
                            int true_start, size_t cap, int64_t* row);
/* The plan over the world's rows (rank order, each packed with the same
 * cap): *rank_out = the first rank to re-walk and *start_out the absolute
 * state to re-walk it from (pos -1: the true walk ended before that rank's
 * core, so it and the ranks after it own no frame), or *rank_out = -1 when
 * every walk is accepted. Rank r is accepted when it was walked from a true
 * state, or when it and rank r-1 located a common frame (same preamble start
 * and lag) no later than r's first owned frame. t2sin_size: the config's
 * (an exit state before the slice moves forward on its own T2 grid). */
int ofdm_stream_stitch_plan(const int64_t* rows, int world, size_t cap, long t2sin_size, int* rank_out,
                            ofdm_walk_state* start_out);

/* ---- stream walk tuning (tests and experiments) --------------------------
 * Per-context settings of the ofdm_rx_stream* walkers; ofdm_create sets the
 * defaults (ofdm_walk_tuning_default), which are the product configuration.
 * chunks_per_slot, halo_milli, ext_milli and lookback change only how the
 * walk is split over walkers: the stitched walk is exact for any values.
 * lookback = 1 (default): each chunk's walker starts at its core (minus
 * halo_milli, default 0) and walks on past the core end until its walk
 * shares a frame with the records the next chunk's walker has published;
 * the chain of joined walks, resolved on the device, is the sequential walk
 * (no host stitching, no re-walks). lookback = 0: every chunk walks in from a
 * halo (default 3 frames) and the host stitches the walks, re-walking a chunk
 * whose walk-in missed the true walk (short halos cost serial re-walks).
 * halo_milli = -1 selects the mode's default. exact_search = 1 replaces the certified FFT
 * preamble search by the reference's serial recurrence; t2_f32 = 0 turns the
 * FP32 T2 screen off (FP64 only). t2_margin is the FP32 screen's
 * certification margin: at or above the default 4e-5 every uncertain block is
 * decided in FP64. A smaller margin would trust raw FP32 ratios near the
 * level and could make the walk differ from the reference, so it is refused
 * (OFDM_ERR_INVALID) unless allow_uncertified = 1, a test-only switch (the
 * tests compare margin 0 against the certified screen). staged_decode = 1
 * decodes through the three staged kernels instead of the one fused decode
 * kernel (same results within the parity bar; for A/B measurements). */
typedef struct ofdm_walk_tuning {
    long chunks_per_slot; /* chunks per resident walker (>= 1; default 1)       */
    long halo_milli;      /* walk-in halo, 1/1000 frames (-1 = default: 0 with
                             lookback, 3000 without)                            */
    long ext_milli;       /* walk-on past the core end, 1/1000 frames (0)       */
    int exact_search;     /* 1: serial-recurrence preamble search (default 0)   */
    int t2_f32;           /* 1: certified FP32 T2 screen (default 1)            */
    double t2_margin;     /* FP32 screen margin (default 4e-5, the certified minimum) */
    int allow_uncertified; /* test only: 1 accepts t2_margin < 4e-5 (default 0) */
    int staged_decode;    /* 1: decode located frames with the staged cfo ->
                             params -> rx kernels even where a fused decode
                             kernel fits (A/B measurements, tests; default 0) */
    int lookback;         /* 1: device-side look-back stitching (default 1)     */
    int max_rec_cap;      /* test only: > 0 caps the records per walker (forces
                             the look-back overflow and its halo-walk fallback;
                             default 0 = the computed bound)                    */
    int pre_f32;          /* 1: certified FP32 tier of the FFT preamble search
                             (an uncertain lag is re-decided in FP64; default 1) */
} ofdm_walk_tuning;
int ofdm_walk_tuning_default(ofdm_walk_tuning* out);
int ofdm_get_walk_tuning(const ofdm_ctx* ctx, ofdm_walk_tuning* out);
int ofdm_set_walk_tuning(ofdm_ctx* ctx, const ofdm_walk_tuning* tuning);

#ifdef __cplusplus
}
#endif
#endif /* OFDM_MI355X_H */
