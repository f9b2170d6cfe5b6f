// ofdm_sync.hpp — argument blocks and launchers of the rx sync front end
// (ofdm_sync.hip), called from ofdm_capi.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include "ofdm_internal.hpp"

namespace ofdm {

struct T2Args {
    const double2* iq;      // stream
    const double2* tw;      // T2sin_size forward twiddles
    long start;             // first sample scanned
    long nblocks;           // floor((n - start) / size)
    int a1, b1, a2, b2;     // detector mask bands (Frame.cpp:120-133)
    double level;           // T2_sin_level / 1000
    double* rel_out;        // nullable: nblocks ratios (0 where <= level)
    int* first_scratch;     // device {min block index above level (INT_MAX between launches), done count (0)}
    int* first_out;         // nullable: find_t2sin's answer, written by the last workgroup
};

struct PreambleArgs {
    const double2* iq;
    long n;
    const int* starts;
    long nstarts;
    int* idx_out;
    const double2* templ;   // pr_sin_len conj template
    int L;                  // pr_sin_len
    int cycles;             // 2*T2sin_size + pr_sin_len
    double level;           // pr_level / 1000
    double* cor_out;        // nullable: find_corr values, cycles per start
    double* hv_scratch;     // nullable: nstarts * cycles (the split form), else one workgroup per start
    unsigned* done;         // nstarts counters, zero between launches (with hv_scratch)
};

struct CfoArgs {
    const double2* x;
    long nframes, frame_stride;
    const long* starts;      // nullable: frame f's form at x + starts[f] (stream decode)
    const short2* x16;       // or: complex<int16> stream (with starts)
    const double2* tw_sub;   // M-point forward twiddles
    const double2* tw_full;  // S-point forward twiddles (G == 5)
    const int* borders;      // P + 2 window borders (Frame.hpp:311-321)
    int P;
    double* cfo_out;
    const long* count;       // nullable: frames beyond min(*count, nframes) are skipped (speculative stream decode)
    int host_out;            // cfo_out may be pinned host memory: fence each store system-wide (ofdm_cfo_estimate)
};

struct ShiftArgs {
    double2* x;
    long nframes, frame_stride, nsamples;
    const double* cfo;
};

struct CpArgs {
    double2* x;
    long nframes, frame_stride;
    int nsym, N, cp;
};

struct PhaseArgs {
    double2* x;
    long nframes, frame_stride, nsamples;
    const double2* pr;
    long pr_len;
};

// freq_shift -> cp_freq_sinh -> pr_phase_sinh of one form per workgroup, the
// form held in LDS; each stage's result optionally copied to out[k] (device
// or page-locked host memory) at out[k] + f * out_stride.
struct SyncChainArgs {
    double2* x;
    long nframes, frame_stride, nsamples;
    const double* cfo;
    int nsym, N, cp;
    const double2* pr;
    long pr_len;
    double2* out[3];
    long out_stride;
};

struct ChanArgs {
    DevTables tab;
    const double2* x;           // preamble form
    long nframes, frame_stride;
    const double2* mod_pre;     // D*npr BPSK points
    double2* chan_out;
    long chan_stride;
    int npr, D, P, cp;
    double pilot_ampl;
};

struct WalkArgs {
    const double2* iq;          // stream
    const short2* iq16;         // or: complex<int16> stream (exact int16 -> double on load)
    long n;
    const double2* t2tw;        // T2sin_size forward twiddles
    int a1, b1, a2, b2;         // T2 mask bands
    double t2_level;
    int t2_f32;                 // screen T2 blocks in FP32 (certified; T2sin_size <= 512)
    double t2_margin;           // FP32 screen: certain when |ratio - level| > t2_margin
    const double2* templ;       // pr_sin_len conj template
    int L, cycles;              // pr_sin_len, 2*T2sin_size + pr_sin_len
    double pr_level;
    long pre, msg;              // preamble / message lengths (samples)
    long chunk, halo;           // core samples per chunk; walk-in before the core
    long start;                 // walk state chunk 0 starts from (0: the stream's first sample)
    // rx.cpp's SDR ring (ring > 0; ofdm_set_stream_ring): the walk state is
    // (pos, ring end); the ring ends lie on ring_phase + k*ring. ring = 0: the
    // continuous walk (no ring state)
    long ring;                  // R = rx_buf_size * output_size, or 0
    long ring_phase;            // ring ends = ring_phase + k * ring (0 <= ring_phase < ring)
    long out_len;               // output_size (frame_len): the carry thresholds
    long start_ring_end;        // ring end of chunk 0's start state
    long core_lo, core_hi;      // the chunk cores tile [core_lo, core_hi) (whole stream: [0, n))
    long ext;                   // walk-on past the core end while looking for the first frame there
    long ext_scan;              // >= ext: the same when the core end falls inside a T2 scan
    const int* chunk_ids;       // nullable: chunk of each workgroup (re-walk launches)
    const long* start_pos;      // nullable: exact start state per workgroup (re-walk)
    const long* start_ring;     //   and its ring end (ring mode)
    int* queue;                 // nullable: chunk counter (zeroed) the workgroups take chunks from until
    long nchunks;               //   nchunks are taken (dynamic balance); else one chunk per workgroup
    int max_rec;                // records per chunk
    long* rec;                  // [chunk][max_rec] preamble starts found (| WALK_REC_LAG: ring mode's
                                //   state after the frame has the later of its two possible ring ends)
    int* nrec;                  // [chunk] frames found (> max_rec: overflow)
    long* exit_pos;             // [chunk] walk state at exit; -1: stream exhausted
    long* exit_ring;            // [chunk] its ring end (ring mode)
    int* ncore;                 // nullable: [chunk] records inside the chunk's own core (a contiguous run:
    int* first_in;              //   the walk only moves forward) and the index of the first of them
    int exact_only;             // 1: always the serial-recurrence preamble search (test hook, OFDM_WALK_EXACT=1)
    // FFT correlation for the preamble search (windows of WALK_FFT_M - L + 1
    // lags, L <= WALK_FFT_M - 63): the template's spectrum and the M-point
    // twiddles, or nullptr (direct search)
    const double2* tw_m;        // WALK_FFT_M forward twiddles
    const double2* tspec;       // sum_j c_j e^{+2 pi i k j / M}, k < M
    double tspec_max;           // max_k |tspec_k| (error bound)
    const float2* tspec32;      // tspec rounded to FP32 (the FP32 tier of the FFT search), or nullptr
    // Look-back stitching on the device (lookback = 1; needs `queue`): chunk
    // c > 0 walks from its core start (minus halo) with no walk-in; past its
    // core end it checks each frame it locates against the records the
    // chunk owning that frame has published so far, and stops at the first
    // frame they share (the two walks are one from there on). A walk that
    // shares none walks on, through later cores, to core_hi. Records are
    // published write-through (sc1) with a per-chunk count (pub, zero before
    // the launch; | WALK_PUB_DONE when the chunk's walk ends); link[3c..3c+2]
    // = {chunk m whose walk it joined (-1: none), index of the shared frame
    // in c's records, its index in m's records}.
    int lookback;
    int* pub;
    int* link;
    // nullable diagnostics (OFDM_WALK_PROF): per chunk {start, core end,
    // end (wall_clock64 ticks), frames past the core end, look-back polls
    // that waited, workgroup, XCC id, frames located, ticks in the T2 scans,
    // ticks in the preamble searches, scan steps, FP64 T2 evaluations,
    // preamble searches}
    long* prof;
};
constexpr int WALK_PROF_FIELDS = 14;
constexpr int WALK_PUB_DONE = 1 << 30;
// set by a chunk's walker when it starts (with the count, until DONE): a
// walker looks back on (waits for) only a chunk whose walker is running
constexpr int WALK_PUB_STARTED = 1 << 29;
constexpr int WALK_PUB_COUNT = WALK_PUB_STARTED - 1;
// a walker waits at most this many polls for the chunk it looks back on
constexpr int WALK_SPIN_MAX = 1 << 16;
// A walk record is a preamble start, plus in ring mode the walk state after
// the frame: (pb + message_len, ring end), where the ring end is the first
// ring end past pb + message_len, or the one after it (the next buffer was
// loaded by a carry, rx.cpp:147-156,180-189): bit 62 marks the second case.
// Two walks with equal records are in equal states from there on.
constexpr long WALK_REC_LAG = 1L << 62;
constexpr long WALK_REC_PB = WALK_REC_LAG - 1;
constexpr int WALK_FFT_LOGM = 9;
constexpr int WALK_FFT_M = 1 << WALK_FFT_LOGM;
// Samples one T2 scan step of a walker covers at most (stream_walk_kernel:
// the FP32 screen's 2*G blocks of T2sin_size = 2 x 128 threads x 8 samples
// for T2sin_size <= 512; G = 1 FP64 block of up to 2048 samples above).
constexpr long WALK_SCAN_MAX = 2048;

struct GatherArgs {
    const double2* iq;
    const short2* iq16;         // or: complex<int16> stream, converted into dst
    long n;
    const long* starts;         // frame f copies [starts[f], starts[f] + span)
    long nframes, span;
    double2* dst;               // nframes * span
};

// Fused stream decode, stage 2 (after cfo_kernel): per located frame, the
// cp_freq_sinh symbol phases, the pr_phase_sinh phase and chan_char_lq, all
// from the raw stream samples (no corrected copy is written), plus for each
// message symbol s the phase ramp theta(m) = A_s + B_s*m (m = sample of the
// CP-stripped body) that freq_shift + cp_freq_sinh + pr_phase_sinh apply to
// it, consumed by the rx kernel's stream mode.
struct StreamParamsArgs {
    DevTables tab;              // BPSK tables (the preamble is a BPSK symbol)
    const double2* iq;          // stream
    const short2* iq16;         // or complex<int16> stream
    const long* starts;         // preamble start of each frame
    long nframes;
    const double* cfo;          // per frame (cfo_kernel)
    const double2* pre;         // ofdm_preamble (npr*L samples)
    const double2* mod_pre;     // D*npr BPSK points
    double2* chan_out;          // nframes * D
    bool chan_recip;            // write 1/chan (for rx's chan_recip mode) instead of chan
    double2* corr_out;          // nframes * S * CORR_PER_SYM: the ramp tables (ofdm_internal.hpp)
    int npr, S, D, P, cp;
    double pilot_ampl;
    const long* count;          // nullable: frames beyond min(*count, nframes) are skipped
};

// Speculative frame list of a stream walk: every chunk's records inside its
// own core [k*chunk, (k+1)*chunk), in chunk order, which is the stitched walk
// whenever no chunk needed a re-walk (the host checks and redoes otherwise).
struct CompactArgs {
    const long* rec;            // [chunk][max_rec]
    const int* ncore;           // [chunk] in-core records (WalkArgs::ncore)
    const int* first_in;        // [chunk] index of the first of them
    long nchunks;
    int max_rec;
    long cap;                   // list capacity (max_frames)
    long* list;                 // cap entries
    long* list2;                // nullable: a second copy (the caller's pb_out)
    long* count;                // total located (uncapped)
    int* queue_reset;           // nullable: the walkers' chunk counter, zeroed at the end
};
hipError_t launch_compact(const CompactArgs& a, hipStream_t st);

// The look-back walk's true walk (WalkArgs::lookback), resolved on the device
// in one workgroup: chunk 0 starts at the true state, so the chain 0 -> link
// -> link ... of the chunks whose walks it joins is the sequential walk; each
// chain chunk contributes its records from its entry index to the shared
// frame. Outputs: the owned frames (pb in [own_lo, own_hi)) in walk order, the
// whole chain's records (nullable), and a status block.
constexpr int RESOLVE_MAX_CHUNKS = 8192;
enum { RESOLVE_OVERFLOW = 1, RESOLVE_NEG_FRAME = 2 };
struct ResolveArgs {
    const long* rec;            // [chunk][max_rec]
    const int* nrec;            // [chunk]
    const int* link;            // [chunk][3]
    const long* exit_pos;       // [chunk]
    const long* exit_ring;      // [chunk] (nullable: ring off)
    long nchunks;
    int max_rec;
    long own_lo, own_hi;        // owned preamble starts; own_lo = LONG_MIN: no lower bound (whole stream:
                                //   a frame before sample 0 is the stream's, as rx.cpp decodes it)
    long cap;                   // list capacity
    long* list;                 // owned preamble starts
    long* list2;                // nullable: a second copy (the caller's pb_out)
    long* count;                // owned frames (uncapped)
    long* chain;                // nullable: records of the true walk: the first chain_head, then the
    long chain_head, chain_tail;  //   last chain_tail (all of them, in order, when they are fewer)
    long* status;               // {owned, flags (RESOLVE_*), exit pos, exit ring end, chain records,
                                //  owned frames before sample 0 (a prefix of the list)}
    int* pub;                   // zeroed for the next call
    int* queue_reset;           // nullable: the walkers' chunk counter, zeroed
};
hipError_t launch_resolve(const ResolveArgs& a, hipStream_t st);

hipError_t launch_stream_params(int logn, const StreamParamsArgs& a, hipStream_t st);
// pilot_freq_sinh + the params stage fused (N = 512, 640-point CFO form);
// hipErrorNotSupported for other geometries (use launch_cfo + launch_stream_params)
// the whole fused decode (sync stage + rx stage) in one kernel for the same
// geometries (r: the stream rx arguments; corr / chan pass through LDS)
hipError_t launch_stream_decode(const CfoArgs& c, const StreamParamsArgs& a, const RxArgs& r, int logn, int logm, int g,
                                hipStream_t st);

// the same for N = 2048 / 4096 with cp = N/4 and a 5 x N/4-point CFO form
// (ofdm_stream_wide.hip): whether the geometry fits, and the launch
bool stream_decode_wide_fits(const StreamParamsArgs& a, int logn, int logm, int g, int cfo_p);
hipError_t launch_stream_decode_wide(const CfoArgs& c, const StreamParamsArgs& a, const RxArgs& r, int logn,
                                     hipStream_t st);

hipError_t launch_stream_walk(int logt, const WalkArgs& a, long nblocks, hipStream_t st);
// stream walkers resident at once on the current device (occupancy of the
// walker with this geometry's LDS: 8 per CU for the default geometries)
long stream_walk_slots(int logt, int L, int C, bool fft);
hipError_t launch_gather(const GatherArgs& a, hipStream_t st);
hipError_t launch_t2_scan(int logn, const T2Args& a, int* first_out, hipStream_t st);
hipError_t launch_find_preamble(const PreambleArgs& a, hipStream_t st);
int preamble_splits(int cycles);  // workgroups per start index
hipError_t launch_cfo(int logm, int g, const CfoArgs& a, hipStream_t st);
hipError_t launch_freq_shift(const ShiftArgs& a, hipStream_t st);
hipError_t launch_cp_sync(const CpArgs& a, hipStream_t st);
hipError_t launch_sync_chain(const SyncChainArgs& a, hipStream_t st);
bool sync_chain_fits(long nsamples);
hipError_t launch_phase_sync(const PhaseArgs& a, hipStream_t st);
hipError_t launch_chan(int logn, const ChanArgs& a, hipStream_t st);

}  // namespace ofdm
