// ofdm_internal.hpp — kernel argument blocks and launcher declarations shared
// by ofdm_kernels.hip (device code) and ofdm_capi.cpp (the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ofdm {

// Per-context constant tables, resident in HBM (tiny; L2-resident in practice).
struct DevTables {
    const double2* tw;          // N forward twiddles exp(-2*pi*i*j/N)
    const int* data_bin;        // D: FFT bin of data index d within a symbol
    const int* data_slot;       // D: pilot slot j = d / seg owning data index d
    const int* pilot_bin;       // P
    const int* bin_map;         // N: >=0 data index, -1 unused bin, -2 pilot
    const int* rx_pack;         // max(D, RX_DPT*N/8): lds_swz(data_bin) | data_slot << 16, 0-padded
    const int* pilot_swz;       // max(P, N/8): lds_swz(pilot_bin), 0-padded
    const int* tx_code;         // N: tx per-bin code (tx_code_data / tx_code_fixed)
    const double2* constell;    // 2^k mapping table (Modulation::constell)
};

struct TxArgs {
    DevTables tab;
    const uint8_t* bytes;       // nframes * bytes_per_frame
    const double2* points;      // nullable: mapped points instead of bytes (FFT_FORM::write)
    double2* iq;                // frame f message at iq + f*frame_stride (+ msg_offset)
    int16_t* iq16;              // nullable, same indexing, 2 x int16 per sample
    const double2* header;      // T2+preamble samples (nullable: message only)
    long nframes;
    long frame_stride;          // samples
    long msg_offset;            // samples from frame start to the message
    int header_len;             // samples of header to copy per frame
    int S, D, P, cp, k;
    long bytes_per_frame;
    double pilot_ampl;
    double inv_sqrt_n;
    double mult;
    // AWGN (noise_std <= 0: off)
    double noise_scale;         // noise_std / sqrt(2)
    unsigned long long seed;
    unsigned long long sample_offset;
};

// The staged stream decode's ramp table, per frame and message symbol:
// CORR_PER_SYM phasors {e^{iA}, e^{iB 2^j} (j < CORR_BITS), e^{iBN/8}}. A
// thread's start phasor e^{i(A + B t)} is e^{iA} times the powers its index
// bits select (t < 2^CORR_BITS = 512 = the largest N/8): products of table
// entries, no sincos in the rx, whose register window leaves no room for one.
constexpr int CORR_BITS = 9;
constexpr int CORR_PER_SYM = CORR_BITS + 2;  // double2 entries

struct RxArgs {
    DevTables tab;
    const double2* iq;          // frame f message at iq + f*frame_stride
    const short2* iq16;         // or: complex<int16> input, same indexing (FRAME_FORM::form_int16_to_double fused)
    long nframes;
    long frame_stride;
    const double2* chan;        // nullable: D divisors per frame
    long chan_stride;           // complex elements between frames (0 = shared)
    bool chan_recip;            // chan holds the divisors' reciprocals (multiply instead of divide)
    double2* constell;          // nullable
    double2* read_out;          // nullable (with chan): FFT_FORM::read's points, before the channel divisor
    uint8_t* bytes;             // nullable
    const uint8_t* ref;         // nullable
    unsigned long long* bit_errors;  // nullable
    double2* ystage;            // staged variant only: nframes*S*D scratch
    // stream mode (staged stream decode): frame f's message body starts at
    // starts[f] + start_off, and message symbol s is multiplied by the phase
    // ramp e^{i(A + B m)} (freq_shift + cp_freq_sinh + pr_phase_sinh) whose
    // table is corr[(f*S + s)*CORR_PER_SYM ..] (ofdm_sync.hip stream_params_kernel)
    const long* starts;         // nullable
    long start_off;
    const long* count;          // nullable: frames beyond min(*count, nframes) are skipped
    int* queue;                 // nullable: {next, done} counters (zero; left zero) for dynamic frames
    const double2* corr;
    int S, D, P, seg, cp, k;
    long bytes_per_frame;
    double pilot_ampl;
};

// Launchers (ofdm_kernels.hip). Return hipSuccess or the launch error.
hipError_t launch_tx(int logn, const TxArgs& a, hipStream_t stream);
hipError_t launch_rx(int logn, const RxArgs& a, hipStream_t stream, bool* staged_needed);
hipError_t launch_copy(void* dst, const void* src, size_t n, hipStream_t stream);  // kernel copy (device / mapped pinned)
hipError_t launch_demap(double2* pts, long n, int k, uint8_t* bytes, hipStream_t stream);
hipError_t launch_map(const uint8_t* bytes, long nbytes, int k, const double2* table, double2* out,
                      hipStream_t stream);
hipError_t launch_bit_convert(const uint8_t* in, long len, int in_bits, int out_bits, uint8_t* out, long out_len,
                              hipStream_t stream);
hipError_t launch_i16_to_f64(const int16_t* in, long n, double* out, hipStream_t stream);
hipError_t launch_f64_to_i16(const double* in, long n, double mult, int16_t* out, hipStream_t stream);

// Register-resident rx limits: S*ceil(D/T) <= RX_REG_SLOTS.
constexpr int RX_SMAX = 8;
// LDS slot of FFT element e (ofdm_fft.hpp lds_swz), for host-built tables
inline int lds_swz_host(int e) { return e ^ ((e >> 3) & 7); }
constexpr int RX_DPT = 4;
// rx: persistent resident waves per CU (2 per SIMD: the register window's occupancy)
constexpr int RX_WAVES_PER_CU = 8;
// tx per-bin code: bits 0-12 data index d, bits 13-20 mask applied to its
// k-bit payload symbol (0xff data, 0 otherwise), bits 21-29 base entry of the
// tx kernel's LDS point table (0 for data; TX_LDS_PILOT / TX_LDS_ZERO hold the
// pilot amplitude and 0), so every bin maps as table[(bits(d) & mask) + base].
constexpr int TX_LDS_PILOT = 256, TX_LDS_ZERO = 257;
inline int tx_code_data(int d) { return d | (0xff << 13); }
inline int tx_code_fixed(int entry) { return entry << 21; }
// tx: persistent grid-stride launch size (symbols per workgroup = nsym / grid)
constexpr long TX_MAX_GRID = 4096;

}  // namespace ofdm
