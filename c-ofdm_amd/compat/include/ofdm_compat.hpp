// ofdm_compat.hpp — shared plumbing of the C++ compatibility layer: one
// cached ofdm_ctx per parameter set (device from $OFDM_DEVICE, default 0),
// grow-on-demand device scratch, a per-thread transfer engine (one
// non-blocking HIP stream, a page-locked bounce arena), and device mirrors of
// a FRAME_FORM's host buffers.
//
// Every compat call leaves its thread's stream idle when it returns (it ends
// with the copy of its results to the host), so host buffers are current on
// return, as the reference's members leave them.
#pragma once
#include <complex>
#include <cstddef>
#include <memory>
#include <string>
#include <vector>

#include <ofdm_mi355x.h>
#include "config/parser.hpp"

namespace ofdm_compat {

void check(int rc, const char* what);  // throws std::runtime_error(ofdm_last_error())

// Per-thread transfers: the stream every compat kernel of this thread runs
// on, and a pinned arena for staging pageable host data (reset at each sync,
// so a staged copy's source stays intact until its copy is done). Copies to
// and from pinned memory are kernels on the same stream (ofdm_copy): the
// per-frame transfers are small, and a DMA-engine hand-off between two
// kernels costs more than the copy itself.
struct Engine {
    ofdm_ctx* ctx = nullptr;  // the context that created the stream (kept alive)
    void* stream = nullptr;
    char* arena = nullptr;
    size_t arena_bytes = 0, arena_used = 0;
    int* t2_word = nullptr;   // pinned: find_t2sin's answer, written by the detector's last workgroup
    void* stage(size_t bytes);                                // arena slice (synchronises when full)
    volatile int* t2_answer();                                // t2_word (allocated on first use)
    void h2d(void* dev, const void* host, size_t bytes);      // staged, asynchronous
    void h2d_pinned(void* dev, const void* pinned, size_t bytes);
    void d2h(void* host, const void* dev, size_t bytes);      // synchronous
    void d2h_pinned(void* pinned, const void* dev, size_t bytes);  // asynchronous
    void sync();
};

struct Context {
    ofdm_ctx* ctx = nullptr;
    ofdm_params params{};
    ofdm_geometry geo{};
    std::vector<std::complex<double>> ofdm_preamble;  // host copy of the context's preamble symbol(s)
    explicit Context(const ofdm_params& p);
    ~Context();
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    void* buf(int slot, size_t bytes);  // device scratch, slot-indexed
    Engine& engine();                   // this thread's engine (created on first use)
    void* stream() { return engine().stream; }
    void h2d(void* dev, const void* host, size_t bytes) { engine().h2d(dev, host, bytes); }
    void d2h(void* host, const void* dev, size_t bytes) { engine().d2h(host, dev, bytes); }
    void sync() { engine().sync(); }

private:
    std::vector<std::pair<void*, size_t>> slots_;

public:
    const int* zero_index();  // a device int holding 0 (uploaded once)

private:
    int* zero_ = nullptr;
};

// Device mirror of one host buffer (FRAME_FORM::buf, from_sdr_buf,
// from_sdr_int16_buf). `shadow` (pinned) holds exactly the bytes the device
// copy holds. push() makes the device copy equal the host on a range: it
// compares host and shadow and uploads only the span that differs (nothing,
// when the host has not been written since the last transfer), so the
// reference's in-place member chain (freq_shift, cp_freq_sinh,
// pr_phase_sinh, chan_char_lq, fft) costs one upload per frame. pull() copies
// a range back after an in-place device operation (host = shadow = device).
// Exact for any host writes in between: a host byte that differs from the
// shadow is uploaded, and a byte equal to it is equal to the device's.
struct Mirror {
    std::shared_ptr<Context> ctx;
    char* host = nullptr;
    size_t bytes = 0;
    char* dev = nullptr;
    char* shadow = nullptr;
    size_t gen = 0;  // bumped by every upload and every copy back (content changed)
    // [stale_lo, stale_hi): bytes whose device copy runs ahead of the shadow
    // (the run-ahead chain works in place); the next push or write settles it
    size_t stale_lo = 0, stale_hi = 0;
    Mirror(std::shared_ptr<Context> c, void* host, size_t bytes);
    ~Mirror();
    Mirror(const Mirror&) = delete;
    Mirror& operator=(const Mirror&) = delete;
    bool covers(const void* p, size_t n) const
    {
        const char* q = static_cast<const char*>(p);
        return q >= host && q + n <= host + bytes;
    }
    void* device(const void* p) const { return dev + (static_cast<const char*>(p) - host); }
    void push(const void* p, size_t n);
    void pull(const void* p, size_t n);
    void settle();  // device := shadow on the stale range
};

// The registered mirror covering [p, p + n), or nullptr.
Mirror* find_mirror(const void* p, size_t n);

// The reference apps' per-frame sync chain (main.cpp:60-71, rx.cpp:200-216)
// run ahead on the device. When PREAMBLE_FORM::pilot_freq_sinh is called on a
// FRAME_FORM's own preamble form, the whole chain is enqueued behind the CFO
// kernel on copies of the frame's device image: freq_shift by that CFO,
// cp_freq_sinh, pr_phase_sinh with the context preamble, chan_char_lq and
// the message FFT, each state and result copied to pinned memory. The later
// member calls are then served from those results, without a device round
// trip, when (and only when) their inputs are the ones speculated: the call
// order, the same CFO value (bitwise), the context's own preamble, and host
// bytes of the frame region unchanged since the previous member returned.
// Any other call runs the ordinary path and ends the speculation; served
// results are the same kernels on the same inputs, so bit-identical.
struct Chain {
    const void* pre_form = nullptr;  // identities of the FRAME_FORM's forms
    const void* msg_form = nullptr;
    const void* mwp_form = nullptr;
    char* region = nullptr;  // host message_with_preamble region (buf + T2sin_size)
    size_t region_bytes = 0, pre_bytes = 0, chan_bytes = 0, cons_bytes = 0;
    std::shared_ptr<Context> pre_ctx, msg_ctx, mwp_ctx;
    int stage = 0;  // 1: freq_shift next, 2: cp_freq_sinh, 3: pr_phase_sinh, 4: chan_char_lq / fft
    size_t gen = 0;  // the frame mirror's generation the stage was reached at
    bool chan_served = false, fft_served = false;
    double cfo = 0.0;
    // the states after freq_shift / cp / phase (pinned), results, events
    char* hstate[3] = {};
    char *dchan = nullptr, *hchan = nullptr, *hcons = nullptr;  // hcons: the message transform (FFT_FORM::read)
    double* hcfo = nullptr;  // two pinned words the CFO kernel writes, frames alternate (cfo_slot)
    int cfo_slot = 0;
    // Modulation::demod of the channel-divided message (rx.cpp:211-220): the
    // points and their decisions, written by the rx kernel to pinned memory
    char* hcons_eq = nullptr;
    uint8_t* hbits = nullptr;
    size_t bits_bytes = 0;
    int bits_k = 0;    // the message's bits per point
    bool demod_armed = false;  // fft() was served: the next demod may be
    // events: [0] the CFO landed, [3] the three states, [6] everything (a
    // served member waits for the point its result needs; fewer records cost
    // less host time than they could save in waiting)
    void* ev[7] = {};
    ~Chain();
    bool alloc(Engine& e);
};

// The chain whose speculated demod the calling thread's next
// Modulation::demod may take (set when OFDM_FORM::fft is served), or nullptr.
void arm_demod(Chain* c);
Chain* armed_demod();

// A FRAME_FORM's mirrors and run-ahead chain (registered while alive).
struct FrameMirrors {
    std::vector<std::unique_ptr<Mirror>> m;
    Chain chain;
    FrameMirrors();
    ~FrameMirrors();
    void add(std::shared_ptr<Context> c, void* host, size_t bytes);
};

// The chain of the FRAME_FORM owning `form` (one of its three OFDM forms), or nullptr.
Chain* chain_of(const void* form);
// True when the host bytes [p, p + n) of a mirrored range equal its shadow
// and the mirror is still at generation `gen`.
bool mirror_clean(const void* p, size_t n, size_t gen);
// The generation of the mirror covering [p, p + n) (0 if none).
size_t mirror_gen(const void* p, size_t n);

std::shared_ptr<Context> context_for(const ofdm_params& p);
ofdm_params params_from(ConfigMap& config);
ofdm_params params_default();

}  // namespace ofdm_compat
