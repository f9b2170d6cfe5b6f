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
// so a staged copy's source stays intact until its DMA is done).
struct Engine {
    ofdm_ctx* ctx = nullptr;  // the context that created the stream (kept alive)
    void* stream = nullptr;
    char* arena = nullptr;
    size_t arena_bytes = 0, arena_used = 0;
    void* stage(size_t bytes);                                // arena slice (synchronises when full)
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
};

// The registered mirror covering [p, p + n), or nullptr.
Mirror* find_mirror(const void* p, size_t n);

// A FRAME_FORM's mirrors (registered while alive).
struct FrameMirrors {
    std::vector<std::unique_ptr<Mirror>> m;
    ~FrameMirrors();
    void add(std::shared_ptr<Context> c, void* host, size_t bytes);
};

std::shared_ptr<Context> context_for(const ofdm_params& p);
ofdm_params params_from(ConfigMap& config);
ofdm_params params_default();

}  // namespace ofdm_compat
