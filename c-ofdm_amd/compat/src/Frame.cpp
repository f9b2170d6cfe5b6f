// Frame.cpp — the FFT_FORM / T2SIN_FORM / OFDM_FORM / PREAMBLE_FORM /
// FRAME_FORM members of the compatibility layer. Each DSP member runs its
// C-ABI entry (HIP kernels) on its thread's compat stream, on the device
// image of its host buffers:
//   - a FRAME_FORM's buf, from_sdr_buf and from_sdr_int16_buf are mirrored
//     on the device (ofdm_compat::Mirror): a member uploads only what the
//     host changed since the last transfer and copies back what it changed
//     in place, so rx.cpp's per-frame chain moves one frame over PCIe once;
//   - any other host buffer is staged through the pinned arena.
// Every member returns with its results in the host buffers, as the
// reference's do.
#include "OFDM/Frame.hpp"

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdint>
#include <cstdio>
#include <optional>
#include <cstdlib>
#include <cstring>

#include "ofdm_compat.hpp"

using ofdm_compat::check;
using ofdm_compat::Context;

namespace {

constexpr size_t CD = sizeof(complex_double);

// OFDM_COMPAT_TRACE=1: one stderr line per compat call with its wall time
// in microseconds (diagnostics).
bool trace_on()
{
    static const bool on = std::getenv("OFDM_COMPAT_TRACE") != nullptr;
    return on;
}
struct TraceScope {
    const char* name;
    std::chrono::steady_clock::time_point t0;
    explicit TraceScope(const char* n) : name(n), t0(std::chrono::steady_clock::now()) {}
    ~TraceScope()
    {
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        std::fprintf(stderr, "[compat] %s %.1f\n", name, us);
    }
};
#define COMPAT_TRACE(name) \
    std::optional<TraceScope> trace_scope_; \
    if (trace_on()) trace_scope_.emplace(name)

ofdm_params form_params(ConfigMap& config, int num_symb, int mod)
{
    ofdm_params p = ofdm_compat::params_from(config);
    p.num_symb = num_symb;
    p.mod_type = mod;
    return p;
}

// The device image of the host range [h, h + n): a mirror's (made current
// with the host) or a staged copy in scratch slot `slot`.
struct DevRange {
    void* d;
    ofdm_compat::Mirror* m;
    void* h;
    size_t n;
};

DevRange stage_in(Context& ctx, int slot, const void* h, size_t n)
{
    if (ofdm_compat::Mirror* m = ofdm_compat::find_mirror(h, n)) {
        m->push(h, n);
        return {m->device(h), m, const_cast<void*>(h), n};
    }
    void* d = ctx.buf(slot, std::max<size_t>(n, 1));
    ctx.h2d(d, h, n);
    return {d, nullptr, const_cast<void*>(h), n};
}

// A device range the kernel is about to overwrite entirely: no upload.
DevRange stage_out_only(Context& ctx, int slot, void* h, size_t n)
{
    if (ofdm_compat::Mirror* m = ofdm_compat::find_mirror(h, n)) {
        m->settle();
        return {m->device(h), m, h, n};
    }
    return {ctx.buf(slot, std::max<size_t>(n, 1)), nullptr, h, n};
}

// The host range takes the device's (after an in-place device operation).
void stage_back(Context& ctx, const DevRange& r)
{
    if (r.m)
        r.m->pull(r.h, r.n);
    else
        ctx.d2h(r.h, r.d, r.n);
}

// The run-ahead chain (ofdm_compat::Chain) of the FRAME_FORM that owns `form`,
// when it is at `stage` and the frame region's host bytes [p, p + n) are the
// ones it speculated on; otherwise the chain ends (nullptr).
ofdm_compat::Chain* served(const void* form, int stage, const void* p, size_t n)
{
    ofdm_compat::Chain* ch = ofdm_compat::chain_of(form);
    if (!ch) return nullptr;
    if (ch->stage == stage && ofdm_compat::mirror_clean(p, n, ch->gen)) return ch;
    ch->stage = 0;
    return nullptr;
}

// Serve state k (after freq_shift / cp_freq_sinh / pr_phase_sinh) of the
// chain: host region and shadow take it; the device image (which the chain
// advanced in place to the last state) equals the shadow again at k = 2.
void serve_state(Context& ctx, ofdm_compat::Chain& ch, int k)
{
    ofdm_compat::Engine& e = ctx.engine();
    check(ofdm_event_synchronize(e.ctx, ch.ev[3]), "ofdm_event_synchronize");  // the three states
    ofdm_compat::Mirror* m = ofdm_compat::find_mirror(ch.region, ch.region_bytes);
    std::memcpy(ch.region, ch.hstate[k], ch.region_bytes);
    const size_t off = ch.region - m->host;
    std::memcpy(m->shadow + off, ch.hstate[k], ch.region_bytes);
    if (k == 2 && m->stale_lo == off && m->stale_hi == off + ch.region_bytes) m->stale_lo = m->stale_hi = 0;
    ch.stage = k + 2;
}

}  // namespace

// ---------------------------------------------------------------- FFT_FORM
FFT_FORM::FFT_FORM(int fft_size, int num_data_subc, int num_pilot_subc, int num_symb, double pilot_ampl)
    : fft_size(fft_size),
      num_data_subc(num_data_subc),
      num_pilot_subc(num_pilot_subc),
      num_symb(num_symb),
      segment_step(num_data_subc / num_pilot_subc + 1),
      segment_size(segment_step - 1),
      segment_byte_size(segment_size * (int)sizeof(complex_double)),
      FFT_buf((size_t)num_symb * fft_size, complex_double(0.0, 0.0)),
      segment((size_t)num_pilot_subc * num_symb, nullptr),
      pilot((size_t)num_pilot_subc * num_symb, nullptr),
      restored_buf((size_t)num_data_subc * num_symb, 0),
      norm_factor(std::sqrt(static_cast<double>(fft_size))),
      pilot_ampl(pilot_ampl)
{
    COMPAT_TRACE("FFT_FORM::FFT_FORM");
    // pilot comb / segment pointers into FFT_buf (the layout of Frame.cpp:31-44)
    const int half = num_pilot_subc / 2;
    for (int s = 0; s < num_symb; ++s) {
        complex_double* base = FFT_buf.data() + (size_t)s * fft_size;
        int j = 0;
        for (int pos = 1 + segment_size; j < half; ++j, pos += segment_step) {
            pilot[s * num_pilot_subc + j] = base + pos;
            segment[s * num_pilot_subc + j] = base + pos - segment_size;
        }
        for (int pos = fft_size - segment_step * half; j < num_pilot_subc; ++j, pos += segment_step) {
            pilot[s * num_pilot_subc + j] = base + pos;
            segment[s * num_pilot_subc + j] = base + pos + 1;
        }
    }
    ofdm_params p = ofdm_compat::params_default();
    p.fft_size = fft_size;
    p.num_data_subc = num_data_subc;
    p.num_pilot_subc = num_pilot_subc;
    p.num_symb = num_symb;
    p.cp_size = 0;
    p.mod_type = 8;  // unused by FFT_FORM; any k keeps D*S*k byte-aligned
    p.pilot_ampl = std::lround(pilot_ampl * 1000);
    p.pr_sin_len = std::min<long>(p.pr_sin_len, fft_size);
    ctx_ = ofdm_compat::context_for(p);
}

FFT_FORM::~FFT_FORM() = default;

void FFT_FORM::write(complex_vector& input)
{
    COMPAT_TRACE("FFT_FORM::write");
    const size_t np = (size_t)num_data_subc * num_symb;
    complex_vector pts(np, 0);
    std::copy_n(input.begin(), std::min(np, input.size()), pts.begin());
    const DevRange in = stage_in(*ctx_, 0, pts.data(), np * CD);
    const DevRange out = stage_out_only(*ctx_, 1, FFT_buf.data(), FFT_buf.size() * CD);
    check(ofdm_fft_write(ctx_->ctx, (const double*)in.d, 1, (double*)out.d, ctx_->stream()), "ofdm_fft_write");
    stage_back(*ctx_, out);
}

complex_vector& FFT_FORM::read()
{
    COMPAT_TRACE("FFT_FORM::read");
    const DevRange in = stage_in(*ctx_, 0, FFT_buf.data(), FFT_buf.size() * CD);
    const DevRange out = stage_out_only(*ctx_, 1, restored_buf.data(), restored_buf.size() * CD);
    check(ofdm_fft_read(ctx_->ctx, (const double*)in.d, 1, (double*)out.d, ctx_->stream()), "ofdm_fft_read");
    stage_back(*ctx_, out);
    return restored_buf;
}

// ---------------------------------------------------------------- T2SIN_FORM
T2SIN_FORM::T2SIN_FORM(ConfigMap& config)
    : config(config),
      size((int)config["T2sin_size"]),
      f1((int)config["T2_sin_f1"]),
      f2((int)config["T2_sin_f2"]),
      smooth((int)config["smooth"]),
      level((double)config["T2_sin_level"] / 1000),
      detect_mask(size, 0.0),
      detect_buf(size, complex_double(0, 0)),
      mean_freq((f1 + f2) / 2),
      min_f1(std::max(0, f1 - smooth)),
      max_f1(std::max(mean_freq, f1 + smooth)),
      min_f2(std::max(mean_freq, f2 - smooth)),
      max_f2(std::max(size, f2 + smooth))
{
    COMPAT_TRACE("T2SIN_FORM::T2SIN_FORM");
    // detector mask (Frame.cpp:120-133): +1 on [f-smooth, f+smooth] clamped, per tone
    for (int f : {f1, f2})
        for (int i = std::max(0, f - smooth); i <= std::min(size - 1, f + smooth); ++i) detect_mask[i] += 1.0;
    ctx_ = ofdm_compat::context_for(ofdm_compat::params_from(config));
}

void T2SIN_FORM::set(complex_double* buf_ptr)
{
    COMPAT_TRACE("T2SIN_FORM::set");
    buf = buf_ptr;
    if (size) check(ofdm_get_t2_symbol(ctx_->ctx, reinterpret_cast<double*>(buf)), "ofdm_get_t2_symbol");
}

std::vector<double> T2SIN_FORM::corr(complex_vector& signal)
{
    COMPAT_TRACE("T2SIN_FORM::corr");
    const size_t n = signal.size();
    std::vector<double> out(size ? n / size : 0, 0.0);
    if (out.empty()) return out;
    const DevRange x = stage_in(*ctx_, 0, signal.data(), n * CD);
    void* dr = ctx_->buf(1, out.size() * sizeof(double));
    check(ofdm_t2_scan(ctx_->ctx, (const double*)x.d, n, 0, (double*)dr, nullptr, ctx_->stream()), "ofdm_t2_scan");
    ctx_->d2h(out.data(), dr, out.size() * sizeof(double));
    return out;
}

int T2SIN_FORM::find_t2sin(complex_vector& signal, int start_index)
{
    COMPAT_TRACE("T2SIN_FORM::find_t2sin");
    // Frame.hpp:150-197 tests the blocks start + b*size in order and returns
    // the first above the level; each block's decision reads only its own
    // samples. So the scan runs over windows of whole blocks from
    // start_index (a frame or two first, then doubling) and stops at the
    // first window with a hit: only the samples it reads are made current on
    // the device (from_sdr_buf's mirror: normally already there).
    const long n = (long)signal.size();
    if (size <= 0 || start_index < 0 || start_index > n) return -1;
    const long nblocks = (n - start_index) / size;
    long b0 = 0, w = std::max<long>(16, 2L * ctx_->geo.frame_len / size + 2);
    while (b0 < nblocks) {
        const long nb = std::min(w, nblocks - b0);
        const size_t len = (size_t)nb * size;
        const DevRange x = stage_in(*ctx_, 0, signal.data() + start_index + b0 * size, len * CD);
        // the launch's last workgroup writes the answer straight to the
        // engine's pinned word (no copy launch, no stream synchronisation):
        // poll it. The detector's tail may still retire when this returns
        // (it writes the word once, before that); the next call on the
        // thread's stream is ordered after it.
        volatile int* hf = ctx_->engine().t2_answer();
        *hf = INT_MIN;
        check(ofdm_t2_scan(ctx_->ctx, (const double*)x.d, len, 0, nullptr, const_cast<int*>(hf), ctx_->stream()),
              "ofdm_t2_scan");
        const auto t0 = std::chrono::steady_clock::now();
        int first = INT_MIN;
        for (long spin = 0; (first = *hf) == INT_MIN; ++spin)
            if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
                ctx_->sync();  // not landed in 200 ms: wait for the stream (errors surface here)
                first = *hf;
                break;
            }
        if (first >= 0) return (int)(start_index + b0 * size + first);
        b0 += nb;
        w *= 2;
    }
    return -1;
}

// ---------------------------------------------------------------- OFDM_FORM
OFDM_FORM::OFDM_FORM(ConfigMap& config, bool data, bool with_preamble)
    : config(config),
      data(data),
      fft_size((int)config["fft_size"]),
      num_data_subc((int)config["num_data_subc"]),
      num_pilot_subc((int)config["num_pilot_subc"]),
      cp_size((int)config["cp_size"]),
      num_symb((int)((with_preamble) ? config["num_symb"] + config["num_pr_symb"]
                                     : (data) ? config["num_symb"] : config["num_pr_symb"])),
      pr_sin_len((int)config["pr_sin_len"]),
      pr_seed((int)config["pr_seed"]),
      modType((data) ? static_cast<mod_type>(config["modType"]) : mod_type(1)),
      ofdm_len(fft_size + cp_size),
      size((fft_size + cp_size) * num_symb),
      usefull_size(num_data_subc * num_symb),
      output(num_symb, nullptr),
      fft_task(fft_size, num_data_subc, num_pilot_subc, num_symb, double(config["pilot_ampl"]) / 1000),
      Mod(modType),
      byte_fft_size(fft_size * (int)sizeof(complex_double)),
      pilot_ampl((int)config["pilot_ampl"])
{
    COMPAT_TRACE("OFDM_FORM::OFDM_FORM");
    ctx_ = ofdm_compat::context_for(form_params(config, num_symb, modType));
}

void OFDM_FORM::set(complex_double* buf_ptr)
{
    COMPAT_TRACE("OFDM_FORM::set");
    for (int i = 0; i < num_symb; i++) output[i] = buf_ptr + (size_t)(cp_size + fft_size) * i;
}

void OFDM_FORM::write(bit_vector& input)
{
    COMPAT_TRACE("OFDM_FORM::write");
    const size_t nb = (size_t)ctx_->geo.bytes_per_frame;
    bit_vector bytes(nb, 0);
    std::copy_n(input.begin(), std::min(nb, input.size()), bytes.begin());
    const DevRange b = stage_in(*ctx_, 0, bytes.data(), nb);
    const DevRange x = stage_out_only(*ctx_, 1, output[0], (size_t)size * CD);
    check(ofdm_tx_modulate(ctx_->ctx, (const uint8_t*)b.d, 1, (double*)x.d, (size_t)size, nullptr, nullptr,
                           ctx_->stream()),
          "ofdm_tx_modulate");
    stage_back(*ctx_, x);
}

bit_vector OFDM_FORM::read()
{
    COMPAT_TRACE("OFDM_FORM::read");
    const size_t nb = ((size_t)usefull_size * modType + 7) / 8;
    bit_vector out(nb);
    const DevRange x = stage_in(*ctx_, 1, output[0], (size_t)size * CD);
    void* db = ctx_->buf(0, nb);
    check(ofdm_rx_demod(ctx_->ctx, (const double*)x.d, 1, (size_t)size, nullptr, 0, nullptr, (uint8_t*)db, nullptr,
                        nullptr, ctx_->stream()),
          "ofdm_rx_demod");
    ctx_->d2h(out.data(), db, nb);
    return out;
}

complex_vector OFDM_FORM::fft()
{
    COMPAT_TRACE("OFDM_FORM::fft");
    const size_t np = (size_t)usefull_size;
    if (ofdm_compat::Chain* ch = served(this, 4, output[0], (size_t)size * CD)) {
        if (this == ch->msg_form && !ch->fft_served && np * CD == ch->cons_bytes) {
            check(ofdm_event_synchronize(ctx_->engine().ctx, ch->ev[6]), "ofdm_event_synchronize");
            std::memcpy(fft_task.restored_buf.data(), ch->hcons, ch->cons_bytes);
            ch->fft_served = true;
            ch->demod_armed = true;
            ofdm_compat::arm_demod(ch);
            if (ch->chan_served) ch->stage = 0;
            return fft_task.restored_buf;
        }
        ch->stage = 0;
    }
    const DevRange x = stage_in(*ctx_, 1, output[0], (size_t)size * CD);
    void* dc = ctx_->buf(2, np * CD);
    check(ofdm_rx_demod(ctx_->ctx, (const double*)x.d, 1, (size_t)size, nullptr, 0, (double*)dc, nullptr, nullptr,
                        nullptr, ctx_->stream()),
          "ofdm_rx_demod");
    ctx_->d2h(fft_task.restored_buf.data(), dc, np * CD);
    return fft_task.restored_buf;
}

void OFDM_FORM::cp_freq_sinh()
{
    COMPAT_TRACE("OFDM_FORM::cp_freq_sinh");
    if (ofdm_compat::Chain* ch = served(this, 2, output[0], (size_t)size * CD)) {
        if (this == ch->mwp_form) return serve_state(*ctx_, *ch, 1);
        ch->stage = 0;
    }
    const DevRange x = stage_in(*ctx_, 1, output[0], (size_t)size * CD);
    check(ofdm_cp_sync(ctx_->ctx, (double*)x.d, 1, (size_t)size, num_symb, ctx_->stream()), "ofdm_cp_sync");
    stage_back(*ctx_, x);
}

void OFDM_FORM::pr_phase_sinh(complex_double* pr, int pr_size)
{
    COMPAT_TRACE("OFDM_FORM::pr_phase_sinh");
    if (ofdm_compat::Chain* ch = served(this, 3, output[0], (size_t)size * CD)) {
        if (this == ch->mwp_form && (size_t)pr_size == ctx_->ofdm_preamble.size() &&
            std::memcmp(pr, ctx_->ofdm_preamble.data(), (size_t)pr_size * CD) == 0)
            return serve_state(*ctx_, *ch, 2);
        ch->stage = 0;
    }
    const DevRange x = stage_in(*ctx_, 1, output[0], (size_t)size * CD);
    // the caller's preamble copy (main.cpp:63 / rx.cpp:208 pass
    // preamble.ofdm_preamble): when it holds the context's own ofdm_preamble,
    // the device copy made at construction is used
    const double* dp = nullptr;
    size_t plen = (size_t)pr_size;
    if (plen == ctx_->ofdm_preamble.size() &&
        std::memcmp(pr, ctx_->ofdm_preamble.data(), plen * CD) == 0) {
        plen = 0;  // ofdm_phase_sync: the context preamble
    } else {
        const DevRange p = stage_in(*ctx_, 3, pr, plen * CD);
        dp = (const double*)p.d;
    }
    check(ofdm_phase_sync(ctx_->ctx, (double*)x.d, 1, (size_t)size, (size_t)size, dp, plen, ctx_->stream()),
          "ofdm_phase_sync");
    stage_back(*ctx_, x);
}

double OFDM_FORM::pilot_freq_sinh()
{
    COMPAT_TRACE("OFDM_FORM::pilot_freq_sinh");
    ofdm_compat::Chain* ch = ofdm_compat::chain_of(this);
    if (ch) ch->stage = 0;
    if (ch && this == ch->pre_form && output[0] == (complex_double*)ch->region &&
        ofdm_compat::find_mirror(ch->region, ch->region_bytes) && ch->alloc(ctx_->engine())) {
        // the frame's whole message_with_preamble region on the device, then
        // pilot_freq_sinh and the rest of main.cpp:60-66 behind it on copies
        ofdm_compat::Engine& e = ctx_->engine();
        const DevRange r = stage_in(*ctx_, 1, ch->region, ch->region_bytes);
        void* st = e.stream;
        // the estimate lands straight in its pinned word (no copy launch);
        // the chain below reads it from there, and the host polls it. Frames
        // alternate between two words: the previous frame's chain may still
        // be queued behind its estimate (which this host thread has seen) and
        // read its word, while this frame's is reset here; the one before it
        // ran ahead of that estimate in stream order.
        ch->cfo_slot ^= 1;
        double* wc = ch->hcfo + ch->cfo_slot;
        volatile double* hc = wc;
        const uint64_t unset = 0x7ff4dead0badf00dull;  // a NaN the estimate never is
        std::memcpy(const_cast<double*>(hc), &unset, sizeof(unset));
        check(ofdm_cfo_estimate(ctx_->ctx, (const double*)r.d, 1, (size_t)size, num_symb, wc, st),
              "ofdm_cfo_estimate");
        check(ofdm_event_record(e.ctx, ch->ev[0], st), "ofdm_event_record");
        // the chain runs in place on the frame's device image: it is marked
        // stale (ahead of the shadow) until its last state is served
        const size_t nw = ch->region_bytes / CD;
        ofdm_ctx* mw = ch->mwp_ctx->ctx;
        const int nsym = (int)(nw / (size_t)ofdm_len);
        char* dr = static_cast<char*>(r.d);
        r.m->stale_lo = ch->region - r.m->host;
        r.m->stale_hi = r.m->stale_lo + ch->region_bytes;
        // main.cpp:61-63 in one launch, each state written straight into its
        // pinned copy (what output[0] holds after each member)
        check(ofdm_sync_chain(mw, (double*)dr, 1, nw, nw, nsym, wc, (double*)ch->hstate[0],
                              (double*)ch->hstate[1], (double*)ch->hstate[2], 0, st),
              "ofdm_sync_chain");
        check(ofdm_event_record(e.ctx, ch->ev[3], st), "ofdm_event_record");
        check(ofdm_chan_estimate(ch->pre_ctx->ctx, (const double*)dr, 1, ch->pre_bytes / CD, (double*)ch->dchan,
                                 ch->chan_bytes / CD, st),
              "ofdm_chan_estimate");
        e.d2h_pinned(ch->hchan, ch->dchan, ch->chan_bytes);
        // the message transform (OFDM_FORM::fft) and rx.cpp:214-220 behind
        // it, the points divided by this channel (the host loop's complex
        // division) with Modulation::demod's decisions: one rx launch writing
        // all three straight into pinned memory
        const size_t nm = (ch->region_bytes - ch->pre_bytes) / CD;
        check(ofdm_rx_demod_read(ch->msg_ctx->ctx, (const double*)(dr + ch->pre_bytes), 1, nm,
                                 (const double*)ch->dchan, 0, (double*)ch->hcons, (double*)ch->hcons_eq, ch->hbits, st),
              "ofdm_rx_demod_read");
        check(ofdm_event_record(e.ctx, ch->ev[6], st), "ofdm_event_record");
        const auto t0 = std::chrono::steady_clock::now();
        for (long spin = 0;; ++spin) {
            uint64_t bits;
            const double v = *hc;
            std::memcpy(&bits, &v, sizeof(bits));
            if (bits != unset) break;
            if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
                // not landed in 200 ms: wait for the estimate (errors surface here)
                check(ofdm_event_synchronize(e.ctx, ch->ev[0]), "ofdm_event_synchronize");
                break;
            }
        }
        const double shift = *hc;
        ch->cfo = shift;
        ch->stage = 1;
        ch->gen = ofdm_compat::mirror_gen(ch->region, ch->region_bytes);
        ch->chan_served = ch->fft_served = ch->demod_armed = false;
        return shift;
    }
    const DevRange x = stage_in(*ctx_, 1, output[0], (size_t)size * CD);
    void* dc = ctx_->buf(4, sizeof(double));
    check(ofdm_cfo_estimate(ctx_->ctx, (const double*)x.d, 1, (size_t)size, num_symb, (double*)dc, ctx_->stream()),
          "ofdm_cfo_estimate");
    double shift = 0;
    ctx_->d2h(&shift, dc, sizeof(double));
    return shift;
}

void OFDM_FORM::freq_shift(double& shift)
{
    COMPAT_TRACE("OFDM_FORM::freq_shift");
    if (ofdm_compat::Chain* ch = served(this, 1, output[0], (size_t)size * CD)) {
        if (this == ch->mwp_form && std::memcmp(&shift, &ch->cfo, sizeof(double)) == 0)
            return serve_state(*ctx_, *ch, 0);
        ch->stage = 0;
    }
    const DevRange x = stage_in(*ctx_, 1, output[0], (size_t)size * CD);
    void* dc = ctx_->buf(4, sizeof(double));
    ctx_->h2d(dc, &shift, sizeof(double));
    check(ofdm_freq_shift(ctx_->ctx, (double*)x.d, 1, (size_t)size, (size_t)size, (const double*)dc, ctx_->stream()),
          "ofdm_freq_shift");
    stage_back(*ctx_, x);
}

// ---------------------------------------------------------------- PREAMBLE_FORM
PREAMBLE_FORM::PREAMBLE_FORM(ConfigMap& config)
    : OFDM_FORM(config, false),
      level((double)config["pr_level"] / 1000),
      preamble((size_t)usefull_size * modType / 8, 0),
      mod_preamble(size, complex_double(0, 0)),
      ofdm_preamble(size, complex_double(0, 0)),
      conjected_sinh_part(pr_sin_len, complex_double(0, 0)),
      cor((size_t)config["T2sin_size"] * 2 + pr_sin_len, 0.0),
      chan_est(num_data_subc, complex_double(0, 0))
{
    COMPAT_TRACE("PREAMBLE_FORM::PREAMBLE_FORM");
    // mt19937(pr_seed) bytes, made by the context exactly as Frame.cpp:269-272
    check(ofdm_get_preamble(ctx_->ctx, preamble.data(), nullptr, nullptr, nullptr), "ofdm_get_preamble");
}

void PREAMBLE_FORM::set(complex_double* buf_ptr)
{
    COMPAT_TRACE("PREAMBLE_FORM::set");
    OFDM_FORM::set(buf_ptr);
    write(preamble);  // BPSK OFDM preamble on the GPU into the frame buffer
    std::copy_n(output[0], ofdm_preamble.size(), ofdm_preamble.begin());
    mod_preamble = Mod.mod(preamble);
    check(ofdm_get_preamble(ctx_->ctx, nullptr, nullptr, nullptr, reinterpret_cast<double*>(conjected_sinh_part.data())),
          "ofdm_get_preamble");
}

void PREAMBLE_FORM::find_corr(complex_vector& input, int start)
{
    COMPAT_TRACE("PREAMBLE_FORM::find_corr");
    const size_t n = input.size();
    const DevRange x = stage_in(*ctx_, 5, input.data(), n * CD);
    void* dc = ctx_->buf(6, cor.size() * sizeof(double));
    check(ofdm_preamble_corr(ctx_->ctx, (const double*)x.d, n, start, (double*)dc, ctx_->stream()),
          "ofdm_preamble_corr");
    ctx_->d2h(cor.data(), dc, cor.size() * sizeof(double));
}

int PREAMBLE_FORM::find_preamble(complex_vector& input, int start)
{
    COMPAT_TRACE("PREAMBLE_FORM::find_preamble");
    // Frame.cpp:338-378 reads input[start .. start + cor.size() + pr_sin_len):
    // only that window is made current on the device (samples past the
    // vector's end read as zero in the kernel, as before)
    const long n = (long)input.size();
    if (start < 0 || start >= n) return -10;
    const long win = std::min<long>(n - start, (long)cor.size() + pr_sin_len);
    const DevRange x = stage_in(*ctx_, 5, input.data() + start, (size_t)win * CD);
    int* ds = (int*)ctx_->buf(7, sizeof(int));
    check(ofdm_find_preamble(ctx_->ctx, (const double*)x.d, (size_t)win, ctx_->zero_index(), 1, ds, ctx_->stream()),
          "ofdm_find_preamble");
    int idx = -10;
    ctx_->d2h(&idx, ds, sizeof(int));
    return idx < 0 ? idx : idx + start;
}

complex_vector PREAMBLE_FORM::chan_char()
{
    COMPAT_TRACE("PREAMBLE_FORM::chan_char");
    // the averaging estimator (Frame.hpp:375-385), unused by the apps:
    // FFT_FORM::read on the GPU (fft()), then the caller-side per-carrier
    // division and the average, written as the reference writes them
    complex_vector pr = fft();
    std::fill(chan_est.begin(), chan_est.end(), complex_double(0.0, 0.0));
    for (int i = 0; i < num_data_subc * num_symb; i++) chan_est[i % num_data_subc] += pr[i] / mod_preamble[i];
    for (int i = 0; i < num_data_subc; i++) chan_est[i] /= complex_double(num_symb, 0);
    return chan_est;
}

complex_vector& PREAMBLE_FORM::chan_char_lq()
{
    COMPAT_TRACE("PREAMBLE_FORM::chan_char_lq");
    if (ofdm_compat::Chain* ch = served(this, 4, output[0], (size_t)size * CD)) {
        if (this == ch->pre_form && !ch->chan_served && chan_est.size() * CD == ch->chan_bytes) {
            check(ofdm_event_synchronize(ctx_->engine().ctx, ch->ev[6]), "ofdm_event_synchronize");
            std::memcpy(chan_est.data(), ch->hchan, ch->chan_bytes);
            ch->chan_served = true;
            if (ch->fft_served) ch->stage = 0;
            return chan_est;
        }
        ch->stage = 0;
    }
    const DevRange x = stage_in(*ctx_, 1, output[0], (size_t)size * CD);
    void* dc = ctx_->buf(2, chan_est.size() * CD);
    check(ofdm_chan_estimate(ctx_->ctx, (const double*)x.d, 1, (size_t)size, (double*)dc, chan_est.size(),
                             ctx_->stream()),
          "ofdm_chan_estimate");
    ctx_->d2h(chan_est.data(), dc, chan_est.size() * CD);
    return chan_est;
}

// ---------------------------------------------------------------- FRAME_FORM
FRAME_FORM::FRAME_FORM(const std::string& CONFIGNAME)
    : config(parse_config(CONFIGNAME)),
      t2sin(config),
      preamble(config),
      message(config),
      message_with_preamble(config, true, true),
      buf(t2sin.size + preamble.size + message.size, complex_double(0.0, 0.0)),
      int16_buf(buf.size()),
      from_sdr_buf(buf.size() * (config["rx_buf_size"] + 1), complex_double(0.0, 0.0)),
      from_sdr_int16_buf(from_sdr_buf.size()),
      usefull_size(message.usefull_size * message.modType / 8),
      output_size((int)buf.size()),
      bit_preambple(usefull_size, 0)
{
    COMPAT_TRACE("FRAME_FORM::FRAME_FORM");
    // the device images of the frame buffer and the rx ring (f64 and int16)
    mirrors_ = std::make_shared<ofdm_compat::FrameMirrors>();
    mirrors_->add(message.ctx_, buf.data(), buf.size() * CD);
    mirrors_->add(message.ctx_, from_sdr_buf.data(), from_sdr_buf.size() * CD);
    mirrors_->add(message.ctx_, from_sdr_int16_buf.data(), from_sdr_int16_buf.size() * sizeof(std::complex<int16_t>));
    t2sin.set(buf.data());
    preamble.set(buf.data() + t2sin.size);
    message.set(buf.data() + t2sin.size + preamble.size);
    message_with_preamble.set(buf.data() + t2sin.size);
    ofdm_compat::Chain& ch = mirrors_->chain;
    ch.pre_form = &preamble;
    ch.msg_form = &message;
    ch.mwp_form = &message_with_preamble;
    ch.region = reinterpret_cast<char*>(buf.data() + t2sin.size);
    ch.region_bytes = (size_t)message_with_preamble.size * CD;
    ch.pre_bytes = (size_t)preamble.size * CD;
    ch.chan_bytes = preamble.chan_est.size() * CD;
    ch.cons_bytes = (size_t)message.usefull_size * CD;
    ch.pre_ctx = preamble.ctx_;
    ch.msg_ctx = message.ctx_;
    ch.mwp_ctx = message_with_preamble.ctx_;
}

void FRAME_FORM::write(bit_vector& input) { message.write(input); }

bit_vector FRAME_FORM::read(void* transmitted_data)
{
    COMPAT_TRACE("FRAME_FORM::read");
    std::memcpy(buf.data(), transmitted_data, sizeof(complex_double) * buf.size());
    return message.read();
}

complex_vector FRAME_FORM::get() { return buf; }

complex16_vector FRAME_FORM::get_int16()
{
    COMPAT_TRACE("FRAME_FORM::get_int16");
    auto& ctx = message.ctx_;
    const DevRange x = stage_in(*ctx, 1, buf.data(), buf.size() * CD);
    void* d16 = ctx->buf(3, buf.size() * sizeof(std::complex<int16_t>));
    check(ofdm_double_to_int16(ctx->ctx, (const double*)x.d, buf.size(), (int16_t*)d16, ctx->stream()),
          "ofdm_double_to_int16");
    ctx->d2h(int16_buf.data(), d16, buf.size() * sizeof(std::complex<int16_t>));
    return int16_buf;
}

void FRAME_FORM::form_int16_to_double()
{
    COMPAT_TRACE("FRAME_FORM::form_int16_to_double");
    auto& ctx = message.ctx_;
    const size_t n = from_sdr_int16_buf.size();
    const DevRange in = stage_in(*ctx, 6, from_sdr_int16_buf.data(), n * sizeof(std::complex<int16_t>));
    const DevRange out = stage_out_only(*ctx, 5, from_sdr_buf.data(), std::min(n, from_sdr_buf.size()) * CD);
    check(ofdm_int16_to_double(ctx->ctx, (const int16_t*)in.d, std::min(n, from_sdr_buf.size()), (double*)out.d,
                               ctx->stream()),
          "ofdm_int16_to_double");
    stage_back(*ctx, out);
}
