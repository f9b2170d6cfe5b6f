// compat.cpp — plumbing (cached contexts, staging), parse_config, psk/qam and
// Modulation of the C++ compatibility layer. Every DSP call goes through the
// C-ABI of include/ofdm_mi355x.h (HIP kernels); there is no CPU DSP path.
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>
#include <emmintrin.h>

#include <algorithm>
#include <cmath>
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>

#include "OFDM/modulation.hpp"
#include "ofdm_compat.hpp"

// ---------------------------------------------------------------- parser
ConfigMap parse_config(const std::string& filename)
{
    std::ifstream file(filename);
    if (!file.is_open()) throw std::runtime_error("Cannot open config file");
    ConfigMap cfg;
    std::string line;
    auto not_space = [](unsigned char ch) { return !std::isspace(ch); };
    while (std::getline(file, line)) {
        line.erase(line.begin(), std::find_if(line.begin(), line.end(), not_space));
        line.erase(std::find_if(line.rbegin(), line.rend(), not_space).base(), line.end());
        if (line.empty() || line[0] == '#') continue;
        const auto pos = line.find('=');
        if (pos == std::string::npos) continue;
        std::string key = line.substr(0, pos), value = line.substr(pos + 1);
        key.erase(std::remove_if(key.begin(), key.end(), ::isspace), key.end());
        value.erase(std::remove_if(value.begin(), value.end(), ::isspace), value.end());
        cfg[key] = std::stol(value);
    }
    return cfg;
}

namespace ofdm_compat {

// OFDM_COMPAT_TRACE set: print a raw backtrace on SIGSEGV/SIGABRT (diagnostics
// for apps linked against the drop-in layer; symbolise with addr2line).
static void crash_handler(int sig)
{
    void* frames[64];
    const int n = backtrace(frames, 64);
    const char msg[] = "[compat] fatal signal, backtrace:\n";
    ssize_t w = write(2, msg, sizeof msg - 1);
    (void)w;
    backtrace_symbols_fd(frames, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

static struct CrashHandlerInstaller {
    CrashHandlerInstaller()
    {
        if (std::getenv("OFDM_COMPAT_TRACE")) {
            signal(SIGSEGV, crash_handler);
            signal(SIGABRT, crash_handler);
        }
    }
} g_crash_handler_installer;

void check(int rc, const char* what)
{
    if (rc != OFDM_OK) throw std::runtime_error(std::string(what) + ": " + ofdm_last_error());
}

static int device_index()
{
    const char* e = std::getenv("OFDM_DEVICE");
    return e ? std::atoi(e) : 0;
}

Context::Context(const ofdm_params& p) : params(p)
{
    check(ofdm_create(&params, device_index(), &ctx), "ofdm_create");
    check(ofdm_get_geometry(ctx, &geo), "ofdm_get_geometry");
    ofdm_preamble.resize((size_t)geo.preamble_len);
    check(ofdm_get_preamble(ctx, nullptr, reinterpret_cast<double*>(ofdm_preamble.data()), nullptr, nullptr),
          "ofdm_get_preamble");
}

const int* Context::zero_index()
{
    if (!zero_) {
        void* d = nullptr;
        check(ofdm_device_alloc(ctx, sizeof(int), &d), "ofdm_device_alloc");
        check(ofdm_memset_device(ctx, d, 0, sizeof(int), engine().stream), "ofdm_memset_device");
        zero_ = static_cast<int*>(d);
    }
    return zero_;
}

Context::~Context()
{
    if (zero_) ofdm_device_free(ctx, zero_);
    for (auto& s : slots_)
        if (s.first) ofdm_device_free(ctx, s.first);
    ofdm_destroy(ctx);
}

void* Context::buf(int slot, size_t bytes)
{
    if ((int)slots_.size() <= slot) slots_.resize(slot + 1, {nullptr, 0});
    auto& s = slots_[slot];
    if (s.second < bytes) {
        if (s.first) ofdm_device_free(ctx, s.first);
        s.first = nullptr;
        check(ofdm_device_alloc(ctx, bytes, &s.first), "ofdm_device_alloc");
        s.second = bytes;
    }
    return s.first;
}

// ---------------------------------------------------------------- engine
Engine& Context::engine()
{
    // one per thread, never destroyed: global FRAME_FORMs (rx.cpp) outlive
    // the thread-local storage at exit, and a leaked stream is harmless
    thread_local Engine* e = nullptr;
    if (!e) {
        auto* n = new Engine;
        ofdm_params p = params_default();
        check(ofdm_create(&p, device_index(), &n->ctx), "ofdm_create (compat engine)");
        check(ofdm_stream_create(n->ctx, &n->stream), "ofdm_stream_create");
        e = n;
    }
    return *e;
}

void* Engine::stage(size_t bytes)
{
    const size_t need = (bytes + 255) & ~(size_t)255;
    if (arena_used + need > arena_bytes) {
        sync();  // every staged copy has landed: the arena is free
        if (need > arena_bytes) {
            if (arena) check(ofdm_host_free(ctx, arena), "ofdm_host_free");
            arena = nullptr;
            arena_bytes = 0;
            const size_t nb = std::max<size_t>(need, (size_t)4 << 20);
            void* h = nullptr;
            check(ofdm_host_alloc(ctx, nb, &h), "ofdm_host_alloc");
            arena = static_cast<char*>(h);
            arena_bytes = nb;
        }
    }
    void* p = arena + arena_used;
    arena_used += need;
    return p;
}

volatile int* Engine::t2_answer()
{
    if (!t2_word) {
        void* h = nullptr;
        check(ofdm_host_alloc(ctx, sizeof(int), &h), "ofdm_host_alloc");
        t2_word = static_cast<int*>(h);
    }
    return t2_word;
}

void Engine::h2d(void* dev, const void* host, size_t bytes)
{
    if (!bytes) return;
    void* st = stage(bytes);
    std::memcpy(st, host, bytes);
    h2d_pinned(dev, st, bytes);
}

void Engine::h2d_pinned(void* dev, const void* pinned, size_t bytes)
{
    if (bytes) check(ofdm_copy(ctx, dev, pinned, bytes, stream), "ofdm_copy");
}

void Engine::d2h_pinned(void* pinned, const void* dev, size_t bytes)
{
    if (bytes) check(ofdm_copy(ctx, pinned, dev, bytes, stream), "ofdm_copy");
}

void Engine::d2h(void* host, const void* dev, size_t bytes)
{
    if (!bytes) {
        sync();
        return;
    }
    void* st = stage(bytes);
    d2h_pinned(st, dev, bytes);
    sync();
    std::memcpy(host, st, bytes);
}

void Engine::sync()
{
    check(ofdm_stream_synchronize(ctx, stream), "ofdm_stream_synchronize");
    arena_used = 0;
}

// ---------------------------------------------------------------- mirrors
namespace {
std::mutex g_mirror_mu;
std::vector<Mirror*> g_mirrors;

// First and last differing 256-byte blocks of a and b over n bytes
// ([lo, hi) in bytes); lo == hi when equal.
void diff_span(const char* a, const char* b, size_t n, size_t& lo, size_t& hi)
{
    constexpr size_t B = 256;
    size_t i = 0;
    while (i < n && std::memcmp(a + i, b + i, std::min(B, n - i)) == 0) i += B;
    if (i >= n) {
        lo = hi = n;
        return;
    }
    size_t j = n;
    while (j > i) {
        const size_t s = j > i + B ? ((j - 1) / B) * B : i;
        const size_t st = std::max(s, i);
        if (std::memcmp(a + st, b + st, j - st) != 0) break;
        j = st;
    }
    lo = i;
    hi = j;
}
}  // namespace

Mirror::Mirror(std::shared_ptr<Context> c, void* h, size_t n) : ctx(std::move(c)), host(static_cast<char*>(h)), bytes(n)
{
    void* d = nullptr;
    void* s = nullptr;
    check(ofdm_device_alloc(ctx->ctx, std::max<size_t>(n, 1), &d), "ofdm_device_alloc");
    dev = static_cast<char*>(d);
    check(ofdm_host_alloc(ctx->ctx, std::max<size_t>(n, 1), &s), "ofdm_host_alloc");
    shadow = static_cast<char*>(s);
    std::memcpy(shadow, host, n);
    Engine& e = ctx->engine();
    e.h2d_pinned(dev, shadow, n);
    e.sync();
    std::lock_guard<std::mutex> lock(g_mirror_mu);
    g_mirrors.push_back(this);
}

Mirror::~Mirror()
{
    {
        std::lock_guard<std::mutex> lock(g_mirror_mu);
        g_mirrors.erase(std::remove(g_mirrors.begin(), g_mirrors.end(), this), g_mirrors.end());
    }
    ofdm_device_free(ctx->ctx, dev);
    ofdm_host_free(ctx->ctx, shadow);
}

void Mirror::settle()
{
    if (stale_lo == stale_hi) return;
    ++gen;
    ctx->engine().h2d_pinned(dev + stale_lo, shadow + stale_lo, stale_hi - stale_lo);
    stale_lo = stale_hi = 0;
}

void Mirror::push(const void* p, size_t n)
{
    settle();
    const size_t off = static_cast<const char*>(p) - host;
    size_t lo, hi;
    diff_span(host + off, shadow + off, n, lo, hi);
    if (lo == hi) return;  // the device already holds these bytes
    ++gen;
    std::memcpy(shadow + off + lo, host + off + lo, hi - lo);
    ctx->engine().h2d_pinned(dev + off + lo, shadow + off + lo, hi - lo);
}

void Mirror::pull(const void* p, size_t n)
{
    const size_t off = static_cast<const char*>(p) - host;
    Engine& e = ctx->engine();
    ++gen;
    e.d2h_pinned(shadow + off, dev + off, n);
    e.sync();
    std::memcpy(host + off, shadow + off, n);
}

Mirror* find_mirror(const void* p, size_t n)
{
    std::lock_guard<std::mutex> lock(g_mirror_mu);
    for (Mirror* m : g_mirrors)
        if (m->covers(p, n)) return m;
    return nullptr;
}

namespace {
std::vector<FrameMirrors*> g_frames;  // guarded by g_mirror_mu
}

FrameMirrors::FrameMirrors()
{
    std::lock_guard<std::mutex> lock(g_mirror_mu);
    g_frames.push_back(this);
}

FrameMirrors::~FrameMirrors()
{
    std::lock_guard<std::mutex> lock(g_mirror_mu);
    g_frames.erase(std::remove(g_frames.begin(), g_frames.end(), this), g_frames.end());
}

Chain* chain_of(const void* form)
{
    std::lock_guard<std::mutex> lock(g_mirror_mu);
    for (FrameMirrors* f : g_frames) {
        Chain& c = f->chain;
        if (form && (form == c.pre_form || form == c.msg_form || form == c.mwp_form)) return &c;
    }
    return nullptr;
}

size_t mirror_gen(const void* p, size_t n)
{
    Mirror* m = find_mirror(p, n);
    return m ? m->gen : 0;
}

bool mirror_clean(const void* p, size_t n, size_t gen)
{
    Mirror* m = find_mirror(p, n);
    if (!m || m->gen != gen) return false;
    const size_t off = static_cast<const char*>(p) - m->host;
    size_t lo, hi;
    diff_span(m->host + off, m->shadow + off, n, lo, hi);
    return lo == hi;
}

namespace {
thread_local Chain* t_demod = nullptr;
}

void arm_demod(Chain* c) { t_demod = c; }
Chain* armed_demod() { return t_demod; }

Chain::~Chain()
{
    if (t_demod == this) t_demod = nullptr;
    if (!mwp_ctx) return;
    ofdm_ctx* c = mwp_ctx->ctx;
    for (int i = 0; i < 3; ++i) {
        if (hstate[i]) ofdm_host_free(c, hstate[i]);
    }
    if (dchan) ofdm_device_free(c, dchan);
    for (void* h : {(void*)hchan, (void*)hcons, (void*)hcfo, (void*)hcons_eq, (void*)hbits})
        if (h) ofdm_host_free(c, h);
    for (void* e : ev)
        if (e) ofdm_event_destroy(c, e);
}

bool Chain::alloc(Engine& e)
{
    (void)e;
    if (hcfo) return true;
    if (!mwp_ctx || !region) return false;
    ofdm_ctx* c = mwp_ctx->ctx;
    void* p = nullptr;
    for (int i = 0; i < 3; ++i) {
        check(ofdm_host_alloc(c, region_bytes, &p), "ofdm_host_alloc");
        hstate[i] = static_cast<char*>(p);
    }
    check(ofdm_device_alloc(c, chan_bytes, &p), "ofdm_device_alloc");
    dchan = static_cast<char*>(p);
    check(ofdm_host_alloc(c, chan_bytes, &p), "ofdm_host_alloc");
    hchan = static_cast<char*>(p);
    check(ofdm_host_alloc(c, cons_bytes, &p), "ofdm_host_alloc");
    hcons = static_cast<char*>(p);
    check(ofdm_host_alloc(c, cons_bytes, &p), "ofdm_host_alloc");
    hcons_eq = static_cast<char*>(p);
    bits_bytes = (size_t)msg_ctx->geo.bytes_per_frame;
    bits_k = msg_ctx->params.mod_type;
    check(ofdm_host_alloc(c, bits_bytes, &p), "ofdm_host_alloc");
    hbits = static_cast<uint8_t*>(p);
    for (auto& v : ev) check(ofdm_event_create(c, &v), "ofdm_event_create");
    check(ofdm_host_alloc(c, 2 * sizeof(double), &p), "ofdm_host_alloc");
    hcfo = static_cast<double*>(p);  // last: the allocation marker
    return true;
}

void FrameMirrors::add(std::shared_ptr<Context> c, void* host, size_t bytes)
{
    m.push_back(std::make_unique<Mirror>(std::move(c), host, bytes));
}

std::shared_ptr<Context> context_for(const ofdm_params& p)
{
    static std::mutex mu;
    static std::map<std::string, std::weak_ptr<Context>> cache;
    const std::string key(reinterpret_cast<const char*>(&p), sizeof p);
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find(key);
    if (it != cache.end())
        if (auto sp = it->second.lock()) return sp;
    auto sp = std::make_shared<Context>(p);
    cache[key] = sp;
    return sp;
}

ofdm_params params_default()
{
    ofdm_params p;
    check(ofdm_params_default(&p), "ofdm_params_default");
    return p;
}

ofdm_params params_from(ConfigMap& c)
{
    ofdm_params p{};
    p.fft_size = c["fft_size"];
    p.num_data_subc = c["num_data_subc"];
    p.num_pilot_subc = c["num_pilot_subc"];
    p.cp_size = c["cp_size"];
    p.num_symb = c["num_symb"];
    p.num_pr_symb = c["num_pr_symb"];
    p.pr_sin_len = c["pr_sin_len"];
    p.pr_seed = c["pr_seed"];
    p.pr_level = c["pr_level"];
    p.t2sin_size = c["T2sin_size"];
    p.t2_sin_f1 = c["T2_sin_f1"];
    p.t2_sin_f2 = c["T2_sin_f2"];
    p.t2_sin_level = c["T2_sin_level"];
    p.smooth = c["smooth"];
    p.mod_type = c["modType"];
    p.pilot_ampl = c["pilot_ampl"];
    p.mult = c["mult"];
    p.rx_buf_size = c["rx_buf_size"];
    p.iterations = c["iterations"];
    return p;
}

}  // namespace ofdm_compat

using ofdm_compat::check;

// ---------------------------------------------------------------- Modulation
// psk / qam: the constellation formulas of modulation.cpp:4-20 (table build, host).
complex_double psk(uint8_t input, double angle, int deg)
{
    const double step = M_PI * 2 / (double)deg;
    const complex_double j(0.0, 1.0);
    return std::exp(j * (step * complex_double(input) + angle));
}

complex_double qam(uint8_t input, int deg)
{
    if ((deg % 2) || deg > 8) return complex_double(0.0, 0.0);
    const uint8_t num = (uint8_t)(1u << (deg / 2));
    return complex_double(2.0 / (num - 1) * double(input % num) - 1.0, 2.0 / (num - 1) * double(input >> (deg / 2)) - 1.0);
}

Modulation::Modulation(mod_type mod) : modulation(mod), constell(1u << mod, 0), mod_index(mod)
{
    for (size_t i = 0; i < constell.size(); i++)
        constell[i] = modulation == bpsk ? psk(uint8_t(i), M_PI_4 * 5, 2) : qam(uint8_t(i), (int)mod_index);
    ofdm_params p = ofdm_compat::params_default();
    p.mod_type = mod;
    ctx_ = ofdm_compat::context_for(p);
}

complex_vector Modulation::mod(std::vector<uint8_t>& in)
{
    const size_t n = (in.size() * 8) / mod_index + ((in.size() * 8) % mod_index > 0);
    complex_vector out(n);
    if (in.empty()) return out;
    void* din = ctx_->buf(0, in.size());
    void* dout = ctx_->buf(1, n * sizeof(complex_double));
    ctx_->h2d(din, in.data(), in.size());
    check(ofdm_map(ctx_->ctx, (const uint8_t*)din, in.size(), (double*)dout, ctx_->stream()), "ofdm_map");
    ctx_->d2h(out.data(), dout, n * sizeof(complex_double));
    return out;
}

// One pass over the caller's points: bitwise equality with the served
// chain's divided points, and (QAM) the in-place clamp to [-1, 1]
// (modulation.cpp:70-75) as max(-1, v) then min(1, v): MAXPD/MINPD return
// their second operand for a NaN, so NaN stays NaN as with std::clamp, and
// -0.0 stays -0.0. Branch-free: noisy points straddle the clamp at random.
static bool equal_then_clamp(double* p, const double* q, size_t nd, bool clamp)
{
    __m128i diff = _mm_setzero_si128();
    const __m128d lo = _mm_set1_pd(-1.0), hi = _mm_set1_pd(1.0);
    for (size_t i = 0; i < nd; i += 2) {  // nd even: complex points
        const __m128d v = _mm_loadu_pd(p + i);
        diff = _mm_or_si128(diff, _mm_xor_si128(_mm_castpd_si128(v),
                                                _mm_loadu_si128(reinterpret_cast<const __m128i*>(q + i))));
        if (clamp) _mm_storeu_pd(p + i, _mm_min_pd(hi, _mm_max_pd(lo, v)));
    }
    return _mm_movemask_epi8(_mm_cmpeq_epi8(diff, _mm_setzero_si128())) == 0xffff;
}

std::vector<uint8_t> Modulation::demod(complex_vector& in)
{
    const size_t n = in.size(), nb = (n * mod_index + 7) / 8;
    std::vector<uint8_t> out(nb);
    if (!n) return out;
    // rx.cpp:214-220 run ahead by the frame's chain: served when these are
    // exactly the points it divided and decided (same kernels, same inputs)
    if (ofdm_compat::Chain* ch = ofdm_compat::armed_demod()) {
        ofdm_compat::arm_demod(nullptr);
        if (ch->demod_armed && (int)mod_index == ch->bits_k && n * sizeof(complex_double) == ch->cons_bytes &&
            nb == ch->bits_bytes) {
            ch->demod_armed = false;
            // (no event wait: the served OFDM_FORM::fft that armed this
            // demod already waited for ev[6], after which the rx kernel's
            // pinned points and decisions are complete)
            if (equal_then_clamp(reinterpret_cast<double*>(in.data()),
                                 reinterpret_cast<const double*>(ch->hcons_eq), 2 * n, modulation != bpsk)) {
                std::memcpy(out.data(), ch->hbits, nb);
                return out;
            }
            // (a mismatch leaves `in` clamped: the demap below decides and
            // clamps clamped points to the same bytes and values)
        }
    }
    void* dp = ctx_->buf(0, n * sizeof(complex_double));
    void* db = ctx_->buf(1, nb);
    ctx_->h2d(dp, in.data(), n * sizeof(complex_double));
    check(ofdm_demap(ctx_->ctx, (double*)dp, n, (uint8_t*)db, ctx_->stream()), "ofdm_demap");
    ctx_->d2h(out.data(), db, nb);
    ctx_->d2h(in.data(), dp, n * sizeof(complex_double));  // clamped in place (modulation.cpp:70-75)
    return out;
}

std::vector<uint8_t> Modulation::bit_stream_converter(size_t ob, size_t ib, std::vector<uint8_t>& in)
{
    const size_t total = in.size() * ib, n = total / ob + (total % ob > 0);
    std::vector<uint8_t> out(n);
    if (in.empty()) return out;
    void* din = ctx_->buf(0, in.size());
    void* dout = ctx_->buf(1, n);
    ctx_->h2d(din, in.data(), in.size());
    size_t m = 0;
    check(ofdm_bit_convert(ctx_->ctx, (const uint8_t*)din, in.size(), (int)ib, (int)ob, (uint8_t*)dout, &m, ctx_->stream()),
          "ofdm_bit_convert");
    ctx_->d2h(out.data(), dout, n);
    return out;
}
