// ofdm_capi.cpp — implementation of include/ofdm_mi355x.h (the C-ABI drop-in
// boundary). Host side: config parsing, validation, the constant tables the
// reference builds in its constructors, and kernel dispatch. Every compute
// entry point launches HIP kernels; there is no CPU compute path.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cctype>
#include <cmath>
#include <complex>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <mutex>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/ofdm_mi355x.h"

// RCCL's types and enum values for the one collective (ofdm_reduce_counters):
// from its header where the build host has it; the library itself is loaded
// at first use, so the core library neither links RCCL nor needs it to run
#if __has_include(<rccl/rccl.h>)
#include <rccl/rccl.h>
static constexpr int kRcclInt64 = ncclInt64, kRcclSum = ncclSum;
#else
static constexpr int kRcclInt64 = 4, kRcclSum = 0;  // rccl.h: ncclInt64, ncclSum (header absent at build time)
#endif
#include "ofdm_internal.hpp"
#include "ofdm_sync.hpp"

using cd = std::complex<double>;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_fail(hipError_t e, const char* what)
{
    return fail(OFDM_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

#define HIP_TRY(expr)                                   \
    do {                                                \
        hipError_t _e = (expr);                         \
        if (_e != hipSuccess) return hip_fail(_e, #expr); \
    } while (0)

int ilog2_exact(long n)
{
    if (n <= 0 || (n & (n - 1))) return -1;
    int l = 0;
    while ((1L << l) < n) ++l;
    return l;
}

// key=value ConfigMap exactly as parse_config (config/parser.cpp:4-33):
// trim, skip blank and '#' lines and lines without '=', strip every space
// from key and value, std::stol the value (throws -> OFDM_ERR_PARSE).
int parse_file(const char* path, std::unordered_map<std::string, long>& cfg)
{
    if (!path) return fail(OFDM_ERR_INVALID, "null config path");
    std::ifstream file(path);
    if (!file.is_open()) return fail(OFDM_ERR_IO, "Cannot open config file");
    std::string line;
    while (std::getline(file, line)) {
        line.erase(line.begin(), std::find_if(line.begin(), line.end(),
                                              [](unsigned char ch) { return !std::isspace(ch); }));
        line.erase(std::find_if(line.rbegin(), line.rend(), [](unsigned char ch) { return !std::isspace(ch); })
                       .base(),
                   line.end());
        if (line.empty() || line[0] == '#') continue;
        auto pos = line.find('=');
        if (pos == std::string::npos) continue;
        std::string key = line.substr(0, pos), value = line.substr(pos + 1);
        key.erase(std::remove_if(key.begin(), key.end(), ::isspace), key.end());
        value.erase(std::remove_if(value.begin(), value.end(), ::isspace), value.end());
        try {
            cfg[key] = std::stol(value);
        } catch (const std::exception& e) {
            return fail(OFDM_ERR_PARSE, "stol failed for key '%s': %s", key.c_str(), e.what());
        }
    }
    return OFDM_OK;
}

template <class T>
int upload(T** dst, const std::vector<T>& v)
{
    HIP_TRY(hipMalloc((void**)dst, std::max<size_t>(1, v.size()) * sizeof(T)));
    if (!v.empty()) HIP_TRY(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return OFDM_OK;
}

}  // namespace

// --------------------------------------------------------------------------
struct ofdm_ctx {
    ofdm_params p{};
    int device = 0;
    int logn = 0;
    int N = 0, D = 0, P = 0, cp = 0, S = 0, k = 0, L = 0, seg = 0, npr = 0, t2 = 0;
    ofdm_geometry geo{};
    // host constants
    std::vector<cd> t2_symbol, ofdm_preamble, mod_preamble, templ;
    std::vector<uint8_t> preamble_bytes;
    std::vector<double> t2_mask;
    // device tables
    double2* d_tw = nullptr;
    int* d_data_bin = nullptr;
    int* d_data_slot = nullptr;
    int* d_pilot_bin = nullptr;
    int* d_bin_map = nullptr;
    int* d_rx_pack = nullptr;
    int* d_pilot_swz = nullptr;
    int* d_tx_code = nullptr;
    double2* d_const = nullptr;
    double2* d_const_bpsk = nullptr;
    double2* d_header = nullptr;   // T2 + preamble
    double2* d_preamble = nullptr; // ofdm_preamble (preamble_len)
    double2* d_templ = nullptr;    // pr_sin_len
    double2* d_tspec = nullptr;    // WALK_FFT_M template spectrum (stream walker FFT search)
    float2* d_tspec32 = nullptr;   // the same rounded to FP32 (the search's FP32 tier)
    double2* d_twm = nullptr;      // WALK_FFT_M twiddles
    double tspec_max = 0.0;
    double2* d_modpre = nullptr;   // D*npr
    double* d_t2mask = nullptr;    // t2 size
    double2* d_t2tw = nullptr;     // t2-size twiddles (T2 detector)
    int* d_first = nullptr;        // T2 detector min-block scratch
    int t2_logn = -1;              // T2sin_size = 2^t2_logn, else -1 (detector unsupported)
    struct CfoPlan {               // pilot_freq_sinh on a form of nsym symbols
        int nsym = 0, logm = -1, g = 0;
        double2* tw_sub = nullptr;
        double2* tw_full = nullptr;
        int* borders = nullptr;
    };
    std::vector<CfoPlan> cfo_plans;
    double* d_cfo_scratch = nullptr;
    size_t cfo_scratch_n = 0;
    // staged-rx scratch (grown on demand, only for num_symb > 8 or D > N/2)
    double2* d_scratch = nullptr;
    size_t scratch_bytes = 0;
    // ofdm_rx_stream scratch (grown on demand): walker records, frame batch,
    // channel estimates, frame starts
    struct Grow {
        void* p = nullptr;
        size_t bytes = 0;
    };
    Grow s_walk, s_batch, s_chan, s_pbs;
    // find_preamble's split form: magnitudes and per-start counters (zero
    // between launches) for up to PRE_SCRATCH_STARTS start indices per call
    static constexpr size_t PRE_SCRATCH_STARTS = 64;
    double* d_pre_hv = nullptr;
    unsigned* d_pre_done = nullptr;
    // pinned host staging for the walk records and the frame list (pageable
    // copies go through a driver bounce buffer and synchronise twice)
    Grow h_walk, h_frames;
    hipStream_t h_frames_stream = nullptr;  // stream of the last copy out of h_frames
    bool h_frames_used = false;
    int* d_queue = nullptr;        // walker chunk counter (zero between calls)
    // rx dynamic-frame counters {next, done}, zero between launches: one slot
    // per HIP stream that launched rx on this context (launches on one stream
    // run in order, so each slot is reset by the launch before the next uses
    // it); streams past RX_QUEUE_SLOTS run with a static frame order
    static constexpr int RX_QUEUE_SLOTS = 32;
    int* d_rxq = nullptr;          // RX_QUEUE_SLOTS x 16 ints (one 64-B line each)
    hipStream_t rxq_stream[RX_QUEUE_SLOTS] = {};
    bool rxq_live[RX_QUEUE_SLOTS] = {};  // slot bound to rxq_stream[i] (false: freed by ofdm_stream_destroy)
    int rxq_used = 0;
    ofdm_walk_tuning walk{};       // stream walker settings (ofdm_set_walk_tuning)
    long ring = 0;                 // rx.cpp's SDR ring R (ofdm_set_stream_ring; 0: the continuous walk)
    bool queue_zero = false;       // the last stream call's compaction left the walker counter zero
    hipEvent_t ev_call = nullptr;  // recorded on call_stream when a stream call comes on another stream
    hipStream_t call_stream = nullptr;  // the last stream call's HIP stream
    bool call_valid = false;       //   (call_stream set)
    hipEvent_t ev_walk = nullptr;  // walk records landed in h_walk
    hipEvent_t ev_wdone = nullptr;  // the walk kernel finished (caller's stream)
    hipStream_t side = nullptr;     // copies the walk records out beside the decode
    // look-back walk: per-chunk publication counts (zero between calls: the
    // resolve kernel clears them), the true walk's records for shard reports,
    // and the resolve kernel's status block (page-locked, written by the kernel)
    Grow s_pub, s_chain, h_status;
    bool pub_zero = false;         // every s_pub word is zero
    // per-phase device times of the last look-back stream call
    // (ofdm_set_stream_timing): events before the walk, after the walk, after
    // the resolve and after the decode, on the call's stream
    bool phase_timing = false;
    bool phase_valid = false;
    hipEvent_t ev_phase[4] = {};

    ofdm::DevTables tables(bool bpsk) const
    {
        ofdm::DevTables t;
        t.tw = d_tw;
        t.data_bin = d_data_bin;
        t.data_slot = d_data_slot;
        t.pilot_bin = d_pilot_bin;
        t.bin_map = d_bin_map;
        t.rx_pack = d_rx_pack;
        t.pilot_swz = d_pilot_swz;
        t.tx_code = d_tx_code;
        t.constell = bpsk ? d_const_bpsk : d_const;
        return t;
    }
};

extern "C" {

const char* ofdm_last_error(void) { return g_err.c_str(); }
int ofdm_abi_version(void) { return OFDM_MI355X_ABI_VERSION; }

int ofdm_params_default(ofdm_params* o)
{
    if (!o) return fail(OFDM_ERR_INVALID, "null params");
    *o = ofdm_params{};
    o->fft_size = 512;
    o->num_data_subc = 256;
    o->num_pilot_subc = 8;
    o->cp_size = 128;
    o->num_symb = 8;
    o->num_pr_symb = 1;
    o->pr_sin_len = 128;
    o->pr_seed = 42;
    o->pr_level = 500;
    o->t2sin_size = 256;
    o->t2_sin_f1 = 17;
    o->t2_sin_f2 = 51;
    o->t2_sin_level = 800;
    o->smooth = 5;
    o->mod_type = 4;
    o->pilot_ampl = 2500;
    o->mult = 200;
    o->rx_buf_size = 40;
    o->iterations = 10000;
    return OFDM_OK;
}

int ofdm_params_from_config(const char* path, ofdm_params* o)
{
    if (!o) return fail(OFDM_ERR_INVALID, "null params");
    std::unordered_map<std::string, long> c;
    int rc = parse_file(path, c);
    if (rc) return rc;
    // ConfigMap::operator[] semantics: missing keys read as 0
    o->fft_size = c["fft_size"];
    o->num_data_subc = c["num_data_subc"];
    o->num_pilot_subc = c["num_pilot_subc"];
    o->cp_size = c["cp_size"];
    o->num_symb = c["num_symb"];
    o->num_pr_symb = c["num_pr_symb"];
    o->pr_sin_len = c["pr_sin_len"];
    o->pr_seed = c["pr_seed"];
    o->pr_level = c["pr_level"];
    o->t2sin_size = c["T2sin_size"];
    o->t2_sin_f1 = c["T2_sin_f1"];
    o->t2_sin_f2 = c["T2_sin_f2"];
    o->t2_sin_level = c["T2_sin_level"];
    o->smooth = c["smooth"];
    o->mod_type = c["modType"];
    o->pilot_ampl = c["pilot_ampl"];
    o->mult = c["mult"];
    o->rx_buf_size = c["rx_buf_size"];
    o->iterations = c["iterations"];
    return OFDM_OK;
}

int ofdm_config_lookup(const char* path, const char* key, long* value)
{
    if (!key || !value) return fail(OFDM_ERR_INVALID, "null key/value");
    std::unordered_map<std::string, long> c;
    int rc = parse_file(path, c);
    if (rc) return rc;
    *value = c[key];
    return OFDM_OK;
}

static int validate(const ofdm_params* p)
{
    const long N = p->fft_size, D = p->num_data_subc, P = p->num_pilot_subc, k = p->mod_type;
    if (ilog2_exact(N) < 6 || ilog2_exact(N) > 12)
        return fail(OFDM_ERR_UNSUPPORTED, "fft_size=%ld: the HIP FFT covers powers of two 64..4096", N);
    if (P < 1 || D < P || D % P)
        return fail(OFDM_ERR_UNSUPPORTED, "num_data_subc=%ld must be a positive multiple of num_pilot_subc=%ld", D,
                    P);
    if (P > 256) return fail(OFDM_ERR_UNSUPPORTED, "num_pilot_subc > 256");
    if (!(k == 1 || k == 2 || k == 4 || k == 6 || k == 8))
        return fail(OFDM_ERR_INVALID, "modType=%ld is not one of 1,2,4,6,8 (OFDM/modulation.hpp:11-17)", k);
    if (p->cp_size < 0 || p->cp_size > N) return fail(OFDM_ERR_INVALID, "cp_size out of range");
    if (p->num_symb < 1 || p->num_pr_symb < 1) return fail(OFDM_ERR_INVALID, "num_symb/num_pr_symb must be >= 1");
    if ((D * p->num_symb * k) % 8 || (D * k) % 8)
        return fail(OFDM_ERR_UNSUPPORTED, "num_data_subc*modType must be a multiple of 8 bits");
    if ((D * p->num_pr_symb) % 8) return fail(OFDM_ERR_UNSUPPORTED, "preamble bits must fill bytes");
    // layout must stay inside [1, N) without collisions: FFT_FORM ctor Frame.cpp:31-44
    {
        std::vector<char> used(N, 0);
        const long step = D / P + 1, seg = D / P, half = P / 2;
        long j = 0;
        auto take = [&](long b) {
            if (b < 1 || b >= N || used[b]) return false;
            used[b] = 1;
            return true;
        };
        for (long pos = 1 + seg; j < half; ++j, pos += step) {
            if (!take(pos)) return fail(OFDM_ERR_INVALID, "pilot comb does not fit fft_size");
            for (long t = 0; t < seg; ++t)
                if (!take(pos - seg + t)) return fail(OFDM_ERR_INVALID, "data segments do not fit fft_size");
        }
        for (long pos = N - step * half; j < P; ++j, pos += step) {
            if (!take(pos)) return fail(OFDM_ERR_INVALID, "pilot comb does not fit fft_size");
            for (long t = 0; t < seg; ++t)
                if (!take(pos + 1 + t)) return fail(OFDM_ERR_INVALID, "data segments do not fit fft_size");
        }
    }
    if (p->t2sin_size < 0 || (p->t2sin_size && (p->t2_sin_f1 < 0 || p->t2_sin_f1 >= p->t2sin_size ||
                                                p->t2_sin_f2 < 0 || p->t2_sin_f2 >= p->t2sin_size)))
        return fail(OFDM_ERR_INVALID, "T2 tones outside T2sin_size");
    if (p->pr_sin_len < 0 || p->pr_sin_len > (N + p->cp_size) * p->num_pr_symb)
        return fail(OFDM_ERR_INVALID, "pr_sin_len exceeds the preamble");
    return OFDM_OK;
}

int ofdm_destroy(ofdm_ctx* c)
{
    if (!c) return OFDM_OK;
    (void)hipSetDevice(c->device);
    void* ptrs[] = {c->d_tw, c->d_data_bin, c->d_data_slot, c->d_pilot_bin, c->d_bin_map, c->d_rx_pack,
                    c->d_pilot_swz, c->d_tx_code, c->d_const,
                    c->d_const_bpsk, c->d_header, c->d_preamble, c->d_templ, c->d_tspec, c->d_tspec32, c->d_twm, c->d_modpre,
                    c->d_t2mask,
                    c->d_t2tw, c->d_first, c->d_scratch, c->d_cfo_scratch, c->d_pre_hv, c->d_pre_done};
    for (void* q : ptrs)
        if (q) (void)hipFree(q);
    for (auto* g : {&c->s_walk, &c->s_batch, &c->s_chan, &c->s_pbs, &c->s_pub, &c->s_chain})
        if (g->p) (void)hipFree(g->p);
    for (auto* g : {&c->h_walk, &c->h_frames, &c->h_status})
        if (g->p) (void)hipHostFree(g->p);
    if (c->d_queue) (void)hipFree(c->d_queue);
    if (c->d_rxq) (void)hipFree(c->d_rxq);
    if (c->ev_call) (void)hipEventDestroy(c->ev_call);
    if (c->ev_walk) (void)hipEventDestroy(c->ev_walk);
    if (c->ev_wdone) (void)hipEventDestroy(c->ev_wdone);
    if (c->side) (void)hipStreamDestroy(c->side);
    for (hipEvent_t ev : c->ev_phase)
        if (ev) (void)hipEventDestroy(ev);
    for (auto& pl : c->cfo_plans) {
        if (pl.tw_sub) (void)hipFree(pl.tw_sub);
        if (pl.tw_full) (void)hipFree(pl.tw_full);
        if (pl.borders) (void)hipFree(pl.borders);
    }
    delete c;
    return OFDM_OK;
}

static std::vector<double2> twiddles(int n)
{
    std::vector<double2> w(n);
    for (int j = 0; j < n; ++j) {
        const double a = 2.0 * M_PI * (double)j / (double)n;
        w[j] = make_double2(std::cos(a), -std::sin(a));
    }
    return w;
}

// Modulation::Modulation table (modulation.cpp:4-36).
static std::vector<double2> constellation(int k)
{
    std::vector<double2> t(1u << k);
    if (k == 1) {
        const double step = M_PI * 2 / (double)2;
        for (int i = 0; i < 2; ++i) {
            const cd z = std::exp(cd(0.0, 1.0) * (step * cd(i) + M_PI_4 * 5));
            t[i] = make_double2(z.real(), z.imag());
        }
    } else {
        const unsigned num = 1u << (k / 2);
        for (unsigned i = 0; i < t.size(); ++i) {
            const uint8_t in = (uint8_t)i;
            t[i] = make_double2(2.0 / (num - 1) * double(in % num) - 1.0, 2.0 / (num - 1) * double(in >> (k / 2)) - 1.0);
        }
    }
    return t;
}

int ofdm_create(const ofdm_params* params, int device, ofdm_ctx** out)
{
    if (!params || !out) return fail(OFDM_ERR_INVALID, "null argument");
    *out = nullptr;
    int rc = validate(params);
    if (rc) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(OFDM_ERR_HIP, "no HIP device available (the modem core has no CPU path)");
    if (device < 0 || device >= ndev) return fail(OFDM_ERR_INVALID, "device %d out of range", device);
    HIP_TRY(hipSetDevice(device));

    ofdm_ctx* c = new ofdm_ctx;
    c->p = *params;
    c->device = device;
    c->N = (int)params->fft_size;
    c->logn = ilog2_exact(c->N);
    c->D = (int)params->num_data_subc;
    c->P = (int)params->num_pilot_subc;
    c->cp = (int)params->cp_size;
    c->S = (int)params->num_symb;
    c->k = (int)params->mod_type;
    c->L = c->N + c->cp;
    c->seg = c->D / c->P;
    c->npr = (int)params->num_pr_symb;
    c->t2 = (int)params->t2sin_size;

    ofdm_geometry& g = c->geo;
    g.symbol_len = c->L;
    g.message_len = (long)c->L * c->S;
    g.preamble_len = (long)c->L * c->npr;
    g.frame_len = c->t2 + g.preamble_len + g.message_len;
    g.ring_len = g.frame_len * (params->rx_buf_size + 1);
    g.data_per_frame = (long)c->D * c->S;
    g.bytes_per_frame = (long)c->D * c->S * c->k / 8;
    g.segment_size = c->seg;

    // FFT_FORM layout (Frame.cpp:31-44)
    std::vector<int> pilot(c->P), segst(c->P), data_bin(c->D), data_slot(c->D), bin_map(c->N, -1);
    {
        const int step = c->seg + 1, half = c->P / 2;
        int j = 0;
        for (int pos = 1 + c->seg; j < half; ++j, pos += step) {
            pilot[j] = pos;
            segst[j] = pos - c->seg;
        }
        for (int pos = c->N - step * half; j < c->P; ++j, pos += step) {
            pilot[j] = pos;
            segst[j] = pos + 1;
        }
        for (int jj = 0; jj < c->P; ++jj) {
            g.pilot_bin[jj] = pilot[jj];
            g.segment_bin[jj] = segst[jj];
            bin_map[pilot[jj]] = -2;
            for (int t = 0; t < c->seg; ++t) {
                const int d = jj * c->seg + t;
                data_bin[d] = segst[jj] + t;
                data_slot[d] = jj;
                bin_map[segst[jj] + t] = d;
            }
        }
    }
    // rx per-thread tables, zero-padded to the rx kernel's fixed per-thread
    // counts (RX_DPT data and one pilot per thread) so it loads them unguarded
    std::vector<int> rx_pack(std::max(c->D, ofdm::RX_DPT * (c->N / 8)), 0),
        pilot_swz(std::max(c->P, c->N / 8), 0);
    for (int d = 0; d < c->D; ++d) rx_pack[d] = ofdm::lds_swz_host(data_bin[d]) | (data_slot[d] << 16);
    for (int j = 0; j < c->P; ++j) pilot_swz[j] = ofdm::lds_swz_host(pilot[j]);
    // tx per-bin codes (ofdm_internal.hpp tx_code): data index + 0xff mask, or
    // the pilot / zero entry of the kernel's LDS point table
    std::vector<int> tx_code(c->N);
    for (int b = 0; b < c->N; ++b)
        tx_code[b] = bin_map[b] >= 0 ? ofdm::tx_code_data(bin_map[b])
                                     : ofdm::tx_code_fixed(bin_map[b] == -2 ? ofdm::TX_LDS_PILOT : ofdm::TX_LDS_ZERO);
    if ((rc = upload(&c->d_rx_pack, rx_pack)) || (rc = upload(&c->d_pilot_swz, pilot_swz)) ||
        (rc = upload(&c->d_tx_code, tx_code)) ||
        (rc = upload(&c->d_tw, twiddles(c->N))) || (rc = upload(&c->d_data_bin, data_bin)) ||
        (rc = upload(&c->d_data_slot, data_slot)) || (rc = upload(&c->d_pilot_bin, pilot)) ||
        (rc = upload(&c->d_bin_map, bin_map)) || (rc = upload(&c->d_const, constellation(c->k))) ||
        (rc = upload(&c->d_const_bpsk, constellation(1)))) {
        ofdm_destroy(c);
        return rc;
    }

    // T2SIN_FORM::set (Frame.cpp:139-154): X[f1] = X[f2] = 0.5, unnormalised
    // backward DFT of T2sin_size points = two complex tones of amplitude 0.5.
    c->t2_symbol.assign(c->t2, cd(0, 0));
    if (c->t2) {
        std::vector<cd> spec(c->t2, cd(0, 0));
        spec[params->t2_sin_f1] = cd(0.5, 0);
        spec[params->t2_sin_f2] = cd(0.5, 0);
        for (int n = 0; n < c->t2; ++n) {
            cd acc(0, 0);
            for (int kk = 0; kk < c->t2; ++kk) {
                if (spec[kk] == cd(0, 0)) continue;
                const double a = 2.0 * M_PI * (double)(((long)kk * n) % c->t2) / (double)c->t2;
                acc += spec[kk] * cd(std::cos(a), std::sin(a));
            }
            c->t2_symbol[n] = acc;
        }
    }
    // T2 detector mask (Frame.cpp:120-133)
    c->t2_mask.assign(std::max(1, c->t2), 0.0);
    if (c->t2) {
        const int sm = (int)params->smooth, f1 = (int)params->t2_sin_f1, f2 = (int)params->t2_sin_f2;
        for (int i = std::max(0, f1 - sm); i <= std::min(c->t2 - 1, f1 + sm); ++i) c->t2_mask[i] += 1.0;
        for (int i = std::max(0, f2 - sm); i <= std::min(c->t2 - 1, f2 + sm); ++i) c->t2_mask[i] += 1.0;
    }

    // PREAMBLE_FORM (Frame.cpp:259-294): mt19937(pr_seed) bytes, BPSK OFDM
    // symbol(s) made by the tx kernel itself, conj template normalised.
    {
        const long nb = (long)c->D * c->npr / 8;
        c->preamble_bytes.resize(nb);
        std::mt19937 rng(params->pr_seed);
        std::uniform_int_distribution<int> dist(0, 255);
        for (auto& b : c->preamble_bytes) b = (uint8_t)dist(rng);

        const long plen = g.preamble_len;
        uint8_t* d_b = nullptr;
        double2* d_pre = nullptr;
        HIP_TRY(hipMalloc((void**)&d_b, std::max<long>(1, nb)));
        HIP_TRY(hipMalloc((void**)&d_pre, plen * sizeof(double2)));
        HIP_TRY(hipMemcpy(d_b, c->preamble_bytes.data(), nb, hipMemcpyHostToDevice));
        ofdm::TxArgs a{};
        a.tab = c->tables(true);
        a.bytes = d_b;
        a.iq = d_pre;
        a.nframes = 1;
        a.frame_stride = plen;
        a.S = c->npr;
        a.D = c->D;
        a.P = c->P;
        a.cp = c->cp;
        a.k = 1;
        a.bytes_per_frame = nb;
        a.pilot_ampl = (double)params->pilot_ampl / 1000;
        a.inv_sqrt_n = 1.0 / std::sqrt((double)c->N);
        a.mult = (double)params->mult;
        hipError_t e = ofdm::launch_tx(c->logn, a, nullptr);
        if (e == hipSuccess) e = hipDeviceSynchronize();
        std::vector<double2> pre(plen);
        if (e == hipSuccess) e = hipMemcpy(pre.data(), d_pre, plen * sizeof(double2), hipMemcpyDeviceToHost);
        (void)hipFree(d_b);
        (void)hipFree(d_pre);
        if (e != hipSuccess) {
            ofdm_destroy(c);
            return hip_fail(e, "preamble synthesis");
        }
        c->ofdm_preamble.resize(plen);
        for (long i = 0; i < plen; ++i) c->ofdm_preamble[i] = cd(pre[i].x, pre[i].y);
        // mod_preamble = Mod.mod(preamble) (BPSK points, bit_stream_converter(1,8))
        const auto bp = constellation(1);
        c->mod_preamble.resize((long)c->D * c->npr);
        for (long i = 0; i < (long)c->mod_preamble.size(); ++i) {
            const int bit = (c->preamble_bytes[i >> 3] >> (7 - (i & 7))) & 1;
            c->mod_preamble[i] = cd(bp[bit].x, bp[bit].y);
        }
        const int Lt = (int)params->pr_sin_len;
        c->templ.resize(Lt);
        double norm = 0.0;
        for (int i = 0; i < Lt; ++i) {
            c->templ[i] = std::conj(c->ofdm_preamble[i]);
            norm += std::abs(c->templ[i] * c->templ[i]);
        }
        norm = std::sqrt(norm);
        for (int i = 0; i < Lt; ++i) c->templ[i] /= cd(norm);
    }
    {
        std::vector<double2> hdr(c->t2 + g.preamble_len), pre(g.preamble_len), tpl(c->templ.size()),
            mp(c->mod_preamble.size());
        for (int i = 0; i < c->t2; ++i) hdr[i] = make_double2(c->t2_symbol[i].real(), c->t2_symbol[i].imag());
        for (long i = 0; i < g.preamble_len; ++i) {
            pre[i] = make_double2(c->ofdm_preamble[i].real(), c->ofdm_preamble[i].imag());
            hdr[c->t2 + i] = pre[i];
        }
        for (size_t i = 0; i < tpl.size(); ++i) tpl[i] = make_double2(c->templ[i].real(), c->templ[i].imag());
        // stream walker FFT search (ofdm_sync.hip walk_preamble_fft): template
        // spectrum tspec_k = sum_j c_j e^{+2 pi i k j / M}, long double
        std::vector<double2> tsp, twm;
        if (params->pr_sin_len <= ofdm::WALK_FFT_M - 63) {  // windows of >= 64 lags
            const int M = ofdm::WALK_FFT_M;
            tsp.resize(M);
            for (int k = 0; k < M; ++k) {
                long double re = 0, im = 0;
                for (size_t j = 0; j < c->templ.size(); ++j) {
                    const long double a = 2.0L * 3.14159265358979323846264338327950288L * (long double)((k * (long)j) % M) / M;
                    const long double cr = c->templ[j].real(), ci = c->templ[j].imag();
                    const long double co = cosl(a), si = sinl(a);
                    re += cr * co - ci * si;
                    im += cr * si + ci * co;
                }
                tsp[k] = make_double2((double)re, (double)im);
                c->tspec_max = std::max(c->tspec_max, std::hypot(tsp[k].x, tsp[k].y));
            }
            twm = twiddles(M);
        }
        for (size_t i = 0; i < mp.size(); ++i) mp[i] = make_double2(c->mod_preamble[i].real(), c->mod_preamble[i].imag());
        std::vector<float2> tsp32(tsp.size());
        for (size_t k = 0; k < tsp.size(); ++k) tsp32[k] = make_float2((float)tsp[k].x, (float)tsp[k].y);
        if ((!tsp.empty() && ((rc = upload(&c->d_tspec, tsp)) || (rc = upload(&c->d_tspec32, tsp32)) ||
                              (rc = upload(&c->d_twm, twm)))) ||
            (rc = upload(&c->d_header, hdr)) || (rc = upload(&c->d_preamble, pre)) || (rc = upload(&c->d_templ, tpl)) ||
            (rc = upload(&c->d_modpre, mp)) || (rc = upload(&c->d_t2mask, c->t2_mask))) {
            ofdm_destroy(c);
            return rc;
        }
    }
    // T2 detector tables
    // T2 detector scratch {min block = INT_MAX, done count = 0} (left so by
    // every t2_scan launch), word 2: preamble_corr's start index
    if ((rc = upload(&c->d_first, std::vector<int>{INT_MAX, 0, 0, 0}))) {
        ofdm_destroy(c);
        return rc;
    }
    // find_preamble's split scratch for up to PRE_SCRATCH_STARTS start indices
    // (counters zero between launches); more starts per call take the
    // one-workgroup form, so the entry point never allocates
    {
        const size_t cyc = 2 * (size_t)c->p.t2sin_size + (size_t)c->p.pr_sin_len;
        if ((rc = upload(&c->d_pre_hv, std::vector<double>(ofdm_ctx::PRE_SCRATCH_STARTS * cyc, 0.0))) ||
            (rc = upload(&c->d_pre_done, std::vector<unsigned>(ofdm_ctx::PRE_SCRATCH_STARTS, 0u)))) {
            ofdm_destroy(c);
            return rc;
        }
    }
    if (c->t2 >= 64 && c->t2 <= 4096 && ilog2_exact(c->t2) > 0) {
        c->t2_logn = ilog2_exact(c->t2);
        if ((rc = upload(&c->d_t2tw, twiddles(c->t2)))) {
            ofdm_destroy(c);
            return rc;
        }
    }
    // rx dynamic-frame counters: zero now, and left zero by every rx launch
    const size_t qbytes = ofdm_ctx::RX_QUEUE_SLOTS * 16 * sizeof(int);
    hipError_t qe = hipMalloc((void**)&c->d_rxq, qbytes);
    if (qe == hipSuccess) qe = hipMemset(c->d_rxq, 0, qbytes);
    if (qe == hipSuccess) qe = hipDeviceSynchronize();
    if (qe != hipSuccess) {
        ofdm_destroy(c);
        return hip_fail(qe, "rx frame counters");
    }
    ofdm_walk_tuning_default(&c->walk);
    c->ring = std::max(0L, c->p.rx_buf_size) * c->geo.frame_len;  // rx.cpp:53 / sdr.hpp:141
    *out = c;
    return OFDM_OK;
}

// The rx frame-queue slot of `st` (nullptr: no slot free, static frame order).
static int* rx_queue(ofdm_ctx* c, hipStream_t st)
{
    int free_slot = -1;
    for (int i = 0; i < c->rxq_used; ++i) {
        if (c->rxq_live[i] && c->rxq_stream[i] == st) return c->d_rxq + 16 * i;
        if (!c->rxq_live[i] && free_slot < 0) free_slot = i;
    }
    if (free_slot < 0) {
        if (c->rxq_used == ofdm_ctx::RX_QUEUE_SLOTS) return nullptr;
        free_slot = c->rxq_used++;
    }
    c->rxq_stream[free_slot] = st;
    c->rxq_live[free_slot] = true;
    return c->d_rxq + 16 * free_slot;
}

// ofdm_stream_destroy: the stream's slot becomes free for a later stream (its
// counters are zero once the stream has drained: the last workgroup of every
// rx launch resets them), so a handle value reused by a new stream starts on
// a clean slot and short-lived streams do not use the slots up.
static void rx_queue_release(ofdm_ctx* c, hipStream_t st)
{
    for (int i = 0; i < c->rxq_used; ++i)
        if (c->rxq_live[i] && c->rxq_stream[i] == st) c->rxq_live[i] = false;
}

// A launch that did not start leaves its slot as it was (zero). One that
// faulted poisons the context anyway (HIP errors are sticky); the slot is
// still zeroed so a recovered context starts clean.
static void rx_queue_reset(ofdm_ctx* c, int* q, hipStream_t st)
{
    if (q) (void)hipMemsetAsync(q, 0, 2 * sizeof(int), st);
}

// pilot_freq_sinh plan for a form of nsym symbols: S = (N+cp)*nsym = M or 5*M,
// M = 2^m; window borders exactly as Frame.hpp:311-321 computes them.
static int cfo_plan(ofdm_ctx* c, int nsym, ofdm_ctx::CfoPlan** out)
{
    for (auto& pl : c->cfo_plans)
        if (pl.nsym == nsym) {
            *out = &pl;
            return OFDM_OK;
        }
    const long S = (long)c->L * nsym;
    ofdm_ctx::CfoPlan pl;
    pl.nsym = nsym;
    if (ilog2_exact(S) >= 6 && ilog2_exact(S) <= 12) {
        pl.g = 1;
        pl.logm = ilog2_exact(S);
    } else if (S % 5 == 0 && ilog2_exact(S / 5) >= 6 && ilog2_exact(S / 5) <= 10) {
        pl.g = 5;
        pl.logm = ilog2_exact(S / 5);
    } else {
        return fail(OFDM_ERR_UNSUPPORTED, "pilot_freq_sinh: form length %ld is not 2^a or 5*2^a (64 <= 2^a <= %d)", S,
                    4096);
    }
    const int P = c->P;
    const double rel_bw = double(c->D + c->P) / (c->N);
    const double rel_pilot_w = rel_bw / P;
    const int pilot_w = int(S * rel_pilot_w);
    std::vector<int> borders(P + 2);
    for (int i = 0, j = int((1.0 - rel_bw - rel_pilot_w) / 2.0 * S); i < P + 2; i++) {
        borders[i] = j;
        j += pilot_w;
    }
    borders[0] = std::max(0, borders[0]);
    for (int b : borders)
        if (b < 0 || b > S) return fail(OFDM_ERR_UNSUPPORTED, "pilot_freq_sinh windows leave the spectrum");
    int rc;
    if ((rc = upload(&pl.tw_sub, twiddles(1 << pl.logm))) || (rc = upload(&pl.borders, borders))) return rc;
    if (pl.g == 5 && (rc = upload(&pl.tw_full, twiddles((int)S)))) return rc;
    c->cfo_plans.push_back(pl);
    *out = &c->cfo_plans.back();
    return OFDM_OK;
}

int ofdm_get_geometry(const ofdm_ctx* c, ofdm_geometry* o)
{
    if (!c || !o) return fail(OFDM_ERR_INVALID, "null argument");
    *o = c->geo;
    return OFDM_OK;
}

int ofdm_get_t2_symbol(const ofdm_ctx* c, double* o)
{
    if (!c || !o) return fail(OFDM_ERR_INVALID, "null argument");
    std::memcpy(o, c->t2_symbol.data(), c->t2_symbol.size() * sizeof(cd));
    return OFDM_OK;
}

int ofdm_get_preamble(const ofdm_ctx* c, uint8_t* bytes, double* pre, double* modp, double* templ)
{
    if (!c) return fail(OFDM_ERR_INVALID, "null ctx");
    if (bytes) std::memcpy(bytes, c->preamble_bytes.data(), c->preamble_bytes.size());
    if (pre) std::memcpy(pre, c->ofdm_preamble.data(), c->ofdm_preamble.size() * sizeof(cd));
    if (modp) std::memcpy(modp, c->mod_preamble.data(), c->mod_preamble.size() * sizeof(cd));
    if (templ) std::memcpy(templ, c->templ.data(), c->templ.size() * sizeof(cd));
    return OFDM_OK;
}

// ---- memory helpers
int ofdm_device_alloc(ofdm_ctx* c, size_t bytes, void** d)
{
    if (!c || !d) return fail(OFDM_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMalloc(d, std::max<size_t>(bytes, 1)));
    return OFDM_OK;
}
int ofdm_device_free(ofdm_ctx* c, void* d)
{
    if (!c) return fail(OFDM_ERR_INVALID, "null ctx");
    if (d) HIP_TRY(hipFree(d));
    return OFDM_OK;
}
int ofdm_memcpy_h2d(ofdm_ctx* c, void* dst, const void* src, size_t n, void* st)
{
    if (!c) return fail(OFDM_ERR_INVALID, "null ctx");
    HIP_TRY(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, (hipStream_t)st));
    return OFDM_OK;
}
int ofdm_memcpy_d2h(ofdm_ctx* c, void* dst, const void* src, size_t n, void* st)
{
    if (!c) return fail(OFDM_ERR_INVALID, "null ctx");
    HIP_TRY(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, (hipStream_t)st));
    return OFDM_OK;
}
int ofdm_memset_device(ofdm_ctx* c, void* dst, int v, size_t n, void* st)
{
    if (!c) return fail(OFDM_ERR_INVALID, "null ctx");
    HIP_TRY(hipMemsetAsync(dst, v, n, (hipStream_t)st));
    return OFDM_OK;
}
int ofdm_stream_synchronize(ofdm_ctx* c, void* st)
{
    if (!c) return fail(OFDM_ERR_INVALID, "null ctx");
    HIP_TRY(hipStreamSynchronize((hipStream_t)st));
    return OFDM_OK;
}

int ofdm_host_alloc(ofdm_ctx* c, size_t bytes, void** h)
{
    if (!c || !h) return fail(OFDM_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipHostMalloc(h, std::max<size_t>(bytes, 1), hipHostMallocDefault));
    return OFDM_OK;
}
int ofdm_host_free(ofdm_ctx* c, void* h)
{
    if (!c) return fail(OFDM_ERR_INVALID, "null ctx");
    if (h) HIP_TRY(hipHostFree(h));
    return OFDM_OK;
}
int ofdm_stream_create(ofdm_ctx* c, void** st)
{
    if (!c || !st) return fail(OFDM_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *st = s;
    return OFDM_OK;
}
int ofdm_stream_destroy(ofdm_ctx* c, void* st)
{
    if (!c) return fail(OFDM_ERR_INVALID, "null ctx");
    if (st) {
        HIP_TRY(hipStreamSynchronize((hipStream_t)st));
        rx_queue_release(c, (hipStream_t)st);
        if (c->call_valid && c->call_stream == (hipStream_t)st) c->call_valid = false;  // drained above
        HIP_TRY(hipStreamDestroy((hipStream_t)st));
    }
    return OFDM_OK;
}
int ofdm_memcpy_d2d(ofdm_ctx* c, void* dst, const void* src, size_t n, void* st)
{
    if (!c) return fail(OFDM_ERR_INVALID, "null ctx");
    if (n) HIP_TRY(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, (hipStream_t)st));
    return OFDM_OK;
}
int ofdm_copy(ofdm_ctx* c, void* dst, const void* src, size_t n, void* st)
{
    if (!c) return fail(OFDM_ERR_INVALID, "null ctx");
    if (n && (!dst || !src)) return fail(OFDM_ERR_INVALID, "null argument");
    hipError_t e = ofdm::launch_copy(dst, src, n, (hipStream_t)st);
    if (e != hipSuccess) return hip_fail(e, "copy launch");
    return OFDM_OK;
}
int ofdm_event_create(ofdm_ctx* c, void** ev)
{
    if (!c || !ev) return fail(OFDM_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    hipEvent_t e = nullptr;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    *ev = e;
    return OFDM_OK;
}
int ofdm_event_record(ofdm_ctx* c, void* ev, void* st)
{
    if (!c || !ev) return fail(OFDM_ERR_INVALID, "null argument");
    HIP_TRY(hipEventRecord((hipEvent_t)ev, (hipStream_t)st));
    return OFDM_OK;
}
int ofdm_event_synchronize(ofdm_ctx* c, void* ev)
{
    if (!c || !ev) return fail(OFDM_ERR_INVALID, "null argument");
    HIP_TRY(hipEventSynchronize((hipEvent_t)ev));
    return OFDM_OK;
}
int ofdm_event_destroy(ofdm_ctx* c, void* ev)
{
    if (!c) return fail(OFDM_ERR_INVALID, "null ctx");
    if (ev) HIP_TRY(hipEventDestroy((hipEvent_t)ev));
    return OFDM_OK;
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Device scratch that only grows (contents not preserved).
static int grow(ofdm_ctx* c, ofdm_ctx::Grow& g, size_t need)
{
    if (need <= g.bytes) return OFDM_OK;
    HIP_TRY(hipSetDevice(c->device));
    if (g.p) HIP_TRY(hipFree(g.p));
    g.p = nullptr;
    g.bytes = 0;
    HIP_TRY(hipMalloc(&g.p, need));
    g.bytes = need;
    return OFDM_OK;
}

// Pinned host staging that only grows (contents not preserved).
static int grow_host(ofdm_ctx* c, ofdm_ctx::Grow& g, size_t need)
{
    if (need <= g.bytes) return OFDM_OK;
    HIP_TRY(hipSetDevice(c->device));
    if (g.p) HIP_TRY(hipHostFree(g.p));
    g.p = nullptr;
    g.bytes = 0;
    HIP_TRY(hipHostMalloc(&g.p, need, hipHostMallocDefault));
    g.bytes = need;
    return OFDM_OK;
}

static void fill_tx(const ofdm_ctx* c, ofdm::TxArgs& a, const uint8_t* bytes, size_t nframes, double* iq,
                    size_t stride, int16_t* iq16, const ofdm_channel* ch)
{
    a.tab = c->tables(false);
    a.bytes = bytes;
    a.iq = reinterpret_cast<double2*>(iq);
    a.iq16 = iq16;
    a.nframes = (long)nframes;
    a.frame_stride = (long)stride;
    a.S = c->S;
    a.D = c->D;
    a.P = c->P;
    a.cp = c->cp;
    a.k = c->k;
    a.bytes_per_frame = c->geo.bytes_per_frame;
    a.pilot_ampl = (double)c->p.pilot_ampl / 1000;
    a.inv_sqrt_n = 1.0 / std::sqrt((double)c->N);
    a.mult = (double)c->p.mult;
    if (ch && ch->noise_std > 0.0) {
        a.noise_scale = ch->noise_std * M_SQRT1_2;
        a.seed = ch->seed;
        a.sample_offset = ch->sample_offset;
    }
}

int ofdm_tx_modulate(ofdm_ctx* c, const uint8_t* bytes, size_t nframes, double* iq_out, size_t frame_stride,
                     int16_t* iq16_out, const ofdm_channel* ch, void* stream)
{
    if (!c || !bytes || !iq_out) return fail(OFDM_ERR_INVALID, "null argument");
    if (frame_stride < (size_t)c->geo.message_len) return fail(OFDM_ERR_INVALID, "frame_stride < message_len");
    if (!aligned16(iq_out)) return fail(OFDM_ERR_INVALID, "iq_out must be 16-byte aligned");
    if (nframes == 0) return OFDM_OK;
    if (nframes * (size_t)c->S > 0x7fffffffu) return fail(OFDM_ERR_INVALID, "too many symbols in one call");
    ofdm::TxArgs a{};
    fill_tx(c, a, bytes, nframes, iq_out, frame_stride, iq16_out, ch);
    hipError_t e = ofdm::launch_tx(c->logn, a, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "tx_kernel launch");
    return OFDM_OK;
}

int ofdm_tx_frames(ofdm_ctx* c, const uint8_t* bytes, size_t nframes, double* frames_out, int16_t* frames16_out,
                   void* stream)
{
    if (!c || !bytes || !frames_out) return fail(OFDM_ERR_INVALID, "null argument");
    if (!aligned16(frames_out)) return fail(OFDM_ERR_INVALID, "frames_out must be 16-byte aligned");
    if (nframes == 0) return OFDM_OK;
    ofdm::TxArgs a{};
    fill_tx(c, a, bytes, nframes, frames_out, (size_t)c->geo.frame_len, frames16_out, nullptr);
    a.header = c->d_header;
    a.header_len = (int)(c->t2 + c->geo.preamble_len);
    a.msg_offset = a.header_len;
    hipError_t e = ofdm::launch_tx(c->logn, a, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "tx_kernel launch");
    return OFDM_OK;
}

}  // extern "C"

// ofdm_rx_demod / ofdm_rx_demod_i16: exactly one of iq, iq16 is set.
static int rx_demod_impl(ofdm_ctx* c, const double* iq, const int16_t* iq16, size_t nframes, size_t frame_stride,
                         const double* chan, size_t chan_stride, double* constell_out, uint8_t* bytes_out,
                         const uint8_t* ref_bytes, unsigned long long* bit_errors, void* stream,
                         double* read_out = nullptr)
{
    if (!c || (!iq && !iq16)) return fail(OFDM_ERR_INVALID, "null argument");
    if (iq16 && ((uintptr_t)iq16 & 3)) return fail(OFDM_ERR_INVALID, "iq16 must be 4-byte aligned");
    if (frame_stride < (size_t)c->geo.message_len) return fail(OFDM_ERR_INVALID, "frame_stride < message_len");
    if ((iq && !aligned16(iq)) || (chan && !aligned16(chan)) || (constell_out && !aligned16(constell_out)))
        return fail(OFDM_ERR_INVALID, "complex buffers must be 16-byte aligned");
    if ((ref_bytes == nullptr) != (bit_errors == nullptr))
        return fail(OFDM_ERR_INVALID, "ref_bytes and bit_errors go together");
    if (nframes == 0) return OFDM_OK;
    if (nframes > 0x7fffffffu) return fail(OFDM_ERR_INVALID, "too many frames in one call");
    ofdm::RxArgs a{};
    a.tab = c->tables(false);
    a.iq = iq16 ? nullptr : reinterpret_cast<const double2*>(iq);
    a.iq16 = reinterpret_cast<const short2*>(iq16);
    a.nframes = (long)nframes;
    a.frame_stride = (long)frame_stride;
    a.chan = reinterpret_cast<const double2*>(chan);
    a.chan_stride = (long)chan_stride;
    a.constell = reinterpret_cast<double2*>(constell_out);
    a.read_out = reinterpret_cast<double2*>(read_out);
    a.bytes = bytes_out;
    a.ref = ref_bytes;
    a.bit_errors = bit_errors;
    a.S = c->S;
    a.D = c->D;
    a.P = c->P;
    a.seg = c->seg;
    a.cp = c->cp;
    a.k = c->k;
    a.bytes_per_frame = c->geo.bytes_per_frame;
    a.pilot_ampl = (double)c->p.pilot_ampl / 1000;
    a.queue = rx_queue(c, (hipStream_t)stream);
    const bool fits = c->S <= ofdm::RX_SMAX && c->D <= ofdm::RX_DPT * (c->N / 8);
    if (!fits) {
        if (c->D > ofdm::RX_DPT * (c->N / 8))
            return fail(OFDM_ERR_UNSUPPORTED, "num_data_subc > fft_size/2 is not covered by the rx kernel");
        if (constell_out) {
            a.ystage = a.constell;
        } else {
            const size_t need = nframes * (size_t)c->S * c->D * sizeof(double2);
            if (need > c->scratch_bytes) {
                HIP_TRY(hipSetDevice(c->device));
                if (c->d_scratch) HIP_TRY(hipFree(c->d_scratch));
                c->d_scratch = nullptr;
                c->scratch_bytes = 0;
                HIP_TRY(hipMalloc((void**)&c->d_scratch, need));
                c->scratch_bytes = need;
            }
            a.ystage = c->d_scratch;
        }
    }
    hipError_t e = ofdm::launch_rx(c->logn, a, (hipStream_t)stream, nullptr);
    if (e != hipSuccess) {
        rx_queue_reset(c, a.queue, (hipStream_t)stream);
        return hip_fail(e, "rx_kernel launch");
    }
    return OFDM_OK;
}

extern "C" {

int ofdm_rx_demod(ofdm_ctx* c, const double* iq, size_t nframes, size_t frame_stride, const double* chan,
                  size_t chan_stride, double* constell_out, uint8_t* bytes_out, const uint8_t* ref_bytes,
                  unsigned long long* bit_errors, void* stream)
{
    if (!iq) return fail(OFDM_ERR_INVALID, "null argument");
    return rx_demod_impl(c, iq, nullptr, nframes, frame_stride, chan, chan_stride, constell_out, bytes_out, ref_bytes,
                         bit_errors, stream);
}

int ofdm_rx_demod_i16(ofdm_ctx* c, const int16_t* iq16, size_t nframes, size_t frame_stride, const double* chan,
                      size_t chan_stride, double* constell_out, uint8_t* bytes_out, const uint8_t* ref_bytes,
                      unsigned long long* bit_errors, void* stream)
{
    if (!iq16) return fail(OFDM_ERR_INVALID, "null argument");
    return rx_demod_impl(c, nullptr, iq16, nframes, frame_stride, chan, chan_stride, constell_out, bytes_out,
                         ref_bytes, bit_errors, stream);
}

int ofdm_rx_demod_read(ofdm_ctx* c, const double* iq, size_t nframes, size_t frame_stride, const double* chan,
                       size_t chan_stride, double* read_out, double* constell_out, uint8_t* bytes_out, void* stream)
{
    if (!iq || !chan || !read_out) return fail(OFDM_ERR_INVALID, "null argument");
    if (!aligned16(read_out)) return fail(OFDM_ERR_INVALID, "complex buffers must be 16-byte aligned");
    return rx_demod_impl(c, iq, nullptr, nframes, frame_stride, chan, chan_stride, constell_out, bytes_out, nullptr,
                         nullptr, stream, read_out);
}

int ofdm_demap(ofdm_ctx* c, double* points, size_t n, uint8_t* bytes_out, void* stream)
{
    if (!c || !points || !bytes_out) return fail(OFDM_ERR_INVALID, "null argument");
    hipError_t e = ofdm::launch_demap(reinterpret_cast<double2*>(points), (long)n, c->k, bytes_out, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "demap launch");
    return OFDM_OK;
}

int ofdm_map(ofdm_ctx* c, const uint8_t* bytes, size_t nbytes, double* points_out, void* stream)
{
    if (!c || !bytes || !points_out) return fail(OFDM_ERR_INVALID, "null argument");
    hipError_t e = ofdm::launch_map(bytes, (long)nbytes, c->k, c->d_const, reinterpret_cast<double2*>(points_out),
                                    (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "map launch");
    return OFDM_OK;
}

int ofdm_fft_write(ofdm_ctx* c, const double* points, size_t nframes, double* fft_buf, void* stream)
{
    if (!c || !points || !fft_buf) return fail(OFDM_ERR_INVALID, "null argument");
    if (!aligned16(points) || !aligned16(fft_buf)) return fail(OFDM_ERR_INVALID, "buffers must be 16-byte aligned");
    if (nframes == 0) return OFDM_OK;
    ofdm::TxArgs a{};
    fill_tx(c, a, nullptr, nframes, fft_buf, (size_t)c->N * c->S, nullptr, nullptr);
    a.points = reinterpret_cast<const double2*>(points);
    a.cp = 0;  // FFT_buf holds bodies only
    hipError_t e = ofdm::launch_tx(c->logn, a, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "fft_write launch");
    return OFDM_OK;
}

int ofdm_fft_read(ofdm_ctx* c, const double* fft_buf, size_t nframes, double* restored, void* stream)
{
    if (!c || !fft_buf || !restored) return fail(OFDM_ERR_INVALID, "null argument");
    if (!aligned16(fft_buf) || !aligned16(restored)) return fail(OFDM_ERR_INVALID, "buffers must be 16-byte aligned");
    if (nframes == 0) return OFDM_OK;
    ofdm::RxArgs a{};
    a.tab = c->tables(false);
    a.iq = reinterpret_cast<const double2*>(fft_buf);
    a.nframes = (long)nframes;
    a.frame_stride = (long)c->N * c->S;
    a.constell = reinterpret_cast<double2*>(restored);
    a.S = c->S;
    a.D = c->D;
    a.P = c->P;
    a.seg = c->seg;
    a.cp = 0;  // no CP in FFT_buf
    a.k = c->k;
    a.bytes_per_frame = c->geo.bytes_per_frame;
    a.pilot_ampl = (double)c->p.pilot_ampl / 1000;
    a.queue = rx_queue(c, (hipStream_t)stream);
    if (!(c->S <= ofdm::RX_SMAX && c->D <= ofdm::RX_DPT * (c->N / 8))) a.ystage = a.constell;
    hipError_t e = ofdm::launch_rx(c->logn, a, (hipStream_t)stream, nullptr);
    if (e != hipSuccess) {
        rx_queue_reset(c, a.queue, (hipStream_t)stream);
        return hip_fail(e, "fft_read launch");
    }
    return OFDM_OK;
}

int ofdm_bit_convert(ofdm_ctx* c, const uint8_t* in, size_t len, int in_bits, int out_bits, uint8_t* out,
                     size_t* out_len, void* stream)
{
    if (!c || (len && (!in || !out))) return fail(OFDM_ERR_INVALID, "null argument");
    if (in_bits < 1 || in_bits > 8 || out_bits < 1 || out_bits > 8) return fail(OFDM_ERR_INVALID, "bits must be 1..8");
    const size_t total = len * (size_t)in_bits;
    const size_t n = total / out_bits + (total % out_bits > 0);
    if (out_len) *out_len = n;
    hipError_t e = ofdm::launch_bit_convert(in, (long)len, in_bits, out_bits, out, (long)n, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "bit_convert launch");
    return OFDM_OK;
}

int ofdm_int16_to_double(ofdm_ctx* c, const int16_t* in, size_t n, double* out, void* stream)
{
    if (!c || (n && (!in || !out))) return fail(OFDM_ERR_INVALID, "null argument");
    if (((uintptr_t)in & 3) || !aligned16(out)) return fail(OFDM_ERR_INVALID, "misaligned buffers");
    hipError_t e = ofdm::launch_i16_to_f64(in, (long)n, out, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "int16_to_double launch");
    return OFDM_OK;
}

int ofdm_double_to_int16(ofdm_ctx* c, const double* in, size_t n, int16_t* out, void* stream)
{
    if (!c || (n && (!in || !out))) return fail(OFDM_ERR_INVALID, "null argument");
    if (!aligned16(in) || ((uintptr_t)out & 3)) return fail(OFDM_ERR_INVALID, "misaligned buffers");
    hipError_t e = ofdm::launch_f64_to_i16(in, (long)n, (double)c->p.mult, out, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "double_to_int16 launch");
    return OFDM_OK;
}

// ---- sync front end (ofdm_sync.hip)
int ofdm_t2_scan(ofdm_ctx* c, const double* iq, size_t n, long start, double* rel_out, int* first_out, void* stream)
{
    if (!c || !iq) return fail(OFDM_ERR_INVALID, "null argument");
    if (c->t2_logn < 0) return fail(OFDM_ERR_UNSUPPORTED, "T2 detector needs T2sin_size = 2^a, 64..4096");
    if (start < 0) return fail(OFDM_ERR_INVALID, "start < 0");
    if (!aligned16(iq)) return fail(OFDM_ERR_INVALID, "iq must be 16-byte aligned");
    ofdm::T2Args a{};
    a.iq = reinterpret_cast<const double2*>(iq);
    a.tw = c->d_t2tw;
    a.start = start;
    a.nblocks = (long)n > start ? ((long)n - start) / c->t2 : 0;
    const int sm = (int)c->p.smooth, f1 = (int)c->p.t2_sin_f1, f2 = (int)c->p.t2_sin_f2;
    a.a1 = std::max(0, f1 - sm);
    a.b1 = std::min(c->t2 - 1, f1 + sm);
    a.a2 = std::max(0, f2 - sm);
    a.b2 = std::min(c->t2 - 1, f2 + sm);
    a.level = (double)c->p.t2_sin_level / 1000;
    a.rel_out = rel_out;
    a.first_scratch = c->d_first;
    hipError_t e = ofdm::launch_t2_scan(c->t2_logn, a, first_out, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "t2_scan launch");
    return OFDM_OK;
}

// find_preamble's split scratch when the call fits it (else the
// one-workgroup form: hv_scratch stays null).
static void preamble_scratch(ofdm_ctx* c, size_t nstarts, ofdm::PreambleArgs& a)
{
    if (nstarts > ofdm_ctx::PRE_SCRATCH_STARTS) return;
    a.hv_scratch = c->d_pre_hv;
    a.done = c->d_pre_done;
}

int ofdm_find_preamble(ofdm_ctx* c, const double* iq, size_t n, const int* starts, size_t nstarts, int* idx_out,
                       void* stream)
{
    if (!c || !iq || (nstarts && (!starts || !idx_out))) return fail(OFDM_ERR_INVALID, "null argument");
    if (!aligned16(iq)) return fail(OFDM_ERR_INVALID, "iq must be 16-byte aligned");
    ofdm::PreambleArgs a{};
    a.iq = reinterpret_cast<const double2*>(iq);
    a.n = (long)n;
    a.starts = starts;
    a.nstarts = (long)nstarts;
    a.idx_out = idx_out;
    a.templ = c->d_templ;
    a.L = (int)c->p.pr_sin_len;
    a.cycles = (int)(2 * c->p.t2sin_size + c->p.pr_sin_len);
    a.level = (double)c->p.pr_level / 1000;
    preamble_scratch(c, nstarts, a);
    hipError_t e = ofdm::launch_find_preamble(a, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "find_preamble launch");
    return OFDM_OK;
}

int ofdm_preamble_corr(ofdm_ctx* c, const double* iq, size_t n, long start, double* cor_out, void* stream)
{
    if (!c || !iq || !cor_out) return fail(OFDM_ERR_INVALID, "null argument");
    if (!aligned16(iq)) return fail(OFDM_ERR_INVALID, "iq must be 16-byte aligned");
    if (start < INT32_MIN || start > INT32_MAX) return fail(OFDM_ERR_INVALID, "start out of range");
    int* d_start = c->d_first + 2;  // scratch word 2: the one start index
    const int s32 = (int)start;
    HIP_TRY(hipMemcpyAsync(d_start, &s32, sizeof(int), hipMemcpyHostToDevice, (hipStream_t)stream));
    ofdm::PreambleArgs a{};
    a.iq = reinterpret_cast<const double2*>(iq);
    a.n = (long)n;
    a.starts = d_start;
    a.nstarts = 1;
    a.idx_out = nullptr;
    a.templ = c->d_templ;
    a.L = (int)c->p.pr_sin_len;
    a.cycles = (int)(2 * c->p.t2sin_size + c->p.pr_sin_len);
    a.level = (double)c->p.pr_level / 1000;
    a.cor_out = cor_out;
    preamble_scratch(c, 1, a);
    hipError_t e = ofdm::launch_find_preamble(a, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "preamble_corr launch");
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));  // the start word is host-staged
    return OFDM_OK;
}

int ofdm_cfo_estimate(ofdm_ctx* c, const double* x, size_t nframes, size_t stride, int nsym, double* cfo_out,
                      void* stream)
{
    if (!c || !x || !cfo_out) return fail(OFDM_ERR_INVALID, "null argument");
    if (nsym < 1 || stride < (size_t)c->L * nsym) return fail(OFDM_ERR_INVALID, "bad nsym / frame_stride");
    if (!aligned16(x)) return fail(OFDM_ERR_INVALID, "x must be 16-byte aligned");
    if (nframes == 0) return OFDM_OK;
    ofdm_ctx::CfoPlan* pl = nullptr;
    int rc = cfo_plan(c, nsym, &pl);
    if (rc) return rc;
    ofdm::CfoArgs a{};
    a.x = reinterpret_cast<const double2*>(x);
    a.nframes = (long)nframes;
    a.frame_stride = (long)stride;
    a.tw_sub = pl->tw_sub;
    a.tw_full = pl->tw_full;
    a.borders = pl->borders;
    a.P = c->P;
    a.cfo_out = cfo_out;
    a.host_out = 1;  // the public entry: cfo_out may be pinned host memory (header)
    hipError_t e = ofdm::launch_cfo(pl->logm, pl->g, a, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "cfo launch");
    return OFDM_OK;
}

int ofdm_freq_shift(ofdm_ctx* c, double* x, size_t nframes, size_t stride, size_t nsamples, const double* cfo,
                    void* stream)
{
    if (!c || !x || !cfo) return fail(OFDM_ERR_INVALID, "null argument");
    if (nframes > 1 && stride < nsamples) return fail(OFDM_ERR_INVALID, "frame_stride < nsamples");
    if (!aligned16(x)) return fail(OFDM_ERR_INVALID, "x must be 16-byte aligned");
    ofdm::ShiftArgs a{reinterpret_cast<double2*>(x), (long)nframes, (long)stride, (long)nsamples, cfo};
    hipError_t e = ofdm::launch_freq_shift(a, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "freq_shift launch");
    return OFDM_OK;
}

int ofdm_cp_sync(ofdm_ctx* c, double* x, size_t nframes, size_t stride, int nsym, void* stream)
{
    if (!c || !x) return fail(OFDM_ERR_INVALID, "null argument");
    if (nsym < 1 || nsym > 64 || (nframes > 1 && stride < (size_t)c->L * nsym))
        return fail(OFDM_ERR_INVALID, "bad nsym / frame_stride");
    if (!aligned16(x)) return fail(OFDM_ERR_INVALID, "x must be 16-byte aligned");
    ofdm::CpArgs a{reinterpret_cast<double2*>(x), (long)nframes, (long)stride, nsym, c->N, c->cp};
    hipError_t e = ofdm::launch_cp_sync(a, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "cp_sync launch");
    return OFDM_OK;
}

int ofdm_phase_sync(ofdm_ctx* c, double* x, size_t nframes, size_t stride, size_t nsamples, const double* pr,
                    size_t pr_len, void* stream)
{
    if (!c || !x) return fail(OFDM_ERR_INVALID, "null argument");
    if (!pr) {
        pr = reinterpret_cast<const double*>(c->d_preamble);
        pr_len = (size_t)c->geo.preamble_len;
    }
    if (pr_len > nsamples && nframes > 1 && stride < pr_len) return fail(OFDM_ERR_INVALID, "pr_len exceeds the form");
    if (!aligned16(x) || !aligned16(pr)) return fail(OFDM_ERR_INVALID, "buffers must be 16-byte aligned");
    ofdm::PhaseArgs a{reinterpret_cast<double2*>(x), (long)nframes, (long)stride, (long)nsamples,
                      reinterpret_cast<const double2*>(pr), (long)pr_len};
    hipError_t e = ofdm::launch_phase_sync(a, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "phase_sync launch");
    return OFDM_OK;
}

int ofdm_sync_chain(ofdm_ctx* c, double* x, size_t nframes, size_t stride, size_t nsamples, int nsym,
                    const double* cfo, double* shift_out, double* cp_out, double* phase_out, size_t out_stride,
                    void* stream)
{
    if (!c || !x || !cfo) return fail(OFDM_ERR_INVALID, "null argument");
    if (nsym < 1 || nsym > 64 || (size_t)c->L * nsym > nsamples) return fail(OFDM_ERR_INVALID, "bad nsym / nsamples");
    if (nframes > 1 && stride < nsamples) return fail(OFDM_ERR_INVALID, "frame_stride < nsamples");
    if ((size_t)c->geo.preamble_len > nsamples) return fail(OFDM_ERR_INVALID, "the preamble exceeds the form");
    double* outs[3] = {shift_out, cp_out, phase_out};
    for (double* o : outs)
        if (o && nframes > 1 && out_stride < nsamples) return fail(OFDM_ERR_INVALID, "out_stride < nsamples");
    if (!aligned16(x) || !aligned16(shift_out) || !aligned16(cp_out) || !aligned16(phase_out))
        return fail(OFDM_ERR_INVALID, "buffers must be 16-byte aligned");
    if (nframes == 0 || nsamples == 0) return OFDM_OK;
    ofdm::SyncChainArgs a{};
    a.x = reinterpret_cast<double2*>(x);
    a.nframes = (long)nframes;
    a.frame_stride = (long)stride;
    a.nsamples = (long)nsamples;
    a.cfo = cfo;
    a.nsym = nsym;
    a.N = c->N;
    a.cp = c->cp;
    a.pr = c->d_preamble;
    a.pr_len = (long)c->geo.preamble_len;
    for (int k = 0; k < 3; ++k) a.out[k] = reinterpret_cast<double2*>(outs[k]);
    a.out_stride = (long)out_stride;
    hipError_t e = ofdm::launch_sync_chain(a, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "sync_chain launch");
    return OFDM_OK;
}

int ofdm_chan_estimate(ofdm_ctx* c, const double* x, size_t nframes, size_t stride, double* chan_out,
                       size_t chan_stride, void* stream)
{
    if (!c || !x || !chan_out) return fail(OFDM_ERR_INVALID, "null argument");
    if (!aligned16(x) || !aligned16(chan_out)) return fail(OFDM_ERR_INVALID, "buffers must be 16-byte aligned");
    if (c->P > c->N / 8) return fail(OFDM_ERR_UNSUPPORTED, "num_pilot_subc > fft_size/8");
    ofdm::ChanArgs a{};
    a.tab = c->tables(true);
    a.x = reinterpret_cast<const double2*>(x);
    a.nframes = (long)nframes;
    a.frame_stride = (long)stride;
    a.mod_pre = c->d_modpre;
    a.chan_out = reinterpret_cast<double2*>(chan_out);
    a.chan_stride = (long)chan_stride;
    a.npr = c->npr;
    a.D = c->D;
    a.P = c->P;
    a.cp = c->cp;
    a.pilot_ampl = (double)c->p.pilot_ampl / 1000;
    hipError_t e = ofdm::launch_chan(c->logn, a, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "chan launch");
    return OFDM_OK;
}

int ofdm_sync_frames(ofdm_ctx* c, double* frames, size_t nframes, size_t stride, int stages, const double* cfo_in,
                     double* cfo_out, double* chan_out, void* stream)
{
    if (!c || !frames) return fail(OFDM_ERR_INVALID, "null argument");
    const int nsym = c->npr + c->S;
    const size_t nsamples = (size_t)c->L * nsym;
    if (nframes > 1 && stride < nsamples) return fail(OFDM_ERR_INVALID, "frame_stride < preamble+message");
    if (nframes == 0) return OFDM_OK;
    const double* cfo = cfo_in;
    int rc;
    if (stages & OFDM_SYNC_CFO) {
        double* dst = cfo_out;
        if (!dst) {
            if (c->cfo_scratch_n < nframes) {
                HIP_TRY(hipSetDevice(c->device));
                if (c->d_cfo_scratch) HIP_TRY(hipFree(c->d_cfo_scratch));
                c->d_cfo_scratch = nullptr;
                c->cfo_scratch_n = 0;
                HIP_TRY(hipMalloc((void**)&c->d_cfo_scratch, nframes * sizeof(double)));
                c->cfo_scratch_n = nframes;
            }
            dst = c->d_cfo_scratch;
        }
        if ((rc = ofdm_cfo_estimate(c, frames, nframes, stride, c->npr, dst, stream))) return rc;
        cfo = dst;
    }
    if (stages & OFDM_SYNC_FREQ_SHIFT) {
        if (!cfo) return fail(OFDM_ERR_INVALID, "freq shift without a CFO (set OFDM_SYNC_CFO or pass cfo_in)");
        if ((rc = ofdm_freq_shift(c, frames, nframes, stride, nsamples, cfo, stream))) return rc;
    }
    if ((stages & OFDM_SYNC_CP) && (rc = ofdm_cp_sync(c, frames, nframes, stride, nsym, stream))) return rc;
    if ((stages & OFDM_SYNC_PHASE) && (rc = ofdm_phase_sync(c, frames, nframes, stride, nsamples, nullptr, 0, stream)))
        return rc;
    if ((stages & OFDM_SYNC_CHAN) && chan_out &&
        (rc = ofdm_chan_estimate(c, frames, nframes, stride, chan_out, (size_t)c->D, stream)))
        return rc;
    return OFDM_OK;
}

}  // extern "C"

// rx.cpp's initial walk state (rx.cpp:105-114): pos = 0 of a buffer whose
// first output_size samples are the zero header before the first SDR buffer,
// i.e. stream position -output_size in a ring ending at R; the continuous
// walk starts at the stream's first sample.
static ofdm_walk_state initial_state(const ofdm_ctx* c)
{
    return c->ring > 0 ? ofdm_walk_state{-c->geo.frame_len, c->ring} : ofdm_walk_state{0, 0};
}

// ofdm_rx_stream / ofdm_rx_stream_i16 / ofdm_rx_stream_shard: exactly one of
// iq, iq16 is set. The walk starts at state `start`; frames located with pb in
// [own_lo, own_hi) are decoded (the whole stream: start = own_lo = 0, own_hi = n).
static int rx_stream_impl(ofdm_ctx* c, const double* iq, const int16_t* iq16, size_t n, size_t max_frames,
                          long chunk, long* pb_out, uint8_t* bytes_out, double* constell_out, double* cfo_out,
                          size_t* nframes_out, void* stream, ofdm_walk_state start_state, long own_lo, long own_hi,
                          long* located, uint8_t* located_lag, size_t located_cap, size_t* nlocated_out,
                          ofdm_walk_state* exit_out, bool force_halo = false)
{
    if (!c || (!iq && !iq16) || !nframes_out) return fail(OFDM_ERR_INVALID, "null argument");
    *nframes_out = 0;
    if (nlocated_out) *nlocated_out = 0;
    if (exit_out) *exit_out = ofdm_walk_state{-1, 0};
    const long R = c->ring, flen0 = c->geo.frame_len;
    const long start = start_state.pos;
    // ring mode: the walk may start in rx.cpp's zero header before the first
    // SDR buffer ([-output_size, 0)); its ring end lies ahead of it, within R.
    // An exit state may also lie a little past its ring end: a walk that
    // crossed own_hi inside a T2 scan whose next block leaves the ring (the
    // state's next step is the refill, pos = ring_end, rx.cpp:137-145)
    const long past = ofdm::WALK_SCAN_MAX + c->t2;
    if (R > 0 ? (start < -flen0 || start_state.ring_end <= start - past || start_state.ring_end > start + R + flen0)
              : start < 0)
        return fail(OFDM_ERR_INVALID, "start state out of range (ring mode: -output_size <= pos, pos - %ld < ring_end "
                                      "<= pos + R + output_size)", past);
    if (own_lo < 0 || own_lo > own_hi || own_hi > (long)n)
        return fail(OFDM_ERR_INVALID, "need 0 <= own_lo <= own_hi <= n");
    if (c->t2_logn < 6 || c->t2_logn > 11) return fail(OFDM_ERR_UNSUPPORTED, "stream walk needs T2sin_size = 2^a, 64..2048");
    if ((iq && !aligned16(iq)) || (iq16 && ((uintptr_t)iq16 & 3)) || (constell_out && !aligned16(constell_out)))
        return fail(OFDM_ERR_INVALID, "misaligned buffer (complex<double> 16 B, complex<int16> 4 B)");
    if (n > (size_t)1 << 40) return fail(OFDM_ERR_INVALID, "stream too long");
    hipStream_t st = (hipStream_t)stream;
    const long L = c->L, pre = (long)L * c->npr, msg = (long)L * c->S, span = pre + msg;
    const long flen = c->geo.frame_len, nn = (long)n;
    if (nn == 0 || start >= nn) return OFDM_OK;
    // walkers: one chunk per resident walker slot by default, each >= 8 frames
    const long slots = ofdm::stream_walk_slots(c->t2_logn, (int)c->p.pr_sin_len,
                                               (int)(2 * c->p.t2sin_size + c->p.pr_sin_len), c->d_tspec != nullptr);
    // Per-context tuning (ofdm_set_walk_tuning): chunks per walker slot,
    // walk-in halo and walk-on extension in 1/1000 frames, look-back
    // stitching. Look-back (the default): chunks start at their core (no
    // walk-in) and each walks on past its core end until its walk joins the
    // next chunk's (a device-side check of the records that chunk publishes);
    // the chain of joined walks is the sequential walk, resolved on the
    // device. Without it (lookback = 0, or the fallback when a walker's
    // records overflow): each chunk walks in from a 3-frame halo and the host
    // stitches the walks, re-walking a chunk whose walk-in did not meet the
    // true walk.
    const ofdm_walk_tuning& tu = c->walk;
    const long qper = std::max(1L, tu.chunks_per_slot);
    const long span_w = own_hi - own_lo;  // the chunk cores tile [own_lo, own_hi)
    if (chunk <= 0) chunk = std::max(8 * flen, (span_w + slots * qper - 1) / (slots * qper));
    chunk = std::max(chunk, (long)c->t2);
    const long nchunks = std::max(1L, (span_w + chunk - 1) / chunk);
    if (nchunks > 1 << 20) return fail(OFDM_ERR_INVALID, "chunk too small for this stream");
    // look-back needs a resolvable chunk count and per-chunk record counts
    // below 2^14 (the resolve kernel's packing): else the halo walk
    bool lbk = tu.lookback && !force_halo && nchunks <= ofdm::RESOLVE_MAX_CHUNKS &&
               (2 * chunk + std::max(0L, own_lo - start)) / msg < 8192;
    const long halo = (tu.halo_milli < 0 ? (lbk ? 0L : 3000L) : tu.halo_milli) * flen / 1000;
    const long ext = std::max(0L, tu.ext_milli) * flen / 1000;
    // each located frame advances the walk by > message_len, and a walker can
    // walk on past its core end by ext plus one scan step (WALK_SCAN_MAX
    // samples) and the preamble window: this many records always suffice
    // (chunk 0 walks in from `start`, the others a halo before their core).
    // A look-back walker may walk on through the next core too (its walk met
    // no record of that chunk's); one more overflows: the host falls back
    int max_rec =
        (int)(((lbk ? 2 : 1) * chunk + std::max(halo, own_lo - start) + std::max(ext, 2 * flen) + ofdm::WALK_SCAN_MAX +
               2 * c->p.t2sin_size + c->p.pr_sin_len) / msg + (lbk ? 8 : 4));
    // test hook: a smaller record buffer makes look-back walkers overflow
    // (the halo walk, which the cap does not touch, then takes the call)
    if (lbk && tu.max_rec_cap > 0) max_rec = std::min(max_rec, tu.max_rec_cap);
    int rc;
    const size_t rec_b = (size_t)nchunks * max_rec * sizeof(long);
    // layout: records | exit states | exit ring ends | re-walk start (pos, ring end) | counts | ...
    const size_t walk_b0 = rec_b + (size_t)nchunks * (2 * sizeof(long) + sizeof(int)) + 2 * sizeof(long) + 64;
    const size_t walk_b = walk_b0 + 2 * (size_t)nchunks * sizeof(int);  // + in-core counts and first indices
    const size_t link_b = 3 * (size_t)nchunks * sizeof(int);            // + look-back links
    if ((rc = grow(c, c->s_walk, walk_b + link_b))) return rc;
    char* wb = static_cast<char*>(c->s_walk.p);
    long* d_rec = reinterpret_cast<long*>(wb);
    long* d_exit = reinterpret_cast<long*>(wb + rec_b);
    long* d_exit_ring = d_exit + nchunks;
    long* d_start = d_exit_ring + nchunks;  // one re-walk start state (pos, ring end)
    int* d_nrec = reinterpret_cast<int*>(d_start + 2);
    int* d_ids = d_nrec + nchunks;     // one re-walk chunk id (in the 64 B slack)
    int* d_ncore = reinterpret_cast<int*>(wb + walk_b0);
    int* d_first_in = d_ncore + nchunks;
    int* d_link = reinterpret_cast<int*>(wb + walk_b);

    ofdm::WalkArgs w{};
    w.exact_only = tu.exact_search != 0;
    w.tw_m = c->d_twm;
    w.tspec = c->d_tspec;  // nullptr: direct certified search
    w.tspec_max = c->tspec_max;
    w.tspec32 = tu.pre_f32 ? c->d_tspec32 : nullptr;  // FP32 tier of the FFT search
    w.iq = reinterpret_cast<const double2*>(iq);
    w.iq16 = reinterpret_cast<const short2*>(iq16);
    w.n = nn;
    w.t2tw = c->d_t2tw;
    const int sm = (int)c->p.smooth, f1 = (int)c->p.t2_sin_f1, f2 = (int)c->p.t2_sin_f2;
    w.a1 = std::max(0, f1 - sm);
    w.b1 = std::min(c->t2 - 1, f1 + sm);
    w.a2 = std::max(0, f2 - sm);
    w.b2 = std::min(c->t2 - 1, f2 + sm);
    w.t2_level = (double)c->p.t2_sin_level / 1000;
    // FP32 T2 screen (certified, FP64 re-evaluation of uncertain steps)
    w.t2_f32 = tu.t2_f32 != 0;
    w.t2_margin = tu.t2_margin;
    w.templ = c->d_templ;
    w.L = (int)c->p.pr_sin_len;
    w.cycles = (int)(2 * c->p.t2sin_size + c->p.pr_sin_len);
    w.pr_level = (double)c->p.pr_level / 1000;
    w.pre = pre;
    w.msg = msg;
    w.chunk = chunk;
    w.halo = halo;
    w.start = start;
    w.ring = R;
    w.out_len = flen;
    w.start_ring_end = start_state.ring_end;
    w.ring_phase = R > 0 ? ((start_state.ring_end % R) + R) % R : 0;
    w.exit_ring = d_exit_ring;
    w.core_lo = own_lo;
    w.core_hi = own_hi;
    w.ext = ext;
    // A chunk whose core end falls inside a T2 scan (its last frame well
    // before the end, e.g. a frame the reference's walk misses) walks on to
    // the next frame it locates: the next chunk's walk locates that frame
    // too, so the two sync without a serial re-walk (2048 chunks of config 4:
    // one re-walk per call without this).
    w.ext_scan = std::max(ext, 2 * flen);
    w.max_rec = max_rec;
    w.rec = d_rec;
    w.nrec = d_nrec;
    w.exit_pos = d_exit;
    w.ncore = d_ncore;
    w.first_in = d_first_in;
    // the walkers take chunks from a queue: one resident round of workgroups
    // drains it, slower walkers taking fewer chunks. The counter is zeroed by
    // the previous call's compaction (stream order), else here.
    if (!c->d_queue) {
        HIP_TRY(hipMalloc((void**)&c->d_queue, 64));
        c->queue_zero = false;
    }
    w.queue = c->d_queue;
    w.nchunks = nchunks;
    // The previous stream call's work must be done before this one rewrites
    // the ctx's scratch (walk records, compacted list, channel): its decodes
    // read them. On the same stream that is stream order; on another stream
    // this call waits for an event recorded now on the previous call's stream
    // (behind that call's decodes; header: overlapping stream calls take two
    // contexts). Recorded here rather than at the end of every call: an event
    // between two dependent kernels of one stream costs a launch gap (the
    // next call's walker started ~15-25 us after the decode ended).
    if (c->call_valid && c->call_stream != st) {
        if (!c->ev_call) HIP_TRY(hipEventCreateWithFlags(&c->ev_call, hipEventDisableTiming));
        if (hipEventRecord(c->ev_call, c->call_stream) == hipSuccess) {
            HIP_TRY(hipStreamWaitEvent(st, c->ev_call, 0));
        } else {
            (void)hipGetLastError();  // that stream is gone (destroyed): wait for the device instead
            HIP_TRY(hipDeviceSynchronize());
        }
    }
    c->call_stream = st;
    c->call_valid = true;
    if (!c->queue_zero) HIP_TRY(hipMemsetAsync(w.queue, 0, sizeof(int), st));
    c->queue_zero = false;
    if (lbk) {
        if (c->s_pub.bytes < (size_t)nchunks * sizeof(int)) {
            if ((rc = grow(c, c->s_pub, (size_t)std::max(nchunks, 2048L) * sizeof(int)))) return rc;
            c->pub_zero = false;
        }
        if (!c->pub_zero) HIP_TRY(hipMemsetAsync(c->s_pub.p, 0, c->s_pub.bytes, st));
        c->pub_zero = false;  // until the resolve kernel clears it again
        w.lookback = 1;
        w.pub = static_cast<int*>(c->s_pub.p);
        w.link = d_link;
    }
    // diagnostics: OFDM_WALK_PROF=<file> appends one JSON line per call with
    // every chunk's walker timeline (WalkArgs::prof)
    const char* prof_path = getenv("OFDM_WALK_PROF");
    long* d_prof = nullptr;
    if (prof_path) HIP_TRY(hipMalloc((void**)&d_prof, (size_t)nchunks * ofdm::WALK_PROF_FIELDS * sizeof(long)));
    w.prof = d_prof;
    c->phase_valid = false;
    const bool timed = c->phase_timing && lbk;  // events between the kernels: measurement calls only
    if (timed) HIP_TRY(hipEventRecord(c->ev_phase[0], st));
    hipError_t e = ofdm::launch_stream_walk(c->t2_logn, w, std::min(nchunks, slots), st);
    if (e != hipSuccess) return hip_fail(e, "stream_walk launch");
    if (timed) HIP_TRY(hipEventRecord(c->ev_phase[1], st));
    if (d_prof) {
        std::vector<long> hp((size_t)nchunks * ofdm::WALK_PROF_FIELDS);
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipMemcpy(hp.data(), d_prof, hp.size() * sizeof(long), hipMemcpyDeviceToHost));
        HIP_TRY(hipFree(d_prof));
        if (FILE* f = fopen(prof_path, "a")) {
            fprintf(f, "{\"nchunks\": %ld, \"chunk\": %ld, \"lookback\": %d, \"grid\": %ld, \"fields\": "
                       "[\"t0\", \"t_core\", \"t_end\", \"ext_frames\", \"waits\", \"block\", \"xcc\", \"nrec\", "
                       "\"t2_ticks\", \"pre_ticks\", \"scan_steps\", \"fp64_evals\", \"searches\", \"hw_id\"], "
                       "\"chunks\": [", nchunks, chunk, (int)lbk, std::min(nchunks, slots));
            for (long k = 0; k < nchunks; ++k) {
                fprintf(f, "%s[", k ? "," : "");
                for (int i = 0; i < ofdm::WALK_PROF_FIELDS; ++i)
                    fprintf(f, "%s%ld", i ? "," : "", hp[(size_t)k * ofdm::WALK_PROF_FIELDS + i]);
                fprintf(f, "]");
            }
            fprintf(f, "]}\n");
            fclose(f);
        }
    }

    // Fused decode: three kernels read each frame from the stream in place
    // (pilot_freq_sinh; the other sync stages' parameters + chan_char_lq;
    // rx with the corrections applied on load), no frame copy, no corrected
    // copy. Needs the register-window rx and a pilot_freq_sinh plan.
    ofdm_ctx::CfoPlan* pl = nullptr;
    const bool fused = c->S <= ofdm::RX_SMAX && c->D <= ofdm::RX_DPT * (c->N / 8) && c->P <= c->N / 8 &&
                       c->npr == 1 && c->S + 1 <= 64 && c->L % (c->N / 8) == 0 && c->L / (c->N / 8) <= 16 &&
                       c->cp <= 2 * (c->N / 8) &&  // stream_params_kernel: CP template in 2 registers
                       cfo_plan(c, c->npr, &pl) == OFDM_OK;
    const size_t per = (size_t)c->D * sizeof(double2) + (size_t)c->S * ofdm::CORR_PER_SYM * sizeof(double2) + sizeof(double);
    const long npts = (long)c->D * c->S;
    // frames [0, nb) of d_list (device count d_cnt, if set, bounds them further)
    auto decode_fused = [&](const long* d_list, size_t nb_total, const long* d_cnt) -> int {
        const size_t bmax = std::max<size_t>(1, ((size_t)256 << 20) / per);
        const size_t nb0 = std::min(nb_total, bmax);
        int r2;
        if ((r2 = grow(c, c->s_chan, nb0 * per))) return r2;
        double2* chan = static_cast<double2*>(c->s_chan.p);
        double2* corr = chan + nb0 * c->D;
        double* cfo_tmp = reinterpret_cast<double*>(corr + nb0 * c->S * ofdm::CORR_PER_SYM);
        for (size_t f0 = 0; f0 < nb_total; f0 += nb0) {
            const size_t nb = std::min(nb0, nb_total - f0);
            double* cfo = cfo_out ? cfo_out + f0 : cfo_tmp;
            ofdm::CfoArgs ca{};
            ca.x = reinterpret_cast<const double2*>(iq);
            ca.x16 = reinterpret_cast<const short2*>(iq16);
            ca.starts = d_list + f0;
            ca.nframes = (long)nb;
            ca.tw_sub = pl->tw_sub;
            ca.tw_full = pl->tw_full;
            ca.borders = pl->borders;
            ca.P = c->P;
            ca.cfo_out = cfo;
            ca.count = d_cnt;  // single batch when set (f0 == 0)
            ofdm::StreamParamsArgs sa{};
            sa.tab = c->tables(true);
            sa.iq = reinterpret_cast<const double2*>(iq);
            sa.iq16 = reinterpret_cast<const short2*>(iq16);
            sa.starts = d_list + f0;
            sa.nframes = (long)nb;
            sa.cfo = cfo;
            sa.pre = c->d_preamble;
            sa.mod_pre = c->d_modpre;
            sa.chan_out = chan;  // internal scratch: reciprocals for rx's multiply
            sa.chan_recip = true;
            sa.corr_out = corr;
            sa.npr = c->npr;
            sa.S = c->S;
            sa.D = c->D;
            sa.P = c->P;
            sa.cp = c->cp;
            sa.pilot_ampl = (double)c->p.pilot_ampl / 1000;
            sa.count = d_cnt;
            ofdm::RxArgs ra{};
            ra.tab = c->tables(false);
            ra.iq = reinterpret_cast<const double2*>(iq);
            ra.iq16 = reinterpret_cast<const short2*>(iq16);
            ra.nframes = (long)nb;
            ra.starts = d_list + f0;
            ra.start_off = pre + c->cp;
            ra.count = d_cnt;
            ra.corr = corr;
            ra.chan = chan;
            ra.chan_stride = c->D;
            ra.chan_recip = true;
            ra.constell = constell_out ? reinterpret_cast<double2*>(constell_out) + f0 * npts : nullptr;
            ra.bytes = bytes_out ? bytes_out + f0 * c->geo.bytes_per_frame : nullptr;
            ra.S = c->S;
            ra.D = c->D;
            ra.P = c->P;
            ra.seg = c->seg;
            ra.cp = c->cp;
            ra.k = c->k;
            ra.bytes_per_frame = c->geo.bytes_per_frame;
            ra.pilot_ampl = (double)c->p.pilot_ampl / 1000;
            // static frame order: the next frame's symbol 0 is fetched ahead of
            // the gains (stream rx 500 -> 416 us with the queue's late fetch)
            ra.queue = nullptr;
            // One kernel for the whole decode where the geometry allows (N =
            // 512, 640-point CFO form: sync stage + rx stage per frame, the
            // ramps and channel through LDS); else pilot_freq_sinh + the
            // params stage (one kernel or two), then the stream rx.
            hipError_t e2 = c->walk.staged_decode
                                ? hipErrorNotSupported
                                : ofdm::launch_stream_decode(ca, sa, ra, c->logn, pl->logm, pl->g, st);
            if (e2 == hipErrorNotSupported) {
                // other geometries: pilot_freq_sinh, the params stage, then
                // the stream rx (two waves per frame at N = 512)
                e2 = ofdm::launch_cfo(pl->logm, pl->g, ca, st);
                if (e2 != hipSuccess) return hip_fail(e2, "stream cfo launch");
                e2 = ofdm::launch_stream_params(c->logn, sa, st);
                if (e2 != hipSuccess) return hip_fail(e2, "stream params launch");
                e2 = ofdm::launch_rx(c->logn, ra, st, nullptr);
                if (e2 != hipSuccess) return hip_fail(e2, "stream rx launch");
            } else if (e2 != hipSuccess) {
                return hip_fail(e2, "stream decode launch");
            }
        }
        return OFDM_OK;
    };
    // Geometries the fused kernels do not take: gather each frame of d_list
    // into a batch, then the staged sync chain + demod
    auto decode_gathered = [&](const long* d_list, size_t nout) -> int {
        const size_t fb = (size_t)span * sizeof(double2);
        const size_t bmax = std::max<size_t>(1, std::min<size_t>(65535, ((size_t)256 << 20) / fb));
        const size_t nb0 = std::min(nout, bmax);
        int r2;
        if ((r2 = grow(c, c->s_batch, nb0 * fb)) || (r2 = grow(c, c->s_chan, nb0 * c->D * sizeof(double2)))) return r2;
        double* batch = static_cast<double*>(c->s_batch.p);
        double* chan = static_cast<double*>(c->s_chan.p);
        for (size_t f0 = 0; f0 < nout; f0 += nb0) {
            const size_t nb = std::min(nb0, nout - f0);
            ofdm::GatherArgs ga{reinterpret_cast<const double2*>(iq), reinterpret_cast<const short2*>(iq16), nn,
                                d_list + f0, (long)nb, span, reinterpret_cast<double2*>(batch)};
            hipError_t e2 = ofdm::launch_gather(ga, st);
            if (e2 != hipSuccess) return hip_fail(e2, "gather launch");
            if ((r2 = ofdm_sync_frames(c, batch, nb, (size_t)span, OFDM_SYNC_ALL, nullptr,
                                       cfo_out ? cfo_out + f0 : nullptr, chan, stream)))
                return r2;
            if ((r2 = ofdm_rx_demod(c, batch + 2 * pre, nb, (size_t)span, chan, (size_t)c->D,
                                    constell_out ? constell_out + 2 * f0 * npts : nullptr,
                                    bytes_out ? bytes_out + f0 * c->geo.bytes_per_frame : nullptr, nullptr, nullptr,
                                    stream)))
                return r2;
        }
        return OFDM_OK;
    };

    if (lbk) {
        // The true walk, resolved on the device: the owned frames straight
        // into the decode's list (and pb_out), a status block to the host.
        // The decode is enqueued behind it before the host reads the status.
        const size_t ub = std::min(max_frames, (size_t)nchunks * max_rec);
        const bool want_chain = (located || located_lag) && located_cap > 0;
        const size_t chain_tail = located_cap / 2, chain_head = located_cap - chain_tail;
        if ((rc = grow(c, c->s_pbs, (ub + 1) * sizeof(long))) || (rc = grow_host(c, c->h_status, 64)) ||
            (want_chain && (rc = grow(c, c->s_chain, located_cap * sizeof(long)))))
            return rc;
        long* d_pbs = static_cast<long*>(c->s_pbs.p);
        volatile long* hs = static_cast<volatile long*>(c->h_status.p);
        hs[1] = -1;  // overwritten by the resolve kernel
        ofdm::ResolveArgs ra{};
        ra.rec = d_rec;
        ra.nrec = d_nrec;
        ra.link = d_link;
        ra.exit_pos = d_exit;
        ra.exit_ring = d_exit_ring;
        ra.nchunks = nchunks;
        ra.max_rec = max_rec;
        // a core starting at the stream's first sample also owns a frame whose
        // preamble starts before it (rx.cpp:105-114,158: its zero header)
        ra.own_lo = own_lo == 0 ? LONG_MIN : own_lo;
        ra.own_hi = own_hi;
        ra.cap = (long)ub;
        ra.list = d_pbs;
        ra.list2 = pb_out;
        ra.count = d_pbs + ub;
        ra.chain = want_chain ? static_cast<long*>(c->s_chain.p) : nullptr;
        ra.chain_head = (long)chain_head;
        ra.chain_tail = (long)chain_tail;
        ra.status = const_cast<long*>(hs);
        ra.pub = w.pub;
        ra.queue_reset = c->d_queue;
        e = ofdm::launch_resolve(ra, st);
        if (e != hipSuccess) return hip_fail(e, "stream resolve launch");
        c->pub_zero = true;    // cleared by the resolve (stream order)
        c->queue_zero = true;  // likewise the chunk counter
        if (timed) HIP_TRY(hipEventRecord(c->ev_phase[2], st));
        const bool spec = fused && ub > 0 && ub * per <= ((size_t)256 << 20);
        if (spec && (rc = decode_fused(d_pbs, ub, d_pbs + ub))) return rc;
        if (timed && spec) {
            HIP_TRY(hipEventRecord(c->ev_phase[3], st));
            c->phase_valid = true;
        }
        // the resolve kernel's last word is the flags word of the status:
        // poll it (no event between the resolve and the decode: a marker
        // between two dependent kernels costs a launch gap); if it has not
        // landed in 2 s, wait for the stream (errors surface there)
        {
            const auto t0 = std::chrono::steady_clock::now();
            for (long spin = 0; hs[1] == -1; ++spin)
                if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
                    HIP_TRY(hipStreamSynchronize(st));
                    break;
                }
        }
        const long owned = hs[0], flags = hs[1], xpos = hs[2], xring = hs[3], nchain = hs[4], nneg = hs[5];
        if (flags < 0) return fail(OFDM_ERR_HIP, "stream resolve wrote no status");
        if (flags & ofdm::RESOLVE_OVERFLOW) {
            // a walker's records overflowed (a walk that met no later chunk's
            // through a whole core): the halo walk with host stitching
            if (getenv("OFDM_STREAM_DEBUG")) fprintf(stderr, "ofdm_rx_stream: look-back overflow, halo walk\n");
            return rx_stream_impl(c, iq, iq16, n, max_frames, chunk, pb_out, bytes_out, constell_out, cfo_out,
                                  nframes_out, stream, start_state, own_lo, own_hi, located, located_lag, located_cap,
                                  nlocated_out, exit_out, true);
        }
        *nframes_out = (size_t)owned;
        if (exit_out) *exit_out = ofdm_walk_state{xpos, xpos < 0 ? 0 : xring};
        if (nlocated_out) *nlocated_out = (size_t)nchain;
        if (want_chain) {
            const size_t nl = std::min((size_t)nchain, located_cap);
            if (nl) {
                std::vector<long> rl(nl);
                HIP_TRY(hipMemcpy(rl.data(), c->s_chain.p, nl * sizeof(long), hipMemcpyDeviceToHost));
                for (size_t i = 0; i < nl; ++i) {
                    const long r = rl[i];
                    if (located) located[i] = r < 0 ? r : (r & ofdm::WALK_REC_PB);
                    if (located_lag) located_lag[i] = r > 0 && (r & ofdm::WALK_REC_LAG) ? 1 : 0;
                }
            }
        }
        if (getenv("OFDM_STREAM_DEBUG"))
            fprintf(stderr, "ofdm_rx_stream: look-back, %ld chunks of %ld samples, halo %ld, %ld frames\n", nchunks,
                    chunk, halo, owned);
        const size_t nout = std::min((size_t)owned, ub);
        // frames before sample 0 (a prefix; the fused kernels skip them): the
        // gather path, whose samples before 0 read as zero like rx.cpp's header
        const size_t neg = (flags & ofdm::RESOLVE_NEG_FRAME) ? std::min((size_t)nneg, nout) : 0;
        if (spec) return neg ? decode_gathered(d_pbs, neg) : OFDM_OK;
        if (nout == 0) return OFDM_OK;
        if (!fused) return decode_gathered(d_pbs, nout);
        if ((rc = decode_fused(d_pbs, nout, nullptr))) return rc;
        return neg ? decode_gathered(d_pbs, neg) : OFDM_OK;
    }

    // records, exit states and counts in one copy of the walk buffer's layout
    if ((rc = grow_host(c, c->h_walk, walk_b))) return rc;
    char* hb = static_cast<char*>(c->h_walk.p);
    long* rec = reinterpret_cast<long*>(hb);
    long* ex = reinterpret_cast<long*>(hb + rec_b);
    long* exr = ex + nchunks;
    int* nrec = reinterpret_cast<int*>(exr + nchunks + 2);
    if (!c->ev_walk) HIP_TRY(hipEventCreateWithFlags(&c->ev_walk, hipEventDisableTiming));
    if (!c->ev_wdone) HIP_TRY(hipEventCreateWithFlags(&c->ev_wdone, hipEventDisableTiming));
    if (!c->side) HIP_TRY(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
    // Speculative decode: every chunk's in-core records, compacted on the
    // device behind the walk, are decoded while the host stitches the walks.
    // That list is the stitched walk unless a chunk needs a re-walk (or the
    // walk ends early); then the host's list is decoded again over it.
    const size_t ub = std::min(max_frames, (size_t)nchunks * max_rec);
    const bool spec = fused && ub > 0 && ub * per <= ((size_t)256 << 20);
    long* d_pbs = nullptr;
    if (spec) {
        if ((rc = grow(c, c->s_pbs, (ub + 1) * sizeof(long)))) return rc;
        d_pbs = static_cast<long*>(c->s_pbs.p);
        ofdm::CompactArgs ka{};
        ka.rec = d_rec;
        ka.ncore = d_ncore;
        ka.first_in = d_first_in;
        ka.nchunks = nchunks;
        ka.max_rec = max_rec;
        ka.cap = (long)ub;
        ka.list = d_pbs;
        ka.list2 = pb_out;
        ka.count = d_pbs + ub;
        ka.queue_reset = c->d_queue;  // after the walk (stream order): zero for the next call
        e = ofdm::launch_compact(ka, st);
        if (e != hipSuccess) return hip_fail(e, "stream compact launch");
    }
    // The walk records go to the host on a side stream, so the decode on the
    // caller's stream does not queue behind the copy. The one event marks the
    // walk and the compaction together: a marker between two dependent
    // kernels costs a launch gap, so walk -> compaction runs back to back.
    HIP_TRY(hipEventRecord(c->ev_wdone, st));
    HIP_TRY(hipStreamWaitEvent(c->side, c->ev_wdone, 0));
    HIP_TRY(hipMemcpyAsync(hb, wb, walk_b, hipMemcpyDeviceToHost, c->side));
    HIP_TRY(hipEventRecord(c->ev_walk, c->side));
    if (spec) {
        if ((rc = decode_fused(d_pbs, ub, d_pbs + ub))) return rc;
        // the queue counter was zeroed by the compaction (stream order)
        c->queue_zero = true;
    }
    HIP_TRY(hipEventSynchronize(c->ev_walk));

    // the speculative list, from the walks as they came back
    // a record's preamble start (ring mode: the lag bit stripped; a frame
    // before the stream's first sample stays negative)
    auto rec_pb = [](long r) { return r < 0 ? r : (r & ofdm::WALK_REC_PB); };
    std::vector<long> spec_list;
    if (spec)
        for (long k = 0; k < nchunks; ++k) {
            const long lo = own_lo + k * chunk, hi = std::min(lo + chunk, own_hi);
            for (int i = 0; i < std::min(nrec[k], max_rec); ++i) {
                const long pb = rec_pb(rec[(size_t)k * max_rec + i]);
                if (pb >= lo && pb < hi) spec_list.push_back(pb);
            }
        }

    // Stitch the chunk walks into the one true walk. Chunk 0 starts at the
    // true initial state. Chunk k is accepted when its walk and the accepted
    // walk before it locate a common frame no later than k's first owned
    // frame (from there on both are the same computation); otherwise it is
    // re-walked from the previous exit state (exact), with one workgroup.
    long nrewalk = 0;
    auto rewalk = [&](long k, long start, long start_ring) -> int {
        ofdm::WalkArgs r = w;
        const int id = (int)k;
        const long st2[2] = {start, start_ring};
        HIP_TRY(hipMemcpyAsync(d_start, st2, sizeof(st2), hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(d_ids, &id, sizeof(int), hipMemcpyHostToDevice, st));
        r.start_pos = d_start;
        r.start_ring = d_start + 1;
        r.chunk_ids = d_ids;
        r.queue = nullptr;
        ++nrewalk;
        hipError_t e2 = ofdm::launch_stream_walk(c->t2_logn, r, 1, st);
        if (e2 != hipSuccess) return hip_fail(e2, "stream_walk re-walk launch");
        HIP_TRY(hipMemcpyAsync(rec + (size_t)k * max_rec, d_rec + (size_t)k * max_rec, max_rec * sizeof(long),
                               hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(&ex[k], d_exit + k, sizeof(long), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(&exr[k], d_exit_ring + k, sizeof(long), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(&nrec[k], d_nrec + k, sizeof(int), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        return OFDM_OK;
    };
    // records compare whole (preamble start and, in ring mode, the ring of the
    // state after the frame): equal records = equal walks from there on
    std::vector<long> frames, walk_in;  // frames: preamble starts; walk_in: records
    std::vector<long> owned_rec;        // the owned frames' records
    std::vector<long> prev;  // every record of the accepted walk of the previous chunk
    long texit = 0, texit_ring = start_state.ring_end, last_k = -1;
    for (long k = 0; k < nchunks; ++k) {
        if (k > 0 && texit < 0) break;  // the true walk ended
        if (nrec[k] > max_rec) return fail(OFDM_ERR_HIP, "stream walk record overflow");
        std::vector<long> lst(rec + (size_t)k * max_rec, rec + (size_t)k * max_rec + nrec[k]);
        const long lo = own_lo + k * chunk, hi = std::min(lo + chunk, own_hi);
        if (k > 0) {
            long first_owned = LONG_MAX;
            for (long r : lst)
                if (rec_pb(r) >= lo && rec_pb(r) < hi) first_owned = std::min(first_owned, rec_pb(r));
            bool sync = false;
            for (long r : lst)
                if (rec_pb(r) <= first_owned && std::find(prev.begin(), prev.end(), r) != prev.end()) sync = true;
            if (!sync) {
                if (getenv("OFDM_STREAM_DEBUG")) {
                    fprintf(stderr, "ofdm_rx_stream: re-walk chunk %ld [%ld, %ld) from (%ld, %ld); its walk:", k, lo, hi,
                            texit, texit_ring);
                    for (long r : lst) fprintf(stderr, " %ld%s", rec_pb(r), r > 0 && (r & ofdm::WALK_REC_LAG) ? "+" : "");
                    fprintf(stderr, " | previous:");
                    for (long r : prev) fprintf(stderr, " %ld%s", rec_pb(r), r > 0 && (r & ofdm::WALK_REC_LAG) ? "+" : "");
                    fprintf(stderr, "\n");
                }
                if ((rc = rewalk(k, texit, texit_ring))) return rc;
                if (nrec[k] > max_rec) return fail(OFDM_ERR_HIP, "stream walk record overflow");
                lst.assign(rec + (size_t)k * max_rec, rec + (size_t)k * max_rec + nrec[k]);
            }
        }
        if (k == 0)  // the walk-in from `start` (true by definition): frames before own_lo; a
            for (long r : lst) {  // core from sample 0 owns a frame before it (rx.cpp's zero header)
                if (rec_pb(r) < lo && !(own_lo == 0 && r < 0)) walk_in.push_back(r);
                if (own_lo == 0 && r < 0) {
                    frames.push_back(r);
                    owned_rec.push_back(r);
                }
            }
        for (long r : lst)
            if (rec_pb(r) >= lo && rec_pb(r) < hi) {
                frames.push_back(rec_pb(r));
                owned_rec.push_back(r);
            }
        prev.swap(lst);
        texit = ex[k];
        texit_ring = exr[k];
        last_k = k;
    }
    *nframes_out = frames.size();
    if (exit_out && last_k == nchunks - 1) *exit_out = ofdm_walk_state{texit, texit < 0 ? 0 : texit_ring};
    if (nlocated_out) {
        // every frame of the stitched walk: the walk-in, the owned frames, and
        // what the last walker located past own_hi before it stopped
        std::vector<long> all(walk_in);
        all.insert(all.end(), owned_rec.begin(), owned_rec.end());
        if (last_k == nchunks - 1)
            for (long r : prev)
                if (rec_pb(r) >= own_hi) all.push_back(r);
        *nlocated_out = all.size();
        // more than located_cap: the first located_cap - located_cap/2 and the last located_cap/2
        if (all.size() > located_cap) {
            const size_t tail = located_cap / 2, head = located_cap - tail;
            std::vector<long> ht(all.begin(), all.begin() + head);
            ht.insert(ht.end(), all.end() - tail, all.end());
            all.swap(ht);
        }
        for (size_t i = 0; i < all.size(); ++i) {
            if (located) located[i] = rec_pb(all[i]);
            if (located_lag) located_lag[i] = all[i] > 0 && (all[i] & ofdm::WALK_REC_LAG) ? 1 : 0;
        }
    }
    if (getenv("OFDM_STREAM_DEBUG"))
        fprintf(stderr, "ofdm_rx_stream: %ld chunks of %ld samples, halo %ld, %ld re-walks, %zu frames, speculative %s\n",
                nchunks, chunk, halo, nrewalk, frames.size(), spec ? (frames == spec_list ? "hit" : "miss") : "off");
    const size_t nout = std::min(frames.size(), max_frames);
    if (spec && frames == spec_list) return OFDM_OK;  // the speculative decode was the true one
    if (nout == 0) return OFDM_OK;

    // located frames -> main.cpp:60-80 chain + demod
    if ((rc = grow(c, c->s_pbs, (std::max(nout, ub) + 1) * sizeof(long))) ||
        (rc = grow_host(c, c->h_frames, nout * sizeof(long))))
        return rc;
    d_pbs = static_cast<long*>(c->s_pbs.p);
    // the previous call's copy out of the pinned stage must have finished: on
    // the same stream the walk-record sync above saw to it
    if (c->h_frames_used && c->h_frames_stream != st) HIP_TRY(hipStreamSynchronize(c->h_frames_stream));
    c->h_frames_stream = st;
    c->h_frames_used = true;
    std::memcpy(c->h_frames.p, frames.data(), nout * sizeof(long));
    HIP_TRY(hipMemcpyAsync(d_pbs, c->h_frames.p, nout * sizeof(long), hipMemcpyHostToDevice, st));
    if (pb_out) HIP_TRY(hipMemcpyAsync(pb_out, d_pbs, nout * sizeof(long), hipMemcpyDeviceToDevice, st));

    if (!fused) return decode_gathered(d_pbs, nout);
    if ((rc = decode_fused(d_pbs, nout, nullptr))) return rc;
    size_t neg = 0;  // frames before sample 0: the gather path (the fused kernels skip them)
    while (neg < nout && frames[neg] < 0) ++neg;
    return neg ? decode_gathered(d_pbs, neg) : OFDM_OK;
}

extern "C" {

int ofdm_rx_stream(ofdm_ctx* c, const double* iq, size_t n, size_t max_frames, long chunk, long* pb_out,
                   uint8_t* bytes_out, double* constell_out, double* cfo_out, size_t* nframes_out, void* stream)
{
    if (!iq) return fail(OFDM_ERR_INVALID, "null argument");
    return rx_stream_impl(c, iq, nullptr, n, max_frames, chunk, pb_out, bytes_out, constell_out, cfo_out,
                          nframes_out, stream, initial_state(c), 0, (long)n, nullptr, nullptr, 0, nullptr, nullptr);
}

int ofdm_rx_stream_i16(ofdm_ctx* c, const int16_t* iq16, size_t n, size_t max_frames, long chunk, long* pb_out,
                       uint8_t* bytes_out, double* constell_out, double* cfo_out, size_t* nframes_out, void* stream)
{
    if (!iq16) return fail(OFDM_ERR_INVALID, "null argument");
    return rx_stream_impl(c, nullptr, iq16, n, max_frames, chunk, pb_out, bytes_out, constell_out, cfo_out,
                          nframes_out, stream, initial_state(c), 0, (long)n, nullptr, nullptr, 0, nullptr, nullptr);
}

int ofdm_stream_shard_margins(const ofdm_ctx* c, long* halo_out, long* tail_out)
{
    if (!c) return fail(OFDM_ERR_INVALID, "null ctx");
    const long flen = c->geo.frame_len, window = 2 * c->p.t2sin_size + c->p.pr_sin_len;
    if (halo_out) *halo_out = std::max(std::max(0L, c->walk.halo_milli) * flen / 1000, flen + window + c->t2);
    if (tail_out)
        *tail_out = ofdm::WALK_SCAN_MAX + c->t2 + window + c->geo.preamble_len + c->geo.message_len + 1;
    return OFDM_OK;
}

int ofdm_walk_tuning_default(ofdm_walk_tuning* o)
{
    if (!o) return fail(OFDM_ERR_INVALID, "null argument");
    *o = ofdm_walk_tuning{};
    o->chunks_per_slot = 1;
    o->halo_milli = -1;
    o->ext_milli = 0;
    o->exact_search = 0;
    o->t2_f32 = 1;
    o->t2_margin = 4e-5;
    o->lookback = 1;
    o->pre_f32 = 1;
    return OFDM_OK;
}

int ofdm_get_walk_tuning(const ofdm_ctx* c, ofdm_walk_tuning* o)
{
    if (!c || !o) return fail(OFDM_ERR_INVALID, "null argument");
    *o = c->walk;
    return OFDM_OK;
}

int ofdm_set_walk_tuning(ofdm_ctx* c, const ofdm_walk_tuning* t)
{
    if (!c || !t) return fail(OFDM_ERR_INVALID, "null argument");
    if (t->staged_decode != 0 && t->staged_decode != 1) return fail(OFDM_ERR_INVALID, "staged_decode must be 0 or 1");
    if (t->lookback != 0 && t->lookback != 1) return fail(OFDM_ERR_INVALID, "lookback must be 0 or 1");
    if (t->pre_f32 != 0 && t->pre_f32 != 1) return fail(OFDM_ERR_INVALID, "pre_f32 must be 0 or 1");
    if (t->chunks_per_slot < 1 || t->halo_milli < -1 || t->ext_milli < 0 || !(t->t2_margin >= 0.0) ||
        t->max_rec_cap < 0)
        return fail(OFDM_ERR_INVALID, "walk tuning out of range");
    if (t->t2_margin < 4e-5 && !t->allow_uncertified)
        return fail(OFDM_ERR_INVALID, "t2_margin %g is below the certified 4e-5 (the walk could differ from the "
                                      "reference); allow_uncertified = 1 is a test-only switch", t->t2_margin);
    c->walk = *t;
    return OFDM_OK;
}

int ofdm_rx_stream_shard(ofdm_ctx* c, const double* iq, const int16_t* iq16, size_t n, const ofdm_walk_state* start,
                         long own_lo, long own_hi, size_t max_frames, long chunk, long* pb_out, uint8_t* bytes_out,
                         double* constell_out, double* cfo_out, size_t* nframes_out, long* located,
                         uint8_t* located_lag, size_t located_cap, size_t* nlocated_out, ofdm_walk_state* exit_out,
                         void* stream)
{
    if (!iq == !iq16) return fail(OFDM_ERR_INVALID, "exactly one of iq, iq16");
    if (!c || !start) return fail(OFDM_ERR_INVALID, "null argument");
    return rx_stream_impl(c, iq, iq16, n, max_frames, chunk, pb_out, bytes_out, constell_out, cfo_out, nframes_out,
                          stream, *start, own_lo, own_hi, located, located_lag, located_cap, nlocated_out, exit_out);
}

int ofdm_set_stream_timing(ofdm_ctx* c, int on)
{
    if (!c || (on != 0 && on != 1)) return fail(OFDM_ERR_INVALID, "need a ctx and on = 0 or 1");
    HIP_TRY(hipSetDevice(c->device));
    for (hipEvent_t& ev : c->ev_phase)
        if (on && !ev) HIP_TRY(hipEventCreate(&ev));
    c->phase_timing = on != 0;
    c->phase_valid = false;
    return OFDM_OK;
}

int ofdm_get_stream_timing(ofdm_ctx* c, float* walk_ms, float* resolve_ms, float* decode_ms)
{
    if (!c || !walk_ms || !resolve_ms || !decode_ms) return fail(OFDM_ERR_INVALID, "null argument");
    if (!c->phase_valid)
        return fail(OFDM_ERR_INVALID, "no timed call: ofdm_set_stream_timing(ctx, 1), then a look-back stream call "
                                      "whose decode runs behind the resolve");
    HIP_TRY(hipEventSynchronize(c->ev_phase[3]));
    HIP_TRY(hipEventElapsedTime(walk_ms, c->ev_phase[0], c->ev_phase[1]));
    HIP_TRY(hipEventElapsedTime(resolve_ms, c->ev_phase[1], c->ev_phase[2]));
    HIP_TRY(hipEventElapsedTime(decode_ms, c->ev_phase[2], c->ev_phase[3]));
    return OFDM_OK;
}

int ofdm_stream_initial_state(const ofdm_ctx* c, ofdm_walk_state* out)
{
    if (!c || !out) return fail(OFDM_ERR_INVALID, "null argument");
    *out = initial_state(c);
    return OFDM_OK;
}

int ofdm_set_stream_ring(ofdm_ctx* c, long ring)
{
    if (!c) return fail(OFDM_ERR_INVALID, "null ctx");
    // R >= output_size: the smallest ring a config makes (rx_buf_size = 1,
    // Frame.cpp:221, sdr.hpp:141), the default ofdm_create sets from it
    if (ring < 0 || (ring > 0 && ring < c->geo.frame_len))
        return fail(OFDM_ERR_INVALID, "ring must be 0 or at least output_size (rx.cpp's buffer holds output_size + R, "
                                      "R = rx_buf_size * output_size)");
    c->ring = ring;
    return OFDM_OK;
}

int ofdm_shard_range(size_t total, int world, int rank, size_t* first, size_t* count)
{
    if (world < 1 || rank < 0 || rank >= world || !first || !count)
        return fail(OFDM_ERR_INVALID, "need world >= 1, 0 <= rank < world and non-null outputs");
    const size_t base = total / (size_t)world, rem = total % (size_t)world;
    *count = base + ((size_t)rank < rem ? 1 : 0);
    *first = (size_t)rank * base + std::min((size_t)rank, rem);
    return OFDM_OK;
}

int ofdm_stream_shard_plan(const ofdm_params* p, size_t n, int world, int rank, long* slice_lo, long* slice_hi,
                           long* own_lo, long* own_hi)
{
    if (!p || !slice_lo || !slice_hi || !own_lo || !own_hi) return fail(OFDM_ERR_INVALID, "null argument");
    size_t first = 0, count = 0;
    int rc = ofdm_shard_range(n, world, rank, &first, &count);
    if (rc) return rc;
    // ofdm_stream.py: stream_halo / stream_tail (the library's shard margins)
    const long L = p->fft_size + p->cp_size, t2 = p->t2sin_size, pre = L * p->num_pr_symb, msg = L * p->num_symb;
    const long flen = t2 + pre + msg, window = 2 * t2 + p->pr_sin_len;
    const long halo = std::max(3 * flen, flen + window + t2);
    const long tail = ofdm::WALK_SCAN_MAX + t2 + window + pre + msg + 1;
    *own_lo = (long)first;
    *own_hi = (long)(first + count);
    *slice_lo = std::max(0L, *own_lo - halo);
    *slice_hi = std::min((long)n, *own_hi + tail);
    return OFDM_OK;
}

int ofdm_reduce_counters(ofdm_ctx* c, int64_t* counters, size_t count, void* comm, void* stream)
{
    if (!c || !counters || !comm) return fail(OFDM_ERR_INVALID, "null argument");
    // RCCL is loaded on first use (the core library does not link it): the
    // one collective of a multi-GPU job, ncclAllReduce(int64, sum)
    using AllReduce = int (*)(const void*, void*, size_t, int, int, void*, hipStream_t);
    using ErrStr = const char* (*)(int);
    static std::mutex mu;
    static AllReduce all_reduce = nullptr;
    static ErrStr err_str = nullptr;
    {
        std::lock_guard<std::mutex> g(mu);
        if (!all_reduce) {
            void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
            if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
            if (!h) return fail(OFDM_ERR_UNSUPPORTED, "RCCL (librccl.so) not found: %s", dlerror());
            all_reduce = reinterpret_cast<AllReduce>(dlsym(h, "ncclAllReduce"));
            err_str = reinterpret_cast<ErrStr>(dlsym(h, "ncclGetErrorString"));
            if (!all_reduce) return fail(OFDM_ERR_UNSUPPORTED, "librccl.so has no ncclAllReduce");
        }
    }
    HIP_TRY(hipSetDevice(c->device));
    const int r = all_reduce(counters, counters, count, kRcclInt64, kRcclSum, comm, (hipStream_t)stream);
    if (r != 0) return fail(OFDM_ERR_HIP, "ncclAllReduce: %s", err_str ? err_str(r) : "error");
    return OFDM_OK;
}

int ofdm_stream_report_pack(int rank, long slice_lo, long own_lo, long own_hi, const long* located,
                            const uint8_t* located_lag, size_t nlocated, const ofdm_walk_state* exit_state,
                            int true_start, size_t cap, int64_t* row)
{
    // ofdm_stream.py pack_report: header, then the walk's first and last cap
    // located frames, each as 2*pb + lag (-1: empty)
    if (!row || !exit_state || (nlocated && !located) || cap < 1) return fail(OFDM_ERR_INVALID, "null argument or cap 0");
    const size_t H = OFDM_STREAM_REPORT_HEADER;
    const int64_t head[H] = {rank, slice_lo, own_lo, own_hi, exit_state->pos, exit_state->ring_end, true_start ? 1 : 0};
    std::copy(head, head + H, row);
    std::fill(row + H, row + H + 2 * cap, (int64_t)-1);
    auto key = [&](size_t i) { return 2 * (int64_t)located[i] + (located_lag && located_lag[i] ? 1 : 0); };
    const size_t nh = std::min(nlocated, cap);
    for (size_t i = 0; i < nh; ++i) row[H + i] = key(i);
    if (nlocated > cap)
        for (size_t i = 0; i < cap; ++i) row[H + cap + i] = key(nlocated - cap + i);
    return OFDM_OK;
}

int ofdm_stream_stitch_plan(const int64_t* rows, int world, size_t cap, long t2, int* rank_out,
                            ofdm_walk_state* start_out)
{
    // ofdm_stream.py unpack_report + stitch_plan + rewalk_start
    if (!rows || !rank_out || !start_out || world < 1 || cap < 1 || t2 < 1)
        return fail(OFDM_ERR_INVALID, "need rows, outputs, world >= 1, cap >= 1, t2sin_size >= 1");
    const size_t H = OFDM_STREAM_REPORT_HEADER, len = H + 2 * cap;
    auto keys = [&](int r) {  // the rank's located keys (2*pb + lag), sorted, unique
        std::vector<int64_t> k;
        for (size_t i = H; i < len; ++i)
            if (rows[r * len + i] >= 0) k.push_back(rows[r * len + i]);
        std::sort(k.begin(), k.end());
        k.erase(std::unique(k.begin(), k.end()), k.end());
        return k;
    };
    *rank_out = -1;
    *start_out = ofdm_walk_state{-1, 0};
    for (int r = 1; r < world; ++r) {
        const int64_t* cur = rows + r * len;
        const int64_t* prev = rows + (r - 1) * len;
        if (cur[6]) continue;  // walked from a true state
        const std::vector<int64_t> kc = keys(r), kp = keys(r - 1);
        int64_t first = INT64_MAX;  // the first owned frame's preamble start
        for (int64_t k : kc)
            if ((k >> 1) >= cur[2] && (k >> 1) < cur[3]) first = std::min(first, k >> 1);
        std::vector<int64_t> common;
        std::set_intersection(kc.begin(), kc.end(), kp.begin(), kp.end(), std::back_inserter(common));
        bool ok = false;
        for (int64_t k : common) ok = ok || (k >> 1) <= first;
        if (ok) continue;
        *rank_out = r;
        if (prev[4] < 0) return OFDM_OK;  // the true walk ran out of samples before this core
        long pos = (long)prev[4];
        const long slice_lo = (long)cur[1];
        if (pos < slice_lo) pos += (slice_lo - pos + t2 - 1) / t2 * t2;  // forward on its own T2 grid
        *start_out = ofdm_walk_state{pos, (long)prev[5]};
        return OFDM_OK;
    }
    return OFDM_OK;
}

int ofdm_device_count(int* count)
{
    if (!count) return fail(OFDM_ERR_INVALID, "null argument");
    *count = 0;
    int n = 0;
    const hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
    *count = n;
    return OFDM_OK;
}

int ofdm_get_stream_ring(const ofdm_ctx* c, long* ring)
{
    if (!c || !ring) return fail(OFDM_ERR_INVALID, "null argument");
    *ring = c->ring;
    return OFDM_OK;
}

}  // extern "C"
