// ofdm_multigpu — the multi-GPU modem job from C++ over the C-ABI alone
// (BASELINE configs[4]): one thread and one ofdm_ctx per GPU,
// each taking a contiguous share of the frames (ofdm_shard_range), running
// the tx (fused AWGN) -> rx loopback on them, and the job's one collective:
// the SUM all-reduce of {bit errors, bits, samples, frames} over RCCL
// (ofdm_reduce_counters; communicators from ncclCommInitAll). No data-path
// collective: frames are independent. The payload is a counter-based
// function of the global byte index and the noise of the global sample
// index (bench.py's definitions), so the counters do not depend on the GPU
// count. Prints one JSON line (bench.py's metric).
//
//   ofdm_multigpu [--gpus N] [--frames F | --total-frames T] [--steps K] [--warmup W]
//                 [--snr-db X] [--plan-only]
//   --plan-only prints each rank's frame range and a stream's shard plan and
//   touches no GPU.
//
// Stream mode (BASELINE configs[3] over N GPUs; the reference's
// receive loop rx.cpp:125-221 sharded by samples):
//   ofdm_multigpu --stream FILE [--f64] [--config CFG] [--shards N] [--gpus G]
//                 [--report-cap C] [--reps K] [--pbs-out FILE]
//   FILE holds the stream as the SDR delivers it, complex<int16> pairs (or
//   complex<double> with --f64). N ranks (default: one per GPU), rank r on
//   device r % G, each with its own ofdm_ctx and thread: it walks and decodes
//   its slice (ofdm_stream_shard_plan, ofdm_rx_stream_shard), packs its
//   report row (ofdm_stream_report_pack), the ranks all-gather the rows
//   (ncclAllGather with one rank per GPU; through host memory when ranks
//   share a GPU, the in-process mode) and all run the same plan
//   (ofdm_stream_stitch_plan): the rank it names re-walks from its
//   predecessor's exit state, and the exchange repeats until every walk is
//   accepted. Prints one JSON line; --pbs-out writes every owned frame's
//   preamble start (int64, stream order): the sequential walk's frames.
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ofdm_mi355x.h"

namespace {

// bench.py CONFIG_B: 2048-subcarrier QPSK frames of 8 symbols (BASELINE configs[1])
ofdm_params config_b()
{
    ofdm_params p{};
    ofdm_params_default(&p);
    p.fft_size = 2048;
    p.num_data_subc = 1024;
    p.num_pilot_subc = 32;
    p.cp_size = 512;
    p.mod_type = 2;
    return p;
}

uint64_t splitmix64(uint64_t z)
{
    z *= 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// byte i of the job = splitmix64(0x5EED + i) & 0xFF (ofdm_synth.payload_bytes)
void payload(uint64_t begin, std::vector<uint8_t>& out)
{
    for (size_t i = 0; i < out.size(); ++i) out[i] = (uint8_t)(splitmix64(0x5EED + begin + i) & 0xFF);
}

struct Barrier {  // the ranks' host barrier (threads of this process)
    std::mutex mu;
    std::condition_variable cv;
    int n, waiting = 0;
    long gen = 0;
    explicit Barrier(int n_) : n(n_) {}
    void wait()
    {
        std::unique_lock<std::mutex> l(mu);
        const long g = gen;
        if (++waiting == n) {
            waiting = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(l, [&] { return gen != g; });
        }
    }
};

[[noreturn]] void die(int rank, const char* what)
{
    std::fprintf(stderr, "rank %d: %s: %s\n", rank, what, ofdm_last_error());
    std::exit(1);
}
#define CHECK(rank, expr) \
    do {                     \
        if ((expr) != OFDM_OK) die(rank, #expr); \
    } while (0)

}  // namespace

// the stream mode (see the header comment); returns the process exit code
int stream_main(const std::string& path, bool f64, const std::string& cfg, int shards, int gpus, size_t cap,
                int reps, const std::string& pbs_out);

int main(int argc, char** argv)
{
    int gpus = 0, steps = 20, warmup = 5;
    long frames = 8192, total_frames = 0;
    double snr_db = 10.0;
    bool plan_only = false;
    std::string stream_path, cfg_path, pbs_out;
    bool f64 = false;
    int shards = 0, reps = 1;
    size_t cap = 64;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() { return i + 1 < argc ? argv[++i] : (std::fprintf(stderr, "%s needs a value\n", a.c_str()), std::exit(2), ""); };
        if (a == "--gpus") gpus = std::atoi(next());
        else if (a == "--frames") frames = std::atol(next());
        else if (a == "--total-frames") total_frames = std::atol(next());
        else if (a == "--steps") steps = std::atoi(next());
        else if (a == "--warmup") warmup = std::atoi(next());
        else if (a == "--snr-db") snr_db = std::atof(next());
        else if (a == "--plan-only") plan_only = true;
        else if (a == "--stream") stream_path = next();
        else if (a == "--f64") f64 = true;
        else if (a == "--config") cfg_path = next();
        else if (a == "--shards") shards = std::atoi(next());
        else if (a == "--report-cap") cap = (size_t)std::atol(next());
        else if (a == "--reps") reps = std::atoi(next());
        else if (a == "--pbs-out") pbs_out = next();
        else {
            std::fprintf(stderr, "usage: %s [--gpus N] [--frames F | --total-frames T] [--steps K] [--warmup W] "
                                 "[--snr-db X] [--plan-only] | --stream FILE [--f64] [--config CFG] [--shards N] "
                                 "[--gpus G] [--report-cap C] [--reps K] [--pbs-out FILE]\n", argv[0]);
            return 2;
        }
    }
    if (!stream_path.empty()) return stream_main(stream_path, f64, cfg_path, shards, gpus, cap, reps, pbs_out);
    const ofdm_params p = config_b();
    const long L = p.fft_size + p.cp_size, msg = L * p.num_symb;
    const long bpf = p.num_data_subc * p.num_symb * p.mod_type / 8;
    if (plan_only) {  // the sharding arithmetic, no GPU: frame ranges, and a stream of 10^8 samples
        const int world = gpus > 0 ? gpus : 8;
        const long total = total_frames > 0 ? total_frames : frames * world;
        std::printf("{\"world\": %d, \"total_frames\": %ld, \"ranks\": [", world, total);
        for (int r = 0; r < world; ++r) {
            size_t f0 = 0, nf = 0;
            long sl, sh, ol, oh;
            if (ofdm_shard_range((size_t)total, world, r, &f0, &nf) ||
                ofdm_stream_shard_plan(&p, 100000000, world, r, &sl, &sh, &ol, &oh))
                die(r, "plan");
            std::printf("%s{\"rank\": %d, \"first\": %zu, \"count\": %zu, \"stream\": [%ld, %ld, %ld, %ld]}",
                        r ? ", " : "", r, f0, nf, sl, sh, ol, oh);
        }
        std::printf("]}\n");
        return 0;
    }
    if (gpus <= 0 && ofdm_device_count(&gpus) != OFDM_OK) die(0, "ofdm_device_count");
    if (gpus <= 0) {
        std::fprintf(stderr, "no GPU\n");
        return 1;
    }
    // RCCL communicators, one per GPU (one process: ncclCommInitAll)
    std::vector<ncclComm_t> comms(gpus);
    std::vector<int> devs(gpus);
    for (int r = 0; r < gpus; ++r) devs[r] = r;
    if (ncclCommInitAll(comms.data(), gpus, devs.data()) != ncclSuccess) {
        std::fprintf(stderr, "ncclCommInitAll failed\n");
        return 1;
    }
    const double es = 2.0;  // QPSK constellation energy
    const double noise_std = std::sqrt(es / std::pow(10.0, snr_db / 10.0));
    Barrier bar(gpus);
    std::vector<double> elapsed(gpus, 0.0), rx_ms(gpus, 0.0);
    std::vector<int64_t> totals(4, 0);
    auto rank_main = [&](int r) {
        size_t f0 = (size_t)r * frames, nf = (size_t)frames;
        if (total_frames > 0) CHECK(r, ofdm_shard_range((size_t)total_frames, gpus, r, &f0, &nf));
        ofdm_ctx* c = nullptr;
        CHECK(r, ofdm_create(&p, r, &c));
        void* st = nullptr;
        CHECK(r, ofdm_stream_create(c, &st));
        std::vector<uint8_t> h_data(nf * bpf);
        payload(f0 * bpf, h_data);
        void *d_data, *d_iq, *d_cons, *d_out, *d_errs, *d_cnt;
        CHECK(r, ofdm_device_alloc(c, h_data.size() ? h_data.size() : 1, &d_data));
        CHECK(r, ofdm_device_alloc(c, std::max<size_t>(1, nf * msg * 16), &d_iq));
        CHECK(r, ofdm_device_alloc(c, std::max<size_t>(1, nf * p.num_data_subc * p.num_symb * 16), &d_cons));
        CHECK(r, ofdm_device_alloc(c, std::max<size_t>(1, h_data.size()), &d_out));
        CHECK(r, ofdm_device_alloc(c, 8, &d_errs));
        CHECK(r, ofdm_device_alloc(c, 4 * sizeof(int64_t), &d_cnt));
        CHECK(r, ofdm_memcpy_h2d(c, d_data, h_data.data(), h_data.size(), st));
        ofdm_channel ch{noise_std, 1, (unsigned long long)(f0 * msg)};
        auto step = [&]() {
            if (!nf) return;
            CHECK(r, ofdm_tx_modulate(c, (const uint8_t*)d_data, nf, (double*)d_iq, (size_t)msg, nullptr, &ch, st));
            CHECK(r, ofdm_rx_demod(c, (const double*)d_iq, nf, (size_t)msg, nullptr, 0, (double*)d_cons,
                                   (uint8_t*)d_out, (const uint8_t*)d_data, (unsigned long long*)d_errs, st));
        };
        for (int i = 0; i < warmup; ++i) step();
        CHECK(r, ofdm_stream_synchronize(c, st));
        bar.wait();
        CHECK(r, ofdm_memset_device(c, d_errs, 0, 8, st));
        const int64_t mine[4] = {0, (int64_t)(steps * nf * bpf * 8), (int64_t)(steps * nf * msg), (int64_t)(steps * nf)};
        CHECK(r, ofdm_memcpy_h2d(c, d_cnt, mine, sizeof(mine), st));
        CHECK(r, ofdm_stream_synchronize(c, st));
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < steps; ++i) step();
        // the one collective: {bit errors, bits, samples, frames} summed over the ranks
        CHECK(r, ofdm_memcpy_d2d(c, d_cnt, d_errs, 8, st));
        CHECK(r, ofdm_reduce_counters(c, (int64_t*)d_cnt, 4, comms[r], st));
        CHECK(r, ofdm_stream_synchronize(c, st));
        bar.wait();
        elapsed[r] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (r == 0) CHECK(r, ofdm_memcpy_d2h(c, totals.data(), d_cnt, 4 * sizeof(int64_t), st));
        CHECK(r, ofdm_stream_synchronize(c, st));
        for (void* d : {d_data, d_iq, d_cons, d_out, d_errs, d_cnt}) ofdm_device_free(c, d);
        ofdm_stream_destroy(c, st);
        ofdm_destroy(c);
    };
    std::vector<std::thread> th;
    for (int r = 0; r < gpus; ++r) th.emplace_back(rank_main, r);
    for (auto& t : th) t.join();
    for (auto& cm : comms) ncclCommDestroy(cm);
    const double el = *std::max_element(elapsed.begin(), elapsed.end());  // max over ranks
    std::printf("{\"metric\": \"IQ-samples/sec (tx IFFT+CP and rx FFT+equalise), 2048-subcarrier frames, "
                "1/2/4/8 GPU\", \"value\": %.6e, \"unit\": \"IQ-samples/s\", \"n_gpus\": %d, \"steps\": %d, "
                "\"warmup\": %d, \"ms_per_step\": %.4f, \"scaling\": \"%s\", \"bit_errors\": %lld, \"bits\": %lld, "
                "\"ber\": %.6e, \"frames\": %lld, \"host\": \"C++ over the C-ABI, one thread + ofdm_ctx per GPU, "
                "RCCL all-reduce of the counters\"}\n",
                totals[2] / el, gpus, steps, warmup, el / steps * 1e3, total_frames > 0 ? "strong" : "weak",
                (long long)totals[0], (long long)totals[1], totals[1] ? (double)totals[0] / totals[1] : 0.0,
                (long long)totals[3]);
    return 0;
}

// ---------------------------------------------------------------- stream mode
namespace {

struct RankRx {  // one rank's context, slice and outputs
    ofdm_ctx* c = nullptr;
    void* st = nullptr;
    long slice_lo = 0, slice_hi = 0, own_lo = 0, own_hi = 0;
    void *d_iq = nullptr, *d_pb = nullptr, *d_bytes = nullptr, *d_cons = nullptr, *d_cfo = nullptr;
    size_t max_frames = 0, n_owned = 0;
    int rewalks = 0;
    std::vector<long> located;
    std::vector<uint8_t> lag;
    std::vector<int64_t> row;
};

}  // namespace

int stream_main(const std::string& path, bool f64, const std::string& cfg, int shards, int gpus, size_t cap,
                int reps, const std::string& pbs_out)
{
    ofdm_params p{};
    if (cfg.empty() ? ofdm_params_default(&p) : ofdm_params_from_config(cfg.c_str(), &p)) die(0, "config");
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) {
        std::fprintf(stderr, "cannot open %s\n", path.c_str());
        return 1;
    }
    std::fseek(f, 0, SEEK_END);
    const long bytes = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    const size_t esz = f64 ? 16 : 4;
    const size_t n = (size_t)bytes / esz;
    std::vector<char> host((size_t)bytes);
    if (std::fread(host.data(), 1, host.size(), f) != host.size()) {
        std::fprintf(stderr, "short read %s\n", path.c_str());
        return 1;
    }
    std::fclose(f);
    int ndev = 0;
    if (ofdm_device_count(&ndev) != OFDM_OK || ndev < 1) die(0, "ofdm_device_count");
    if (gpus <= 0 || gpus > ndev) gpus = ndev;
    const int world = shards > 0 ? shards : gpus;
    // one rank per GPU: RCCL moves the rows; ranks sharing a GPU: host memory
    const bool rccl = world == gpus && world > 1;
    std::vector<ncclComm_t> comms;
    if (rccl) {
        comms.resize(world);
        std::vector<int> devs(world);
        for (int r = 0; r < world; ++r) devs[r] = r;
        if (ncclCommInitAll(comms.data(), world, devs.data()) != ncclSuccess) {
            std::fprintf(stderr, "ncclCommInitAll failed\n");
            return 1;
        }
    }
    const size_t len = OFDM_STREAM_REPORT_HEADER + 2 * cap;
    const long L = p.fft_size + p.cp_size, flen = p.t2sin_size + L * (p.num_pr_symb + p.num_symb);
    const long bpf = p.num_data_subc * p.num_symb * p.mod_type / 8, npts = (long)p.num_data_subc * p.num_symb;
    std::vector<RankRx> rk(world);
    std::vector<int64_t> rows(world * len);  // the all-gathered rows (every rank reads them)
    Barrier bar(world);
    std::vector<double> elapsed(world, 0.0);
    std::vector<int> plan_rank(1, -1);
    std::vector<ofdm_walk_state> plan_start(1);
    std::vector<std::vector<long>> owned(world);

    auto rank_main = [&](int r) {
        RankRx& x = rk[r];
        CHECK(r, ofdm_create(&p, r % gpus, &x.c));
        CHECK(r, ofdm_stream_create(x.c, &x.st));
        CHECK(r, ofdm_stream_shard_plan(&p, n, world, r, &x.slice_lo, &x.slice_hi, &x.own_lo, &x.own_hi));
        const size_t ns = (size_t)(x.slice_hi - x.slice_lo);
        x.max_frames = ns / (size_t)flen + 16;
        CHECK(r, ofdm_device_alloc(x.c, std::max<size_t>(1, ns * esz), &x.d_iq));
        CHECK(r, ofdm_device_alloc(x.c, x.max_frames * sizeof(long), &x.d_pb));
        CHECK(r, ofdm_device_alloc(x.c, x.max_frames * bpf, &x.d_bytes));
        CHECK(r, ofdm_device_alloc(x.c, x.max_frames * npts * 16, &x.d_cons));
        CHECK(r, ofdm_device_alloc(x.c, x.max_frames * sizeof(double), &x.d_cfo));
        CHECK(r, ofdm_memcpy_h2d(x.c, x.d_iq, host.data() + (size_t)x.slice_lo * esz, ns * esz, x.st));
        long ring = 0;
        CHECK(r, ofdm_get_stream_ring(x.c, &ring));
        x.located.resize(2 * cap);
        x.lag.resize(2 * cap);
        x.row.resize(len);
        void *d_row = nullptr, *d_rows = nullptr;
        if (rccl) {
            CHECK(r, ofdm_device_alloc(x.c, len * sizeof(int64_t), &d_row));
            CHECK(r, ofdm_device_alloc(x.c, world * len * sizeof(int64_t), &d_rows));
        }
        // walk from an absolute state, pack the report row
        auto walk = [&](ofdm_walk_state s, bool true_start) {
            ofdm_walk_state rel{s.pos - x.slice_lo, ring ? s.ring_end - x.slice_lo : 0}, ex{};
            size_t nl = 0, nf = 0;
            if (s.pos < 0 && r > 0) {  // the true walk ended before this core: nothing owned
                x.n_owned = 0;
                nl = 0;
                ex = ofdm_walk_state{-1, 0};
            } else {
                CHECK(r, ofdm_rx_stream_shard(x.c, f64 ? (const double*)x.d_iq : nullptr,
                                              f64 ? nullptr : (const int16_t*)x.d_iq, ns, &rel, x.own_lo - x.slice_lo,
                                              x.own_hi - x.slice_lo, x.max_frames, 0, (long*)x.d_pb,
                                              (uint8_t*)x.d_bytes, (double*)x.d_cons, (double*)x.d_cfo, &nf,
                                              x.located.data(), x.lag.data(), 2 * cap, &nl, &ex, x.st));
                x.n_owned = std::min(nf, x.max_frames);
                if (ex.pos >= 0) ex = ofdm_walk_state{ex.pos + x.slice_lo, ring ? ex.ring_end + x.slice_lo : 0};
            }
            const size_t k = std::min(nl, 2 * cap);
            for (size_t i = 0; i < k; ++i) x.located[i] += x.slice_lo;
            CHECK(r, ofdm_stream_report_pack(r, x.slice_lo, x.own_lo, x.own_hi, x.located.data(), x.lag.data(), k,
                                             &ex, true_start ? 1 : 0, cap, x.row.data()));
        };
        auto exchange = [&]() {
            if (rccl) {
                CHECK(r, ofdm_memcpy_h2d(x.c, d_row, x.row.data(), len * sizeof(int64_t), x.st));
                if (ncclAllGather(d_row, d_rows, len, ncclInt64, comms[r], (hipStream_t)x.st) != ncclSuccess)
                    die(r, "ncclAllGather");
                std::vector<int64_t> all(world * len);
                CHECK(r, ofdm_memcpy_d2h(x.c, all.data(), d_rows, all.size() * sizeof(int64_t), x.st));
                CHECK(r, ofdm_stream_synchronize(x.c, x.st));
                bar.wait();
                if (r == 0) rows = all;
                bar.wait();
            } else {
                bar.wait();  // every rank's row is final
                std::copy(x.row.begin(), x.row.end(), rows.begin() + r * len);
                bar.wait();
            }
        };
        for (int it = 0; it < reps; ++it) {
            bar.wait();
            const auto t0 = std::chrono::steady_clock::now();
            ofdm_walk_state s0{};
            if (r == 0) {
                CHECK(r, ofdm_stream_initial_state(x.c, &s0));
            } else {
                s0 = ofdm_walk_state{x.slice_lo, ring ? (x.slice_lo / ring + 1) * ring : 0};
            }
            walk(s0, r == 0);
            x.rewalks = 0;
            for (;;) {
                exchange();
                if (r == 0) CHECK(r, ofdm_stream_stitch_plan(rows.data(), world, cap, p.t2sin_size, &plan_rank[0],
                                                             &plan_start[0]));
                bar.wait();
                const int pr = plan_rank[0];
                const ofdm_walk_state ps = plan_start[0];
                bar.wait();  // every rank has read the plan
                if (pr < 0) break;
                if (pr == r) {
                    walk(ps, true);
                    ++x.rewalks;
                }
            }
            CHECK(r, ofdm_stream_synchronize(x.c, x.st));  // the decodes
            bar.wait();
            elapsed[r] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        }
        std::vector<long> pb(x.n_owned);
        if (x.n_owned) CHECK(r, ofdm_memcpy_d2h(x.c, pb.data(), x.d_pb, x.n_owned * sizeof(long), x.st));
        CHECK(r, ofdm_stream_synchronize(x.c, x.st));
        for (long& v : pb) v += x.slice_lo;
        owned[r] = pb;
        for (void* d : {x.d_iq, x.d_pb, x.d_bytes, x.d_cons, x.d_cfo, d_row, d_rows})
            if (d) ofdm_device_free(x.c, d);
        ofdm_stream_destroy(x.c, x.st);
        ofdm_destroy(x.c);
    };
    std::vector<std::thread> th;
    for (int r = 0; r < world; ++r) th.emplace_back(rank_main, r);
    for (auto& t : th) t.join();
    for (auto& cm : comms) ncclCommDestroy(cm);
    size_t total = 0;
    int rewalks = 0;
    for (int r = 0; r < world; ++r) {
        total += owned[r].size();
        rewalks += rk[r].rewalks;
    }
    if (!pbs_out.empty()) {
        FILE* o = std::fopen(pbs_out.c_str(), "wb");
        if (!o) die(0, "pbs-out");
        for (int r = 0; r < world; ++r)
            if (!owned[r].empty()) std::fwrite(owned[r].data(), sizeof(long), owned[r].size(), o);
        std::fclose(o);
    }
    const double el = *std::max_element(elapsed.begin(), elapsed.end());
    std::printf("{\"metric\": \"stream samples/s (T2 walk + preamble sync + CFO/CP/phase/chan sync + demod), "
                "sharded stream\", \"value\": %.6e, \"unit\": \"stream samples/s\", \"ranks\": %d, \"gpus\": %d, "
                "\"exchange\": \"%s\", \"stream_samples\": %zu, \"format\": \"%s\", \"frames\": %zu, "
                "\"rewalks\": %d, \"ms_per_stream\": %.4f, \"host\": \"C++ over the C-ABI, one thread + ofdm_ctx per "
                "rank, report rows all-gathered, ofdm_stream_stitch_plan\"}\n",
                n / el, world, gpus, rccl ? "ncclAllGather" : "host memory (ranks share a GPU)", n,
                f64 ? "complex<double>" : "complex<int16>", total, rewalks, el * 1e3);
    return 0;
}
