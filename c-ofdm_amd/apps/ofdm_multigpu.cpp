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

int main(int argc, char** argv)
{
    int gpus = 0, steps = 20, warmup = 5;
    long frames = 8192, total_frames = 0;
    double snr_db = 10.0;
    bool plan_only = false;
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
        else {
            std::fprintf(stderr, "usage: %s [--gpus N] [--frames F | --total-frames T] [--steps K] [--warmup W] "
                                 "[--snr-db X] [--plan-only]\n", argv[0]);
            return 2;
        }
    }
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
