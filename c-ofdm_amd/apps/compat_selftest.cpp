// compat_selftest — checks of the drop-in layer's device mirrors
// (ofdm_compat::Mirror) on the GPU:
//   1. the rx chain of main.cpp / rx.cpp (pilot_freq_sinh, freq_shift,
//      cp_freq_sinh, pr_phase_sinh, chan_char_lq, fft) on a FRAME_FORM's
//      mirrored buf equals, bit for bit, the same chain on forms bound to a
//      plain vector (staged through the arena, no mirror) — for fresh
//      frames, for the same frame copied in again after the in-place
//      members ran (the host bytes then equal neither the shadow's nor the
//      device's), for partial host writes between members, and with the
//      run-ahead chain (ofdm_compat::Chain) served, refused (another CFO
//      value, a skipped member) and taken in another order;
//   2. form_int16_to_double, find_t2sin, find_preamble and corr on the
//      mirrored rx ring equal the staged path, also after direct host writes
//      to from_sdr_buf;
//      the chain also serves Modulation::demod after rx.cpp's division:
//      its bytes and in-place clamp equal the unserved demod's, and a point
//      moved after the division makes it refuse;
//   3. PREAMBLE_FORM::chan_char equals the reference's formula
//      (Frame.hpp:375-385) evaluated here on fft()'s output.
// Usage: compat_selftest <config.txt> [frames]. Prints "SELFTEST OK ...".
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>

#include "OFDM/Frame.hpp"

static int g_fail = 0;

#define CHECK(cond, ...)                          \
    do {                                          \
        if (!(cond)) {                            \
            std::fprintf(stderr, "FAIL: " __VA_ARGS__); \
            std::fprintf(stderr, "\n");           \
            ++g_fail;                             \
        }                                         \
    } while (0)

static bool same(const complex_double* a, const complex_double* b, size_t n)
{
    return std::memcmp(a, b, n * sizeof(complex_double)) == 0;
}

int main(int argc, char** argv)
{
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s config.txt [frames]\n", argv[0]);
        return 2;
    }
    const std::string cfg = argv[1];
    const int nframes = argc > 2 ? std::atoi(argv[2]) : 12;
    FRAME_FORM tx(cfg), rx(cfg);
    ConfigMap c = parse_config(cfg);
    // the same forms bound to a plain vector: no mirror covers it
    PREAMBLE_FORM pre2(c);
    OFDM_FORM msg2(c);
    OFDM_FORM mwp2(c, true, true);
    const int t2 = rx.t2sin.size, npre = rx.preamble.size, nmsg = rx.message.size;
    complex_vector plain(rx.buf.size(), complex_double(0, 0));
    pre2.set(plain.data() + t2);
    msg2.set(plain.data() + t2 + npre);
    mwp2.set(plain.data() + t2);
    CHECK(same(rx.preamble.ofdm_preamble.data(), pre2.ofdm_preamble.data(), npre), "preamble symbols differ");

    std::mt19937 rng(7);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    std::normal_distribution<double> Nn(0.0, 0.02);
    const size_t span = (size_t)npre + nmsg;
    auto run_chain = [&](const char* what, int k) {
        complex_double* a = rx.buf.data() + t2;
        complex_double* b = plain.data() + t2;
        double c1 = rx.preamble.pilot_freq_sinh(), c2 = pre2.pilot_freq_sinh();
        CHECK(c1 == c2, "%s frame %d: pilot_freq_sinh %.17g vs %.17g", what, k, c1, c2);
        rx.message_with_preamble.freq_shift(c1);
        mwp2.freq_shift(c2);
        CHECK(same(a, b, span), "%s frame %d: freq_shift", what, k);
        rx.message_with_preamble.cp_freq_sinh();
        mwp2.cp_freq_sinh();
        CHECK(same(a, b, span), "%s frame %d: cp_freq_sinh", what, k);
        rx.message_with_preamble.pr_phase_sinh(rx.preamble.ofdm_preamble.data(), rx.preamble.size);
        mwp2.pr_phase_sinh(pre2.ofdm_preamble.data(), pre2.size);
        CHECK(same(a, b, span), "%s frame %d: pr_phase_sinh", what, k);
        auto& h1 = rx.preamble.chan_char_lq();
        auto& h2 = pre2.chan_char_lq();
        CHECK(h1.size() == h2.size() && same(h1.data(), h2.data(), h1.size()), "%s frame %d: chan_char_lq", what, k);
        auto f1 = rx.message.fft(), f2 = msg2.fft();
        CHECK(f1.size() == f2.size() && same(f1.data(), f2.data(), f1.size()), "%s frame %d: fft", what, k);
        // rx.cpp:214-221: the division by chan_char, then Modulation::demod
        // (served from the chain's decisions for the mirrored form when the
        // points are the chain's, bit for bit; every fourth frame one point
        // is moved after the division, so the served demod must refuse)
        complex_vector d1(f1), d2(f2);
        for (size_t j = 0; j < d1.size(); j++) {
            d1[j] /= h1[j % h1.size()];
            d2[j] /= h2[j % h2.size()];
        }
        if (k % 4 == 2 && d1.size() > 7) {
            d1[7] += complex_double(1e-3, 0.0);
            d2[7] += complex_double(1e-3, 0.0);
        }
        const bit_vector b1 = rx.message.Mod.demod(d1), b2 = msg2.Mod.demod(d2);
        CHECK(b1 == b2, "%s frame %d: demod bytes", what, k);
        CHECK(same(d1.data(), d2.data(), d1.size()), "%s frame %d: demod's in-place clamp", what, k);
    };

    std::vector<complex_vector> sent;
    for (int k = 0; k < nframes; ++k) {
        bit_vector bytes(rx.usefull_size);
        for (auto& v : bytes) v = (uint8_t)(rng() & 0xff);
        tx.write(bytes);
        complex_vector f = tx.get();
        const double cfo = 0.003 * U(rng), ph = 3.0 * U(rng);
        for (size_t n = 0; n < f.size(); ++n)
            f[n] = f[n] * std::polar(1.0, 2 * M_PI * cfo * (double)n + ph) + complex_double(Nn(rng), Nn(rng));
        sent.push_back(f);
        std::copy(f.begin(), f.end(), rx.buf.begin());
        std::copy(f.begin(), f.end(), plain.begin());
        run_chain("fresh", k);
        if (k % 3 == 1) {
            // the same frame copied in again: the host now holds what the
            // mirror's shadow held before the in-place members ran
            std::copy(f.begin(), f.end(), rx.buf.begin());
            std::copy(f.begin(), f.end(), plain.begin());
            run_chain("recopied", k);
        }
        if (k % 4 == 3) {
            // the run-ahead chain must not be served for another CFO value,
            // nor out of order (fft before chan_char_lq, cp_freq_sinh skipped)
            std::copy(f.begin(), f.end(), rx.buf.begin());
            std::copy(f.begin(), f.end(), plain.begin());
            double c1 = rx.preamble.pilot_freq_sinh(), c2 = pre2.pilot_freq_sinh();
            CHECK(c1 == c2, "other-cfo frame %d: pilot_freq_sinh", k);
            c1 += 1e-7;
            c2 += 1e-7;
            rx.message_with_preamble.freq_shift(c1);
            mwp2.freq_shift(c2);
            CHECK(same(rx.buf.data() + t2, plain.data() + t2, span), "other-cfo frame %d: freq_shift", k);
            rx.message_with_preamble.pr_phase_sinh(rx.preamble.ofdm_preamble.data(), rx.preamble.size);
            mwp2.pr_phase_sinh(pre2.ofdm_preamble.data(), pre2.size);
            CHECK(same(rx.buf.data() + t2, plain.data() + t2, span), "other-cfo frame %d: pr_phase_sinh", k);
            auto f1 = rx.message.fft(), f2 = msg2.fft();
            CHECK(same(f1.data(), f2.data(), f1.size()), "other-cfo frame %d: fft", k);
            auto& h1 = rx.preamble.chan_char_lq();
            auto& h2 = pre2.chan_char_lq();
            CHECK(same(h1.data(), h2.data(), h1.size()), "other-cfo frame %d: chan_char_lq", k);
            // the full chain in the reference's order again, fft before chan_char_lq
            std::copy(f.begin(), f.end(), rx.buf.begin());
            std::copy(f.begin(), f.end(), plain.begin());
            c1 = rx.preamble.pilot_freq_sinh();
            c2 = pre2.pilot_freq_sinh();
            rx.message_with_preamble.freq_shift(c1);
            mwp2.freq_shift(c2);
            rx.message_with_preamble.cp_freq_sinh();
            mwp2.cp_freq_sinh();
            rx.message_with_preamble.pr_phase_sinh(rx.preamble.ofdm_preamble.data(), rx.preamble.size);
            mwp2.pr_phase_sinh(pre2.ofdm_preamble.data(), pre2.size);
            auto g1 = rx.message.fft(), g2 = msg2.fft();
            CHECK(same(g1.data(), g2.data(), g1.size()), "fft-first frame %d: fft", k);
            auto& q1 = rx.preamble.chan_char_lq();
            auto& q2 = pre2.chan_char_lq();
            CHECK(same(q1.data(), q2.data(), q1.size()), "fft-first frame %d: chan_char_lq", k);
            CHECK(same(rx.buf.data() + t2, plain.data() + t2, span), "fft-first frame %d: buffer", k);
        }
        if (k % 3 == 2) {
            // partial host writes between members
            const double c1 = rx.preamble.pilot_freq_sinh();
            (void)pre2.pilot_freq_sinh();
            rx.message_with_preamble.freq_shift(const_cast<double&>(c1));
            double c2 = c1;
            mwp2.freq_shift(c2);
            for (int j = 0; j < 37; ++j) {
                const size_t at = (size_t)t2 + (rng() % span);
                const complex_double v(U(rng), U(rng));
                rx.buf[at] = v;
                plain[at] = v;
            }
            rx.message_with_preamble.cp_freq_sinh();
            mwp2.cp_freq_sinh();
            CHECK(same(rx.buf.data() + t2, plain.data() + t2, span), "partial writes frame %d: cp_freq_sinh", k);
            auto f1 = rx.message.fft(), f2 = msg2.fft();
            CHECK(same(f1.data(), f2.data(), f1.size()), "partial writes frame %d: fft", k);
        }
    }

    // chan_char (Frame.hpp:375-385): the reference's formula on fft()
    {
        complex_vector pr = rx.preamble.fft();
        complex_vector want(rx.preamble.num_data_subc, complex_double(0, 0));
        for (int i = 0; i < rx.preamble.num_data_subc * rx.preamble.num_symb; i++)
            want[i % rx.preamble.num_data_subc] += pr[i] / rx.preamble.mod_preamble[i];
        for (auto& v : want) v /= complex_double(rx.preamble.num_symb, 0);
        complex_vector got = rx.preamble.chan_char();
        CHECK(got.size() == want.size() && same(got.data(), want.data(), got.size()), "chan_char vs Frame.hpp:375-385");
    }

    // the rx ring: int16 capture of the sent frames with gaps
    {
        const size_t ring = rx.from_sdr_int16_buf.size();
        std::fill(rx.from_sdr_int16_buf.begin(), rx.from_sdr_int16_buf.end(), std::complex<int16_t>(0, 0));
        size_t pos = 1000;
        const int mult = (int)c["mult"];
        for (size_t k = 0; k < sent.size() && pos + sent[k].size() < ring; ++k) {
            for (size_t n = 0; n < sent[k].size(); ++n)
                rx.from_sdr_int16_buf[pos + n] = std::complex<int16_t>((int16_t)(sent[k][n].real() * mult),
                                                                       (int16_t)(sent[k][n].imag() * mult));
            pos += sent[k].size() + 777 + 313 * (k % 4);
        }
        rx.form_int16_to_double();
        bool conv = true;
        for (size_t i = 0; i < ring; ++i)
            conv = conv && rx.from_sdr_buf[i] == complex_double(rx.from_sdr_int16_buf[i].real(),
                                                                rx.from_sdr_int16_buf[i].imag());
        CHECK(conv, "form_int16_to_double");
        for (int round = 0; round < 2; ++round) {
            complex_vector copy(rx.from_sdr_buf);  // not mirrored: the staged path
            auto c1 = rx.t2sin.corr(rx.from_sdr_buf), c2 = rx.t2sin.corr(copy);
            CHECK(c1 == c2, "corr round %d", round);
            int p1 = 0, p2 = 0, found = 0;
            for (int it = 0; it < 64; ++it) {
                p1 = rx.t2sin.find_t2sin(rx.from_sdr_buf, p1);
                p2 = rx.t2sin.find_t2sin(copy, p2);
                CHECK(p1 == p2, "find_t2sin round %d step %d: %d vs %d", round, it, p1, p2);
                if (p1 < 0 || p1 != p2) break;
                const int q1 = rx.preamble.find_preamble(rx.from_sdr_buf, p1), q2 = rx.preamble.find_preamble(copy, p2);
                CHECK(q1 == q2, "find_preamble round %d step %d: %d vs %d", round, it, q1, q2);
                if (q1 >= 0) {
                    ++found;
                    p1 = p2 = q1 + 1 + rx.message.size;
                } else {
                    p1 = p2 = p1 + rx.message.size;
                }
            }
            CHECK(found >= 2, "round %d: only %d frames located in the ring", round, found);
            // direct host writes to the ring (no form_int16_to_double): the
            // mirror must pick them up
            for (size_t i = 500; i < ring; i += 4099) rx.from_sdr_buf[i] *= -1.0;
            for (size_t i = 1000; i < 1000 + 6000 && i < ring; ++i) rx.from_sdr_buf[i] *= complex_double(0.0, 1.0);
        }
    }
    if (g_fail) {
        std::fprintf(stderr, "SELFTEST FAILED: %d checks\n", g_fail);
        return 1;
    }
    std::printf("SELFTEST OK frames=%d\n", nframes);
    return 0;
}
