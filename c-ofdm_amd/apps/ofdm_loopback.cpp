// ofdm_loopback — one-shot tx -> air -> rx over the drop-in class surface
// (the flow of the reference's main.cpp:21-113, written against the compat
// headers): MAC-frame a payload, FRAME_FORM::write, get_int16, SDR::send x2,
// SDR::recv, form_int16_to_double, T2 + preamble detection, CFO / CP / phase
// sync, chan_char_lq, FFT + equalise, demod, MAC::read, accuracy, and the
// data/*.bin dumps python_code/ reads. Every DSP step runs on the GPU.
//
//   ofdm_loopback CONFIG [PAYLOAD_FILE] [OUT_DIR]     exit 0 iff the payload decodes exactly
#include <cstdio>
#include <cstring>
#include <iostream>
#include <string>
#include <sys/stat.h>

#include "OFDM/Frame.hpp"
#include "OFDM/modulation.hpp"
#include "io/io.hpp"
#include "mac/mac_frame.hpp"
#include "sdr/sdr.hpp"

int main(int argc, char** argv)
{
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s CONFIG [PAYLOAD_FILE] [OUT_DIR]\n", argv[0]);
        return 2;
    }
    const std::string cfg = argv[1];
    const std::string out_dir = argc > 3 ? argv[3] : "data";
    FRAME_FORM tx_frame(cfg);
    FRAME_FORM rx_frame(cfg);
    MAC mac(1, 0, rx_frame.usefull_size);
    SDR tx_sdr(0, tx_frame.output_size, cfg);
    SDR rx_sdr(1, rx_frame.output_size, cfg);

    bit_vector origin(mac.payload);
    if (argc > 2) {
        if (FILE* f = std::fopen(argv[2], "rb")) {
            size_t got = std::fread(origin.data(), 1, origin.size(), f);
            (void)got;
            std::fclose(f);
        }
    } else {
        for (size_t i = 0; i < origin.size(); ++i) origin[i] = (uint8_t)(i * 37 + 11);
    }

    auto tx_mac_frame = mac.write(origin, 0);
    tx_frame.write(tx_mac_frame);
    auto tx_data = tx_frame.get_int16();
    tx_sdr.send(tx_data);
    tx_sdr.send(tx_data);
    rx_sdr.recv(rx_frame.from_sdr_int16_buf);
    rx_frame.form_int16_to_double();

    auto corr = rx_frame.t2sin.corr(rx_frame.from_sdr_buf);
    const int t2 = rx_frame.t2sin.find_t2sin(rx_frame.from_sdr_buf, 0);
    const int pr = rx_frame.preamble.find_preamble(rx_frame.from_sdr_buf, t2) + 1;
    if (t2 < 0 || pr < rx_frame.t2sin.size) {
        std::fprintf(stderr, "no frame found (t2 %d, preamble %d)\n", t2, pr);
        return 1;
    }
    std::copy(rx_frame.from_sdr_buf.begin() + pr - rx_frame.t2sin.size,
              rx_frame.from_sdr_buf.begin() + pr - rx_frame.t2sin.size + rx_frame.output_size, rx_frame.buf.begin());

    double cfo = rx_frame.preamble.pilot_freq_sinh();
    rx_frame.message_with_preamble.freq_shift(cfo);
    rx_frame.message_with_preamble.cp_freq_sinh();
    rx_frame.message_with_preamble.pr_phase_sinh(rx_frame.preamble.ofdm_preamble.data(), rx_frame.preamble.size);
    auto chan = rx_frame.preamble.chan_char_lq();
    auto constell = rx_frame.message.fft();
    for (size_t i = 0; i < constell.size(); ++i) constell[i] /= chan[i % chan.size()];

    mkdir(out_dir.c_str(), 0755);
    write_complex_to_file(out_dir + "/source.bin", tx_frame.int16_buf);
    write_complex_to_file(out_dir + "/data.bin", rx_frame.from_sdr_buf);
    write_double_to_file(out_dir + "/t2_sin_corr.bin", corr);
    write_complex_to_file(out_dir + "/phases.bin", chan);
    write_complex_to_file(out_dir + "/constell.bin", constell);

    auto bits = rx_frame.message.Mod.demod(constell);
    auto res = mac.read(bits);
    size_t byte_ok = 0, bit_ok = 0;
    for (size_t i = 0; i < res.size(); ++i) {
        byte_ok += res[i] == origin[i];
        for (int b = 0; b < 8; ++b) bit_ok += (((res[i] ^ origin[i]) >> b) & 1) == 0;
    }
    std::cout << "t2 " << t2 << " preamble " << pr << " cfo " << cfo << "\n";
    std::cout << "FRAME FROM " << mac.input_tx_id << " TO " << mac.input_rx_id << " SEQ " << mac.input_seq_num << "\n";
    std::cout << "ACCURACY: " << (double)byte_ok / res.size() << "\n";
    std::cout << "Bit-level ACCURACY: " << (double)bit_ok / (res.size() * 8) << "\n";
    return byte_ok == res.size() ? 0 : 1;
}
