// mac/mac_frame.hpp — recreation of the reference's missing MAC header (the
// tree includes "mac/mac_frame.hpp" from main.cpp:18, tx.cpp:16, rx.cpp:17 but
// does not ship it). Layout from the DWARF of the reference's build/main.o
// (class MAC, decl lines 7-61): uint16 tx_id, rx_id, seq_num, cs; input_*
// copies parsed on read; const size_t header_len; size_t frame_len, payload;
// bit_vector mes; MAC(uint32_t, uint32_t, size_t), calc_cs(), write(bit_vector,
// size_t) -> bit_vector&, read(bit_vector) -> bit_vector. Wire format: 8-byte
// little-endian header {tx_id, rx_id, seq_num, cs} + payload; cs = sum of the
// bytes of (header with cs = 0) ++ payload, mod 2^16 (0x577E on the golden
// frame, data/source.bin). Host framing: not part of the GPU modem.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

class MAC {
public:
    uint16_t tx_id;
    uint16_t rx_id;
    uint16_t seq_num;
    uint16_t cs;
    uint16_t input_tx_id = 0;
    uint16_t input_rx_id = 0;
    uint16_t input_seq_num = 0;
    uint16_t input_cs = 0;
    const size_t header_len = 8;
    size_t frame_len;
    size_t payload;
    std::vector<uint8_t> mes;

    MAC(uint32_t tx, uint32_t rx, size_t frame_len)
        : tx_id((uint16_t)tx), rx_id((uint16_t)rx), seq_num(0), cs(0), frame_len(frame_len),
          payload(frame_len > 8 ? frame_len - 8 : 0), mes(frame_len, 0)
    {
    }

    void calc_cs()
    {
        unsigned sum = 0;
        for (size_t i = 0; i < mes.size(); ++i)
            if (i != 6 && i != 7) sum += mes[i];
        cs = (uint16_t)sum;
        if (mes.size() >= 8) {
            mes[6] = (uint8_t)(cs & 0xff);
            mes[7] = (uint8_t)(cs >> 8);
        }
    }

    std::vector<uint8_t>& write(std::vector<uint8_t> input, size_t seq)
    {
        seq_num = (uint16_t)seq;
        std::fill(mes.begin(), mes.end(), 0);
        const uint16_t h[4] = {tx_id, rx_id, seq_num, 0};
        for (int i = 0; i < 4 && 2 * i + 1 < (int)mes.size(); ++i) {
            mes[2 * i] = (uint8_t)(h[i] & 0xff);
            mes[2 * i + 1] = (uint8_t)(h[i] >> 8);
        }
        for (size_t i = 0; i < payload && i < input.size(); ++i) mes[header_len + i] = input[i];
        calc_cs();
        return mes;
    }

    std::vector<uint8_t> read(std::vector<uint8_t> input)
    {
        auto u16 = [&](size_t i) { return (uint16_t)(i + 1 < input.size() ? input[i] | (input[i + 1] << 8) : 0); };
        input_tx_id = u16(0);
        input_rx_id = u16(2);
        input_seq_num = u16(4);
        input_cs = u16(6);
        std::vector<uint8_t> out(payload, 0);
        for (size_t i = 0; i < payload && header_len + i < input.size(); ++i) out[i] = input[header_len + i];
        return out;
    }
};
