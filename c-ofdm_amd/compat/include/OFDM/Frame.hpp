// OFDM/Frame.hpp — drop-in for the reference's OFDM/Frame.hpp class surface
// (FFT_FORM, T2SIN_FORM, OFDM_FORM, PREAMBLE_FORM, FRAME_FORM).
// Same class/member names, buffer ownership and in-place semantics, so
// main.cpp / tx.cpp / rx.cpp build unchanged; every DSP member runs on the GPU
// through the C-ABI of include/ofdm_mi355x.h. A FRAME_FORM keeps device
// images of its buffers (ofdm_compat::Mirror): the forms' members move only
// what the host changed and copy back what they change in place; the batched
// device-pointer C-ABI is the throughput path.
#pragma once
#include <math.h>
#include <stdlib.h>

#include <algorithm>
#include <complex>
#include <cstring>
#include <fstream>
#include <memory>
#include <optional>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "config/parser.hpp"
#include "OFDM/modulation.hpp"

const complex_double REAL_ONE(1.0, 0.0);

namespace ofdm_compat {
struct Context;
struct FrameMirrors;
}

class FFT_FORM {
public:
    int fft_size;
    int num_data_subc;
    int num_pilot_subc;
    int num_symb;
    int segment_step;
    int segment_size;
    int segment_byte_size;

    complex_vector FFT_buf;
    std::vector<complex_double*> segment;  // data segment starts inside FFT_buf
    std::vector<complex_double*> pilot;    // pilot bins inside FFT_buf

    complex_vector restored_buf;
    double norm_factor;
    double pilot_ampl;

    FFT_FORM(int fft_size, int num_data_subc, int num_pilot_subc, int num_symb, double pilot_ampl = 1.0);
    ~FFT_FORM();
    void write(complex_vector& input);   // FFT_buf <- IFFT(pilots + segments)/sqrt(N)   (Frame.cpp:54-70)
    complex_vector& read();              // restored_buf <- equalised FFT_buf           (Frame.cpp:73-96)

    std::shared_ptr<ofdm_compat::Context> ctx_;
};

class T2SIN_FORM {
private:
    ConfigMap& config;

public:
    int size;
    int f1;
    int f2;
    int smooth;
    double level;
    std::vector<double> detect_mask;
    complex_vector detect_buf;
    int mean_freq;
    int min_f1;
    int max_f1;
    int min_f2;
    int max_f2;
    int real_f1 = 0;
    int real_f2 = 0;
    int real_f1_ampl = 0;
    int real_f2_ampl = 0;
    double freq_shift = 0;
    complex_double* buf = nullptr;

    T2SIN_FORM(ConfigMap& config);
    void set(complex_double* buf_ptr);
    std::vector<double> corr(complex_vector& signal);           // Frame.hpp:96-147
    int find_t2sin(complex_vector& signal, int start_index);    // Frame.hpp:150-197

    std::shared_ptr<ofdm_compat::Context> ctx_;
};

class OFDM_FORM {
private:
    ConfigMap& config;

public:
    bool data;
    int fft_size;
    int num_data_subc;
    int num_pilot_subc;
    int cp_size;
    int num_symb;
    int pr_sin_len;
    int pr_seed;
    mod_type modType;
    int ofdm_len;
    int size;
    int usefull_size;
    std::vector<complex_double*> output;  // views into the owner's frame buffer
    FFT_FORM fft_task;
    Modulation Mod;
    int byte_fft_size;
    int pilot_ampl;

    OFDM_FORM(ConfigMap& config, bool data = true, bool with_preamble = false);
    virtual ~OFDM_FORM() = default;
    virtual void set(complex_double* buf_ptr);
    void write(bit_vector& input);                               // Frame.cpp:185-198
    bit_vector read();                                           // Frame.cpp:201-208
    void cp_freq_sinh();                                         // Frame.hpp:238-263
    void pr_phase_sinh(complex_double* pr, int pr_size);         // Frame.hpp:265-274
    complex_vector fft();                                        // Frame.hpp:276-282
    double pilot_freq_sinh();                                    // Frame.hpp:285-337
    void freq_shift(double& shift);                              // Frame.hpp:340-348

    std::shared_ptr<ofdm_compat::Context> ctx_;
};

class PREAMBLE_FORM : public OFDM_FORM {
public:
    double level;
    bit_vector preamble;
    complex_vector mod_preamble;
    complex_vector ofdm_preamble;
    complex_vector conjected_sinh_part;
    std::vector<double> cor;
    complex_vector chan_est;

    PREAMBLE_FORM(ConfigMap& config);
    void set(complex_double* buf_ptr) override;                  // Frame.cpp:276-294
    void find_corr(complex_vector& input, int start);            // Frame.cpp:297-335
    int find_preamble(complex_vector& input, int start);         // Frame.cpp:338-378
    complex_vector chan_char();                                  // Frame.hpp:375-385
    complex_vector& chan_char_lq();                              // Frame.hpp:389-434
};

class FRAME_FORM {
public:
    ConfigMap config;
    T2SIN_FORM t2sin;
    PREAMBLE_FORM preamble;
    OFDM_FORM message;
    OFDM_FORM message_with_preamble;

    complex_vector buf;
    complex16_vector int16_buf;
    complex_vector from_sdr_buf;
    complex16_vector from_sdr_int16_buf;

    int usefull_size;
    int output_size;
    bit_vector bit_preambple;

    FRAME_FORM(const std::string& CONFIGNAME);                   // Frame.cpp:213-232
    void write(bit_vector& input);                               // Frame.cpp:235-237
    bit_vector read(void* transmitted_data);                     // Frame.cpp:239-242
    complex_vector get();                                        // Frame.cpp:244-246
    complex16_vector get_int16();                                // Frame.cpp:249-256
    void form_int16_to_double();                                 // Frame.hpp:472-481

    std::shared_ptr<ofdm_compat::FrameMirrors> mirrors_;  // device images of buf / from_sdr_buf / from_sdr_int16_buf
};
