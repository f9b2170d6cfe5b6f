// ofdm_compat.hpp — shared plumbing of the C++ compatibility layer: one
// cached ofdm_ctx per parameter set (device from $OFDM_DEVICE, default 0),
// grow-on-demand device staging buffers, synchronous host<->device copies.
// The compat classes are a drop-in for the reference's single-frame, host
// std::vector API; the batched device-pointer C-ABI is the fast path.
#pragma once
#include <cstddef>
#include <memory>
#include <string>
#include <vector>

#include <ofdm_mi355x.h>
#include "config/parser.hpp"

namespace ofdm_compat {

void check(int rc, const char* what);  // throws std::runtime_error(ofdm_last_error())

struct Context {
    ofdm_ctx* ctx = nullptr;
    ofdm_params params{};
    ofdm_geometry geo{};
    explicit Context(const ofdm_params& p);
    ~Context();
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    void* buf(int slot, size_t bytes);  // device scratch, slot-indexed
    void h2d(void* dev, const void* host, size_t bytes);
    void d2h(void* host, const void* dev, size_t bytes);
    void sync();

private:
    std::vector<std::pair<void*, size_t>> slots_;
};

std::shared_ptr<Context> context_for(const ofdm_params& p);
ofdm_params params_from(ConfigMap& config);
ofdm_params params_default();

}  // namespace ofdm_compat
