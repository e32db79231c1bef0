// Shared internals of libldm_amd (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "ldm_capi.h"

namespace ldm {

// thread-local last error (ldm_last_error)
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define LDM_HIP_TRY(expr)                                                                      \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess)                                                                  \
            return ::ldm::fail(1000 + (int)_e, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

#define LDM_CHECK_LAUNCH(name)                                                                 \
    do {                                                                                       \
        hipError_t _e = hipGetLastError();                                                     \
        if (_e != hipSuccess)                                                                  \
            return ::ldm::fail(1000 + (int)_e, std::string("launch ") + name + ": " + hipGetErrorString(_e)); \
    } while (0)

#define LDM_REQUIRE(cond, msg)                                                                 \
    do {                                                                                       \
        if (!(cond)) return ::ldm::fail(2, std::string(msg));                                  \
    } while (0)

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kMaxPhase = 4;
constexpr int kMaxTap = 9;

// Sub-pixel phase decomposition of a (transposed) convolution, see conv.hip.
struct PhaseTable {
    int32_t nphase;
    int32_t Hq, Wq;   // phase output grid
    int32_t sy;       // input step per q (conv: stride, convT: 1)
    int32_t osy;      // output step per q (conv: 1, convT: 2)
    int32_t ry[kMaxPhase], rx[kMaxPhase];
    int32_t ntap[kMaxPhase];
    int8_t dy[kMaxPhase][kMaxTap], dx[kMaxPhase][kMaxTap];
    int8_t kk[kMaxPhase][kMaxTap];   // kernel-window index kh*KW+kw of the tap
    int64_t wofs[kMaxPhase];         // packed-weight offset (floats) of each phase
    int32_t kchunks[kMaxPhase];      // K chunks of each phase
};

int build_phase_table(const ldm_conv_desc& d, PhaseTable& pt);

// Device-side epilogue parameters (by value in kernel args).
struct EpiArgs {
    const float* bias;
    const float* bn_w;
    const float* bn_b;
    const float* bn_m;
    const float* bn_v;
    float bn_eps;
    int32_t act;
    const float* bcast;
    const float* skip;
};

__device__ __forceinline__ float apply_act(float v, int act) {
    if (act == LDM_ACT_RELU) return v < 0.f ? 0.f : v;   // F.relu; NaN propagates like torch
    if (act == LDM_ACT_TANH) return tanhf(v);
    if (act == LDM_ACT_TANH_HALF) {
        float th = tanhf(v);
        float s = th + 1.0f;
        return s / 2.0f;
    }
    if (act == LDM_ACT_GELU) return v * 0.5f * (1.0f + erff(v * 0.70710678118654752440f));
    return v;
}

}  // namespace ldm
