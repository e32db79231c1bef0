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
typedef _Float16 halfx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short shortx4 __attribute__((ext_vector_type(4)));

// Operand precision of the reduced-precision step kernels (ldm_capi.h LDM_DT_*): fp32 operands rounded to
// nearest-even fp16 / bf16 in registers, one v_mfma_f32_16x16x16_{f16,bf16} per 16-deep K chunk (the
// 4 consecutive elements a lane holds are exactly that MFMA's per-lane operand), fp32 accumulation.
template <int DT>
__device__ __forceinline__ floatx16 mma32_lowp(floatx4 a, floatx4 b, floatx16 c) {
    if constexpr (DT == 1) {
        return __builtin_amdgcn_mfma_f32_32x32x8f16(__builtin_convertvector(a, halfx4), __builtin_convertvector(b, halfx4),
                                                    c, 0, 0, 0);
    } else {
        return __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(__builtin_bit_cast(shortx4, __builtin_convertvector(a, bf16x4)),
                                                        __builtin_bit_cast(shortx4, __builtin_convertvector(b, bf16x4)),
                                                        c, 0, 0, 0);
    }
}

template <int DT>
__device__ __forceinline__ floatx4 mma16_lowp(floatx4 a, floatx4 b, floatx4 c) {
    if constexpr (DT == 1) {
        return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_convertvector(a, halfx4), __builtin_convertvector(b, halfx4),
                                                     c, 0, 0, 0);
    } else {
        return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(shortx4, __builtin_convertvector(a, bf16x4)),
                                                         __builtin_bit_cast(shortx4, __builtin_convertvector(b, bf16x4)),
                                                         c, 0, 0, 0);
    }
}

// the same with A already rounded to 16 bits (a packed weight fragment, 4 x f16 / bf16 bit patterns)
template <int DT>
__device__ __forceinline__ floatx4 mma16_lowp(shortx4 a16, floatx4 b, floatx4 c) {
    if constexpr (DT == 1) {
        return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(halfx4, a16), __builtin_convertvector(b, halfx4),
                                                     c, 0, 0, 0);
    } else {
        return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a16, __builtin_bit_cast(shortx4, __builtin_convertvector(b, bf16x4)),
                                                         c, 0, 0, 0);
    }
}

// Division of a non-negative int < 2^31 by a runtime constant with one mul_hi + shift (Granlund-
// Montgomery, round-up multiplier): the GPU's integer division is a ~30-instruction VALU sequence.
// Pin a wave-uniform value to an SGPR (a buffer soffset / resource the compiler leaves in a VGPR is
// legalised with a waterfall loop around every load).
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ void* uni_ptr(const void* p) {
    const uint64_t u = (uint64_t)p;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32));
    return (void*)(((uint64_t)hi << 32) | lo);
}

// n / d for 0 <= n < 2^31 by multiply-high and shift; branch-free (d == 1 folds in through `one`,
// so the quotient is umulhi(n, 0) + n) — a data-independent select costs a branch at one wave/SIMD.
struct FastDiv {
    int32_t d;
    uint32_t mul, shr, one;
    static FastDiv make(int32_t dv) {
        FastDiv f{dv, 0u, 0u, 0xffffffffu};
        if (dv > 1) {
            uint32_t l = 0;
            while ((1u << l) < (uint32_t)dv) ++l;   // ceil(log2 d)
            const uint32_t p = 31 + l;
            f.mul = (uint32_t)(((1ull << p) + (uint32_t)dv - 1) / (uint32_t)dv);
            f.shr = p - 32;
            f.one = 0u;
        }
        return f;
    }
    __device__ __forceinline__ int div(int n) const {
        return (int)((__umulhi((uint32_t)n, mul) >> shr) + ((uint32_t)n & one));
    }
};

constexpr int kMaxPhase = 4;
constexpr int kMaxTap = 16;   // 4x4 windows: the decoder's k4 convT and its k4 s2 data-gradient conv

// Sub-pixel phase decomposition of a (transposed) convolution, see conv.hip.
struct PhaseTable {
    int32_t nphase;
    int32_t Hq, Wq;   // phase output grid
    int32_t sy;       // input step per q (conv: stride, convT: 1)
    int32_t osy;      // output step per q (conv: 1, convT: 2)
    int32_t ry[kMaxPhase], rx[kMaxPhase];
    int32_t ntap[kMaxPhase];
    // int32 (not int8): the kernels index these with a wave-uniform tap, which must compile to a
    // scalar s_load_dword from the kernarg segment; byte fields force per-lane global loads.
    int32_t dy[kMaxPhase][kMaxTap], dx[kMaxPhase][kMaxTap];
    int32_t kk[kMaxPhase][kMaxTap];   // kernel-window index kh*KW+kw of the tap
    int64_t wofs[kMaxPhase];         // packed-weight offset (floats) of each phase
    int32_t kchunks[kMaxPhase];      // K chunks of each phase
};

int build_phase_table(const ldm_conv_desc& d, PhaseTable& pt);

// One weight re-pack of a multi-tensor pack launch (pack.hip): the packed layout of a conv.hip MFMA plan
// (kind 1 / 2: fp32, CK = 8 / 16 channels per fragment) or of a tconv.hip plan (kind 3: 16-bit, 32-channel
// chunks), read from the torch-layout weight w.
struct PackJob {   // one weight of a multi-tensor re-pack (pack.hip); filled by conv_pack_job / tconv_pack_job
    const float* w;
    void* out;
    int64_t first_block, total;   // this job's first block of the launch; its element count (< 2^31)
    int32_t kind, dt, Cin, Cout, KK, transposed, Mpad, nphase;
    int32_t ntap[kMaxPhase];
    int64_t wofs[kMaxPhase];
    int32_t kk[kMaxPhase][kMaxTap];
    FastDiv fd_mpad, fd_cin, fd_ntap[kMaxPhase];
    FastDiv fd_kr;                 // kinds 1/2 with remap: 8-element runs per packed row (K / 8)
    int32_t remap;
};
int conv_pack_job(const ldm_conv_desc& d, const ldm_conv_plan& p, PackJob& j);    // kinds 1, 2 (conv.hip)
int tconv_pack_job(const ldm_conv_desc& d, const ldm_conv_plan& p, PackJob& j);   // kind 3 (tconv.hip)

// tconv.hip: the LDS-staged 16-bit-operand implicit GEMM (plan kind 3) for large-plane NCHW layers
struct EpiArgs;
bool tconv_plan(const ldm_conv_desc& d, int dtype, ldm_conv_plan& plan);
int tconv_pack(const ldm_conv_desc& d, const ldm_conv_plan& p, const float* w, float* packed, hipStream_t st);
int tconv_forward(const ldm_conv_desc& d, const ldm_conv_plan& p, const float* x, const float* w, const EpiArgs& ep,
                  float* y, hipStream_t st);
// plan kind 4 (sconv.hip): small-plane 16-bit-operand implicit GEMM, packed like kind 3 (tm = 1)
bool sconv_plan(const ldm_conv_desc& d, int dtype, ldm_conv_plan& plan);
int sconv_forward(const ldm_conv_desc& d, const ldm_conv_plan& p, const float* x, const float* w, const EpiArgs& ep,
                  float* y, hipStream_t st);

// Device-side epilogue parameters (by value in kernel args).
struct EpiArgs {
    const float* bias;
    const float* bn_w;
    const float* bn_b;
    const float* bn_m;
    const float* bn_v;
    float bn_eps;
    int32_t act;
    const float* pos_bias;   // [Cout, Hout, Wout] added in place of `bias` (a projection folded into the
                             // conv, whose bias reaches each output through the taps inside the window)
    const float* bcast;
    const float* skip;
    float* act_out;   // post-activation value before the adds (training), or NULL
    // fused DDIM reverse update (model.py:442-458) on the conv output eps = noise_pred:
    // x <- sqrt(ab_n)*x0 + sqrt(1-ab_n)*eps + eta*(...) in place, with pred_x0 / noise_pred logs.
    const float* ddim_coef;   // [4] {sqrt(ab_t), sqrt(1-ab_t), sqrt(ab_n), sqrt(1-ab_n)} or NULL
    float ddim_eta;
    float* ddim_x;
    float* ddim_x0_log;
    float* ddim_eps_log;
    int32_t lowp;   // operand precision LDM_DT_* (MFMA kernels; the VALU conv kernels round their operands too)
    // LDM_DT_F16 / LDM_DT_BF16: round the conv output, the eval-BN output, the activation and each add to that
    // type, as ATen's autocast does (its conv / linear outputs are 16-bit tensors); 0: fp32 outputs
    int32_t round_out;
    // 16-bit storage (LDM_DT_X16 / LDM_DT_Y16, in the lowp type): the input x, and the output y with act_out
    int32_t x16, y16;
};

// conv.hip: implicit-GEMM conv with the full internal epilogue (incl. the fused DDIM update); y may be
// NULL when ep.ddim_coef is set; ws: p.ws_floats floats (split-K counters + partials) or NULL.
int conv_forward_ex(const ldm_conv_desc& d, const ldm_conv_plan& p, const float* x, const float* w, const EpiArgs& ep,
                    float* y, float* ws, hipStream_t st);

// misc.hip: cross-attention core; tok = q / out token-major [B,L,E] (else channel-major [B,E,L]);
// kv is always channel-major [B,2E,S].
int attention_core_ex(const float* q, const float* kv, float* out, int32_t B, int32_t E, int32_t heads, int32_t L,
                      int32_t S, float scale, bool tok, hipStream_t st);

// flash.hip: KV-tiled online-softmax attention for any L, S (head dim 64 or 128); lse [B,heads,L] (channel-major
// q only) or NULL
bool attention_flash_supported(int E, int heads);
int attention_flash(const float* q, const float* kv, float* out, float* lse, int32_t B, int32_t E, int32_t heads,
                    int32_t L, int32_t S, float scale, bool tok, hipStream_t st);

int attention_folded(const float* z, const float* kv, const float* kf, const float* bf, float* out, int32_t B,
                     int32_t E, int32_t heads, int32_t L, int32_t S, hipStream_t st);
int attention_fold_keys(const float* kv, const float* wq, const float* bq, int32_t B, int32_t E, int32_t heads,
                        int32_t S, float scale, float* kf, float* bf, hipStream_t st);
int attention_folded_probs(const float* z, const float* kf, const float* bf, float* p, int32_t B, int32_t E,
                           int32_t heads, int32_t L, int32_t S, hipStream_t st);
// bfold.hip: the reverse loop's bottleneck with CA1's values folded into its weights (U, once per loop)
bool bneck_fold_supported(int B, int H, int W);
int bneck_fold_values(const float* wf, const float* kv, float* u, int B, hipStream_t st);
int bneck_pv(const float* u, const float* p, const float* pb, float* y, int B, int dtype, hipStream_t st);

// uconv.hip: the step kernels of the reverse loop (NHWC activations, see ldm_capi.h)
struct StepConv {
    const float* x;
    const float* w;
    float* y;
    const float* bias;    // [Cout] or, for enc4 / bottleneck, the folded position bias [Hout*Wout][Cout]
    const float* bcast;   // enc2: t_emb [B][128]
    const float* skip;    // dec4..dec2
    const float* coef;    // dec1: DDIM coefficients of the step
    float eta;
    float* xs;            // dec1: sampler state (NHWC), updated in place
    float* x0_log;        // dec1: NCHW logs (or NULL)
    float* eps_log;
    int dtype;            // operand precision: LDM_DT_F32 / LDM_DT_F16 / LDM_DT_BF16 (uconv.hip)
    float* ws;            // split-K workspace (step_ws_floats; zero-filled once) for the K-split layers
};
int step_conv(int layer, int B, int H, int W, const StepConv& s, hipStream_t st);
int64_t step_ws_floats(int B, int H, int W, int64_t* cnt_floats = nullptr);
int step_ks_mask();   // layers running the K-split step form (LDM_UCONV_KS)
// LDM_DEBUG_BOUNDS (make DIAG=1: the diagnostic library lib/libldm_amd_diag.so): the multi-tensor optimizer kernels check the chunk map they
// index the slot table with (chunk_tensor[i] in [0, nchunks), chunk_start >= 0, a non-null gradient) and print
// and skip a bad chunk instead of dereferencing it (round 5's aperture violation in unscale_check_kernel read
// a slot table that the graph's own scratch had overwritten)
#ifndef LDM_DEBUG_BOUNDS
#define LDM_DEBUG_BOUNDS 0
#endif
int step_layout(const float* x, float* y, int B, int C, int HW, bool to_nhwc, hipStream_t st);

// wgrad.hip: the tap-shared weight-gradient kernel (ldm_conv_backward_weight where it applies)
bool wgrad2_plan_ws(const ldm_conv_desc& d, int64_t& ws_floats);
int wgrad2_run(const ldm_conv_desc& d, const float* dense, const float* gath, float* partial, int& splits, int dtype,
               hipStream_t st, int st16 = 0, float* dw_direct = nullptr);   // splits = 0: written to dw_direct
int wgrad2_storage16(const ldm_conv_desc& d);

// One DDIM step for one element, one fp32 rounding per reference op (no contraction: callers compile
// with fp contract off).  Returns x_next; x0 out.
__device__ __forceinline__ float ddim_update(float xv, float e, const float* coef, float eta, float& x0) {
#pragma clang fp contract(off)
    const float sat = coef[0], s1t = coef[1], san = coef[2], s1n = coef[3];
    const float dxt = s1t * e;            // sqrt(1-ab_t) * noise_pred (also inside predict_start)
    x0 = (xv - dxt) / sat;                // predict_start_from_noise
    const float dxn = s1n * e;            // direction_xt_next
    const float nc = eta * (dxn - dxt);   // noise_contribution
    const float t1 = san * x0;
    return (t1 + dxn) + nc;
}

// v rounded to a 16-bit type (LDM_DT_F16 / LDM_DT_BF16, round to nearest even), or unchanged (0)
__device__ __forceinline__ float round16(float v, int mode) {
    if (mode == LDM_DT_F16) return (float)(_Float16)v;
    if (mode == LDM_DT_BF16) return (float)(__bf16)v;
    return v;
}

// ---- 16-bit activation storage (the train step's large maps inside an autocast region: ATen stores them as
// fp16 / bf16 tensors).  ST = the 16-bit type (LDM_DT_F16 / LDM_DT_BF16); a tensor is read / written in it
// when its flag `h` is set, else as fp32.  Stores convert round-to-nearest-even (a value already rounded to the
// type, as the autocast output semantics leave it, is stored exactly).
template <int ST>
__device__ __forceinline__ float from16(unsigned short u) {
    if constexpr (ST == LDM_DT_F16) return (float)__builtin_bit_cast(_Float16, u);
    else return __builtin_bit_cast(float, (unsigned)u << 16);
}
template <int ST>
__device__ __forceinline__ unsigned short to16s(float v) {
    if constexpr (ST == LDM_DT_F16) return __builtin_bit_cast(unsigned short, (_Float16)v);
    else return __builtin_bit_cast(unsigned short, (__bf16)v);
}
// W consecutive values at element offset o of p (fp32, or 16-bit when ST != 0 and h)
template <int ST, int W>
__device__ __forceinline__ void ld_st(const void* p, size_t o, bool h, float (&v)[W]) {
    if (ST != 0 && h) {
        const unsigned short* q = reinterpret_cast<const unsigned short*>(p) + o;
        if constexpr (W == 8) {   // one 16-byte load
            const uint4 t = *reinterpret_cast<const uint4*>(q);
            const unsigned u[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
            for (int j = 0; j < 4; ++j)
                v[2 * j] = from16<ST>((unsigned short)(u[j] & 0xffff)), v[2 * j + 1] = from16<ST>((unsigned short)(u[j] >> 16));
        } else if constexpr (W == 4) {
            const uint2 t = *reinterpret_cast<const uint2*>(q);
            v[0] = from16<ST>((unsigned short)(t.x & 0xffff)), v[1] = from16<ST>((unsigned short)(t.x >> 16));
            v[2] = from16<ST>((unsigned short)(t.y & 0xffff)), v[3] = from16<ST>((unsigned short)(t.y >> 16));
        } else {
#pragma unroll
            for (int j = 0; j < W; ++j) v[j] = from16<ST>(q[j]);
        }
    } else {
        const float* q = reinterpret_cast<const float*>(p) + o;
        if constexpr (W % 4 == 0) {
#pragma unroll
            for (int j = 0; j < W; j += 4) {
                const float4 t = *reinterpret_cast<const float4*>(q + j);
                v[j] = t.x, v[j + 1] = t.y, v[j + 2] = t.z, v[j + 3] = t.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < W; ++j) v[j] = q[j];
        }
    }
}
// The same load split in two, for loops that keep several pieces in flight: ld_raw issues the load(s) of W
// consecutive values into raw registers (16-bit: W / 2 words; fp32: W words), cvt_raw converts them once the
// values are used.  Same values as ld_st.
template <int W>
struct RawW {
    float v[W];
};
template <int ST, int W>
__device__ __forceinline__ void ld_raw(const void* p, size_t o, bool h, RawW<W>& r) {
    if (ST != 0 && h) {
        const unsigned short* q = reinterpret_cast<const unsigned short*>(p) + o;
        if constexpr (W == 8) {
            const uint4 t = *reinterpret_cast<const uint4*>(q);
            r.v[0] = __builtin_bit_cast(float, t.x), r.v[1] = __builtin_bit_cast(float, t.y);
            r.v[2] = __builtin_bit_cast(float, t.z), r.v[3] = __builtin_bit_cast(float, t.w);
        } else if constexpr (W == 4) {
            const uint2 t = *reinterpret_cast<const uint2*>(q);
            r.v[0] = __builtin_bit_cast(float, t.x), r.v[1] = __builtin_bit_cast(float, t.y);
        } else {
#pragma unroll
            for (int j = 0; j < W; ++j) r.v[j] = __builtin_bit_cast(float, (unsigned)q[j]);
        }
    } else {
        float t[W];
        ld_st<0, W>(p, o, false, t);
#pragma unroll
        for (int j = 0; j < W; ++j) r.v[j] = t[j];
    }
}
template <int ST, int W>
__device__ __forceinline__ void cvt_raw(const RawW<W>& r, bool h, float (&v)[W]) {
    if (ST != 0 && h) {
        if constexpr (W == 8 || W == 4) {
#pragma unroll
            for (int j = 0; j < W / 2; ++j) {
                const unsigned u = __builtin_bit_cast(unsigned, r.v[j]);
                v[2 * j] = from16<ST>((unsigned short)(u & 0xffff)), v[2 * j + 1] = from16<ST>((unsigned short)(u >> 16));
            }
        } else {
#pragma unroll
            for (int j = 0; j < W; ++j) v[j] = from16<ST>((unsigned short)__builtin_bit_cast(unsigned, r.v[j]));
        }
    } else {
#pragma unroll
        for (int j = 0; j < W; ++j) v[j] = r.v[j];
    }
}
template <int ST, int W>
__device__ __forceinline__ void st_st(void* p, size_t o, bool h, const float (&v)[W]) {
    if (ST != 0 && h) {
        unsigned short* q = reinterpret_cast<unsigned short*>(p) + o;
        if constexpr (W == 8) {   // one 16-byte store
            unsigned u[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                u[j] = (unsigned)to16s<ST>(v[2 * j]) | ((unsigned)to16s<ST>(v[2 * j + 1]) << 16);
            *reinterpret_cast<uint4*>(q) = make_uint4(u[0], u[1], u[2], u[3]);
        } else if constexpr (W == 4) {
            uint2 t;
            t.x = (unsigned)to16s<ST>(v[0]) | ((unsigned)to16s<ST>(v[1]) << 16);
            t.y = (unsigned)to16s<ST>(v[2]) | ((unsigned)to16s<ST>(v[3]) << 16);
            *reinterpret_cast<uint2*>(q) = t;
        } else {
#pragma unroll
            for (int j = 0; j < W; ++j) q[j] = to16s<ST>(v[j]);
        }
    } else {
        float* q = reinterpret_cast<float*>(p) + o;
        if constexpr (W % 4 == 0) {
#pragma unroll
            for (int j = 0; j < W; j += 4)
                *reinterpret_cast<float4*>(q + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
        } else {
#pragma unroll
            for (int j = 0; j < W; ++j) q[j] = v[j];
        }
    }
}
template <int ST>
__device__ __forceinline__ float ld1_st(const void* p, size_t o, bool h) {
    if (ST != 0 && h) return from16<ST>(reinterpret_cast<const unsigned short*>(p)[o]);
    return reinterpret_cast<const float*>(p)[o];
}
template <int ST>
__device__ __forceinline__ void st1_st(void* p, size_t o, bool h, float v) {
    if (ST != 0 && h) reinterpret_cast<unsigned short*>(p)[o] = to16s<ST>(v);
    else reinterpret_cast<float*>(p)[o] = v;
}

__device__ __forceinline__ float apply_act(float v, int act) {
#pragma clang fp contract(off)
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
