// Per-channel reductions of the train path, sliced for the whole chip:
//   * train-mode BatchNorm2d forward (batch stats -> normalise + act + running stats),
//   * its backward (sum g, sum g*xhat -> dx),
//   * the fused-epilogue activation backward (dv, dbias[c], dbcast[b,c]).
// Reference semantics: nn.BatchNorm2d / the conv epilogues of model.py:10-49 (VAE) and
// model.py:163-231 (UNet) under .train(); the backward follows torch's native_batch_norm_backward.
//
// Layout: NCHW fp32.  A channel's B*HW elements are cut into P contiguous slices of the flattened
// (b, hw) index (slice length a multiple of 4, float4 loads when HW % 4 == 0), one 256-thread block
// per (slice, channel), so a C=64..128 layer launches >= 1024 blocks instead of C.  Every reduction
// has a fixed partition and a fixed order (thread stride -> wave shuffle tree -> waves in order ->
// slices in order), so results are bitwise reproducible run to run.  BatchNorm statistics are fp64
// (sum x, sum x^2) so the per-rank sums can be all-reduced for SyncBatchNorm between the two stages
// (ldm_batchnorm_stats -> all-reduce -> ldm_batchnorm_apply; likewise the backward).
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace ldm {
namespace {

constexpr int kThreads = 256;

// blocks a BatchNorm pass aims for (LDM_BN_BLOCKS, default 2048: 8 blocks of 256 threads per CU, so 32 waves
// keep enough 16-byte loads in flight; 1024 left the normalise / backward passes at 2.4-3.5 TB/s)
inline int64_t bn_blocks() {
    static const int64_t v = [] {
        const char* e = getenv("LDM_BN_BLOCKS");
        const long x = e ? atol(e) : 2048;
        return (int64_t)(x >= 256 && x <= 16384 ? x : 2048);
    }();
    return v;
}

// slices per channel for a reduction over n = B*HW elements across C channels
inline int bn_slices(int64_t n, int C) {
    int64_t p = (bn_blocks() + C - 1) / C;          // >= bn_blocks() blocks in total
    const int64_t by_len = (n + 2047) / 2048;       // but >= ~2048 elements per slice
    if (p > by_len) p = by_len;
    if (p < 1) p = 1;
    if (p > 256) p = 256;
    return (int)p;
}
// slice length: a multiple of the access width W (4 or 8 elements; 4 for the scalar form, as before)
inline int64_t slice_len(int64_t n, int P, int W = 4) {
    const int64_t a = W > 4 ? W : 4;
    return ((n + P - 1) / P + a - 1) / a * a;
}

// slices per (b,c) plane for the activation backward
inline int act_slices(int B, int C, int HW) {
    int64_t q = (2048 + (int64_t)B * C - 1) / ((int64_t)B * C);
    const int64_t by_len = (HW + 1023) / 1024;
    if (q > by_len) q = by_len;
    if (q < 1) q = 1;
    return (int)q;
}

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    T s = 0;
    for (int w = 0; w < kThreads / 64; ++w) s += red[w];
    return s;
}

__device__ __forceinline__ float act_grad(int act, float a) {
    switch (act) {
        case LDM_ACT_RELU: return a > 0.f ? 1.f : 0.f;
        case LDM_ACT_TANH: return 1.f - a * a;
        case LDM_ACT_TANH_HALF: {   // a = (tanh(v)+1)/2 -> da/dv = (1 - tanh^2)/2
            const float th = 2.f * a - 1.f;
            return 0.5f * (1.f - th * th);
        }
        default: return 1.f;
    }
}

template <int W>
__device__ __forceinline__ void ld(const float* p, float (&v)[W]) {
    ld_st<0, W>(p, 0, false, v);
}

// Visit channel c's elements with flattened (b, hw) index in [e0, e1): f(offset) for W consecutive
// elements of one plane.  Plane-by-plane, so no per-element division.
template <int W, class F>
__device__ __forceinline__ void slice_for(int64_t e0, int64_t e1, int C, int c, int HW, F&& f) {
    if (e0 >= e1) return;
    int b = (int)(e0 / HW);
    int p = (int)(e0 - (int64_t)b * HW);
    int64_t e = e0;
    while (e < e1) {
        const int64_t left = e1 - e;
        const int n = (int)((int64_t)(HW - p) < left ? (int64_t)(HW - p) : left);
        const size_t base = ((size_t)b * C + c) * HW + p;
        for (int i = threadIdx.x * W; i < n; i += kThreads * W) f(base + i);
        e += n;
        ++b;
        p = 0;
    }
}

// HM: how a BatchNorm kernel instance reads its tensors' storage flags.  0: at run time, per tensor (a mixed call);
// 1: every tensor of the call 16-bit; 2: every tensor fp32.  With 1 / 2 the flag is a constant, so the load / store
// paths carry no branch: a branch around a load makes the compiler drain vmcnt at the join, which serialises the
// pieces slice_for_u keeps in flight (measured: 2-3.5x slower sweeps with run-time flags and U = 2).
template <int HM>
__device__ __forceinline__ bool st_flag(int sf, int bit) {
    if constexpr (HM == 0) return (sf & bit) != 0;
    else return HM == 1;
}

// slice_for with U pieces of a thread in flight at once: within a plane, the loads of U consecutive pieces
// (ldf(offset, u)) are issued before the first is used (usef(offset, u), in offset order), so a wave keeps U
// 16-byte loads outstanding instead of one (a sweep at one load per wave ran at 3.4-4.3 TB/s).  The pieces a
// thread visits and the order it uses them in are slice_for's: every sum keeps its bits.
template <int N, class F, int I = 0>
__device__ __forceinline__ void unroll_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        unroll_for<N, F, I + 1>(static_cast<F&&>(f));
    }
}
template <int W, int U, class L, class F>
__device__ __forceinline__ void slice_for_u(int64_t e0, int64_t e1, int C, int c, int HW, L&& ldf, F&& usef) {
    if (e0 >= e1) return;
    constexpr int STEP = kThreads * W;
    int b = (int)(e0 / HW);
    int p = (int)(e0 - (int64_t)b * HW);
    int64_t e = e0;
    while (e < e1) {
        const int64_t left = e1 - e;
        const int n = (int)((int64_t)(HW - p) < left ? (int64_t)(HW - p) : left);
        const size_t base = ((size_t)b * C + c) * HW + p;
        int i = threadIdx.x * W;
        if constexpr (U > 1) {
            for (; i + (U - 1) * STEP < n; i += U * STEP) {
                unroll_for<U>([&](auto uc) { ldf(base + i + decltype(uc)::value * STEP, uc); });
                unroll_for<U>([&](auto uc) { usef(base + i + decltype(uc)::value * STEP, uc); });
            }
        }
        for (; i < n; i += STEP) {
            ldf(base + i, std::integral_constant<int, 0>{});
            usef(base + i, std::integral_constant<int, 0>{});
        }
        e += n;
        ++b;
        p = 0;
    }
}

// the normalisation of the forward (and its re-evaluation for the ReLU mask in the backward): one
// helper, so both sides compute the same bits
__device__ __forceinline__ float bn_affine(float v, float alpha, float beta) { return v * alpha + beta; }

// g * act'(output) of the BN backward: from the saved output y, or, when y is NULL (act NONE / RELU), from
// the input x through the forward's affine map (alpha = invstd * w, beta = b - mean * alpha)
__device__ __forceinline__ float bn_act_grad(int act, float g, bool has_y, float yv, float xv, float alpha,
                                             float beta) {
    if (has_y) return g * act_grad(act, yv);
    if (act == LDM_ACT_RELU) return bn_affine(xv, alpha, beta) > 0.f ? g : 0.f;
    return g;
}

// ---- BatchNorm forward ---------------------------------------------------------------------------
template <int W, int ST, int U, int HM>
__global__ __launch_bounds__(kThreads) void bn_stats_partial_kernel(const void* __restrict__ x, int sf, int C, int HW,
                                                                    int64_t n, int64_t S,
                                                                    double* __restrict__ part) {
    const bool xh = st_flag<HM>(sf, LDM_ST_X16);
    __shared__ double red[kThreads / 64];
    const int k = blockIdx.x, c = blockIdx.y, P = gridDim.x;
    const int64_t e0 = (int64_t)k * S, e1 = e0 + S < n ? e0 + S : n;
    double s = 0.0, q = 0.0;
    RawW<W> rv[U];
    slice_for_u<W, U>(
        e0, e1, C, c, HW, [&](size_t o, auto u) { ld_raw<ST, W>(x, o, xh, rv[decltype(u)::value]); },
        [&](size_t, auto u) {
            float v[W];
            cvt_raw<ST, W>(rv[decltype(u)::value], xh, v);
#pragma unroll
            for (int j = 0; j < W; ++j) {
                s += (double)v[j];
                q += (double)v[j] * (double)v[j];
            }
        });
    s = block_sum(s, red);
    q = block_sum(q, red);
    if (threadIdx.x == 0) {
        part[((size_t)c * P + k) * 2 + 0] = s;
        part[((size_t)c * P + k) * 2 + 1] = q;
    }
}

// stats[2c+j] = sum_k part[c][k][j] (slices in order); optional float copies out0/out1.  stats[2C] =
// the element count per channel on this rank (n): all-reduced together with the sums, it becomes the
// global count that the apply stages read on the device (no separate collective, no host sync).
__global__ __launch_bounds__(kThreads) void slices_finalize_kernel(const double* __restrict__ part, int C, int P,
                                                                   double* __restrict__ stats,
                                                                   float* __restrict__ out0,
                                                                   float* __restrict__ out1, double n) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c == 0) stats[2 * C] = n;
    if (c >= C) return;
    double a = 0.0, b = 0.0;
    for (int k = 0; k < P; ++k) {
        a += part[((size_t)c * P + k) * 2 + 0];
        b += part[((size_t)c * P + k) * 2 + 1];
    }
    stats[2 * c] = a;
    stats[2 * c + 1] = b;
    if (out0) out0[c] = (float)a;
    if (out1) out1[c] = (float)b;
}

template <int W, int ST, int U, int HM>
__global__ __launch_bounds__(kThreads) void bn_apply_kernel(const void* src, void* x, int sf, int C,
                                                            int HW, int64_t n, int64_t S,
                                                            const double* __restrict__ stats, double count_arg,
                                                            const float* __restrict__ weight,
                                                            const float* __restrict__ bias, float* __restrict__ rmean,
                                                            float* __restrict__ rvar, float momentum, float eps,
                                                            int act, float* __restrict__ save_mean,
                                                            float* __restrict__ save_invstd,
                                                            const double* __restrict__ part, int P) {
    const int k = blockIdx.x, c = blockIdx.y;
    const double count = count_arg > 0.0 ? count_arg : stats[2 * C];   // <= 0: the all-reduced count
    // part: the slice partials of bn_stats_partial_kernel, summed here in slice order exactly as
    // slices_finalize_kernel sums them (same bits), so the rank-local path needs no finalize launch
    double s1 = 0.0, s2 = 0.0;
    if (part) {
        for (int q = 0; q < P; ++q) {
            s1 += part[((size_t)c * P + q) * 2 + 0];
            s2 += part[((size_t)c * P + q) * 2 + 1];
        }
    } else {
        s1 = stats[2 * c];
        s2 = stats[2 * c + 1];
    }
    const double mean = s1 / count;
    double var_sum = s2 - mean * s1;   // sum (x - mean)^2
    if (var_sum < 0.0) var_sum = 0.0;
    const float mean_f = (float)mean;
    const float invstd = (float)(1.0 / sqrt(var_sum / count + (double)eps));
    const float alpha = invstd * (weight ? weight[c] : 1.0f);
    const float beta = (bias ? bias[c] : 0.0f) - mean_f * alpha;
    const int64_t e0 = (int64_t)k * S, e1 = e0 + S < n ? e0 + S : n;
    const int ro = (act >> 8) & 0xff, ac = act & 0xff;   // LDM_ACT_ROUND_*: the output of a 16-bit input's BN (autocast)
    const bool xh = st_flag<HM>(sf, LDM_ST_X16), yh = st_flag<HM>(sf, LDM_ST_Y16);
    RawW<W> rv[U];
    slice_for_u<W, U>(
        e0, e1, C, c, HW, [&](size_t o, auto u) { ld_raw<ST, W>(src, o, xh, rv[decltype(u)::value]); },
        [&](size_t o, auto u) {
            float v[W];
            cvt_raw<ST, W>(rv[decltype(u)::value], xh, v);
#pragma unroll
            for (int j = 0; j < W; ++j) v[j] = apply_act(round16(bn_affine(v[j], alpha, beta), ro), ac);
            st_st<ST, W>(x, o, yh, v);
        });
    if (k == 0 && threadIdx.x == 0) {
        if (rmean) rmean[c] = (float)((double)momentum * mean + (1.0 - (double)momentum) * (double)rmean[c]);
        if (rvar) {
            const double unbiased = count > 1.0 ? var_sum / (count - 1.0) : var_sum;
            rvar[c] = (float)((double)momentum * unbiased + (1.0 - (double)momentum) * (double)rvar[c]);
        }
        if (save_mean) save_mean[c] = mean_f;
        if (save_invstd) save_invstd[c] = invstd;
    }
}

// ---- BatchNorm backward: g = dy*act'(y); sums (sum g, sum g*xhat); dx = w*invstd*(g - sg/N - xhat*sgx/N)
template <int W, int ST, int U, int HM>
__global__ __launch_bounds__(kThreads) void bn_bwd_partial_kernel(const void* __restrict__ dy,
                                                                  const void* __restrict__ y,
                                                                  const void* __restrict__ x, int sf,
                                                                  const float* __restrict__ mean,
                                                                  const float* __restrict__ invstd,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ bias, int act, int C,
                                                                  int HW, int64_t n, int64_t S,
                                                                  double* __restrict__ part) {
    __shared__ double red[kThreads / 64];
    const int k = blockIdx.x, c = blockIdx.y, P = gridDim.x;
    const float mu = mean[c], is = invstd[c];
    const float alpha = is * (w ? w[c] : 1.0f);
    const float beta = (bias ? bias[c] : 0.0f) - mu * alpha;
    const int64_t e0 = (int64_t)k * S, e1 = e0 + S < n ? e0 + S : n;
    float sg = 0.f, sgx = 0.f;
    const bool dyh = st_flag<HM>(sf, LDM_ST_DY16), yh = st_flag<HM>(sf, LDM_ST_Y16), xh = st_flag<HM>(sf, LDM_ST_X16);
    RawW<W> rg[U], ry[U] = {}, rx[U];
    slice_for_u<W, U>(
        e0, e1, C, c, HW,
        [&](size_t o, auto u) {
            constexpr int q = decltype(u)::value;
            ld_raw<ST, W>(dy, o, dyh, rg[q]);
            if (y) ld_raw<ST, W>(y, o, yh, ry[q]);
            ld_raw<ST, W>(x, o, xh, rx[q]);
        },
        [&](size_t, auto u) {
            constexpr int q = decltype(u)::value;
            float g[W], yv[W] = {}, xv[W];
            cvt_raw<ST, W>(rg[q], dyh, g);
            if (y) cvt_raw<ST, W>(ry[q], yh, yv);
            cvt_raw<ST, W>(rx[q], xh, xv);
#pragma unroll
            for (int j = 0; j < W; ++j) {
                const float gj = bn_act_grad(act, g[j], y != nullptr, yv[j], xv[j], alpha, beta);
                sg += gj;
                sgx += gj * ((xv[j] - mu) * is);
            }
        });
    const double a = block_sum((double)sg, red);
    const double b = block_sum((double)sgx, red);
    if (threadIdx.x == 0) {
        part[((size_t)c * P + k) * 2 + 0] = a;
        part[((size_t)c * P + k) * 2 + 1] = b;
    }
}

template <int W, int ST, int U, int HM>
__global__ __launch_bounds__(kThreads) void bn_bwd_apply_kernel(const void* __restrict__ dy,
                                                                const void* __restrict__ y,
                                                                const void* __restrict__ x, int sf,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ invstd,
                                                                const float* __restrict__ w,
                                                                const float* __restrict__ bias, int act, int C, int HW,
                                                                int64_t n, int64_t S, const double* __restrict__ sums,
                                                                double count_arg, void* __restrict__ dx,
                                                                const double* __restrict__ part, int P,
                                                                float* __restrict__ dweight, float* __restrict__ dbias,
                                                                float* __restrict__ dxs_part) {
    __shared__ float redf[kThreads / 64];
    const int k = blockIdx.x, c = blockIdx.y;
    const double count = count_arg > 0.0 ? count_arg : sums[2 * C];
    const float mu = mean[c], is = invstd[c];
    // part: bn_bwd_partial_kernel's slice partials, summed in slice order as slices_finalize_kernel does
    double a = 0.0, b = 0.0;
    if (part) {
        for (int q = 0; q < P; ++q) {
            a += part[((size_t)c * P + q) * 2 + 0];
            b += part[((size_t)c * P + q) * 2 + 1];
        }
        if (k == 0 && threadIdx.x == 0) {
            if (dbias) dbias[c] = (float)a;
            if (dweight) dweight[c] = (float)b;
        }
    } else {
        a = sums[2 * c];
        b = sums[2 * c + 1];
    }
    const float sgN = (float)(a / count), sgxN = (float)(b / count);
    const float kk = (w ? w[c] : 1.f) * is;
    const float alpha = is * (w ? w[c] : 1.0f);
    const float beta = (bias ? bias[c] : 0.0f) - mu * alpha;
    const int64_t e0 = (int64_t)k * S, e1 = e0 + S < n ? e0 + S : n;
    const bool dyh = st_flag<HM>(sf, LDM_ST_DY16), yh = st_flag<HM>(sf, LDM_ST_Y16), xh = st_flag<HM>(sf, LDM_ST_X16),
               dxh = st_flag<HM>(sf, LDM_ST_DX16);
    float sdx = 0.f;
    RawW<W> rg[U], ry[U] = {}, rx[U];
    slice_for_u<W, U>(
        e0, e1, C, c, HW,
        [&](size_t o, auto u) {
            constexpr int q = decltype(u)::value;
            ld_raw<ST, W>(dy, o, dyh, rg[q]);
            if (y) ld_raw<ST, W>(y, o, yh, ry[q]);
            ld_raw<ST, W>(x, o, xh, rx[q]);
        },
        [&](size_t o, auto u) {
            constexpr int q = decltype(u)::value;
            float g[W], yv[W] = {}, xv[W], d[W];
            cvt_raw<ST, W>(rg[q], dyh, g);
            if (y) cvt_raw<ST, W>(ry[q], yh, yv);
            cvt_raw<ST, W>(rx[q], xh, xv);
#pragma unroll
            for (int j = 0; j < W; ++j) {
                const float gj = bn_act_grad(act, g[j], y != nullptr, yv[j], xv[j], alpha, beta);
                d[j] = kk * ((gj - sgN) - ((xv[j] - mu) * is) * sgxN);
            }
            st_st<ST, W>(dx, o, dxh, d);
            if (dxs_part) {   // the sum of dx as stored (a 16-bit dx: its rounded values)
#pragma unroll
                for (int j = 0; j < W; ++j) sdx += dxh ? round16(d[j], ST) : d[j];
            }
        });
    // dxs_part: this slice's sum of dx (fixed order: thread stride, wave tree, waves in order), for the bias
    // gradient of the conv that produced x (chan_sum_finalize_kernel sums the slices in order)
    if (dxs_part) {
        const float t = block_sum(sdx, redf);
        if (threadIdx.x == 0) dxs_part[(size_t)c * gridDim.x + k] = t;
    }
}

// out[c] = sum_k part[c][k] (slices in order)
__global__ __launch_bounds__(kThreads) void chan_sum_finalize_kernel(const float* __restrict__ part, int C, int P,
                                                                     float* __restrict__ out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    float a = 0.f;
    for (int k = 0; k < P; ++k) a += part[(size_t)c * P + k];
    out[c] = a;
}

// ---- fused-epilogue activation backward: dv = dy*act'(v); partial sums of dv and dy per (b,c,slice)
template <int W, int ST>
__global__ __launch_bounds__(kThreads) void act_bwd_kernel(const void* dy,
                                                           const void* __restrict__ aval,
                                                           const float* __restrict__ pre, int act, int sf, int C,
                                                           int HW, int64_t S, void* dv,
                                                           float* __restrict__ part) {
    const bool dyh = sf & LDM_ST_DY16, ah = sf & LDM_ST_X16, dvh = sf & LDM_ST_DX16;
    __shared__ float red[kThreads / 64];
    const int k = blockIdx.x, plane = blockIdx.y, Q = gridDim.x;
    const int b = plane / C, c = plane - b * C;
    const int64_t e0 = (int64_t)b * HW + (int64_t)k * S;
    const int64_t pe = (int64_t)b * HW + HW;
    const int64_t e1 = e0 + S < pe ? e0 + S : pe;
    float sd = 0.f, sg = 0.f;
    slice_for<W>(e0, e1, C, c, HW, [&](size_t o) {
        float g[W], d[W];
        ld_st<ST, W>(dy, o, dyh, g);
        if (act == LDM_ACT_GELU) {
            float v[W];
            ld<W>(pre + o, v);
#pragma unroll
            for (int j = 0; j < W; ++j) {
                const float cdf = 0.5f * (1.0f + erff(v[j] * 0.70710678118654752440f));
                const float pdf = 0.39894228040143267794f * expf(-0.5f * v[j] * v[j]);
                d[j] = g[j] * (cdf + v[j] * pdf);
            }
        } else if (aval) {
            float a[W];
            ld_st<ST, W>(aval, o, ah, a);
#pragma unroll
            for (int j = 0; j < W; ++j) d[j] = g[j] * act_grad(act, a[j]);
        } else {
#pragma unroll
            for (int j = 0; j < W; ++j) d[j] = g[j];
        }
        if (dv) st_st<ST, W>(dv, o, dvh, d);
#pragma unroll
        for (int j = 0; j < W; ++j) {
            sd += d[j];
            sg += g[j];
        }
    });
    if (part) {
        sd = block_sum(sd, red);
        sg = block_sum(sg, red);
        if (threadIdx.x == 0) {
            part[((size_t)plane * Q + k) * 2 + 0] = sd;
            part[((size_t)plane * Q + k) * 2 + 1] = sg;
        }
    }
}

// The same for planes of 64..1024 elements (the UNet's latent-scale maps at the train batch): the sliced
// kernel gives such a plane a whole 256-thread block, with a two-level block reduction for as little as 64
// elements (8192 blocks, 10-12 us per launch).  Here TP = HW / 4 threads own one plane (one float4 each) and
// a block holds 256 / TP planes; the plane's sums reduce over its TP lanes (shuffles within the segment, then
// the plane's waves in order through LDS when TP > 64).  One partial per plane (Q = 1) for the finalize.
template <int TP, int ST>
__global__ __launch_bounds__(kThreads) void act_bwd_planes_kernel(const void* __restrict__ dy,
                                                                  const void* __restrict__ aval, int act, int sf,
                                                                  int nplanes, void* dv, float* __restrict__ part) {
    const bool dyh = sf & LDM_ST_DY16, ah = sf & LDM_ST_X16, dvh = sf & LDM_ST_DX16;
    constexpr int PPB = kThreads / TP;
    __shared__ float red[2][kThreads / 64];
    const int pl = blockIdx.x * PPB + (int)threadIdx.x / TP;
    const int t = (int)threadIdx.x % TP;
    float sd = 0.f, sg = 0.f;
    if (pl < nplanes) {
        const size_t o = (size_t)pl * (TP * 4) + (size_t)t * 4;
        float g[4], d[4];
        ld_st<ST, 4>(dy, o, dyh, g);
        if (aval) {
            float a[4];
            ld_st<ST, 4>(aval, o, ah, a);
#pragma unroll
            for (int j = 0; j < 4; ++j) d[j] = g[j] * act_grad(act, a[j]);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) d[j] = g[j];
        }
        if (dv) st_st<ST, 4>(dv, o, dvh, d);
        sd = ((d[0] + d[1]) + d[2]) + d[3];
        sg = ((g[0] + g[1]) + g[2]) + g[3];
    }
    constexpr int SEG = TP < 64 ? TP : 64;
#pragma unroll
    for (int o = SEG / 2; o > 0; o >>= 1) {
        sd += __shfl_xor(sd, o);
        sg += __shfl_xor(sg, o);
    }
    if constexpr (TP > 64) {   // the plane spans TP / 64 waves: add their sums in wave order
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        if (lane == 0) {
            red[0][wave] = sd;
            red[1][wave] = sg;
        }
        __syncthreads();
        if (t == 0) {
            const int w0 = wave;   // the plane's first wave
            sd = red[0][w0];
            sg = red[1][w0];
#pragma unroll
            for (int w = 1; w < TP / 64; ++w) {
                sd += red[0][w0 + w];
                sg += red[1][w0 + w];
            }
        }
    }
    if (part && t == 0 && pl < nplanes) {
        part[(size_t)pl * 2 + 0] = sd;
        part[(size_t)pl * 2 + 1] = sg;
    }
}

// dbias[c] = sum_b sum_k part_dv;  dbcast[b,c] = sum_k part_dy.  One block per channel: a plane's Q slice
// partials go to QP lanes (QP = Q rounded up to a power of two, at most 64; lane stride past 64), so a wave
// takes 64 / QP planes per step (wave w the planes from w * 64 / QP on, stepping by 256 / QP) and sums each
// plane by a segmented shuffle tree; the plane sums meet in a full-wave tree, the four wave sums in wave
// order.  A fixed partition and order, so bitwise reproducible (a single thread walking B*Q partials
// serially took 150 us for the decoder's one-channel output layer at B = 32; one plane per wave step left
// the Q = 1 finalize of the plane kernels at 8 serial load round trips per wave).
__device__ __forceinline__ void act_fin_body(const float* __restrict__ part, int B, int C, int Q, int QP,
                                             float* __restrict__ dbias, float* __restrict__ dbcast, int c) {
    __shared__ float wsum[kThreads / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int ppw = 64 / QP, sub = lane / QP, k0 = lane % QP;
    float sb = 0.f;
    for (int b0 = wave * ppw; b0 < B; b0 += (kThreads / 64) * ppw) {
        const int b = b0 + sub;
        const size_t pl = (size_t)b * C + c;
        float sd = 0.f, sg = 0.f;
        if (b < B)
            for (int k = k0; k < Q; k += QP) {
                sd += part[(pl * Q + k) * 2 + 0];
                sg += part[(pl * Q + k) * 2 + 1];
            }
        for (int o = QP / 2; o > 0; o >>= 1) {
            sd += __shfl_xor(sd, o);
            sg += __shfl_xor(sg, o);
        }
        if (k0 == 0 && b < B) {
            sb += sd;
            if (dbcast) dbcast[pl] = sg;
        }
    }
    for (int o = 32; o > 0; o >>= 1) sb += __shfl_xor(sb, o);
    if (lane == 0) wsum[wave] = sb;
    __syncthreads();
    if (threadIdx.x == 0 && dbias) {
        float s = 0.f;
        for (int w = 0; w < kThreads / 64; ++w) s += wsum[w];
        dbias[c] = s;
    }
}
__global__ __launch_bounds__(kThreads) void act_bwd_finalize_kernel(const float* __restrict__ part, int B, int C,
                                                                    int Q, int QP, float* __restrict__ dbias,
                                                                    float* __restrict__ dbcast) {
    act_fin_body(part, B, C, Q, QP, dbias, dbcast, blockIdx.x);
}

// The finalizes of several activation backwards in one launch (ldm_act_finalize_many): the bias gradients of a
// train step's convs are read only by the optimizer, so their finalize launches (one per conv, ~16 per step) can
// wait for the end of the backward and go as one.  Block -> (job, channel) by the jobs' first blocks c0; each
// channel's sums are act_bwd_finalize_kernel's (act_fin_body), so the same bits.
struct FinJob {
    const float* part;
    float* dbias;
    int32_t B, C, Q, QP, c0, kind;   // kind 0: act_fin_body; 1: chan_sum_finalize_kernel's sum (Q = its P)
};
constexpr int kMaxFinJobs = 24;
struct FinJobs {
    FinJob j[kMaxFinJobs];
    int32_t n;
};
__global__ __launch_bounds__(kThreads) void act_bwd_finalize_many_kernel(FinJobs jobs) {
    int k = 0;
    while (k + 1 < jobs.n && (int)blockIdx.x >= jobs.j[k + 1].c0) ++k;
    const FinJob& J = jobs.j[k];
    const int c = (int)blockIdx.x - J.c0;
    if (J.kind == 0) {
        act_fin_body(J.part, J.B, J.C, J.Q, J.QP, J.dbias, nullptr, c);
    } else if (threadIdx.x == 0) {   // the slices in order, as chan_sum_finalize_kernel sums them
        float a = 0.f;
        for (int q = 0; q < J.Q; ++q) a += J.part[(size_t)c * J.Q + q];
        J.dbias[c] = a;
    }
}
static int finalize_lanes(int Q) {
    int qp = 1;
    while (qp < Q && qp < 64) qp *= 2;
    return qp;
}

// Small planes (HW <= 16: the Linear layers, HW = 1, and the 2x8 projections): one block per channel
// over its B*HW elements (dv elementwise, dbias by a block sum, dbcast[b] by the first B lanes over their
// HW elements) -- one launch instead of the sliced kernel's B*C tiny blocks plus the finalize pass.
template <int ST>
__global__ __launch_bounds__(kThreads) void act_bwd_small_kernel(const void* __restrict__ dy,
                                                                 const void* __restrict__ aval,
                                                                 const float* __restrict__ pre, int act, int sf, int B,
                                                                 int C, int HW, void* __restrict__ dv,
                                                                 float* __restrict__ dbias, float* __restrict__ dbcast) {
    __shared__ float red[kThreads / 64];
    const int c = blockIdx.x;
    const bool dyh = sf & LDM_ST_DY16, ah = sf & LDM_ST_X16, dvh = sf & LDM_ST_DX16;
    auto dval = [&](size_t o) {
        const float g = ld1_st<ST>(dy, o, dyh);
        if (act == LDM_ACT_GELU) {
            const float v = pre[o];
            const float cdf = 0.5f * (1.0f + erff(v * 0.70710678118654752440f));
            const float pdf = 0.39894228040143267794f * expf(-0.5f * v * v);
            return g * (cdf + v * pdf);
        }
        return aval ? g * act_grad(act, ld1_st<ST>(aval, o, ah)) : g;
    };
    float sd = 0.f;
    for (int e = threadIdx.x; e < B * HW; e += blockDim.x) {
        const int b = e / HW, i = e - b * HW;
        const size_t o = ((size_t)b * C + c) * HW + i;
        const float d = dval(o);
        if (dv) st1_st<ST>(dv, o, dvh, d);
        sd += d;
    }
    if (dbias) {
        sd = block_sum(sd, red);
        if (threadIdx.x == 0) dbias[c] = sd;
    }
    if (dbcast) {
        for (int b = threadIdx.x; b < B; b += blockDim.x) {
            const size_t o = ((size_t)b * C + c) * HW;
            float sg = 0.f;
            for (int i = 0; i < HW; ++i) sg += ld1_st<ST>(dy, o + i, dyh);
            dbcast[(size_t)b * C + c] = sg;
        }
    }
}

bool vec_ok(int HW, const void* a, const void* b = nullptr, const void* c = nullptr, const void* d = nullptr) {
    auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    return HW % 4 == 0 && al(a) && al(b) && al(c) && al(d);
}

// elements per thread access of the sliced kernels: 8 (one 16-byte load of a 16-bit map, two float4 of an fp32
// one) when HW % 8 == 0 and the pointers are 16-byte aligned, else 4 (float4 / 8-byte), else 1.  The width
// depends only on HW and alignment, never on the storage type, so a map's sums keep the same order (and bits)
// in 16-bit and fp32 storage.  LDM_REDUCE_W8=0: 4 at most.
inline int vec_width(int HW, const void* a, const void* b = nullptr, const void* c = nullptr, const void* d = nullptr) {
    static const bool w8 = [] {
        const char* e = getenv("LDM_REDUCE_W8");
        return !(e && e[0] == '0');
    }();
    if (!vec_ok(HW, a, b, c, d)) return 1;
    return w8 && HW % 8 == 0 ? 8 : 4;
}
template <class F>
void w_dispatch(int w, F&& f) {
    if (w == 8) f(std::integral_constant<int, 8>{});
    else if (w == 4) f(std::integral_constant<int, 4>{});
    else f(std::integral_constant<int, 1>{});
}

// pieces of a thread in flight in the BatchNorm sweeps (slice_for_u): LDM_BN_UNROLL = 1, 2 or 4 (default 2)
inline int bn_unroll() {
    static const int v = [] {
        const char* e = getenv("LDM_BN_UNROLL");
        const int x = e ? atoi(e) : 2;
        return x == 1 || x == 4 ? x : 2;
    }();
    return v;
}
// (U, HM) instances: HM 0 (run-time flags) only with U = 1; HM 1 / 2 with U = bn_unroll()
template <class F>
void uh_dispatch(int hm, F&& f) {
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I4 = std::integral_constant<int, 4>;
    using H0 = std::integral_constant<int, 0>;
    if (hm == 0) return f(I1{}, H0{});
    const int u = bn_unroll();
    auto go = [&](auto hc) {
        if (u == 4) f(I4{}, hc);
        else if (u == 1) f(I1{}, hc);
        else f(I2{}, hc);
    };
    if (hm == 1) go(std::integral_constant<int, 1>{});
    else go(std::integral_constant<int, 2>{});
}
// the storage fields of an act code (ldm_capi.h LDM_ST_*): 16-bit type, per-tensor flags, and the act + round
// bits the kernels read
struct StCode {
    int st, sf, act;
};
inline StCode st_code(int32_t code) {
    StCode c{(code >> LDM_ST_SHIFT) & 3, code & (LDM_ST_X16 | LDM_ST_Y16 | LDM_ST_DY16 | LDM_ST_DX16), code & 0xffff};
    if (c.st != LDM_DT_F16 && c.st != LDM_DT_BF16) c.st = 0, c.sf = 0;
    return c;
}
// the HM of a call: which of `bits` (the flags of the tensors it reads / writes) are set
inline int bn_hm(const StCode& sc, int bits) {
    if (sc.st == 0) return 2;
    const int f = sc.sf & bits;
    return f == bits ? 1 : (f == 0 ? 2 : 0);
}
// f(integral_constant<int, ST>) for the code's storage type
template <class F>
void st_dispatch(const StCode& c, F&& f) {
    if (c.st == LDM_DT_F16) f(std::integral_constant<int, LDM_DT_F16>{});
    else if (c.st == LDM_DT_BF16) f(std::integral_constant<int, LDM_DT_BF16>{});
    else f(std::integral_constant<int, 0>{});
}

}  // namespace
}  // namespace ldm

using namespace ldm;

extern "C" int64_t ldm_reduce_workspace_floats(int32_t B, int32_t C, int32_t HW) {
    if (B < 0 || C <= 0 || HW <= 0) return 0;
    if (B == 0) B = 1;   // an empty local shard (SyncBatchNorm) still runs the finalize stage
    const int64_t n = (int64_t)B * HW;
    // doubles -> floats, + the dx-sum slice partials of ldm_batchnorm_backward_dxsum (C * P floats)
    const int64_t bn = 2 * ((int64_t)C * bn_slices(n, C) * 2 + 2 * (int64_t)C + 2) + (int64_t)C * bn_slices(n, C);
    const int64_t ac = (int64_t)B * C * act_slices(B, C, HW) * 2;
    return bn > ac ? bn : ac;
}

static int bn_stats_launch(const void* x, const StCode& sc, int32_t B, int32_t C, int32_t HW, double* part,
                           void* stream) {
    const int64_t n = (int64_t)B * HW;
    const int P = bn_slices(n, C);
    const int vw = vec_width(HW, x);
    const int64_t S = slice_len(n, P, vw);
    const dim3 grid(P, C);
    const int hm = bn_hm(sc, LDM_ST_X16);
    st_dispatch(sc, [&](auto stc) {
        w_dispatch(vw, [&](auto wc) { uh_dispatch(hm, [&](auto uc, auto hc) {
            hipLaunchKernelGGL((bn_stats_partial_kernel<decltype(wc)::value, decltype(stc)::value, decltype(uc)::value, decltype(hc)::value>), grid, dim3(kThreads),
                               0, (hipStream_t)stream, x, sc.sf, C, HW, n, S, part);
        }); });
    });
    LDM_CHECK_LAUNCH("bn_stats_partial_kernel");
    return 0;
}

// SyncBatchNorm stage 1 with a storage code (LDM_ST_X16 | type << LDM_ST_SHIFT for a 16-bit input)
extern "C" int ldm_batchnorm_stats_code(const float* x, int32_t code, int32_t B, int32_t C, int32_t HW, double* stats,
                                        float* workspace, void* stream) {
    LDM_REQUIRE(stats && workspace && B >= 0 && C > 0 && HW > 0 && (x || B == 0), "batchnorm_stats: bad argument");
    LDM_REQUIRE(((uintptr_t)workspace & 7) == 0, "batchnorm_stats: workspace must be 8-byte aligned");
    const int64_t n = (int64_t)B * HW;
    const int P = bn_slices(n, C);
    double* part = reinterpret_cast<double*>(workspace);
    const int rc = bn_stats_launch(x, st_code(code), B, C, HW, part, stream);   // (B = 0: zero partials)
    if (rc) return rc;
    hipLaunchKernelGGL(slices_finalize_kernel, dim3((C + kThreads - 1) / kThreads), dim3(kThreads), 0,
                       (hipStream_t)stream, part, C, P, stats, nullptr, nullptr, (double)n);
    LDM_CHECK_LAUNCH("slices_finalize_kernel");
    return 0;
}

extern "C" int ldm_batchnorm_stats(const float* x, int32_t B, int32_t C, int32_t HW, double* stats, float* workspace,
                                   void* stream) {
    return ldm_batchnorm_stats_code(x, 0, B, C, HW, stats, workspace, stream);
}

// part != NULL: the statistics are summed from bn_stats_partial_kernel's slice partials inside the apply
static int bn_apply_launch(const float* x, float* y, int32_t B, int32_t C, int32_t HW, const double* stats,
                           double count, const float* weight, const float* bias, float* running_mean,
                           float* running_var, float momentum, float eps, int32_t act, float* save_mean,
                           float* save_invstd, const double* part, void* stream) {
    const int64_t n = (int64_t)B * HW;
    const int P = bn_slices(n, C);
    const StCode sc = st_code(act);
    const int vw = vec_width(HW, x, y);
    const int64_t S = slice_len(n, P, vw);
    const dim3 grid(P, C);
    const int hm = bn_hm(sc, LDM_ST_X16 | LDM_ST_Y16);
    st_dispatch(sc, [&](auto stc) {
        w_dispatch(vw, [&](auto wc) { uh_dispatch(hm, [&](auto uc, auto hc) {
            hipLaunchKernelGGL((bn_apply_kernel<decltype(wc)::value, decltype(stc)::value, decltype(uc)::value, decltype(hc)::value>), grid, dim3(kThreads), 0,
                               (hipStream_t)stream, x, y, sc.sf, C, HW, n, S, stats, count, weight, bias, running_mean,
                               running_var, momentum, eps, sc.act, save_mean, save_invstd, part, part ? P : 0);
        }); });
    });
    LDM_CHECK_LAUNCH("bn_apply_kernel");
    return 0;
}

extern "C" int ldm_batchnorm_apply_out(const float* x, float* y, int32_t B, int32_t C, int32_t HW, const double* stats,
                                       double count, const float* weight, const float* bias, float* running_mean,
                                       float* running_var, float momentum, float eps, int32_t act, float* save_mean,
                                       float* save_invstd, void* stream) {
    LDM_REQUIRE(stats && B >= 0 && C > 0 && HW > 0 && ((x && y) || B == 0), "batchnorm_apply: bad argument");
    return bn_apply_launch(x, y, B, C, HW, stats, count, weight, bias, running_mean, running_var, momentum, eps, act,
                           save_mean, save_invstd, nullptr, stream);
}

extern "C" int ldm_batchnorm_apply(float* x, int32_t B, int32_t C, int32_t HW, const double* stats, double count,
                                   const float* weight, const float* bias, float* running_mean, float* running_var,
                                   float momentum, float eps, int32_t act, float* save_mean, float* save_invstd,
                                   void* stream) {
    return ldm_batchnorm_apply_out(x, x, B, C, HW, stats, count, weight, bias, running_mean, running_var, momentum,
                                   eps, act, save_mean, save_invstd, stream);
}

extern "C" int ldm_batchnorm_train_out(const float* x, float* y, int32_t B, int32_t C, int32_t HW, const float* weight,
                                       const float* bias, float* running_mean, float* running_var, float momentum,
                                       float eps, int32_t act, float* save_mean, float* save_invstd, float* workspace,
                                       void* stream) {
    LDM_REQUIRE(x && y && workspace && B > 0 && C > 0 && HW > 0, "batchnorm: bad argument");
    LDM_REQUIRE(((uintptr_t)workspace & 7) == 0, "batchnorm: workspace must be 8-byte aligned");
    const int64_t n = (int64_t)B * HW;
    const int P = bn_slices(n, C);
    const int64_t S = slice_len(n, P);
    double* part = reinterpret_cast<double*>(workspace);
    // rank-local: partials, then the apply sums them itself (two launches; the SyncBatchNorm path keeps the
    // finalize stage, whose sums it all-reduces)
    (void)P, (void)S;
    const int rc = bn_stats_launch(x, st_code(act), B, C, HW, part, stream);
    if (rc) return rc;
    return bn_apply_launch(x, y, B, C, HW, nullptr, (double)n, weight, bias, running_mean, running_var, momentum, eps,
                           act, save_mean, save_invstd, part, stream);
}

extern "C" int ldm_batchnorm_train(float* x, int32_t B, int32_t C, int32_t HW, const float* weight, const float* bias,
                                   float* running_mean, float* running_var, float momentum, float eps, int32_t act,
                                   float* save_mean, float* save_invstd, float* workspace, void* stream) {
    return ldm_batchnorm_train_out(x, x, B, C, HW, weight, bias, running_mean, running_var, momentum, eps, act,
                                   save_mean, save_invstd, workspace, stream);
}

// y may be NULL when act is NONE or RELU (bn_act_grad: the mask is re-evaluated from x)
static bool bn_need_y(int act) { return act != LDM_ACT_NONE && act != LDM_ACT_RELU; }

// the kernels' partial stage (dx == NULL) / apply stage of the BN backward under storage code sc
static int bn_bwd_partial_launch(const void* dy, const void* y, const void* x, const float* save_mean,
                                  const float* save_invstd, const float* weight, const float* bias, const StCode& sc,
                                  int act, int32_t B, int32_t C, int32_t HW, double* part, void* stream) {
    const int64_t n = (int64_t)B * HW;
    const int P = bn_slices(n, C);
    const int vw = vec_width(HW, dy, y, x);
    const int64_t S = slice_len(n, P, vw);
    const dim3 grid(P, C);
    const int hm = bn_hm(sc, LDM_ST_DY16 | LDM_ST_X16 | (y ? LDM_ST_Y16 : 0));
    st_dispatch(sc, [&](auto stc) {
        w_dispatch(vw, [&](auto wc) { uh_dispatch(hm, [&](auto uc, auto hc) {
            hipLaunchKernelGGL((bn_bwd_partial_kernel<decltype(wc)::value, decltype(stc)::value, decltype(uc)::value, decltype(hc)::value>), grid, dim3(kThreads),
                               0, (hipStream_t)stream, dy, y, x, sc.sf, save_mean, save_invstd, weight, bias, act, C, HW,
                               n, S, part);
        }); });
    });
    LDM_CHECK_LAUNCH("bn_bwd_partial_kernel");
    return 0;
}

extern "C" int ldm_batchnorm_backward_reduce(const float* dy, const float* y, const float* x, const float* save_mean,
                                             const float* save_invstd, const float* weight, const float* bias,
                                             int32_t act_code, int32_t B, int32_t C, int32_t HW, double* sums,
                                             float* dweight, float* dbias, float* workspace, void* stream) {
    const StCode sc = st_code(act_code);
    const int act = sc.act & 0xff;
    LDM_REQUIRE(save_mean && save_invstd && sums && workspace && B >= 0 && C > 0 && HW > 0 &&
                    ((dy && x && (y || !bn_need_y(act))) || B == 0),
                "bn_backward_reduce: bad argument");
    LDM_REQUIRE(((uintptr_t)workspace & 7) == 0, "bn_backward_reduce: workspace must be 8-byte aligned");
    const int64_t n = (int64_t)B * HW;
    const int P = bn_slices(n, C);
    double* part = reinterpret_cast<double*>(workspace);
    const int rc = bn_bwd_partial_launch(dy, y, x, save_mean, save_invstd, weight, bias, sc, act, B, C, HW, part, stream);
    if (rc) return rc;
    // local sums: db = sum g, dw = sum g*xhat (SyncBatchNorm keeps the parameter grads local)
    hipLaunchKernelGGL(slices_finalize_kernel, dim3((C + kThreads - 1) / kThreads), dim3(kThreads), 0,
                       (hipStream_t)stream, part, C, P, sums, dbias, dweight, (double)n);
    LDM_CHECK_LAUNCH("slices_finalize_kernel");
    return 0;
}

// part != NULL: the sums come from bn_bwd_partial_kernel's slice partials, and dweight / dbias are written here
static int bn_bwd_apply_launch(const void* dy, const void* y, const void* x, const float* save_mean,
                               const float* save_invstd, const float* weight, const float* bias, const StCode& sc,
                               int act, int32_t B, int32_t C, int32_t HW, const double* sums, double count, void* dx,
                               const double* part, float* dweight, float* dbias, void* stream, float* dxs_part = nullptr) {
    if (B == 0) return 0;
    const int64_t n = (int64_t)B * HW;
    const int P = bn_slices(n, C);
    const int vw = vec_width(HW, dy, y, x, dx);
    const int64_t S = slice_len(n, P, vw);
    const dim3 grid(P, C);
    const int hm = bn_hm(sc, LDM_ST_DY16 | LDM_ST_X16 | LDM_ST_DX16 | (y ? LDM_ST_Y16 : 0));
    st_dispatch(sc, [&](auto stc) {
        w_dispatch(vw, [&](auto wc) { uh_dispatch(hm, [&](auto uc, auto hc) {
            hipLaunchKernelGGL((bn_bwd_apply_kernel<decltype(wc)::value, decltype(stc)::value, decltype(uc)::value, decltype(hc)::value>), grid, dim3(kThreads), 0,
                               (hipStream_t)stream, dy, y, x, sc.sf, save_mean, save_invstd, weight, bias, act, C, HW, n,
                               S, sums, count, dx, part, part ? P : 0, dweight, dbias, dxs_part);
        }); });
    });
    LDM_CHECK_LAUNCH("bn_bwd_apply_kernel");
    return 0;
}

extern "C" int ldm_batchnorm_backward_apply(const float* dy, const float* y, const float* x, const float* save_mean,
                                            const float* save_invstd, const float* weight, const float* bias,
                                            int32_t act_code, int32_t B, int32_t C, int32_t HW, const double* sums,
                                            double count, float* dx, void* stream) {
    const StCode sc = st_code(act_code);
    const int act = sc.act & 0xff;
    LDM_REQUIRE(save_mean && save_invstd && sums && B >= 0 && C > 0 && HW > 0 &&
                    ((dy && x && dx && (y || !bn_need_y(act))) || B == 0),
                "bn_backward_apply: bad argument");
    return bn_bwd_apply_launch(dy, y, x, save_mean, save_invstd, weight, bias, sc, act, B, C, HW, sums, count, dx,
                               nullptr, nullptr, nullptr, stream);
}

extern "C" int ldm_batchnorm_backward(const float* dy, const float* y, const float* x, const float* save_mean,
                                      const float* save_invstd, const float* weight, const float* bias, int32_t act_code,
                                      int32_t B, int32_t C, int32_t HW, float* dx, float* dweight, float* dbias,
                                      float* workspace, void* stream) {
    LDM_REQUIRE(workspace && B > 0 && C > 0 && HW > 0, "bn_backward: bad argument");
    const StCode sc = st_code(act_code);
    const int act = sc.act & 0xff;
    const int64_t n = (int64_t)B * HW;
    double* sums = reinterpret_cast<double*>(workspace) + (size_t)C * bn_slices(n, C) * 2;
    if (!dx)   // parameter grads only: partials + finalize
        return ldm_batchnorm_backward_reduce(dy, y, x, save_mean, save_invstd, weight, bias, act_code, B, C, HW, sums,
                                             dweight, dbias, workspace, stream);
    LDM_REQUIRE(dy && x && save_mean && save_invstd && (y || !bn_need_y(act)), "bn_backward: bad argument");
    LDM_REQUIRE(((uintptr_t)workspace & 7) == 0, "bn_backward: workspace must be 8-byte aligned");
    double* part = reinterpret_cast<double*>(workspace);
    const int rc = bn_bwd_partial_launch(dy, y, x, save_mean, save_invstd, weight, bias, sc, act, B, C, HW, part, stream);
    if (rc) return rc;
    // the apply sums the partials itself and writes dweight / dbias (no finalize launch)
    return bn_bwd_apply_launch(dy, y, x, save_mean, save_invstd, weight, bias, sc, act, B, C, HW, nullptr, (double)n,
                               dx, part, dweight, dbias, stream);
}

static int bn_backward_dxsum_impl(const float* dy, const float* y, const float* x, const float* save_mean,
                                  const float* save_invstd, const float* weight, const float* bias, int32_t act_code,
                                  int32_t B, int32_t C, int32_t HW, float* dx, float* dweight, float* dbias,
                                  float* dx_sum, float* dxs_ext, int32_t* p_out, float* workspace, void* stream) {
    LDM_REQUIRE(workspace && dx && dx_sum && B > 0 && C > 0 && HW > 0, "bn_backward_dxsum: bad argument");
    const StCode sc = st_code(act_code);
    const int act = sc.act & 0xff;
    LDM_REQUIRE(dy && x && save_mean && save_invstd && (y || !bn_need_y(act)), "bn_backward_dxsum: bad argument");
    LDM_REQUIRE(((uintptr_t)workspace & 7) == 0, "bn_backward_dxsum: workspace must be 8-byte aligned");
    const int64_t n = (int64_t)B * HW;
    const int P = bn_slices(n, C);
    double* part = reinterpret_cast<double*>(workspace);
    float* dxs = dxs_ext ? dxs_ext : workspace + 2 * ((int64_t)C * P * 2 + 2 * (int64_t)C + 2);
    int rc = bn_bwd_partial_launch(dy, y, x, save_mean, save_invstd, weight, bias, sc, act, B, C, HW, part, stream);
    if (rc) return rc;
    rc = bn_bwd_apply_launch(dy, y, x, save_mean, save_invstd, weight, bias, sc, act, B, C, HW, nullptr, (double)n, dx,
                             part, dweight, dbias, stream, dxs);
    if (rc) return rc;
    if (p_out) {   // deferred: ldm_act_finalize_many sums the slices later (job kind 1)
        *p_out = P;
        return 0;
    }
    hipLaunchKernelGGL(chan_sum_finalize_kernel, dim3((C + kThreads - 1) / kThreads), dim3(kThreads), 0,
                       (hipStream_t)stream, dxs, C, P, dx_sum);
    LDM_CHECK_LAUNCH("chan_sum_finalize_kernel");
    return 0;
}

// ldm_batchnorm_backward plus dx_sum[c] = sum of dx over (b, h, w): the bias gradient of the conv whose output is
// the BN's input (no separate sweep over dx for it).  The slice partials go after the backward's own workspace.
extern "C" int ldm_batchnorm_backward_dxsum(const float* dy, const float* y, const float* x, const float* save_mean,
                                            const float* save_invstd, const float* weight, const float* bias,
                                            int32_t act_code, int32_t B, int32_t C, int32_t HW, float* dx,
                                            float* dweight, float* dbias, float* dx_sum, float* workspace, void* stream) {
    return bn_backward_dxsum_impl(dy, y, x, save_mean, save_invstd, weight, bias, act_code, B, C, HW, dx, dweight, dbias,
                                  dx_sum, nullptr, nullptr, workspace, stream);
}

// The same with the dx-sum's slice partials in `dxs_part` (ldm_bn_dxsum_partial_floats(B, C, HW) floats, kept until
// the finalize) and the finalize deferred: *p_out = the slice count for an ldm_act_finalize_many job of kind 1.
extern "C" int ldm_batchnorm_backward_dxsum_defer(const float* dy, const float* y, const float* x, const float* save_mean,
                                                  const float* save_invstd, const float* weight, const float* bias,
                                                  int32_t act_code, int32_t B, int32_t C, int32_t HW, float* dx,
                                                  float* dweight, float* dbias, float* dx_sum, float* dxs_part,
                                                  int32_t* p_out, float* workspace, void* stream) {
    LDM_REQUIRE(dxs_part && p_out, "bn_backward_dxsum_defer: bad argument");
    return bn_backward_dxsum_impl(dy, y, x, save_mean, save_invstd, weight, bias, act_code, B, C, HW, dx, dweight, dbias,
                                  dx_sum, dxs_part, p_out, workspace, stream);
}

extern "C" int64_t ldm_bn_dxsum_partial_floats(int32_t B, int32_t C, int32_t HW) {
    if (B <= 0 || C <= 0 || HW <= 0) return -1;
    return (int64_t)C * bn_slices((int64_t)B * HW, C);
}

// defer_q != NULL (ldm_act_backward_defer): the slice partials stay in `workspace` for ldm_act_finalize_many and
// *defer_q receives their slice count Q (0: nothing deferred, the small-plane kernel wrote dbias itself)
static int act_backward_impl(const float* dy, const float* act_out, const float* pre_act, int32_t act_code, int32_t B,
                             int32_t C, int32_t HW, float* dv, float* dbias, float* dbcast, float* workspace,
                             int32_t* defer_q, void* stream) {
    if (defer_q) *defer_q = 0;
    const StCode sc = st_code(act_code);
    const int act = sc.act & 0xff;
    LDM_REQUIRE(dy && B > 0 && C > 0 && HW > 0, "act_backward: bad argument");
    LDM_REQUIRE(act != LDM_ACT_GELU || pre_act, "act_backward: GELU needs the pre-activation");
    LDM_REQUIRE(act == LDM_ACT_NONE || act == LDM_ACT_GELU || act_out, "act_backward: needs the activation output");
    const bool sums = dbias || dbcast;
    const float* aval0 = act == LDM_ACT_NONE || act == LDM_ACT_GELU ? nullptr : act_out;
    hipStream_t st = (hipStream_t)stream;
    if (HW <= 16) {
        st_dispatch(sc, [&](auto stc) {
            hipLaunchKernelGGL((act_bwd_small_kernel<decltype(stc)::value>), dim3(C), dim3(kThreads), 0, st, dy, aval0,
                               pre_act, act, sc.sf, B, C, HW, dv, dbias, dbcast);
        });
        LDM_CHECK_LAUNCH("act_bwd_small_kernel");
        return 0;
    }
    LDM_REQUIRE(!sums || workspace, "act_backward: bias / bcast sums need the workspace");
    // act none: dv = dy, so the write is dropped only when dv IS dy (a separate dv buffer is still written)
    float* dvp = act == LDM_ACT_NONE && dv == dy ? nullptr : dv;
    if (HW >= 64 && HW <= 1024 && (HW & (HW - 1)) == 0 && act != LDM_ACT_GELU && vec_ok(HW, dy, aval0, nullptr, dvp)) {
        const int nplanes = B * C;
        float* part = sums ? workspace : nullptr;
        const int tp = HW / 4;
        const unsigned blocks = (unsigned)((nplanes + kThreads / tp - 1) / (kThreads / tp));
        st_dispatch(sc, [&](auto stc) {
            constexpr int ST = decltype(stc)::value;
            switch (tp) {
                case 16: hipLaunchKernelGGL((act_bwd_planes_kernel<16, ST>), dim3(blocks), dim3(kThreads), 0, st, dy, aval0, act, sc.sf, nplanes, dvp, part); break;
                case 32: hipLaunchKernelGGL((act_bwd_planes_kernel<32, ST>), dim3(blocks), dim3(kThreads), 0, st, dy, aval0, act, sc.sf, nplanes, dvp, part); break;
                case 64: hipLaunchKernelGGL((act_bwd_planes_kernel<64, ST>), dim3(blocks), dim3(kThreads), 0, st, dy, aval0, act, sc.sf, nplanes, dvp, part); break;
                case 128: hipLaunchKernelGGL((act_bwd_planes_kernel<128, ST>), dim3(blocks), dim3(kThreads), 0, st, dy, aval0, act, sc.sf, nplanes, dvp, part); break;
                default: hipLaunchKernelGGL((act_bwd_planes_kernel<256, ST>), dim3(blocks), dim3(kThreads), 0, st, dy, aval0, act, sc.sf, nplanes, dvp, part); break;
            }
        });
        LDM_CHECK_LAUNCH("act_bwd_planes_kernel");
        if (sums && defer_q) {
            *defer_q = 1;
        } else if (sums) {
            hipLaunchKernelGGL(act_bwd_finalize_kernel, dim3(C), dim3(kThreads), 0, st, part, B, C, 1, 1, dbias, dbcast);
            LDM_CHECK_LAUNCH("act_bwd_finalize_kernel");
        }
        return 0;
    }
    const int Q = act_slices(B, C, HW);
    const float* aval = aval0;
    float* part = sums ? workspace : nullptr;
    const int vw = vec_width(HW, dy, aval, pre_act, dv);
    const int64_t S = slice_len(HW, Q, vw);
    const dim3 grid(Q, B * C);
    st_dispatch(sc, [&](auto stc) {
        w_dispatch(vw, [&](auto wc) {
            hipLaunchKernelGGL((act_bwd_kernel<decltype(wc)::value, decltype(stc)::value>), grid, dim3(kThreads), 0, st,
                               dy, aval, pre_act, act, sc.sf, C, HW, S, dv, part);
        });
    });
    LDM_CHECK_LAUNCH("act_bwd_kernel");
    if (sums && defer_q) {
        *defer_q = Q;
    } else if (sums) {
        hipLaunchKernelGGL(act_bwd_finalize_kernel, dim3(C), dim3(kThreads), 0, st, part, B, C, Q,
                           finalize_lanes(Q), dbias, dbcast);
        LDM_CHECK_LAUNCH("act_bwd_finalize_kernel");
    }
    return 0;
}

extern "C" int ldm_act_backward(const float* dy, const float* act_out, const float* pre_act, int32_t act_code,
                                int32_t B, int32_t C, int32_t HW, float* dv, float* dbias, float* dbcast, float* workspace,
                                void* stream) {
    return act_backward_impl(dy, act_out, pre_act, act_code, B, C, HW, dv, dbias, dbcast, workspace, nullptr, stream);
}

extern "C" int ldm_act_backward_defer(const float* dy, const float* act_out, const float* pre_act, int32_t act_code,
                                      int32_t B, int32_t C, int32_t HW, float* dv, float* dbias, float* workspace,
                                      int32_t* q_out, void* stream) {
    LDM_REQUIRE(q_out && dbias && workspace, "act_backward_defer: bad argument");
    return act_backward_impl(dy, act_out, pre_act, act_code, B, C, HW, dv, dbias, nullptr, workspace, q_out, stream);
}

extern "C" int64_t ldm_act_partial_floats(int32_t B, int32_t C, int32_t HW) {
    if (B <= 0 || C <= 0 || HW <= 0) return -1;
    return (int64_t)B * C * act_slices(B, C, HW) * 2;
}

extern "C" int ldm_act_finalize_many(const ldm_act_fin_job* jobs, int32_t n, void* stream) {
    LDM_REQUIRE(jobs && n >= 0, "act_finalize_many: bad argument");
    hipStream_t st = (hipStream_t)stream;
    for (int i0 = 0; i0 < n; i0 += kMaxFinJobs) {
        FinJobs fj{};
        int blocks = 0;
        fj.n = n - i0 < kMaxFinJobs ? n - i0 : kMaxFinJobs;
        for (int i = 0; i < fj.n; ++i) {
            const ldm_act_fin_job& J = jobs[i0 + i];
            LDM_REQUIRE(J.part && J.dbias && J.C > 0 && J.Q > 0 && (J.kind == 1 || (J.kind == 0 && J.B > 0)),
                        "act_finalize_many: bad job");
            fj.j[i] = FinJob{J.part, J.dbias, J.B, J.C, J.Q, finalize_lanes(J.Q), blocks, J.kind};
            blocks += J.C;
        }
        if (blocks == 0) continue;
        hipLaunchKernelGGL(act_bwd_finalize_many_kernel, dim3(blocks), dim3(kThreads), 0, st, fj);
        LDM_CHECK_LAUNCH("act_bwd_finalize_many_kernel");
    }
    return 0;
}
