// The VGGish style / feature loss of the train step (reference loss.py:52-101,
// VGGishFeatureLoss.forward, called as style_loss at train.py:183): the conv stack itself runs on the conv
// kernels (conv.hip, ReLU fused into the epilogue, so every conv launch yields one feature tap); this file
// holds what is left of the path:
//   * nn.MaxPool2d(2, 2) on NCHW (floor mode, NaN-propagating like torch's max_pool2d): one float2 x 2
//     rows per output pair, HBM-bound (read 16 B, write 8 B per output pair);
//   * the std-normalised MSE of one tap,  mse(p / (std(p) + eps), t / (std(t) + eps))  with torch.std's
//     per-sample unbiased std over (C, H, W): ONE pass over p and t collects the per-sample fp64 moments
//     (sum p, sum p^2, sum t, sum t^2, sum p*t) and the loss is their closed form
//       sum_i (p_i/a - t_i/b)^2 = Sp2/a^2 - 2 Spt/(a b) + St2/b^2     (a, b per sample)
//     -- the reference's two normalised copies and the squared difference are never materialised.
// Reductions are sliced (fixed slices per sample, fixed block order, fp64): bitwise reproducible.
#include "common.h"

namespace ldm {
namespace {

constexpr int kT = 256;

__device__ __forceinline__ float max_nan(float a, float b) { return (a > b || a != a) ? a : b; }

__global__ __launch_bounds__(kT) void maxpool2x2_kernel(const float* __restrict__ x, float* __restrict__ y, int H,
                                                        int W, int Ho, int Wo, int64_t planes, int vec) {
    const int64_t Wp = vec ? (Wo >> 1) : Wo;                    // lanes per output row
    const int64_t total = planes * Ho * Wp;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t pr = i / Wp;
        const int ox = (int)(i - pr * Wp) * (vec ? 2 : 1);
        const int64_t pl = pr / Ho;
        const int oy = (int)(pr - pl * Ho);
        const float* r0 = x + (pl * H + 2 * oy) * W + 2 * ox;
        const float* r1 = r0 + W;
        float* o = y + (pl * Ho + oy) * Wo + ox;
        if (vec) {   // two outputs from one float4 of each input row
            const float4 a = *reinterpret_cast<const float4*>(r0);
            const float4 b = *reinterpret_cast<const float4*>(r1);
            float2 v;
            v.x = max_nan(max_nan(a.x, a.y), max_nan(b.x, b.y));
            v.y = max_nan(max_nan(a.z, a.w), max_nan(b.z, b.w));
            *reinterpret_cast<float2*>(o) = v;
        } else {
            o[0] = max_nan(max_nan(r0[0], r0[1]), max_nan(r1[0], r1[1]));
        }
    }
}

// slices per sample for the moment pass: >= ~1024 blocks in all, >= 4096 elements per slice
inline int mom_slices(int B, int64_t n) {
    int64_t p = (1024 + B - 1) / B;
    const int64_t by_len = (n + 4095) / 4096;
    if (p > by_len) p = by_len;
    if (p < 1) p = 1;
    return (int)p;
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double s = 0.0;
    for (int w = 0; w < kT / 64; ++w) s += red[w];
    return s;
}

// part[b][k][5] over slice k of sample b: sum p, sum p^2, sum t, sum t^2, sum p*t
__global__ __launch_bounds__(kT) void std_mse_partial_kernel(const float* __restrict__ p, const float* __restrict__ t,
                                                             int64_t n, int64_t S, int vec,
                                                             double* __restrict__ part) {
    __shared__ double red[kT / 64];
    const int k = blockIdx.x, b = blockIdx.y, P = gridDim.x;
    const int64_t e0 = (int64_t)k * S, e1 = min(e0 + S, n);
    const float* pb = p + (size_t)b * n;
    const float* tb = t + (size_t)b * n;
    double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    auto acc = [&](float pv, float tv) {
        const double dp = pv, dt = tv;
        s[0] += dp;
        s[1] += dp * dp;
        s[2] += dt;
        s[3] += dt * dt;
        s[4] += dp * dt;
    };
    if (vec) {   // e0 is a multiple of 4 (S is), so are the sample bases (n % 4 == 0)
        for (int64_t i = e0 + 4 * (int64_t)threadIdx.x; i < e1; i += 4 * kT) {
            const float4 a = *reinterpret_cast<const float4*>(pb + i);
            const float4 c = *reinterpret_cast<const float4*>(tb + i);
            acc(a.x, c.x);
            acc(a.y, c.y);
            acc(a.z, c.z);
            acc(a.w, c.w);
        }
    } else {
        for (int64_t i = e0 + threadIdx.x; i < e1; i += kT) acc(pb[i], tb[i]);
    }
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const double v = block_sum_d(s[j], red);
        if (threadIdx.x == 0) part[((size_t)b * P + k) * 5 + j] = v;
    }
}

// moments[b][j] = sum_k part[b][k][j] (slices in order)
__global__ void std_mse_finalize_kernel(const double* __restrict__ part, int B, int P, double* __restrict__ mom) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * 5) return;
    const int b = i / 5, j = i - b * 5;
    double s = 0.0;
    for (int k = 0; k < P; ++k) s += part[((size_t)b * P + k) * 5 + j];
    mom[i] = s;
}

// acc += scale * mean over (B, n) of (p/a - t/b)^2, a = std(p_b) + eps (unbiased); out = (float)acc
__global__ void std_mse_accumulate_kernel(const double* __restrict__ mom, int B, int64_t n, double eps, double scale,
                                          double* __restrict__ acc, float* __restrict__ out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const double N = (double)n;
    double tot = 0.0;
    for (int b = 0; b < B; ++b) {
        const double* m = mom + (size_t)b * 5;
        double vp = (m[1] - m[0] * m[0] / N) / (N - 1.0);
        double vt = (m[3] - m[2] * m[2] / N) / (N - 1.0);
        vp = vp > 0.0 ? vp : 0.0;
        vt = vt > 0.0 ? vt : 0.0;
        const double a = sqrt(vp) + eps, c = sqrt(vt) + eps;
        tot += m[1] / (a * a) - 2.0 * m[4] / (a * c) + m[3] / (c * c);
    }
    acc[0] += scale * (tot / ((double)B * N));
    if (out) out[0] = (float)acc[0];
}

}  // namespace
}  // namespace ldm

using namespace ldm;

extern "C" int ldm_maxpool2x2(const float* x, float* y, int32_t B, int32_t C, int32_t H, int32_t W, void* stream) {
    LDM_REQUIRE(x && y && B > 0 && C > 0 && H >= 2 && W >= 2, "maxpool2x2: bad argument");
    const int Ho = H / 2, Wo = W / 2;
    const int64_t planes = (int64_t)B * C;
    const int vec = (W % 4 == 0 && Wo % 2 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 7) == 0) ? 1 : 0;
    const int64_t lanes = planes * Ho * (vec ? Wo / 2 : Wo);
    const unsigned blocks = (unsigned)std::min<int64_t>((lanes + kT - 1) / kT, 65536);
    hipLaunchKernelGGL(maxpool2x2_kernel, dim3(blocks), dim3(kT), 0, (hipStream_t)stream, x, y, H, W, Ho, Wo, planes,
                       vec);
    LDM_CHECK_LAUNCH("maxpool2x2_kernel");
    return 0;
}

extern "C" int64_t ldm_std_mse_workspace_floats(int32_t B, int64_t n) {
    if (B <= 0 || n <= 0) return 0;
    return (int64_t)B * mom_slices(B, n) * 5 * 2;   // doubles -> floats
}

extern "C" int ldm_std_mse_moments(const float* p, const float* t, int32_t B, int64_t n, double* moments,
                                   float* workspace, void* stream) {
    LDM_REQUIRE(p && t && moments && workspace && B > 0 && n > 1, "std_mse_moments: bad argument");
    LDM_REQUIRE(((uintptr_t)workspace & 7) == 0, "std_mse_moments: workspace must be 8-byte aligned");
    const int P = mom_slices(B, n);
    const int64_t S = ((n + P - 1) / P + 3) & ~(int64_t)3;
    const int vec = (n % 4 == 0 && ((uintptr_t)p & 15) == 0 && ((uintptr_t)t & 15) == 0) ? 1 : 0;
    double* part = reinterpret_cast<double*>(workspace);
    hipLaunchKernelGGL(std_mse_partial_kernel, dim3(P, B), dim3(kT), 0, (hipStream_t)stream, p, t, n, S, vec, part);
    LDM_CHECK_LAUNCH("std_mse_partial_kernel");
    hipLaunchKernelGGL(std_mse_finalize_kernel, dim3((B * 5 + 255) / 256), dim3(256), 0, (hipStream_t)stream, part, B,
                       P, moments);
    LDM_CHECK_LAUNCH("std_mse_finalize_kernel");
    return 0;
}

extern "C" int ldm_std_mse_accumulate(const double* moments, int32_t B, int64_t n, double eps, double scale,
                                      double* acc, float* out, void* stream) {
    LDM_REQUIRE(moments && acc && B > 0 && n > 1, "std_mse_accumulate: bad argument");
    hipLaunchKernelGGL(std_mse_accumulate_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, moments, B, n, eps, scale,
                       acc, out);
    LDM_CHECK_LAUNCH("std_mse_accumulate_kernel");
    return 0;
}
