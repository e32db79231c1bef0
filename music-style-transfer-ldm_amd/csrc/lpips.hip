// LPIPS-AlexNet perceptual distance (reference loss.py:6-21: perceptual_loss_old builds lpips==0.1.4
// LPIPS(net='alex') and takes LPIPS(2x-1, 2y-1).mean(); the compression loss' 0.1-weighted term, the only
// perceptual term that carries gradient in the reference's train steps).  SURVEY §8(f) row 2.
//
// The AlexNet convolutions run on the conv kernels (conv.hip / tconv.hip, ReLU fused): the 3x3 layers
// directly, the 11x11 / stride-4 and 5x5 layers as explicit im2col + one 1x1 implicit GEMM (their windows
// exceed the phase tables' 16 taps), whose data gradient is the 1x1 dual conv + col2im here.  This file holds
// the rest, all fp32, deterministic (gathers, fixed-order fp64 reductions):
//   * im2col with the LPIPS ScalingLayer fused: a 1-channel mel in [0,1] -> t = 2x - 1 (perceptual_loss_old)
//     -> v_c = (t - shift_c) / scale_c broadcast to the 3 "RGB" channels (lpips ScalingLayer), zero padding
//     applied after the scaling as the conv pads the scaled tensor; col2im gathers the taps back and
//     folds d v_c / d x = 2 / scale_c summed over the broadcast channels;
//   * nn.MaxPool2d(3, 2) (floor) and its backward as a gather over the windows whose first-occurrence argmax
//     (torch's CPU rule: strictly greater, NaN wins) is the input pixel;
//   * one LPIPS layer: normalize_tensor over channels (x / (sqrt(sum x^2) + 1e-10)), squared difference, the
//     1x1 "lin" head (no bias), spatial mean -> added to val[b]; and its backward to either feature map,
//     following torch autograd's expression order (so an all-zero feature pixel gives NaN like torch's
//     sqrt backward does).
#include <cmath>

#include "common.h"

namespace ldm {
namespace {

constexpr int kT = 256;

__device__ __forceinline__ float lp_in(const float* x, int unit) {
#pragma clang fp contract(off)
    const float v = *x;
    if (!unit) return v;
    const float t = 2.0f * v;   // 2 * original - 1   (loss.py:17-18)
    return t - 1.0f;
}

// col[b][k][oy][ox], k = (c*kh + ky)*kw + kx (the torch weight [Cout][Cin][kh][kw] flattened), k >= Cv*kh*kw: 0
__global__ __launch_bounds__(kT) void im2col_kernel(const float* __restrict__ x, int C, int H, int W, int kh, int kw,
                                                    int stride, int pad, int Ho, int Wo, int Kpad,
                                                    const float* __restrict__ shift, const float* __restrict__ scale,
                                                    int Cv, int unit, float* __restrict__ col, int64_t n) {
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int P = Ho * Wo;
    const int p = (int)(i % P);
    const int64_t r = i / P;
    const int k = (int)(r % Kpad);
    const int64_t b = r / Kpad;
    float v = 0.f;
    if (k < Cv * kh * kw) {
        const int kx = k % kw, ky = (k / kw) % kh, c = k / (kw * kh);
        const int oy = p / Wo, ox = p % Wo;
        const int iy = oy * stride - pad + ky, ix = ox * stride - pad + kx;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
            const int cs = (shift && C == 1) ? 0 : c;   // a 1-channel mel broadcasts over the 3 channels
            const float t = lp_in(x + ((b * C + cs) * H + iy) * (int64_t)W + ix, unit);
            v = shift ? (t - shift[c]) / scale[c] : t;   // ScalingLayer: (inp - shift) / scale
        }
    }
    col[i] = v;
}

// dx[b][c][iy][ix] = sum over the taps whose window covers (iy, ix) of dcol (x d/dx of the fused transform)
__global__ __launch_bounds__(kT) void col2im_kernel(const float* __restrict__ col, int C, int H, int W, int kh, int kw,
                                                    int stride, int pad, int Ho, int Wo, int Kpad,
                                                    const float* __restrict__ scale, int Cv, int unit,
                                                    float* __restrict__ dx, int64_t n) {
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int ix = (int)(i % W);
    const int iy = (int)((i / W) % H);
    const int c = (int)((i / ((int64_t)W * H)) % C);
    const int64_t b = i / ((int64_t)W * H * C);
    const int P = Ho * Wo;
    const float* cb = col + b * Kpad * (int64_t)P;
    const bool bcast = scale && C == 1;
    const int c0 = bcast ? 0 : c, c1 = bcast ? Cv : c + 1;
    float acc = 0.f;
    for (int cv = c0; cv < c1; ++cv) {
        float g = 0.f;
        for (int ky = 0; ky < kh; ++ky) {
            const int ty = iy + pad - ky;
            if (ty < 0 || ty % stride) continue;
            const int oy = ty / stride;
            if (oy >= Ho) continue;
            for (int kx = 0; kx < kw; ++kx) {
                const int tx = ix + pad - kx;
                if (tx < 0 || tx % stride) continue;
                const int ox = tx / stride;
                if (ox >= Wo) continue;
                g += cb[(int64_t)((cv * kh + ky) * kw + kx) * P + oy * Wo + ox];
            }
        }
        acc += scale ? g / scale[cv] : g;   // d((t - shift)/scale)/dt = 1/scale, summed over the broadcast
    }
    dx[i] = unit ? 2.0f * acc : acc;        // d(2x - 1)/dx
}

__device__ __forceinline__ bool gt_nan(float v, float m) { return v > m || v != v; }

__global__ __launch_bounds__(kT) void maxpool3s2_kernel(const float* __restrict__ x, float* __restrict__ y, int H, int W,
                                                        int Ho, int Wo, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int ox = (int)(i % Wo);
    const int oy = (int)((i / Wo) % Ho);
    const int64_t pl = i / ((int64_t)Wo * Ho);
    const float* xp = x + (pl * H + 2 * oy) * (int64_t)W + 2 * ox;
    float m = xp[0];
    for (int ky = 0; ky < 3; ++ky)
        for (int kx = 0; kx < 3; ++kx) {
            const float v = xp[ky * W + kx];
            if (gt_nan(v, m)) m = v;
        }
    y[i] = m;
}

// dx[p] = sum of dy over the windows (<= 4 per axis pair) whose first-occurrence argmax is p
__global__ __launch_bounds__(kT) void maxpool3s2_backward_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                                 float* __restrict__ dx, int H, int W, int Ho, int Wo,
                                                                 int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int ix = (int)(i % W);
    const int iy = (int)((i / W) % H);
    const int64_t pl = i / ((int64_t)W * H);
    const float* xb = x + pl * H * (int64_t)W;
    float g = 0.f;
    for (int oy = max(0, (iy - 1) / 2); oy <= min(Ho - 1, iy / 2); ++oy) {
        if (iy < 2 * oy || iy > 2 * oy + 2) continue;
        for (int ox = max(0, (ix - 1) / 2); ox <= min(Wo - 1, ix / 2); ++ox) {
            if (ix < 2 * ox || ix > 2 * ox + 2) continue;
            const float* xp = xb + (2 * oy) * (int64_t)W + 2 * ox;
            float m = xp[0];
            int am = 0;
            for (int ky = 0; ky < 3; ++ky)
                for (int kx = 0; kx < 3; ++kx) {
                    const float v = xp[ky * W + kx];
                    if (gt_nan(v, m)) {
                        m = v;
                        am = ky * 3 + kx;
                    }
                }
            if (am == (iy - 2 * oy) * 3 + (ix - 2 * ox)) g += dy[(pl * Ho + oy) * (int64_t)Wo + ox];
        }
    }
    dx[i] = g;
}

// d[b][p] = sum_c w_c (f0_c/(|f0|+eps) - f1_c/(|f1|+eps))^2 over channels c (stride HW)
__global__ __launch_bounds__(kT) void lpips_dist_kernel(const float* __restrict__ f0, const float* __restrict__ f1,
                                                        const float* __restrict__ w, int C, int HW,
                                                        float* __restrict__ d, int64_t n) {
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int p = (int)(i % HW);
    const int64_t b = i / HW;
    const float* a0 = f0 + b * C * (int64_t)HW + p;
    const float* a1 = f1 + b * C * (int64_t)HW + p;
    float s0 = 0.f, s1 = 0.f;
    for (int c = 0; c < C; ++c) {
        const float u = a0[(int64_t)c * HW], v = a1[(int64_t)c * HW];
        s0 += u * u;
        s1 += v * v;
    }
    const float n0 = sqrtf(s0) + 1e-10f, n1 = sqrtf(s1) + 1e-10f;   // normalize_tensor, eps 1e-10
    float acc = 0.f;
    for (int c = 0; c < C; ++c) {
        const float df = a0[(int64_t)c * HW] / n0 - a1[(int64_t)c * HW] / n1;
        acc += w[c] * (df * df);
    }
    d[i] = acc;
}

// val[b] += mean_p d[b][p]  (one block per sample, fp64 fixed-order sum)
__global__ __launch_bounds__(kT) void lpips_mean_kernel(const float* __restrict__ d, int HW, float* __restrict__ val) {
    __shared__ double red[kT / 64];
    const int b = blockIdx.x;
    double s = 0.0;
    for (int p = threadIdx.x; p < HW; p += kT) s += (double)d[(int64_t)b * HW + p];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < kT / 64; ++w) t += red[w];
        val[b] = val[b] + (float)(t / (double)HW);
    }
}

// gradient of val[b] (upstream gval[b]) w.r.t. f1 (side 1) or f0 (side 0) of one layer, accumulated into df
// (accumulate) or written.  With n = sqrt(s) and q = f / (n + eps):
//   dq_c = gval/HW * w_c * 2 (a_c - b_c) * (side 0 ? +1 : -1)
//   df_k = dq_k / (n + eps) + f_k * ( -(sum_c dq_c f_c) / (n + eps)^2 ) / n     (torch's chain: /, +, sqrt, pow)
__global__ __launch_bounds__(kT) void lpips_dist_backward_kernel(const float* __restrict__ f0, const float* __restrict__ f1,
                                                                 const float* __restrict__ w, const float* __restrict__ gval,
                                                                 int C, int HW, int side, int accumulate,
                                                                 float* __restrict__ df, int64_t n) {
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int p = (int)(i % HW);
    const int64_t b = i / HW;
    const float* a0 = f0 + b * C * (int64_t)HW + p;
    const float* a1 = f1 + b * C * (int64_t)HW + p;
    float s0 = 0.f, s1 = 0.f;
    for (int c = 0; c < C; ++c) {
        const float u = a0[(int64_t)c * HW], v = a1[(int64_t)c * HW];
        s0 += u * u;
        s1 += v * v;
    }
    const float r0 = sqrtf(s0), r1 = sqrtf(s1);
    const float n0 = r0 + 1e-10f, n1 = r1 + 1e-10f;
    const float gd = gval[b] / (float)HW;
    const float* fs = side ? a1 : a0;
    const float ns = side ? n1 : n0, rs = side ? r1 : r0;
    float dot = 0.f;
    for (int c = 0; c < C; ++c) {
        const float df_ = a0[(int64_t)c * HW] / n0 - a1[(int64_t)c * HW] / n1;
        float dq = gd * w[c] * 2.0f * df_;
        if (side) dq = -dq;
        dot += dq * fs[(int64_t)c * HW];
    }
    const float dn = -dot / (ns * ns);         // d/dn of f / (n + eps)
    const float ds = dn / (2.0f * rs);          // sqrt backward (NaN at an all-zero pixel, as torch)
    float* o = df + b * C * (int64_t)HW + p;
    for (int c = 0; c < C; ++c) {
        const float df_ = a0[(int64_t)c * HW] / n0 - a1[(int64_t)c * HW] / n1;
        float dq = gd * w[c] * 2.0f * df_;
        if (side) dq = -dq;
        const float fk = fs[(int64_t)c * HW];
        const float g = dq / ns + 2.0f * fk * ds;
        o[(int64_t)c * HW] = accumulate ? o[(int64_t)c * HW] + g : g;
    }
}

unsigned nb(int64_t n) { return (unsigned)((n + kT - 1) / kT); }

}  // namespace
}  // namespace ldm

using namespace ldm;

extern "C" int ldm_im2col(const float* x, int32_t B, int32_t C, int32_t H, int32_t W, int32_t kh, int32_t kw,
                          int32_t stride, int32_t pad, int32_t Kpad, const float* shift, const float* scale, int32_t Cv,
                          int32_t unit, float* col, void* stream) {
    LDM_REQUIRE(x && col && B > 0 && C > 0 && H > 0 && W > 0 && kh > 0 && kw > 0 && stride > 0 && pad >= 0,
                "im2col: bad argument");
    LDM_REQUIRE(!shift == !scale && (!shift || C == 1 || C == Cv), "im2col: scaling layer needs C = 1 or C = Cv");
    const int cv = shift ? Cv : C;
    LDM_REQUIRE(cv > 0 && Kpad >= cv * kh * kw, "im2col: Kpad below C*kh*kw");
    const int Ho = (H + 2 * pad - kh) / stride + 1, Wo = (W + 2 * pad - kw) / stride + 1;
    LDM_REQUIRE(Ho > 0 && Wo > 0, "im2col: empty output");
    const int64_t n = (int64_t)B * Kpad * Ho * Wo;
    hipLaunchKernelGGL(im2col_kernel, dim3(nb(n)), dim3(kT), 0, (hipStream_t)stream, x, C, H, W, kh, kw, stride, pad, Ho,
                       Wo, Kpad, shift, scale, cv, unit, col, n);
    LDM_CHECK_LAUNCH("im2col_kernel");
    return 0;
}

extern "C" int ldm_col2im(const float* col, int32_t B, int32_t C, int32_t H, int32_t W, int32_t kh, int32_t kw,
                          int32_t stride, int32_t pad, int32_t Kpad, const float* scale, int32_t Cv, int32_t unit,
                          float* dx, void* stream) {
    LDM_REQUIRE(col && dx && B > 0 && C > 0 && H > 0 && W > 0 && kh > 0 && kw > 0 && stride > 0 && pad >= 0,
                "col2im: bad argument");
    LDM_REQUIRE(!scale || C == 1 || C == Cv, "col2im: scaling layer needs C = 1 or C = Cv");
    const int cv = scale ? Cv : C;
    LDM_REQUIRE(cv > 0 && Kpad >= cv * kh * kw, "col2im: Kpad below C*kh*kw");
    const int Ho = (H + 2 * pad - kh) / stride + 1, Wo = (W + 2 * pad - kw) / stride + 1;
    const int64_t n = (int64_t)B * C * H * W;
    hipLaunchKernelGGL(col2im_kernel, dim3(nb(n)), dim3(kT), 0, (hipStream_t)stream, col, C, H, W, kh, kw, stride, pad,
                       Ho, Wo, Kpad, scale, cv, unit, dx, n);
    LDM_CHECK_LAUNCH("col2im_kernel");
    return 0;
}

extern "C" int ldm_maxpool3s2(const float* x, float* y, int32_t B, int32_t C, int32_t H, int32_t W, void* stream) {
    LDM_REQUIRE(x && y && B > 0 && C > 0 && H >= 3 && W >= 3, "maxpool3s2: bad argument");
    const int Ho = (H - 3) / 2 + 1, Wo = (W - 3) / 2 + 1;
    const int64_t n = (int64_t)B * C * Ho * Wo;
    hipLaunchKernelGGL(maxpool3s2_kernel, dim3(nb(n)), dim3(kT), 0, (hipStream_t)stream, x, y, H, W, Ho, Wo, n);
    LDM_CHECK_LAUNCH("maxpool3s2_kernel");
    return 0;
}

extern "C" int ldm_maxpool3s2_backward(const float* x, const float* dy, float* dx, int32_t B, int32_t C, int32_t H,
                                       int32_t W, void* stream) {
    LDM_REQUIRE(x && dy && dx && B > 0 && C > 0 && H >= 3 && W >= 3, "maxpool3s2_backward: bad argument");
    const int Ho = (H - 3) / 2 + 1, Wo = (W - 3) / 2 + 1;
    const int64_t n = (int64_t)B * C * H * W;
    hipLaunchKernelGGL(maxpool3s2_backward_kernel, dim3(nb(n)), dim3(kT), 0, (hipStream_t)stream, x, dy, dx, H, W, Ho,
                       Wo, n);
    LDM_CHECK_LAUNCH("maxpool3s2_backward_kernel");
    return 0;
}

extern "C" int ldm_lpips_layer(const float* f0, const float* f1, const float* w, int32_t B, int32_t C, int32_t HW,
                               float* val, float* workspace, void* stream) {
    LDM_REQUIRE(f0 && f1 && w && val && workspace && B > 0 && C > 0 && HW > 0, "lpips_layer: bad argument");
    const int64_t n = (int64_t)B * HW;
    hipLaunchKernelGGL(lpips_dist_kernel, dim3(nb(n)), dim3(kT), 0, (hipStream_t)stream, f0, f1, w, C, HW, workspace, n);
    LDM_CHECK_LAUNCH("lpips_dist_kernel");
    hipLaunchKernelGGL(lpips_mean_kernel, dim3(B), dim3(kT), 0, (hipStream_t)stream, workspace, HW, val);
    LDM_CHECK_LAUNCH("lpips_mean_kernel");
    return 0;
}

extern "C" int ldm_lpips_layer_backward(const float* f0, const float* f1, const float* w, const float* gval, int32_t B,
                                        int32_t C, int32_t HW, int32_t side, int32_t accumulate, float* df,
                                        void* stream) {
    LDM_REQUIRE(f0 && f1 && w && gval && df && B > 0 && C > 0 && HW > 0 && (side == 0 || side == 1),
                "lpips_layer_backward: bad argument");
    const int64_t n = (int64_t)B * HW;
    hipLaunchKernelGGL(lpips_dist_backward_kernel, dim3(nb(n)), dim3(kT), 0, (hipStream_t)stream, f0, f1, w, gval, C, HW,
                       side, accumulate, df, n);
    LDM_CHECK_LAUNCH("lpips_dist_backward_kernel");
    return 0;
}
