// The reverse loop's bottleneck with CA1's values folded into its weights (UNet.forward, model.py:214-217).
//
// After CA1 the bottleneck reads a = concat_h(P_h V_h), P_h = softmax(z4 . kf_h + bf_h) [L = 16 queries x S = 16
// keys] on the 2 x 8 plane and V_h = Wv_h s6 + bv_h [S x d = 128] (fixed for the whole loop: the style maps and
// the weights do not change), through W' = W_bottleneck o Wo (the out-projection already folded,
// ldm_fold_conv_proj).  Re-associating the contraction over the head dimension d:
//
//   y[l, co] = sum_t sum_{ci} W'[co, ci, t] a[l_t, ci] + pb[l, co]
//            = sum_t sum_h sum_s P_h[l_t, s] U[co, t, h, s] + pb[l, co],   U[co, t, h, s] = sum_d W'[co, h d, t] V_h[s, d]
//
// (l_t = the input position tap t of output l reads; taps outside the plane read the zero padding of a, so they
// drop out; pb = the bias with bo carried through the taps inside the plane, uconv's step_pb[1]).  U is per
// sample (V is): 512 x (9 taps x 4 heads x 16 keys) = 576-deep rows, 1.18 MB per sample — at B <= 8 no more
// bytes than W' itself (9.4 MB), but the bottleneck becomes a K = 576 contraction per sample instead of
// K = 4608 shared over the batch: every block owns one sample's 16 x 16 output tile and streams 37 KB of U
// instead of the K-split uconv form's 147 KB of W' plus partial slabs, and the CA1 launch writes P only (no
// P V product).  U is formed once per loop (bneck_fold_values_kernel), like the folded keys.
#include <cstdlib>
#include <type_traits>

#include "common.h"

#pragma clang fp contract(off)

namespace ldm {
namespace bf {

constexpr int E = 512, HEADS = 4, DH = 128, S = 16, L = 16, TAPS = 9;
constexpr int K = TAPS * HEADS * S;   // 576: k = (t * HEADS + h) * S + s

// U[b][co][k] = sum_d W'[co][h*DH + d][t] * V[b][h][s][d]; kv = the style K/V projection [B][2E][S] (V rows
// E + h*DH + d, channel-major).  Block (b, h, 32-row co tile), 288 threads = 32 co x 9 taps, V_h staged in LDS.
__global__ __launch_bounds__(288) void bneck_fold_values_kernel(const float* __restrict__ wf, const float* __restrict__ kv,
                                                                float* __restrict__ u) {
    __shared__ float vs[DH][S];
    const int co0 = blockIdx.x * 32, h = blockIdx.y, b = blockIdx.z;
    const float* vb = kv + ((size_t)b * 2 * E + E + (size_t)h * DH) * S;
    for (int e = threadIdx.x; e < DH * S; e += blockDim.x) vs[e / S][e % S] = vb[e];
    __syncthreads();
    const int co = co0 + threadIdx.x / TAPS, t = threadIdx.x % TAPS;
    const float* wr = wf + ((size_t)co * E + (size_t)h * DH) * TAPS + t;
    float acc[S];
#pragma unroll
    for (int s = 0; s < S; ++s) acc[s] = 0.f;
    for (int d = 0; d < DH; ++d) {
        const float w = wr[(size_t)d * TAPS];
#pragma unroll
        for (int s = 0; s < S; ++s) acc[s] = fmaf(w, vs[d][s], acc[s]);
    }
    float4* out = reinterpret_cast<float4*>(u + ((size_t)b * E + co) * K + (size_t)(t * HEADS + h) * S);
#pragma unroll
    for (int q = 0; q < S / 4; ++q) out[q] = make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
}

// y[b][l][co] (NHWC on the 2 x 8 plane) = relu(sum_k U[b][co][k] B[k][l] + pb[l][co]), B[(t,h,s)][l] = P[b][h][l_t][s]
// (0 where tap t of l falls outside the plane).  Block = (16-row co tile, sample b); its NWV waves (9 by default) split
// the 36 chunks of 16 k (one (tap, head) pair each), all their operand loads in flight before the MFMAs
// (v_mfma_f32_16x16x4_f32: lane (row = l & 15, lg = l >> 4) holds A[row][4 lg + j] and B[4 lg + j][col = l & 15]
// for step j — one 16-byte load each per chunk), and meet in LDS in wave order.  DT != 0: the output is rounded to
// the 16-bit type, as the reference's autocast conv returns it (the operands stay fp32).
template <int DT, int NWV>
__global__ __launch_bounds__(64 * NWV) void bneck_pv_kernel(const float* __restrict__ u, const float* __restrict__ p,
                                                            const float* __restrict__ pb, float* __restrict__ y) {
    constexpr int NCH = K / 16, PER = NCH / NWV;   // 36 chunks, PER per wave
    static_assert(NCH % NWV == 0, "chunks per wave");
    __shared__ floatx4 red[NWV][64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int row = lane & 15, lg = lane >> 4;
    const int co0 = blockIdx.x * 16, b = blockIdx.y;
    const int l = lane & 15, oy = l >> 3, ox = l & 7;
    const floatx4* ua = reinterpret_cast<const floatx4*>(u + ((size_t)b * E + co0 + row) * K) + lg;
    const float* pbb = p + (size_t)b * HEADS * L * S;
    floatx4 fa[PER], fb[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int c = wave * PER + i;   // chunk = (tap, head)
        fa[i] = ua[c * 4];
        const int t = c / HEADS, h = c % HEADS;
        const int iy = oy - 1 + t / 3, ix = ox - 1 + t % 3;
        const bool in = (unsigned)iy < 2u && (unsigned)ix < 8u;
        const floatx4 v = *reinterpret_cast<const floatx4*>(pbb + ((size_t)h * L + (in ? iy * 8 + ix : 0)) * S + 4 * lg);
        fb[i] = in ? v : floatx4{0.f, 0.f, 0.f, 0.f};
    }
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < PER; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][j], fb[i][j], acc, 0, 0, 0);
    red[wave][lane] = acc;
    __syncthreads();
    if (wave != 0) return;
    floatx4 v = red[0][lane];
#pragma unroll
    for (int w = 1; w < NWV; ++w) v = v + red[w][lane];
    const int co = co0 + 4 * lg;   // D rows 4 lg + r, column l
    const floatx4 bias = *reinterpret_cast<const floatx4*>(pb + (size_t)l * E + co);
    floatx4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float sv = round16(v[r] + bias[r], DT);
        o[r] = sv < 0.f ? 0.f : sv;
    }
    *reinterpret_cast<floatx4*>(y + ((size_t)b * L + l) * E + co) = o;
}

// CA1's probabilities alone, one block of eight waves per (sample, head) (round 5) — the scores' E = 512 contraction split over the eight waves (v_mfma_f32_16x16x4_f32,
// two 16-byte loads per lane per 16 e), the partial score tiles summed in wave order in LDS, the bias and the
// softmax over the 16 keys by wave 0, P stored with plain stores (the next launch reads it).  The generic
// attention kernel's PONLY instance runs the same contraction through its query / key staging.
__global__ __launch_bounds__(512) void ca1_probs_kernel(const float* __restrict__ z, const float* __restrict__ kf,
                                                         const float* __restrict__ bfv, float* __restrict__ p) {
    __shared__ floatx4 red[8][64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int col = lane & 15, lg = lane >> 4;
    const int b = blockIdx.x / HEADS, h = blockIdx.x % HEADS;
    const int e0 = wave * (E / 8);
    const float* za = z + ((size_t)b * L + col) * E + e0 + 4 * lg;
    const float* ka = kf + (((size_t)b * HEADS + h) * S + col) * E + e0 + 4 * lg;
    floatx4 zz[4], kk[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        zz[i] = *reinterpret_cast<const floatx4*>(za + 16 * i);
        kk[i] = *reinterpret_cast<const floatx4*>(ka + 16 * i);
    }
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(zz[i][j], kk[i][j], acc, 0, 0, 0);
    red[wave][lane] = acc;
    __syncthreads();
    if (wave != 0) return;
    floatx4 v = red[0][lane];
#pragma unroll
    for (int w = 1; w < 8; ++w) v = v + red[w][lane];
    const float bias = bfv[((size_t)b * HEADS + h) * S + col];
    float* pb = p + ((size_t)(b * HEADS + h) * L) * S;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float x = v[r] + bias;
        float mx = x;
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
        const float ex = expf(x - mx);
        float sum = ex;
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
        pb[(size_t)(4 * lg + r) * S + col] = ex / sum;
    }
}

}  // namespace bf

// The fold applies on the canonical 2 x 8 bottleneck plane while U is no larger than W' (B <= 8);
// LDM_BNECK_FOLD=0 keeps CA1 + the uconv bottleneck (A/B timing).
bool bneck_fold_supported(int B, int H, int W) {
    static const bool on = [] {
        const char* e = std::getenv("LDM_BNECK_FOLD");
        return !e || std::atoi(e) != 0;
    }();
    return on && B >= 1 && B <= 8 && H / 8 == 2 && W / 8 == 8 && H % 8 == 0 && W % 8 == 0;
}

int bneck_fold_values(const float* wf, const float* kv, float* u, int B, hipStream_t st) {
    LDM_REQUIRE(wf && kv && u && B > 0, "bottleneck fold values: bad argument");
    hipLaunchKernelGGL(bf::bneck_fold_values_kernel, dim3(bf::E / 32, bf::HEADS, B), dim3(288), 0, st, wf, kv, u);
    LDM_CHECK_LAUNCH("bneck_fold_values_kernel");
    return 0;
}

int bneck_pv(const float* u, const float* p, const float* pb, float* y, int B, int dtype, hipStream_t st) {
    LDM_REQUIRE(u && p && pb && y && B > 0, "bottleneck (folded values): bad argument");
    LDM_REQUIRE((((uintptr_t)u | (uintptr_t)p | (uintptr_t)pb | (uintptr_t)y) & 15) == 0,
                "bottleneck (folded values): operands must be 16-byte aligned");
    LDM_REQUIRE(dtype >= LDM_DT_F32 && dtype <= LDM_DT_BF16, "bottleneck (folded values): unknown operand precision");
    // waves per block splitting the 36 chunks (LDM_BNECK_WAVES: 4, 6, 9 or 12).  Measured in the loop
    // (gpurun_out/ab1, two rounds): 4 waves 75.30 / 75.34 us per iteration, 6: 74.08 / 73.84, 9: 73.48 / 73.22,
    // 12: 73.48 / 73.55 — more loads in flight per CU; 9 (four chunks per wave) kept
    static const int nwv = [] {
        const char* e = std::getenv("LDM_BNECK_WAVES");
        const int v = e ? std::atoi(e) : 9;
        return (v == 4 || v == 6 || v == 12) ? v : 9;
    }();
    const dim3 grid(bf::E / 16, B);
    auto go = [&](auto dtc, auto nwc) {
        constexpr int DT = decltype(dtc)::value, NW = decltype(nwc)::value;
        hipLaunchKernelGGL((bf::bneck_pv_kernel<DT, NW>), grid, dim3(64 * NW), 0, st, u, p, pb, y);
    };
    auto by_waves = [&](auto dtc) {
        switch (nwv) {
            case 6: go(dtc, std::integral_constant<int, 6>{}); break;
            case 9: go(dtc, std::integral_constant<int, 9>{}); break;
            case 12: go(dtc, std::integral_constant<int, 12>{}); break;
            default: go(dtc, std::integral_constant<int, 4>{}); break;
        }
    };
    if (dtype == LDM_DT_F16) by_waves(std::integral_constant<int, LDM_DT_F16>{});
    else if (dtype == LDM_DT_BF16) by_waves(std::integral_constant<int, LDM_DT_BF16>{});
    else by_waves(std::integral_constant<int, 0>{});
    LDM_CHECK_LAUNCH("bneck_pv_kernel");
    return 0;
}

// CA1's probabilities on ca1_probs_kernel (LDM_CA1P_FORM=0: the generic attention kernel's PONLY instance)
bool ca1_probs_own() {
    static const bool on = [] {
        const char* e = std::getenv("LDM_CA1P_FORM");
        return !e || std::atoi(e) != 0;
    }();
    return on;
}

int ca1_probs(const float* z, const float* kf, const float* bfv, float* p, int B, hipStream_t st) {
    LDM_REQUIRE(z && kf && bfv && p && B > 0, "CA1 probabilities: bad argument");
    LDM_REQUIRE((((uintptr_t)z | (uintptr_t)kf) & 15) == 0, "CA1 probabilities: operands must be 16-byte aligned");
    hipLaunchKernelGGL(bf::ca1_probs_kernel, dim3(B * bf::HEADS), dim3(512), 0, st, z, kf, bfv, p);
    LDM_CHECK_LAUNCH("ca1_probs_kernel");
    return 0;
}

}  // namespace ldm

extern "C" int32_t ldm_bneck_fold_supported(int32_t B, int32_t H, int32_t W) {
    return ldm::bneck_fold_supported(B, H, W) ? 1 : 0;
}

extern "C" int ldm_bneck_fold_values(const float* w_fold, const float* kv, float* u, int32_t B, void* stream) {
    return ldm::bneck_fold_values(w_fold, kv, u, B, (hipStream_t)stream);
}

extern "C" int ldm_bneck_pv(const float* u, const float* p, const float* pos_bias, float* y, int32_t B, int32_t dtype,
                            void* stream) {
    return ldm::bneck_pv(u, p, pos_bias, y, B, dtype, (hipStream_t)stream);
}

extern "C" int ldm_ca1_probs(const float* z4, const float* kf, const float* bf, float* p, int32_t B, void* stream) {
    return ldm::ca1_probs(z4, kf, bf, p, B, (hipStream_t)stream);
}

extern "C" int32_t ldm_ca1_probs_form(void) { return ldm::ca1_probs_own() ? 1 : 0; }
