// Backward kernels of the LDM train step (LDMTrainer.train_step, train.py:163-208): conv weight
// gradients, activation / bias / time-embedding gradients, train-mode BatchNorm backward,
// cross-attention backward, and the Adam update with GradScaler semantics (train.py:156-157,189-201).
// Data gradients of convs reuse the forward implicit-GEMM kernel (conv <-> transposed conv duality).
// Every reduction has a fixed partition and order: results are bitwise reproducible run to run.
#include <algorithm>
#include <cstdlib>

#include "common.h"

#pragma clang fp contract(off)

namespace ldm {

// ================================================================================================
// weight gradient:  out[m][c][t] = sum_{b,q} Dense[b][m][q] * Gath[b][c][q*s + d_t]
//   conv  (w [Cout][Cin][k][k]):  Dense = dY (m = co, q over Hout x Wout), Gath = X,  s = stride
//   convT (w [Cin][Cout][k][k]):  Dense = X  (m = ci, q over Hin  x Win ), Gath = dY, s = stride
//   d_t = (kh - pad, kw - pad); out-of-window gathers are 0.
// GEMM M = m, N = C*T, K = B*Hq*Wq on v_mfma_f32_16x16x4_f32.  A 16-deep K chunk is 16 consecutive q
// of one sample; lane group g holds k = 4g + j at MFMA step j (A arrives as one float4 per lane).
// K is split over blocks (grid.z); partial tiles go to a workspace and a second kernel sums them in
// split order.
// ================================================================================================
struct WgradArgs {
    const float* dense;
    const float* gath;
    float* partial;   // [S][M][N]
    int32_t B, M, C, T, N;
    int32_t Hq, Wq, Hg, Wg, s;
    int32_t cpb;      // chunks per sample = ceil(Hq*Wq / 16)
    int32_t nchunk;   // B * cpb
    int32_t per_split;
    int32_t kw, pad;
    FastDiv fd_cpb, fd_wq, fd_t, fd_kw;
};

__global__ __launch_bounds__(64) void wgrad_kernel(WgradArgs a) {
    const int lane = threadIdx.x;
    const int col = lane & 15, g = lane >> 4;
    const int m0 = blockIdx.y * 16, n0 = blockIdx.x * 16;
    const int split = blockIdx.z;
    const int HQ = a.Hq * a.Wq, HG = a.Hg * a.Wg;
    // B-operand lane state: n -> (c, t)
    const int n = n0 + col;
    const bool nok = n < a.N;
    const int c = nok ? a.fd_t.div(n) : 0;
    const int t = nok ? n - c * a.T : 0;
    const int kh = a.fd_kw.div(t);
    const int dy = kh - a.pad, dx = (t - kh * a.kw) - a.pad;
    const int m = m0 + col;
    const bool mok = m < a.M;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    const int c_begin = split * a.per_split;
    const int c_end = min(a.nchunk, c_begin + a.per_split);
    const bool vec4 = (HQ % 4) == 0;
    for (int ch = c_begin; ch < c_end; ++ch) {
        const int b = a.fd_cpb.div(ch);
        const int q0 = (ch - b * a.cpb) * 16 + 4 * g;
        // A: Dense[b][m][q0 .. q0+3]
        floatx4 av = {0.f, 0.f, 0.f, 0.f};
        const float* dp = a.dense + ((size_t)b * a.M + (mok ? m : 0)) * HQ;
        if (vec4 && q0 + 3 < HQ) {
            av = *(const floatx4*)(dp + q0);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) av[j] = q0 + j < HQ ? dp[q0 + j] : 0.f;
        }
        if (!mok) av = floatx4{0.f, 0.f, 0.f, 0.f};
        float bv[4];
        const float* gp = a.gath + ((size_t)b * a.C + c) * HG;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int q = q0 + j;
            const int qy = a.fd_wq.div(q), qx = q - qy * a.Wq;
            const int iy = qy * a.s + dy, ix = qx * a.s + dx;
            const bool ok = nok && q < HQ && (unsigned)iy < (unsigned)a.Hg && (unsigned)ix < (unsigned)a.Wg;
            const float v = gp[ok ? iy * a.Wg + ix : 0];
            bv[j] = ok ? v : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], bv[j], acc, 0, 0, 0);
    }
    float* out = a.partial + (size_t)split * a.M * a.N;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int mm = m0 + 4 * g + r;
        if (mm < a.M && nok) out[(size_t)mm * a.N + n] = acc[r];
    }
}

// sum of split partials in split order.  Tap t is the kernel-window index (kh*kw + kw), so the
// [m][c*T + t] GEMM layout IS the torch weight layout [m][c][kh][kw].
// 256 threads = (256 / G) outputs x G split groups: group g sums its contiguous range of splits serially,
// then the G group sums meet in a pairwise tree in LDS (a fixed partition and order: bitwise
// reproducible).  G grows as M*N shrinks, so that ~2^18 threads share the S*M*N partial reads: one thread
// per output walking all S splits serially was latency-bound at small M*N (60 us for 1024 outputs x 256
// splits), while at large M*N that form (G = 1) streams whole 256-B rows per wave.
inline int wgrad_groups(int S, int MN) {
    int G = 1;
    while (G < S && G < 256 && (int64_t)MN * G < (1 << 18)) G *= 2;
    return G;
}
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ partial, int S, int MN,
                                                           float* __restrict__ dw, int accumulate, int G) {
    __shared__ float red[256];
    const int NO = 256 / G;
    const int ol = threadIdx.x % NO, g = threadIdx.x / NO;
    const int i = blockIdx.x * NO + ol;
    const int per = (S + G - 1) / G;
    float v = 0.f;
    if (i < MN) {
        // eight splits' loads in flight per step, summed in split order (same roundings as one at a time)
        const int s1 = min(S, (g + 1) * per);
        int s = g * per;
        for (; s + 8 <= s1; s += 8) {
            float p[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) p[u] = partial[(size_t)(s + u) * MN + i];
#pragma unroll
            for (int u = 0; u < 8; ++u) v = v + p[u];
        }
        for (; s < s1; ++s) v = v + partial[(size_t)s * MN + i];
    }
    if (G > 1) {
        red[threadIdx.x] = v;
        for (int st = G / 2; st >= 1; st /= 2) {
            __syncthreads();
            if (g < st) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + st * NO];
        }
        __syncthreads();
        v = red[ol];
    }
    if (g == 0 && i < MN) dw[i] = accumulate ? dw[i] + v : v;
}
// The same sums on 16-byte pieces (round 6): a thread owns four consecutive outputs, each summed in the order
// above, so a wave-load moves 1 KB instead of 256 B (the partials of the train step's layers are ~38 MB per
// layer: the scalar form read them at ~4.5 TB/s).  G comes from the piece count, ~2^18 threads as before.
__device__ __forceinline__ void wgrad_reduce4_body(const floatx4* __restrict__ partial, int S, int MN4,
                                                   floatx4* __restrict__ dw, int accumulate, int G, int blk) {
    __shared__ floatx4 red[256];
    const int NO = 256 / G;
    const int ol = threadIdx.x % NO, g = threadIdx.x / NO;
    const int i = blk * NO + ol;
    const int per = (S + G - 1) / G;
    floatx4 v = {0.f, 0.f, 0.f, 0.f};
    if (i < MN4) {
        const int s1 = min(S, (g + 1) * per);
        int s = g * per;
        for (; s + 8 <= s1; s += 8) {
            floatx4 p[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) p[u] = partial[(size_t)(s + u) * MN4 + i];
#pragma unroll
            for (int u = 0; u < 8; ++u) v = v + p[u];
        }
        for (; s < s1; ++s) v = v + partial[(size_t)s * MN4 + i];
    }
    if (G > 1) {
        red[threadIdx.x] = v;
        for (int st = G / 2; st >= 1; st /= 2) {
            __syncthreads();
            if (g < st) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + st * NO];
        }
        __syncthreads();
        v = red[ol];
    }
    if (g == 0 && i < MN4) dw[i] = accumulate ? dw[i] + v : v;
}
__global__ __launch_bounds__(256) void wgrad_reduce4_kernel(const floatx4* __restrict__ partial, int S, int MN4,
                                                            floatx4* __restrict__ dw, int accumulate, int G) {
    wgrad_reduce4_body(partial, S, MN4, dw, accumulate, G, blockIdx.x);
}

// The split-K reductions of several weight gradients in one launch (ldm_wgrad_reduce_many): the train step's weight
// gradients are read only by the optimizer, so their reductions can wait for the end of the backward and go as one
// launch.  Block -> (job, block of the job) by the jobs' first blocks b0; each job's blocks run wgrad_reduce4_kernel's
// code with its G, so the same bits.
struct RedJob {
    const floatx4* partial;
    floatx4* dw;
    int32_t S, MN4, accumulate, G, b0;
};
constexpr int kMaxRedJobs = 24;
struct RedJobs {
    RedJob j[kMaxRedJobs];
    int32_t n;
};
__global__ __launch_bounds__(256) void wgrad_reduce_many_kernel(RedJobs jobs) {
    int k = 0;
    while (k + 1 < jobs.n && (int)blockIdx.x >= jobs.j[k + 1].b0) ++k;
    const RedJob& J = jobs.j[k];
    wgrad_reduce4_body(J.partial, J.S, J.MN4, J.dw, J.accumulate, J.G, (int)blockIdx.x - J.b0);
}
static void wgrad_reduce(const float* partial, int S, int MN, float* dw, int accumulate, hipStream_t st) {
    static const bool vec = [] {   // LDM_WGRAD_REDUCE4=0: the scalar form (A/B timing)
        const char* e = std::getenv("LDM_WGRAD_REDUCE4");
        return !e || std::atoi(e) != 0;
    }();
    if (vec && MN % 4 == 0 && (((uintptr_t)partial | (uintptr_t)dw) & 15) == 0) {
        const int MN4 = MN / 4, G = wgrad_groups(S, MN4), NO = 256 / G;
        hipLaunchKernelGGL(wgrad_reduce4_kernel, dim3((MN4 + NO - 1) / NO), dim3(256), 0, st,
                           reinterpret_cast<const floatx4*>(partial), S, MN4, reinterpret_cast<floatx4*>(dw), accumulate, G);
        return;
    }
    const int G = wgrad_groups(S, MN), NO = 256 / G;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((MN + NO - 1) / NO), dim3(256), 0, st, partial, S, MN, dw, accumulate,
                       G);
}

// ================================================================================================
// cross-attention backward, one block per (b, head); recomputes P from q, k:
//   dV = dO P ; dP = dO^T V ; dS = P*(dP - rowsum(dP*P)) ; dq = scale*(K dS^T) ; dK = qs dS
// q [B,E,L], kv [B,2E,S] (K then V), dout [B,E,L] -> dq [B,E,L], dkv [B,2E,S].
// LDS: X1 [d][L], X2 [d][S] (Q,K then dO,V then Q,K again), P [L][S], dP [L][S].
// ================================================================================================
__global__ __launch_bounds__(256) void attention_backward_kernel(const float* __restrict__ q,
                                                                 const float* __restrict__ kv,
                                                                 const float* __restrict__ dout, float* __restrict__ dq,
                                                                 float* __restrict__ dkv, int E, int heads, int L, int S,
                                                                 float scale) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int d = E / heads;
    const int h = blockIdx.x % heads, b = blockIdx.x / heads;
    float* X1 = sm;              // [d][L]
    float* X2 = X1 + d * L;      // [d][S]
    float* P = X2 + d * S;       // [L][S]
    float* dP = P + L * S;       // [L][S]
    const size_t qo = ((size_t)b * E + (size_t)h * d) * L;
    const size_t ko = ((size_t)b * 2 * E + (size_t)h * d) * S;
    const size_t vo = ((size_t)b * 2 * E + E + (size_t)h * d) * S;
    const int tid = threadIdx.x, nt = blockDim.x;
    const int lane = tid & 63, wave = tid >> 6, nw = nt >> 6;
    // phase 1: P = softmax((q*scale)^T k)
    for (int e = tid; e < d * L; e += nt) X1[e] = q[qo + e] * scale;
    for (int e = tid; e < d * S; e += nt) X2[e] = kv[ko + e];
    __syncthreads();
    for (int e = tid; e < L * S; e += nt) {
        const int l = e / S, s = e - l * S;
        float acc = 0.f;
        for (int c = 0; c < d; ++c) acc = fmaf(X1[c * L + l], X2[c * S + s], acc);
        P[e] = acc;
    }
    __syncthreads();
    for (int l = wave; l < L; l += nw) {
        float* row = P + l * S;
        float mx = -INFINITY;
        for (int s = lane; s < S; s += 64) mx = fmaxf(mx, row[s]);
        for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
        float sum = 0.f;
        for (int s = lane; s < S; s += 64) {
            const float ex = expf(row[s] - mx);
            row[s] = ex;
            sum += ex;
        }
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
        for (int s = lane; s < S; s += 64) row[s] = row[s] / sum;
    }
    __syncthreads();
    // phase 2: X1 <- dO [d][L], X2 <- V [d][S]; dV = dO P -> global; dP = dO^T V -> LDS
    for (int e = tid; e < d * L; e += nt) X1[e] = dout[qo + e];
    for (int e = tid; e < d * S; e += nt) X2[e] = kv[vo + e];
    __syncthreads();
    for (int e = tid; e < d * S; e += nt) {
        const int c = e / S, s = e - c * S;
        float acc = 0.f;
        for (int l = 0; l < L; ++l) acc = fmaf(X1[c * L + l], P[l * S + s], acc);
        dkv[vo + e] = acc;
    }
    for (int e = tid; e < L * S; e += nt) {
        const int l = e / S, s = e - l * S;
        float acc = 0.f;
        for (int c = 0; c < d; ++c) acc = fmaf(X1[c * L + l], X2[c * S + s], acc);
        dP[e] = acc;
    }
    __syncthreads();
    // phase 3: dS = P * (dP - rowsum(dP * P))  (in place in dP)
    for (int l = wave; l < L; l += nw) {
        float s0 = 0.f;
        for (int s = lane; s < S; s += 64) s0 += dP[l * S + s] * P[l * S + s];
        for (int o = 32; o > 0; o >>= 1) s0 += __shfl_xor(s0, o);
        for (int s = lane; s < S; s += 64) dP[l * S + s] = P[l * S + s] * (dP[l * S + s] - s0);
    }
    __syncthreads();
    // phase 4: X1 <- qs, X2 <- K; dq = scale * K dS^T ; dK = qs dS
    for (int e = tid; e < d * L; e += nt) X1[e] = q[qo + e] * scale;
    for (int e = tid; e < d * S; e += nt) X2[e] = kv[ko + e];
    __syncthreads();
    for (int e = tid; e < d * L; e += nt) {
        const int c = e / L, l = e - c * L;
        float acc = 0.f;
        for (int s = 0; s < S; ++s) acc = fmaf(dP[l * S + s], X2[c * S + s], acc);
        dq[qo + e] = acc * scale;
    }
    for (int e = tid; e < d * S; e += nt) {
        const int c = e / S, s = e - c * S;
        float acc = 0.f;
        for (int l = 0; l < L; ++l) acc = fmaf(dP[l * S + s], X1[c * L + l], acc);
        dkv[ko + e] = acc;
    }
}

// The same backward on f32 MFMA (v_mfma_f32_16x16x4_f32, exact fp32 products) when L, S and d are
// multiples of 16 (the UNet's CA2: d 64, L = S = 64; CA1: d 128, L = S = 16 at the canonical latent): every
// product of the five is a sweep of 16x16 output tiles over the block's 4 waves with both operands read
// from LDS (the scalar form above spent ~6K dependent LDS-operand FMAs per thread: 128 us per call at B=32).
// Operand (m, k) of a product lives at base[m * sm + k * sk]; the lane's D rows 4 lg + r, column lane & 15.
template <class FA, class FB, class FO>
__device__ __forceinline__ void lds_mfma_gemm(int M, int N, int K, FA&& fa, FB&& fb, FO&& out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int col = lane & 15, lg = lane >> 4;
    const int tn = N / 16, tiles = (M / 16) * tn;
    for (int t = wave; t < tiles; t += nw) {
        const int m0 = (t / tn) * 16, n0 = (t % tn) * 16;
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int k0 = 0; k0 < K; k0 += 16) {
            float a[4], b[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                a[j] = fa(m0 + col, k0 + 4 * j + lg);
                b[j] = fb(k0 + 4 * j + lg, n0 + col);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) out(m0 + 4 * lg + r, n0 + col, acc[r]);
    }
}

__global__ __launch_bounds__(256) void attention_backward_mfma_kernel(const float* __restrict__ q,
                                                                      const float* __restrict__ kv,
                                                                      const float* __restrict__ dout,
                                                                      float* __restrict__ dq, float* __restrict__ dkv,
                                                                      int E, int heads, int L, int S, float scale) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int d = E / heads;
    const int h = blockIdx.x % heads, b = blockIdx.x / heads;
    // row pitches padded by one float so that the 16 lanes of an MFMA operand column hit 16 banks
    const int pL = L + 1, pS = S + 1;
    float* X1 = sm;              // [d][L+1]
    float* X2 = X1 + d * pL;     // [d][S+1]
    float* P = X2 + d * pS;      // [L][S+1]
    float* dP = P + L * pS;      // [L][S+1]
    const size_t qo = ((size_t)b * E + (size_t)h * d) * L;
    const size_t ko = ((size_t)b * 2 * E + (size_t)h * d) * S;
    const size_t vo = ((size_t)b * 2 * E + E + (size_t)h * d) * S;
    const int tid = threadIdx.x, nt = blockDim.x;
    const int lane = tid & 63, wave = tid >> 6, nw = nt >> 6;
    auto load2 = [&](const float* s1, float m1, const float* s2) {
        for (int e = tid; e < d * L; e += nt) X1[(e / L) * pL + e % L] = s1[e] * m1;
        for (int e = tid; e < d * S; e += nt) X2[(e / S) * pS + e % S] = s2[e];
    };
    // phase 1: P[l][s] = sum_c (q*scale)[c][l] K[c][s], softmax over s
    load2(q + qo, scale, kv + ko);
    __syncthreads();
    lds_mfma_gemm(L, S, d, [&](int l, int c) { return X1[c * pL + l]; }, [&](int c, int s) { return X2[c * pS + s]; },
                  [&](int l, int s, float v) { P[l * pS + s] = v; });
    __syncthreads();
    for (int l = wave; l < L; l += nw) {
        float* row = P + l * pS;
        float mx = -INFINITY;
        for (int s = lane; s < S; s += 64) mx = fmaxf(mx, row[s]);
        for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
        float sum = 0.f;
        for (int s = lane; s < S; s += 64) {
            const float ex = expf(row[s] - mx);
            row[s] = ex;
            sum += ex;
        }
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
        for (int s = lane; s < S; s += 64) row[s] = row[s] / sum;
    }
    __syncthreads();
    // phase 2: X1 <- dO, X2 <- V; dV[c][s] = sum_l dO[c][l] P[l][s] (global); dP[l][s] = sum_c dO[c][l] V[c][s]
    load2(dout + qo, 1.f, kv + vo);
    __syncthreads();
    lds_mfma_gemm(d, S, L, [&](int c, int l) { return X1[c * pL + l]; }, [&](int l, int s) { return P[l * pS + s]; },
                  [&](int c, int s, float v) { dkv[vo + (size_t)c * S + s] = v; });
    lds_mfma_gemm(L, S, d, [&](int l, int c) { return X1[c * pL + l]; }, [&](int c, int s) { return X2[c * pS + s]; },
                  [&](int l, int s, float v) { dP[l * pS + s] = v; });
    __syncthreads();
    // phase 3: dS = P * (dP - rowsum(dP * P)), in place in dP
    for (int l = wave; l < L; l += nw) {
        float s0 = 0.f;
        for (int s = lane; s < S; s += 64) s0 += dP[l * pS + s] * P[l * pS + s];
        for (int o = 32; o > 0; o >>= 1) s0 += __shfl_xor(s0, o);
        for (int s = lane; s < S; s += 64) dP[l * pS + s] = P[l * pS + s] * (dP[l * pS + s] - s0);
    }
    __syncthreads();
    // phase 4: X1 <- q*scale, X2 <- K; dq[c][l] = scale sum_s K[c][s] dS[l][s]; dK[c][s] = sum_l qs[c][l] dS[l][s]
    load2(q + qo, scale, kv + ko);
    __syncthreads();
    lds_mfma_gemm(d, L, S, [&](int c, int s) { return X2[c * pS + s]; }, [&](int s, int l) { return dP[l * pS + s]; },
                  [&](int c, int l, float v) { dq[qo + (size_t)c * L + l] = v * scale; });
    lds_mfma_gemm(d, S, L, [&](int c, int l) { return X1[c * pL + l]; }, [&](int l, int s) { return dP[l * pS + s]; },
                  [&](int c, int s, float v) { dkv[ko + (size_t)c * S + s] = v; });
}

// ================================================================================================
// multi-tensor Adam (torch.optim.Adam, train.py:156) with GradScaler unscale / inf check / skip
// ================================================================================================
// A chunk's elements, float4 at a time where every pointer of the slot is 16-byte aligned (the chunk
// start is a multiple of 4 elements), the ragged tail one at a time; f(i, W) handles elements i..i+W-1.
template <class F4, class F1>
__device__ __forceinline__ void chunk_for(int64_t s0, int64_t e0, bool vec, F4&& f4, F1&& f1) {
    int64_t t0 = s0;
    if (vec) {
        const int64_t n4 = (e0 - s0) >> 2;
        for (int64_t j = threadIdx.x; j < n4; j += blockDim.x) f4(s0 + 4 * j);
        t0 = s0 + 4 * n4;
    }
    for (int64_t i = t0 + threadIdx.x; i < e0; i += blockDim.x) f1(i);
}
__device__ __forceinline__ bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

__global__ __launch_bounds__(256) void unscale_check_kernel(const ldm_tensor_slot* __restrict__ slots,
                                                            const int32_t* __restrict__ chunk_tensor,
                                                            const int64_t* __restrict__ chunk_start, int chunk_len,
                                                            const float* __restrict__ inv_scale,
                                                            int32_t* __restrict__ found_inf) {
#define KNAME "unscale_check_kernel"
#if LDM_DEBUG_BOUNDS
    {
        const int32_t ti = chunk_tensor[blockIdx.x];
        const bool bad_ix = ti < 0 || ti >= (int32_t)gridDim.x || chunk_start[blockIdx.x] < 0;
        if (bad_ix || slots[ti].grad == nullptr) {
            if (threadIdx.x == 0) printf("%s: chunk %u: bad slot index %d / start %ld\n", KNAME, blockIdx.x, ti, (long)chunk_start[blockIdx.x]);
            return;
        }
    }
#endif
#undef KNAME
    const ldm_tensor_slot sl = slots[chunk_tensor[blockIdx.x]];
    const int64_t s0 = chunk_start[blockIdx.x];
    const int64_t e0 = min(s0 + (int64_t)chunk_len, sl.numel);
    const float is = inv_scale ? inv_scale[0] : 1.f;
    bool bad = false;
    chunk_for(
        s0, e0, al16(sl.grad + s0),
        [&](int64_t i) {
            float4 g = *reinterpret_cast<const float4*>(sl.grad + i);
            g.x *= is, g.y *= is, g.z *= is, g.w *= is;
            *reinterpret_cast<float4*>(sl.grad + i) = g;
            bad |= !isfinite(g.x) || !isfinite(g.y) || !isfinite(g.z) || !isfinite(g.w);
        },
        [&](int64_t i) {
            const float g = sl.grad[i] * is;
            sl.grad[i] = g;
            bad |= !isfinite(g);
        });
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(found_inf, 1);   // a flag, not a sum: order-free
}

struct AdamScalars {
    float one_m_beta1, beta2, one_m_beta2, eps, weight_decay, decay_mul, step_size, bc2_sqrt;
};
// torch.optim.Adam / AdamW (_single_tensor_adam, non-capturable) on one element
__device__ __forceinline__ void adam_elem(const AdamScalars& k, float& p, float g, float& m, float& v) {
    if (k.decay_mul != 1.f) p = p * k.decay_mul;                 // AdamW: param.mul_(1 - lr * weight_decay)
    else if (k.weight_decay != 0.f) g = g + k.weight_decay * p;  // Adam: grad.add(param, alpha=wd)
    m = m + k.one_m_beta1 * (g - m);                              // exp_avg.lerp_(grad, 1 - beta1)
    v = v * k.beta2;                                              // exp_avg_sq.mul_(beta2)
    v = v + (k.one_m_beta2 * g) * g;                              //   .addcmul_(grad, grad, value=1 - beta2)
    const float denom = sqrtf(v) / k.bc2_sqrt + k.eps;
    p = p + (-k.step_size) * (m / denom);                         // param.addcdiv_(exp_avg, denom, value=-step_size)
}

__global__ __launch_bounds__(256) void adam_kernel(const ldm_tensor_slot* __restrict__ slots,
                                                   const int32_t* __restrict__ chunk_tensor,
                                                   const int64_t* __restrict__ chunk_start, int chunk_len,
                                                   AdamScalars k, const int32_t* __restrict__ found_inf,
                                                   const AdamScalars* __restrict__ kdev = nullptr) {
    if (found_inf && found_inf[0]) return;   // GradScaler.step skips the update on inf/nan
    if (kdev) k = *kdev;                     // capturable form: scalars of the device-side step count
#define KNAME "adam_kernel"
#if LDM_DEBUG_BOUNDS
    {
        const int32_t ti = chunk_tensor[blockIdx.x];
        const bool bad_ix = ti < 0 || ti >= (int32_t)gridDim.x || chunk_start[blockIdx.x] < 0;
        if (bad_ix || slots[ti].grad == nullptr) {
            if (threadIdx.x == 0) printf("%s: chunk %u: bad slot index %d / start %ld\n", KNAME, blockIdx.x, ti, (long)chunk_start[blockIdx.x]);
            return;
        }
    }
#endif
#undef KNAME
    const ldm_tensor_slot sl = slots[chunk_tensor[blockIdx.x]];
    const int64_t s0 = chunk_start[blockIdx.x];
    const int64_t e0 = min(s0 + (int64_t)chunk_len, sl.numel);
    // scalars arrive as torch's: host doubles cast once to fp32 (1-beta computed in double)
    const bool vec = al16(sl.grad + s0) && al16(sl.param + s0) && al16(sl.exp_avg + s0) && al16(sl.exp_avg_sq + s0);
    chunk_for(
        s0, e0, vec,
        [&](int64_t i) {
            const float4 g = *reinterpret_cast<const float4*>(sl.grad + i);
            float4 p = *reinterpret_cast<const float4*>(sl.param + i);
            float4 m = *reinterpret_cast<const float4*>(sl.exp_avg + i);
            float4 v = *reinterpret_cast<const float4*>(sl.exp_avg_sq + i);
            adam_elem(k, p.x, g.x, m.x, v.x);
            adam_elem(k, p.y, g.y, m.y, v.y);
            adam_elem(k, p.z, g.z, m.z, v.z);
            adam_elem(k, p.w, g.w, m.w, v.w);
            *reinterpret_cast<float4*>(sl.exp_avg + i) = m;
            *reinterpret_cast<float4*>(sl.exp_avg_sq + i) = v;
            *reinterpret_cast<float4*>(sl.param + i) = p;
        },
        [&](int64_t i) {
            float p = sl.param[i], m = sl.exp_avg[i], v = sl.exp_avg_sq[i];
            adam_elem(k, p, sl.grad[i], m, v);
            sl.exp_avg[i] = m;
            sl.exp_avg_sq[i] = v;
            sl.param[i] = p;
        });
}

// Capturable step (hipGraph replay): the step count lives on the device and advances only on applied
// steps (found_inf clear), and the derived scalars are formed from it exactly as the host form forms them
// (double, one cast to fp32), so graphed and eager steps are bitwise equal.
__global__ void adam_prep_kernel(float* step, const int32_t* found_inf, double lr, double beta1, double beta2,
                                 double eps, double weight_decay, int decoupled, AdamScalars* out) {
    if (found_inf && found_inf[0]) return;
    const float st = step[0] + 1.f;
    step[0] = st;
    const double bc1 = 1.0 - pow(beta1, (double)st);
    const double bc2 = 1.0 - pow(beta2, (double)st);
    AdamScalars k;
    k.one_m_beta1 = (float)(1.0 - beta1);
    k.beta2 = (float)beta2;
    k.one_m_beta2 = (float)(1.0 - beta2);
    k.eps = (float)eps;
    k.weight_decay = (float)weight_decay;
    k.decay_mul = decoupled ? (float)(1.0 - lr * weight_decay) : 1.f;
    k.step_size = (float)(lr / bc1);
    k.bc2_sqrt = (float)sqrt(bc2);
    *out = k;
}

// torch.amp.GradScaler._amp_update_scale_: backoff on inf, grow after growth_interval clean steps
__global__ void update_scale_kernel(float* scale, int32_t* growth_tracker, const int32_t* found_inf,
                                    float growth_factor, float backoff_factor, int growth_interval) {
    if (found_inf[0]) {
        scale[0] = scale[0] * backoff_factor;
        growth_tracker[0] = 0;
    } else {
        const int successful = growth_tracker[0] + 1;
        if (successful == growth_interval) {
            scale[0] = scale[0] * growth_factor;
            growth_tracker[0] = 0;
        } else {
            growth_tracker[0] = successful;
        }
    }
}

}  // namespace ldm

using namespace ldm;

// ---- weight gradient ------------------------------------------------------------------------------
// ---- weight gradient of a 1x1 conv (the cross-attention projections): dW[m][c] = sum_b sum_n dy[b][m][n] x[b][c][n]
// over HW % 16 == 0 planes, an NT GEMM whose K (b, n) is contiguous in both NCHW operands.  A block owns a 32 x 32
// tile of dW; its eight waves take interleaved shares of the 16-position k-steps (two steps per iteration, the
// next two steps' loads issued before these MFMAs) and meet in LDS in wave order, so no split-K partials and no
// reduction launch (the tap-shared form above ran these at 16 x 16 tiles of one wave plus a reduction).  DT 0: fp32 operands on
// v_mfma_f32_32x32x2f32 (the k-pairs in a fixed permutation); DT 1 / 2: operands rounded to fp16 / bf16 on the
// double-rate 32x32x16 MFMA (the autocast region's weight gradients).
typedef __bf16 wbf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 whalfx8 __attribute__((ext_vector_type(8)));
typedef float wfloatx8 __attribute__((ext_vector_type(8)));

struct W1Args {
    const float* dy;   // [B][M][HW]
    const float* x;    // [B][C][HW]
    float* dw;         // [M][C]
    int32_t B, M, C, HW, accumulate;
};

constexpr int kW1Waves = 8;   // waves per block of wgrad_1x1_kernel (interleaved k-step shares; 16: 88 vs 79 us per step)

template <int DT>
__device__ __forceinline__ floatx16 w1_mma(const floatx4 (&ca)[2], const floatx4 (&cb)[2], floatx16 acc) {
    if constexpr (DT == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ca[j >> 2][j & 3], cb[j >> 2][j & 3], acc, 0, 0, 0);
        return acc;
    } else {
        const wfloatx8 fa{ca[0][0], ca[0][1], ca[0][2], ca[0][3], ca[1][0], ca[1][1], ca[1][2], ca[1][3]};
        const wfloatx8 fb{cb[0][0], cb[0][1], cb[0][2], cb[0][3], cb[1][0], cb[1][1], cb[1][2], cb[1][3]};
        if constexpr (DT == 1)
            return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_convertvector(fa, whalfx8),
                                                          __builtin_convertvector(fb, whalfx8), acc, 0, 0, 0);
        else
            return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_convertvector(fa, wbf16x8),
                                                           __builtin_convertvector(fb, wbf16x8), acc, 0, 0, 0);
    }
}

// wave w takes k-steps w, w + 8, ...: two steps per iteration, the next two steps' loads issued before these
// MFMAs (the chain is load latency-bound, not MFMA-bound)
template <int DT>
__global__ __launch_bounds__(64 * kW1Waves) void wgrad_1x1_kernel(W1Args a) {
    __shared__ float red[kW1Waves][16][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int m0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
    const int spp = a.HW / 16;                 // k-steps per sample
    const int nsteps = a.B * spp;
    const size_t sa = (size_t)a.M * a.HW, sb = (size_t)a.C * a.HW;
    const float* pa = a.dy + (size_t)(m0 + r) * a.HW + 8 * h;
    const float* pb = a.x + (size_t)(c0 + r) * a.HW + 8 * h;
    // step st (clamped to the last one: a re-load whose MFMA is skipped)
    auto load = [&](int st, floatx4 (&va)[2], floatx4 (&vb)[2]) {
        st = st < nsteps ? st : nsteps - 1;
        const int b = st / spp, n0 = (st - b * spp) * 16;
        const float* qa = pa + b * sa + n0;
        const float* qb = pb + b * sb + n0;
        va[0] = *reinterpret_cast<const floatx4*>(qa);
        va[1] = *reinterpret_cast<const floatx4*>(qa + 4);
        vb[0] = *reinterpret_cast<const floatx4*>(qb);
        vb[1] = *reinterpret_cast<const floatx4*>(qb + 4);
    };
    floatx16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    constexpr int W = kW1Waves;
    floatx4 ca0[2], cb0[2], ca1[2], cb1[2], na0[2], nb0[2], na1[2], nb1[2];
    load(wave, ca0, cb0);
    load(wave + W, ca1, cb1);
    for (int st = wave; st < nsteps; st += 2 * W) {
        load(st + 2 * W, na0, nb0);
        load(st + 3 * W, na1, nb1);
        acc = w1_mma<DT>(ca0, cb0, acc);
        if (st + W < nsteps) acc = w1_mma<DT>(ca1, cb1, acc);
#pragma unroll
        for (int i = 0; i < 2; ++i) ca0[i] = na0[i], cb0[i] = nb0[i], ca1[i] = na1[i], cb1[i] = nb1[i];
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) red[wave][i][lane] = acc[i];
    __syncthreads();
    // 1024 outputs, two per thread: the wave partials summed in wave order
    for (int o = threadIdx.x; o < 16 * 64; o += 64 * W) {
        const int reg = o >> 6, l = o & 63;
        float v = red[0][reg][l];
#pragma unroll
        for (int w = 1; w < W; ++w) v += red[w][reg][l];
        const int m = m0 + (reg & 3) + 8 * (reg >> 2) + 4 * (l >> 5), c = c0 + (l & 31);
        float* d = a.dw + (size_t)m * a.C + c;
        *d = a.accumulate ? *d + v : v;
    }
}

static int wgrad_setup(const ldm_conv_desc& d, WgradArgs& a, int& kk_count) {
    a = WgradArgs{};
    LDM_REQUIRE(d.kh > 0 && d.kw > 0 && d.B > 0, "wgrad: bad descriptor");
    a.B = d.B;
    a.T = d.kh * d.kw;
    kk_count = a.T;
    if (!d.transposed) {
        a.M = d.Cout;
        a.C = d.Cin;
        a.Hq = d.Hout;
        a.Wq = d.Wout;
        a.Hg = d.Hin;
        a.Wg = d.Win;
    } else {
        a.M = d.Cin;
        a.C = d.Cout;
        a.Hq = d.Hin;
        a.Wq = d.Win;
        a.Hg = d.Hout;
        a.Wg = d.Wout;
    }
    a.s = d.stride;
    a.N = a.C * a.T;
    a.kw = d.kw;
    a.pad = d.pad;
    a.fd_kw = FastDiv::make(d.kw);
    a.cpb = (a.Hq * a.Wq + 15) / 16;
    a.nchunk = a.B * a.cpb;
    a.fd_cpb = FastDiv::make(a.cpb);
    a.fd_wq = FastDiv::make(a.Wq);
    a.fd_t = FastDiv::make(a.T);
    return 0;
}

static int wgrad_splits(const WgradArgs& a) {
    const int tiles = ((a.M + 15) / 16) * ((a.N + 15) / 16);
    int S = 1;
    while (S < 256 && tiles * S < 2048 && a.nchunk / (S * 2) >= 4) S *= 2;
    return S;
}

extern "C" int64_t ldm_conv_wgrad_workspace_floats(const ldm_conv_desc* d) {
    if (!d) return -1;
    int64_t f2 = 0;
    if (wgrad2_plan_ws(*d, f2)) return f2;
    WgradArgs a;
    int kk;
    if (wgrad_setup(*d, a, kk)) return -1;
    const int S = wgrad_splits(a);
    return (int64_t)S * a.M * a.N;
}

extern "C" int32_t ldm_conv_wgrad_storage16(const ldm_conv_desc* d) { return d ? wgrad2_storage16(*d) : 0; }

extern "C" int ldm_conv_backward_weight(const ldm_conv_desc* d, const float* x, const float* dy, float* dw,
                                        int32_t accumulate, float* workspace, void* stream) {
    return ldm_conv_backward_weight_dt(d, x, dy, dw, accumulate, workspace, LDM_DT_F32, stream);
}

static int conv_backward_weight_impl(const ldm_conv_desc* d, const float* x, const float* dy, float* dw,
                                     int32_t accumulate, float* workspace, int32_t dtype, int32_t* defer_s, void* stream);

extern "C" int ldm_conv_backward_weight_dt(const ldm_conv_desc* d, const float* x, const float* dy, float* dw,
                                           int32_t accumulate, float* workspace, int32_t dtype, void* stream) {
    return conv_backward_weight_impl(d, x, dy, dw, accumulate, workspace, dtype, nullptr, stream);
}

extern "C" int ldm_conv_backward_weight_defer(const ldm_conv_desc* d, const float* x, const float* dy, float* dw,
                                              int32_t accumulate, float* workspace, int32_t dtype, int32_t* splits_out,
                                              void* stream) {
    LDM_REQUIRE(splits_out, "wgrad_defer: bad argument");
    return conv_backward_weight_impl(d, x, dy, dw, accumulate, workspace, dtype, splits_out, stream);
}

extern "C" int ldm_wgrad_reduce_many(const ldm_wgrad_red_job* jobs, int32_t n, void* stream) {
    LDM_REQUIRE(jobs && n >= 0, "wgrad_reduce_many: bad argument");
    hipStream_t st = (hipStream_t)stream;
    for (int i0 = 0; i0 < n; i0 += kMaxRedJobs) {
        RedJobs rj{};
        int blocks = 0;
        rj.n = n - i0 < kMaxRedJobs ? n - i0 : kMaxRedJobs;
        for (int i = 0; i < rj.n; ++i) {
            const ldm_wgrad_red_job& J = jobs[i0 + i];
            LDM_REQUIRE(J.partial && J.dw && J.S > 0 && J.MN > 0 && J.MN % 4 == 0 &&
                            (((uintptr_t)J.partial | (uintptr_t)J.dw) & 15) == 0,
                        "wgrad_reduce_many: bad job");
            const int MN4 = J.MN / 4, G = wgrad_groups(J.S, MN4), NO = 256 / G;
            rj.j[i] = RedJob{reinterpret_cast<const floatx4*>(J.partial), reinterpret_cast<floatx4*>(J.dw), J.S, MN4,
                             J.accumulate, G, blocks};
            blocks += (MN4 + NO - 1) / NO;
        }
        if (blocks == 0) continue;
        hipLaunchKernelGGL(wgrad_reduce_many_kernel, dim3(blocks), dim3(256), 0, st, rj);
        LDM_CHECK_LAUNCH("wgrad_reduce_many_kernel");
    }
    return 0;
}

// defer_s != NULL: a tap-shared gradient split over S > 1 K ranges leaves its partials in `workspace` and *defer_s = S
// (the caller reduces them later with ldm_wgrad_reduce_many); any other form runs as ldm_conv_backward_weight_dt and
// *defer_s = 0
static int conv_backward_weight_impl(const ldm_conv_desc* d, const float* x, const float* dy, float* dw,
                                     int32_t accumulate, float* workspace, int32_t dtype, int32_t* defer_s, void* stream) {
    if (defer_s) *defer_s = 0;
    LDM_REQUIRE(d && x && dy && dw && workspace, "wgrad: null argument");
    const int st16 = dtype & (LDM_DT_X16 | LDM_DT_DY16);
    dtype &= ~(LDM_DT_X16 | LDM_DT_DY16);
    LDM_REQUIRE(dtype >= LDM_DT_F32 && dtype <= LDM_DT_BF16, "wgrad: unknown operand precision");
    LDM_REQUIRE(!st16 || dtype != LDM_DT_F32, "wgrad: 16-bit storage needs a 16-bit dtype");
    static const bool w1 = [] {   // LDM_WGRAD_1X1=0: the tap-shared form for 1x1 convs too (A/B timing)
        const char* e = std::getenv("LDM_WGRAD_1X1");
        return !e || e[0] != '0';
    }();
    if (w1 && !st16 && d->kh == 1 && d->kw == 1 && d->stride == 1 && d->pad == 0 && !d->transposed && d->B > 0 &&
        d->Cout % 32 == 0 && d->Cin % 32 == 0 && (d->Hout * d->Wout) % 16 == 0 &&
        ((uintptr_t)x & 15) == 0 && ((uintptr_t)dy & 15) == 0) {
        W1Args w{dy, x, dw, d->B, d->Cout, d->Cin, d->Hout * d->Wout, accumulate};
        const dim3 grid(d->Cin / 32, d->Cout / 32);
        hipStream_t s1 = (hipStream_t)stream;
        const dim3 blk(64 * kW1Waves);
        if (dtype == LDM_DT_F16) hipLaunchKernelGGL(wgrad_1x1_kernel<1>, grid, blk, 0, s1, w);
        else if (dtype == LDM_DT_BF16) hipLaunchKernelGGL(wgrad_1x1_kernel<2>, grid, blk, 0, s1, w);
        else hipLaunchKernelGGL(wgrad_1x1_kernel<0>, grid, blk, 0, s1, w);
        LDM_CHECK_LAUNCH("wgrad_1x1_kernel");
        return 0;
    }
    WgradArgs a;
    int kk;
    int rc = wgrad_setup(*d, a, kk);
    if (rc) return rc;
    a.dense = d->transposed ? x : dy;
    a.gath = d->transposed ? dy : x;
    hipStream_t st = (hipStream_t)stream;
    const int MN = a.M * a.N;
    int S2 = 0;
    // 16-bit storage (LDM_DT_X16 / LDM_DT_DY16) as Dense / Gath flags: Dense = dy (conv) or x (convT)
    const int d16 = (st16 & (d->transposed ? LDM_DT_X16 : LDM_DT_DY16)) ? 1 : 0;
    const int g16 = (st16 & (d->transposed ? LDM_DT_DY16 : LDM_DT_X16)) ? 1 : 0;
    rc = wgrad2_run(*d, a.dense, a.gath, workspace, S2, dtype, st, d16 | (g16 << 1),   // (wgrad.hip) where it applies
                    accumulate ? nullptr : dw);
    if (rc > 0) return rc;
    LDM_REQUIRE(rc == 0 || !st16, "wgrad: 16-bit storage on a layer without the tap-shared form (ldm_conv_wgrad_storage16)");
    if (rc == 0 && S2 == 0) return 0;   // one K range, written to dw by the kernel
    if (rc == 0 && defer_s && MN % 4 == 0 && (((uintptr_t)workspace | (uintptr_t)dw) & 15) == 0) {
        *defer_s = S2;
        return 0;
    }
    if (rc == 0) {
        wgrad_reduce((const float*)workspace, S2, MN, dw, accumulate, st);
        LDM_CHECK_LAUNCH("wgrad_reduce_kernel");
        return 0;
    }
    const int S = wgrad_splits(a);
    a.per_split = (a.nchunk + S - 1) / S;
    a.partial = workspace;
    dim3 grid((a.N + 15) / 16, (a.M + 15) / 16, S);
    hipLaunchKernelGGL(wgrad_kernel, grid, dim3(64), 0, st, a);
    LDM_CHECK_LAUNCH("wgrad_kernel");
    wgrad_reduce((const float*)a.partial, S, MN, dw, accumulate, st);
    LDM_CHECK_LAUNCH("wgrad_reduce_kernel");
    return 0;
}

extern "C" int ldm_attention_backward(const float* q, const float* kv, const float* dout, float* dq, float* dkv,
                                      int32_t B, int32_t E, int32_t heads, int32_t L, int32_t S, float scale,
                                      void* stream) {
    LDM_REQUIRE(q && kv && dout && dq && dkv && B > 0 && heads > 0 && E % heads == 0, "attention_backward: bad argument");
    const int d = E / heads;
    if (L % 16 == 0 && S % 16 == 0 && d % 16 == 0) {
        const size_t lds = ((size_t)d * (L + 1) + (size_t)d * (S + 1) + 2 * (size_t)L * (S + 1)) * sizeof(float);
        if (lds <= 160 * 1024) {
            static bool opted = false;
            if (!opted) {
                LDM_HIP_TRY(hipFuncSetAttribute((const void*)attention_backward_mfma_kernel,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
                opted = true;
            }
            hipLaunchKernelGGL(attention_backward_mfma_kernel, dim3(B * heads), dim3(256), lds, (hipStream_t)stream, q,
                               kv, dout, dq, dkv, E, heads, L, S, scale);
            LDM_CHECK_LAUNCH("attention_backward_mfma_kernel");
            return 0;
        }
    }
    const size_t lds = ((size_t)d * L + (size_t)d * S + 2 * (size_t)L * S) * sizeof(float);
    LDM_REQUIRE(lds <= 64 * 1024, "attention_backward: head tile exceeds LDS budget");
    hipLaunchKernelGGL(attention_backward_kernel, dim3(B * heads), dim3(256), lds, (hipStream_t)stream, q, kv, dout, dq,
                       dkv, E, heads, L, S, scale);
    LDM_CHECK_LAUNCH("attention_backward_kernel");
    return 0;
}

extern "C" int ldm_unscale_check(const ldm_tensor_slot* slots, const int32_t* chunk_tensor, const int64_t* chunk_start,
                                 int32_t nchunks, int32_t chunk_len, const float* inv_scale, int32_t* found_inf,
                                 void* stream) {
    LDM_REQUIRE(slots && chunk_tensor && chunk_start && found_inf && nchunks >= 0, "unscale_check: bad argument");
    if (nchunks == 0) return 0;
    hipLaunchKernelGGL(unscale_check_kernel, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, slots, chunk_tensor,
                       chunk_start, chunk_len, inv_scale, found_inf);
    LDM_CHECK_LAUNCH("unscale_check_kernel");
    return 0;
}

extern "C" int ldm_adam_step(const ldm_tensor_slot* slots, const int32_t* chunk_tensor, const int64_t* chunk_start,
                             int32_t nchunks, int32_t chunk_len, double lr, double beta1, double beta2, double eps,
                             double weight_decay, int32_t decoupled, int32_t step, const int32_t* found_inf,
                             void* stream) {
    LDM_REQUIRE(slots && chunk_tensor && chunk_start && nchunks >= 0 && step >= 1, "adam_step: bad argument");
    if (nchunks == 0) return 0;
    // torch/optim/adam.py (_single_tensor_adam / _multi_tensor_adam, non-capturable): python floats
    const double bc1 = 1.0 - std::pow(beta1, (double)step);
    const double bc2 = 1.0 - std::pow(beta2, (double)step);
    const double step_size = lr / bc1;
    AdamScalars k;
    k.one_m_beta1 = (float)(1.0 - beta1);
    k.beta2 = (float)beta2;
    k.one_m_beta2 = (float)(1.0 - beta2);
    k.eps = (float)eps;
    k.weight_decay = (float)weight_decay;
    k.decay_mul = decoupled ? (float)(1.0 - lr * weight_decay) : 1.f;
    k.step_size = (float)step_size;
    k.bc2_sqrt = (float)std::sqrt(bc2);
    hipLaunchKernelGGL(adam_kernel, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, slots, chunk_tensor, chunk_start,
                       chunk_len, k, found_inf);
    LDM_CHECK_LAUNCH("adam_kernel");
    return 0;
}

extern "C" int ldm_adam_step_dev(const ldm_tensor_slot* slots, const int32_t* chunk_tensor, const int64_t* chunk_start,
                                 int32_t nchunks, int32_t chunk_len, double lr, double beta1, double beta2, double eps,
                                 double weight_decay, int32_t decoupled, float* step, const int32_t* found_inf,
                                 float* scalars, void* stream) {
    LDM_REQUIRE(slots && chunk_tensor && chunk_start && nchunks >= 0 && step && scalars, "adam_step_dev: bad argument");
    static_assert(sizeof(AdamScalars) == 8 * sizeof(float), "AdamScalars is 8 floats");
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(adam_prep_kernel, dim3(1), dim3(1), 0, st, step, found_inf, lr, beta1, beta2, eps, weight_decay,
                       (int)decoupled, reinterpret_cast<AdamScalars*>(scalars));
    LDM_CHECK_LAUNCH("adam_prep_kernel");
    if (nchunks == 0) return 0;
    hipLaunchKernelGGL(adam_kernel, dim3(nchunks), dim3(256), 0, st, slots, chunk_tensor, chunk_start, chunk_len,
                       AdamScalars{}, found_inf, reinterpret_cast<const AdamScalars*>(scalars));
    LDM_CHECK_LAUNCH("adam_kernel");
    return 0;
}

extern "C" int ldm_update_scale(float* scale, int32_t* growth_tracker, const int32_t* found_inf, float growth_factor,
                                float backoff_factor, int32_t growth_interval, void* stream) {
    LDM_REQUIRE(scale && growth_tracker && found_inf, "update_scale: bad argument");
    hipLaunchKernelGGL(update_scale_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, scale, growth_tracker, found_inf,
                       growth_factor, backoff_factor, growth_interval);
    LDM_CHECK_LAUNCH("update_scale_kernel");
    return 0;
}
