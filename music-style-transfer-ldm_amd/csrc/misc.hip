// Small fused kernels of the hot path: time MLP, cross-attention core, DDPM/DDIM scheduler updates,
// train-mode BatchNorm, activations.  All fp32; elementwise op order mirrors the reference's
// separate fp32 ATen ops exactly (no FMA contraction), so the scheduler updates are bitwise the
// reference's for identical inputs.
#include <algorithm>

#include "common.h"

#pragma clang fp contract(off)

namespace ldm {

// ------------------------------------------------------------------------------------------------
// time MLP (model.py:170-175, :239-246): one block per batch element, one thread per feature
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void time_mlp_kernel(const void* t, int t_is_float, int dim, const float* __restrict__ freqs,
                                                       const float* __restrict__ w1, const float* __restrict__ b1,
                                                       const float* __restrict__ w2, const float* __restrict__ b2,
                                                       float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* emb = sm;
    float* hid = sm + dim;
    const int b = blockIdx.x, i = threadIdx.x;
    // time[:, None] * freqs[None, :] with int64 time promoted to fp32 (model.py:244)
    const float tv = t_is_float ? ((const float*)t)[b] : (float)((const int64_t*)t)[b];
    const int half = dim / 2;
    if (i < dim) {
        const float arg = tv * freqs[i < half ? i : i - half];
        emb[i] = i < half ? sinf(arg) : cosf(arg);
    }
    __syncthreads();
    if (i < dim) {
        const float* wr = w1 + (size_t)i * dim;
        float acc = 0.f;
        for (int k = 0; k < dim; ++k) acc = fmaf(wr[k], emb[k], acc);
        const float x = acc + b1[i];
        // nn.GELU() (exact): x * 0.5 * (1 + erf(x / sqrt(2)))
        hid[i] = x * 0.5f * (1.0f + erff(x * 0.70710678118654752440f));
    }
    __syncthreads();
    if (i < dim) {
        const float* wr = w2 + (size_t)i * dim;
        float acc = 0.f;
        for (int k = 0; k < dim; ++k) acc = fmaf(wr[k], hid[k], acc);
        out[(size_t)b * dim + i] = acc + b2[i];
    }
}

// ------------------------------------------------------------------------------------------------
// cross-attention core: one block per (b, head, 16-query tile).  q [B,E,L], kv [B,2E,S] channel-major.
// out[b][h*d+c][l] = sum_s softmax_s((q*scale)[.,l] . k[.,s]) v[c][s]
// (torch.nn.functional.multi_head_attention_forward, need_weights=True path: q_scaled = q*sqrt(1/d),
//  bmm, softmax, bmm; dropout 0 in nn.MultiheadAttention(E, 4) as built at model.py:132)
// ------------------------------------------------------------------------------------------------
constexpr int kAttnLT = 16;

__global__ __launch_bounds__(256) void attention_core_kernel(const float* __restrict__ q, const float* __restrict__ kv,
                                                             float* __restrict__ out, int E, int heads, int L, int S,
                                                             float scale) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int d = E / heads;
    const int ltiles = (L + kAttnLT - 1) / kAttnLT;
    const int lt = blockIdx.x % ltiles;
    const int h = (blockIdx.x / ltiles) % heads;
    const int b = blockIdx.x / (ltiles * heads);
    const int l0 = lt * kAttnLT;
    const int nl = min(kAttnLT, L - l0);
    float* Qs = sm;                    // [d][LT]
    float* Ks = Qs + d * kAttnLT;      // [d][S]
    float* Vs = Ks + d * S;            // [d][S]
    float* Ps = Vs + d * S;            // [LT][S]
    const float* qb = q + ((size_t)b * E + (size_t)h * d) * L;
    const float* kb = kv + ((size_t)b * 2 * E + (size_t)h * d) * S;
    const float* vb = kv + ((size_t)b * 2 * E + E + (size_t)h * d) * S;
    for (int e = threadIdx.x; e < d * kAttnLT; e += blockDim.x) {
        const int c = e / kAttnLT, l = e - c * kAttnLT;
        Qs[e] = l < nl ? qb[(size_t)c * L + l0 + l] * scale : 0.f;
    }
    for (int e = threadIdx.x; e < d * S; e += blockDim.x) {
        Ks[e] = kb[e];
        Vs[e] = vb[e];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < kAttnLT * S; e += blockDim.x) {
        const int l = e / S, s = e - l * S;
        float acc = 0.f;
        for (int c = 0; c < d; ++c) acc = fmaf(Qs[c * kAttnLT + l], Ks[c * S + s], acc);
        Ps[e] = acc;
    }
    __syncthreads();
    // softmax over s: one wave per query row
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int l = wave; l < nl; l += nw) {
        float* row = Ps + l * S;
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
    float* ob = out + ((size_t)b * E + (size_t)h * d) * L;
    for (int e = threadIdx.x; e < d * kAttnLT; e += blockDim.x) {
        const int c = e / kAttnLT, l = e - c * kAttnLT;
        if (l >= nl) continue;
        float acc = 0.f;
        const float* pr = Ps + l * S;
        const float* vr = Vs + c * S;
        for (int s = 0; s < S; ++s) acc = fmaf(pr[s], vr[s], acc);
        ob[(size_t)c * L + l0 + l] = acc;
    }
}

// ------------------------------------------------------------------------------------------------
// cross-attention core on f32 MFMA: one block (4 waves) per (b, head).
//   S = (q*scale)^T k   : A[m=l][k=c] = q[c][l], B[k=c][n=s] = k[c][s] — both read straight from the
//                         channel-major projections (lanes walk l / s: coalesced), tiles round-robin
//                         over waves, written to LDS
//   P = softmax_s(S)    : one wave per query row, padded columns -> 0
//   O = V P^T           : A[m=c][k=s] = V[c][s] (staged in LDS), B[k=s][n=l] = P[l][s] (LDS),
//                         stored channel-major out[b][h*d+c][l] (coalesced along l)
// KIND 1 = v_mfma_f32_32x32x2_f32 (L, S > 16), KIND 2 = v_mfma_f32_16x16x4_f32 (small maps).
// ------------------------------------------------------------------------------------------------
template <int KIND>
struct AMfma;
template <>
struct AMfma<1> {
    static constexpr int TILE = 32, NLG = 2, NACC = 16;
    typedef floatx16 acc_t;
    static __device__ __forceinline__ acc_t mma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int r, int lg) { return (r & 3) + 8 * (r >> 2) + 4 * lg; }
};
template <>
struct AMfma<2> {
    static constexpr int TILE = 16, NLG = 4, NACC = 4;
    typedef floatx4 acc_t;
    static __device__ __forceinline__ acc_t mma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int r, int lg) { return 4 * lg + r; }
};

// Compile-time padded sizes LP x SP and head dim D (instances in ldm_attention_core); the actual L, S
// (<= LP, SP) are runtime and masked.  All index math folds to shifts.
// Each block owns LT query rows of one (b, head): grid = B * heads * (LP / LT).
// TOK: q and out are token-major [B,L,E] (the UNet engine's NHWC activations) instead of [B,E,L].
// EQ > 0 (folded query projection, token-major only): `q` is the projection's INPUT z [B,L,E=EQ] and
// the scores are z^T kf[b,h] + bf[b,h] with kf [B,heads,S,E] = scale*Wq_h^T K_h and bf [B,heads,S] =
// scale*bq_h^T K_h (ldm_attention_fold_keys) — the same scores as ((Wq z + bq)*scale)^T K re-associated,
// so the Q in-projection needs no launch of its own.
// PONLY (folded instances): stop after the softmax and write the probabilities P [B, heads, L, S] (S fastest) to
// `out` instead of P V — the bottleneck after CA1 contracts P with values folded into its weights (bfold.hip).
template <int KIND, int LP, int SP, int D, int LT, bool TOK, int EQ = 0, int NW = 4, bool PONLY = false>
__global__ __launch_bounds__(64 * NW) void attention_mfma_kernel(const float* __restrict__ q, const float* __restrict__ kv,
                                                             float* __restrict__ out, int E, int heads, int L, int S,
                                                             float scale, const float* __restrict__ kf = nullptr,
                                                             const float* __restrict__ bf = nullptr) {
    using MF = AMfma<KIND>;
    constexpr int TILE = MF::TILE, NLG = MF::NLG;
    static_assert(LT % TILE == 0 && LP % LT == 0, "query split");
    static_assert(EQ == 0 || TOK, "folded queries are token-major");
    constexpr int DQ = EQ ? EQ : D;                       // contraction length of the scores
    constexpr int KBQ = DQ / NLG < 16 ? DQ / NLG : 16;   // k-steps per register batch (QK^T)
    constexpr int KBP = SP / NLG < 16 ? SP / NLG : 16;    // (PV)
    static_assert(LP % TILE == 0 && SP % TILE == 0 && D % TILE == 0 && DQ % (KBQ * NLG) == 0 &&
                      SP % (KBP * NLG) == 0 && SP <= 64 * 64,
                  "attention instance shape");
    constexpr int LDP = SP + 1;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* Ps = sm;                                // [LT][SP+1]  (rows l0 .. l0+LT-1); folded: 4 slabs
    float* Vs = sm + (EQ > 0 ? NW : 1) * LT * LDP;  // [D][SP+1]
    constexpr int NSPLIT = LP / LT;
    const int l0 = (blockIdx.x % NSPLIT) * LT;
    const int bh = blockIdx.x / NSPLIT;
    const int h = bh % heads, b = bh / heads;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int col = lane % TILE, lg = lane / TILE;
    const float* qb = EQ ? q + (size_t)b * L * E
                         : (TOK ? q + (size_t)b * L * E + (size_t)h * D : q + ((size_t)b * E + (size_t)h * D) * L);
    const int qcs = TOK ? 1 : L, qls = TOK ? E : 1;   // q element (c, l) at qb[c*qcs + l*qls]
    const float* kb = EQ ? kf + (size_t)(b * heads + h) * E * S : kv + ((size_t)b * 2 * E + (size_t)h * D) * S;
    const float* vb = kv + ((size_t)b * 2 * E + E + (size_t)h * D) * S;

    // stage V [D][S] -> LDS [D][SP+1]: every load of this thread issues before any LDS store
    if constexpr (PONLY) {
    } else if (S == SP && (D * SP) % (256 * NW) == 0 && D * SP >= 256 * NW) {   // full rows: 16-byte loads
        constexpr int NV4 = D * SP >= 256 * NW ? D * SP / (256 * NW) : 1;
        float4 v[NV4];
#pragma unroll
        for (int u = 0; u < NV4; ++u) v[u] = reinterpret_cast<const float4*>(vb)[u * 64 * NW + (int)threadIdx.x];
#pragma unroll
        for (int u = 0; u < NV4; ++u) {
            const int e = 4 * (u * 64 * NW + (int)threadIdx.x);
            const int c = e / SP, s = e % SP;
            float* dst = Vs + c * LDP + s;
            dst[0] = v[u].x;
            dst[1] = v[u].y;
            dst[2] = v[u].z;
            dst[3] = v[u].w;
        }
    } else {
        constexpr int NV = (D * SP + 64 * NW - 1) / (64 * NW);
        float v[NV];
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const int e = u * 64 * NW + (int)threadIdx.x;
            const int c = e / SP, s = e % SP;
            v[u] = vb[(e < D * SP && s < S) ? c * S + s : 0];
        }
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const int e = u * 64 * NW + (int)threadIdx.x;
            const int c = e / SP, s = e % SP;
            if (e < D * SP) Vs[c * LDP + s] = s < S ? v[u] : 0.f;
        }
    }
    constexpr int NTL = LT / TILE, NTS = SP / TILE;
    if constexpr (EQ > 0) {
        // Folded scores z^T kf: the E-long contraction is split over the 4 waves (each covers every tile
        // of the block over E/4, all of its operand loads in flight at once — a single memory round
        // trip), partial tiles go to 4 LDS slabs and the softmax pass below sums them in wave order.
        // Both operands are E-contiguous (z token-major, kf [B,heads,S,E]), so MFMA step j = 4*jj + i
        // takes lane group lg's k = kbase + 16*jj + 4*lg + i: one 16-byte load feeds 4 steps.
        constexpr int NSTEP = DQ / NW / NLG;
        static_assert(NLG == 4 && DQ % (NW * 16) == 0 && NTL * NSTEP + NTS * NSTEP <= 96, "folded score tile");
        const int kbase = wave * (DQ / NW);
        float av[NTL][NSTEP], bv[NTS][NSTEP];
#pragma unroll
        for (int lt = 0; lt < NTL; ++lt) {
            const int l = l0 + lt * TILE + col;
            const float4* zp = reinterpret_cast<const float4*>(qb + (size_t)(l < L ? l : 0) * E + kbase + 4 * lg);
#pragma unroll
            for (int jj = 0; jj < NSTEP / 4; ++jj) {
                const float4 v = zp[4 * jj];
                av[lt][4 * jj + 0] = l < L ? v.x : 0.f;
                av[lt][4 * jj + 1] = l < L ? v.y : 0.f;
                av[lt][4 * jj + 2] = l < L ? v.z : 0.f;
                av[lt][4 * jj + 3] = l < L ? v.w : 0.f;
            }
        }
#pragma unroll
        for (int st = 0; st < NTS; ++st) {
            const int s = st * TILE + col;
            const float4* kp = reinterpret_cast<const float4*>(kb + (size_t)(s < S ? s : 0) * E + kbase + 4 * lg);
#pragma unroll
            for (int jj = 0; jj < NSTEP / 4; ++jj) {
                const float4 v = kp[4 * jj];
                bv[st][4 * jj + 0] = s < S ? v.x : 0.f;
                bv[st][4 * jj + 1] = s < S ? v.y : 0.f;
                bv[st][4 * jj + 2] = s < S ? v.z : 0.f;
                bv[st][4 * jj + 3] = s < S ? v.w : 0.f;
            }
        }
        float* Pw = Ps + (size_t)wave * LT * LDP;
#pragma unroll
        for (int lt = 0; lt < NTL; ++lt)
#pragma unroll
            for (int st = 0; st < NTS; ++st) {
                typename MF::acc_t acc;
#pragma unroll
                for (int r = 0; r < MF::NACC; ++r) acc[r] = 0.f;
#pragma unroll
                for (int j = 0; j < NSTEP; ++j) acc = MF::mma(av[lt][j], bv[st][j], acc);
#pragma unroll
                for (int r = 0; r < MF::NACC; ++r) Pw[(lt * TILE + MF::row(r, lg)) * LDP + st * TILE + col] = acc[r];
            }
    }
    // S = (q*scale)^T k for this block's LT rows: tiles round-robin over the 4 waves
    for (int tile = wave; tile < (EQ > 0 ? 0 : NTL * NTS); tile += NW) {
        const int lt = tile / NTS, st = tile % NTS;
        const int l = l0 + lt * TILE + col, s = st * TILE + col;
        const bool lok = l < L, sok = s < S;
        typename MF::acc_t acc;
#pragma unroll
        for (int r = 0; r < MF::NACC; ++r) acc[r] = 0.f;
        const float* qp = qb + lg * qcs + (lok ? l : 0) * qls;
        const float* kp = kb + lg * S + (sok ? s : 0);
#pragma unroll
        for (int k0 = 0; k0 < DQ; k0 += KBQ * NLG) {
            float av[KBQ], bv[KBQ];
#pragma unroll
            for (int j = 0; j < KBQ; ++j) {   // the whole batch in flight before its MFMAs
                av[j] = qp[(k0 + NLG * j) * qcs];
                bv[j] = kp[(k0 + NLG * j) * S];
            }
#pragma unroll
            for (int j = 0; j < KBQ; ++j) {
                if constexpr (EQ) acc = MF::mma(lok ? av[j] : 0.f, sok ? bv[j] : 0.f, acc);
                else acc = MF::mma(lok ? av[j] * scale : 0.f, sok ? bv[j] : 0.f, acc);   // q_scaled = q * sqrt(1/d)
            }
        }

#pragma unroll
        for (int r = 0; r < MF::NACC; ++r) Ps[(lt * TILE + MF::row(r, lg)) * LDP + st * TILE + col] = acc[r];
    }
    __syncthreads();
    // softmax over s: RPW = 64/SP rows per wave pass, one lane per column, segmented shuffles
    {
        constexpr int RPW = SP >= 64 ? 1 : 64 / SP;
        constexpr int SEG = SP >= 64 ? 64 : SP;
        const int sub = lane / SEG, s0 = lane % SEG;
        for (int r0 = wave * RPW; r0 < LT; r0 += NW * RPW) {
            const int r = r0 + sub;             // local row; global query row l0 + r
            float* row = Ps + r * LDP;
            float x[SP / SEG];
            float mx = -INFINITY;
#pragma unroll
            for (int u = 0; u < SP / SEG; ++u) {
                const int s = s0 + u * SEG;
                if constexpr (EQ > 0) {   // sum the 4 wave slabs in wave order, then the folded bias
                    float v = row[s];
#pragma unroll
                    for (int w = 1; w < NW; ++w) v = v + row[s + w * LT * LDP];
                    x[u] = v + (s < S ? bf[(size_t)(b * heads + h) * S + s] : 0.f);
                } else {
                    x[u] = row[s];
                }
                if (s < S) mx = fmaxf(mx, x[u]);
            }
#pragma unroll
            for (int o = SEG / 2; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
            float sum = 0.f;
#pragma unroll
            for (int u = 0; u < SP / SEG; ++u) {
                const int s = s0 + u * SEG;
                x[u] = s < S ? expf(x[u] - mx) : 0.f;
                sum += x[u];
            }
#pragma unroll
            for (int o = SEG / 2; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
#pragma unroll
            for (int u = 0; u < SP / SEG; ++u) row[s0 + u * SEG] = l0 + r < L ? x[u] / sum : 0.f;
        }
    }
    __syncthreads();
    if constexpr (PONLY) {
        float* pb = out + ((size_t)(b * heads + h) * L + l0) * S;
        for (int e = threadIdx.x; e < LT * SP; e += 64 * NW) {
            const int r = e / SP, s = e % SP;
            if (l0 + r < L && s < S) pb[(size_t)r * S + s] = Ps[r * LDP + s];
        }
        return;
    }
    // O[c][l] = sum_s V[c][s] P[l][s]
    constexpr int NTC = D / TILE;
    float* ob = TOK ? out + (size_t)b * L * E + (size_t)h * D : out + ((size_t)b * E + (size_t)h * D) * L;
    for (int tile = wave; tile < NTC * NTL; tile += NW) {
        const int ct = tile / NTL, lt = tile % NTL;
        typename MF::acc_t acc;
#pragma unroll
        for (int r = 0; r < MF::NACC; ++r) acc[r] = 0.f;
        const float* va = Vs + (ct * TILE + col) * LDP + lg;
        const float* pb = Ps + (lt * TILE + col) * LDP + lg;
#pragma unroll
        for (int k0 = 0; k0 < SP; k0 += KBP * NLG) {
            float av[KBP], bv[KBP];
#pragma unroll
            for (int j = 0; j < KBP; ++j) {
                av[j] = va[k0 + NLG * j];
                bv[j] = pb[k0 + NLG * j];
            }
#pragma unroll
            for (int j = 0; j < KBP; ++j) acc = MF::mma(av[j], bv[j], acc);
        }
        const int l = l0 + lt * TILE + col;
        if (l < L) {
            if constexpr (TOK && KIND == 2) {   // rows 4*lg .. 4*lg+3 = 4 consecutive channels of token l
                *reinterpret_cast<float4*>(ob + (size_t)l * E + ct * TILE + 4 * lg) = make_float4(acc[0], acc[1], acc[2], acc[3]);
            } else {
#pragma unroll
                for (int r = 0; r < MF::NACC; ++r) ob[(ct * TILE + MF::row(r, lg)) * qcs + l * qls] = acc[r];
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Folds for the reverse loop (style fixed over the loop, weights fixed between optimiser steps).
// ------------------------------------------------------------------------------------------------
// kf[b,h,s,e] = scale * sum_c Wq[h*d+c, e] K[b, h*d+c, s];  bf[b,h,s] = scale * sum_c bq[h*d+c] K[b,h*d+c,s]
// (fp64 accumulation, one rounding to fp32).  kv [B,2E,S] channel-major; wq [E,E] torch Linear layout.
__global__ __launch_bounds__(256) void attention_fold_keys_kernel(const float* __restrict__ kv, const float* __restrict__ wq,
                                                                  const float* __restrict__ bq, int B, int E, int heads,
                                                                  int S, float scale, float* __restrict__ kf,
                                                                  float* __restrict__ bf, int64_t first) {
    const int d = E / heads;
    const int64_t nk = (int64_t)B * heads * E * S;
    const int64_t idx = first + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // first = nk: bf only
    if (idx < nk) {   // kf [B,heads,S,E]: e fastest (the attention reads 16-byte runs along E)
        const int e = (int)(idx % E);
        int64_t r = idx / E;
        const int s = (int)(r % S);
        r /= S;
        const int h = (int)(r % heads), b = (int)(r / heads);
        const float* kr = kv + ((int64_t)b * 2 * E + (int64_t)h * d) * S + s;
        const float* wr = wq + (int64_t)h * d * E + e;
        double acc = 0.0;
        // 16 channels' loads in flight per step: the sum stays serial in c (same roundings), but the loads no
        // longer wait one L2 round trip each (64-128 dependent rounds made this a 30 us launch)
        int c = 0;
        for (; c + 16 <= d; c += 16) {
            float wv[16], kvv[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                wv[u] = wr[(int64_t)(c + u) * E];
                kvv[u] = kr[(int64_t)(c + u) * S];
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) acc += (double)wv[u] * (double)kvv[u];
        }
        for (; c < d; ++c) acc += (double)wr[(int64_t)c * E] * (double)kr[(int64_t)c * S];
        kf[idx] = (float)(acc * (double)scale);
    } else if (idx < nk + (int64_t)B * heads * S) {
        const int64_t j = idx - nk;
        const int s = (int)(j % S);
        const int bh = (int)(j / S);
        const int h = bh % heads, b = bh / heads;
        const float* kr = kv + ((int64_t)b * 2 * E + (int64_t)h * d) * S + s;
        double acc = 0.0;
        for (int c = 0; c < d; ++c) acc += (double)bq[h * d + c] * (double)kr[(int64_t)c * S];
        bf[j] = (float)(acc * (double)scale);
    }
}

// The same folded keys, four key positions per thread (S % 4 == 0): each Wq element loaded once feeds four
// fp64 sums (the one-output-per-thread form re-reads Wq once per key position: 268 MB of L1/L2 traffic for
// CA2 at B = 8), the four K values of a channel are one 16-byte broadcast load, and 16 channels' loads are
// in flight per step.  Each sum runs serially in c as in attention_fold_keys_kernel: the same roundings.
__global__ __launch_bounds__(256) void attention_fold_keys4_kernel(const float* __restrict__ kv, const float* __restrict__ wq,
                                                                   const float* __restrict__ bq, int B, int E, int heads,
                                                                   int S, float scale, float* __restrict__ kf,
                                                                   float* __restrict__ bf) {
    // column e == E of the (b, h, key group) row is the bias fold bf (w = bq instead of a Wq column)
    const int d = E / heads;
    const int SG = S / 4;
    const int64_t n = (int64_t)B * heads * SG * (E + 1);
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n) return;
    const int e = (int)(idx % (E + 1));
    int64_t r = idx / (E + 1);
    const int sg = (int)(r % SG);
    r /= SG;
    const int h = (int)(r % heads), b = (int)(r / heads);
    const float* kr = kv + ((int64_t)b * 2 * E + (int64_t)h * d) * S + sg * 4;
    const bool isb = e == E;
    const float* wr = isb ? bq + h * d : wq + (int64_t)h * d * E + e;
    const int64_t ws = isb ? 1 : E;
    double acc[4] = {0., 0., 0., 0.};
    int c = 0;
    for (; c + 16 <= d; c += 16) {
        float wv[16];
        float4 kq[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            wv[u] = wr[(int64_t)(c + u) * ws];
            kq[u] = *reinterpret_cast<const float4*>(kr + (int64_t)(c + u) * S);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const double w = (double)wv[u];
            acc[0] += w * (double)kq[u].x;
            acc[1] += w * (double)kq[u].y;
            acc[2] += w * (double)kq[u].z;
            acc[3] += w * (double)kq[u].w;
        }
    }
    for (; c < d; ++c) {
        const double w = (double)wr[(int64_t)c * ws];
        const float4 k = *reinterpret_cast<const float4*>(kr + (int64_t)c * S);
        acc[0] += w * (double)k.x;
        acc[1] += w * (double)k.y;
        acc[2] += w * (double)k.z;
        acc[3] += w * (double)k.w;
    }
    if (isb) {
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[((int64_t)b * heads + h) * S + sg * 4 + j] = (float)(acc[j] * (double)scale);
        return;
    }
    float* out = kf + (((int64_t)b * heads + h) * S + sg * 4) * E + e;
#pragma unroll
    for (int j = 0; j < 4; ++j) out[(int64_t)j * E] = (float)(acc[j] * (double)scale);
}

// W'[co, ci, t] = sum_j Wc[co, j, t] Wp[j, ci]  (conv after a Linear/1x1 projection, composed), and the
// projection bias pushed through the window: pb[co, oy, ox] = bc[co] + sum_{taps t inside the input}
// sum_j Wc[co, j, t] bp[j].  fp64 accumulation, one rounding.
__global__ __launch_bounds__(256) void fold_conv_proj_kernel(const float* __restrict__ wc, const float* __restrict__ bc,
                                                             const float* __restrict__ wp, const float* __restrict__ bp,
                                                             int Cout, int Cmid, int Cin, int kh, int kw, int stride,
                                                             int pad, int Hin, int Win, int Hout, int Wout,
                                                             float* __restrict__ w_out, float* __restrict__ pb_out) {
    const int KK = kh * kw;
    const int64_t nw = (int64_t)Cout * Cin * KK;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx < nw) {
        const int t = (int)(idx % KK);
        const int64_t r = idx / KK;
        const int ci = (int)(r % Cin), co = (int)(r / Cin);
        const float* wr = wc + (int64_t)co * Cmid * KK + t;
        double acc = 0.0;
        for (int j = 0; j < Cmid; ++j) acc += (double)wr[(int64_t)j * KK] * (double)wp[(int64_t)j * Cin + ci];
        w_out[idx] = (float)acc;
    } else if (idx < nw + (int64_t)Cout * Hout * Wout) {
        const int64_t p = idx - nw;
        const int ox = (int)(p % Wout);
        const int oy = (int)((p / Wout) % Hout);
        const int co = (int)(p / ((int64_t)Hout * Wout));
        double acc = bc ? (double)bc[co] : 0.0;
        for (int ky = 0; ky < kh; ++ky) {
            const int iy = oy * stride - pad + ky;
            if (iy < 0 || iy >= Hin) continue;
            for (int kx = 0; kx < kw; ++kx) {
                const int ix = ox * stride - pad + kx;
                if (ix < 0 || ix >= Win) continue;
                const float* wr = wc + (int64_t)co * Cmid * KK + ky * kw + kx;
                for (int j = 0; j < Cmid; ++j) acc += (double)wr[(int64_t)j * KK] * (double)bp[j];
            }
        }
        pb_out[p] = (float)acc;
    }
}

// ------------------------------------------------------------------------------------------------
// scheduler updates
// ------------------------------------------------------------------------------------------------
// coef_table [T,2] = {sqrt(ab), sqrt(1-ab)} per timestep (host-computed with the reference's fp32
// torch.sqrt); t [B] int64 on device.  An out-of-range t (the reference raises IndexError,
// model.py:107) poisons the sample with NaN instead of reading out of bounds.
__device__ __forceinline__ bool load_coef(const float* table, int T, const int64_t* t, int b, float& sa, float& s1) {
    const int64_t tb = t[b];
    if (tb < 0 || tb >= T) {
        sa = s1 = __builtin_nanf("");
        return false;
    }
    sa = table[2 * tb];
    s1 = table[2 * tb + 1];
    return true;
}

__global__ __launch_bounds__(256) void q_sample_kernel(const float* __restrict__ x0, const float* __restrict__ eps,
                                                       const float* __restrict__ table, int T,
                                                       const int64_t* __restrict__ t, float* __restrict__ zt,
                                                       int64_t per_sample, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float sa, s1;
    load_coef(table, T, t, (int)(i / per_sample), sa, s1);
    // torch.sqrt(alpha_bar_t) * x_0 + torch.sqrt(1 - alpha_bar_t) * eps   (model.py:113)
    const float u = sa * x0[i];
    const float v = s1 * eps[i];
    zt[i] = u + v;
}

__global__ __launch_bounds__(256) void predict_start_kernel(const float* __restrict__ zt, const float* __restrict__ eps,
                                                            const float* __restrict__ table, int T,
                                                            const int64_t* __restrict__ t, float* __restrict__ x0,
                                                            int64_t per_sample, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float sa, s1;
    load_coef(table, T, t, (int)(i / per_sample), sa, s1);
    // (z_t - torch.sqrt(1 - alpha_bar_t) * noise_pred) / torch.sqrt(alpha_bar_t)   (model.py:124)
    const float v = s1 * eps[i];
    x0[i] = (zt[i] - v) / sa;
}

// backward of q_sample (kind 0: ga = sa*g, gb = s1*g) and predict_start (kind 1: ga = g/sa, gb = -(s1*g)/sa)
__global__ __launch_bounds__(256) void sched_backward_kernel(int kind, const float* __restrict__ g,
                                                             const float* __restrict__ table, int T,
                                                             const int64_t* __restrict__ t, float* __restrict__ ga,
                                                             float* __restrict__ gb, int64_t per_sample, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float sa, s1;
    load_coef(table, T, t, (int)(i / per_sample), sa, s1);
    const float gv = g[i];
    if (kind == 0) {
        if (ga) ga[i] = sa * gv;
        if (gb) gb[i] = s1 * gv;
    } else {
        if (ga) ga[i] = gv / sa;
        if (gb) gb[i] = -(s1 * gv) / sa;
    }
}

__global__ __launch_bounds__(256) void ddim_step_kernel(float* __restrict__ x, const float* __restrict__ eps,
                                                        const float* __restrict__ coef, float eta,
                                                        float* __restrict__ x0_log, float* __restrict__ eps_log,
                                                        int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float e = eps[i];
    float x0;
    x[i] = ddim_update(x[i], e, coef, eta, x0);   // model.py:446-458
    if (x0_log) x0_log[i] = x0;
    if (eps_log) eps_log[i] = e;
}

// (train-mode BatchNorm2d lives in reduce.hip)

__global__ __launch_bounds__(256) void activation_kernel(const float* x, float* y, int64_t n, int act) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = apply_act(x[i], act);
}

__global__ __launch_bounds__(256) void batchnorm_eval_kernel(const float* x, float* y, int C, int HW, int64_t n,
                                                             const float* __restrict__ w, const float* __restrict__ b,
                                                             const float* __restrict__ rm, const float* __restrict__ rv,
                                                             float eps, int act) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int c = (int)((i / HW) % C);
    const float invstd = 1.0f / sqrtf(rv[c] + eps);
    const float alpha = invstd * (w ? w[c] : 1.0f);
    const float beta = (b ? b[c] : 0.0f) - rm[c] * alpha;
    y[i] = apply_act(x[i] * alpha + beta, act);
}

__global__ __launch_bounds__(256) void sinusoid_kernel(const void* t, int t_is_float, int B, int dim,
                                                       const float* __restrict__ freqs, float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * dim) return;
    const int b = i / dim, k = i - b * dim, half = dim / 2;
    const float tv = t_is_float ? ((const float*)t)[b] : (float)((const int64_t*)t)[b];
    const float arg = tv * freqs[k < half ? k : k - half];
    out[i] = k < half ? sinf(arg) : cosf(arg);
}

// ------------------------------------------------------------------------------------------------
// loss reductions (deterministic: fixed block partition, fp64 partials, one final block)
//   kind 0: mean((a-b)^2)                                  F.mse_loss / nn.MSELoss (loss.py:35,49)
//   kind 1: mean(0.5*(a^2 - 1 - log(a^2 + 1e-8)))          kl_regularization_loss (loss.py:31-32)
// ------------------------------------------------------------------------------------------------
constexpr int kLossBlocks = 512;

__device__ __forceinline__ float loss_term(int kind, float a, float b) {
    if (kind == 0) {
        const float d = a - b;
        return d * d;
    }
    const float a2 = a * a;
    return 0.5f * ((a2 - 1.0f) - logf(a2 + 1e-8f));
}

__global__ __launch_bounds__(256) void loss_partial_kernel(int kind, const float* __restrict__ a,
                                                           const float* __restrict__ b, int64_t n,
                                                           double* __restrict__ partial) {
    __shared__ double red[16];
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        s += (double)loss_term(kind, a[i], b ? b[i] : 0.f);
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
        partial[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(64) void loss_final_kernel(const double* __restrict__ partial, int np, int64_t n,
                                                        float* __restrict__ out) {
    double s = 0.0;
    for (int i = threadIdx.x; i < np; i += 64) s += partial[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (threadIdx.x == 0) out[0] = (float)(s / (double)n);
}

// d/da of the mean loss times upstream scalar gradient g (device scalar)
__global__ __launch_bounds__(256) void loss_backward_kernel(int kind, const float* __restrict__ a,
                                                            const float* __restrict__ b, int64_t n,
                                                            const float* __restrict__ g, float* __restrict__ ga,
                                                            float* __restrict__ gb) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float scale = g[0] / (float)n;
    if (kind == 0) {
        const float d = 2.0f * (a[i] - (b ? b[i] : 0.f)) * scale;
        if (ga) ga[i] = d;
        if (gb) gb[i] = -d;
    } else {
        // d/da 0.5*(a^2 - 1 - log(a^2+eps)) = a - a/(a^2+eps)
        const float av = a[i];
        const float a2 = av * av;
        if (ga) ga[i] = (av - av / (a2 + 1e-8f)) * scale;
    }
}

static unsigned blocks_for(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

}  // namespace ldm

using namespace ldm;

extern "C" int ldm_time_mlp_forward(const void* t, int32_t t_is_float, int32_t B, int32_t dim, const float* freqs,
                                    const float* w1, const float* b1, const float* w2, const float* b2, float* out,
                                    void* stream) {
    LDM_REQUIRE(t && freqs && w1 && b1 && w2 && b2 && out, "time_mlp: null argument");
    LDM_REQUIRE(B > 0 && dim > 1 && dim % 2 == 0 && dim <= 256, "time_mlp: unsupported dim");
    const int threads = (dim + 63) / 64 * 64;
    hipLaunchKernelGGL(time_mlp_kernel, dim3(B), dim3(threads), 2 * dim * sizeof(float), (hipStream_t)stream, t,
                       t_is_float, dim, freqs, w1, b1, w2, b2, out);
    LDM_CHECK_LAUNCH("time_mlp_kernel");
    return 0;
}

namespace ldm {
int attention_folded(const float* z, const float* kv, const float* kf, const float* bf, float* out, int32_t B,
                     int32_t E, int32_t heads, int32_t L, int32_t S, hipStream_t st) {
    LDM_REQUIRE(z && kv && kf && bf && out, "attention (folded): null argument");
    LDM_REQUIRE(B > 0 && heads == 4 && L > 0 && S > 0, "attention (folded): bad shape");
    const int d = E / heads;
#define LDM_ATTF(LP, SP, D, LT, EQV, NWV)                                                                \
    if (d == D && E == EQV && L <= LP && S <= SP) {                                                      \
        const size_t lds = ((size_t)NWV * LT * (SP + 1) + (size_t)D * (SP + 1)) * sizeof(float);       \
        if (lds > 64 * 1024) {                                                                           \
            static bool opted = false;                                                                   \
            if (!opted) {                                                                                \
                LDM_HIP_TRY(hipFuncSetAttribute(                                                         \
                    (const void*)attention_mfma_kernel<2, LP, SP, D, LT, true, EQV, NWV>,                  \
                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));                            \
                opted = true;                                                                            \
            }                                                                                            \
        }                                                                                                \
        hipLaunchKernelGGL((attention_mfma_kernel<2, LP, SP, D, LT, true, EQV, NWV>), dim3(B * heads * (LP / LT)), \
                           dim3(64 * NWV), lds, st, z, kv, out, E, heads, L, S, 1.0f, kf, bf);           \
        LDM_CHECK_LAUNCH("attention_mfma_kernel (folded)");                                              \
        return 0;                                                                                        \
    }
    LDM_ATTF(16, 16, 128, 16, 512, 8)
    LDM_ATTF(64, 64, 64, 16, 256, 16)
    LDM_ATTF(32, 32, 64, 16, 256, 8)
    LDM_ATTF(32, 32, 128, 16, 512, 8)
    LDM_ATTF(16, 16, 64, 16, 256, 4)
#undef LDM_ATTF
    return fail(3, "attention (folded): no instance for this shape");
}

// The probabilities of the folded cross-attention only (P [B, heads, L, S]): the CA1 instance of
// attention_folded without its P V product.
int attention_folded_probs(const float* z, const float* kf, const float* bf, float* p, int32_t B, int32_t E,
                           int32_t heads, int32_t L, int32_t S, hipStream_t st) {
    LDM_REQUIRE(z && kf && bf && p, "attention probs (folded): null argument");
    LDM_REQUIRE(B > 0 && heads == 4 && E == 512 && L > 0 && L <= 16 && S > 0 && S <= 16,
                "attention probs (folded): instances for CA1's 2 x 8 plane only (E 512, L, S <= 16)");
    // waves splitting the E-long score contraction (LDM_CA1P_WAVES: 8 or 16; A/B timing)
    static const int nw = [] {
        const char* e = std::getenv("LDM_CA1P_WAVES");
        return e && std::atoi(e) == 16 ? 16 : 8;
    }();
    if (nw == 16) {
        auto kfn = attention_mfma_kernel<2, 16, 16, 128, 16, true, 512, 16, true>;
        const size_t lds = ((size_t)16 * 16 * 17 + (size_t)128 * 17) * sizeof(float);
        hipLaunchKernelGGL(kfn, dim3(B * heads), dim3(64 * 16), lds, st, z, kf, p, E, heads, L, S, 1.0f, kf, bf);
    } else {
        auto kfn = attention_mfma_kernel<2, 16, 16, 128, 16, true, 512, 8, true>;
        const size_t lds = ((size_t)8 * 16 * 17 + (size_t)128 * 17) * sizeof(float);
        hipLaunchKernelGGL(kfn, dim3(B * heads), dim3(64 * 8), lds, st, z, kf, p, E, heads, L, S, 1.0f, kf, bf);   // (kv unread)
    }
    LDM_CHECK_LAUNCH("attention_mfma_kernel (folded, probabilities)");
    return 0;
}

int attention_fold_keys(const float* kv, const float* wq, const float* bq, int32_t B, int32_t E, int32_t heads,
                        int32_t S, float scale, float* kf, float* bf, hipStream_t st) {
    LDM_REQUIRE(kv && wq && bq && kf && bf && B > 0 && heads > 0 && E % heads == 0 && S > 0, "fold keys: bad argument");
    const int64_t nk = (int64_t)B * heads * E * S, nb = (int64_t)B * heads * S;
    static const bool k4_on = [] {   // LDM_FOLD_KEYS4=0: the one-output-per-thread kernel only (A/B timing)
        const char* e = std::getenv("LDM_FOLD_KEYS4");
        return e ? std::atoi(e) != 0 : true;
    }();
    const bool k4 = k4_on && S % 4 == 0 && ((uintptr_t)kv & 15) == 0;
    if (k4) {   // keys and bias in one launch
        const int64_t n4 = (int64_t)B * heads * (S / 4) * (E + 1);
        hipLaunchKernelGGL(attention_fold_keys4_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, kv, wq, bq,
                           B, E, heads, S, scale, kf, bf);
        LDM_CHECK_LAUNCH("attention_fold_keys4_kernel");
        return 0;
    }
    const int64_t first = 0, n = nk + nb - first;
    hipLaunchKernelGGL(attention_fold_keys_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, kv, wq, bq, B,
                       E, heads, S, scale, kf, bf, first);
    LDM_CHECK_LAUNCH("attention_fold_keys_kernel");
    return 0;
}

int attention_core_ex(const float* q, const float* kv, float* out, int32_t B, int32_t E, int32_t heads, int32_t L,
                      int32_t S, float scale, bool tok, hipStream_t st) {
    LDM_REQUIRE(q && kv && out, "attention: null argument");
    LDM_REQUIRE(B > 0 && heads > 0 && E % heads == 0 && L > 0 && S > 0, "attention: bad shape");
    const int d = E / heads;
    {
        // compile-time instances covering the UNet's maps (128x512 mel: L=64 / 16; 128x128: 16 / 4)
        const dim3 blk(256);
#define LDM_ATT(KIND, LP, SP, D, LT)                                                                      \
    if (d == D && L <= LP && S <= SP) {                                                                   \
        const size_t lds = ((size_t)LT * (SP + 1) + (size_t)D * (SP + 1)) * sizeof(float);              \
        if (tok)                                                                                          \
            hipLaunchKernelGGL((attention_mfma_kernel<KIND, LP, SP, D, LT, true>), dim3(B * heads * (LP / LT)), blk, \
                               lds, st, q, kv, out, E, heads, L, S, scale);                               \
        else                                                                                              \
            hipLaunchKernelGGL((attention_mfma_kernel<KIND, LP, SP, D, LT, false>), dim3(B * heads * (LP / LT)), \
                               blk, lds, st, q, kv, out, E, heads, L, S, scale);                          \
        LDM_CHECK_LAUNCH("attention_mfma_kernel");                                                        \
        return 0;                                                                                         \
    }
        LDM_ATT(2, 16, 16, 64, 16)
        LDM_ATT(2, 16, 16, 128, 16)
        LDM_ATT(2, 32, 32, 64, 16)
        LDM_ATT(2, 32, 32, 128, 16)
        LDM_ATT(2, 64, 64, 64, 16)
        LDM_ATT(2, 64, 64, 128, 16)
#undef LDM_ATT
    }
    // wider maps (L or S > 64: mels wider than 512 frames, SURVEY's shape S): KV-tiled online softmax
    if (attention_flash_supported(E, heads)) return attention_flash(q, kv, out, nullptr, B, E, heads, L, S, scale, tok, st);
    // generic VALU fallback (head dims not a multiple of the MFMA tile)
    LDM_REQUIRE(!tok, "attention: token-major layout needs an MFMA instance for this head size");
    const size_t lds = ((size_t)d * kAttnLT + 2 * (size_t)d * S + (size_t)kAttnLT * S) * sizeof(float);
    LDM_REQUIRE(lds <= 64 * 1024, "attention: head tile exceeds LDS budget");
    const int ltiles = (L + kAttnLT - 1) / kAttnLT;
    hipLaunchKernelGGL(attention_core_kernel, dim3(B * heads * ltiles), dim3(256), lds, st, q, kv, out, E, heads, L, S,
                       scale);
    LDM_CHECK_LAUNCH("attention_core_kernel");
    return 0;
}
}  // namespace ldm

extern "C" int ldm_attention_core(const float* q, const float* kv, float* out, int32_t B, int32_t E, int32_t heads,
                                  int32_t L, int32_t S, float scale, void* stream) {
    return ldm::attention_core_ex(q, kv, out, B, E, heads, L, S, scale, false, (hipStream_t)stream);
}

extern "C" int ldm_q_sample(const float* x0, const float* eps, const float* coef_table, int32_t T, const int64_t* t,
                            float* zt, int32_t B, int64_t per_sample, void* stream) {
    LDM_REQUIRE(x0 && eps && coef_table && t && zt && B > 0 && per_sample > 0 && T > 0, "q_sample: bad argument");
    const int64_t n = (int64_t)B * per_sample;
    hipLaunchKernelGGL(q_sample_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, x0, eps,
                       coef_table, T, t, zt, per_sample, n);
    LDM_CHECK_LAUNCH("q_sample_kernel");
    return 0;
}

extern "C" int ldm_predict_start(const float* zt, const float* eps, const float* coef_table, int32_t T,
                                 const int64_t* t, float* x0, int32_t B, int64_t per_sample, void* stream) {
    LDM_REQUIRE(x0 && eps && coef_table && t && zt && B > 0 && per_sample > 0 && T > 0, "predict_start: bad argument");
    const int64_t n = (int64_t)B * per_sample;
    hipLaunchKernelGGL(predict_start_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, zt, eps,
                       coef_table, T, t, x0, per_sample, n);
    LDM_CHECK_LAUNCH("predict_start_kernel");
    return 0;
}

extern "C" int ldm_sched_backward(int32_t kind, const float* grad, const float* coef_table, int32_t T, const int64_t* t,
                                  float* grad_a, float* grad_b, int32_t B, int64_t per_sample, void* stream) {
    LDM_REQUIRE(grad && coef_table && t && B > 0 && per_sample > 0 && T > 0 && (kind == 0 || kind == 1),
                "sched_backward: bad argument");
    const int64_t n = (int64_t)B * per_sample;
    hipLaunchKernelGGL(sched_backward_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, kind, grad,
                       coef_table, T, t, grad_a, grad_b, per_sample, n);
    LDM_CHECK_LAUNCH("sched_backward_kernel");
    return 0;
}

extern "C" int ldm_ddim_step(float* x, const float* eps, const float* coef, float eta, float* x0_log, float* eps_log,
                             int64_t n, void* stream) {
    LDM_REQUIRE(x && eps && coef && n > 0, "ddim_step: bad argument");
    hipLaunchKernelGGL(ddim_step_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, x, eps, coef, eta,
                       x0_log, eps_log, n);
    LDM_CHECK_LAUNCH("ddim_step_kernel");
    return 0;
}

extern "C" int ldm_activation(const float* x, float* y, int64_t n, int32_t act, void* stream) {
    LDM_REQUIRE(x && y && n >= 0, "activation: bad argument");
    if (n == 0) return 0;
    hipLaunchKernelGGL(activation_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, x, y, n, act);
    LDM_CHECK_LAUNCH("activation_kernel");
    return 0;
}

extern "C" int ldm_batchnorm_eval(const float* x, float* y, int32_t B, int32_t C, int32_t HW, const float* weight,
                                  const float* bias, const float* running_mean, const float* running_var, float eps,
                                  int32_t act, void* stream) {
    LDM_REQUIRE(x && y && running_mean && running_var && B > 0 && C > 0 && HW > 0, "batchnorm_eval: bad argument");
    const int64_t n = (int64_t)B * C * HW;
    hipLaunchKernelGGL(batchnorm_eval_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, x, y, C, HW,
                       n, weight, bias, running_mean, running_var, eps, act);
    LDM_CHECK_LAUNCH("batchnorm_eval_kernel");
    return 0;
}

extern "C" int ldm_sinusoid_embed(const void* t, int32_t t_is_float, int32_t B, int32_t dim, const float* freqs,
                                  float* out, void* stream) {
    LDM_REQUIRE(t && freqs && out && B > 0 && dim > 1 && dim % 2 == 0, "sinusoid: bad argument");
    hipLaunchKernelGGL(sinusoid_kernel, dim3(blocks_for((int64_t)B * dim, 256)), dim3(256), 0, (hipStream_t)stream, t,
                       t_is_float, B, dim, freqs, out);
    LDM_CHECK_LAUNCH("sinusoid_kernel");
    return 0;
}

extern "C" int ldm_loss_forward(int32_t kind, const float* a, const float* b, int64_t n, void* workspace, float* out,
                                void* stream) {
    LDM_REQUIRE(a && workspace && out && n > 0 && (kind == 0 || kind == 1), "loss_forward: bad argument");
    LDM_REQUIRE(kind != 0 || b, "loss_forward: mse needs two inputs");
    const int np = (int)std::min<int64_t>(kLossBlocks, (n + 255) / 256);
    hipLaunchKernelGGL(loss_partial_kernel, dim3(np), dim3(256), 0, (hipStream_t)stream, kind, a, b, n,
                       (double*)workspace);
    LDM_CHECK_LAUNCH("loss_partial_kernel");
    hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const double*)workspace, np, n, out);
    LDM_CHECK_LAUNCH("loss_final_kernel");
    return 0;
}

extern "C" int ldm_loss_backward(int32_t kind, const float* a, const float* b, int64_t n, const float* grad_out,
                                 float* grad_a, float* grad_b, void* stream) {
    LDM_REQUIRE(a && grad_out && n > 0 && (kind == 0 || kind == 1), "loss_backward: bad argument");
    hipLaunchKernelGGL(loss_backward_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, kind, a, b, n,
                       grad_out, grad_a, grad_b);
    LDM_CHECK_LAUNCH("loss_backward_kernel");
    return 0;
}

extern "C" int ldm_attention_fold_keys(const float* kv, const float* wq, const float* bq, int32_t B, int32_t E,
                                       int32_t heads, int32_t S, float scale, float* kf, float* bf, void* stream) {
    return ldm::attention_fold_keys(kv, wq, bq, B, E, heads, S, scale, kf, bf, (hipStream_t)stream);
}

extern "C" int ldm_attention_folded(const float* z, const float* kv, const float* kf, const float* bf, float* out,
                                    int32_t B, int32_t E, int32_t heads, int32_t L, int32_t S, void* stream) {
    return ldm::attention_folded(z, kv, kf, bf, out, B, E, heads, L, S, (hipStream_t)stream);
}

extern "C" int ldm_attention_folded_probs(const float* z, const float* kf, const float* bf, float* p, int32_t B,
                                          int32_t E, int32_t heads, int32_t L, int32_t S, void* stream) {
    return ldm::attention_folded_probs(z, kf, bf, p, B, E, heads, L, S, (hipStream_t)stream);
}

extern "C" int ldm_fold_conv_proj(const ldm_conv_desc* d, const float* w_conv, const float* b_conv, const float* w_proj,
                                  const float* b_proj, int32_t Cmid, float* w_out, float* pos_bias_out, void* stream) {
    LDM_REQUIRE(d && w_conv && w_proj && b_proj && w_out && pos_bias_out, "fold conv/proj: null argument");
    LDM_REQUIRE(!d->transposed && d->kh * d->kw > 0 && Cmid > 0, "fold conv/proj: a plain conv after the projection");
    const int64_t n = (int64_t)d->Cout * d->Cin * d->kh * d->kw + (int64_t)d->Cout * d->Hout * d->Wout;
    hipLaunchKernelGGL(ldm::fold_conv_proj_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       w_conv, b_conv, w_proj, b_proj, d->Cout, Cmid, d->Cin, d->kh, d->kw, d->stride, d->pad, d->Hin,
                       d->Win, d->Hout, d->Wout, w_out, pos_bias_out);
    LDM_CHECK_LAUNCH("fold_conv_proj_kernel");
    return 0;
}
