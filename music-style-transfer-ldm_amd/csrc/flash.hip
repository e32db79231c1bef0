// Width-general cross-attention (CrossAttention, model.py:126-160) for any number of query tokens L and
// key tokens S: KV-tiled online-softmax forward and the matching two-kernel backward, on the exact-fp32
// v_mfma_f32_16x16x4_f32.  The UNet's attention tokens grow linearly with the mel width (L = S = H*W/16
// for CA2, H*W/64 for CA1: 64 / 16 at the canonical 16x64 latent, 128 / 32 at 16x128, 4096 / 1024 for
// SURVEY's stress shape S), so the LDS-resident instances of misc.hip (L, S <= 64) hand over to these.
//
// One block = 4 waves = 64 query rows (forward, dQ) or 64 key columns (dK/dV) of one (batch, head); each
// wave owns 16 of them as the N (or M) side of its MFMA tiles.  K / V (forward, dQ) or q / dO (dK/dV)
// stream through LDS in tiles of 64 tokens, staged by all four waves, pitch D+4 / 68 floats (= 4 mod 64:
// the 16 lanes of one b128 read and the 64 lanes of one b32 read hit distinct banks).
//
// The products are laid out so that no fragment is ever transposed through LDS: the scores are computed
// transposed (S^T = K (q*scale)^T, M = key, N = query), whose accumulator layout — lane (col, lg) holds
// keys 4 lg + r of query col — is exactly the B operand of O^T = V P^T (K index s = 16 st + 4 lg + r), and
// the softmax statistics of query col live in the lanes that accumulate its output column.  Row max / sum
// take two xor-shuffles across the lane groups.  Deterministic: fixed tile order, no atomics.
//
// Layouts: kv [B, 2E, S] channel-major (K rows then V rows, as the K/V projection writes them); q / out
// [B, E, L] channel-major or token-major [B, L, E] (TOK, the UNet engine's NHWC activations); lse / delta
// [B, heads, L].
#include <cmath>
#include <cstdlib>

#include "common.h"

namespace ldm {
namespace fa {

constexpr int kTok = 64;            // tokens per block and per streamed tile
constexpr int kKP = kTok + 4;       // LDS pitch of a channel-major [c][s] tile

__device__ __forceinline__ floatx4 mma(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// [D][64] tile of a channel-major slab (row c at src + c*n, tokens t0 .. t0+63, zero past n) -> registers
// (every load of the thread in flight at once), then -> LDS [D][kKP].  Split in two so that a kernel can issue
// the next tile's loads before it computes on the current one.
template <int D>
constexpr int cs_pieces() { return D * (kTok / 4) / 256; }
// Branch-free: a piece past n is loaded from a valid address (the slab's first element) and replaced by zero
// after the load, so no load sits inside a branch (a load under a branch whose register the other arm writes makes
// the compiler wait for it at the join, which drains the look-ahead).  VEC: n % 4 == 0, so a float4 of a row is
// wholly inside or wholly past it.
template <int D, bool VEC>
__device__ __forceinline__ void load_cs(const float* __restrict__ src, int n, int t0, float4 (&v)[cs_pieces<D>()],
                                        int tid = (int)threadIdx.x) {
    constexpr int NIT = cs_pieces<D>();
#pragma unroll
    for (int u = 0; u < NIT; ++u) {
        const int e = u * 256 + tid;
        const int c = e / (kTok / 4), t = t0 + 4 * (e % (kTok / 4));
        const float* p = src + (size_t)c * n + t;
        if constexpr (VEC) {
            const bool in = t < n;
            const float4 x = *reinterpret_cast<const float4*>(in ? p : src);
            v[u] = in ? x : make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
            float x[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool in = t + k < n;
                const float y = *(in ? p + k : src);
                x[k] = in ? y : 0.f;
            }
            v[u] = make_float4(x[0], x[1], x[2], x[3]);
        }
    }
}
template <int D>
__device__ __forceinline__ void store_cs(const float4 (&v)[cs_pieces<D>()], float* __restrict__ dst,
                                         int tid = (int)threadIdx.x) {
#pragma unroll
    for (int u = 0; u < cs_pieces<D>(); ++u) {
        const int e = u * 256 + tid;
        *reinterpret_cast<float4*>(dst + (e / (kTok / 4)) * kKP + 4 * (e % (kTok / 4))) = v[u];
    }
}

// [D][64] channel-major tile (tokens t0..) -> LDS token-major [64][D+4], times mul; zero past n.
template <int D>
__device__ __forceinline__ void stage_tc(const float* __restrict__ src, int n, int t0, float mul, float* __restrict__ dst) {
    constexpr int NIT = D * (kTok / 4) / 256, P = D + 4;
    float4 v[NIT];
    const bool vec = (n & 3) == 0 && t0 + kTok <= n;
#pragma unroll
    for (int u = 0; u < NIT; ++u) {
        const int e = u * 256 + (int)threadIdx.x;
        const int c = e / (kTok / 4), t = t0 + 4 * (e % (kTok / 4));
        const float* p = src + (size_t)c * n + t;
        if (vec) {
            v[u] = *reinterpret_cast<const float4*>(p);
        } else {
            v[u].x = t + 0 < n ? p[0] : 0.f;
            v[u].y = t + 1 < n ? p[1] : 0.f;
            v[u].z = t + 2 < n ? p[2] : 0.f;
            v[u].w = t + 3 < n ? p[3] : 0.f;
        }
    }
#pragma unroll
    for (int u = 0; u < NIT; ++u) {
        const int e = u * 256 + (int)threadIdx.x;
        const int c = e / (kTok / 4), tl = 4 * (e % (kTok / 4));
        dst[(tl + 0) * P + c] = v[u].x * mul;
        dst[(tl + 1) * P + c] = v[u].y * mul;
        dst[(tl + 2) * P + c] = v[u].z * mul;
        dst[(tl + 3) * P + c] = v[u].w * mul;
    }
}

// The 16 query rows' fragment a lane holds as the N operand: frag[jj][i] = x[l][16 jj + 4 lg + i] * mul.
template <int D, bool TOK>
__device__ __forceinline__ void load_qfrag(const float* __restrict__ base, int E, int L, int l, int lg, float mul,
                                           float (&f)[D / 16][4]) {
    if constexpr (TOK) {
        const float* p = base + (size_t)l * E + 4 * lg;
#pragma unroll
        for (int jj = 0; jj < D / 16; ++jj) {
            const float4 v = *reinterpret_cast<const float4*>(p + 16 * jj);
            f[jj][0] = v.x * mul;
            f[jj][1] = v.y * mul;
            f[jj][2] = v.z * mul;
            f[jj][3] = v.w * mul;
        }
    } else {
        const float* p = base + (size_t)(4 * lg) * L + l;
#pragma unroll
        for (int jj = 0; jj < D / 16; ++jj)
#pragma unroll
            for (int i = 0; i < 4; ++i) f[jj][i] = p[(size_t)(16 * jj + i) * L] * mul;
    }
}

// ---- forward ---------------------------------------------------------------------------------------
// KH > 1: the block's KH groups of four waves take the same 64 queries over KH contiguous ranges of key tiles (each
// group stages its own tiles), and the groups' (m, l, O) meet in LDS at the end (O = sum_g e^(m_g - M) O_g over the
// same sum of l_g): KH waves per SIMD where the grid has one block per CU.  NBUF: K / V buffers per group (1: the
// next tile is stored after a barrier that closes the current one; the D = 128, KH = 2 form needs it to fit LDS).
//
// SPL (round 6): the key tiles split over gridDim.y blocks as well (fewer (query tile, head) blocks than a quarter of
// the CUs: CA1 at shape S, L = S = 1024, d = 128, 64 blocks).  Each block leaves its unnormalised O, m and l in the
// workspace `part` ([split][B heads][L] rows of D + 4: O, m, l) and flash_combine_kernel merges the splits in split order.
template <int D, bool TOK, bool LSE, bool VEC, int KH, int NBUF, bool SPL = false>
__global__ __launch_bounds__(256 * KH) void flash_fwd_kernel(const float* __restrict__ q, const float* __restrict__ kv,
                                                        float* __restrict__ out, float* __restrict__ lse, int E,
                                                        int heads, int L, int S, float scale,
                                                        float* __restrict__ part = nullptr) {
    constexpr int NJ = D / 16;
    extern __shared__ __attribute__((aligned(16))) float smem_all[];   // KH x NBUF x {K [D][kKP], V [D][kKP]}
    const int nqt = (L + kTok - 1) / kTok;
    const int qt = blockIdx.x % nqt, bh = blockIdx.x / nqt;
    const int h = bh % heads, b = bh / heads;
    const int lane = threadIdx.x & 63, wave = (threadIdx.x >> 6) & 3, col = lane & 15, lg = lane >> 4;
    const int kg = KH > 1 ? (int)(threadIdx.x >> 8) : 0;   // key group
    const int gtid = (int)threadIdx.x & 255;
    float* sm = smem_all + kg * (NBUF * 2 * D * kKP);
    const int l = qt * kTok + wave * 16 + col;
    const bool lok = l < L;
    const int lc = lok ? l : L - 1;

    // q_scaled = q * sqrt(1/d) (the reference's elementwise product), N operand of S^T
    float qf[NJ][4];
    const float* qb = TOK ? q + (size_t)b * L * E + (size_t)h * D : q + ((size_t)b * E + (size_t)h * D) * L;
    load_qfrag<D, TOK>(qb, E, L, lc, lg, scale, qf);

    const float* kb = kv + ((size_t)b * 2 * E + (size_t)h * D) * S;
    const float* vb = kb + (size_t)E * S;
    floatx4 o[NJ];
#pragma unroll
    for (int ct = 0; ct < NJ; ++ct) o[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, lsum = 0.f;

    // K / V tiles double-buffered in LDS, the next tile's loads in registers while the current one is multiplied:
    // tile t+1 is stored into the buffer tile t-1 used (every wave left it at the barrier closing iteration t-1),
    // then tile t+2's loads are issued; one barrier per tile.  (Round 6: the single-buffered form waited out
    // a load round trip per 64-key tile, 364 us per launch at L = S = 4096.)
    const int ntall = (S + kTok - 1) / kTok;
    // SPL: this block's contiguous range of tiles [sb, sb + nts) (the last split may have fewer, or none)
    const int tps = SPL ? (ntall + (int)gridDim.y - 1) / (int)gridDim.y : ntall;
    const int sb = SPL ? (int)blockIdx.y * tps : 0;
    const int nts = SPL ? max(0, min(ntall - sb, tps)) : ntall;
    const int ntg = (nts + KH - 1) / KH;                  // tiles per key group (the last group may have fewer)
    const int tb = sb + kg * ntg, nt = min(sb + nts - tb, ntg);   // this group's first tile and its count (<= 0: none)
    float4 rk[cs_pieces<D>()], rv[cs_pieces<D>()];
    if (nt > 0) {
        load_cs<D, VEC>(kb, S, tb * kTok, rk, gtid);
        load_cs<D, VEC>(vb, S, tb * kTok, rv, gtid);
        store_cs<D>(rk, sm, gtid);
        store_cs<D>(rv, sm + D * kKP, gtid);
        if (nt > 1) {
            load_cs<D, VEC>(kb, S, (tb + 1) * kTok, rk, gtid);
            load_cs<D, VEC>(vb, S, (tb + 1) * kTok, rv, gtid);
        }
    }
    __syncthreads();
    for (int t = 0; t < ntg; ++t) {   // every group runs ntg iterations: the barriers are the whole block's
      if (t < nt) {
        const int s0 = (tb + t) * kTok;
        const float* Ks = sm + (NBUF == 2 ? (t & 1) : 0) * (2 * D * kKP);   // [D][kKP]
        const float* Vs = Ks + D * kKP;                   // [D][kKP]
        // S^T[s][l] for the tile's 64 keys (4 tiles of 16): lane holds keys s0 + 16 st + 4 lg + r of query l; the
        // four key tiles' chains interleaved (each chain still sums jj, i in order)
        floatx4 sc[4];
#pragma unroll
        for (int st = 0; st < 4; ++st) sc[st] = floatx4{0.f, 0.f, 0.f, 0.f};
        // the K fragments of channel group jj + 1 are read while group jj's 16 MFMAs run (one LDS round trip per
        // group instead of one per MFMA pair)
        float ka[2][4][4];
        auto read_k = [&](int jj, float (&f)[4][4]) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int st = 0; st < 4; ++st) f[i][st] = Ks[(16 * jj + 4 * lg + i) * kKP + 16 * st + col];
        };
        read_k(0, ka[0]);
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj) {
            if (jj + 1 < NJ) read_k(jj + 1, ka[(jj + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);   // (the scheduler would sink the reads back next to their MFMAs)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int st = 0; st < 4; ++st) sc[st] = mma(ka[jj & 1][i][st], qf[jj][i], sc[st]);
            __builtin_amdgcn_sched_barrier(0);
        }
        // online softmax over s (the 4 lanes of query col share its statistics)
        float tmax = -INFINITY;
#pragma unroll
        for (int st = 0; st < 4; ++st)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (s0 + 16 * st + 4 * lg + r < S) tmax = fmaxf(tmax, sc[st][r]);
        tmax = fmaxf(tmax, __shfl_xor(tmax, 16));
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
        const float mnew = fmaxf(m, tmax);
        const float alpha = expf(m - mnew);
        float p[4][4], tsum = 0.f;
#pragma unroll
        for (int st = 0; st < 4; ++st)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                p[st][r] = s0 + 16 * st + 4 * lg + r < S ? expf(sc[st][r] - mnew) : 0.f;
                tsum += p[st][r];
            }
        tsum += __shfl_xor(tsum, 16);
        tsum += __shfl_xor(tsum, 32);
        lsum = lsum * alpha + tsum;
        m = mnew;
        // O^T[c][l] = alpha O^T + sum_s V[c][s] P[l][s] (the NJ channel tiles' chains interleaved)
#pragma unroll
        for (int ct = 0; ct < NJ; ++ct) o[ct] *= alpha;
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            float4 va[NJ];
#pragma unroll
            for (int ct = 0; ct < NJ; ++ct) va[ct] = *reinterpret_cast<const float4*>(Vs + (16 * ct + col) * kKP + 16 * st + 4 * lg);
#pragma unroll
            for (int ct = 0; ct < NJ; ++ct) o[ct] = mma(va[ct].x, p[st][0], o[ct]);
#pragma unroll
            for (int ct = 0; ct < NJ; ++ct) o[ct] = mma(va[ct].y, p[st][1], o[ct]);
#pragma unroll
            for (int ct = 0; ct < NJ; ++ct) o[ct] = mma(va[ct].z, p[st][2], o[ct]);
#pragma unroll
            for (int ct = 0; ct < NJ; ++ct) o[ct] = mma(va[ct].w, p[st][3], o[ct]);
        }
      }
        if constexpr (NBUF == 1) __syncthreads();   // every wave is done with the single buffer
        if (t + 1 < nt) {
            float* nb = sm + (NBUF == 2 ? ((t + 1) & 1) : 0) * (2 * D * kKP);
            store_cs<D>(rk, nb, gtid);
            store_cs<D>(rv, nb + D * kKP, gtid);
            if (t + 2 < nt) {
                load_cs<D, VEC>(kb, S, (tb + t + 2) * kTok, rk, gtid);
                load_cs<D, VEC>(vb, S, (tb + t + 2) * kTok, rv, gtid);
            }
        }
        __syncthreads();
    }
    if constexpr (KH > 1) {
        // the key groups' (m, l, O) meet in LDS (the K / V buffers are free after the loop's last barrier): groups
        // 1.. publish theirs, group 0 combines them in group order
        float* xs = smem_all + (size_t)wave * (KH - 1) * 64 * (4 * NJ + 2);
        if (kg > 0) {
            float* my = xs + (size_t)(kg - 1) * 64 * (4 * NJ + 2);
#pragma unroll
            for (int ct = 0; ct < NJ; ++ct)
#pragma unroll
                for (int r = 0; r < 4; ++r) my[(ct * 4 + r) * 64 + lane] = o[ct][r];
            my[(4 * NJ) * 64 + lane] = m;
            my[(4 * NJ + 1) * 64 + lane] = lsum;
        }
        __syncthreads();
        if (kg > 0) return;
#pragma unroll
        for (int g = 1; g < KH; ++g) {
            const float* ot = xs + (size_t)(g - 1) * 64 * (4 * NJ + 2);
            const float mg = ot[(4 * NJ) * 64 + lane], lg2 = ot[(4 * NJ + 1) * 64 + lane];
            const float M = fmaxf(m, mg);
            const float w0 = m == -INFINITY ? 0.f : expf(m - M), w1 = mg == -INFINITY ? 0.f : expf(mg - M);
#pragma unroll
            for (int ct = 0; ct < NJ; ++ct)
#pragma unroll
                for (int r = 0; r < 4; ++r) o[ct][r] = o[ct][r] * w0 + ot[(ct * 4 + r) * 64 + lane] * w1;
            lsum = lsum * w0 + lg2 * w1;
            m = M;
        }
    }
    if (!lok) return;
    if constexpr (SPL) {   // unnormalised O[l][16 ct + 4 lg + r], then m and l (lane group 0)
        const int BH = (int)gridDim.x / nqt;
        float* pb = part + (((size_t)blockIdx.y * BH + bh) * L + l) * (D + 4);
#pragma unroll
        for (int ct = 0; ct < NJ; ++ct) *reinterpret_cast<floatx4*>(pb + 16 * ct + 4 * lg) = o[ct];
        if (lg == 0) *reinterpret_cast<float2*>(pb + D) = make_float2(m, lsum);
        return;
    }
    // lane holds O[l][c] for c = 16 ct + 4 lg + r
    if constexpr (TOK) {
        float* ob = out + ((size_t)b * L + l) * E + (size_t)h * D + 4 * lg;
#pragma unroll
        for (int ct = 0; ct < NJ; ++ct)
            *reinterpret_cast<float4*>(ob + 16 * ct) =
                make_float4(o[ct][0] / lsum, o[ct][1] / lsum, o[ct][2] / lsum, o[ct][3] / lsum);
    } else {
        float* ob = out + ((size_t)b * E + (size_t)h * D + 4 * lg) * L + l;
#pragma unroll
        for (int ct = 0; ct < NJ; ++ct)
#pragma unroll
            for (int r = 0; r < 4; ++r) ob[(size_t)(16 * ct + r) * L] = o[ct][r] / lsum;
    }
    if (LSE && lg == 0) lse[(size_t)bh * L + l] = m + logf(lsum);
}

// Merge of the key splits (SPL), token-major outputs: per (b, h, l) M = max m_i, w_i = e^(m_i - M) (0 for a split with
// no keys), O = sum_i w_i O_i / sum_i w_i l_i, folded in split order (the KH groups' merge, over blocks).  Thread = 4
// channels of one query row, channels fastest (reads and writes both along the row).
template <int D, bool LSE>
__global__ __launch_bounds__(256) void flash_combine_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                            float* __restrict__ lse, int nsp, int BH, int E, int heads,
                                                            int L) {
    constexpr int C4 = D / 4, P = D + 4;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)BH * L * C4) return;
    const int c4 = (int)(i % C4);
    const int64_t r = i / C4;
    const int l = (int)(r % L), bh = (int)(r / L);
    const size_t split_stride = (size_t)BH * L * P;
    const float* pr = part + ((size_t)bh * L + l) * P;
    float M = -INFINITY;
    for (int s = 0; s < nsp; ++s) M = fmaxf(M, pr[s * split_stride + D]);
    floatx4 o = {0.f, 0.f, 0.f, 0.f};
    float lsum = 0.f;
    for (int s = 0; s < nsp; ++s) {
        const float* ps = pr + s * split_stride;
        const float ms = ps[D];
        const float w = ms == -INFINITY ? 0.f : expf(ms - M);
        o = o + w * *reinterpret_cast<const floatx4*>(ps + 4 * c4);
        lsum = lsum + w * ps[D + 1];
    }
    const int h = bh % heads, b = bh / heads, c = 4 * c4;
    *reinterpret_cast<float4*>(out + ((size_t)b * L + l) * E + (size_t)h * D + c) =
        make_float4(o[0] / lsum, o[1] / lsum, o[2] / lsum, o[3] / lsum);
    if (LSE && c4 == 0) lse[(size_t)bh * L + l] = M + logf(lsum);
}

// The channel-major form: a block merges 16 query rows x D channels (threads along the channels of a row: the
// partial rows read whole), parks O / l in LDS and writes it along L (out [B, E, L]).  Same arithmetic per output.
template <int D, bool LSE>
__global__ __launch_bounds__(256) void flash_combine_cm_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                               float* __restrict__ lse, int nsp, int BH, int E,
                                                               int heads, int L) {
    constexpr int C4 = D / 4, P = D + 4, RB = 16;   // (64 rows: 64 blocks at CA1's shape S, 21 us; 16: 256 blocks)
    __shared__ float tile[D][RB + 1];
    const int bh = (int)blockIdx.y, l0 = (int)blockIdx.x * RB;
    const size_t split_stride = (size_t)BH * L * P;
    for (int it = (int)threadIdx.x; it < RB * C4; it += 256) {
        const int lr = it / C4, c4 = it % C4, l = l0 + lr;
        if (l >= L) continue;
        const float* pr = part + ((size_t)bh * L + l) * P;
        float M = -INFINITY;
        for (int s = 0; s < nsp; ++s) M = fmaxf(M, pr[s * split_stride + D]);
        floatx4 o = {0.f, 0.f, 0.f, 0.f};
        float lsum = 0.f;
        for (int s = 0; s < nsp; ++s) {
            const float* ps = pr + s * split_stride;
            const float ms = ps[D];
            const float w = ms == -INFINITY ? 0.f : expf(ms - M);
            o = o + w * *reinterpret_cast<const floatx4*>(ps + 4 * c4);
            lsum = lsum + w * ps[D + 1];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) tile[4 * c4 + r][lr] = o[r] / lsum;
        if (LSE && c4 == 0) lse[(size_t)bh * L + l] = M + logf(lsum);
    }
    __syncthreads();
    const int h = bh % heads, b = bh / heads;
    float* ob = out + ((size_t)b * E + (size_t)h * D) * L;
    for (int it = (int)threadIdx.x; it < D * RB; it += 256) {
        const int c = it / RB, lr = it % RB, l = l0 + lr;
        if (l < L) ob[(size_t)c * L + l] = tile[c][lr];
    }
}

// ---- backward ----------------------------------------------------------------------------------------
// delta[b,h,l] = sum_c dO[c][l] O[c][l] over the head's channels (= rowsum(P * dP), channel-major)
__global__ __launch_bounds__(256) void flash_delta_kernel(const float* __restrict__ out, const float* __restrict__ dout,
                                                          float* __restrict__ delta, int E, int heads, int L, int D,
                                                          int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int l = (int)(i % L);
    const int64_t bh = i / L;
    const int h = (int)(bh % heads);
    const int64_t b = bh / heads;
    const size_t base = ((size_t)b * E + (size_t)h * D) * L + l;
    float acc = 0.f;
    for (int c = 0; c < D; ++c) acc = fmaf(dout[base + (size_t)c * L], out[base + (size_t)c * L], acc);
    delta[i] = acc;
}

// dK, dV for 64 keys per block (wave: 16 keys, the N side), streaming q*scale and dO through LDS:
//   S = qs K^T, P = exp(S - lse), dP = dO V^T, dS = P (dP - delta);  dV^T += dO^T P, dK^T += qs^T dS
template <int D>
__global__ __launch_bounds__(256) void flash_bwd_dkv_kernel(const float* __restrict__ q, const float* __restrict__ kv,
                                                            const float* __restrict__ dout, const float* __restrict__ lse,
                                                            const float* __restrict__ delta, float* __restrict__ dkv,
                                                            int E, int heads, int L, int S, float scale) {
    constexpr int NJ = D / 16, P = D + 4;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* Qs = sm;                  // [64][D+4]  q * scale, token-major
    float* Os = Qs + kTok * P;       // [64][D+4]  dO
    float* Ls = Os + kTok * P;       // [64] lse (+inf past L: P = 0)
    float* Ds = Ls + kTok;           // [64] delta
    const int nkt = (S + kTok - 1) / kTok;
    const int kt = blockIdx.x % nkt, bh = blockIdx.x / nkt;
    const int h = bh % heads, b = bh / heads;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, lg = lane >> 4;
    const int s = kt * kTok + wave * 16 + col;
    const bool sok = s < S;
    const int sc = sok ? s : S - 1;
    const float* kb = kv + ((size_t)b * 2 * E + (size_t)h * D) * S;
    const float* vb = kb + (size_t)E * S;
    float kf[NJ][4], vf[NJ][4];   // B operands: K[c][s], V[c][s] for c = 16 jj + 4 lg + i
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            kf[jj][i] = kb[(size_t)(16 * jj + 4 * lg + i) * S + sc];
            vf[jj][i] = vb[(size_t)(16 * jj + 4 * lg + i) * S + sc];
        }
    const float* qb = q + ((size_t)b * E + (size_t)h * D) * L;
    const float* ob = dout + ((size_t)b * E + (size_t)h * D) * L;
    const float* lb = lse + (size_t)bh * L;
    const float* db = delta + (size_t)bh * L;
    floatx4 dk[NJ], dv[NJ];
#pragma unroll
    for (int ct = 0; ct < NJ; ++ct) dk[ct] = dv[ct] = floatx4{0.f, 0.f, 0.f, 0.f};

    for (int l0 = 0; l0 < L; l0 += kTok) {
        __syncthreads();
        stage_tc<D>(qb, L, l0, scale, Qs);
        stage_tc<D>(ob, L, l0, 1.f, Os);
        if (threadIdx.x < kTok) {
            const int l = l0 + (int)threadIdx.x;
            Ls[threadIdx.x] = l < L ? lb[l] : INFINITY;
            Ds[threadIdx.x] = l < L ? db[l] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int lt = 0; lt < 4; ++lt) {
            // S[l][s], dP[l][s]: lane holds queries l0 + 16 lt + 4 lg + r of key s
            floatx4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
            const float* qrow = Qs + (16 * lt + col) * P + 4 * lg;
            const float* orow = Os + (16 * lt + col) * P + 4 * lg;
#pragma unroll
            for (int jj = 0; jj < NJ; ++jj) {
                const float4 a = *reinterpret_cast<const float4*>(qrow + 16 * jj);
                const float4 g = *reinterpret_cast<const float4*>(orow + 16 * jj);
                sv = mma(a.x, kf[jj][0], sv);
                sv = mma(a.y, kf[jj][1], sv);
                sv = mma(a.z, kf[jj][2], sv);
                sv = mma(a.w, kf[jj][3], sv);
                dp = mma(g.x, vf[jj][0], dp);
                dp = mma(g.y, vf[jj][1], dp);
                dp = mma(g.z, vf[jj][2], dp);
                dp = mma(g.w, vf[jj][3], dp);
            }
            float pv[4], ds[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int li = 16 * lt + 4 * lg + r;
                pv[r] = expf(sv[r] - Ls[li]);
                ds[r] = pv[r] * (dp[r] - Ds[li]);
            }
            // dV^T[c][s] += sum_l dO[l][c] P[l][s];  dK^T[c][s] += sum_l qs[l][c] dS[l][s]
#pragma unroll
            for (int ct = 0; ct < NJ; ++ct)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int li = 16 * lt + 4 * lg + r;
                    dv[ct] = mma(Os[li * P + 16 * ct + col], pv[r], dv[ct]);
                    dk[ct] = mma(Qs[li * P + 16 * ct + col], ds[r], dk[ct]);
                }
        }
    }
    if (!sok) return;
    float* dkb = dkv + ((size_t)b * 2 * E + (size_t)h * D) * S + s;
    float* dvb = dkb + (size_t)E * S;
#pragma unroll
    for (int ct = 0; ct < NJ; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            dkb[(size_t)(16 * ct + 4 * lg + r) * S] = dk[ct][r];
            dvb[(size_t)(16 * ct + 4 * lg + r) * S] = dv[ct][r];
        }
}

// dQ for 64 queries per block (wave: 16 queries, the N side), streaming K and V through LDS:
//   S^T = K qs^T, dP^T = V dO^T, dS = P (dP - delta);  dQ^T += K dS^T, times scale
template <int D, bool VEC>
__global__ __launch_bounds__(256) void flash_bwd_dq_kernel(const float* __restrict__ q, const float* __restrict__ kv,
                                                           const float* __restrict__ dout, const float* __restrict__ lse,
                                                           const float* __restrict__ delta, float* __restrict__ dq,
                                                           int E, int heads, int L, int S, float scale) {
    constexpr int NJ = D / 16;
    extern __shared__ __attribute__((aligned(16))) float sm[];   // 2 x {K [D][kKP], V [D][kKP]}
    const int nqt = (L + kTok - 1) / kTok;
    const int qt = blockIdx.x % nqt, bh = blockIdx.x / nqt;
    const int h = bh % heads, b = bh / heads;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, lg = lane >> 4;
    const int l = qt * kTok + wave * 16 + col;
    const bool lok = l < L;
    const int lc = lok ? l : L - 1;
    const float* qb = q + ((size_t)b * E + (size_t)h * D) * L;
    const float* ob = dout + ((size_t)b * E + (size_t)h * D) * L;
    float qf[NJ][4], of[NJ][4];
    load_qfrag<D, false>(qb, E, L, lc, lg, scale, qf);
    load_qfrag<D, false>(ob, E, L, lc, lg, 1.f, of);
    const float ll = lse[(size_t)bh * L + lc], dl = delta[(size_t)bh * L + lc];
    const float* kb = kv + ((size_t)b * 2 * E + (size_t)h * D) * S;
    const float* vb = kb + (size_t)E * S;
    floatx4 acc[NJ];
#pragma unroll
    for (int ct = 0; ct < NJ; ++ct) acc[ct] = floatx4{0.f, 0.f, 0.f, 0.f};

    // K / V tiles double-buffered as in flash_fwd_kernel
    const int nt = (S + kTok - 1) / kTok;
    float4 rk[cs_pieces<D>()], rv[cs_pieces<D>()];
    load_cs<D, VEC>(kb, S, 0, rk);
    load_cs<D, VEC>(vb, S, 0, rv);
    store_cs<D>(rk, sm);
    store_cs<D>(rv, sm + D * kKP);
    if (nt > 1) {
        load_cs<D, VEC>(kb, S, kTok, rk);
        load_cs<D, VEC>(vb, S, kTok, rv);
    }
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
        const int s0 = t * kTok;
        const float* Ks = sm + (t & 1) * (2 * D * kKP);   // [D][kKP]
        const float* Vs = Ks + D * kKP;                   // [D][kKP]
        float ds[4][4];
        floatx4 sv[4], dp[4];
#pragma unroll
        for (int st = 0; st < 4; ++st) sv[st] = dp[st] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int st = 0; st < 4; ++st) {
                    const int a = (16 * jj + 4 * lg + i) * kKP + 16 * st + col;
                    sv[st] = mma(Ks[a], qf[jj][i], sv[st]);
                    dp[st] = mma(Vs[a], of[jj][i], dp[st]);
                }
#pragma unroll
        for (int st = 0; st < 4; ++st)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const bool ok = s0 + 16 * st + 4 * lg + r < S;
                const float pv = ok ? expf(sv[st][r] - ll) : 0.f;
                ds[st][r] = pv * (dp[st][r] - dl);
            }
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            float4 ka[NJ];
#pragma unroll
            for (int ct = 0; ct < NJ; ++ct) ka[ct] = *reinterpret_cast<const float4*>(Ks + (16 * ct + col) * kKP + 16 * st + 4 * lg);
#pragma unroll
            for (int ct = 0; ct < NJ; ++ct) acc[ct] = mma(ka[ct].x, ds[st][0], acc[ct]);
#pragma unroll
            for (int ct = 0; ct < NJ; ++ct) acc[ct] = mma(ka[ct].y, ds[st][1], acc[ct]);
#pragma unroll
            for (int ct = 0; ct < NJ; ++ct) acc[ct] = mma(ka[ct].z, ds[st][2], acc[ct]);
#pragma unroll
            for (int ct = 0; ct < NJ; ++ct) acc[ct] = mma(ka[ct].w, ds[st][3], acc[ct]);
        }
        if (t + 1 < nt) {
            float* nb = sm + ((t + 1) & 1) * (2 * D * kKP);
            store_cs<D>(rk, nb);
            store_cs<D>(rv, nb + D * kKP);
            if (t + 2 < nt) {
                load_cs<D, VEC>(kb, S, (t + 2) * kTok, rk);
                load_cs<D, VEC>(vb, S, (t + 2) * kTok, rv);
            }
        }
        __syncthreads();
    }
    if (!lok) return;
    float* db = dq + ((size_t)b * E + (size_t)h * D + 4 * lg) * L + l;
#pragma unroll
    for (int ct = 0; ct < NJ; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) db[(size_t)(16 * ct + r) * L] = acc[ct][r] * scale;
}

template <class K>
static int opt_in_lds(K kernel, size_t bytes) {
    if (bytes > 64 * 1024) LDM_HIP_TRY(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                           (int)bytes));
    return 0;
}

// key groups per block (flash_fwd_kernel's KH): 2 where the grid has at most one block per CU and the keys span
// two tiles or more (LDM_FLASH_KH = 1 / 2 forces it, A/B timing)
static int flash_kh(int64_t blocks, int ntiles) {
    static const int forced = [] {
        const char* e = std::getenv("LDM_FLASH_KH");
        return e ? std::atoi(e) : 0;
    }();
    if (forced == 1 || forced == 2) return ntiles >= 2 ? forced : 1;
    return blocks <= 256 && ntiles >= 2 ? 2 : 1;
}

// key splits over blocks (flash_fwd_kernel's SPL): doubled while the grid stays within 256 blocks and every split
// keeps 4 key tiles or more; g_flash_split = 0 (LDM_FLASH_SPLIT=0, ldm_set_flash_split(0)) keeps one block per
// (query tile, head)
static int g_flash_split = [] {
    const char* e = std::getenv("LDM_FLASH_SPLIT");
    return e ? std::atoi(e) : 1;
}();
// (LDM_FLASH_SPLIT = 8, A/B timing: up to 8 splits within 512 blocks, 2 tiles per split)
static int flash_splits(int64_t blocks, int ntiles) {
    if (!g_flash_split) return 1;
    const bool wide = g_flash_split == 8;
    const int maxsp = wide ? 8 : 4, maxb = wide ? 512 : 256, mint = wide ? 2 : 4;
    int nsp = 1;
    while (nsp < maxsp && blocks * 2 * nsp <= maxb && ntiles / (2 * nsp) >= mint) nsp *= 2;
    return nsp;
}

// The splits' workspace: per device one buffer of kLanes lanes, each stream that launches a split forward owning a
// lane (assigned on first use, inside a capture too: no allocation needed), so launches on two streams (concurrent
// sub-batch chains, a captured graph beside its eager warm-up) never share partials, and launches on one stream are
// ordered.  The buffer grows (never freed: a captured graph may still hold the old one) outside stream capture only;
// nullptr — the caller then runs unsplit — when a capture would need it to grow or the lanes are all taken.
static float* split_workspace(size_t floats, hipStream_t st) {
    constexpr int kLanes = 8, kDev = 16;
    static float* buf[kDev];
    static size_t cap[kDev];   // floats per lane
    static hipStream_t lane_st[kDev][kLanes];
    static int lanes[kDev];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kDev) return nullptr;
    int lane = -1;
    for (int i = 0; i < lanes[dev]; ++i)
        if (lane_st[dev][i] == st) lane = i;
    if (lane < 0) {
        if (lanes[dev] == kLanes) return nullptr;
        lane = lanes[dev]++;
        lane_st[dev][lane] = st;
    }
    if (cap[dev] < floats) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
        float* p = nullptr;
        if (hipMalloc(&p, floats * kLanes * sizeof(float)) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        buf[dev] = p;
        cap[dev] = floats;
    }
    return buf[dev] + (size_t)lane * cap[dev];
}

template <int D, bool TOK, bool LSE, bool VEC, int KH>
static int fwd_launch_k(const float* q, const float* kv, float* out, float* lse, int B, int E, int heads, int L, int S,
                        float scale, int nsp, hipStream_t st) {
    constexpr int NBUF = (KH == 2 && D == 128) ? 1 : 2;   // (D = 128 with two groups: one buffer each fits LDS)
    const size_t lds = (size_t)KH * NBUF * 2 * D * kKP * sizeof(float);
    const unsigned grid = (unsigned)B * heads * ((L + kTok - 1) / kTok);
    float* part = nullptr;
    if (nsp > 1) part = split_workspace((size_t)nsp * B * heads * L * (D + 4), st);
    if (part) {
        static int opted_s = opt_in_lds(flash_fwd_kernel<D, TOK, false, VEC, KH, NBUF, true>, lds);
        if (opted_s) return opted_s;
        hipLaunchKernelGGL((flash_fwd_kernel<D, TOK, false, VEC, KH, NBUF, true>), dim3(grid, (unsigned)nsp), dim3(256 * KH),
                           lds, st, q, kv, out, nullptr, E, heads, L, S, scale, part);
        LDM_CHECK_LAUNCH("flash_fwd_kernel (key splits)");
        if constexpr (TOK) {
            const int64_t n = (int64_t)B * heads * L * (D / 4);
            hipLaunchKernelGGL((flash_combine_kernel<D, LSE>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                               part, out, lse, nsp, B * heads, E, heads, L);
            LDM_CHECK_LAUNCH("flash_combine_kernel");
        } else {
            hipLaunchKernelGGL((flash_combine_cm_kernel<D, LSE>), dim3((unsigned)((L + 15) / 16), (unsigned)(B * heads)),
                               dim3(256), 0, st, part, out, lse, nsp, B * heads, E, heads, L);
            LDM_CHECK_LAUNCH("flash_combine_cm_kernel");
        }
        return 0;
    }
    static int opted = opt_in_lds(flash_fwd_kernel<D, TOK, LSE, VEC, KH, NBUF>, lds);
    if (opted) return opted;
    hipLaunchKernelGGL((flash_fwd_kernel<D, TOK, LSE, VEC, KH, NBUF>), dim3(grid), dim3(256 * KH), lds, st, q, kv, out,
                       lse, E, heads, L, S, scale, nullptr);
    LDM_CHECK_LAUNCH("flash_fwd_kernel");
    return 0;
}

template <int D, bool TOK, bool LSE>
static int fwd_launch(const float* q, const float* kv, float* out, float* lse, int B, int E, int heads, int L, int S,
                      float scale, hipStream_t st) {
    const int64_t blocks = (int64_t)B * heads * ((L + kTok - 1) / kTok);
    const int ntiles = (S + kTok - 1) / kTok;
    const int nsp = flash_splits(blocks, ntiles);
    const int kh = flash_kh(blocks * nsp, (ntiles + nsp - 1) / nsp);
    if (S % 4 == 0) {
        if (kh == 2) return fwd_launch_k<D, TOK, LSE, true, 2>(q, kv, out, lse, B, E, heads, L, S, scale, nsp, st);
        return fwd_launch_k<D, TOK, LSE, true, 1>(q, kv, out, lse, B, E, heads, L, S, scale, nsp, st);
    }
    if (kh == 2) return fwd_launch_k<D, TOK, LSE, false, 2>(q, kv, out, lse, B, E, heads, L, S, scale, nsp, st);
    return fwd_launch_k<D, TOK, LSE, false, 1>(q, kv, out, lse, B, E, heads, L, S, scale, nsp, st);
}

template <int D>
static int bwd_launch(const float* q, const float* kv, const float* out, const float* lse, const float* dout, float* dq,
                      float* dkv, float* delta, int B, int E, int heads, int L, int S, float scale, hipStream_t st) {
    const int64_t n = (int64_t)B * heads * L;
    hipLaunchKernelGGL(flash_delta_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, dout, delta, E, heads,
                       L, D, n);
    LDM_CHECK_LAUNCH("flash_delta_kernel");
    const size_t lds_kv = (2 * (size_t)kTok * (D + 4) + 2 * kTok) * sizeof(float);
    static int o1 = opt_in_lds(flash_bwd_dkv_kernel<D>, lds_kv);
    if (o1) return o1;
    hipLaunchKernelGGL(flash_bwd_dkv_kernel<D>, dim3((unsigned)B * heads * ((S + kTok - 1) / kTok)), dim3(256), lds_kv,
                       st, q, kv, dout, lse, delta, dkv, E, heads, L, S, scale);
    LDM_CHECK_LAUNCH("flash_bwd_dkv_kernel");
    const size_t lds_q = 4 * (size_t)D * kKP * sizeof(float);   // K and V, two buffers each
    static int o2 = opt_in_lds(flash_bwd_dq_kernel<D, true>, lds_q) | opt_in_lds(flash_bwd_dq_kernel<D, false>, lds_q);
    if (o2) return o2;
    if (S % 4 == 0)
        hipLaunchKernelGGL((flash_bwd_dq_kernel<D, true>), dim3((unsigned)B * heads * ((L + kTok - 1) / kTok)), dim3(256),
                           lds_q, st, q, kv, dout, lse, delta, dq, E, heads, L, S, scale);
    else
        hipLaunchKernelGGL((flash_bwd_dq_kernel<D, false>), dim3((unsigned)B * heads * ((L + kTok - 1) / kTok)), dim3(256),
                           lds_q, st, q, kv, dout, lse, delta, dq, E, heads, L, S, scale);
    LDM_CHECK_LAUNCH("flash_bwd_dq_kernel");
    return 0;
}

}  // namespace fa

bool attention_flash_supported(int E, int heads) {
    if (heads <= 0 || E % heads) return false;
    const int d = E / heads;
    return d == 64 || d == 128;
}

int attention_flash(const float* q, const float* kv, float* out, float* lse, int32_t B, int32_t E, int32_t heads,
                    int32_t L, int32_t S, float scale, bool tok, hipStream_t st) {
    LDM_REQUIRE(q && kv && out && B > 0 && L > 0 && S > 0, "attention (flash): bad argument");
    LDM_REQUIRE(attention_flash_supported(E, heads), "attention (flash): head dim must be 64 or 128");
    LDM_REQUIRE(!(tok && lse), "attention (flash): lse output with channel-major q only");
    const int d = E / heads;
#define LDM_FA(D)                                                                                   \
    if (d == D) {                                                                                   \
        if (tok) return fa::fwd_launch<D, true, false>(q, kv, out, nullptr, B, E, heads, L, S, scale, st); \
        if (lse) return fa::fwd_launch<D, false, true>(q, kv, out, lse, B, E, heads, L, S, scale, st);     \
        return fa::fwd_launch<D, false, false>(q, kv, out, nullptr, B, E, heads, L, S, scale, st);         \
    }
    LDM_FA(64)
    LDM_FA(128)
#undef LDM_FA
    return fail(3, "attention (flash): no instance");
}

}  // namespace ldm

using namespace ldm;

// A/B switch of the flash forward's key splits over blocks (bitwise-stable per setting; tests compare the two within
// fp32 rounding); returns the previous setting
extern "C" int ldm_set_flash_split(int on) {
    const int prev = fa::g_flash_split;
    fa::g_flash_split = on ? (on == 8 ? 8 : 1) : 0;
    return prev;
}

extern "C" int ldm_attention_forward_lse(const float* q, const float* kv, float* out, float* lse, int32_t B, int32_t E,
                                         int32_t heads, int32_t L, int32_t S, float scale, void* stream) {
    LDM_REQUIRE(lse, "attention_forward_lse: null lse");
    return attention_flash(q, kv, out, lse, B, E, heads, L, S, scale, false, (hipStream_t)stream);
}

extern "C" int ldm_attention_backward_flash(const float* q, const float* kv, const float* out, const float* lse,
                                            const float* dout, float* dq, float* dkv, float* delta_ws, int32_t B,
                                            int32_t E, int32_t heads, int32_t L, int32_t S, float scale, void* stream) {
    LDM_REQUIRE(q && kv && out && lse && dout && dq && dkv && delta_ws && B > 0 && L > 0 && S > 0,
                "attention_backward_flash: bad argument");
    LDM_REQUIRE(attention_flash_supported(E, heads), "attention_backward_flash: head dim must be 64 or 128");
    const int d = E / heads;
    if (d == 64)
        return fa::bwd_launch<64>(q, kv, out, lse, dout, dq, dkv, delta_ws, B, E, heads, L, S, scale, (hipStream_t)stream);
    return fa::bwd_launch<128>(q, kv, out, lse, dout, dq, dkv, delta_ws, B, E, heads, L, S, scale, (hipStream_t)stream);
}

extern "C" int ldm_attention_flash_supported(int32_t E, int32_t heads) { return attention_flash_supported(E, heads) ? 1 : 0; }
