// Implicit-GEMM 2-D convolution / transposed convolution for gfx950 (CDNA4), fp32.
//
// Replaces the reference's nn.Conv2d / nn.ConvTranspose2d (+BatchNorm2d eval, ReLU, Tanh, time-emb
// and skip adds) — model.py:16-25, :37-46, :61-79, :178-194, :205-229.
//
// GEMM view (per sub-pixel phase p of the output grid):
//     Y[m = cout][n = (b, qy, qx)] = sum_k A_p[m][k] * X_p[k][n],   k = tap * Cin + ci  (tap-major)
// A conv has one phase (q = output pixel).  A stride-2 transposed conv is split into its 4 output
// parities (ry, rx); each parity is an ordinary gather-conv over the input grid with only the taps
// that hit it (k3: 1/2/2/4 taps, k4: 4/4/4/4), so no multiply is spent on the zeros a
// zero-insertion formulation would create.
//
// A (weights) is re-laid once per weight version into the exact fragment order of the MFMA used
// (pack kernel below), so every lane's A operand arrives with one 16-byte load and a wave reads
// 1 KiB contiguous.  X is gathered straight from the NCHW activation: within a K-chunk the tap is
// wave-uniform, so a lane's 4 operand loads differ only by a channel stride and consecutive lanes
// read consecutive output pixels (coalesced).  Waves of a block split K; their partial tiles are
// summed in LDS in a fixed order (deterministic) and the fused epilogue runs once per output.
//
// The K loop is software-pipelined in registers: chunks are loaded in groups of kGroup, and the
// loads of group g+1 are issued before the MFMAs of group g, so at ~1-2 waves per SIMD (these GEMMs
// are small) the L2/HBM latency hides under matrix work instead of serialising every chunk.
//
// Matrix instructions (exact fp32, bitwise an fmaf chain — cdna_hip_programming.md §3):
//   kind 1: v_mfma_f32_32x32x2_f32  lane l: A[l&31][k=l>>5], B[k=l>>5][l&31]; D row=(r&3)+8(r>>2)+4(l>>5), col=l&31
//   kind 2: v_mfma_f32_16x16x4_f32  lane l: A[l&15][k=l>>4], B[k=l>>4][l&15]; D row=4(l>>4)+r,            col=l&15
// Within a K-chunk, lane group lg = lane/TILE holds k = NLG*j + lg for MFMA step j = 0..3 (NLG = 64/TILE).
#include <algorithm>
#include <cstdio>

#include "common.h"

#pragma clang fp contract(off)

namespace ldm {

struct ConvArgs {
    const float* x;
    const float* w;
    float* y;
    int32_t B, Cin, Hin, Win, Cout, Hout, Wout;
    int32_t KK;     // kh*kw
    int32_t Mpad;   // rows of the packed weight
    int32_t transposed;
    FastDiv fd_hw, fd_w;   // n -> (b, q) and q -> (qy, qx) of the phase grid
    PhaseTable pt;
    EpiArgs ep;
};

// ------------------------------------------------------------------------------------------------
// phase / tap tables
// ------------------------------------------------------------------------------------------------
int build_phase_table(const ldm_conv_desc& d, PhaseTable& pt) {
    pt = PhaseTable{};
    LDM_REQUIRE(d.B > 0 && d.Cin > 0 && d.Hin > 0 && d.Win > 0 && d.Cout > 0, "conv: empty dimension");
    LDM_REQUIRE(d.kh > 0 && d.kw > 0 && d.kh * d.kw <= kMaxTap, "conv: kernel larger than 4x4 unsupported");
    if (!d.transposed) {
        const int ho = (d.Hin + 2 * d.pad - d.kh) / d.stride + 1;
        const int wo = (d.Win + 2 * d.pad - d.kw) / d.stride + 1;
        LDM_REQUIRE(d.stride >= 1 && d.Hout == ho && d.Wout == wo, "conv: output size mismatch");
        pt.nphase = 1;
        pt.Hq = d.Hout;
        pt.Wq = d.Wout;
        pt.sy = d.stride;
        pt.osy = 1;
        pt.ry[0] = pt.rx[0] = 0;
        int n = 0;
        for (int a = 0; a < d.kh; ++a)
            for (int b = 0; b < d.kw; ++b) {
                pt.dy[0][n] = (int32_t)(a - d.pad);
                pt.dx[0][n] = (int32_t)(b - d.pad);
                pt.kk[0][n] = (int32_t)(a * d.kw + b);
                ++n;
            }
        pt.ntap[0] = n;
        return 0;
    }
    const int ho = (d.Hin - 1) * d.stride - 2 * d.pad + d.kh + d.out_pad;
    const int wo = (d.Win - 1) * d.stride - 2 * d.pad + d.kw + d.out_pad;
    LDM_REQUIRE(d.Hout == ho && d.Wout == wo, "conv_transpose: output size mismatch");
    if (d.stride == 1) {
        // stride-1 transposed conv (= the data gradient of a stride-1 conv): one phase,
        // out[o] += x[o + pad - k] * w[k]  ->  dy = pad - kh
        pt.nphase = 1;
        pt.Hq = d.Hout;
        pt.Wq = d.Wout;
        pt.sy = 1;
        pt.osy = 1;
        int n = 0;
        for (int a = 0; a < d.kh; ++a)
            for (int b = 0; b < d.kw; ++b) {
                pt.dy[0][n] = (int32_t)(d.pad - a);
                pt.dx[0][n] = (int32_t)(d.pad - b);
                pt.kk[0][n] = (int32_t)(a * d.kw + b);
                ++n;
            }
        pt.ntap[0] = n;
        return 0;
    }
    // transposed: stride 2 with Hout == 2*Hin (k3 p1 op1, k4 p1 op0) -> 4 parity phases
    LDM_REQUIRE(d.stride == 2 && d.Hout == 2 * d.Hin && d.Wout == 2 * d.Win,
                "conv_transpose: only stride 2 with Hout == 2*Hin is supported");
    pt.nphase = 4;
    pt.Hq = d.Hin;
    pt.Wq = d.Win;
    pt.sy = 1;
    pt.osy = 2;
    for (int ry = 0; ry < 2; ++ry)
        for (int rx = 0; rx < 2; ++rx) {
            const int p = ry * 2 + rx;
            pt.ry[p] = ry;
            pt.rx[p] = rx;
            int n = 0;
            for (int a = 0; a < d.kh; ++a) {
                const int vy = ry + d.pad - a;
                if (vy & 1) continue;
                for (int b = 0; b < d.kw; ++b) {
                    const int vx = rx + d.pad - b;
                    if (vx & 1) continue;
                    LDM_REQUIRE(n < kMaxTap, "conv_transpose: too many taps");
                    pt.dy[p][n] = (int32_t)(vy >> 1);
                    pt.dx[p][n] = (int32_t)(vx >> 1);
                    pt.kk[p][n] = (int32_t)(a * d.kw + b);
                    ++n;
                }
            }
            pt.ntap[p] = n;
        }
    return 0;
}

static int chunk_k(int kind) { return kind == 1 ? 8 : 16; }
static int tile_m(int kind) { return kind == 1 ? 32 : 16; }

// fill wofs / kchunks / Mpad for a plan
static int layout_for_plan(const ldm_conv_desc& d, const ldm_conv_plan& p, PhaseTable& pt, int& Mpad, int64_t& floats) {
    int rc = build_phase_table(d, pt);
    if (rc) return rc;
    floats = 0;
    Mpad = d.Cout;
    if (p.kind == 0) {
        for (int i = 0; i < pt.nphase; ++i) pt.wofs[i] = 0, pt.kchunks[i] = 0;
        return 0;
    }
    const int ck = chunk_k(p.kind);
    LDM_REQUIRE(d.Cin % ck == 0, "conv: MFMA plan needs Cin % chunk == 0");
    const int bm = tile_m(p.kind) * p.tm;
    Mpad = (d.Cout + bm - 1) / bm * bm;
    for (int i = 0; i < pt.nphase; ++i) {
        pt.kchunks[i] = pt.ntap[i] * (d.Cin / ck);
        pt.wofs[i] = floats;
        floats += (int64_t)pt.kchunks[i] * Mpad * ck;
    }
    return 0;
}

// ------------------------------------------------------------------------------------------------
// epilogue (op order of the reference: conv+bias -> BN(eval) -> act -> +bcast -> +skip)
// ------------------------------------------------------------------------------------------------
// Epilogue operands of one output element, loaded ahead of time (before the K loop) so their memory
// latency overlaps the GEMM instead of trailing it.
struct EpiPre {
    float bias, bcast, skip, x;
};

__device__ __forceinline__ EpiPre epi_prefetch(const ConvArgs& a, int m, int b, size_t oidx) {
    const EpiArgs& e = a.ep;
    EpiPre p;
    p.bias = e.bias ? e.bias[m] : 0.f;
    p.bcast = e.bcast ? e.bcast[(size_t)b * a.Cout + m] : 0.f;
    p.skip = e.skip ? e.skip[oidx] : 0.f;
    p.x = e.ddim_coef ? e.ddim_x[oidx] : 0.f;
    return p;
}

__device__ __forceinline__ void epi_finish(const ConvArgs& a, int m, size_t oidx, float v, const EpiPre& p) {
    const EpiArgs& e = a.ep;
    if (e.bias) v = v + p.bias;
    if (e.bn_w) {
        // aten batch_norm_cpu_collect_linear_and_constant_terms: alpha = invstd*w, beta = b - mean*alpha
        const float invstd = 1.0f / sqrtf(e.bn_v[m] + e.bn_eps);
        const float alpha = invstd * e.bn_w[m];
        const float beta = e.bn_b[m] - e.bn_m[m] * alpha;
        v = v * alpha + beta;
    }
    v = apply_act(v, e.act);
    if (e.act_out) e.act_out[oidx] = v;
    if (e.bcast) v = v + p.bcast;
    if (e.skip) v = v + p.skip;
    if (e.ddim_coef) {
        float x0;
        e.ddim_x[oidx] = ddim_update(p.x, v, e.ddim_coef, e.ddim_eta, x0);
        if (e.ddim_x0_log) e.ddim_x0_log[oidx] = x0;
        if (e.ddim_eps_log) e.ddim_eps_log[oidx] = v;
        if (a.y) a.y[oidx] = v;
        return;
    }
    a.y[oidx] = v;
}

__device__ __forceinline__ void epilogue_store(const ConvArgs& a, int m, int b, int oy, int ox, float v) {
    const size_t oidx = (((size_t)b * a.Cout + m) * a.Hout + oy) * a.Wout + ox;
    epi_finish(a, m, oidx, v, epi_prefetch(a, m, b, oidx));
}

// ------------------------------------------------------------------------------------------------
// MFMA traits
// ------------------------------------------------------------------------------------------------
template <int KIND>
struct Mfma;

template <>
struct Mfma<1> {
    static constexpr int TILE = 32, NLG = 2, NACC = 16;
    typedef floatx16 acc_t;
    static __device__ __forceinline__ acc_t mma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int r, int lg) { return (r & 3) + 8 * (r >> 2) + 4 * lg; }
};

template <>
struct Mfma<2> {
    static constexpr int TILE = 16, NLG = 4, NACC = 4;
    typedef floatx4 acc_t;
    static __device__ __forceinline__ acc_t mma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int r, int lg) { return 4 * lg + r; }
};

constexpr int kGroup = 4;   // K-chunks per prefetch group

template <int TM, int TN>
struct Frag {
    floatx4 a[TM];
    float b[TN][4];
};

// ------------------------------------------------------------------------------------------------
// kinds 1/2: block = WK waves over one (TILE*TM x TILE*TN) output tile of one phase; each wave owns
// every WK-th K-chunk, register-pipelined in groups of kGroup chunks.
// ------------------------------------------------------------------------------------------------
template <int KIND, int TM, int TN, int WK>
__global__ __launch_bounds__(64 * WK) void conv_mfma_kernel(ConvArgs a) {
    using MF = Mfma<KIND>;
    constexpr int TILE = MF::TILE, NLG = MF::NLG, CK = 4 * NLG;
    constexpr int BM = TILE * TM, BN = TILE * TN;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int lane = threadIdx.x & 63;
    // wave index made provably uniform: chunk / tap indices then live in SGPRs and the tap-table
    // lookups below are scalar kernarg loads (lgkmcnt), not per-lane global loads that would force a
    // vmcnt(0) drain of the prefetched operands on every chunk.
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ph = blockIdx.z;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const int HqWq = a.pt.Hq * a.pt.Wq;
    const int Nq = a.B * HqWq;
    const int HWin = a.Hin * a.Win;
    const int col = lane % TILE, lg = lane / TILE;

    // Operands come through bounds-checked buffer loads: one SGPR descriptor per tensor, a per-lane
    // 32-bit byte offset fixed for a whole tap, and a scalar soffset that walks the K chunks — so the
    // K loop spends no VALU on addressing, and an input pixel outside the window (padding) is simply an
    // out-of-range offset that the hardware returns as 0.
    constexpr int kOOB = 0x7ffffff0;
    // per output column: top-left input pixel (iy0, ix0) of its window and the byte offset of
    // (b, channel lg, iy0, ix0); a tap then only adds the uniform (dy, dx).  Invalid columns get
    // iy0 = -0x4000000 so every tap falls outside the window.
    int iy0[TN], ix0[TN], base4[TN];
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
        const int n = n0 + TILE * ni + col;
        const bool nv = n < Nq;
        const int nn = nv ? n : 0;
        const int b = a.fd_hw.div(nn);
        const int r = nn - b * HqWq;
        const int qy = a.fd_w.div(r);
        const int qx = r - qy * a.pt.Wq;
        iy0[ni] = nv ? qy * a.pt.sy : -0x4000000;
        ix0[ni] = qx * a.pt.sy;
        base4[ni] = ((b * a.Cin + lg) * HWin + iy0[ni] * a.Win + ix0[ni]) * 4;
    }

    typename MF::acc_t acc[TM][TN];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni)
#pragma unroll
            for (int r = 0; r < MF::NACC; ++r) acc[mi][ni][r] = 0.f;

    const int cpt = a.Cin / CK;   // chunks per tap
    const int nchunk = a.pt.kchunks[ph];
    const int wstride_b = a.Mpad * CK * 4;                 // bytes per packed chunk
    const int nmine = nchunk > wave ? (nchunk - wave + WK - 1) / WK : 0;
    const int ngrp = (nmine + kGroup - 1) / kGroup;
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.B * a.Cin * HWin * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.w + a.pt.wofs[ph]), (short)0, nchunk * wstride_b, 0x00020000);
    const int a_voff = ((m0 + col) * CK + lg * 4) * 4;
    const int cstep_b = CK * HWin * 4;                     // bytes per channel chunk in x

    // Epilogue operands of the outputs this thread will finish (element e = tid + k*64*WK of the tile),
    // issued now so they land while the K loop runs.
    constexpr int EPT = (BM * BN + 64 * WK - 1) / (64 * WK);
    constexpr bool kPre = EPT <= 8;
    EpiPre pre[kPre ? EPT : 1];
    int po[kPre ? EPT : 1], pm[kPre ? EPT : 1];
    if constexpr (kPre) {
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const int e = (int)threadIdx.x + k * 64 * WK;
            const int mloc = e / BN, nloc = e - mloc * BN;
            const int m = m0 + mloc, n = n0 + nloc;
            const bool valid = e < BM * BN && m < a.Cout && n < Nq;
            const int mm = valid ? m : 0, nn = valid ? n : 0;
            const int b = a.fd_hw.div(nn);
            const int r = nn - b * HqWq;
            const int qyy = a.fd_w.div(r);
            const int qxx = r - qyy * a.pt.Wq;
            const int oy = qyy * a.pt.osy + a.pt.ry[ph], ox = qxx * a.pt.osy + a.pt.rx[ph];
            const size_t oidx = (((size_t)b * a.Cout + mm) * a.Hout + oy) * a.Wout + ox;
            pre[k] = epi_prefetch(a, mm, b, oidx);
            po[k] = valid ? (int)oidx : -1;
            pm[k] = mm;
        }
    }

    // K cursor (wave-uniform): chunk c = wave + WK*i  <->  (tap t, channel chunk cc), advanced without
    // division; per-lane tap offsets are recomputed only when the tap changes.
    int t_ld = wave / cpt, cc_ld = wave - (wave / cpt) * cpt, c_ld = wave;
    int tcur = -1;
    int voff[TN];
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) voff[ni] = kOOB;

    // Loads are unconditional (past this wave's range the cursor stays on its last chunk and the
    // compute is skipped): every path has the same loads in flight, so the vmcnt bookkeeping stays
    // exact and the next group's loads really overlap this group's MFMAs.
    auto load = [&](Frag<TM, TN>(&f)[kGroup], int grp) {
#pragma unroll
        for (int q = 0; q < kGroup; ++q) {
            const int i = grp * kGroup + q;
            if (t_ld != tcur) {
                tcur = t_ld;
                const int dy = a.pt.dy[ph][t_ld], dx = a.pt.dx[ph][t_ld];
                const int dxy4 = (dy * a.Win + dx) * 4;   // uniform
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {
                    const bool ok = (unsigned)(iy0[ni] + dy) < (unsigned)a.Hin && (unsigned)(ix0[ni] + dx) < (unsigned)a.Win;
                    voff[ni] = ok ? base4[ni] + dxy4 : kOOB;
                }
            }
            const int soff_a = c_ld * wstride_b;
            const int soff_b = cc_ld * cstep_b;
#pragma unroll
            for (int mi = 0; mi < TM; ++mi)
                f[q].a[mi] = __builtin_bit_cast(
                    floatx4, __builtin_amdgcn_raw_buffer_load_b128(wr, a_voff + mi * TILE * CK * 4, soff_a, 0));
#pragma unroll
            for (int ni = 0; ni < TN; ++ni)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    f[q].b[ni][j] = __builtin_bit_cast(
                        float, __builtin_amdgcn_raw_buffer_load_b32(xr, voff[ni], soff_b + NLG * j * HWin * 4, 0));
            if (i + 1 < nmine) {   // advance the cursor to this wave's next chunk
                c_ld += WK;
                cc_ld += WK;
                while (cc_ld >= cpt) {
                    cc_ld -= cpt;
                    ++t_ld;
                }
            }
        }
    };
    auto compute = [&](const Frag<TM, TN>(&f)[kGroup], int grp) {
#pragma unroll
        for (int q = 0; q < kGroup; ++q) {
            if (grp * kGroup + q < nmine) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                        for (int ni = 0; ni < TN; ++ni)
                            acc[mi][ni] = MF::mma(f[q].a[mi][j], f[q].b[ni][j], acc[mi][ni]);
            }
        }
    };

    Frag<TM, TN> f0[kGroup], f1[kGroup];
    if (ngrp > 0) {
        load(f0, 0);
        for (int g = 0; g < ngrp; g += 2) {
            load(f1, g + 1);    // may be past the end: clamped + masked
            compute(f0, g);
            if (g + 2 < ngrp) load(f0, g + 2);
            compute(f1, g + 1);
        }
    }

    // split-K partial tiles -> LDS, fixed-order sum, fused epilogue
    float* sw = smem + wave * BM * BN;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni)
#pragma unroll
            for (int r = 0; r < MF::NACC; ++r)
                sw[(TILE * mi + MF::row(r, lg)) * BN + TILE * ni + col] = acc[mi][ni][r];
    __syncthreads();
    if constexpr (kPre) {
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const int e = (int)threadIdx.x + k * 64 * WK;
            if (po[k] < 0) continue;
            float v = smem[e];
#pragma unroll
            for (int w = 1; w < WK; ++w) v = v + smem[w * BM * BN + e];
            epi_finish(a, pm[k], (size_t)po[k], v, pre[k]);
        }
    } else {
        for (int e = threadIdx.x; e < BM * BN; e += 64 * WK) {
            const int mloc = e / BN, nloc = e - mloc * BN;
            const int m = m0 + mloc, n = n0 + nloc;
            if (m >= a.Cout || n >= Nq) continue;
            float v = smem[e];
#pragma unroll
            for (int w = 1; w < WK; ++w) v = v + smem[w * BM * BN + e];
            const int b = n / HqWq;
            const int r = n - b * HqWq;
            const int qyy = r / a.pt.Wq;
            const int qxx = r - qyy * a.pt.Wq;
            epilogue_store(a, m, b, qyy * a.pt.osy + a.pt.ry[ph], qxx * a.pt.osy + a.pt.rx[ph], v);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// kind 0: direct VALU conv (Cin not a multiple of 8, or tiny Cout: VAE first/last layers)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_direct_kernel(ConvArgs a) {
    const int64_t total = (int64_t)a.B * a.Cout * a.Hout * a.Wout;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int ox = (int)(idx % a.Wout);
    int64_t rest = idx / a.Wout;
    const int oy = (int)(rest % a.Hout);
    rest /= a.Hout;
    const int co = (int)(rest % a.Cout);
    const int b = (int)(rest / a.Cout);
    int ph, qy, qx;
    if (a.pt.osy == 1) {
        ph = 0;
        qy = oy;
        qx = ox;
    } else {
        ph = (oy & 1) * 2 + (ox & 1);
        qy = oy >> 1;
        qx = ox >> 1;
    }
    const int HWin = a.Hin * a.Win;
    const float* xb = a.x + (size_t)b * a.Cin * HWin;
    const size_t wci = a.transposed ? (size_t)a.Cout * a.KK : (size_t)a.KK;
    const float* wb = a.w + (a.transposed ? (size_t)co * a.KK : (size_t)co * a.Cin * a.KK);
    float acc = 0.f;
    const int nt = a.pt.ntap[ph];
    for (int t = 0; t < nt; ++t) {
        const int iy = qy * a.pt.sy + a.pt.dy[ph][t];
        const int ix = qx * a.pt.sy + a.pt.dx[ph][t];
        if (iy < 0 || iy >= a.Hin || ix < 0 || ix >= a.Win) continue;
        const float* xp = xb + iy * a.Win + ix;
        const float* wq = wb + a.pt.kk[ph][t];
        for (int ci = 0; ci < a.Cin; ++ci) acc = fmaf(xp[(size_t)ci * HWin], wq[ci * wci], acc);
    }
    epilogue_store(a, co, b, oy, ox, acc);
}

// ------------------------------------------------------------------------------------------------
// weight packing into fragment order: packed[phase][chunk][Mpad][NLG][4], k = chunk*CK + NLG*j + lg
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_pack_kernel(const float* __restrict__ w, float* __restrict__ out, ConvArgs a,
                                                        int kind, int64_t total) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int nlg = kind == 1 ? 2 : 4;
    const int ck = 4 * nlg;
    int ph = 0;
    for (int p = 1; p < a.pt.nphase; ++p)
        if (idx >= a.pt.wofs[p]) ph = p;
    const int64_t local = idx - a.pt.wofs[ph];
    const int slot = (int)(local % ck);
    const int64_t rowid = local / ck;
    const int m = (int)(rowid % a.Mpad);
    const int c = (int)(rowid / a.Mpad);
    const int lg = slot >> 2, j = slot & 3;
    const int k = c * ck + nlg * j + lg;
    const int t = k / a.Cin, ci = k - t * a.Cin;
    float v = 0.f;
    if (m < a.Cout && t < a.pt.ntap[ph]) {
        const int kk = a.pt.kk[ph][t];
        v = a.transposed ? w[((size_t)ci * a.Cout + m) * a.KK + kk] : w[((size_t)m * a.Cin + ci) * a.KK + kk];
    }
    out[idx] = v;
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
static int make_args(const ldm_conv_desc& d, const ldm_conv_plan& p, ConvArgs& a) {
    a = ConvArgs{};
    int64_t floats = 0;
    int rc = layout_for_plan(d, p, a.pt, a.Mpad, floats);
    if (rc) return rc;
    a.B = d.B;
    a.Cin = d.Cin;
    a.Hin = d.Hin;
    a.Win = d.Win;
    a.Cout = d.Cout;
    a.Hout = d.Hout;
    a.Wout = d.Wout;
    a.KK = d.kh * d.kw;
    a.transposed = d.transposed;
    a.fd_hw = FastDiv::make(a.pt.Hq * a.pt.Wq);
    a.fd_w = FastDiv::make(a.pt.Wq);
    return 0;
}

static bool plan_ok(const ldm_conv_desc& d, int kind, int tm, int tn, int wk) {
    if (kind == 0) return true;
    if (kind != 1 && kind != 2) return false;
    if (tm < 1 || tm > 2 || tn < 1 || tn > 2) return false;
    if (wk != 1 && wk != 2 && wk != 4 && wk != 8) return false;
    if (d.Cin % chunk_k(kind) != 0) return false;
    const int bm = tile_m(kind) * tm, bn = tile_m(kind) * tn;
    if ((int64_t)wk * bm * bn * 4 > 64 * 1024) return false;
    return true;
}

}  // namespace ldm

using namespace ldm;

extern "C" int ldm_conv_make_plan_forced(const ldm_conv_desc* d, int kind, int tm, int tn, int wk, ldm_conv_plan* plan) {
    LDM_REQUIRE(d && plan, "conv plan: null argument");
    LDM_REQUIRE(plan_ok(*d, kind, tm, tn, wk), "conv plan: unsupported (kind, tm, tn, wk) for this layer");
    ldm_conv_plan p{};
    p.kind = kind;
    p.tm = kind ? tm : 1;
    p.tn = kind ? tn : 1;
    p.wk = kind ? wk : 1;
    PhaseTable pt;
    int Mpad;
    int64_t floats;
    int rc = layout_for_plan(*d, p, pt, Mpad, floats);
    if (rc) return rc;
    p.packed_floats = floats;
    *plan = p;
    return 0;
}

extern "C" int ldm_conv_make_plan(const ldm_conv_desc* d, ldm_conv_plan* plan) {
    LDM_REQUIRE(d && plan, "conv plan: null argument");
    PhaseTable pt;
    int rc = build_phase_table(*d, pt);
    if (rc) return rc;
    const int M = d->Cout;
    const int64_t Nq = (int64_t)d->B * pt.Hq * pt.Wq;
    int maxtap = 0;
    for (int i = 0; i < pt.nphase; ++i) maxtap = std::max(maxtap, pt.ntap[i]);
    // direct VALU path: no 8-aligned channel chunks, or tiny output channel count
    if (d->Cin % 8 != 0 || M < 16) return ldm_conv_make_plan_forced(d, 0, 1, 1, 1, plan);
    // Heuristic (refined by the Python-side autotuner): fill >= ~2048 waves (2 per SIMD).
    auto tiles_for = [&](int kind, int tm, int tn) {
        const int bm = tile_m(kind) * tm, bn = tile_m(kind) * tn;
        return (int64_t)((M + bm - 1) / bm) * ((Nq + bn - 1) / bn) * pt.nphase;
    };
    int kind = (M >= 32 && Nq >= 32) ? 1 : 2;
    if (kind == 2 && d->Cin % 16 != 0) return ldm_conv_make_plan_forced(d, 0, 1, 1, 1, plan);
    int64_t tiles = tiles_for(kind, 1, 1);
    if (kind == 1 && tiles * 8 < 1024 && d->Cin % 16 == 0) {
        kind = 2;
        tiles = tiles_for(kind, 1, 1);
    }
    const int64_t chunks = (int64_t)maxtap * (d->Cin / chunk_k(kind));
    int wk = 1;
    while (wk < 8 && tiles * wk < 2048 && chunks / (wk * 2) >= 2) wk *= 2;
    return ldm_conv_make_plan_forced(d, kind, 1, 1, wk, plan);
}

extern "C" int ldm_conv_pack_weight(const ldm_conv_desc* d, const ldm_conv_plan* plan, const float* w, float* packed,
                                    void* stream) {
    LDM_REQUIRE(d && plan && w, "conv pack: null argument");
    if (plan->kind == 0) return 0;
    LDM_REQUIRE(packed, "conv pack: null output");
    ConvArgs a;
    int rc = make_args(*d, *plan, a);
    if (rc) return rc;
    const int64_t total = plan->packed_floats;
    const int threads = 256;
    const int64_t blocks = (total + threads - 1) / threads;
    hipLaunchKernelGGL(conv_pack_kernel, dim3((unsigned)blocks), dim3(threads), 0, (hipStream_t)stream, w, packed, a,
                       plan->kind, total);
    LDM_CHECK_LAUNCH("conv_pack_kernel");
    return 0;
}

template <int KIND>
static int launch_mfma(const ConvArgs& a, const ldm_conv_plan& p, int64_t Nq, hipStream_t st) {
    const int TILE = Mfma<KIND>::TILE;
    const int BMx = TILE * p.tm, BNx = TILE * p.tn;
    const size_t lds = (size_t)p.wk * BMx * BNx * sizeof(float);
    dim3 grid((unsigned)((Nq + BNx - 1) / BNx), (unsigned)((a.Cout + BMx - 1) / BMx), a.pt.nphase);
    dim3 block(64 * p.wk);
    const int code = (p.tm - 1) * 2 + (p.tn - 1);
#define LDM_CASE(WK, C, TM, TN) \
    case WK * 10 + C: hipLaunchKernelGGL((conv_mfma_kernel<KIND, TM, TN, WK>), grid, block, lds, st, a); break;
    switch (p.wk * 10 + code) {
        LDM_CASE(1, 0, 1, 1) LDM_CASE(1, 1, 1, 2) LDM_CASE(1, 2, 2, 1) LDM_CASE(1, 3, 2, 2)
        LDM_CASE(2, 0, 1, 1) LDM_CASE(2, 1, 1, 2) LDM_CASE(2, 2, 2, 1) LDM_CASE(2, 3, 2, 2)
        LDM_CASE(4, 0, 1, 1) LDM_CASE(4, 1, 1, 2) LDM_CASE(4, 2, 2, 1) LDM_CASE(4, 3, 2, 2)
        LDM_CASE(8, 0, 1, 1) LDM_CASE(8, 1, 1, 2) LDM_CASE(8, 2, 2, 1) LDM_CASE(8, 3, 2, 2)
        default: return fail(3, "conv: no kernel instance for plan");
    }
#undef LDM_CASE
    LDM_CHECK_LAUNCH("conv_mfma_kernel");
    return 0;
}

namespace ldm {

int conv_forward_ex(const ldm_conv_desc& d, const ldm_conv_plan& p, const float* x, const float* w, const EpiArgs& ep,
                    float* y, hipStream_t st) {
    LDM_REQUIRE(x && w && (y || ep.ddim_coef), "conv forward: null argument");
    LDM_REQUIRE(!ep.ddim_coef || ep.ddim_x, "conv forward: fused DDIM update needs x");
    ConvArgs a;
    int rc = make_args(d, p, a);
    if (rc) return rc;
    a.x = x;
    a.w = w;
    a.y = y;
    a.ep = ep;
    LDM_REQUIRE(!a.ep.bn_w || (a.ep.bn_b && a.ep.bn_m && a.ep.bn_v), "conv: incomplete BatchNorm parameters");
    const int64_t Nq = (int64_t)d.B * a.pt.Hq * a.pt.Wq;
    if (p.kind == 0) {
        const int64_t total = (int64_t)d.B * d.Cout * d.Hout * d.Wout;
        hipLaunchKernelGGL(conv_direct_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a);
        LDM_CHECK_LAUNCH("conv_direct_kernel");
        return 0;
    }
    LDM_REQUIRE(plan_ok(d, p.kind, p.tm, p.tn, p.wk), "conv forward: invalid plan");
    // buffer descriptors use 32-bit byte offsets; padding lanes use offset 0x7ffffff0 (out of range)
    LDM_REQUIRE((int64_t)d.B * d.Cin * d.Hin * d.Win * 4 < 0x7ff00000LL &&
                    p.packed_floats * 4 < 0x7ff00000LL,
                "conv forward: tensor too large for 32-bit buffer offsets (split the batch)");
    return p.kind == 1 ? launch_mfma<1>(a, p, Nq, st) : launch_mfma<2>(a, p, Nq, st);
}

}  // namespace ldm

extern "C" int ldm_conv_forward(const ldm_conv_desc* d, const ldm_conv_plan* plan, const float* x, const float* w,
                                const ldm_epilogue* ep, float* y, void* stream) {
    LDM_REQUIRE(d && plan && x && w && y, "conv forward: null argument");
    EpiArgs e{};
    if (ep) {
        e.bias = ep->bias;
        e.bn_w = ep->bn_weight;
        e.bn_b = ep->bn_bias;
        e.bn_m = ep->bn_mean;
        e.bn_v = ep->bn_var;
        e.bn_eps = ep->bn_eps;
        e.act = ep->act;
        e.bcast = ep->bcast_add;
        e.skip = ep->skip_add;
        e.act_out = ep->act_out;
    }
    return conv_forward_ex(*d, *plan, x, w, e, y, (hipStream_t)stream);
}
