// LDS-staged fp16 / bf16 implicit-GEMM convolution for the large-plane layers of the train step and the
// VGGish feature stack (plan kind 3): NCHW fp32 activations, operands rounded to the autocast precision,
// fp32 accumulation on the gfx950 double-rate v_mfma_f32_32x32x16_{bf16,f16}.
//
// Why: at B = 32 on 1x128x512 mels (VAE encoder / decoder, style encoder, and their data gradients) and
// in the VGGish stack, the general kernel (conv.hip) gives each wave its own operand stream with no
// sharing inside a block; its 1-wave blocks re-fetched ~1 GB per launch of the decoder's 128 -> 64 convT
// and ran its 32x32x8 MFMAs at 10 % busy (profiles/r02/train_pmc.json).  Here a block owns a BM x 128
// output tile (BM output channels x 128 positions of one phase grid), K = taps x Cin in chunks of 32
// (a chunk is one tap and 32 channels; channel-chunk major, tap minor, so the 3-9 taps that read one
// input window run back to back and find its lines in L2 — tap-major order re-fetched each input line
// from the Infinity Cache once per tap), and per chunk:
//   * every lane gathers 16 channels of one position at the chunk's tap (each load instruction is 64
//     consecutive positions: coalesced for stride 1, 2 lines per 64 lanes at stride 2), rounds them to
//     16-bit and writes them as two 16-byte LDS stores: B tile [128 positions][32 k] (double-buffered);
//   * the 4 waves (2 along M x 2 along N) read their B fragments from LDS (one ds_read_b128 per 32x16
//     fragment) and their A fragments straight from the pre-packed 16-bit weights (L2-resident, one
//     16-byte load per fragment, issued one chunk ahead), and issue BM/32 x 2 x 2 MFMAs;
//   * the next chunk's gather is in flight while the MFMAs run; one barrier per chunk.
// Transposed convs run as their sub-pixel phases (build_phase_table), one phase per block.
//
// MFMA operand maps (cdna_hip_programming.md §3): lane l (r = l & 31, h = l >> 5) holds A[row r][k = 8h + j]
// and B[k = 8h + j][col r], j = 0..7; D: col = l & 31, row = (reg & 3) + 8 (reg >> 2) + 4h.
#include <cstdlib>
#include <type_traits>

#include "common.h"

// Diagnostic builds only (tools/build_diag.sh): TCONV_DIAG bit 0 = no gather loads (B from registers),
// bit 1 = no MFMAs.
#ifndef TCONV_DIAG
#define TCONV_DIAG 0
#endif

namespace ldm {
namespace tc {

constexpr int BN = 128;   // positions per block
constexpr int KC = 32;    // k per chunk (one tap, 32 input channels)
constexpr int KP = 40;    // LDS row pitch (16-bit elements): 80-B rows keep 16 lanes' 16-B accesses conflict-free
constexpr int kOOB = 0x7ffffff0;

typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef float floatx8 __attribute__((ext_vector_type(8)));

struct TArgs {
    const float* x;
    const unsigned short* w;   // packed [phase][chunk][Mpad][32] 16-bit
    float* y;
    int32_t B, Cin, Hin, Win, Cout, Hout, Wout;
    int32_t Mpad, nM, nN, cpt;   // cpt = Cin / KC chunks per tap
    int32_t xcd_chunk;           // > 0: tiles per XCD of the XCD-contiguous block order (blocks % 8 == 0)
    int64_t N;                   // positions per phase (B * Hq * Wq)
    FastDiv fd_hw, fd_w;
    PhaseTable pt;               // wofs in 16-bit elements
    EpiArgs ep;
};

template <int DT>
__device__ __forceinline__ u16x8 to16(const floatx8& v) {
    if constexpr (DT == 1)
        return __builtin_bit_cast(u16x8, __builtin_convertvector(v, halfx8));
    else
        return __builtin_bit_cast(u16x8, __builtin_convertvector(v, bf16x8));
}

template <int DT>
__device__ __forceinline__ floatx16 mma(const u16x8& a, const u16x8& b, const floatx16& c) {
    if constexpr (DT == 1)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(halfx8, a), __builtin_bit_cast(halfx8, b), c, 0,
                                                      0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                       0, 0, 0);
}

template <int BM, int DT>
__global__ __launch_bounds__(256) void tconv_kernel(TArgs a) {
    constexpr int MT = BM / 64;   // 32-row tiles per wave (2 waves along M)
    __shared__ __attribute__((aligned(16))) unsigned short bt[2][BN * KP];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int r = lane & 31, h = lane >> 5;

    // block -> (N tile, phase, M tile), M fastest, then the phases: the blocks of one N tile gather the same
    // input window.  Blocks go round-robin to the 8 XCDs (block b to XCD b % 8), so with xcd_chunk each XCD
    // walks its own contiguous run of tiles: the windows of neighbouring N tiles and all phases of one N
    // tile meet in that XCD's L2 instead of being fetched by every XCD from the Infinity Cache.
    int t = blockIdx.x;
    if (a.xcd_chunk > 0) t = (t & 7) * a.xcd_chunk + (t >> 3);
    const int mt = t % a.nM;
    const int rest = t / a.nM;
    const int ph = rest % a.pt.nphase;
    const int nt = rest / a.pt.nphase;
    const int ntap = a.pt.ntap[ph];
    const int nch = ntap * a.cpt;
    const int64_t n0 = (int64_t)nt * BN;
    const int HWin = a.Hin * a.Win;

    // ---- gather role: position gp = tid & 127, channels 16 * (tid >> 7) .. +15 of each chunk
    const int gp = tid & (BN - 1), gk = tid >> 7;
    int gb = 0, gqy = 0, gqx = 0;
    bool gval;
    {
        const int64_t n = n0 + gp;
        gval = n < a.N;
        const int nn = gval ? (int)n : 0;
        gb = a.fd_hw.div(nn);
        const int rr = nn - gb * (a.pt.Hq * a.pt.Wq);
        gqy = a.fd_w.div(rr);
        gqx = rr - gqy * a.pt.Wq;
    }
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(a.x), (short)0, uni(a.B * a.Cin * HWin * 4), 0x00020000);
    const int gbase = (gb * a.Cin + gk * 16) * HWin;   // floats
    auto gather = [&](int c, float (&gv)[16]) {
        const int cc = c / ntap;   // channel-chunk major, tap minor: the taps of a window run back to back
        const int t = c - cc * ntap;   // (wave-uniform)
        const int ci0 = cc * KC;
        const int iy = gqy * a.pt.sy + a.pt.dy[ph][t];
        const int ix = gqx * a.pt.sy + a.pt.dx[ph][t];
        const bool ok = gval && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
        const int voff = ok ? (gbase + ci0 * HWin + iy * a.Win + ix) * 4 : kOOB;
#pragma unroll
        for (int j = 0; j < 16; ++j)
            gv[j] = (TCONV_DIAG & 1) ? (float)(voff + j)
                                     : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, voff, uni(j * HWin * 4), 0));
    };
    auto stage = [&](int buf, const float (&gv)[16]) {
        floatx8 lo, hi;
#pragma unroll
        for (int j = 0; j < 8; ++j) lo[j] = gv[j], hi[j] = gv[8 + j];
        u16x8* dst = reinterpret_cast<u16x8*>(&bt[buf][gp * KP + gk * 16]);
        dst[0] = to16<DT>(lo);
        dst[1] = to16<DT>(hi);
    };

    // ---- A fragments: rows mbase + 32 i + r, k = 16 s + 8 h .. +7 of chunk c
    const int mbase = mt * BM + wm * (BM / 2);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(a.w), (short)0, 0x7ffffff0, 0x00020000);
    const int wph = (int)a.pt.wofs[ph];   // 16-bit elements
    u16x8 aset[3][MT][2];   // A fragments of chunks c, c+1, c+2 (two chunks of weight loads in flight)
    auto loadA = [&](int c, u16x8 (&dst)[MT][2]) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int e = wph + (c * a.Mpad + mbase + 32 * i + r) * KC + 16 * s + 8 * h;
                dst[i][s] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(wr, e * 2, 0, 0));
            }
    };

    floatx16 acc[MT][2];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

    float gv[2][16];
    gather(0, gv[0]);
    loadA(0, aset[0]);
    loadA(min(1, nch - 1), aset[1]);
    stage(0, gv[0]);
    __syncthreads();
    gather(min(1, nch - 1), gv[0]);
    // step c (G = c % 2, A = c % 3, compile-time so every register set is named, never copied): chunk
    // c+2's weights and gather are issued, chunk c is multiplied, chunk c+1's gather (issued one step
    // earlier, in gv[G]) is staged; weights are consumed two steps after their loads, gathers one
    auto step = [&](int c, auto Gc, auto Ac) {
        constexpr int G = decltype(Gc)::value, A = decltype(Ac)::value;
        const int buf = c & 1;
        // unconditional (clamped past the end: a harmless re-load), so that every step issues the same
        // loads and the waitcnt pass can count them exactly across the unrolled steps
        const int c2 = min(c + 2, nch - 1);
        loadA(c2, aset[(A + 2) % 3]);
        gather(c2, gv[G ^ 1]);
        const unsigned short* bs = bt[buf];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            u16x8 bf[2];
#pragma unroll
            for (int j = 0; j < 2; ++j)
                bf[j] = *reinterpret_cast<const u16x8*>(&bs[(wn * 64 + 32 * j + r) * KP + 16 * s + 8 * h]);
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if constexpr ((TCONV_DIAG & 2) != 0)
                        acc[i][j][0] = acc[i][j][0] + (float)(aset[A][i][s][0] ^ bf[j][1]);
                    else
                        acc[i][j] = mma<DT>(aset[A][i][s], bf[j], acc[i][j]);
                }
        }
        stage(buf ^ 1, gv[G]);   // past the end it fills the idle buffer, which nothing reads
        __syncthreads();
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    // exits only right after a step, so the only path into a step is the one through the step before it
    for (int c = 0;; c += 6) {
        step(c, I0{}, I0{});
        if (c + 1 >= nch) break;
        step(c + 1, I1{}, I1{});
        if (c + 2 >= nch) break;
        step(c + 2, I0{}, I2{});
        if (c + 3 >= nch) break;
        step(c + 3, I1{}, I0{});
        if (c + 4 >= nch) break;
        step(c + 4, I0{}, I1{});
        if (c + 5 >= nch) break;
        step(c + 5, I1{}, I2{});
        if (c + 6 >= nch) break;
    }

    // ---- epilogue: bias -> eval-BN -> act (-> act_out), NCHW store
    const EpiArgs& e = a.ep;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int64_t n = n0 + wn * 64 + 32 * j + r;
        if (n >= a.N) continue;
        const int nn = (int)n;
        const int b = a.fd_hw.div(nn);
        const int rr = nn - b * (a.pt.Hq * a.pt.Wq);
        const int qy = a.fd_w.div(rr);
        const int qx = rr - qy * a.pt.Wq;
        const int oy = qy * a.pt.osy + a.pt.ry[ph], ox = qx * a.pt.osy + a.pt.rx[ph];
        const size_t obase = (size_t)b * a.Cout * a.Hout * a.Wout + (size_t)oy * a.Wout + ox;
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int co = mbase + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
                if (co >= a.Cout) continue;
                float v = acc[i][j][q];
                if (e.bias) v = v + e.bias[co];
                if (e.bn_w) {   // as epi_finish (conv.hip)
                    const float invstd = 1.0f / sqrtf(e.bn_v[co] + e.bn_eps);
                    const float alpha = invstd * e.bn_w[co];
                    const float beta = e.bn_b[co] - e.bn_m[co] * alpha;
                    v = v * alpha + beta;
                }
                v = apply_act(v, e.act);
                const size_t o = obase + (size_t)co * a.Hout * a.Wout;
                if (e.act_out) e.act_out[o] = v;
                a.y[o] = v;
            }
    }
}

// packed[p][c][m][e] = w(co = m, tap t = c % ntap, ci = (c / ntap) * 32 + e) in 16 bits, zero past Cout
template <int DT>
__global__ __launch_bounds__(256) void tconv_pack_kernel(const float* __restrict__ w, unsigned short* __restrict__ out,
                                                         PhaseTable pt, int Cin, int Cout, int KK, int transposed,
                                                         int Mpad, int cpt, int64_t total) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    int p = 0;
    for (int q = 1; q < pt.nphase; ++q)
        if (idx >= pt.wofs[q]) p = q;
    const int64_t local = idx - pt.wofs[p];
    const int e = (int)(local % KC);
    const int64_t row = local / KC;
    const int m = (int)(row % Mpad);
    const int c = (int)(row / Mpad);
    const int ntap = pt.ntap[p];
    const int cc = c / ntap, t = c - cc * ntap, ci = cc * KC + e;
    float v = 0.f;
    if (m < Cout) {
        const int kk = pt.kk[p][t];
        v = transposed ? w[((size_t)ci * Cout + m) * KK + kk] : w[((size_t)m * Cin + ci) * KK + kk];
    }
    if constexpr (DT == 1)
        out[idx] = __builtin_bit_cast(unsigned short, (_Float16)v);
    else
        out[idx] = __builtin_bit_cast(unsigned short, (__bf16)v);
}

// geometry of a kind-3 plan: tm = BM / 64, tn = operand precision (LDM_DT_F16 / LDM_DT_BF16)
static int layout(const ldm_conv_desc& d, int bm, PhaseTable& pt, int& Mpad, int64_t& halfs) {
    int rc = build_phase_table(d, pt);
    if (rc) return rc;
    Mpad = (d.Cout + bm - 1) / bm * bm;
    halfs = 0;
    for (int p = 0; p < pt.nphase; ++p) {
        pt.wofs[p] = halfs;
        pt.kchunks[p] = pt.ntap[p] * (d.Cin / KC);
        halfs += (int64_t)pt.kchunks[p] * Mpad * KC;
    }
    return 0;
}

}  // namespace tc

// A kind-3 plan for `d` at operand precision `dtype`; false when the layer is not of this kernel's class
// (16-bit operands, NCHW, Cin % 32 == 0, Cout >= 16, a phase grid of >= 4096 positions, tensors < 2 GiB).
bool tconv_plan(const ldm_conv_desc& d, int dtype, ldm_conv_plan& plan) {
    if (dtype != LDM_DT_F16 && dtype != LDM_DT_BF16) return false;
    if (d.layout != 0 || d.Cin % tc::KC != 0 || d.B <= 0) return false;
    if (d.Cout < 16) return false;   // a 64- / 128-row tile would be > 90 % padding (the decoder's 64 -> 1 convT)
    PhaseTable pt;
    int Mpad;
    int64_t halfs;
    const int bm = d.Cout > 64 ? 128 : 64;
    if (tc::layout(d, bm, pt, Mpad, halfs)) return false;
    const int64_t N = (int64_t)d.B * pt.Hq * pt.Wq;
    if (N < 4096 || N >= (1LL << 31)) return false;
    if ((int64_t)d.B * d.Cin * d.Hin * d.Win * 4 >= 0x7ff00000LL || halfs * 2 >= 0x7ff00000LL) return false;
    plan = ldm_conv_plan{};
    plan.kind = 3;
    plan.tm = bm / 64;
    plan.tn = dtype;
    plan.wk = 1;
    plan.ks = 1;
    plan.packed_floats = (halfs + 1) / 2;
    plan.ws_floats = 0;
    return true;
}

int tconv_pack_job(const ldm_conv_desc& d, const ldm_conv_plan& p, PackJob& j) {
    LDM_REQUIRE(p.kind == 3 && (p.tn == LDM_DT_F16 || p.tn == LDM_DT_BF16), "pack job: not a kind-3 plan");
    PhaseTable pt;
    int Mpad;
    int64_t halfs;
    int rc = tc::layout(d, 64 * p.tm, pt, Mpad, halfs);
    if (rc) return rc;
    j.kind = 3;
    j.dt = p.tn;
    j.Cin = d.Cin;
    j.Cout = d.Cout;
    j.KK = d.kh * d.kw;
    j.transposed = d.transposed;
    j.Mpad = Mpad;
    j.nphase = pt.nphase;
    for (int q = 0; q < kMaxPhase; ++q) {
        j.ntap[q] = pt.ntap[q];
        j.wofs[q] = pt.wofs[q];
        for (int t = 0; t < kMaxTap; ++t) j.kk[q][t] = pt.kk[q][t];
    }
    j.total = halfs;
    return 0;
}

int tconv_pack(const ldm_conv_desc& d, const ldm_conv_plan& p, const float* w, float* packed, hipStream_t st) {
    PhaseTable pt;
    int Mpad;
    int64_t halfs;
    int rc = tc::layout(d, 64 * p.tm, pt, Mpad, halfs);
    if (rc) return rc;
    const unsigned blocks = (unsigned)((halfs + 255) / 256);
    auto* out = reinterpret_cast<unsigned short*>(packed);
    if (p.tn == LDM_DT_F16)
        hipLaunchKernelGGL(tc::tconv_pack_kernel<1>, dim3(blocks), dim3(256), 0, st, w, out, pt, d.Cin, d.Cout,
                           d.kh * d.kw, d.transposed, Mpad, d.Cin / tc::KC, halfs);
    else
        hipLaunchKernelGGL(tc::tconv_pack_kernel<2>, dim3(blocks), dim3(256), 0, st, w, out, pt, d.Cin, d.Cout,
                           d.kh * d.kw, d.transposed, Mpad, d.Cin / tc::KC, halfs);
    LDM_CHECK_LAUNCH("tconv_pack_kernel");
    return 0;
}

int tconv_forward(const ldm_conv_desc& d, const ldm_conv_plan& p, const float* x, const float* w, const EpiArgs& ep,
                  float* y, hipStream_t st) {
    LDM_REQUIRE(p.kind == 3 && (p.tm == 1 || p.tm == 2) && (p.tn == LDM_DT_F16 || p.tn == LDM_DT_BF16),
                "tconv: not a kind-3 plan");
    LDM_REQUIRE(ep.lowp == p.tn, "tconv: the plan's operand precision differs from the call's");
    LDM_REQUIRE(!ep.pos_bias && !ep.bcast && !ep.skip && !ep.ddim_coef && y,
                "tconv: only bias / eval-BN / activation epilogues");
    ldm_conv_plan chk;
    LDM_REQUIRE(tconv_plan(d, p.tn, chk) && chk.tm == p.tm && chk.packed_floats == p.packed_floats,
                "tconv: plan does not match the descriptor");
    tc::TArgs a{};
    int64_t halfs;
    int rc = tc::layout(d, 64 * p.tm, a.pt, a.Mpad, halfs);
    if (rc) return rc;
    a.x = x;
    a.w = reinterpret_cast<const unsigned short*>(w);
    a.y = y;
    a.B = d.B, a.Cin = d.Cin, a.Hin = d.Hin, a.Win = d.Win, a.Cout = d.Cout, a.Hout = d.Hout, a.Wout = d.Wout;
    a.cpt = d.Cin / tc::KC;
    a.N = (int64_t)d.B * a.pt.Hq * a.pt.Wq;
    a.nM = a.Mpad / (64 * p.tm);
    a.nN = (int)((a.N + tc::BN - 1) / tc::BN);
    a.fd_hw = FastDiv::make(a.pt.Hq * a.pt.Wq);
    a.fd_w = FastDiv::make(a.pt.Wq);
    a.ep = ep;
    const int64_t blocks = (int64_t)a.pt.nphase * a.nM * a.nN;
    static const int order = [] {   // LDM_TCONV_XCD=0: plain order (A/B timing)
        const char* e = std::getenv("LDM_TCONV_XCD");
        return e ? std::atoi(e) : 1;
    }();
    a.xcd_chunk = (order && blocks % 8 == 0) ? (int)(blocks / 8) : 0;
    LDM_REQUIRE(blocks < (1LL << 31), "tconv: grid too large");
    hipStream_t s = st;
    if (p.tm == 2) {
        if (p.tn == LDM_DT_F16)
            hipLaunchKernelGGL((tc::tconv_kernel<128, 1>), dim3((unsigned)blocks), dim3(256), 0, s, a);
        else
            hipLaunchKernelGGL((tc::tconv_kernel<128, 2>), dim3((unsigned)blocks), dim3(256), 0, s, a);
    } else {
        if (p.tn == LDM_DT_F16)
            hipLaunchKernelGGL((tc::tconv_kernel<64, 1>), dim3((unsigned)blocks), dim3(256), 0, s, a);
        else
            hipLaunchKernelGGL((tc::tconv_kernel<64, 2>), dim3((unsigned)blocks), dim3(256), 0, s, a);
    }
    LDM_CHECK_LAUNCH("tconv_kernel");
    return 0;
}

}  // namespace ldm

using namespace ldm;

extern "C" int ldm_conv_tiled_plan(const ldm_conv_desc* d, int32_t dtype, ldm_conv_plan* plan) {
    if (!d || !plan) return fail(2, "conv_tiled_plan: null argument");
    return tconv_plan(*d, dtype, *plan) ? 0 : 1;
}
