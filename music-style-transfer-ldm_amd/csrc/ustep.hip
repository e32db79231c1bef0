// LDS-staged step kernels of the reverse loop at the canonical latent (16 x 64, i.e. a 1x128x512 mel), the
// nine UNet convolutions (model.py:178-194, :205-229) of the folded DDIM step.
//
// What limits a conv launch here (measured on MI355X, tools/step_times.py + rocprofv3): the operand loads.
// Every kernel starts with cold L2s, so each load pays Infinity-Cache latency, and a CU keeps only so many
// line requests in flight: a register-direct implicit GEMM (uconv.hip) spends ~7 cycles per 128-B line
// request, and its fragment-shaped activation loads (16 pixels x 64 B per instruction, each tap of the
// 3x3 window fetched again) make 2-9x more requests than the layer has unique bytes.  So here each block
//   * DMAs its weight tile and the unique input window of its output tile into LDS once, in full lines
//     (buffer_load ... lds, 16 B per lane; out-of-image window positions come back as zeros, which is the
//     convolution's padding), in two K stages so stage 1 streams in while stage 0 is being multiplied;
//   * reads every MFMA fragment from LDS (16-B slots XOR-swizzled by row / pixel: conflict-free
//     ds_read_b128 for 16 consecutive rows or pixels; stride-2 windows store even and odd columns apart);
//   * splits K over waves (LDS reduction) and, for the deep layers whose output is only 64K values, over
//     up to four blocks (sc1 slabs + an arrival counter, the last block sums in slot order: deterministic),
//     so that every layer runs as 256 blocks of 4 (bottleneck: 8) waves, 144 MFMAs per wave.
// Geometry is compile-time (latent 16 x 64; batch runtime, a multiple of 4); other shapes use uconv.hip.
// The stride-2 transposed convs run over the input grid with four parity accumulators (see uconv.hip).
// MFMA v_mfma_f32_16x16x4_f32 (exact fp32): lane l = (col l&15, lane group lg = l>>4); MFMA step j of a
// 16-channel chunk uses channel 4*lg + j; D rows 4*lg..4*lg+3 = 4 consecutive output channels.
#include <array>
#include <map>
#include <set>
#include <type_traits>
#include <utility>

#include "common.h"

#pragma clang fp contract(off)

// Diagnostic build only (make DIAG=1 -> lib/libldm_amd_diag.so): no layer runs these kernels by default
// (unet.hip ustep_mask), so the shipped library carries the entry points as stubs that report it.
#if LDM_STEP_DIAG

namespace ldm {
namespace us {

enum : int { EPI_RELU = 1, EPI_BCAST = 2, EPI_SKIP = 4, EPI_POSB = 8, EPI_DDIM = 16 };

struct Cfg {
    int mode, cin, cout, div, bm, bn, ks, kc, wm, wn, wk, nst, epi;
};
constexpr int kH = 16, kW = 64;   // the latent of a 1x128x512 mel spectrogram
constexpr int kOOB = 0x7ffffff0;  // a buffer offset past every range: the DMA lands zeros
// mode 0 conv3x3 s1, 1 conv3x3 s2, 2 convT3x3 s2 p1 op1 (over the input grid).  bm x bn block tile, ks
// blocks splitting K, kc 16-channel chunks per block; wm / wn waves splitting M / N, wk waves splitting K;
// nst K stages (stage s+1 is DMA'd while stage s is multiplied).  Every layer: 256 blocks.
constexpr Cfg kCfg[9] = {
    {0, 32, 64, 1, 32, 64, 1, 2, 1, 4, 1, 2, EPI_RELU},               // enc1
    {1, 64, 128, 1, 32, 32, 1, 4, 2, 2, 1, 4, EPI_RELU | EPI_BCAST},  // enc2 (+ t_emb)
    {1, 128, 256, 2, 32, 32, 2, 4, 2, 2, 1, 4, EPI_RELU},             // enc3
    {1, 256, 512, 4, 16, 64, 4, 4, 1, 4, 1, 4, EPI_RELU | EPI_POSB},  // enc4 (folded CA2 out-proj)
    {0, 512, 512, 8, 16, 64, 4, 8, 1, 4, 2, 4, EPI_RELU | EPI_POSB},  // bottleneck (folded CA1 out-proj)
    {2, 512, 256, 8, 16, 32, 4, 8, 1, 2, 2, 4, EPI_RELU | EPI_SKIP},  // dec4 (+ z3)
    {2, 256, 128, 4, 16, 32, 2, 8, 1, 2, 2, 4, EPI_RELU | EPI_SKIP},  // dec3 (+ z2)
    {2, 128, 64, 2, 16, 32, 1, 8, 1, 2, 2, 4, EPI_RELU | EPI_SKIP},   // dec2 (+ z1)
    {0, 64, 32, 1, 32, 32, 1, 4, 2, 2, 1, 4, EPI_DDIM},               // dec1 (+ DDIM update)
};

template <int L>
struct G {
    static constexpr Cfg c = kCfg[L];
    static constexpr int MODE = c.mode, CIN = c.cin, COUT = c.cout, BM = c.bm, BN = c.bn, KS = c.ks, KC = c.kc;
    static constexpr int WM = c.wm, WN = c.wn, WK = c.wk, EPI = c.epi, NW = WM * WN * WK, NST = c.nst;
    static constexpr int NWL = 4, NT = NW + NWL;      // + loader waves (one per SIMD): they issue every DMA
    static constexpr int Hin = kH / c.div, Win = kW / c.div;
    static constexpr int Hq = MODE == 1 ? Hin / 2 : Hin, Wq = MODE == 1 ? Win / 2 : Win;   // column grid
    static constexpr int Hout = MODE == 2 ? 2 * Hin : Hq, Wout = MODE == 2 ? 2 * Win : Wq;
    static constexpr int NPH = MODE == 2 ? 4 : 1;
    static constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
    // the N tile: BN consecutive columns of the (b, qy, qx) grid = whole rows (possibly whole samples) or a
    // part of one row
    static constexpr bool FULLROW = BN >= Wq;
    static constexpr int R = FULLROW ? BN / Wq : 1;
    static constexpr int SPT = R >= Hq ? R / Hq : 1;   // samples per tile
    static constexpr int RS = R >= Hq ? Hq : R;        // grid rows per sample in the tile
    static constexpr int COLS = FULLROW ? Wq : BN;     // grid columns per tile row
    // input window per sample, borders included (out-of-image positions are DMA'd as zeros)
    static constexpr int WR = MODE == 0 ? RS + 2 : (MODE == 1 ? 2 * RS + 1 : RS + 1);
    static constexpr int WC = MODE == 0 ? COLS + 2 : (MODE == 1 ? 2 * COLS + 1 : COLS + 1);
    static constexpr int WE = (WC + 1) / 2;            // stride 2: even window columns first, then odd
    static constexpr int WPIX = SPT * WR * WC;
    static constexpr int WSLOTS = (WPIX + 15) / 16 * 16;
    static constexpr int KCS = KC / NST;               // channel chunks per stage
    static constexpr int CPW = KCS / WK;               // channel chunks per stage per wave
    static constexpr int NIT = CPW * 9;                // (chunk, tap) steps per stage per wave
    // DMA instructions (1 KB each) per stage: A rows, B window; padded to a multiple of the loader waves
    static constexpr int GA = KCS * 9 * BM / 16, GB = KCS * WSLOTS / 16;
    static constexpr int GS = (GA + GB + NWL - 1) / NWL * NWL, GPL = GS / NWL;
    static constexpr int LDS_A = KC * 9 * BM * 64, LDS_B = KC * WSLOTS * 64, LDS_DUMMY = 1024;
    static constexpr int LDS_RED = NW * NPH * TM * TN * 64 * 16;
    static constexpr int LDS = (LDS_A + LDS_B + LDS_DUMMY) > LDS_RED ? (LDS_A + LDS_B + LDS_DUMMY) : LDS_RED;
    static_assert(KC * KS == CIN / 16 && KC % (NST * WK) == 0, "K split");
    static_assert(COUT % BM == 0 && BM % (16 * WM) == 0 && BN % (16 * WN) == 0 && TM >= 1 && TN >= 1, "tile");
    static_assert(FULLROW ? (R % Hq == 0 || Hq % R == 0) : (Wq % BN == 0), "the tile is whole rows or samples");
    static_assert(LDS <= 160 * 1024, "LDS budget");
    static_assert(NST * GPL <= 63, "a loader wave's DMAs must fit the vmcnt counter");
};

struct Args {
    const float* x;       // NHWC input [B, Hin, Win, CIN]
    const float* w;       // step-packed weights [9*CIN/16][COUT][16] (ldm_step_pack_weight)
    float* y;             // NHWC output
    const float* bias;    // [COUT], or with EPI_POSB [Hout*Wout][COUT]
    const float* bcast;   // [B][COUT]
    const float* skip;    // NHWC like y
    const float* coef;    // EPI_DDIM: [4]
    float* xs;            // EPI_DDIM: sampler state (NHWC)
    float* x0_log;        // EPI_DDIM: NCHW logs or NULL
    float* eps_log;
    float* slab;          // KS > 1: partial tiles [tile][KS][WM*WN][NPH*TM*TN][64] float4
    int32_t* cnt;         // KS > 1: arrival counter per tile (zero between launches)
    float eta;
    int32_t B, nNt;
    int32_t xm, xn, xk;   // the (M tiles, N tiles, K slices) box of blocks one XCD runs (choose_box)
};

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

__device__ __forceinline__ int swz(int slot, int q) { return q ^ ((slot >> 2) & 3); }   // 16-B quarter swizzle

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// Diagnostic builds only (never shipped; tools/step_diag.sh ustep): USTEP_DIAG bit 0 = no MFMAs, bit 1 = no
// DMAs, bit 2 = per-block timestamps of thread 0 (entry / exit in 100 MHz wall ticks, phases in shader
// clocks) into g_ustep_stamps, read back with ldm_debug_ustep_stamps.
// Loader look-ahead: 1 = issue stage s+1, wait for stage s, release it; 2 = keep stages s+1 and s+2 in
// flight while stage s is released (issue s+2 right after the release).
#ifndef USTEP_LA
#define USTEP_LA 2
#endif
#ifndef USTEP_DIAG
#define USTEP_DIAG 0
#endif
#if (USTEP_DIAG & 4)
__device__ unsigned long long g_ustep_stamps[4096][8];
#define USTEP_STAMP(k)                                                                                  \
    do {                                                                                                \
        if (threadIdx.x == 0 && blockIdx.x < 4096)                                                      \
            g_ustep_stamps[blockIdx.x][k] = ((k) == 0 || (k) == 7) ? __builtin_amdgcn_s_memrealtime()   \
                                                                   : __builtin_amdgcn_s_memtime();     \
    } while (0)
#else
#define USTEP_STAMP(k) \
    do {               \
    } while (0)
#endif

template <int L>
__global__ __launch_bounds__(64 * G<L>::NT) __attribute__((amdgpu_waves_per_eu((G<L>::NT + 3) / 4, (G<L>::NT + 3) / 4)))
void ustep_kernel(Args a) {
    using g = G<L>;
    constexpr int MODE = g::MODE, CIN = g::CIN, COUT = g::COUT, BM = g::BM, BN = g::BN, KS = g::KS, KC = g::KC;
    constexpr int WM = g::WM, WN = g::WN, WK = g::WK, NW = g::NW, TM = g::TM, TN = g::TN, NPH = g::NPH, EPI = g::EPI;
    constexpr int WMN = WM * WN, NST = g::NST, NIT = g::NIT;
    constexpr int Hin = g::Hin, Win = g::Win, Hq = g::Hq, Wq = g::Wq, Hout = g::Hout, Wout = g::Wout;
    constexpr int WR = g::WR, WC = g::WC, WE = g::WE, WPIX = g::WPIX, WSLOTS = g::WSLOTS;
    constexpr int KCS = g::KCS, GA = g::GA, GB = g::GB, GPL = g::GPL, NWL = g::NWL;
    constexpr int NFR = NPH * TM * TN, NMY = (NFR + WK - 1) / WK;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    char* const lds = reinterpret_cast<char*>(smem);
    constexpr int OFF_B = g::LDS_A, OFF_D = g::LDS_A + g::LDS_B;

    USTEP_STAMP(0);
    USTEP_STAMP(1);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool loader = wave >= NW;   // waves NW.. only issue DMAs; 0..NW-1 only multiply
    const int wn = wave % WN, wm = (wave / WN) % WM, wk = (wave / WMN) % WK, wmn = wave % WMN;
    const int col = lane & 15, lg = lane >> 4;

    // block -> (M tile, N tile, K slice).  Blocks are dealt to the 8 XCDs round-robin (bid % 8; for speed
    // only, nothing depends on it) and every kernel starts with cold L2s, so the blocks of one XCD get one
    // xm x xn x xk box of the tile grid: what its L2 fetches is xm*xk weight tiles and the union of xn
    // neighbouring input windows (xk channel slices), instead of scattered tiles.
    constexpr int nMt = COUT / BM;
    const int bid = blockIdx.x;
    const int per_xcd = uni((int)gridDim.x >> 3);
    const int lidx = (bid & 7) * per_xcd + (bid >> 3);
    const int xm = uni(a.xm), xn = uni(a.xn), xmn = xm * uni(a.xn), box = xmn * uni(a.xk);
    const int bx = lidx / box, w_in = lidx - bx * box;
    const int nbm = nMt / xm, nbn = uni(a.nNt) / xn;
    const int bxm = bx % nbm, bxn = (bx / nbm) % nbn, bxk = bx / (nbm * nbn);
    const int mt = bxm * xm + w_in % xm;
    const int nt = bxn * xn + (w_in / xm) % xn;
    const int ks = bxk * uni(a.xk) + w_in / xmn;
    const int m0 = mt * BM;
    const int kc0 = ks * KC;

    // tile origin: first sample, first grid row, first grid column
    int b0, qy0, qx0;
    if constexpr (g::FULLROW) {
        if constexpr (g::SPT > 1) {
            b0 = nt * g::SPT, qy0 = 0;
        } else {
            const int row = nt * g::R;
            b0 = row / Hq, qy0 = row % Hq;
        }
        qx0 = 0;
    } else {
        constexpr int TPR = Wq / BN;   // tiles per grid row
        const int row = nt / TPR;
        b0 = row / Hq, qy0 = row % Hq;
        qx0 = (nt % TPR) * BN;
    }
    // window origin in input coordinates
    const int row0 = MODE == 0 ? qy0 - 1 : (MODE == 1 ? 2 * qy0 - 1 : qy0);
    const int col0 = MODE == 0 ? qx0 - 1 : (MODE == 1 ? 2 * qx0 - 1 : qx0);

    // ---- DMA both stages of the block's A tile and input window into LDS (16 B per lane, full lines) -----
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc(uni_ptr(a.w), (short)0, 9 * CIN * COUT * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(uni_ptr(a.x), (short)0, uni(a.B * Hin * Win * CIN * 4), 0x00020000);

    // DMA instruction k (of GPL) of loader wave lw for stage st
    auto dma_one = [&](int st, int lw, auto kc_) {
        if constexpr ((USTEP_DIAG & 2) != 0) return;
        constexpr int k = decltype(kc_)::value;
        const int gi = k * NWL + lw;   // wave-uniform
        if (gi < GA) {
            constexpr int RB = BM / 16;
            const int cl = gi / RB, rb = gi - cl * RB;
            const int c = st * KCS * 9 + cl;                       // (chunk, tap) row block within the block
            const int row = rb * 16 + (lane >> 2);
            const int q = swz(row, lane & 3);
            const int voff = (((kc0 * 9 + c) * COUT + m0 + row) * 16 + q * 4) * 4;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_ptr_t)(lds + (c * BM + rb * 16) * 64), 16, voff, 0, 0, 0);
        } else if (gi < GA + GB) {
            constexpr int NGR = WSLOTS / 16;
            const int gb = gi - GA;
            const int kcl = gb / NGR, grp = gb - kcl * NGR;
            const int kc = st * KCS + kcl;
            const int p = grp * 16 + (lane >> 2);
            const int q = swz(p, lane & 3);
            const int s = p / (WR * WC), r2 = p - s * (WR * WC);
            const int wrr = r2 / WC, pc = r2 - wrr * WC;
            const int wc = MODE == 1 ? (pc < WE ? 2 * pc : 2 * (pc - WE) + 1) : pc;
            const int iy = row0 + wrr, ix = col0 + wc, b = b0 + s;
            const bool ok = p < WPIX && (unsigned)iy < (unsigned)Hin && (unsigned)ix < (unsigned)Win;
            const int voff = ok ? (((b * Hin + iy) * Win + ix) * CIN + (kc0 + kc) * 16 + q * 4) * 4 : kOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_ptr_t)(lds + OFF_B + (kc * WSLOTS + grp * 16) * 64), 16,
                                                     voff, 0, 0, 0);
        } else {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_ptr_t)(lds + OFF_D), 16, kOOB, 0, 0, 0);
        }
    };

    // ---- per-lane column geometry and the LDS slot of every tap ---------------------------------------
    int cb[TN], cqy[TN], cqx[TN], slot[9][TN];
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
        const int j = wn * (TN * 16) + ni * 16 + col;   // column within the tile
        int s, r, c;
        if constexpr (g::FULLROW) {
            s = j / (g::RS * Wq);
            r = (j / Wq) % g::RS;
            c = j % Wq;
        } else {
            s = 0, r = 0, c = j;
        }
        cb[ni] = b0 + s;
        cqy[ni] = qy0 + r;
        cqx[ni] = qx0 + c;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int ky = t / 3, kx = t % 3;
            const int wrr = MODE == 0 ? r + ky : (MODE == 1 ? 2 * r + ky : r + (ky == 0 ? 1 : 0));
            const int wc = MODE == 0 ? c + kx : (MODE == 1 ? 2 * c + kx : c + (kx == 0 ? 1 : 0));
            const int pc = MODE == 1 ? ((wc & 1) ? WE + (wc >> 1) : (wc >> 1)) : wc;
            slot[t][ni] = (s * WR + wrr) * WC + pc;
        }
    }

    // ---- epilogue operands of the fragments this thread finishes (f = k*WK + wk), in flight meanwhile ---
    auto colsel = [&](const int (&arr)[TN], int ni) -> int {
        const int v0 = arr[0], v1 = arr[TN - 1];
        return TN == 1 ? v0 : (v0 ^ ((v0 ^ v1) & -(int)(ni != 0)));
    };
    struct Out {
        int b, oy, ox, pix, m;
        bool ok;
    };
    auto out_of = [&](int f) {
        const int fc = f < NFR ? f : NFR - 1;
        const int p = fc / (TM * TN), mi = (fc / TN) % TM, ni = fc % TN;
        Out o;
        o.b = colsel(cb, ni);
        o.oy = MODE == 2 ? 2 * colsel(cqy, ni) + (p >> 1) : colsel(cqy, ni);
        o.ox = MODE == 2 ? 2 * colsel(cqx, ni) + (p & 1) : colsel(cqx, ni);
        o.pix = (o.b * Hout + o.oy) * Wout + o.ox;
        o.m = m0 + wm * (TM * 16) + 16 * mi + 4 * lg;
        o.ok = f < NFR && !loader;
        return o;
    };
    auto frag = [&](int k) { return WK == 1 ? k : k * WK + wk; };
    floatx4 pre_b[NMY], pre_c[NMY], pre_s[NMY];
    USTEP_STAMP(2);
    if (!loader) static_for<0, NMY>([&](auto kc_) {
        constexpr int k = decltype(kc_)::value;
        const Out o = out_of(frag(k));
        pre_b[k] = (EPI & EPI_POSB) ? *reinterpret_cast<const floatx4*>(a.bias + (size_t)(o.oy * Wout + o.ox) * COUT + o.m)
                                    : *reinterpret_cast<const floatx4*>(a.bias + o.m);
        if constexpr ((EPI & EPI_BCAST) != 0) pre_c[k] = *reinterpret_cast<const floatx4*>(a.bcast + (size_t)o.b * COUT + o.m);
        if constexpr ((EPI & EPI_SKIP) != 0) pre_s[k] = *reinterpret_cast<const floatx4*>(a.skip + (size_t)o.pix * COUT + o.m);
        if constexpr ((EPI & EPI_DDIM) != 0) pre_s[k] = *reinterpret_cast<const floatx4*>(a.xs + (size_t)o.pix * COUT + o.m);
    });
    USTEP_STAMP(3);

    // ---- MFMAs from LDS ---------------------------------------------------------------------------------
    floatx4 acc[NPH][TM][TN];
#pragma unroll
    for (int p = 0; p < NPH; ++p)
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) acc[p][mi][ni] = floatx4{0.f, 0.f, 0.f, 0.f};
    int aoff[TM];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
        const int row = wm * (TM * 16) + mi * 16 + col;
        aoff[mi] = row * 64 + swz(row, lg) * 16;
    }
    int boff[9][TN];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) boff[t][ni] = OFF_B + slot[t][ni] * 64 + swz(slot[t][ni], lg) * 16;

    // fragments of step it (chunk it / 9 of this wave, tap it % 9) of stage st
    auto load_frag = [&](int st, int it, floatx4 (&fa)[TM], floatx4 (&fb)[TN]) {
        const int u = it / 9, t = it - u * 9;
        const int kc = st * KCS + u * WK + wk;     // this wave's channel chunk (wave-uniform)
        const int c = kc * 9 + t;
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) fa[mi] = *reinterpret_cast<const floatx4*>(lds + c * (BM * 64) + aoff[mi]);
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) fb[ni] = *reinterpret_cast<const floatx4*>(lds + kc * (WSLOTS * 64) + boff[t][ni]);
    };
    // The loader waves keep two stages of DMAs in flight and release stage s to the multiplying waves
    // (barrier s) once their own DMAs of it landed (nothing is overwritten: every stage stays resident).
    if (loader) {
        const int lw = wave - NW;
        auto issue = [&](auto sc) { static_for<0, GPL>([&](auto kc_) { dma_one(decltype(sc)::value, lw, kc_); }); };
        issue(std::integral_constant<int, 0>{});
        if constexpr (USTEP_LA == 2 && NST > 1) issue(std::integral_constant<int, 1>{});
        static_for<0, NST>([&](auto sc) {
            constexpr int st = decltype(sc)::value;
            if constexpr (USTEP_LA == 1 && st + 1 < NST) issue(std::integral_constant<int, st + 1>{});
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(st + 1 < NST ? GPL : 0) : "memory");
            __builtin_amdgcn_s_barrier();
            if constexpr (USTEP_LA == 2 && st + 2 < NST) issue(std::integral_constant<int, st + 2>{});
        });
    } else {
        static_for<0, NST>([&](auto sc) {
            constexpr int st = decltype(sc)::value;
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if constexpr (st == 0) USTEP_STAMP(4);
            floatx4 fa[2][TM], fb[2][TN];
            load_frag(st, 0, fa[0], fb[0]);
            static_for<0, NIT>([&](auto ic) {
                constexpr int it = decltype(ic)::value, cur = it & 1;
                constexpr int t = it % 9;
                constexpr int p = MODE == 2 ? ((t / 3 != 1 ? 2 : 0) + (t % 3 != 1 ? 1 : 0)) : 0;
                if constexpr (it + 1 < NIT) load_frag(st, it + 1, fa[cur ^ 1], fb[cur ^ 1]);
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                        for (int ni = 0; ni < TN; ++ni) {
                            if constexpr ((USTEP_DIAG & 1) != 0) {   // diagnostic: no MFMAs (operands kept live)
                                if (j == 0) acc[p][mi][ni][0] = acc[p][mi][ni][0] + fa[cur][mi][j] * fb[cur][ni][j];
                            } else {
                                acc[p][mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[cur][mi][j], fb[cur][ni][j],
                                                                                      acc[p][mi][ni], 0, 0, 0);
                            }
                        }
            });
        });
    }
    USTEP_STAMP(5);

    // ---- K reduction: waves (LDS), then blocks (sc1 slabs, last arriver) ------------------------------
    floatx4* red = reinterpret_cast<floatx4*>(smem);
    floatx4 v[NMY];
    if constexpr (WK > 1) {
        __syncthreads();   // every wave is done reading the staged operands
        static_for<0, NFR>([&](auto fc) {
            constexpr int f = decltype(fc)::value;
            constexpr int p = f / (TM * TN), mi = (f / TN) % TM, ni = f % TN;
            if (!loader) red[((wk * WMN + wmn) * NFR + f) * 64 + lane] = acc[p][mi][ni];
        });
        __syncthreads();
        static_for<0, NMY>([&](auto kc_) {
            constexpr int k = decltype(kc_)::value;
            const int f = frag(k);
            const int fc = f < NFR ? f : NFR - 1;
            floatx4 sum = red[wmn * NFR * 64 + fc * 64 + lane];
#pragma unroll
            for (int k2 = 1; k2 < WK; ++k2) sum = sum + red[((k2 * WMN + wmn) * NFR + fc) * 64 + lane];
            v[k] = sum;
        });
    } else {
        static_for<0, NMY>([&](auto kc_) {
            constexpr int k = decltype(kc_)::value;
            constexpr int p = k / (TM * TN), mi = (k / TN) % TM, ni = k % TN;
            v[k] = acc[p][mi][ni];
        });
    }
    if constexpr (KS > 1) {
        const int tile = nt * nMt + mt;
        const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(uni_ptr(a.slab), (short)0, 0x7fffffff, 0x00020000);
        auto slab_off = [&](int kk, int f) { return ((((tile * KS + kk) * WMN + wmn) * NFR + f) * 64 + lane) * 16; };
        static_for<0, NMY>([&](auto kc_) {
            constexpr int k = decltype(kc_)::value;
            const int f = frag(k);
            if (f < NFR && !loader)   // write-through (sc1) partial tile
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v[k]), sr,
                                                       slab_off(ks, f), 0, 16);
        });
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int* flag = reinterpret_cast<int*>(lds + OFF_D);
        if (threadIdx.x == 0) {
            const int old = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = old == KS - 1;
            if (last) __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *flag = last;
        }
        __syncthreads();
        if (!*flag) {
            USTEP_STAMP(6);
            USTEP_STAMP(7);
            return;
        }
        // the last block: every partial in split order (sc1 loads; its own from registers)
        static_for<0, NMY>([&](auto kc_) {
            constexpr int k = decltype(kc_)::value;
            const int f = frag(k);
            const int fc = f < NFR ? f : NFR - 1;
            floatx4 part[KS];
#pragma unroll
            for (int kk = 0; kk < KS; ++kk)
                part[kk] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(sr, slab_off(kk, fc), 0, 16));
            floatx4 sum = ks == 0 ? v[k] : part[0];
#pragma unroll
            for (int kk = 1; kk < KS; ++kk) sum = sum + (kk == ks ? v[k] : part[kk]);
            v[k] = sum;
        });
    }

    USTEP_STAMP(6);
    // ---- fused epilogue (reference op order: +bias -> ReLU -> +t_emb / +skip; or the DDIM update) -------
    static_for<0, NMY>([&](auto kc_) {
        constexpr int k = decltype(kc_)::value;
        const Out ot = out_of(frag(k));
        if (!ot.ok) return;
        floatx4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float sv = v[k][r] + pre_b[k][r];
            if (EPI & EPI_RELU) sv = sv < 0.f ? 0.f : sv;
            o[r] = sv;
        }
        if constexpr ((EPI & EPI_BCAST) != 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = o[r] + pre_c[k][r];
        }
        if constexpr ((EPI & EPI_SKIP) != 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = o[r] + pre_s[k][r];
        }
        if constexpr ((EPI & EPI_DDIM) != 0) {
            const floatx4 xv = pre_s[k];
            floatx4 xn;
            constexpr size_t hw = (size_t)Hout * Wout;
            const size_t lbase = ((size_t)ot.b * COUT + ot.m) * hw + (size_t)ot.oy * Wout + ot.ox;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float x0;
                xn[r] = ddim_update(xv[r], o[r], a.coef, a.eta, x0);
                if (a.x0_log) a.x0_log[lbase + r * hw] = x0;
                if (a.eps_log) a.eps_log[lbase + r * hw] = o[r];
            }
            *reinterpret_cast<floatx4*>(a.xs + (size_t)ot.pix * COUT + ot.m) = xn;
        } else {
            *reinterpret_cast<floatx4*>(a.y + (size_t)ot.pix * COUT + ot.m) = o;
        }
    });
    USTEP_STAMP(7);
}

// Input pixels (with halo) of the windows of n consecutive N tiles starting at tile 0 (host, exact).
template <int L>
int64_t window_union(int n) {
    using g = G<L>;
    const int nNt1 = g::Hq * g::Wq / g::BN;   // tiles per sample (or a fraction, SPT > 1)
    std::set<int64_t> px;
    for (int nt = 0; nt < n; ++nt) {
        int b0, qy0, qx0;
        if (g::FULLROW) {
            const int row = nt * g::R;
            b0 = row / g::Hq, qy0 = row % g::Hq, qx0 = 0;
        } else {
            const int row = nt / (g::Wq / g::BN);
            b0 = row / g::Hq, qy0 = row % g::Hq, qx0 = (nt % (g::Wq / g::BN)) * g::BN;
        }
        const int row0 = g::MODE == 0 ? qy0 - 1 : (g::MODE == 1 ? 2 * qy0 - 1 : qy0);
        const int col0 = g::MODE == 0 ? qx0 - 1 : (g::MODE == 1 ? 2 * qx0 - 1 : qx0);
        for (int s = 0; s < g::SPT; ++s)
            for (int r = 0; r < g::WR; ++r)
                for (int c = 0; c < g::WC; ++c) {
                    const int iy = row0 + r, ix = col0 + c;
                    if (iy >= 0 && iy < g::Hin && ix >= 0 && ix < g::Win)
                        px.insert(((int64_t)(b0 + s) * g::Hin + iy) * g::Win + ix);
                }
    }
    (void)nNt1;
    return (int64_t)px.size();
}

// The per-XCD box (xm, xn, xk) of the tile grid with the fewest bytes fetched per XCD: xm*xk weight
// tiles + xk channel slices of the union of xn consecutive windows.  Cached per batch.
template <int L>
std::array<int, 3> choose_box(int B) {
    using g = G<L>;
    static std::map<int, std::array<int, 3>> cache;
    auto it = cache.find(B);
    if (it != cache.end()) return it->second;
    const int nMt = g::COUT / g::BM, nNt = B * g::Hq * g::Wq / g::BN;
    const int per_xcd = nMt * nNt * g::KS / 8;
    const int64_t a_tile = (int64_t)g::KC * 9 * g::BM * 64;
    std::array<int, 3> best{1, 1, per_xcd};
    int64_t best_cost = -1;
    for (int xk = 1; xk <= g::KS; ++xk) {
        if (g::KS % xk || per_xcd % xk) continue;
        for (int xm = 1; xm <= nMt; ++xm) {
            if (nMt % xm || (per_xcd / xk) % xm) continue;
            const int xn = per_xcd / xk / xm;
            if (xn < 1 || nNt % xn) continue;
            const int64_t cost = (int64_t)xm * xk * a_tile + (int64_t)xk * g::KC * 64 * window_union<L>(xn);
            if (best_cost < 0 || cost < best_cost) best_cost = cost, best = {xm, xn, xk};
        }
    }
    if (best_cost < 0) best = {0, 0, 0};   // no box tiles this grid (launch refuses)
    cache[B] = best;
    return best;
}

template <int L>
int launch(const Args& a0, hipStream_t st) {
    using g = G<L>;
    Args a = a0;
    a.nNt = a.B * g::Hq * g::Wq / g::BN;
    const int blocks = (g::COUT / g::BM) * a.nNt * g::KS;
    LDM_REQUIRE(blocks % 8 == 0, "ustep: the grid is dealt to 8 XCDs");
    const std::array<int, 3> box = choose_box<L>(a.B);
    LDM_REQUIRE(box[0] * box[1] * box[2] == blocks / 8, "ustep: no XCD box tiles this grid");
    a.xm = box[0], a.xn = box[1], a.xk = box[2];
    auto kfn = ustep_kernel<L>;
    static bool opted = false;
    if (!opted) {
        LDM_HIP_TRY(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, g::LDS));
        opted = true;
    }
    hipLaunchKernelGGL(kfn, dim3((unsigned)blocks), dim3(64 * g::NT), g::LDS, st, a);
    LDM_CHECK_LAUNCH("ustep_kernel");
    return 0;
}

// split-K workspace at batch B: the arrival counters (int32, one per output tile, zero between launches),
// sized for the layer with the most tiles so that layers sharing a workspace never write their slabs over
// another layer's counters, then layer L's partial slabs
template <int L>
int64_t tiles(int B) {
    using g = G<L>;
    return g::KS == 1 ? 0 : (int64_t)(g::COUT / g::BM) * (B * g::Hq * g::Wq / g::BN);
}
inline int64_t cnt_floats(int B) {
    const int64_t t[9] = {tiles<0>(B), tiles<1>(B), tiles<2>(B), tiles<3>(B), tiles<4>(B),
                          tiles<5>(B), tiles<6>(B), tiles<7>(B), tiles<8>(B)};
    int64_t m = 0;
    for (int64_t v : t) m = m > v ? m : v;
    return (m + 63) / 64 * 64;
}
template <int L>
int64_t ws_floats(int B, int64_t* cnt = nullptr) {
    using g = G<L>;
    if (g::KS == 1) return 0;
    const int64_t c = cnt_floats(B);
    if (cnt) *cnt = c;
    return c + tiles<L>(B) * g::KS * g::BM * g::BN * g::NPH;
}

}  // namespace us

bool ustep_supported(int B, int H, int W) { return H == us::kH && W == us::kW && B > 0 && B % 4 == 0; }

int64_t ustep_workspace_floats(int layer, int B, int64_t* cnt_floats) {
    switch (layer) {
        case 0: return us::ws_floats<0>(B, cnt_floats);
        case 1: return us::ws_floats<1>(B, cnt_floats);
        case 2: return us::ws_floats<2>(B, cnt_floats);
        case 3: return us::ws_floats<3>(B, cnt_floats);
        case 4: return us::ws_floats<4>(B, cnt_floats);
        case 5: return us::ws_floats<5>(B, cnt_floats);
        case 6: return us::ws_floats<6>(B, cnt_floats);
        case 7: return us::ws_floats<7>(B, cnt_floats);
        default: return us::ws_floats<8>(B, cnt_floats);
    }
}

int ustep_conv(int layer, int B, const StepConv& s, float* ws, hipStream_t st) {
    LDM_REQUIRE(ustep_supported(B, us::kH, us::kW) && layer >= 0 && layer <= 8, "ustep: unsupported shape / layer");
    us::Args a{};
    a.x = s.x;
    a.w = s.w;
    a.y = s.y;
    a.bias = s.bias;
    a.bcast = s.bcast;
    a.skip = s.skip;
    a.coef = s.coef;
    a.xs = s.xs;
    a.x0_log = s.x0_log;
    a.eps_log = s.eps_log;
    a.eta = s.eta;
    a.B = B;
    int64_t cnt_floats = 0;
    const int64_t wsf = ustep_workspace_floats(layer, B, &cnt_floats);
    if (wsf > 0) {
        LDM_REQUIRE(ws, "ustep: this layer splits K across blocks and needs its (zero-filled) workspace");
        LDM_REQUIRE(wsf * 4 < 0x7fffffffLL, "ustep: split-K workspace beyond 32-bit buffer offsets");
        a.cnt = reinterpret_cast<int32_t*>(ws);
        a.slab = ws + cnt_floats;
    }
    switch (layer) {
        case 0: return us::launch<0>(a, st);
        case 1: LDM_REQUIRE(s.bcast, "enc2: t_emb"); return us::launch<1>(a, st);
        case 2: return us::launch<2>(a, st);
        case 3: return us::launch<3>(a, st);
        case 4: return us::launch<4>(a, st);
        case 5: LDM_REQUIRE(s.skip, "dec4: skip"); return us::launch<5>(a, st);
        case 6: LDM_REQUIRE(s.skip, "dec3: skip"); return us::launch<6>(a, st);
        case 7: LDM_REQUIRE(s.skip, "dec2: skip"); return us::launch<7>(a, st);
        default: LDM_REQUIRE(s.xs && s.coef, "dec1: sampler state"); return us::launch<8>(a, st);
    }
}

}  // namespace ldm

using namespace ldm;

#if (USTEP_DIAG & 4)
extern "C" int ldm_debug_ustep_stamps(unsigned long long* host, int nblocks) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(us::g_ustep_stamps), sizeof(unsigned long long) * 8 * nblocks, 0,
                                    hipMemcpyDeviceToHost);
}
#endif

extern "C" int64_t ldm_ustep_workspace_floats(int32_t layer, int32_t B) {
    if (layer < 0 || layer > 8 || !ustep_supported(B, us::kH, us::kW)) return -1;
    return ustep_workspace_floats(layer, B);
}

extern "C" int ldm_ustep_conv(int32_t layer, int32_t B, const float* x, const float* packed, const float* bias,
                              const float* bcast, const float* skip, float* y, float* workspace, void* stream) {
    LDM_REQUIRE(x && packed && bias && y, "ldm_ustep_conv: null argument");
    LDM_REQUIRE(layer != 8, "ldm_ustep_conv: dec1 runs fused with the DDIM update (ldm_ddim_sample)");
    StepConv s{};
    s.x = x;
    s.w = packed;
    s.y = y;
    s.bias = bias;
    s.bcast = bcast;
    s.skip = skip;
    return ustep_conv(layer, B, s, workspace, (hipStream_t)stream);
}

#else   // !LDM_STEP_DIAG

namespace ldm {
bool ustep_supported(int, int, int) { return false; }
int64_t ustep_workspace_floats(int, int, int64_t* cnt_floats) {
    if (cnt_floats) *cnt_floats = 0;
    return 0;
}
int ustep_conv(int, int, const StepConv&, float*, hipStream_t) {
    return fail(2, "ustep: the LDS-staged step kernels are in the diagnostic build only (make DIAG=1)");
}
}  // namespace ldm

extern "C" int64_t ldm_ustep_workspace_floats(int32_t, int32_t) { return -1; }

extern "C" int ldm_ustep_conv(int32_t, int32_t, const float*, const float*, const float*, const float*, const float*,
                              float*, float*, void*) {
    return ldm::fail(2, "ldm_ustep_conv: the LDS-staged step kernels are in the diagnostic build only (make DIAG=1)");
}

#endif  // LDM_STEP_DIAG
