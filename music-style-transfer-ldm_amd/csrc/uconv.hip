// Step kernels of the reverse loop: the nine convolutions of UNet.forward (model.py:178-194, :205-229)
// as fixed-structure implicit GEMMs for gfx950, used by ldm_ddim_sample when use_step != 0.
//
// Why a second conv family next to conv.hip: at the sampling batch (B = 8 on a 16x64 latent) every layer
// is a 0.3-0.6 GFLOP GEMM whose output is only 64K-512K values, so a launch is ~256 blocks that each own
// one output tile and split K over their waves.  conv.hip's general kernel (runtime tap tables, phase
// tables, K cursors, split-K hand-off) spends most of such a launch on dependent operand rounds and
// address arithmetic.  Here the channel counts, the tap structure and the per-wave K range are template
// constants, so:
//   * the K order is channel-chunk major, tap minor (chunk c = cc*9 + tap): a wave's chunk range is a
//     whole number of channel chunks times the 9 taps, every chunk's tap is a compile-time constant, and
//     the per-lane input offset of each tap is computed once — the K loop is loads + MFMAs only;
//   * every operand load of a stage is issued before the first MFMA of that stage (one memory round trip
//     per stage; most layers are a single stage, so the whole K range is in flight at once);
//   * activations are NHWC: a lane's 4 channels of a 16-channel chunk are one 16-byte load, and the
//     16x16 accumulator rows of a lane (4 consecutive output channels) are one 16-byte store.
// The stride-2 transposed convolutions (dec4..dec2) run over the INPUT grid with 4 accumulator sets, one
// per output parity: tap (ky, kx) of ConvTranspose2d(k3, s2, p1, op1) reads input (qy + [ky==0],
// qx + [kx==0]) and feeds output (2qy + [ky!=1], 2qx + [kx!=1]) — every block carries the same 9-tap K,
// so the four parities need no separate (unequal) launches.
//
// MFMA: v_mfma_f32_16x16x4_f32 (exact fp32, = an fmaf chain, cdna_hip_programming.md §3).  Lane l holds
// A[row = l & 15][k] and B[k][col = l & 15] for its lane group lg = l >> 4; within a 16-channel chunk,
// MFMA step j uses k-local channel 4*lg + j.  D: row 4*lg + r, col l & 15.
// Summation order differs from torch's (K blocked over waves, fixed order), well inside 1e-4.
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "common.h"

#pragma clang fp contract(off)

#define UC_TRY(expr)             \
    do {                         \
        int _rc = (expr);        \
        if (_rc) return _rc;     \
    } while (0)

namespace ldm {
namespace uc {

enum : int { EPI_RELU = 1, EPI_BCAST = 2, EPI_SKIP = 4, EPI_POSB = 8, EPI_DDIM = 16, EPI_PLANE = 32, EPI_WINDOW = 64 };
// EPI_PLANE (a geometry flag carried with the epilogue bits): the layer's plane is 2 x 8 (the bottleneck at the
// canonical 16 x 64 latent), so the 16 columns of a lane group are one sample's whole plane and every tap of a
// stride-1 3x3 conv reads a position some lane of the group already holds.  Each channel chunk's activation
// fragment is loaded once (the centre tap), parked in the wave's own LDS window, and the other eight taps are
// read back shifted by 8 dy + dx positions (zero outside the plane): 1 global load per channel chunk instead of
// 9.  The stride-2 layer onto that plane (enc4, input 4 x 16) parks each sample's whole input plane instead:
// 4 loads instead of 9.  Needs MODE 0 / 1, a single stage, whole channel chunks per stage.
// EPI_WINDOW (likewise a geometry flag): a layer whose wave covers 16 TN consecutive columns of ONE row of its
// column grid (Wq a multiple of the block's columns): the wave loads the input rows and columns those columns'
// taps read (stride 1: 3 x (16 TN + 2); stride 2: 3 x (32 TN + 1); transposed: 2 x (16 TN + 1); halo and
// padding included, zeros outside the image) once per channel chunk, parks them in LDS and reads every tap from
// there: ceil(positions / 16) global loads per channel chunk instead of 9 TN (4 TN transposed).

struct UArgs {
    const float* x;       // NHWC [B, Hin, Win, CIN]
    const float* w;       // packed [9*CIN/16][COUT][16]
    float* y;             // NHWC [B, Hout, Wout, COUT] (unused with EPI_DDIM)
    const float* bias;    // [COUT], or with EPI_POSB [Hout*Wout][COUT]
    const float* bcast;   // [B][COUT]
    const float* skip;    // NHWC like y
    const float* coef;    // EPI_DDIM: [4] {sqrt(ab_t), sqrt(1-ab_t), sqrt(ab_n), sqrt(1-ab_n)}
    float* xs;            // EPI_DDIM: sampler state x, NHWC, updated in place
    float* x0_log;        // EPI_DDIM: pred_x0 log, NCHW [B, COUT, Hout, Wout] (or NULL)
    float* eps_log;       // EPI_DDIM: noise_pred log, NCHW (or NULL)
    float eta;
    int32_t B, Hin, Win, Hout, Wout;
    int32_t Hq, Wq, Nq;   // column grid: output pixels (conv) or input pixels (transposed)
    int32_t nMt, nNt, order;
    int32_t xpm, xpn;     // order 2: the 8 XCDs as an xpm x xpn grid over (M tiles, N tiles), contiguous slices
    FastDiv fd_hw, fd_w, fd_mt, fd_nt, fd_tiles;
    float* slab;          // KS > 1: partial tiles [tile][KS][NFR][64] float4 (write-through)
    int32_t* cnt;         // KS > 1: arrival counter per tile (zero between launches)
};

// (ky, kx) of tap t and the conv input offset / the transposed conv's output parity
__host__ __device__ constexpr int tky(int t) { return t / 3; }
__host__ __device__ constexpr int tkx(int t) { return t % 3; }
__host__ __device__ constexpr int tphase(int t) { return (tky(t) != 1 ? 2 : 0) + (tkx(t) != 1 ? 1 : 0); }
// The transposed layers read only four distinct input offsets over their nine taps (tap (ky, kx) reads input
// (qy + [ky == 0], qx + [kx == 0])): the activation fragment of a tap is loaded once per (channel chunk,
// offset) within a stage and reused by the other taps with that offset.  B_SRC<MODE, S>(i): the chunk of the
// stage whose fragment chunk i uses (i itself when it loads).
__host__ __device__ constexpr int toff(int t) { return (tky(t) == 0 ? 2 : 0) + (tkx(t) == 0 ? 1 : 0); }
template <int MODE>
__host__ __device__ constexpr int b_src(int st, int S, int i) {
    if (MODE != 2) return i;
    const int c = st * S + i;
    for (int j = 0; j < i; ++j) {
        const int cj = st * S + j;
        if (cj / 9 == c / 9 && toff(cj % 9) == toff(c % 9)) return j;
    }
    return i;
}

// Diagnostic builds only (never shipped; tools/step_diag.sh): UCONV_DIAG bit 0 = no MFMAs, bit 1 = no
// operand loads, bit 2 = per-block timestamps of wave 0 (entry and exit in 100 MHz wall ticks, the
// phases between in shader clocks) into g_uconv_stamps, read back with ldm_debug_uconv_stamps.
#ifndef UCONV_DIAG
#define UCONV_DIAG 0
#endif
// cache policy of the activation (B operand) loads: 0 default; experiment builds set 2 (nt: streamed, so that
// they do not push the layer weights out of the XCD's L2 between iterations)
#ifndef UCONV_XAUX
#define UCONV_XAUX 0
#endif
#if (UCONV_DIAG & 4)
__device__ unsigned long long g_uconv_stamps[4096][5];
#define UCONV_STAMP(k)                                                                                 \
    do {                                                                                               \
        if (threadIdx.x == 0 && blockIdx.x < 4096u)                                                    \
            g_uconv_stamps[blockIdx.x][k] = ((k) == 0 || (k) == 4) ? __builtin_amdgcn_s_memrealtime() \
                                                                   : __builtin_amdgcn_s_memtime();    \
    } while (0)
#else
#define UCONV_STAMP(k) \
    do {               \
    } while (0)
#endif

// compile-time loop: f(integral_constant<int, I>) for I in [B, E)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

template <int MODE, int CIN, int COUT, int TM, int TN, int WN, int WK, int NCH, int S, int EPI, int DT, int KS>
__device__ __forceinline__ void uconv_body(const UArgs& a, int bid_in) {
    constexpr int NPH = MODE == 2 ? 4 : 1;
    constexpr int NST = NCH / S;
    constexpr int CPC = 9;                        // chunks per channel chunk (the 9 taps)
    static_assert(NCH % S == 0 && NCH % CPC == 0, "stage / chunk structure");
    static_assert(CIN % 16 == 0 && COUT % (16 * TM) == 0, "channel tiling");
    static_assert((9 * CIN / 16) == NCH * WK * KS, "the grid's waves cover K exactly once");
    // a lone accumulator chain of 16x16x4 (40-cycle dependent latency, 32-cycle issue) alternates two
    constexpr int NACC2 = (NPH * TM * TN == 1) ? 2 : 1;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    UCONV_STAMP(0);

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wn = wave % WN, wk = wave / WN;
    const int col = lane & 15, lg = lane >> 4;

    // block -> (K split ks, M tile, N tile).  The KS blocks of one tile are tiles apart, so with a tile count
    // that is a multiple of 8 they share an XCD (round-robin placement): the last one reads the others'
    // partials from its own L2.
    int mt, nt, ks = 0;
    {
        int bid = bid_in;
        if constexpr (KS > 1) {
            ks = a.fd_tiles.div(bid);
            bid -= ks * (a.nMt * a.nNt);
        }
        if (a.order == 2) {
            // XCD-aware: tile T goes to XCD T % 8 (round-robin placement); XCD x = (xm, xn) owns the contiguous
            // M-tile slice xm and N-tile slice xn, so it fetches 1/xpm of the weights and 1/xpn of the input
            // (and the input rows a slice shares with its neighbour once)
            const int x = bid & 7, l = bid >> 3;
            const int xm = x / a.xpn, xn = x - xm * a.xpn;
            const int mloc = a.nMt / a.xpm, nloc = a.nNt / a.xpn;
            const int ln = l / mloc;
            mt = xm * mloc + (l - ln * mloc);
            nt = xn * nloc + ln;
        } else {
            const int q1 = a.fd_mt.div(bid), q2 = a.fd_nt.div(bid);
            mt = a.order == 0 ? bid - q1 * a.nMt : q2;
            nt = a.order == 0 ? q1 : bid - q2 * a.nNt;
        }
    }
    const int m0 = mt * (16 * TM);
    const int nbase = nt * (16 * TN * WN) + wn * (16 * TN);

    // per column: (b, qy, qx) and the per-tap input byte offsets (kOOB: padding / outside the image)
    constexpr int kOOB = 0x7ffffff0;
    int vt[9][TN];
    int cb[TN], cqy[TN], cqx[TN];
    bool cval[TN];
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
        const int n = nbase + 16 * ni + col;
        const bool nv = n < a.Nq;
        const int nn = nv ? n : 0;
        const int b = a.fd_hw.div(nn);
        const int r = nn - b * (a.Hq * a.Wq);
        const int qy = a.fd_w.div(r);
        const int qx = r - qy * a.Wq;
        cb[ni] = b;
        cqy[ni] = qy;
        cqx[ni] = qx;
        cval[ni] = nv;
        const int iy0 = MODE == 0 ? qy - 1 : (MODE == 1 ? 2 * qy - 1 : qy);
        const int ix0 = MODE == 0 ? qx - 1 : (MODE == 1 ? 2 * qx - 1 : qx);
        const int base = ((b * a.Hin + iy0) * a.Win + ix0) * (CIN * 4) + lg * 16;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int ky = tky(t), kx = tkx(t);
            const int dy = MODE == 2 ? (ky == 0 ? 1 : 0) : ky;
            const int dx = MODE == 2 ? (kx == 0 ? 1 : 0) : kx;
            const bool ok = nv && (unsigned)(iy0 + dy) < (unsigned)a.Hin && (unsigned)(ix0 + dx) < (unsigned)a.Win;
            vt[t][ni] = ok ? base + (dy * a.Win + dx) * (CIN * 4) : kOOB;
        }
    }

    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(a.x), (short)0, uni(a.B * a.Hin * a.Win * CIN * 4), 0x00020000);
    // 16-bit operands read 16-bit packed weights (ldm_step_pack_weight_dt): half the A bytes of the fp32 pack,
    // which matters because a block's operand stream through its CU's L1 is what bounds these launches
    constexpr int AE = DT != 0 ? 2 : 4;                        // bytes per packed weight element
    using AT = std::conditional_t<DT != 0, shortx4, floatx4>;
    constexpr int WBYTES = 9 * CIN * COUT * AE;
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc(uni_ptr(a.w), (short)0, WBYTES, 0x00020000);
    const int va = ((m0 + col) * 16 + lg * 4) * AE;            // A: row m0+col, k-local 4*lg .. +3
    const int kw0 = ks * WK + wk;                              // this wave's slice of K
    const int sa0 = uni(kw0 * NCH * COUT * 16 * AE);           // first chunk of this wave
    const int sb0 = uni(kw0 * (NCH / CPC) * 64);               // its first channel chunk (16 ch x 4 B)

    floatx4 acc[NACC2][NPH][TM][TN];
#pragma unroll
    for (int u = 0; u < NACC2; ++u)
#pragma unroll
        for (int p = 0; p < NPH; ++p)
#pragma unroll
            for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) acc[u][p][mi][ni] = floatx4{0.f, 0.f, 0.f, 0.f};

    constexpr int XAUX = UCONV_XAUX;
    AT fa[NST > 1 ? 2 : 1][S][TM];
    floatx4 fb[NST > 1 ? 2 : 1][S][TN];
    // PART bit 0: weight (A) fragments, bit 1: activation (B) fragments
    auto load_stage = [&](auto stc, auto partc) {
        constexpr int st = decltype(stc)::value;
        constexpr int PART = decltype(partc)::value;
        constexpr int bf = NST > 1 ? (st & 1) : 0;
        static_for<0, S>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            constexpr int c = st * S + i;                 // chunk within this wave's range
            constexpr int t = c % CPC, cc = c / CPC;
            if constexpr ((PART & 1) != 0)
#pragma unroll
            for (int mi = 0; mi < TM; ++mi) {
                const int so = sa0 + (c * COUT * 16 + mi * 256) * AE;
                if constexpr ((UCONV_DIAG & 2) != 0)
                    fa[bf][i][mi] = AT{};
                else if constexpr (DT != 0)
                    fa[bf][i][mi] = __builtin_bit_cast(shortx4, __builtin_amdgcn_raw_buffer_load_b64(wr, va, so, 0));
                else
                    fa[bf][i][mi] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(wr, va, so, 0));
            }
            if constexpr ((PART & 2) != 0 && b_src<MODE>(st, S, i) == i)
#pragma unroll
            for (int ni = 0; ni < TN; ++ni)
                fb[bf][i][ni] = (UCONV_DIAG & 2) ? floatx4{(float)vt[t][ni], 1.f, 2.f, 3.f}
                                                 : __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                                   xr, vt[t][ni], sb0 + cc * 64, XAUX));
            __builtin_amdgcn_sched_barrier(0);        // chunks issue in consumption order
        });
    };
    auto compute_stage = [&](auto stc) {
        constexpr int st = decltype(stc)::value;
        constexpr int bf = NST > 1 ? (st & 1) : 0;
        static_for<0, S>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            constexpr int c = st * S + i;
            constexpr int p = MODE == 2 ? tphase(c % CPC) : 0;
            constexpr int ib = b_src<MODE>(st, S, i);   // the fragment this chunk's taps share
            if constexpr (DT != 0) {   // fp16 / bf16 operands: the whole 16-channel chunk in one MFMA
                constexpr int u = NACC2 == 2 ? (c & 1) : 0;
#pragma unroll
                for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni)
                        acc[u][p][mi][ni] = mma16_lowp<DT>(fa[bf][i][mi], fb[bf][ib][ni], acc[u][p][mi][ni]);
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                        for (int ni = 0; ni < TN; ++ni) {
                            const int u = NACC2 == 2 ? (j & 1) : 0;
                            if constexpr ((UCONV_DIAG & 1) != 0) {   // diagnostic: no MFMAs (operands kept live)
                                if (j == 0)
                                    acc[u][p][mi][ni][0] = acc[u][p][mi][ni][0] + fa[bf][i][mi][j] * fb[bf][ib][ni][j];
                            } else {
                                acc[u][p][mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                                    fa[bf][i][mi][j], fb[bf][ib][ni][j], acc[u][p][mi][ni], 0, 0, 0);
                            }
                        }
            }
        });
    };
    // Epilogue operands of the fragments this thread finishes — fragment f = k*WK + wk for k < NMY (all
    // of them when WK == 1) — loaded right after the last operand stage is issued: they arrive while the
    // MFMAs run and never hold up an operand wait.  Branch-free (a fragment index past NFR is clamped
    // and its result dropped), so the waitcnt pass sees one straight-line load sequence.
    constexpr int NFR = NPH * TM * TN;   // accumulator fragments per wave
    constexpr int NMY = (NFR + WK - 1) / WK;
    static_assert(TN <= 2, "column selects below assume TN <= 2");
    auto frag = [&](int k) { return WK == 1 ? k : k * WK + wk; };
    // (a bitwise blend of two scalars: a ?: over array elements gets folded into a dynamically indexed
    // array, which lives in scratch memory)
    auto colsel = [&](const auto& arr, int ni) -> int {
        const int v0 = (int)arr[0], v1 = (int)arr[TN - 1];
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
        o.pix = (o.b * a.Hout + o.oy) * a.Wout + o.ox;
        o.m = m0 + 16 * mi + 4 * lg;
        o.ok = f < NFR && colsel(cval, ni) != 0;
        return o;
    };
    floatx4 pre_b[NMY], pre_c[NMY], pre_s[NMY];
    auto epi_prefetch = [&]() {
        static_for<0, NMY>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const Out o = out_of(frag(k));
            pre_b[k] = (EPI & EPI_POSB)
                           ? *reinterpret_cast<const floatx4*>(a.bias + (size_t)(o.oy * a.Wout + o.ox) * COUT + o.m)
                           : *reinterpret_cast<const floatx4*>(a.bias + o.m);
            if constexpr ((EPI & EPI_BCAST) != 0) pre_c[k] = *reinterpret_cast<const floatx4*>(a.bcast + (size_t)o.b * COUT + o.m);
            if constexpr ((EPI & EPI_SKIP) != 0) pre_s[k] = *reinterpret_cast<const floatx4*>(a.skip + (size_t)o.pix * COUT + o.m);
            if constexpr ((EPI & EPI_DDIM) != 0) pre_s[k] = *reinterpret_cast<const floatx4*>(a.xs + (size_t)o.pix * COUT + o.m);
        });
    };

    // scheduling fences keep each stage's loads ahead of the MFMAs that consume the previous stage (the
    // default scheduler would interleave them to save registers and expose one latency per chunk); the
    // waitcnt pass then waits progressively, chunk by chunk, in issue order
    UCONV_STAMP(1);
    using AB = std::integral_constant<int, 3>;
    constexpr bool PLANE = (EPI & EPI_PLANE) != 0;
    static_assert(!PLANE || (NST == 1 && S % CPC == 0), "EPI_PLANE geometry");
    if constexpr (PLANE && MODE == 1) {
        // stride 2 onto a 2 x 8 output plane: each sample's whole 4 x 16 input plane (64 positions, 4 loads per
        // lane per channel chunk) goes to the wave's LDS window; tap (ky, kx) of output (qy, qx) reads input
        // (2 qy - 1 + ky, 2 qx - 1 + kx), zero where that is -1 (the top / left padding; the bottom / right
        // never pass the plane)
        constexpr int NCC = S / CPC;
        floatx4 wl[NCC][TN][4];
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
            const int bs = colsel(cb, ni);   // this column set's sample (16 columns = one sample)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int e = k * 64 + lane, pos = e >> 2, g4 = e & 3;
                const int off = colsel(cval, ni) ? ((bs * 4 + (pos >> 4)) * 16 + (pos & 15)) * (CIN * 4) + g4 * 16 : kOOB;
                static_for<0, NCC>([&](auto ccc) {
                    constexpr int cc = decltype(ccc)::value;
                    wl[cc][ni][k] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, sb0 + cc * 64, XAUX));
                });
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        load_stage(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
        epi_prefetch();
        __builtin_amdgcn_sched_barrier(0);
        constexpr int kRedFloats = WK > 1 ? WK * WN * NPH * TM * TN * 64 * 4 : 0;
        float* win = smem + kRedFloats + wave * (NCC * TN * 1024);
        static_for<0, NCC>([&](auto ccc) {
            constexpr int cc = decltype(ccc)::value;
#pragma unroll
            for (int ni = 0; ni < TN; ++ni)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    *reinterpret_cast<floatx4*>(win + (cc * TN + ni) * 1024 + (k * 64 + lane) * 4) = wl[cc][ni][k];
        });
        // the taps read what OTHER lanes of this wave wrote: the compiler, which reasons per lane, may otherwise
        // hoist a read above a write it cannot alias (and the LDS hand back the previous launch's window).  A
        // wave's LDS operations execute in order, so the wave only waits for its own writes: no block barrier.
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int qy = col >> 3, qx = col & 7;
        static_for<0, NCC>([&](auto ccc) {
            constexpr int cc = decltype(ccc)::value;
            static_for<0, CPC>([&](auto tc) {
                constexpr int t = decltype(tc)::value;
                const int iy = 2 * qy - 1 + tky(t), ix = 2 * qx - 1 + tkx(t);
                const bool in = iy >= 0 && ix >= 0;
                const int o = in ? (iy * 16 + ix) * 16 + lg * 4 : 0;
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {
                    const floatx4 v = *reinterpret_cast<const floatx4*>(win + (cc * TN + ni) * 1024 + o);
                    fb[0][cc * CPC + t][ni] = in ? v : floatx4{0.f, 0.f, 0.f, 0.f};
                }
            });
        });
    } else if constexpr (PLANE && MODE == 2) {
        // transposed conv over a 2 x 8 input plane: the four offsets a tap reads, (qy + oy, qx + ox) with oy, ox in
        // {0, 1}, are all in the sample's own plane (zero past its last row / column): one load per channel chunk
        constexpr int NCC = S / CPC;
        static_for<0, NCC>([&](auto ccc) {
            constexpr int cc = decltype(ccc)::value;
#pragma unroll
            for (int ni = 0; ni < TN; ++ni)   // tap 8 = (2, 2) reads offset (0, 0): the lane's own position
                fb[0][cc * CPC + 4][ni] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                          xr, vt[8][ni], sb0 + cc * 64, XAUX));
        });
        __builtin_amdgcn_sched_barrier(0);
        load_stage(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
        epi_prefetch();
        __builtin_amdgcn_sched_barrier(0);
        constexpr int kRedFloats = WK > 1 ? WK * WN * NPH * TM * TN * 64 * 4 : 0;
        float* win = smem + kRedFloats + wave * (NCC * TN * 256);
        const int py = col >> 3, px = col & 7;
        static_for<0, NCC>([&](auto ccc) {
            constexpr int cc = decltype(ccc)::value;
#pragma unroll
            for (int ni = 0; ni < TN; ++ni)
                *reinterpret_cast<floatx4*>(win + ((cc * TN + ni) * 16 + col) * 16 + lg * 4) = fb[0][cc * CPC + 4][ni];
        });
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // cross-lane through LDS: see the stride-2 plane branch
        static_for<0, NCC>([&](auto ccc) {
            constexpr int cc = decltype(ccc)::value;
            static_for<0, CPC>([&](auto tc) {
                constexpr int t = decltype(tc)::value;
                constexpr int i = cc * CPC + t;
                if constexpr (b_src<MODE>(0, S, i) == i) {
                    constexpr int oy = tky(t) == 0 ? 1 : 0, ox = tkx(t) == 0 ? 1 : 0;
                    const bool in = py + oy < 2 && px + ox < 8;
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni) {
                        const floatx4 v =
                            *reinterpret_cast<const floatx4*>(win + ((cc * TN + ni) * 16 + col + 8 * oy + ox) * 16 + lg * 4);
                        fb[0][i][ni] = in ? v : floatx4{0.f, 0.f, 0.f, 0.f};
                    }
                }
            });
        });
    } else if constexpr (PLANE) {
        constexpr int NCC = S / CPC;   // channel chunks of this wave
        // centre taps first (the window waits on them only), then the weight stream, then the epilogue operands
        static_for<0, NCC>([&](auto ccc) {
            constexpr int cc = decltype(ccc)::value;
#pragma unroll
            for (int ni = 0; ni < TN; ++ni)
                fb[0][cc * CPC + 4][ni] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                          xr, vt[4][ni], sb0 + cc * 64, XAUX));
        });
        __builtin_amdgcn_sched_barrier(0);
        load_stage(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
        epi_prefetch();
        __builtin_amdgcn_sched_barrier(0);
        // the wave's window: [cc][ni][16 positions][16 channels] fp32, after the K-reduction buffer
        constexpr int kRedFloats = WK > 1 ? WK * WN * NPH * TM * TN * 64 * 4 : 0;
        float* win = smem + kRedFloats + wave * (NCC * TN * 256);
        const int py = col >> 3, px = col & 7;
        static_for<0, NCC>([&](auto ccc) {
            constexpr int cc = decltype(ccc)::value;
#pragma unroll
            for (int ni = 0; ni < TN; ++ni)
                *reinterpret_cast<floatx4*>(win + ((cc * TN + ni) * 16 + col) * 16 + lg * 4) = fb[0][cc * CPC + 4][ni];
        });
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // cross-lane through LDS: see the stride-2 plane branch
        static_for<0, NCC>([&](auto ccc) {
            constexpr int cc = decltype(ccc)::value;
            static_for<0, CPC>([&](auto tc) {
                constexpr int t = decltype(tc)::value;
                if constexpr (t != 4) {
                    constexpr int dy = tky(t) - 1, dx = tkx(t) - 1;
                    const bool in = (unsigned)(py + dy) < 2u && (unsigned)(px + dx) < 8u;
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni) {
                        const floatx4 v =
                            *reinterpret_cast<const floatx4*>(win + ((cc * TN + ni) * 16 + col + 8 * dy + dx) * 16 + lg * 4);
                        fb[0][cc * CPC + t][ni] = in ? v : floatx4{0.f, 0.f, 0.f, 0.f};
                    }
                }
            });
        });
    } else if constexpr ((EPI & EPI_WINDOW) != 0) {
        static_assert(NST == 1 && S % CPC == 0, "EPI_WINDOW geometry");
        constexpr int NCC = S / CPC;           // channel chunks of this wave
        // the input rows and columns the wave's 16 TN output columns (one row of the column grid) read:
        // stride 1: rows y0-1..y0+1, columns x0-1..x0+16TN; stride 2: rows 2y0-1..2y0+1, columns
        // 2x0-1..2x0+32TN-1; transposed (input grid): rows y0..y0+1, columns x0..x0+16TN
        constexpr int WR = MODE == 2 ? 2 : 3;
        constexpr int WC = MODE == 0 ? 16 * TN + 2 : (MODE == 1 ? 32 * TN + 1 : 16 * TN + 1);
        constexpr int WPOS = WR * WC;          // window positions
        constexpr int NLD = (WPOS * 4 + 63) / 64;   // 16-byte loads per lane per channel chunk
        const int b0 = a.fd_hw.div(nbase);
        const int rem = nbase - b0 * (a.Hq * a.Wq);
        const int y0 = a.fd_w.div(rem);
        const int x0 = rem - y0 * a.Wq;
        const int iy0 = MODE == 0 ? y0 - 1 : (MODE == 1 ? 2 * y0 - 1 : y0);
        const int ix0 = MODE == 0 ? x0 - 1 : (MODE == 1 ? 2 * x0 - 1 : x0);
        floatx4 wl[NCC][NLD];
        int wpos[NLD];
        static_for<0, NLD>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const int e = k * 64 + lane;       // window slot: (position, 4-channel group)
            const int pos = e >> 2, g4 = e & 3;
            const int r = pos / WC, cx = pos - r * WC;
            const int iy = iy0 + r, ix = ix0 + cx;
            const bool ok = e < WPOS * 4 && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win && nbase < a.Nq;
            const int off = ok ? ((b0 * a.Hin + iy) * a.Win + ix) * (CIN * 4) + g4 * 16 : kOOB;
            wpos[k] = e < WPOS * 4 ? pos * 16 + g4 * 4 : -1;
            static_for<0, NCC>([&](auto ccc) {
                constexpr int cc = decltype(ccc)::value;
                wl[cc][k] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, sb0 + cc * 64, XAUX));
            });
        });
        __builtin_amdgcn_sched_barrier(0);
        load_stage(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
        epi_prefetch();
        __builtin_amdgcn_sched_barrier(0);
        constexpr int kRedFloats = WK > 1 ? WK * WN * NPH * TM * TN * 64 * 4 : 0;
        float* win = smem + kRedFloats + wave * (NCC * WPOS * 16);
        static_for<0, NLD>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            static_for<0, NCC>([&](auto ccc) {
                constexpr int cc = decltype(ccc)::value;
                if (wpos[k] >= 0) *reinterpret_cast<floatx4*>(win + cc * WPOS * 16 + wpos[k]) = wl[cc][k];
            });
        });
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // cross-lane through LDS: see the stride-2 plane branch
        static_for<0, NCC>([&](auto ccc) {
            constexpr int cc = decltype(ccc)::value;
            static_for<0, CPC>([&](auto tc) {
                constexpr int t = decltype(tc)::value;
                constexpr int i = cc * CPC + t;
                if constexpr (b_src<MODE>(0, S, i) == i) {   // transposed: one read per distinct offset
                    constexpr int wr = MODE == 2 ? (tky(t) == 0 ? 1 : 0) : tky(t);
                    constexpr int wx = MODE == 2 ? (tkx(t) == 0 ? 1 : 0) : tkx(t);
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni) {
                        const int cx = MODE == 1 ? 2 * (16 * ni + col) + wx : 16 * ni + col + wx;
                        fb[0][i][ni] = *reinterpret_cast<const floatx4*>(win + cc * WPOS * 16 + (wr * WC + cx) * 16 + lg * 4);
                    }
                }
            });
        });
    } else {
        load_stage(std::integral_constant<int, 0>{}, AB{});
        if constexpr (NST == 1) epi_prefetch();
    }
    __builtin_amdgcn_sched_barrier(0);
    static_for<0, NST>([&](auto stc) {
        constexpr int st = decltype(stc)::value;
        if constexpr (st + 1 < NST) {
            load_stage(std::integral_constant<int, st + 1>{}, AB{});
            if constexpr (st + 2 == NST) epi_prefetch();
        }
        __builtin_amdgcn_sched_barrier(0);
        compute_stage(stc);
        __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr (NACC2 == 2) {
#pragma unroll
        for (int p = 0; p < NPH; ++p)
#pragma unroll
            for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) acc[0][p][mi][ni] = acc[0][p][mi][ni] + acc[1][p][mi][ni];
    }

    UCONV_STAMP(2);
    // ---- in-block K reduction (fixed order) and the fused epilogue ------------------------------------
    floatx4* red = reinterpret_cast<floatx4*>(smem);
    if constexpr (WK > 1) {
        static_for<0, NFR>([&](auto fc) {
            constexpr int f = decltype(fc)::value;
            constexpr int p = f / (TM * TN), mi = (f / TN) % TM, ni = f % TN;
            red[((wk * WN + wn) * NFR + f) * 64 + lane] = acc[0][p][mi][ni];
        });
        __syncthreads();
    }
    UCONV_STAMP(3);
    floatx4 vv[NMY];
    static_for<0, NMY>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const int f = frag(k);
        if constexpr (WK > 1) {
            const int fc = f < NFR ? f : NFR - 1;
            floatx4 v = red[((0 * WN + wn) * NFR + fc) * 64 + lane];
#pragma unroll
            for (int k2 = 1; k2 < WK; ++k2) v = v + red[((k2 * WN + wn) * NFR + fc) * 64 + lane];
            vv[k] = v;
        } else {
            constexpr int p = k / (TM * TN), mi = (k / TN) % TM, ni = k % TN;
            vv[k] = acc[0][p][mi][ni];
        }
    });
    if constexpr (KS > 1) {
        // ---- K split over blocks: write-through (sc1) partial tile, arrival counter, the last block of the
        //      tile sums the KS partials in split order (deterministic) and runs the epilogue ---------------
        const int tile = mt + nt * a.nMt;
        const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(uni_ptr(a.slab), (short)0, 0x7fffffff, 0x00020000);
        auto slab_off = [&](int kk, int f) { return ((((tile * KS + kk) * WN + wn) * NFR + f) * 64 + lane) * 16; };
        static_for<0, NMY>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const int f = frag(k);
            if (f < NFR)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, vv[k]),
                                                       sr, slab_off(ks, f), 0, 16);
        });
        // Ordering of the hand-off: the partial tile is stored write-through (sc1) and drained (vmcnt(0)) before
        // the block's barrier, and thread 0 counts the block only after that barrier; the last arriver reads the
        // other partials with sc1 loads after its own barrier, whose workgroup-scope acquire keeps the compiler
        // from hoisting them above the counter.  An agent-scope acq_rel RMW would order the same traffic through
        // the memory model, but on gfx950 it lowers to an L2 write-back + invalidate per block (the plain-store +
        // release form the guide's handoff-flag / publish-large rows price at 2-2.7x the sc1 form).
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int* flag = reinterpret_cast<int*>(smem);
        if (threadIdx.x == 0) {
            const int old = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = old == KS - 1;
            if (last) __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *flag = last;
        }
        __syncthreads();
        if (!*flag) return;
        static_for<0, NMY>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const int f = frag(k);
            const int fc = f < NFR ? f : NFR - 1;
            floatx4 part[KS];
#pragma unroll
            for (int kk = 0; kk < KS; ++kk)
                part[kk] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(sr, slab_off(kk, fc), 0, 16));
            floatx4 sum = ks == 0 ? vv[k] : part[0];
#pragma unroll
            for (int kk = 1; kk < KS; ++kk) sum = sum + (kk == ks ? vv[k] : part[kk]);
            vv[k] = sum;
        });
    }
    static_for<0, NMY>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const int f = frag(k);
        const floatx4 v = vv[k];
        const Out ot = out_of(f);
        if (!ot.ok) return;
        const floatx4 bias = pre_b[k];
        floatx4 o;
        // 16-bit operands (a sampling loop inside torch.autocast): the conv output and each add rounded to that
        // type as well, as the reference's autocast convs return 16-bit tensors; the DDIM update stays fp32
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float sv = round16(v[r] + bias[r], DT);
            if (EPI & EPI_RELU) sv = sv < 0.f ? 0.f : sv;
            o[r] = sv;
        }
        if constexpr ((EPI & EPI_BCAST) != 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = round16(o[r] + pre_c[k][r], DT);
        }
        if constexpr ((EPI & EPI_SKIP) != 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = round16(o[r] + pre_s[k][r], DT);
        }
        if constexpr ((EPI & EPI_DDIM) != 0) {
            // noise_pred = o; the reverse update of model.py:442-458 (ddim_update, one rounding per op)
            const floatx4 xv = pre_s[k];
            floatx4 xn;
            const size_t hw = (size_t)a.Hout * a.Wout;
            const size_t lbase = ((size_t)ot.b * COUT + ot.m) * hw + (size_t)ot.oy * a.Wout + ot.ox;
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
    UCONV_STAMP(4);
}

// The plain step kernel: one layer per launch.
template <int MODE, int CIN, int COUT, int TM, int TN, int WN, int WK, int NCH, int S, int EPI, int DT, int KS = 1>
__global__ __launch_bounds__(64 * WN * WK) __attribute__((amdgpu_waves_per_eu((WN * WK + 3) / 4, (WN * WK + 3) / 4)))
void uconv_kernel(UArgs a) {
    uconv_body<MODE, CIN, COUT, TM, TN, WN, WK, NCH, S, EPI, DT, KS>(a, blockIdx.x);
}

// packed[c][m][16], c = cc*9 + t, element e = 4*lg + j  ->  input channel cc*16 + e, tap t = ky*3 + kx.
// conv: w [COUT][CIN][3][3]; transposed conv: w [CIN][COUT][3][3] (torch layouts).  DT: element type of the
// pack (0 fp32; LDM_DT_F16 / LDM_DT_BF16: rounded once here, to nearest even, as the kernels would round it).
template <int DT>
__global__ __launch_bounds__(256) void uconv_pack_kernel(const float* __restrict__ w, void* __restrict__ outp,
                                                         int CIN, int COUT, int transposed) {
    const int64_t total = (int64_t)9 * CIN * COUT;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int e = (int)(idx % 16);
    const int m = (int)((idx / 16) % COUT);
    const int c = (int)(idx / (16 * (int64_t)COUT));
    const int cc = c / 9, t = c % 9;
    const int ci = cc * 16 + e;
    const float v = transposed ? w[((int64_t)ci * COUT + m) * 9 + t] : w[((int64_t)m * CIN + ci) * 9 + t];
    if constexpr (DT == 0)
        reinterpret_cast<float*>(outp)[idx] = v;
    else if constexpr (DT == LDM_DT_F16)
        reinterpret_cast<_Float16*>(outp)[idx] = (_Float16)v;
    else
        reinterpret_cast<__bf16*>(outp)[idx] = (__bf16)v;
}

// NCHW <-> NHWC for the sampler state (once before / after the loop)
__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(const float* __restrict__ x, float* __restrict__ y, int C,
                                                           int HW, int64_t n) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // over y (NHWC)
    if (idx >= n) return;
    const int c = (int)(idx % C);
    const int64_t r = idx / C;
    const int p = (int)(r % HW);
    const int64_t b = r / HW;
    y[idx] = x[(b * C + c) * HW + p];
}
__global__ __launch_bounds__(256) void nhwc_to_nchw_kernel(const float* __restrict__ x, float* __restrict__ y, int C,
                                                           int HW, int64_t n) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // over y (NCHW)
    if (idx >= n) return;
    const int p = (int)(idx % HW);
    const int64_t r = idx / HW;
    const int c = (int)(r % C);
    const int64_t b = r / C;
    y[idx] = x[(b * HW + p) * C + c];
}

// ------------------------------------------------------------------------------------------------------
// Layer table: the instance each of the nine layers runs (the batch only changes the grid).
// Chosen so that at the sampling batch (B = 8, 16x64 latent) a launch is 256 equal blocks (dec4: 128),
// one wave per SIMD (bottleneck / dec4: two) and 144 MFMAs per wave.
// ------------------------------------------------------------------------------------------------------
struct LayerGeo {
    int mode, cin, cout, tm, tn, wn, wk;
};

template <int MODE, int CIN, int COUT, int TM, int TN, int WN, int WK, int NCH, int S, int EPI, int DT, int KS>
static int launch_dt(const UArgs& a, hipStream_t st) {
    constexpr int NPH = MODE == 2 ? 4 : 1;
    const int blocks = a.nMt * a.nNt * KS;
    size_t lds = std::max<size_t>(WK > 1 ? (size_t)WK * WN * NPH * TM * TN * 64 * 16 : 0, KS > 1 ? 16 : 0);
    if constexpr ((EPI & EPI_PLANE) != 0)   // + each wave's activation window (see EPI_PLANE; 4 KB per sample at stride 2)
        lds = (WK > 1 ? (size_t)WK * WN * NPH * TM * TN * 64 * 16 : 0) + (size_t)WN * WK * (S / 9) * TN * (MODE == 1 ? 4096 : 1024);
    if constexpr ((EPI & EPI_WINDOW) != 0) {   // + each wave's row window (see EPI_WINDOW)
        constexpr int WR = MODE == 2 ? 2 : 3;
        constexpr int WC = MODE == 0 ? 16 * TN + 2 : (MODE == 1 ? 32 * TN + 1 : 16 * TN + 1);
        lds = (WK > 1 ? (size_t)WK * WN * NPH * TM * TN * 64 * 16 : 0) + (size_t)WN * WK * (S / 9) * WR * WC * 64;
    }
    auto kfn = uconv_kernel<MODE, CIN, COUT, TM, TN, WN, WK, NCH, S, EPI, DT, KS>;
    if (lds > 64 * 1024) {   // dynamic LDS past 64 KiB needs the per-function opt-in, once
        static bool opted = false;
        if (!opted) {
            LDM_HIP_TRY(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
            opted = true;
        }
    }
    hipLaunchKernelGGL(kfn, dim3((unsigned)blocks), dim3(64 * WN * WK), lds, st, a);
    LDM_CHECK_LAUNCH("uconv_kernel");
    return 0;
}

// operand precision (StepConv::dtype) -> instance
template <int MODE, int CIN, int COUT, int TM, int TN, int WN, int WK, int NCH, int S, int EPI, int KS = 1>
static int launch(const UArgs& a, int dtype, hipStream_t st) {
    switch (dtype) {
        case LDM_DT_F32: return launch_dt<MODE, CIN, COUT, TM, TN, WN, WK, NCH, S, EPI, 0, KS>(a, st);
        case LDM_DT_F16: return launch_dt<MODE, CIN, COUT, TM, TN, WN, WK, NCH, S, EPI, 1, KS>(a, st);
        case LDM_DT_BF16: return launch_dt<MODE, CIN, COUT, TM, TN, WN, WK, NCH, S, EPI, 2, KS>(a, st);
        default: return fail(2, "step conv: unknown operand precision");
    }
}

// The K-split form of the deep layers (variant 1): a 32 x 32 block tile (2 x 2 MFMA tiles per wave) instead of
// 16 x 16, so a block pulls half the operand bytes per MFMA, with K split over KS blocks to keep 256 blocks
// (write-through partial tiles, last arriver sums in split order).  {tm, tn, wk, ks}; ks 0 = no variant.
struct KsGeo {
    int tm, tn, wk, ks, wn = 1;
};
constexpr KsGeo kKs[9] = {
    {0, 0, 0, 0},   // enc1
    {0, 0, 0, 0},   // enc2
    {2, 2, 4, 2},   // enc3        128 tiles x 2
    {2, 2, 4, 4},   // enc4        64 tiles x 4
    {2, 2, 8, 4},   // bottleneck  64 tiles x 4, 8 waves
    {2, 2, 4, 8},   // dec4        32 tiles x 8
    {2, 2, 4, 4},   // dec3        64 tiles x 4
    {0, 0, 0, 0},   // dec2
    {0, 0, 0, 0},   // dec1
};

// Variant 2 ("thin"): a 16 x 32 block tile with K split over 2-4 blocks of 8 waves: the same weight bytes per
// block as variant 1, a partial tile of a quarter / half the size for the last arriver to gather (its hand-off
// cost grows with KS x the tile).  Selected by bit l of LDM_UCONV_KS2 for a layer also in LDM_UCONV_KS.
constexpr KsGeo kKs2[9] = {
    {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0},
    {1, 2, 8, 2},   // enc4        128 tiles x 2
    {1, 2, 4, 4, 2},   // bottleneck  64 tiles (16 x 64: 2 wave columns) x 4, two channel chunks per wave
    {1, 2, 8, 4},   // dec4        64 tiles x 4
    {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0},
};

// Variant 3 ("wide", round 6): 16 x 16 tiles with one channel chunk per wave and 16 waves per block (4 per SIMD), so a
// block keeps 16 x 9 operand loads in flight across four times the waves: enc4 with K in one block (256 tiles, no
// partial slabs), dec4 with K over 2 blocks (128 tiles; half the slab bytes of variant 2).  Bit l of LDM_UCONV_KS3
// (default 0xED: every layer that has one; it takes precedence over LDM_UCONV_KS / _KS2 for that layer).  Measured
// in the fp32 loop (B = 8, one box each): none 75.28, enc4 73.47-73.68, dec4 74.28-74.37, both 72.21-72.69 us per
// iteration (gpurun_out/r6b7); then on another box from enc4 + dec4 (72.15-72.39): + enc1 71.59-71.74, + enc3
// 71.41-71.71, + dec3 71.44-71.56, + dec2 72.34-72.50, all six 70.12-70.18 (gpurun_out/r6b8); the fp16 loop
// 57.97 -> 56.70-57.06 with enc4 + dec4, unchanged by the other four; + dec1 with its DDIM update 70.30-70.44 ->
// 69.72-69.87, fp16 55.50-55.73 -> 55.19-55.23 (gpurun_out/r6b9).
constexpr KsGeo kKs3[9] = {
    {2, 1, 2, 1, 4},   // enc1        32 x 64 tiles (4 wave columns), K (2 channel chunks) over 2 waves: 8 waves
    {2, 1, 4, 1, 2},   // enc2        32 x 32 tiles (2 wave columns of 16), K over 4 waves: 8 waves
    {2, 1, 8, 1},    // enc3        32 x 16 tiles, K over 8 waves
    {1, 1, 16, 1},   // enc4        256 tiles, K whole
    {0, 0, 0, 0},
    {1, 1, 16, 2},   // dec4        128 tiles x 2
    {1, 1, 16, 1},   // dec3        256 tiles, K over 16 waves
    {1, 2, 8, 1},    // dec2        16 x 32 tiles, K over 8 waves
    {1, 2, 4, 1, 2}, // dec1 + DDIM 16 x 64 tiles (2 wave columns), K over 4 waves: 8 waves
};
constexpr int kKs3Default = 0x1ED;   // enc1, enc3, enc4, dec4, dec3, dec2, dec1 (gpurun_out/r6b7, r6b8, r6b9)
static int ks3_mask() {
    static const int m = [] {
        const char* e = std::getenv("LDM_UCONV_KS3");
        return e ? (int)std::strtol(e, nullptr, 0) : kKs3Default;
    }();
    return m;
}

constexpr LayerGeo kGeo[9] = {
    {0, 32, 64, 2, 1, 4, 1},     // enc1        conv3x3 s1
    {1, 64, 128, 2, 2, 1, 4},    // enc2        conv3x3 s2 (+ t_emb)
    {1, 128, 256, 2, 1, 1, 4},   // enc3        conv3x3 s2
    {1, 256, 512, 1, 1, 1, 4},   // enc4        conv3x3 s2 (folded with CA2's out-projection)
    {0, 512, 512, 1, 1, 1, 8},   // bottleneck  conv3x3 s1 (folded with CA1's out-projection)
    {2, 512, 256, 1, 1, 1, 8},   // dec4        convT k3 s2 (+ skip z3)
    {2, 256, 128, 1, 1, 1, 4},   // dec3        convT (+ skip z2)
    {2, 128, 64, 1, 2, 1, 4},    // dec2        convT (+ skip z1)
    {0, 64, 32, 2, 2, 1, 4},     // dec1        conv3x3 s1 (+ fused DDIM update)
};

}  // namespace uc

// Packed floats of layer `layer`'s step weights (9*Cin*Cout).
int64_t step_packed_floats(int layer) {
    if (layer < 0 || layer > 8) return -1;
    return (int64_t)9 * uc::kGeo[layer].cin * uc::kGeo[layer].cout;
}

namespace uc {
// Layers that run the K-split variant: bit l of LDM_UCONV_KS (read once; default kKsDefault).
// Round 2, in the loop's chain timing (B = 8): the split form gained 0.4 us on the bottleneck and 0.2 us on enc4
// and lost 0.9-1.5 us on enc3, dec4 and dec3.  Round 3, with the taps formed from LDS windows, the loop with
// enc4, the bottleneck and dec4 split (enc4 and dec4 on the thin variant kKs2) measured best (79.7-79.9 us per
// iteration against 84.0 for the round-2 choice, profiles/r03/ks2, profiles/r03/geo).
constexpr int kKsDefault = (1 << 3) | (1 << 4) | (1 << 5);
static int ks_mask() {
    static const int m = [] {
        const char* e = std::getenv("LDM_UCONV_KS");
        return e ? (int)std::strtol(e, nullptr, 0) : kKsDefault;
    }();
    return m;
}
// 16-bit operands (config 5) stream half the weight bytes per block, so the split that pays for fp32 need not pay
// there: their own mask, LDM_UCONV_KS_LOWP (default kKsDefaultLowp, measured in the fp16 loop)
constexpr int kKsDefaultLowp = kKsDefault;
static int ks_mask_lowp() {
    static const int m = [] {
        const char* e = std::getenv("LDM_UCONV_KS_LOWP");
        return e ? (int)std::strtol(e, nullptr, 0) : kKsDefaultLowp;
    }();
    return m;
}
static bool ks_on(int layer, int dtype = LDM_DT_F32) {
    return kKs[layer].ks > 1 && (((dtype == LDM_DT_F32 ? ks_mask() : ks_mask_lowp()) >> layer) & 1);
}
// (the bottleneck's variants measured alike: 16 x 32 KS 2 79.7, 16 x 64 KS 4 80.1, 32 x 32 KS 4 79.9 us per
// iteration, profiles/r03/geo; it keeps variant 1)
constexpr int kKs2Default = (1 << 3) | (1 << 5);
static int ks2_mask() {
    static const int m = [] {
        const char* e = std::getenv("LDM_UCONV_KS2");
        return e ? (int)std::strtol(e, nullptr, 0) : kKs2Default;
    }();
    return m;
}
// K-split form of a layer: 0 none, 1 variant 1 (kKs), 2 variant 2 (kKs2)
static bool plane_taps();
static bool window_taps();
// (variant 3 runs at the canonical 16 x 64 latent only: enc4 / dec4 on its 2 x 8 planes (EPI_PLANE), the others on
// whole rows of their column grids (EPI_WINDOW))
static int ks_form(int layer, int dtype = LDM_DT_F32, int H = 16, int W = 64) {
    if (layer >= 0 && layer <= 8 && kKs3[layer].wk > 0 && ((ks3_mask() >> layer) & 1) && H == 16 && W == 64 &&
        (layer == 3 || layer == 5 ? plane_taps() : window_taps()))
        return 3;
    if (layer < 0 || layer > 8 || !ks_on(layer, dtype)) return 0;
    return (kKs2[layer].ks > 1 && ((ks2_mask() >> layer) & 1)) ? 2 : 1;
}
// dec1 on 16-row x 64-position tiles: half of the 32 output channels per block, so a block streams half of the
// layer's weights (every block streams all of them in the 32-row form): loop 81.2 -> 80.7 us per iteration
// (profiles/r03/dec1_thin); LDM_UCONV_DEC1_THIN=0 keeps the 32-row form
static bool dec1_thin(int W) {
    static const bool on = [] {
        const char* e = std::getenv("LDM_UCONV_DEC1_THIN");
        return e ? std::atoi(e) != 0 : true;
    }();
    return on && W % 32 == 0;
}
// enc2 on 16-row x 64-position tiles (four wave columns sharing each weight fragment through L1): half the weight
// bytes per block of the 32 x 32 form, measured slower in the loop (81.6 vs 80.1 us per iteration,
// profiles/r03/geo); LDM_UCONV_ENC2_WIDE=1 (A/B timing)
static bool enc2_wide(int W) {
    static const bool on = [] {
        const char* e = std::getenv("LDM_UCONV_ENC2_WIDE");
        return e ? std::atoi(e) != 0 : false;
    }();
    return on && (W / 2) % 16 == 0;
}
// enc3 on 16-row tiles (half the weight bytes per block of the 32-row form), each wave one 16-column row of the
// 4 x 16 output plane so that its taps come from a row window.  Measured in the loop: 80.9 against 80.5 us per
// iteration for the 32-row form (profiles/r03/enc3_thin), so off unless LDM_UCONV_ENC3_THIN=1.
static bool enc3_thin(int W) {
    static const bool on = [] {
        const char* e = std::getenv("LDM_UCONV_ENC3_THIN");
        return e ? std::atoi(e) != 0 : false;
    }();
    return on && (W / 4) % 16 == 0;   // enc3's output row (W / 4 columns) holds whole 16-column groups
}
// EPI_WINDOW instances where the geometry allows (LDM_UCONV_WINDOW=0 turns them off for A/B timing)
static bool window_taps() {
    static const bool on = [] {
        const char* e = std::getenv("LDM_UCONV_WINDOW");
        return e ? std::atoi(e) != 0 : true;
    }();
    return on;
}
// XCD-grid block order (order 2 in make_args); LDM_UCONV_XCD=0 turns it off for A/B timing
static bool xcd_grid() {
    static const bool on = [] {
        const char* e = std::getenv("LDM_UCONV_XCD");
        return e ? std::atoi(e) != 0 : true;
    }();
    return on;
}
// EPI_PLANE instances where the geometry allows (LDM_UCONV_PLANE=0 turns them off for A/B timing)
static bool plane_taps() {
    static const bool on = [] {
        const char* e = std::getenv("LDM_UCONV_PLANE");
        return e ? std::atoi(e) != 0 : true;
    }();
    return on;
}
// spatial size divisor of each layer's input (model.py:178-194)
constexpr int kDiv[9] = {1, 1, 2, 4, 8, 8, 4, 2, 1};
static void ks_tiles(int layer, int B, int H, int W, int64_t& tiles, int64_t& slab_floats, int form = 1) {
    const LayerGeo& g = kGeo[layer];
    const KsGeo& k = form == 3 ? kKs3[layer] : (form == 2 ? kKs2[layer] : kKs[layer]);
    const int Hin = H / kDiv[layer], Win = W / kDiv[layer];
    const int64_t nq = (int64_t)B * (g.mode == 1 ? (Hin / 2) * (Win / 2) : Hin * Win);
    tiles = (int64_t)(g.cout / (16 * k.tm)) * ((nq + 16 * k.tn * k.wn - 1) / (16 * k.tn * k.wn));
    slab_floats = tiles * k.ks * (g.mode == 2 ? 4 : 1) * k.tm * k.tn * k.wn * 256;
}
}  // namespace uc

// Split-K workspace of the step kernels at this shape: arrival counters (one int32 per tile, zero between
// launches) sized for the layer with the most tiles, then the largest layer's partial slabs.
// the layers on a K-split form (ldm_step_layer_forms): LDM_UCONV_KS's, with the wide variant's layers counted by its
// own split (enc4's wide form keeps K in one block)
int step_ks_mask() {
    int m = uc::ks_mask();
    for (int l = 0; l < 9; ++l)
        if (uc::kKs3[l].wk > 0 && ((uc::ks3_mask() >> l) & 1)) m = uc::kKs3[l].ks > 1 ? (m | (1 << l)) : (m & ~(1 << l));
    return m;
}

int64_t step_ws_floats(int B, int H, int W, int64_t* cnt_floats) {
    using namespace uc;
    int64_t mt = 0, ms = 0;
    for (int l = 0; l < 9; ++l) {
        for (int form = 1; form <= 3; ++form) {   // every K-split geometry, whatever the masks select
            if ((form == 1 ? kKs[l].ks : (form == 2 ? kKs2[l].ks : kKs3[l].ks)) <= 1) continue;
            int64_t t, sf;
            ks_tiles(l, B, H, W, t, sf, form);
            mt = std::max(mt, t);
            ms = std::max(ms, sf);
        }
    }
    const int64_t c = (mt + 63) / 64 * 64;
    if (cnt_floats) *cnt_floats = c;
    return c + ms;
}

namespace uc {
// The launch arguments of layer `layer` (ksv: the K-split form).
static int make_args(int layer, int B, int H, int W, const StepConv& s, int ksv, UArgs& a) {
    LDM_REQUIRE(layer >= 0 && layer <= 8, "step conv: layer index");
    LDM_REQUIRE(B > 0 && H % 8 == 0 && W % 8 == 0, "step conv: latent H, W must be multiples of 8");
    LayerGeo g = kGeo[layer];
    if (ksv) {
        const KsGeo& k = ksv == 3 ? kKs3[layer] : (ksv == 2 ? kKs2[layer] : kKs[layer]);
        g.tm = k.tm, g.tn = k.tn, g.wn = k.wn, g.wk = k.wk;
    } else if (layer == 8 && dec1_thin(W)) {
        g = LayerGeo{0, 64, 32, 1, 2, 2, 2};   // 16 of the 32 rows x 64 positions (2 wave columns), K over 2 waves
    } else if (layer == 1 && enc2_wide(W)) {
        g = LayerGeo{1, 64, 128, 1, 1, 4, 1};   // 16 rows x 4 wave columns of 16 (64 positions), whole K per wave
    } else if (layer == 2 && enc3_thin(W)) {
        g = LayerGeo{1, 128, 256, 1, 1, 2, 2};   // 16 rows x 2 column groups of one row each, K over 2 waves
    }
    const int Hin = H / kDiv[layer], Win = W / kDiv[layer];
    a = UArgs{};
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
    a.Hin = Hin;
    a.Win = Win;
    if (g.mode == 0) {
        a.Hout = Hin, a.Wout = Win, a.Hq = Hin, a.Wq = Win;
    } else if (g.mode == 1) {
        a.Hout = Hin / 2, a.Wout = Win / 2, a.Hq = a.Hout, a.Wq = a.Wout;
    } else {
        a.Hout = 2 * Hin, a.Wout = 2 * Win, a.Hq = Hin, a.Wq = Win;
    }
    a.Nq = B * a.Hq * a.Wq;
    const int bm = 16 * g.tm, bn = 16 * g.tn * g.wn;
    a.nMt = g.cout / bm;
    a.nNt = (a.Nq + bn - 1) / bn;
    // weight-heavy layers keep one M tile's blocks together (N tile fastest would spread a weight slab
    // over every XCD's L2); activation-heavy ones walk M fastest
    const int64_t wbytes = (int64_t)9 * g.cin * g.cout * 4, xbytes = (int64_t)B * Hin * Win * g.cin * 4;
    a.order = wbytes > xbytes ? 0 : 1;
    // XCD grid (order 2, LDM_UCONV_XCD=0 keeps orders 0 / 1): the split of the 8 XCDs over (M, N) tiles with
    // the fewest bytes fetched into the eight L2s, xpn x weights + xpm x input (each XCD its weight and input
    // slices; contiguous N slices share their halo rows); only where both tile counts divide
    if (xcd_grid() && ((int64_t)a.nMt * a.nNt) % 8 == 0) {
        int64_t best = -1;
        for (int pm = 1; pm <= 8; pm *= 2) {
            const int pn = 8 / pm;
            if (a.nMt % pm || ((a.Nq + bn - 1) / bn) % pn) continue;
            const int64_t est = pn * wbytes + pm * xbytes;
            if (best < 0 || est < best) best = est, a.xpm = pm, a.xpn = pn;
        }
        if (best >= 0) a.order = 2;
    }
    a.fd_hw = FastDiv::make(a.Hq * a.Wq);
    a.fd_w = FastDiv::make(a.Wq);
    a.fd_mt = FastDiv::make(a.nMt);
    a.fd_nt = FastDiv::make(a.nNt);
    a.fd_tiles = FastDiv::make(a.nMt * a.nNt);
    if (ksv && (ksv == 3 ? kKs3[layer] : (ksv == 2 ? kKs2[layer] : kKs[layer])).ks > 1) {
        int64_t cnt = 0;
        const int64_t wsf = step_ws_floats(B, H, W, &cnt);
        int64_t tiles, sf;
        ks_tiles(layer, B, H, W, tiles, sf, ksv);
        LDM_REQUIRE(tiles == (int64_t)a.nMt * a.nNt && wsf >= cnt + sf && (cnt + sf) * 4 < 0x7fffffffLL,
                    "step conv: split-K workspace geometry");
        a.cnt = reinterpret_cast<int32_t*>(s.ws);
        a.slab = s.ws + cnt;
    }
    LDM_REQUIRE((int64_t)B * Hin * Win * g.cin * 4 < 0x7ff00000LL && (int64_t)B * a.Hout * a.Wout * g.cout * 4 < 0x7ff00000LL,
                "step conv: tensor too large for 32-bit buffer offsets");
    LDM_REQUIRE(s.x && s.w && s.bias, "step conv: null operand");
    return 0;
}
}  // namespace uc

int step_conv(int layer, int B, int H, int W, const StepConv& s, hipStream_t st) {
    using namespace uc;
    const int ksv = s.ws ? ks_form(layer, s.dtype, H, W) : 0;   // without a workspace: the single-block form
    UArgs a;
    UC_TRY(make_args(layer, B, H, W, s, ksv, a));
    if (ksv == 3) {
        const bool win = window_taps();
        switch (layer) {
            case 0: LDM_REQUIRE(s.y && win && a.Wq % 64 == 0, "enc1 (variant 3): y, 64-column rows");
                return launch<0, 32, 64, 2, 1, 4, 2, 9, 9, EPI_RELU | EPI_WINDOW, 1>(a, s.dtype, st);
            case 1: LDM_REQUIRE(s.y && s.bcast && win && a.Wq % 32 == 0, "enc2 (variant 3): y, t_emb, 32-column rows");
                return launch<1, 64, 128, 2, 1, 2, 4, 9, 9, EPI_RELU | EPI_BCAST | EPI_WINDOW, 1>(a, s.dtype, st);
            case 2: LDM_REQUIRE(s.y && win && a.Wq % 16 == 0, "enc3 (variant 3): y, 16-column rows");
                return launch<1, 128, 256, 2, 1, 1, 8, 9, 9, EPI_RELU | EPI_WINDOW, 1>(a, s.dtype, st);
            case 6: LDM_REQUIRE(s.y && s.skip && win && a.Wq % 16 == 0, "dec3 (variant 3): y, skip, 16-column rows");
                return launch<2, 256, 128, 1, 1, 1, 16, 9, 9, EPI_RELU | EPI_SKIP | EPI_WINDOW, 1>(a, s.dtype, st);
            case 7: LDM_REQUIRE(s.y && s.skip && win && a.Wq % 32 == 0, "dec2 (variant 3): y, skip, 32-column rows");
                return launch<2, 128, 64, 1, 2, 1, 8, 9, 9, EPI_RELU | EPI_SKIP | EPI_WINDOW, 1>(a, s.dtype, st);
            case 8: LDM_REQUIRE(s.xs && s.coef && win && a.Wq % 64 == 0, "dec1 (variant 3): sampler state, 64-column rows");
                return launch<0, 64, 32, 1, 2, 2, 4, 9, 9, EPI_DDIM | EPI_WINDOW, 1>(a, s.dtype, st);
            case 3: LDM_REQUIRE(s.y && a.Hin == 4 && a.Win == 16 && plane_taps(), "enc4 (variant 3): y, 4 x 16 input plane");
                return launch<1, 256, 512, 1, 1, 1, 16, 9, 9, EPI_RELU | EPI_POSB | EPI_PLANE, 1>(a, s.dtype, st);
            case 5: LDM_REQUIRE(s.y && s.skip && a.Hin == 2 && a.Win == 8 && plane_taps(), "dec4 (variant 3): y, skip, 2 x 8 plane");
                return launch<2, 512, 256, 1, 1, 1, 16, 9, 9, EPI_RELU | EPI_SKIP | EPI_PLANE, 2>(a, s.dtype, st);
            default: return fail(2, "step conv: no K-split variant 3 for this layer");
        }
    }
    if (ksv == 2) {
        const bool pl = plane_taps();
        switch (layer) {
            case 3: LDM_REQUIRE(s.y, "enc4: y");
                if (a.Hin == 4 && a.Win == 16 && pl)
                    return launch<1, 256, 512, 1, 2, 1, 8, 9, 9, EPI_RELU | EPI_POSB | EPI_PLANE, 2>(a, s.dtype, st);
                return launch<1, 256, 512, 1, 2, 1, 8, 9, 9, EPI_RELU | EPI_POSB, 2>(a, s.dtype, st);
            case 4: LDM_REQUIRE(s.y, "bottleneck: y");
                if (a.Hin == 2 && a.Win == 8 && pl)
                    return launch<0, 512, 512, 1, 2, 2, 4, 18, 18, EPI_RELU | EPI_POSB | EPI_PLANE, 4>(a, s.dtype, st);
                return launch<0, 512, 512, 1, 2, 2, 4, 18, 18, EPI_RELU | EPI_POSB, 4>(a, s.dtype, st);
            case 5: LDM_REQUIRE(s.y && s.skip, "dec4: y, skip");
                if (a.Hin == 2 && a.Win == 8 && pl)
                    return launch<2, 512, 256, 1, 2, 1, 8, 9, 9, EPI_RELU | EPI_SKIP | EPI_PLANE, 4>(a, s.dtype, st);
                return launch<2, 512, 256, 1, 2, 1, 8, 9, 9, EPI_RELU | EPI_SKIP, 4>(a, s.dtype, st);
            default: return fail(2, "step conv: no K-split variant 2 for this layer");
        }
    }
    if (ksv) {
        switch (layer) {
            case 2: LDM_REQUIRE(s.y, "enc3: y"); return launch<1, 128, 256, 2, 2, 1, 4, 9, 9, EPI_RELU, 2>(a, s.dtype, st);
            case 3: LDM_REQUIRE(s.y, "enc4: y");
                if (a.Hin == 4 && a.Win == 16 && plane_taps())   // the canonical latent: a 2 x 8 output plane
                    return launch<1, 256, 512, 2, 2, 1, 4, 9, 9, EPI_RELU | EPI_POSB | EPI_PLANE, 4>(a, s.dtype, st);
                return launch<1, 256, 512, 2, 2, 1, 4, 9, 9, EPI_RELU | EPI_POSB, 4>(a, s.dtype, st);
            case 4: LDM_REQUIRE(s.y, "bottleneck: y");
                if (a.Hin == 2 && a.Win == 8 && plane_taps())   // the canonical latent: one sample per lane group
                    return launch<0, 512, 512, 2, 2, 1, 8, 9, 9, EPI_RELU | EPI_POSB | EPI_PLANE, 4>(a, s.dtype, st);
                return launch<0, 512, 512, 2, 2, 1, 8, 9, 9, EPI_RELU | EPI_POSB, 4>(a, s.dtype, st);
            case 5: LDM_REQUIRE(s.y && s.skip, "dec4: y, skip");
                if (a.Hin == 2 && a.Win == 8 && plane_taps())
                    return launch<2, 512, 256, 2, 2, 1, 4, 9, 9, EPI_RELU | EPI_SKIP | EPI_PLANE, 8>(a, s.dtype, st);
                return launch<2, 512, 256, 2, 2, 1, 4, 9, 9, EPI_RELU | EPI_SKIP, 8>(a, s.dtype, st);
            case 6: LDM_REQUIRE(s.y && s.skip, "dec3: y, skip");
                return launch<2, 256, 128, 2, 2, 1, 4, 9, 9, EPI_RELU | EPI_SKIP, 4>(a, s.dtype, st);
            default: return fail(2, "step conv: no K-split variant for this layer");
        }
    }
    switch (layer) {
        case 0: LDM_REQUIRE(s.y, "enc1: y");
            if (window_taps() && a.Wq % 64 == 0)   // a block's 64 columns lie in one row
                return launch<0, 32, 64, 2, 1, 4, 1, 18, 18, EPI_RELU | EPI_WINDOW>(a, s.dtype, st);
            return launch<0, 32, 64, 2, 1, 4, 1, 18, 18, EPI_RELU>(a, s.dtype, st);
        case 1: LDM_REQUIRE(s.y && s.bcast, "enc2: y, t_emb");
            if (enc2_wide(W)) {
                if (window_taps()) return launch<1, 64, 128, 1, 1, 4, 1, 36, 36, EPI_RELU | EPI_BCAST | EPI_WINDOW>(a, s.dtype, st);
                return launch<1, 64, 128, 1, 1, 4, 1, 36, 36, EPI_RELU | EPI_BCAST>(a, s.dtype, st);
            }
            if (window_taps() && a.Wq % 32 == 0)
                return launch<1, 64, 128, 2, 2, 1, 4, 9, 9, EPI_RELU | EPI_BCAST | EPI_WINDOW>(a, s.dtype, st);
            return launch<1, 64, 128, 2, 2, 1, 4, 9, 9, EPI_RELU | EPI_BCAST>(a, s.dtype, st);
        case 2: LDM_REQUIRE(s.y, "enc3: y");
            if (enc3_thin(W)) {
                if (window_taps()) return launch<1, 128, 256, 1, 1, 2, 2, 36, 36, EPI_RELU | EPI_WINDOW>(a, s.dtype, st);
                return launch<1, 128, 256, 1, 1, 2, 2, 36, 36, EPI_RELU>(a, s.dtype, st);
            }
            if (window_taps() && a.Wq % 16 == 0) return launch<1, 128, 256, 2, 1, 1, 4, 18, 18, EPI_RELU | EPI_WINDOW>(a, s.dtype, st);
            return launch<1, 128, 256, 2, 1, 1, 4, 18, 18, EPI_RELU>(a, s.dtype, st);
        case 3: LDM_REQUIRE(s.y, "enc4: y"); return launch<1, 256, 512, 1, 1, 1, 4, 36, 36, EPI_RELU | EPI_POSB>(a, s.dtype, st);
        case 4: LDM_REQUIRE(s.y, "bottleneck: y"); return launch<0, 512, 512, 1, 1, 1, 8, 36, 12, EPI_RELU | EPI_POSB>(a, s.dtype, st);
        case 5: LDM_REQUIRE(s.y && s.skip, "dec4: y, skip");
            return launch<2, 512, 256, 1, 1, 1, 8, 36, 12, EPI_RELU | EPI_SKIP>(a, s.dtype, st);
        case 6: LDM_REQUIRE(s.y && s.skip, "dec3: y, skip");
            if (window_taps() && a.Wq % 16 == 0)
                return launch<2, 256, 128, 1, 1, 1, 4, 36, 36, EPI_RELU | EPI_SKIP | EPI_WINDOW>(a, s.dtype, st);
            return launch<2, 256, 128, 1, 1, 1, 4, 36, 36, EPI_RELU | EPI_SKIP>(a, s.dtype, st);
        case 7: LDM_REQUIRE(s.y && s.skip, "dec2: y, skip");
            if (window_taps() && a.Wq % 32 == 0)
                return launch<2, 128, 64, 1, 2, 1, 4, 18, 18, EPI_RELU | EPI_SKIP | EPI_WINDOW>(a, s.dtype, st);
            return launch<2, 128, 64, 1, 2, 1, 4, 18, 18, EPI_RELU | EPI_SKIP>(a, s.dtype, st);
        default: LDM_REQUIRE(s.xs && s.coef, "dec1: sampler state, coefficients");
            if (dec1_thin(W)) {
                if (window_taps()) return launch<0, 64, 32, 1, 2, 2, 2, 18, 18, EPI_DDIM | EPI_WINDOW>(a, s.dtype, st);
                return launch<0, 64, 32, 1, 2, 2, 2, 18, 18, EPI_DDIM>(a, s.dtype, st);
            }
            if (window_taps() && a.Wq % 32 == 0)   // a block's 32 columns lie in one row
                return launch<0, 64, 32, 2, 2, 1, 4, 9, 9, EPI_DDIM | EPI_WINDOW>(a, s.dtype, st);
            return launch<0, 64, 32, 2, 2, 1, 4, 9, 9, EPI_DDIM>(a, s.dtype, st);
    }
}

int step_layout(const float* x, float* y, int B, int C, int HW, bool to_nhwc, hipStream_t st) {
    const int64_t n = (int64_t)B * C * HW;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    if (to_nhwc)
        hipLaunchKernelGGL(uc::nchw_to_nhwc_kernel, dim3(blocks), dim3(256), 0, st, x, y, C, HW, n);
    else
        hipLaunchKernelGGL(uc::nhwc_to_nchw_kernel, dim3(blocks), dim3(256), 0, st, x, y, C, HW, n);
    LDM_CHECK_LAUNCH("layout transpose");
    return 0;
}

}  // namespace ldm

using namespace ldm;

extern "C" int64_t ldm_step_packed_floats(int32_t layer) { return step_packed_floats(layer); }

#if (UCONV_DIAG & 4)
extern "C" int ldm_debug_uconv_stamps(unsigned long long* host, int nblocks) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(uc::g_uconv_stamps), sizeof(unsigned long long) * 5 * nblocks, 0,
                                    hipMemcpyDeviceToHost);
}
#endif

extern "C" int ldm_step_pack_weight_dt(int32_t layer, int32_t dtype, const float* w, float* packed, void* stream) {
    LDM_REQUIRE(layer >= 0 && layer <= 8 && w && packed, "step pack: bad argument");
    LDM_REQUIRE(dtype >= LDM_DT_F32 && dtype <= LDM_DT_BF16, "step pack: unknown operand precision");
    const uc::LayerGeo& g = uc::kGeo[layer];
    const int64_t total = step_packed_floats(layer);
    const dim3 grid((unsigned)((total + 255) / 256));
    const int tr = g.mode == 2 ? 1 : 0;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == LDM_DT_F32)
        hipLaunchKernelGGL(uc::uconv_pack_kernel<0>, grid, dim3(256), 0, st, w, packed, g.cin, g.cout, tr);
    else if (dtype == LDM_DT_F16)
        hipLaunchKernelGGL(uc::uconv_pack_kernel<LDM_DT_F16>, grid, dim3(256), 0, st, w, packed, g.cin, g.cout, tr);
    else
        hipLaunchKernelGGL(uc::uconv_pack_kernel<LDM_DT_BF16>, grid, dim3(256), 0, st, w, packed, g.cin, g.cout, tr);
    LDM_CHECK_LAUNCH("uconv_pack_kernel");
    return 0;
}

extern "C" int ldm_step_pack_weight(int32_t layer, const float* w, float* packed, void* stream) {
    return ldm_step_pack_weight_dt(layer, LDM_DT_F32, w, packed, stream);
}

extern "C" int ldm_step_conv(int32_t layer, int32_t B, int32_t H, int32_t W, const float* x, const float* packed,
                             const float* bias, const float* bcast, const float* skip, float* y, void* stream) {
    return ldm_step_conv_dt(layer, B, H, W, x, packed, bias, bcast, skip, y, LDM_DT_F32, stream);
}

extern "C" int64_t ldm_step_workspace_floats(int32_t B, int32_t H, int32_t W) {
    if (B <= 0 || H % 8 || W % 8) return -1;
    return step_ws_floats(B, H, W, nullptr);
}

extern "C" int64_t ldm_step_workspace_counter_floats(int32_t B, int32_t H, int32_t W) {
    if (B <= 0 || H % 8 || W % 8) return -1;
    int64_t c = 0;
    step_ws_floats(B, H, W, &c);
    return c;
}

extern "C" int ldm_step_conv_ws(int32_t layer, int32_t B, int32_t H, int32_t W, const float* x, const float* packed,
                                const float* bias, const float* bcast, const float* skip, float* y, int32_t dtype,
                                float* workspace, void* stream) {
    StepConv s{};
    s.dtype = dtype;
    s.x = x;
    s.w = packed;
    s.bias = bias;
    s.bcast = bcast;
    s.skip = skip;
    s.y = y;
    s.ws = workspace;
    LDM_REQUIRE(layer != 8, "ldm_step_conv: dec1 runs fused with the DDIM update (ldm_ddim_sample)");
    return step_conv(layer, B, H, W, s, (hipStream_t)stream);
}

extern "C" int ldm_step_dec1_ddim(int32_t B, int32_t H, int32_t W, const float* d2, const float* packed, const float* bias,
                                  const float* coef, float eta, float* xs, float* x0_log, float* eps_log, int32_t dtype,
                                  void* stream) {
    LDM_REQUIRE(d2 && packed && bias && coef && xs, "ldm_step_dec1_ddim: null argument");
    StepConv s{};
    s.dtype = dtype;
    s.x = d2;
    s.w = packed;
    s.bias = bias;
    s.coef = coef;
    s.eta = eta;
    s.xs = xs;
    s.x0_log = x0_log;
    s.eps_log = eps_log;
    return step_conv(8, B, H, W, s, (hipStream_t)stream);
}

extern "C" int ldm_step_conv_dt(int32_t layer, int32_t B, int32_t H, int32_t W, const float* x, const float* packed,
                                const float* bias, const float* bcast, const float* skip, float* y, int32_t dtype,
                                void* stream) {
    StepConv s{};
    s.dtype = dtype;
    s.x = x;
    s.w = packed;
    s.bias = bias;
    s.bcast = bcast;
    s.skip = skip;
    s.y = y;
    LDM_REQUIRE(layer != 8, "ldm_step_conv: dec1 runs fused with the DDIM update (ldm_ddim_sample)");
    return step_conv(layer, B, H, W, s, (hipStream_t)stream);
}
