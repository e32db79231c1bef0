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
#include <algorithm>
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

template <int BM, int DT, int XS>
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
    // XS: x stored in 16 bits (LDM_DT_X16, the operand type DT): 2-byte gathers, staged without conversion
    constexpr int XB = XS ? 2 : 4;   // bytes per input element
    using GT = std::conditional_t<XS != 0, unsigned short, float>;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(a.x), (short)0, uni(a.B * a.Cin * HWin * XB), 0x00020000);
    const int gbase = (gb * a.Cin + gk * 16) * HWin;   // elements
    auto gather = [&](int c, GT (&gv)[16]) {
        const int cc = c / ntap;   // channel-chunk major, tap minor: the taps of a window run back to back
        const int t = c - cc * ntap;   // (wave-uniform)
        const int ci0 = cc * KC;
        const int iy = gqy * a.pt.sy + a.pt.dy[ph][t];
        const int ix = gqx * a.pt.sy + a.pt.dx[ph][t];
        const bool ok = gval && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
        const int voff = ok ? (gbase + ci0 * HWin + iy * a.Win + ix) * XB : kOOB;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if constexpr (XS != 0)
                gv[j] = (TCONV_DIAG & 1) ? (GT)(voff + j)
                                         : __builtin_amdgcn_raw_buffer_load_b16(xr, voff, uni(j * HWin * XB), 0);
            else
                gv[j] = (TCONV_DIAG & 1) ? (float)(voff + j)
                                         : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, voff, uni(j * HWin * XB), 0));
        }
    };
    auto stage = [&](int buf, const GT (&gv)[16]) {
        u16x8* dst = reinterpret_cast<u16x8*>(&bt[buf][gp * KP + gk * 16]);
        if constexpr (XS != 0) {
            u16x8 lo, hi;
#pragma unroll
            for (int j = 0; j < 8; ++j) lo[j] = gv[j], hi[j] = gv[8 + j];
            dst[0] = lo;
            dst[1] = hi;
        } else {
            floatx8 lo, hi;
#pragma unroll
            for (int j = 0; j < 8; ++j) lo[j] = gv[j], hi[j] = gv[8 + j];
            dst[0] = to16<DT>(lo);
            dst[1] = to16<DT>(hi);
        }
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

    GT gv[2][16];
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

    // ---- epilogue: bias -> eval-BN -> act (-> act_out), NCHW store.  Per channel (i, q) the bias / BN constants
    // are read once for the lane's two positions; the activation, the BN flag and the storage type are
    // compile-time forms dispatched once (per-value runtime switches and loads were the epilogue's cost).
    const EpiArgs& e = a.ep;
    const bool ro = e.round_out != 0;   // a select per value: DT is known here, the mode test is not per value
    auto rnd = [ro](float v) { return ro ? round16(v, DT) : v; };
    size_t obase[2];
    bool nok[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int64_t n = n0 + wn * 64 + 32 * j + r;
        nok[j] = n < a.N;
        const int nn = nok[j] ? (int)n : 0;
        const int b = a.fd_hw.div(nn);
        const int rr = nn - b * (a.pt.Hq * a.pt.Wq);
        const int qy = a.fd_w.div(rr);
        const int qx = rr - qy * a.pt.Wq;
        const int oy = qy * a.pt.osy + a.pt.ry[ph], ox = qx * a.pt.osy + a.pt.rx[ph];
        obase[j] = (size_t)b * a.Cout * a.Hout * a.Wout + (size_t)oy * a.Wout + ox;
    }
    const size_t HWo = (size_t)a.Hout * a.Wout;
    auto store_lane = [&](auto actc, auto bnc, auto y16c) {
        constexpr int ACT = decltype(actc)::value;   // LDM_ACT_NONE, LDM_ACT_RELU, or -1: e.act at run time
        constexpr bool BNF = decltype(bnc)::value, Y16 = decltype(y16c)::value;
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int co = mbase + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
                if (co >= a.Cout) continue;
                const float bias = e.bias ? e.bias[co] : 0.f;
                float alpha = 0.f, beta = 0.f;
                if constexpr (BNF) {   // as epi_finish (conv.hip)
                    const float invstd = 1.0f / sqrtf(e.bn_v[co] + e.bn_eps);
                    alpha = invstd * e.bn_w[co];
                    beta = e.bn_b[co] - e.bn_m[co] * alpha;
                }
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if (!nok[j]) continue;
                    float v = acc[i][j][q];
                    if (e.bias) v = v + bias;
                    v = rnd(v);   // (autocast output semantics: round_out is 0 or DT)
                    if constexpr (BNF) v = rnd(v * alpha + beta);
                    if constexpr (ACT == LDM_ACT_RELU) v = v < 0.f ? 0.f : v;
                    else if constexpr (ACT < 0) v = apply_act(v, e.act);
                    v = rnd(v);
                    const size_t o = obase[j] + (size_t)co * HWo;
                    if (e.act_out) st1_st<DT>(e.act_out, o, Y16, v);
                    st1_st<DT>(a.y, o, Y16, v);
                }
            }
    };
    auto by_store = [&](auto actc, auto bnc) {
        if (e.y16) store_lane(actc, bnc, std::true_type{});
        else store_lane(actc, bnc, std::false_type{});
    };
    using A0 = std::integral_constant<int, LDM_ACT_NONE>;
    using A1 = std::integral_constant<int, LDM_ACT_RELU>;
    using AG = std::integral_constant<int, -1>;
    if (e.bn_w) {
        if (e.act == LDM_ACT_NONE) by_store(A0{}, std::true_type{});
        else if (e.act == LDM_ACT_RELU) by_store(A1{}, std::true_type{});
        else by_store(AG{}, std::true_type{});
    } else {
        if (e.act == LDM_ACT_NONE) by_store(A0{}, std::false_type{});
        else if (e.act == LDM_ACT_RELU) by_store(A1{}, std::false_type{});
        else by_store(AG{}, std::false_type{});
    }
}

// ---------------------------------------------------------------------------------------------------------
// Window form (tconvw_kernel): the same tiles, plan and packed weights, but the activation operand is staged
// once per 16-channel window instead of once per (tap, 32-channel chunk).  tconv_kernel's time went into its
// per-chunk instruction stream (16 four-byte gathers per lane per chunk of K = 32, one barrier per chunk):
// here a block loads, for 16 input channels, the whole input window its 128 positions' taps read (rows x
// columns incl. halo and zero padding) with 16-byte loads along the NCHW rows, converts it to 16 bits and
// parks it position-major in LDS ([window position][16 channels + 8 pad], 48-B rows: the 32-position B-fragment
// reads are conflict-free).  Every tap then reads its B fragment (8 channels of one position, one ds_read_b128)
// at a tap-constant offset from that image: K = 16 x taps per barrier (144 for a 3x3 conv) instead of 32.
//   * stride-2 windows are stored with even and odd columns apart, so that the 32 consecutive positions of a
//     fragment read consecutive image positions for every tap;
//   * the next window's loads are issued before this window's MFMAs and written to the other LDS buffer after
//     them; the A fragments (weights) of every tap of the next window are issued as soon as this window's tap
//     has consumed its set, so the in-order vector-memory returns never make a tap wait for the window loads;
//   * one phase per block and the same tap count for every block of a launch (template NT): transposed convs
//     whose phases differ in taps run one launch per tap count.
// Geometry (tconvw_geometry): a tile of 128 positions is R = 128 / Cq rows x Cq columns of the phase grid (Cq =
// 128 or Wq | 128, inside one sample); Win % 4 == 0 (a 16-byte quad is wholly inside or outside a row).
// compile-time loop: f(integral_constant<int, I>) for I in [B, E)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

constexpr int WCH = 16;   // input channels per window
constexpr int WP = 24;    // 16-bit elements per image position (48-B rows)

struct WArgs {
    const float* x;
    const unsigned short* w;   // packed [phase][chunk][Mpad][32] 16-bit (as tconv_kernel)
    float* y;
    int32_t B, Cin, Hin, Win, Cout, Hout, Wout;
    int32_t Mpad, nM, nN, cpt;
    int32_t xcd_chunk;
    int32_t nph;                      // phases in this launch
    int32_t phs[kMaxPhase];           // their indices
    int64_t N;                        // positions per phase
    FastDiv fd_hw, fd_w;
    int32_t cq_log2;                  // tile columns Cq = 1 << cq_log2
    int32_t NQ, rowp, half, nsu;      // window: quads per row, image positions per row, odd-column plane, super-units
    int32_t imgsz;                    // 16-bit elements per image buffer
    int32_t ybase[kMaxPhase], xbase[kMaxPhase];   // window origin = (qy0 * sy + ybase, qx0 * sy + xbase)
    int32_t toff[kMaxPhase][kMaxTap];             // image-position offset of each tap
    PhaseTable pt;
    EpiArgs ep;
};

// PK = 1: the four output-parity phases of a k3 s2 p1 op1 transposed conv (the data gradient of a 3x3 stride-2
// conv) in ONE block over one shared window — phases (0,0), (0,1), (1,0), (1,1) have 1, 2, 2, 4 taps, all reading
// input offsets {0, 1} x {0, 1}, so the block runs nine (phase, tap) pairs per window into four accumulator sets,
// the compute density of a 3x3 conv (a launch per phase reloads the window for one to four taps).
// PK = 2 (round 5): the same for the four phases of a k4 s2 p1 transposed conv (the decoder's 128 -> 64 layer): four
// taps each, all reading input offsets {-1, 0, 1} x {-1, 0, 1}: sixteen (phase, tap) pairs per shared window.
template <int PK>
__host__ __device__ constexpr int pk_phase(int i) {
    return PK == 2 ? i / 4 : (i < 1 ? 0 : (i < 3 ? 1 : (i < 5 ? 2 : 3)));
}
template <int PK>
__host__ __device__ constexpr int pk_tap(int i) {
    return PK == 2 ? i % 4 : (i < 1 ? i : (i < 3 ? i - 1 : (i < 5 ? i - 3 : i - 5)));
}
template <int PK>
__host__ __device__ constexpr int pk_ntap(int p) { return PK == 2 ? 4 : (p == 0 ? 1 : (p == 3 ? 4 : 2)); }

// WNW: waves along the positions.  2: a 2 x 2 wave grid (BM / 2 rows x 64 positions per wave); 1 (round 5,
// BM = 128): four waves of 32 rows x all 128 positions, so no two waves load the same weight fragments — the
// weights were 3x the window's bytes per block (four waves x 9 taps x 2 row tiles x 1 KB per window)
template <int BM, int NT, int SY, int DT, int NS, int PK = 0, int XS = 0, int WNW = 2>
__global__ __launch_bounds__(256, 2) void tconvw_kernel(WArgs a) {
    constexpr int WMW = 4 / WNW;              // waves along the rows
    constexpr int MT = BM / (32 * WMW);       // 32-row tiles per wave
    constexpr int NJ = 4 / WNW;               // 32-position tiles per wave
    static_assert(MT >= 1 && MT * 32 * WMW == BM, "wave grid");
    constexpr int NACC = PK ? 4 : 1;
    static_assert(!PK || (NT == (PK == 2 ? 16 : 9) && SY == 1),
                  "PK 1 / 2: the nine / sixteen (phase, tap) pairs of a k3 op1 / k4 p1 transposed conv");
    extern __shared__ __attribute__((aligned(16))) unsigned short img[];   // [2][image]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WNW, wn = wave % WNW;
    const int r = lane & 31, h = lane >> 5;

    int t = blockIdx.x;
    if (a.xcd_chunk > 0) t = (t & 7) * a.xcd_chunk + (t >> 3);
    const int mt = t % a.nM;
    const int rest = t / a.nM;
    const int ph = PK ? 0 : a.phs[rest % a.nph];   // (PK 1: every phase; the window origin is phase 0's)
    const int nt = PK ? rest : rest / a.nph;
    const int n0 = nt * BN;
    const int HWq = a.pt.Hq * a.pt.Wq;
    const int b = a.fd_hw.div(n0);
    const int rem = n0 - b * HWq;
    const int qy0 = a.fd_w.div(rem);
    const int qx0 = rem - qy0 * a.pt.Wq;
    const int iyb = qy0 * SY + a.ybase[ph], ixb = qx0 * SY + a.xbase[ph];
    const int HWin = a.Hin * a.Win;
    const int imgsz = a.imgsz;   // 16-bit elements per image buffer (+ a 48-B dummy row after it)

    // ---- window super-units of this thread: 4 channels x one 16-byte column quad of one window row
    // XS: x stored in 16 bits (the operand type DT): a quad is one 8-byte load, parked without conversion
    constexpr int XB = XS ? 2 : 4;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(a.x), (short)0, uni(a.B * a.Cin * HWin * XB), 0x00020000);
    int svo[NS], slp[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int su = s * 256 + tid;
        const bool valid = su < a.nsu;
        const int q4 = a.NQ * 4;
        const int wr = su / q4;
        const int rr = su - wr * q4;
        const int q = rr >> 2, cg = rr & 3;
        const int iy = iyb + wr, ix = ixb + 4 * q;
        const bool ok = valid && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
        svo[s] = ok ? ((b * a.Cin + 4 * cg) * HWin + iy * a.Win + ix) * XB : kOOB;
        // (a slot past the window writes to the dummy row after the image: the store stays branch-free)
        slp[s] = valid ? (wr * a.rowp + (SY == 2 ? 2 * q : 4 * q)) * WP + 4 * cg : imgsz;
    }
    using WV = std::conditional_t<XS != 0, uint2, floatx4>;   // one channel's column quad
    WV wv[NS][4];
    auto load_win = [&](int w) {   // channels 16 w + 4 cg + i of every super-unit
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if constexpr (XS != 0)
                    wv[s][i] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(
                                                             xr, svo[s], uni((w * WCH + i) * HWin * XB), 0));
                else
                    wv[s][i] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                                               xr, svo[s], uni((w * WCH + i) * HWin * XB), 0));
            }
    };
    auto store_win = [&](int buf) {
        unsigned short* base = img + buf * (imgsz + WP);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int col = slp[s] == imgsz ? 0 : (SY == 2 ? ((k & 1) * a.half + (k >> 1)) : k);
                uint2 pk;
                if constexpr (XS != 0) {
                    // column k of channels 0..3: the k-th 16-bit half of each channel's quad
                    auto el = [&](int i) { return (k < 2 ? wv[s][i].x : wv[s][i].y) >> (16 * (k & 1)) & 0xffffu; };
                    pk.x = el(0) | (el(1) << 16);
                    pk.y = el(2) | (el(3) << 16);
                } else {
                    floatx4 v{wv[s][0][k], wv[s][1][k], wv[s][2][k], wv[s][3][k]};
                    if constexpr (DT == 1)
                        pk = __builtin_bit_cast(uint2, __builtin_convertvector(v, halfx4));
                    else
                        pk = __builtin_bit_cast(uint2, __builtin_convertvector(v, bf16x4));
                }
                *reinterpret_cast<uint2*>(base + slp[s] + col * WP) = pk;
            }
        }
    };

    // ---- B fragments: this lane's two 32-column tiles, image position of tap 0's origin
    int lb[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int nl = wn * 32 * NJ + 32 * j + r;
        const int rrow = nl >> a.cq_log2, cx = nl & ((1 << a.cq_log2) - 1);
        lb[j] = (rrow * SY * a.rowp + cx) * WP + 8 * h;
    }

    // ---- A fragments: rows mbase + 32 i + r, k = 16 (w & 1) + 8 h of chunk (w / 2) * NT + tap
    const int mbase = mt * BM + wm * 32 * MT;
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(uni_ptr(a.w), (short)0, 0x7ffffff0, 0x00020000);
    u16x8 af[NT][MT];
    // pair tp: phase PK ? pk_phase(tp) : ph, tap in that phase PK ? pk_tap(tp) : tp
    auto loadA = [&](int w, auto tpc, u16x8 (&dst)[MT]) {
        constexpr int tp = decltype(tpc)::value;
        const int pp = PK ? pk_phase<PK>(tp) : ph;
        const int c = (w >> 1) * (PK ? pk_ntap<PK>(pk_phase<PK>(tp)) : NT) + (PK ? pk_tap<PK>(tp) : tp);
        const int wph = (int)a.pt.wofs[pp];
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const int e = wph + (c * a.Mpad + mbase + 32 * i + r) * KC + 16 * (w & 1) + 8 * h;
            dst[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, e * 2, 0, 0));
        }
    };

    floatx16 acc[NACC][MT][NJ];
#pragma unroll
    for (int u = 0; u < NACC; ++u)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int q = 0; q < 16; ++q) acc[u][i][j][q] = 0.f;

    const int NW = a.Cin / WCH;
    static_for<0, NT>([&](auto tpc) { loadA(0, tpc, af[decltype(tpc)::value]); });
    load_win(0);
    store_win(0);
    __syncthreads();
    // Every iteration issues the same instruction stream (past the end: re-loads of the last window and its
    // weights, stored into the idle buffer, which nothing reads), so that the loads are never sunk into a
    // conditional store and the waitcnt pass counts them exactly; the scheduling fences keep the window
    // loads ahead of the MFMAs and each tap's weight loads right after the tap that frees their registers.
    for (int w = 0; w < NW; ++w) {
        const int buf = w & 1;
        const int wn1 = w + 1 < NW ? w + 1 : w;
        load_win(wn1);
        __builtin_amdgcn_sched_barrier(0);
        const unsigned short* bimg = img + buf * (imgsz + WP);
        static_for<0, NT>([&](auto tpc) {
            constexpr int tp = decltype(tpc)::value;
            constexpr int u = PK ? pk_phase<PK>(tp) : 0;
            const int to = (PK ? a.toff[u][pk_tap<PK>(tp)] : a.toff[ph][tp]) * WP;
            u16x8 bf[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j) bf[j] = *reinterpret_cast<const u16x8*>(bimg + lb[j] + to);
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j) acc[u][i][j] = mma<DT>(af[tp][i], bf[j], acc[u][i][j]);
            loadA(wn1, tpc, af[tp]);   // this tap's set is free: the next window's weights for it
            __builtin_amdgcn_sched_barrier(0);
        });
        store_win(buf ^ 1);
        __syncthreads();
    }

    // ---- epilogue: bias -> eval-BN -> act (-> act_out)
    const EpiArgs& e = a.ep;
    const bool ro = e.round_out != 0;   // a select per value: DT is known here, the mode test is not per value
    auto rnd = [ro](float v) { return ro ? round16(v, DT) : v; };
    if constexpr (NT == 4) {
        // a single transposed-conv phase: its outputs sit two columns apart, so each lane stores its own values.
        // Per channel (i, q) the bias / BN constants are read once for the lane's two positions, and the
        // activation, the BN flag and the storage type are compile-time forms dispatched once (see below).
        size_t obase[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int nn = n0 + wn * 32 * NJ + 32 * j + r;
            const int bb = a.fd_hw.div(nn);
            const int rr = nn - bb * HWq;
            const int qy = a.fd_w.div(rr);
            const int qx = rr - qy * a.pt.Wq;
            const int oy = qy * a.pt.osy + a.pt.ry[ph], ox = qx * a.pt.osy + a.pt.rx[ph];
            obase[j] = (size_t)bb * a.Cout * a.Hout * a.Wout + (size_t)oy * a.Wout + ox;
        }
        const size_t HWo = (size_t)a.Hout * a.Wout;
        auto store_lane = [&](auto actc, auto bnc, auto y16c) {
            constexpr int ACT = decltype(actc)::value;   // LDM_ACT_NONE, LDM_ACT_RELU, or -1: e.act at run time
            constexpr bool BNF = decltype(bnc)::value, Y16 = decltype(y16c)::value;
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int co = mbase + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
                    if (co >= a.Cout) continue;
                    const float bias = e.bias ? e.bias[co] : 0.f;
                    float alpha = 0.f, beta = 0.f;
                    if constexpr (BNF) {   // as epi_finish (conv.hip)
                        const float invstd = 1.0f / sqrtf(e.bn_v[co] + e.bn_eps);
                        alpha = invstd * e.bn_w[co];
                        beta = e.bn_b[co] - e.bn_m[co] * alpha;
                    }
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        float v = acc[0][i][j][q];
                        if (e.bias) v = v + bias;
                        v = rnd(v);
                        if constexpr (BNF) v = rnd(v * alpha + beta);
                        if constexpr (ACT == LDM_ACT_RELU) v = v < 0.f ? 0.f : v;
                        else if constexpr (ACT < 0) v = apply_act(v, e.act);
                        v = rnd(v);
                        const size_t o = obase[j] + (size_t)co * HWo;
                        if (e.act_out) st1_st<DT>(e.act_out, o, Y16, v);
                        st1_st<DT>(a.y, o, Y16, v);
                    }
                }
        };
        auto by_store = [&](auto actc, auto bnc) {
            if (e.y16) store_lane(actc, bnc, std::true_type{});
            else store_lane(actc, bnc, std::false_type{});
        };
        using A0 = std::integral_constant<int, LDM_ACT_NONE>;
        using A1 = std::integral_constant<int, LDM_ACT_RELU>;
        using AG = std::integral_constant<int, -1>;
        if (e.bn_w) {
            if (e.act == LDM_ACT_NONE) by_store(A0{}, std::true_type{});
            else if (e.act == LDM_ACT_RELU) by_store(A1{}, std::true_type{});
            else by_store(AG{}, std::true_type{});
        } else {
            if (e.act == LDM_ACT_NONE) by_store(A0{}, std::false_type{});
            else if (e.act == LDM_ACT_RELU) by_store(A1{}, std::false_type{});
            else by_store(AG{}, std::false_type{});
        }
    } else {
        // Staged through LDS (the image buffers are free now) as [channel][output row segment], then written
        // with 16-byte stores along the NCHW rows: a lane's accumulator holds one position of 16 channels, so
        // direct stores are 4-byte scalars (64-128 per lane), and the store issue, not the bytes, bounded the
        // large-plane layers.  One pass for a single phase (the tile's R rows x Cq columns); PK 1: one pass per
        // output row parity ry, holding phases (ry, 0) and (ry, 1) interleaved into whole output rows.
        // The raw accumulators are staged; the epilogue runs in the store pass, on a 16-byte piece of one output
        // channel at a time (its bias / BN constants loaded once per piece, not once per value), with the
        // activation and the BN flag as compile-time forms (dispatched once: per-value runtime switches and the
        // inlined tanh / erf paths of every value made the epilogue the kernel's largest VALU stream).
        constexpr int NPASS = PK ? 2 : 1;
        constexpr int SEG = BN * (PK ? 2 : 1);          // floats per channel in one pass (R rows x rowlen)
        const int cq = 1 << a.cq_log2;
        const int rl_log2 = a.cq_log2 + (PK ? 1 : 0);   // rowlen = floats per staged output row
        const int rowlen = 1 << rl_log2;
        constexpr int pitch = SEG + 4;                  // (+16 B: consecutive channels start on different banks)
        float* stg = reinterpret_cast<float*>(img);
        const int HWo = a.Hout * a.Wout;
        const int b = a.fd_hw.div(n0);
        const int rem0 = n0 - b * HWq;
        const int qy0 = a.fd_w.div(rem0), qx0 = rem0 - qy0 * a.pt.Wq;
        static_for<0, NPASS>([&](auto passc) {
            constexpr int pass = decltype(passc)::value;
            __syncthreads();   // every wave is done with the image (pass 0) / the previous pass's reads
            static_for<0, NACC>([&](auto uc) {
                constexpr int u = decltype(uc)::value;
                if constexpr (PK && (u >> 1) != pass) return;
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const int nl = wn * 32 * NJ + 32 * j + r;
                    const int rr = nl >> a.cq_log2, cx = nl & (cq - 1);
                    const int col = rr * rowlen + (PK ? 2 * cx + (u & 1) : cx);
#pragma unroll
                    for (int i = 0; i < MT; ++i)
#pragma unroll
                        for (int q = 0; q < 16; ++q) {
                            const int cl = wm * 32 * MT + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
                            stg[cl * pitch + col] = acc[u][i][j][q];
                        }
                }
            });
            __syncthreads();
            constexpr int nv = BM * SEG / 4;           // 16-byte pieces of the staged tile
            auto store_pass = [&](auto actc, auto bnc) {
                constexpr int ACT = decltype(actc)::value;   // LDM_ACT_NONE, LDM_ACT_RELU, or -1: e.act at run time
                constexpr bool BNF = decltype(bnc)::value;
                for (int k = tid; k < nv; k += 256) {
                    const int cl = k / (SEG / 4);
                    const int rest4 = (k - cl * (SEG / 4)) * 4;
                    const int co = mt * BM + cl;
                    if (co >= a.Cout) continue;
                    const int rr = rest4 >> rl_log2, c0 = rest4 - (rr << rl_log2);
                    const int oy = PK ? 2 * (qy0 + rr) + pass : qy0 + rr;
                    const int ox = PK ? 2 * qx0 + c0 : qx0 + c0;
                    const floatx4 raw = *reinterpret_cast<const floatx4*>(stg + cl * pitch + rest4);
                    const float bias = e.bias ? e.bias[co] : 0.f;
                    float alpha = 0.f, beta = 0.f;
                    if constexpr (BNF) {   // as epi_finish (conv.hip)
                        const float invstd = 1.0f / sqrtf(e.bn_v[co] + e.bn_eps);
                        alpha = invstd * e.bn_w[co];
                        beta = e.bn_b[co] - e.bn_m[co] * alpha;
                    }
                    float vv[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        float v = raw[q];
                        if (e.bias) v = v + bias;
                        v = rnd(v);   // (autocast output semantics: round_out is 0 or DT)
                        if constexpr (BNF) v = rnd(v * alpha + beta);
                        if constexpr (ACT == LDM_ACT_RELU) v = v < 0.f ? 0.f : v;
                        else if constexpr (ACT < 0) v = apply_act(v, e.act);
                        vv[q] = rnd(v);
                    }
                    const size_t o = ((size_t)b * a.Cout + co) * HWo + (size_t)oy * a.Wout + ox;
                    if (e.y16) {   // 16-bit storage: 8-byte stores of the four values
                        if (e.act_out) st_st<DT, 4>(e.act_out, o, true, vv);
                        st_st<DT, 4>(a.y, o, true, vv);
                    } else {
                        const floatx4 v4{vv[0], vv[1], vv[2], vv[3]};
                        if (e.act_out) *reinterpret_cast<floatx4*>(e.act_out + o) = v4;
                        *reinterpret_cast<floatx4*>(a.y + o) = v4;
                    }
                }
            };
            using A0 = std::integral_constant<int, LDM_ACT_NONE>;
            using A1 = std::integral_constant<int, LDM_ACT_RELU>;
            using AG = std::integral_constant<int, -1>;
            using BT = std::true_type;
            using BF = std::false_type;
            if (e.bn_w) {
                if (e.act == LDM_ACT_NONE) store_pass(A0{}, BT{});
                else if (e.act == LDM_ACT_RELU) store_pass(A1{}, BT{});
                else store_pass(AG{}, BT{});
            } else {
                if (e.act == LDM_ACT_NONE) store_pass(A0{}, BF{});
                else if (e.act == LDM_ACT_RELU) store_pass(A1{}, BF{});
                else store_pass(AG{}, BF{});
            }
        });
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

// ---- the window form's geometry and launch ------------------------------------------------------------
// Tap count and stride of one launch of the window form (template NT, SY); its image sizes (NS super-unit
// slots per thread, LDS bytes) are checked here against the instance.
// LDM_TCONVW_WNW: the 128-row instances' wave grid (1: four waves along the rows, default; 2: the 2 x 2 grid)
static int tconvw_wnw() {
    static const int v = [] {
        const char* e = std::getenv("LDM_TCONVW_WNW");
        return (e && e[0] == '2') ? 2 : 1;
    }();
    return v;
}

template <int BM, int NT, int SY, int DT, int NS, int PK, int XS>
static int launch_wx(WArgs& a, hipStream_t st) {
    LDM_REQUIRE(a.nsu <= NS * 256, "tconvw: window larger than the instance's register slots");
    // the image double buffer, or the epilogue's staged output tile if larger (BM channels x the pass's floats)
    const int cq = 1 << a.cq_log2;
    const size_t stage = NT == 4 ? 0 : (size_t)BM * ((PK ? 2 * BN : BN) + 4) * 4;
    const size_t lds = std::max((size_t)2 * (a.imgsz + WP) * 2, stage);
    (void)cq;
    // (a 16-tap 128-row tile only on the four-waves-along-rows grid: two row tiles x 16 taps of fragments spill)
    constexpr int WNW0 = (BM == 128 && NT == 16) ? 1 : 2;
    auto kfn = tconvw_kernel<BM, NT, SY, DT, NS, PK, XS, WNW0>;
    if constexpr (BM == 128 && WNW0 == 2)
        if (tconvw_wnw() == 1) kfn = tconvw_kernel<BM, NT, SY, DT, NS, PK, XS, 1>;
    if (lds > 64 * 1024) {
        static bool opted[2] = {false, false};
        const int k = BM == 128 ? tconvw_wnw() - 1 : 1;
        if (!opted[k]) {
            LDM_HIP_TRY(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
            opted[k] = true;
        }
    }
    const int64_t blocks = (int64_t)a.nph * a.nM * a.nN;
    a.xcd_chunk = blocks % 8 == 0 ? (int)(blocks / 8) : 0;
    hipLaunchKernelGGL(kfn, dim3((unsigned)blocks), dim3(256), lds, st, a);
    LDM_CHECK_LAUNCH("tconvw_kernel");
    return 0;
}

template <int BM, int NT, int SY, int DT, int NS, int PK = 0>
static int launch_w(WArgs& a, hipStream_t st) {
    if (a.ep.x16) return launch_wx<BM, NT, SY, DT, NS, PK, DT>(a, st);
    return launch_wx<BM, NT, SY, DT, NS, PK, 0>(a, st);
}

// Window geometry of the phases `phs` (same tap count) of a kind-3 conv; false when the tile / window shape
// does not fit the window form (tconv_kernel then runs).
static bool w_geometry(const ldm_conv_desc& d, const PhaseTable& pt, const int* phs, int nph, WArgs& a,
                       bool shared = false) {
    if (d.Win % 4 || d.Wout % 4 || d.Cin % WCH) return false;   // 16-byte window quads and output stores
    const int HWq = pt.Hq * pt.Wq;
    if (HWq % BN) return false;
    int cq;
    if (pt.Wq % BN == 0) cq = BN;
    else if (BN % pt.Wq == 0) cq = pt.Wq;
    else return false;
    int l2 = 0;
    while ((1 << l2) < cq) ++l2;
    if ((1 << l2) != cq) return false;
    const int R = BN / cq, sy = pt.sy;
    if (sy != 1 && sy != 2) return false;
    int NR = 0, NQ = 0;
    a.nph = nph;
    for (int i = 0; i < nph; ++i) {
        const int p = phs[i];
        a.phs[i] = p;
        int dy0 = 1 << 20, dy1 = -(1 << 20), dx0 = 1 << 20, dx1 = -(1 << 20);
        for (int t = 0; t < pt.ntap[p]; ++t) {
            dy0 = std::min(dy0, (int)pt.dy[p][t]), dy1 = std::max(dy1, (int)pt.dy[p][t]);
            dx0 = std::min(dx0, (int)pt.dx[p][t]), dx1 = std::max(dx1, (int)pt.dx[p][t]);
        }
        const int xb = dx0 >= 0 ? (dx0 / 4) * 4 : -((-dx0 + 3) / 4) * 4;   // 4 * floor(dx0 / 4)
        a.ybase[p] = dy0;
        a.xbase[p] = xb;
        NR = std::max(NR, (R - 1) * sy + (dy1 - dy0) + 1);
        NQ = std::max(NQ, ((cq - 1) * sy + dx1 - xb) / 4 + 1);
    }
    if (shared) {   // one window for every phase of the block: the common origin and extent
        int y0 = 1 << 20, x0 = 1 << 20, y1 = -(1 << 20), x1 = -(1 << 20);
        for (int i = 0; i < nph; ++i)
            for (int t = 0; t < pt.ntap[phs[i]]; ++t) {
                y0 = std::min(y0, (int)pt.dy[phs[i]][t]), y1 = std::max(y1, (int)pt.dy[phs[i]][t]);
                x0 = std::min(x0, (int)pt.dx[phs[i]][t]), x1 = std::max(x1, (int)pt.dx[phs[i]][t]);
            }
        const int xb = x0 >= 0 ? (x0 / 4) * 4 : -((-x0 + 3) / 4) * 4;
        for (int i = 0; i < nph; ++i) a.ybase[phs[i]] = y0, a.xbase[phs[i]] = xb;
        NR = (R - 1) * sy + (y1 - y0) + 1;
        NQ = ((cq - 1) * sy + x1 - xb) / 4 + 1;
    }
    a.NQ = NQ;
    a.rowp = 4 * NQ;
    a.half = 2 * NQ;
    a.nsu = 4 * NR * NQ;
    a.imgsz = NR * a.rowp * WP;
    if ((size_t)2 * a.imgsz * 2 > 150 * 1024) return false;
    for (int i = 0; i < nph; ++i) {
        const int p = phs[i];
        for (int t = 0; t < pt.ntap[p]; ++t) {
            const int c0 = pt.dx[p][t] - a.xbase[p];
            a.toff[p][t] = (pt.dy[p][t] - a.ybase[p]) * a.rowp + (sy == 2 ? ((c0 & 1) * a.half + (c0 >> 1)) : c0);
        }
    }
    a.cq_log2 = l2;
    return true;
}

// The window form of one kind-3 conv: one launch per group of phases with equal tap counts.  Returns 1 (and
// launches nothing) when some group's geometry does not fit an instance.
static int forward_window(const ldm_conv_desc& d, const TArgs& t, int bm, int dt, hipStream_t st, bool any_density,
                          bool four_phase_k4) {
    const PhaseTable& pt = t.pt;
    auto fill = [&](WArgs& a) {
        a.x = t.x, a.w = t.w, a.y = t.y;
        a.B = t.B, a.Cin = t.Cin, a.Hin = t.Hin, a.Win = t.Win, a.Cout = t.Cout, a.Hout = t.Hout, a.Wout = t.Wout;
        a.Mpad = t.Mpad, a.nM = t.nM, a.nN = t.nN, a.cpt = t.cpt;
        a.N = t.N, a.fd_hw = t.fd_hw, a.fd_w = t.fd_w, a.pt = t.pt, a.ep = t.ep;
    };
    // the data gradient of a 3x3 stride-2 conv (k3 s2 p1 op1 transposed: phases of 1, 2, 2, 4 taps): all four
    // phases in one block over a shared window, on 64-row tiles (four accumulator sets)
    if (pt.nphase == 4 && pt.sy == 1 && pt.ntap[0] == 1 && pt.ntap[1] == 2 && pt.ntap[2] == 2 && pt.ntap[3] == 4) {
        WArgs a{};
        const int all[4] = {0, 1, 2, 3};
        if (bm != 64 || !w_geometry(d, pt, all, 4, a, true) || a.nsu > 2 * 256) return 1;
        fill(a);
        a.nph = 1;
        return dt == LDM_DT_F16 ? launch_w<64, 9, 1, 1, 2, 1>(a, st) : launch_w<64, 9, 1, 2, 2, 1>(a, st);
    }
    // a k4 s2 p1 transposed conv (the decoder's upsampling layers: four phases of four taps): likewise
    if (four_phase_k4 && pt.nphase == 4 && pt.sy == 1 && pt.ntap[0] == 4 && pt.ntap[1] == 4 && pt.ntap[2] == 4 &&
        pt.ntap[3] == 4) {
        WArgs a{};
        const int all[4] = {0, 1, 2, 3};
        if (bm != 64 || !w_geometry(d, pt, all, 4, a, true) || a.nsu > 2 * 256) return 1;
        fill(a);
        a.nph = 1;
        return dt == LDM_DT_F16 ? launch_w<64, 16, 1, 1, 2, 2>(a, st) : launch_w<64, 16, 1, 2, 2, 2>(a, st);
    }
    int groups[kMaxPhase][kMaxPhase], gn[kMaxPhase], gt[kMaxPhase], ng = 0;
    for (int p = 0; p < pt.nphase; ++p) {
        int g = 0;
        while (g < ng && gt[g] != pt.ntap[p]) ++g;
        if (g == ng) gt[ng] = pt.ntap[p], gn[ng] = 0, ++ng;
        groups[g][gn[g]++] = p;
    }
    WArgs w[kMaxPhase];
    for (int g = 0; g < ng; ++g) {
        w[g] = WArgs{};
        if (!w_geometry(d, pt, groups[g], gn[g], w[g])) return 1;
        const int nt = gt[g], sy = pt.sy;
        const int ns = (w[g].nsu + 255) / 256;
        // measured (profiles/r04/tconv_window): the window form wins for 3x3 convs (5-25 %) and where a window
        // feeds >= 16 MFMAs per wave with one M tile (the decoder's 32 -> 128 convT and its data gradient); with
        // fewer taps x rows per window, or a window re-loaded by two M tiles, the per-chunk form is faster
        const bool dense = (nt * (bm / 64) >= 8 || any_density) && t.nM == 1;
        const bool ok = (nt == 9 && ns <= (sy == 2 ? 4 : 2)) || (nt == 16 && sy == 2 && ns <= 5 && dense) ||
                        (nt == 4 && sy == 1 && ns <= 2 && dense);
        if (!ok) return 1;
    }
    for (int g = 0; g < ng; ++g) {
        WArgs& a = w[g];
        fill(a);
        const int nt = gt[g], sy = pt.sy;
        int rc;
#define TCW(BM_, NT_, SY_, NS_)                                                                          \
    (dt == LDM_DT_F16 ? launch_w<BM_, NT_, SY_, 1, NS_>(a, st) : launch_w<BM_, NT_, SY_, 2, NS_>(a, st))
        if (nt == 16) rc = bm == 128 ? TCW(128, 16, 2, 5) : TCW(64, 16, 2, 5);
        else if (nt == 9 && sy == 2) rc = bm == 128 ? TCW(128, 9, 2, 4) : TCW(64, 9, 2, 4);
        else if (nt == 9) rc = bm == 128 ? TCW(128, 9, 1, 2) : TCW(64, 9, 1, 2);
        else rc = bm == 128 ? TCW(128, 4, 1, 2) : TCW(64, 4, 1, 2);
#undef TCW
        if (rc) return rc;
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
    // the window form where the geometry allows (LDM_TCONV_WIN=0: the per-chunk gather form, A/B timing).
    // 16-tap (4x4 stride-2) convs run it on 64-row tiles: their image needs five register slots per thread.
    // LDM_TCONV_WIN: bit 0 the single-phase window forms, bit 1 the four-phase form of the k3 s2 op1 transposed
    // convs (0 = the per-chunk gather form everywhere); bit 3 (with bit 1): the four-phase form of the k4 s2 p1
    // transposed convs too.  Default before round 5: bit 0 only: in the train step (B = 32, bf16)
    // 4.899 ms per step on the gather form, 4.823 with bit 0, 4.874 with both — the four-phase form won only on
    // style_enc3's data gradient (85 -> 71 us) and lost 5-16 us on the other four (profiles/r04/tconv_window);
    // re-measured with the maps in 16 bits: 909 vs 724 us for those layers, 3.98-4.00 vs 3.86-3.95 ms per step
    // Round 5: with the epilogue's per-value branches and loads gone (tconvw_kernel's store pass) the four-phase
    // form wins on every k3 s2 data gradient of the step (tools/one_conv.py, B = 32 bf16: 64 -> 128 104.9 -> 66.7
    // us, 128 -> 256 91.3 -> 53.1, 256 -> 256 52.5 -> 32.7, 128 -> 32 46.1 -> 22.7), and its k4 s2 p1 form (bit 3)
    // on the decoder's convT forwards (128 -> 64 113.2 -> 90.1 us, 32 -> 128 34.6 -> 26.0; train step 3.48-3.49 ->
    // 3.40-3.44 ms): default 11.  Bit 2: the single-phase window form for the 4-tap phases whatever their density.
    // Bit 4 (round 5): the 16-tap convs with a 128-row pack on 128-row window tiles (four waves along the rows):
    // the decoder convT 128 -> 64's data gradient 134.2 -> 100.8 us, train step 3.33-3.34 -> 3.28-3.31 ms
    // (gpurun_out/k16): default 27.
    static const int win = [] {
        const char* e = std::getenv("LDM_TCONV_WIN");
        return e ? (int)std::strtol(e, nullptr, 0) : 27;
    }();
    if (win) {
        const bool k16 = a.pt.nphase == 1 && a.pt.ntap[0] == 16;
        const bool k3t = a.pt.nphase == 4 && a.pt.ntap[0] == 1 && a.pt.ntap[3] == 4;   // k3 s2 op1 transposed
        const bool k4t = a.pt.nphase == 4 && a.pt.ntap[0] == 4 && a.pt.ntap[3] == 4 && (win & 8);   // k4 s2 p1
        if (((k3t || k4t) && (win & 2)) || (!k3t && (win & 1))) {
            tc::TArgs t = a;
            // bit 4: a 16-tap conv with a 128-row pack keeps it (four waves along the rows, WNW 1: 16 taps x one
            // row tile of weight fragments per wave fit the registers the 2 x 2 grid's two row tiles did not)
            const bool k16w = k16 && p.tm == 2 && (win & 16);
            const bool r64 = (k16 && !k16w) || k3t || k4t;   // the 64-row tilings (their image needs 5 slots / 4 acc sets)
            if (r64 && p.tm == 2) t.nM = a.Mpad / 64;   // the 128-row pack is also a valid 64-row tiling
            const int rc = tc::forward_window(d, t, r64 ? 64 : 64 * p.tm, p.tn, s, (win & 4) != 0, k4t);
            if (rc != 1) return rc;
        }
    }
    const dim3 g((unsigned)blocks);
#define TCK(BM_, DT_)                                                                          \
    do {                                                                                       \
        if (ep.x16) hipLaunchKernelGGL((tc::tconv_kernel<BM_, DT_, DT_>), g, dim3(256), 0, s, a); \
        else hipLaunchKernelGGL((tc::tconv_kernel<BM_, DT_, 0>), g, dim3(256), 0, s, a);        \
    } while (0)
    if (p.tm == 2) {
        if (p.tn == LDM_DT_F16) TCK(128, 1);
        else TCK(128, 2);
    } else {
        if (p.tn == LDM_DT_F16) TCK(64, 1);
        else TCK(64, 2);
    }
#undef TCK
    LDM_CHECK_LAUNCH("tconv_kernel");
    return 0;
}

}  // namespace ldm

using namespace ldm;

extern "C" int ldm_conv_tiled_plan(const ldm_conv_desc* d, int32_t dtype, ldm_conv_plan* plan) {
    if (!d || !plan) return fail(2, "conv_tiled_plan: null argument");
    return tconv_plan(*d, dtype, *plan) ? 0 : 1;
}
