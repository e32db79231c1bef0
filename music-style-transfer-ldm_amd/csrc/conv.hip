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
#include <type_traits>
#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "conv_epi.h"

#pragma clang fp contract(off)

#ifndef LDM_DIAG
#define LDM_DIAG 0
#endif

namespace ldm {

// mask-and-or select (a ?: chain is turned into branches by the compiler); single-phase kernels
// (PH4 = false) read slot 0 only, which keeps 27 scalars of kernarg traffic out of their prologue
template <bool PH4 = true>
__device__ __forceinline__ int sel_phase(const int32_t (&v)[kMaxPhase], int ph) {
    if constexpr (!PH4) return v[0];
    const int x0 = v[0], x1 = v[1], x2 = v[2], x3 = v[3];
    return (x0 & -(int)(ph == 0)) | (x1 & -(int)(ph == 1)) | (x2 & -(int)(ph == 2)) | (x3 & -(int)(ph == 3));
}

// ------------------------------------------------------------------------------------------------
// phase / tap tables
// ------------------------------------------------------------------------------------------------
int build_phase_table(const ldm_conv_desc& d, PhaseTable& pt) {
    pt = PhaseTable{};
    // unused tap slots point far outside any input: the kernel can scan all kMaxTap slots branch-free
    for (int p = 0; p < kMaxPhase; ++p)
        for (int t = 0; t < kMaxTap; ++t) pt.dy[p][t] = -0x4000;
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
    // the 4 consecutive k of a lane's fragment as one reduced-precision MFMA (32x32x8)
    template <int DT>
    static __device__ __forceinline__ acc_t mma4(floatx4 a, floatx4 b, acc_t c) { return mma32_lowp<DT>(a, b, c); }
};

template <>
struct Mfma<2> {
    static constexpr int TILE = 16, NLG = 4, NACC = 4;
    typedef floatx4 acc_t;
    static __device__ __forceinline__ acc_t mma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int r, int lg) { return 4 * lg + r; }
    template <int DT>
    static __device__ __forceinline__ acc_t mma4(floatx4 a, floatx4 b, acc_t c) { return mma16_lowp<DT>(a, b, c); }
};

constexpr int kMaxKSplit = 16;   // blocks splitting K (ldm_conv_plan.ks)
constexpr int kMaxConvLds = 160 * 1024;   // gfx950 LDS per CU (dynamic LDS above 64 KiB is opted into per kernel)

template <int TM, int TN>
struct Frag {
    floatx4 a[TM];
    float b[TN][4];
};

// ------------------------------------------------------------------------------------------------
// kinds 1/2: block = WK waves over one (TILE*TM x TILE*TN) output tile of one phase; the ks blocks of a
// tile and the WK waves of a block deal the K-chunks round-robin, register-pipelined in groups of
// kGroup chunks per wave.
// ------------------------------------------------------------------------------------------------
#ifndef LDM_DIAG   // diagnostic builds only (timing experiments, never shipped): 4 = per-block phase
#define LDM_DIAG 0 // timestamps (tools/stamp_probe.py); 8 = no K-loop operand loads (MFMAs on register
#endif             // garbage: the kernel's cost without its operand traffic)
#if (LDM_DIAG & 4)
__device__ unsigned long long g_ldm_stamps[1 << 16][6];
#define LDM_STAMP(k)                                                                               \
    do {                                                                                           \
        if (threadIdx.x == 0 && blockIdx.x < (1u << 16))                                          \
            g_ldm_stamps[blockIdx.x][k] = ((k) == 0 || (k) == 5) ? __builtin_amdgcn_s_memrealtime()           \
                                                                 : __builtin_amdgcn_s_memtime();          \
    } while (0)
#else
#define LDM_STAMP(k) \
    do {             \
    } while (0)
#endif

// Partial-tile hand-off between the ks blocks of one output tile (cross-block split-K).  Stores and
// loads are agent-scope relaxed atomics, i.e. `global_store/load ... sc1`: written through past the
// writer's L2 and read past the reader's L1, so no release / acquire fence (each ~1.7 us on gfx950)
// is needed — MI355X_MICROARCH.md "Workgroup dispatch ... Valid forms", first table row.
__device__ __forceinline__ void part_store(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float part_load(const float* p) {
    return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// NT = tap slots scanned per phase (1 for 1x1 projections, 4 for transposed-conv phases, 9 for 3x3,
// 16 for 4x4): the per-lane tap offsets are precomputed for NT slots only.
// DT: operand precision (0 fp32; 2 bf16 operands with fp32 accumulation, NCHW instances only).
template <int KIND, int TM, int TN, int WK, int NT, bool NHWC, int DT>
__global__ __launch_bounds__(64 * WK) void conv_mfma_kernel(ConvArgs a) {
    LDM_STAMP(0);
    using MF = Mfma<KIND>;
    constexpr bool PH4 = NT == 4;   // the 4-phase (stride-2 transposed) instances; all others are 1-phase
    // prefetch depth scaled to the register tile: 8 chunks per group for 1x1 tiles, 4 for 2x1, 2 for
    // 2x2 (the same register budget; short K loops then expose one memory latency, not one per group)
    constexpr int kGroup = TM * TN == 1 ? 8 : (TM * TN == 2 ? 4 : 2);
    constexpr int TILE = MF::TILE, NLG = MF::NLG, CK = 4 * NLG;
    constexpr int BM = TILE * TM, BN = TILE * TN;
    constexpr int LDB = BN + 1, SLAB = BM * LDB;   // LDS partial tile [BM][BN+1]: conflict-free both ways
    extern __shared__ __attribute__((aligned(16))) float smem[];
    __shared__ int s_last;
    const int lane = threadIdx.x & 63;
    // wave index made provably uniform: chunk / tap indices then live in SGPRs and the tap-table
    // lookups below are scalar kernarg loads (lgkmcnt), not per-lane global loads that would force a
    // vmcnt(0) drain of the prefetched operands on every chunk.
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int HqWq = a.pt.Hq * a.pt.Wq;
    const int Nq = a.B * HqWq;
    // XCD-aware tile order (bijective for any grid size): the dispatcher deals blocks round-robin over
    // the 8 XCDs, so block b lands with the blocks b' = b mod 8.  Renumber so that each such group gets
    // a contiguous run of tiles: phase fastest (transposed-conv phases differ in tap count, so every
    // XCD gets the same mix), then along the operand that is cheaper to re-fetch.  Weight-heavy layers
    // (a.xcd_nfast) walk N first, so one weight row-block's N-tiles share an XCD's L2 and the packed
    // weights are fetched once per launch instead of once per XCD; activation-heavy layers walk M
    // first, so the M-tiles reading the same input columns share it.  The M index is extended by the
    // K split (mt' = mt * ks + s): blocks with the same weight slice (mt, s) are the ones grouped.
    int ph, mt, nt, ksp;
    {
        // (divisions by host-precomputed multiply-high constants: no runtime integer division; both
        // orders are computed and selected arithmetically — a branch on tile_order splits the kernarg
        // loads of the prologue into dependent rounds)
        const int nwg = gridDim.x, orig = blockIdx.x;
        // natural order: N-tile fastest, then M-tile', then phase
        const int rest = a.fd_nn.div(orig);
        const int nt0 = orig - rest * a.fd_nn.d;
        const int ph0 = PH4 ? a.fd_nm.div(rest) : 0;
        const int mx0 = rest - ph0 * a.fd_nm.d;
        // XCD-grouped order
        const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
        const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
        const int tile = PH4 ? (wgid >> 2) : wgid;
        const int ph1 = PH4 ? (wgid & 3) : 0;
        const int outer = a.fd_inner.div(tile);
        const int inner = tile - outer * a.fd_inner.d;
        const int o = a.tile_order;
        const int m0_ = -(int)(o == 0), m1_ = -(int)(o == 1), m2_ = -(int)(o == 2);
        ph = (ph0 & m0_) | (ph1 & ~m0_);
        const int mtx = (mx0 & m0_) | (outer & m1_) | (inner & m2_);
        nt = (nt0 & m0_) | (inner & m1_) | (outer & m2_);
        mt = a.fd_ks.div(mtx);
        ksp = mtx - mt * a.ks;
        if constexpr (PH4) {
            if (a.balance) {
                // phase-balanced split: phase p's tiles are split ks_p = ks * ntap_p ways, so every block
                // carries the same K; consecutive (XCD-grouped) blocks walk one phase's N-tiles, then its
                // (M-tile, split) pairs
                const int p = (int)(wgid >= a.bofs[1]) + (int)(wgid >= a.bofs[2]) + (int)(wgid >= a.bofs[3]);
                const int local = wgid - sel_phase<true>(a.bofs, p);
                const int lks = sel_phase<true>(a.bks_log2, p);
                const int r2 = a.fd_nn.div(local);
                nt = local - r2 * a.fd_nn.d;
                mt = r2 >> lks;
                ksp = r2 - (mt << lks);
                ph = p;
            }
        }
    }
    // K splits of this block's tile (ks_p in balance mode), and the partial-tile slots per tile
    const int ksn = uni((PH4 && a.balance) ? 1 << sel_phase<PH4>(a.bks_log2, ph) : a.ks);
    const int m0 = mt * BM, n0 = nt * BN;
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
        const int iyv = qy * a.pt.sy;
        iy0[ni] = nv ? iyv : -0x4000000;
        ix0[ni] = qx * a.pt.sy;
        // lane group lg holds k-local 4*lg + j at MFMA step j: channels 4*lg .. 4*lg+3 of each chunk,
        // which NHWC stores contiguously (one 16-byte load per chunk instead of four 4-byte ones)
        base4[ni] = NHWC ? (((b * a.Hin + iyv) * a.Win + ix0[ni]) * a.Cin + 4 * lg) * 4
                         : ((b * a.Cin + 4 * lg) * HWin + iyv * a.Win + ix0[ni]) * 4;
    }

    typename MF::acc_t acc[TM][TN];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni)
#pragma unroll
            for (int r = 0; r < MF::NACC; ++r) acc[mi][ni][r] = 0.f;

    const int cpt = a.Cin / CK;   // chunks per tap
    const int nchunk = sel_phase<PH4>(a.pk.kchunks, ph);
    const int ph_ry = sel_phase<PH4>(a.pk.ry, ph), ph_rx = sel_phase<PH4>(a.pk.rx, ph);
    const int wstride_b = a.Mpad * CK * 4;                 // bytes per packed chunk
    // K chunks are dealt round-robin over the ks*WK waves that share this output tile: wave `wave` of
    // split `ksp` owns chunks g, g + G, g + 2G, ...
    const int G = uni(ksn * WK), g = uni(ksp * WK + wave);
    const int nmine = nchunk > g ? uni((nchunk - g + G - 1) / G) : 0;
    const int ngrp = (nmine + kGroup - 1) / kGroup;
    // (uniform values pinned to SGPRs with readfirstlane: a buffer resource or soffset that the
    // compiler parks in a VGPR turns every load into a waterfall loop)
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(uni_ptr(a.x), (short)0, uni(a.B * a.Cin * HWin * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(a.w + sel_phase<PH4>(a.pk.wofs, ph)), (short)0, uni(nchunk * wstride_b), 0x00020000);
    const int a_voff = ((m0 + col) * CK + lg * 4) * 4;
    const int cstep_b = NHWC ? CK * 4 : CK * HWin * 4;     // bytes per channel chunk in x
    const int tap_mul = NHWC ? a.Cin * 4 : 4;              // bytes per input pixel step

    constexpr int EPT = (BM * BN + 64 * WK - 1) / (64 * WK);
    constexpr bool kPre = EPT <= 8;
    EpiPre pre[kPre ? EPT : 1];
    int po[kPre ? EPT : 1], pm[kPre ? EPT : 1], ps[kPre ? EPT : 1];
    // epilogue element e of the tile -> (mloc, nloc): consecutive threads walk the output's contiguous
    // dimension (n for NCHW, m = channel for NHWC) so the stores coalesce
    const bool onhwc = a.out_nhwc != 0;
    auto elem = [&](int e, int& mloc, int& nloc) {
        const int nl_c = e / BM, ml_c = e - nl_c * BM;   // NHWC order
        const int ml_n = e / BN, nl_n = e - ml_n * BN;   // NCHW order
        mloc = onhwc ? ml_c : ml_n;
        nloc = onhwc ? nl_c : nl_n;
    };

    // Epilogue operands of the outputs this thread will finish (element e = tid + k*64*WK of the tile),
    // issued first so their latency (and that of the epilogue pointers' kernarg reads) overlaps the
    // offset precompute below and the K loop (all index math in 32 bits: the tensors are < 2^31
    // elements, checked on the host).  With a K split only the last-arriving block runs the epilogue,
    // so nobody prefetches.
    LDM_STAMP(1);
    if constexpr (kPre) {
        // (issued unconditionally — with a K split only the last block runs the epilogue, and its
        // sources get zero records instead, so the loads return 0 without touching memory)
        const EpiSrc esrc = epi_sources(a, ksn == 1);
        {
#pragma unroll
            for (int k = 0; k < EPT; ++k) {
                const int e = (int)threadIdx.x + k * 64 * WK;
                int mloc, nloc;
                elem(e, mloc, nloc);
                const int m = m0 + mloc, n = n0 + nloc;
                const bool valid = e < BM * BN && m < a.Cout && n < Nq;
                const int mm = valid ? m : 0, nn = valid ? n : 0;
                const int b = a.fd_hw.div(nn);
                const int r = nn - b * HqWq;
                const int qyy = a.fd_w.div(r);
                const int qxx = r - qyy * a.pt.Wq;
                const int oy = qyy * a.pt.osy + ph_ry, ox = qxx * a.pt.osy + ph_rx;
                const int oidx = out_index(a, mm, b, oy, ox);
                const int boff = (a.ep.pos_bias ? mm * a.Hout * a.Wout + oy * a.Wout + ox : mm) * 4;
                pre[k] = epi_prefetch_buf(esrc, a.Cout, mm, b, oidx, boff);
                po[k] = valid ? oidx : -1;
                pm[k] = mm;
                ps[k] = mloc * LDB + nloc;
            }
        }
    }

    // Per-tap input offsets of this lane's columns, computed once: a tap change in the K loop is a
    // register pick by a wave-uniform index (no tap-table loads, no divergent branch, no VALU temps
    // that could alias prefetched registers).
    // (taps generated arithmetically from the phase's (dy0, dx0, na, nb) — no table loads; slots past
    // na*nb are out of window)
#ifndef LDM_TAP_ARITH
#define LDM_TAP_ARITH 1
#endif
    // tap t -> (dy, dx) = (dy0 + sg*ja, dx0 + sg*jb), (ja, jb) = divmod(t, nb), nb <= 4, t < 16
    const int tp_dy0 = sel_phase<PH4>(a.pk.dy0, ph), tp_dx0 = sel_phase<PH4>(a.pk.dx0, ph);
    const int tp_nb = sel_phase<PH4>(a.pk.nb, ph), tp_ntap = sel_phase<PH4>(a.pk.na, ph) * tp_nb;
    const int tp_mul = uni((32 + tp_nb - 1) / tp_nb), tp_sg = a.pk.sg;
    const int tp_win = a.Win, tp_hin = a.Hin;
    auto tap_off = [&](int t, int ni) {   // per-lane byte offset of tap t for column ni (kOOB if padding)
        const int ja = uni((t * tp_mul) >> 5), jb = uni(t - ja * tp_nb);
        const int dy = uni(t < tp_ntap ? tp_dy0 + tp_sg * ja : -0x4000), dx = uni(tp_dx0 + tp_sg * jb);
        const bool ok = (unsigned)(iy0[ni] + dy) < (unsigned)tp_hin && (unsigned)(ix0[ni] + dx) < (unsigned)tp_win;
        return ok ? base4[ni] + (dy * tp_win + dx) * tap_mul : kOOB;
    };
    int vtap[LDM_TAP_ARITH ? 1 : NT][TN];
    if constexpr (!LDM_TAP_ARITH) {
        const int dy0 = tp_dy0, dx0 = tp_dx0, nb = tp_nb;
        const int sg = a.pk.sg, ntap = tp_ntap;
        int ja = 0, jb = 0;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int dy = t < ntap ? dy0 + sg * ja : -0x4000;
            const int dx = dx0 + sg * jb;
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) {
                const bool ok = (unsigned)(iy0[ni] + dy) < (unsigned)a.Hin && (unsigned)(ix0[ni] + dx) < (unsigned)a.Win;
                vtap[t][ni] = ok ? base4[ni] + (dy * a.Win + dx) * tap_mul : kOOB;
            }
            const bool wrap = jb + 1 == nb;
            jb = wrap ? 0 : jb + 1;
            ja += wrap ? 1 : 0;
        }
    }

    // The K cursor is branch-free scalar arithmetic: chunk c = g + G*i -> (tap t, channel chunk cc) by
    // a multiply-high division.  Loads are unconditional; a chunk past this wave's range loads from
    // out-of-range offsets (the hardware returns 0 without touching memory) and its MFMAs are skipped
    // by a wave-uniform branch (measured: the padding MFMAs of short K loops cost up to 1.6x the
    // useful ones).
    constexpr int kSkipA = 0x40000000;   // soffset past any packed weight buffer
    // K cursor of this wave (wave-uniform, SGPRs), advanced incrementally chunk by chunk in issue order:
    // chunk c = g + G*i sits at tap t = c / cpt, channel chunk cc = c % cpt, packed-weight byte offset
    // c * wstride_b.  (A per-chunk division and the liveness selects cost ~25 scalar instructions per
    // chunk, issued in one block ahead of the group's MFMAs.)
    int cur_t = uni(a.fd_cpt.div(g));
    int cur_cc = uni(g - cur_t * cpt);
    int cur_sa = uni(g * wstride_b);
    const int adv_t = uni(G / cpt), adv_cc = uni(G - (G / cpt) * cpt), adv_sa = uni(G * wstride_b);
    // ALL_LIVE: every chunk of the group is one of this wave's (no liveness selects, no clamping)
    auto load = [&](Frag<TM, TN>(&f)[kGroup], int grp, auto all_live) {
        constexpr bool ALL_LIVE = decltype(all_live)::value;
#pragma unroll
        for (int q = 0; q < kGroup; ++q) {
            const bool live = ALL_LIVE || grp * kGroup + q < nmine;
            const int t_ld = ALL_LIVE ? cur_t : uni(cur_t < NT - 1 ? cur_t : NT - 1);
            const int soff_a = uni(live ? cur_sa : kSkipA);
            const int soff_b = uni(live ? cur_cc * cstep_b : kSkipA);
            cur_sa += adv_sa;
            cur_t += adv_t;
            cur_cc += adv_cc;
            const bool wrap = cur_cc >= cpt;
            cur_cc = uni(wrap ? cur_cc - cpt : cur_cc);
            cur_t = uni(cur_t + (wrap ? 1 : 0));
            int voff[TN];
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) voff[ni] = LDM_TAP_ARITH ? tap_off(t_ld, ni) : vtap[LDM_TAP_ARITH ? 0 : t_ld][ni];
#pragma unroll
            for (int mi = 0; mi < TM; ++mi) {
                if constexpr (LDM_DIAG & 8) {
                    const float g0 = (float)(soff_a + mi) * 1e-30f;
                    f[q].a[mi] = floatx4{g0, g0, g0, g0};
                } else {
                    f[q].a[mi] = __builtin_bit_cast(
                        floatx4, __builtin_amdgcn_raw_buffer_load_b128(wr, a_voff + mi * TILE * CK * 4, soff_a, 0));
                }
            }
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) {
                if constexpr (LDM_DIAG & 8) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) f[q].b[ni][j] = (float)(voff[ni] + soff_b + j) * 1e-30f;
                } else if constexpr (NHWC) {
                    const floatx4 v = __builtin_bit_cast(
                        floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, voff[ni], soff_b, 0));
#pragma unroll
                    for (int j = 0; j < 4; ++j) f[q].b[ni][j] = v[j];
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        f[q].b[ni][j] = __builtin_bit_cast(
                            float, __builtin_amdgcn_raw_buffer_load_b32(xr, voff[ni], uni(soff_b + j * HWin * 4), 0));
                }
            }
        }
    };
    // 16x16x4 f32 has a 40-cycle dependent latency vs a 32-cycle issue: a lone accumulator chain
    // alternates two accumulators (summed before the reduction).
    constexpr int NCH = (KIND == 2 && TM * TN == 1) ? 2 : 1;
    typename MF::acc_t acc2[TM][TN];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni)
#pragma unroll
            for (int r = 0; r < MF::NACC; ++r) acc2[mi][ni][r] = 0.f;
    auto compute = [&](const Frag<TM, TN>(&f)[kGroup], int grp, auto all_live) {
#pragma unroll
        for (int q = 0; q < kGroup; ++q) {
            if (!decltype(all_live)::value && grp * kGroup + q >= nmine) break;   // wave-uniform: no MFMAs on padding
            if constexpr (LDM_DIAG & 16) {          // diagnostic: no MFMAs either (fixed cost only)
                acc[0][0][0] = acc[0][0][0] + f[q].a[0][0] * f[q].b[0][0];
                continue;
            }
            if constexpr (DT != 0) {   // fp16 / bf16 operands: a lane's 4 consecutive k in one MFMA
#pragma unroll
                for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni) {
                        const floatx4 bv = {f[q].b[ni][0], f[q].b[ni][1], f[q].b[ni][2], f[q].b[ni][3]};
                        if (NCH == 2 && (q & 1)) acc2[mi][ni] = MF::template mma4<DT>(f[q].a[mi], bv, acc2[mi][ni]);
                        else acc[mi][ni] = MF::template mma4<DT>(f[q].a[mi], bv, acc[mi][ni]);
                    }
                continue;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni) {
                        if (NCH == 2 && (j & 1))
                            acc2[mi][ni] = MF::mma(f[q].a[mi][j], f[q].b[ni][j], acc2[mi][ni]);
                        else
                            acc[mi][ni] = MF::mma(f[q].a[mi][j], f[q].b[ni][j], acc[mi][ni]);
                    }
        }
    };

    // Group pairs: an odd group count is padded with one all-zero group, so the loop has no tail and
    // every register in flight keeps one home across iterations (a tail compute after the loop makes
    // the compiler rotate the prefetch registers with copies, and a copy waits for its load).
    Frag<TM, TN> f0[kGroup], f1[kGroup];
    LDM_STAMP(2);
    // Groups past this wave's range are not loaded at all: an out-of-range buffer load moves no data
    // but still costs texture-address cycles, and with short K loops padding groups were ~half of all
    // vector-memory instructions (rocprofv3 TA_BUSY).  The steady-state loop runs while both next
    // groups are full (no liveness checks, unconditional loads, so the waitcnt pass keeps the next
    // group in flight across each compute); the last <= 3 groups are peeled.
    using Live = std::true_type;
    using Maybe = std::false_type;
    const int nfull = nmine / kGroup;
    if (ngrp > 0) load(f0, 0, Maybe{});
    int gi = 0;
    for (; gi + 2 < nfull; gi += 2) {
        load(f1, gi + 1, Live{});
        compute(f0, gi, Live{});
        load(f0, gi + 2, Live{});
        compute(f1, gi + 1, Live{});
    }
    while (gi < ngrp) {   // tail: group gi is in f0
        if (gi + 1 < ngrp) {
            load(f1, gi + 1, Maybe{});
            compute(f0, gi, Maybe{});
            if (gi + 2 < ngrp) load(f0, gi + 2, Maybe{});
            compute(f1, gi + 1, Maybe{});
            gi += 2;
        } else {
            compute(f0, gi, Maybe{});
            gi += 1;
        }
    }
    if constexpr (NCH == 2) {
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
            for (int ni = 0; ni < TN; ++ni)
#pragma unroll
                for (int r = 0; r < MF::NACC; ++r) acc[mi][ni][r] = acc[mi][ni][r] + acc2[mi][ni][r];
    }
    LDM_STAMP(3);

    // in-block split-K partial tiles -> LDS, fixed-order sum over the WK waves
    float* sw = smem + wave * SLAB;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni)
#pragma unroll
            for (int r = 0; r < MF::NACC; ++r)
                sw[(TILE * mi + MF::row(r, lg)) * LDB + TILE * ni + col] = acc[mi][ni][r];
    __syncthreads();
    LDM_STAMP(4);
    if (ksn == 1) {
        if constexpr (kPre) {
#pragma unroll
            for (int k = 0; k < EPT; ++k) {
                if (po[k] < 0) continue;
                const int si = ps[k];
                float v = smem[si];
#pragma unroll
                for (int w = 1; w < WK; ++w) v = v + smem[w * SLAB + si];
                epi_finish(a, pm[k], (size_t)po[k], v, pre[k]);
            }
        } else {
            for (int e = threadIdx.x; e < BM * BN; e += 64 * WK) {
                int mloc, nloc;
                elem(e, mloc, nloc);
                const int m = m0 + mloc, n = n0 + nloc;
                if (m >= a.Cout || n >= Nq) continue;
                const int si = mloc * LDB + nloc;
                float v = smem[si];
#pragma unroll
                for (int w = 1; w < WK; ++w) v = v + smem[w * SLAB + si];
                const int b = n / HqWq;
                const int r = n - b * HqWq;
                const int qyy = r / a.pt.Wq;
                const int qxx = r - qyy * a.pt.Wq;
                epilogue_store(a, m, b, qyy * a.pt.osy + ph_ry, qxx * a.pt.osy + ph_rx, v);
            }
        }
        LDM_STAMP(5);
        return;
    }

    // Cross-block split-K: publish this block's partial tile, count arrivals; the block that arrives
    // last sums the ks partials in split order (bitwise independent of arrival order) and runs the
    // fused epilogue.  No block waits for another: nothing here can hang.
    const int tile = (ph * a.nM + mt) * a.nN + nt;
    float* tpart = a.part + (size_t)tile * a.ks * (BM * BN);
    for (int e = threadIdx.x; e < BM * BN; e += 64 * WK) {
        int mloc, nloc;
        elem(e, mloc, nloc);
        const int si = mloc * LDB + nloc;
        float v = smem[si];
#pragma unroll
        for (int w = 1; w < WK; ++w) v = v + smem[w * SLAB + si];
        part_store(tpart + (size_t)ksp * (BM * BN) + e, v);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int old = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == ksn - 1;
        if (last) __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    for (int e = threadIdx.x; e < BM * BN; e += 64 * WK) {
        int mloc, nloc;
        elem(e, mloc, nloc);
        const int m = m0 + mloc, n = n0 + nloc;
        if (m >= a.Cout || n >= Nq) continue;
        const int si = mloc * LDB + nloc;
        float own = smem[si];
#pragma unroll
        for (int w = 1; w < WK; ++w) own = own + smem[w * SLAB + si];
        float pv[kMaxKSplit];
#pragma unroll
        for (int s2 = 0; s2 < kMaxKSplit; ++s2)
            if (s2 < ksn && s2 != ksp) pv[s2] = part_load(tpart + (size_t)s2 * (BM * BN) + e);
        float v = ksp == 0 ? own : pv[0];
#pragma unroll
        for (int s2 = 1; s2 < kMaxKSplit; ++s2)
            if (s2 < ksn) v = v + (s2 == ksp ? own : pv[s2]);
        const int b = n / HqWq;
        const int r = n - b * HqWq;
        const int qyy = r / a.pt.Wq;
        const int qxx = r - qyy * a.pt.Wq;
        epilogue_store(a, m, b, qyy * a.pt.osy + ph_ry, qxx * a.pt.osy + ph_rx, v);
    }
    LDM_STAMP(5);
}
#if (LDM_DIAG & 4)
extern "C" int ldm_debug_stamps(unsigned long long* host, int nblocks) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ldm_stamps), sizeof(unsigned long long) * 6 * nblocks, 0,
                                    hipMemcpyDeviceToHost);
}
#endif

// ------------------------------------------------------------------------------------------------
// kind 0: direct VALU conv (Cin not a multiple of 8, or tiny Cout: VAE first/last layers)
// ------------------------------------------------------------------------------------------------
// One output per lane, 32-bit index arithmetic by multiply-high (the host guarantees < 2^31 outputs): the
// 64-bit div/mod chains of a per-lane decomposition cost more than the arithmetic of these thin layers.
// The phase table is indexed by a per-lane phase (the output parity of a transposed conv): it is copied
// to LDS once per block, since a kernarg array indexed by a VGPR compiles to per-lane global loads.  The
// taps' offsets and validity are resolved first, so that each channel's tap loads are independent (no
// branch between them) and issue back to back.
__global__ __launch_bounds__(256) void conv_direct_kernel(ConvArgs a) {
    __shared__ int tab[kMaxPhase * kMaxTap * 3 + kMaxPhase];   // dy, dx, kk [phase][tap], ntap[phase]
    for (int i = threadIdx.x; i < kMaxPhase * kMaxTap * 3 + kMaxPhase; i += blockDim.x) {
        const int which = i / (kMaxPhase * kMaxTap), e = i - which * (kMaxPhase * kMaxTap);
        const int ph = e / kMaxTap, t = e - ph * kMaxTap;
        tab[i] = which == 0 ? a.pt.dy[ph][t] : which == 1 ? a.pt.dx[ph][t] : which == 2 ? a.pt.kk[ph][t]
                                                                                      : a.pt.ntap[e < kMaxPhase ? e : 0];
    }
    __syncthreads();
    const int total = a.B * a.Cout * a.Hout * a.Wout;
    const int idx = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (idx >= total) return;
    int rest = a.fd_dwo.div(idx);
    const int ox = idx - rest * a.Wout;
    int r2 = a.fd_dho.div(rest);
    const int oy = rest - r2 * a.Hout;
    const int b = a.fd_dco.div(r2);
    const int co = r2 - b * a.Cout;
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
    const int wci = a.transposed ? a.Cout * a.KK : a.KK;
    const float* wb = a.w + (a.transposed ? (size_t)co * a.KK : (size_t)co * a.Cin * a.KK);
    const int nt = tab[kMaxPhase * kMaxTap * 3 + ph];
    int off[kMaxTap], wkk[kMaxTap];
    bool ok[kMaxTap];
#pragma unroll
    for (int t = 0; t < kMaxTap; ++t) {
        const int e = ph * kMaxTap + t;
        const int iy = qy * a.pt.sy + tab[e];
        const int ix = qx * a.pt.sy + tab[kMaxPhase * kMaxTap + e];
        ok[t] = t < nt && iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win;
        off[t] = ok[t] ? iy * a.Win + ix : 0;
        wkk[t] = t < nt ? tab[2 * kMaxPhase * kMaxTap + e] : 0;
    }
    float acc = 0.f;
    for (int ci = 0; ci < a.Cin; ++ci) {
        const float* xp = xb + (size_t)ci * HWin;
        const float* wq = wb + (size_t)ci * wci;
        float xv[kMaxTap], wv[kMaxTap];
#pragma unroll
        for (int t = 0; t < kMaxTap; ++t) {   // (operands rounded to the autocast type, as the MFMA kernels do)
            xv[t] = round16(t < nt ? xp[off[t]] : 0.f, a.ep.lowp);
            wv[t] = round16(t < nt ? wq[wkk[t]] : 0.f, a.ep.lowp);
        }
#pragma unroll
        for (int t = 0; t < kMaxTap; ++t)
            if (ok[t]) acc = fmaf(xv[t], wv[t], acc);
    }
    epilogue_store(a, co, b, oy, ox, acc);
}

// Cin -> 1 conv, k3 s1 p1 (the UNet's dec1 on a raw mel, SURVEY shape S: 64 -> 1 on 128 x 512 at B = 1).
// conv_direct_kernel gives such a layer one lane per output (65,536 lanes = 1 wave per SIMD) walking all Cin x 9
// taps serially: 240 us per launch for 16.8 MB of input.  Here a lane owns 4 adjacent outputs of a row (their
// 3 x 6 window per channel: one 16-byte load and two scalars per row) and one of G = 8 channel groups; the G
// partial sums of a quad meet in LDS in group order.  Each output's sum: per group, channels ascending, taps in
// window order (fmaf), then the groups in order — a fixed order, so bitwise reproducible.
constexpr int kC1Groups = 8;
__global__ __launch_bounds__(256) void conv_cout1_k3_kernel(ConvArgs a) {
    constexpr int G = kC1Groups, QB = 256 / G;   // channel groups, output quads per block
    __shared__ float wsm[512 * 9];
    __shared__ float4 red[G][QB];
    const int Cin = a.Cin;
    for (int i = threadIdx.x; i < Cin * 9; i += 256) wsm[i] = round16(a.w[i], a.ep.lowp);   // [ci][ky*3 + kx]
    __syncthreads();
    const int g = threadIdx.x / QB, ql = threadIdx.x - g * QB;
    const int wq = a.Wout >> 2;
    const int quad = blockIdx.x * QB + ql;
    const int nquad = a.B * a.Hout * wq;
    const bool qv = quad < nquad;
    const int qq = qv ? quad : 0;
    const int rest = a.fd_dwo.div(qq);   // (b, oy)
    const int ox0 = (qq - rest * wq) * 4;
    const int b = a.fd_dho.div(rest);
    const int oy = rest - b * a.Hout;
    const int HW = a.Hin * a.Win;
    const int cpg = Cin / G;
    const float* xb = a.x + ((size_t)b * Cin + (size_t)g * cpg) * HW;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    bool rok[3];
    int roff[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const int iy = oy - 1 + r;
        rok[r] = iy >= 0 && iy < a.Hin;
        roff[r] = (rok[r] ? iy : 0) * a.Win + ox0;
    }
    const bool lok = ox0 > 0, rgt = ox0 + 4 < a.Win;
    for (int c = 0; c < cpg; ++c) {
        const float* xp = xb + (size_t)c * HW;
        const float* wc = wsm + (g * cpg + c) * 9;
        float win[3][6];
#pragma unroll
        for (int r = 0; r < 3; ++r) {   // loads first (no branch around them: the masks apply after)
            const float4 m = *reinterpret_cast<const float4*>(xp + roff[r]);
            const float l = xp[roff[r] + (lok ? -1 : 0)], rr = xp[roff[r] + (rgt ? 4 : 0)];
            win[r][0] = rok[r] && lok ? l : 0.f;
            win[r][1] = rok[r] ? m.x : 0.f;
            win[r][2] = rok[r] ? m.y : 0.f;
            win[r][3] = rok[r] ? m.z : 0.f;
            win[r][4] = rok[r] ? m.w : 0.f;
            win[r][5] = rok[r] && rgt ? rr : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx)
                    acc[j] = fmaf(round16(win[ky][j + kx], a.ep.lowp), wc[ky * 3 + kx], acc[j]);
    }
    red[g][ql] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    __syncthreads();
    if (g != 0 || !qv) return;
    float4 s = red[0][ql];
#pragma unroll
    for (int k = 1; k < G; ++k) {
        const float4 t = red[k][ql];
        s.x = s.x + t.x, s.y = s.y + t.y, s.z = s.z + t.z, s.w = s.w + t.w;
    }
    epilogue_store(a, 0, b, oy, ox0 + 0, s.x);
    epilogue_store(a, 0, b, oy, ox0 + 1, s.y);
    epilogue_store(a, 0, b, oy, ox0 + 2, s.z);
    epilogue_store(a, 0, b, oy, ox0 + 3, s.w);
}

// Single-input-channel conv (the VAE encoder's and the style encoder's first layers, 1 -> 64 on 128x512
// mels): one lane per output pixel computes every output channel from one k x k window read, with the
// Cout x k*k weights in LDS; the stores stay coalesced (consecutive lanes = consecutive ox per channel).
__global__ __launch_bounds__(256) void conv_cin1_kernel(ConvArgs a) {
    __shared__ float ws[64 * 16];
    for (int i = threadIdx.x; i < a.Cout * a.KK; i += blockDim.x) ws[i] = round16(a.w[i], a.ep.lowp);   // [co][kh*kw]
    __syncthreads();
    const int total = a.B * a.Hout * a.Wout;
    const int idx = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (idx >= total) return;
    const int rest = a.fd_dwo.div(idx);
    const int ox = idx - rest * a.Wout;
    const int b = a.fd_dho.div(rest);
    const int oy = rest - b * a.Hout;
    const float* xb = a.x + (size_t)b * a.Hin * a.Win;
    float xv[kMaxTap];
    bool ok[kMaxTap];
    const int nt = a.pt.ntap[0];
#pragma unroll
    for (int t = 0; t < kMaxTap; ++t) {
        const int iy = oy * a.pt.sy + a.pt.dy[0][t];
        const int ix = ox * a.pt.sy + a.pt.dx[0][t];
        ok[t] = t < nt && iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win;
        xv[t] = round16(xb[ok[t] ? iy * a.Win + ix : 0], a.ep.lowp);
    }
    for (int co = 0; co < a.Cout; ++co) {
        float acc = 0.f;
#pragma unroll
        for (int t = 0; t < kMaxTap; ++t)
            if (ok[t]) acc = fmaf(xv[t], ws[co * a.KK + a.pt.kk[0][t]], acc);
        epilogue_store(a, co, b, oy, ox, acc);
    }
}

// ------------------------------------------------------------------------------------------------
// Thin VAE layers at full mel resolution (B = 32 in the train step: 134 MB activations each), four
// adjacent output columns per lane so that every store is one 16-byte store and each input window is
// loaded once for 4 (or 16) outputs.  Simple epilogues only (bias, eval-BN, act, act_out: the host
// routes anything else to the kernels above); arithmetic and accumulation order equal conv_cin1_kernel /
// conv_direct_kernel's, so the results are the same bits.
// ------------------------------------------------------------------------------------------------
// the operand / output rounding modes of EpiArgs as compile-time constants: f(lp, ro) with integral_constants,
// ro in {0, lp} (round_out is either off or the operand type)
template <class F>
static void lp_dispatch(const EpiArgs& e, F&& f) {
    using Z = std::integral_constant<int, 0>;
    using H = std::integral_constant<int, LDM_DT_F16>;
    using Bf = std::integral_constant<int, LDM_DT_BF16>;
    if (e.lowp == LDM_DT_BF16) {
        if (e.round_out) f(Bf{}, Bf{}); else f(Bf{}, Z{});
    } else if (e.lowp == LDM_DT_F16) {
        if (e.round_out) f(H{}, H{}); else f(H{}, Z{});
    } else {
        f(Z{}, Z{});
    }
}

struct ChanEpi {
    float bias, alpha, beta;
};
__device__ __forceinline__ ChanEpi chan_epi(const ConvArgs& a, int m) {
    const EpiArgs& e = a.ep;
    ChanEpi c{0.f, 1.f, 0.f};
    if (e.bias) c.bias = e.bias[m];
    if (e.bn_w) {   // as epi_finish
        const float invstd = 1.0f / sqrtf(e.bn_v[m] + e.bn_eps);
        c.alpha = invstd * e.bn_w[m];
        c.beta = e.bn_b[m] - e.bn_m[m] * c.alpha;
    }
    return c;
}
// RO: the output rounding (a.ep.round_out) as a template argument, so that the VALU kernels below carry no
// per-element mode test (they do a few FMAs per output; a runtime round16 costs as much as the conv)
template <int RO>
__device__ __forceinline__ float chan_apply(const ConvArgs& a, const ChanEpi& c, float v) {
    constexpr int ro = RO;
    if (a.ep.bias) v = v + c.bias;
    v = round16(v, ro);
    if (a.ep.bn_w) v = round16(v * c.alpha + c.beta, ro);
    return round16(apply_act(v, a.ep.act), ro);
}
// YS: 0 fp32 outputs, else the 16-bit storage type of y / act_out (LDM_DT_Y16)
template <int YS = 0>
__device__ __forceinline__ void store4(const ConvArgs& a, size_t o, const float (&v)[4]) {
    if constexpr (YS != 0) {
        if (a.ep.act_out) st_st<YS, 4>(a.ep.act_out, o, true, v);
        st_st<YS, 4>(a.y, o, true, v);
    } else {
        const float4 t = make_float4(v[0], v[1], v[2], v[3]);
        if (a.ep.act_out) *reinterpret_cast<float4*>(a.ep.act_out + o) = t;
        *reinterpret_cast<float4*>(a.y + o) = t;
    }
}

// Cin = 1, stride SD = 2, k x k (the VAE / style encoders' first layers, and the data gradient of the decoder's
// 64 -> 1 output layer): lane = (b, oy, 4 output columns), its K x (3 SD + K) input window in registers,
// every output channel from it, weights in LDS.  SD = 1 (round 6): the UNet's first layer on the raw mel
// (shape S, UNet(1, 1): 1 -> 32, k3 s1 on 128 x 512), which ran on conv_cin1_kernel (one lane per pixel).
// PK = 1 (round 6): two output channels per packed FMA.  v_pk_fma_f32 computes each half exactly as v_fma_f32
// does, so each output's chain fma(x, w, acc) over (ky, kx) is the scalar form's, bit for bit; the halves are
// channels co and co + 1 (their weights one aligned 8-byte LDS read from a [tap][channel] copy), the input value
// the same register for both (op_sel).  Round 5's packed attempt paired the FOUR OUTPUT COLUMNS instead; the
// columns' inputs win[ky][kx + 2j] are not register pairs, and that variant failed the config-3 parity bound —
// which fma rounding cannot explain.
template <int K, int LP, int RO, int YS, int PK = 0, int SD = 2>
__global__ __launch_bounds__(256) void conv_cin1_x4_kernel(ConvArgs a) {
    __shared__ float ws[64 * K * K];
    __shared__ __attribute__((aligned(8))) float wt[PK ? K * K * 64 : 1];   // PK: [ky*K + kx][co]
    __shared__ ChanEpi es[64];   // per-channel epilogue constants, formed once per block (not per lane and channel)
    for (int i = threadIdx.x; i < a.Cout * K * K; i += blockDim.x) {
        const float w = round16(a.w[i], LP);
        ws[i] = w;   // [co][ky*K + kx]
        if constexpr (PK != 0) wt[(i % (K * K)) * 64 + i / (K * K)] = w;
    }
    for (int i = threadIdx.x; i < a.Cout; i += blockDim.x) es[i] = chan_epi(a, i);
    __syncthreads();
    const int W4 = a.Wout >> 2;
    const int idx = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (idx >= a.B * a.Hout * W4) return;
    const int r = a.fd_dwo.div(idx);   // fd_dwo = W4 here
    const int ox0 = (idx - r * W4) * 4;
    const int b = a.fd_dho.div(r);
    const int oy = r - b * a.Hout;
    constexpr int NC = 3 * SD + K;
    const int pad = -a.pt.dy[0][0];
    const int iy0 = SD * oy - pad, ix0 = SD * ox0 - pad;
    const float* xb = a.x + (size_t)b * a.Hin * a.Win;
    float win[K][NC];
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
        const int iy = iy0 + ky;
        const bool rok = (unsigned)iy < (unsigned)a.Hin;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int ix = ix0 + c;
            const bool ok = rok && (unsigned)ix < (unsigned)a.Win;
            win[ky][c] = round16(ok ? xb[iy * a.Win + ix] : 0.f, LP);
        }
    }
    // the output channels [c0, c1) of this block (gridDim.y > 1 splits them when the pixel grid alone is under
    // a block per CU: B = 1 at shape S; the host keeps Cout / gridDim.y even)
    const int cpb = a.Cout / (int)gridDim.y, c0 = (int)blockIdx.y * cpb, c1 = c0 + cpb;
    const size_t plane = (size_t)a.Hout * a.Wout;
    size_t o = (((size_t)b * a.Cout + c0) * a.Hout + oy) * a.Wout + ox0;
    if constexpr (PK != 0) {   // (the host takes this form for an even Cout only)
        typedef float f2 __attribute__((ext_vector_type(2)));
        for (int co = c0; co < c1; co += 2, o += 2 * plane) {
            f2 acc[4] = {f2{0.f, 0.f}, f2{0.f, 0.f}, f2{0.f, 0.f}, f2{0.f, 0.f}};
#pragma unroll
            for (int ky = 0; ky < K; ++ky)
#pragma unroll
                for (int kx = 0; kx < K; ++kx) {
                    const f2 w2 = *reinterpret_cast<const f2*>(wt + (ky * K + kx) * 64 + co);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float xv = win[ky][kx + SD * j];
                        acc[j] = __builtin_elementwise_fma(f2{xv, xv}, w2, acc[j]);
                    }
                }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const ChanEpi ce = es[co + h];
                float v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = chan_apply<RO>(a, ce, acc[j][h]);
                store4<YS>(a, o + h * plane, v);
            }
        }
        return;
    }
    for (int co = c0; co < c1; ++co, o += plane) {
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ky = 0; ky < K; ++ky)
#pragma unroll
            for (int kx = 0; kx < K; ++kx) {
                const float w = ws[co * K * K + ky * K + kx];
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[j] = fmaf(win[ky][kx + SD * j], w, acc[j]);
            }
        const ChanEpi ce = es[co];
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = chan_apply<RO>(a, ce, acc[j]);
        store4<YS>(a, o, v);
    }
}

// conv_cout1_k3_kernel for the Cin -> 1 k3 s1 convs (LDM_COUT1=0: conv_direct_kernel, A/B timing)
static bool cout1_on() {
    static const bool on = [] {
        const char* e = std::getenv("LDM_COUT1");
        return !e || std::atoi(e) != 0;
    }();
    return on;
}

// the packed form of conv_cin1_x4_kernel: LDM_CIN1_PK (default 1: the B = 32 first layer 48.5 -> 44.6 us per
// launch, gpurun_out/r6b1), or ldm_set_cin1_packed; LDM_CIN1_PK=0 keeps the scalar form
static int g_cin1_packed = [] {
    const char* e = std::getenv("LDM_CIN1_PK");
    return e ? std::atoi(e) : 1;
}();

// conv_cin1_x4_kernel's stride-1 form for the k3 Cin = 1 convs (LDM_CIN1_S1=0 or ldm_set_cin1_s1(0):
// conv_cin1_kernel, for A/B timing and the bitwise test)
static int g_cin1_s1 = [] {
    const char* e = std::getenv("LDM_CIN1_S1");
    return e ? std::atoi(e) : 1;
}();
static bool cin1_s1_on() { return g_cin1_s1 != 0; }

// ConvTranspose2d(Cin -> 1, k4, s2, p1) (the decoder's output layer): lane = (b, qy, 4 input columns
// qx0..qx0+3) -> the 2 x 8 outputs they feed (all four parities); per input channel a 3 x 6 window.
// Taps in the phase-table order of build_phase_table: parity r uses kernel rows {1, 3} (r = 0, input
// offsets 0, -1) or {0, 2} (r = 1, offsets +1, 0).
__host__ __device__ constexpr int ct4_tap(int r, int i) { return r == 0 ? (i == 0 ? 1 : 3) : (i == 0 ? 0 : 2); }
__host__ __device__ constexpr int ct4_off(int r, int i) { return (r + 1 - ct4_tap(r, i)) >> 1; }

template <int LP, int RO, int XS>
__global__ __launch_bounds__(256) void convT4_cout1_kernel(ConvArgs a) {
    const int W4 = a.Win >> 2;
    const int idx = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (idx >= a.B * a.Hin * W4) return;
    const int r = a.fd_dwo.div(idx);   // fd_dwo = W4 here
    const int qx0 = (idx - r * W4) * 4;
    const int b = a.fd_dho.div(r);     // fd_dho = Hin here
    const int qy = r - b * a.Hin;
    const int HW = a.Hin * a.Win;
    float acc[2][8];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
    bool rok[3], cok[6];
#pragma unroll
    for (int i = 0; i < 3; ++i) rok[i] = (unsigned)(qy - 1 + i) < (unsigned)a.Hin;
#pragma unroll
    for (int c = 0; c < 6; ++c) cok[c] = (unsigned)(qx0 - 1 + c) < (unsigned)a.Win;
    const float* xp = a.x + (size_t)b * a.Cin * HW + (qy - 1) * a.Win + (qx0 - 1);
    for (int ci = 0; ci < a.Cin; ++ci, xp += HW) {
        float xr[3][6];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int c = 0; c < 6; ++c)
                xr[i][c] = (rok[i] && cok[c]) ? (XS ? ld1_st<XS>(a.x, (size_t)(xp - a.x) + i * a.Win + c, true)
                                                    : round16(xp[i * a.Win + c], LP))
                                              : 0.f;
        const float* wq = a.w + ci * 16;   // w [Cin][1][4][4]
#pragma unroll
        for (int ry = 0; ry < 2; ++ry)
#pragma unroll
            for (int rx = 0; rx < 2; ++rx)
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int ia = t >> 1, ib = t & 1;
                    const int dy = ct4_off(ry, ia), dx = ct4_off(rx, ib);
                    const float w = round16(wq[ct4_tap(ry, ia) * 4 + ct4_tap(rx, ib)], LP);
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
                        acc[ry][2 * jj + rx] = fmaf(xr[1 + dy][1 + jj + dx], w, acc[ry][2 * jj + rx]);
                }
    }
    const ChanEpi ce = chan_epi(a, 0);
#pragma unroll
    for (int ry = 0; ry < 2; ++ry) {
        const size_t o = ((size_t)b * a.Hout + 2 * qy + ry) * a.Wout + 2 * qx0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = chan_apply<RO>(a, ce, acc[ry][4 * h + j]);
            store4(a, o + 4 * h, v);
        }
    }
}

// The same layer with two input rows per lane (four output rows x 8 columns): per input channel a lane
// reads its four window rows as one 16-byte run plus the two border columns (12 loads for two rows instead
// of 36 single-float gathers), and the channel loop keeps two channels of loads in flight.  Hin even.
template <int LP, int RO, int XS>
__global__ __launch_bounds__(256) void convT4_cout1_r2_kernel(ConvArgs a) {
    const int W4 = a.Win >> 2, H2 = a.Hin >> 1;
    const int idx = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (idx >= a.B * H2 * W4) return;
    const int r = a.fd_dwo.div(idx);   // fd_dwo = W4
    const int qx0 = (idx - r * W4) * 4;
    const int b = a.fd_dho.div(r);     // fd_dho = Hin / 2
    const int qy0 = (r - b * H2) * 2;
    const int HW = a.Hin * a.Win;
    float acc[2][2][8];   // [input row][ry][2 jj + rx]
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[u][i][j] = 0.f;
    bool rok[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) rok[i] = (unsigned)(qy0 - 1 + i) < (unsigned)a.Hin;
    const bool lok = qx0 > 0, hok = qx0 + 4 < a.Win;
    const float* xp = a.x + (size_t)b * a.Cin * HW + (qy0 - 1) * a.Win + qx0;
    auto load = [&](const float* p, float (&xr)[4][6]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float* row = p + i * a.Win;
            if constexpr (XS != 0) {   // 16-bit storage: the operands are in the MFMA-free VALU type already
                const size_t ro_ = (size_t)(row - a.x);
                float m[4] = {0.f, 0.f, 0.f, 0.f};
                if (rok[i]) ld_st<XS, 4>(a.x, ro_, true, m);
                xr[i][0] = (rok[i] && lok) ? ld1_st<XS>(a.x, ro_ - 1, true) : 0.f;
                xr[i][1] = m[0], xr[i][2] = m[1], xr[i][3] = m[2], xr[i][4] = m[3];
                xr[i][5] = (rok[i] && hok) ? ld1_st<XS>(a.x, ro_ + 4, true) : 0.f;
            } else {
                const float4 m = rok[i] ? *reinterpret_cast<const float4*>(row) : make_float4(0.f, 0.f, 0.f, 0.f);
                xr[i][0] = (rok[i] && lok) ? row[-1] : 0.f;
                xr[i][1] = m.x, xr[i][2] = m.y, xr[i][3] = m.z, xr[i][4] = m.w;
                xr[i][5] = (rok[i] && hok) ? row[4] : 0.f;
#pragma unroll
                for (int c = 0; c < 6; ++c) xr[i][c] = round16(xr[i][c], LP);
            }
        }
    };
    auto mac = [&](const float (&xr)[4][6], const float* wq) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int ry = 0; ry < 2; ++ry)
#pragma unroll
                for (int rx = 0; rx < 2; ++rx)
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const int ia = t >> 1, ib = t & 1;
                        const int dy = ct4_off(ry, ia), dx = ct4_off(rx, ib);
                        const float w = round16(wq[ct4_tap(ry, ia) * 4 + ct4_tap(rx, ib)], LP);
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj)
                            acc[u][ry][2 * jj + rx] = fmaf(xr[1 + u + dy][1 + jj + dx], w, acc[u][ry][2 * jj + rx]);
                    }
    };
    float xa[4][6], xb[4][6];
    int ci = 0;
    for (; ci + 1 < a.Cin; ci += 2, xp += 2 * HW) {   // channel order kept: ci, then ci + 1
        load(xp, xa);
        load(xp + HW, xb);
        mac(xa, a.w + ci * 16);
        mac(xb, a.w + (ci + 1) * 16);
    }
    if (ci < a.Cin) {
        load(xp, xa);
        mac(xa, a.w + ci * 16);
    }
    const ChanEpi ce = chan_epi(a, 0);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int ry = 0; ry < 2; ++ry) {
            const size_t o = ((size_t)b * a.Hout + 2 * (qy0 + u) + ry) * a.Wout + 2 * qx0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = chan_apply<RO>(a, ce, acc[u][ry][4 * h + j]);
                store4(a, o + 4 * h, v);
            }
        }
}

// The same tiles with the input channels split over the block's four waves (Cin % 8 == 0): wave g sums the
// quarter g * Cin / 4 .. of the channels for the 64 tiles of its block, then the quarters meet in LDS in wave
// order.  At B = 32 the two-rows-per-lane kernel has 65,536 lanes, one 4-wave block per CU walking all 64
// channels in a chain of dependent loads (119 us per launch); here 4x the waves walk a quarter each.
template <int LP, int RO, int XS>
__global__ __launch_bounds__(256, 4) void convT4_cout1_r2s_kernel(ConvArgs a) {
    __shared__ float part[3][32][64];
    const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int W4 = a.Win >> 2, H2 = a.Hin >> 1;
    const int idx = (int)(blockIdx.x * 64 + lane);
    const bool valid = idx < a.B * H2 * W4;
    const int id = valid ? idx : 0;
    const int r = a.fd_dwo.div(id);   // fd_dwo = W4
    const int qx0 = (id - r * W4) * 4;
    const int b = a.fd_dho.div(r);     // fd_dho = Hin / 2
    const int qy0 = (r - b * H2) * 2;
    const int HW = a.Hin * a.Win;
    const int cq = a.Cin >> 2, c0 = g * cq;
    float acc[2][2][8];   // [input row][ry][2 jj + rx]
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[u][i][j] = 0.f;
    bool rok[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) rok[i] = valid && (unsigned)(qy0 - 1 + i) < (unsigned)a.Hin;
    const bool lok = qx0 > 0, hok = qx0 + 4 < a.Win;
    const float* xp = a.x + ((size_t)b * a.Cin + c0) * HW + (qy0 - 1) * a.Win + qx0;
    auto load = [&](const float* p, float (&xr)[4][6]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float* row = p + i * a.Win;
            if constexpr (XS != 0) {   // 16-bit storage: the operands are in the MFMA-free VALU type already
                const size_t ro_ = (size_t)(row - a.x);
                float m[4] = {0.f, 0.f, 0.f, 0.f};
                if (rok[i]) ld_st<XS, 4>(a.x, ro_, true, m);
                xr[i][0] = (rok[i] && lok) ? ld1_st<XS>(a.x, ro_ - 1, true) : 0.f;
                xr[i][1] = m[0], xr[i][2] = m[1], xr[i][3] = m[2], xr[i][4] = m[3];
                xr[i][5] = (rok[i] && hok) ? ld1_st<XS>(a.x, ro_ + 4, true) : 0.f;
            } else {
                const float4 m = rok[i] ? *reinterpret_cast<const float4*>(row) : make_float4(0.f, 0.f, 0.f, 0.f);
                xr[i][0] = (rok[i] && lok) ? row[-1] : 0.f;
                xr[i][1] = m.x, xr[i][2] = m.y, xr[i][3] = m.z, xr[i][4] = m.w;
                xr[i][5] = (rok[i] && hok) ? row[4] : 0.f;
#pragma unroll
                for (int c = 0; c < 6; ++c) xr[i][c] = round16(xr[i][c], LP);
            }
        }
    };
    auto mac = [&](const float (&xr)[4][6], const float* wq) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int ry = 0; ry < 2; ++ry)
#pragma unroll
                for (int rx = 0; rx < 2; ++rx)
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const int ia = t >> 1, ib = t & 1;
                        const int dy = ct4_off(ry, ia), dx = ct4_off(rx, ib);
                        const float w = round16(wq[ct4_tap(ry, ia) * 4 + ct4_tap(rx, ib)], LP);
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj)
                            acc[u][ry][2 * jj + rx] = fmaf(xr[1 + u + dy][1 + jj + dx], w, acc[u][ry][2 * jj + rx]);
                    }
    };
    // cq even; channel order kept within the quarter.  No register prefetch of the next pair: without it the
    // kernel fits 128 VGPRs, so the 1024 blocks of B = 32 are resident at once (4 waves per SIMD) instead of
    // 3 + 1 rounds at 164 VGPRs, and the other waves hide the loads
    float xa[4][6], xb[4][6];
    for (int ci = c0; ci < c0 + cq; ci += 2, xp += 2 * HW) {
        load(xp, xa);
        load(xp + HW, xb);
        mac(xa, a.w + ci * 16);
        mac(xb, a.w + (ci + 1) * 16);
    }
    if (g > 0) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 8; ++j) part[g - 1][u * 16 + i * 8 + j][lane] = acc[u][i][j];
    }
    __syncthreads();
    if (g > 0 || !valid) return;
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[u][i][j] = acc[u][i][j] + part[q][u * 16 + i * 8 + j][lane];
    const ChanEpi ce = chan_epi(a, 0);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int ry = 0; ry < 2; ++ry) {
            const size_t o = ((size_t)b * a.Hout + 2 * (qy0 + u) + ry) * a.Wout + 2 * qx0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = chan_apply<RO>(a, ce, acc[u][ry][4 * h + j]);
                store4(a, o + 4 * h, v);
            }
        }
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
    const int k = c * ck + 4 * lg + j;   // MFMA step j, lane group lg <- k-local 4*lg + j (see the kernel)
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
    a.out_nhwc = (d.layout >> 1) & 1;
    // weights vs input bytes: group tiles on an XCD along the operand that is larger
    a.xcd_nfast = (int64_t)d.Cout * d.Cin * d.kh * d.kw > (int64_t)d.B * d.Cin * d.Hin * d.Win;
    a.fd_hw = FastDiv::make(a.pt.Hq * a.pt.Wq);
    a.fd_w = FastDiv::make(a.pt.Wq);
    a.fd_cpt = FastDiv::make(p.kind ? d.Cin / chunk_k(p.kind) : 1);
    a.fd_np = FastDiv::make(a.pt.nphase);
    // per-phase scalars + the arithmetic tap form (dy0 + sg*ja, dx0 + sg*jb), verified against the table
    a.pk = {};
    a.pk.sg = d.transposed ? -1 : 1;
    for (int ph = 0; ph < a.pt.nphase; ++ph) {
        const int n = a.pt.ntap[ph];
        int nb = 1;
        while (nb < n && a.pt.dy[ph][nb] == a.pt.dy[ph][0]) ++nb;
        LDM_REQUIRE(n % nb == 0, "conv: tap table is not a rectangle");
        a.pk.ry[ph] = a.pt.ry[ph];
        a.pk.rx[ph] = a.pt.rx[ph];
        a.pk.dy0[ph] = a.pt.dy[ph][0];
        a.pk.dx0[ph] = a.pt.dx[ph][0];
        a.pk.na[ph] = n / nb;
        a.pk.nb[ph] = nb;
        for (int t = 0; t < n; ++t)
            LDM_REQUIRE(a.pt.dy[ph][t] == a.pk.dy0[ph] + a.pk.sg * (t / nb) &&
                            a.pt.dx[ph][t] == a.pk.dx0[ph] + a.pk.sg * (t % nb),
                        "conv: tap table not in (dy0 + sg*ja, dx0 + sg*jb) order");
        a.pk.kchunks[ph] = a.pt.kchunks[ph];
        LDM_REQUIRE(a.pt.wofs[ph] < 0x7fffffff, "conv: packed weights too large");
        a.pk.wofs[ph] = (int32_t)a.pt.wofs[ph];
    }
    // tile order: XCD-grouped N-fast for weight-heavy layers (measured: bottleneck -12 %, dec4 -9 %),
    // natural order otherwise; LDM_TILE_ORDER=0/1/2 forces one (experiments)
    a.tile_order = a.xcd_nfast ? 1 : 0;
    if (const char* env = std::getenv("LDM_TILE_ORDER")) a.tile_order = std::atoi(env) % 3;
    int nN = 1, nM = 1;
    if (p.kind) {
        const int bm = tile_m(p.kind) * p.tm, bn = tile_m(p.kind) * p.tn;
        nN = (int)(((int64_t)d.B * a.pt.Hq * a.pt.Wq + bn - 1) / bn);
        nM = (d.Cout + bm - 1) / bm;
    }
    a.ks = p.kind ? std::max(1, (int)p.ks) : 1;
    a.nN = nN;
    a.nM = nM;
    a.balance = p.kind && p.balance;
    for (int i = 0; i < kMaxPhase; ++i) a.bofs[i] = a.bks_log2[i] = 0;
    if (a.balance) {
        int ofs = 0, kmax = 1;
        for (int ph = 0; ph < a.pt.nphase; ++ph) {
            const int ksp = a.ks * a.pt.ntap[ph];
            int l2 = 0;
            while ((1 << l2) < ksp) ++l2;
            a.bofs[ph] = ofs;
            a.bks_log2[ph] = l2;
            ofs += nN * nM * ksp;
            kmax = std::max(kmax, ksp);
        }
        a.nblocks_bal = ofs;
        a.ks = kmax;   // partial slots per tile
    }
    a.fd_ks = FastDiv::make(a.ks);
    a.fd_inner = FastDiv::make(a.tile_order == 1 ? nN : nM * a.ks);
    a.fd_nn = FastDiv::make(nN);
    a.fd_nm = FastDiv::make(nM * a.ks);
    return 0;
}

// Workspace of a split-K plan: a fixed region of kSplitCounters int32 arrival counters (one per output
// tile, all phases), then ks partial tiles of BM x BN floats per output tile.  The counter region has
// the same size and place for every plan, so one zero-filled workspace can serve any sequence of
// plans: partials never land on a counter word, and every launch leaves its counters zero.
constexpr int64_t kSplitCounters = 1 << 16;

static int64_t split_tiles(const ldm_conv_desc& d, const ldm_conv_plan& p, const PhaseTable& pt) {
    const int bm = tile_m(p.kind) * p.tm, bn = tile_m(p.kind) * p.tn;
    const int64_t nN = ((int64_t)d.B * pt.Hq * pt.Wq + bn - 1) / bn;
    const int64_t nM = (d.Cout + bm - 1) / bm;
    return nN * nM * pt.nphase;
}

static int split_slots(const ldm_conv_plan& p, const PhaseTable& pt) {
    int k = p.ks;
    if (p.balance)
        for (int i = 0; i < pt.nphase; ++i) k = std::max(k, p.ks * pt.ntap[i]);
    return k;
}

static int64_t split_ws_floats(const ldm_conv_desc& d, const ldm_conv_plan& p, const PhaseTable& pt) {
    if (p.kind == 0 || split_slots(p, pt) <= 1) return 0;
    const int bm = tile_m(p.kind) * p.tm, bn = tile_m(p.kind) * p.tn;
    return kSplitCounters + split_tiles(d, p, pt) * split_slots(p, pt) * bm * bn;
}

static bool plan_ok(const ldm_conv_desc& d, int kind, int tm, int tn, int wk, int ks) {
    if (d.layout & ~3) return false;
    if (kind == 0) return ks == 1 && d.layout == 0;   // the direct VALU kernel is NCHW only
    if (kind != 1 && kind != 2) return false;
    if (tm < 1 || tm > 2 || tn < 1 || tn > 2) return false;
    if (wk != 1 && wk != 2 && wk != 4 && wk != 8) return false;
    if (ks < 1 || ks > kMaxKSplit || (ks & (ks - 1))) return false;
    if (d.Cin % chunk_k(kind) != 0) return false;
    const int bm = tile_m(kind) * tm, bn = tile_m(kind) * tn;
    if ((int64_t)wk * bm * (bn + 1) * 4 > kMaxConvLds) return false;
    return true;
}

}  // namespace ldm

using namespace ldm;

extern "C" int ldm_conv_make_plan_forced(const ldm_conv_desc* d, int kind, int tm, int tn, int wk, int ks,
                                         ldm_conv_plan* plan) {
    LDM_REQUIRE(d && plan, "conv plan: null argument");
    const bool balance = ks < 0;   // ks = -k: phase-balanced split (4-phase layers), base k
    if (balance) ks = -ks;
    LDM_REQUIRE(plan_ok(*d, kind, tm, tn, wk, ks), "conv plan: unsupported (kind, tm, tn, wk, ks) for this layer");
    ldm_conv_plan p{};
    p.kind = kind;
    p.tm = kind ? tm : 1;
    p.tn = kind ? tn : 1;
    p.wk = kind ? wk : 1;
    p.ks = kind ? ks : 1;
    p.balance = balance ? 1 : 0;
    PhaseTable pt;
    int Mpad;
    int64_t floats;
    int rc = layout_for_plan(*d, p, pt, Mpad, floats);
    if (rc) return rc;
    if (balance) {
        LDM_REQUIRE(kind != 0 && pt.nphase == 4, "conv plan: a phase-balanced split needs a 4-phase (stride-2 transposed) layer");
        for (int i = 0; i < 4; ++i)
            LDM_REQUIRE(pt.ntap[i] > 0 && (pt.ntap[i] & (pt.ntap[i] - 1)) == 0 && ks * pt.ntap[i] <= kMaxKSplit,
                        "conv plan: phase-balanced split needs power-of-two taps per phase and ks*taps <= 16");
    }
    p.packed_floats = floats;
    LDM_REQUIRE(split_slots(p, pt) == 1 || split_tiles(*d, p, pt) <= kSplitCounters, "conv plan: too many tiles for a K split");
    p.ws_floats = split_ws_floats(*d, p, pt);
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
    if (d->Cin % 8 != 0 || M < 16) return ldm_conv_make_plan_forced(d, 0, 1, 1, 1, 1, plan);
    // Heuristic (refined by the Python-side autotuner): fill >= ~2048 waves (2 per SIMD).
    auto tiles_for = [&](int kind, int tm, int tn) {
        const int bm = tile_m(kind) * tm, bn = tile_m(kind) * tn;
        return (int64_t)((M + bm - 1) / bm) * ((Nq + bn - 1) / bn) * pt.nphase;
    };
    int kind = (M >= 32 && Nq >= 32) ? 1 : 2;
    if (kind == 2 && d->Cin % 16 != 0) return ldm_conv_make_plan_forced(d, 0, 1, 1, 1, 1, plan);
    int64_t tiles = tiles_for(kind, 1, 1);
    if (kind == 1 && tiles * 8 < 1024 && d->Cin % 16 == 0) {
        kind = 2;
        tiles = tiles_for(kind, 1, 1);
    }
    const int64_t chunks = (int64_t)maxtap * (d->Cin / chunk_k(kind));
    int wk = 1;
    while (wk < 8 && tiles * wk < 2048 && chunks / (wk * 2) >= 2) wk *= 2;
    return ldm_conv_make_plan_forced(d, kind, 1, 1, wk, 1, plan);
}

extern "C" int ldm_conv_pack_weight(const ldm_conv_desc* d, const ldm_conv_plan* plan, const float* w, float* packed,
                                    void* stream) {
    LDM_REQUIRE(d && plan && w, "conv pack: null argument");
    if (plan->kind == 0) return 0;
    LDM_REQUIRE(packed, "conv pack: null output");
    if (plan->kind == 3) return tconv_pack(*d, *plan, w, packed, (hipStream_t)stream);
    if (plan->kind == 4) {   // sconv.hip reads the kind-3 pack with 64-row padding
        ldm_conv_plan k3 = *plan;
        k3.kind = 3, k3.tm = 1;
        return tconv_pack(*d, k3, w, packed, (hipStream_t)stream);
    }
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

namespace ldm {
int conv_pack_job(const ldm_conv_desc& d, const ldm_conv_plan& p, PackJob& j) {
    LDM_REQUIRE(p.kind == 1 || p.kind == 2, "pack job: not an MFMA plan");
    ConvArgs a;
    int rc = make_args(d, p, a);
    if (rc) return rc;
    j.kind = p.kind;
    j.dt = 0;
    j.Cin = a.Cin;
    j.Cout = a.Cout;
    j.KK = a.KK;
    j.transposed = a.transposed;
    j.Mpad = a.Mpad;
    j.nphase = a.pt.nphase;
    for (int q = 0; q < kMaxPhase; ++q) {
        j.ntap[q] = a.pt.ntap[q];
        j.wofs[q] = a.pt.wofs[q];
        for (int t = 0; t < kMaxTap; ++t) j.kk[q][t] = a.pt.kk[q][t];
    }
    j.total = p.packed_floats;
    return 0;
}
}  // namespace ldm

template <int KIND, int NT, bool NHWC, int DT>
static int launch_mfma_nt(const ConvArgs& a, const ldm_conv_plan& p, int64_t Nq, hipStream_t st) {
    const int TILE = Mfma<KIND>::TILE;
    const int BMx = TILE * p.tm, BNx = TILE * p.tn;
    const size_t lds = (size_t)p.wk * BMx * (BNx + 1) * sizeof(float);
    // 1-D grid, tile order remapped XCD-aware inside the kernel
    dim3 grid((unsigned)(a.balance ? a.nblocks_bal
                                   : ((Nq + BNx - 1) / BNx) * ((a.Cout + BMx - 1) / BMx) * a.ks * a.pt.nphase));
    dim3 block(64 * p.wk);
    const int code = (p.tm - 1) * 2 + (p.tn - 1);
#define LDM_CASE(WK, C, TM, TN)                                                                              \
    case WK * 10 + C: {                                                                                      \
        auto kfn = conv_mfma_kernel<KIND, TM, TN, WK, NT, NHWC, DT>;                                        \
        if (lds > 64 * 1024) {                                                                               \
            static size_t opted = 0;                                                                         \
            if (opted < lds) {                                                                               \
                LDM_HIP_TRY(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                                (int)lds));                                                  \
                opted = lds;                                                                                 \
            }                                                                                                \
        }                                                                                                    \
        hipLaunchKernelGGL(kfn, grid, block, lds, st, a);                                                    \
        break;                                                                                               \
    }
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

template <int KIND, bool NHWC, int DT>
static int launch_mfma(const ConvArgs& a, const ldm_conv_plan& p, int64_t Nq, hipStream_t st) {
    int maxtap = 0;
    for (int i = 0; i < a.pt.nphase; ++i) maxtap = std::max(maxtap, a.pt.ntap[i]);
    // NT = 4 <=> the 4-phase kernels (kMaxTap per phase of a stride-2 transposed conv with k <= 4 is 4)
    if (a.pt.nphase == 4) {
        if (maxtap > 4) return fail(3, "conv: 4-phase layer with more than 4 taps per phase");
        return launch_mfma_nt<KIND, 4, NHWC, DT>(a, p, Nq, st);
    }
    if (a.pt.nphase != 1) return fail(3, "conv: unsupported phase count");
    if (maxtap <= 1) return launch_mfma_nt<KIND, 1, NHWC, DT>(a, p, Nq, st);
    if (maxtap <= 9) return launch_mfma_nt<KIND, 9, NHWC, DT>(a, p, Nq, st);
    return launch_mfma_nt<KIND, 16, NHWC, DT>(a, p, Nq, st);
}

namespace ldm {

int conv_forward_ex(const ldm_conv_desc& d, const ldm_conv_plan& p, const float* x, const float* w, const EpiArgs& ep,
                    float* y, float* ws, hipStream_t st) {
    LDM_REQUIRE(x && w && (y || ep.ddim_coef), "conv forward: null argument");
    LDM_REQUIRE(p.ws_floats == 0 || ws, "conv forward: this plan splits K across blocks and needs a workspace");
    LDM_REQUIRE(!ep.ddim_coef || ep.ddim_x, "conv forward: fused DDIM update needs x");
    if (p.kind == 3) return tconv_forward(d, p, x, w, ep, y, st);
    if (p.kind == 4) return sconv_forward(d, p, x, w, ep, y, st);
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
        LDM_REQUIRE(d.layout == 0, "conv: the direct kernel supports NCHW tensors only");
        const int64_t total = (int64_t)d.B * d.Cout * d.Hout * d.Wout;
        LDM_REQUIRE(total < 0x7fffffffLL, "conv: the direct kernel indexes outputs in 32 bits");
        a.fd_dwo = FastDiv::make(d.Wout);
        a.fd_dho = FastDiv::make(d.Hout);
        a.fd_dco = FastDiv::make(d.Cout);
        const bool simple_epi = !ep.pos_bias && !ep.bcast && !ep.skip && !ep.ddim_coef && y;
        if (simple_epi && d.Cin == 1 && !d.transposed && d.Cout <= 64 && d.kh == d.kw &&
            ((d.stride == 2 && (d.kh == 3 || d.kh == 4)) || (d.stride == 1 && d.kh == 3 && cin1_s1_on())) && d.Wout % 4 == 0 && a.pt.dy[0][0] == -d.pad && a.pt.dx[0][0] == -d.pad &&
            ((uintptr_t)y & 15) == 0 && (!ep.act_out || ((uintptr_t)ep.act_out & 15) == 0)) {
            a.fd_dwo = FastDiv::make(d.Wout / 4);
            const int64_t lanes = (int64_t)d.B * d.Hout * (d.Wout / 4);
            LDM_REQUIRE(!ep.x16, "conv: the Cin = 1 kernel reads fp32 inputs only");
            const bool pk = g_cin1_packed != 0 && d.Cout % 2 == 0;
            // under 512 pixel blocks (B = 1 at shape S: 64): split the output channels over grid.y
            // (each split re-reads its lanes' windows; the arithmetic per output is unchanged)
            const int64_t pblocks = (lanes + 255) / 256;
            int csplit = 1;
            while (pblocks * csplit < 512 && d.Cout % (csplit * 4) == 0 && d.Cout / (csplit * 2) >= 4) csplit *= 2;
            lp_dispatch(a.ep, [&](auto lp, auto ro) {
                constexpr int LP = decltype(lp)::value, RO = decltype(ro)::value;
                const dim3 g((unsigned)pblocks, (unsigned)csplit);
                auto go = [&](auto pkc) {
                    constexpr int PK = decltype(pkc)::value;
                    if (d.stride == 1) {
                        if (LP != 0 && ep.y16) hipLaunchKernelGGL((conv_cin1_x4_kernel<3, LP, RO, LP, PK, 1>), g, dim3(256), 0, st, a);
                        else hipLaunchKernelGGL((conv_cin1_x4_kernel<3, LP, RO, 0, PK, 1>), g, dim3(256), 0, st, a);
                    } else if (LP != 0 && ep.y16) {
                        if (d.kh == 3) hipLaunchKernelGGL((conv_cin1_x4_kernel<3, LP, RO, LP, PK>), g, dim3(256), 0, st, a);
                        else hipLaunchKernelGGL((conv_cin1_x4_kernel<4, LP, RO, LP, PK>), g, dim3(256), 0, st, a);
                    } else {
                        if (d.kh == 3) hipLaunchKernelGGL((conv_cin1_x4_kernel<3, LP, RO, 0, PK>), g, dim3(256), 0, st, a);
                        else hipLaunchKernelGGL((conv_cin1_x4_kernel<4, LP, RO, 0, PK>), g, dim3(256), 0, st, a);
                    }
                };
                if (pk) go(std::integral_constant<int, 1>{}); else go(std::integral_constant<int, 0>{});
            });
            LDM_CHECK_LAUNCH("conv_cin1_x4_kernel");
            return 0;
        }
        if (simple_epi && !ep.y16 && d.transposed && d.Cout == 1 && d.kh == 4 && d.kw == 4 && d.stride == 2 && d.pad == 1 &&
            d.out_pad == 0 && d.Win % 4 == 0 && a.pt.nphase == 4 && ((uintptr_t)y & 15) == 0 &&
            (!ep.act_out || ((uintptr_t)ep.act_out & 15) == 0)) {
            a.fd_dwo = FastDiv::make(d.Win / 4);
            static const bool split = [] {   // LDM_CT4_SPLIT=0: the unsplit channel walk (A/B timing)
                const char* e = std::getenv("LDM_CT4_SPLIT");
                return !e || std::atoi(e) != 0;
            }();
            if (d.Hin % 2 == 0 && d.Cin % 8 == 0 && split) {
                a.fd_dho = FastDiv::make(d.Hin / 2);
                const int64_t tiles = (int64_t)d.B * (d.Hin / 2) * (d.Win / 4);
                lp_dispatch(a.ep, [&](auto lp, auto ro) {
                    constexpr int LP = decltype(lp)::value, RO = decltype(ro)::value;
                    if (LP != 0 && ep.x16)
                        hipLaunchKernelGGL((convT4_cout1_r2s_kernel<LP, RO, LP>), dim3((unsigned)((tiles + 63) / 64)), dim3(256), 0, st, a);
                    else
                        hipLaunchKernelGGL((convT4_cout1_r2s_kernel<LP, RO, 0>), dim3((unsigned)((tiles + 63) / 64)), dim3(256), 0, st, a);
                });
                LDM_CHECK_LAUNCH("convT4_cout1_r2s_kernel");
                return 0;
            }
            if (d.Hin % 2 == 0) {
                a.fd_dho = FastDiv::make(d.Hin / 2);
                const int64_t lanes = (int64_t)d.B * (d.Hin / 2) * (d.Win / 4);
                lp_dispatch(a.ep, [&](auto lp, auto ro) {
                    constexpr int LP = decltype(lp)::value, RO = decltype(ro)::value;
                    if (LP != 0 && ep.x16)
                        hipLaunchKernelGGL((convT4_cout1_r2_kernel<LP, RO, LP>), dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, st, a);
                    else
                        hipLaunchKernelGGL((convT4_cout1_r2_kernel<LP, RO, 0>), dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, st, a);
                });
                LDM_CHECK_LAUNCH("convT4_cout1_r2_kernel");
                return 0;
            }
            a.fd_dho = FastDiv::make(d.Hin);
            const int64_t lanes = (int64_t)d.B * d.Hin * (d.Win / 4);
            lp_dispatch(a.ep, [&](auto lp, auto ro) {
                    constexpr int LP = decltype(lp)::value, RO = decltype(ro)::value;
                    if (LP != 0 && ep.x16)
                        hipLaunchKernelGGL((convT4_cout1_kernel<LP, RO, LP>), dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, st, a);
                    else
                        hipLaunchKernelGGL((convT4_cout1_kernel<LP, RO, 0>), dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, st, a);
                });
            LDM_CHECK_LAUNCH("convT4_cout1_kernel");
            return 0;
        }
        LDM_REQUIRE(!ep.x16 && !ep.y16, "conv: 16-bit storage on a path without it (ldm_conv_storage16)");
        if (d.Cin == 1 && !d.transposed && d.Cout <= 64 && a.KK <= 16) {
            const int64_t pix = (int64_t)d.B * d.Hout * d.Wout;
            hipLaunchKernelGGL(conv_cin1_kernel, dim3((unsigned)((pix + 255) / 256)), dim3(256), 0, st, a);
            LDM_CHECK_LAUNCH("conv_cin1_kernel");
            return 0;
        }
        if (!d.transposed && d.Cout == 1 && d.kh == 3 && d.kw == 3 && d.stride == 1 && d.pad == 1 && d.Cin % kC1Groups == 0 &&
            d.Cin <= 512 && d.Wout % 4 == 0 && d.Win == d.Wout && d.Hin == d.Hout && ((uintptr_t)x & 15) == 0 && cout1_on()) {
            a.fd_dwo = FastDiv::make(d.Wout / 4);
            a.fd_dho = FastDiv::make(d.Hout);
            const int64_t quads = (int64_t)d.B * d.Hout * (d.Wout / 4);
            constexpr int QB = 256 / kC1Groups;
            hipLaunchKernelGGL(conv_cout1_k3_kernel, dim3((unsigned)((quads + QB - 1) / QB)), dim3(256), 0, st, a);
            LDM_CHECK_LAUNCH("conv_cout1_k3_kernel");
            return 0;
        }
        hipLaunchKernelGGL(conv_direct_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a);
        LDM_CHECK_LAUNCH("conv_direct_kernel");
        return 0;
    }
    LDM_REQUIRE(plan_ok(d, p.kind, p.tm, p.tn, p.wk, p.ks), "conv forward: invalid plan");
    LDM_REQUIRE(!ep.x16 && !ep.y16, "conv: 16-bit storage on a path without it (ldm_conv_storage16)");
    if (a.ks > 1) {   // (balance: a.ks = the largest per-phase split)
        PhaseTable pt2;
        LDM_REQUIRE(build_phase_table(d, pt2) == 0 && p.ws_floats == split_ws_floats(d, p, pt2),
                    "conv forward: plan workspace size does not match the descriptor");
        a.cnt = reinterpret_cast<int32_t*>(ws);
        a.part = ws + kSplitCounters;
    }
    // buffer descriptors use 32-bit byte offsets; padding lanes use offset 0x7ffffff0 (out of range)
    LDM_REQUIRE((int64_t)d.B * d.Cin * d.Hin * d.Win * 4 < 0x7ff00000LL &&
                    p.packed_floats * 4 < 0x7ff00000LL && (int64_t)d.B * d.Cout * d.Hout * d.Wout * 4 < 0x7ff00000LL,
                "conv forward: tensor too large for 32-bit buffer offsets (split the batch)");
    const bool in_nhwc = d.layout & 1;
    // reduced-precision operands (autocast): bf16 instances for NCHW tensors (the train step's convs);
    // fp16 autocast runs the fp32 kernels (exact operands, wider than asked)
    if (a.ep.lowp == LDM_DT_BF16 && !in_nhwc)
        return p.kind == 1 ? launch_mfma<1, false, 2>(a, p, Nq, st) : launch_mfma<2, false, 2>(a, p, Nq, st);
    if (p.kind == 1) return in_nhwc ? launch_mfma<1, true, 0>(a, p, Nq, st) : launch_mfma<1, false, 0>(a, p, Nq, st);
    return in_nhwc ? launch_mfma<2, true, 0>(a, p, Nq, st) : launch_mfma<2, false, 0>(a, p, Nq, st);
}

}  // namespace ldm

extern "C" int ldm_conv_forward_ws(const ldm_conv_desc* d, const ldm_conv_plan* plan, const float* x, const float* w,
                                   const ldm_epilogue* ep, float* y, float* workspace, void* stream) {
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
        e.lowp = ep->dtype & 0xff;
        LDM_REQUIRE(e.lowp >= LDM_DT_F32 && e.lowp <= LDM_DT_BF16 &&
                        (ep->dtype & ~(0xff | LDM_DT_ROUND_OUT | LDM_DT_X16 | LDM_DT_Y16)) == 0,
                    "conv forward: unknown operand precision");
        e.round_out = (ep->dtype & LDM_DT_ROUND_OUT) ? e.lowp : 0;
        e.x16 = (ep->dtype & LDM_DT_X16) ? 1 : 0;
        e.y16 = (ep->dtype & LDM_DT_Y16) ? 1 : 0;
        LDM_REQUIRE(e.lowp != LDM_DT_F32 || (!e.x16 && !e.y16), "conv forward: 16-bit storage needs a 16-bit dtype");
    }
    return conv_forward_ex(*d, *plan, x, w, e, y, workspace, (hipStream_t)stream);
}

// The 16-bit storage flags (LDM_DT_X16 / LDM_DT_Y16) ldm_conv_forward takes for (d, plan) at a 16-bit operand
// precision: kind 3 both; the Cin = 1 stride-2 kernel a 16-bit output; the 64 -> 1 k4 s2 transposed conv a
// 16-bit input (simple epilogues, 16-byte aligned tensors, as those kernels require); else none.
extern "C" int32_t ldm_conv_storage16(const ldm_conv_desc* d, const ldm_conv_plan* plan) {
    if (!d || !plan) return 0;
    if (plan->kind == 3) return LDM_DT_X16 | LDM_DT_Y16;
    if (plan->kind != 0 || d->layout != 0) return 0;
    if (d->Cin == 1 && !d->transposed && d->Cout <= 64 && d->kh == d->kw && (d->kh == 3 || d->kh == 4) &&
        d->stride == 2 && d->Wout % 4 == 0)
        return LDM_DT_Y16;
    if (d->transposed && d->Cout == 1 && d->kh == 4 && d->kw == 4 && d->stride == 2 && d->pad == 1 && d->out_pad == 0 &&
        d->Win % 4 == 0)
        return LDM_DT_X16;
    return 0;
}

extern "C" int ldm_conv_forward(const ldm_conv_desc* d, const ldm_conv_plan* plan, const float* x, const float* w,
                                const ldm_epilogue* ep, float* y, void* stream) {
    return ldm_conv_forward_ws(d, plan, x, w, ep, y, nullptr, stream);
}

// A/B switch of the Cin = 1 kernel's packed form (tests/test_gpu_store16.py compares both bitwise); returns the
// previous setting
extern "C" int ldm_set_cin1_packed(int on) {
    const int prev = ldm::g_cin1_packed;
    ldm::g_cin1_packed = on ? 1 : 0;
    return prev;
}

// A/B switch of the Cin = 1 kernel's stride-1 form (conv_cin1_x4_kernel<3, ..., SD = 1> against conv_cin1_kernel,
// compared bitwise in tests/test_gpu_store16.py); returns the previous setting
extern "C" int ldm_set_cin1_s1(int on) {
    const int prev = ldm::g_cin1_s1;
    ldm::g_cin1_s1 = on ? 1 : 0;
    return prev;
}
