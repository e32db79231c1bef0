// Small-plane 16-bit-operand implicit-GEMM convolution (plan kind 4, round 6): the train step's UNet layers at
// the bottom of the U (model.py:178-194, :205-229 under train.py:174's autocast) and their data gradients.
//
// Why: at B = 32 on the 16 x 64 latent these layers have 512-2048 positions per phase (2 x 8 / 4 x 16 planes),
// K = 1152-4608, and carry +t_emb / +skip epilogues.  The LDS-window kernel (tconv.hip, kind 3) needs >= 4096
// positions and a bias / BN / activation epilogue only; the general kernel (conv.hip kinds 1 / 2) gathers every
// B operand from the NCHW map one scalar per (k, position) and ran them at 25-57 us per call (10 calls per step,
// ~0.43 ms of the step's kernel time, profiles/r05/train_kernel_stats.csv).
//
// A block owns a 32 x 32 output tile of every phase: 32 output channels x 32 positions of the phase grid q
// (ST samples x R rows x TW columns: a whole 2 x 8 plane pair, half a 4 x 16 plane, one 32-column row run).
//   * Staging: the tile's input window — every input channel, halo and zero padding included — is loaded once,
//     cooperatively (consecutive threads read consecutive positions of one channel row: coalesced), rounded to
//     the operand type and parked position-major in LDS ([position][Cin], 16-byte channel runs, a row pitch of
//     Cin * 2 + 16 bytes so 16 lanes' 16-byte reads of 16 positions are conflict-free).  One barrier.
//   * K: the NW waves deal the 32-channel chunks round-robin.  Per chunk the nine taps (conv: one phase; the k3 s2
//     op1 transposed conv: its four phases' 1 / 2 / 2 / 4 taps) each run two v_mfma_f32_32x32x16_{bf16,f16}: the A
//     fragment is one 16-byte load of the kind-3 weight pack ([phase][chunk = cc * ntap + t][Mpad][32], 16-bit;
//     tconv_pack), the B fragment one ds_read_b128 of the window at the tap's shifted position.  The next chunk's
//     A fragments are loaded while this chunk's MFMAs run.
//   * The waves' partial tiles meet in LDS (the window is dead by then) and are summed in wave order (fixed:
//     deterministic), then conv.hip's epilogue (bias -> BN -> act -> act_out -> + bcast -> + skip, autocast output
//     rounding) stores NCHW, consecutive threads along a row of positions.
// MFMA maps (cdna_hip_programming.md §3): lane l (r = l & 31, h = l >> 5) holds A[row r][k = 8h + j] and
// B[k = 8h + j][col r], j = 0..7; D: col = l & 31, row = (reg & 3) + 8 (reg >> 2) + 4h.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "conv_epi.h"

#pragma clang fp contract(off)

namespace ldm {
namespace sc {

typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef float floatx8 __attribute__((ext_vector_type(8)));

constexpr int kTaps = 9;    // k3: nine taps per chunk in both forms
constexpr int kLdsMax = 160 * 1024;

struct SArgs {
    ConvArgs c;                   // dimensions, phase table, epilogue (conv.hip's)
    const unsigned short* wp;     // kind-3 pack, 16-bit
    int32_t nM, ntx, nty, nsg;    // 32-row M tiles; position tiles along q columns / q rows / sample groups
    int32_t ST, R, TW;            // a tile: ST samples x R q-rows x TW q-columns (= 32 positions)
    int32_t sy, osy;              // input step per q, output step per q
    int32_t dylo, dxlo, WR, WC;   // the tile's input window per sample: rows qy0 * sy + dylo + [0, WR), cols likewise
    int32_t pitch;                // LDS bytes per window position
    int32_t nchunk;               // Cin / 32
    // the nine taps in phase-table order (phase 0's taps, then phase 1's, ...): LDS position offset dy * WC + dx,
    // and the pack offset of chunk 0 (16-bit elements) and its stride per chunk
    int32_t toff[kTaps];
    int64_t tw0[kTaps], twst[kTaps];
    int32_t ry[kMaxPhase], rx[kMaxPhase];
};

// phase of tap i (phase-table order) for the one-phase conv / the four-phase k3 s2 op1 transposed conv
template <int NPH>
__host__ __device__ constexpr int tap_phase(int i) {
    return NPH == 1 ? 0 : (i == 0 ? 0 : (i < 3 ? 1 : (i < 5 ? 2 : 3)));
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

template <int DT>
__device__ __forceinline__ u16x8 to16(const floatx8& v) {
    if constexpr (DT == 1)
        return __builtin_bit_cast(u16x8, __builtin_convertvector(v, halfx8));
    else
        return __builtin_bit_cast(u16x8, __builtin_convertvector(v, bf16x8));
}

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

template <int NPH, int DT, int NW>
__global__ __launch_bounds__(64 * NW) void sconv_kernel(SArgs s) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const ConvArgs& a = s.c;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int mt = blockIdx.x % s.nM;
    const int tile = blockIdx.x / s.nM;
    const int tx = tile % s.ntx;
    const int rest = tile / s.ntx;
    const int ty = rest % s.nty, sg = rest / s.nty;
    const int b0 = sg * s.ST, qy0 = ty * s.R, qx0 = tx * s.TW;
    const int m0 = mt * 32;
    const int HWin = a.Hin * a.Win;
    const int wps = s.WR * s.WC;             // window positions per sample
    const int npos = s.ST * wps;

    // ---- the tile's input window, every channel, 16-bit, [position][Cin] --------------------------------------
    {
        const int ncg = a.Cin >> 3;          // 8-channel groups
        const int per = (64 * NW) / npos;    // channel groups staged per pass (npos <= the block's threads)
        const int pos = tid % npos, cg0 = tid / npos;
        const int sm = pos / wps, rem = pos - sm * wps;
        const int wr = rem / s.WC, wc = rem - wr * s.WC;
        const int b = b0 + sm;
        const int iy = qy0 * s.sy + s.dylo + wr, ix = qx0 * s.sy + s.dxlo + wc;
        const bool ok = cg0 < per && b < a.B && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
        const float* src = a.x + (size_t)(ok ? b : 0) * a.Cin * HWin + (ok ? iy * a.Win + ix : 0);
        char* dst = lds + pos * s.pitch;
        if (cg0 < per) {
            for (int cg = cg0; cg < ncg; cg += per) {
                floatx8 v;
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = ok ? src[(size_t)(cg * 8 + j) * HWin] : 0.f;
                *reinterpret_cast<u16x8*>(dst + cg * 16) = to16<DT>(v);
            }
        }
    }
    __syncthreads();

    // ---- K: this wave's 32-channel chunks, nine taps each, two 16-deep MFMAs per tap ----------------------------
    // lane r's column: position r of the tile -> its window position (tap (dy, dx) adds toff)
    const int spos = s.R * s.TW;
    const int rs = r / spos, rr = r - rs * spos;
    const int ryl = rr / s.TW, cx = rr - ryl * s.TW;
    const int lpos0 = rs * wps + (ryl * s.sy - s.dylo) * s.WC + (cx * s.sy - s.dxlo);
    const char* lb = lds + h * 16;           // lane's 8-channel half of each 16-deep k-step
    const __amdgpu_buffer_rsrc_t wr_ = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(s.wp), (short)0, 0x7ffffff0, 0x00020000);
    const int arow = ((m0 + r) * 32 + h * 8) * 2;   // bytes: row m0 + r of a chunk, k 8h .. 8h + 7

    floatx16 acc[NPH];
#pragma unroll
    for (int p = 0; p < NPH; ++p)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[p][i] = 0.f;

    // two register sets of A fragments (compile-time set index: the chunk loop is unrolled by two), the next
    // chunk's set loading while this chunk's MFMAs run — except at two waves per SIMD with four phase accumulators,
    // where the second set does not fit the 256 registers (the other wave of the SIMD covers the wait)
    constexpr bool DB = !(NPH == 4 && NW == 8);
    u16x8 fa[DB ? 2 : 1][kTaps][2];
    auto load_a = [&](auto setc, int cc) {
        constexpr int S = decltype(setc)::value;
        static_for<0, kTaps>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const int off = (int)((s.tw0[i] + (int64_t)cc * s.twst[i]) * 2) + arow;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
                fa[S][i][ks] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(wr_, off + ks * 32, 0, 0));
        });
    };
    auto compute = [&](auto setc, int cc) {
        constexpr int S = decltype(setc)::value;
        static_for<0, kTaps>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            constexpr int p = tap_phase<NPH>(i);
            const char* bp = lb + (lpos0 + s.toff[i]) * s.pitch + cc * 64;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const u16x8 fb = *reinterpret_cast<const u16x8*>(bp + ks * 32);
                acc[p] = mma<DT>(fa[S][i][ks], fb, acc[p]);
            }
        });
    };
    using Z = std::integral_constant<int, 0>;
    using O = std::integral_constant<int, DB ? 1 : 0>;
    int cc = wave;
    if constexpr (DB) {
        if (cc < s.nchunk) load_a(Z{}, cc);
        while (cc < s.nchunk) {
            if (cc + NW < s.nchunk) load_a(O{}, cc + NW);
            compute(Z{}, cc);
            cc += NW;
            if (cc >= s.nchunk) break;
            if (cc + NW < s.nchunk) load_a(Z{}, cc + NW);
            compute(O{}, cc);
            cc += NW;
        }
    } else {
        for (; cc < s.nchunk; cc += NW) {
            load_a(Z{}, cc);
            compute(Z{}, cc);
        }
    }

    // ---- the waves' partial tiles meet in LDS in wave order; epilogue, NCHW ------------------------------------
    __syncthreads();   // every wave is done with the window
    float* red = reinterpret_cast<float*>(lds);   // [wave][phase][reg][lane]
#pragma unroll
    for (int p = 0; p < NPH; ++p)
#pragma unroll
        for (int g = 0; g < 16; ++g) red[((wave * NPH + p) * 16 + g) * 64 + lane] = acc[p][g];
    __syncthreads();
    for (int o = tid; o < NPH * 1024; o += 64 * NW) {
        const int p = o >> 10, mn = o & 1023;
        const int ml = mn >> 5, n = mn & 31;                 // row of the tile, position of the tile
        const int g = (ml & 3) + 4 * (ml >> 3), ln = n + 32 * ((ml >> 2) & 1);
        float v = red[((0 * NPH + p) * 16 + g) * 64 + ln];
#pragma unroll
        for (int w = 1; w < NW; ++w) v = v + red[((w * NPH + p) * 16 + g) * 64 + ln];
        const int ns = n / spos, nr = n - ns * spos;
        const int qyl = nr / s.TW, qx = qx0 + nr - qyl * s.TW;
        const int b = b0 + ns, m = m0 + ml;
        if (b >= a.B || m >= a.Cout) continue;
        const int oy = (qy0 + qyl) * s.osy + s.ry[p], ox = qx * s.osy + s.rx[p];
        epilogue_store(a, m, b, oy, ox, v);
    }
}

}  // namespace sc

// Geometry of a kind-4 plan for d; false when the layer is not of its class.
static bool sconv_geometry(const ldm_conv_desc& d, sc::SArgs& s, int& nph, int& nw, size_t& lds) {
    if (d.layout != 0 || d.kh != 3 || d.kw != 3 || d.pad != 1 || d.B <= 0) return false;
    if (d.Cin % 32 != 0 || d.Cin < 64 || d.Cout % 64 != 0) return false;
    const bool conv = !d.transposed && (d.stride == 1 || d.stride == 2);
    const bool convt = d.transposed && d.stride == 2 && d.out_pad == 1;
    const bool convt1 = d.transposed && d.stride == 1;   // the data gradient of a stride-1 conv
    if (!conv && !convt && !convt1) return false;
    PhaseTable pt;
    if (build_phase_table(d, pt)) return false;
    nph = pt.nphase;
    if (nph == 4 && !(pt.ntap[0] == 1 && pt.ntap[1] == 2 && pt.ntap[2] == 2 && pt.ntap[3] == 4)) return false;
    if (nph == 1 && pt.ntap[0] != 9) return false;
    const int Hq = pt.Hq, Wq = pt.Wq;
    int TW, R, ST;
    if (Wq <= 32) {
        if (32 % Wq) return false;
        TW = Wq, R = 32 / Wq, ST = 1;
        if (R > Hq) {
            if (R % Hq) return false;
            ST = R / Hq, R = Hq;
        } else if (Hq % R) {
            return false;
        }
    } else {
        if (Wq % 32) return false;
        TW = 32, R = 1, ST = 1;
    }
    int dylo = 1 << 20, dyhi = -(1 << 20), dxlo = 1 << 20, dxhi = -(1 << 20);
    int i = 0;
    for (int p = 0; p < nph; ++p)
        for (int t = 0; t < pt.ntap[p]; ++t, ++i) {
            dylo = std::min(dylo, pt.dy[p][t]), dyhi = std::max(dyhi, pt.dy[p][t]);
            dxlo = std::min(dxlo, pt.dx[p][t]), dxhi = std::max(dxhi, pt.dx[p][t]);
        }
    if (i != sc::kTaps) return false;
    s = sc::SArgs{};
    s.ST = ST, s.R = R, s.TW = TW;
    s.sy = pt.sy, s.osy = pt.osy;
    s.dylo = dylo, s.dxlo = dxlo;
    s.WR = (R - 1) * pt.sy + dyhi - dylo + 1;
    s.WC = (TW - 1) * pt.sy + dxhi - dxlo + 1;
    s.pitch = d.Cin * 2 + 16;
    s.nchunk = d.Cin / 32;
    s.ntx = Wq / TW, s.nty = Hq / R, s.nsg = (d.B + ST - 1) / ST;
    s.nM = d.Cout / 32;
    nw = s.nchunk >= 8 ? 8 : 4;
    const int npos = ST * s.WR * s.WC;
    if (npos > 64 * nw) return false;                   // one staging pass covers every window position
    lds = std::max((size_t)npos * s.pitch, (size_t)nw * nph * 16 * 64 * 4);
    if (lds > (size_t)sc::kLdsMax) return false;
    const int64_t blocks = (int64_t)s.nM * s.ntx * s.nty * s.nsg;
    if (blocks >= (1LL << 31)) return false;
    if ((int64_t)d.B * d.Cin * d.Hin * d.Win >= (1LL << 31) || (int64_t)d.B * d.Cout * d.Hout * d.Wout >= (1LL << 31))
        return false;
    return true;
}

bool sconv_plan(const ldm_conv_desc& d, int dtype, ldm_conv_plan& plan) {
    if (dtype != LDM_DT_F16 && dtype != LDM_DT_BF16) return false;
    static const bool on = [] {   // LDM_AMD_SCONV=0: the layers keep conv.hip's plans (A/B timing)
        const char* e = std::getenv("LDM_AMD_SCONV");
        return !e || std::atoi(e) != 0;
    }();
    if (!on) return false;
    sc::SArgs s;
    int nph, nw;
    size_t lds;
    if (!sconv_geometry(d, s, nph, nw, lds)) return false;
    // the weights: tconv.hip's kind-3 pack with 64-row padding (Cout % 64 == 0: no padding rows)
    ldm_conv_plan k3{};
    k3.kind = 3, k3.tm = 1, k3.tn = dtype, k3.wk = 1, k3.ks = 1;
    PhaseTable pt;
    int Mpad = 0;
    int64_t halfs = 0;
    if (build_phase_table(d, pt)) return false;
    halfs = 0;
    for (int p = 0; p < pt.nphase; ++p) halfs += (int64_t)pt.ntap[p] * (d.Cin / 32) * d.Cout * 32;
    (void)Mpad;
    plan = ldm_conv_plan{};
    plan.kind = 4;
    plan.tm = 1;
    plan.tn = dtype;
    plan.wk = nw;
    plan.ks = 1;
    plan.packed_floats = (halfs + 1) / 2;
    plan.ws_floats = 0;
    return true;
}

int sconv_forward(const ldm_conv_desc& d, const ldm_conv_plan& p, const float* x, const float* w, const EpiArgs& ep,
                  float* y, hipStream_t st) {
    LDM_REQUIRE(p.kind == 4 && (p.tn == LDM_DT_F16 || p.tn == LDM_DT_BF16), "sconv: not a kind-4 plan");
    LDM_REQUIRE(ep.lowp == p.tn, "sconv: the plan's operand precision differs from the call's");
    LDM_REQUIRE(!ep.x16 && !ep.y16, "sconv: fp32 maps only");
    LDM_REQUIRE(!ep.ddim_coef && !ep.pos_bias && y, "sconv: no fused update / position bias");
    sc::SArgs s;
    int nph, nw;
    size_t lds;
    LDM_REQUIRE(sconv_geometry(d, s, nph, nw, lds) && nw == p.wk, "sconv: plan does not match the descriptor");
    ConvArgs& a = s.c;
    a = ConvArgs{};
    a.x = x;
    a.w = w;
    a.y = y;
    a.B = d.B, a.Cin = d.Cin, a.Hin = d.Hin, a.Win = d.Win, a.Cout = d.Cout, a.Hout = d.Hout, a.Wout = d.Wout;
    a.out_nhwc = 0;
    a.ep = ep;
    LDM_REQUIRE(!a.ep.bn_w || (a.ep.bn_b && a.ep.bn_m && a.ep.bn_v), "sconv: incomplete BatchNorm parameters");
    PhaseTable pt;
    LDM_REQUIRE(build_phase_table(d, pt) == 0, "sconv: phase table");
    // tconv_pack's layout: phase segments in 16-bit elements, chunk c = cc * ntap + t of rows [Mpad = Cout][32]
    int64_t wofs = 0;
    int i = 0;
    for (int q = 0; q < pt.nphase; ++q) {
        s.ry[q] = pt.ry[q], s.rx[q] = pt.rx[q];
        for (int t = 0; t < pt.ntap[q]; ++t, ++i) {
            s.toff[i] = pt.dy[q][t] * s.WC + pt.dx[q][t];
            s.tw0[i] = wofs + (int64_t)t * d.Cout * 32;
            s.twst[i] = (int64_t)pt.ntap[q] * d.Cout * 32;
        }
        wofs += (int64_t)pt.ntap[q] * (d.Cin / 32) * d.Cout * 32;
    }
    LDM_REQUIRE(wofs * 2 < 0x7ffffff0LL, "sconv: weight pack too large for 32-bit offsets");
    s.wp = reinterpret_cast<const unsigned short*>(w);
    const unsigned blocks = (unsigned)((int64_t)s.nM * s.ntx * s.nty * s.nsg);
    auto go = [&](auto nphc, auto dtc, auto nwc) {
        constexpr int NPH = decltype(nphc)::value, DT = decltype(dtc)::value, NW = decltype(nwc)::value;
        auto kfn = sc::sconv_kernel<NPH, DT, NW>;
        static bool opted = false;
        if (!opted) {
            LDM_HIP_TRY(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, sc::kLdsMax));
            opted = true;
        }
        hipLaunchKernelGGL(kfn, dim3(blocks), dim3(64 * NW), lds, st, s);
        return 0;
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I4 = std::integral_constant<int, 4>;
    using I8 = std::integral_constant<int, 8>;
    int rc;
    auto by_nw = [&](auto nphc, auto dtc) { return nw == 8 ? go(nphc, dtc, I8{}) : go(nphc, dtc, I4{}); };
    auto by_dt = [&](auto nphc) { return p.tn == LDM_DT_F16 ? by_nw(nphc, I1{}) : by_nw(nphc, I2{}); };
    rc = nph == 4 ? by_dt(I4{}) : by_dt(I1{});
    if (rc) return rc;
    LDM_CHECK_LAUNCH("sconv_kernel");
    return 0;
}

}  // namespace ldm

using namespace ldm;

extern "C" int ldm_conv_sconv_plan(const ldm_conv_desc* d, int32_t dtype, ldm_conv_plan* plan) {
    if (!d || !plan) return fail(2, "conv_sconv_plan: null argument");
    return sconv_plan(*d, dtype, *plan) ? 0 : 1;
}
