// Conv / transposed-conv weight gradient of the train step (LDMTrainer.train_step, train.py:163-208:
// scaler.scale(loss).backward() through every trained conv) as a tap-shared implicit GEMM for gfx950.
//
//   dW[m][c][t] = sum_{b,q} Dense[b][m][q] * Gath[b][c][q*s + d_t],   d_t = (kh - pad, kw - pad)
//   conv  (w [Cout][Cin][k][k]):  Dense = dY (m = co, q over Hout x Wout), Gath = X,  s = stride
//   convT (w [Cin][Cout][k][k]):  Dense = X  (m = ci, q over Hin  x Win ), Gath = dY, s = stride
//
// One block owns a BM (m) x BC (c) tile for ALL k*k taps and walks a slice of K = (b, q) in chunks of 64
// output positions (one 64-wide row segment, or 64/Wq whole rows).  Per chunk it DMAs into LDS (16 B per
// lane, buffer_load ... lds) the Dense rows [BM][64] and the Gath window the chunk's taps touch,
// [BC][WR][WCa] (borders and channels past C arrive as zeros: the window origin is aligned down to 4
// floats, so a 16-B piece is either inside the image row or wholly outside it).  Every Dense fragment is
// then read once per 16 positions and reused by all k*k taps, every window value by every tap that
// covers it: the previous kernel (backward.hip) gathered 4 scalars per lane per tap from global memory.
// Chunks are double-buffered: the DMAs of chunk i+1 are issued before chunk i is multiplied.
// K is split over blocks (grid.z) into fixed ranges; wgrad_reduce_kernel sums the partials in split
// order, so the result is bitwise reproducible.
// MFMA v_mfma_f32_16x16x4_f32: lane l = (col l&15, group g = l>>4); for the 16 positions of step u the
// lane supplies positions 16u + 4g + j at MFMA j (A as one float4 from LDS, B as 4 window values).
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "common.h"

#pragma clang fp contract(off)

namespace ldm {
namespace wg {

struct Args {
    const float* dense;   // [B][M][Hq*Wq]
    const float* gath;    // [B][C][Hg][Wg]
    float* partial;       // [S][M][C*T]
    int32_t B, M, C, Hq, Wq, Hg, Wg, pad;
    int32_t cols, rows;   // chunk = rows x cols output positions (cols = min(Wq, 64), rows = 64 / cols)
    int32_t cps;          // chunks per sample
    int32_t nchunk, per_split;
    int32_t wr, wca, e;   // window rows, row pitch (floats, multiple of 4), column shift of the aligned origin
    int32_t pitch_c;      // floats per channel in the window (wr * wca)
    int32_t lowp;         // LDM_DT_*: operands rounded to fp16 / bf16, fp32 accumulation
    int32_t dense16;      // wgrad_c1_kernel XS != 0: Dense stored in 16 bits (register-staged, see wgrad_lp_kernel)
};

template <int B_, int E_, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B_ < E_) {
        f(std::integral_constant<int, B_>{});
        static_for<B_ + 1, E_>(f);
    }
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;
constexpr int kOOB = 0x7ffffff0;
constexpr int kKQ = 64;   // output positions per chunk

template <int S, int KK, int BM, int BC>
struct Cfg {
    static constexpr int T = KK * KK;
    static constexpr int WCF = BC / 16, WMF = 4 / WCF, FM = BM / 16 / WMF;   // 4 waves: WMF x WCF, FM m-frags each
    static_assert(WMF * WCF == 4 && FM >= 1 && FM * 16 * WMF == BM, "wave layout");
    static constexpr int A_FLOATS = BM * kKQ;
};

// floats of one LDS buffer: A rows + the window rounded up to whole wave-instructions (64 pieces)
__host__ __device__ inline int buf_floats(int a_floats, int bc, int pitch_c) {
    return a_floats + (bc * pitch_c + 255) / 256 * 256;
}

template <int S, int KK, int BM, int BC, int DT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void wgrad_kernel(Args a) {
    using g = Cfg<S, KK, BM, BC>;
    constexpr int T = g::T, WCF = g::WCF, FM = g::FM, AF = g::A_FLOATS;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wc = wave % WCF, wm = wave / WCF;
    const int col = lane & 15, lg = lane >> 4;
    const int m0 = blockIdx.y * BM, c0 = blockIdx.x * BC;
    const int HQ = a.Hq * a.Wq;
    const int bufF = buf_floats(AF, BC, a.pitch_c);
    const int ch_begin = blockIdx.z * a.per_split;
    const int ch_end = min(a.nchunk, ch_begin + a.per_split);

    const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(a.dense), (short)0, uni(a.B * a.M * HQ * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(a.gath), (short)0, uni(a.B * a.C * a.Hg * a.Wg * 4), 0x00020000);

    // chunk -> (sample, first output row, first output column)
    auto chunk_geo = [&](int ch, int& b, int& qy0, int& qx0) {
        b = ch / a.cps;
        const int r = ch - b * a.cps;
        if (a.cols == a.Wq) {   // whole rows
            qy0 = r * a.rows, qx0 = 0;
        } else {                // 64-wide segments of one row
            const int segs = a.Wq / kKQ;
            qy0 = r / segs, qx0 = (r - qy0 * segs) * kKQ;
        }
    };
    // DMA of chunk ch into buffer buf: A = BM rows x 64 positions (XOR-swizzled 16-B pieces), then the
    // window [BC][wr][wca]; the work is dealt round-robin over all 256 lanes' 16-B pieces.
    auto issue = [&](int ch, int buf) {
        int b, qy0, qx0;
        chunk_geo(ch, b, qy0, qx0);
        char* base = reinterpret_cast<char*>(smem + buf * bufF);
        // A: BM*16 pieces = BM/4 wave-instructions
        for (int gi = wave; gi < BM / 4; gi += 4) {
            const int row = gi * 4 + (lane >> 4);
            const int p = lane & 15;                       // destination piece
            const int sp = p ^ (row & 15);                  // source piece
            const int m = m0 + row;
            const int ql = sp * 4;                          // chunk-local position of the piece
            const int qy = qy0 + ql / a.cols, qx = qx0 + ql % a.cols;
            const bool ok = m < a.M && qy < a.Hq;
            const int voff = ok ? (((b * a.M + m) * HQ + qy * a.Wq + qx) * 4) : kOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(dr, (lds_ptr_t)(base + gi * 1024), 16, voff, 0, 0, 0);
        }
        // window: BC * wr * wca / 4 pieces
        const int wq4 = a.wca >> 2;
        const int npiece = BC * a.wr * wq4;
        const int row0 = qy0 * S - a.pad, colA = qx0 * S - a.pad - a.e;
        for (int gi = wave; gi * 64 < npiece; gi += 4) {
            const int pc = gi * 64 + lane;
            const int cl = pc / (a.wr * wq4);
            const int rem = pc - cl * (a.wr * wq4);
            const int wrow = rem / wq4, wp = rem - wrow * wq4;
            const int c = c0 + cl, iy = row0 + wrow, ix = colA + wp * 4;
            const bool ok = pc < npiece && c < a.C && (unsigned)iy < (unsigned)a.Hg && (unsigned)ix < (unsigned)a.Wg;
            const int voff = ok ? ((((b * a.C + c) * a.Hg + iy) * a.Wg + ix) * 4) : kOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(gr, (lds_ptr_t)(base + AF * 4 + gi * 1024), 16, voff, 0, 0, 0);
        }
    };

    floatx4 acc[T][FM];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int f = 0; f < FM; ++f) acc[t][f] = floatx4{0.f, 0.f, 0.f, 0.f};

    // per-lane LDS offsets inside a buffer: A row pieces, window column of position 16u + 4g (+ j*S)
    int aoff[FM][4];
#pragma unroll
    for (int f = 0; f < FM; ++f)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int row = (wm * FM + f) * 16 + col;
            aoff[f][u] = row * kKQ + (((4 * u + lg) ^ (row & 15)) << 2);
        }
    int boff[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        // positions past the chunk's rows (a small image zero-padded to 64) multiply zeros of A: point them
        // at position 0 so that they read finite window values (0 * NaN from stale LDS would be NaN)
        const int ql = (16 * u + 4 * lg < a.rows * a.cols) ? 16 * u + 4 * lg : 0;
        const int rl = ql / a.cols, xl = ql - rl * a.cols;
        boff[u] = AF + (wc * 16 + col) * a.pitch_c + rl * S * a.wca + a.e + xl * S;
    }

    if (ch_begin < ch_end) issue(ch_begin, 0);
    for (int ch = ch_begin; ch < ch_end; ++ch) {
        const int buf = (ch - ch_begin) & 1;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();   // chunk ch landed everywhere; every wave is done with the other buffer
        if (ch + 1 < ch_end) issue(ch + 1, buf ^ 1);
        const float* sb = smem + buf * bufF;
        {   // DT = operand precision (compile time: a runtime branch between MFMA forms miscompiled in conv.hip)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                floatx4 fa[FM];
#pragma unroll
                for (int f = 0; f < FM; ++f) fa[f] = *reinterpret_cast<const floatx4*>(sb + aoff[f][u]);
                static_for<0, T>([&](auto tc) {
                    constexpr int t = decltype(tc)::value;
                    constexpr int ky = t / KK, kx = t % KK;
                    const float* bp = sb + boff[u] + ky * a.wca + kx;
                    floatx4 bv;
#pragma unroll
                    for (int j = 0; j < 4; ++j) bv[j] = bp[j * S];
                    if constexpr (DT == 0) {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
#pragma unroll
                            for (int f = 0; f < FM; ++f)
                                acc[t][f] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[f][j], bv[j], acc[t][f], 0, 0, 0);
                    } else {
#pragma unroll
                        for (int f = 0; f < FM; ++f) acc[t][f] = mma16_lowp<DT>(fa[f], bv, acc[t][f]);
                    }
                });
            }
        }
    }

    // partial tile: rows m = m0 + 16*(wm*FM+f) + 4g + r, column c = c0 + 16*wc + col, T taps contiguous
    const int N = a.C * T;
    const int c = c0 + wc * 16 + col;
    if (c < a.C) {
        float* out = a.partial + (size_t)blockIdx.z * a.M * N;
#pragma unroll
        for (int f = 0; f < FM; ++f)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + (wm * FM + f) * 16 + 4 * lg + r;
                if (m < a.M) {
                    float* o = out + (size_t)m * N + (size_t)c * T;
#pragma unroll
                    for (int t = 0; t < T; ++t) o[t] = acc[t][f][r];
                }
            }
    }
}

// One gathered channel (C = 1: the Cin = 1 first layers of the VAE / style encoders, and the decoder's
// 64 -> 1 output convT): the N dimension of the GEMM is the k*k taps instead of 16 channels (the general
// kernel spent 15/16 of its window DMAs and MFMAs on padding channels there).  Block = 4 waves x 16 rows
// (m) x 16 columns (taps; k = 3 leaves 7 idle); the lane of column t reads its tap's window value, so the
// whole 16 x 16 x (64 positions) product of a chunk is 4 (16 in f32) MFMAs per wave.
template <int S, int KK, int DT, int XS = 0>
__global__ __launch_bounds__(256) void wgrad_c1_kernel(Args a) {
    constexpr int T = KK * KK, BM = 64, AF = BM * kKQ;
    static_assert(T <= 16, "taps per column tile");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int col = lane & 15, lg = lane >> 4;
    const int m0 = blockIdx.y * BM;
    const int HQ = a.Hq * a.Wq;
    const int bufF = buf_floats(AF, 1, a.pitch_c);
    const int ch_begin = blockIdx.z * a.per_split;
    const int ch_end = min(a.nchunk, ch_begin + a.per_split);
    const bool d16 = XS != 0 && a.dense16;
    const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(a.dense), (short)0, uni(a.B * a.M * HQ * (d16 ? 2 : 4)), 0x00020000);
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(a.gath), (short)0, uni(a.B * a.Hg * a.Wg * 4), 0x00020000);

    // XS != 0: the Dense rows register-staged (16-bit quads widened when parked at the DMA's addresses); the
    // window (the fp32 input of a Cin = 1 layer) keeps its DMA
    uint4 rd[XS ? BM / 16 : 1];
    auto fetch_dense = [&](int ch) {
        const int b = ch / a.cps;
        const int r = ch - b * a.cps;
        int qy0, qx0;
        if (a.cols == a.Wq) {
            qy0 = r * a.rows, qx0 = 0;
        } else {
            const int segs = a.Wq / kKQ;
            qy0 = r / segs, qx0 = (r - qy0 * segs) * kKQ;
        }
#pragma unroll
        for (int i = 0; i < BM / 16; ++i) {
            const int gi = wave + 4 * i;
            const int row = gi * 4 + (lane >> 4);
            const int p = lane & 15;
            const int sp = p ^ (row & 15);
            const int m = m0 + row;
            const int ql = sp * 4;
            const int qy = qy0 + ql / a.cols, qx = qx0 + ql % a.cols;
            const bool ok = m < a.M && qy < a.Hq;
            const int el = ((b * a.M + m) * HQ + qy * a.Wq + qx);
            if (d16) {
                const uint2 t = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(dr, ok ? el * 2 : kOOB, 0, 0));
                rd[i] = uint4{t.x, t.y, 0u, 0u};
            } else {
                rd[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(dr, ok ? el * 4 : kOOB, 0, 0));
            }
        }
    };
    auto park_dense = [&](int buf) {
        char* base = reinterpret_cast<char*>(smem + buf * bufF);
#pragma unroll
        for (int i = 0; i < BM / 16; ++i) {
            const int gi = wave + 4 * i;
            floatx4 v;
            if (d16)
                v = floatx4{from16<XS>((unsigned short)(rd[i].x & 0xffff)), from16<XS>((unsigned short)(rd[i].x >> 16)),
                            from16<XS>((unsigned short)(rd[i].y & 0xffff)), from16<XS>((unsigned short)(rd[i].y >> 16))};
            else
                v = __builtin_bit_cast(floatx4, rd[i]);
            *reinterpret_cast<floatx4*>(base + gi * 1024 + lane * 16) = v;
        }
    };

    auto issue = [&](int ch, int buf) {
        int b, qy0, qx0;
        b = ch / a.cps;
        const int r = ch - b * a.cps;
        if (a.cols == a.Wq) {
            qy0 = r * a.rows, qx0 = 0;
        } else {
            const int segs = a.Wq / kKQ;
            qy0 = r / segs, qx0 = (r - qy0 * segs) * kKQ;
        }
        char* base = reinterpret_cast<char*>(smem + buf * bufF);
        for (int gi = wave; gi < (XS ? 0 : BM / 4); gi += 4) {
            const int row = gi * 4 + (lane >> 4);
            const int p = lane & 15;
            const int sp = p ^ (row & 15);
            const int m = m0 + row;
            const int ql = sp * 4;
            const int qy = qy0 + ql / a.cols, qx = qx0 + ql % a.cols;
            const bool ok = m < a.M && qy < a.Hq;
            const int voff = ok ? (((b * a.M + m) * HQ + qy * a.Wq + qx) * 4) : kOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(dr, (lds_ptr_t)(base + gi * 1024), 16, voff, 0, 0, 0);
        }
        const int wq4 = a.wca >> 2;
        const int npiece = a.wr * wq4;
        const int row0 = qy0 * S - a.pad, colA = qx0 * S - a.pad - a.e;
        for (int gi = wave; gi * 64 < npiece; gi += 4) {
            const int pc = gi * 64 + lane;
            const int wrow = pc / wq4, wp = pc - wrow * wq4;
            const int iy = row0 + wrow, ix = colA + wp * 4;
            const bool ok = pc < npiece && (unsigned)iy < (unsigned)a.Hg && (unsigned)ix < (unsigned)a.Wg;
            const int voff = ok ? (((b * a.Hg + iy) * a.Wg + ix) * 4) : kOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(gr, (lds_ptr_t)(base + AF * 4 + gi * 1024), 16, voff, 0, 0, 0);
        }
    };

    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    int aoff[4], boff[4];
    const int row = wave * 16 + col;
    const int tcol = col < T ? col : 0;   // idle columns (k = 3) re-read tap 0; their results are dropped
    const int ky = tcol / KK, kx = tcol - ky * KK;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        aoff[u] = row * kKQ + (((4 * u + lg) ^ (row & 15)) << 2);
        const int ql = (16 * u + 4 * lg < a.rows * a.cols) ? 16 * u + 4 * lg : 0;
        const int rl = ql / a.cols, xl = ql - rl * a.cols;
        boff[u] = AF + (rl * S + ky) * a.wca + a.e + xl * S + kx;
    }

    if (ch_begin < ch_end) {
        issue(ch_begin, 0);
        if constexpr (XS != 0) {
            fetch_dense(ch_begin);
            park_dense(0);
        }
    }
    for (int ch = ch_begin; ch < ch_end; ++ch) {
        const int buf = (ch - ch_begin) & 1;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (ch + 1 < ch_end) {
            issue(ch + 1, buf ^ 1);
            if constexpr (XS != 0) fetch_dense(ch + 1);
        }
        const float* sb = smem + buf * bufF;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const floatx4 fa = *reinterpret_cast<const floatx4*>(sb + aoff[u]);
            floatx4 bv;
#pragma unroll
            for (int j = 0; j < 4; ++j) bv[j] = sb[boff[u] + j * S];
            if constexpr (DT == 0) {
#pragma unroll
                for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[j], bv[j], acc, 0, 0, 0);
            } else {
                acc = mma16_lowp<DT>(fa, bv, acc);
            }
        }
        if constexpr (XS != 0) {
            if (ch + 1 < ch_end) park_dense(buf ^ 1);
        }
    }
    // D: row m = m0 + 16*wave + 4*lg + r, column = tap col
    if (col < T) {
        float* out = a.partial + (size_t)blockIdx.z * a.M * T;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + wave * 16 + 4 * lg + r;
            if (m < a.M) out[(size_t)m * T + col] = acc[r];
        }
    }
}

// ------------------------------------------------------------------------------------------------------
// The same weight gradient with 16-bit operands (the train step's torch.autocast region) on the gfx950
// double-rate v_mfma_f32_32x32x16_{f16,bf16}: K = 16 positions per MFMA instead of 4 per f32 MFMA.
//
// The fp32 form above reads its gathered operand one scalar per position per tap, so at 16-bit rates
// it would be bound by LDS reads and their conversions.  Here a block owns BM rows (m) x 32 gathered
// channels (c) x all k*k taps; its NW = WM * KK waves split the rows (wm) and the tap rows (ky): a wave
// covers BM/WM rows and the KK taps (ky, 0..KK-1) of 32 channels.  K is walked in chunks of 32 output
// positions (one 32-wide row segment, or two 16-wide rows), two MFMA k-steps of 16 positions each.
// Per k-step a lane of column c needs positions q0 .. q0+7 (q0 = 16 ks + 8 h) of every kx tap, i.e.
// window columns 3 + kx + S j of one window row; their union is one aligned run of 4*NB floats, read as
// NB ds_read_b128 (channel pitch = 4 mod 64 floats: 16 lanes' 16-B reads are conflict-free), and each
// tap's fragment is 8 of those registers rounded to 16 bits.  The Dense rows are read two pieces
// (8 positions) per fragment from an XOR-swizzled [BM][32] tile.  Both tiles arrive by LDS DMA, double-
// buffered.  Requires pad = 1 (every k3 / k4 layer of the model), so the window origin shift e = 3.
// MFMA maps (cdna_hip_programming.md §3): lane l (r = l & 31, h = l >> 5) holds A[row r][k = 8h + j] and
// B[k = 8h + j][col r]; D col = l & 31, row = (reg & 3) + 8 (reg >> 2) + 4h.
// ------------------------------------------------------------------------------------------------------
constexpr int kLC = 32;    // gathered channels per block
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef float floatx8 __attribute__((ext_vector_type(8)));

template <int DT>
__device__ __forceinline__ floatx16 mma32x16(const floatx8& a, const floatx8& b, const floatx16& c) {
    if constexpr (DT == 1)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_convertvector(a, halfx8), __builtin_convertvector(b, halfx8),
                                                      c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_convertvector(a, bf16x8),
                                                       __builtin_convertvector(b, bf16x8), c, 0, 0, 0);
}

struct LpArgs {
    const float* dense;   // [B][M][Hq*Wq]
    const float* gath;    // [B][C][Hg][Wg]
    float* partial;       // [splits][M][C*T]
    int32_t B, M, C, Hq, Wq, Hg, Wg;
    int32_t cols, rows, cps, nchunk, per_split;
    int32_t wr, wca, pitch_c;   // window rows, row pitch, channel pitch (floats)
    int32_t dense16, gath16;    // 16-bit storage of dense / gath (the register-staged instances, XS != 0)
};
// window pieces per lane of a register-staged instance: the largest window lp_plan makes for (S, KK, QC) over
// the instance's NW waves (the window of one chunk: 32 channels x the padded channel pitch, in 4-float pieces)
__host__ __device__ constexpr int lp_pitch(int S, int KK, int rows, int cols) {
    const int wr = (rows - 1) * S + KK, wca = (3 + (cols - 1) * S + KK + 3) / 4 * 4;
    int pc = wr * wca;
    while (pc % 64 != 4) pc += 4;
    return pc;
}
__host__ __device__ constexpr int lp_staged_pieces(int S, int KK, int QC, int NW) {
    const int p1 = QC == 32 ? lp_pitch(S, KK, 1, 32) : lp_pitch(S, KK, 1, 16);
    const int p2 = QC == 32 ? lp_pitch(S, KK, 2, 16) : lp_pitch(S, KK, 2, 8);
    const int pc = p1 > p2 ? p1 : p2;
    return (32 * (pc / 4) + 64 * NW - 1) / (64 * NW);
}
constexpr int kLpStagedPieces = 12;   // (upper bound over the instances)

__host__ __device__ constexpr int lp_nb(int S, int KK) { return (3 + 7 * S + KK + 3) / 4; }   // b128 reads per k-step
__host__ __device__ inline int lp_buf_floats(int bm, int qc, int pitch_c) {
    return bm * qc + (kLC * pitch_c + 255) / 256 * 256;
}
// XOR swizzle of a Dense row's 16-B pieces (PPR per row): 16 consecutive rows' fragment reads land on
// distinct bank groups
template <int PPR>
__host__ __device__ constexpr int lp_swz(int row) { return (row >> 1) & (PPR - 1); }

// QC positions per chunk: 32 (two k-steps), or 16 (one; the 2 x 8 planes of the UNet bottom)
// XS = 0: both tiles arrive by LDS DMA (fp32 tensors).  XS = the 16-bit storage type (LDM_DT_X16 / _DY16
// tensors): the tiles are register-staged instead (a DMA cannot widen 16-bit elements to the floats the
// compute side reads): the next chunk's pieces are loaded into registers during this chunk's MFMAs, widened
// and parked in LDS at the addresses the DMA would have written, so the compute side is the same.
template <int S, int KK, int BM, int WM, int QC, int DT, int XS = 0>
__global__ __launch_bounds__(64 * WM * KK) void wgrad_lp_kernel(LpArgs a) {
    constexpr int NW = WM * KK, MF = BM / WM / 32, T = KK * KK, NB = lp_nb(S, KK);
    constexpr int PPR = QC / 4, RPI = 64 / PPR, NKS = QC / 16;   // pieces per row, rows per DMA instr, k-steps
    static_assert(MF >= 1 && MF * 32 * WM == BM, "row split");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ky = wave % KK, wm = wave / KK;
    const int r = lane & 31, h = lane >> 5;
    const int m0 = blockIdx.y * BM, c0 = blockIdx.x * kLC;
    const int HQ = a.Hq * a.Wq;
    const int bufF = lp_buf_floats(BM, QC, a.pitch_c);
    const int ch_begin = blockIdx.z * a.per_split;
    const int ch_end = min(a.nchunk, ch_begin + a.per_split);
    const bool d16 = XS != 0 && a.dense16, g16 = XS != 0 && a.gath16;
    const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(a.dense), (short)0, uni(a.B * a.M * HQ * (d16 ? 2 : 4)), 0x00020000);
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(a.gath), (short)0, uni(a.B * a.C * a.Hg * a.Wg * (g16 ? 2 : 4)), 0x00020000);

    // chunk ch -> sample, first row, first column; its DMAs into buffer buf
    auto issue = [&](int ch, int buf) {
        const int b = ch / a.cps;
        const int rr = ch - b * a.cps;
        int qy0, qx0;
        if (a.cols == a.Wq) {
            qy0 = rr * a.rows, qx0 = 0;
        } else {
            const int segs = a.Wq / QC;
            qy0 = rr / segs, qx0 = (rr - qy0 * segs) * QC;
        }
        char* base = reinterpret_cast<char*>(smem + buf * bufF);
        // Dense: BM rows x PPR pieces; one wave-instruction = RPI rows
        for (int gi = wave; gi < BM / RPI; gi += NW) {
            const int row = gi * RPI + lane / PPR;
            const int sp = (lane % PPR) ^ lp_swz<PPR>(row);   // source piece landing in destination piece lane % PPR
            const int ql = sp * 4;
            const int qy = qy0 + ql / a.cols, qx = qx0 + ql % a.cols;
            const int m = m0 + row;
            const int voff = m < a.M ? (((b * a.M + m) * HQ + qy * a.Wq + qx) * 4) : kOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(dr, (lds_ptr_t)(base + gi * 1024), 16, voff, 0, 0, 0);
        }
        // window [32][pitch_c]: rows of wca floats, pieces past wr * wca in a channel are padding (zeros)
        const int wq4 = a.wca >> 2, pq = a.pitch_c >> 2;
        const int npiece = kLC * pq;
        const int row0 = qy0 * S - 1, colA = qx0 * S - 4;   // pad 1, e = 3
        for (int gi = wave; gi * 64 < npiece; gi += NW) {
            const int pc = gi * 64 + lane;
            const int cl = pc / pq;
            const int rem = pc - cl * pq;
            const int wrow = rem / wq4, wp = rem - wrow * wq4;
            const int c = c0 + cl, iy = row0 + wrow, ix = colA + wp * 4;
            const bool ok = pc < npiece && c < a.C && wrow < a.wr && (unsigned)iy < (unsigned)a.Hg &&
                            (unsigned)ix < (unsigned)a.Wg;
            const int voff = ok ? ((((b * a.C + c) * a.Hg + iy) * a.Wg + ix) * 4) : kOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(gr, (lds_ptr_t)(base + BM * QC * 4 + gi * 1024), 16, voff, 0, 0, 0);
        }
    };

    // ---- register-staged form (XS != 0): the same pieces as issue(), loaded as 16-byte fp32 quads or 8-byte
    //      16-bit quads (element offsets as issue()'s), widened to floats when parked
    constexpr int ND = (BM / RPI + NW - 1) / NW, NWPC = lp_staged_pieces(S, KK, QC, NW);
    static_assert(NWPC <= kLpStagedPieces, "staged window pieces");
    uint4 rd[XS ? ND : 1], rw[XS ? NWPC : 1];
    auto fetch = [&](int ch) {
        const int b = ch / a.cps;
        const int rr = ch - b * a.cps;
        int qy0, qx0;
        if (a.cols == a.Wq) {
            qy0 = rr * a.rows, qx0 = 0;
        } else {
            const int segs = a.Wq / QC;
            qy0 = rr / segs, qx0 = (rr - qy0 * segs) * QC;
        }
#pragma unroll
        for (int i = 0; i < ND; ++i) {
            const int gi = wave + i * NW;
            const int row = gi * RPI + lane / PPR;
            const int sp = (lane % PPR) ^ lp_swz<PPR>(row);
            const int ql = sp * 4;
            const int qy = qy0 + ql / a.cols, qx = qx0 + ql % a.cols;
            const int m = m0 + row;
            const int el = ((b * a.M + m) * HQ + qy * a.Wq + qx);
            const bool ok = gi < BM / RPI && m < a.M;
            if (d16) {
                const uint2 t = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(dr, ok ? el * 2 : kOOB, 0, 0));
                rd[i] = uint4{t.x, t.y, 0u, 0u};
            } else {
                rd[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(dr, ok ? el * 4 : kOOB, 0, 0));
            }
        }
        const int wq4 = a.wca >> 2, pq = a.pitch_c >> 2;
        const int npiece = kLC * pq;
        const int row0 = qy0 * S - 1, colA = qx0 * S - 4;
#pragma unroll
        for (int i = 0; i < NWPC; ++i) {
            const int pc = (wave + i * NW) * 64 + lane;
            const int cl = pc / pq;
            const int rem = pc - cl * pq;
            const int wrow = rem / wq4, wp = rem - wrow * wq4;
            const int c = c0 + cl, iy = row0 + wrow, ix = colA + wp * 4;
            const bool ok = pc < npiece && c < a.C && wrow < a.wr && (unsigned)iy < (unsigned)a.Hg &&
                            (unsigned)ix < (unsigned)a.Wg;
            const int el = (((b * a.C + c) * a.Hg + iy) * a.Wg + ix);
            if (g16) {
                const uint2 t = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(gr, ok ? el * 2 : kOOB, 0, 0));
                rw[i] = uint4{t.x, t.y, 0u, 0u};
            } else {
                rw[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(gr, ok ? el * 4 : kOOB, 0, 0));
            }
        }
    };
    auto widen = [&](const uint4& v, bool h16) {
        if (!h16) return __builtin_bit_cast(floatx4, v);
        return floatx4{from16<XS>((unsigned short)(v.x & 0xffff)), from16<XS>((unsigned short)(v.x >> 16)),
                       from16<XS>((unsigned short)(v.y & 0xffff)), from16<XS>((unsigned short)(v.y >> 16))};
    };
    auto park = [&](int buf) {
        char* base = reinterpret_cast<char*>(smem + buf * bufF);
#pragma unroll
        for (int i = 0; i < ND; ++i) {
            const int gi = wave + i * NW;
            if (gi < BM / RPI) *reinterpret_cast<floatx4*>(base + gi * 1024 + lane * 16) = widen(rd[i], d16);
        }
        const int npiece = kLC * (a.pitch_c >> 2);
#pragma unroll
        for (int i = 0; i < NWPC; ++i) {
            const int gi = wave + i * NW;
            if (gi * 64 < npiece)
                *reinterpret_cast<floatx4*>(base + BM * QC * 4 + gi * 1024 + lane * 16) = widen(rw[i], g16);
        }
    };

    floatx16 acc[MF][KK];
#pragma unroll
    for (int f = 0; f < MF; ++f)
#pragma unroll
        for (int t = 0; t < KK; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[f][t][i] = 0.f;

    // per-lane LDS offsets (floats) inside a buffer for k-step ks: A pieces of fragment f, window run start
    int aoff[NKS][MF][2], boff[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
        const int q0 = ks * 16 + 8 * h;
        const int rl = q0 / a.cols, xl0 = q0 - rl * a.cols;
#pragma unroll
        for (int f = 0; f < MF; ++f) {
            const int row = (wm * MF + f) * 32 + r;
#pragma unroll
            for (int u = 0; u < 2; ++u) aoff[ks][f][u] = row * QC + ((((q0 >> 2) + u) ^ lp_swz<PPR>(row)) << 2);
        }
        boff[ks] = BM * QC + r * a.pitch_c + (rl * S + ky) * a.wca + xl0 * S;
    }

    auto compute = [&](const float* sb) {
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            floatx8 fa[MF];
#pragma unroll
            for (int f = 0; f < MF; ++f) {
                const floatx4 lo = *reinterpret_cast<const floatx4*>(sb + aoff[ks][f][0]);
                const floatx4 hi = *reinterpret_cast<const floatx4*>(sb + aoff[ks][f][1]);
                fa[f] = floatx8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            }
            float v[4 * NB];
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const floatx4 p = *reinterpret_cast<const floatx4*>(sb + boff[ks] + 4 * i);
                v[4 * i + 0] = p[0], v[4 * i + 1] = p[1], v[4 * i + 2] = p[2], v[4 * i + 3] = p[3];
            }
#pragma unroll
            for (int kx = 0; kx < KK; ++kx) {
                floatx8 fb;
#pragma unroll
                for (int j = 0; j < 8; ++j) fb[j] = v[3 + kx + S * j];
#pragma unroll
                for (int f = 0; f < MF; ++f) acc[f][kx] = mma32x16<DT>(fa[f], fb, acc[f][kx]);
            }
        }
    };
    if constexpr (XS == 0) {
        if (ch_begin < ch_end) issue(ch_begin, 0);
        for (int ch = ch_begin; ch < ch_end; ++ch) {
            const int buf = (ch - ch_begin) & 1;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();   // chunk ch landed; every wave is done with the other buffer
            if (ch + 1 < ch_end) issue(ch + 1, buf ^ 1);
            compute(smem + buf * bufF);
        }
    } else {
        if (ch_begin < ch_end) {
            fetch(ch_begin);
            park(0);
        }
        for (int ch = ch_begin; ch < ch_end; ++ch) {
            const int buf = (ch - ch_begin) & 1;
            __syncthreads();   // chunk ch parked by every wave; every wave is done with the other buffer
            const bool more = ch + 1 < ch_end;
            if (more) fetch(ch + 1);   // in flight during this chunk's MFMAs
            compute(smem + buf * bufF);
            if (more) park(buf ^ 1);
        }
    }

    // partial[z][m][c*T + ky*KK + kx]: D col = channel c0 + r, rows (reg & 3) + 8 (reg >> 2) + 4h
    const int c = c0 + r;
    if (c < a.C) {
        float* out = a.partial + (size_t)blockIdx.z * a.M * a.C * T + (size_t)c * T + ky * KK;
#pragma unroll
        for (int f = 0; f < MF; ++f)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int m = m0 + (wm * MF + f) * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
                if (m < a.M) {
                    float* o = out + (size_t)m * a.C * T;
                    if constexpr (KK == 4) {
                        *reinterpret_cast<floatx4*>(o) = floatx4{acc[f][0][reg], acc[f][1][reg], acc[f][2][reg], acc[f][3][reg]};
                    } else {
#pragma unroll
                        for (int kx = 0; kx < KK; ++kx) o[kx] = acc[f][kx][reg];
                    }
                }
            }
    }
}

// ------------------------------------------------------------------------------------------------------
// The double-rate weight gradient on 16-bit maps (both Dense and Gath stored in the operand type, LDM_DT_X16 +
// LDM_DT_DY16): the tiles arrive by LDS DMA as they are stored, 16 bits, and the MFMA operands are read from
// LDS without any conversion.  Same blocks, waves, chunks and k-steps as wgrad_lp_kernel, so the same sums in
// the same order (bitwise equal to the fp32-storage form on the same values).  Layout in 16-bit elements:
//   Dense [BM][QC], 16-B pieces of 8 positions, XOR-swizzled per row pair (a fragment is one ds_read_b128);
//   window [32][pitch16] of rows of wca16 elements from the 8-aligned origin qx0*S - 8 (so e = 7; Wg % 8 == 0:
//   a piece is wholly inside or outside the image row), channel pitch = 8 mod 128 elements.
// B fragment of tap (ky, kx) for positions q0 + j: window elements 7 + kx + S j of the lane's channel row run
// (read as NB16 16-byte loads); stride 2 takes every other 16-bit element (one v_perm per dword), stride 1
// eight consecutive ones (aligned, or a funnel shift).
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
__host__ __device__ constexpr int lp16_nb(int S, int KK) { return (7 + KK + 7 * S + 7) / 8; }   // b128 per k-step
__host__ __device__ inline int lp16_buf_bytes(int bm, int qc, int pitch16) {
    return bm * qc * 2 + (kLC * pitch16 * 2 + 1023) / 1024 * 1024;
}
template <int PPR>
__host__ __device__ constexpr int lp16_swz(int row) { return (row >> 1) & (PPR - 1); }

// 8 consecutive 16-bit elements starting at element `e` (compile-time) of the dword array w, stride S
template <int S, int E, int N>
__device__ __forceinline__ u16x8 lp16_frag(const unsigned (&w)[N]) {
    static_assert((E >> 1) + (S == 2 ? 8 : 5) <= N, "fragment past the loaded run");
    unsigned d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if constexpr (S == 2) {
            // elements E + 4i and E + 4i + 2: the same half of dwords (E + 4i) / 2 and (E + 4i) / 2 + 1
            constexpr int h = E & 1;
            const unsigned lo = w[(E >> 1) + 2 * i], hi = w[(E >> 1) + 2 * i + 1];
            d[i] = h ? ((lo >> 16) | (hi & 0xffff0000u)) : ((lo & 0xffffu) | (hi << 16));
        } else {
            if constexpr ((E & 1) == 0) {
                d[i] = w[(E >> 1) + i];
            } else {
                const unsigned lo = w[(E >> 1) + i], hi = w[(E >> 1) + i + 1];
                d[i] = (lo >> 16) | (hi << 16);
            }
        }
    }
    return __builtin_bit_cast(u16x8, (uint4){d[0], d[1], d[2], d[3]});
}

template <int DT>
__device__ __forceinline__ floatx16 mma16x(const u16x8& a, const u16x8& b, const floatx16& c) {
    if constexpr (DT == 1)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(halfx8, a), __builtin_bit_cast(halfx8, b), c, 0,
                                                      0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                       0, 0, 0);
}

template <int S, int KK, int BM, int WM, int QC, int DT>
__global__ __launch_bounds__(64 * WM * KK) void wgrad_lp16_kernel(LpArgs a) {
    constexpr int NW = WM * KK, MF = BM / WM / 32, T = KK * KK, NB = lp16_nb(S, KK);
    constexpr int PPR = QC / 8, RPI = 64 / PPR, NKS = QC / 16;
    static_assert(MF >= 1 && MF * 32 * WM == BM, "row split");
    extern __shared__ __attribute__((aligned(16))) unsigned short smem16[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ky = wave % KK, wm = wave / KK;
    const int r = lane & 31, h = lane >> 5;
    const int m0 = blockIdx.y * BM, c0 = blockIdx.x * kLC;
    const int HQ = a.Hq * a.Wq;
    const int bufB = lp16_buf_bytes(BM, QC, a.pitch_c);   // (LpArgs.wca / pitch_c hold the 16-bit geometry here)
    const int ch_begin = blockIdx.z * a.per_split;
    const int ch_end = min(a.nchunk, ch_begin + a.per_split);
    const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(a.dense), (short)0, uni(a.B * a.M * HQ * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(a.gath), (short)0, uni(a.B * a.C * a.Hg * a.Wg * 2), 0x00020000);

    auto issue = [&](int ch, int buf) {
        const int b = ch / a.cps;
        const int rr = ch - b * a.cps;
        int qy0, qx0;
        if (a.cols == a.Wq) {
            qy0 = rr * a.rows, qx0 = 0;
        } else {
            const int segs = a.Wq / QC;
            qy0 = rr / segs, qx0 = (rr - qy0 * segs) * QC;
        }
        char* base = reinterpret_cast<char*>(smem16) + buf * bufB;
        for (int gi = wave; gi < BM / RPI; gi += NW) {
            const int row = gi * RPI + lane / PPR;
            const int sp = (lane % PPR) ^ lp16_swz<PPR>(row);
            const int ql = sp * 8;
            const int qy = qy0 + ql / a.cols, qx = qx0 + ql % a.cols;
            const int m = m0 + row;
            const int voff = m < a.M ? (((b * a.M + m) * HQ + qy * a.Wq + qx) * 2) : kOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(dr, (lds_ptr_t)(base + gi * 1024), 16, voff, 0, 0, 0);
        }
        const int wq8 = a.wca >> 3, pq = a.pitch_c >> 3;
        const int npiece = kLC * pq;
        const int row0 = qy0 * S - 1, colA = qx0 * S - 8;   // pad 1, e = 7
        for (int gi = wave; gi * 64 < npiece; gi += NW) {
            const int pc = gi * 64 + lane;
            const int cl = pc / pq;
            const int rem = pc - cl * pq;
            const int wrow = rem / wq8, wp = rem - wrow * wq8;
            const int c = c0 + cl, iy = row0 + wrow, ix = colA + wp * 8;
            const bool ok = pc < npiece && c < a.C && wrow < a.wr && (unsigned)iy < (unsigned)a.Hg &&
                            (unsigned)ix < (unsigned)a.Wg;
            const int voff = ok ? ((((b * a.C + c) * a.Hg + iy) * a.Wg + ix) * 2) : kOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(gr, (lds_ptr_t)(base + BM * QC * 2 + gi * 1024), 16, voff, 0, 0, 0);
        }
    };

    floatx16 acc[MF][KK];
#pragma unroll
    for (int f = 0; f < MF; ++f)
#pragma unroll
        for (int t = 0; t < KK; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[f][t][i] = 0.f;

    // per-lane byte offsets inside a buffer for k-step ks: the A piece of fragment f, the window run start
    int aoff[NKS][MF], boff[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
        const int q0 = ks * 16 + 8 * h;
        const int rl = q0 / a.cols, xl0 = q0 - rl * a.cols;
#pragma unroll
        for (int f = 0; f < MF; ++f) {
            const int row = (wm * MF + f) * 32 + r;
            aoff[ks][f] = row * QC * 2 + (((q0 >> 3) ^ lp16_swz<PPR>(row)) << 4);
        }
        boff[ks] = BM * QC * 2 + (r * a.pitch_c + (rl * S + ky) * a.wca + xl0 * S) * 2;
    }

    if (ch_begin < ch_end) issue(ch_begin, 0);
    for (int ch = ch_begin; ch < ch_end; ++ch) {
        const int buf = (ch - ch_begin) & 1;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();   // chunk ch landed; every wave is done with the other buffer
        if (ch + 1 < ch_end) issue(ch + 1, buf ^ 1);
        const char* sb = reinterpret_cast<const char*>(smem16) + buf * bufB;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            u16x8 fa[MF];
#pragma unroll
            for (int f = 0; f < MF; ++f) fa[f] = *reinterpret_cast<const u16x8*>(sb + aoff[ks][f]);
            unsigned w[4 * NB];
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const uint4 p = *reinterpret_cast<const uint4*>(sb + boff[ks] + 16 * i);
                w[4 * i + 0] = p.x, w[4 * i + 1] = p.y, w[4 * i + 2] = p.z, w[4 * i + 3] = p.w;
            }
            static_for<0, KK>([&](auto kxc) {
                constexpr int kx = decltype(kxc)::value;
                const u16x8 fb = lp16_frag<S, 7 + kx, 4 * NB>(w);
#pragma unroll
                for (int f = 0; f < MF; ++f) acc[f][kx] = mma16x<DT>(fa[f], fb, acc[f][kx]);
            });
        }
    }

    const int c = c0 + r;
    if (c < a.C) {
        float* out = a.partial + (size_t)blockIdx.z * a.M * a.C * T + (size_t)c * T + ky * KK;
#pragma unroll
        for (int f = 0; f < MF; ++f)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int m = m0 + (wm * MF + f) * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
                if (m < a.M) {
                    float* o = out + (size_t)m * a.C * T;
                    if constexpr (KK == 4) {
                        *reinterpret_cast<floatx4*>(o) = floatx4{acc[f][0][reg], acc[f][1][reg], acc[f][2][reg], acc[f][3][reg]};
                    } else {
#pragma unroll
                        for (int kx = 0; kx < KK; ++kx) o[kx] = acc[f][kx][reg];
                    }
                }
            }
    }
}

// The same sums on an NBUF-deep ring of chunk buffers: the double-buffered form keeps one chunk's DMAs (~25 KB
// per CU) in flight, which at the grid's one block per CU leaves the HBM pipe latency-bound (tools/pmc_one_conv.sh:
// 64 -> 128 s2 weight gradient, 172 MB fetched in ~60 us, waves mostly waiting).  Here chunks ch + 1 .. ch + NBUF - 1
// are in flight while chunk ch computes.  Every wave issues exactly NL = ND + NG DMAs per chunk (slots past the
// tile's pieces load nothing into a trash KB), so "chunk ch landed" is one vmcnt immediate; the per-slot offsets
// are chunk-invariant and computed once (the chunk loop walks the chunk coordinates without divisions).  Same
// blocks, chunks, k-steps and fragments as wgrad_lp16_kernel: the sums are bitwise those of the double-buffered
// form.
// Synchronisation (round 6; the round-5 form waited one chunk short and was rescued by hipcc): at iteration k the
// chunks k .. min(n - 1, k + NBUF - 2) are outstanding, so "chunk k landed" is vmcnt(ahead * NL) with ahead the
// chunks issued after k; then a RAW s_barrier (every wave's share of chunk k landed, every wave done reading chunk
// k - 1), then chunk k + NBUF - 1 is issued into chunk k - 1's buffer.  hipcc would drain the ring twice per
// chunk: __syncthreads()'s workgroup fence waits vmcnt(0) (an LDS DMA is a pending LDS write), and an ordinary
// ds_read after any LDS DMA waits for all of them (it may alias).  So the wait + barrier is one asm statement
// and the fragment reads are asm ds_read_b128 that end in their own lgkmcnt(0) (cdna_hip_programming.md §5,
// "Pipelining across barriers"): the emitted loop holds no vmcnt but the counted one.
__host__ __device__ constexpr int lp16_pitch(int S, int KK, int rows, int cols) {
    const int wr = (rows - 1) * S + KK, wca = (7 + (cols - 1) * S + KK + 7) / 8 * 8;
    int pc = wr * wca;
    while (pc % 128 != 8) pc += 8;
    return pc;
}
// the window's 1-KB DMA groups per wave: the larger of the two geometries a QC allows (rows 1 / 2)
__host__ __device__ constexpr int lp16_ng(int S, int KK, int QC, int NW) {
    const int p1 = lp16_pitch(S, KK, 1, QC), p2 = lp16_pitch(S, KK, 2, QC / 2);
    const int pmax = p1 > p2 ? p1 : p2;
    const int groups = (kLC * pmax / 8 + 63) / 64;
    return (groups + NW - 1) / NW;
}

// this wave's DMAs but the N youngest have landed, then the block's raw barrier (no fence: see above)
template <int N>
__device__ __forceinline__ void lp_wait_vm_barrier() {
    static_assert(N >= 0 && N <= 63, "vmcnt immediate");
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
// a ds_read_b128 the compiler's waitcnt pass does not see (the caller waits lgkmcnt(0) before the use)
__device__ __forceinline__ u32x4 lp_lds_read(const char* p) {
    u32x4 v;
    const unsigned addr = (unsigned)(uintptr_t)(lds_ptr_t)p;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
    return v;
}

template <int S, int KK, int BM, int WM, int QC, int DT, int NBUF>
__global__ __launch_bounds__(64 * WM * KK) void wgrad_lp16p_kernel(LpArgs a) {
    constexpr int NW = WM * KK, MF = BM / WM / 32, T = KK * KK, NB = lp16_nb(S, KK);
    constexpr int PPR = QC / 8, RPI = 64 / PPR, NKS = QC / 16;
    constexpr int NDG = BM / RPI, ND = (NDG + NW - 1) / NW, NG = lp16_ng(S, KK, QC, NW), NL = ND + NG;
    static_assert(MF >= 1 && MF * 32 * WM == BM, "row split");
    static_assert(NBUF >= 3 && (NBUF - 2) * NL <= 63, "ring depth (vmcnt immediate)");
    extern __shared__ __attribute__((aligned(16))) unsigned short smem16[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ky = wave % KK, wm = wave / KK;
    const int r = lane & 31, h = lane >> 5;
    const int m0 = blockIdx.y * BM, c0 = blockIdx.x * kLC;
    const int HQ = a.Hq * a.Wq;
    const int bufB = lp16_buf_bytes(BM, QC, a.pitch_c);
    char* const trash = reinterpret_cast<char*>(smem16) + NBUF * bufB;
    const int ch_begin = blockIdx.z * a.per_split;
    const int ch_end = min(a.nchunk, ch_begin + a.per_split);
    const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(a.dense), (short)0, uni(a.B * a.M * HQ * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(
        uni_ptr(a.gath), (short)0, uni(a.B * a.C * a.Hg * a.Wg * 2), 0x00020000);

    // chunk-invariant slot offsets (elements): Dense row m's position run, window piece (channel, row, column)
    int doff[ND], goff[NG], grow[NG], gcol[NG];
#pragma unroll
    for (int j = 0; j < ND; ++j) {
        const int gi = wave + j * NW;
        const int row = gi * RPI + lane / PPR;
        const int ql = (((lane % PPR) ^ lp16_swz<PPR>(row))) * 8;
        const int m = m0 + row;
        doff[j] = (gi < NDG && m < a.M) ? m * HQ + (ql / a.cols) * a.Wq + ql % a.cols : -1;
    }
    const int wq8 = a.wca >> 3, pq = a.pitch_c >> 3, npiece = kLC * pq;
#pragma unroll
    for (int j = 0; j < NG; ++j) {
        const int pc = (wave + j * NW) * 64 + lane;
        const int cl = pc / pq, rem = pc - (pc / pq) * pq;
        const int wrow = rem / wq8, wx = (rem - wrow * wq8) * 8;
        const bool ok = pc < npiece && c0 + cl < a.C && wrow < a.wr;
        goff[j] = ((c0 + cl) * a.Hg + wrow) * a.Wg + wx;
        grow[j] = ok ? wrow : -(1 << 20);   // (an invalid piece fails the row test of every chunk)
        gcol[j] = wx;
    }

    auto issue = [&](int buf, int b, int qy0, int qx0) {
        char* base = reinterpret_cast<char*>(smem16) + buf * bufB;
        const int dbase = b * a.M * HQ + qy0 * a.Wq + qx0;
#pragma unroll
        for (int j = 0; j < ND; ++j) {
            const int gi = wave + j * NW;
            const int voff = doff[j] >= 0 ? (dbase + doff[j]) * 2 : kOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(dr, (lds_ptr_t)(gi < NDG ? base + gi * 1024 : trash), 16, voff, 0, 0, 0);
        }
        const int row0 = qy0 * S - 1, colA = qx0 * S - 8;   // pad 1, e = 7
        const int gbase = (b * a.C * a.Hg + row0) * a.Wg + colA;
#pragma unroll
        for (int j = 0; j < NG; ++j) {
            const int gi = wave + j * NW;
            const bool ok = (unsigned)(row0 + grow[j]) < (unsigned)a.Hg && (unsigned)(colA + gcol[j]) < (unsigned)a.Wg;
            const int voff = ok ? (gbase + goff[j]) * 2 : kOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(gr, (lds_ptr_t)(gi * 64 < npiece ? base + BM * QC * 2 + gi * 1024 : trash),
                                                     16, voff, 0, 0, 0);
        }
    };

    floatx16 acc[MF][KK];
#pragma unroll
    for (int f = 0; f < MF; ++f)
#pragma unroll
        for (int t = 0; t < KK; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[f][t][i] = 0.f;

    int aoff[NKS][MF], boff[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
        const int q0 = ks * 16 + 8 * h;
        const int rl = q0 / a.cols, xl0 = q0 - rl * a.cols;
#pragma unroll
        for (int f = 0; f < MF; ++f) {
            const int row = (wm * MF + f) * 32 + r;
            aoff[ks][f] = row * QC * 2 + (((q0 >> 3) ^ lp16_swz<PPR>(row)) << 4);
        }
        boff[ks] = BM * QC * 2 + (r * a.pitch_c + (rl * S + ky) * a.wca + xl0 * S) * 2;
    }

    // the issue cursor (chunk ch_begin + k, walked without divisions): sample, chunk row / column origin
    int ib = ch_begin / a.cps, iqy, iqx;
    {
        const int rr = ch_begin - ib * a.cps;
        if (a.cols == a.Wq) {
            iqy = rr * a.rows, iqx = 0;
        } else {
            const int segs = a.Wq / QC;
            iqy = rr / segs, iqx = (rr - iqy * segs) * QC;
        }
    }
    auto advance = [&]() {
        iqx += a.cols;
        if (iqx >= a.Wq) {
            iqx = 0, iqy += a.rows;
            if (iqy >= a.Hq) iqy = 0, ++ib;
        }
    };
    const int n = ch_end - ch_begin;
#pragma unroll
    for (int k = 0; k < NBUF - 1; ++k)
        if (k < n) issue(k, ib, iqy, iqx), advance();
    int buf = 0, ibuf = NBUF - 1;   // ibuf = (k + NBUF - 1) % NBUF: chunk k - 1's buffer
    for (int k = 0; k < n; ++k) {
        // outstanding: chunks k .. k + ahead; chunk k must land, the ahead younger ones may stay in flight
        const int ahead = min(n - 1 - k, NBUF - 2);
        if constexpr (NBUF == 3) {
            if (ahead >= 1) lp_wait_vm_barrier<NL>(); else lp_wait_vm_barrier<0>();
        } else {
            static_assert(NBUF == 4, "ring depth 3 or 4");
            if (ahead >= 2) lp_wait_vm_barrier<2 * NL>(); else if (ahead == 1) lp_wait_vm_barrier<NL>(); else lp_wait_vm_barrier<0>();
        }
        // chunk k landed for every wave; every wave is done with chunk k - 1's buffer: refill it
        if (k + NBUF - 1 < n) {
            issue(ibuf, ib, iqy, iqx);
            advance();
        }
        ibuf = ibuf + 1 == NBUF ? 0 : ibuf + 1;
        const char* sb = reinterpret_cast<const char*>(smem16) + buf * bufB;
        buf = buf + 1 == NBUF ? 0 : buf + 1;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            u32x4 ra[MF], rb[NB];
#pragma unroll
            for (int f = 0; f < MF; ++f) ra[f] = lp_lds_read(sb + aoff[ks][f]);
#pragma unroll
            for (int i = 0; i < NB; ++i) rb[i] = lp_lds_read(sb + boff[ks] + 16 * i);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int f = 0; f < MF; ++f) asm volatile("" : "+v"(ra[f]));
#pragma unroll
            for (int i = 0; i < NB; ++i) asm volatile("" : "+v"(rb[i]));
            u16x8 fa[MF];
#pragma unroll
            for (int f = 0; f < MF; ++f) fa[f] = __builtin_bit_cast(u16x8, ra[f]);
            unsigned w[4 * NB];
#pragma unroll
            for (int i = 0; i < NB; ++i) w[4 * i + 0] = rb[i][0], w[4 * i + 1] = rb[i][1], w[4 * i + 2] = rb[i][2], w[4 * i + 3] = rb[i][3];
            static_for<0, KK>([&](auto kxc) {
                constexpr int kx = decltype(kxc)::value;
                const u16x8 fb = lp16_frag<S, 7 + kx, 4 * NB>(w);
#pragma unroll
                for (int f = 0; f < MF; ++f) acc[f][kx] = mma16x<DT>(fa[f], fb, acc[f][kx]);
            });
        }
    }

    const int c = c0 + r;
    if (c < a.C) {
        float* out = a.partial + (size_t)blockIdx.z * a.M * a.C * T + (size_t)c * T + ky * KK;
#pragma unroll
        for (int f = 0; f < MF; ++f)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int m = m0 + (wm * MF + f) * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
                if (m < a.M) {
                    float* o = out + (size_t)m * a.C * T;
                    if constexpr (KK == 4) {
                        *reinterpret_cast<floatx4*>(o) = floatx4{acc[f][0][reg], acc[f][1][reg], acc[f][2][reg], acc[f][3][reg]};
                    } else {
#pragma unroll
                        for (int kx = 0; kx < KK; ++kx) o[kx] = acc[f][kx][reg];
                    }
                }
            }
    }
}

// The fp32-map form (wgrad_lp_kernel, XS = 0: the train step's UNet layers, whose maps stay fp32) on the same
// NBUF-deep ring as wgrad_lp16p_kernel (round 6): the double-buffered form waited vmcnt(0) + __syncthreads() per
// chunk and hipcc drained its one in-flight DMA before the first ds_read, so every chunk paid a whole memory round
// trip.  Here every wave issues exactly NL = ND + NG DMAs per chunk (slots past the tile's pieces load nothing
// into a trash KB), "chunk k landed" is vmcnt(ahead * NL) + a raw s_barrier, chunk k + NBUF - 1 refills chunk
// k - 1's buffer, and the fragment reads are asm ds_read_b128 (see wgrad_lp16p_kernel).  Same blocks, chunks,
// k-steps, fragments and MFMA order as wgrad_lp_kernel: bitwise its sums.
template <int S, int KK, int BM, int WM, int QC, int DT, int NBUF>
__global__ __launch_bounds__(64 * WM * KK) void wgrad_lpp_kernel(LpArgs a) {
    constexpr int NW = WM * KK, MF = BM / WM / 32, T = KK * KK, NB = lp_nb(S, KK);
    constexpr int PPR = QC / 4, RPI = 64 / PPR, NKS = QC / 16;
    constexpr int NDG = BM / RPI, ND = (NDG + NW - 1) / NW, NG = lp_staged_pieces(S, KK, QC, NW), NL = ND + NG;
    static_assert(MF >= 1 && MF * 32 * WM == BM, "row split");
    static_assert(NBUF >= 3 && NBUF <= 4 && (NBUF - 2) * NL <= 63, "ring depth (vmcnt immediate)");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ky = wave % KK, wm = wave / KK;
    const int r = lane & 31, h = lane >> 5;
    const int m0 = blockIdx.y * BM, c0 = blockIdx.x * kLC;
    const int HQ = a.Hq * a.Wq;
    const int bufF = lp_buf_floats(BM, QC, a.pitch_c);
    char* const trash = reinterpret_cast<char*>(smem + NBUF * bufF);
    const int ch_begin = blockIdx.z * a.per_split;
    const int ch_end = min(a.nchunk, ch_begin + a.per_split);
    const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(uni_ptr(a.dense), (short)0, uni(a.B * a.M * HQ * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(uni_ptr(a.gath), (short)0, uni(a.B * a.C * a.Hg * a.Wg * 4), 0x00020000);

    // chunk-invariant slot offsets (floats): Dense row m's 4-position piece, window piece (channel, row, column)
    int doff[ND], goff[NG], grow[NG], gcol[NG];
#pragma unroll
    for (int j = 0; j < ND; ++j) {
        const int gi = wave + j * NW;
        const int row = gi * RPI + lane / PPR;
        const int ql = ((lane % PPR) ^ lp_swz<PPR>(row)) * 4;
        const int m = m0 + row;
        doff[j] = (gi < NDG && m < a.M) ? m * HQ + (ql / a.cols) * a.Wq + ql % a.cols : -1;
    }
    const int wq4 = a.wca >> 2, pq = a.pitch_c >> 2, npiece = kLC * pq;
#pragma unroll
    for (int j = 0; j < NG; ++j) {
        const int pc = (wave + j * NW) * 64 + lane;
        const int cl = pc / pq, rem = pc - (pc / pq) * pq;
        const int wrow = rem / wq4, wx = (rem - wrow * wq4) * 4;
        const bool ok = pc < npiece && c0 + cl < a.C && wrow < a.wr;
        goff[j] = ((c0 + cl) * a.Hg + wrow) * a.Wg + wx;
        grow[j] = ok ? wrow : -(1 << 20);   // (an invalid piece fails the row test of every chunk)
        gcol[j] = wx;
    }
    auto issue = [&](int buf, int b, int qy0, int qx0) {
        char* base = reinterpret_cast<char*>(smem + buf * bufF);
        const int dbase = b * a.M * HQ + qy0 * a.Wq + qx0;
#pragma unroll
        for (int j = 0; j < ND; ++j) {
            const int gi = wave + j * NW;
            const int voff = doff[j] >= 0 ? (dbase + doff[j]) * 4 : kOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(dr, (lds_ptr_t)(gi < NDG ? base + gi * 1024 : trash), 16, voff, 0, 0, 0);
        }
        const int row0 = qy0 * S - 1, colA = qx0 * S - 4;   // pad 1, e = 3
        const int gbase = (b * a.C * a.Hg + row0) * a.Wg + colA;
#pragma unroll
        for (int j = 0; j < NG; ++j) {
            const int gi = wave + j * NW;
            const bool ok = (unsigned)(row0 + grow[j]) < (unsigned)a.Hg && (unsigned)(colA + gcol[j]) < (unsigned)a.Wg;
            const int voff = ok ? (gbase + goff[j]) * 4 : kOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(gr, (lds_ptr_t)(gi * 64 < npiece ? base + BM * QC * 4 + gi * 1024 : trash),
                                                     16, voff, 0, 0, 0);
        }
    };

    floatx16 acc[MF][KK];
#pragma unroll
    for (int f = 0; f < MF; ++f)
#pragma unroll
        for (int t = 0; t < KK; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[f][t][i] = 0.f;
    // per-lane LDS byte offsets inside a buffer for k-step ks: A pieces of fragment f, window run start
    int aoff[NKS][MF][2], boff[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
        const int q0 = ks * 16 + 8 * h;
        const int rl = q0 / a.cols, xl0 = q0 - rl * a.cols;
#pragma unroll
        for (int f = 0; f < MF; ++f) {
            const int row = (wm * MF + f) * 32 + r;
#pragma unroll
            for (int u = 0; u < 2; ++u) aoff[ks][f][u] = (row * QC + ((((q0 >> 2) + u) ^ lp_swz<PPR>(row)) << 2)) * 4;
        }
        boff[ks] = (BM * QC + r * a.pitch_c + (rl * S + ky) * a.wca + xl0 * S) * 4;
    }

    int ib = ch_begin / a.cps, iqy, iqx;   // the issue cursor, walked without divisions
    {
        const int rr = ch_begin - ib * a.cps;
        if (a.cols == a.Wq) {
            iqy = rr * a.rows, iqx = 0;
        } else {
            const int segs = a.Wq / QC;
            iqy = rr / segs, iqx = (rr - iqy * segs) * QC;
        }
    }
    auto advance = [&]() {
        iqx += a.cols;
        if (iqx >= a.Wq) {
            iqx = 0, iqy += a.rows;
            if (iqy >= a.Hq) iqy = 0, ++ib;
        }
    };
    const int n = ch_end - ch_begin;
#pragma unroll
    for (int k = 0; k < NBUF - 1; ++k)
        if (k < n) issue(k, ib, iqy, iqx), advance();
    int buf = 0, ibuf = NBUF - 1;
    for (int k = 0; k < n; ++k) {
        const int ahead = min(n - 1 - k, NBUF - 2);
        if constexpr (NBUF == 3) {
            if (ahead >= 1) lp_wait_vm_barrier<NL>(); else lp_wait_vm_barrier<0>();
        } else {
            if (ahead >= 2) lp_wait_vm_barrier<2 * NL>(); else if (ahead == 1) lp_wait_vm_barrier<NL>(); else lp_wait_vm_barrier<0>();
        }
        if (k + NBUF - 1 < n) {
            issue(ibuf, ib, iqy, iqx);
            advance();
        }
        ibuf = ibuf + 1 == NBUF ? 0 : ibuf + 1;
        const char* sb = reinterpret_cast<const char*>(smem + buf * bufF);
        buf = buf + 1 == NBUF ? 0 : buf + 1;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            u32x4 ra[MF][2], rb[NB];
#pragma unroll
            for (int f = 0; f < MF; ++f)
#pragma unroll
                for (int u = 0; u < 2; ++u) ra[f][u] = lp_lds_read(sb + aoff[ks][f][u]);
#pragma unroll
            for (int i = 0; i < NB; ++i) rb[i] = lp_lds_read(sb + boff[ks] + 16 * i);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int f = 0; f < MF; ++f)
#pragma unroll
                for (int u = 0; u < 2; ++u) asm volatile("" : "+v"(ra[f][u]));
#pragma unroll
            for (int i = 0; i < NB; ++i) asm volatile("" : "+v"(rb[i]));
            floatx8 fa[MF];
#pragma unroll
            for (int f = 0; f < MF; ++f) {
                const floatx4 lo = __builtin_bit_cast(floatx4, ra[f][0]), hi = __builtin_bit_cast(floatx4, ra[f][1]);
                fa[f] = floatx8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            }
            float v[4 * NB];
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const floatx4 p = __builtin_bit_cast(floatx4, rb[i]);
                v[4 * i + 0] = p[0], v[4 * i + 1] = p[1], v[4 * i + 2] = p[2], v[4 * i + 3] = p[3];
            }
#pragma unroll
            for (int kx = 0; kx < KK; ++kx) {
                floatx8 fb;
#pragma unroll
                for (int j = 0; j < 8; ++j) fb[j] = v[3 + kx + S * j];
#pragma unroll
                for (int f = 0; f < MF; ++f) acc[f][kx] = mma32x16<DT>(fa[f], fb, acc[f][kx]);
            }
        }
    }

    const int c = c0 + r;
    if (c < a.C) {
        float* out = a.partial + (size_t)blockIdx.z * a.M * a.C * T + (size_t)c * T + ky * KK;
#pragma unroll
        for (int f = 0; f < MF; ++f)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int m = m0 + (wm * MF + f) * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
                if (m < a.M) {
                    float* o = out + (size_t)m * a.C * T;
                    if constexpr (KK == 4) {
                        *reinterpret_cast<floatx4*>(o) = floatx4{acc[f][0][reg], acc[f][1][reg], acc[f][2][reg], acc[f][3][reg]};
                    } else {
#pragma unroll
                        for (int kx = 0; kx < KK; ++kx) o[kx] = acc[f][kx][reg];
                    }
                }
            }
    }
}

struct LpPlan {
    int S, KK, BM, WM, QC, splits, lds_bytes;
    int lds16;   // 1: a and lds_bytes hold the 16-bit geometry (wgrad_lp16_kernel)
    int nbuf;    // the 16-bit form's chunk ring depth: 2 (wgrad_lp16_kernel) or 3 / 4 (wgrad_lp16p_kernel)
    LpArgs a;
};

// 16-bit form: pad 1, k 3 / 4, stride 1 / 2, rows of 16 or a multiple of 32 positions, C >= 16.  K is
// split over blocks until the grid covers the 256 CUs (one block per CU: the double buffer takes
// 60-110 KB of LDS); the workspace query (wgrad2_plan_ws) sizes the partials for the larger of the forms.
bool lp_plan(const ldm_conv_desc& d, LpPlan& p) {
    if (d.kh != d.kw || (d.kh != 3 && d.kh != 4) || (d.stride != 1 && d.stride != 2) || d.pad != 1) return false;
    LpArgs a{};
    a.B = d.B;
    if (!d.transposed) {
        a.M = d.Cout, a.C = d.Cin, a.Hq = d.Hout, a.Wq = d.Wout, a.Hg = d.Hin, a.Wg = d.Win;
    } else {
        a.M = d.Cin, a.C = d.Cout, a.Hq = d.Hin, a.Wq = d.Win, a.Hg = d.Hout, a.Wg = d.Wout;
    }
    if (a.C < 16 || a.Wg % 4) return false;
    int qc = 32;
    if (a.Wq % 32 == 0) {
        a.cols = 32, a.rows = 1;
    } else if (a.Wq == 16 && a.Hq % 2 == 0) {
        a.cols = 16, a.rows = 2;
    } else if (a.Wq == 16) {
        qc = 16, a.cols = 16, a.rows = 1;
    } else if (a.Wq == 8 && a.Hq % 2 == 0) {
        qc = 16, a.cols = 8, a.rows = 2;
    } else {
        return false;
    }
    const int S = d.stride, KK = d.kh;
    p.QC = qc;
    a.cps = a.Hq * a.Wq / qc;
    a.nchunk = a.B * a.cps;
    a.wr = (a.rows - 1) * S + KK;
    a.wca = (3 + (a.cols - 1) * S + KK + 3) / 4 * 4;
    int pc = a.wr * a.wca;
    while (pc % 64 != 4) pc += 4;
    a.pitch_c = pc;
    p.S = S, p.KK = KK;
    p.BM = a.M >= 128 ? 128 : (a.M > 32 ? 64 : 32);
    p.WM = p.BM == 128 ? 2 : 1;
    p.lds_bytes = 2 * lp_buf_floats(p.BM, qc, a.pitch_c) * 4;
    p.lds16 = 0;
    p.nbuf = 2;
    if (p.lds_bytes > 160 * 1024) return false;
    const int tiles = ((a.M + p.BM - 1) / p.BM) * ((a.C + kLC - 1) / kLC);
    static const int smax = [] {   // LDM_WGRAD_SPLITS: the largest K split (A/B timing; default 256)
        const char* e = std::getenv("LDM_WGRAD_SPLITS");
        const int v = e ? (int)std::strtol(e, nullptr, 0) : 256;
        return v < 1 ? 1 : (v > 256 ? 256 : v);
    }();
    int s = 1;
    while (s < smax && tiles * s < 256 && a.nchunk / (s * 2) >= 4) s *= 2;
    p.splits = s;
    a.per_split = (a.nchunk + s - 1) / s;
    p.a = a;
    return true;
}

// the 16-bit geometry of a plan (wgrad_lp16_kernel): window rows of wca16 elements from the 8-aligned origin,
// channel pitch = 8 mod 128 elements; false when Wg % 8 != 0 or the double buffer exceeds the LDS
bool lp16_plan(LpPlan& p) {
    LpArgs& a = p.a;
    if (a.Wg % 8) return false;
    a.wca = (7 + (a.cols - 1) * p.S + p.KK + 7) / 8 * 8;
    int pc = a.wr * a.wca;
    while (pc % 128 != 8) pc += 8;
    a.pitch_c = pc;
    p.lds_bytes = 2 * lp16_buf_bytes(p.BM, p.QC, a.pitch_c) + 64;   // (+ the tail a last run may read past)
    if (p.lds_bytes > 160 * 1024) return false;
    // the ring (wgrad_lp16p_kernel): LDM_WGRAD_RING = 2 / 3 / 4 (default 3: train step 3.279-3.282 ms against 3.288-3.304 with 4, gpurun_out/trab7), shallower where the LDS is short
    static const int ring = [] {
        const char* e = std::getenv("LDM_WGRAD_RING");
        const int v = e ? (int)std::strtol(e, nullptr, 0) : 3;
        return v < 2 ? 2 : (v > 4 ? 4 : v);
    }();
    p.nbuf = 2;
    for (int nb = ring; nb >= 3; --nb) {
        const int bytes = nb * lp16_buf_bytes(p.BM, p.QC, a.pitch_c) + 1024 + 64;   // (+ the trash KB)
        if (bytes <= 160 * 1024) {
            p.nbuf = nb;
            p.lds_bytes = bytes;
            break;
        }
    }
    return true;
}

// the fp32-map ring (wgrad_lpp_kernel): the depth LDM_WGRAD_RING asks for (default 3), shallower where the LDS is
// short; 2 keeps the double-buffered wgrad_lp_kernel
static int lp_ring_depth() {
    static const int ring = [] {
        const char* e = std::getenv("LDM_WGRAD_RING");
        const int v = e ? (int)std::strtol(e, nullptr, 0) : 3;
        return v < 2 ? 2 : (v > 4 ? 4 : v);
    }();
    return ring;
}
void lp32_ring(LpPlan& p) {
    for (int nb = lp_ring_depth(); nb >= 3; --nb) {
        const int bytes = nb * lp_buf_floats(p.BM, p.QC, p.a.pitch_c) * 4 + 1024;   // (+ the trash KB)
        if (bytes <= 160 * 1024) {
            p.nbuf = nb;
            p.lds_bytes = bytes;
            return;
        }
    }
}

template <int S, int KK, int BM, int WM, int QC, int DT, int NBUF>
int launch_lpp(const LpPlan& p, hipStream_t st) {
    constexpr int NW = WM * KK;
    LDM_REQUIRE((kLC * (p.a.pitch_c / 4) + 63) / 64 <= lp_staged_pieces(S, KK, QC, NW) * NW, "wgrad ring (fp32): window slots");
    LDM_REQUIRE(p.a.cols * p.a.rows == QC, "wgrad ring (fp32): chunk geometry");
    auto kfn = wgrad_lpp_kernel<S, KK, BM, WM, QC, DT, NBUF>;
    static bool opted = false;
    if (!opted) {
        LDM_HIP_TRY(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        opted = true;
    }
    dim3 grid((p.a.C + kLC - 1) / kLC, (p.a.M + BM - 1) / BM, p.splits);
    hipLaunchKernelGGL(kfn, grid, dim3(64 * NW), p.lds_bytes, st, p.a);
    LDM_CHECK_LAUNCH("wgrad_lpp_kernel");
    return 0;
}

template <int S, int KK, int BM, int WM, int QC, int DT>
int launch_lp16(const LpPlan& p, hipStream_t st) {
    auto kfn = wgrad_lp16_kernel<S, KK, BM, WM, QC, DT>;
    static bool opted = false;
    if (!opted) {
        LDM_HIP_TRY(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        opted = true;
    }
    dim3 grid((p.a.C + kLC - 1) / kLC, (p.a.M + BM - 1) / BM, p.splits);
    hipLaunchKernelGGL(kfn, grid, dim3(64 * WM * KK), p.lds_bytes, st, p.a);
    LDM_CHECK_LAUNCH("wgrad_lp16_kernel");
    return 0;
}

template <int S, int KK, int BM, int WM, int QC, int DT, int NBUF>
int launch_lp16p(const LpPlan& p, hipStream_t st) {
    constexpr int NW = WM * KK;
    // the slot counts the kernel assumes cover this plan's pieces (its window groups fit NG slots per wave)
    LDM_REQUIRE((kLC * (p.a.pitch_c / 8) + 63) / 64 <= lp16_ng(S, KK, QC, NW) * NW, "wgrad ring: window slots");
    LDM_REQUIRE(p.a.cols * p.a.rows == QC, "wgrad ring: chunk geometry");
    auto kfn = wgrad_lp16p_kernel<S, KK, BM, WM, QC, DT, NBUF>;
    static bool opted = false;
    if (!opted) {
        LDM_HIP_TRY(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        opted = true;
    }
    dim3 grid((p.a.C + kLC - 1) / kLC, (p.a.M + BM - 1) / BM, p.splits);
    hipLaunchKernelGGL(kfn, grid, dim3(64 * NW), p.lds_bytes, st, p.a);
    LDM_CHECK_LAUNCH("wgrad_lp16p_kernel");
    return 0;
}

template <int S, int KK, int BM, int WM, int QC, int DT, int XS>
int launch_lp_xs(const LpPlan& p, hipStream_t st) {
    auto kfn = wgrad_lp_kernel<S, KK, BM, WM, QC, DT, XS>;
    static bool opted = false;
    if (!opted) {
        LDM_HIP_TRY(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        opted = true;
    }
    dim3 grid((p.a.C + kLC - 1) / kLC, (p.a.M + BM - 1) / BM, p.splits);
    hipLaunchKernelGGL(kfn, grid, dim3(64 * WM * KK), p.lds_bytes, st, p.a);
    LDM_CHECK_LAUNCH("wgrad_lp_kernel");
    return 0;
}
template <int S, int KK, int BM, int WM, int QC, int DT>
int launch_lp_dt(const LpPlan& p, hipStream_t st) {
    if (p.a.dense16 && p.a.gath16 && p.lds16) {   // both 16-bit
        if (p.nbuf == 4) return launch_lp16p<S, KK, BM, WM, QC, DT, 4>(p, st);
        if (p.nbuf == 3) return launch_lp16p<S, KK, BM, WM, QC, DT, 3>(p, st);
        return launch_lp16<S, KK, BM, WM, QC, DT>(p, st);
    }
    if (p.a.dense16 || p.a.gath16) return launch_lp_xs<S, KK, BM, WM, QC, DT, DT>(p, st);
    if (p.nbuf == 4) return launch_lpp<S, KK, BM, WM, QC, DT, 4>(p, st);
    if (p.nbuf == 3) return launch_lpp<S, KK, BM, WM, QC, DT, 3>(p, st);
    return launch_lp_xs<S, KK, BM, WM, QC, DT, 0>(p, st);
}
template <int S, int KK, int QC, int DT>
int launch_lp_bm(const LpPlan& p, hipStream_t st) {
    switch (p.BM) {
        case 128: return launch_lp_dt<S, KK, 128, 2, QC, DT>(p, st);
        case 64: return launch_lp_dt<S, KK, 64, 1, QC, DT>(p, st);
        default: return launch_lp_dt<S, KK, 32, 1, QC, DT>(p, st);
    }
}
template <int S, int KK, int DT>
int launch_lp_qc(const LpPlan& p, hipStream_t st) {
    return p.QC == 16 ? launch_lp_bm<S, KK, 16, DT>(p, st) : launch_lp_bm<S, KK, 32, DT>(p, st);
}
template <int DT>
int launch_lp(const LpPlan& p, hipStream_t st) {
    switch (p.S * 10 + p.KK) {
        case 13: return launch_lp_qc<1, 3, DT>(p, st);
        case 23: return launch_lp_qc<2, 3, DT>(p, st);
        case 14: return launch_lp_qc<1, 4, DT>(p, st);
        default: return launch_lp_qc<2, 4, DT>(p, st);
    }
}

struct Plan {
    int S, KK, BM, BC, splits;
    Args a;
    int lds_bytes;
};

// Geometry and instance choice; false when this form does not apply (the caller keeps backward.hip's).
bool plan(const ldm_conv_desc& d, Plan& p) {
    if (d.kh != d.kw || (d.kh != 3 && d.kh != 4) || (d.stride != 1 && d.stride != 2) || d.pad < 0 || d.pad > 3)
        return false;
    Args a{};
    a.B = d.B;
    if (!d.transposed) {
        a.M = d.Cout, a.C = d.Cin, a.Hq = d.Hout, a.Wq = d.Wout, a.Hg = d.Hin, a.Wg = d.Win;
    } else {
        a.M = d.Cin, a.C = d.Cout, a.Hq = d.Hin, a.Wq = d.Win, a.Hg = d.Hout, a.Wg = d.Wout;
    }
    a.pad = d.pad;
    if (a.Wq % 4 || a.Wg % 4) return false;
    if (a.Wq >= kKQ ? (a.Wq % kKQ != 0) : (kKQ % a.Wq != 0)) return false;
    a.cols = a.Wq >= kKQ ? kKQ : a.Wq;
    a.rows = kKQ / a.cols;
    if (a.rows > a.Hq) a.rows = a.Hq;   // a small image: one chunk per sample, the rest zero-padded
    a.cps = a.Wq >= kKQ ? a.Hq * (a.Wq / kKQ) : (a.Hq + a.rows - 1) / a.rows;
    a.nchunk = a.B * a.cps;
    const int KK = d.kh, S = d.stride;
    a.e = ((a.pad % 4) == 0) ? 0 : 4 - (a.pad % 4);          // origin qx0*S - pad, qx0*S a multiple of 4
    a.wr = (a.rows - 1) * S + KK;
    const int wc = (a.cols - 1) * S + KK;
    a.wca = (a.e + wc + 3) / 4 * 4;
    a.pitch_c = a.wr * a.wca;
    p.S = S, p.KK = KK;
    p.BC = a.C == 1 ? 1 : (a.C <= 16 || KK == 4) ? 16 : 32;
    p.BM = (p.BC == 32 && a.M <= 32) ? 32 : 64;
    p.lds_bytes = 2 * buf_floats(p.BM * kKQ, p.BC, a.pitch_c) * 4;
    if (p.lds_bytes > 160 * 1024) return false;
    const int tiles = ((a.M + p.BM - 1) / p.BM) * ((a.C + p.BC - 1) / p.BC);
    // the one-channel kernel keeps 4 blocks per CU resident: up to 1024 splits
    const int smax = p.BC == 1 ? 1024 : 256, want = p.BC == 1 ? 1024 : 512;
    int s = 1;
    while (s < smax && tiles * s < want && a.nchunk / (s * 2) >= 2) s *= 2;
    p.splits = s;
    a.per_split = (a.nchunk + s - 1) / s;
    p.a = a;
    return true;
}

template <int S, int KK, int BM, int BC, int DT>
int launch_dt(const Plan& p, hipStream_t st) {
    auto kfn = wgrad_kernel<S, KK, BM, BC, DT>;
    static bool opted = false;
    if (!opted) {
        LDM_HIP_TRY(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        opted = true;
    }
    dim3 grid((p.a.C + BC - 1) / BC, (p.a.M + BM - 1) / BM, p.splits);
    hipLaunchKernelGGL(kfn, grid, dim3(256), p.lds_bytes, st, p.a);
    LDM_CHECK_LAUNCH("wgrad_kernel (tap-shared)");
    return 0;
}

template <int S, int KK, int DT>
int launch_c1_dt(const Plan& p, hipStream_t st) {
    dim3 grid(1, (p.a.M + 63) / 64, p.splits);
    if (DT != 0 && p.a.dense16)
        hipLaunchKernelGGL((wgrad_c1_kernel<S, KK, DT, DT>), grid, dim3(256), p.lds_bytes, st, p.a);
    else
        hipLaunchKernelGGL((wgrad_c1_kernel<S, KK, DT, 0>), grid, dim3(256), p.lds_bytes, st, p.a);
    LDM_CHECK_LAUNCH("wgrad_c1_kernel");
    return 0;
}
template <int S, int KK>
int launch_c1(const Plan& p, hipStream_t st) {
    switch (p.a.lowp) {
        case LDM_DT_F32: return launch_c1_dt<S, KK, 0>(p, st);
        case LDM_DT_F16: return launch_c1_dt<S, KK, 1>(p, st);
        default: return launch_c1_dt<S, KK, 2>(p, st);
    }
}

template <int S, int KK, int BM, int BC>
int launch(const Plan& p, hipStream_t st) {
    switch (p.a.lowp) {
        case LDM_DT_F32: return launch_dt<S, KK, BM, BC, 0>(p, st);
        case LDM_DT_F16: return launch_dt<S, KK, BM, BC, 1>(p, st);
        default: return launch_dt<S, KK, BM, BC, 2>(p, st);
    }
}

}  // namespace wg

// LDM_WGRAD_LP=0 in the environment keeps 16-bit weight gradients on the tap-shared kernel (A/B timing
// and the parity test of both forms).
static bool wgrad_lp_disabled() {
    const char* e = getenv("LDM_WGRAD_LP");
    return e && e[0] == '0';
}

bool wgrad2_plan_ws(const ldm_conv_desc& d, int64_t& ws_floats) {
    wg::Plan p;
    if (!wg::plan(d, p)) return false;
    ws_floats = (int64_t)p.splits * p.a.M * p.a.C * p.KK * p.KK;
    wg::LpPlan lp;
    if (wg::lp_plan(d, lp)) ws_floats = std::max(ws_floats, (int64_t)lp.splits * lp.a.M * lp.a.C * lp.KK * lp.KK);
    return true;
}

// Runs the tap-shared kernel into `partial` ([splits][M][N]); returns the split count through `splits`,
// or -1 when the form does not apply.
// the register-staged instances hold at most kLpStagedPieces window pieces per lane
static bool lp_staged_fits(const wg::LpPlan& lp) {
    const int nw = lp.WM * lp.KK;
    const int npiece = wg::kLC * (lp.a.pitch_c >> 2);
    return (npiece + 64 * nw - 1) / (64 * nw) <= wg::lp_staged_pieces(lp.S, lp.KK, lp.QC, nw);
}

// Which tensors of the weight gradient of d may be stored in 16 bits (LDM_DT_X16 | LDM_DT_DY16) at a 16-bit
// operand precision: the double-rate form's register-staged instances take both, the one-channel kernel
// (Cin = 1 layers) a 16-bit Dense (dy of a conv); else none.
int wgrad2_storage16(const ldm_conv_desc& d) {
    wg::Plan p;
    if (!wg::plan(d, p)) return 0;
    wg::LpPlan lp;
    if (!wgrad_lp_disabled() && wg::lp_plan(d, lp) && lp_staged_fits(lp)) return LDM_DT_X16 | LDM_DT_DY16;
    if (p.BC == 1) return d.transposed ? LDM_DT_X16 : LDM_DT_DY16;
    return 0;
}

// st16: bit 0 Dense, bit 1 Gath stored in 16 bits (-2: not on this layer's forms)
int wgrad2_run(const ldm_conv_desc& d, const float* dense, const float* gath, float* partial, int& splits, int dtype,
               hipStream_t st, int st16, float* dw_direct) {
    wg::Plan p;
    if (!wg::plan(d, p)) return -1;
    if (dtype != LDM_DT_F32 && !wgrad_lp_disabled()) {   // 16-bit operands: the double-rate MFMA form
        wg::LpPlan lp;
        bool ok = wg::lp_plan(d, lp);
        if (ok && st16 == 3) {
            wg::LpPlan l16 = lp;   // both maps 16-bit: the 16-bit DMA form where its geometry fits
            if (wg::lp16_plan(l16)) {
                lp = l16;
                lp.lds16 = 1;
            }
        }
        if (ok && !st16) wg::lp32_ring(lp);   // both maps fp32: the LDS-DMA ring
        if (ok && (!st16 || lp.lds16 || lp_staged_fits(lp))) {
            lp.a.dense = dense;
            lp.a.gath = gath;
            lp.a.partial = partial;
            lp.a.dense16 = st16 & 1;
            lp.a.gath16 = (st16 >> 1) & 1;
            splits = lp.splits;
            if (lp.splits == 1 && dw_direct) {   // one K range: its partial is the gradient (no reduce launch)
                lp.a.partial = dw_direct;
                splits = 0;
            }
            return dtype == LDM_DT_F16 ? wg::launch_lp<1>(lp, st) : wg::launch_lp<2>(lp, st);
        }
    }
    if (st16 && (p.BC != 1 || (st16 & 2) || dtype == LDM_DT_F32)) return -2;
    p.a.dense16 = st16 & 1;
    p.a.lowp = dtype;
    p.a.dense = dense;
    p.a.gath = gath;
    p.a.partial = partial;
    splits = p.splits;
    if (p.BC == 1) {
        switch (p.S * 10 + p.KK) {
            case 13: return wg::launch_c1<1, 3>(p, st);
            case 23: return wg::launch_c1<2, 3>(p, st);
            case 14: return wg::launch_c1<1, 4>(p, st);
            case 24: return wg::launch_c1<2, 4>(p, st);
            default: return -1;
        }
    }
    const int key = p.S * 1000 + p.KK * 100 + (p.BM == 64 ? 10 : 0) + (p.BC == 32 ? 1 : 0);
    switch (key) {
        case 1311: return wg::launch<1, 3, 64, 32>(p, st);
        case 1301: return wg::launch<1, 3, 32, 32>(p, st);
        case 1310: return wg::launch<1, 3, 64, 16>(p, st);
        case 2311: return wg::launch<2, 3, 64, 32>(p, st);
        case 2301: return wg::launch<2, 3, 32, 32>(p, st);
        case 2310: return wg::launch<2, 3, 64, 16>(p, st);
        case 2410: return wg::launch<2, 4, 64, 16>(p, st);
        case 1410: return wg::launch<1, 4, 64, 16>(p, st);
        default: return -1;
    }
}

}  // namespace ldm
