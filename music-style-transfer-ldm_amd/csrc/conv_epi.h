// ConvArgs and the conv epilogue (conv.hip's implicit-GEMM kernels and sconv.hip's small-plane kernel share them):
// the reference's op order conv + bias -> BN(eval) -> act -> + bcast -> + skip (model.py:16-25, :205-229), with
// autocast output rounding and the fused DDIM update.
#pragma once
#include "common.h"

namespace ldm {

struct ConvArgs {
    const float* x;
    const float* w;
    float* y;
    int32_t B, Cin, Hin, Win, Cout, Hout, Wout;
    int32_t KK;     // kh*kw
    int32_t Mpad;   // rows of the packed weight
    int32_t transposed;
    int32_t xcd_nfast;     // weight-heavy layer (weights > input bytes)
    int32_t tile_order;    // 0 natural (N, M, phase), 1 XCD-grouped N-fast, 2 XCD-grouped M-fast
    int32_t ks;            // blocks splitting K (cross-block split-K)
    int32_t out_nhwc;      // output / skip / fused-update tensors are NHWC (the input layout is a template flag)
    int32_t nN, nM;        // N / M tiles per phase
    int32_t balance;       // 4-phase layers: phase p splits K ks_p = ks_base * ntap_p ways (equal work per block)
    int32_t bofs[kMaxPhase];    // balance: first block of each phase (after the XCD renumbering)
    int32_t bks_log2[kMaxPhase];  // balance: log2 ks_p
    int32_t nblocks_bal;          // balance: grid size
    float* part;           // ks > 1: partial tiles [phase][M-tile][N-tile][ks][BM*BN]
    int32_t* cnt;          // ks > 1: arrival counter per tile (zero between launches)
    FastDiv fd_ks;         // M-tile' -> (M-tile, split)
    FastDiv fd_hw, fd_w;   // n -> (b, q) and q -> (qy, qx) of the phase grid
    FastDiv fd_cpt;        // K chunk -> (tap, channel chunk)
    FastDiv fd_np, fd_inner;   // block -> (phase, tile), tile -> (outer, inner) of the XCD order
    FastDiv fd_nn, fd_nm;      // natural order: block -> (N-tile, M-tile, phase)
    FastDiv fd_dwo, fd_dho, fd_dco;   // direct kernel: output index -> (b, co, oy, ox)
    PhaseTable pt;
    // Per-phase scalars of the MFMA kernel, indexed [phase] and read at static offsets (one batch of
    // scalar loads, then a select by phase: a load indexed by the runtime phase would be a second,
    // dependent round of kernarg reads).  Tap t = ja*nb + jb of a phase sits at
    // (dy, dx) = (dy0 + sg*ja, dx0 + sg*jb) — the same order as pt.dy / pt.dx (checked on the host).
    struct {
        int32_t ry[kMaxPhase], rx[kMaxPhase];
        int32_t dy0[kMaxPhase], dx0[kMaxPhase];
        int32_t na[kMaxPhase], nb[kMaxPhase];
        int32_t kchunks[kMaxPhase], wofs[kMaxPhase];
        int32_t sg;
    } pk;
    EpiArgs ep;
};

// ------------------------------------------------------------------------------------------------
// epilogue (op order of the reference: conv+bias -> BN(eval) -> act -> +bcast -> +skip)
// ------------------------------------------------------------------------------------------------
// Epilogue operands of one output element, loaded ahead of time (before the K loop) so their memory
// latency overlaps the GEMM instead of trailing it.
struct EpiPre {
    float bias, bcast, skip, x;
};

__device__ __forceinline__ EpiPre epi_prefetch(const ConvArgs& a, int m, int b, size_t oidx, int pix) {
    const EpiArgs& e = a.ep;
    EpiPre p;
    p.bias = e.pos_bias ? e.pos_bias[m * a.Hout * a.Wout + pix] : (e.bias ? e.bias[m] : 0.f);
    p.bcast = e.bcast ? e.bcast[(size_t)b * a.Cout + m] : 0.f;
    p.skip = e.skip ? e.skip[oidx] : 0.f;
    p.x = e.ddim_coef ? e.ddim_x[oidx] : 0.f;
    return p;
}

// The same loads, unconditional: one buffer resource per optional operand, with zero records when the
// operand is absent (its loads then return 0 without touching memory).  No branch, so the loads issue
// back to back and the waitcnt pass can count them (a branchy prefetch ends in a vmcnt(0) drain
// in front of the K loop).
struct EpiSrc {
    __amdgpu_buffer_rsrc_t bias, bcast, skip, x;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t opt_rsrc(const float* p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(uni_ptr(p), (short)0, uni(p ? bytes : 0), 0x00020000);
}

__device__ __forceinline__ EpiSrc epi_sources(const ConvArgs& a, bool live) {
    const EpiArgs& e = a.ep;
    const int ybytes = live ? a.B * a.Cout * a.Hout * a.Wout * 4 : 0;
    EpiSrc s;
    s.bias = e.pos_bias ? opt_rsrc(e.pos_bias, live ? a.Cout * a.Hout * a.Wout * 4 : 0)
                        : opt_rsrc(e.bias, live ? a.Cout * 4 : 0);
    s.bcast = opt_rsrc(e.bcast, live ? a.B * a.Cout * 4 : 0);
    s.skip = opt_rsrc(e.skip, ybytes);
    s.x = opt_rsrc(e.ddim_coef ? e.ddim_x : nullptr, ybytes);
    return s;
}

__device__ __forceinline__ EpiPre epi_prefetch_buf(const EpiSrc& s, int Cout, int m, int b, int oidx, int boff) {
    EpiPre p;
    p.bias = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(s.bias, boff, 0, 0));
    p.bcast = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(s.bcast, (b * Cout + m) * 4, 0, 0));
    p.skip = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(s.skip, oidx * 4, 0, 0));
    p.x = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(s.x, oidx * 4, 0, 0));
    return p;
}

__device__ __forceinline__ void epi_finish(const ConvArgs& a, int m, size_t oidx, float v, const EpiPre& p) {
    const EpiArgs& e = a.ep;
#if (LDM_DIAG & 32)   // diagnostic: minimal epilogue (bias + relu + store) to size the code-footprint cost
    v = v + p.bias;
    a.y[oidx] = v < 0.f ? 0.f : v;
    return;
#endif
    const int ro = e.round_out;   // autocast output semantics (EpiArgs::round_out): 0 leaves every value as is
    if (e.bias || e.pos_bias) v = v + p.bias;
    v = round16(v, ro);
    if (e.bn_w) {
        // aten batch_norm_cpu_collect_linear_and_constant_terms: alpha = invstd*w, beta = b - mean*alpha
        const float invstd = 1.0f / sqrtf(e.bn_v[m] + e.bn_eps);
        const float alpha = invstd * e.bn_w[m];
        const float beta = e.bn_b[m] - e.bn_m[m] * alpha;
        v = round16(v * alpha + beta, ro);
    }
    v = round16(apply_act(v, e.act), ro);
    if (e.act_out) e.act_out[oidx] = v;
    if (e.bcast) v = round16(v + p.bcast, ro);
    if (e.skip) v = round16(v + p.skip, ro);
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

__device__ __forceinline__ int out_index(const ConvArgs& a, int m, int b, int oy, int ox) {
    return a.out_nhwc ? ((b * a.Hout + oy) * a.Wout + ox) * a.Cout + m : ((b * a.Cout + m) * a.Hout + oy) * a.Wout + ox;
}

__device__ __forceinline__ void epilogue_store(const ConvArgs& a, int m, int b, int oy, int ox, float v) {
    const size_t oidx = out_index(a, m, b, oy, ox);
    epi_finish(a, m, oidx, v, epi_prefetch(a, m, b, oidx, oy * a.Wout + ox));
}

}  // namespace ldm
