// Whole-UNet forward (UNet.forward, model.py:196-231) and the DDIM reverse loop
// (style_conditioned_ddim_sample model.py:409-465 / content_style_ddim_sample :503-559) as one C call:
// ~16 launches per denoising step, no host synchronisation, no allocation — the Python layer
// captures the full loop into a single hipGraph.
#include <cmath>
#include <cstdlib>

#include "common.h"

namespace ldm {

// Layer index -> geometry.  0..8: enc1 enc2 enc3 enc4 bottleneck dec4 dec3 dec2 dec1 (model.py:178-194)
// 9..14: [CA2 q, CA2 kv, CA2 out, CA1 q, CA1 kv, CA1 out] 1x1 projections of the packed
// nn.MultiheadAttention in_proj / out_proj (model.py:132, :184-185).
static int layer_desc(const ldm_unet_shape& s, int layer, ldm_conv_desc& d) {
    LDM_REQUIRE(s.B > 0 && s.C > 0 && s.nf > 0, "unet: bad shape");
    LDM_REQUIRE(s.H % 8 == 0 && s.W % 8 == 0 && s.H >= 8 && s.W >= 8,
                "unet: latent H and W must be multiples of 8 (skip connections, model.py:221-227)");
    LDM_REQUIRE(s.nf * 4 == 256, "unet: CrossAttention dims are fixed at 512/256 (model.py:184-185) -> num_filters 64");
    d = ldm_conv_desc{};
    d.B = s.B;
    const int nf = s.nf;
    const int H = s.H, W = s.W;
    auto conv = [&](int cin, int hin, int win, int cout, int stride) {
        d.Cin = cin;
        d.Hin = hin;
        d.Win = win;
        d.Cout = cout;
        d.kh = d.kw = 3;
        d.stride = stride;
        d.pad = 1;
        d.out_pad = 0;
        d.transposed = 0;
        d.Hout = (hin + 2 - 3) / stride + 1;
        d.Wout = (win + 2 - 3) / stride + 1;
    };
    auto convT = [&](int cin, int hin, int win, int cout) {
        d.Cin = cin;
        d.Hin = hin;
        d.Win = win;
        d.Cout = cout;
        d.kh = d.kw = 3;
        d.stride = 2;
        d.pad = 1;
        d.out_pad = 1;
        d.transposed = 1;
        d.Hout = 2 * hin;
        d.Wout = 2 * win;
    };
    auto proj = [&](int cin, int cout, int hw) {
        d.Cin = cin;
        d.Hin = 1;
        d.Win = hw;
        d.Cout = cout;
        d.kh = d.kw = 1;
        d.stride = 1;
        d.pad = 0;
        d.out_pad = 0;
        d.transposed = 0;
        d.Hout = 1;
        d.Wout = hw;
    };
    const int L2 = (H / 4) * (W / 4), L1 = (H / 8) * (W / 8);
    switch (layer) {
        case 0: conv(s.C, H, W, nf, 1); break;
        case 1: conv(nf, H, W, 2 * nf, 2); break;
        case 2: conv(2 * nf, H / 2, W / 2, 4 * nf, 2); break;
        case 3: conv(4 * nf, H / 4, W / 4, 8 * nf, 2); break;
        case 4: conv(8 * nf, H / 8, W / 8, 8 * nf, 1); break;
        case 5: convT(8 * nf, H / 8, W / 8, 4 * nf); break;
        case 6: convT(4 * nf, H / 4, W / 4, 2 * nf); break;
        case 7: convT(2 * nf, H / 2, W / 2, nf); break;
        case 8: conv(nf, H, W, s.C, 1); break;
        case 9: proj(256, 256, L2); break;
        case 10: proj(256, 512, L2); break;
        case 11: proj(256, 256, L2); break;
        case 12: proj(512, 512, L1); break;
        case 13: proj(512, 1024, L1); break;
        case 14: proj(512, 512, L1); break;
        default: return fail(2, "unet: layer index out of range");
    }
    // Activation layouts inside the UNet: everything between the latent input (NCHW, read by enc1)
    // and the noise prediction (NCHW, written by dec1) is NHWC, so each K-chunk of an implicit-GEMM
    // operand is one 16-byte load per lane; the style-map K/V projections read the NCHW style maps and
    // stay channel-major (the attention reads K/V that way); q and the attention output are token-major.
    switch (layer) {
        case 0: d.layout = 2; break;           // z (NCHW) -> z1 (NHWC)
        case 8: d.layout = 1; break;           // d2 (NHWC) -> eps / fused update (NCHW)
        case 10: case 13: d.layout = 0; break; // s5 / s6 -> kv (channel-major)
        default: d.layout = 3; break;
    }
    return 0;
}

struct UNetWs {
    float *convws, *temb, *z1, *z2, *z3, *q2, *kv2, *a2, *c2, *z4, *q1, *kv1, *a1, *c1, *zb, *d4, *d3, *d2, *eps;
    float *kf2, *bf2, *kf1, *bf1;   // folded keys of both cross-attentions (reverse loop, use_fold)
    float* xs;                      // the sampler state in NHWC (reverse loop with the step kernels)
    float* uks;                     // split-K counters + slabs of the K-split step kernels (uconv.hip)
    float *ubn, *p1;                // the bottleneck's folded values U and CA1's probabilities (bfold.hip)
    int64_t total;
};

// Largest split-K workspace over the 15 layers' plans (layers run one after another on one stream, so
// they share it; its counters are zero between launches).
static int64_t conv_ws_floats(const ldm_unet_weights* w) {
    if (!w) return 0;
    int64_t m = 0;
    for (int i = 0; i < 9; ++i) m = m > w->conv_plan[i].ws_floats ? m : w->conv_plan[i].ws_floats;
    for (int j = 0; j < 2; ++j) {
        m = m > w->ca_plan_q[j].ws_floats ? m : w->ca_plan_q[j].ws_floats;
        m = m > w->ca_plan_kv[j].ws_floats ? m : w->ca_plan_kv[j].ws_floats;
        m = m > w->ca_plan_o[j].ws_floats ? m : w->ca_plan_o[j].ws_floats;
    }
    return m;
}

// The reverse loop's bottleneck on CA1's folded values (bfold.hip) at the canonical plane, B <= 8.
bool ca1_probs_own();   // (bfold.hip)
int ca1_probs(const float* z, const float* kf, const float* bfv, float* p, int B, hipStream_t st);

static bool use_bneck_fold(const ldm_unet_shape& s, const ldm_unet_weights* w) {
    return w && w->use_fold && w->use_step && w->step_bneck_w && s.C == 32 && s.nf == 64 &&
           bneck_fold_supported(s.B, s.H, s.W);
}

static UNetWs carve(const ldm_unet_shape& s, const ldm_unet_weights* wts, float* base) {
    const int64_t B = s.B, nf = s.nf, HW = (int64_t)s.H * s.W;
    const int64_t HW2 = HW / 4, L2 = HW / 16, L1 = HW / 64;
    UNetWs w{};
    int64_t off = 0;
    auto take = [&](int64_t n) {
        float* p = base ? base + off : nullptr;
        off += (n + 63) / 64 * 64;   // 256-byte aligned sub-buffers
        return p;
    };
    w.convws = take(conv_ws_floats(wts));   // first: the zero-filled counters live here
    w.temb = take(B * 128);
    w.z1 = take(B * nf * HW);
    w.z2 = take(B * 2 * nf * HW2);
    w.z3 = take(B * 4 * nf * L2);
    w.q2 = take(B * 256 * L2);
    w.kv2 = take(B * 512 * L2);
    w.a2 = take(B * 256 * L2);
    w.c2 = take(B * 256 * L2);
    w.z4 = take(B * 8 * nf * L1);
    w.q1 = take(B * 512 * L1);
    w.kv1 = take(B * 1024 * L1);
    w.a1 = take(B * 512 * L1);
    w.c1 = take(B * 512 * L1);
    w.zb = take(B * 8 * nf * L1);
    w.d4 = take(B * 4 * nf * L2);
    w.d3 = take(B * 2 * nf * HW2);
    w.d2 = take(B * nf * HW);
    w.eps = take(B * (int64_t)s.C * HW);
    w.kf2 = take(B * 4 * 256 * L2);
    w.bf2 = take(B * 4 * L2);
    w.kf1 = take(B * 4 * 512 * L1);
    w.bf1 = take(B * 4 * L1);
    w.xs = take(B * (int64_t)s.C * HW);
    w.uks = take(wts && wts->use_step ? step_ws_floats(s.B, s.H, s.W) : 0);
    const bool bfold = use_bneck_fold(s, wts);
    w.ubn = take(bfold ? B * 512 * 576 : 0);
    w.p1 = take(bfold ? B * 4 * L1 * L1 : 0);
    w.total = off;
    return w;
}

// Optional fusion of the reverse-loop update into dec1's epilogue (see EpiArgs::ddim_*).
struct DdimFuse {
    const float* coef;
    float eta;
    float* x;
    float* x0_log;
    float* eps_log;
};

static int conv_call(const ldm_unet_shape& s, float* convws, int layer, const ldm_conv_plan& plan, const float* x, const float* w,
                     const float* bias, int act, const float* bcast, const float* skip, float* y, hipStream_t st,
                     const DdimFuse* fuse = nullptr, const float* pos_bias = nullptr) {
    ldm_conv_desc d;
    int rc = layer_desc(s, layer, d);
    if (rc) return rc;
    EpiArgs ep{};
    ep.bias = pos_bias ? nullptr : bias;
    ep.pos_bias = pos_bias;
    ep.act = act;
    ep.bcast = bcast;
    ep.skip = skip;
    if (fuse) {
        ep.ddim_coef = fuse->coef;
        ep.ddim_eta = fuse->eta;
        ep.ddim_x = fuse->x;
        ep.ddim_x0_log = fuse->x0_log;
        ep.ddim_eps_log = fuse->eps_log;
    }
    return conv_forward_ex(d, plan, x, w, ep, y, convws, st);
}

#define LDM_TRY(expr)            \
    do {                         \
        int _rc = (expr);        \
        if (_rc) return _rc;     \
    } while (0)

// K/V projections of the style maps (the key/value half of both cross-attentions' in_proj,
// model.py:153).  They depend only on s5 / s6, which are fixed for a whole reverse loop.
static int style_kv(const ldm_unet_shape& s, const ldm_unet_weights& w, const float* s5, const float* s6,
                    const UNetWs& ws, hipStream_t st) {
    LDM_TRY(conv_call(s, ws.convws, 10, w.ca_plan_kv[0], s5, w.ca_wkv[0], w.ca_bkv[0], 0, nullptr, nullptr, ws.kv2, st));
    LDM_TRY(conv_call(s, ws.convws, 13, w.ca_plan_kv[1], s6, w.ca_wkv[1], w.ca_bkv[1], 0, nullptr, nullptr, ws.kv1, st));
    return 0;
}

// kv_ready: ws.kv2 / ws.kv1 already hold style_kv() of these s5 / s6 (the reverse loop computes them
// once, before its first step — the same kernel on the same inputs, so bitwise what each step's
// in-loop projection would produce).
static int unet_forward(const ldm_unet_shape& s, const ldm_unet_weights& w, const float* z, const void* t,
                        int t_is_float, const float* s5, const float* s6, float* out, const UNetWs& ws,
                        hipStream_t st, const float* temb_pre = nullptr, const DdimFuse* fuse = nullptr,
                        bool kv_ready = false) {
    const int HW = s.H * s.W;
    const int L2 = HW / 16, L1 = HW / 64;
    // t_embedding = time_mlp(t)[:, :, None, None]                               (model.py:203)
    const float* temb = temb_pre;
    if (!temb) {
        LDM_TRY(ldm_time_mlp_forward(t, t_is_float, s.B, 128, w.t_freqs, w.t_w1, w.t_b1, w.t_w2, w.t_b2, ws.temb, st));
        temb = ws.temb;
    }
    // z1 = relu(enc1(z)); z2 = relu(enc2(z1)) + t_emb; z3 = relu(enc3(z2))      (model.py:205-209)
    LDM_TRY(conv_call(s, ws.convws, 0, w.conv_plan[0], z, w.conv_w[0], w.conv_b[0], LDM_ACT_RELU, nullptr, nullptr, ws.z1, st));
    LDM_TRY(conv_call(s, ws.convws, 1, w.conv_plan[1], ws.z1, w.conv_w[1], w.conv_b[1], LDM_ACT_RELU, temb, nullptr, ws.z2, st));
    LDM_TRY(conv_call(s, ws.convws, 2, w.conv_plan[2], ws.z2, w.conv_w[2], w.conv_b[2], LDM_ACT_RELU, nullptr, nullptr, ws.z3, st));
    // z3 = cross_attention2(z3, s5)                                              (model.py:211)
    if (!kv_ready) LDM_TRY(style_kv(s, w, s5, s6, ws, st));
    LDM_TRY(conv_call(s, ws.convws, 9, w.ca_plan_q[0], ws.z3, w.ca_wq[0], w.ca_bq[0], 0, nullptr, nullptr, ws.q2, st));
    LDM_TRY(attention_core_ex(ws.q2, ws.kv2, ws.a2, s.B, 256, 4, L2, L2, (float)std::sqrt(1.0 / 64.0), true, st));
    LDM_TRY(conv_call(s, ws.convws, 11, w.ca_plan_o[0], ws.a2, w.ca_wo[0], w.ca_bo[0], 0, nullptr, nullptr, ws.c2, st));
    // z4 = relu(enc4(z3)); z4 = cross_attention1(z4, s6)                         (model.py:212-214)
    LDM_TRY(conv_call(s, ws.convws, 3, w.conv_plan[3], ws.c2, w.conv_w[3], w.conv_b[3], LDM_ACT_RELU, nullptr, nullptr, ws.z4, st));
    LDM_TRY(conv_call(s, ws.convws, 12, w.ca_plan_q[1], ws.z4, w.ca_wq[1], w.ca_bq[1], 0, nullptr, nullptr, ws.q1, st));
    LDM_TRY(attention_core_ex(ws.q1, ws.kv1, ws.a1, s.B, 512, 4, L1, L1, (float)std::sqrt(1.0 / 128.0), true, st));
    LDM_TRY(conv_call(s, ws.convws, 14, w.ca_plan_o[1], ws.a1, w.ca_wo[1], w.ca_bo[1], 0, nullptr, nullptr, ws.c1, st));
    // bottleneck + decoder with skips (ReLU before the add)                     (model.py:217-229)
    LDM_TRY(conv_call(s, ws.convws, 4, w.conv_plan[4], ws.c1, w.conv_w[4], w.conv_b[4], LDM_ACT_RELU, nullptr, nullptr, ws.zb, st));
    LDM_TRY(conv_call(s, ws.convws, 5, w.conv_plan[5], ws.zb, w.conv_w[5], w.conv_b[5], LDM_ACT_RELU, nullptr, ws.z3, ws.d4, st));
    LDM_TRY(conv_call(s, ws.convws, 6, w.conv_plan[6], ws.d4, w.conv_w[6], w.conv_b[6], LDM_ACT_RELU, nullptr, ws.z2, ws.d3, st));
    LDM_TRY(conv_call(s, ws.convws, 7, w.conv_plan[7], ws.d3, w.conv_w[7], w.conv_b[7], LDM_ACT_RELU, nullptr, ws.z1, ws.d2, st));
    LDM_TRY(conv_call(s, ws.convws, 8, w.conv_plan[8], ws.d2, w.conv_w[8], w.conv_b[8], LDM_ACT_NONE, nullptr, nullptr, out, st,
                      fuse));
    return 0;
}

// The reverse loop's step with both cross-attentions re-associated (style and weights are fixed for the
// whole loop): the Q in-projection folds into the keys (ldm_attention_fold_keys, once per loop) and the
// out-projection into the following conv (ldm_fold_conv_proj, once per weight version).  11 launches per
// step instead of 15; the same arithmetic up to fp32 re-association.
static int unet_forward_folded(const ldm_unet_shape& s, const ldm_unet_weights& w, const float* z, const UNetWs& ws,
                               hipStream_t st, const float* temb, const DdimFuse* fuse) {
    const int HW = s.H * s.W;
    const int L2 = HW / 16, L1 = HW / 64;
    LDM_TRY(conv_call(s, ws.convws, 0, w.conv_plan[0], z, w.conv_w[0], w.conv_b[0], LDM_ACT_RELU, nullptr, nullptr, ws.z1, st));
    LDM_TRY(conv_call(s, ws.convws, 1, w.conv_plan[1], ws.z1, w.conv_w[1], w.conv_b[1], LDM_ACT_RELU, temb, nullptr, ws.z2, st));
    LDM_TRY(conv_call(s, ws.convws, 2, w.conv_plan[2], ws.z2, w.conv_w[2], w.conv_b[2], LDM_ACT_RELU, nullptr, nullptr, ws.z3, st));
    // cross_attention2 then enc4 (model.py:211-212)
    LDM_TRY(attention_folded(ws.z3, ws.kv2, ws.kf2, ws.bf2, ws.a2, s.B, 256, 4, L2, L2, st));
    LDM_TRY(conv_call(s, ws.convws, 3, w.conv_plan[3], ws.a2, w.fold_w[0], nullptr, LDM_ACT_RELU, nullptr, nullptr, ws.z4, st,
                      nullptr, w.fold_pb[0]));
    // cross_attention1 then bottleneck (model.py:214-217)
    LDM_TRY(attention_folded(ws.z4, ws.kv1, ws.kf1, ws.bf1, ws.a1, s.B, 512, 4, L1, L1, st));
    LDM_TRY(conv_call(s, ws.convws, 4, w.conv_plan[4], ws.a1, w.fold_w[1], nullptr, LDM_ACT_RELU, nullptr, nullptr, ws.zb, st,
                      nullptr, w.fold_pb[1]));
    LDM_TRY(conv_call(s, ws.convws, 5, w.conv_plan[5], ws.zb, w.conv_w[5], w.conv_b[5], LDM_ACT_RELU, nullptr, ws.z3, ws.d4, st));
    LDM_TRY(conv_call(s, ws.convws, 6, w.conv_plan[6], ws.d4, w.conv_w[6], w.conv_b[6], LDM_ACT_RELU, nullptr, ws.z2, ws.d3, st));
    LDM_TRY(conv_call(s, ws.convws, 7, w.conv_plan[7], ws.d3, w.conv_w[7], w.conv_b[7], LDM_ACT_RELU, nullptr, ws.z1, ws.d2, st));
    LDM_TRY(conv_call(s, ws.convws, 8, w.conv_plan[8], ws.d2, w.conv_w[8], w.conv_b[8], LDM_ACT_NONE, nullptr, nullptr, nullptr,
                      st, fuse));
    return 0;
}

// The same folded step on the step kernels (uconv.hip): x and every activation NHWC, 11 launches, the
// DDIM update fused into dec1.  z (the sampler state) is ws.xs.
static int unet_step_kernels(const ldm_unet_shape& s, const ldm_unet_weights& w, const UNetWs& ws, hipStream_t st,
                             const float* temb, const DdimFuse& fuse) {
    const int HW = s.H * s.W;
    const int L2 = HW / 16, L1 = HW / 64;
    // the nine convs' operands: enc1..enc3, enc4 (after CA2), bottleneck (after CA1), dec4..dec2, dec1 + DDIM
    const float* xin[9] = {ws.xs, ws.z1, ws.z2, ws.a2, ws.a1, ws.zb, ws.d4, ws.d3, ws.d2};
    float* yout[9] = {ws.z1, ws.z2, ws.z3, ws.z4, ws.zb, ws.d4, ws.d3, ws.d2, nullptr};
    const float* bias[9] = {w.conv_b[0], w.conv_b[1], w.conv_b[2], w.step_pb[0], w.step_pb[1], w.conv_b[5], w.conv_b[6],
                            w.conv_b[7], w.conv_b[8]};
    const float* skip[9] = {nullptr, nullptr, nullptr, nullptr, nullptr, ws.z3, ws.z2, ws.z1, nullptr};
    StepConv c[9];
    for (int l = 0; l < 9; ++l) {
        c[l] = StepConv{};
        c[l].x = xin[l];
        c[l].w = w.step_w[l];
        c[l].y = yout[l];
        c[l].bias = bias[l];
        c[l].skip = skip[l];
        c[l].dtype = w.step_dtype;
        c[l].ws = ws.uks;
    }
    c[1].bcast = temb;
    c[8].coef = fuse.coef;
    c[8].eta = fuse.eta;
    c[8].xs = ws.xs;
    c[8].x0_log = fuse.x0_log;
    c[8].eps_log = fuse.eps_log;
    auto run = [&](int l0, int l1) -> int {   // layers [l0, l1]
        for (int l = l0; l <= l1; ++l) LDM_TRY(step_conv(l, s.B, s.H, s.W, c[l], st));
        return 0;
    };
    LDM_TRY(run(0, 2));
    LDM_TRY(attention_folded(ws.z3, ws.kv2, ws.kf2, ws.bf2, ws.a2, s.B, 256, 4, L2, L2, st));
    LDM_TRY(run(3, 3));
    if (use_bneck_fold(s, &w)) {
        // CA1's probabilities, then the bottleneck on its folded values U (formed before the loop)
        if (ca1_probs_own()) LDM_TRY(ca1_probs(ws.z4, ws.kf1, ws.bf1, ws.p1, s.B, st));
        else LDM_TRY(attention_folded_probs(ws.z4, ws.kf1, ws.bf1, ws.p1, s.B, 512, 4, L1, L1, st));
        LDM_TRY(bneck_pv(ws.ubn, ws.p1, w.step_pb[1], ws.zb, s.B, w.step_dtype, st));
        return run(5, 8);
    }
    LDM_TRY(attention_folded(ws.z4, ws.kv1, ws.kf1, ws.bf1, ws.a1, s.B, 512, 4, L1, L1, st));
    return run(4, 8);
}

}  // namespace ldm

using namespace ldm;

extern "C" int ldm_step_layer_forms(int32_t* ks_layers) {
    LDM_REQUIRE(ks_layers, "step_layer_forms: null argument");
    *ks_layers = step_ks_mask();   // (their K-split geometry: LDM_UCONV_KS2, uconv.hip kKs2)
    return 0;
}

extern "C" int ldm_unet_layer_desc(const ldm_unet_shape* s, int32_t layer, ldm_conv_desc* d) {
    LDM_REQUIRE(s && d, "unet_layer_desc: null argument");
    return layer_desc(*s, layer, *d);
}

extern "C" int64_t ldm_unet_workspace_floats(const ldm_unet_shape* s, const ldm_unet_weights* w) {
    if (!s) return -1;
    return carve(*s, w, nullptr).total;
}

extern "C" int ldm_unet_make_plans(const ldm_unet_shape* s, ldm_unet_weights* w) {
    LDM_REQUIRE(s && w, "unet_make_plans: null argument");
    for (int l = 0; l < 15; ++l) {
        ldm_conv_desc d;
        LDM_TRY(layer_desc(*s, l, d));
        ldm_conv_plan* p = l < 9 ? &w->conv_plan[l]
                                 : ((l - 9) % 3 == 0 ? &w->ca_plan_q[(l - 9) / 3]
                                                     : ((l - 9) % 3 == 1 ? &w->ca_plan_kv[(l - 9) / 3]
                                                                         : &w->ca_plan_o[(l - 9) / 3]));
        LDM_TRY(ldm_conv_make_plan(&d, p));
    }
    return 0;
}

extern "C" int ldm_unet_forward(const ldm_unet_shape* s, const ldm_unet_weights* w, const float* z, const void* t,
                                int32_t t_is_float, const float* s5, const float* s6, float* out, float* workspace,
                                void* stream) {
    LDM_REQUIRE(s && w && z && t && s5 && s6 && out && workspace, "unet_forward: null argument");
    UNetWs ws = carve(*s, w, workspace);
    return unet_forward(*s, *w, z, t, t_is_float, s5, s6, out, ws, (hipStream_t)stream);
}

extern "C" int ldm_ddim_sample(const ldm_unet_shape* s, const ldm_unet_weights* w, float* x, const float* s5,
                               const float* s6, const int64_t* t_table, const float* coef_table, int32_t nsteps,
                               float eta, float* x0_logs, float* eps_logs, int64_t log_step_stride, float* workspace,
                               void* stream) {
    LDM_REQUIRE(s && w && x && s5 && s6 && t_table && coef_table && workspace, "ddim_sample: null argument");
    LDM_REQUIRE(nsteps >= 0, "ddim_sample: negative step count");
    if (nsteps == 0) return 0;
    UNetWs ws = carve(*s, w, workspace);
    float* temb_all = workspace + ws.total;   // [nsteps*B, 128] (ldm_ddim_workspace_floats)
    const int64_t dense = (int64_t)s->B * s->C * s->H * s->W;
    LDM_REQUIRE(log_step_stride == 0 || log_step_stride >= dense, "ddim_sample: log stride smaller than a step");
    const int64_t n = log_step_stride ? log_step_stride : dense;
    hipStream_t st = (hipStream_t)stream;
    // The time MLP depends only on t: all nsteps*B embeddings in one launch before the loop (the same
    // evaluations the reference makes one step at a time, model.py:203).
    LDM_TRY(ldm_time_mlp_forward(t_table, 0, nsteps * s->B, 128, w->t_freqs, w->t_w1, w->t_b1, w->t_w2, w->t_b2,
                                 temb_all, st));
    // Likewise the style maps' K/V projections (model.py:153 with kv = s5 / s6, fixed for the loop).
    LDM_TRY(style_kv(*s, *w, s5, s6, ws, st));
    const int HW = s->H * s->W;
    if (w->use_fold) {
        LDM_REQUIRE(w->ca_wq_raw[0] && w->ca_wq_raw[1] && w->fold_w[0] && w->fold_w[1] && w->fold_pb[0] && w->fold_pb[1],
                    "ddim_sample: use_fold needs the folded weights");
        LDM_TRY(attention_fold_keys(ws.kv2, w->ca_wq_raw[0], w->ca_bq[0], s->B, 256, 4, HW / 16,
                                    (float)std::sqrt(1.0 / 64.0), ws.kf2, ws.bf2, st));
        LDM_TRY(attention_fold_keys(ws.kv1, w->ca_wq_raw[1], w->ca_bq[1], s->B, 512, 4, HW / 64,
                                    (float)std::sqrt(1.0 / 128.0), ws.kf1, ws.bf1, st));
        if (w->use_step) {
            LDM_REQUIRE(s->C == 32 && s->nf == 64, "ddim_sample: the step kernels are built for latent 32 / 64 filters");
            for (int l = 0; l < 9; ++l) LDM_REQUIRE(w->step_w[l], "ddim_sample: use_step needs the step weights");
            LDM_REQUIRE(w->step_pb[0] && w->step_pb[1], "ddim_sample: use_step needs the folded biases");
            LDM_REQUIRE(w->step_dtype >= LDM_DT_F32 && w->step_dtype <= LDM_DT_BF16, "ddim_sample: step_dtype");
            if (use_bneck_fold(*s, w)) LDM_TRY(bneck_fold_values(w->step_bneck_w, ws.kv1, ws.ubn, s->B, st));
            LDM_TRY(step_layout(x, ws.xs, s->B, s->C, HW, true, st));
            for (int i = 0; i < nsteps; ++i) {
                DdimFuse fuse{coef_table + 4 * (size_t)i, eta, ws.xs, x0_logs ? x0_logs + (size_t)i * n : nullptr,
                              eps_logs ? eps_logs + (size_t)i * n : nullptr};
                LDM_TRY(unet_step_kernels(*s, *w, ws, st, temb_all + (size_t)i * s->B * 128, fuse));
            }
            return step_layout(ws.xs, x, s->B, s->C, HW, false, st);
        }
        for (int i = 0; i < nsteps; ++i) {
            DdimFuse fuse{coef_table + 4 * (size_t)i, eta, x, x0_logs ? x0_logs + (size_t)i * n : nullptr,
                          eps_logs ? eps_logs + (size_t)i * n : nullptr};
            LDM_TRY(unet_forward_folded(*s, *w, x, ws, st, temb_all + (size_t)i * s->B * 128, &fuse));
        }
        return 0;
    }
    for (int i = 0; i < nsteps; ++i) {
        // noise_pred = unet(x, t, style_embedding)                                (model.py:439)
        // and, fused into dec1's epilogue, the x0 / direction / eta update and the two log clones
        // (model.py:442-463) — bitwise the same fp32 op sequence as ldm_ddim_step.
        DdimFuse fuse{coef_table + 4 * (size_t)i, eta, x, x0_logs ? x0_logs + (size_t)i * n : nullptr,
                      eps_logs ? eps_logs + (size_t)i * n : nullptr};
        LDM_TRY(unet_forward(*s, *w, x, t_table + (size_t)i * s->B, 0, s5, s6, nullptr, ws, st,
                             temb_all + (size_t)i * s->B * 128, &fuse, /*kv_ready=*/true));
    }
    return 0;
}

extern "C" int64_t ldm_ddim_workspace_floats(const ldm_unet_shape* s, const ldm_unet_weights* w, int32_t nsteps) {
    if (!s || nsteps < 0) return -1;
    return carve(*s, w, nullptr).total + (int64_t)nsteps * s->B * 128;
}
