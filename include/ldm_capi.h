/*
 * ldm_capi.h — C ABI of the MI355X-native latent-diffusion hot path (libldm_amd.so).
 *
 * The reference (PrioteasaAndrei/music-style-transfer-ldm) has no native boundary: its hot path is
 * nn.Module.__call__ -> ATen.  This header is the thin C ABI the drop-in Python
 * modules (music-style-transfer-ldm_amd/models/ (*.py)) call through ctypes.  Each entry point names the
 * reference code it replaces.
 *
 * Conventions
 *   - Plain pointers + sizes; every tensor is a contiguous fp32 NCHW device buffer unless stated.
 *   - `stream` is a hipStream_t passed as void* (torch.cuda.current_stream().cuda_stream); every
 *     launch goes on it, nothing is synchronised, nothing is allocated: workspaces come from the
 *     caller (graph-capture safe, §8(b) "Ownership").
 *   - Return 0 on success, otherwise a nonzero code; ldm_last_error() gives the message
 *     (thread-local).  The Python layer raises RuntimeError with it.
 */
#ifndef LDM_CAPI_H
#define LDM_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDM_CAPI_VERSION 1

/* ---- errors / introspection --------------------------------------------------------------- */
const char* ldm_last_error(void);
int ldm_capi_version(void);
/* Number of HIP devices visible to the runtime this library is bound to (no kernel launch). */
int ldm_device_count(int* count);

/* ---- 2-D convolution / transposed convolution -----------------------------------------------
 * Replaces nn.Conv2d / nn.ConvTranspose2d (+ following BatchNorm2d(eval) / ReLU / Tanh / time-emb
 * add / skip add) at model.py:16-25 (encoder), :37-46 (decoder), :61-79 (style encoder),
 * :178-194 + :205-229 (UNet).  Implicit GEMM on f32 MFMA (v_mfma_f32_32x32x2_f32 /
 * v_mfma_f32_16x16x4_f32), transposed convs as sub-pixel phases, fused epilogue. */
typedef struct ldm_conv_desc {
    int32_t B, Cin, Hin, Win;
    int32_t Cout, Hout, Wout;
    int32_t kh, kw, stride, pad, out_pad;
    int32_t transposed; /* 0: Conv2d weight [Cout,Cin,kh,kw]; 1: ConvTranspose2d weight [Cin,Cout,kh,kw] */
    int32_t layout;     /* activation layouts: bit 0 input NHWC, bit 1 output (and skip) NHWC; 0 = NCHW  */
} ldm_conv_desc;

enum {
    LDM_ACT_NONE = 0,
    LDM_ACT_RELU = 1,
    LDM_ACT_TANH = 2,
    LDM_ACT_TANH_HALF = 3, /* (tanh(x)+1)/2: decoder output rescale, model.py:371,:405,:498 */
    LDM_ACT_GELU = 4       /* exact erf GELU (nn.GELU(), model.py:173)                     */
};

/* Operand precision of the MFMA kernels: fp32 operands (exact), or rounded to fp16 / bf16 in registers
 * with fp32 accumulation, fp32 epilogue and fp32 outputs / sampler state (the torch.autocast fp16 / bf16
 * regions of the train step and of a sampling loop; BASELINE configs 3 and 5). */
enum { LDM_DT_F32 = 0, LDM_DT_F16 = 1, LDM_DT_BF16 = 2 };
/* Or'ed into ldm_epilogue.dtype (with LDM_DT_F16 / LDM_DT_BF16): ATen's autocast OUTPUT semantics as well —
 * the conv output, the eval-BN output, the activation and each add are rounded to that type (stored in the
 * fp32 tensor), as the reference's conv / linear outputs are 16-bit tensors inside torch.autocast
 * (train.py:174).  Or'ed into the act code of ldm_batchnorm_train_out / ldm_batchnorm_apply_out as
 * LDM_ACT_ROUND_F16 / LDM_ACT_ROUND_BF16: the BatchNorm output likewise (a 16-bit input's BN output). */
enum { LDM_DT_ROUND_OUT = 0x100 };
enum { LDM_ACT_ROUND_F16 = LDM_DT_F16 << 8, LDM_ACT_ROUND_BF16 = LDM_DT_BF16 << 8 };
/* 16-bit storage of the train step's large maps (ATen keeps the outputs of an autocast region in fp16 / bf16):
 *  - conv entry points, or'ed into ldm_epilogue.dtype with LDM_DT_F16 / _BF16: the input x (LDM_DT_X16), the
 *    output y and act_out (LDM_DT_Y16) are stored in that type; ldm_conv_backward_weight_dt's dtype takes
 *    LDM_DT_X16 (x) and LDM_DT_DY16 (dy);
 *  - BatchNorm / activation-backward entry points: bits 16-17 of the act code name the 16-bit type
 *    (LDM_DT_F16 / _BF16 << LDM_ST_SHIFT), and LDM_ST_* which of the call's tensors are stored in it: X16 the
 *    BatchNorm input x (activation backward: act_out), Y16 the BatchNorm output y, DY16 the incoming gradient,
 *    DX16 the outgoing gradient (dx / dv).  The pointers stay typed float* in the signatures. */
enum { LDM_DT_X16 = 0x200, LDM_DT_Y16 = 0x400, LDM_DT_DY16 = 0x800 };
enum { LDM_ST_SHIFT = 16, LDM_ST_X16 = 1 << 18, LDM_ST_Y16 = 1 << 19, LDM_ST_DY16 = 1 << 20, LDM_ST_DX16 = 1 << 21 };

typedef struct ldm_epilogue {
    const float* bias;      /* [Cout] or NULL                                                */
    const float* bn_weight; /* eval-mode BatchNorm2d after bias (NULL = none): gamma [Cout]    */
    const float* bn_bias;   /*   beta [Cout]                                                   */
    const float* bn_mean;   /*   running_mean [Cout]                                           */
    const float* bn_var;    /*   running_var [Cout]                                            */
    float bn_eps;
    int32_t act;            /* LDM_ACT_*                                                       */
    const float* bcast_add; /* [B,Cout] added after act (UNet time embedding, model.py:206)   */
    const float* skip_add;  /* [B,Cout,Hout,Wout] added after act (UNet skips, model.py:221) */
    float* act_out;         /* [B,Cout,Hout,Wout] or NULL: also store act(.) before the adds  */
                            /* (training: the activation's backward needs it)                */
    int32_t dtype;          /* operand precision LDM_DT_* of the conv kernels: fp32, or x and w rounded */
                            /* to fp16 / bf16 with fp32 accumulation (autocast); | LDM_DT_ROUND_OUT */
} ldm_epilogue;

typedef struct ldm_conv_plan {
    int32_t kind;          /* 0 direct (VALU), 1 MFMA 32x32x2 f32, 2 MFMA 16x16x4 f32, 3 LDS-staged */
                           /* 16-bit-operand MFMA 32x32x16 (tm = BM/64, tn = LDM_DT_F16 / _BF16),    */
                           /* 4 small-plane 16-bit-operand MFMA 32x32x16 (sconv.hip; tn = the dtype, */
                           /* wk = waves per block)                                                  */
    int32_t tm, tn, wk;    /* MFMA tiles per wave along M / N, waves splitting K per block      */
    int32_t ks;            /* blocks splitting K (>1: partial tiles + fixed-order last-arriver sum) */
    int32_t balance;       /* 4-phase transposed convs: phase p splits K ks*ntap_p ways (equal K per block) */
    int64_t packed_floats; /* size of the packed-weight buffer ldm_conv_pack_weight fills (0 = none) */
    int64_t ws_floats;     /* workspace floats the plan needs (ks > 1): tile counters, then partials */
} ldm_conv_plan;

int ldm_conv_make_plan(const ldm_conv_desc* d, ldm_conv_plan* plan);
/* The kind-3 plan for d at operand precision dtype (LDM_DT_F16 / LDM_DT_BF16): the LDS-staged implicit
 * GEMM for large-plane NCHW layers (Cin % 32 == 0, >= 4096 positions per phase; bias / eval-BN /
 * activation epilogues only).  Returns 0 and fills plan, or 1 when the layer is not of that class. */
int ldm_conv_tiled_plan(const ldm_conv_desc* d, int32_t dtype, ldm_conv_plan* plan);
/* The kind-4 plan for d at operand precision dtype (LDM_DT_F16 / LDM_DT_BF16): the small-plane implicit GEMM
 * (sconv.hip) for k3 p1 convs (stride 1 / 2) and k3 s2 op1 / stride-1 transposed convs whose phase grid tiles into
 * 32-position runs (Wq | 32, or Wq % 32 == 0), Cin % 32 == 0 (>= 64), Cout % 64 == 0, fp32 NCHW maps; every
 * epilogue but the position bias and the fused DDIM update.  Its weights use the kind-3 pack (ldm_conv_pack_weight).
 * Returns 0 and fills plan, or 1 when the layer is not of that class (LDM_AMD_SCONV=0: never). */
int ldm_conv_sconv_plan(const ldm_conv_desc* d, int32_t dtype, ldm_conv_plan* plan);
/* Force a specific plan (autotuning / tests).  Fills packed_floats / ws_floats; validates.
 * ks < 0 requests the phase-balanced split with base -ks (4-phase layers only). */
int ldm_conv_make_plan_forced(const ldm_conv_desc* d, int kind, int tm, int tn, int wk, int ks,
                              ldm_conv_plan* plan);
/* Re-lay the torch weight into the MFMA fragment order of `plan` (tap-major K, zero padded). */
int ldm_conv_pack_weight(const ldm_conv_desc* d, const ldm_conv_plan* plan, const float* w,
                         float* packed, void* stream);
/* y = epilogue(conv(x, w)).  `w` is the packed buffer for MFMA plans, the torch weight for direct.
 * Plans with ks > 1 need ldm_conv_forward_ws. */
/* The 16-bit storage flags (LDM_DT_X16 | LDM_DT_Y16) ldm_conv_forward takes for (d, plan) at a 16-bit operand
 * precision: both on kind-3 plans, a 16-bit output on the Cin = 1 stride-2 kernel, a 16-bit input on the
 * 64 -> 1 k4 s2 transposed conv; else 0. */
int32_t ldm_conv_storage16(const ldm_conv_desc* d, const ldm_conv_plan* plan);
int ldm_conv_forward(const ldm_conv_desc* d, const ldm_conv_plan* plan, const float* x, const float* w,
                     const ldm_epilogue* ep, float* y, void* stream);
/* The same with a caller-owned workspace of plan->ws_floats floats (may be NULL when that is 0).
 * Its leading counter words must be zero before the first call; every call leaves them zero again,
 * so one zero-initialised workspace serves any number of stream-ordered calls (not concurrent ones). */
int ldm_conv_forward_ws(const ldm_conv_desc* d, const ldm_conv_plan* plan, const float* x, const float* w,
                        const ldm_epilogue* ep, float* y, float* workspace, void* stream);

/* ---- BatchNorm2d, train mode (model.py:18,21,24,39,42 under .train(); model.py:307,344-347) ----
 * Batch statistics over (B,H,W) per channel, normalise in place, optional activation, and the
 * running-stat update (momentum, unbiased variance) exactly as nn.BatchNorm2d.  save_mean /
 * save_invstd [C] are written for the backward pass (may be NULL).  workspace:
 * ldm_reduce_workspace_floats(B,C,HW) floats, 8-byte aligned (reduce.hip).  Each channel is reduced
 * by a fixed set of slices in a fixed order (fp64 sums): bitwise reproducible. */
int64_t ldm_reduce_workspace_floats(int32_t B, int32_t C, int32_t HW);
int ldm_batchnorm_train(float* x, int32_t B, int32_t C, int32_t HW, const float* weight, const float* bias,
                        float* running_mean, float* running_var, float momentum, float eps, int32_t act,
                        float* save_mean, float* save_invstd, float* workspace, void* stream);
/* Out-of-place form (y may equal x): statistics of x, the normalised result into y.  The autograd path
 * uses it so that no copy of the input is made for the in-place kernel (functional.batchnorm). */
int ldm_batchnorm_train_out(const float* x, float* y, int32_t B, int32_t C, int32_t HW, const float* weight,
                            const float* bias, float* running_mean, float* running_var, float momentum, float eps,
                            int32_t act, float* save_mean, float* save_invstd, float* workspace, void* stream);
/* The same in two stages, for SyncBatchNorm (replaces torch.nn.SyncBatchNorm's batch_norm_stats /
 * batch_norm_gather_stats_with_counts / batch_norm_elemt for the data-parallel train path):
 * stats[2c] = sum x, stats[2c+1] = sum x^2 over this rank's batch (fp64) and stats[2C] = this rank's
 * B*H*W (stats holds 2C+1 doubles) -> the caller all-reduces all 2C+1 doubles over ranks (one collective;
 * the count rides along) -> apply.  apply's count > 0 is used as given; count <= 0 reads the global count
 * from stats[2C] on the device (no host synchronisation).  B may be 0 (an empty local shard joins the
 * all-reduce with zero sums and still updates the running statistics). */
int ldm_batchnorm_stats(const float* x, int32_t B, int32_t C, int32_t HW, double* stats, float* workspace,
                        void* stream);
/* ldm_batchnorm_stats with a storage code (LDM_ST_X16 | type << LDM_ST_SHIFT: a 16-bit input) */
int ldm_batchnorm_stats_code(const float* x, int32_t code, int32_t B, int32_t C, int32_t HW, double* stats,
                             float* workspace, void* stream);
int ldm_batchnorm_apply(float* x, int32_t B, int32_t C, int32_t HW, const double* stats, double count,
                        const float* weight, const float* bias, float* running_mean, float* running_var,
                        float momentum, float eps, int32_t act, float* save_mean, float* save_invstd, void* stream);
int ldm_batchnorm_apply_out(const float* x, float* y, int32_t B, int32_t C, int32_t HW, const double* stats,
                            double count, const float* weight, const float* bias, float* running_mean,
                            float* running_var, float momentum, float eps, int32_t act, float* save_mean,
                            float* save_invstd, void* stream);

/* ---- eval-mode BatchNorm2d (+activation) as a standalone op, out-of-place (y may equal x) ------ */
int ldm_batchnorm_eval(const float* x, float* y, int32_t B, int32_t C, int32_t HW, const float* weight,
                       const float* bias, const float* running_mean, const float* running_var, float eps, int32_t act,
                       void* stream);

/* ---- elementwise activation, out-of-place (y may equal x): ReLU / Tanh / (tanh+1)/2 / GELU ------ */
int ldm_activation(const float* x, float* y, int64_t n, int32_t act, void* stream);

/* ---- SinusoidalPositionEmbeddings.forward (model.py:239-246) alone: out [B,dim] ---------------- */
int ldm_sinusoid_embed(const void* t, int32_t t_is_float, int32_t B, int32_t dim, const float* freqs, float* out,
                       void* stream);

/* ---- time MLP: SinusoidalPositionEmbeddings -> Linear -> GELU -> Linear (model.py:170-175,
 * :239-246).  t: [B] int64 (t_is_float=0) or float32 (t_is_float=1); freqs [dim/2] = the
 * reference's exp(arange(half)*-(ln 1e4/(half-1))) table; w1,w2 [dim,dim] torch Linear layout. */
int ldm_time_mlp_forward(const void* t, int32_t t_is_float, int32_t B, int32_t dim, const float* freqs,
                         const float* w1, const float* b1, const float* w2, const float* b2, float* out,
                         void* stream);

/* ---- cross-attention core (nn.MultiheadAttention inside CrossAttention, model.py:126-160) -------
 * q [B,E,L] (the Q in-projection output in NCHW token order), kv [B,2E,S] (K channels then V
 * channels), out [B,E,L] = softmax((q*scale)^T k) v per head, written channel-major so the
 * out-projection reads it as NCHW (the reference's two permutes, model.py:144-158, vanish). */
/* Folded-query form for a fixed key set (the reverse loop's style maps): kf [B,heads,S,E] =
 * scale * Wq_h^T K_h, bf [B,heads,S] = scale * bq_h^T K_h from kv [B,2E,S] and the Q in-projection
 * (wq [E,E] torch layout, bq [E]); ldm_attention_folded then takes the projection's input z [B,L,E]
 * (token-major) and writes out [B,L,E] (token-major) = the same attention as q = Wq z + bq.
 * Replaces the Q in-projection + score product of nn.MultiheadAttention (model.py:153). */
int ldm_attention_fold_keys(const float* kv, const float* wq, const float* bq, int32_t B, int32_t E, int32_t heads,
                            int32_t S, float scale, float* kf, float* bf, void* stream);
int ldm_attention_folded(const float* z, const float* kv, const float* kf, const float* bf, float* out, int32_t B,
                         int32_t E, int32_t heads, int32_t L, int32_t S, void* stream);
/* The folded attention's probabilities only: p [B,heads,L,S] = softmax(z^T kf_h + bf_h) (CA1's instance: E 512,
 * 4 heads, L, S <= 16).  The reverse loop's bottleneck then contracts them with its folded values (below). */
int ldm_attention_folded_probs(const float* z, const float* kf, const float* bf, float* p, int32_t B, int32_t E,
                               int32_t heads, int32_t L, int32_t S, void* stream);
/* The bottleneck after CA1 with the attention's values folded into its weights (bfold.hip; model.py:214-217):
 * u [B,512,576] = W' (x) V once per loop, u[b][co][(t*4 + h)*16 + s] = sum_d w_fold[co][h*128 + d][t] *
 * kv[b][512 + h*128 + d][s] (w_fold = the bottleneck o out-projection fold of ldm_fold_conv_proj, torch layout
 * [512,512,3,3]; kv the CA1 K/V projection [B,1024,16]); then per step y [B,2,8,512] (NHWC) = relu(sum over
 * (t, h, s) of u * p[b][h][l_t][s] + pos_bias[l][co]) with pos_bias [16][512] (position-major) and p from
 * ldm_attention_folded_probs.  dtype LDM_DT_F16 / _BF16 rounds the output to that type (operands stay fp32).
 * Used by ldm_ddim_sample when ldm_bneck_fold_supported(B, H, W): the canonical 16 x 64 latent, B <= 8
 * (LDM_BNECK_FOLD=0 turns it off). */
int32_t ldm_bneck_fold_supported(int32_t B, int32_t H, int32_t W);
int ldm_bneck_fold_values(const float* w_fold, const float* kv, float* u, int32_t B, void* stream);
int ldm_bneck_pv(const float* u, const float* p, const float* pos_bias, float* y, int32_t B, int32_t dtype,
                 void* stream);
/* CA1's probabilities P [B,4,16,16] only, one block of eight waves per (sample, head): the reverse loop's form
 * (LDM_CA1P_FORM=0 keeps ldm_attention_folded_probs).  z4 token-major [B,16,512], kf [B,4,16,512], bf [B,4,16]. */
int ldm_ca1_probs(const float* z4, const float* kf, const float* bf, float* p, int32_t B, void* stream);
/* 1 when the reverse loop forms CA1's probabilities with ldm_ca1_probs, 0 when with ldm_attention_folded_probs
 * (LDM_CA1P_FORM=0): what bench.py times for the loop's CA1 launch. */
int32_t ldm_ca1_probs_form(void);
/* A/B switch of the Cin = 1 stride-2 conv's packed form (two output channels per v_pk_fma_f32; bitwise the scalar
 * form's results): 1 on, 0 off; returns the previous setting.  Default: LDM_CIN1_PK. */
int ldm_set_cin1_packed(int on);
/* A/B switch of the Cin = 1 k3 stride-1 conv's four-column form (conv_cin1_x4_kernel, SD = 1: the UNet's first layer on
 * the raw mel, UNet(1, 1) at shape S; models/model.py:178 Conv2d(in_channels, num_filters, 3, 1, 1)) against the one-lane-per-pixel
 * kernel, bitwise the same results: 1 on, 0 off; returns the previous setting.  Default: LDM_CIN1_S1. */
int ldm_set_cin1_s1(int on);
/* A/B switch of the flash attention forward's key splits over blocks (flash.hip: where one block per (query tile,
 * head) fills under a quarter of the CUs — CA1 at shape S — the key tiles split over up to 4 blocks and a combine pass
 * merges their (O, m, l); CrossAttention, models/model.py:126-160): 1 on, 0 off; returns the previous setting.
 * Default: LDM_FLASH_SPLIT. */
int ldm_set_flash_split(int on);
/* A conv (descriptor d, weight w_conv [Cout,Cmid,kh,kw], bias b_conv or NULL) applied to the output of a
 * Linear/1x1 projection (w_proj [Cmid,Cin], b_proj [Cmid]) as ONE conv: w_out [Cout,Cin,kh,kw] =
 * w_conv o w_proj and pos_bias_out [Cout,Hout,Wout] = b_conv + the projection bias through the taps that
 * fall inside the input (padding taps see zeros).  Used for out_proj -> enc4 / bottleneck
 * (model.py:155-160 then :212 / :217) in the reverse loop. */
int ldm_fold_conv_proj(const ldm_conv_desc* d, const float* w_conv, const float* b_conv, const float* w_proj,
                       const float* b_proj, int32_t Cmid, float* w_out, float* pos_bias_out, void* stream);
int ldm_attention_core(const float* q, const float* kv, float* out, int32_t B, int32_t E, int32_t heads,
                       int32_t L, int32_t S, float scale, void* stream);
/* Width-general form (flash.hip; any L, S, head dim 64 or 128 — the UNet's token counts grow with the mel
 * width, model.py:140-153): KV-tiled online softmax, channel-major q / out as ldm_attention_core, plus
 * lse [B,heads,L] = the log-sum-exp of each query's scaled scores for ldm_attention_backward_flash.
 * ldm_attention_core itself hands over to this kernel when L or S exceeds its LDS-resident instances. */
int ldm_attention_flash_supported(int32_t E, int32_t heads);
int ldm_attention_forward_lse(const float* q, const float* kv, float* out, float* lse, int32_t B, int32_t E,
                              int32_t heads, int32_t L, int32_t S, float scale, void* stream);

/* ---- DDPM forward noising q_sample (ForwardDiffusion.forward, model.py:102-115) ----------------
 * z_t = sqrt(ab[t_b]) * x0 + sqrt(1-ab[t_b]) * eps.  coef_table [T,2] = {sqrt(ab), sqrt(1-ab)} per
 * timestep (device), t [B] int64 (device).  t outside [0,T) yields NaN for that sample (the
 * reference raises IndexError, model.py:107; the Python layer checks host-known t up front). */
int ldm_q_sample(const float* x0, const float* eps, const float* coef_table, int32_t T, const int64_t* t, float* zt,
                 int32_t B, int64_t per_sample, void* stream);
/* predict_start_from_noise (model.py:117-124): x0 = (z_t - sqrt(1-ab) * eps) / sqrt(ab), table as above. */
int ldm_predict_start(const float* zt, const float* eps, const float* coef_table, int32_t T, const int64_t* t,
                      float* x0, int32_t B, int64_t per_sample, void* stream);
/* Backward of the two gathers above: kind 0 (q_sample): grad_a = sqrt(ab)*g -> d x0, grad_b = sqrt(1-ab)*g
 * -> d eps; kind 1 (predict_start): grad_a = g/sqrt(ab) -> d z_t, grad_b = -sqrt(1-ab)*g/sqrt(ab) -> d eps.
 * Either output may be NULL. */
int ldm_sched_backward(int32_t kind, const float* grad, const float* coef_table, int32_t T, const int64_t* t,
                       float* grad_a, float* grad_b, int32_t B, int64_t per_sample, void* stream);
/* One reverse step of style_conditioned_ddim_sample / content_style_ddim_sample (model.py:439-463):
 * coef[4] = {sqrt(ab_t), sqrt(1-ab_t), sqrt(ab_next), sqrt(1-ab_next)} (device, uniform over the
 * batch), eta as in the reference (deterministic term).  x is updated in place; x0_log / eps_log
 * (may be NULL) receive pred_x0 / noise_pred clones.  Bitwise equal to the reference's fp32 op
 * sequence for identical inputs (no FMA contraction). */
int ldm_ddim_step(float* x, const float* eps, const float* coef, float eta, float* x0_log, float* eps_log,
                  int64_t n, void* stream);

/* ---- loss reductions (loss.py): kind 0 = mean((a-b)^2) (diffusion_loss :48-49, nn.MSELoss :35),
 * kind 1 = mean(0.5*(a^2-1-log(a^2+1e-8))) (kl_regularization_loss :31-32, b unused).
 * Deterministic: fixed partition, fp64 partials.  workspace >= 512 doubles; out is a device scalar. */
int ldm_loss_forward(int32_t kind, const float* a, const float* b, int64_t n, void* workspace, float* out,
                     void* stream);
/* grad_a / grad_b (may be NULL) = d(loss)/d(a|b) * grad_out[0] (device scalar). */
int ldm_loss_backward(int32_t kind, const float* a, const float* b, int64_t n, const float* grad_out, float* grad_a,
                      float* grad_b, void* stream);

/* ---- whole UNet forward (UNet.forward, model.py:196-231) and the DDIM sampling loop ------------- */
typedef struct ldm_unet_weights {
    /* conv layers in order enc1, enc2, enc3, enc4, bottleneck, dec4, dec3, dec2, dec1:
     * packed (or raw, for direct plans) weights and biases */
    const float* conv_w[9];
    const float* conv_b[9];
    ldm_conv_plan conv_plan[9];
    /* cross_attention2 (E=256) then cross_attention1 (E=512): packed Q-proj / KV-proj / out-proj */
    const float* ca_wq[2];
    const float* ca_bq[2];
    ldm_conv_plan ca_plan_q[2];
    const float* ca_wkv[2];
    const float* ca_bkv[2];
    ldm_conv_plan ca_plan_kv[2];
    const float* ca_wo[2];
    const float* ca_bo[2];
    ldm_conv_plan ca_plan_o[2];
    /* time MLP */
    const float* t_freqs;
    const float* t_w1;
    const float* t_b1;
    const float* t_w2;
    const float* t_b2;
    /* Re-associated forms used by the reverse loop when use_fold != 0 (ldm_fold_conv_proj,
     * ldm_attention_fold_keys): raw Q in-projection rows (in_proj_weight[:E], torch layout) of both
     * cross-attentions, and enc4 / bottleneck composed with the preceding out-projection
     * (packed with conv_plan[3] / conv_plan[4]) plus their position-dependent biases [Cout,Hout,Wout]. */
    const float* ca_wq_raw[2];
    const float* fold_w[2];
    const float* fold_pb[2];
    int32_t use_fold;
    /* Step kernels of the reverse loop (used when use_step != 0 together with use_fold, for latent C = 32
     * and num_filters = 64): the nine convs packed by ldm_step_pack_weight (enc4 / bottleneck: their
     * folded weights), and the folded position biases transposed to [Hout*Wout][Cout].  use_step 1: the
     * register-direct kernels (uconv.hip, any latent with H, W multiples of 8); 2: the same (it selected the
     * LDS-staged kernels of rounds 2-5, measured slower and removed in round 6). */
    const float* step_w[9];
    const float* step_pb[2];
    int32_t use_step;
    int32_t step_dtype;   /* LDM_DT_*: operand precision of the step kernels (not F32: uconv.hip only) */
    /* The bottleneck o CA1 out-projection fold in the torch layout [512,512,3,3] (ldm_fold_conv_proj's w_out,
     * unpacked): the source of the folded values U when the loop runs the bottleneck on them
     * (ldm_bneck_fold_supported; ldm_bneck_fold_values).  NULL: the uconv bottleneck. */
    const float* step_bneck_w;
} ldm_unet_weights;

typedef struct ldm_unet_shape {
    int32_t B, C, H, W;   /* latent [B,C,H,W]; style s5 [B,256,H/4,W/4], s6 [B,512,H/8,W/8] */
    int32_t nf;           /* num_filters (64)                                                   */
} ldm_unet_shape;

/* Workspace floats needed by ldm_unet_forward for this shape and these plans (w may be NULL: plans
 * without cross-block K splits).  The workspace must be zero-filled once before its first use (it
 * holds the split-K tile counters, which every call leaves zero again). */
int64_t ldm_unet_workspace_floats(const ldm_unet_shape* s, const ldm_unet_weights* w);
/* Fill the 9+6 conv plans of `w` for this shape (weights must then be packed by the caller). */
int ldm_unet_make_plans(const ldm_unet_shape* s, ldm_unet_weights* w);
/* Conv descriptors of the 9 convs + 6 projection GEMMs (index order as in ldm_unet_weights). */
int ldm_unet_layer_desc(const ldm_unet_shape* s, int32_t layer, ldm_conv_desc* d);
int ldm_unet_forward(const ldm_unet_shape* s, const ldm_unet_weights* w, const float* z, const void* t,
                     int32_t t_is_float, const float* s5, const float* s6, float* out, float* workspace,
                     void* stream);

/* Reverse loop (style_conditioned_ddim_sample model.py:409-465 / content_style_ddim_sample :503-559):
 * x [B,C,H,W] updated in place over nsteps = len(times)-1 steps.  t_table [nsteps,B] int64 holds
 * times[i] repeated over the batch, coef_table [nsteps,4] the per-step coefficients.  x0_logs /
 * eps_logs (may be NULL) hold step i at x0_logs + i*log_step_stride ([B,C,H,W] each; stride 0 = dense
 * B*C*H*W), so a sub-batch can write straight into its slice of the full-batch logs.
 * workspace: ldm_ddim_workspace_floats(s, w, nsteps) floats, zero-filled before first use.
 * The time MLP for all steps is one launch before the loop; each step's update is fused into dec1's
 * epilogue.  Only launches: the caller may capture the whole loop into one hipGraph (the Python layer
 * does, with torch.cuda.CUDAGraph, splitting the batch into independent sub-batch chains on separate
 * streams so that one chain's launch / memory latency overlaps another's work). */
int64_t ldm_ddim_workspace_floats(const ldm_unet_shape* s, const ldm_unet_weights* w, int32_t nsteps);
int ldm_ddim_sample(const ldm_unet_shape* s, const ldm_unet_weights* w, float* x, const float* s5,
                    const float* s6, const int64_t* t_table, const float* coef_table, int32_t nsteps, float eta,
                    float* x0_logs, float* eps_logs, int64_t log_step_stride, float* workspace, void* stream);

/* ---- data formats either side of the path (dataio.hip) ---------------------------
 * ldm_mel_quantize: the reference's 8-bit mel PNG pixels, uint8(clip((db + max_db) * 255/max_db, 0, 255)
 * + 0.5) (audio_processor.py:55-73, fp32 arithmetic, bit-exact with its numpy); ldm_mel_dequantize: its
 * inverse db = u8 * max_db/255 - max_db (audio_processor.py:91-93); ldm_u8_to_unit: the [0,1] tensor the
 * model consumes, u8 / 255 (dataset.py:258, torchvision ToTensor). */
int ldm_mel_quantize(const float* db, uint8_t* out, int64_t n, float max_db, void* stream);
int ldm_mel_dequantize(const uint8_t* in, float* db, int64_t n, float max_db, void* stream);
int ldm_u8_to_unit(const uint8_t* in, float* out, int64_t n, void* stream);

/* ---- step kernels (uconv.hip): fixed-structure implicit GEMMs of the nine UNet convs -------------------
 * Packed size (floats) of layer `layer` (0..8 = enc1..dec1) and its packing from the torch weight layout
 * (conv [Cout][Cin][3][3], transposed conv [Cin][Cout][3][3]).  ldm_step_conv runs one layer on NHWC
 * activations (latent [B,H,W] with H, W multiples of 8): y = act(conv(x) + bias) (+ bcast[b][c] for
 * enc2) (+ skip for dec4..dec2); bias is [Cout], or [Hout*Wout][Cout] for the folded enc4 / bottleneck.
 * dec1 only runs fused with the DDIM update inside ldm_ddim_sample. */
int64_t ldm_step_packed_floats(int32_t layer);
int ldm_step_pack_weight(int32_t layer, const float* w, float* packed, void* stream);
/* The pack for an operand precision: LDM_DT_F32 as ldm_step_pack_weight; LDM_DT_F16 / LDM_DT_BF16 write the
 * same layout in 16-bit elements (ldm_step_packed_floats / 2 floats of storage), which is what every step
 * conv with that dtype reads (ldm_step_conv_dt, _ws, ldm_step_dec1_ddim, ldm_unet_weights.step_w). */
int ldm_step_pack_weight_dt(int32_t layer, int32_t dtype, const float* w, float* packed, void* stream);
int ldm_step_conv(int32_t layer, int32_t B, int32_t H, int32_t W, const float* x, const float* packed,
                  const float* bias, const float* bcast, const float* skip, float* y, void* stream);
/* The step kernels of the deep layers (enc3, enc4, bottleneck, dec4, dec3) also come in a K-split form: a
 * 32x32 block tile with K split over 2-8 blocks (write-through partial tiles, the last block of a tile sums
 * them in split order), half the operand bytes per block.  It runs when a workspace is given (and
 * LDM_UCONV_KS, a layer bit mask, selects the layer; default all five): ldm_step_workspace_floats(B, H, W)
 * floats, zero-filled once (its counters return to zero after every launch); launches on one stream may
 * share it.  ldm_step_conv / ldm_step_conv_dt run the single-block form. */
int64_t ldm_step_workspace_floats(int32_t B, int32_t H, int32_t W);
/* The leading part of that workspace that holds the split-K tile counters (one int32 per tile of the layer with
 * the most tiles, rounded up to 64): zero between launches, like the 64 layer-pair counters at its end. */
int64_t ldm_step_workspace_counter_floats(int32_t B, int32_t H, int32_t W);
int ldm_step_conv_ws(int32_t layer, int32_t B, int32_t H, int32_t W, const float* x, const float* packed,
                     const float* bias, const float* bcast, const float* skip, float* y, int32_t dtype,
                     float* workspace, void* stream);
/* dec1 with the fused DDIM update, as the reverse loop runs it: d2 [B,H,W,64] NHWC, xs [B,H,W,32] NHWC sampler
 * state updated in place, coef [4] {sqrt(ab_t), sqrt(1-ab_t), sqrt(ab_next), sqrt(1-ab_next)}, x0_log /
 * eps_log NCHW [B,32,H,W] or NULL (model.py:442-463). */
int ldm_step_dec1_ddim(int32_t B, int32_t H, int32_t W, const float* d2, const float* packed, const float* bias,
                       const float* coef, float eta, float* xs, float* x0_log, float* eps_log, int32_t dtype,
                       void* stream);
/* Which reverse-loop layers run uconv.hip's K-split form (bit l = layer l; LDM_UCONV_KS, default enc4 +
 * bottleneck + dec4); every other layer runs the single-block form. */
int ldm_step_layer_forms(int32_t* ks_layers);
/* ldm_step_conv with an operand precision LDM_DT_* (ldm_step_conv = LDM_DT_F32). */
int ldm_step_conv_dt(int32_t layer, int32_t B, int32_t H, int32_t W, const float* x, const float* packed,
                     const float* bias, const float* bcast, const float* skip, float* y, int32_t dtype, void* stream);

/* ---- train step backward (LDMTrainer.train_step, train.py:163-208: scaler.scale(loss).backward()) ---
 * Data gradients of a conv are the forward kernel on the dual descriptor (conv <-> transposed conv);
 * these are the remaining pieces.  All reductions are fixed-order (bitwise reproducible). */
/* dW of nn.Conv2d / nn.ConvTranspose2d for descriptor d (the FORWARD descriptor): x = layer input,
 * dy = gradient at the layer's pre-epilogue output.  dw in the torch weight layout; accumulate != 0 adds.
 * workspace: ldm_conv_wgrad_workspace_floats(d) floats. */
int64_t ldm_conv_wgrad_workspace_floats(const ldm_conv_desc* d);
/* ldm_conv_backward_weight with an operand precision LDM_DT_* (the tap-shared kernel rounds x and dy;
 * shapes it does not cover run the fp32 kernel). */
int ldm_conv_backward_weight_dt(const ldm_conv_desc* d, const float* x, const float* dy, float* dw,
                                int32_t accumulate, float* workspace, int32_t dtype, void* stream);
/* ldm_conv_backward_weight_dt with a tap-shared gradient's split-K reduction deferred (the train step's weight
 * gradients are read only by the optimizer): the partials stay in `workspace` (ldm_conv_wgrad_workspace_floats,
 * kept until the reduction) and *splits_out receives their count S (0: nothing deferred, dw written).
 * ldm_wgrad_reduce_many then reduces every job in one launch per 24 jobs, bitwise ldm_conv_backward_weight_dt's
 * result (MN = the gradient's element count, a multiple of 4; partial and dw 16-byte aligned). */
int ldm_conv_backward_weight_defer(const ldm_conv_desc* d, const float* x, const float* dy, float* dw,
                                   int32_t accumulate, float* workspace, int32_t dtype, int32_t* splits_out,
                                   void* stream);
typedef struct ldm_wgrad_red_job {
    const float* partial;   /* [S][MN] */
    float* dw;              /* [MN] */
    int32_t S, MN, accumulate;
} ldm_wgrad_red_job;
int ldm_wgrad_reduce_many(const ldm_wgrad_red_job* jobs, int32_t n, void* stream);
/* The 16-bit storage flags (LDM_DT_X16 | LDM_DT_DY16) ldm_conv_backward_weight_dt takes for d at a 16-bit
 * operand precision (0: neither; the caller then passes fp32 tensors). */
int32_t ldm_conv_wgrad_storage16(const ldm_conv_desc* d);
int ldm_conv_backward_weight(const ldm_conv_desc* d, const float* x, const float* dy, float* dw, int32_t accumulate,
                             float* workspace, void* stream);
/* Backward of the fused epilogue act(v) (+bcast[b,c]) (+skip): dv = dy*act'(v) (from act_out = act(v);
 * GELU from pre_act = v), dbias[c] = sum dv, dbcast[b,c] = sum_hw dy.  dv / dbias / dbcast may be NULL;
 * dv may alias dy.  workspace: ldm_reduce_workspace_floats(B,C,HW) floats (NULL when no sums). */
int ldm_act_backward(const float* dy, const float* act_out, const float* pre_act, int32_t act, int32_t B, int32_t C,
                     int32_t HW, float* dv, float* dbias, float* dbcast, float* workspace, void* stream);
/* ldm_act_backward with the bias gradient's finalize deferred (the train step's convs: their bias gradients are read
 * only by the optimizer): the slice partials go to `workspace` (ldm_act_partial_floats(B, C, HW) floats, kept until
 * the finalize), *q_out receives their slice count for the job (0: nothing deferred — the small-plane kernel
 * wrote dbias itself).  No bcast gradient.  ldm_act_finalize_many then writes every job's dbias in one launch per 24
 * jobs, bitwise what ldm_act_backward writes. */
int ldm_act_backward_defer(const float* dy, const float* act_out, const float* pre_act, int32_t act_code, int32_t B,
                           int32_t C, int32_t HW, float* dv, float* dbias, float* workspace, int32_t* q_out, void* stream);
int64_t ldm_act_partial_floats(int32_t B, int32_t C, int32_t HW);
typedef struct ldm_act_fin_job {
    const float* part;   /* the deferred call's partials */
    float* dbias;        /* [C]: the sums */
    int32_t B, C, Q;     /* Q: the call's *q_out (kind 1: *p_out) */
    int32_t kind;        /* 0: ldm_act_backward_defer; 1: ldm_batchnorm_backward_dxsum_defer's dx sum */
} ldm_act_fin_job;
int ldm_act_finalize_many(const ldm_act_fin_job* jobs, int32_t n, void* stream);
/* train-mode BatchNorm2d (+ReLU/Tanh) backward from the saved batch stats of ldm_batchnorm_train:
 * y = its output, x = its input, weight / bias its affine parameters (NULL = 1 / 0); dx / dweight / dbias
 * may be NULL.  y may be NULL when act is NONE or RELU: the ReLU mask is then re-evaluated from x with the
 * forward's own arithmetic (one tensor read less per pass).  workspace as ldm_batchnorm_train. */
int ldm_batchnorm_backward(const float* dy, const float* y, const float* x, const float* save_mean,
                           const float* save_invstd, const float* weight, const float* bias, int32_t act, int32_t B,
                           int32_t C, int32_t HW, float* dx, float* dweight, float* dbias, float* workspace,
                           void* stream);
/* ldm_batchnorm_backward (dx required) that also writes dx_sum[c] = the sum of dx (as stored) over (b, h, w): the
 * bias gradient of the conv whose output x is, without a sweep of its own over dx (round 6).  workspace as
 * ldm_batchnorm_train (ldm_reduce_workspace_floats covers the extra slice partials). */
int ldm_batchnorm_backward_dxsum(const float* dy, const float* y, const float* x, const float* save_mean,
                                 const float* save_invstd, const float* weight, const float* bias, int32_t act,
                                 int32_t B, int32_t C, int32_t HW, float* dx, float* dweight, float* dbias,
                                 float* dx_sum, float* workspace, void* stream);
/* ldm_batchnorm_backward_dxsum with the dx sum's finalize deferred to ldm_act_finalize_many (a job of kind 1 with
 * part = dxs_part, dbias = dx_sum, Q = *p_out); dxs_part holds ldm_bn_dxsum_partial_floats(B, C, HW) floats. */
int ldm_batchnorm_backward_dxsum_defer(const float* dy, const float* y, const float* x, const float* save_mean,
                                       const float* save_invstd, const float* weight, const float* bias, int32_t act_code,
                                       int32_t B, int32_t C, int32_t HW, float* dx, float* dweight, float* dbias,
                                       float* dx_sum, float* dxs_part, int32_t* p_out, float* workspace, void* stream);
int64_t ldm_bn_dxsum_partial_floats(int32_t B, int32_t C, int32_t HW);
/* The same in two stages for SyncBatchNorm: sums[2c] = sum g, sums[2c+1] = sum g*xhat over this rank
 * (g = dy*act'(y)) and sums[2C] = this rank's B*H*W (sums holds 2C+1 doubles); dbias / dweight get the
 * local sums (parameter grads stay local, as in torch.nn.SyncBatchNorm; the DP gradient all-reduce
 * averages them) -> the caller all-reduces all 2C+1 doubles -> apply (count <= 0: read sums[2C]). */
int ldm_batchnorm_backward_reduce(const float* dy, const float* y, const float* x, const float* save_mean,
                                  const float* save_invstd, const float* weight, const float* bias, int32_t act,
                                  int32_t B, int32_t C, int32_t HW, double* sums, float* dweight, float* dbias,
                                  float* workspace, void* stream);
int ldm_batchnorm_backward_apply(const float* dy, const float* y, const float* x, const float* save_mean,
                                 const float* save_invstd, const float* weight, const float* bias, int32_t act,
                                 int32_t B, int32_t C, int32_t HW, const double* sums, double count, float* dx,
                                 void* stream);
/* Backward of ldm_attention_core: dq [B,E,L], dkv [B,2E,S] (dK then dV). */
int ldm_attention_backward(const float* q, const float* kv, const float* dout, float* dq, float* dkv, int32_t B,
                           int32_t E, int32_t heads, int32_t L, int32_t S, float scale, void* stream);
/* The same backward for any L, S (flash.hip), from the forward's out and lse (ldm_attention_forward_lse):
 * delta = rowsum(dO * O) into delta_ws [B,heads,L], then dK/dV (64 keys per block, q and dO streamed) and
 * dQ (64 queries per block, K and V streamed), deterministic. */
int ldm_attention_backward_flash(const float* q, const float* kv, const float* out, const float* lse,
                                 const float* dout, float* dq, float* dkv, float* delta_ws, int32_t B, int32_t E,
                                 int32_t heads, int32_t L, int32_t S, float scale, void* stream);

/* ---- multi-tensor weight re-pack (the train step refreshes every packed trainable conv weight after the
 * optimizer step in one launch instead of one per weight; pack.hip).  ldm_pack_many_prepare fills
 * n * ldm_pack_job_bytes() bytes of host_jobs with the jobs for (descs[i], plans[i]) reading the torch-layout
 * weight w[i] into out[i] (the buffer ldm_conv_pack_weight would fill, kinds 1-3) and returns the launch
 * size; copy the table to device memory once, then ldm_pack_many(table, n, launch_size, stream) re-packs
 * them all (same values as ldm_conv_pack_weight). */
int64_t ldm_pack_job_bytes(void);
int ldm_pack_many_prepare(const ldm_conv_desc* descs, const ldm_conv_plan* plans, const float* const* w,
                          void* const* out, int32_t n, void* host_jobs, int64_t* launch_size);
int ldm_pack_many(const void* device_jobs, int32_t n, int64_t launch_size, void* stream);

/* ---- LPIPS-AlexNet perceptual distance (loss.py:6-21: lpips==0.1.4 LPIPS(net='alex') on 2x-1)
 * The AlexNet convs run on ldm_conv_forward: 3x3 directly, 11x11/s4 and 5x5 as ldm_im2col + a 1x1 conv (their
 * data gradient: the 1x1 dual conv + ldm_col2im).  col [B,Kpad,Ho,Wo], k = (c*kh+ky)*kw+kx, rows >= Cv*kh*kw
 * zero.  shift/scale (or NULL): the LPIPS ScalingLayer fused, a 1-channel input broadcast to Cv channels
 * (t - shift_c)/scale_c; unit=1 first maps x -> 2x - 1 (perceptual_loss_old); col2im folds both back into dx.
 * ldm_maxpool3s2: nn.MaxPool2d(3, 2) (floor); its backward routes dy to torch's first-occurrence argmax.
 * ldm_lpips_layer: val[b] += mean_p sum_c w_c (f0_c/(|f0|+1e-10) - f1_c/(|f1|+1e-10))^2 (normalize_tensor,
 * squared difference, 1x1 lin head without bias, spatial average); workspace >= B*HW floats.
 * ldm_lpips_layer_backward: d val / d f1 (side 1) or d f0 (side 0) times gval[b], written or accumulated. */
int ldm_im2col(const float* x, int32_t B, int32_t C, int32_t H, int32_t W, int32_t kh, int32_t kw, int32_t stride,
               int32_t pad, int32_t Kpad, const float* shift, const float* scale, int32_t Cv, int32_t unit, float* col,
               void* stream);
int ldm_col2im(const float* col, int32_t B, int32_t C, int32_t H, int32_t W, int32_t kh, int32_t kw, int32_t stride,
               int32_t pad, int32_t Kpad, const float* scale, int32_t Cv, int32_t unit, float* dx, void* stream);
int ldm_maxpool3s2(const float* x, float* y, int32_t B, int32_t C, int32_t H, int32_t W, void* stream);
int ldm_maxpool3s2_backward(const float* x, const float* dy, float* dx, int32_t B, int32_t C, int32_t H, int32_t W,
                            void* stream);
int ldm_lpips_layer(const float* f0, const float* f1, const float* w, int32_t B, int32_t C, int32_t HW, float* val,
                    float* workspace, void* stream);
int ldm_lpips_layer_backward(const float* f0, const float* f1, const float* w, const float* gval, int32_t B,
                             int32_t C, int32_t HW, int32_t side, int32_t accumulate, float* df, void* stream);

/* ---- VGGish feature / style loss (loss.py:52-101, VGGishFeatureLoss.forward) ----
 * The conv stack runs on ldm_conv_forward (ReLU fused: each conv launch yields one feature tap).
 * ldm_maxpool2x2: nn.MaxPool2d(2, 2) on NCHW fp32 (floor mode, NaN-propagating), y [B,C,H/2,W/2].
 * ldm_std_mse_moments: per sample b of p, t [B][n] (n = C*H*W contiguous): moments[b][0..4] = sum p,
 *   sum p^2, sum t, sum t^2, sum p*t (fp64, fixed slices and order; workspace
 *   ldm_std_mse_workspace_floats(B, n) floats, 8-byte aligned).
 * ldm_std_mse_accumulate: *acc += scale * mse(p / (std(p) + eps), t / (std(t) + eps)) from the moments
 *   (torch.std per sample over dims 1..3, unbiased), and *out = (float)*acc when out is not NULL. */
int ldm_maxpool2x2(const float* x, float* y, int32_t B, int32_t C, int32_t H, int32_t W, void* stream);
int64_t ldm_std_mse_workspace_floats(int32_t B, int64_t n);
int ldm_std_mse_moments(const float* p, const float* t, int32_t B, int64_t n, double* moments, float* workspace,
                        void* stream);
int ldm_std_mse_accumulate(const double* moments, int32_t B, int64_t n, double eps, double scale, double* acc,
                           float* out, void* stream);

/* ---- optimiser: torch.optim.Adam (train.py:156) + torch.amp.GradScaler (train.py:157,189-201) ----
 * Multi-tensor: `slots` (device array) lists the parameters; the work is cut into chunks of
 * chunk_len elements, chunk i covering slots[chunk_tensor[i]] from element chunk_start[i]. */
typedef struct ldm_tensor_slot {
    float* param;
    float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    int64_t numel;
} ldm_tensor_slot;
/* scaler.unscale_: grad *= inv_scale[0] (device scalar, NULL = 1); found_inf[0] |= any non-finite. */
int ldm_unscale_check(const ldm_tensor_slot* slots, const int32_t* chunk_tensor, const int64_t* chunk_start,
                      int32_t nchunks, int32_t chunk_len, const float* inv_scale, int32_t* found_inf, void* stream);
/* optimizer.step() (skipped entirely when found_inf[0] != 0, as scaler.step does). step = 1-based.
 * decoupled = 0: torch.optim.Adam (L2 added to the gradient); 1: torch.optim.AdamW (train.py:44).
 * Hyper-parameters are the optimizer's python floats (double); derived scalars are formed in double
 * and cast once to fp32, as torch's Adam does. */
int ldm_adam_step(const ldm_tensor_slot* slots, const int32_t* chunk_tensor, const int64_t* chunk_start,
                  int32_t nchunks, int32_t chunk_len, double lr, double beta1, double beta2, double eps,
                  double weight_decay, int32_t decoupled, int32_t step, const int32_t* found_inf, void* stream);
/* The capturable form of ldm_adam_step (hipGraph-captured train steps, LDMTrainer.graph_step): the step
 * count is the device float step[0], advanced by one only when found_inf[0] == 0 (or found_inf NULL);
 * the derived scalars are formed from it on the device exactly as ldm_adam_step forms them on the host,
 * into the caller's 8-float device workspace `scalars`.  Replaces torch.optim.Adam(capturable=True)'s
 * _single_tensor_adam capturable branch (train.py:156's optimizer when the step is graph-captured). */
int ldm_adam_step_dev(const ldm_tensor_slot* slots, const int32_t* chunk_tensor, const int64_t* chunk_start,
                      int32_t nchunks, int32_t chunk_len, double lr, double beta1, double beta2, double eps,
                      double weight_decay, int32_t decoupled, float* step, const int32_t* found_inf, float* scalars,
                      void* stream);
/* scaler.update(): scale *= backoff on inf (tracker = 0), *= growth after growth_interval clean steps. */
int ldm_update_scale(float* scale, int32_t* growth_tracker, const int32_t* found_inf, float growth_factor,
                     float backoff_factor, int32_t growth_interval, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LDM_CAPI_H */
