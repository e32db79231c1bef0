"""ORACLE — test infrastructure only.  CPU restatement of the reference's latent-diffusion hot path in
functional PyTorch-CPU fp32 (the same ATen kernels the reference's CPU path dispatches to).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only
as the checker / the timed CPU baseline — never as the product path (the product path has no CPU
fallback and raises without its HIP library).

Every function takes a flat state dict (reference key names) and cites the
reference lines it restates.  Pinned against tests/golden/ref_goldens.npz (captured by importing the
reference itself) by tests/test_oracle_golden.py.
"""
import math

import torch
import torch.nn.functional as F


def _g(sd, k):
    v = sd[k]
    return v if isinstance(v, torch.Tensor) else torch.from_numpy(v)


# ---- schedule (model.py:90-100) ------------------------------------------------------------------
def schedule(T):
    beta = torch.linspace(0.0001, 0.02, T)
    alpha = 1 - beta
    return beta, alpha, torch.cumprod(alpha, dim=0)


def ddim_times(num_timesteps, timesteps):
    """style_conditioned_ddim_sample index list (model.py:420)."""
    return torch.linspace(num_timesteps - 1, 0, timesteps).long()


def content_times(timesteps):
    """content_style_ddim_sample index list (model.py:514)."""
    return torch.linspace(timesteps - 1, 0, timesteps).long()


# ---- time embedding (model.py:170-175, 234-246) ---------------------------------------------------
def sinusoid(t, dim=128):
    half = dim // 2
    e = math.log(10000) / (half - 1)
    f = torch.exp(torch.arange(half) * -e)
    a = t[:, None] * f[None, :]
    return torch.cat((a.sin(), a.cos()), dim=-1)


def time_mlp(sd, p, t):
    w1 = _g(sd, p + "time_mlp.1.weight")
    # the embedding is fp32 in the reference (model.py:239-246); a float64 restatement widens it afterwards
    h = F.linear(sinusoid(t).to(w1.dtype), w1, _g(sd, p + "time_mlp.1.bias"))
    h = F.gelu(h)
    return F.linear(h, _g(sd, p + "time_mlp.3.weight"), _g(sd, p + "time_mlp.3.bias"))


# ---- attention (model.py:126-160; nn.MultiheadAttention need_weights=True path) --------------------
def cross_attention(sd, p, x, s, heads=4):
    B, C, h, w = x.shape
    q_in = x.permute(2, 3, 0, 1).reshape(h * w, B, C)
    kv_in = s.permute(2, 3, 0, 1).reshape(h * w, B, C)
    W = _g(sd, p + "multihead_attn.in_proj_weight")
    b = _g(sd, p + "multihead_attn.in_proj_bias")
    q = F.linear(q_in, W[:C], b[:C])
    k = F.linear(kv_in, W[C:2 * C], b[C:2 * C])
    v = F.linear(kv_in, W[2 * C:], b[2 * C:])
    d = C // heads
    L_, S_ = q.shape[0], k.shape[0]
    q = q.reshape(L_, B * heads, d).transpose(0, 1)
    k = k.reshape(S_, B * heads, d).transpose(0, 1)
    v = v.reshape(S_, B * heads, d).transpose(0, 1)
    att = torch.softmax(torch.bmm(q * math.sqrt(1.0 / d), k.transpose(1, 2)), dim=-1)
    o = torch.bmm(att, v).transpose(0, 1).reshape(L_ * B, C)
    o = F.linear(o, _g(sd, p + "multihead_attn.out_proj.weight"), _g(sd, p + "multihead_attn.out_proj.bias"))
    return o.reshape(h, w, B, C).permute(2, 3, 0, 1)


# ---- UNet (model.py:163-231) -------------------------------------------------------------------------
def unet(sd, z, t, s5, s6, p="unet."):
    def cv(name, x, stride=1):
        return F.conv2d(x, _g(sd, p + name + ".weight"), _g(sd, p + name + ".bias"), stride=stride, padding=1)

    def ct(name, x):
        return F.conv_transpose2d(x, _g(sd, p + name + ".weight"), _g(sd, p + name + ".bias"), stride=2, padding=1,
                                  output_padding=1)

    temb = time_mlp(sd, p, t)[:, :, None, None]
    z1 = F.relu(cv("enc1", z))
    z2 = F.relu(cv("enc2", z1, 2)) + temb
    z3 = F.relu(cv("enc3", z2, 2))
    z3a = cross_attention(sd, p + "cross_attention2.", z3, s5)
    z4 = F.relu(cv("enc4", z3a, 2))
    z4a = cross_attention(sd, p + "cross_attention1.", z4, s6)
    zb = F.relu(cv("bottleneck", z4a))
    d4 = F.relu(ct("dec4", zb)) + z3
    d3 = F.relu(ct("dec3", d4)) + z2
    d2 = F.relu(ct("dec2", d3)) + z1
    return cv("dec1", d2)


# ---- VAE + style encoder (model.py:10-88) --------------------------------------------------------------
def _bn(sd, p, x, train, state=None):
    rm, rv = _g(sd, p + ".running_mean"), _g(sd, p + ".running_var")
    if train:   # running-stat updates go to `state` (a scratch dict), never into sd
        state = {} if state is None else state
        rm, rv = state.setdefault(p + ".running_mean", rm.clone()), state.setdefault(p + ".running_var", rv.clone())
    return F.batch_norm(x, rm, rv, _g(sd, p + ".weight"), _g(sd, p + ".bias"), training=train, momentum=0.1, eps=1e-5)


def encoder(sd, x, train=False, p="encoder.", state=None):
    e = p + "encoder."
    h = F.relu(_bn(sd, e + "1", F.conv2d(x, _g(sd, e + "0.weight"), _g(sd, e + "0.bias"), stride=2, padding=1),
                   train, state))
    h = F.relu(_bn(sd, e + "4", F.conv2d(h, _g(sd, e + "3.weight"), _g(sd, e + "3.bias"), stride=2, padding=1),
                   train, state))
    return _bn(sd, e + "7", F.conv2d(h, _g(sd, e + "6.weight"), _g(sd, e + "6.bias"), stride=2, padding=1), train,
               state)


def decoder(sd, z, train=False, p="decoder.", state=None):
    d = p + "decoder."

    def ct(i, x):
        return F.conv_transpose2d(x, _g(sd, d + f"{i}.weight"), _g(sd, d + f"{i}.bias"), stride=2, padding=1)

    h = F.relu(_bn(sd, d + "1", ct(0, z), train, state))
    h = F.relu(_bn(sd, d + "4", ct(3, h), train, state))
    return torch.tanh(ct(6, h))


def style_encoder(sd, x, p="style_encoder."):
    out = {}
    for i in range(1, 7):
        x = F.relu(F.conv2d(x, _g(sd, p + f"enc{i}.weight"), _g(sd, p + f"enc{i}.bias"), stride=2, padding=1))
        out[f"s{i}"] = x
    return out


# ---- diffusion (model.py:102-124, 409-465, 503-559) --------------------------------------------------
def q_sample(alpha_bar, x0, t, eps):
    ab = alpha_bar[t].view(-1, 1, 1, 1)
    return torch.sqrt(ab) * x0 + torch.sqrt(1 - ab) * eps


def predict_start(alpha_bar, zt, t, eps):
    ab = alpha_bar[t].view(-1, 1, 1, 1)
    return (zt - torch.sqrt(1 - ab) * eps) / torch.sqrt(ab)


def ddim_step(alpha_bar, x, eps, t, t_next, eta):
    ab_t = alpha_bar[t].view(-1, 1, 1, 1)
    ab_n = alpha_bar[t_next].view(-1, 1, 1, 1)
    x0 = predict_start(alpha_bar, x, t, eps)
    dxt = torch.sqrt(1 - ab_t) * eps
    dxn = torch.sqrt(1 - ab_n) * eps
    return torch.sqrt(ab_n) * x0 + dxn + eta * (dxn - dxt), x0


def reverse_loop(sd, alpha_bar, x, s5, s6, times, eta, p="unet.", logs=None):
    B = x.shape[0]
    for i in range(len(times) - 1):
        t = times[i].repeat(B)
        eps = unet(sd, x, t, s5, s6, p)
        x, x0 = ddim_step(alpha_bar, x, eps, t, times[i + 1].repeat(B), eta)
        if logs is not None:
            logs["timesteps"].append(int(t[0]))
            logs["pred_x0"].append(x0)
            logs["noise_pred"].append(eps)
    return x


def ldm_forward(sd, x, style, t, noise, alpha_bar, train_decoder=False, train_encoder=False, state=None):
    """LDM.forward (model.py:355-379) with injected noise."""
    z0 = encoder(sd, x, train_encoder, state=state)
    emb = style_encoder(sd, style)
    zt = q_sample(alpha_bar, z0, t, noise)
    eps = unet(sd, zt, t, emb["s5"], emb["s6"])
    z0p = predict_start(alpha_bar, zt, t, eps)
    rec = (decoder(sd, z0p, train_decoder, state=state) + 1) / 2
    return {"z_t": zt, "noise": noise, "noise_pred": eps, "z_0": z0, "reconstructed": rec}


def kl_loss(z):
    return torch.mean(0.5 * (z.pow(2) - 1 - torch.log(z.pow(2) + 1e-8)))


VGGISH_CFG = (64, "M", 128, "M", 256, 256, "M", 512, 512, "M")


def vggish_feature_loss(sd, predicted, target, cfg=VGGISH_CFG):
    """VGGishFeatureLoss.forward (reference loss.py:64-101) over a VGGish-shaped stack whose state dict `sd`
    uses the nn.Sequential keys '<index>.weight' / '<index>.bias': every 3x3 conv (padding 1) is followed by
    a ReLU whose output is a tap, 'M' is max_pool2d(2, 2); per tap the per-sample unbiased std over dims
    1..3 normalises both sides (+1e-8), the tap loss is their MSE, the result the mean over taps."""
    xp, xt = predicted, target
    taps, i = [], 0
    for v in cfg:
        if v == "M":
            xp, xt = F.max_pool2d(xp, 2, 2), F.max_pool2d(xt, 2, 2)
            i += 1
            continue
        w, b = sd[f"{i}.weight"], sd[f"{i}.bias"]
        xp = torch.relu(F.conv2d(xp, w, b, padding=1))
        xt = torch.relu(F.conv2d(xt, w, b, padding=1))
        taps.append((xp, xt))
        i += 2
    total = 0
    for p_, t_ in taps:
        p_ = p_ / (torch.std(p_, dim=[1, 2, 3], keepdim=True) + 1e-8)
        t_ = t_ / (torch.std(t_, dim=[1, 2, 3], keepdim=True) + 1e-8)
        total = total + F.mse_loss(p_, t_)
    return total / len(taps)



# ---- LPIPS-AlexNet (loss.py:6-21: lpips==0.1.4 LPIPS(net='alex'), not vendored, not installed) ----------------
# Restated from lpips 0.1.4's published forward (net='alex', lpips=True, spatial=False, version '0.1'); PARITY
# UNPINNED: no output of the package exists here to pin it to.  sd uses lpips.LPIPS state_dict keys.
LPIPS_SHIFT = (-0.030, -0.088, -0.188)
LPIPS_SCALE = (0.458, 0.448, 0.450)
_ALEX = (("net.slice1.0", 4, 2, False), ("net.slice2.3", 1, 2, True), ("net.slice3.6", 1, 1, True),
         ("net.slice4.8", 1, 1, False), ("net.slice5.10", 1, 1, False))


def lpips_alex(sd, in0, in1):
    """LPIPS.forward(in0, in1) -> [B,1,1,1] (inputs already in [-1, 1], as perceptual_loss_old passes them)."""
    dt = in0.dtype
    shift = torch.tensor(LPIPS_SHIFT, dtype=dt).view(1, 3, 1, 1)
    scale = torch.tensor(LPIPS_SCALE, dtype=dt).view(1, 3, 1, 1)

    def feats(x):
        h = (x - shift) / scale                       # ScalingLayer (a 1-channel input broadcasts)
        out = []
        for name, stride, pad, pool in _ALEX:
            if pool:
                h = F.max_pool2d(h, kernel_size=3, stride=2)
            h = F.relu(F.conv2d(h, _g(sd, name + ".weight"), _g(sd, name + ".bias"), stride=stride, padding=pad))
            out.append(h)
        return out

    def normalize(f, eps=1e-10):
        return f / (torch.sqrt(torch.sum(f ** 2, dim=1, keepdim=True)) + eps)

    val = None
    for i, (a, b) in enumerate(zip(feats(in0), feats(in1))):
        d = (normalize(a) - normalize(b)) ** 2
        r = F.conv2d(d, _g(sd, f"lin{i}.model.1.weight")).mean([2, 3], keepdim=True)
        val = r if val is None else val + r
    return val
