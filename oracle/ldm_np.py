"""ORACLE — test infrastructure only.  Independent float64 numpy restatement of the reference's forward
hot path (no torch): DDPM tables bit-exact to torch's fp32 algorithms, and the UNet / VAE / style
encoder / cross-attention / DDIM update in float64 — a higher-precision reference for small cases.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.  Pinned against
tests/golden/ref_goldens.npz (made by importing the reference) in tests/test_oracle_golden.py.
"""
import math

import numpy as np
from scipy.special import erf


# ---- DDPM tables, bit-exact to the reference's fp32 torch calls ------------------------------------
def linspace_f32(start, end, n):
    """torch.linspace(start, end, n) for float32 (aten RangeFactoriesKernel: step = (end-start)/(n-1)
    in fp32; start + step*i for i < n/2, end - step*(n-1-i) above, each with ONE rounding)."""
    start, end = np.float32(start), np.float32(end)
    if n == 1:
        return np.array([start], dtype=np.float32)
    step = np.float32((end - start) / np.float32(n - 1))
    i = np.arange(n)
    lo = (np.float64(start) + np.float64(step) * i).astype(np.float32)
    hi = (np.float64(end) - np.float64(step) * (n - 1 - i)).astype(np.float32)
    return np.where(i < n // 2, lo, hi).astype(np.float32)


def schedule(T):
    """beta, alpha, alpha_bar of ForwardDiffusion (model.py:96-100); cumprod accumulates in double
    like aten's CPU cumprod (acc_type<float> = double)."""
    beta = linspace_f32(0.0001, 0.02, T)
    alpha = (np.float32(1) - beta).astype(np.float32)
    alpha_bar = np.cumprod(alpha.astype(np.float64)).astype(np.float32)
    return beta, alpha, alpha_bar


def ddim_times(num_timesteps, timesteps):
    """torch.linspace(T-1, 0, n).long() (model.py:420): truncation toward zero."""
    return linspace_f32(num_timesteps - 1, 0, timesteps).astype(np.int64)


def content_times(timesteps):
    return linspace_f32(timesteps - 1, 0, timesteps).astype(np.int64)


# ---- layers (float64) --------------------------------------------------------------------------------
def _f(sd, k):
    return np.asarray(sd[k], dtype=np.float64)


def conv2d(x, w, b, stride, pad):
    B, C, H, W = x.shape
    O, _, kh, kw = w.shape
    Ho = (H + 2 * pad - kh) // stride + 1
    Wo = (W + 2 * pad - kw) // stride + 1
    xp = np.pad(x, ((0, 0), (0, 0), (pad, pad), (pad, pad)))
    out = np.zeros((B, O, Ho, Wo))
    for i in range(kh):
        for j in range(kw):
            patch = xp[:, :, i:i + stride * Ho:stride, j:j + stride * Wo:stride]
            out += np.einsum("bchw,oc->bohw", patch, w[:, :, i, j], optimize=True)
    return out + b[None, :, None, None]


def conv_transpose2d(x, w, b, stride, pad, out_pad):
    """Scatter form: out_full[ih*s+i, iw*s+j] += x[ih,iw] w[:, :, i, j], then crop by `pad`."""
    B, C, H, W = x.shape
    _, O, kh, kw = w.shape
    Hf, Wf = (H - 1) * stride + kh, (W - 1) * stride + kw
    full = np.zeros((B, O, Hf + out_pad, Wf + out_pad))
    for i in range(kh):
        for j in range(kw):
            full[:, :, i:i + stride * H:stride, j:j + stride * W:stride] += np.einsum("bchw,co->bohw", x, w[:, :, i, j],
                                                                                      optimize=True)
    Ho = (H - 1) * stride - 2 * pad + kh + out_pad
    Wo = (W - 1) * stride - 2 * pad + kw + out_pad
    return full[:, :, pad:pad + Ho, pad:pad + Wo] + b[None, :, None, None]


def relu(x):
    return np.maximum(x, 0.0)


def gelu(x):
    return 0.5 * x * (1.0 + erf(x / math.sqrt(2.0)))


def bn_eval(sd, p, x):
    m, v, g, b = _f(sd, p + ".running_mean"), _f(sd, p + ".running_var"), _f(sd, p + ".weight"), _f(sd, p + ".bias")
    return (x - m[None, :, None, None]) / np.sqrt(v[None, :, None, None] + 1e-5) * g[None, :, None, None] + \
        b[None, :, None, None]


def bn_train(sd, p, x):
    g, b = _f(sd, p + ".weight"), _f(sd, p + ".bias")
    m = x.mean(axis=(0, 2, 3))
    v = x.var(axis=(0, 2, 3))
    return (x - m[None, :, None, None]) / np.sqrt(v[None, :, None, None] + 1e-5) * g[None, :, None, None] + \
        b[None, :, None, None]


def sinusoid(t, dim=128):
    half = dim // 2
    f = np.exp(np.arange(half) * -(math.log(10000) / (half - 1)))
    a = np.asarray(t, dtype=np.float64)[:, None] * f[None, :]
    return np.concatenate([np.sin(a), np.cos(a)], axis=-1)


def time_mlp(sd, p, t):
    h = sinusoid(t) @ _f(sd, p + "time_mlp.1.weight").T + _f(sd, p + "time_mlp.1.bias")
    h = gelu(h)
    return h @ _f(sd, p + "time_mlp.3.weight").T + _f(sd, p + "time_mlp.3.bias")


def cross_attention(sd, p, x, s, heads=4):
    """nn.MultiheadAttention(E, heads)(q, kv, kv) over H*W tokens, no residual (model.py:135-160)."""
    B, C, h, w = x.shape
    q_in = x.reshape(B, C, h * w).transpose(0, 2, 1)         # [B, L, C]
    kv_in = s.reshape(B, C, -1).transpose(0, 2, 1)
    W = _f(sd, p + "multihead_attn.in_proj_weight")
    bb = _f(sd, p + "multihead_attn.in_proj_bias")
    q = q_in @ W[:C].T + bb[:C]
    k = kv_in @ W[C:2 * C].T + bb[C:2 * C]
    v = kv_in @ W[2 * C:].T + bb[2 * C:]
    d = C // heads
    out = np.empty_like(q)
    for hd in range(heads):
        sl = slice(hd * d, (hd + 1) * d)
        sc = np.einsum("bld,bsd->bls", q[:, :, sl] / math.sqrt(d), k[:, :, sl])
        sc = np.exp(sc - sc.max(axis=-1, keepdims=True))
        sc /= sc.sum(axis=-1, keepdims=True)
        out[:, :, sl] = np.einsum("bls,bsd->bld", sc, v[:, :, sl])
    o = out @ _f(sd, p + "multihead_attn.out_proj.weight").T + _f(sd, p + "multihead_attn.out_proj.bias")
    return o.transpose(0, 2, 1).reshape(B, C, h, w)


def unet(sd, z, t, s5, s6, p="unet."):
    def cv(n, x, s=1):
        return conv2d(x, _f(sd, p + n + ".weight"), _f(sd, p + n + ".bias"), s, 1)

    def ct(n, x):
        return conv_transpose2d(x, _f(sd, p + n + ".weight"), _f(sd, p + n + ".bias"), 2, 1, 1)

    z = np.asarray(z, dtype=np.float64)
    temb = time_mlp(sd, p, t)[:, :, None, None]
    z1 = relu(cv("enc1", z))
    z2 = relu(cv("enc2", z1, 2)) + temb
    z3 = relu(cv("enc3", z2, 2))
    z3a = cross_attention(sd, p + "cross_attention2.", z3, np.asarray(s5, np.float64))
    z4 = relu(cv("enc4", z3a, 2))
    z4a = cross_attention(sd, p + "cross_attention1.", z4, np.asarray(s6, np.float64))
    zb = relu(cv("bottleneck", z4a))
    d4 = relu(ct("dec4", zb)) + z3
    d3 = relu(ct("dec3", d4)) + z2
    d2 = relu(ct("dec2", d3)) + z1
    return cv("dec1", d2)


def encoder(sd, x, train=False, p="encoder."):
    e = p + "encoder."
    bn = bn_train if train else bn_eval
    h = np.asarray(x, dtype=np.float64)
    h = relu(bn(sd, e + "1", conv2d(h, _f(sd, e + "0.weight"), _f(sd, e + "0.bias"), 2, 1)))
    h = relu(bn(sd, e + "4", conv2d(h, _f(sd, e + "3.weight"), _f(sd, e + "3.bias"), 2, 1)))
    return bn(sd, e + "7", conv2d(h, _f(sd, e + "6.weight"), _f(sd, e + "6.bias"), 2, 1))


def decoder(sd, z, train=False, p="decoder."):
    d = p + "decoder."
    bn = bn_train if train else bn_eval
    h = np.asarray(z, dtype=np.float64)
    h = relu(bn(sd, d + "1", conv_transpose2d(h, _f(sd, d + "0.weight"), _f(sd, d + "0.bias"), 2, 1, 0)))
    h = relu(bn(sd, d + "4", conv_transpose2d(h, _f(sd, d + "3.weight"), _f(sd, d + "3.bias"), 2, 1, 0)))
    return np.tanh(conv_transpose2d(h, _f(sd, d + "6.weight"), _f(sd, d + "6.bias"), 2, 1, 0))


def style_encoder(sd, x, p="style_encoder."):
    out = {}
    h = np.asarray(x, dtype=np.float64)
    for i in range(1, 7):
        h = relu(conv2d(h, _f(sd, p + f"enc{i}.weight"), _f(sd, p + f"enc{i}.bias"), 2, 1))
        out[f"s{i}"] = h
    return out


def ddim_step(alpha_bar, x, eps, t, t_next, eta):
    """model.py:442-458 (float64)."""
    ab_t, ab_n = np.float64(alpha_bar[t]), np.float64(alpha_bar[t_next])
    x0 = (x - math.sqrt(1 - ab_t) * eps) / math.sqrt(ab_t)
    dxt = math.sqrt(1 - ab_t) * eps
    dxn = math.sqrt(1 - ab_n) * eps
    return math.sqrt(ab_n) * x0 + dxn + eta * (dxn - dxt), x0
