"""Drop-in for the reference's models/model.py: same classes, constructor signatures and defaults,
parameter names and shapes (state_dicts interchange), forward semantics and return values — with every
tensor operation of the path executed by libldm_amd.so (hand-written HIP for gfx950).

Deliberate, documented deviations:
  * style_conditioned_ddim_sample / content_style_ddim_sample log timesteps as int(t[0]) instead of
    t.item(), which raises for batch > 1 in the reference (model.py:461, :555).  Numerics unchanged.
  * ForwardDiffusion.forward and LDM.forward accept an optional `noise=` to inject epsilon (parity
    tests); without it epsilon is drawn on the device exactly like torch.randn_like.
  * SpectrogramDecoder.forward(z, rescale=True) fuses the reference's `(decoder(z) + 1) / 2`
    (model.py:371, :405, :498) into the final Tanh epilogue with the same fp32 op order.
  * The sampling loops are inference-only: they build no autograd graph.
No tensor op falls back to the CPU: a CPU tensor on the hot path raises.
"""
import math
import weakref
from typing import Dict, List, Optional, Tuple  # noqa: F401  (API-compat with the reference imports)

import torch
import torch.nn as nn

try:
    from .config import config
except ImportError:
    from config import config

try:
    from . import _pathfix  # noqa: F401
except ImportError:
    import _pathfix  # noqa: F401

try:
    from .loss import VGGishFeatureLoss
except ImportError:
    from loss import VGGishFeatureLoss

from ldm_amd import functional as HF
from ldm_amd import graphs as hgraphs
from ldm_amd import nn as hnn
from ldm_amd import ops
from ldm_amd.engine import UNetEngine


# ------------------------------------------------------------------------------------------------
# fused helpers
# ------------------------------------------------------------------------------------------------
def _bn_is_eval(bn):
    return not (bn.training or not bn.track_running_stats)


def _conv_bn_act(conv, bn, act, x, transposed=False):
    """conv -> BatchNorm2d -> activation, reference op order.  Eval-mode BN (with frozen affine) is folded
    into the conv epilogue; train-mode BN runs the batch-statistics kernel after the conv."""
    kw = dict(stride=conv.stride[0], padding=conv.padding[0], transposed=transposed,
              output_padding=conv.output_padding[0] if transposed else 0)
    if bn is not None and _bn_is_eval(bn) and not HF._needs_grad(bn.weight, bn.bias):
        return HF.conv(x, conv.weight, conv.bias, act=act,
                       bn_eval=(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps), **kw)
    if bn is None:
        return HF.conv(x, conv.weight, conv.bias, act=act, **kw)
    y = HF.conv(x, conv.weight, conv.bias, act="none", **kw)
    return HF.batchnorm(y, bn, act)


# ------------------------------------------------------------------------------------------------
# VAE
# ------------------------------------------------------------------------------------------------
class SpectrogramEncoder(nn.Module):
    """[B,1,H,W] -> [B,latent_dim,H/8,W/8]: 3 x (conv3x3 s2 + BN) with ReLU after the first two
    (reference model.py:10-28)."""

    def __init__(self, latent_dim=4):
        super(SpectrogramEncoder, self).__init__()
        self.encoder = nn.Sequential(
            hnn.Conv2d(1, 64, kernel_size=3, stride=2, padding=1),
            hnn.BatchNorm2d(64),
            hnn.ReLU(),
            hnn.Conv2d(64, 128, kernel_size=3, stride=2, padding=1),
            hnn.BatchNorm2d(128),
            hnn.ReLU(),
            hnn.Conv2d(128, latent_dim, kernel_size=3, stride=2, padding=1),
            hnn.BatchNorm2d(latent_dim),
        )

    def forward(self, x):
        e = self.encoder
        h = _conv_bn_act(e[0], e[1], "relu", x)
        h = _conv_bn_act(e[3], e[4], "relu", h)
        return _conv_bn_act(e[6], e[7], "none", h)


class SpectrogramDecoder(nn.Module):
    """[B,latent_dim,h,w] -> [B,1,8h,8w]: 3 x convT k4 s2 p1 (+BN+ReLU, last Tanh) (reference
    model.py:31-49).  rescale=True returns (tanh(.)+1)/2 in the same fused epilogue."""

    def __init__(self, latent_dim=4):
        super(SpectrogramDecoder, self).__init__()
        self.decoder = nn.Sequential(
            hnn.ConvTranspose2d(latent_dim, 128, kernel_size=4, stride=2, padding=1),
            hnn.BatchNorm2d(128),
            hnn.ReLU(),
            hnn.ConvTranspose2d(128, 64, kernel_size=4, stride=2, padding=1),
            hnn.BatchNorm2d(64),
            hnn.ReLU(),
            hnn.ConvTranspose2d(64, 1, kernel_size=4, stride=2, padding=1),
            hnn.Tanh(),
        )

    def forward(self, z, rescale=False):
        d = self.decoder
        h = _conv_bn_act(d[0], d[1], "relu", z, transposed=True)
        h = _conv_bn_act(d[3], d[4], "relu", h, transposed=True)
        return _conv_bn_act(d[6], None, "tanh_half" if rescale else "tanh", h, transposed=True)


class StyleEncoder(nn.Module):
    """6 x (conv3x3 s2 + ReLU) -> {'s1'..'s6'} (reference model.py:51-88)."""

    def __init__(self, in_channels=1, num_filters=64):
        super().__init__()
        nf = num_filters
        self.enc1 = hnn.Conv2d(in_channels, nf, kernel_size=3, stride=2, padding=1)
        self.enc2 = hnn.Conv2d(nf, nf * 2, kernel_size=3, stride=2, padding=1)
        self.enc3 = hnn.Conv2d(nf * 2, nf * 4, kernel_size=3, stride=2, padding=1)
        self.enc4 = hnn.Conv2d(nf * 4, nf * 4, kernel_size=3, stride=2, padding=1)
        self.enc5 = hnn.Conv2d(nf * 4, nf * 4, kernel_size=3, stride=2, padding=1)
        self.enc6 = hnn.Conv2d(nf * 4, nf * 8, kernel_size=3, stride=2, padding=1)

    def forward(self, style_spectrogram):
        out = {}
        h = style_spectrogram
        for i in range(1, 7):
            h = getattr(self, f"enc{i}")(h, act="relu")
            out[f"s{i}"] = h
        return out


# ------------------------------------------------------------------------------------------------
# DDPM schedule
# ------------------------------------------------------------------------------------------------
class ForwardDiffusion(nn.Module):
    """beta = linspace(1e-4, 0.02, T); alpha = 1 - beta; alpha_bar = cumprod(alpha) (reference
    model.py:90-124).  The tables are host constants computed with the reference's own torch calls;
    q_sample / predict_start_from_noise run on the device with per-sample gathers of {sqrt(ab),
    sqrt(1-ab)}."""

    def __init__(self, num_timesteps=config["forward_diffusion_num_timesteps"]):
        super().__init__()
        self.num_timesteps = num_timesteps
        beta_start, beta_end = 0.0001, 0.02
        self.register_buffer("beta_t", torch.linspace(beta_start, beta_end, num_timesteps))
        self.register_buffer("alpha_t", 1 - self.beta_t)
        self.register_buffer("alpha_bar_t", torch.cumprod(self.alpha_t, dim=0))

    def _check_t(self, t):
        if not t.is_cuda:
            T = self.alpha_bar_t.shape[0]
            bad = (t >= T) | (t < -T)
            if bool(bad.any()):
                raise IndexError(f"index {int(t[bad][0])} is out of bounds for dimension 0 with size {T}")
            t = torch.where(t < 0, t + T, t)
        return t

    def coef_table(self, device):
        return ops.alpha_bar_coef_table(self.alpha_bar_t, device)

    def forward(self, x_0, t, noise=None):
        device = x_0.device
        t = self._check_t(t).to(device)
        self.alpha_bar_t = self.alpha_bar_t.to(device)   # reference side effect (model.py:106)
        eps = torch.randn_like(x_0, device=device) if noise is None else noise.to(device)
        z_t = HF.q_sample(x_0, eps, self.coef_table(device), t)
        return z_t, eps

    def predict_start_from_noise(self, z_t, t, noise_pred):
        device = z_t.device
        t = self._check_t(t).to(device)
        self.alpha_bar_t = self.alpha_bar_t.to(device)   # reference side effect (model.py:121)
        return HF.predict_start(z_t, noise_pred, self.coef_table(device), t)

    def reverse_coefs(self, times):
        """[n,4] {sqrt(ab_t), sqrt(1-ab_t), sqrt(ab_next), sqrt(1-ab_next)} for consecutive `times`."""
        ab = self.alpha_bar_t.detach().to("cpu", torch.float32)
        T = ab.shape[0]
        if times.numel() and (int(times.max()) >= T or int(times.min()) < -T):
            bad = int(times.max()) if int(times.max()) >= T else int(times.min())
            raise IndexError(f"index {bad} is out of bounds for dimension 0 with size {T}")
        a_t, a_n = ab[times[:-1]], ab[times[1:]]
        return torch.stack([torch.sqrt(a_t), torch.sqrt(1 - a_t), torch.sqrt(a_n), torch.sqrt(1 - a_n)], 1).contiguous()


# ------------------------------------------------------------------------------------------------
# UNet
# ------------------------------------------------------------------------------------------------
class CrossAttention(nn.Module):
    """nn.MultiheadAttention(E, heads) over the H*W tokens of two NCHW maps, no residual (reference
    model.py:126-160).  Runs on the channel-major maps directly: the reference's permute/reshape pairs
    are folded into the projection GEMMs' addressing."""

    def __init__(self, embed_dim, num_heads=4):
        super().__init__()
        self.multihead_attn = hnn.MultiheadAttention(embed_dim, num_heads)
        self.embed_dim = embed_dim

    def forward(self, unet_features, style_embedding):
        B, c, h, w = unet_features.shape
        if style_embedding.shape[0] != B or style_embedding.shape[1] != c or \
                style_embedding.shape[2] * style_embedding.shape[3] != h * w:
            raise RuntimeError(f"CrossAttention: style map {tuple(style_embedding.shape)} cannot be viewed as "
                               f"[{h * w}, {B}, {c}] (reference model.py:150)")
        kv = style_embedding.reshape(B, c, h, w) if tuple(style_embedding.shape[2:]) != (h, w) else style_embedding
        return hnn.attention_nchw(self.multihead_attn, unet_features, kv)


class SinusoidalPositionEmbeddings(nn.Module):
    """[sin(t f_i), cos(t f_i)], f_i = exp(-i ln(1e4)/(dim/2-1)) (reference model.py:234-246)."""

    def __init__(self, dim):
        super().__init__()
        self.dim = dim

    def forward(self, time):
        if not time.is_cuda:
            raise RuntimeError("SinusoidalPositionEmbeddings: time must be a GPU tensor (no CPU fallback)")
        return ops.sinusoid_embed(time, self.dim, time.device)


class _TimeMLP(nn.Sequential):
    """nn.Sequential(Sinusoid, Linear, GELU, Linear) whose inference forward is one fused kernel."""

    def forward(self, t):
        lin1, lin2 = self[1], self[3]
        if HF._needs_grad(lin1.weight, lin1.bias, lin2.weight, lin2.bias):
            emb = ops.sinusoid_embed(t, self[0].dim, lin1.weight.device)
            h = HF.activation(HF.linear(emb, lin1.weight, lin1.bias), "gelu")
            return HF.linear(h, lin2.weight, lin2.bias)
        return ops.time_mlp(t, lin1.weight, lin1.bias, lin2.weight, lin2.bias)


_ENGINES = weakref.WeakKeyDictionary()


def engine_for(unet):
    eng = _ENGINES.get(unet)
    if eng is None:
        eng = UNetEngine(unet)
        _ENGINES[unet] = eng
    return eng


class UNet(nn.Module):
    """Style-conditioned denoiser (reference model.py:163-231): conv encoder, two cross-attentions,
    bottleneck, transposed-conv decoder with additive skips, sinusoid time MLP added after enc2."""

    def __init__(self, in_channels=1, out_channels=1, num_filters=64):
        super(UNet, self).__init__()
        time_emb_dim = 128
        self.num_filters = num_filters
        self.time_mlp = _TimeMLP(
            SinusoidalPositionEmbeddings(time_emb_dim),
            hnn.Linear(time_emb_dim, time_emb_dim),
            hnn.GELU(),
            hnn.Linear(time_emb_dim, time_emb_dim),
        )
        nf = num_filters
        self.enc1 = hnn.Conv2d(in_channels, nf, kernel_size=3, stride=1, padding=1)
        self.enc2 = hnn.Conv2d(nf, nf * 2, kernel_size=3, stride=2, padding=1)
        self.enc3 = hnn.Conv2d(nf * 2, nf * 4, kernel_size=3, stride=2, padding=1)
        self.enc4 = hnn.Conv2d(nf * 4, nf * 8, kernel_size=3, stride=2, padding=1)
        self.cross_attention1 = CrossAttention(embed_dim=512, num_heads=4)
        self.cross_attention2 = CrossAttention(embed_dim=256, num_heads=4)
        self.bottleneck = hnn.Conv2d(nf * 8, nf * 8, kernel_size=3, stride=1, padding=1)
        self.dec4 = hnn.ConvTranspose2d(nf * 8, nf * 4, kernel_size=3, stride=2, padding=1, output_padding=1)
        self.dec3 = hnn.ConvTranspose2d(nf * 4, nf * 2, kernel_size=3, stride=2, padding=1, output_padding=1)
        self.dec2 = hnn.ConvTranspose2d(nf * 2, nf, kernel_size=3, stride=2, padding=1, output_padding=1)
        self.dec1 = hnn.Conv2d(nf, out_channels, kernel_size=3, stride=1, padding=1)

    def _layerwise(self, z, t, s5, s6):
        """Same kernels and plans as the fused engine, one autograd node per layer (training)."""
        temb = self.time_mlp(t)
        z1 = self.enc1(z, act="relu")
        z2 = self.enc2(z1, act="relu", bcast=temb)            # relu(enc2(z1)) + t_emb   (model.py:206)
        z3 = self.enc3(z2, act="relu")
        z3a = self.cross_attention2(z3, s5)
        z4 = self.enc4(z3a, act="relu")
        z4a = self.cross_attention1(z4, s6)
        zb = self.bottleneck(z4a, act="relu")
        d4 = self.dec4(zb, act="relu", skip=z3)                 # relu(dec4(.)) + z3_original  (model.py:220-221)
        d3 = self.dec3(d4, act="relu", skip=z2)
        d2 = self.dec2(d3, act="relu", skip=z1)
        return self.dec1(d2)

    def forward(self, z, t, style_embedding: dict = None):
        s5, s6 = style_embedding["s5"], style_embedding["s6"]
        if HF._needs_grad(z, s5, s6, *self.parameters()) or not UNetEngine.supports(z.shape[1]):
            return self._layerwise(z, t, s5, s6)
        return engine_for(self).forward(z, t, s5, s6)


# ------------------------------------------------------------------------------------------------
# LDM
# ------------------------------------------------------------------------------------------------
class LDM(nn.Module):
    """VAE + style encoder + DDPM schedule + UNet (reference model.py:249-559)."""

    def __init__(self, latent_dim, pretrained_path: str = "models/pretrained/", pretraind_filename: str = "ldm.pth",
                 num_timesteps=config["forward_diffusion_num_timesteps"], load_full_model=False):
        super(LDM, self).__init__()
        self.encoder = SpectrogramEncoder(latent_dim=latent_dim)
        self.decoder = SpectrogramDecoder(latent_dim=latent_dim)
        self.unet = UNet(in_channels=latent_dim, out_channels=latent_dim, num_filters=64)
        self.noise_scheduler = ForwardDiffusion(num_timesteps=num_timesteps)
        self.style_encoder = StyleEncoder(in_channels=1, num_filters=64)
        self.num_timesteps = num_timesteps
        self.feature_loss_net = VGGishFeatureLoss()

        if pretrained_path:
            if load_full_model:
                try:
                    sd = torch.load(pretrained_path + pretraind_filename, map_location="cpu", weights_only=True)
                    for prefix, mod in (("encoder.", self.encoder), ("decoder.", self.decoder), ("unet.", self.unet),
                                        ("style_encoder.", self.style_encoder),
                                        ("noise_scheduler.", self.noise_scheduler)):
                        mod.load_state_dict({k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)})
                    print(f"Loaded full pretrained LDM components from {pretrained_path + 'ldm.pth'}")
                    self.encoder.eval()
                    self.decoder.train()
                    self.unet.train()
                    self.style_encoder.train()
                    for p in self.encoder.parameters():
                        p.requires_grad = False
                    for p in self.decoder.parameters():
                        p.requires_grad = True
                    return
                except (FileNotFoundError, RuntimeError) as e:
                    print(f"Could not load full LDM model: {e}")
                    print("Falling back to loading just encoder/decoder weights")
            self.encoder.load_state_dict(torch.load(pretrained_path + "encoder.pth", map_location="cpu",
                                                    weights_only=True))
            self.decoder.load_state_dict(torch.load(pretrained_path + "decoder.pth", map_location="cpu",
                                                    weights_only=True))
            print("Loaded pretrained weights from", pretrained_path)
            for p in self.encoder.parameters():
                p.requires_grad = False
            for p in self.decoder.parameters():
                p.requires_grad = True
            self.encoder.eval()
            self.decoder.train()
            self.style_encoder.train()

        # The reference rebuilds these three after loading (model.py:350-353); mirrored so that the
        # parameter-init RNG draws match it.
        self.unet = UNet(in_channels=latent_dim, out_channels=latent_dim, num_filters=64)
        self.noise_scheduler = ForwardDiffusion(num_timesteps=num_timesteps)
        self.style_encoder = StyleEncoder(in_channels=1, num_filters=64)
        self.num_timesteps = num_timesteps

    # -------------------------------------------------------------------------------------------
    def forward(self, x, style, t, noise=None):
        x = x.float()
        style = style.float()
        # the style encoder depends on nothing the VAE encoder / scheduler compute: on a side stream it overlaps
        # them (and, through the autograd engine's stream semantics, its backward overlaps theirs)
        with hgraphs.branch(style.device, "style_encoder") as side:
            style_embedding = self.style_encoder(style)
        z_0 = self.encoder(x)
        z_t, noise = self.noise_scheduler(z_0, t, noise=noise)
        hgraphs.join(side, style.device)
        noise_pred = self.unet(z_t, t, style_embedding)
        z_0_pred = self.noise_scheduler.predict_start_from_noise(z_t, t, noise_pred)
        reconstructed = self.decoder(z_0_pred, rescale=True)       # (decoder(.) + 1) / 2  (model.py:369-371)
        return {
            "z_t": z_t,
            "noise": noise,
            "noise_pred": noise_pred,
            "z_0": z_0,
            "reconstructed": reconstructed,
        }

    # -------------------------------------------------------------------------------------------
    def _reverse(self, z_t, style_embedding, times, eta):
        """The shared body of the two samplers: len(times)-1 UNet + update steps in one C call."""
        n = int(times.numel()) - 1
        logs = {"timesteps": [], "pred_x0": [], "noise_pred": []}
        if n <= 0:
            return z_t, logs
        coefs = self.noise_scheduler.reverse_coefs(times)
        dev = z_t.device
        x = ops.f32c(z_t).clone()
        B = x.shape[0]
        t_table = times[:-1].view(n, 1).expand(n, B).contiguous().to(dev)
        x0_logs = torch.empty((n,) + tuple(x.shape), device=dev, dtype=torch.float32)
        eps_logs = torch.empty_like(x0_logs)
        s5 = ops.f32c(style_embedding["s5"])
        s6 = ops.f32c(style_embedding["s6"])
        coefs = coefs.to(dev)
        with torch.no_grad():
            if UNetEngine.supports(x.shape[1]):
                engine_for(self.unet).ddim_loop(x, s5, s6, t_table, coefs, float(eta), x0_logs, eps_logs)
            else:   # latent widths the fused engine does not take: per-layer UNet + the DDIM update kernel
                emb = {"s5": s5, "s6": s6}
                for i in range(n):
                    eps = self.unet(x, t_table[i], emb)
                    ops.ddim_step_(x, eps, coefs[i].contiguous(), float(eta), x0_logs[i], eps_logs[i])
        logs["timesteps"] = [int(v) for v in times[:-1]]
        logs["pred_x0"] = list(x0_logs.unbind(0))
        logs["noise_pred"] = list(eps_logs.unbind(0))
        return x, logs

    def style_ddim_sample_wrapper(self, z_shape, style_spec, timesteps=100, eta=0.0):
        z_t = torch.randn(z_shape).to(style_spec.device)            # CPU generator (model.py:394)
        style_embedding = self.style_encoder(style_spec)
        sampled, _ = self.style_conditioned_ddim_sample(z_t, style_embedding, timesteps, eta)
        return self.decoder(sampled, rescale=True)

    def style_conditioned_ddim_sample(self, z_t, style_embedding, timesteps=100, eta=0.0):
        times = torch.linspace(self.num_timesteps - 1, 0, timesteps).long()    # (model.py:420)
        return self._reverse(z_t, style_embedding, times, eta)

    def content_style_transfer_wrapper(self, content_spec, style_spec, num_timesteps=250, eta=0.0, noise=None):
        """Encode content, q_sample it at T'-1, run the T'-step content/style loop, decode (reference
        model.py:468-501).  `noise` (optional, [B, latent, H/8, W/8]) injects the q_sample epsilon that
        the reference draws with randn_like (parity tests); by default it is drawn on the device."""
        content_spec = content_spec.float()
        style_spec = style_spec.float()
        z_0 = self.encoder(content_spec)
        t = torch.full((content_spec.shape[0],), num_timesteps - 1, dtype=torch.long)
        self.noise_scheduler._check_t(t)                                        # IndexError like model.py:107
        z_t, noise = self.noise_scheduler(z_0, t.to(content_spec.device), noise=noise)
        style_embedding = self.style_encoder(style_spec)
        sampled, _ = self.content_style_ddim_sample(z_t, style_embedding, num_timesteps, eta)
        decoded = self.decoder(sampled, rescale=True)
        z_t_decoded = self.decoder(z_t)
        return decoded, z_t_decoded

    def content_style_ddim_sample(self, z_t, style_embedding, timesteps=250, eta=0.0):
        times = torch.linspace(timesteps - 1, 0, timesteps).long()              # (model.py:514)
        return self._reverse(z_t, style_embedding, times, eta)
