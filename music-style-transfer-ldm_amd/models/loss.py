"""Losses of the LDM path — drop-in for the reference's models/loss.py, computed on libldm_amd.

In scope and parity-pinned: diffusion_loss, the MSE term of
compression_loss, kl_regularization_loss.  Out of scope offline: the
LPIPS-AlexNet perceptual term and the VGGish feature loss — their weights are remote downloads in the
reference (loss.py:10, :56).  Both are pluggable here:

  * set_perceptual_backend(fn)   fn(original, reconstructed) -> scalar tensor (e.g. an LPIPS model
                                 loaded from local weights).  Unset: the term is 0 (warned once).
  * VGGishFeatureLoss(features)  takes a VGGish `features` nn.Sequential (vggish_features() with
                                 local weights) and computes the loss on the HIP kernels (conv +
                                 fused ReLU taps, ldm_maxpool2x2, one-pass std-normalised MSE);
                                 without one the style term is a zero constant.  In the reference it
                                 is computed under torch.no_grad() (loss.py:78), so it never changes
                                 an update — only the reported loss value.
"""
import warnings

import torch
import torch.nn as nn

try:
    from .config import config
except ImportError:  # reference-style flat import (models/ on sys.path)
    from config import config

try:
    from . import _pathfix  # noqa: F401
except ImportError:
    import _pathfix  # noqa: F401

from ldm_amd import functional as HF

_PERCEPTUAL_BACKEND = None
_WARNED = set()


def _const_zero(device):
    """The 0-d zero an absent offline term returns: a new tensor on every call, as the reference's
    torch.zeros, so a caller's in-place update of it reaches no later call; it is marked so that the sums
    below skip adding it (x + w * 0 == x for every finite x: the same value, two fewer launches per use)."""
    z = torch.zeros((), device=device, dtype=torch.float32)
    z._ldm_const_zero = True
    return z


def is_const_zero(t):
    return getattr(t, "_ldm_const_zero", False)


def _warn_once(key, msg):
    if key not in _WARNED:
        _WARNED.add(key)
        warnings.warn(msg, RuntimeWarning, stacklevel=3)


def set_perceptual_backend(fn):
    """Install the LPIPS-style perceptual metric used by perceptual_loss_old (None to clear)."""
    global _PERCEPTUAL_BACKEND
    _PERCEPTUAL_BACKEND = fn


def perceptual_loss_old(original, reconstructed):
    """LPIPS(net='alex') on inputs mapped [0,1] -> [-1,1] (reference loss.py:6-21).

    With an ldm_amd.lpips.LPIPSAlex backend (local weights, load_lpips_alex) the whole term runs on the HIP
    kernels, the 2x - 1 map fused into its first layer; any other backend is called as fn(2x - 1, 2y - 1).
    The reference's two range asserts (loss.py:14-15, two host syncs) are not repeated: the decoder's
    (tanh + 1) / 2 output and ToTensor'd mels are in [0, 1] by construction."""
    if _PERCEPTUAL_BACKEND is None:
        _warn_once("lpips", "perceptual_loss_old: no LPIPS backend installed (weights are not available "
                            "offline); the perceptual term is 0. Use loss.set_perceptual_backend(fn).")
        return _const_zero(original.device)
    from ldm_amd.lpips import LPIPSAlex
    if isinstance(_PERCEPTUAL_BACKEND, LPIPSAlex):
        return _PERCEPTUAL_BACKEND(original, reconstructed, unit=True).mean()
    return _PERCEPTUAL_BACKEND(2 * original - 1, 2 * reconstructed - 1).mean()


def load_lpips_alex(state_dict_or_path, device="cuda"):
    """An LPIPS(net='alex') backend on the HIP kernels from LOCAL weights: an lpips.LPIPS state_dict, or
    torchvision alexnet 'features.*' + the lpips v0.1 'lin<i>.model.1.weight' tensors in one dict (or a file
    holding either, loaded with weights_only=True).  Install it with set_perceptual_backend."""
    from ldm_amd.lpips import LPIPSAlex
    sd = state_dict_or_path
    if isinstance(sd, str):
        sd = torch.load(sd, map_location="cpu", weights_only=True)
    return LPIPSAlex.from_state_dict(sd).to(device)


def perceptual_loss(original, reconstructed, feature_extractor_type: str = "vggish", feature_extractor=None):
    if feature_extractor_type == "vggish":
        assert feature_extractor is not None, "Feature extractor must be provided for VGGish"
        return feature_extractor(original, reconstructed)
    return perceptual_loss_old(original, reconstructed)


def kl_regularization_loss(latent):
    """mean(0.5 * (z^2 - 1 - log(z^2 + 1e-8)))  (reference loss.py:31-32)"""
    return HF.kl_loss(latent)


def compression_loss(original, reconstructed, latent, feature_extractor):
    """MSE(recon, x) + 0.1 * perceptual + 0.01 * KL(latent)  (reference loss.py:34-45)"""
    mse = HF.mse_loss(reconstructed, original)
    perc = perceptual_loss(original, reconstructed, config["compression_feature_extractor"],
                           feature_extractor=feature_extractor)
    kl = kl_regularization_loss(latent)
    if is_const_zero(perc):
        return mse + 0.01 * kl
    return mse + 0.1 * perc + 0.01 * kl


def diffusion_loss(noise_pred, noise_target):
    """F.mse_loss(noise_pred, noise_target)  (reference loss.py:48-49)"""
    return HF.mse_loss(noise_pred, noise_target)


def vggish_features():
    """The VGGish `features` stack (torchvggish VGG.features: 3x3 convs 64-M-128-M-256-256-M-512-512-M, each
    conv followed by ReLU, M = MaxPool2d(2, 2)), randomly initialised: load local weights into it
    (state_dict keys '0.weight', '0.bias', '3.weight', ...) and pass it to VGGishFeatureLoss."""
    layers, cin = [], 1
    for v in (64, "M", 128, "M", 256, 256, "M", 512, 512, "M"):
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers += [nn.Conv2d(cin, v, kernel_size=3, padding=1), nn.ReLU(inplace=True)]
            cin = v
    return nn.Sequential(*layers)


class VGGishFeatureLoss(nn.Module):
    """Std-normalised multi-tap feature MSE of a frozen VGGish conv stack (reference loss.py:52-101).

    `features`: the VGGish `features` nn.Sequential (vggish_features() + local weights).  The reference
    fetches it with torch.hub (remote), which this offline build never does; without it the loss is a zero
    constant (see module docstring).

    With features, forward runs on the HIP kernels (no_grad, as the reference's loss.py:78): predicted and
    target go through the stack as ONE batch (each Conv2d + ReLU pair is one conv launch with the ReLU
    fused, MaxPool2d(2, 2) is ldm_maxpool2x2), and each ReLU tap's std-normalised MSE comes from one moment
    pass (ldm_std_mse_moments / _accumulate: the normalised copies are never materialised).  Convs run at
    the caller's autocast precision, like the reference's (the style loss sits inside train.py:174's
    autocast region)."""

    def __init__(self, features=None):
        super().__init__()
        self.features = features
        if self.features is not None:
            self.features.eval()
            for p in self.features.parameters():
                p.requires_grad = False

    def forward(self, predicted, target):
        if self.features is None:
            _warn_once("vggish", "VGGishFeatureLoss: no VGGish weights (remote torch.hub in the reference); "
                                 "style loss is 0 (it is gradient-free in the reference, loss.py:78).")
            return _const_zero(predicted.device)
        from ldm_amd import ops
        layers = list(self.features)
        ntaps = sum(isinstance(m, nn.ReLU) for m in layers)
        if ntaps == 0:
            raise RuntimeError("VGGishFeatureLoss: the feature stack has no ReLU taps")
        ops.require_device(predicted, target, what="VGGishFeatureLoss")
        B = predicted.shape[0]
        dev = predicted.device
        acc = torch.zeros(1, device=dev, dtype=torch.float64)
        out = torch.empty((), device=dev, dtype=torch.float32)
        with torch.no_grad():
            x = torch.cat([ops.f32c(predicted), ops.f32c(target)], 0)
            i = 0
            while i < len(layers):
                m = layers[i]
                if isinstance(m, nn.Conv2d):
                    if (m.groups != 1 or m.dilation != (1, 1) or m.stride[0] != m.stride[1]
                            or m.padding[0] != m.padding[1] or m.padding_mode != "zeros"):
                        raise NotImplementedError(f"VGGishFeatureLoss: unsupported conv {m}")
                    relu = i + 1 < len(layers) and isinstance(layers[i + 1], nn.ReLU)
                    x = ops.conv_forward(x, m.weight, m.bias, stride=m.stride[0], padding=m.padding[0],
                                         act="relu" if relu else "none")
                    i += 2 if relu else 1
                    if not relu:
                        continue
                elif isinstance(m, nn.ReLU):
                    x = ops.activation(x, "relu")
                    i += 1
                elif isinstance(m, nn.MaxPool2d):
                    k, s_ = m.kernel_size, m.stride
                    if (k not in (2, (2, 2)) or s_ not in (2, (2, 2)) or m.padding not in (0, (0, 0))
                            or m.ceil_mode or m.dilation not in (1, (1, 1))):
                        raise NotImplementedError(f"VGGishFeatureLoss: unsupported pooling {m}")
                    x = ops.maxpool2x2(x)
                    i += 1
                    continue
                else:
                    raise NotImplementedError(f"VGGishFeatureLoss: unsupported layer {type(m).__name__}")
                # a ReLU tap: std-normalised MSE of the predicted half against the target half
                ops.std_mse_accumulate(x[:B], x[B:], acc, 1.0 / ntaps, eps=1e-8, out=out)
        return out


def style_loss(reconstructed, style_spec, feature_loss_net):
    return feature_loss_net(reconstructed, style_spec)


def gram_matrix(features):
    """(B,C,H,W) -> F F^T / (C H W).  Unused by the reference's training (loss.py:108-112)."""
    B, C, H, W = features.size()
    f = features.reshape(B, C, H * W)
    return torch.bmm(f, f.transpose(1, 2)) / (C * H * W)
