"""Losses of the LDM path — drop-in for the reference's models/loss.py, computed on libldm_amd.

In scope and parity-pinned: diffusion_loss, the MSE term of
compression_loss, kl_regularization_loss.  Out of scope offline: the
LPIPS-AlexNet perceptual term and the VGGish feature loss — their weights are remote downloads in the
reference (loss.py:10, :56).  Both are pluggable here:

  * set_perceptual_backend(fn)   fn(original, reconstructed) -> scalar tensor (e.g. an LPIPS model
                                 loaded from local weights).  Unset: the term is 0 (warned once).
  * VGGishFeatureLoss(features)  takes a user-supplied VGGish `features` nn.Sequential; without one
                                 the style term is a zero constant.  In the reference it is computed
                                 under torch.no_grad() (loss.py:78), so it never changes an update —
                                 only the reported loss value.
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


def _warn_once(key, msg):
    if key not in _WARNED:
        _WARNED.add(key)
        warnings.warn(msg, RuntimeWarning, stacklevel=3)


def set_perceptual_backend(fn):
    """Install the LPIPS-style perceptual metric used by perceptual_loss_old (None to clear)."""
    global _PERCEPTUAL_BACKEND
    _PERCEPTUAL_BACKEND = fn


def perceptual_loss_old(original, reconstructed):
    """LPIPS(net='alex') on inputs mapped [0,1] -> [-1,1] (reference loss.py:6-21)."""
    if _PERCEPTUAL_BACKEND is None:
        _warn_once("lpips", "perceptual_loss_old: no LPIPS backend installed (weights are not available "
                            "offline); the perceptual term is 0. Use loss.set_perceptual_backend(fn).")
        return torch.zeros((), device=original.device, dtype=torch.float32)
    return _PERCEPTUAL_BACKEND(2 * original - 1, 2 * reconstructed - 1).mean()


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
    return mse + 0.1 * perc + 0.01 * kl


def diffusion_loss(noise_pred, noise_target):
    """F.mse_loss(noise_pred, noise_target)  (reference loss.py:48-49)"""
    return HF.mse_loss(noise_pred, noise_target)


class VGGishFeatureLoss(nn.Module):
    """Std-normalised multi-tap feature MSE of a frozen VGGish conv stack (reference loss.py:52-101).

    `features`: the VGGish `features` nn.Sequential with weights loaded from a local file.  The
    reference fetches it with torch.hub (remote), which this offline build never does; without it the
    loss is a zero constant (see module docstring)."""

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
            return torch.zeros((), device=predicted.device, dtype=torch.float32)
        pred_feats, targ_feats = [], []
        with torch.no_grad():
            xp, xt = predicted, target
            for layer in self.features:
                xp, xt = layer(xp), layer(xt)
                if isinstance(layer, nn.ReLU):
                    pred_feats.append(xp)
                    targ_feats.append(xt)
        total = 0
        for p, t in zip(pred_feats, targ_feats):
            p = p / (torch.std(p, dim=[1, 2, 3], keepdim=True) + 1e-8)
            t = t / (torch.std(t, dim=[1, 2, 3], keepdim=True) + 1e-8)
            total = total + HF.mse_loss(p, t)
        return total / len(pred_feats)


def style_loss(reconstructed, style_spec, feature_loss_net):
    return feature_loss_net(reconstructed, style_spec)


def gram_matrix(features):
    """(B,C,H,W) -> F F^T / (C H W).  Unused by the reference's training (loss.py:108-112)."""
    B, C, H, W = features.size()
    f = features.reshape(B, C, H * W)
    return torch.bmm(f, f.transpose(1, 2)) / (C * H * W)
