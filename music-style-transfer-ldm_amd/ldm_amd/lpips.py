"""LPIPS-AlexNet on the HIP kernels: the perceptual term of the reference's compression loss.

Reference: loss.py:6-21 -- perceptual_loss_old builds ``lpips.LPIPS(net='alex', verbose=False).eval()``
(lpips==0.1.4, requirements.txt:43) and returns ``LPIPS(2*original - 1, 2*reconstructed - 1).mean()``; with
config['compression_feature_extractor'] = 'lpips' (config.py:17) it is the 0.1-weighted term of
compression_loss (loss.py:34-45) in both the AE pre-training and the LDM train step, and it carries
gradient.  lpips is not installed here and its weights (torchvision AlexNet + the lpips v0.1 lin heads) are
remote downloads, so this module takes LOCAL weights and its parity is UNPINNED: it is checked against a
float64 torch restatement of lpips 0.1.4's published forward (oracle/ldm_torch_cpu.py lpips_alex), not
against the package.

The algorithm (lpips 0.1.4, net='alex', lpips=True, spatial=False, version '0.1'):
  ScalingLayer (x - shift) / scale, shift = [-.030, -.088, -.188], scale = [.458, .448, .450] (a 1-channel
  mel broadcasts to the 3 channels); AlexNet features relu1..relu5 (conv 11x11/4 p2 3->64, maxpool 3/2,
  conv 5x5 p2 ->192, maxpool 3/2, conv 3x3 ->384, ->256, ->256, each + ReLU); per layer normalize_tensor over
  channels (eps 1e-10), squared difference, the 1x1 lin head (dropout is inactive in eval), spatial mean; the
  five layers summed -> val [B,1,1,1].

Every tensor operation runs in libldm_amd: the 3x3 convs on ldm_conv_forward (ReLU fused), the 11x11 and 5x5
convs as ldm_im2col + a 1x1 conv (the ScalingLayer and perceptual_loss_old's 2x - 1 fused into the im2col),
ldm_maxpool3s2, ldm_lpips_layer; the backward (to either input) on the dual convs, ldm_col2im,
ldm_maxpool3s2_backward, ldm_act_backward, ldm_lpips_layer_backward.  The state_dict keys are lpips.LPIPS's
(scaling_layer.*, net.sliceN.<idx>.*, linN.model.1.weight and the lins.N.* aliases), so its weight files load
directly: ``LPIPSAlex.from_state_dict(torch.load(path, weights_only=True))``.
"""
import collections

import torch
import torch.nn as nn

from . import _lib as L
from . import ops

CHNS = (64, 192, 384, 256, 256)
SHIFT = (-0.030, -0.088, -0.188)
SCALE = (0.458, 0.448, 0.450)
# (slice, module index in torchvision's alexnet.features, Cin, Cout, kernel, stride, pad)
CONVS = ((1, 0, 3, 64, 11, 4, 2), (2, 3, 64, 192, 5, 1, 2), (3, 6, 192, 384, 3, 1, 1), (4, 8, 384, 256, 3, 1, 1),
         (5, 10, 256, 256, 3, 1, 1))


class _ScalingLayer(nn.Module):
    def __init__(self):
        super().__init__()
        self.register_buffer("shift", torch.tensor(SHIFT)[None, :, None, None])
        self.register_buffer("scale", torch.tensor(SCALE)[None, :, None, None])


class _AlexSlices(nn.Module):
    """lpips.pretrained_networks.alexnet: slice1..slice5 holding torchvision alexnet.features[0:12] under their
    original indices (only the convs carry state)."""

    def __init__(self):
        super().__init__()
        for sl, idx, cin, cout, k, s, p in CONVS:
            mods = collections.OrderedDict()
            if sl in (2, 3):
                mods[str(idx - 1)] = nn.MaxPool2d(kernel_size=3, stride=2)
            mods[str(idx)] = nn.Conv2d(cin, cout, kernel_size=k, stride=s, padding=p)
            mods[str(idx + 1)] = nn.ReLU(inplace=False)
            self.add_module(f"slice{sl}", nn.Sequential(mods))

    def conv(self, i):
        sl, idx = CONVS[i][0], CONVS[i][1]
        return getattr(self, f"slice{sl}")._modules[str(idx)]


class _NetLinLayer(nn.Module):
    def __init__(self, chn_in):
        super().__init__()
        self.model = nn.Sequential(nn.Dropout(), nn.Conv2d(chn_in, 1, 1, stride=1, padding=0, bias=False))


def _kpad(k):
    return (k + 15) // 16 * 16


class LPIPSAlex(nn.Module):
    """lpips.LPIPS(net='alex') forward (in0, in1 -> [B,1,1,1]) on HIP, differentiable in both inputs.

    unit=True takes inputs in [0, 1] and applies perceptual_loss_old's ``2 * x - 1`` inside the first layer's
    im2col (same fp32 op order)."""

    def __init__(self):
        super().__init__()
        self.scaling_layer = _ScalingLayer()
        self.net = _AlexSlices()
        for i, c in enumerate(CHNS):
            setattr(self, f"lin{i}", _NetLinLayer(c))
        self.lins = nn.ModuleList([getattr(self, f"lin{i}") for i in range(5)])
        for p in self.parameters():
            p.requires_grad_(False)
        self.eval()
        self._cache = {}

    @classmethod
    def from_state_dict(cls, sd):
        """Weights from an lpips.LPIPS state_dict or the pieces lpips loads them from: torchvision alexnet
        ('features.<idx>.*') and the v0.1 lin file ('lin<i>.model.1.weight')."""
        m = cls()
        own = m.state_dict()
        out = {}
        for k, v in sd.items():
            if k.startswith("features."):
                idx = int(k.split(".")[1])
                for sl, i, *_ in CONVS:
                    if i == idx:
                        k = f"net.slice{sl}.{k[len('features.'):]}"
            if k in own:
                out[k] = v
            if k.startswith("lin") and not k.startswith("lins"):
                alias = "lins." + k[3:]
                if alias in own:
                    out[alias] = v
        missing = [k for k in own if k not in out and not k.startswith("scaling_layer")]
        if missing:
            raise KeyError(f"LPIPSAlex.from_state_dict: missing {missing[:4]}{'...' if len(missing) > 4 else ''}")
        m.load_state_dict(out, strict=False)
        return m

    # ------------------------------------------------------------------------------------------------
    def _weights(self, i, dev):
        """(weight, bias) of conv i; the im2col layers' weights as a zero-padded [Cout, Kpad, 1, 1] GEMM operand
        (a re-layout, cached per parameter version)."""
        conv = self.net.conv(i)
        w, b = conv.weight, conv.bias
        if i >= 2:
            return w, b
        key = (i, w._version, str(dev))
        hit = self._cache.get(i)
        if hit is None or hit[0] != key:
            cout, cin, k = w.shape[0], w.shape[1], w.shape[2]
            wp = torch.zeros((cout, _kpad(cin * k * k), 1, 1), device=dev, dtype=torch.float32)
            wp[:, :cin * k * k, 0, 0] = w.detach().reshape(cout, -1)
            hit = (key, wp)
            self._cache[i] = hit
        return hit[1], b

    def forward(self, in0, in1, unit=False):
        ops.require_device(in0, in1, what="LPIPSAlex")
        if in0.shape != in1.shape or in0.dim() != 4 or in0.shape[1] not in (1, 3):
            raise RuntimeError(f"LPIPSAlex: inputs must be [B,1|3,H,W] of one shape, got {tuple(in0.shape)}, "
                               f"{tuple(in1.shape)}")
        return _LPIPSFn.apply(self, bool(unit), ops.f32c(in0), ops.f32c(in1))


def _features(m, x, unit, dt):
    """relu1..relu5 of one input (and what their backward needs)."""
    dev = x.device
    B, C, H, W = x.shape
    sc = m.scaling_layer
    shift, scale = ops.f32c(sc.shift.reshape(3)), ops.f32c(sc.scale.reshape(3))
    feats = []
    h = x
    for i, (_sl, _idx, cin, cout, k, s, p) in enumerate(CONVS):
        w, b = m._weights(i, dev)
        if i == 2 or i == 1:
            h = _maxpool(h)
        if i < 2:
            Bh, Ch, Hh, Wh = h.shape
            Ho, Wo = (Hh + 2 * p - k) // s + 1, (Wh + 2 * p - k) // s + 1
            kp = _kpad(cin * k * k)
            col = torch.empty((Bh, kp, Ho, Wo), device=dev, dtype=torch.float32)
            L.call("ldm_im2col", h.data_ptr(), Bh, Ch, Hh, Wh, k, k, s, p, kp,
                   shift.data_ptr() if i == 0 else None, scale.data_ptr() if i == 0 else None, 3 if i == 0 else Ch,
                   int(unit and i == 0), col.data_ptr(), ops.stream_handle())
            h = ops.conv_forward(col, w, b, stride=1, padding=0, act="relu", dtype=dt)
        else:
            h = ops.conv_forward(h, w, b, stride=1, padding=1, act="relu", dtype=dt)
        feats.append(h)
    return feats


def _maxpool(x):
    B, C, H, W = x.shape
    y = torch.empty((B, C, (H - 3) // 2 + 1, (W - 3) // 2 + 1), device=x.device, dtype=torch.float32)
    L.call("ldm_maxpool3s2", x.data_ptr(), y.data_ptr(), B, C, H, W, ops.stream_handle())
    return y


def _maxpool_backward(x, dy):
    B, C, H, W = x.shape
    dx = torch.empty_like(x)
    L.call("ldm_maxpool3s2_backward", x.data_ptr(), ops.f32c(dy).data_ptr(), dx.data_ptr(), B, C, H, W,
           ops.stream_handle())
    return dx


def _lin(m, i):
    return ops.f32c(getattr(m, f"lin{i}").model[1].weight.detach().reshape(-1))


class _LPIPSFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, m, unit, in0, in1):
        dt = ops.autocast_dt()
        need = (ctx.needs_input_grad[2], ctx.needs_input_grad[3])
        f0 = _features(m, in0, unit, dt)
        f1 = _features(m, in1, unit, dt)
        B = in0.shape[0]
        val = torch.zeros(B, device=in0.device, dtype=torch.float32)
        ws = ops.scratch("lpips", B * f0[0].shape[2] * f0[0].shape[3], in0.device)
        for i in range(5):
            _b, c, h, w = f0[i].shape
            L.call("ldm_lpips_layer", f0[i].data_ptr(), f1[i].data_ptr(), _lin(m, i).data_ptr(), B, c, h * w,
                   val.data_ptr(), ws.data_ptr(), ops.stream_handle())
        ctx.m, ctx.unit, ctx.dt, ctx.shape = m, unit, dt, tuple(in0.shape)
        ctx.need = need
        if any(need):
            ctx.save_for_backward(*(f0 + f1))
        return val.reshape(B, 1, 1, 1)

    @staticmethod
    def backward(ctx, gout):
        m = ctx.m
        f = ctx.saved_tensors
        f0, f1 = list(f[:5]), list(f[5:])
        gval = ops.f32c(gout.reshape(-1))
        grads = []
        for side, feats in ((0, f0), (1, f1)):
            grads.append(_feature_backward(m, f0, f1, feats, gval, side, ctx) if ctx.need[side] else None)
        return (None, None) + tuple(grads)


def _feature_backward(m, f0, f1, feats, gval, side, ctx):
    """d val / d input `side` through the five LPIPS heads and the AlexNet stack."""
    dev = gval.device
    B = gval.shape[0]
    sc = m.scaling_layer
    scale = ops.f32c(sc.scale.reshape(3))
    g = None
    for i in range(4, -1, -1):
        _b, c, h, w = feats[i].shape
        if g is None:
            g = torch.empty_like(feats[i])
            acc = 0
        else:
            acc = 1
        L.call("ldm_lpips_layer_backward", f0[i].data_ptr(), f1[i].data_ptr(), _lin(m, i).data_ptr(), gval.data_ptr(),
               B, c, h * w, side, acc, g.data_ptr(), ops.stream_handle())
        gv, _, _ = ops.act_backward(g, "relu", act_out=feats[i])                # ReLU (fused in the forward)
        _sl, _idx, cin, cout, k, s, p = CONVS[i]
        wgt, _bias = m._weights(i, dev)
        if i >= 2:
            desc = ops.make_desc(B, cin, h, w, cout, 3, 3, 1, 1)
            gx = ops.conv_backward_data(gv, wgt, desc, dtype=ctx.dt)
            if i == 2:
                g = _maxpool_backward(feats[1], gx)                           # pool2 (input: relu2)
            else:
                g = gx
            continue
        # im2col layers: the 1x1 GEMM's data gradient, then col2im
        kp = _kpad(cin * k * k)
        desc = ops.make_desc(B, kp, h, w, cout, 1, 1, 1, 0)
        dcol = ops.conv_backward_data(gv, wgt, desc, dtype=ctx.dt)
        if i == 1:
            Hp, Wp = feats[0].shape[2], feats[0].shape[3]
            Hin, Win = (Hp - 3) // 2 + 1, (Wp - 3) // 2 + 1                     # pool1 output = conv2 input
            gp = torch.empty((B, cin, Hin, Win), device=dev, dtype=torch.float32)
            L.call("ldm_col2im", dcol.data_ptr(), B, cin, Hin, Win, k, k, s, p, kp, None, cin, 0, gp.data_ptr(),
                   ops.stream_handle())
            g = _maxpool_backward(feats[0], gp)                               # pool1 (input: relu1)
        else:
            _b0, C0, H0, W0 = ctx.shape
            dx = torch.empty(ctx.shape, device=dev, dtype=torch.float32)
            L.call("ldm_col2im", dcol.data_ptr(), B, C0, H0, W0, k, k, s, p, kp, scale.data_ptr(), 3, int(ctx.unit),
                   dx.data_ptr(), ops.stream_handle())
            return dx
    raise AssertionError("unreachable")
