"""The Cin -> 1 k3 s1 p1 conv (csrc/conv.hip conv_cout1_k3_kernel: the UNet's dec1 on SURVEY shape S, 64 -> 1 on
128 x 512) against float64 torch, with and without its ReLU / bias epilogue, ragged row counts included, and its
reruns bitwise equal (the channel groups meet in a fixed order).

Tolerance: 1e-5 relative (max-norm) against float64 (fp32 fmaf chains per channel group, groups summed in order).
Reference: /root/reference/models/model.py:194 (dec1 = Conv2d(num_filters, out_channels, 3, padding=1)).
"""
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_err

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(1, 64, 128, 512), (2, 64, 16, 64), (3, 32, 5, 24), (1, 512, 4, 8)])
@pytest.mark.parametrize("act", ["none", "relu"])
def test_cout1_conv_vs_float64(cuda, shape, act):
    from ldm_amd import functional as HF
    B, Cin, H, W = shape
    g = torch.Generator().manual_seed(B * 1000 + Cin + H)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(1, Cin, 3, 3, generator=g) * (1.0 / (Cin * 9) ** 0.5)
    b = torch.randn(1, generator=g)
    xd, wd, bd = x.to(cuda), w.to(cuda), b.to(cuda)
    with torch.no_grad():
        y = HF.conv(xd, wd, bd, stride=1, padding=1, act=act)
        y2 = HF.conv(xd, wd, bd, stride=1, padding=1, act=act)
    torch.cuda.synchronize()
    ref = F.conv2d(x.double(), w.double(), b.double(), stride=1, padding=1)
    if act == "relu":
        ref = ref.clamp_min(0)
    assert y.shape == ref.shape
    assert rel_err(y.double().cpu().numpy(), ref.numpy()) < 1e-5
    assert torch.equal(y, y2)
