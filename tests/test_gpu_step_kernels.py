"""Step kernels (csrc/uconv.hip) of the reverse loop: every layer against float64 torch, and the whole
loop on them against the general-kernel loop and the oracle.

Tolerance: 1e-5 relative (max-norm) per layer against float64 — fp32 MFMA accumulation in a different
order than torch; the loop to 1e-5 against the general kernels and 1e-4 (north_star) against the oracle.
Reference: model.py:178-194 (layers), :205-229 (epilogue order: ReLU, then + t_emb / + skip),
:409-465 (loop).
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import recipe
from conftest import rel_err

pytestmark = pytest.mark.gpu

# (Cin, Cout, mode) of the nine layers; mode 0 conv s1, 1 conv s2, 2 convT k3 s2 p1 op1
LAYERS = [(32, 64, 0), (64, 128, 1), (128, 256, 1), (256, 512, 1), (512, 512, 0), (512, 256, 2), (256, 128, 2),
          (128, 64, 2), (64, 32, 0)]
DIV = [1, 1, 2, 4, 8, 8, 4, 2, 1]


def npy(t):
    return t.detach().double().cpu().numpy()


def _case(variant, layer, shape):
    return variant, layer, shape


@pytest.mark.parametrize("variant,layer,shape",
                         [_case("uconv", l, s) for l in range(8) for s in [(8, 16, 64), (2, 16, 16), (3, 8, 24)]] +
                         [_case("ksplit", l, s) for l in (2, 3, 4, 5, 6) for s in [(8, 16, 64), (2, 16, 16), (3, 8, 24),
                                                                                  (5, 16, 64)]])
def test_step_layer_vs_float64(cuda, variant, layer, shape):
    """uconv: ldm_step_conv (register-direct, any latent with H, W multiples of 8); ksplit: ldm_step_conv_ws
    (the same kernel with 32x32 tiles and K split over blocks).  The split form runs twice on one workspace:
    bitwise-equal results (the split-K sum is in slot order) and the counters left zero."""
    from ldm_amd import _lib as L
    B, H, W = shape
    Cin, Cout, mode = LAYERS[layer]
    Hin, Win = H // DIV[layer], W // DIV[layer]
    Hout, Wout = (Hin, Win) if mode == 0 else ((Hin // 2, Win // 2) if mode == 1 else (2 * Hin, 2 * Win))
    g = torch.Generator().manual_seed(100 * layer + B)
    x = torch.randn(B, Cin, Hin, Win, generator=g)
    wshape = (Cin, Cout, 3, 3) if mode == 2 else (Cout, Cin, 3, 3)
    w = torch.randn(wshape, generator=g) * (1.0 / (Cin * 9) ** 0.5)
    posb = layer in (3, 4)
    bias = torch.randn((Hout, Wout, Cout) if posb else (Cout,), generator=g) * 0.1
    bc = torch.randn(B, Cout, generator=g) if layer == 1 else None
    sk = torch.randn(B, Cout, Hout, Wout, generator=g) if mode == 2 else None
    lib = L.load()
    st = torch.cuda.current_stream().cuda_stream
    packed = torch.empty(int(lib.ldm_step_packed_floats(layer)), device=cuda)
    wd = w.to(cuda).contiguous()
    L.call("ldm_step_pack_weight", layer, wd.data_ptr(), packed.data_ptr(), st)
    xd = x.permute(0, 2, 3, 1).contiguous().to(cuda)
    y = torch.full((B, Hout, Wout, Cout), float("nan"), device=cuda)
    bd = bias.contiguous().to(cuda)
    bcd = bc.to(cuda) if bc is not None else None
    skd = sk.permute(0, 2, 3, 1).contiguous().to(cuda) if sk is not None else None
    bcp = None if bcd is None else bcd.data_ptr()
    skp = None if skd is None else skd.data_ptr()
    if variant == "uconv":
        L.call("ldm_step_conv", layer, B, H, W, xd.data_ptr(), packed.data_ptr(), bd.data_ptr(), bcp, skp,
               y.data_ptr(), st)
    elif variant == "ksplit":   # the K-split form (32x32 tiles, K over 2-8 blocks, last arriver sums)
        nws = int(lib.ldm_step_workspace_floats(B, H, W))
        assert nws > 0
        ws = torch.zeros(nws, device=cuda)
        for yy in (y, y2 := torch.full_like(y, float("nan"))):
            L.call("ldm_step_conv_ws", layer, B, H, W, xd.data_ptr(), packed.data_ptr(), bd.data_ptr(), bcp, skp,
                   yy.data_ptr(), 0, ws.data_ptr(), st)
        torch.cuda.synchronize()
        assert torch.equal(y, y2)
        ncnt = int(lib.ldm_step_workspace_counter_floats(B, H, W))
        assert 64 <= ncnt < nws
        # every tile counter is back to zero
        assert int(ws[:ncnt].view(torch.int32).abs().sum()) == 0
    torch.cuda.synchronize()
    x64, w64 = x.double(), w.double()
    if mode == 2:
        ref = F.conv_transpose2d(x64, w64, None, stride=2, padding=1, output_padding=1)
    else:
        ref = F.conv2d(x64, w64, None, stride=1 if mode == 0 else 2, padding=1)
    ref = ref + (bias.double().permute(2, 0, 1)[None] if posb else bias.double()[None, :, None, None])
    ref = ref.clamp_min(0)
    if bc is not None:
        ref = ref + bc.double()[:, :, None, None]
    if sk is not None:
        ref = ref + sk.double()
    got = y.permute(0, 3, 1, 2)
    assert rel_err(npy(got), ref.numpy()) < 1e-5


@pytest.mark.parametrize("shape,eta", [((8, 16, 64), 0.0), ((2, 16, 16), 1.0), ((3, 8, 24), 0.4), ((1, 16, 64), 0.0),
                                       ((4, 16, 64), 0.7)])
def test_step_loop_equals_general_loop(M, cuda, shape, eta):
    """The reverse loop on the step kernels (NHWC state, fused dec1 update; use_step 1 and 2 =
    uconv.hip) == the same folded loop on conv.hip's general kernel, final x and
    both logs."""
    from ldm_amd.engine import UNetEngine
    B, H, W = shape
    unet = M.UNet(32, 32, 64)
    recipe.fill_module(unet, seed=100)
    unet = unet.to(cuda)
    fd = M.ForwardDiffusion(200)
    times = torch.linspace(199, 0, 6).long()
    coefs = fd.reverse_coefs(times).to(cuda)
    x0 = torch.from_numpy(recipe.normal((B, 32, H, W), 41)).to(cuda)
    s5 = torch.from_numpy(recipe.uniform01((B, 256, H // 4, W // 4), 42)).to(cuda)
    s6 = torch.from_numpy(recipe.uniform01((B, 512, H // 8, W // 8), 43)).to(cuda)
    tt = times[:-1].view(-1, 1).expand(-1, B).contiguous().to(cuda)
    outs = []
    with torch.no_grad():
        for step in (0, 1, 2):   # (2: the nine layers share one split-K workspace)
            eng = UNetEngine(unet, fold=True, step=step)
            x = x0.clone()
            lg = (torch.empty((5, B, 32, H, W), device=cuda), torch.empty((5, B, 32, H, W), device=cuda))
            eng.ddim_loop(x, s5, s6, tt, coefs, eta, *lg)
            assert eng.weights(eng.shape(B, 32, H, W)).use_step == step
            outs.append((x, lg[0], lg[1]))
    torch.cuda.synchronize()
    for k in (1, 2):
        for a, b in zip(outs[0], outs[k]):
            assert rel_err(npy(b), npy(a)) < 1e-5


@pytest.fixture(scope="module")
def M():
    import models.model as M
    return M
