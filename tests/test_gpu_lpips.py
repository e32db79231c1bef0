"""LPIPS-AlexNet on HIP (ldm_amd/lpips.py; reference loss.py:6-21, lpips==0.1.4 LPIPS(net='alex')).

PARITY UNPINNED: lpips and its weights are not available here, so the reference cannot be run; the HIP path is
checked against the float64 restatement of lpips 0.1.4's forward (oracle/ldm_torch_cpu.py lpips_alex) on
recipe weights, and its backward against float64 autograd of that restatement.  Tolerance 1e-4 relative to
max (fp32 sums).  The building blocks (im2col / col2im, MaxPool2d(3, 2) and its backward) against torch's own
float64 unfold / fold / max_pool2d.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import recipe
from conftest import rel_err

pytestmark = pytest.mark.gpu
TOL = 1e-4


def npy(t):
    return t.detach().double().cpu().numpy()


def _module(seed=950):
    from ldm_amd.lpips import LPIPSAlex
    m = LPIPSAlex()
    vals = recipe.make_state({k: tuple(v.shape) for k, v in m.state_dict().items()
                              if not k.startswith(("scaling_layer", "lins."))}, seed)
    # lpips' lin heads are non-negative (it clamps them in training): |recipe| so the distance is a distance
    sd = {k: torch.from_numpy(np.abs(v) if k.startswith("lin") else v) for k, v in vals.items()}
    return LPIPSAlex.from_state_dict(sd), sd


@pytest.mark.parametrize("case", [(2, 3, 20, 26, 5, 1, 2), (2, 64, 15, 31, 5, 1, 2), (2, 3, 37, 50, 11, 4, 2)])
def test_im2col_col2im(cuda, case):
    from ldm_amd import _lib as L, ops
    B, C, H, W, k, s, p = case
    g = torch.Generator().manual_seed(sum(case))
    x = torch.randn(B, C, H, W, generator=g)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    kp = (C * k * k + 15) // 16 * 16
    col = torch.empty(B, kp, Ho, Wo, device=cuda)
    xd = x.to(cuda)
    L.call("ldm_im2col", xd.data_ptr(), B, C, H, W, k, k, s, p, kp, None, None, C, 0, col.data_ptr(),
           ops.stream_handle())
    ref = F.unfold(x.double(), k, padding=p, stride=s).reshape(B, C * k * k, Ho, Wo)
    assert torch.equal(col[:, :C * k * k].cpu().double(), ref)
    assert bool((col[:, C * k * k:] == 0).all())
    dcol = torch.randn(B, kp, Ho, Wo, generator=g)
    dx = torch.empty(B, C, H, W, device=cuda)
    L.call("ldm_col2im", dcol.to(cuda).data_ptr(), B, C, H, W, k, k, s, p, kp, None, C, 0, dx.data_ptr(),
           ops.stream_handle())
    refx = F.fold(dcol[:, :C * k * k].double().reshape(B, C * k * k, Ho * Wo), (H, W), k, padding=p, stride=s)
    assert rel_err(npy(dx), refx.numpy()) < 1e-6


@pytest.mark.parametrize("shape", [(2, 64, 31, 127), (1, 3, 9, 10), (2, 192, 15, 63)])
def test_maxpool3s2(cuda, shape):
    from ldm_amd import lpips as LP
    g = torch.Generator().manual_seed(shape[1])
    x = torch.relu(torch.randn(shape, generator=g))          # ReLU outputs: many tied zeros (first-occurrence rule)
    xr = x.double().requires_grad_(True)
    y = F.max_pool2d(xr, 3, 2)
    dy = torch.randn(tuple(y.shape), generator=g)
    (y * dy.double()).sum().backward()
    yd = LP._maxpool(x.to(cuda))
    dx = LP._maxpool_backward(x.to(cuda), dy.to(cuda))
    assert torch.equal(yd.cpu().double(), y.detach())
    assert rel_err(npy(dx), xr.grad.numpy()) < 1e-6


@pytest.mark.parametrize("shape", [(2, 1, 128, 128), (2, 1, 128, 512), (2, 3, 64, 96)])
def test_lpips_forward_backward(cuda, shape):
    from oracle import ldm_torch_cpu as TC
    m, sd = _module()
    m = m.to(cuda)
    sd64 = {k: v.double() for k, v in sd.items()}
    g = torch.Generator().manual_seed(shape[3])
    a = torch.rand(shape, generator=g)
    b = torch.rand(shape, generator=g)
    # unit=True: inputs in [0, 1], the 2x - 1 of perceptual_loss_old fused
    a64, b64 = a.double().requires_grad_(True), b.double().requires_grad_(True)
    ref = TC.lpips_alex(sd64, 2 * a64 - 1, 2 * b64 - 1)
    gv = torch.rand(shape[0], 1, 1, 1, generator=g) + 0.5
    (ref * gv.double()).sum().backward()
    ad, bd = a.to(cuda).requires_grad_(True), b.to(cuda).requires_grad_(True)
    val = m(ad, bd, unit=True)
    (val * gv.to(cuda)).sum().backward()
    torch.cuda.synchronize()
    assert val.shape == (shape[0], 1, 1, 1)
    assert rel_err(npy(val), ref.detach().numpy()) < TOL
    assert rel_err(npy(bd.grad), b64.grad.numpy()) < TOL
    assert rel_err(npy(ad.grad), a64.grad.numpy()) < TOL


def test_lpips_in_the_train_step(cuda, goldens):
    """loss.set_perceptual_backend(LPIPSAlex): the compression loss' 0.1 * LPIPS term enters the train step and
    its gradient reaches the decoder and the UNet (the restated step of test_gpu_train, B=2 128x128) -- against
    the float64 oracle step with the same LPIPS term."""
    import models.loss as Lm
    import models.model as M
    from oracle import ldm_torch_cpu as TC
    m, sdl = _module(960)
    ldm = M.LDM(32, pretrained_path="")
    recipe.fill_module(ldm, seed=700)
    sd64 = {k: v.detach().double().clone() for k, v in ldm.state_dict().items()}
    ldm = ldm.to(cuda).train()
    for p in ldm.encoder.parameters():
        p.requires_grad_(False)
    content = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 710))
    style = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 711))
    t = torch.from_numpy(goldens["fwd_eval_t"])
    noise = torch.from_numpy(goldens["train_noise"])
    Lm.set_perceptual_backend(m.to(cuda))
    try:
        out = ldm(content.to(cuda), style.to(cuda), t.to(cuda), noise=noise.to(cuda))
        perc = Lm.perceptual_loss_old(content.to(cuda), out["reconstructed"])
        total = Lm.compression_loss(content.to(cuda), out["reconstructed"], out["z_0"], None) + \
            Lm.diffusion_loss(out["noise_pred"], out["noise"])
        total.backward()
    finally:
        Lm.set_perceptual_backend(None)
    keys = ("decoder.decoder.6.weight", "decoder.decoder.1.weight", "unet.dec1.weight")
    for k in keys:
        sd64[k].requires_grad_(True)
    ab = TC.schedule(200)[2].double()
    o = TC.ldm_forward(sd64, content.double(), style.double(), t, noise.double(), ab, train_decoder=True,
                       train_encoder=True, state={})
    sdl64 = {k: v.double() for k, v in sdl.items()}
    perc64 = TC.lpips_alex(sdl64, 2 * content.double() - 1, 2 * o["reconstructed"] - 1).mean()
    tot64 = torch.mean((o["reconstructed"] - content.double()) ** 2) + 0.1 * perc64 + \
        0.01 * TC.kl_loss(o["z_0"]) + torch.mean((o["noise_pred"] - o["noise"]) ** 2)
    tot64.backward()
    assert float(perc) > 0
    assert rel_err(npy(perc), perc64.detach().numpy()) < TOL
    assert rel_err(npy(total), tot64.detach().numpy()) < TOL
    named = dict(ldm.named_parameters())
    for k in keys:
        assert rel_err(npy(named[k].grad), sd64[k].grad.numpy()) < TOL, k
