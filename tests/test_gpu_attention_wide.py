"""Width-general cross-attention (flash.hip; reference model.py:126-160 / :140-153): the KV-tiled online-softmax
forward and its backward for any L, S, and the UNet on latents wider than the LDS-resident instances cover.

* kernel forward / lse / backward against float64 torch of the same attention (1e-4 relative; fp32 sums);
* the UNet on a [1,32,16,128] latent (a 1x128x1024 mel: CA2 L = S = 128) and a 5-step DDIM there, against
  the REFERENCE (tests/golden/ref_goldens_r3.npz, make_goldens.py --r3), both the fused engine (literal loop:
  the folded cross-attentions only pay below ~64 keys) and the per-layer autograd path; 1e-4;
* a reduced SURVEY shape S: UNet(1, 1, 64) on a [1,1,64,256] mel (CA2 L = S = 1024), against the reference;
* CrossAttention forward + backward at L = S = 128 against float64 autograd of the oracle's restatement.
"""
import math
import os

import numpy as np
import pytest
import torch

import recipe
from conftest import ROOT, rel_err

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.fixture(scope="module")
def g3():
    return np.load(os.path.join(ROOT, "tests", "golden", "ref_goldens_r3.npz"))


def npy(t):
    return t.detach().double().cpu().numpy()


def _ref_attn(q, kv, heads):
    """float64 softmax((q*scale)^T k) v per head; q [B,E,L], kv [B,2E,S] channel-major."""
    B, E, L = q.shape
    S = kv.shape[2]
    d = E // heads
    qh = q.reshape(B, heads, d, L).transpose(2, 3) * math.sqrt(1.0 / d)        # [B,h,L,d]
    k = kv[:, :E].reshape(B, heads, d, S)                                       # [B,h,d,S]
    v = kv[:, E:].reshape(B, heads, d, S)
    sc = qh @ k                                                                 # [B,h,L,S]
    p = torch.softmax(sc, -1)
    o = (v @ p.transpose(2, 3))                                                 # [B,h,d,L]
    return o.reshape(B, E, L), torch.logsumexp(sc, -1)


CASES = {"ca2_w128": (2, 256, 128, 128), "ca1_ragged": (2, 512, 40, 200), "ca2_ragged": (1, 256, 100, 77),
         "ca2_long": (1, 256, 1024, 1024), "ca1_256": (1, 512, 256, 256), "s_gt_64_l_small": (3, 256, 16, 130),
         "one_key_tile": (2, 256, 70, 40),   # S <= 64: the double-buffered K/V loop's single-tile path
         # key splits over blocks (flash_combine_kernel): CA1 at shape S (d = 128, 4 splits), ragged S with 13
         # tiles over 2 splits (S % 4 == 0), and S % 4 != 0 over 4 splits
         "ca1_shape_s": (1, 512, 1024, 1024), "split_13_tiles": (1, 256, 200, 800), "split_ragged": (1, 512, 130, 1001)}


@pytest.mark.parametrize("case", sorted(CASES))
def test_flash_forward(cuda, case):
    from ldm_amd import ops
    B, E, L, S = CASES[case]
    g = torch.Generator().manual_seed(L * 7 + S)
    q = torch.randn(B, E, L, generator=g)
    kv = torch.randn(B, 2 * E, S, generator=g)
    ref, lse_ref = _ref_attn(q.double(), kv.double(), 4)
    assert ops.attention_uses_flash(E, 4, L, S)
    out = ops.attention_core(q.to(cuda), kv.to(cuda), 4)               # ldm_attention_core hands over
    out2, lse = ops.attention_forward_lse(q.to(cuda), kv.to(cuda), 4)
    torch.cuda.synchronize()
    assert rel_err(npy(out), ref.numpy()) < TOL
    assert torch.equal(out, out2)
    assert rel_err(npy(lse), lse_ref.numpy()) < 1e-5


SPLIT = ("ca2_long", "ca1_shape_s", "split_13_tiles", "split_ragged")


@pytest.mark.parametrize("case", SPLIT)
def test_flash_key_splits_match_one_block(cuda, case):
    """The forward with its key tiles split over blocks and merged by flash_combine_kernel against the one-block-per-
    (query tile, head) form (ldm_set_flash_split): O and lse within fp32 rounding of each other (the merge re-groups
    the sums: 1e-5 relative), both within the float64 bound (channel-major, the per-layer path's layout)."""
    from ldm_amd import _lib as L, ops
    B, E, Lq, S = CASES[case]
    g = torch.Generator().manual_seed(Lq * 5 + S)
    q = torch.randn(B, E, Lq, generator=g).to(cuda)
    kv = torch.randn(B, 2 * E, S, generator=g).to(cuda)
    lib = L.load()
    res = {}
    prev = lib.ldm_set_flash_split(1)
    try:
        for sp in (0, 1, 8):   # 8: the A/B form with up to 8 splits
            lib.ldm_set_flash_split(sp)
            o, lse = ops.attention_forward_lse(q, kv, 4)
            o2 = ops.attention_core(q, kv, 4)
            torch.cuda.synchronize()
            assert torch.equal(o, o2)
            res[sp] = (o, lse)
    finally:
        lib.ldm_set_flash_split(prev)
    ref, lse_ref = _ref_attn(q.cpu().double(), kv.cpu().double(), 4)
    for sp in (0, 1, 8):
        assert rel_err(npy(res[sp][0]), ref.numpy()) < TOL
        assert rel_err(npy(res[sp][1]), lse_ref.numpy()) < 1e-5
    for sp in (1, 8):
        assert rel_err(npy(res[sp][0]), npy(res[0][0])) < 1e-5
        assert rel_err(npy(res[sp][1]), npy(res[0][1])) < 1e-6


BWD = {"ca2_w128": (2, 256, 128, 128), "ca1_ragged": (1, 512, 96, 200), "ca2_ragged": (2, 256, 70, 33)}


@pytest.mark.parametrize("case", sorted(BWD))
def test_flash_backward(cuda, case):
    from ldm_amd import functional as HF
    B, E, L, S = BWD[case]
    g = torch.Generator().manual_seed(L + 3 * S)
    q = torch.randn(B, E, L, generator=g)
    kv = torch.randn(B, 2 * E, S, generator=g)
    dout = torch.randn(B, E, L, generator=g)
    q64, kv64 = q.double().requires_grad_(True), kv.double().requires_grad_(True)
    ref, _ = _ref_attn(q64, kv64, 4)
    (ref * dout.double()).sum().backward()
    qd, kvd = q.to(cuda).requires_grad_(True), kv.to(cuda).requires_grad_(True)
    y = HF.attention_core(qd, kvd, 4)
    (y * dout.to(cuda)).sum().backward()
    torch.cuda.synchronize()
    assert rel_err(npy(y), ref.detach().numpy()) < TOL
    assert rel_err(npy(qd.grad), q64.grad.numpy()) < TOL
    assert rel_err(npy(kvd.grad[:, :E]), kv64.grad[:, :E].numpy()) < TOL      # dK
    assert rel_err(npy(kvd.grad[:, E:]), kv64.grad[:, E:].numpy()) < TOL      # dV


def _unet(seed, cin):
    import models.model as M
    u = M.UNet(cin, cin, 64)
    recipe.fill_module(u, seed=seed)
    return u


@pytest.mark.parametrize("grad", [False, True])
def test_unet_wide_latent(g3, cuda, grad):
    u = _unet(100, 32).to(cuda)
    z = torch.from_numpy(recipe.normal((1, 32, 16, 128), 770)).to(cuda)
    s5 = torch.from_numpy(recipe.uniform01((1, 256, 4, 32), 771)).to(cuda)
    s6 = torch.from_numpy(recipe.uniform01((1, 512, 2, 16), 772)).to(cuda)
    with torch.set_grad_enabled(grad):
        y = u(z, torch.tensor([117], device=cuda), {"s5": s5, "s6": s6})
    assert y.requires_grad == grad
    assert rel_err(npy(y), g3["w128_unet_out"]) < TOL


def test_ddim_wide_latent(g3, cuda):
    """style_conditioned_ddim_sample on [1,32,16,128] (5 steps, eta 0) through the graphed C loop."""
    import models.model as M
    ldm = M.LDM(32, pretrained_path="")
    recipe.fill_module(ldm, seed=700)
    ldm = ldm.to(cuda).eval()
    style = torch.from_numpy(recipe.uniform01((1, 1, 128, 1024), 773)).to(cuda)
    zT = torch.from_numpy(recipe.normal((1, 32, 16, 128), 774)).to(cuda)
    with torch.no_grad():
        emb = ldm.style_encoder(style)
        x, logs = ldm.style_conditioned_ddim_sample(zT, emb, timesteps=5, eta=0.0)
    assert logs["timesteps"] == [199, 149, 99, 49]
    assert rel_err(npy(x), g3["w128_ddim5_x"]) < TOL


def test_unet_engine_key_splits_token_major(cuda):
    """The fused engine's token-major flash attention with its key tiles split over blocks (flash_combine_kernel): the
    UNet on a [1,32,16,512] latent (CA2 over 512 tokens: 32 blocks, 2 splits) through the engine (no grad) against the
    per-layer autograd path (channel-major attention, merged by flash_combine_cm_kernel) and against the engine with
    the splits off (ldm_set_flash_split(0)); 1e-5 relative to each other (fp32 regroupings only)."""
    from ldm_amd import _lib as L
    u = _unet(102, 32).to(cuda)
    z = torch.from_numpy(recipe.normal((1, 32, 16, 512), 780)).to(cuda)
    s5 = torch.from_numpy(recipe.uniform01((1, 256, 4, 128), 781)).to(cuda)
    s6 = torch.from_numpy(recipe.uniform01((1, 512, 2, 64), 782)).to(cuda)
    t = torch.tensor([321], device=cuda)
    emb = {"s5": s5, "s6": s6}
    lib = L.load()
    prev = lib.ldm_set_flash_split(1)
    try:
        with torch.no_grad():
            y_eng = u(z, t, emb)
        with torch.enable_grad():
            y_layer = u(z, t, emb).detach()
        lib.ldm_set_flash_split(0)
        with torch.no_grad():
            y_one = u(z, t, emb)
        torch.cuda.synchronize()
    finally:
        lib.ldm_set_flash_split(prev)
    assert torch.isfinite(y_eng).all()
    assert rel_err(npy(y_eng), npy(y_one)) < 1e-5
    assert rel_err(npy(y_eng), npy(y_layer)) < 1e-5


@pytest.mark.parametrize("grad", [False, True])
def test_unet_shape_s_reduced(g3, cuda, grad):
    """UNet(1, 1, 64) directly on a [1,1,64,256] mel (SURVEY §0.4 shape S, reduced 2x per side)."""
    u = _unet(101, 1).to(cuda)
    z = torch.from_numpy(recipe.normal((1, 1, 64, 256), 775)).to(cuda)
    s5 = torch.from_numpy(recipe.uniform01((1, 256, 16, 64), 776)).to(cuda)
    s6 = torch.from_numpy(recipe.uniform01((1, 512, 8, 32), 777)).to(cuda)
    with torch.set_grad_enabled(grad):
        y = u(z.requires_grad_(grad), torch.tensor([42], device=cuda), {"s5": s5, "s6": s6})
        if grad:
            y.sum().backward()
            assert torch.isfinite(z.grad).all()
    assert rel_err(npy(y), g3["shapeS_unet_out"]) < TOL


def test_cross_attention_module_backward_wide(cuda):
    """CrossAttention(256) on 8x16 maps (L = S = 128): output, input and in/out-projection gradients against
    float64 autograd of the oracle's restatement (oracle/ldm_torch_cpu.py cross_attention)."""
    import models.model as M
    from oracle import ldm_torch_cpu as TC
    ca = M.CrossAttention(256, 4)
    recipe.fill_module(ca, seed=910)
    sd64 = {k: v.detach().double().clone().requires_grad_(True) for k, v in ca.state_dict().items()}
    x = torch.from_numpy(recipe.normal((2, 256, 8, 16), 911))
    s = torch.from_numpy(recipe.uniform01((2, 256, 8, 16), 912))
    gy = torch.from_numpy(recipe.normal((2, 256, 8, 16), 913))
    x64, s64 = x.double().requires_grad_(True), s.double().requires_grad_(True)
    ref = TC.cross_attention(sd64, "", x64, s64)
    (ref * gy.double()).sum().backward()
    ca = ca.to(cuda)
    xd, sdv = x.to(cuda).requires_grad_(True), s.to(cuda).requires_grad_(True)
    y = ca(xd, sdv)
    (y * gy.to(cuda)).sum().backward()
    torch.cuda.synchronize()
    assert rel_err(npy(y), ref.detach().numpy()) < TOL
    assert rel_err(npy(xd.grad), x64.grad.numpy()) < TOL
    assert rel_err(npy(sdv.grad), s64.grad.numpy()) < TOL
    named = dict(ca.named_parameters())
    for k in ("multihead_attn.in_proj_weight", "multihead_attn.in_proj_bias", "multihead_attn.out_proj.weight"):
        assert rel_err(npy(named[k].grad), sd64[k].grad.numpy()) < TOL, k
