"""GPU parity of the HIP path against golden vectors captured from the REFERENCE (tests/golden/).

Tolerance (north_star: "within 1e-4 rel-fp32"): max|y - y_ref| <= 1e-4 * max|y_ref| for every float
output; scheduler indexing (timestep lists) bit-exact.  Weights/inputs come from tests/golden/recipe.py,
the same streams the goldens were made with.
"""
import numpy as np
import pytest
import torch

import recipe
from conftest import rel_err

pytestmark = pytest.mark.gpu
TOL = 1e-4


def T(a, dev, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return t if dtype is None else t.to(dtype)


def npy(t):
    return t.detach().float().cpu().numpy()


@pytest.fixture(scope="module")
def M():
    import models.model as M
    return M


@pytest.fixture(scope="module")
def L_():
    import models.loss as L
    return L


def test_library_is_loaded_from_tree(cuda):
    from ldm_amd import _lib
    lib = _lib.load()
    n = _lib.c_int32()
    _lib.check(lib.ldm_device_count(_lib.ctypes.byref(n)), "device_count")
    assert n.value >= 1


@pytest.mark.parametrize("tag", ["s", "c"])
def test_unet_forward(M, goldens, cuda, tag):
    B, H, W, seed = {"s": (2, 16, 16, 1), "c": (1, 16, 64, 2)}[tag]
    unet = M.UNet(32, 32, 64)
    recipe.fill_module(unet, seed=100)
    unet = unet.to(cuda)
    z = T(recipe.normal((B, 32, H, W), seed), cuda)
    s5 = T(recipe.uniform01((B, 256, H // 4, W // 4), seed + 10), cuda)
    s6 = T(recipe.uniform01((B, 512, H // 8, W // 8), seed + 20), cuda)
    t = T(goldens[f"unet_{tag}_t"], cuda)
    with torch.no_grad():
        out = unet(z, t, {"s5": s5, "s6": s6})
        temb = unet.time_mlp(t)
    assert rel_err(npy(temb), goldens[f"unet_{tag}_temb"]) < TOL
    assert rel_err(npy(out), goldens[f"unet_{tag}_out"]) < TOL


def test_unet_engine_equals_layerwise(M, cuda):
    """The fused single-call engine and the per-layer autograd path use the same kernels and plans."""
    unet = M.UNet(32, 32, 64)
    recipe.fill_module(unet, seed=100)
    unet = unet.to(cuda)
    z = T(recipe.normal((3, 32, 16, 32), 5), cuda)
    s5 = T(recipe.uniform01((3, 256, 4, 8), 6), cuda)
    s6 = T(recipe.uniform01((3, 512, 2, 4), 7), cuda)
    t = torch.tensor([3, 77, 199], device=cuda)
    with torch.no_grad():
        a = unet(z, t, {"s5": s5, "s6": s6})
        b = unet._layerwise(z, t, s5, s6)
    # the time MLP differs (fused kernel vs two GEMMs): not bitwise, but within fp32 rounding
    assert rel_err(npy(a), npy(b)) < 1e-5


@pytest.mark.parametrize("E,h,w", [(256, 4, 16), (512, 2, 8)])
def test_cross_attention(M, goldens, cuda, E, h, w):
    ca = M.CrossAttention(E, 4)
    recipe.fill_module(ca, seed=200 + E)
    ca = ca.to(cuda)
    q = T(recipe.normal((2, E, h, w), 300 + E), cuda)
    kv = T(recipe.uniform01((2, E, h, w), 400 + E), cuda)
    with torch.no_grad():
        out = ca(q, kv)
    assert rel_err(npy(out), goldens[f"ca{E}_out"]) < TOL


def _vae(M, cuda):
    enc, dec, sty = M.SpectrogramEncoder(32), M.SpectrogramDecoder(32), M.StyleEncoder(1, 64)
    recipe.fill_module(enc, seed=500)
    recipe.fill_module(dec, seed=501)
    recipe.fill_module(sty, seed=502)
    return enc.to(cuda), dec.to(cuda), sty.to(cuda)


def test_vae_and_style_encoder(M, goldens, cuda):
    enc, dec, sty = _vae(M, cuda)
    x_s = T(recipe.uniform01((2, 1, 128, 128), 600), cuda)
    x_c = T(recipe.uniform01((1, 1, 128, 512), 601), cuda)
    zl = T(recipe.normal((2, 32, 16, 16), 602), cuda)
    with torch.no_grad():
        enc.eval()
        dec.eval()
        assert rel_err(npy(enc(x_s)), goldens["enc_eval_s_out"]) < TOL
        assert rel_err(npy(enc(x_c)), goldens["enc_eval_c_out"]) < TOL
        assert rel_err(npy(dec(zl)), goldens["dec_eval_s_out"]) < TOL
        enc.train()
        dec.train()
        assert rel_err(npy(enc(x_s)), goldens["enc_train_s_out"]) < TOL
        assert rel_err(npy(enc.encoder[1].running_mean), goldens["enc_train_s_rm0"]) < TOL
        assert rel_err(npy(enc.encoder[1].running_var), goldens["enc_train_s_rv0"]) < TOL
        assert rel_err(npy(dec(zl)), goldens["dec_train_s_out"]) < TOL
        assert rel_err(npy(dec.decoder[4].running_mean), goldens["dec_train_s_rm1"]) < TOL
        assert rel_err(npy(dec.decoder[4].running_var), goldens["dec_train_s_rv1"]) < TOL
        so = sty(x_s)
        assert rel_err(npy(so["s1"][:, :8]), goldens["style_s_s1_slice"]) < TOL
        for k in ("s5", "s6"):
            assert rel_err(npy(so[k]), goldens[f"style_s_{k}"]) < TOL
        so = sty(x_c)
        for k in ("s5", "s6"):
            assert rel_err(npy(so[k]), goldens[f"style_c_{k}"]) < TOL


@pytest.fixture(scope="module")
def ldm(M, cuda):
    m = M.LDM(32, pretrained_path="")
    recipe.fill_module(m, seed=700)
    m = m.to(cuda)
    m.eval()
    return m


@pytest.mark.parametrize("eta", [0, 1])
def test_ddim50(ldm, goldens, cuda, eta):
    style = T(recipe.uniform01((1, 1, 128, 128), 701), cuda)
    zT = T(recipe.normal((1, 32, 16, 16), 702), cuda)
    with torch.no_grad():
        emb = ldm.style_encoder(style)
        x, logs = ldm.style_conditioned_ddim_sample(zT, emb, timesteps=50, eta=float(eta))
    assert logs["timesteps"] == goldens[f"ddim50_eta{eta}_times"].tolist()
    assert rel_err(npy(logs["pred_x0"][0]), goldens[f"ddim50_eta{eta}_x0_first"]) < TOL
    assert rel_err(npy(logs["noise_pred"][-1]), goldens[f"ddim50_eta{eta}_eps_last"]) < TOL
    assert rel_err(npy(x), goldens[f"ddim50_eta{eta}_x"]) < TOL


def test_content_style_ddim(ldm, goldens, cuda):
    style = T(recipe.uniform01((1, 1, 128, 128), 701), cuda)
    zT = T(recipe.normal((1, 32, 16, 16), 702), cuda)
    with torch.no_grad():
        emb = ldm.style_encoder(style)
        x, logs = ldm.content_style_ddim_sample(zT, emb, timesteps=10, eta=1.0)
    assert logs["timesteps"] == goldens["cs10_eta1_times"].tolist()
    assert rel_err(npy(x), goldens["cs10_eta1_x"]) < TOL


def test_ddim_canonical_128x512(ldm, goldens, cuda):
    style = T(recipe.uniform01((1, 1, 128, 512), 703), cuda)
    zT = T(recipe.normal((1, 32, 16, 64), 704), cuda)
    with torch.no_grad():
        emb = ldm.style_encoder(style)
        x, _ = ldm.style_conditioned_ddim_sample(zT, emb, timesteps=5, eta=0.0)
    assert rel_err(npy(x), goldens["ddim5_c_x"]) < TOL


def test_style_wrapper_cpu_generator(ldm, goldens, cuda):
    style = T(recipe.uniform01((1, 1, 128, 128), 701), cuda)
    torch.manual_seed(1234)
    with torch.no_grad():
        out = ldm.style_ddim_sample_wrapper((1, 32, 16, 16), style, timesteps=8, eta=0.0)
    assert rel_err(npy(out), goldens["wrap8_decoded"]) < TOL


def test_ldm_forward_injected_noise(ldm, goldens, L_, cuda):
    content = T(recipe.uniform01((2, 1, 128, 128), 710), cuda)
    style = T(recipe.uniform01((2, 1, 128, 128), 711), cuda)
    t = T(goldens["fwd_eval_t"], cuda)
    noise = T(goldens["fwd_eval_noise"], cuda)
    with torch.no_grad():
        out = ldm(content, style, t, noise=noise)
    for k in ("z_t", "noise_pred", "z_0", "reconstructed"):
        assert rel_err(npy(out[k]), goldens[f"fwd_eval_{k}"]) < TOL, k
    with torch.no_grad():
        dl = L_.diffusion_loss(out["noise_pred"], out["noise"])
        kl = L_.kl_regularization_loss(out["z_0"])
    assert rel_err(npy(dl), goldens["loss_diffusion"]) < TOL
    assert rel_err(npy(kl), goldens["loss_kl"]) < TOL


def test_batched_sampling_matches_per_sample(ldm, cuda):
    """The reference crashes for B>1 (model.py:461); here B=3 must equal three B=1 runs."""
    style = T(recipe.uniform01((3, 1, 128, 128), 720), cuda)
    zT = T(recipe.normal((3, 32, 16, 16), 721), cuda)
    with torch.no_grad():
        emb = ldm.style_encoder(style)
        xb, logs = ldm.style_conditioned_ddim_sample(zT, emb, timesteps=6, eta=0.5)
        for i in range(3):
            e1 = {k: v[i:i + 1] for k, v in emb.items()}
            x1, _ = ldm.style_conditioned_ddim_sample(zT[i:i + 1], e1, timesteps=6, eta=0.5)
            assert rel_err(npy(xb[i:i + 1]), npy(x1)) < 1e-5
    assert len(logs["timesteps"]) == 5 and len(logs["pred_x0"]) == 5


def test_graph_replay_equals_eager(M, cuda):
    from ldm_amd.engine import GraphedDDIM
    unet = M.UNet(32, 32, 64)
    recipe.fill_module(unet, seed=100)
    unet = unet.to(cuda)
    fd = M.ForwardDiffusion(200)
    times = torch.linspace(199, 0, 7).long()
    coefs = fd.reverse_coefs(times).to(cuda)
    B = 2
    x0 = T(recipe.normal((B, 32, 16, 64), 9), cuda)
    s5 = T(recipe.uniform01((B, 256, 4, 16), 10), cuda)
    s6 = T(recipe.uniform01((B, 512, 2, 8), 11), cuda)
    tt = times[:-1].view(-1, 1).expand(-1, B).contiguous().to(cuda)
    eng = M.engine_for(unet)
    with torch.no_grad():
        x = x0.clone()
        eng.ddim_loop(x, s5, s6, tt, coefs, 0.0)
        g = GraphedDDIM(eng, x0, s5, s6, tt, coefs, 0.0)
        y = g.replay().clone()
        y2 = g.replay().clone()
    torch.cuda.synchronize()
    assert torch.equal(x, y) and torch.equal(y, y2)


@pytest.mark.parametrize("split", [2, 3, 4])
def test_split_chains_match_single_chain(M, cuda, split):
    """Sub-batch chains on separate streams (eager and graph-captured) == one chain, logs included."""
    from ldm_amd.engine import GraphedDDIM
    unet = M.UNet(32, 32, 64)
    recipe.fill_module(unet, seed=100)
    unet = unet.to(cuda)
    fd = M.ForwardDiffusion(200)
    times = torch.linspace(199, 0, 6).long()
    coefs = fd.reverse_coefs(times).to(cuda)
    B, n = 4, 5
    x0 = T(recipe.normal((B, 32, 16, 64), 19), cuda)
    s5 = T(recipe.uniform01((B, 256, 4, 16), 20), cuda)
    s6 = T(recipe.uniform01((B, 512, 2, 8), 21), cuda)
    tt = times[:-1].view(-1, 1).expand(-1, B).contiguous().to(cuda)
    eng = M.engine_for(unet)
    with torch.no_grad():
        x1 = x0.clone()
        l1 = (torch.empty((n, B, 32, 16, 64), device=cuda), torch.empty((n, B, 32, 16, 64), device=cuda))
        eng.ddim_loop(x1, s5, s6, tt, coefs, 0.3, *l1)
        x2 = x0.clone()
        l2 = (torch.empty_like(l1[0]), torch.empty_like(l1[1]))
        eng.ddim_loop(x2, s5, s6, tt, coefs, 0.3, *l2, split=split)
        g = GraphedDDIM(eng, x0, s5, s6, tt, coefs, 0.3, logs=True, split=split)
        y = g.replay().clone()
    torch.cuda.synchronize()
    for a, b in ((x1, x2), (x1, y), (l1[0], l2[0]), (l1[1], l2[1]), (l1[0], g.x0_logs), (l1[1], g.eps_logs)):
        assert rel_err(npy(b), npy(a)) < 1e-5


def test_content_style_transfer_wrapper(ldm, goldens2, cuda):
    """The config-5 entry point end to end (model.py:468-501): encode, q_sample at T'-1 with the
    reference's epsilon (injected), 99-step eta=1 loop, (decoder+1)/2, and the undecorated decoder(z_t)."""
    content = T(recipe.uniform01((1, 1, 128, 128), 720), cuda)
    style = T(recipe.uniform01((1, 1, 128, 128), 721), cuda)
    eps = T(goldens2["cst100_eps"], cuda)
    with torch.no_grad():
        decoded, ztd = ldm.content_style_transfer_wrapper(content, style, num_timesteps=100, eta=1.0, noise=eps)
    assert rel_err(npy(decoded), goldens2["cst100_decoded"]) < TOL
    assert rel_err(npy(ztd), goldens2["cst100_zt_decoded"]) < TOL


def test_index_error_like_reference(ldm, cuda):
    style = T(recipe.uniform01((1, 1, 128, 128), 701), cuda)
    with pytest.raises(IndexError):
        ldm.content_style_transfer_wrapper(style, style, num_timesteps=250)


_SPLIT_CASES = {
    # name: (B, Cin, H, W, Cout, k, stride, transposed, plans)
    "bottleneck": (8, 512, 2, 8, 512, 3, 1, False, [(1, 1, 1, 4, 4), (1, 2, 2, 2, 8), (2, 1, 1, 2, 16), (1, 1, 2, 1, 16)]),
    "enc4": (8, 256, 4, 16, 512, 3, 2, False, [(1, 2, 1, 4, 2), (1, 1, 1, 2, 8)]),
    "dec4": (8, 512, 2, 8, 256, 3, 2, True, [(1, 1, 1, 4, 4), (2, 2, 2, 2, 8), (1, 2, 2, 1, 16), (2, 2, 1, 8, -1),
                                              (2, 2, 2, 4, -2), (1, 1, 1, 2, -4)]),
    "dec2k4": (2, 64, 32, 32, 16, 4, 2, True, [(2, 1, 1, 2, -1), (2, 1, 2, 4, -2)]),
    "enc1": (2, 32, 16, 64, 64, 3, 1, False, [(1, 2, 2, 4, 2), (1, 1, 2, 8, 4)]),
    "proj": (8, 512, 1, 16, 1024, 1, 1, False, [(1, 1, 1, 4, 4), (2, 2, 1, 1, 8)]),
}


@pytest.mark.parametrize("name", sorted(_SPLIT_CASES))
def test_split_k_plans(cuda, name):
    """Cross-block split-K (partial tiles + last-arriver fixed-order sum): equal to the unsplit plan up
    to fp32 summation order, bitwise reproducible across launches, and never stale when the input
    changes between launches (the partial buffers and counters are reused)."""
    from ldm_amd import _lib as L, ops
    B, Cin, H, W, Cout, k, stride, tr, plans = _SPLIT_CASES[name]
    g = torch.Generator().manual_seed(42)
    wshape = (Cin, Cout, k, k) if tr else (Cout, Cin, k, k)
    w = (torch.randn(wshape, generator=g) * 0.05).to(cuda)
    bias = torch.randn(Cout, generator=g).to(cuda)
    pad, op = ((1, 1) if k == 3 else (1, 0)) if tr else (k // 2, 0)
    desc = ops.make_desc(B, Cin, H, W, Cout, k, k, stride, pad, op if tr else 0, tr)
    xs = [torch.randn(B, Cin, H, W, generator=g).to(cuda) for _ in range(3)]
    base = ops.get_plan(desc, force=(2, 1, 1, 1, 1))

    def run(x, plan):
        return ops.conv_forward(x, w, bias, stride=stride, padding=pad, transposed=tr, output_padding=op if tr else 0,
                                act="relu", plan=plan)

    with torch.no_grad():
        refs = [run(x, base) for x in xs]
        x64 = xs[0].double().cpu()
        if tr:
            y64 = torch.nn.functional.conv_transpose2d(x64, w.double().cpu(), bias.double().cpu(), stride, pad, op)
        else:
            y64 = torch.nn.functional.conv2d(x64, w.double().cpu(), bias.double().cpu(), stride, pad)
        assert rel_err(npy(refs[0]), y64.clamp_min(0).numpy()) < 1e-5
        for pl in plans:
            plan = ops.get_plan(desc, force=pl)
            assert plan.ks == abs(pl[4]) and plan.balance == (pl[4] < 0) and plan.ws_floats > 0
            outs = [run(xs[i % 3], plan) for i in range(9)]
            torch.cuda.synchronize()
            for i, y in enumerate(outs):
                assert rel_err(npy(y), npy(refs[i % 3])) < 1e-5, (pl, i)
                assert torch.equal(y, outs[i % 3]), (pl, i)


@pytest.mark.parametrize("shape", [(2, 16, 64), (3, 16, 32), (1, 16, 16)])
def test_folded_reverse_loop_matches_literal(M, cuda, shape):
    """The reverse loop with both cross-attentions re-associated (Q projection folded into the keys,
    out-projection folded into enc4 / bottleneck) equals the literal per-op loop to fp32 rounding."""
    from ldm_amd.engine import UNetEngine
    B, H, W = shape
    unet = M.UNet(32, 32, 64)
    recipe.fill_module(unet, seed=100)
    unet = unet.to(cuda)
    fd = M.ForwardDiffusion(200)
    times = torch.linspace(199, 0, 6).long()
    coefs = fd.reverse_coefs(times).to(cuda)
    x0 = T(recipe.normal((B, 32, H, W), 31), cuda)
    s5 = T(recipe.uniform01((B, 256, H // 4, W // 4), 32), cuda)
    s6 = T(recipe.uniform01((B, 512, H // 8, W // 8), 33), cuda)
    tt = times[:-1].view(-1, 1).expand(-1, B).contiguous().to(cuda)
    outs, logs = [], []
    with torch.no_grad():
        for fold in (False, True):
            eng = UNetEngine(unet, fold=fold)
            x = x0.clone()
            lg = (torch.empty((5, B, 32, H, W), device=cuda), torch.empty((5, B, 32, H, W), device=cuda))
            eng.ddim_loop(x, s5, s6, tt, coefs, 0.0, *lg)
            outs.append(x)
            logs.append(lg)
    torch.cuda.synchronize()
    assert rel_err(npy(outs[1]), npy(outs[0])) < 1e-5
    assert rel_err(npy(logs[1][1]), npy(logs[0][1])) < 1e-5
