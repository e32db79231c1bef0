"""Reduced-precision reverse loops (BASELINE configs 3 / 5: fp16 / bf16 with fp32 scheduler accumulators)
against the reference run under torch.autocast("cpu", dtype) (tests/golden/make_goldens.py --amp).

Our loop under torch.autocast("cuda", dtype) rounds every step-kernel operand (activations and weights) to
fp16 / bf16, accumulates in fp32 and (round 4) rounds each conv output and skip / time-embedding add to the
16-bit type as the reference's autocast convs do, while the sampler state stays fp32; the reference also rounds
its attention matmuls (ours keep them fp32: the folded cross-attentions).  Both differ from the fp32 loop
by a few x 1e-4 (fp16) / 1e-3 (bf16) relative; the stated tolerances (max-norm relative, against the
autocast golden) are 1e-3 for fp16 and 8e-3 for bf16, about 3x the reference's own autocast-vs-fp32 gap.
Reference: model.py:409-465 (DDIM loop), :503-559 (content-style loop).
"""
import numpy as np
import pytest
import torch

import recipe
from conftest import ROOT, rel_err

pytestmark = pytest.mark.gpu

TOLS = {"fp16": 1e-3, "bf16": 8e-3}
DTYPES = {"fp16": torch.float16, "bf16": torch.bfloat16}


@pytest.fixture(scope="module")
def gamp():
    return np.load(f"{ROOT}/tests/golden/ref_goldens_amp.npz")


@pytest.fixture(scope="module")
def ldm(cuda):
    import models.model as M
    m = M.LDM(32, pretrained_path="")
    recipe.fill_module(m, seed=700)
    return m.to(cuda).eval()


def _inputs(ldm, cuda):
    style = torch.from_numpy(recipe.uniform01((1, 1, 128, 512), 741)).to(cuda)
    zT = torch.from_numpy(recipe.normal((1, 32, 16, 64), 742)).to(cuda)
    with torch.no_grad():
        emb = ldm.style_encoder(style)
    return zT, emb


def npy(t):
    return t.detach().double().cpu().numpy()


@pytest.mark.parametrize("name", ["fp16", "bf16"])
def test_ddim10_autocast(ldm, gamp, cuda, name):
    import models.model as M
    zT, emb = _inputs(ldm, cuda)
    with torch.no_grad(), torch.autocast("cuda", dtype=DTYPES[name]):
        x, logs = ldm.style_conditioned_ddim_sample(zT, emb, timesteps=10, eta=0.0)
        eng = M.engine_for(ldm.unet)
        assert eng.weights(eng.shape(1, 32, 16, 64)).step_dtype == (1 if name == "fp16" else 2)
    assert x.dtype == torch.float32
    assert logs["timesteps"] == gamp[f"amp10_{name}_times"].tolist()
    err = rel_err(npy(x), gamp[f"amp10_{name}_x"])
    print(f"ours vs reference {name} {err:.2e}; reference {name} vs fp32 "
          f"{rel_err(gamp[f'amp10_{name}_x'], gamp['amp10_fp32_x']):.2e}")
    assert err < TOLS[name], err
    # and it really ran at reduced precision: farther from the fp32 golden than the fp32 path's 1e-5
    assert rel_err(npy(x), gamp["amp10_fp32_x"]) > 1e-5


def test_ddim10_fp32_outside_autocast(ldm, gamp, cuda):
    zT, emb = _inputs(ldm, cuda)
    with torch.no_grad():
        x, _ = ldm.style_conditioned_ddim_sample(zT, emb, timesteps=10, eta=0.0)
    assert rel_err(npy(x), gamp["amp10_fp32_x"]) < 1e-4


def test_content_style_100_fp16(ldm, gamp, cuda):
    """Config 5's loop: T'=100, eta=1, fp16 operands, fp32 scheduler accumulators."""
    zT, emb = _inputs(ldm, cuda)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        x, _ = ldm.content_style_ddim_sample(zT, emb, timesteps=100, eta=1.0)
    err = rel_err(npy(x), gamp["cs100_fp16_x"])
    print(f"ours vs reference fp16 {err:.2e}; reference fp16 vs fp32 {rel_err(gamp['cs100_fp16_x'], gamp['cs100_fp32_x']):.2e}")
    assert err < TOLS["fp16"], err


@pytest.fixture(scope="module")
def gamp8():
    return np.load(f"{ROOT}/tests/golden/ref_goldens_amp8.npz")


@pytest.mark.parametrize("path", ["sampler", "bench_object"])
def test_content_style_100_fp16_b8(ldm, gamp8, cuda, path):
    """Config 5 at its bench shard: batch 8, [8,32,16,64], T'=100, eta=1, fp16 step-kernel operands, fp32
    scheduler accumulators, against the reference's autocast-fp16 loop (make_goldens.py --amp8: eight batch-1
    runs stacked, since the reference loop raises for batch > 1 at model.py:555).  "sampler" runs
    LDM.content_style_ddim_sample under torch.autocast("cuda", float16); "bench_object" the object bench.py
    --workload transfer times (a GraphedDDIM replay with the engine's dtype set to fp16).  Tolerance 1e-3
    (max-norm relative, as the batch-1 test); the reference's own fp16-vs-fp32 gap is printed."""
    import models.model as M
    from ldm_amd.engine import GraphedDDIM
    B = 8
    style = torch.from_numpy(recipe.uniform01((B, 1, 128, 512), 751)).to(cuda)
    zT = torch.from_numpy(recipe.normal((B, 32, 16, 64), 752)).to(cuda)
    with torch.no_grad():
        emb = ldm.style_encoder(style)
        if path == "sampler":
            with torch.autocast("cuda", dtype=torch.float16):
                x, _ = ldm.content_style_ddim_sample(zT, emb, timesteps=100, eta=1.0)
        else:
            times = torch.linspace(99, 0, 100).long()
            coefs = ldm.noise_scheduler.reverse_coefs(times).to(cuda)
            t_table = times[:-1].view(-1, 1).expand(-1, B).contiguous().to(cuda)
            eng = M.engine_for(ldm.unet)
            prev = eng.dtype
            eng.dtype = "fp16"
            try:
                gd = GraphedDDIM(eng, zT, emb["s5"], emb["s6"], t_table, coefs, 1.0, logs=True)
                gd.replay()
                x = gd.replay().clone()       # a second replay restarts from z_T: same result
            finally:
                eng.dtype = prev
    ref16, ref32 = gamp8["cs100b8_fp16_x"], gamp8["cs100b8_fp32_x"]
    err = rel_err(npy(x), ref16)
    print(f"ours vs reference fp16 {err:.2e}; reference fp16 vs fp32 {rel_err(ref16, ref32):.2e}")
    assert err < TOLS["fp16"], err
    for b in range(B):   # and per sample, so that no sample hides behind the batch's max norm
        assert rel_err(npy(x[b]), ref16[b]) < TOLS["fp16"], b


@pytest.mark.parametrize("name,layer,ksplit", [(n, l, k) for n in ("fp16", "bf16") for l in (0, 4, 5)
                                               for k in ((False, True) if l in (4, 5) else (False,))])
def test_step_layer_lowp(cuda, name, layer, ksplit):
    """One step-kernel layer at fp16 / bf16 operands (weights packed in 16 bits, ldm_step_pack_weight_dt) ==
    float64 conv of the operands rounded the same way, with the autocast output semantics: the conv output
    (+ bias) and the skip add rounded to the 16-bit type (ReLU exact).  Accumulation order aside, each output
    is within one ulp of the 16-bit type of the float64 value rounded the same way (a sum that lands within
    fp32 noise of a 16-bit rounding boundary may round either way), and almost all are equal; single-block and
    K-split forms."""
    import torch.nn.functional as F
    from ldm_amd import _lib as L
    LAYERS = [(32, 64, 0, 1), None, None, None, (512, 512, 0, 8), (512, 256, 2, 8)]
    Cin, Cout, mode, div = LAYERS[layer]
    B, H, W = 8, 16, 64
    Hin, Win = H // div, W // div
    Hout, Wout = (Hin, Win) if mode == 0 else (2 * Hin, 2 * Win)
    g = torch.Generator().manual_seed(300 + layer)
    x = torch.randn(B, Cin, Hin, Win, generator=g)
    w = torch.randn((Cin, Cout, 3, 3) if mode == 2 else (Cout, Cin, 3, 3), generator=g) / (Cin * 9) ** 0.5
    posb = layer == 4
    bias = torch.randn((Hout, Wout, Cout) if posb else (Cout,), generator=g) * 0.1
    sk = torch.randn(B, Cout, Hout, Wout, generator=g) if mode == 2 else None
    lib = L.load()
    st = torch.cuda.current_stream().cuda_stream
    dt = 1 if name == "fp16" else 2
    packed = torch.empty(int(lib.ldm_step_packed_floats(layer)) // 2, device=cuda)     # 16-bit pack
    L.call("ldm_step_pack_weight_dt", layer, dt, w.to(cuda).contiguous().data_ptr(), packed.data_ptr(), st)
    xd = x.permute(0, 2, 3, 1).contiguous().to(cuda)
    bd = bias.contiguous().to(cuda)
    skd = sk.permute(0, 2, 3, 1).contiguous().to(cuda) if sk is not None else None
    y = torch.full((B, Hout, Wout, Cout), float("nan"), device=cuda)
    if ksplit:
        ws = torch.zeros(int(lib.ldm_step_workspace_floats(B, H, W)), device=cuda)
        L.call("ldm_step_conv_ws", layer, B, H, W, xd.data_ptr(), packed.data_ptr(), bd.data_ptr(), None,
               None if skd is None else skd.data_ptr(), y.data_ptr(), dt, ws.data_ptr(), st)
    else:
        L.call("ldm_step_conv_dt", layer, B, H, W, xd.data_ptr(), packed.data_ptr(), bd.data_ptr(), None,
               None if skd is None else skd.data_ptr(), y.data_ptr(), dt, st)
    torch.cuda.synchronize()
    rnd = (lambda t: t.half().double()) if name == "fp16" else (lambda t: t.bfloat16().double())
    x64, w64 = rnd(x), rnd(w)
    ref = F.conv_transpose2d(x64, w64, stride=2, padding=1, output_padding=1) if mode == 2 else \
        F.conv2d(x64, w64, padding=1)
    ref = rnd(ref + (bias.double().permute(2, 0, 1)[None] if posb else bias.double()[None, :, None, None]))
    ref = ref.clamp_min(0)
    if sk is not None:
        ref = rnd(ref + sk.double())
    got = torch.from_numpy(npy(y.permute(0, 3, 1, 2)))
    ulp = 2.0 ** -10 if name == "fp16" else 2.0 ** -7     # one ulp, relative to the value (upper bound)
    diff = (got - ref).abs()
    # two roundings (conv output, skip add): at most two ulps of the larger magnitude, or two subnormal steps
    sub = 2.0 ** -24 if name == "fp16" else 2.0 ** -133     # the subnormal spacing (fp16 outputs below 6e-5)
    bad = diff > 2 * ulp * torch.maximum(ref.abs(), got.abs()) + 2 * sub
    i = int((diff / (torch.maximum(ref.abs(), got.abs()) + 1e-30)).argmax())
    assert not bool(bad.any()), (int(bad.sum()), float(diff.max()), np.unravel_index(i, tuple(ref.shape)),
                                 float(ref.flatten()[i]), float(got.flatten()[i]))
    assert float((diff > 0).double().mean()) < 0.01       # (boundary cases only)


TRAIN_GRAD_KEYS = ("unet.time_mlp.1.weight", "unet.dec1.weight", "unet.dec1.bias", "unet.enc1.weight",
                   "unet.cross_attention1.multihead_attn.in_proj_weight", "unet.bottleneck.bias",
                   "decoder.decoder.6.weight", "decoder.decoder.1.weight", "style_encoder.enc6.bias",
                   "style_encoder.enc1.weight")


def test_train_step_bf16_autocast(gamp, goldens, cuda):
    """Config 3's arithmetic: the restated train step (test_gpu_train.test_train_step_matches_reference)
    with its forward and losses under torch.autocast("cuda", bfloat16) and backward outside, against the
    reference under torch.autocast("cpu", bfloat16) (ref_goldens_amp.npz trainbf16_*) and fp32 (train_*).

    The reference rounds every conv / linear output to bf16 as well, which moves its gradients up to ~14 %
    (max-norm relative) from fp32; ours rounds operands only and accumulates in fp32.  Stated bound, per
    quantity: within 2 e + 1e-3 of both the fp32 and the bf16 golden, e = the reference's own
    bf16-vs-fp32 distance (two independent bf16 perturbations of about that size: the triangle bound);
    and not bitwise fp32 (the bf16 path really ran).  Measured (MI355X): 10 of 12 quantities closer to
    fp32 than the reference's bf16 (e.g. recon 4.2e-2 vs 6.3e-2), the CA1 in-projection and bottleneck
    bias gradients 1.4x e."""
    import models.loss as Lm
    import models.model as M
    ldm = M.LDM(32, pretrained_path="")
    recipe.fill_module(ldm, seed=700)
    ldm = ldm.to(cuda)
    ldm.train()
    for p in ldm.encoder.parameters():
        p.requires_grad_(False)
    content = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 710)).to(cuda)
    style = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 711)).to(cuda)
    t = torch.from_numpy(goldens["fwd_eval_t"]).to(cuda)
    noise = torch.from_numpy(goldens["train_noise"]).to(cuda)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = ldm(content, style, t, noise=noise)
        total = Lm.compression_loss(content, out["reconstructed"], out["z_0"], None) + \
            Lm.diffusion_loss(out["noise_pred"], out["noise"])
    total.backward()
    pairs = [("recon", npy(out["reconstructed"]), "trainbf16_recon", "train_recon"),
             ("total", npy(total), "trainbf16_total", "train_total")]
    named = dict(ldm.named_parameters())
    for k in TRAIN_GRAD_KEYS:
        g = named[k].grad
        g = g[:256] if g.dim() == 2 and g.shape[0] > 256 else g
        pairs.append((k, npy(g), "trainbf16_grad_" + k, "grad_" + k))
    moved, rows, bad = 0.0, [], []
    for name, ours, kb, kf in pairs:
        e = rel_err(gamp[kb], goldens[kf])
        to32, tobf = rel_err(ours, goldens[kf]), rel_err(ours, gamp[kb])
        rows.append(f"{name}: ref bf16-vs-fp32 {e:.2e}, ours-vs-fp32 {to32:.2e}, ours-vs-bf16 {tobf:.2e}")
        if to32 > 2 * e + 1e-3 or tobf > 2 * e + 1e-3:
            bad.append(name)
        moved = max(moved, to32)
    print("\n".join(rows))
    assert not bad, (bad, rows)
    assert moved > 1e-5


@pytest.mark.parametrize("name", ["fp16", "bf16"])
@pytest.mark.parametrize("case", [(2, 64, 32, 128, 128, 3, 2, 1, 0, False, (1, 2, 2, 1, 1)),   # kind 1 (32x32)
                                  (2, 64, 32, 128, 128, 3, 2, 1, 0, False, (2, 2, 2, 1, 1)),   # kind 2 (16x16)
                                  (2, 128, 16, 64, 64, 4, 2, 1, 0, True, (2, 1, 1, 2, 1))])    # 4-phase convT
def test_conv_fwd_wgrad_lowp(cuda, name, case):
    """conv forward (dtype in the epilogue) and the tap-shared weight gradient at fp16 / bf16 operands ==
    float64 of the same-rounded operands (1e-5: only the fp32 accumulation order differs).  The general
    conv kernel has bf16 instances only (config 3); under fp16 it runs fp32 operands (exact)."""
    import torch.nn.functional as F
    from ldm_amd import ops
    B, Cin, H, W, Cout, k, s, p, op, tr, plan = case
    g = torch.Generator().manual_seed(17)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn((Cin, Cout, k, k) if tr else (Cout, Cin, k, k), generator=g) / (Cin * k * k) ** 0.5
    dt = 1 if name == "fp16" else 2
    rnd = (lambda t: t.half().double()) if name == "fp16" else (lambda t: t.bfloat16().double())
    desc = ops.make_desc(B, Cin, H, W, Cout, k, k, s, p, op, tr)
    pl = ops.get_plan(desc, force=plan)
    xd, wd = x.to(cuda), w.to(cuda)
    y = ops.conv_forward(xd, wd, None, stride=s, padding=p, transposed=tr, output_padding=op, plan=pl, dtype=dt)
    frnd = rnd if name == "bf16" else (lambda t: t.double())
    ref = F.conv_transpose2d(frnd(x), frnd(w), stride=s, padding=p, output_padding=op) if tr else \
        F.conv2d(frnd(x), frnd(w), stride=s, padding=p)
    assert rel_err(npy(y), ref.numpy()) < 1e-5
    dy = torch.randn(tuple(ref.shape), generator=g)
    xr = rnd(x).requires_grad_(False)
    wr = rnd(w).requires_grad_(True)
    yr = F.conv_transpose2d(xr, wr, stride=s, padding=p, output_padding=op) if tr else F.conv2d(xr, wr, stride=s, padding=p)
    (yr * rnd(dy)).sum().backward()
    dw = ops.conv_backward_weight(xd, dy.to(cuda), desc, dtype=dt)
    assert rel_err(npy(dw), wr.grad.numpy()) < 1e-5


# the double-rate 16-bit weight-gradient form (wgrad.hip wgrad_lp_kernel) at every geometry class it takes:
# (B, Cin, H, W, Cout, k, s, p, op, transposed)
WGRAD_LP_CASES = {
    "k3s2_vae_enc2": (2, 64, 32, 128, 128, 3, 2, 1, 0, False),     # Wq 64, BM 128, C 64
    "k3s1_unet_enc1": (2, 32, 16, 64, 64, 3, 1, 1, 0, False),      # stride 1, BM 64, C 32
    "k3s2_wq32": (2, 128, 16, 64, 256, 3, 2, 1, 0, False),         # Wq 32, M 256 (two row tiles)
    "k3s2_wq16_rows2": (2, 256, 8, 32, 256, 3, 2, 1, 0, False),    # Wq 16: two rows per chunk
    "k4s2_convT_m32": (2, 32, 16, 64, 128, 4, 2, 1, 0, True),      # decoder convT 32 -> 128, BM 32
    "k4s2_convT_m128": (2, 128, 16, 64, 64, 4, 2, 1, 0, True),     # decoder convT 128 -> 64, BM 128
    "k3s2_convT_op1": (2, 64, 8, 32, 32, 3, 2, 1, 1, True),        # UNet decoder convT (k3 s2 op1)
    "ragged_m40_c48": (3, 48, 8, 32, 40, 3, 1, 1, 0, False),       # M, C not multiples of the tiles
    "k3s1_bottleneck_2x8": (4, 512, 2, 8, 512, 3, 1, 1, 0, False),  # 16-position chunks (2 rows of 8)
    "k3s2_to_2x8": (4, 256, 4, 16, 512, 3, 2, 1, 0, False),         # UNet enc4: output 2 x 8
    "k3s2_convT_from_2x8": (4, 512, 2, 8, 256, 3, 2, 1, 1, True),   # UNet dec4: input grid 2 x 8
    "k3s2_wq16_odd_rows": (2, 64, 6, 32, 64, 3, 2, 1, 0, False),    # 3 x 16 output: one 16-wide row per chunk
}


@pytest.mark.parametrize("name", ["fp16", "bf16"])
@pytest.mark.parametrize("case", sorted(WGRAD_LP_CASES))
def test_wgrad_lowp_double_rate(cuda, name, case, monkeypatch):
    """16-bit dW (32x32x16 MFMA form) == float64 of the same-rounded operands to 1e-5 (fp32 accumulation
    order only), bitwise reproducible, accumulate=1 adds onto dW, and equal within 1e-5 to the tap-shared
    16-bit form (LDM_WGRAD_LP=0)."""
    import torch.nn.functional as F
    import zlib
    from ldm_amd import ops
    B, Cin, H, W, Cout, k, s, p, op, tr = WGRAD_LP_CASES[case]
    g = torch.Generator().manual_seed(zlib.crc32(case.encode()) % 1000)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn((Cin, Cout, k, k) if tr else (Cout, Cin, k, k), generator=g) / (Cin * k * k) ** 0.5
    dt = 1 if name == "fp16" else 2
    rnd = (lambda t: t.half().double()) if name == "fp16" else (lambda t: t.bfloat16().double())
    xr = rnd(x)
    wr = w.double().requires_grad_(True)
    yr = F.conv_transpose2d(xr, wr, stride=s, padding=p, output_padding=op) if tr else F.conv2d(xr, wr, stride=s, padding=p)
    dy = torch.randn(tuple(yr.shape), generator=g)
    (yr * rnd(dy)).sum().backward()
    desc = ops.make_desc(B, Cin, H, W, Cout, k, k, s, p, op, tr)
    xd, dyd = x.to(cuda), dy.to(cuda)
    dw1 = ops.conv_backward_weight(xd, dyd, desc, dtype=dt)
    dw2 = ops.conv_backward_weight(xd, dyd, desc, dtype=dt)
    acc = torch.ones_like(dw1)
    ops.conv_backward_weight(xd, dyd, desc, dw=acc, accumulate=True, dtype=dt)
    monkeypatch.setenv("LDM_WGRAD_LP", "0")
    dw_ts = ops.conv_backward_weight(xd, dyd, desc, dtype=dt)
    torch.cuda.synchronize()
    assert torch.equal(dw1, dw2)
    assert rel_err(npy(dw1), wr.grad.numpy()) < 1e-5
    assert rel_err(npy(acc), wr.grad.numpy() + 1.0) < 1e-5
    assert rel_err(npy(dw1), npy(dw_ts)) < 1e-5
