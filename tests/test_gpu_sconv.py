"""Plan kind 4 (csrc/sconv.hip, round 6): the small-plane 16-bit-operand implicit GEMM that the train step's UNet
layers at the bottom of the U take under autocast (reference model.py:178-194, :205-229 run under train.py:174's
torch.autocast) — forwards with their + t_emb / + skip epilogues, and the data gradients (the forward kernel on the
dual descriptor).

Against float64 of the identically rounded operands (x and w rounded to the operand type, fp32 accumulation in the
kernel): max |y - y64| <= 1e-5 max |y64|; reruns bitwise (fixed-order wave sums); under bf16 the general kernel's plan
(conv.hip) on the same call within 1e-5 of it (both bf16 operands, different summation order; under fp16 the general
kernel keeps fp32 operands, so only the float64 check applies)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

T = {1: torch.float16, 2: torch.bfloat16}
CASES = {   # (B, Cin, H, W, Cout, stride, transposed, epilogue): the UNet layers at B = 8 on the 16 x 64 latent
    "enc2_s2_bcast": (8, 64, 16, 64, 128, 2, False, "bcast"),
    "enc3_s2": (8, 128, 8, 32, 256, 2, False, "relu"),
    "enc4_s2": (8, 256, 4, 16, 512, 2, False, "relu"),
    "bneck_s1": (8, 512, 2, 8, 512, 1, False, "relu"),
    "dec4_T_skip": (8, 512, 2, 8, 256, 2, True, "skip"),
    "dec3_T_skip": (8, 256, 4, 16, 128, 2, True, "skip"),
    "dec2_T_skip": (8, 128, 8, 32, 64, 2, True, "skip"),
    "odd_batch_s1": (3, 128, 2, 8, 128, 1, False, "relu"),
}


def _rand(shape, seed, lo=-1.0, hi=1.0):
    g = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(g.uniform(lo, hi, shape).astype(np.float32))


def _ref64(x, w, b, stride, tr, dt, bcast=None, skip=None):
    xr = x.to(T[dt]).double().cpu()
    wr = w.to(T[dt]).double().cpu()
    if tr:
        y = F.conv_transpose2d(xr, wr, b.double().cpu(), stride=stride, padding=1, output_padding=1)
    else:
        y = F.conv2d(xr, wr, b.double().cpu(), stride=stride, padding=1)
    y = torch.relu(y)
    if bcast is not None:
        y = y + bcast.double().cpu()[:, :, None, None]
    if skip is not None:
        y = y + skip.double().cpu()
    return y


def _rel(a, b):
    return float((a.double().cpu() - b).abs().max()) / max(float(b.abs().max()), 1e-30)


@pytest.fixture(autouse=True)
def _sconv_f16(monkeypatch):
    monkeypatch.setenv("LDM_AMD_SCONV_F16", "1")   # fp16 takes kind 4 here too (the train step: bf16 only)


@pytest.mark.parametrize("dt", [2, 1])
@pytest.mark.parametrize("case", sorted(CASES))
def test_sconv_forward_vs_float64(cuda, case, dt):
    from ldm_amd import ops
    B, Cin, H, W, Cout, s, tr, epi = CASES[case]
    op = 1 if tr else 0
    desc = ops.make_desc(B, Cin, H, W, Cout, 3, 3, s, 1, op, tr)
    plan = ops.tiled_plan(desc, dt, adds=epi in ("bcast", "skip"))
    assert plan is not None and plan.kind == 4, case
    x = _rand((B, Cin, H, W), 61).to(cuda)
    w = _rand((Cin, Cout, 3, 3) if tr else (Cout, Cin, 3, 3), 62, -0.05, 0.05).to(cuda)
    b = _rand((Cout,), 63, -0.1, 0.1).to(cuda)
    bc = _rand((B, Cout), 64).to(cuda) if epi == "bcast" else None
    sk = _rand((B, Cout, desc.Hout, desc.Wout), 65).to(cuda) if epi == "skip" else None
    kw = dict(stride=s, padding=1, transposed=tr, output_padding=op, act="relu", bcast=bc, skip=sk, dtype=dt)
    y = ops.conv_forward(x, w, b, **kw)
    y2 = ops.conv_forward(x, w, b, **kw)
    yg = ops.conv_forward(x, w, b, plan=ops.get_plan(desc), **kw)   # conv.hip's general kernel
    torch.cuda.synchronize()
    assert torch.equal(y, y2)
    ref = _ref64(x, w, b, s, tr, dt, bc, sk)
    assert _rel(y, ref) <= 1e-5, _rel(y, ref)
    if dt == 2:   # (the general kernel rounds bf16 operands too; under fp16 it keeps fp32 operands)
        assert _rel(y, yg.double().cpu()) <= 1e-5


@pytest.mark.parametrize("dt", [2, 1])
@pytest.mark.parametrize("case", ["enc3_s2", "enc4_s2", "bneck_s1", "dec4_T_skip", "dec3_T_skip", "odd_batch_s1"])
def test_sconv_data_gradient_vs_float64(cuda, case, dt):
    """The data gradient of each layer (conv <-> transposed conv on the same weights) on kind 4."""
    from ldm_amd import ops
    B, Cin, H, W, Cout, s, tr, _ = CASES[case]
    op = 1 if tr else 0
    desc = ops.make_desc(B, Cin, H, W, Cout, 3, 3, s, 1, op, tr)
    dplan = ops.tiled_plan(ops.dual_desc(desc), dt)
    assert dplan is not None and dplan.kind == 4, case
    w = _rand((Cin, Cout, 3, 3) if tr else (Cout, Cin, 3, 3), 72, -0.05, 0.05).to(cuda)
    g = _rand((B, Cout, desc.Hout, desc.Wout), 73).to(cuda)
    dx = ops.conv_backward_data(g, w, desc, dtype=dt)
    torch.cuda.synchronize()
    xr = torch.zeros(B, Cin, H, W, dtype=torch.float64, requires_grad=True)
    wr = w.to(T[dt]).double().cpu()
    if tr:
        y = F.conv_transpose2d(xr, wr, stride=s, padding=1, output_padding=op)
    else:
        y = F.conv2d(xr, wr, stride=s, padding=1)
    (y * g.to(T[dt]).double().cpu()).sum().backward()
    assert _rel(dx, xr.grad) <= 1e-5, _rel(dx, xr.grad)


def test_sconv_act_out_and_autocast_rounding(cuda):
    """act_out (the post-activation value before the adds, saved for the backward) and, inside a bf16 autocast
    region, the output rounding of every epilogue step: equal to the general kernel's within one bf16 ulp of
    disagreement on the rounded values (different fp32 summation order before the rounding)."""
    from ldm_amd import ops
    B, Cin, H, W, Cout, s, tr, _ = CASES["dec3_T_skip"]
    desc = ops.make_desc(B, Cin, H, W, Cout, 3, 3, s, 1, 1, tr)
    x = _rand((B, Cin, H, W), 81).to(cuda)
    w = _rand((Cin, Cout, 3, 3), 82, -0.05, 0.05).to(cuda)
    b = _rand((Cout,), 83, -0.1, 0.1).to(cuda)
    sk = _rand((B, Cout, desc.Hout, desc.Wout), 84).to(cuda)
    outs = []
    with torch.autocast("cuda", dtype=torch.bfloat16):
        for plan in (None, ops.get_plan(desc)):
            ao = torch.empty(B, Cout, desc.Hout, desc.Wout, device=cuda)
            y = ops.conv_forward(x, w, b, stride=2, padding=1, transposed=True, output_padding=1, act="relu",
                                 skip=sk, act_out=ao, plan=plan)
            outs.append((y, ao))
    torch.cuda.synchronize()
    (y4, a4), (yg, ag) = outs
    assert torch.equal(y4, y4.to(torch.bfloat16).float()) and torch.equal(a4, a4.to(torch.bfloat16).float())
    assert bool((a4 >= 0).all())
    for p, q in ((y4, yg), (a4, ag)):
        d = (p - q).abs()
        assert float(d.max()) <= 2 ** -7 * float(q.abs().max()) + 1e-6
        assert float((d > 0).float().mean()) < 0.02
