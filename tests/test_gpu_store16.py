"""16-bit storage of the train step's large maps (ldm_capi.h LDM_DT_X16 / _Y16 / _DY16, LDM_ST_*): every
kernel that reads or writes a map in 16 bits gives the SAME result as its fp32-storage form on the same values.

Inputs are bf16 / fp16-representable (a 16-bit map holds exactly those), so a 16-bit read is exact; the kernels
then compute in fp32 as before, and a 16-bit write is the round-to-nearest-even of the fp32 result.  So, bit for
bit: outputs stored in 16 bits == the fp32-storage outputs rounded to the type; fp32 outputs (weight / BN
parameter gradients, statistics) == the fp32-storage outputs.  Covers the kind-3 convs (window and gather
forms, forward and data gradient), the Cin = 1 / Cout = 1 VALU convs, the weight gradient's register-staged
instances (double-rate and one-channel), BatchNorm forward / backward (rank-local and the SyncBatchNorm stages
with a stub group) and the activation backward.  Reference semantics: torch.autocast keeps these maps as
16-bit tensors (train.py:174; models/model.py:10-88 layers)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

T = {1: torch.float16, 2: torch.bfloat16}


def _rand(shape, seed, lo=-1.0, hi=1.0):
    g = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(g.uniform(lo, hi, shape).astype(np.float32))


def _q(t, dt):
    """t rounded to the 16-bit type (as a 16-bit tensor) and its exact fp32 copy."""
    t16 = t.to(T[dt])
    return t16, t16.float()


def _same(a16, b32, dt):
    """a (16-bit) == b (fp32) rounded to the type, bitwise."""
    assert a16.dtype == T[dt], a16.dtype
    assert torch.equal(a16, b32.to(T[dt])), float((a16.float() - b32.to(T[dt]).float()).abs().max())


CONV = {   # (B, Cin, H, W, Cout, k, stride, pad, out_pad, transposed)
    "w_k3s2": (2, 64, 64, 256, 128, 3, 2, 1, 0, False),          # tconvw, stride 2
    "w_k3s1": (4, 32, 16, 64, 256, 3, 1, 1, 0, False),           # tconvw, stride 1
    "g_convT_k4": (2, 128, 32, 64, 64, 4, 2, 1, 0, True),        # tconv gather form (4 taps, one M tile)
    "w_convT_k4_128": (2, 128, 32, 128, 64, 4, 2, 1, 0, True),
    "k4s2_dgrad": (2, 128, 64, 128, 64, 4, 2, 1, 0, False),
}


@pytest.mark.parametrize("dt", [2, 1])
@pytest.mark.parametrize("case", sorted(CONV))
def test_kind3_conv_store16(cuda, case, dt):
    from ldm_amd import ops
    B, Cin, H, W, Cout, k, s, p, op, tr = CONV[case]
    x16, x32 = _q(_rand((B, Cin, H, W), 11), dt)
    w = _rand((Cin, Cout, k, k) if tr else (Cout, Cin, k, k), 12, -0.1, 0.1).to(cuda)
    b = _rand((Cout,), 13, -0.1, 0.1).to(cuda)
    kw = dict(stride=s, padding=p, transposed=tr, output_padding=op, act="relu", dtype=dt)
    y32 = ops.conv_forward(x32.to(cuda), w, b, **kw)
    y16 = ops.conv_forward(x16.to(cuda), w, b, out_dtype=T[dt], **kw)
    torch.cuda.synchronize()
    _same(y16, y32, dt)
    # the data gradient (forward kernel on the dual descriptor) and the weight gradient from 16-bit maps
    desc = ops.make_desc(B, Cin, H, W, Cout, k, k, s, p, op, tr)
    g16, g32 = _q(_rand(tuple(y32.shape), 14), dt)
    dx32 = ops.conv_backward_data(g32.to(cuda), w, desc, dtype=dt)
    dx16 = ops.conv_backward_data(g16.to(cuda), w, desc, dtype=dt, out_dtype=T[dt])
    dw32 = ops.conv_backward_weight(x32.to(cuda), g32.to(cuda), desc, dtype=dt)
    dw16 = ops.conv_backward_weight(x16.to(cuda), g16.to(cuda), desc, dtype=dt)
    torch.cuda.synchronize()
    _same(dx16, dx32, dt)
    assert ops.wgrad_storage16(desc, dt), "the double-rate weight gradient must take 16-bit maps here"
    assert torch.equal(dw16, dw32)


# weight gradients whose splits run several chunks each, so the chunk ring (wgrad_lp16p_kernel, LDM_WGRAD_RING)
# cycles through all its buffers and the issue cursor crosses rows and samples: every chunk geometry of the form
# (rows of 32 positions; 16 x 2; 16 x 1; 8 x 2) and the k3 / k4, stride 1 / 2, transposed layers of the step
RING = {   # (B, Cin, H, W, Cout, k, stride, pad, out_pad, transposed)
    "k3s2_64_128": (16, 64, 64, 256, 128, 3, 2, 1, 0, False),
    "k3s2_128_256": (16, 128, 32, 128, 256, 3, 2, 1, 0, False),
    "k3s1_32_64": (16, 32, 16, 64, 64, 3, 1, 1, 0, False),
    "k3s2_rows16x2": (16, 64, 8, 32, 64, 3, 2, 1, 0, False),
    "k3s1_rows16x2": (16, 64, 4, 16, 64, 3, 1, 1, 0, False),
    "k3s1_rows16x1": (16, 32, 5, 16, 32, 3, 1, 1, 0, False),
    "k3s1_rows8x2": (16, 64, 2, 8, 64, 3, 1, 1, 0, False),
    "k4s2T_128_64": (16, 128, 32, 64, 64, 4, 2, 1, 0, True),
    "k3s2T_256_128": (16, 256, 8, 32, 128, 3, 2, 1, 1, True),
}


@pytest.mark.parametrize("dt", [2, 1])
@pytest.mark.parametrize("case", sorted(RING))
def test_wgrad_ring_equals_fp32_storage(cuda, case, dt):
    from ldm_amd import ops
    B, Cin, H, W, Cout, k, s, p, op, tr = RING[case]
    desc = ops.make_desc(B, Cin, H, W, Cout, k, k, s, p, op, tr)
    x16, x32 = _q(_rand((B, Cin, H, W), 21), dt)
    g16, g32 = _q(_rand((B, Cout, desc.Hout, desc.Wout), 22), dt)
    assert ops.wgrad_storage16(desc, dt), case
    dw32 = ops.conv_backward_weight(x32.to(cuda), g32.to(cuda), desc, dtype=dt)
    dw16 = ops.conv_backward_weight(x16.to(cuda), g16.to(cuda), desc, dtype=dt)
    torch.cuda.synchronize()
    assert torch.equal(dw16, dw32), float((dw16 - dw32).abs().max())


@pytest.mark.parametrize("k", [3, 4])
def test_cin1_and_cout1_store16(cuda, k):
    """The Cin = 1 first layers (16-bit output), the 64 -> 1 output convT (16-bit input), the data gradient of
    the latter (a Cin = 1 conv: 16-bit output) and the one-channel weight gradients (16-bit Dense)."""
    from ldm_amd import ops
    dt = 2
    x = _rand((4, 1, 64, 256), 21)                      # fp32 mel
    w1 = _rand((64, 1, k, k), 22, -0.3, 0.3).to(cuda)
    b1 = _rand((64,), 23, -0.1, 0.1).to(cuda)
    kw = dict(stride=2, padding=1, act="relu", dtype=dt)
    y32 = ops.conv_forward(x.to(cuda), w1, b1, **kw)
    y16 = ops.conv_forward(x.to(cuda), w1, b1, out_dtype=T[dt], **kw)
    torch.cuda.synchronize()
    _same(y16, y32, dt)
    d1 = ops.make_desc(4, 1, 64, 256, 64, k, k, 2, 1)
    g16, g32 = _q(_rand(tuple(y32.shape), 24), dt)
    assert ops.wgrad_storage16(d1, dt) & 0x800
    assert torch.equal(ops.conv_backward_weight(x.to(cuda), g16.to(cuda), d1, dtype=dt),
                       ops.conv_backward_weight(x.to(cuda), g32.to(cuda), d1, dtype=dt))
    # decoder output layer: convT 64 -> 1, k4 s2 p1, tanh
    h16, h32 = _q(_rand((4, 64, 32, 128), 25, 0.0, 1.0), dt)
    w2 = _rand((64, 1, 4, 4), 26, -0.2, 0.2).to(cuda)
    b2 = _rand((1,), 27, -0.1, 0.1).to(cuda)
    kt = dict(stride=2, padding=1, transposed=True, act="tanh", dtype=dt)
    o32 = ops.conv_forward(h32.to(cuda), w2, b2, **kt)
    o16 = ops.conv_forward(h16.to(cuda), w2, b2, **kt)
    torch.cuda.synchronize()
    assert o16.dtype == torch.float32 and torch.equal(o16, o32)
    d2 = ops.make_desc(4, 64, 32, 128, 1, 4, 4, 2, 1, 0, True)
    r = _rand(tuple(o32.shape), 28).to(cuda)
    _same(ops.conv_backward_data(r, w2, d2, dtype=dt, out_dtype=T[dt]), ops.conv_backward_data(r, w2, d2, dtype=dt), dt)
    assert torch.equal(ops.conv_backward_weight(h16.to(cuda), r, d2, dtype=dt),
                       ops.conv_backward_weight(h32.to(cuda), r, d2, dtype=dt))


def test_cin1_cout1_with_skip_fall_back_to_fp32_maps(cuda):
    """The 16-bit VALU convs run only with a simple epilogue: a Cin = 1 stride-2 conv asked for a 16-bit output
    with a skip / broadcast add, and the 64 -> 1 convT handed a 16-bit input with a skip, take the general kernel
    on fp32 maps (an fp32 y) instead of failing, with the same values as the all-fp32 call."""
    from ldm_amd import ops
    dt = 2
    x = _rand((4, 1, 64, 256), 51).to(cuda)
    w1 = _rand((64, 1, 3, 3), 52, -0.3, 0.3).to(cuda)
    b1 = _rand((64,), 53, -0.1, 0.1).to(cuda)
    sk = _rand((4, 64, 32, 128), 54).to(cuda)
    bc = _rand((4, 64), 55).to(cuda)
    kw = dict(stride=2, padding=1, act="relu", dtype=dt)
    for extra in (dict(skip=sk), dict(bcast=bc)):
        ref = ops.conv_forward(x, w1, b1, **kw, **extra)
        got = ops.conv_forward(x, w1, b1, out_dtype=T[dt], **kw, **extra)
        torch.cuda.synchronize()
        assert got.dtype == torch.float32 and torch.equal(got, ref)
    h16, h32 = _q(_rand((4, 64, 32, 128), 56, 0.0, 1.0), dt)
    w2 = _rand((64, 1, 4, 4), 57, -0.2, 0.2).to(cuda)
    sk2 = _rand((4, 1, 64, 256), 58).to(cuda)
    kt = dict(stride=2, padding=1, transposed=True, act="tanh", dtype=dt, skip=sk2)
    ref = ops.conv_forward(h32.to(cuda), w2, None, **kt)
    got = ops.conv_forward(h16.to(cuda), w2, None, **kt)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


class _StubGroup:
    """A world-1 stand-in for a SyncBatchNorm group: the two-stage kernels with an identity all-reduce."""

    def ldm_allreduce_sum(self, t):
        pass


@pytest.mark.parametrize("sync", [False, True])
@pytest.mark.parametrize("act", ["relu", "none"])
def test_batchnorm_store16(cuda, act, sync):
    from ldm_amd import ops
    dt = 2
    B, C, H, W = 4, 64, 32, 64
    x16, x32 = _q(_rand((B, C, H, W), 31, -2.0, 3.0), dt)
    w = _rand((C,), 32, 0.5, 1.5).to(cuda)
    b = _rand((C,), 33, -0.2, 0.2).to(cuda)
    grp = _StubGroup() if sync else False
    outs = {}
    for name, xin in (("32", x32), ("16", x16)):
        rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
        xd = xin.to(cuda)
        y = torch.empty_like(xd)
        sm, si = ops.batchnorm_train_(xd, w, b, rm, rv, 0.1, 1e-5, act, save=True, sync=grp, out=y)
        outs[name] = (xd, y, sm, si, rm, rv)
    torch.cuda.synchronize()
    _same(outs["16"][1], outs["32"][1], dt)
    for i in (2, 3, 4, 5):
        assert torch.equal(outs["16"][i], outs["32"][i]), i
    g16, g32 = _q(_rand((B, C, H, W), 34), dt)
    r32 = ops.batchnorm_backward(g32.to(cuda), None, outs["32"][0], outs["32"][2], outs["32"][3], w, act, sync=grp, bias=b)
    r16 = ops.batchnorm_backward(g16.to(cuda), None, outs["16"][0], outs["16"][2], outs["16"][3], w, act, sync=grp, bias=b)
    torch.cuda.synchronize()
    _same(r16[0], r32[0], dt)
    assert torch.equal(r16[1], r32[1]) and torch.equal(r16[2], r32[2])


@pytest.mark.parametrize("shape", [(4, 64, 32, 64), (8, 32, 16, 16), (32, 64, 3, 3)])
def test_act_backward_store16(cuda, shape):
    """The sliced, per-plane and small-plane activation-backward kernels with 16-bit dy / act_out / dv."""
    from ldm_amd import ops
    dt = 2
    a16, a32 = _q(torch.relu(_rand(shape, 41)), dt)
    g16, g32 = _q(_rand(shape, 42), dt)
    dv32, db32, dc32 = ops.act_backward(g32.to(cuda), "relu", act_out=a32.to(cuda), need_bias=True, need_bcast=True)
    dv16, db16, dc16 = ops.act_backward(g16.to(cuda), "relu", act_out=a16.to(cuda), need_bias=True, need_bcast=True)
    torch.cuda.synchronize()
    _same(dv16, dv32, dt)
    assert torch.equal(db16, db32) and torch.equal(dc16, dc32)


def test_store16_policy():
    """Which maps are stored in 16 bits: >= LDM_AMD_STORE16_MIN elements at a 16-bit operand precision."""
    from ldm_amd import ops
    assert ops.store16_dtype(1 << 22, 2) == torch.bfloat16
    assert ops.store16_dtype(1 << 22, 1) == torch.float16
    assert ops.store16_dtype((1 << 22) - 1, 2) == torch.float32
    assert ops.store16_dtype(1 << 24, 0) == torch.float32


@pytest.mark.parametrize("which", ["x16", "dy16"])
def test_wgrad_mixed_maps(cuda, which):
    """A weight gradient with one 16-bit and one fp32 map (the VAE's third layer: 16-bit input, fp32 output
    gradient; the decoder's first layer the other way round): the fp32 map is rounded to the operand type
    first, as the kernel rounds it, so the result equals the all-fp32-storage form."""
    from ldm_amd import ops
    dt = 2
    B, Cin, H, W, Cout = 2, 64, 32, 128, 32
    desc = ops.make_desc(B, Cin, H, W, Cout, 3, 3, 2, 1)
    x16, x32 = _q(_rand((B, Cin, H, W), 61), dt)
    g = _rand((B, Cout, desc.Hout, desc.Wout), 62)
    g16, g32 = _q(g, dt)
    ref = ops.conv_backward_weight(x32.to(cuda), g32.to(cuda), desc, dtype=dt)
    if which == "x16":
        got = ops.conv_backward_weight(x16.to(cuda), g.to(cuda), desc, dtype=dt)   # dy fp32, rounded inside
    else:
        got = ops.conv_backward_weight(_rand((B, Cin, H, W), 61).to(cuda), g16.to(cuda), desc, dtype=dt)   # x fp32
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


@pytest.mark.parametrize("dt", [0, 2])
@pytest.mark.parametrize("k", [3, 4])
def test_cin1_packed_form_is_bitwise_the_scalar_form(cuda, k, dt):
    """conv_cin1_x4_kernel's packed form (two output channels per v_pk_fma_f32, each half an fma exactly as
    v_fma_f32 rounds it, the same (ky, kx) order per output) against the scalar form, bitwise: the VAE / style
    encoders' first layers (fp32 and bf16 operands, 16-bit output under bf16) and the data gradient of the decoder's
    64 -> 1 output convT (a Cin = 1 conv); plus the fp32 form against float64 torch (1e-5).  Reference layers:
    model.py:17 (Conv2d(1, 64, 3, 2, 1)), model.py:49 (ConvTranspose2d(64, 1, 4, 2, 1))."""
    from ldm_amd import _lib as L, ops
    lib = L.load()
    x = _rand((4, 1, 64, 256), 41 + k)
    w1 = _rand((64, 1, k, k), 42, -0.3, 0.3).to(cuda)
    b1 = _rand((64,), 43, -0.1, 0.1).to(cuda)
    kw = dict(stride=2, padding=1, act="relu", dtype=dt)
    if dt:
        kw["out_dtype"] = T[dt]
    d2 = ops.make_desc(4, 64, 32, 128, 1, 4, 4, 2, 1, 0, True)
    w2 = _rand((64, 1, 4, 4), 44, -0.2, 0.2).to(cuda)
    r = _rand((4, 1, 64, 256), 45).to(cuda)
    outs = []
    prev = lib.ldm_set_cin1_packed(0)
    try:
        for pk in (0, 1):
            lib.ldm_set_cin1_packed(pk)
            y = ops.conv_forward(x.to(cuda), w1, b1, **kw)
            dx = ops.conv_backward_data(r, w2, d2, dtype=dt)
            torch.cuda.synchronize()
            outs.append((y, dx))
    finally:
        lib.ldm_set_cin1_packed(prev)
    (y0, dx0), (y1, dx1) = outs
    assert torch.equal(y0, y1), float((y0.float() - y1.float()).abs().max())
    assert torch.equal(dx0, dx1), float((dx0 - dx1).abs().max())
    if dt == 0:
        import torch.nn.functional as F
        y64 = torch.relu(F.conv2d(x.double(), w1.cpu().double(), b1.cpu().double(), stride=2, padding=1))
        assert float((y1.cpu().double() - y64).abs().max()) <= 1e-5 * float(y64.abs().max())


@pytest.mark.parametrize("store16", [False, True])
def test_conv_bias_grad_from_batchnorm_dx_sum(cuda, store16, monkeypatch):
    """conv -> train-mode BatchNorm + ReLU (the VAE blocks, model.py:16-25, as models.model._conv_bn_act runs them):
    the BN backward sums its dx per channel as it writes it (ldm_batchnorm_backward_dxsum) and the conv's backward
    takes that sum as its bias gradient instead of sweeping dx again.  It equals the sum of the gradient reaching the
    conv output (a tensor hook) to fp32 summation order, 16-bit storage included; LDM_AMD_BN_DXSUM=0 runs the sweep."""
    from ldm_amd import functional as HF
    if store16:
        monkeypatch.setenv("LDM_AMD_STORE16_MIN", "1")
    conv = torch.nn.Conv2d(64, 128, 3, stride=2, padding=1).to(cuda)
    bn = torch.nn.BatchNorm2d(128).to(cuda).train()
    x = _rand((4, 64, 64, 128), 902).to(cuda)
    gy = _rand((4, 128, 32, 64), 903).to(cuda)
    res = []
    for flag in ("1", "0"):
        monkeypatch.setenv("LDM_AMD_BN_DXSUM", flag)
        conv.zero_grad()
        seen = {}
        before = HF.STATS["conv_bias_from_bn"]
        ctx = torch.autocast("cuda", dtype=torch.bfloat16) if store16 else torch.autocast("cuda", enabled=False)
        with ctx:
            y = HF.conv(x, conv.weight, conv.bias, stride=2, padding=1, act="none")
            y.register_hook(lambda g: seen.__setitem__("g", g))
            z = HF.batchnorm(y, bn, "relu")
        (z.float() * gy).sum().backward()
        torch.cuda.synchronize()
        took = HF.STATS["conv_bias_from_bn"] - before
        g = seen["g"].float()
        want = g.sum((0, 2, 3))
        got = conv.bias.grad.clone()
        scale = float(g.abs().sum((0, 2, 3)).max())
        assert float((got - want).abs().max()) <= 1e-5 * scale, (flag, float((got - want).abs().max()), scale)
        res.append(took)
    assert res[0] > 0 and res[1] == 0


@pytest.mark.parametrize("dt", [0, 2])
@pytest.mark.parametrize("cout", [32, 64])
def test_cin1_stride1_form_is_bitwise_the_pixel_kernel(cuda, cout, dt):
    """The Cin = 1, k3, stride-1 conv (the UNet's first layer on the raw mel, UNet(1, 1) at shape S;
    models/model.py:178 Conv2d(in_channels, num_filters, 3, 1, 1)) on conv_cin1_x4_kernel's stride-1 form (four
    output columns per lane from one 3 x 6 window) against conv_cin1_kernel (one lane per pixel), bitwise, with the
    packed and scalar channel walks, fp32 and bf16 operands; the fp32 form against float64 torch (1e-5); and a width
    that is not a multiple of 4 (the pixel kernel) against float64 torch."""
    from ldm_amd import _lib as L, ops
    import torch.nn.functional as F
    lib = L.load()
    x = _rand((2, 1, 64, 256), 71).to(cuda)
    w = _rand((cout, 1, 3, 3), 72, -0.3, 0.3).to(cuda)
    b = _rand((cout,), 73, -0.1, 0.1).to(cuda)
    kw = dict(stride=1, padding=1, act="relu", dtype=dt)
    outs = []
    prev_s1, prev_pk = lib.ldm_set_cin1_s1(0), lib.ldm_set_cin1_packed(1)
    try:
        for s1, pk in ((0, 1), (1, 0), (1, 1)):
            lib.ldm_set_cin1_s1(s1)
            lib.ldm_set_cin1_packed(pk)
            outs.append(ops.conv_forward(x, w, b, **kw))
            torch.cuda.synchronize()
    finally:
        lib.ldm_set_cin1_s1(prev_s1)
        lib.ldm_set_cin1_packed(prev_pk)
    for y in outs[1:]:
        assert torch.equal(y, outs[0]), float((y.float() - outs[0].float()).abs().max())
    if dt == 0:
        y64 = torch.relu(F.conv2d(x.cpu().double(), w.cpu().double(), b.cpu().double(), stride=1, padding=1))
        assert float((outs[-1].cpu().double() - y64).abs().max()) <= 1e-5 * float(y64.abs().max())
        xr = _rand((2, 1, 20, 130), 74).to(cuda)   # Wout = 130: not a multiple of 4
        yr = ops.conv_forward(xr, w, b, **kw)
        torch.cuda.synchronize()
        y64 = torch.relu(F.conv2d(xr.cpu().double(), w.cpu().double(), b.cpu().double(), stride=1, padding=1))
        assert float((yr.cpu().double() - y64).abs().max()) <= 1e-5 * float(y64.abs().max())
