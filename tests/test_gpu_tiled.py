"""GPU parity of the LDS-staged 16-bit-operand conv (tconv.hip, plan kind 3): the path the train step's
large-plane layers (VAE encoder / decoder, style encoder, their data gradients) and the VGGish stack take
inside a torch.autocast(bf16 / fp16) region.  Reference: float64 torch conv / conv_transpose of the SAME
operands rounded to the 16-bit type (what the kernel multiplies; fp32 accumulation), tolerance 1e-5 of
max |y| (fp32 sums over K <= 1152 of exact 16-bit products), plus the fused epilogues and run-to-run
bitwise equality."""
import zlib

import numpy as np
import pytest
import torch
import torch.nn.functional as tF

from conftest import rel_err

pytestmark = pytest.mark.gpu

# (B, Cin, H, W, Cout, k, stride, pad, out_pad, transposed)
CASES = {
    "k3s1_64to128": (2, 64, 32, 64, 128, 3, 1, 1, 0, False),
    "k3s2_64to128": (4, 64, 64, 128, 128, 3, 2, 1, 0, False),
    "k4s2_128to64": (2, 128, 64, 128, 64, 4, 2, 1, 0, False),        # the decoder convT's data gradient
    "convT_k4_128to64": (2, 128, 32, 64, 64, 4, 2, 1, 0, True),       # decoder.3 class: 4 phases x 4 taps
    "convT_k3op1_64to32": (2, 64, 32, 64, 32, 3, 2, 1, 1, True),      # style-encoder dgrad class: 1/2/2/4 taps
    "ragged_32to40": (3, 32, 17, 97, 40, 3, 1, 1, 0, False),          # N % 128 != 0, Cout % 32 != 0
    # window-form geometries (tconvw_kernel): 128-position tiles of one output row (Wq = 128) or of R rows
    "w_k3s2_row128": (2, 64, 64, 256, 128, 3, 2, 1, 0, False),        # VAE / style enc2 class, Wq = 128
    "w_k3s2_cout32": (4, 128, 32, 128, 32, 3, 2, 1, 0, False),        # VAE enc3 class: 64-row tiles, Wq = 64
    "w_k3s2_wq16": (32, 64, 16, 32, 128, 3, 2, 1, 0, False),           # 8 rows of 16 per tile
    "w_k4s2_row128": (2, 128, 64, 256, 64, 4, 2, 1, 0, False),        # 16 taps, five register slots
    "w_k4s2_cout128": (2, 64, 64, 256, 128, 4, 2, 1, 0, False),       # 16 taps on the 128-row pack as 64-row tiles
    "w_convT_k4_row128": (2, 128, 32, 128, 64, 4, 2, 1, 0, True),     # decoder.3 class, phase grid Wq = 128
    "w_convT_k3op1_row128": (2, 64, 32, 128, 32, 3, 2, 1, 1, True),   # 1/2/2/4-tap phases, three launches
    "w_k3s1_cout256": (4, 32, 16, 64, 256, 3, 1, 1, 0, False),        # stride 1, two M tiles
}
EPIS = {"plain": {}, "bias_relu_actout": {"bias": True, "act": "relu", "act_out": True},
        "bn_relu": {"bias": True, "bn": True, "act": "relu"}, "tanh": {"act": "tanh"}}


def _rand(shape, seed, lo=-1.0, hi=1.0):
    g = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(g.uniform(lo, hi, shape).astype(np.float32))


@pytest.mark.parametrize("dt", [2, 1])
@pytest.mark.parametrize("epi", sorted(EPIS))
@pytest.mark.parametrize("case", sorted(CASES))
def test_tiled_conv(cuda, case, epi, dt):
    from ldm_amd import ops
    if dt == 1 and epi != "bias_relu_actout":
        pytest.skip("fp16: one epilogue per shape is enough")
    B, Cin, H, W, Cout, k, s, p, op, tr = CASES[case]
    e = EPIS[epi]
    seed = zlib.crc32((case + epi).encode()) % 1000
    x = _rand((B, Cin, H, W), seed)
    wshape = (Cin, Cout, k, k) if tr else (Cout, Cin, k, k)
    w = _rand(wshape, seed + 1, -0.1, 0.1)
    b = _rand((Cout,), seed + 2, -0.1, 0.1) if e.get("bias") else None
    bn = None
    if e.get("bn"):
        bn = (_rand((Cout,), seed + 3, 0.5, 1.5), _rand((Cout,), seed + 4, -0.1, 0.1),
              _rand((Cout,), seed + 5, -0.2, 0.2), _rand((Cout,), seed + 6, 0.5, 1.5), 1e-5)
    desc = ops.make_desc(B, Cin, H, W, Cout, k, k, s, p, op, tr)
    assert ops.tiled_plan(desc, dt) is not None, "the case must take the kind-3 path"
    tdt = torch.bfloat16 if dt == 2 else torch.float16
    xr, wr = x.to(tdt).double(), w.to(tdt).double()
    if tr:
        v = tF.conv_transpose2d(xr, wr, None if b is None else b.double(), stride=s, padding=p, output_padding=op)
    else:
        v = tF.conv2d(xr, wr, None if b is None else b.double(), stride=s, padding=p)
    if bn is not None:
        g_, be, m, var, eps = bn
        v = (v - m.double()[None, :, None, None]) / torch.sqrt(var.double()[None, :, None, None] + eps) \
            * g_.double()[None, :, None, None] + be.double()[None, :, None, None]
    act = e.get("act", "none")
    ref = {"none": lambda u: u, "relu": torch.relu, "tanh": torch.tanh}[act](v)
    dev = lambda t: None if t is None else t.to(cuda)   # noqa: E731
    aout = torch.empty(tuple(ref.shape), device=cuda) if e.get("act_out") else None
    bng = None if bn is None else tuple(dev(t) for t in bn[:4]) + (bn[4],)
    y = ops.conv_forward(dev(x), dev(w), dev(b), stride=s, padding=p, transposed=tr, output_padding=op, act=act,
                         bn=bng, act_out=aout, dtype=dt)
    y2 = ops.conv_forward(dev(x), dev(w), dev(b), stride=s, padding=p, transposed=tr, output_padding=op, act=act,
                          bn=bng, dtype=dt)
    torch.cuda.synchronize()
    assert y.shape == ref.shape
    assert rel_err(y.double().cpu().numpy(), ref.numpy()) < 1e-5
    assert torch.equal(y, y2)
    if aout is not None:
        assert torch.equal(aout, y)


def test_tiled_plan_classes(cuda, monkeypatch):
    """Which layers take the LDS-staged paths: 16-bit operands only, Cin % 32 == 0; kind 3 (tconv.hip) from 4096
    positions, kind 4 (sconv.hip, round 6) for the small planes under bf16 (fp16: the general kernel unless
    LDM_AMD_SCONV_F16=1)."""
    from ldm_amd import ops
    monkeypatch.delenv("LDM_AMD_SCONV_F16", raising=False)
    big = ops.make_desc(32, 128, 32, 128, 64, 4, 4, 2, 1, 0, True)        # decoder.3 at B = 32
    assert ops.tiled_plan(big, 2) is not None and ops.tiled_plan(big, 0) is None
    assert int(ops.tiled_plan(big, 2).kind) == 3
    unet = ops.make_desc(8, 256, 4, 16, 512, 3, 3, 2, 1)                   # UNet-sized
    assert int(ops.tiled_plan(unet, 2).kind) == 4                            # bf16: sconv.hip
    assert ops.tiled_plan(unet, 1) is None                                   # fp16: general
    assert ops.tiled_plan(ops.make_desc(32, 1, 128, 512, 64, 3, 3, 2, 1), 2) is None      # Cin = 1: x4 kernel
    assert ops.tiled_plan(ops.make_desc(32, 48, 64, 64, 64, 3, 3, 1, 1), 2) is None       # Cin % 32 != 0


@pytest.mark.parametrize("shape", [(2, 64, 64, 256), (3, 64, 8, 16), (5, 8, 6, 12), (2, 12, 6, 8), (2, 16, 5, 8)])
@pytest.mark.parametrize("act", ["none", "tanh"])
def test_convT_cout1(cuda, shape, act):
    """The decoder's 64 -> 1 output convT (k4 s2 p1; model.py:44) on its own kernels (conv.hip): channel
    quarters over a block's four waves (Cin % 8 == 0, Hin even), two input rows per lane (other even Hin),
    one row (odd Hin).  fp32 against float64 torch, 1e-5 of max |y|, run-to-run bitwise."""
    from ldm_amd import ops
    B, Cin, H, W = shape
    seed = B * 1000 + Cin * 10 + H
    x = _rand((B, Cin, H, W), seed)
    w = _rand((Cin, 1, 4, 4), seed + 1, -0.2, 0.2)
    b = _rand((1,), seed + 2, -0.1, 0.1)
    v = tF.conv_transpose2d(x.double(), w.double(), b.double(), stride=2, padding=1)
    ref = torch.tanh(v) if act == "tanh" else v
    y = ops.conv_forward(x.to(cuda), w.to(cuda), b.to(cuda), stride=2, padding=1, transposed=True, act=act)
    y2 = ops.conv_forward(x.to(cuda), w.to(cuda), b.to(cuda), stride=2, padding=1, transposed=True, act=act)
    torch.cuda.synchronize()
    assert y.shape == ref.shape
    assert rel_err(y.double().cpu().numpy(), ref.numpy()) < 1e-5
    assert torch.equal(y, y2)


@pytest.mark.parametrize("case", sorted(c for c in CASES if c.startswith("w_")) + ["k3s1_64to128", "k4s2_128to64"])
def test_tiled_conv_window_vs_gather(cuda, case, monkeypatch):
    """The window form (tconvw_kernel) and the per-chunk gather form (tconv_kernel, LDM_TCONV_WIN=0) of the
    same kind-3 plan: both within 1e-5 of float64 of the bf16-rounded operands, and of each other (they sum K
    in different orders).  The env switch is read once per process, so the gather form runs in a child."""
    import os
    import subprocess
    import sys
    from ldm_amd import ops
    B, Cin, H, W, Cout, k, s, p, op, tr = CASES[case]
    x = _rand((B, Cin, H, W), 5)
    w = _rand((Cin, Cout, k, k) if tr else (Cout, Cin, k, k), 6, -0.1, 0.1)
    y = ops.conv_forward(x.to(cuda), w.to(cuda), None, stride=s, padding=p, transposed=tr, output_padding=op, dtype=2)
    xr, wr = x.to(torch.bfloat16).double(), w.to(torch.bfloat16).double()
    ref = tF.conv_transpose2d(xr, wr, stride=s, padding=p, output_padding=op) if tr else tF.conv2d(xr, wr, stride=s, padding=p)
    assert rel_err(y.double().cpu().numpy(), ref.numpy()) < 1e-5
    here = os.path.dirname(os.path.abspath(__file__))
    code = ("import sys, torch, numpy as np; sys.path.insert(0, %r); import conftest, test_gpu_tiled as t; "
            "from ldm_amd import ops; c = t.CASES[%r]; B, Cin, H, W, Cout, k, s, p, op, tr = c; "
            "x = t._rand((B, Cin, H, W), 5); w = t._rand((Cin, Cout, k, k) if tr else (Cout, Cin, k, k), 6, -0.1, 0.1); "
            "y = ops.conv_forward(x.cuda(), w.cuda(), None, stride=s, padding=p, transposed=tr, output_padding=op, "
            "dtype=2); np.save(sys.argv[1], y.double().cpu().numpy())" % (here, case))
    out = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"tcw_{case}_{os.getpid()}.npy")
    env = dict(os.environ, LDM_TCONV_WIN="0")
    r = subprocess.run([sys.executable, "-c", code, out], env=env, cwd=here, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    y_gather = np.load(out)
    os.remove(out)
    assert rel_err(y_gather, ref.numpy()) < 1e-5
    assert rel_err(y.double().cpu().numpy(), y_gather) < 1e-5

