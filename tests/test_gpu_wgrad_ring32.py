"""The fp32-map weight gradient on its LDS-DMA chunk ring (csrc/wgrad.hip wgrad_lpp_kernel, round 6): the train
step's UNet-level layers (maps below the 16-bit storage threshold stay fp32; reference layers model.py:178-194,
their gradients under train.py:174's autocast) at bf16 / fp16 operand precision.

* against float64 of the identically rounded operands (the weight gradient of a conv is the correlation of the
  input with the output gradient): max |dw - dw64| <= 1e-5 max |dw64|;
* bitwise against the double-buffered form it replaces (wgrad_lp_kernel, LDM_WGRAD_RING=2, run in a child
  process): same blocks, chunks, k-steps and MFMA order, so the same bits."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
T = {1: torch.float16, 2: torch.bfloat16}
CASES = {   # (B, Cin, H, W, Cout, k, stride, pad, out_pad, transposed): UNet layers at the canonical latent
    "enc2_64_128_s2": (8, 64, 16, 64, 128, 3, 2, 1, 0, False),
    "enc3_128_256_s2": (8, 128, 8, 32, 256, 3, 2, 1, 0, False),
    "enc4_256_512_s2": (8, 256, 4, 16, 512, 3, 2, 1, 0, False),
    "bneck_512_s1": (8, 512, 2, 8, 512, 3, 1, 1, 0, False),
    "enc1_32_64_s1": (8, 32, 16, 64, 64, 3, 1, 1, 0, False),
    "dec4_T_512_256": (8, 512, 2, 8, 256, 3, 2, 1, 1, True),
}


def _rand(shape, seed):
    g = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(g.uniform(-1.0, 1.0, shape).astype(np.float32))


def _dw(case, dt, dev):
    from ldm_amd import ops
    B, Cin, H, W, Cout, k, s, p, op, tr = CASES[case]
    desc = ops.make_desc(B, Cin, H, W, Cout, k, k, s, p, op, tr)
    x = _rand((B, Cin, H, W), 51).to(dev)
    g = _rand((B, Cout, desc.Hout, desc.Wout), 52).to(dev)
    dw = ops.conv_backward_weight(x, g, desc, dtype=dt)
    torch.cuda.synchronize()
    return x, g, dw


def _ref64(case, x, g, dt):
    import torch.nn.functional as F
    B, Cin, H, W, Cout, k, s, p, op, tr = CASES[case]
    xr = x.to(T[dt]).double().cpu().requires_grad_(True)
    gr = g.to(T[dt]).double().cpu()
    if tr:
        w = torch.zeros(Cin, Cout, k, k, dtype=torch.float64, requires_grad=True)
        y = F.conv_transpose2d(xr, w, stride=s, padding=p, output_padding=op)
    else:
        w = torch.zeros(Cout, Cin, k, k, dtype=torch.float64, requires_grad=True)
        y = F.conv2d(xr, w, stride=s, padding=p)
    (y * gr).sum().backward()
    return w.grad


@pytest.mark.parametrize("dt", [2, 1])
@pytest.mark.parametrize("case", sorted(CASES))
def test_wgrad_fp32_maps_ring_vs_float64(cuda, case, dt):
    x, g, dw = _dw(case, dt, cuda)
    ref = _ref64(case, x, g, dt)
    err = float((dw.double().cpu() - ref).abs().max()) / float(ref.abs().max())
    assert err <= 1e-5, err


def test_wgrad_fp32_maps_ring_bitwise_double_buffered(cuda, tmp_path):
    out = tmp_path / "db.pt"
    code = ("import sys, torch; sys.path[:0] = [%r, %r, %r]; import test_gpu_wgrad_ring32 as m; "
            "torch.save({c: m._dw(c, 2, torch.device('cuda:0'))[2].cpu() for c in sorted(m.CASES)}, %r)"
            % (ROOT, os.path.join(ROOT, "music-style-transfer-ldm_amd"), os.path.join(ROOT, "tests"), str(out)))
    env = dict(os.environ, LDM_WGRAD_RING="2")
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=240)
    db = torch.load(str(out), weights_only=True)
    for c in sorted(CASES):
        dw = _dw(c, 2, cuda)[2].cpu()
        assert torch.equal(dw, db[c]), (c, float((dw - db[c]).abs().max()))
