"""Weight gradient of a 1x1 conv (the cross-attention in-projections at the train batch: backward.hip
wgrad_1x1_kernel) against float64 torch: dW[m][c] = sum_{b,n} dy[b][m][n] x[b][c][n] of the operands as the
kernel sees them (fp32, or rounded to fp16 / bf16 inside an autocast region), tolerance 1e-5 of max |dW|
(fp32 sums over K = B*HW <= 2048), accumulate mode, and run-to-run bitwise equality.  Reference semantics:
nn.MultiheadAttention's in-projection weight gradient (model.py:126-160, reached through train.py:163-208)."""
import numpy as np
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu


def _rand(shape, seed):
    g = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(g.uniform(-1.0, 1.0, shape).astype(np.float32))


@pytest.mark.parametrize("dt", [0, 2, 1])
@pytest.mark.parametrize("shape", [(32, 512, 1024, 2, 8), (32, 256, 512, 4, 16), (3, 64, 96, 4, 4)])
def test_wgrad_1x1(cuda, shape, dt):
    from ldm_amd import ops
    B, Cin, Cout, H, W = shape
    x = _rand((B, Cin, H, W), 1)
    dy = _rand((B, Cout, H, W), 2)
    desc = ops.make_desc(B, Cin, H, W, Cout, 1, 1, 1, 0)
    dw = ops.conv_backward_weight(x.to(cuda), dy.to(cuda), desc, dtype=dt)
    dw2 = ops.conv_backward_weight(x.to(cuda), dy.to(cuda), desc, dtype=dt)
    base = torch.full_like(dw, 0.5)
    acc = base.clone()
    ops.conv_backward_weight(x.to(cuda), dy.to(cuda), desc, dw=acc, accumulate=True, dtype=dt)
    torch.cuda.synchronize()
    rnd = {0: lambda t: t.double(), 1: lambda t: t.half().double(), 2: lambda t: t.bfloat16().double()}[dt]
    ref = torch.einsum("bmn,bcn->mc", rnd(dy).reshape(B, Cout, -1), rnd(x).reshape(B, Cin, -1))
    got = dw.double().cpu().reshape(Cout, Cin)
    assert rel_err(got.numpy(), ref.numpy()) < 1e-5
    assert torch.equal(dw, dw2)
    assert torch.equal(acc, base + dw)
