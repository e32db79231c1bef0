"""GPU parity of the VGGish feature / style loss path (reference loss.py:52-101) on the
HIP kernels: ldm_maxpool2x2 against torch's max_pool2d (bit-exact: a max is exact), the one-pass
std-normalised MSE against float64 torch, and VGGishFeatureLoss end to end against the golden captured
from the REFERENCE's forward on the same recipe-filled VGGish-shaped stack (1e-4 relative; the real
VGGish weights are a remote download, so parity is pinned on recipe weights only)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as tF

import recipe
from conftest import VGG_CASES, rel_err

pytestmark = pytest.mark.gpu


def _rand(shape, seed, lo=-1.0, hi=1.0):
    g = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(g.uniform(lo, hi, shape).astype(np.float32))


@pytest.mark.parametrize("shape", [(2, 3, 8, 16), (1, 4, 7, 9), (3, 2, 6, 10), (2, 64, 128, 512)])
def test_maxpool2x2_bitexact(cuda, shape):
    from ldm_amd import ops
    x = _rand(shape, sum(shape))
    if shape[2] >= 4:
        x[0, 0, 1, 1] = float("nan")   # NaN propagates like torch
    y = ops.maxpool2x2(x.to(cuda))
    ref = tF.max_pool2d(x, 2, 2)
    assert y.shape == ref.shape
    assert torch.equal(torch.isnan(y.cpu()), torch.isnan(ref))
    m = ~torch.isnan(ref)
    assert torch.equal(y.cpu()[m], ref[m])


@pytest.mark.parametrize("shape", [(2, 64, 16, 32), (3, 5, 7, 9), (1, 512, 2, 4)])
def test_std_mse_against_float64(cuda, shape):
    from ldm_amd import ops
    p = _rand(shape, 3, 0, 2)
    t = _rand(shape, 4, 0, 1.5)
    acc = torch.zeros(1, device=cuda, dtype=torch.float64)
    out = torch.empty((), device=cuda)
    ops.std_mse_accumulate(p.to(cuda), t.to(cuda), acc, 0.5, out=out)
    pd, td = p.double(), t.double()
    pn = pd / (torch.std(pd, dim=[1, 2, 3], keepdim=True) + 1e-8)
    tn = td / (torch.std(td, dim=[1, 2, 3], keepdim=True) + 1e-8)
    ref = 0.5 * tF.mse_loss(pn, tn)
    assert abs(float(acc) - float(ref)) <= 1e-9 * abs(float(ref))
    assert abs(float(out) - float(ref)) <= 1e-6 * abs(float(ref))


@pytest.mark.parametrize("case", sorted(VGG_CASES))
def test_vggish_feature_loss_matches_reference(cuda, goldens_vgg, case):
    from models.loss import VGGishFeatureLoss, vggish_features
    shape, seed = VGG_CASES[case]
    feats = vggish_features()
    recipe.fill_module(feats, seed=seed)
    loss = VGGishFeatureLoss(feats.to(cuda))
    p = torch.from_numpy(recipe.uniform01(shape, seed + 1)).to(cuda)
    t = torch.from_numpy(recipe.uniform01(shape, seed + 2)).to(cuda)
    out = loss(p, t)
    assert out.shape == () and out.dtype == torch.float32
    assert rel_err(out.item(), goldens_vgg[f"vgg_{case}_loss"]) < 1e-4
    assert torch.equal(loss(p, t), out)   # fixed-order reductions: bitwise reproducible


def test_vggish_loss_zero_without_weights(cuda):
    import models.loss as ML
    from models.loss import VGGishFeatureLoss
    ML._WARNED.discard("vggish")
    x = torch.rand(1, 1, 16, 16, device=cuda)
    with pytest.warns(RuntimeWarning):
        assert float(VGGishFeatureLoss()(x, x)) == 0.0
