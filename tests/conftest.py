import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "music-style-transfer-ldm_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def goldens():
    return np.load(os.path.join(ROOT, "tests", "golden", "ref_goldens.npz"))


@pytest.fixture(scope="session")
def goldens2():
    """Round-2 fixtures (make_goldens.py --r2): content/style transfer wrapper, one autoencoder step."""
    return np.load(os.path.join(ROOT, "tests", "golden", "ref_goldens_r2.npz"))


@pytest.fixture(scope="session")
def goldens_vgg():
    """VGGishFeatureLoss.forward of the reference on recipe-filled VGGish-shaped stacks (make_goldens.py --vggish)."""
    return np.load(os.path.join(ROOT, "tests", "golden", "ref_goldens_vggish.npz"))


VGG_CASES = {"a": ((2, 1, 32, 64), 800), "odd": ((2, 1, 20, 36), 810)}   # as make_goldens.VGG_CASES


AE_KEYS = ("encoder.encoder.0.weight", "encoder.encoder.1.weight", "encoder.encoder.4.bias", "encoder.encoder.6.bias",
           "encoder.encoder.7.weight", "decoder.decoder.0.weight", "decoder.decoder.1.bias", "decoder.decoder.4.weight",
           "decoder.decoder.6.weight", "decoder.decoder.6.bias")


def rel_err(y, ref):
    """max |y - ref| / max |ref|  — the parity metric (tolerance stated per test)."""
    y = np.asarray(y, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert y.shape == ref.shape, (y.shape, ref.shape)
    den = max(np.abs(ref).max(), 1e-30)
    return float(np.abs(y - ref).max() / den)


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def adam_step_err(new, ref_new, grad_ref, lr, rel=1e-3, grad=None):
    """Parity of one Adam/AdamW first step, which moves each element by ~lr * sign(g).

    Elements whose reference gradient is above the fp32 noise (|g_ref| > rel x max|g_ref|) must agree to the
    returned rel_err.  Below it an element may legitimately step the other way, so it is held to 2 lr; with
    `grad` (our gradient) given, a sign flip above the noise fails outright, and a below-noise element whose
    gradient sign agrees with the reference's is held to 1 lr (both steps point the same way)."""
    new = np.asarray(new, dtype=np.float64)
    ref_new = np.asarray(ref_new, dtype=np.float64)
    gr = np.asarray(grad_ref, dtype=np.float64)
    big = np.abs(gr) > rel * np.abs(gr).max()
    bound = np.full(gr.shape, 2.0 * lr)
    if grad is not None:
        g = np.asarray(grad, dtype=np.float64)
        same = np.sign(g) == np.sign(gr)
        assert not np.any(~same & big), "a gradient above the noise level has the wrong sign"
        bound[same] = lr
    free = ~big
    small_ok = bool(np.all(np.abs(new - ref_new)[free] <= bound[free] * (1 + 1e-3) + 1e-7))
    assert small_ok, "a below-noise element moved further than its gradient signs allow"
    if not big.any():
        return 0.0
    return float(np.abs(new - ref_new)[big].max() / max(np.abs(ref_new).max(), 1e-30))
