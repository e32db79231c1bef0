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

    grad (our gradient, recommended): where its sign agrees with the reference gradient's, the update must
    agree too, however small g is; a sign disagreement is allowed only inside the fp32 gradient noise
    (|g_ref| <= rel x max|g_ref|), and only there may an element move the other way (held to 2 lr).
    Without grad, every element below the noise level is held to 2 lr only.  Returns the rel_err of the
    elements that must agree."""
    new = np.asarray(new, dtype=np.float64)
    ref_new = np.asarray(ref_new, dtype=np.float64)
    gr = np.asarray(grad_ref, dtype=np.float64)
    big = np.abs(gr) > rel * np.abs(gr).max()
    must = big
    if grad is not None:
        g = np.asarray(grad, dtype=np.float64)
        # (|g| well above Adam's eps = 1e-8, where the step is lr * sign(g) whatever the magnitude)
        agree = (np.sign(g) == np.sign(gr)) & (np.minimum(np.abs(g), np.abs(gr)) > 1e-6)
        assert not np.any(~agree & big), "a gradient above the noise level has the wrong sign"
        must = big | agree
    free = ~must
    small_ok = bool(np.all(np.abs(new - ref_new)[free] <= 2.0 * lr * (1 + 1e-3) + 1e-7))
    assert small_ok, "an element moved by more than one Adam step"
    if not must.any():
        return 0.0
    return float(np.abs(new - ref_new)[must].max() / max(np.abs(ref_new).max(), 1e-30))
