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


def adam_step_err(new, ref_new, grad_ref, lr, rel=1e-3):
    """Parity of one Adam/AdamW first step.  The first step moves each element by ~lr * g / (|g| + eps):
    elements whose reference gradient is below `rel` x max|g| sit inside fp32 gradient noise and may move
    the other way, so they are only held to 2 lr; the rest must agree to the returned rel_err."""
    new = np.asarray(new, dtype=np.float64)
    ref_new = np.asarray(ref_new, dtype=np.float64)
    g = np.abs(np.asarray(grad_ref, dtype=np.float64))
    big = g > rel * g.max()
    small_ok = bool(np.all(np.abs(new - ref_new)[~big] <= 2.0 * lr * (1 + 1e-3) + 1e-7))
    assert small_ok, "an element moved by more than one Adam step"
    if not big.any():
        return 0.0
    return float(np.abs(new - ref_new)[big].max() / max(np.abs(ref_new).max(), 1e-30))
