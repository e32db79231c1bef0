"""Deterministic weight / input recipe shared by the golden generator and the tests.

Test infrastructure only. Both the reference modules (when the goldens are made, in the
build container) and this repo's modules (when the goldens are checked, on the GPU box)
are filled from the same PCG64 streams, so no weight file has to be committed.

Rules (keyed on the state_dict name and shape, iterated in sorted-key order):
  * ``*.num_batches_tracked``            -> 0
  * ``*.running_mean``                   -> U(-0.2, 0.2)
  * ``*.running_var``                    -> U(0.5, 1.5)
  * 1-D ``*weight`` (BatchNorm gamma)    -> U(0.5, 1.5)
  * 1-D bias-like tensors                -> U(-0.1, 0.1)
  * >=2-D tensors                        -> U(-b, b), b = sqrt(3 / prod(shape[1:]))
  * ``noise_scheduler.*`` buffers are left untouched (they are computed, not learned).
"""
import math

import numpy as np

SKIP_PREFIXES = ("noise_scheduler.", "feature_loss_net.")


def _gen(seed):
    return np.random.Generator(np.random.PCG64(seed))


def make_state(shapes, seed=0):
    """shapes: dict name -> tuple. Returns dict name -> float32/int64 numpy array."""
    g = _gen(seed)
    out = {}
    for name in sorted(shapes):
        shape = tuple(shapes[name])
        if name.startswith(SKIP_PREFIXES):
            continue
        if name.endswith("num_batches_tracked"):
            out[name] = np.zeros(shape, dtype=np.int64)
            continue
        n = int(np.prod(shape)) if shape else 1
        if name.endswith("running_mean"):
            v = g.uniform(-0.2, 0.2, n)
        elif name.endswith("running_var"):
            v = g.uniform(0.5, 1.5, n)
        elif len(shape) == 1 and name.endswith("weight"):
            v = g.uniform(0.5, 1.5, n)
        elif len(shape) <= 1:
            v = g.uniform(-0.1, 0.1, n)
        else:
            b = math.sqrt(3.0 / float(np.prod(shape[1:])))
            v = g.uniform(-b, b, n)
        out[name] = v.astype(np.float32).reshape(shape)
    return out


def fill_module(module, seed=0):
    """Fill a torch module's parameters/buffers in place from the recipe."""
    import torch

    sd = module.state_dict()
    vals = make_state({k: tuple(v.shape) for k, v in sd.items()}, seed)
    with torch.no_grad():
        for k, v in vals.items():
            t = sd[k]
            t.copy_(torch.from_numpy(v).to(dtype=t.dtype, device=t.device))
    return vals


def uniform01(shape, seed):
    return _gen(seed).random(int(np.prod(shape))).astype(np.float32).reshape(shape)


def normal(shape, seed):
    return _gen(seed).standard_normal(int(np.prod(shape))).astype(np.float32).reshape(shape)


def timesteps(batch, seed, T=200):
    return _gen(seed).integers(0, T, batch).astype(np.int64)
