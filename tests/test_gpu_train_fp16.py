"""The reference's DEFAULT train-step precision: LDMTrainer.train_step under torch.autocast on the device with
no dtype (float16 on a GPU, reference train.py:174) and its GradScaler (train.py:157, :189-201), against the
reference's own fp16 + GradScaler step (tests/golden/ref_goldens_fp16.npz, make_goldens.py --fp16train) at
config 3's shape and inputs (batch 32, 1x128x512, recipe weights, train mode, q_sample noise injected).

The drop-in is built as a user gets it: LDMTrainer(model, loader, device, lr=1e-4) with autocast_dtype left at
None (the fp16 region) and the default scaler (init 2^16).  Eager and graphed (graph_step: two warm-up steps at
lr = 0, so the weights stay the recipe's, then the captured step replayed).

Step A (scale 2^16): the reference finds no inf; ours must not either, the scale stays 2^16, and the loss
terms, reconstructed samples 0 / 31 and the ten TRAIN_GRAD_KEYS gradients (unscaled) agree with the reference's
fp16 step by the rule of test_gpu_train_config3.py's bf16 case: per quantity within 1.5 e + 1e-4 of the fp16
reference and 2 e + 1e-4 of the fp32 one (e = the reference's own fp16-vs-fp32 distance, ref_goldens_r3.npz
r3_fp32_*; measured on MI355X: every quantity within 1.48 e of the fp16 reference); the Adam update is
checked against float64 Adam on our own gradients from the moments before the step.
Step B (the scale set to 2^40 first, update(new_scale=...) as on torch's scaler): the fp16 backward overflows
in the reference; ours must find the inf too, skip the step (parameters and Adam moments / step count bitwise
unchanged) and back the scale off to 2^39, like the reference.  Step C (the scale reset to 2^16): a normal
step again (finite, parameters move).
"""
import math
import os

import numpy as np
import pytest
import torch

import recipe
from conftest import ROOT, rel_err

pytestmark = pytest.mark.gpu

GRAD_KEYS = ("unet.time_mlp.1.weight", "unet.dec1.weight", "unet.dec1.bias", "unet.enc1.weight",
             "unet.cross_attention1.multihead_attn.in_proj_weight", "unet.bottleneck.bias",
             "decoder.decoder.6.weight", "decoder.decoder.1.weight", "style_encoder.enc6.bias",
             "style_encoder.enc1.weight")
B, H, W = 32, 128, 512


@pytest.fixture(scope="module")
def gf():
    return np.load(os.path.join(ROOT, "tests", "golden", "ref_goldens_fp16.npz"))


@pytest.fixture(scope="module")
def g3():
    return np.load(os.path.join(ROOT, "tests", "golden", "ref_goldens_r3.npz"))


def npy(t):
    return t.detach().double().cpu().numpy()


def _inputs(cuda):
    content = torch.from_numpy(recipe.uniform01((B, 1, H, W), 760)).to(cuda)
    style = torch.from_numpy(recipe.uniform01((B, 1, H, W), 761)).to(cuda)
    t = torch.from_numpy(recipe.timesteps(B, 762)).to(cuda)
    noise = torch.from_numpy(recipe.normal((B, 32, H // 8, W // 8), 763)).to(cuda)
    return content, style, t, noise


def test_golden_is_the_reference_default_sequence(gf):
    assert float(gf["fp16_a_found_inf"]) == 0.0 and float(gf["fp16_a_scale_after"]) == 2.0 ** 16
    assert float(gf["fp16_b_found_inf"]) == 1.0 and float(gf["fp16_b_scale_after"]) == 2.0 ** 39
    assert float(gf["fp16_b_params_unchanged"]) == 1.0 and float(gf["fp16_b_adam_step_unchanged"]) == 1.0


@pytest.mark.parametrize("graph", [False, True])
def test_default_fp16_gradscaler_step_matches_reference(gf, g3, cuda, graph):
    import models.model as M
    import models.train as TR
    m = M.LDM(32, pretrained_path="")
    recipe.fill_module(m, seed=700)
    m = m.to(cuda).train()
    tr = TR.LDMTrainer(m, None, cuda, lr=1e-4)
    assert tr.autocast_dtype is None and tr.autocast_enabled     # the reference's default region
    tr.graph_step = graph
    content, style, t, noise = _inputs(cuda)
    named = dict(m.named_parameters())
    lr = 1e-4
    tr.optimizer.param_groups[0]["lr"] = 0.0
    for _ in range(2):
        tr.train_step(content, style, t=t, noise=noise)
    assert tr._graph is None
    snap = {}
    for k in GRAD_KEYS:
        st = tr.optimizer.state[named[k]]
        snap[k] = (st["exp_avg"].double().cpu(), st["exp_avg_sq"].double().cpu(), named[k].detach().double().cpu())
    tr.optimizer.param_groups[0]["lr"] = lr

    # ---- step A: scale 2^16, no overflow (as the reference) ----
    losses = tr.train_step(content, style, t=t, noise=noise)
    assert (tr._graph is not None) == graph
    torch.cuda.synchronize()
    assert int(tr.scaler._found_inf.item()) == 0
    assert tr.scaler.get_scale() == float(gf["fp16_a_scale_after"])
    rec = tr.last_outputs["reconstructed"][[0, B - 1]]
    grads = {k: (named[k].grad[:256] if named[k].grad.dim() == 2 and named[k].grad.shape[0] > 256 else named[k].grad)
             for k in GRAD_KEYS}
    pairs = [("compression", np.float64(losses["compression_loss"]), "compression"),
             ("diffusion", np.float64(losses["denoisinsg_loss"]), "diffusion"),
             ("total", np.float64(losses["total_loss"]), "total"),
             ("recon", npy(rec), "recon_0_31")] + [(k, npy(grads[k]), "grad_" + k) for k in GRAD_KEYS]
    assert losses["style_loss"] == 0.0
    rows, bad = [], []
    for name, ours, key in pairs:
        f32, f16 = g3[f"r3_fp32_{key}"], gf[f"fp16_{key}"]
        ours = np.asarray(ours).reshape(np.shape(f32))
        e = rel_err(f16, f32)
        to32, to16 = rel_err(ours, f32), rel_err(ours, f16)
        rows.append(f"{name}: ref fp16-vs-fp32 {e:.2e}, ours-vs-fp32 {to32:.2e}, ours-vs-fp16 {to16:.2e}")
        if to32 > 2 * e + 1e-4 or to16 > 1.5 * e + 1e-4:
            bad.append(name)
    print("\n".join(rows))
    assert not bad, (bad, rows)
    b1, b2, eps = 0.9, 0.999, 1e-8
    after_a = {}
    for k in GRAD_KEYS:
        p = named[k]
        g = p.grad.double().cpu()
        m2, v2, p2 = snap[k]
        m3 = b1 * m2 + (1 - b1) * g
        v3 = b2 * v2 + (1 - b2) * g * g
        st = tr.optimizer.state[p]
        assert rel_err(npy(st["exp_avg"]), m3.numpy()) < 1e-6, k
        assert rel_err(npy(st["exp_avg_sq"]), v3.numpy()) < 1e-6, k
        p3 = p2 - (lr / (1 - b1 ** 3)) * m3 / (v3.sqrt() / math.sqrt(1 - b2 ** 3) + eps)
        err = (p.detach().double().cpu() - p3).abs()
        assert bool((err <= 2 * np.finfo(np.float32).eps * p3.abs() + 1e-3 * lr).all()), (k, float(err.max()))
        after_a[k] = (p.detach().clone(), st["exp_avg"].clone(), st["exp_avg_sq"].clone(), st["step"].clone())

    # ---- step B: scale 2^40, the fp16 backward overflows: skip and back off (as the reference) ----
    tr.scaler.update(new_scale=2.0 ** 40)
    lb = tr.train_step(content, style, t=t, noise=noise)
    torch.cuda.synchronize()
    assert int(tr.scaler._found_inf.item()) == 1 == int(gf["fp16_b_found_inf"])
    assert tr.scaler.get_scale() == float(gf["fp16_b_scale_after"])
    assert np.isfinite(lb["total_loss"])     # the loss itself is finite; its scaled gradients are not
    for k in GRAD_KEYS:
        p, ea, es, sc = after_a[k]
        st = tr.optimizer.state[named[k]]
        assert torch.equal(named[k].detach(), p), k
        assert torch.equal(st["exp_avg"], ea) and torch.equal(st["exp_avg_sq"], es) and torch.equal(st["step"], sc), k

    # ---- step C: back at 2^16, a normal step ----
    tr.scaler.update(new_scale=2.0 ** 16)
    lc = tr.train_step(content, style, t=t, noise=noise)
    torch.cuda.synchronize()
    assert int(tr.scaler._found_inf.item()) == 0 and np.isfinite(lc["total_loss"])
    moved = max(float((named[k].detach() - after_a[k][0]).abs().max()) for k in GRAD_KEYS)
    assert moved > 0.5 * lr
