"""CPU: host-side logic of the drop-in (no kernel launches): API surface vs the reference, state_dict
keys/shapes, schedule tables, reverse-loop coefficient tables and index lists, plans / phase tables,
no-CPU-fallback behaviour."""
import ctypes
import inspect
import json
import os

import numpy as np
import pytest
import torch

from oracle import ldm_np as NP

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def M():
    import models.model as M
    return M


def test_state_dict_keys_and_shapes_match_reference(M):
    ref = json.load(open(os.path.join(HERE, "golden", "ref_state_dict_keys.json")))
    mine = {k: list(v.shape) for k, v in M.LDM(32, pretrained_path="").state_dict().items()}
    assert mine == ref


def test_api_signatures(M):
    import models.loss as L
    import models.train as T
    from models.config import config
    assert config["forward_diffusion_num_timesteps"] == 200 and config["latent_dim_encoder"] == 32
    sig = inspect.signature(M.LDM.__init__)
    assert list(sig.parameters)[1:] == ["latent_dim", "pretrained_path", "pretraind_filename", "num_timesteps",
                                        "load_full_model"]
    assert sig.parameters["pretrained_path"].default == "models/pretrained/"
    assert inspect.signature(M.LDM.style_ddim_sample_wrapper).parameters["timesteps"].default == 100
    assert inspect.signature(M.LDM.content_style_transfer_wrapper).parameters["num_timesteps"].default == 250
    assert inspect.signature(M.UNet.__init__).parameters["in_channels"].default == 1
    for name in ("diffusion_loss", "compression_loss", "kl_regularization_loss", "perceptual_loss", "style_loss",
                 "VGGishFeatureLoss", "gram_matrix", "perceptual_loss_old"):
        assert hasattr(L, name)
    for name in ("LDMTrainer", "train_autoencoder", "train_ldm", "main"):
        assert hasattr(T, name)
    p = inspect.signature(T.LDMTrainer.__init__).parameters
    assert p["lr"].default == 1e-4 and p["style_loss_weight"].default == 0.1


def test_parameter_counts(M):
    n = lambda m: sum(p.numel() for p in m.parameters())  # noqa: E731
    assert n(M.UNet(32, 32, 64)) == 6841504
    assert n(M.SpectrogramEncoder(32)) == 111840
    assert n(M.SpectrogramDecoder(32)) == 198209
    assert n(M.StyleEncoder(1, 64)) == 2729984


def test_schedule_buffers_bitexact(M, goldens):
    fd = M.ForwardDiffusion(200)
    assert np.array_equal(fd.beta_t.numpy(), goldens["sched_beta"])
    assert np.array_equal(fd.alpha_bar_t.numpy(), goldens["sched_alpha_bar"])


def test_reverse_coefficients_are_torch_fp32(M):
    fd = M.ForwardDiffusion(200)
    times = torch.linspace(199, 0, 50).long()
    c = fd.reverse_coefs(times)
    ab = fd.alpha_bar_t
    assert c.shape == (49, 4) and c.dtype == torch.float32
    assert torch.equal(c[:, 0], torch.sqrt(ab[times[:-1]]))
    assert torch.equal(c[:, 3], torch.sqrt(1 - ab[times[1:]]))
    assert np.array_equal(times.numpy(), NP.ddim_times(200, 50))


def test_out_of_range_timesteps_raise_index_error(M):
    fd = M.ForwardDiffusion(200)
    with pytest.raises(IndexError):
        fd.reverse_coefs(torch.linspace(249, 0, 250).long())      # content_style_transfer default (§0.5b)
    with pytest.raises(IndexError):
        fd._check_t(torch.tensor([0, 200]))


def test_no_cpu_fallback(M):
    unet = M.UNet(32, 32, 64)
    z = torch.zeros(1, 32, 16, 16)
    emb = {"s5": torch.zeros(1, 256, 4, 4), "s6": torch.zeros(1, 512, 2, 2)}
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        with torch.no_grad():
            unet(z, torch.zeros(1, dtype=torch.long), emb)


def test_conv_plans_and_layer_descs():
    from ldm_amd import _lib as L
    shape = L.UNetShape(8, 32, 16, 64, 64)
    outs = []
    for layer in range(15):
        d = L.ConvDesc()
        L.call("ldm_unet_layer_desc", ctypes.byref(shape), layer, ctypes.byref(d))
        p = L.ConvPlan()
        L.call("ldm_conv_make_plan", ctypes.byref(d), ctypes.byref(p))
        outs.append((d.Cout, d.Hout, d.Wout))
        assert p.kind in (1, 2) and p.packed_floats > 0
    assert outs[0] == (64, 16, 64) and outs[4] == (512, 2, 8) and outs[5] == (256, 4, 16) and outs[8] == (32, 16, 64)
    assert L.load().ldm_unet_workspace_floats(ctypes.byref(shape), None) > 0
    assert L.load().ldm_ddim_workspace_floats(ctypes.byref(shape), None, 49) > L.load().ldm_unet_workspace_floats(
        ctypes.byref(shape), None)
    # plans with cross-block K splits need counter + partial space on top
    w = L.UNetWeights()
    L.call("ldm_unet_make_plans", ctypes.byref(shape), ctypes.byref(w))
    d = L.ConvDesc()
    L.call("ldm_unet_layer_desc", ctypes.byref(shape), 4, ctypes.byref(d))
    L.call("ldm_conv_make_plan_forced", ctypes.byref(d), 1, 1, 1, 4, 4, ctypes.byref(w.conv_plan[4]))
    assert w.conv_plan[4].ws_floats == 4 * 512 * 128 + (1 << 16)
    assert L.load().ldm_unet_workspace_floats(ctypes.byref(shape), ctypes.byref(w)) >= \
        L.load().ldm_unet_workspace_floats(ctypes.byref(shape), None) + w.conv_plan[4].ws_floats


def test_split_k_plan_validation():
    from ldm_amd import _lib as L
    d = L.ConvDesc(8, 512, 2, 8, 512, 2, 8, 3, 3, 1, 1, 0, 0)
    p = L.ConvPlan()
    for ks in (1, 2, 4, 8, 16):
        L.call("ldm_conv_make_plan_forced", ctypes.byref(d), 1, 2, 2, 2, ks, ctypes.byref(p))
        assert p.ks == ks and (p.ws_floats == 0) == (ks == 1)
    assert L.load().ldm_conv_make_plan_forced(ctypes.byref(d), 1, 1, 1, 1, 3, ctypes.byref(p)) != 0
    assert L.load().ldm_conv_make_plan_forced(ctypes.byref(d), 1, 1, 1, 1, 64, ctypes.byref(p)) != 0


def test_transposed_conv_phase_geometry():
    """k3 s2 p1 op1 and k4 s2 p1 transposed convs: the 4 parity phases cover each output once with the
    right tap counts (1/2/2/4 and 4/4/4/4) — checked through the packed-weight size."""
    from ldm_amd import _lib as L
    for k, op, taps in ((3, 1, 9), (4, 0, 16)):
        d = L.ConvDesc(2, 16, 5, 7, 32, 10, 14, k, k, 2, 1, op, 1)
        p = L.ConvPlan()
        L.call("ldm_conv_make_plan_forced", ctypes.byref(d), 2, 1, 1, 1, 1, ctypes.byref(p))
        assert p.packed_floats == taps * 16 * 32   # sum over phases of ntap * Cin * Mpad(=32)


def test_fast_plan_override_table_loads():
    from ldm_amd import autotune, ops
    path = autotune.TUNED_PATH
    if not os.path.exists(path):
        pytest.skip("no tuned table")
    n = autotune.load_tuned(path)
    assert n > 0 and len(ops._PLAN_OVERRIDE) >= n


def test_lpips_alex_state_dict_forms():
    """LPIPSAlex takes lpips.LPIPS state_dict keys, or torchvision alexnet 'features.<idx>.*' + the lpips v0.1
    'lin<i>.model.1.weight' file, and refuses an incomplete set (loss.py:6-21)."""
    import pytest as _pytest
    import torch as _torch
    from ldm_amd.lpips import CONVS, LPIPSAlex
    m = LPIPSAlex()
    sd = {k: _torch.randn(v.shape) for k, v in m.state_dict().items() if not k.startswith("lins.")}
    sd.update({f"lins.{i}.model.1.weight": sd[f"lin{i}.model.1.weight"] for i in range(5)})   # one tensor, two keys
    m2 = LPIPSAlex.from_state_dict(sd)
    assert all(_torch.equal(m2.state_dict()[k], sd[k]) for k in sd if not k.startswith("scaling_layer"))
    tv = {}
    for sl, idx, *_ in CONVS:
        tv[f"features.{idx}.weight"] = sd[f"net.slice{sl}.{idx}.weight"]
        tv[f"features.{idx}.bias"] = sd[f"net.slice{sl}.{idx}.bias"]
    for i in range(5):
        tv[f"lin{i}.model.1.weight"] = sd[f"lin{i}.model.1.weight"]
    m3 = LPIPSAlex.from_state_dict(tv)
    assert _torch.equal(m3.lins[2].model[1].weight, sd["lin2.model.1.weight"])
    assert _torch.equal(m3.net.conv(1).weight, sd["net.slice2.3.weight"])
    with _pytest.raises(KeyError):
        LPIPSAlex.from_state_dict({k: v for k, v in tv.items() if not k.startswith("lin4")})


def test_store16_policy_and_codes(monkeypatch):
    """16-bit storage of large maps (ops.store16_dtype, in16, st_code; ldm_capi.h LDM_ST_* / LDM_DT_*16) and
    which conv forms take it (host-side plan queries, no GPU): every large-map layer of the B = 32 train step."""
    from ldm_amd import _lib as L
    from ldm_amd import ops
    assert ops.store16_dtype(1 << 22, 2) == torch.bfloat16 and ops.store16_dtype(1 << 22, 1) == torch.float16
    assert ops.store16_dtype((1 << 22) - 1, 2) == torch.float32 and ops.store16_dtype(1 << 24, 0) == torch.float32
    monkeypatch.setenv("LDM_AMD_STORE16", "0")
    assert ops.store16_dtype(1 << 24, 2) == torch.float32
    monkeypatch.delenv("LDM_AMD_STORE16")
    t, h = ops.in16(torch.zeros(4, dtype=torch.bfloat16), 2)
    assert h and t.dtype == torch.bfloat16
    t, h = ops.in16(torch.zeros(4, dtype=torch.bfloat16), 1)          # another 16-bit type: read as fp32
    assert not h and t.dtype == torch.float32
    t, h = ops.in16(torch.zeros(4, dtype=torch.bfloat16), 2, ok=False)
    assert not h and t.dtype == torch.float32
    assert ops.st_code(2, x16=True, dx16=True) == (2 << L.ST_SHIFT) | L.ST_X16 | L.ST_DX16
    assert ops.st_code(2) == 0
    layers = [(1, 128, 512, 64, 3, 2, 0, False), (64, 64, 256, 128, 3, 2, 0, False), (128, 32, 128, 32, 3, 2, 0, False),
              (32, 16, 64, 128, 4, 2, 0, True), (128, 32, 128, 64, 4, 2, 0, True), (64, 64, 256, 1, 4, 2, 0, True),
              (128, 32, 128, 256, 3, 2, 0, False), (256, 16, 64, 256, 3, 2, 0, False)]
    for Cin, H, W, Cout, k, s, op, tr in layers:
        d = ops.make_desc(32, Cin, H, W, Cout, k, k, s, 1, op, tr)
        dd = ops.dual_desc(d)
        pf = ops.tiled_plan(d, 2) or ops.get_plan(d)
        pd = ops.tiled_plan(dd, 2) or ops.get_plan(dd)
        big_in, big_out = 32 * Cin * H * W >= 1 << 22, 32 * Cout * d.Hout * d.Wout >= 1 << 22
        f, b, w = ops.conv_storage16(d, pf, 2), ops.conv_storage16(dd, pd, 2), ops.wgrad_storage16(d, 2)
        if big_out:   # (a Cin = 1 first layer has no data gradient: its input is the mel)
            assert f & L.DT_Y16 and (Cin == 1 or b & L.DT_X16) and w & L.DT_DY16, \
                (Cin, Cout, f, b, w)
        if big_in and Cin > 1:
            assert f & L.DT_X16 and b & L.DT_Y16 and w & L.DT_X16, (Cin, Cout, f, b, w)
        assert ops.conv_storage16(d, pf, 0) == 0 and ops.wgrad_storage16(d, 0) == 0
