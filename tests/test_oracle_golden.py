"""CPU: pin both oracles (oracle/ldm_np.py float64 numpy, oracle/ldm_torch_cpu.py fp32 torch-CPU) to the
golden vectors captured from the reference itself (tests/golden/make_goldens.py).

Tolerances: schedule tables / index lists bit-exact; fp32 torch-CPU restatement 2e-6 relative (same ATen
kernels, different op grouping); float64 numpy restatement 2e-5 relative (the goldens are fp32).
"""
import numpy as np
import pytest
import torch

import recipe
from conftest import rel_err
from oracle import ldm_np as NP
from oracle import ldm_torch_cpu as TC


def sd_for(module_ctor, seed):
    m = module_ctor()
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    vals = recipe.make_state(shapes, seed)
    return {k: torch.from_numpy(v) for k, v in vals.items()}


@pytest.fixture(scope="module")
def M():
    import models.model as M
    return M


# ---- scheduler: bit-exact ----------------------------------------------------------------------------
def test_schedule_tables_bitexact(goldens):
    b, a, ab = NP.schedule(200)
    assert np.array_equal(b, goldens["sched_beta"])
    assert np.array_equal(a, goldens["sched_alpha"])
    assert np.array_equal(ab, goldens["sched_alpha_bar"])
    for T in (10, 50, 100, 250, 1000):
        assert np.array_equal(NP.schedule(T)[2], goldens[f"sched_alpha_bar_T{T}"])
        assert np.array_equal(TC.schedule(T)[2].numpy(), goldens[f"sched_alpha_bar_T{T}"])


@pytest.mark.parametrize("start,n", [(199, 50), (199, 100), (199, 200), (49, 50), (99, 100), (199, 250), (199, 2),
                                     (9, 10)])
def test_index_lists_bitexact(goldens, start, n):
    ref = goldens[f"times_{start}_{n}"]
    assert np.array_equal(NP.linspace_f32(start, 0, n).astype(np.int64), ref)
    assert np.array_equal(TC.ddim_times(start + 1, n).numpy(), ref)


def test_reference_step_lists(goldens):
    assert np.array_equal(NP.ddim_times(200, 50)[:-1], goldens["ddim50_eta0_times"])
    assert np.array_equal(NP.content_times(10)[:-1], goldens["cs10_eta1_times"])


def test_sinusoid(goldens):
    # float64 vs the reference's fp32 (t * f with t up to 199 amplifies the fp32 rounding of f)
    assert rel_err(NP.sinusoid(goldens["sinus_t"]), goldens["sinus_emb"]) < 2e-5
    assert rel_err(TC.sinusoid(torch.from_numpy(goldens["sinus_t"])).numpy(), goldens["sinus_emb"]) < 1e-7


# ---- UNet / attention ----------------------------------------------------------------------------------
@pytest.mark.parametrize("tag", ["s", "c"])
def test_unet(M, goldens, tag):
    B, H, W, seed = {"s": (2, 16, 16, 1), "c": (1, 16, 64, 2)}[tag]
    sd = sd_for(lambda: M.UNet(32, 32, 64), 100)
    z = recipe.normal((B, 32, H, W), seed)
    s5 = recipe.uniform01((B, 256, H // 4, W // 4), seed + 10)
    s6 = recipe.uniform01((B, 512, H // 8, W // 8), seed + 20)
    t = goldens[f"unet_{tag}_t"]
    with torch.no_grad():
        y = TC.unet(sd, torch.from_numpy(z), torch.from_numpy(t), torch.from_numpy(s5), torch.from_numpy(s6), p="")
    assert rel_err(y.numpy(), goldens[f"unet_{tag}_out"]) < 2e-6
    assert rel_err(NP.time_mlp(sd, "", t), goldens[f"unet_{tag}_temb"]) < 2e-5
    if tag == "s":
        assert rel_err(NP.unet(sd, z, t, s5, s6, p=""), goldens["unet_s_out"]) < 2e-5


@pytest.mark.parametrize("E,h,w", [(256, 4, 16), (512, 2, 8)])
def test_cross_attention(M, goldens, E, h, w):
    sd = sd_for(lambda: M.CrossAttention(E, 4), 200 + E)
    q = recipe.normal((2, E, h, w), 300 + E)
    kv = recipe.uniform01((2, E, h, w), 400 + E)
    with torch.no_grad():
        y = TC.cross_attention(sd, "", torch.from_numpy(q), torch.from_numpy(kv))
    assert rel_err(y.numpy(), goldens[f"ca{E}_out"]) < 2e-6
    assert rel_err(NP.cross_attention(sd, "", q.astype(np.float64), kv.astype(np.float64)), goldens[f"ca{E}_out"]) < 2e-5


# ---- VAE / style encoder -------------------------------------------------------------------------------
def test_vae_style(M, goldens):
    sde = sd_for(lambda: M.SpectrogramEncoder(32), 500)
    sdd = sd_for(lambda: M.SpectrogramDecoder(32), 501)
    sds = sd_for(lambda: M.StyleEncoder(1, 64), 502)
    x_s = recipe.uniform01((2, 1, 128, 128), 600)
    zl = recipe.normal((2, 32, 16, 16), 602)
    with torch.no_grad():
        assert rel_err(TC.encoder(sde, torch.from_numpy(x_s), p="").numpy(), goldens["enc_eval_s_out"]) < 2e-6
        assert rel_err(TC.decoder(sdd, torch.from_numpy(zl), p="").numpy(), goldens["dec_eval_s_out"]) < 2e-6
        st = {}
        assert rel_err(TC.encoder(sde, torch.from_numpy(x_s), True, p="", state=st).numpy(),
                       goldens["enc_train_s_out"]) < 2e-6
        assert rel_err(st["encoder.1.running_mean"].numpy(), goldens["enc_train_s_rm0"]) < 2e-6
        assert rel_err(TC.decoder(sdd, torch.from_numpy(zl), True, p="").numpy(), goldens["dec_train_s_out"]) < 2e-6
        so = TC.style_encoder(sds, torch.from_numpy(x_s), p="")
        for k in ("s5", "s6"):
            assert rel_err(so[k].numpy(), goldens[f"style_s_{k}"]) < 2e-6
    assert rel_err(NP.encoder(sde, x_s, p=""), goldens["enc_eval_s_out"]) < 2e-5
    assert rel_err(NP.encoder(sde, x_s, True, p=""), goldens["enc_train_s_out"]) < 2e-5
    assert rel_err(NP.decoder(sdd, zl, p=""), goldens["dec_eval_s_out"]) < 2e-5
    assert rel_err(NP.decoder(sdd, zl, True, p=""), goldens["dec_train_s_out"]) < 2e-5
    assert rel_err(NP.style_encoder(sds, x_s, p="")["s6"], goldens["style_s_s6"]) < 2e-5


# ---- sampling loops ------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def ldm_sd(M):
    return sd_for(lambda: M.LDM(32, pretrained_path=""), 700)


@pytest.mark.parametrize("eta", [0, 1])
def test_ddim50(ldm_sd, goldens, eta):
    ab = TC.schedule(200)[2]
    style = torch.from_numpy(recipe.uniform01((1, 1, 128, 128), 701))
    zT = torch.from_numpy(recipe.normal((1, 32, 16, 16), 702))
    logs = {"timesteps": [], "pred_x0": [], "noise_pred": []}
    with torch.no_grad():
        emb = TC.style_encoder(ldm_sd, style)
        x = TC.reverse_loop(ldm_sd, ab, zT, emb["s5"], emb["s6"], TC.ddim_times(200, 50), float(eta), logs=logs)
    assert logs["timesteps"] == goldens[f"ddim50_eta{eta}_times"].tolist()
    assert rel_err(x.numpy(), goldens[f"ddim50_eta{eta}_x"]) < 1e-5
    assert rel_err(logs["pred_x0"][0].numpy(), goldens[f"ddim50_eta{eta}_x0_first"]) < 2e-6


def test_content_style(ldm_sd, goldens):
    ab = TC.schedule(200)[2]
    style = torch.from_numpy(recipe.uniform01((1, 1, 128, 128), 701))
    zT = torch.from_numpy(recipe.normal((1, 32, 16, 16), 702))
    with torch.no_grad():
        emb = TC.style_encoder(ldm_sd, style)
        x = TC.reverse_loop(ldm_sd, ab, zT, emb["s5"], emb["s6"], TC.content_times(10), 1.0)
    assert rel_err(x.numpy(), goldens["cs10_eta1_x"]) < 1e-5


def test_ldm_forward_and_losses(ldm_sd, goldens):
    ab = TC.schedule(200)[2]
    content = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 710))
    style = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 711))
    t = torch.from_numpy(goldens["fwd_eval_t"])
    noise = torch.from_numpy(goldens["fwd_eval_noise"])
    with torch.no_grad():
        out = TC.ldm_forward(ldm_sd, content, style, t, noise, ab)
    for k in ("z_t", "noise_pred", "z_0", "reconstructed"):
        assert rel_err(out[k].numpy(), goldens[f"fwd_eval_{k}"]) < 2e-6, k
    assert rel_err(torch.nn.functional.mse_loss(out["noise_pred"], noise).numpy(), goldens["loss_diffusion"]) < 2e-6
    assert rel_err(TC.kl_loss(out["z_0"]).numpy(), goldens["loss_kl"]) < 2e-6


def test_train_step_gradients(ldm_sd, goldens):
    """Restated LDMTrainer.train_step (train.py:163-208) in fp32 without LPIPS/VGGish: encoder frozen,
    whole model in train mode (train_epoch calls model.train(), train.py:212)."""
    ab = TC.schedule(200)[2]
    sd = {k: (v.clone().requires_grad_(not k.startswith("encoder.") and v.is_floating_point()
                                       and "running" not in k)) for k, v in ldm_sd.items()}
    content = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 710))
    style = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 711))
    t = torch.from_numpy(goldens["fwd_eval_t"])
    noise = torch.from_numpy(goldens["train_noise"])
    out = TC.ldm_forward(sd, content, style, t, noise, ab, train_decoder=True, train_encoder=True, state={})
    total = torch.nn.functional.mse_loss(out["reconstructed"], content) + 0.01 * TC.kl_loss(out["z_0"]) + \
        torch.nn.functional.mse_loss(out["noise_pred"], noise)
    total.backward()
    assert rel_err(total.detach().numpy(), goldens["train_total"]) < 2e-6
    for k in ("unet.time_mlp.1.weight", "unet.dec1.weight", "unet.dec1.bias", "unet.enc1.weight",
              "unet.cross_attention1.multihead_attn.in_proj_weight", "unet.bottleneck.bias",
              "decoder.decoder.6.weight", "decoder.decoder.1.weight", "style_encoder.enc6.bias",
              "style_encoder.enc1.weight"):
        g = sd[k].grad
        g = g[:256] if g.dim() == 2 and g.shape[0] > 256 else g
        assert rel_err(g.numpy(), goldens["grad_" + k]) < 1e-4, k


# ---- round-2 fixtures ------------------------------------------------------------------------------------
def test_content_style_transfer_wrapper(ldm_sd, goldens2):
    """content_style_transfer_wrapper (model.py:468-501) at T'=100, eta=1 with the recorded epsilon."""
    ab = TC.schedule(200)[2]
    content = torch.from_numpy(recipe.uniform01((1, 1, 128, 128), 720))
    style = torch.from_numpy(recipe.uniform01((1, 1, 128, 128), 721))
    eps = torch.from_numpy(goldens2["cst100_eps"])
    with torch.no_grad():
        z0 = TC.encoder(ldm_sd, content)
        zt = TC.q_sample(ab, z0, torch.tensor([99]), eps)
        emb = TC.style_encoder(ldm_sd, style)
        x = TC.reverse_loop(ldm_sd, ab, zt, emb["s5"], emb["s6"], TC.content_times(100), 1.0)
        dec = (TC.decoder(ldm_sd, x) + 1) / 2
        ztd = TC.decoder(ldm_sd, zt)
    assert rel_err(dec.numpy(), goldens2["cst100_decoded"]) < 1e-5
    assert rel_err(ztd.numpy(), goldens2["cst100_zt_decoded"]) < 2e-6


def test_autoencoder_step(M, goldens2):
    """One train_autoencoder step (train.py:59-82) restated: train-mode BN in encoder and decoder,
    MSE + 0.01 KL (LPIPS term out of scope), torch AdamW(lr=5e-4)."""
    from conftest import AE_KEYS
    sde = {"encoder." + k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k)
           for k, v in sd_for(lambda: M.SpectrogramEncoder(32), 730).items()}
    sdd = {"decoder." + k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k)
           for k, v in sd_for(lambda: M.SpectrogramDecoder(32), 731).items()}
    sd = {**sde, **sdd}
    spec = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 732))
    state = {}
    lat = TC.encoder(sd, spec, True, state=state)
    rec = TC.decoder(sd, lat, True, state=state)
    loss = torch.nn.functional.mse_loss(rec, spec) + 0.01 * TC.kl_loss(lat)
    loss.backward()
    assert rel_err(lat.detach().numpy(), goldens2["ae_latent"]) < 2e-6
    assert rel_err(rec.detach().numpy(), goldens2["ae_recon"]) < 2e-6
    assert rel_err(loss.detach().numpy(), goldens2["ae_loss"]) < 2e-6
    for k in AE_KEYS:
        assert rel_err(sd[k].grad.numpy(), goldens2["ae_grad_" + k]) < 1e-4, k
    params = [v for k, v in sd.items() if v.requires_grad]
    opt = torch.optim.AdamW(params, lr=5e-4)
    opt.step()
    for k in AE_KEYS:
        assert rel_err(sd[k].detach().numpy(), goldens2["ae_adamw1_" + k]) < 1e-6, k
    assert rel_err(state["encoder.encoder.4.running_mean"].numpy(), goldens2["ae_enc_rm4"]) < 2e-6
    assert rel_err(state["decoder.decoder.1.running_var"].numpy(), goldens2["ae_dec_rv1"]) < 2e-6


@pytest.mark.parametrize("case", ["a", "odd"])
def test_vggish_feature_loss(goldens_vgg, case):
    """oracle restatement of VGGishFeatureLoss.forward (loss.py:64-101) vs the reference's own forward on
    the same recipe-filled VGGish-shaped stack (fp32 CPU both: 2e-6)."""
    from conftest import VGG_CASES
    from models.loss import vggish_features
    shape, seed = VGG_CASES[case]
    sd = sd_for(vggish_features, seed)
    p = torch.from_numpy(recipe.uniform01(shape, seed + 1))
    t = torch.from_numpy(recipe.uniform01(shape, seed + 2))
    out = TC.vggish_feature_loss(sd, p, t)
    assert rel_err(out.numpy(), goldens_vgg[f"vgg_{case}_loss"]) < 2e-6



# ---- round 3: config 3's shape, wide latents (ref_goldens_r3.npz) ----------------------------------------
@pytest.fixture(scope="module")
def goldens3():
    import os
    from conftest import ROOT
    return np.load(os.path.join(ROOT, "tests", "golden", "ref_goldens_r3.npz"))


def test_wide_latent_unet_and_ddim(M, ldm_sd, goldens3):
    """UNet on a [1,32,16,128] latent (CA2 L = S = 128) and a 5-step DDIM there; UNet(1, 1, 64) on a
    [1,1,64,256] mel (reduced SURVEY shape S: CA2 L = S = 1024)."""
    sd = sd_for(lambda: M.UNet(32, 32, 64), 100)
    z = torch.from_numpy(recipe.normal((1, 32, 16, 128), 770))
    s5 = torch.from_numpy(recipe.uniform01((1, 256, 4, 32), 771))
    s6 = torch.from_numpy(recipe.uniform01((1, 512, 2, 16), 772))
    with torch.no_grad():
        y = TC.unet(sd, z, torch.tensor([117]), s5, s6, p="")
        assert rel_err(y.numpy(), goldens3["w128_unet_out"]) < 2e-6
        ab = TC.schedule(200)[2]
        style = torch.from_numpy(recipe.uniform01((1, 1, 128, 1024), 773))
        emb = TC.style_encoder(ldm_sd, style)
        zT = torch.from_numpy(recipe.normal((1, 32, 16, 128), 774))
        x = TC.reverse_loop(ldm_sd, ab, zT, emb["s5"], emb["s6"], TC.ddim_times(200, 5), 0.0)
        assert rel_err(x.numpy(), goldens3["w128_ddim5_x"]) < 1e-5
        sds = sd_for(lambda: M.UNet(1, 1, 64), 101)
        zs = torch.from_numpy(recipe.normal((1, 1, 64, 256), 775))
        s5s = torch.from_numpy(recipe.uniform01((1, 256, 16, 64), 776))
        s6s = torch.from_numpy(recipe.uniform01((1, 512, 8, 32), 777))
        ys = TC.unet(sds, zs, torch.tensor([42]), s5s, s6s, p="")
        assert rel_err(ys.numpy(), goldens3["shapeS_unet_out"]) < 2e-6


def test_config3_train_step(M, goldens3):
    """The restated train step at config 3's shape (batch 32, 1x128x512, every module in train mode) against
    the reference's fp32 golden: losses, reconstructed samples 0 / 31, two gradients."""
    sd = sd_for(lambda: M.LDM(32, pretrained_path=""), 700)
    trained = [k for k in sd if sd[k].is_floating_point() and "running_" not in k and "num_batches" not in k]
    for k in trained:
        sd[k].requires_grad_(True)
    B = 32
    content = torch.from_numpy(recipe.uniform01((B, 1, 128, 512), 760))
    style = torch.from_numpy(recipe.uniform01((B, 1, 128, 512), 761))
    t = torch.from_numpy(recipe.timesteps(B, 762))
    noise = torch.from_numpy(recipe.normal((B, 32, 16, 64), 763))
    assert np.array_equal(t.numpy(), goldens3["r3_t"])
    ab = TC.schedule(200)[2]
    o = TC.ldm_forward(sd, content, style, t, noise, ab, train_decoder=True, train_encoder=True, state={})
    dl = torch.mean((o["noise_pred"] - o["noise"]) ** 2)
    comp = torch.mean((o["reconstructed"] - content) ** 2) + 0.01 * TC.kl_loss(o["z_0"])
    (comp + dl).backward()
    assert rel_err(comp.detach().numpy(), goldens3["r3_fp32_compression"]) < 1e-5
    assert rel_err(dl.detach().numpy(), goldens3["r3_fp32_diffusion"]) < 1e-5
    assert rel_err(o["reconstructed"].detach()[[0, B - 1]].numpy(), goldens3["r3_fp32_recon_0_31"]) < 1e-5
    for k in ("unet.dec1.weight", "decoder.decoder.6.weight"):
        assert rel_err(sd[k].grad.numpy(), goldens3["r3_fp32_grad_" + k]) < 1e-4, k
