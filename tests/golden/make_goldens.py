"""Generate golden vectors by running the REFERENCE implementation on CPU (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py          # ref_goldens.npz
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py --r2     # ref_goldens_r2.npz
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py --amp    # ref_goldens_amp.npz
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py --amp8   # ref_goldens_amp8.npz
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py --vggish # ref_goldens_vggish.npz
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py --r3     # ref_goldens_r3.npz
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py --fp16train   # ref_goldens_fp16.npz

Imports /root/reference/models/model.py and loss.py with two absent, unused-on-this-path imports
stubbed (``pytorch_lightning`` at model.py:4 and ``lpips`` at loss.py:3) and with
``model.VGGishFeatureLoss`` swapped for an empty module (its constructor is a remote
torch.hub fetch, model.py:260 -> loss.py:56).  Every weight and input comes from
tests/golden/recipe.py, so only inputs/outputs are stored: tests/golden/ref_goldens.npz.
The reference never travels to the GPU box; only this .npz does.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import recipe  # noqa: E402

REF = "/root/reference/models"


def import_reference():
    sys.dont_write_bytecode = True
    sys.modules.setdefault("pytorch_lightning", types.ModuleType("pytorch_lightning"))
    lp = types.ModuleType("lpips")
    lp.LPIPS = None
    sys.modules.setdefault("lpips", lp)
    sys.path.insert(0, REF)
    import model as ref_model  # noqa: E402
    import loss as ref_loss  # noqa: E402

    class _NoVGGish(torch.nn.Module):
        def forward(self, a, b):
            return torch.zeros((), dtype=a.dtype)

    ref_model.VGGishFeatureLoss = _NoVGGish
    return ref_model, ref_loss


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def main():
    torch.set_num_threads(8)
    M, L = import_reference()
    G = {}

    # ---- (1) schedule tables, index lists, sinusoid ------------------------------------------
    fd = M.ForwardDiffusion(200)
    G["sched_beta"] = np32(fd.beta_t)
    G["sched_alpha"] = np32(fd.alpha_t)
    G["sched_alpha_bar"] = np32(fd.alpha_bar_t)
    for T in (10, 50, 100, 250, 1000):
        f = M.ForwardDiffusion(T)
        G[f"sched_alpha_bar_T{T}"] = np32(f.alpha_bar_t)
    for start, n in ((199, 50), (199, 100), (199, 200), (49, 50), (99, 100), (199, 250), (199, 2), (9, 10)):
        G[f"times_{start}_{n}"] = torch.linspace(start, 0, n).long().numpy()
    sp = M.SinusoidalPositionEmbeddings(128)
    tt = torch.tensor([0, 1, 57, 199], dtype=torch.long)
    G["sinus_t"] = tt.numpy()
    G["sinus_emb"] = np32(sp(tt))

    with torch.no_grad():
        # ---- (2) UNet forward -------------------------------------------------------------
        unet = M.UNet(32, 32, 64)
        recipe.fill_module(unet, seed=100)
        for tag, (B, H, W, seed) in {"s": (2, 16, 16, 1), "c": (1, 16, 64, 2)}.items():
            z = torch.from_numpy(recipe.normal((B, 32, H, W), seed))
            s5 = torch.from_numpy(recipe.uniform01((B, 256, H // 4, W // 4), seed + 10))
            s6 = torch.from_numpy(recipe.uniform01((B, 512, H // 8, W // 8), seed + 20))
            t = torch.from_numpy(recipe.timesteps(B, seed + 30))
            out = unet(z, t, {"s5": s5, "s6": s6})
            G[f"unet_{tag}_t"] = t.numpy()
            G[f"unet_{tag}_out"] = np32(out)
            G[f"unet_{tag}_temb"] = np32(unet.time_mlp(t))

        # ---- (3) CrossAttention standalone ------------------------------------------------
        for E, (h, w) in ((256, (4, 16)), (512, (2, 8))):
            ca = M.CrossAttention(E, 4)
            recipe.fill_module(ca, seed=200 + E)
            q = torch.from_numpy(recipe.normal((2, E, h, w), 300 + E))
            kv = torch.from_numpy(recipe.uniform01((2, E, h, w), 400 + E))
            G[f"ca{E}_out"] = np32(ca(q, kv))

        # ---- (4) VAE encoder / decoder (eval and train BN), style encoder ----------------
        enc = M.SpectrogramEncoder(32)
        dec = M.SpectrogramDecoder(32)
        sty = M.StyleEncoder(1, 64)
        recipe.fill_module(enc, seed=500)
        recipe.fill_module(dec, seed=501)
        recipe.fill_module(sty, seed=502)
        x_s = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 600))
        x_c = torch.from_numpy(recipe.uniform01((1, 1, 128, 512), 601))
        enc.eval()
        dec.eval()
        G["enc_eval_s_out"] = np32(enc(x_s))
        G["enc_eval_c_out"] = np32(enc(x_c))
        zl = torch.from_numpy(recipe.normal((2, 32, 16, 16), 602))
        G["dec_eval_s_out"] = np32(dec(zl))
        enc.train()
        dec.train()
        G["enc_train_s_out"] = np32(enc(x_s))
        G["enc_train_s_rm0"] = np32(enc.encoder[1].running_mean)
        G["enc_train_s_rv0"] = np32(enc.encoder[1].running_var)
        G["dec_train_s_out"] = np32(dec(zl))
        G["dec_train_s_rm1"] = np32(dec.decoder[4].running_mean)
        G["dec_train_s_rv1"] = np32(dec.decoder[4].running_var)
        so = sty(x_s)
        G["style_s_s1_slice"] = np32(so["s1"][:, :8])
        for k in ("s5", "s6"):
            G[f"style_s_{k}"] = np32(so[k])
        so = sty(x_c)
        for k in ("s5", "s6"):
            G[f"style_c_{k}"] = np32(so[k])

        # ---- (5) DDIM loops (B=1: the reference crashes for B>1 at model.py:461) -------------
        ldm = M.LDM(32, pretrained_path="")
        recipe.fill_module(ldm, seed=700)
        ldm.eval()
        style = torch.from_numpy(recipe.uniform01((1, 1, 128, 128), 701))
        emb = ldm.style_encoder(style)
        zT = torch.from_numpy(recipe.normal((1, 32, 16, 16), 702))
        for eta in (0.0, 1.0):
            x, logs = ldm.style_conditioned_ddim_sample(zT, emb, timesteps=50, eta=eta)
            e = int(eta)
            G[f"ddim50_eta{e}_x"] = np32(x)
            G[f"ddim50_eta{e}_x0_first"] = np32(logs["pred_x0"][0])
            G[f"ddim50_eta{e}_eps_last"] = np32(logs["noise_pred"][-1])
            G[f"ddim50_eta{e}_times"] = np.array(logs["timesteps"], dtype=np.int64)
        x, logs = ldm.content_style_ddim_sample(zT, emb, timesteps=10, eta=1.0)
        G["cs10_eta1_x"] = np32(x)
        G["cs10_eta1_times"] = np.array(logs["timesteps"], dtype=np.int64)
        # canonical 128x512 latent, a short DDIM (5 steps) to bound fixture cost
        style_c = torch.from_numpy(recipe.uniform01((1, 1, 128, 512), 703))
        emb_c = ldm.style_encoder(style_c)
        zT_c = torch.from_numpy(recipe.normal((1, 32, 16, 64), 704))
        x, _ = ldm.style_conditioned_ddim_sample(zT_c, emb_c, timesteps=5, eta=0.0)
        G["ddim5_c_x"] = np32(x)
        # decoded sample through the full wrapper path (CPU generator z_T, model.py:394)
        torch.manual_seed(1234)
        dec_out = ldm.style_ddim_sample_wrapper((1, 32, 16, 16), style, timesteps=8, eta=0.0)
        G["wrap8_decoded"] = np32(dec_out)

        # ---- (6) LDM.forward with recorded noise ------------------------------------------
        content = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 710))
        style2 = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 711))
        t2 = torch.from_numpy(recipe.timesteps(2, 712))
        torch.manual_seed(11)
        out = ldm(content, style2, t2)
        G["fwd_eval_t"] = t2.numpy()
        for k in ("z_t", "noise", "noise_pred", "z_0", "reconstructed"):
            G[f"fwd_eval_{k}"] = np32(out[k])
        G["loss_diffusion"] = np32(L.diffusion_loss(out["noise_pred"], out["noise"]))
        G["loss_kl"] = np32(L.kl_regularization_loss(out["z_0"]))
        G["loss_mse"] = np32(torch.nn.MSELoss()(out["reconstructed"], content))

    # ---- (7) restated train step (train_step, train.py:163-208, fp32, no LPIPS / VGGish) --------
    ldm.train()
    for p in ldm.encoder.parameters():
        p.requires_grad_(False)
    trainable = [p for p in ldm.parameters() if p.requires_grad]
    opt = torch.optim.Adam(trainable, lr=5e-4)
    opt.zero_grad()
    torch.manual_seed(12)
    out = ldm(content, style2, t2)
    dl = L.diffusion_loss(out["noise_pred"], out["noise"])
    mse = torch.nn.MSELoss()(out["reconstructed"], content)
    kl = L.kl_regularization_loss(out["z_0"])
    total = mse + 0.01 * kl + dl
    total.backward()
    G["train_noise"] = np32(out["noise"])
    G["train_total"] = np32(total)
    G["train_recon"] = np32(out["reconstructed"])
    named = dict(ldm.named_parameters())
    for k in ("unet.time_mlp.1.weight", "unet.dec1.weight", "unet.dec1.bias", "unet.enc1.weight",
              "unet.cross_attention1.multihead_attn.in_proj_weight", "unet.bottleneck.bias",
              "decoder.decoder.6.weight", "decoder.decoder.1.weight", "style_encoder.enc6.bias",
              "style_encoder.enc1.weight"):
        g = named[k].grad
        G["grad_" + k] = np32(g[:256] if g.dim() == 2 and g.shape[0] > 256 else g)
    opt.step()
    for k in ("unet.dec1.weight", "decoder.decoder.6.weight", "style_encoder.enc6.bias"):
        G["adam1_" + k] = np32(named[k])
    G["train_enc_rm0"] = np32(ldm.encoder.encoder[1].running_mean)
    G["train_dec_rv1"] = np32(ldm.decoder.decoder[4].running_var)

    # API surface: state_dict keys / shapes of the reference LDM (checkpoint interchange, §8(b))
    import json
    ref = M.LDM(32, pretrained_path="")
    keys = {k: list(v.shape) for k, v in ref.state_dict().items()}
    with open(os.path.join(HERE, "ref_state_dict_keys.json"), "w") as f:
        json.dump(keys, f, indent=0, sort_keys=True)

    path = os.path.join(HERE, "ref_goldens.npz")
    np.savez_compressed(path, **G)
    print("wrote", path, os.path.getsize(path), "bytes,", len(G), "arrays")


def round2():
    """Round-2 fixtures -> tests/golden/ref_goldens_r2.npz (the round-1 file is left untouched).

    (8) content_style_transfer_wrapper end to end (model.py:468-501) at T'=100, eta=1 (config 5's
        "100-step DDPM"), B=1, 128x128 content/style: the wrapper draws its q_sample noise with
        torch.randn_like on the CPU generator right after torch.manual_seed(21) (nothing before it
        consumes RNG), so the same epsilon is regenerated here and stored for injection.
    (9) one train_autoencoder step (train.py:59-82): encoder + decoder in train mode (batch-statistics
        BN in both, gradients through the whole encoder), loss = compression_loss with the LPIPS term
        left out (weights are remote; loss.py:10) = MSE(recon, x) + 0.01 KL(latent), AdamW(lr=5e-4)."""
    torch.set_num_threads(8)
    M, L = import_reference()
    G = {}
    with torch.no_grad():
        ldm = M.LDM(32, pretrained_path="")
        recipe.fill_module(ldm, seed=700)
        ldm.eval()
        content = torch.from_numpy(recipe.uniform01((1, 1, 128, 128), 720))
        style = torch.from_numpy(recipe.uniform01((1, 1, 128, 128), 721))
        torch.manual_seed(21)
        decoded, z_t_decoded = ldm.content_style_transfer_wrapper(content, style, num_timesteps=100, eta=1.0)
        torch.manual_seed(21)
        eps = torch.randn((1, 32, 16, 16))
        # self-check: the wrapper's z_t is q_sample(encoder(content), T'-1, eps)
        z0 = ldm.encoder(content)
        ab = ldm.noise_scheduler.alpha_bar_t[99]
        zt = torch.sqrt(ab) * z0 + torch.sqrt(1 - ab) * eps
        assert torch.allclose((ldm.decoder(zt)), z_t_decoded, atol=0, rtol=0)
        G["cst100_eps"] = np32(eps)
        G["cst100_decoded"] = np32(decoded)
        G["cst100_zt_decoded"] = np32(z_t_decoded)

    enc = M.SpectrogramEncoder(32)
    dec = M.SpectrogramDecoder(32)
    recipe.fill_module(enc, seed=730)
    recipe.fill_module(dec, seed=731)
    enc.train()
    dec.train()
    opt = torch.optim.AdamW(list(enc.parameters()) + list(dec.parameters()), lr=5e-4)
    spec = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 732))
    latent = enc(spec)
    rec = dec(latent)
    loss = torch.nn.MSELoss()(rec, spec) + 0.01 * L.kl_regularization_loss(latent)
    opt.zero_grad()
    loss.backward()
    G["ae_latent"] = np32(latent)
    G["ae_recon"] = np32(rec)
    G["ae_loss"] = np32(loss)
    named = dict([("encoder." + k, v) for k, v in enc.named_parameters()] +
                 [("decoder." + k, v) for k, v in dec.named_parameters()])
    for k in AE_KEYS:
        G["ae_grad_" + k] = np32(named[k].grad)
    opt.step()
    for k in AE_KEYS:
        G["ae_adamw1_" + k] = np32(named[k])
    G["ae_enc_rm4"] = np32(enc.encoder[4].running_mean)
    G["ae_dec_rv1"] = np32(dec.decoder[1].running_var)
    path = os.path.join(HERE, "ref_goldens_r2.npz")
    np.savez_compressed(path, **G)
    print("wrote", path, os.path.getsize(path), "bytes,", len(G), "arrays")


def amp():
    """Reduced-precision fixtures -> tests/golden/ref_goldens_amp.npz: the reference reverse loops run under
    torch.autocast("cpu", dtype) (convs / linears / attention matmuls in fp16 or bf16, the scheduler
    arithmetic on the fp32 latent), at the canonical latent [1,32,16,64] (the reference loop logs t.item(),
    so it runs batch 1): a 10-step DDIM (eta 0, config 2's loop) in fp32 / bf16 / fp16, and the T'=100
    content-style loop (eta 1, config 5's "fp16 with fp32 scheduler accumulators") in fp32 / fp16.
    Style embedding computed in fp32 outside the autocast region."""
    torch.set_num_threads(8)
    M, L = import_reference()
    G = {}
    with torch.no_grad():
        ldm = M.LDM(32, pretrained_path="")
        recipe.fill_module(ldm, seed=700)
        ldm.eval()
        style = torch.from_numpy(recipe.uniform01((1, 1, 128, 512), 741))
        zT = torch.from_numpy(recipe.normal((1, 32, 16, 64), 742))
        emb = ldm.style_encoder(style)
        for name, dt in (("fp32", None), ("bf16", torch.bfloat16), ("fp16", torch.float16)):
            if dt is None:
                x, logs = ldm.style_conditioned_ddim_sample(zT, emb, timesteps=10, eta=0.0)
            else:
                with torch.autocast("cpu", dtype=dt):
                    x, logs = ldm.style_conditioned_ddim_sample(zT, emb, timesteps=10, eta=0.0)
            G[f"amp10_{name}_x"] = np32(x.float())
            G[f"amp10_{name}_times"] = np.array(logs["timesteps"], dtype=np.int64)
        for name, dt in (("fp32", None), ("fp16", torch.float16)):
            if dt is None:
                x, _ = ldm.content_style_ddim_sample(zT, emb, timesteps=100, eta=1.0)
            else:
                with torch.autocast("cpu", dtype=dt):
                    x, _ = ldm.content_style_ddim_sample(zT, emb, timesteps=100, eta=1.0)
            G[f"cs100_{name}_x"] = np32(x.float())
        # the restated train step of part (7) (fp32 golden: ref_goldens.npz train_*) with its forward and
        # losses under torch.autocast("cpu", bfloat16) -- the reference's own train_step region on a CPU
        # device (train.py:174) -- and backward outside it; the q_sample noise is injected (fp32, the
        # recorded train_noise) by standing in for torch.randn_like, which would otherwise draw it in the
        # autocast dtype of the encoder output.
    g1 = np.load(os.path.join(HERE, "ref_goldens.npz"))
    ldm = M.LDM(32, pretrained_path="")
    recipe.fill_module(ldm, seed=700)
    ldm.train()
    for p_ in ldm.encoder.parameters():
        p_.requires_grad_(False)
    content = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 710))
    style2 = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 711))
    t2 = torch.from_numpy(recipe.timesteps(2, 712))
    noise = torch.from_numpy(g1["train_noise"])
    real_randn_like = torch.randn_like
    torch.randn_like = lambda t, *a, **k: noise.clone()
    try:
        with torch.autocast("cpu", dtype=torch.bfloat16):
            out = ldm(content, style2, t2)
            dl = L.diffusion_loss(out["noise_pred"], out["noise"])
            mse = torch.nn.MSELoss()(out["reconstructed"], content)
            kl = L.kl_regularization_loss(out["z_0"])
            total = mse + 0.01 * kl + dl
    finally:
        torch.randn_like = real_randn_like
    total.backward()
    G["trainbf16_total"] = np32(total.float())
    G["trainbf16_recon"] = np32(out["reconstructed"].float())
    named = dict(ldm.named_parameters())
    for k in TRAIN_GRAD_KEYS:
        g = named[k].grad
        G["trainbf16_grad_" + k] = np32(g[:256] if g.dim() == 2 and g.shape[0] > 256 else g)
    path = os.path.join(HERE, "ref_goldens_amp.npz")
    np.savez_compressed(path, **G)
    print("wrote", path, os.path.getsize(path), "bytes,", len(G), "arrays")


def amp8():
    """Config 5 at its bench shard -> tests/golden/ref_goldens_amp8.npz: content_style_ddim_sample (T'=100,
    eta=1) at batch 8 on the canonical [8,32,16,64] latent under torch.autocast("cpu", float16), as
    bench.py --workload transfer runs it per GPU.  The reference loop logs t.item(), which raises for batch >
    1 (model.py:555), so it runs eight times at batch 1 (sample b: z_T[b], style[b]; the loop and the UNet are
    per-sample) and the results are stacked; fp32 likewise, for the reference's own autocast-vs-fp32 gap.
    Style embeddings in fp32 outside the autocast region, as in amp()."""
    torch.set_num_threads(8)
    M, L = import_reference()
    G = {}
    B = 8
    with torch.no_grad():
        ldm = M.LDM(32, pretrained_path="")
        recipe.fill_module(ldm, seed=700)
        ldm.eval()
        style = torch.from_numpy(recipe.uniform01((B, 1, 128, 512), 751))
        zT = torch.from_numpy(recipe.normal((B, 32, 16, 64), 752))
        for name, dt in (("fp32", None), ("fp16", torch.float16)):
            xs = []
            for b in range(B):
                emb = ldm.style_encoder(style[b:b + 1])
                if dt is None:
                    x, _ = ldm.content_style_ddim_sample(zT[b:b + 1], emb, timesteps=100, eta=1.0)
                else:
                    with torch.autocast("cpu", dtype=dt):
                        x, _ = ldm.content_style_ddim_sample(zT[b:b + 1], emb, timesteps=100, eta=1.0)
                xs.append(x.float())
            G[f"cs100b8_{name}_x"] = np32(torch.cat(xs, 0))
    path = os.path.join(HERE, "ref_goldens_amp8.npz")
    np.savez_compressed(path, **G)
    print("wrote", path, os.path.getsize(path), "bytes,", len(G), "arrays")


def vggish_stack():
    """A VGGish-shaped `features` stack (3x3 convs 64-M-128-M-256-256-M-512-512-M, ReLU after each conv,
    MaxPool2d(2, 2)): the architecture torchvggish's VGG.features is built from; the weights are the
    recipe's (the real ones are a remote download, loss.py:56)."""
    layers, cin = [], 1
    for v in (64, "M", 128, "M", 256, 256, "M", 512, 512, "M"):
        if v == "M":
            layers.append(torch.nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers += [torch.nn.Conv2d(cin, v, kernel_size=3, padding=1), torch.nn.ReLU(inplace=True)]
            cin = v
    return torch.nn.Sequential(*layers)


VGG_CASES = {"a": ((2, 1, 32, 64), 800), "odd": ((2, 1, 20, 36), 810)}


def vggish():
    """(10) VGGishFeatureLoss.forward (loss.py:64-101) -> tests/golden/ref_goldens_vggish.npz: the REFERENCE
    class, instantiated without its constructor (a remote torch.hub fetch, loss.py:56) and given a recipe-
    filled VGGish-shaped stack; inputs U[0,1) like spectrograms.  Case 'odd' exercises floor-mode pooling."""
    torch.set_num_threads(8)
    _, L = import_reference()
    G = {}
    for name, (shape, seed) in VGG_CASES.items():
        feats = vggish_stack()
        recipe.fill_module(feats, seed=seed)
        feats.eval()
        obj = L.VGGishFeatureLoss.__new__(L.VGGishFeatureLoss)
        torch.nn.Module.__init__(obj)
        obj.features = feats
        pred = torch.from_numpy(recipe.uniform01(shape, seed + 1))
        targ = torch.from_numpy(recipe.uniform01(shape, seed + 2))
        G[f"vgg_{name}_loss"] = np32(obj(pred, targ))
    path = os.path.join(HERE, "ref_goldens_vggish.npz")
    np.savez_compressed(path, **G)
    print("wrote", path, os.path.getsize(path), "bytes,", len(G), "arrays", {k: float(v) for k, v in G.items()})


R3_B, R3_H, R3_W = 32, 128, 512


def r3_inputs():
    """Config 3's benchmarked shape: batch 32, 1x128x512 content / style mels, t, injected q_sample noise."""
    content = torch.from_numpy(recipe.uniform01((R3_B, 1, R3_H, R3_W), 760))
    style = torch.from_numpy(recipe.uniform01((R3_B, 1, R3_H, R3_W), 761))
    t = torch.from_numpy(recipe.timesteps(R3_B, 762))
    noise = torch.from_numpy(recipe.normal((R3_B, 32, R3_H // 8, R3_W // 8), 763))
    return content, style, t, noise


def round3():
    """(11) LDMTrainer.train_step's arithmetic at config 3's benchmarked shape -> ref_goldens_r3.npz: batch 32,
    1x128x512 mels, LDM(32, pretrained_path='') with recipe weights (seed 700) and every module in train mode
    (the bench's model: the encoder is trainable too, its BN uses batch statistics), loss = MSE(recon, x) +
    0.01 KL(z0) + MSE(eps_pred, eps) (LPIPS / VGGish left out: remote weights), q_sample noise injected.  Once
    in fp32 and once with forward + losses under torch.autocast("cpu", bfloat16) (train.py:174's region),
    backward outside.  Stored: the loss terms, reconstructed samples 0 and 31, the ten TRAIN_GRAD_KEYS
    gradients (in_proj rows 0..255); and all of it again with the reference model in float64."""
    torch.set_num_threads(8)
    M, L = import_reference()
    G = {}
    content, style, t, noise = r3_inputs()
    G["r3_t"] = t.numpy()
    for name, dt in (("fp32", None), ("bf16", torch.bfloat16)):
        ldm = M.LDM(32, pretrained_path="")
        recipe.fill_module(ldm, seed=700)
        ldm.train()
        real_randn_like = torch.randn_like
        torch.randn_like = lambda x, *a, **k: noise.clone()
        try:
            with torch.autocast("cpu", dtype=torch.bfloat16, enabled=dt is not None):
                out = ldm(content, style, t)
                dl = L.diffusion_loss(out["noise_pred"], out["noise"])
                mse = torch.nn.MSELoss()(out["reconstructed"], content)
                kl = L.kl_regularization_loss(out["z_0"])
                comp = mse + 0.01 * kl
                total = comp + dl
        finally:
            torch.randn_like = real_randn_like
        total.backward()
        G[f"r3_{name}_compression"] = np32(comp.float())
        G[f"r3_{name}_diffusion"] = np32(dl.float())
        G[f"r3_{name}_total"] = np32(total.float())
        G[f"r3_{name}_recon_0_31"] = np32(out["reconstructed"].float()[[0, R3_B - 1]])
        named = dict(ldm.named_parameters())
        for k in TRAIN_GRAD_KEYS:
            g = named[k].grad
            G[f"r3_{name}_grad_" + k] = np32(g[:256] if g.dim() == 2 and g.shape[0] > 256 else g)
        print(name, float(total), flush=True)
    # the same step in float64 (LDM.forward casts its inputs to fp32, model.py:357, so the reference cannot run
    # it in float64 itself): the oracle's restatement (oracle/ldm_torch_cpu.py, pinned to the fp32 golden by
    # tests/test_oracle_golden.py) on float64 recipe weights -- the reference's own fp32 error, per quantity
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import ldm_torch_cpu as TC
    ldm = M.LDM(32, pretrained_path="")
    recipe.fill_module(ldm, seed=700)
    sd = {k: v.detach().double().clone() for k, v in ldm.state_dict().items()}
    for k, v in sd.items():
        if v.is_floating_point() and "running_" not in k and not k.startswith("noise_scheduler"):
            v.requires_grad_(True)
    ab = M.ForwardDiffusion(200).alpha_bar_t.double()
    o = TC.ldm_forward(sd, content.double(), style.double(), t, noise.double(), ab, train_decoder=True,
                       train_encoder=True, state={})
    dl = torch.mean((o["noise_pred"] - o["noise"]) ** 2)
    comp = torch.mean((o["reconstructed"] - content.double()) ** 2) + 0.01 * TC.kl_loss(o["z_0"])
    (comp + dl).backward()
    G["r3_fp64_compression"] = comp.detach().numpy()
    G["r3_fp64_diffusion"] = dl.detach().numpy()
    G["r3_fp64_total"] = (comp + dl).detach().numpy()
    G["r3_fp64_recon_0_31"] = o["reconstructed"].detach()[[0, R3_B - 1]].numpy()
    for k in TRAIN_GRAD_KEYS:
        g = sd[k].grad
        G["r3_fp64_grad_" + k] = (g[:256] if g.dim() == 2 and g.shape[0] > 256 else g).numpy()

    # (12) width-general attention: the UNet on a latent wider than 64 tokens per cross-attention --
    # [1,32,16,128] (a 1x128x1024 mel: CA2 L = S = 128, CA1 32) -- forward and a 5-step DDIM (eta 0); and
    # a reduced SURVEY shape S: UNet(1, 1, 64) straight on a [1,1,64,256] mel with s5 [1,256,16,64] and
    # s6 [1,512,8,32] (CA2 L = S = 1024, CA1 256).
    with torch.no_grad():
        unet = M.UNet(32, 32, 64)
        recipe.fill_module(unet, seed=100)
        z = torch.from_numpy(recipe.normal((1, 32, 16, 128), 770))
        s5 = torch.from_numpy(recipe.uniform01((1, 256, 4, 32), 771))
        s6 = torch.from_numpy(recipe.uniform01((1, 512, 2, 16), 772))
        t = torch.tensor([117])
        G["w128_unet_out"] = np32(unet(z, t, {"s5": s5, "s6": s6}))
        ldm = M.LDM(32, pretrained_path="")
        recipe.fill_module(ldm, seed=700)
        ldm.eval()
        style = torch.from_numpy(recipe.uniform01((1, 1, 128, 1024), 773))
        emb = ldm.style_encoder(style)
        zT = torch.from_numpy(recipe.normal((1, 32, 16, 128), 774))
        x, _ = ldm.style_conditioned_ddim_sample(zT, emb, timesteps=5, eta=0.0)
        G["w128_ddim5_x"] = np32(x)
        us = M.UNet(1, 1, 64)
        recipe.fill_module(us, seed=101)
        zs = torch.from_numpy(recipe.normal((1, 1, 64, 256), 775))
        s5s = torch.from_numpy(recipe.uniform01((1, 256, 16, 64), 776))
        s6s = torch.from_numpy(recipe.uniform01((1, 512, 8, 32), 777))
        G["shapeS_unet_out"] = np32(us(zs, torch.tensor([42]), {"s5": s5s, "s6": s6s}))
    path = os.path.join(HERE, "ref_goldens_r3.npz")
    np.savez_compressed(path, **G)
    print("wrote", path, os.path.getsize(path), "bytes,", len(G), "arrays")


def fp16train():
    """(13) The reference's DEFAULT train-step precision -> ref_goldens_fp16.npz: LDMTrainer.train_step
    (train.py:163-208) with its own torch.autocast region (device default: float16 on a GPU, train.py:174) and
    its GradScaler (train.py:157, :189-201; init scale 2^16, growth 2, backoff 0.5, interval 2000), Adam(lr=1e-4)
    (LDMTrainer default), at config 3's shape and inputs (r3_inputs: batch 32, 1x128x512, recipe seed 700,
    every module in train mode, q_sample noise injected).  On the CPU the region is torch.autocast("cpu",
    float16) and the scaler torch.amp.GradScaler("cpu") (same defaults and the same unscale / inf-check / update
    arithmetic as 'cuda').  Loss = compression (MSE + 0.01 KL; LPIPS left out, remote weights) + diffusion +
    0.1 x style (VGGish stubbed to 0), as the reference adds them.

    Two steps: (A) at the default scale 2^16 -- loss terms, reconstructed samples 0 / 31, the unscaled
    TRAIN_GRAD_KEYS gradients, whether the scaler found an inf, the scale after update(); (B) the scale set
    to 2^40 with update(new_scale=...) first, so the fp16 backward overflows: found-inf, the step skipped
    (parameters and Adam state untouched), the scale backed off to 2^39."""
    torch.set_num_threads(8)
    M, L = import_reference()
    G = {}
    content, style, t, noise = r3_inputs()
    ldm = M.LDM(32, pretrained_path="")
    recipe.fill_module(ldm, seed=700)
    ldm.train()
    trainable = [p for p in ldm.parameters() if p.requires_grad]
    opt = torch.optim.Adam(trainable, lr=1e-4)
    scaler = torch.amp.GradScaler("cpu")
    named = dict(ldm.named_parameters())

    def train_step():
        opt.zero_grad()
        real_randn_like = torch.randn_like
        torch.randn_like = lambda x, *a, **k: noise.clone()
        try:
            with torch.autocast("cpu", dtype=torch.float16):
                out = ldm(content.float(), style.float(), t)
            # the loss terms with CUDA autocast's semantics: mse_loss, pow and log are on its fp32 list (their
            # 16-bit inputs cast to fp32), so on a GPU the reference computes every term below in fp32.  CPU
            # autocast keeps pow / log in fp16, where KL's + 1e-8 underflows to 0 and log(0) makes the loss inf,
            # which the reference on a GPU never sees: the terms are taken on the fp32 casts instead.
            dl = L.diffusion_loss(out["noise_pred"].float(), out["noise"].float())
            mse = torch.nn.MSELoss()(out["reconstructed"].float(), content)
            kl = L.kl_regularization_loss(out["z_0"].float())
            comp = mse + 0.01 * kl
            style_l = torch.zeros(())
            total = comp + dl + 0.1 * style_l
        finally:
            torch.randn_like = real_randn_like
        scaler.scale(total).backward()
        scaler.step(opt)
        found = float(sum(v.item() for v in scaler._found_inf_per_device(opt).values()))
        scaler.update()
        return out, comp, dl, total, found

    before = {k: named[k].detach().clone() for k in TRAIN_GRAD_KEYS}
    out, comp, dl, total, found = train_step()
    G["fp16_a_found_inf"] = np.float32(found)
    G["fp16_a_scale_after"] = np.float32(scaler.get_scale())
    G["fp16_compression"] = np32(comp.float())
    G["fp16_diffusion"] = np32(dl.float())
    G["fp16_total"] = np32(total.float())
    G["fp16_recon_0_31"] = np32(out["reconstructed"].float()[[0, R3_B - 1]])
    for k in TRAIN_GRAD_KEYS:
        g = named[k].grad
        G["fp16_grad_" + k] = np32(g[:256] if g.dim() == 2 and g.shape[0] > 256 else g)
    G["fp16_a_param_moved"] = np.array([float((named[k].detach() - before[k]).abs().max()) for k in TRAIN_GRAD_KEYS],
                                       dtype=np.float32)
    print("step A: compression", float(comp), "diffusion", float(dl), "total", float(total), "found_inf", found, "scale after", scaler.get_scale(), flush=True)
    snap = {k: named[k].detach().clone() for k in TRAIN_GRAD_KEYS}
    steps = [opt.state[named[k]]["step"].clone() if named[k] in opt.state else None for k in TRAIN_GRAD_KEYS]
    scaler.update(new_scale=2.0 ** 40)
    out, comp, dl, total, found = train_step()
    G["fp16_b_found_inf"] = np.float32(found)
    G["fp16_b_scale_after"] = np.float32(scaler.get_scale())
    G["fp16_b_total"] = np32(total.float())
    G["fp16_b_params_unchanged"] = np.float32(all(torch.equal(named[k], snap[k]) for k in TRAIN_GRAD_KEYS))
    G["fp16_b_adam_step_unchanged"] = np.float32(all(
        s is None or torch.equal(opt.state[named[k]]["step"], s) for k, s in zip(TRAIN_GRAD_KEYS, steps)))
    print("step B: total", float(total), "found_inf", found, "scale after", scaler.get_scale(),
          "params unchanged", bool(G["fp16_b_params_unchanged"]), flush=True)
    path = os.path.join(HERE, "ref_goldens_fp16.npz")
    np.savez_compressed(path, **G)
    print("wrote", path, os.path.getsize(path), "bytes,", len(G), "arrays")


TRAIN_GRAD_KEYS = ("unet.time_mlp.1.weight", "unet.dec1.weight", "unet.dec1.bias", "unet.enc1.weight",
                   "unet.cross_attention1.multihead_attn.in_proj_weight", "unet.bottleneck.bias",
                   "decoder.decoder.6.weight", "decoder.decoder.1.weight", "style_encoder.enc6.bias",
                   "style_encoder.enc1.weight")

AE_KEYS = ("encoder.encoder.0.weight", "encoder.encoder.1.weight", "encoder.encoder.4.bias", "encoder.encoder.6.bias",
           "encoder.encoder.7.weight", "decoder.decoder.0.weight", "decoder.decoder.1.bias", "decoder.decoder.4.weight",
           "decoder.decoder.6.weight", "decoder.decoder.6.bias")


if __name__ == "__main__":
    if "--fp16train" in sys.argv:
        fp16train()
    elif "--r2" in sys.argv:
        round2()
    elif "--r3" in sys.argv:
        round3()
    elif "--amp8" in sys.argv:
        amp8()
    elif "--amp" in sys.argv:
        amp()
    elif "--vggish" in sys.argv:
        vggish()
    else:
        main()
