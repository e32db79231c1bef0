"""The reference's own model tests, mirrored 1:1 on the drop-in API (reference models/tests.py:153-463).

Each test keeps the reference's shapes, batch size, input distribution and assertions (output shapes, the
tanh range, finiteness), runs the modules in their default (train-mode BatchNorm) state exactly as the
reference constructs them, and adds one value check the reference does not make: the HIP result against
the oracle's fp32 CPU restatement on the same weights and inputs, max|y - y_ref| <= 1e-4 * max|y_ref|
(north_star tolerance).  Weights: torch's default init under a fixed seed (the reference's tests use the
default init too).
"""
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _sd(m):
    return {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}


def _randn(shape, seed):
    return torch.randn(shape, generator=torch.Generator().manual_seed(seed))


def test_encoder_dimensions(cuda):
    """tests.py:153-174: B=4, 1x128x128 -> [4, latent_dim, 16, 16]."""
    import models.model as M
    from models.config import config
    from oracle import ldm_torch_cpu as TC
    torch.manual_seed(1)
    latent_dim = config["latent_dim_encoder"]
    enc = M.SpectrogramEncoder(latent_dim=latent_dim)
    sd = {"encoder." + k: v for k, v in _sd(enc).items()}
    enc = enc.to(cuda)
    x = _randn((4, 1, 128, 128), 11)
    latent = enc(x.to(cuda))
    assert latent.shape == (4, latent_dim, 16, 16)
    ref = TC.encoder(sd, x, train=True, state={})
    assert rel_err(latent.detach().cpu().numpy(), ref.numpy()) < TOL


def test_decoder_dimensions(cuda):
    """tests.py:176-195: B=4, [4, latent_dim, 16, 16] -> [4, 1, 128, 128]."""
    import models.model as M
    from models.config import config
    from oracle import ldm_torch_cpu as TC
    torch.manual_seed(2)
    latent_dim = config["latent_dim_encoder"]
    dec = M.SpectrogramDecoder(latent_dim=latent_dim)
    sd = {"decoder." + k: v for k, v in _sd(dec).items()}
    dec = dec.to(cuda)
    z = _randn((4, latent_dim, 16, 16), 12)
    out = dec(z.to(cuda))
    assert out.shape == (4, 1, 128, 128)
    ref = TC.decoder(sd, z, train=True, state={})
    assert rel_err(out.detach().cpu().numpy(), ref.numpy()) < TOL


def test_encoder_decoder_pipeline(cuda):
    """tests.py:197-222: latent_dim 4, B=4, 1x256x256 in U[-1,1) -> same shape, output in [-1, 1]."""
    import models.model as M
    from oracle import ldm_torch_cpu as TC
    torch.manual_seed(3)
    enc, dec = M.SpectrogramEncoder(latent_dim=4), M.SpectrogramDecoder(latent_dim=4)
    sd = {**{"encoder." + k: v for k, v in _sd(enc).items()}, **{"decoder." + k: v for k, v in _sd(dec).items()}}
    enc, dec = enc.to(cuda), dec.to(cuda)
    x = torch.rand((4, 1, 256, 256), generator=torch.Generator().manual_seed(13)) * 2 - 1
    latent = enc(x.to(cuda))
    rec = dec(latent)
    assert x.shape == rec.shape
    assert bool(torch.all(rec >= -1)) and bool(torch.all(rec <= 1))
    ref = TC.decoder(sd, TC.encoder(sd, x, train=True, state={}), train=True, state={})
    assert rel_err(rec.detach().cpu().numpy(), ref.numpy()) < TOL


def test_decoder_output_range(cuda):
    """tests.py:224-242: latent_dim 4, B=4, 8x8 latent: finite, in the tanh range."""
    import models.model as M
    from oracle import ldm_torch_cpu as TC
    torch.manual_seed(4)
    dec = M.SpectrogramDecoder(latent_dim=4)
    sd = {"decoder." + k: v for k, v in _sd(dec).items()}
    dec = dec.to(cuda)
    z = _randn((4, 4, 8, 8), 14)
    out = dec(z.to(cuda))
    assert out.shape == (4, 1, 64, 64)
    assert bool(torch.all(torch.isfinite(out)))
    assert bool(torch.all(out >= -1)) and bool(torch.all(out <= 1))
    ref = TC.decoder(sd, z, train=True, state={})
    assert rel_err(out.detach().cpu().numpy(), ref.numpy()) < TOL


def test_style_encoder_dimensions(cuda):
    """tests.py:378-421: B=4, 1x128x128 -> s1..s6 at the six resolutions."""
    import models.model as M
    from oracle import ldm_torch_cpu as TC
    torch.manual_seed(5)
    se = M.StyleEncoder(in_channels=1, num_filters=64)
    sd = {"style_encoder." + k: v for k, v in _sd(se).items()}
    assert sum(p.numel() for p in se.parameters()) == 2729984
    se = se.to(cuda)
    x = _randn((4, 1, 128, 128), 15)
    emb = se(x.to(cuda))
    expected = {"s1": (4, 64, 64, 64), "s2": (4, 128, 32, 32), "s3": (4, 256, 16, 16), "s4": (4, 256, 8, 8),
                "s5": (4, 256, 4, 4), "s6": (4, 512, 2, 2)}
    ref = TC.style_encoder(sd, x)
    for k, shp in expected.items():
        assert emb[k].shape == shp, k
        assert rel_err(emb[k].detach().cpu().numpy(), ref[k].numpy()) < TOL, k


@pytest.mark.parametrize("grad", [False, True])
def test_unet_dimensions(cuda, grad):
    """tests.py:424-463: UNet(32, 32, 64), B=4, 16x16 latent, FLOAT t = zeros, s1..s6 dict -> same shape.
    grad=False runs the fused engine (no-grad), grad=True the per-layer autograd path."""
    import models.model as M
    from oracle import ldm_torch_cpu as TC
    torch.manual_seed(6)
    unet = M.UNet(in_channels=32, out_channels=32, num_filters=64)
    assert sum(p.numel() for p in unet.parameters()) == 6841504
    sd = {"unet." + k: v for k, v in _sd(unet).items()}
    unet = unet.to(cuda)
    x = _randn((4, 32, 16, 16), 16)
    t = torch.zeros(4)
    shapes = {"s1": (4, 64, 64, 64), "s2": (4, 128, 32, 32), "s3": (4, 256, 16, 16), "s4": (4, 256, 8, 8),
              "s5": (4, 256, 4, 4), "s6": (4, 512, 2, 2)}
    style = {k: _randn(s, 20 + i) for i, (k, s) in enumerate(shapes.items())}
    xd = x.to(cuda).requires_grad_(grad)
    with torch.set_grad_enabled(grad):
        z = unet(xd, t.to(cuda), {k: v.to(cuda) for k, v in style.items()})
    assert z.shape == (4, 32, 16, 16)
    assert z.requires_grad == grad
    ref = TC.unet(sd, x, t, style["s5"], style["s6"])
    assert rel_err(z.detach().cpu().numpy(), ref.numpy()) < TOL


def test_ldm_latent_dim4_sampling(cuda):
    """A latent width the fused engine does not take (the VAE's default latent_dim=4, model.py:14): the UNet
    runs per layer and the reverse loop is the per-step UNet + DDIM-update kernel.  3 DDIM steps (eta 1)
    against the oracle's reverse loop on the same weights, 1e-4."""
    import models.model as M
    from oracle import ldm_torch_cpu as TC
    torch.manual_seed(7)
    ldm = M.LDM(4, pretrained_path="").eval()
    sd = _sd(ldm)
    ldm = ldm.to(cuda)
    style = torch.rand((2, 1, 64, 64), generator=torch.Generator().manual_seed(17))
    zT = _randn((2, 4, 8, 8), 18)
    with torch.no_grad():
        emb = ldm.style_encoder(style.to(cuda))
        x, logs = ldm.style_conditioned_ddim_sample(zT.to(cuda), emb, timesteps=4, eta=1.0)
        embr = TC.style_encoder(sd, style)
        xr = TC.reverse_loop(sd, TC.schedule(200)[2], zT, embr["s5"], embr["s6"], TC.ddim_times(200, 4), 1.0)
    assert logs["timesteps"] == TC.ddim_times(200, 4)[:-1].tolist()
    assert rel_err(x.cpu().numpy(), xr.numpy()) < TOL
