"""Layer pairs of the reverse loop (csrc/uconv.hip upair_kernel, ldm_step_set_pairs).

A pair runs two consecutive step layers as ONE launch: the first layer's blocks publish their output tiles with
write-through stores and count themselves on a sharded counter; the second layer's blocks stream their weights,
wait for the count, then read the tiles.  These tests run the benchmarked configuration (config 2: B = 8,
[8,32,16,64] latent, 50-step DDIM, folded cross-attentions, step kernels, one hipGraph) with each pair on, and
with all of them on, against the fixture-pinned oracle (1e-4, north_star) and against the loop without pairs
(1e-5: a pair changes only which step instance runs a layer, e.g. uconv instead of ustep for enc1, so the
summation order of that layer's K reduction).  Replaying a graph several times checks that the counters return
to zero after every launch.

Reference: /root/reference/models/model.py:409-465 (the loop), :163-231 (the UNet).
"""
import numpy as np
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _diag_build_only(cuda):
    from ldm_amd import _lib as L
    if not L.load().ldm_step_diag_build():
        pytest.skip("layer pairs are in the diagnostic build only (make DIAG=1, LDM_AMD_LIB=lib/libldm_amd_diag.so)")
TOL = 1e-4
PAIRS = [0x1, 0x40, 0x80, 0x1 | 0x40, 0x1 | 0x80]


def npy(t):
    return t.detach().double().cpu().numpy()


@pytest.fixture(scope="module")
def loop_setup(cuda):
    import models.model as M
    torch.manual_seed(0)
    ldm = M.LDM(32, pretrained_path="").to(cuda).eval()
    B = 8
    g = torch.Generator().manual_seed(1)
    style = torch.rand(B, 1, 128, 512, generator=g).to(cuda)
    torch.manual_seed(1234)
    z_T = torch.randn((B, 32, 16, 64)).to(cuda)
    times = torch.linspace(ldm.num_timesteps - 1, 0, 50).long()
    coefs = ldm.noise_scheduler.reverse_coefs(times).to(cuda)
    t_table = times[:-1].view(-1, 1).expand(-1, B).contiguous().to(cuda)
    with torch.no_grad():
        emb = ldm.style_encoder(style)
    return dict(ldm=ldm, style=style, z_T=z_T, times=times, coefs=coefs, t_table=t_table, emb=emb)


def _run(o, mask, replays=3):
    import models.model as M
    from ldm_amd import _lib as L
    from ldm_amd.engine import GraphedDDIM
    lib = L.load()
    prev = lib.ldm_step_set_pairs(mask)
    try:
        with torch.no_grad():
            eng = M.engine_for(o["ldm"].unet)
            gd = GraphedDDIM(eng, o["z_T"], o["emb"]["s5"], o["emb"]["s6"], o["t_table"], o["coefs"], 0.0, logs=True)
            outs = []
            for _ in range(replays):
                gd.replay()
                outs.append(gd.x.clone())
        torch.cuda.synchronize()
    finally:
        lib.ldm_step_set_pairs(prev)
    return outs, gd


@pytest.fixture(scope="module")
def oracle_x(loop_setup):
    from oracle import ldm_torch_cpu as TC
    o = loop_setup
    sd = {k: v.detach().float().cpu() for k, v in o["ldm"].state_dict().items()}
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    with torch.no_grad():
        emb_ref = TC.style_encoder(sd, o["style"].cpu())
        ab = TC.schedule(200)[2]
        x_ref = TC.reverse_loop(sd, ab, o["z_T"].cpu(), emb_ref["s5"], emb_ref["s6"], o["times"], 0.0)
    return x_ref.double().numpy()


@pytest.fixture(scope="module")
def no_pair_x(loop_setup):
    outs, _ = _run(loop_setup, 0, replays=1)
    return npy(outs[0])


@pytest.mark.parametrize("mask", PAIRS, ids=[hex(m) for m in PAIRS])
def test_pairs_match_oracle_and_unpaired_loop(loop_setup, oracle_x, no_pair_x, mask):
    outs, gd = _run(loop_setup, mask)
    for x in outs:   # every replay restarts from z_T: the counters were back at zero
        assert torch.equal(x, outs[0]), "a replay of the paired loop differs from the first"
    x = npy(outs[0])
    assert np.isfinite(x).all()
    assert rel_err(x, oracle_x) < TOL
    assert rel_err(x, no_pair_x) < 1e-5


def test_set_pairs_roundtrip():
    from ldm_amd import _lib as L
    lib = L.load()
    prev = lib.ldm_step_set_pairs(-1)
    assert lib.ldm_step_set_pairs(0x41) == prev
    assert lib.ldm_step_set_pairs(-1) == 0x41
    lib.ldm_step_set_pairs(prev)
