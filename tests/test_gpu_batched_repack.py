"""Batched weight re-pack of the train step (pack.hip ldm_pack_many, ops.PackSet, models/train.py).

* Every recorded pack (conv kinds 1/2 in fp32, the 16-bit kind-3 tconv packs under fp16 and bf16 autocast,
  forward and data-gradient duals, in_proj slices) re-packed by the one launch equals the pack
  ldm_conv_pack_weight makes of the same weight, bitwise.
* A trainer with the batched re-pack and one without it (LDM_AMD_BATCHED_REPACK=0 path) take bitwise equal
  steps, eager and graphed, and an eager forward after the steps reads current packs.
"""
import ctypes

import pytest
import torch

import recipe

pytestmark = pytest.mark.gpu


class _ZeroFeat(torch.nn.Module):
    def forward(self, a, b):
        return torch.zeros((), device=a.device)


def _model(cuda, seed=700):
    import models.model as M
    m = M.LDM(32, pretrained_path="")
    recipe.fill_module(m, seed=seed)
    m.feature_loss_net = _ZeroFeat()
    return m.to(cuda).train()


def _inputs(cuda, seed, B=2):
    content = torch.from_numpy(recipe.uniform01((B, 1, 128, 128), seed)).to(cuda)
    style = torch.from_numpy(recipe.uniform01((B, 1, 128, 128), seed + 1)).to(cuda)
    t = torch.tensor([17, 160] * (B // 2), device=cuda)
    noise = torch.from_numpy(recipe.normal((B, 32, 16, 16), seed + 2)).to(cuda)
    return content, style, t, noise


@pytest.mark.parametrize("precision", ["fp32", "fp16", "bf16"])
def test_pack_many_equals_single_packs(cuda, precision):
    import models.train as TR
    from ldm_amd import _lib as L
    from ldm_amd import ops
    m = _model(cuda)
    tr = TR.LDMTrainer(m, [], cuda, lr=1e-3)
    tr.autocast_enabled = precision != "fp32"
    tr.autocast_dtype = {"fp16": torch.float16, "bf16": torch.bfloat16}.get(precision)
    tr.train_step(*_inputs(cuda, 300, B=8))       # B = 8: the 64-channel VAE / style layers take kind 3
    ps = tr._packset
    assert ps is not None and ps.n >= 40, "the step's trainable packs were not recorded"
    kinds = {int(p.kind) for p in ps.plans}
    assert kinds >= ({1, 3} if precision != "fp32" else {1}), kinds
    if precision == "bf16":   # the small-plane layers' kind-4 packs (sconv.hip) are refreshed by the batch too
        assert 4 in kinds, kinds
    assert any(t[0] is not None for t in ps.tails), "no in_proj slice pack recorded"
    for b in ps.bufs:
        b.zero_()
    ps.repack()
    torch.cuda.synchronize()
    for i, (buf, wptr) in enumerate(zip(ps.bufs, ps.wptrs)):
        d, p = ps.descs[i], ps.plans[i]
        fresh = torch.zeros_like(buf)
        L.call("ldm_conv_pack_weight", ctypes.byref(d), ctypes.byref(p), wptr, fresh.data_ptr(),
               ops.stream_handle())
        torch.cuda.synchronize()
        assert torch.equal(buf, fresh), (i, int(p.kind), ps.tails[i])


@pytest.mark.parametrize("graph", [False, True])
def test_trainer_with_and_without_batched_repack(cuda, graph):
    import models.train as TR
    res = []
    for batched in (False, True):
        m = _model(cuda, seed=710)
        tr = TR.LDMTrainer(m, [], cuda, lr=1e-3)
        tr.autocast_dtype = torch.float16
        tr.batched_repack = batched
        tr.graph_step = graph
        losses = [tr.train_step(*_inputs(cuda, 320 + 3 * i, B=8)) for i in range(5)]
        assert (tr._packset is not None) == batched
        m.eval()
        with torch.no_grad():
            out = m(*_inputs(cuda, 400)[:3], noise=_inputs(cuda, 400)[3])["reconstructed"].clone()
        m.train()
        res.append((losses, {k: v.detach().clone() for k, v in m.state_dict().items()}, out))
    (l0, s0, o0), (l1, s1, o1) = res
    assert l0 == l1
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k
    assert torch.equal(o0, o1)


def test_weights_changed_between_replays_are_repacked(cuda):
    """load_state_dict between graph replays (in-place copies into the same storage): the next replay reads
    packs of the loaded weights (the graph's forward no longer packs them itself)."""
    import models.train as TR
    ins = _inputs(cuda, 500)
    m = _model(cuda, seed=720)
    tr = TR.LDMTrainer(m, [], cuda, lr=1e-3)
    tr.autocast_enabled = False
    tr.graph_step = True
    for _ in range(4):
        tr.train_step(*ins)
    assert tr._graph is not None
    donor = _model(cuda, seed=721)
    m.load_state_dict(donor.state_dict())
    got = tr.train_step(*ins)
    # the same single step from the loaded state on an eager trainer without the batched re-pack
    ref_m = _model(cuda, seed=721)
    ref_tr = TR.LDMTrainer(ref_m, [], cuda, lr=1e-3)
    ref_tr.autocast_enabled = False
    ref_tr.batched_repack = False
    ref = ref_tr.train_step(*ins)      # (the optimizer states differ; the step's losses come before it)
    assert got["compression_loss"] == ref["compression_loss"]
    assert got["denoisinsg_loss"] == ref["denoisinsg_loss"]
