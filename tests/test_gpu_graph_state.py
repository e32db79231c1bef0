"""State that a graph-replayed train step leaves behind (reference train.py:163-208 run as one hipGraph).

* Version-keyed caches (ops.packed_weight, UNetEngine bound weights) must never serve weights packed before
  a replay: graphed steps, an eager forward, more replays, another eager forward -- each eager forward equals
  the same forward of a fresh model loaded from the trainer's current state_dict (bitwise: same kernels).
* A learning-rate change after an eager forward re-captures with the pack inside the new graph: the run's
  parameters equal an all-eager trainer's bitwise.
* The capturable Adam's state_dict carries a CPU step per param (no shared device count, no private group
  entries): it loads into torch.optim.Adam and into the eager form, and the next step there matches
  torch.optim.Adam continuing from the same state (1e-6).
"""
import copy

import numpy as np
import pytest
import torch

import recipe
from conftest import rel_err

pytestmark = pytest.mark.gpu


class _ZeroFeat(torch.nn.Module):
    def forward(self, a, b):
        return torch.zeros((), device=a.device)


def _model(cuda):
    import models.model as M
    m = M.LDM(32, pretrained_path="")
    recipe.fill_module(m, seed=700)
    m.feature_loss_net = _ZeroFeat()
    return m.to(cuda).train()


def _eval_outputs(m, content, style, t, noise):
    """An eager no-grad forward through the packed-weight caches (LDM.forward) and the UNet engine."""
    m.eval()
    with torch.no_grad():
        out = m(content, style, t, noise=noise)
        z = out["z_t"]
        s = m.style_encoder(style)
        eps = m.unet(z, t, s)
    m.train()
    return out["reconstructed"].clone(), eps.clone()


def _fresh_outputs(m, cuda, content, style, t, noise):
    import models.model as M
    f = M.LDM(32, pretrained_path="")
    f.feature_loss_net = _ZeroFeat()
    f.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()})
    f = f.to(cuda)
    return _eval_outputs(f, content, style, t, noise)


def test_eager_forward_between_replays_sees_current_weights(cuda):
    import models.train as TR
    content = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 880)).to(cuda)
    style = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 881)).to(cuda)
    t = torch.tensor([20, 120], device=cuda)
    noise = torch.from_numpy(recipe.normal((2, 32, 16, 16), 882)).to(cuda)
    m = _model(cuda)
    tr = TR.LDMTrainer(m, [], cuda, lr=1e-3)
    tr.autocast_enabled = False
    tr.graph_step = True
    for _ in range(4):
        tr.train_step(content, style, t=t, noise=noise)
    assert tr._graph is not None
    for round_ in range(2):
        got = _eval_outputs(m, content, style, t, noise)
        ref = _fresh_outputs(m, cuda, content, style, t, noise)
        for a, b in zip(got, ref):
            assert torch.equal(a, b), f"eager forward after replays served stale packed weights (round {round_})"
        for _ in range(2):
            tr.train_step(content, style, t=t, noise=noise)


def test_recapture_after_eager_forward_equals_eager_trainer(cuda):
    import models.train as TR
    content = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 890)).to(cuda)
    style = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 891)).to(cuda)
    t = torch.tensor([5, 190], device=cuda)
    noise = torch.from_numpy(recipe.normal((2, 32, 16, 16), 892)).to(cuda)
    res = []
    for graph in (False, True):
        m = _model(cuda)
        tr = TR.LDMTrainer(m, [], cuda, lr=1e-3)
        tr.autocast_enabled = False
        tr.graph_step = graph
        losses = [tr.train_step(content, style, t=t, noise=noise) for _ in range(4)]
        _eval_outputs(m, content, style, t, noise)        # packs at the current version, outside any graph
        tr.optimizer.param_groups[0]["lr"] *= 0.5          # re-capture (graph) / next eager step
        losses += [tr.train_step(content, style, t=t, noise=noise) for _ in range(4)]
        res.append((losses, {k: v.detach().clone() for k, v in m.state_dict().items()}))
    (le, sde), (lg, sdg) = res
    for a, b in zip(le, lg):
        for k in a:
            assert a[k] == b[k], (k, a[k], b[k])
    for k in sde:
        assert torch.equal(sde[k], sdg[k]), k


def _rand(shape, seed):
    g = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(g.uniform(-1, 1, shape).astype(np.float32))


@pytest.mark.parametrize("target", ["torch", "eager", "capturable"])
def test_capturable_adam_state_dict_round_trip(cuda, target):
    from ldm_amd import optim as hoptim
    shapes = [(64, 32, 3, 3), (64,), (5000,)]
    ps = [torch.nn.Parameter(_rand(s, 10 + i).to(cuda)) for i, s in enumerate(shapes)]
    ps_ref = [torch.nn.Parameter(p.detach().cpu().clone()) for p in ps]
    mine = hoptim.Adam(ps, lr=5e-4, capturable=True)
    ref = torch.optim.Adam(ps_ref, lr=5e-4)
    for step in range(3):
        for i, (a, b) in enumerate(zip(ps_ref, ps)):
            g = _rand(a.shape, 100 * step + i)
            a.grad = g.clone()
            b.grad = g.to(cuda)
        ref.step()
        mine.step()
    sd = mine.state_dict()
    assert all(not k.startswith("_ldm") for g in sd["param_groups"] for k in g)
    steps = [st["step"] for st in sd["state"].values()]
    assert all(s.device.type == "cpu" and float(s) == 3.0 for s in steps)
    assert len({id(s) for s in steps}) == len(steps), "params share one step tensor"
    # load into a new optimizer over copies of the current parameters, one more step there and in ref
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    if target == "torch":
        qs = [torch.nn.Parameter(q.detach().cpu()) for q in qs]
        other = torch.optim.Adam(qs, lr=5e-4)
    else:
        other = hoptim.Adam(qs, lr=5e-4, capturable=(target == "capturable"))
    other.load_state_dict(copy.deepcopy(sd))   # (load_state_dict keeps same-device tensors by reference)
    for i, (a, b) in enumerate(zip(ps_ref, qs)):
        g = _rand(a.shape, 900 + i)
        a.grad = g.clone()
        b.grad = g.to(b.device)
    ref.step()
    other.step()
    for a, b in zip(ps_ref, qs):
        assert rel_err(b.detach().double().cpu().numpy(), a.detach().double().numpy()) < 1e-6
    st = other.state_dict()["state"]
    assert all(float(s["step"]) == 4.0 for s in st.values())
    # and the original (capturable) optimizer leaving its capturable form counts once per step too
    mine.capturable = False
    for i, b in enumerate(ps):
        b.grad = _rand(b.shape, 900 + i).to(cuda)
    mine.step()
    assert all(float(mine.state[p]["step"]) == 4.0 for p in ps)
    for a, b in zip(ps_ref, ps):
        assert rel_err(b.detach().double().cpu().numpy(), a.detach().double().numpy()) < 1e-6


def test_capture_allocation_reuses_a_scratch_block_of_the_same_capture(cuda):
    """The mechanism behind round 5's aperture violation in unscale_check_kernel: a tensor
    allocated while capturing may be a block that a temporary of the same capture used and freed, so the graph
    itself rewrites it at every replay.  A table written into such a block once, outside the graph's stream
    order (the reverted side-stream upload of the optimizer's slot rows), holds the scratch values by the time
    a later node reads it.  Plain torch ops, no kernel of this package: the allocator's behaviour alone."""
    from ldm_amd.graphs import capture
    n = 4096
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with capture(g):
        tmp = torch.empty(n, dtype=torch.int64, device=cuda)
        tmp.fill_(-7)                                   # a step's scratch: written, then freed
        scratch_ptr = tmp.data_ptr()
        del tmp
        table = torch.empty(n, dtype=torch.int64, device=cuda)
        seen = table * 1                                # a later node reads the "table"
    assert table.data_ptr() == scratch_ptr              # the capture handed the freed scratch block out again
    table.copy_(torch.arange(n, device=cuda))           # filled once, eagerly, after the capture
    g.replay()
    torch.cuda.synchronize()
    assert bool((seen == -7).all())                     # the replay's scratch write clobbered it


def test_slot_tables_are_built_and_filled_outside_the_capture(cuda):
    """ldm_amd.optim builds no device table inside a capture: without reserved buffers it raises; with them the
    captured launch reads a buffer allocated before the capture, which fill_captured() uploads after it ends
    (so no graph scratch can alias it and no copy node runs per replay)."""
    from ldm_amd import optim as hoptim
    from ldm_amd.graphs import capture
    ps = [torch.randn(1000, device=cuda), torch.randn(5000, device=cuda)]
    gs = [torch.randn_like(p) for p in ps]
    hoptim.scale_tensors_(gs, 1.0)                      # the chunk map of this size list: built eagerly
    torch.cuda.synchronize()
    hoptim._SlotTable._cache.clear()
    hoptim._SlotTable._reserve.clear()
    g = torch.cuda.CUDAGraph()
    with pytest.raises(RuntimeError, match="outside a graph capture"):
        with capture(g):
            hoptim.scale_tensors_(gs, 0.5)
    torch.cuda.synchronize()
    hoptim._SlotTable._cache.clear()
    tables = hoptim.reserve_capture_buffers(device=cuda)
    reserved = {int(r[1].data_ptr()) for r in hoptim._SlotTable._reserve}
    want = [gg.clone() * 0.5 for gg in gs]
    g = torch.cuda.CUDAGraph()
    with capture(g):
        hoptim.scale_tensors_(gs, 0.5)
    assert len(tables) == 1 and int(tables[0].slots.data_ptr()) in reserved
    hoptim.fill_captured(tables)
    g.replay()
    torch.cuda.synchronize()
    for a, b in zip(gs, want):
        assert torch.equal(a, b)
    hoptim.release_captured(tables)
