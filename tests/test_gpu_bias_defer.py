"""The convs' bias-gradient finalizes deferred to the end of the backward (ops.bias_grads_deferred,
ldm_act_backward_defer + ldm_act_finalize_many; LDMTrainer's step without a gradient all-reduce): trainers with and
without the deferral take bitwise equal steps, eager and graph-replayed, fp32 and bf16 autocast; every gradient the
deferral touches equals the immediate finalize's bits; the bcast (time-embedding) gradient is never deferred.
Reference: /root/reference/models/train.py:163-208 (the step), model.py:205-229 (the convs' biases).
"""
import pytest
import torch

import recipe

pytestmark = pytest.mark.gpu


class _ZeroFeat(torch.nn.Module):
    def forward(self, a, b):
        return torch.zeros((), device=a.device)


def _model(cuda, seed):
    import models.model as M
    m = M.LDM(32, pretrained_path="")
    recipe.fill_module(m, seed=seed)
    m.feature_loss_net = _ZeroFeat()
    return m.to(cuda).train()


def _inputs(cuda, seed, B=4):
    content = torch.from_numpy(recipe.uniform01((B, 1, 128, 128), seed)).to(cuda)
    style = torch.from_numpy(recipe.uniform01((B, 1, 128, 128), seed + 1)).to(cuda)
    t = torch.tensor([17, 160] * (B // 2), device=cuda)
    noise = torch.from_numpy(recipe.normal((B, 32, 16, 16), seed + 2)).to(cuda)
    return content, style, t, noise


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_trainer_with_and_without_deferred_bias_grads(cuda, monkeypatch, graph, precision):
    import models.train as TR
    res = []
    for defer in ("0", "1"):
        monkeypatch.setenv("LDM_AMD_DEFER_BIAS", defer)
        m = _model(cuda, seed=730)
        tr = TR.LDMTrainer(m, [], cuda, lr=1e-3)
        tr.autocast_enabled = precision != "fp32"
        tr.autocast_dtype = torch.bfloat16 if precision == "bf16" else None
        tr.graph_step = graph
        losses = [tr.train_step(*_inputs(cuda, 340 + 3 * i)) for i in range(4)]
        grads = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
        res.append((losses, grads, {k: v.detach().clone() for k, v in m.state_dict().items()}))
    (l0, g0, s0), (l1, g1, s1) = res
    assert l0 == l1
    assert g0.keys() == g1.keys() and any(k.endswith("bias") for k in g0)
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k


def test_finalize_many_equals_immediate(cuda):
    """ldm_act_backward_defer + ldm_act_finalize_many == ldm_act_backward for dbias, over the kernel classes
    (planes of 64..1024 positions, sliced planes), relu and none, with more jobs than one launch takes (24)."""
    from ldm_amd import ops
    g = torch.Generator().manual_seed(5)
    cases = [(32, 64, 16, 64), (32, 128, 8, 32), (32, 256, 4, 16), (4, 64, 64, 256), (8, 32, 32, 128)] * 6
    imm, dfr = [], []
    with torch.no_grad():
        for i, (B, C, H, W) in enumerate(cases):
            dy = torch.randn(B, C, H, W, generator=g).to(cuda)
            a = torch.randn(B, C, H, W, generator=g).clamp_min(0).to(cuda)
            act = "relu" if i % 2 else "none"
            _, db, _ = ops.act_backward(dy, act, act_out=a, need_dv=True, need_bias=True)
            imm.append(db.clone())
        with ops.bias_grads_deferred():
            g = torch.Generator().manual_seed(5)
            for i, (B, C, H, W) in enumerate(cases):
                dy = torch.randn(B, C, H, W, generator=g).to(cuda)
                a = torch.randn(B, C, H, W, generator=g).clamp_min(0).to(cuda)
                act = "relu" if i % 2 else "none"
                _, db, _ = ops.act_backward(dy, act, act_out=a, need_dv=True, need_bias=True)
                dfr.append(db)
    torch.cuda.synchronize()
    for i, (x, y) in enumerate(zip(imm, dfr)):
        assert torch.equal(x, y), (i, cases[i])


@pytest.mark.parametrize("dtype", [0, 2])
def test_wgrad_reduce_many_equals_immediate(cuda, dtype):
    """ldm_conv_backward_weight_defer + ldm_wgrad_reduce_many (inside bias_grads_deferred) == ldm_conv_backward_weight_dt
    bitwise, over conv / convT weight gradients that split K (the train step's classes), more jobs than one launch."""
    from ldm_amd import ops
    descs = [ops.make_desc(8, 64, 64, 256, 128, 3, 3, 2, 1), ops.make_desc(8, 128, 32, 128, 256, 3, 3, 2, 1),
             ops.make_desc(8, 128, 16, 64, 64, 3, 3, 2, 1, 1, True), ops.make_desc(8, 256, 8, 32, 256, 3, 3, 1, 1),
             ops.make_desc(8, 64, 16, 64, 32, 3, 3, 1, 1)] * 6
    g = torch.Generator().manual_seed(9)
    data = []
    for d in descs:
        x = torch.randn(d.B, d.Cin, d.Hin, d.Win, generator=g).to(cuda)
        dy = torch.randn(d.B, d.Cout, d.Hout, d.Wout, generator=g).to(cuda)
        data.append((x, dy))
    with torch.no_grad():
        imm = [ops.conv_backward_weight(x, dy, d, dtype=dtype).clone() for d, (x, dy) in zip(descs, data)]
        with ops.bias_grads_deferred():
            dfr = [ops.conv_backward_weight(x, dy, d, dtype=dtype) for d, (x, dy) in zip(descs, data)]
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(imm, dfr)):
        assert torch.equal(a, b), i
