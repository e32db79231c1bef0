"""SyncBatchNorm and the data-parallel trainer on the HIP path.

1. Two-stage BN kernels in one process: a batch split into two "ranks", per-half fp64 stats (plus the
   per-half count) summed on the device exactly as the RCCL all-reduce sums them, then the apply stage
   reading the global count on the device.  Outputs, running statistics and the backward (dx, dw, db)
   must equal single-call BN on the whole batch and float64 torch autograd.
2. LDMTrainer at world size 2: two processes on the one GPU over gloo (CUDA tensors), each training on
   half of a batch with SyncBatchNorm + the bucketed gradient all-reduce + GradScaler's 1/world divisor,
   against one process training on the whole batch, both with the autocast region off (fp32 operands).
   Gradients, BN running statistics and the Adam update must agree to fp32 rounding (1e-4 relative; the
   update 1e-5).

Reference: nn.BatchNorm2d train mode in model.py:10-49 (encoder/decoder), LDMTrainer train.py:163-208.
"""
import os
import socket

import numpy as np
import pytest
import torch

import recipe
from conftest import adam_step_err, rel_err

pytestmark = pytest.mark.gpu
TOL = 1e-4
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def npy(t):
    return t.detach().double().cpu().numpy()


def _rand(shape, seed, lo=-1.0, hi=1.0):
    g = np.random.Generator(np.random.PCG64(seed))
    return g.uniform(lo, hi, shape).astype(np.float32)


@pytest.mark.parametrize("shape", [(4, 64, 8, 8), (4, 8, 36, 36), (6, 4, 30, 31), (2, 16, 3, 5)])
@pytest.mark.parametrize("act", ["none", "relu"])
@pytest.mark.parametrize("pass_y", [True, False])
def test_two_stage_bn_equals_single_call(cuda, shape, act, pass_y):
    """pass_y False: the backward re-evaluates the ReLU mask from x, weight and bias (no output read)."""
    from ldm_amd import _lib as L, ops
    B, C, H, W = shape
    HW = H * W
    x = torch.from_numpy(_rand(shape, 5, -2, 2))
    g = torch.from_numpy(_rand((C,), 6, 0.5, 1.5))
    b = torch.from_numpy(_rand((C,), 7, -0.1, 0.1))
    rm0 = torch.from_numpy(_rand((C,), 8, -0.2, 0.2))
    rv0 = torch.from_numpy(_rand((C,), 9, 0.5, 1.5))
    dy = torch.from_numpy(_rand(shape, 10))
    st = ops.stream_handle()
    A = L.ACT[act]
    # --- single call over the whole batch
    x1 = x.clone().to(cuda)
    rm1, rv1 = rm0.clone().to(cuda), rv0.clone().to(cuda)
    gd, bd = g.to(cuda), b.to(cuda)
    sm1, si1 = torch.empty(C, device=cuda), torch.empty(C, device=cuda)
    ws = ops.reduce_workspace(B, C, HW, cuda)
    L.call("ldm_batchnorm_train", x1.data_ptr(), B, C, HW, gd.data_ptr(), bd.data_ptr(), rm1.data_ptr(), rv1.data_ptr(),
           0.1, 1e-5, A, sm1.data_ptr(), si1.data_ptr(), ws.data_ptr(), st)
    # out-of-place form: the same bits, input untouched
    xo, yo = x.clone().to(cuda), torch.empty((B, C, H, W), device=cuda)
    rmo, rvo = rm0.clone().to(cuda), rv0.clone().to(cuda)
    L.call("ldm_batchnorm_train_out", xo.data_ptr(), yo.data_ptr(), B, C, HW, gd.data_ptr(), bd.data_ptr(),
           rmo.data_ptr(), rvo.data_ptr(), 0.1, 1e-5, A, None, None, ops.reduce_workspace(B, C, HW, cuda).data_ptr(), st)
    torch.cuda.synchronize()
    assert torch.equal(yo, x1) and torch.equal(xo.cpu(), x) and torch.equal(rmo, rm1) and torch.equal(rvo, rv1)
    # --- two halves: stats per half, summed (what the all-reduce does), apply with the device count
    h = B // 2
    halves = [x[:h].clone().to(cuda), x[h:].clone().to(cuda)]
    stats = []
    for xh in halves:
        s = torch.empty(2 * C + 1, device=cuda, dtype=torch.float64)
        wsh = ops.reduce_workspace(xh.shape[0], C, HW, cuda).clone()
        L.call("ldm_batchnorm_stats", xh.data_ptr(), xh.shape[0], C, HW, s.data_ptr(), wsh.data_ptr(), st)
        stats.append(s)
    tot = stats[0] + stats[1]
    assert float(tot[2 * C]) == B * HW
    outs, rms = [], []
    for xh in halves:
        rm, rv = rm0.clone().to(cuda), rv0.clone().to(cuda)
        sm, si = torch.empty(C, device=cuda), torch.empty(C, device=cuda)
        L.call("ldm_batchnorm_apply", xh.data_ptr(), xh.shape[0], C, HW, tot.data_ptr(), -1.0, gd.data_ptr(),
               bd.data_ptr(), rm.data_ptr(), rv.data_ptr(), 0.1, 1e-5, A, sm.data_ptr(), si.data_ptr(), st)
        outs.append(xh)
        rms.append((rm, rv, sm, si))
    y2 = torch.cat(outs, 0)
    # float64 torch reference
    xt = x.double().requires_grad_()
    bn = torch.nn.BatchNorm2d(C).double()
    with torch.no_grad():
        bn.weight.copy_(g.double())
        bn.bias.copy_(b.double())
        bn.running_mean.copy_(rm0.double())
        bn.running_var.copy_(rv0.double())
    ref = bn(xt)
    if act == "relu":
        ref = torch.relu(ref)
    assert rel_err(npy(x1), ref.detach().numpy()) < TOL
    assert rel_err(npy(y2), npy(x1)) < 1e-5
    for rm, rv, sm, si in rms:
        assert rel_err(npy(rm), bn.running_mean.numpy()) < TOL
        assert rel_err(npy(rv), bn.running_var.numpy()) < TOL
        assert rel_err(npy(sm), npy(sm1)) < 1e-5 and rel_err(npy(si), npy(si1)) < 1e-5
    # --- backward: single call vs per-half reduce -> sum -> apply
    (ref * dy.double()).sum().backward()
    dyd = dy.to(cuda)
    xin = x.to(cuda)
    dx1, dw1, db1 = torch.empty_like(xin), torch.empty(C, device=cuda), torch.empty(C, device=cuda)
    L.call("ldm_batchnorm_backward", dyd.data_ptr(), x1.data_ptr() if pass_y else None, xin.data_ptr(), sm1.data_ptr(),
           si1.data_ptr(), gd.data_ptr(), bd.data_ptr(), A, B, C, HW, dx1.data_ptr(), dw1.data_ptr(), db1.data_ptr(),
           ws.data_ptr(), st)
    sums, parts = [], []
    for i, sl in enumerate((slice(0, h), slice(h, B))):
        s = torch.empty(2 * C + 1, device=cuda, dtype=torch.float64)
        dwh, dbh = torch.empty(C, device=cuda), torch.empty(C, device=cuda)
        n = sl.stop - sl.start
        wsh = ops.reduce_workspace(n, C, HW, cuda).clone()
        L.call("ldm_batchnorm_backward_reduce", dyd[sl].contiguous().data_ptr(),
               outs[i].data_ptr() if pass_y else None, xin[sl].contiguous().data_ptr(), rms[i][2].data_ptr(),
               rms[i][3].data_ptr(), gd.data_ptr(), bd.data_ptr(), A, n, C, HW, s.data_ptr(), dwh.data_ptr(),
               dbh.data_ptr(), wsh.data_ptr(), st)
        torch.cuda.synchronize()
        sums.append(s)
        parts.append((dwh, dbh))
    tot_b = sums[0] + sums[1]
    assert float(tot_b[2 * C]) == B * HW
    dxs = []
    for i, sl in enumerate((slice(0, h), slice(h, B))):
        n = sl.stop - sl.start
        dxh = torch.empty((n, C, H, W), device=cuda)
        L.call("ldm_batchnorm_backward_apply", dyd[sl].contiguous().data_ptr(),
               outs[i].data_ptr() if pass_y else None, xin[sl].contiguous().data_ptr(), rms[i][2].data_ptr(),
               rms[i][3].data_ptr(), gd.data_ptr(), bd.data_ptr(), A, n, C, HW, tot_b.data_ptr(), -1.0,
               dxh.data_ptr(), st)
        dxs.append(dxh)
    torch.cuda.synchronize()
    dx2 = torch.cat(dxs, 0)
    assert rel_err(npy(dx1), xt.grad.numpy()) < TOL
    assert rel_err(npy(dx2), xt.grad.numpy()) < TOL
    assert rel_err(npy(parts[0][0] + parts[1][0]), bn.weight.grad.numpy()) < TOL      # local dw summed = DP sum
    assert rel_err(npy(parts[0][1] + parts[1][1]), bn.bias.grad.numpy()) < TOL
    assert rel_err(npy(dw1), bn.weight.grad.numpy()) < TOL and rel_err(npy(db1), bn.bias.grad.numpy()) < TOL


def test_empty_shard_joins_with_zero_sums(cuda):
    """B = 0 on this rank: stats are zero, the count is 0, and apply still updates the running stats from
    the (here: injected) global sums."""
    from ldm_amd import _lib as L, ops
    C, HW = 8, 16
    st = ops.stream_handle()
    s = torch.full((2 * C + 1,), 7.0, device=cuda, dtype=torch.float64)
    ws = ops.reduce_workspace(0, C, HW, cuda)
    L.call("ldm_batchnorm_stats", None, 0, C, HW, s.data_ptr(), ws.data_ptr(), st)
    torch.cuda.synchronize()
    assert torch.count_nonzero(s).item() == 0
    glob = torch.zeros(2 * C + 1, device=cuda, dtype=torch.float64)
    glob[0:2 * C:2] = 32.0          # sum x over 16 elements of mean 2
    glob[1:2 * C:2] = 16 * 5.0      # sum x^2 -> var 1
    glob[2 * C] = 16
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    L.call("ldm_batchnorm_apply", None, 0, C, HW, glob.data_ptr(), -1.0, None, None, rm.data_ptr(), rv.data_ptr(),
           0.1, 1e-5, 0, None, None, st)
    torch.cuda.synchronize()
    assert torch.allclose(rm, torch.full_like(rm, 0.2))
    assert torch.allclose(rv, torch.full_like(rv, 0.9 + 0.1 * 16.0 / 15.0))


# ---- LDMTrainer at world size 2 (gloo over CUDA tensors, both ranks on the one GPU) -------------------------
KEYS = ("unet.dec1.weight", "unet.enc1.weight", "unet.bottleneck.bias",
        "unet.cross_attention1.multihead_attn.in_proj_weight", "decoder.decoder.0.weight",
        "decoder.decoder.1.weight", "decoder.decoder.4.bias", "decoder.decoder.6.weight",
        "style_encoder.enc1.weight", "style_encoder.enc6.bias")
BUFS = ("decoder.decoder.1.running_mean", "decoder.decoder.4.running_var", "encoder.encoder.4.running_var")


class _ZeroFeat(torch.nn.Module):
    def forward(self, a, b):
        return torch.zeros((), device=a.device)


def _train_once(rank, world, cuda):
    import models.model as M
    import models.train as TR
    from ldm_amd import dist as D
    Bt = 4
    content = torch.from_numpy(recipe.uniform01((Bt, 1, 128, 128), 810))
    style = torch.from_numpy(recipe.uniform01((Bt, 1, 128, 128), 811))
    noise = torch.from_numpy(recipe.normal((Bt, 32, 16, 16), 812))
    t = torch.tensor([5, 60, 120, 190])
    lo, hi = D.shard_bounds(Bt, rank, world)
    ldm = M.LDM(32, pretrained_path="")
    recipe.fill_module(ldm, seed=700)
    ldm.feature_loss_net = _ZeroFeat()
    ldm = ldm.to(cuda)
    for p in ldm.encoder.parameters():
        p.requires_grad_(False)
    ldm.train()
    tr = TR.LDMTrainer(ldm, [], cuda, lr=5e-4)
    # fp32 step: under the default fp16 autocast region the two shardings round slightly different fp32
    # intermediates to fp16 operands, which alone moves a gradient by ~2e-4 (measured) — not a DP defect
    tr.autocast_enabled = False
    losses = tr.train_step(content[lo:hi].to(cuda), style[lo:hi].to(cuda), t=t[lo:hi].to(cuda),
                           noise=noise[lo:hi].to(cuda))
    named = dict(ldm.named_parameters())
    out = {"grad/" + k: npy(named[k].grad) for k in KEYS}
    out.update({"param/" + k: npy(named[k]) for k in KEYS})
    sd = ldm.state_dict()
    out.update({"buf/" + k: npy(sd[k]) for k in BUFS})
    out["loss"] = np.array([losses["total_loss"]])
    return out


def _worker(rank, world, port, q):
    import sys
    for p in (ROOT, os.path.join(ROOT, "music-style-transfer-ldm_amd"), os.path.join(ROOT, "tests", "golden"),
              os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as tdist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        tdist.init_process_group("gloo", rank=rank, world_size=world)
        out = _train_once(rank, world, torch.device("cuda:0"))
        tdist.barrier()
        tdist.destroy_process_group()
        q.put((rank, out, None))
    except Exception as e:   # report instead of hanging the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))
        raise


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_trainer_world2_syncbn_equals_world1(cuda):
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            r, out, err = q.get(timeout=240)
            assert err is None, f"rank {r} failed:\n{err}"
            res[r] = out
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    ref = _train_once(0, 1, cuda)
    for k in KEYS:
        for r in range(world):
            assert rel_err(res[r]["grad/" + k], ref["grad/" + k]) < TOL, (r, k)
            assert adam_step_err(res[r]["param/" + k], ref["param/" + k], ref["grad/" + k], 5e-4,
                                 grad=res[r]["grad/" + k]) < 1e-5, (r, k)
    for k in BUFS:
        for r in range(world):
            assert rel_err(res[r]["buf/" + k], ref["buf/" + k]) < TOL, (r, k)
    # each rank reports its local loss; their mean is the whole-batch loss
    assert abs(0.5 * (res[0]["loss"][0] + res[1]["loss"][0]) - ref["loss"][0]) <= 1e-4 * abs(ref["loss"][0])
