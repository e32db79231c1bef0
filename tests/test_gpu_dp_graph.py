"""The data-parallel train step captured into a hipGraph (reference train.py:163-208).

One GPU box holds one GPU, so:
  * the RCCL path runs in a world-1 'nccl' (= RCCL) process group rendezvoused exactly as bench.py does
    (env://, a TCPStore on 127.0.0.1, TORCH_NCCL_ASYNC_ERROR_HANDLING and the heartbeat monitor left at
    their defaults), in this process: the trainer gets the bucketed GradAllReduce it builds for world > 1
    (post-accumulate-grad hooks, per-bucket copies, asynchronous RCCL all-reduces and their joins),
    graph_step captures all of it, and the replays must equal an eager trainer without a reducer BITWISE
    (a one-rank sum is the identity);
  * the watchdog race behind round 3's intermittent abort (ldm_amd/graphs.py) is exercised on
    purpose: an eager collective immediately followed by a capture that spans several watchdog passes;
  * what only fires for world > 1 — SyncBatchNorm's in-graph statistic all-reduces and N > 1 bucket sums —
    runs against a capturable stub group that simulates a second rank holding the same shard (sum = 2x),
    graphed against eager, bitwise.
What stays unmeasured on hardware: more than one RCCL rank, and the scaling curve.
"""
import os
import socket
import time

import pytest
import torch

import recipe

pytestmark = pytest.mark.gpu


class _ZeroFeat(torch.nn.Module):
    def forward(self, a, b):
        return torch.zeros((), device=a.device)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def nccl_world1(cuda):
    import torch.distributed as tdist
    assert not tdist.is_initialized()
    env = {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_free_port()), "RANK": "0", "WORLD_SIZE": "1",
           "LOCAL_RANK": "0"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    tdist.init_process_group("nccl", device_id=cuda)          # env:// -> TCPStore, as bench.py:main
    try:
        yield tdist
    finally:
        torch.cuda.synchronize()
        tdist.destroy_process_group()
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _inputs(cuda):
    content = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 930)).to(cuda)
    style = torch.from_numpy(recipe.uniform01((2, 1, 128, 128), 931)).to(cuda)
    t = torch.tensor([33, 144], device=cuda)
    noise = torch.from_numpy(recipe.normal((2, 32, 16, 16), 932)).to(cuda)
    return content, style, t, noise


def _trainer(cuda, seed=700):
    import models.model as M
    import models.train as TR
    m = M.LDM(32, pretrained_path="")
    recipe.fill_module(m, seed=seed)
    m.feature_loss_net = _ZeroFeat()
    m = m.to(cuda).train()
    tr = TR.LDMTrainer(m, [], cuda, lr=1e-3)
    tr.autocast_enabled = False
    return m, tr


def _run(tr, m, args, n1=5, n2=3):
    losses = [tr.train_step(*args) for _ in range(n1)]
    tr.optimizer.param_groups[0]["lr"] *= 0.5                 # a re-capture mid-run
    losses += [tr.train_step(*args) for _ in range(n2)]
    return losses, {k: v.detach().clone() for k, v in m.state_dict().items()}


def _assert_bitwise(res_e, res_g):
    (le, sde), (lg, sdg) = res_e, res_g
    for a, b in zip(le, lg):
        for k in a:
            assert a[k] == b[k], (k, a[k], b[k])
    for k in sde:
        assert torch.equal(sde[k], sdg[k]), k


def test_capture_right_after_eager_collective(cuda, nccl_world1):
    """An eager all-reduce (left on the watchdog's work list until its next pass) immediately followed by a
    0.4 s capture through ldm_amd.graphs.capture, a captured all-reduce, then replays: three times.  In the
    global capture mode the watchdog's event query inside the window is refused and the process aborts."""
    from ldm_amd import graphs as hgraphs
    tdist = nccl_world1
    x = torch.ones(1 << 16, device=cuda)
    y = torch.zeros_like(x)
    for _ in range(3):
        tdist.all_reduce(x, async_op=True).wait()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        t0 = time.time()
        with hgraphs.capture(g):
            while time.time() - t0 < 0.4:
                y.add_(x)
                time.sleep(0.01)
            tdist.all_reduce(y, async_op=True).wait()
        y.zero_()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        assert torch.isfinite(y).all() and float(y[0]) > 0
        time.sleep(0.15)


def test_graphed_step_with_rccl_reducer_equals_eager(cuda, nccl_world1):
    from ldm_amd import dist as hdist
    args = _inputs(cuda)
    m, tr = _trainer(cuda)
    res_e = _run(tr, m, args)
    assert tr._graph is None
    m, tr = _trainer(cuda)
    tr.reducer = hdist.GradAllReduce([p for p in m.parameters() if p.requires_grad], bucket_mb=8.0)
    assert tr.reducer.capturable and len(tr.reducer.buckets) > 1
    tr.graph_step = True
    res_g = _run(tr, m, args)
    assert tr._graph is not None
    torch.cuda.synchronize()
    tr.reducer.remove()
    _assert_bitwise(res_e, res_g)


class _Work:
    def wait(self):
        pass


class _StubWorld2:
    """A capturable stand-in for a 2-rank group whose other rank holds the same shard: sum = 2x, in place,
    on the current stream (so it is recorded into the graph like RCCL's kernels)."""
    capturable = True

    def __init__(self):
        self.calls = 0

    def ldm_allreduce_sum(self, t):                             # SyncBatchNorm statistics / backward sums
        self.calls += 1
        t.mul_(2.0)

    def __call__(self, flat, group):                           # GradAllReduce bucket collective
        self.calls += 1
        flat.mul_(2.0)
        return _Work()


def _stub_dp_trainer(cuda, graph):
    from ldm_amd import dist as hdist
    m, tr = _trainer(cuda)
    stub = _StubWorld2()
    hdist.convert_sync_batchnorm(m, group=stub)
    tr.reducer = hdist.GradAllReduce([p for p in m.parameters() if p.requires_grad], bucket_mb=8.0,
                                     collective=stub)
    tr.scaler.set_grad_divisor(2)
    tr.graph_step = graph
    return m, tr, stub


def test_graphed_world2_stub_syncbn_equals_eager(cuda):
    """SyncBatchNorm's statistic all-reduces and the N > 1 bucket sums inside the captured step (stub world
    of 2), graphed == eager bitwise; and the stubbed world-2 step stays close to the plain one-rank step
    (same batch statistics, gradients summed then halved; only running-variance unbias factors and
    summation order differ)."""
    args = _inputs(cuda)
    m, tr, stub_e = _stub_dp_trainer(cuda, graph=False)
    res_e = _run(tr, m, args)
    assert stub_e.calls > 0
    m, tr, stub_g = _stub_dp_trainer(cuda, graph=True)
    res_g = _run(tr, m, args)
    assert tr._graph is not None
    _assert_bitwise(res_e, res_g)
    # the SyncBN collectives were recorded: the eager run issues them every step, the graphed one only in its
    # eager warm-ups and its two captures
    assert 0 < stub_g.calls < stub_e.calls
    m, tr = _trainer(cuda)
    res_1 = _run(tr, m, args, n1=1, n2=0)
    m, tr, _ = _stub_dp_trainer(cuda, graph=False)
    res_2 = _run(tr, m, args, n1=1, n2=0)
    for k in res_1[0][0]:
        assert abs(res_1[0][0][k] - res_2[0][0][k]) <= 1e-5 * max(1.0, abs(res_1[0][0][k])), k
