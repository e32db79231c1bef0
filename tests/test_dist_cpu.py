"""CPU, world_size 2 over gloo: the data-parallel pieces of ldm_amd.dist (batch sharding, all-gather of
samples, bucketed gradient all-reduce driven by post-accumulate-grad hooks).  The same code runs over
RCCL ('nccl') with one process per GPU; the HIP kernels are not involved in these host-side paths
(averaging is folded into the GPU-side GradScaler unscale, tested in tests/test_gpu_train.py)."""
import copy
import os
import socket

import pytest
import torch
import torch.distributed as tdist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)


def _worker_gather(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "music-style-transfer-ldm_amd"))
    from ldm_amd import dist as D
    _init(rank, world, port)
    try:
        n = 5
        full = torch.arange(n * 3, dtype=torch.float32).reshape(n, 3)
        mine = D.shard_batch(full)
        got = D.gather_batch(mine * 1.0, n)
        q.put((rank, bool(torch.equal(got, full)), tuple(mine.shape)))
    finally:
        tdist.destroy_process_group()


def _worker_grads(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "music-style-transfer-ldm_amd"))
    from ldm_amd import dist as D
    _init(rank, world, port)
    try:
        torch.manual_seed(0)                   # identical init on both ranks
        net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4),
                                  torch.nn.Linear(4, 4))
        unused = torch.nn.Parameter(torch.ones(3))          # gets no gradient: must reduce as zeros
        params = list(net.parameters()) + [unused]
        net_ref = copy.deepcopy(net)                          # un-hooked twin for the expected sums
        # tiny buckets so several all-reduces are in flight during backward
        red = D.GradAllReduce(params, bucket_mb=0.0005)
        torch.manual_seed(100)
        xs = torch.randn(world, 8, 16)
        ok = True
        for step in range(2):
            for p in params:
                p.grad = None
            net(xs[rank] * (step + 1)).pow(2).sum().backward()
            red.finish()
            # expected: sum over ranks of the per-rank gradients
            ref = [torch.zeros_like(p) for p in params]
            for r in range(world):
                net_ref.zero_grad(set_to_none=True)
                net_ref(xs[r] * (step + 1)).pow(2).sum().backward()
                for i, p in enumerate(net_ref.parameters()):
                    ref[i] += p.grad
            for i, p in enumerate(params):
                ok &= bool(torch.allclose(p.grad, ref[i], rtol=1e-5, atol=1e-5))
                b = red._owner[id(p)]
                ok &= p.grad.data_ptr() == b.flat[b.offsets[id(p)]:].data_ptr()   # a view of the bucket
        q.put((rank, ok, len(red.buckets)))
    finally:
        tdist.destroy_process_group()


def _worker_ldm_params(rank, world, port, q):
    """GradAllReduce over the real LDM trainable-parameter list (UNet + StyleEncoder + Decoder, 9.77 M
    params in ~25 MB buckets, encoder frozen as LDMTrainer sees it), then the 1/world divisor that
    GradScaler.set_grad_divisor folds into its unscale: the result must be the mean of the ranks' grads."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "music-style-transfer-ldm_amd"))
    import models.model as M
    from ldm_amd import dist as D
    _init(rank, world, port)
    try:
        torch.manual_seed(0)
        ldm = M.LDM(32, pretrained_path="")
        for p in ldm.encoder.parameters():
            p.requires_grad_(False)
        params = [p for p in ldm.parameters() if p.requires_grad]
        red = D.GradAllReduce(params)
        scale = 65536.0
        ok = True
        for step in range(2):
            for p in params:
                p.grad = None
            # per-rank gradient G_r(p) = scale * rand(seed(step, rank, i)), delivered through autograd so the
            # post-accumulate-grad hooks fire in backward order
            loss = 0.0
            for i, p in enumerate(params):
                g = torch.Generator().manual_seed(1000 * step + 100 * rank + i)
                loss = loss + (p * (torch.rand(p.shape, generator=g) * scale)).sum()
            loss.backward()
            red.finish()
            inv = 1.0 / (scale * world)          # GradScaler.unscale_ with set_grad_divisor(world)
            for i, p in enumerate(params):
                exp = sum(torch.rand(p.shape, generator=torch.Generator().manual_seed(1000 * step + 100 * r + i))
                          for r in range(world)) / world
                ok &= bool(torch.allclose(p.grad * inv, exp, rtol=1e-6, atol=1e-6))
        n = sum(p.numel() for p in params)
        q.put((rank, ok, (len(red.buckets), n)))
    finally:
        tdist.destroy_process_group()


class _StubCollective:
    """A capturable-declared stand-in for the RCCL all-reduce: records the bucket it is handed, reduces it with a
    synchronous gloo all_reduce, returns a finished work object."""
    capturable = True

    def __init__(self):
        self.calls = []

    def __call__(self, flat, group):
        self.calls.append((flat.data_ptr(), flat.numel()))
        tdist.all_reduce(flat, op=tdist.ReduceOp.SUM, group=group)

        class _Done:
            def wait(self):
                return True
        return _Done()


def _worker_stubbed_capture_path(rank, world, port, q):
    """The hook / bucket logic LDMTrainer's graphed data-parallel step captures (GradAllReduce with a collective
    declared capturable): one collective per bucket per step, on the bucket's persistent flat buffer (the same
    address every step, as a replayed graph needs), in completion order during backward, every p.grad a view of
    its bucket afterwards, sums right; the default gloo reducer reports itself not capturable."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "music-style-transfer-ldm_amd"))
    from ldm_amd import dist as D
    _init(rank, world, port)
    try:
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
        params = list(net.parameters())
        net_ref = copy.deepcopy(net)
        stub = _StubCollective()
        red = D.GradAllReduce(params, bucket_mb=0.001, collective=stub)
        ok = red.capturable and not D.GradAllReduce(params).capturable
        flats = [(b.flat.data_ptr(), b.flat.numel()) for b in red.buckets]
        torch.manual_seed(7)
        xs = torch.randn(world, 8, 16)
        for step in range(3):
            stub.calls.clear()
            for p in params:
                p.grad = None
            net(xs[rank] + step).pow(2).sum().backward()
            in_backward = list(stub.calls)            # launched by the hooks, before finish()
            red.finish()
            ok &= sorted(stub.calls) == sorted(flats) and len(stub.calls) == len(flats)
            ok &= len(in_backward) == len(flats)      # every bucket completed inside backward
            ref = [torch.zeros_like(p) for p in params]
            for r in range(world):
                net_ref.zero_grad(set_to_none=True)
                net_ref(xs[r] + step).pow(2).sum().backward()
                for i, p in enumerate(net_ref.parameters()):
                    ref[i] += p.grad
            for i, p in enumerate(params):
                ok &= bool(torch.allclose(p.grad, ref[i], rtol=1e-5, atol=1e-5))
                b = red._owner[id(p)]
                ok &= p.grad.data_ptr() == b.flat[b.offsets[id(p)]:].data_ptr()
        q.put((rank, ok, len(flats)))
    finally:
        tdist.destroy_process_group()


def _run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res)


def test_shard_bounds_partition():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "music-style-transfer-ldm_amd"))
    from ldm_amd import dist as D
    for n in (0, 1, 5, 8, 64, 257):
        for w in (1, 2, 3, 8):
            spans = [D.shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


def test_gather_batch_world2():
    res = _run(_worker_gather)
    assert [r[1] for r in res] == [True, True]
    assert [r[2] for r in res] == [(3, 3), (2, 3)]


def test_bucketed_grad_allreduce_world2():
    res = _run(_worker_grads)
    assert all(r[1] for r in res), res
    assert res[0][2] > 1   # several buckets


def test_grad_allreduce_ldm_parameter_list_world2():
    res = _run(_worker_ldm_params)
    assert all(r[1] for r in res), res
    nb, n = res[0][2]
    assert n == 6_841_504 + 2_729_984 + 198_209                                     # UNet + style + decoder
    assert nb >= 2                                                                     # 39 MB in ~25 MB buckets


def test_stubbed_capturable_reducer_world2():
    res = _run(_worker_stubbed_capture_path)
    assert all(r[1] for r in res), res
    assert res[0][2] > 1


if __name__ == "__main__":
    pytest.main([__file__, "-q"])
