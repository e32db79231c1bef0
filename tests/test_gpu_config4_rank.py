"""Config 4's per-rank workload at its size: the B = 32 bf16 graphed train step (config 3's shape) with the
trainer built as LDMTrainer builds it for world > 1 (reference train.py:163-208 split over ranks; SURVEY
§8(e)): the bucketed GradAllReduce from post-accumulate-grad hooks, SyncBatchNorm on every BatchNorm, and the
1/world divisor folded into the GradScaler's unscale.  One GPU per box, so two forms:

  * world-1 RCCL: a 'nccl' process group rendezvoused over env:// as bench.py does; the reducer's bucket
    all-reduces and SyncBN's statistic / backward-sum all-reduces are real RCCL collectives, captured into the
    step's hipGraph (a one-rank sum is the identity);
  * a capturable world-2 stub: the collectives sum as if a second rank held the same shard (x 2), with
    set_grad_divisor(2), so the averaged gradients and the global batch statistics equal the one-rank ones.

Each is checked against the reference's config-3 step (ref_goldens_r3.npz) at test_gpu_train_config3.py's
bf16 bounds: 1.5 e + 1e-4 of the reference's bf16 step and 2 e + 1e-4 of its fp32 step per quantity, and the
Adam update against float64.  N > 1 over RCCL stays unmeasured here (the driver's 8-GPU node runs it)."""
import os
import socket

import pytest
import torch

import test_gpu_train_config3 as C3

pytestmark = pytest.mark.gpu


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
    tdist.init_process_group("nccl", device_id=cuda)
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


class _Work:
    def wait(self):
        pass


class _StubWorld2:
    """A capturable 2-rank group whose other rank holds the same shard: every sum is x 2, in place, on the
    current stream (recorded into the graph like RCCL's kernels)."""
    capturable = True

    def __init__(self):
        self.calls = 0

    def ldm_allreduce_sum(self, t):                      # SyncBatchNorm statistics / backward sums
        self.calls += 1
        t.mul_(2.0)

    def __call__(self, flat, group):                    # GradAllReduce bucket collective
        self.calls += 1
        flat.mul_(2.0)
        return _Work()


def test_config4_rank_step_rccl_world1(C3g3, cuda, nccl_world1):
    from ldm_amd import dist as hdist
    m, tr = C3._bench_trainer(cuda, "bf16")
    hdist.convert_sync_batchnorm(m)                      # the default group: RCCL
    tr.reducer = hdist.GradAllReduce(tr._trainable)      # 25 MB buckets, RCCL all-reduce per bucket
    assert tr.reducer.capturable and len(tr.reducer.buckets) >= 2
    tr.scaler.set_grad_divisor(hdist.world_size())
    C3.check_graphed_step(C3g3, cuda, "bf16", m, tr)
    tr.reducer.remove()


def test_config4_rank_step_stub_world2(C3g3, cuda):
    from ldm_amd import dist as hdist
    m, tr = C3._bench_trainer(cuda, "bf16")
    stub = _StubWorld2()
    hdist.convert_sync_batchnorm(m, group=stub)
    tr.reducer = hdist.GradAllReduce(tr._trainable, collective=stub)
    tr.scaler.set_grad_divisor(2)
    C3.check_graphed_step(C3g3, cuda, "bf16", m, tr)
    assert stub.calls > 0
    tr.reducer.remove()


@pytest.fixture(scope="module")
def C3g3():
    import numpy as np
    from conftest import ROOT
    return np.load(os.path.join(ROOT, "tests", "golden", "ref_goldens_r3.npz"))
