"""Data parallelism for the LDM path: one process per GPU, torch.distributed over RCCL ('nccl' backend
on ROCm, xGMI between the GPUs of a node); 'gloo' works for the same code on CPU tensors (tests).

SURVEY.md §8(e):
  * Sampling shards by sample: every rank runs the whole reverse loop on its slice of the batch, no
    collective inside the loop; the decoded results are all-gathered once at the end
    (``shard_batch`` / ``gather_batch`` / ``sharded_style_sample``).
  * Training is data-parallel: each rank computes gradients on its batch shard, and the gradients of
    the trainable parameters (UNet + StyleEncoder + Decoder, 9.77 M fp32 = 39 MB) are summed across
    ranks before the optimiser step (``GradAllReduce``).  Buckets of ~``bucket_mb`` are launched as
    asynchronous all-reduces from post-accumulate-grad hooks, i.e. while the backward pass is still
    producing the gradients of earlier layers (overlap), and the 1/world averaging is folded into
    the GradScaler's unscale kernel (no extra pass over the gradients).
"""
import contextlib

import torch
import torch.distributed as tdist


def is_distributed():
    return tdist.is_available() and tdist.is_initialized()


def world_size():
    return tdist.get_world_size() if is_distributed() else 1


def rank():
    return tdist.get_rank() if is_distributed() else 0


# ------------------------------------------------------------------------------------------------
# sampling: batch sharding
# ------------------------------------------------------------------------------------------------
def shard_bounds(n, r=None, w=None):
    """[lo, hi) of rank r's contiguous share of n items (the first n % w ranks get one more)."""
    r = rank() if r is None else r
    w = world_size() if w is None else w
    base, extra = divmod(n, w)
    lo = r * base + min(r, extra)
    return lo, lo + base + (1 if r < extra else 0)


def shard_batch(x, r=None, w=None):
    lo, hi = shard_bounds(x.shape[0], r, w)
    return x[lo:hi]


def gather_batch(x, n_total):
    """All-gather the per-rank batch shards back into the full [n_total, ...] batch (rank order)."""
    w = world_size()
    if w == 1:
        return x
    sizes = [shard_bounds(n_total, r, w) for r in range(w)]
    cap = max(hi - lo for lo, hi in sizes)
    pad = torch.zeros((cap,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    pad[: x.shape[0]].copy_(x)
    if tdist.get_backend() == "gloo":        # CPU tests: gloo has no all_gather_into_tensor
        chunks = [torch.empty_like(pad) for _ in range(w)]
        tdist.all_gather(chunks, pad)
        out = torch.cat(chunks, 0)
    else:
        out = torch.empty((w * cap,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        tdist.all_gather_into_tensor(out, pad)
    parts = [out[r * cap: r * cap + (hi - lo)] for r, (lo, hi) in enumerate(sizes)]
    return torch.cat(parts, 0)


def sharded_style_sample(model, z_T, style_spec, timesteps=100, eta=0.0):
    """style_ddim_sample_wrapper over a batch split across ranks: z_T [B,...] is the FULL starting
    noise (identical on every rank, e.g. from a seeded CPU generator as model.py:394 does), each rank
    samples and decodes its shard, the decoded spectrograms are all-gathered.

    The style encoder, UNet and sampler are per-sample, so each shard's latents equal the single-GPU
    ones.  The decoder's BatchNorm layers couple the batch when the decoder is in train mode (the
    reference samples that way, model.py:344-347 / tests.py:803-810): they are synchronised over the
    group here, so the decoded batch equals the single-GPU result up to fp32 summation order.  A rank
    whose shard is empty (B < world size) still joins those collectives."""
    B = z_T.shape[0]
    z = shard_batch(z_T).to(style_spec.device)
    s = shard_batch(style_spec)
    with torch.no_grad():
        if z.shape[0]:
            emb = model.style_encoder(s)
            x, _ = model.style_conditioned_ddim_sample(z, emb, timesteps, eta)
        else:
            x = z.float()
        with batchnorm_sync(True):
            dec = model.decoder(x, rescale=True)
    return gather_batch(dec.contiguous(), B)


# ------------------------------------------------------------------------------------------------
# training: bucketed gradient all-reduce overlapped with backward
# ------------------------------------------------------------------------------------------------
class _Bucket:
    def __init__(self, params, device):
        self.params = params
        self.numel = sum(p.numel() for p in params)
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.offsets = {}
        off = 0
        for p in params:
            self.offsets[id(p)] = off
            off += p.numel()
        self.ready = set()
        self.work = None
        self.streams = {}    # the streams that copied gradients in (the train step's branch streams)


class GradAllReduce:
    """Sum gradients of `params` over the process group, bucket by bucket, as backward produces them.

    Usage per step:   loss.backward(); reducer.finish(); optimizer.step()
    After finish() every p.grad is a view into a flat bucket holding the SUM over ranks; divide by
    world_size() before applying it (GradScaler.set_grad_divisor folds that into its unscale kernel,
    or pass average=True to scale here with the HIP kernel)."""

    def __init__(self, params, bucket_mb=25.0, group=None, average=False, collective=None):
        self.group = group
        self.average = average
        # collective(flat, group) -> work with .wait(): the bucket all-reduce (default: an async RCCL / gloo
        # all_reduce(SUM)); tests inject a stub
        self._collective = collective
        params = [p for p in params if p.requires_grad]
        if not params:
            raise ValueError("GradAllReduce: no parameters require grad")
        dev = params[0].device
        # backward visits parameters roughly in reverse registration order: fill buckets that way so
        # the first bucket completes first
        cap = int(bucket_mb * (1 << 20) / 4)
        self.buckets, cur, cur_n = [], [], 0
        for p in reversed(params):
            if cur and cur_n + p.numel() > cap:
                self.buckets.append(_Bucket(cur, dev))
                cur, cur_n = [], 0
            cur.append(p)
            cur_n += p.numel()
        if cur:
            self.buckets.append(_Bucket(cur, dev))
        self._owner = {}
        for b in self.buckets:
            for p in b.params:
                self._owner[id(p)] = b
        self._handles = [p.register_post_accumulate_grad_hook(self._on_grad) for p in params]

    def remove(self):
        for h in self._handles:
            h.remove()
        self._handles = []

    @property
    def capturable(self):
        """True when the whole step, these hooks and collectives included, can be captured into a hipGraph:
        every piece is then a device operation on fixed buffers (the bucket copies, the RCCL all-reduces on
        the process group's stream joined back by events, the views into the flat buckets) and nothing reads
        the device from the host.  RCCL ('nccl') collectives are capturable; gloo's (host staging) are not.
        A stub collective declares it with a `capturable` attribute."""
        if self._collective is not None:
            return bool(getattr(self._collective, "capturable", False))
        return is_distributed() and tdist.get_backend(self.group) == "nccl"

    def _launch(self, b):
        # gradients of a branch (e.g. the style encoder's, graphs.branch) were copied in on that branch's
        # stream: the launching stream waits for every stream that wrote into the bucket
        if b.flat.is_cuda:
            cur = torch.cuda.current_stream(b.flat.device)
            for st in b.streams.values():
                if st.cuda_stream != cur.cuda_stream:
                    cur.wait_stream(st)
        b.streams.clear()
        if self._collective is not None:
            b.work = self._collective(b.flat, self.group)
            return
        b.work = tdist.all_reduce(b.flat, op=tdist.ReduceOp.SUM, group=self.group, async_op=True)

    def _on_grad(self, p):
        b = self._owner[id(p)]
        if b.work is not None or id(p) in b.ready:
            return
        off = b.offsets[id(p)]
        b.flat[off: off + p.numel()].copy_(p.grad.reshape(-1))
        if b.flat.is_cuda:
            st = torch.cuda.current_stream(b.flat.device)
            b.streams[st.cuda_stream] = st
        b.ready.add(id(p))
        if len(b.ready) == len(b.params):
            self._launch(b)

    def finish(self):
        """Launch the buckets still open (params that got no gradient contribute zeros), wait for all
        reductions, and point every p.grad at its reduced slice."""
        for b in self.buckets:
            if b.work is None:
                for p in b.params:
                    if id(p) not in b.ready:
                        off = b.offsets[id(p)]
                        seg = b.flat[off: off + p.numel()]
                        if p.grad is None:
                            seg.zero_()
                        else:
                            seg.copy_(p.grad.reshape(-1))
                self._launch(b)
        for b in self.buckets:
            b.work.wait()
            b.work = None
            b.ready.clear()
            for p in b.params:
                off = b.offsets[id(p)]
                p.grad = b.flat[off: off + p.numel()].view_as(p)
        if self.average and world_size() > 1:
            from .optim import scale_tensors_
            scale_tensors_([b.flat for b in self.buckets], 1.0 / world_size())


def broadcast_parameters(module, src=0, group=None):
    """Make every rank start from rank `src`'s parameters and buffers."""
    if world_size() == 1:
        return
    for t in list(module.parameters()) + list(module.buffers()):
        tdist.broadcast(t.data, src=src, group=group)


def convert_sync_batchnorm(module, group=True):
    """SyncBatchNorm for the data-parallel train path (torch.nn.SyncBatchNorm.convert_sync_batchnorm
    semantics, in place): every BatchNorm2d of `module` that runs in training mode normalises with the
    batch statistics of the whole process group (fp64 (sum x, sum x^2, count) and the backward sums
    all-reduced between the two stages of reduce.hip, one collective each), so N ranks x B samples train
    like one process on N*B.  group=True means the default group; group=False turns it off again.  No
    effect in eval mode or single-process runs.  For rank-local use of a converted model (e.g. sampling
    on rank 0 only) wrap the calls in ``batchnorm_sync(False)``: every rank must otherwise make the same
    train-mode BatchNorm calls, in the same order, or the collectives wait for each other."""
    for m in module.modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            m.ldm_sync_group = group
    return module


@contextlib.contextmanager
def batchnorm_sync(group=True):
    """Within the block, every train-mode BatchNorm uses `group` (True = default group, a ProcessGroup,
    or False = local statistics), whatever convert_sync_batchnorm set on the module."""
    from . import functional as HF
    HF._SYNC_OVERRIDE.append(group)
    try:
        yield
    finally:
        HF._SYNC_OVERRIDE.pop()
