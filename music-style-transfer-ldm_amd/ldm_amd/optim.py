"""Optimiser step of the train path on the HIP kernels.

``Adam`` / ``AdamW`` are torch.optim.Optimizer subclasses (same param_groups, state keys 'step',
'exp_avg', 'exp_avg_sq', state_dict format, so ReduceLROnPlateau and checkpoints work unchanged) whose
step() is ONE multi-tensor launch per param group (ldm_adam_step).  ``GradScaler`` mirrors
torch.amp.GradScaler's API and semantics (scale / unscale_ / step / update, backoff and growth) with
the unscale + inf check and the scale update as device kernels (ldm_unscale_check, ldm_update_scale).

Reference call sites: torch.optim.Adam + torch.amp.GradScaler in LDMTrainer (train.py:156-157,
:189-201); torch.optim.AdamW in train_autoencoder (train.py:44).
"""
import numpy as np
import torch

from . import _lib as L
from .ops import require_device, stream_handle

CHUNK = 1 << 12   # elements per workgroup-chunk of the multi-tensor kernels (4 float4 per thread)


class _SlotTable:
    """Device table of ldm_tensor_slot {param, grad, exp_avg, exp_avg_sq, numel} + chunk map.

    Tables are cached by the tensors' addresses (the same parameters, gradients and state give the same
    table every step).  The chunk map depends only on the sizes and is uploaded once per size list; the
    slot rows (whose gradient addresses move when zero_grad() drops the grads) go up with an asynchronous
    copy from pinned memory, so building a table never synchronises the host with the device.

    Inside a graph capture a table is neither allocated nor filled on the device.  Its rows go to a pinned
    host buffer and its device rows are a buffer reserved BEFORE the capture (reserve_capture_buffers), and
    fill_captured() uploads them after the capture has ended.  Why (round 6): a device buffer
    allocated while capturing comes from the graph's private pool and may be a block that a temporary of the
    SAME capture used and freed earlier (the forward / backward scratch).  Every replay then rewrites that
    block before the optimizer reads it, so a table written there once, outside the graph's own stream order,
    is garbage by the time unscale_check_kernel indexes slots[chunk_tensor[i]]: round 5's side-stream
    upload variant faulted on exactly that (HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION in unscale_check_kernel
    at the first replay).  A chunk map for a new size list would be a captured copy from a pageable numpy
    buffer that is freed after the capture; both are refused while capturing."""

    _cache = {}
    _maps = {}
    _captured = []
    _reserve = []   # (pinned host int64 buffer, device int64 buffer) pairs, allocated outside any capture

    def __new__(cls, params, grads, m, v):
        key = tuple((p.data_ptr(), g.data_ptr(), 0 if a is None else a.data_ptr(), 0 if b is None else b.data_ptr(),
                     p.numel()) for p, g, a, b in zip(params, grads, m, v))
        dev = params[0].device
        hit = cls._cache.get((dev, key))
        if hit is not None:
            return hit
        capturing = torch.cuda.is_current_stream_capturing()
        self = super().__new__(cls)
        rows = np.array(key, dtype=np.int64).reshape(-1, 5)
        numels = tuple(int(k[4]) for k in key)
        mp = cls._maps.get((dev, numels))
        if mp is None:
            if capturing:
                raise RuntimeError("ldm_amd.optim: a slot table's chunk map is built outside a graph capture only "
                                   "(run the step eagerly once before capturing it)")
            nch = (rows[:, 4] + CHUNK - 1) // CHUNK
            ct = np.repeat(np.arange(len(rows), dtype=np.int32), nch)
            first = np.repeat(np.cumsum(nch) - nch, nch)
            cs = (np.arange(int(nch.sum()), dtype=np.int64) - first) * CHUNK
            mp = (torch.from_numpy(ct).to(dev), torch.from_numpy(cs).to(dev), int(len(ct)))
            cls._maps[(dev, numels)] = mp
        self.chunk_tensor, self.chunk_start, self.nchunks = mp
        if capturing:
            res = cls._reserve[-1] if cls._reserve else None
            if res is None or res[0].numel() < rows.size or res[1].device != dev:
                raise RuntimeError("ldm_amd.optim: slot tables are built and filled outside a graph capture only; "
                                   "call reserve_capture_buffers(device=...) before capturing an optimizer step")
            host, dbuf = cls._reserve.pop()
            host = host[:rows.size].view(rows.shape)
            host.copy_(torch.from_numpy(rows))
            self._host = host
            self.slots = dbuf[:rows.size].view(rows.shape)   # reserved before the capture: never a graph-pool block
            self._filled = False
            cls._captured.append(self)
            self._captured_key = (dev, key)
        else:
            self.slots = torch.empty(rows.shape, dtype=torch.int64, device=dev)
            host = torch.from_numpy(rows).pin_memory()    # caching host allocator: reused once the copy ran
            self.slots.copy_(host, non_blocking=True)
        self.key = key
        if len(cls._cache) > 64:
            cls._cache.clear()
        cls._cache[(dev, key)] = self
        return self

    def __init__(self, *args):
        pass


def reserve_capture_buffers(n=4, words=1 << 14, device="cuda"):
    """Pinned host buffers and device buffers for the slot tables built while a step is being captured into
    a hipGraph (one pair per optimizer / unscale table in the step); call before torch.cuda.graph, outside
    the capture.  Returns the list that will hold the tables the capture builds: pass it to fill_captured()
    once the capture has ended (before the first replay), and to release_captured() when the graph is
    dropped."""
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("ldm_amd.optim.reserve_capture_buffers: call it before the capture starts")
    dev = torch.device(device)
    _SlotTable._reserve = [r for r in _SlotTable._reserve if r[1].device == dev]
    while len(_SlotTable._reserve) < n:
        _SlotTable._reserve.append((torch.empty(words, dtype=torch.int64, pin_memory=True),
                                    torch.empty(words, dtype=torch.int64, device=dev)))
    _SlotTable._captured = []
    return _SlotTable._captured


def fill_captured(tables):
    """Upload the rows of the slot tables a capture built (on the current stream, outside the capture; the
    graph's replays on this stream come after the copies).  Idempotent."""
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("ldm_amd.optim.fill_captured: the tables are filled after the capture has ended")
    for tab in tables:
        if not tab._filled:
            tab.slots.copy_(tab._host, non_blocking=True)
            tab._filled = True


def release_captured(tables):
    """Forget the slot tables (and their pinned host rows) of a captured graph that is being replaced: they
    leave the table cache, so the pinned buffers and device tables die with the graph."""
    if not tables:
        return
    for tab in tables:
        k = getattr(tab, "_captured_key", None)
        if k is not None and _SlotTable._cache.get(k) is tab:
            del _SlotTable._cache[k]
    tables.clear()
    _SlotTable._reserve.clear()


def scale_tensors_(tensors, factor):
    """t *= factor for every (contiguous fp32 device) tensor, one multi-tensor launch; returns a device
    int32 [1] flag, nonzero if any result is non-finite."""
    tensors = [t for t in tensors if t.numel()]
    if not tensors:
        return False
    require_device(*tensors, what="scale_tensors_")
    tab = _SlotTable(tensors, tensors, [None] * len(tensors), [None] * len(tensors))
    f = torch.full((1,), float(factor), dtype=torch.float32, device=tensors[0].device)
    bad = torch.zeros((1,), dtype=torch.int32, device=tensors[0].device)
    L.call("ldm_unscale_check", tab.slots.data_ptr(), tab.chunk_tensor.data_ptr(), tab.chunk_start.data_ptr(),
           tab.nchunks, CHUNK, f.data_ptr(), bad.data_ptr(), stream_handle())
    return bad


def _check_params(params):
    for p in params:
        require_device(p, what="ldm_amd.optim")
        if not p.is_contiguous() or (p.grad is not None and not p.grad.is_contiguous()):
            raise RuntimeError("ldm_amd.optim: parameters and gradients must be contiguous")
        if p.grad is not None and p.grad.is_sparse:
            raise RuntimeError("ldm_amd.optim: sparse gradients are not supported")


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad=False, maximize=False, no capturable/differentiable) on one fused
    multi-tensor kernel per param group."""

    _decoupled = 0

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False,
                 capturable=False):
        if amsgrad:
            raise NotImplementedError("ldm_amd.optim.Adam: amsgrad is not supported")
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameters: {betas}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False))
        self._tables = {}
        # capturable (torch.optim.Adam(capturable=True)): the step count is a device tensor advanced by the
        # kernel itself, so step() never reads it on the host and can be captured into a hipGraph
        self.capturable = bool(capturable)

    @torch.no_grad()
    def step(self, closure=None, found_inf=None):
        """One Adam update.  found_inf (device int32 [1], optional): skip on the device if set."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            _check_params(params)
            beta1, beta2 = group["betas"]
            if self.capturable:
                self._step_capturable(gi, group, params, found_inf, beta1, beta2)
                continue
            if "_ldm_step" in group:
                # leaving the capturable form: every param gets its own host step count again (the shared
                # device count must not be advanced once per param by the eager loop below)
                self._unshare_steps(group)
            # group the params by their step count (all equal unless params were added later)
            by_step = {}
            for p in params:
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                by_step.setdefault(int(st["step"].item()), []).append(p)
            for step, ps in by_step.items():
                grads = [p.grad for p in ps]
                tab = _SlotTable(ps, grads, [self.state[p]["exp_avg"] for p in ps],
                                 [self.state[p]["exp_avg_sq"] for p in ps])
                L.call("ldm_adam_step", tab.slots.data_ptr(), tab.chunk_tensor.data_ptr(), tab.chunk_start.data_ptr(),
                       tab.nchunks, CHUNK, float(group["lr"]), float(beta1), float(beta2), float(group["eps"]),
                       float(group["weight_decay"]), self._decoupled, step,
                       None if found_inf is None else found_inf.data_ptr(), stream_handle())
                # the tables are read by the kernel asynchronously: keep them alive until it ran
                self._tables[(gi, step)] = tab
                # the kernel wrote the parameters through raw pointers: move their autograd versions the
                # way an in-place torch update does, so that version-keyed caches (packed conv weights,
                # ops.packed_weight; the UNet engine's step weights) re-pack them
                for p in ps:
                    torch.autograd.graph.increment_version(p)
        return loss


    _GROUP_PRIVATE = ("_ldm_step", "_ldm_scalars", "_ldm_tabs")

    def _unshare_steps(self, group):
        gstep = group.pop("_ldm_step")
        group.pop("_ldm_scalars", None)
        n = float(gstep)
        for p in group["params"]:
            st = self.state.get(p)
            if st and st.get("step") is gstep:
                st["step"] = torch.tensor(n)

    def state_dict(self):
        """torch.optim state_dict, with every param's 'step' a CPU tensor of its own (the capturable form
        shares one device count per group) and without this class's private per-group device tensors, so
        that it loads into torch.optim.Adam or into an eager / capturable instance of this class alike."""
        sd = super().state_dict()
        for g in sd["param_groups"]:
            for k in self._GROUP_PRIVATE:
                g.pop(k, None)
        state = {}
        for idx, st in sd["state"].items():
            st = dict(st)
            if "step" in st and torch.is_tensor(st["step"]):
                st["step"] = torch.tensor(float(st["step"]))
            state[idx] = st
        sd["state"] = state
        return sd

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        for g in self.param_groups:
            for k in self._GROUP_PRIVATE:
                g.pop(k, None)
            for p in g["params"]:
                st = self.state.get(p)
                if st and "step" in st and torch.is_tensor(st["step"]):
                    st["step"] = torch.tensor(float(st["step"]))
        self._tables.clear()
        # a captured train step holds the old state tensors: LDMTrainer re-captures when this moves
        self.state_epoch = getattr(self, "state_epoch", 0) + 1

    def _step_capturable(self, gi, group, params, found_inf, beta1, beta2):
        """One launch pair for the group: ldm_adam_step_dev advances the group's device step count (shared
        by its params' state["step"]) unless found_inf is set and forms the scalars from it on the device."""
        dev = params[0].device
        gstep = group.get("_ldm_step")
        if gstep is None:
            prev = [self.state[p]["step"] for p in params if len(self.state[p]) > 0]
            init = float(prev[0]) if prev else 0.0
            if any(float(s) != init for s in prev):
                raise RuntimeError("ldm_amd.optim.Adam(capturable=True): params of a group at different steps")
            gstep = torch.full((), init, dtype=torch.float32, device=dev)
            group["_ldm_step"] = gstep
            group["_ldm_scalars"] = torch.zeros(8, dtype=torch.float32, device=dev)
        for p in params:
            st = self.state[p]
            if len(st) == 0 or "exp_avg" not in st:
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["step"] = gstep
        tab = _SlotTable(params, [p.grad for p in params], [self.state[p]["exp_avg"] for p in params],
                         [self.state[p]["exp_avg_sq"] for p in params])
        L.call("ldm_adam_step_dev", tab.slots.data_ptr(), tab.chunk_tensor.data_ptr(), tab.chunk_start.data_ptr(),
               tab.nchunks, CHUNK, float(group["lr"]), float(beta1), float(beta2), float(group["eps"]),
               float(group["weight_decay"]), self._decoupled, gstep.data_ptr(),
               None if found_inf is None else found_inf.data_ptr(), group["_ldm_scalars"].data_ptr(), stream_handle())
        self._tables[(gi, "dev")] = tab
        for p in params:
            torch.autograd.graph.increment_version(p)


class AdamW(Adam):
    """torch.optim.AdamW (decoupled weight decay, default 1e-2)."""

    _decoupled = 1

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False,
                 capturable=False):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad,
                         capturable=capturable)


class GradScaler:
    """torch.amp.GradScaler('cuda') semantics: scale(loss) multiplies by the current scale, step()
    unscales the grads (device kernel), skips the optimiser step when any grad is inf/nan, update()
    backs the scale off (x0.5) on inf or grows it (x2) after growth_interval clean steps."""

    def __init__(self, device="cuda", init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5,
                 growth_interval=2000, enabled=True):
        self._device = device
        self._init_scale = init_scale
        self._growth_factor = growth_factor
        self._backoff_factor = backoff_factor
        self._growth_interval = growth_interval
        self._enabled = enabled
        self._scale = None
        self._tracker = None
        self._found_inf = None
        self._unscaled = set()
        self._divisor = 1.0

    def is_enabled(self):
        return self._enabled

    def set_grad_divisor(self, d):
        """Extra factor 1/d folded into unscale_ (data-parallel gradient averaging: d = world size)."""
        self._divisor = float(d)

    def _lazy_init(self, dev):
        if self._scale is None:
            self._scale = torch.full((1,), self._init_scale, dtype=torch.float32, device=dev)
            self._tracker = torch.zeros((1,), dtype=torch.int32, device=dev)
            self._found_inf = torch.zeros((1,), dtype=torch.int32, device=dev)

    def get_scale(self):
        return float(self._scale.item()) if self._scale is not None else self._init_scale

    def scale(self, outputs):
        if not self._enabled:
            return outputs
        self._lazy_init(outputs.device)
        return outputs * self._scale.to(outputs.device)

    def unscale_(self, optimizer):
        if not self._enabled or id(optimizer) in self._unscaled:
            return
        self._lazy_init(next(p.device for g in optimizer.param_groups for p in g["params"]))
        # GradScaler: scale.double().reciprocal().float()  (x 1/divisor for data-parallel averaging)
        inv = torch.reciprocal(self._scale.double() * self._divisor).float()
        self._found_inf.zero_()
        for group in optimizer.param_groups:
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            _check_params(ps)
            tab = _SlotTable(ps, [p.grad for p in ps], [None] * len(ps), [None] * len(ps))
            L.call("ldm_unscale_check", tab.slots.data_ptr(), tab.chunk_tensor.data_ptr(), tab.chunk_start.data_ptr(),
                   tab.nchunks, CHUNK, inv.data_ptr(), self._found_inf.data_ptr(), stream_handle())
            group.setdefault("_ldm_tabs", []).append(tab)   # keep alive until the launch ran
        self._unscaled.add(id(optimizer))

    def step(self, optimizer, *args, **kwargs):
        if not self._enabled:
            return optimizer.step(*args, **kwargs)
        self.unscale_(optimizer)
        for group in optimizer.param_groups:
            group.pop("_ldm_tabs", None)
        if getattr(optimizer, "capturable", False):
            # device-side skip: the kernel pair reads found_inf and leaves the step count alone on inf/nan
            return optimizer.step(*args, found_inf=self._found_inf, **kwargs)
        # torch's GradScaler also syncs here (found_inf.item()) so that the optimiser's step counters
        # only advance on applied steps
        if int(self._found_inf.item()) == 0:
            return optimizer.step(*args, **kwargs)
        return None

    def update(self, new_scale=None):
        if not self._enabled:
            return
        if new_scale is not None:
            self._scale.fill_(float(new_scale))
        else:
            L.call("ldm_update_scale", self._scale.data_ptr(), self._tracker.data_ptr(), self._found_inf.data_ptr(),
                   float(self._growth_factor), float(self._backoff_factor), int(self._growth_interval),
                   stream_handle())
        self._unscaled.clear()

    def state_dict(self):
        if not self._enabled:
            return {}
        return {"scale": self.get_scale(), "growth_factor": self._growth_factor,
                "backoff_factor": self._backoff_factor, "growth_interval": self._growth_interval,
                "_growth_tracker": int(self._tracker.item()) if self._tracker is not None else 0}

    def load_state_dict(self, sd):
        if not sd:
            return
        self._init_scale = sd["scale"]
        self._growth_factor = sd["growth_factor"]
        self._backoff_factor = sd["backoff_factor"]
        self._growth_interval = sd["growth_interval"]
        if self._scale is not None:
            self._scale.fill_(sd["scale"])
            self._tracker.fill_(sd["_growth_tracker"])
