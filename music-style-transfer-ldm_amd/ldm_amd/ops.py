"""Tensor-level entry points over the C ABI (torch tensors in, torch tensors out).

torch is only the owner of device memory and streams here; every arithmetic operation of the hot
path runs in libldm_amd.so.  Inputs must be contiguous float32 tensors on a HIP device: there is no
CPU fallback (a CPU tensor raises).
"""
import ctypes
import math
import weakref

import os

import torch

from . import _lib as L

byref = ctypes.byref


# ------------------------------------------------------------------------------------------------
# helpers
# ------------------------------------------------------------------------------------------------
def stream_handle():
    """Raw hipStream_t of the caller's current stream (the direct C query: torch.cuda.current_stream()
    costs ~10 us of Python per call, ~0.5 ms per train step)."""
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def _p(t):
    return None if t is None else t.data_ptr()


def require_device(*ts, dtype=torch.float32, what="music-style-transfer-ldm_amd"):
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError(f"{what}: tensor on {t.device}; the HIP kernels need a GPU tensor "
                               "(there is no CPU fallback)")
        if dtype is not None and t.dtype != dtype:
            raise RuntimeError(f"{what}: expected {dtype}, got {t.dtype}")


def f32c(t):
    """contiguous float32 view/copy on the same device (a dtype cast is a device copy, not compute)."""
    if t.dtype != torch.float32:
        t = t.to(torch.float32)
    return t.contiguous()


# ---- 16-bit storage of the train step's large maps -------------------------------------------------------
# Inside a torch.autocast region ATen stores conv / BatchNorm / activation outputs as fp16 / bf16 tensors (and
# autograd their gradients likewise).  Maps of at least LDM_AMD_STORE16_MIN elements (default 2^22: the VAE and
# style-encoder maps at the train batch) are stored that way here too, where the kernels that produce and read
# them take 16-bit storage (ldm_conv_storage16 / ldm_conv_wgrad_storage16; BatchNorm and the activation
# backward always); anything else reads a 16-bit tensor through an fp32 copy.  LDM_AMD_STORE16=0: fp32 maps.
T16 = {torch.float16: 1, torch.bfloat16: 2}
TORCH16 = {1: torch.float16, 2: torch.bfloat16}


def store16_dtype(numel, dt):
    """The torch dtype a new map of `numel` elements is stored in at operand precision dt (fp32 or 16-bit)."""
    if dt in TORCH16 and os.environ.get("LDM_AMD_STORE16", "1") != "0" and \
            numel >= int(os.environ.get("LDM_AMD_STORE16_MIN", str(1 << 22))):
        return TORCH16[dt]
    return torch.float32


def in16(t, dt, ok=True):
    """(contiguous tensor, is16) as a kernel reads t: a 16-bit t of type dt as it is when ok, else fp32."""
    if t.dtype == torch.float32:
        return t.contiguous(), False
    if ok and T16.get(t.dtype) == dt:
        return t.contiguous(), True
    return f32c(t), False


def st_code(dt, **flags):
    """BatchNorm / activation-backward storage bits of an act code: the 16-bit type and the LDM_ST_* flags
    (x16, y16, dy16, dx16) that are set."""
    names = {"x16": L.ST_X16, "y16": L.ST_Y16, "dy16": L.ST_DY16, "dx16": L.ST_DX16}
    bits = 0
    for k, v in flags.items():
        if v:
            bits |= names[k]
    return ((int(dt) << L.ST_SHIFT) | bits) if bits else 0


_ST16_CACHE = {}


def conv_storage16(desc, plan, dt):
    """LDM_DT_X16 | LDM_DT_Y16 bits the conv kernels take for (desc, plan) at operand precision dt."""
    if not dt:
        return 0
    key = ("f", desc.key(), plan.kind, plan.tm, plan.tn)
    v = _ST16_CACHE.get(key)
    if v is None:
        v = _ST16_CACHE[key] = int(L.load().ldm_conv_storage16(byref(desc), byref(plan)))
    return v


def wgrad_storage16(desc, dt):
    if not dt:
        return 0
    key = ("w", desc.key())
    v = _ST16_CACHE.get(key)
    if v is None:
        v = _ST16_CACHE[key] = int(L.load().ldm_conv_wgrad_storage16(byref(desc)))
    return v


# ------------------------------------------------------------------------------------------------
# plans and packed weights
# ------------------------------------------------------------------------------------------------
class IdCache:
    """Per-object cache keyed by identity (tensors cannot key a WeakKeyDictionary: their __eq__ is
    elementwise).  Entries die with their key object."""

    def __init__(self):
        self._d = {}

    def get(self, obj, default=None):
        hit = self._d.get(id(obj))
        if hit is None or hit[0]() is not obj:
            return default
        return hit[1]

    def __setitem__(self, obj, value):
        k = id(obj)
        self._d[k] = (weakref.ref(obj, lambda _r, k=k, d=self._d: d.pop(k, None)), value)

    def clear(self):
        self._d.clear()


_PLAN_CACHE = {}
_PLAN_OVERRIDE = {}      # desc.key() -> (kind, tm, tn, wk, ks), filled by the autotuner / tests
_PACK_CACHE = IdCache()


def make_desc(B, Cin, Hin, Win, Cout, kh, kw, stride, pad, out_pad=0, transposed=False):
    if transposed:
        Hout = (Hin - 1) * stride - 2 * pad + kh + out_pad
        Wout = (Win - 1) * stride - 2 * pad + kw + out_pad
    else:
        Hout = (Hin + 2 * pad - kh) // stride + 1
        Wout = (Win + 2 * pad - kw) // stride + 1
    return L.ConvDesc(B, Cin, Hin, Win, Cout, Hout, Wout, kh, kw, stride, pad, out_pad, int(bool(transposed)))


def get_plan(desc, force=None):
    key = desc.key()
    force = force or _PLAN_OVERRIDE.get(key)
    if force is not None:
        force = tuple(force) + (1,) * (5 - len(force))     # (kind, tm, tn, wk[, ks])
        plan = L.ConvPlan()
        L.call("ldm_conv_make_plan_forced", byref(desc), *force, byref(plan))
        return plan
    plan = _PLAN_CACHE.get(key)
    if plan is None:
        plan = L.ConvPlan()
        L.call("ldm_conv_make_plan", byref(desc), byref(plan))
        _PLAN_CACHE[key] = plan
    return plan


_TILED_CACHE = {}


def tiled_plan(desc, dt, adds=False):
    """The 16-bit-operand LDS-staged plan for desc at operand precision dt: kind 3 (tconv.hip, large planes; no
    + bcast / + skip epilogue, so not when `adds`), else kind 4 (sconv.hip, small planes, any epilogue), or None
    when the layer is of neither class.  LDM_AMD_TILED=0 turns both off (LDM_AMD_SCONV=0 kind 4 alone)."""
    if dt == 0 or os.environ.get("LDM_AMD_TILED", "1") == "0":
        return None
    # kind 4 under fp16 only with LDM_AMD_SCONV_F16=1: there the general kernel keeps fp32 operands, and the
    # reference-fp16 GradScaler step's parity bound (tests/test_gpu_train_fp16.py) was set on that form
    k4 = int(dt) == 2 or os.environ.get("LDM_AMD_SCONV_F16", "0") == "1"
    key = (desc.key(), int(dt), bool(adds), k4)
    if key not in _TILED_CACHE:
        lib = L.load()
        plan = L.ConvPlan()
        ok = not adds and lib.ldm_conv_tiled_plan(byref(desc), int(dt), byref(plan)) == 0
        if not ok and k4:
            plan = L.ConvPlan()
            ok = lib.ldm_conv_sconv_plan(byref(desc), int(dt), byref(plan)) == 0
        _TILED_CACHE[key] = plan if ok else None
    return _TILED_CACHE[key]


def set_plan_override(desc, kind, tm=1, tn=1, wk=1, ks=1):
    _PLAN_OVERRIDE[desc.key()] = (kind, tm, tn, wk, ks)


def clear_plan_overrides():
    _PLAN_OVERRIDE.clear()


def packed_weight(weight, desc, plan, owner=None, tag=None):
    """Weight re-laid into the plan's MFMA fragment order; cached per (owner tensor, _version, layout).

    `owner`/`tag` let a slice of a parameter (the q / kv rows of in_proj_weight) be cached against the
    parameter itself, whose _version moves on every in-place update."""
    if plan.kind == 0:
        return weight
    owner = weight if owner is None else owner
    key = (owner._version, tag, desc.Cin, desc.Cout, desc.kh, desc.kw, desc.stride, desc.pad, desc.out_pad,
           desc.transposed, plan.kind, plan.tm, plan.tn if plan.kind in (3, 4) else 0)
    per = _PACK_CACHE.get(owner)
    if per is None:
        per = {}
        _PACK_CACHE[owner] = per
    buf = per.get(key)
    w = None
    if buf is None:
        # drop stale versions of this weight
        for k in [k for k in per if k[0] != owner._version]:
            del per[k]
        w = f32c(weight.detach())
        buf = torch.empty(int(plan.packed_floats), device=weight.device, dtype=torch.float32)
        L.call("ldm_conv_pack_weight", byref(desc), byref(plan), w.data_ptr(), buf.data_ptr(), stream_handle())
        per[key] = buf
    if _RECORD is not None and owner.requires_grad and owner.grad_fn is None:
        _RECORD.add(owner, key[1:], weight.detach() if w is None else w, desc, plan, buf)
    return buf


_RECORD = None


class _PackRecord:
    """The packs of trainable weights one step reads (filled by packed_weight while record_packs is open)."""

    def __init__(self):
        self.entries = {}

    def add(self, owner, tail, w, desc, plan, buf):
        # only a pack that reads the owner's own storage can be refreshed from it later (not a cast copy)
        if plan.kind not in (1, 2, 3, 4) or w.dtype != torch.float32 or not w.is_contiguous() or \
                w.untyped_storage().data_ptr() != owner.untyped_storage().data_ptr():
            return
        # no reference to w itself: a slice of a parameter (in_proj rows) keeps its autograd node alive, and
        # an AccumulateGrad node from an eager step breaks a later graph capture of the step
        self.entries.setdefault((id(owner), tail), (owner, tail, w.data_ptr() - owner.data_ptr(),
                                                    L.ConvDesc.from_buffer_copy(desc),
                                                    L.ConvPlan.from_buffer_copy(plan), buf))


class record_packs:
    """with record_packs() as rec: ... -- rec.entries then lists every trainable-weight pack read inside."""

    def __enter__(self):
        global _RECORD
        self._prev, _RECORD = _RECORD, _PackRecord()
        return _RECORD

    def __exit__(self, *exc):
        global _RECORD
        _RECORD = self._prev
        return False


class PackSet:
    """Every packed trainable conv weight of a train step re-packed by ONE launch (pack.hip ldm_pack_many)
    after the optimizer step, instead of one ldm_conv_pack_weight launch per weight at its first use in the
    next step's forward / backward (51 launches per step at B = 32).  The buffers are packed_weight's own
    cache entries; after a re-pack they are re-keyed to their owners' current _version, so the next step's
    packed_weight calls hit them.  Built from a record_packs() pass over one step."""

    def __init__(self, record, device):
        ents = list(record.entries.values())
        self.owners = [e[0] for e in ents]
        self.tails = [e[1] for e in ents]
        self.bufs = [e[5] for e in ents]
        self.ptrs = tuple(o.data_ptr() for o in self.owners)
        self.wptrs = [o.data_ptr() + e[2] for o, e in zip(self.owners, ents)]   # the packed weights (or slices)
        self.descs = [e[3] for e in ents]
        self.plans = [e[4] for e in ents]
        self.n = n = len(ents)
        descs = (L.ConvDesc * n)(*self.descs)
        plans = (L.ConvPlan * n)(*self.plans)
        wptr = (ctypes.c_void_p * n)(*self.wptrs)
        optr = (ctypes.c_void_p * n)(*[e[5].data_ptr() for e in ents])
        host = ctypes.create_string_buffer(int(L.load().ldm_pack_job_bytes()) * n)
        launch = ctypes.c_int64()
        L.call("ldm_pack_many_prepare", descs, plans, wptr, optr, n, ctypes.addressof(host), byref(launch))
        self.launch = int(launch.value)
        self.table = torch.frombuffer(bytearray(host.raw), dtype=torch.uint8).to(device)
        self.versions = None

    def valid(self):
        """False once a weight moved to other storage (the job table holds raw pointers)."""
        return all(o.data_ptr() == p for o, p in zip(self.owners, self.ptrs))

    def current(self):
        return self.versions == tuple(o._version for o in self.owners)

    def repack(self):
        """Launch the re-pack on the current stream, then re-key the buffers.  Inside a graph capture only the
        launch is recorded: the buffers hold the new packs once the replay ran (the caller re-keys then)."""
        if not self.valid():
            raise RuntimeError("PackSet: a recorded weight moved to new storage; build a new PackSet")
        L.call("ldm_pack_many", self.table.data_ptr(), self.n, self.launch, stream_handle())
        if not torch.cuda.is_current_stream_capturing():
            self.rekey()

    def rekey(self):
        """Declare the buffers packs of the owners' current versions (the caller knows they are)."""
        for owner, tail, buf in zip(self.owners, self.tails, self.bufs):
            v = owner._version
            per = _PACK_CACHE.get(owner)
            if per is None:
                per = {}
                _PACK_CACHE[owner] = per
            for k in [k for k in per if k[0] != v]:
                del per[k]
            per[(v,) + tail] = buf
        self.versions = tuple(o._version for o in self.owners)


# ------------------------------------------------------------------------------------------------
# convolution with fused epilogue
# ------------------------------------------------------------------------------------------------
def conv_forward(x, weight, bias=None, *, stride=1, padding=1, transposed=False, output_padding=0, bn=None,
                 act="none", bcast=None, skip=None, out=None, plan=None, wkey=None, act_out=None, dtype=None,
                 out_dtype=None):
    """act(BN_eval(conv(x, w) + bias)) (+ bcast[b, c]) (+ skip).  bn = (gamma, beta, mean, var, eps).
    act_out (preallocated, output-shaped) also receives act(.) before the adds.  x may be a 16-bit map of the
    operand type; out_dtype = that 16-bit type asks for a 16-bit y where the kernel stores one (else fp32)."""
    require_device(x, bcast, skip, dtype=None)   # (bcast / skip: read through fp32 copies when 16-bit)
    require_device(weight, bias)
    B, Cin, H, W = x.shape
    if transposed:
        cin_w, Cout, kh, kw = weight.shape
    else:
        Cout, cin_w, kh, kw = weight.shape
    if cin_w != Cin:
        raise RuntimeError(f"conv: input has {Cin} channels, weight expects {cin_w}")
    desc = make_desc(B, Cin, H, W, Cout, kh, kw, stride, padding, output_padding, transposed)
    if desc.Hout <= 0 or desc.Wout <= 0:
        raise RuntimeError("conv: non-positive output size")
    if B == 0:   # an empty batch shard (data-parallel sampling with B < world size): nothing to launch
        return out if out is not None else torch.empty((0, Cout, desc.Hout, desc.Wout), device=x.device,
                                                       dtype=torch.float32)
    dt = autocast_dt() if dtype is None else int(dtype)
    if plan is None:
        plan = tiled_plan(desc, dt, adds=bcast is not None or skip is not None)
    plan = plan or get_plan(desc)
    wbuf = packed_weight(weight, desc, plan, *(wkey or ()))
    st = conv_storage16(desc, plan, dt)
    if st and plan.kind == 0 and (bcast is not None or skip is not None or
                                  (out is not None and out.data_ptr() % 16) or
                                  (act_out is not None and act_out.data_ptr() % 16)):
        # the VALU convs that take 16-bit maps (Cin = 1 stride 2: y; 64 -> 1 k4 s2 convT: x) run only with a
        # simple epilogue and 16-byte aligned y / act_out (conv.hip conv_forward_ex); any other call of those
        # shapes takes the general direct kernel with fp32 maps
        st = 0
    x, xh = in16(x, dt, st & L.DT_X16)
    y16 = out is None and act_out is None and T16.get(out_dtype) == dt and bool(st & L.DT_Y16)
    y = out if out is not None else torch.empty((B, Cout, desc.Hout, desc.Wout), device=x.device,
                                                dtype=out_dtype if y16 else torch.float32)
    ep = L.Epilogue()
    ep.bias = _p(bias)
    ep.dtype = autocast_out(dt) | (L.DT_X16 if xh else 0) | (L.DT_Y16 if y16 else 0)
    keep = []
    if bn is not None:
        g, b_, m, v, eps = bn
        require_device(g, b_, m, v)
        ep.bn_weight, ep.bn_bias, ep.bn_mean, ep.bn_var = _p(g), _p(b_), _p(m), _p(v)
        ep.bn_eps = float(eps)
    ep.act = L.ACT[act]
    if bcast is not None:
        bcast = f32c(bcast)
        keep.append(bcast)
        ep.bcast_add = bcast.data_ptr()
    if skip is not None:
        skip = f32c(skip)
        keep.append(skip)
        ep.skip_add = skip.data_ptr()
    if act_out is not None:
        require_device(act_out)
        assert act_out.is_contiguous() and act_out.shape == y.shape
        ep.act_out = act_out.data_ptr()
    L.call("ldm_conv_forward_ws", byref(desc), byref(plan), x.data_ptr(), _p(wbuf), byref(ep), y.data_ptr(),
           split_workspace(plan, x.device), stream_handle())
    return y


def autocast_out(dt, round_out=None):
    """The ldm_epilogue.dtype bits for operand precision dt.  round_out=None: inside a torch.autocast region
    (and dt != 0) the outputs are rounded to dt as well (LDM_DT_ROUND_OUT), as ATen's autocast conv / linear /
    BatchNorm return 16-bit tensors (the reference's train step, train.py:174); outside one (explicit-dtype
    kernel calls) operands only.  True / False force it (the backward passes what its forward did).
    LDM_AMD_AUTOCAST_OUT=0: operands only everywhere (rounds 1-3)."""
    dt = int(dt)
    if round_out is None:
        round_out = torch.is_autocast_enabled("cuda")
    if dt and round_out and os.environ.get("LDM_AMD_AUTOCAST_OUT", "1") != "0":
        return dt | L.DT_ROUND_OUT
    return dt


def autocast_dt(device_type="cuda"):
    """LDM_DT_* for the MFMA kernels from the caller's torch.autocast region: fp16 / bf16 operands (fp32
    accumulation, epilogue and outputs) inside one, fp32 outside.  LDM_AMD_DTYPE=fp32 turns it off."""
    if os.environ.get("LDM_AMD_DTYPE", "") in ("fp32", "f32"):
        return 0
    if not torch.is_autocast_enabled(device_type):
        return 0
    dt = torch.get_autocast_dtype(device_type)
    return 1 if dt == torch.float16 else (2 if dt == torch.bfloat16 else 0)


def dual_desc(desc):
    """Descriptor whose forward is the data gradient of `desc`: conv <-> transposed conv with the same
    kernel, stride and padding (the torch weight tensor is reused unchanged in both directions)."""
    d = L.ConvDesc(desc.B, desc.Cout, desc.Hout, desc.Wout, desc.Cin, desc.Hin, desc.Win, desc.kh, desc.kw,
                   desc.stride, desc.pad, 0, 1 - desc.transposed)
    if d.transposed:
        d.out_pad = desc.Hin - ((desc.Hout - 1) * desc.stride - 2 * desc.pad + desc.kh)
        if d.out_pad != desc.Win - ((desc.Wout - 1) * desc.stride - 2 * desc.pad + desc.kw) or \
                not 0 <= d.out_pad < max(1, desc.stride):
            raise RuntimeError("conv backward: input size not reachable by a transposed conv (ragged stride)")
    return d


def conv_backward_data(dy, weight, desc, wkey=None, dtype=0, round_out=False, out_dtype=None):
    """dX of the conv/convT `desc` for the pre-epilogue gradient dy (forward kernel on the dual desc);
    dtype = LDM_DT_* operand precision (the forward's autocast precision); round_out: dX rounded to it as well
    (the reference's data gradient of a 16-bit conv is a 16-bit tensor); out_dtype: a 16-bit dX where the
    kernel stores one (the gradient of a 16-bit map; fp32 otherwise)."""
    dd = dual_desc(desc)
    dtype = int(dtype)
    plan = tiled_plan(dd, dtype) or get_plan(dd)
    wbuf = packed_weight(weight, dd, plan, *(wkey or ()))
    st = conv_storage16(dd, plan, dtype)
    dy, dyh = in16(dy, dtype, st & L.DT_X16)
    d16 = T16.get(out_dtype) == dtype and bool(st & L.DT_Y16)
    dx = torch.empty((desc.B, desc.Cin, desc.Hin, desc.Win), device=dy.device,
                     dtype=out_dtype if d16 else torch.float32)
    ep = L.Epilogue()
    ep.dtype = autocast_out(dtype, round_out) | (L.DT_X16 if dyh else 0) | (L.DT_Y16 if d16 else 0)
    L.call("ldm_conv_forward_ws", byref(dd), byref(plan), dy.data_ptr(), _p(wbuf), byref(ep), dx.data_ptr(),
           split_workspace(plan, dy.device), stream_handle())
    return dx


_WS = {}


def _stream_key(device):
    d = torch.device(device)
    return torch.cuda.current_stream(d).cuda_stream if d.type == "cuda" else 0


def scratch(name, nfloats, device):
    """Per-(device, stream) scratch buffer reused across stream-ordered calls (grown on demand): the train
    step runs independent branches on their own streams (graphs.branch), each with its own buffers.

    Memory: one buffer per (name, device, stream) at the largest size asked for, kept until release_workspaces()
    — at config 3 (B = 32) the weight-gradient scratch is the largest (the split-K partials of the biggest layer,
    ~38 MB) and exists once per stream that ran a backward (the origin stream and graphs.branch's pool, three
    streams: ~0.1 GB); a program that creates streams of its own should call release_workspaces() when done."""
    key = (name, str(device), _stream_key(device))
    buf = _WS.get(key)
    if buf is None or buf.numel() < nfloats:
        buf = torch.empty(max(int(nfloats), 1), device=device, dtype=torch.float32)
        _WS[key] = buf
    return buf


_SPLIT_WS = {}


def release_workspaces():
    """Drop every cached scratch / split-K workspace (all devices and streams); the next call re-allocates.
    Not while a captured graph that uses them may still replay: the graph keeps the addresses it recorded."""
    _WS.clear()
    _SPLIT_WS.clear()


def split_workspace(plan, device):
    """Zero-initialised workspace for a plan that splits K across blocks (None when it does not).  One
    buffer per (device, stream): its tile counters return to zero after every launch, so stream-ordered
    calls share it; another stream gets its own."""
    if plan.ws_floats <= 0:
        return None
    key = (str(device), torch.cuda.current_stream(device).cuda_stream)
    buf = _SPLIT_WS.get(key)
    if buf is None or buf.numel() < plan.ws_floats:
        buf = torch.zeros(int(plan.ws_floats), device=device, dtype=torch.float32)
        _SPLIT_WS[key] = buf
    return buf.data_ptr()


def conv_backward_weight(x, dy, desc, dw=None, accumulate=False, dtype=0):
    """dW (torch layout) of conv/convT `desc` from its input x and pre-epilogue gradient dy; dtype =
    LDM_DT_* operand precision."""
    dtype = int(dtype)
    st = wgrad_storage16(desc, dtype)
    if st == L.DT_X16 | L.DT_DY16 and (T16.get(x.dtype) == dtype) != (T16.get(dy.dtype) == dtype):
        # one 16-bit map and one fp32 map: the fp32 one rounded to the operand type first (the kernel rounds
        # it the same way, RNE), so both tiles take the 16-bit DMA form (wgrad_lp16_kernel) — same result
        if T16.get(x.dtype) == dtype:
            dy = dy.to(TORCH16[dtype])
        else:
            x = x.to(TORCH16[dtype])
    x, xh = in16(x, dtype, st & L.DT_X16)
    dy, dyh = in16(dy, dtype, st & L.DT_DY16)
    if desc.transposed:
        shape = (desc.Cin, desc.Cout, desc.kh, desc.kw)
    else:
        shape = (desc.Cout, desc.Cin, desc.kh, desc.kw)
    if dw is None:
        dw = torch.empty(shape, device=x.device, dtype=torch.float32)
    nws = int(L.load().ldm_conv_wgrad_workspace_floats(byref(desc)))
    code = dtype | (L.DT_X16 if xh else 0) | (L.DT_DY16 if dyh else 0)
    if _BIAS_DEFER:   # the split-K reduction waits for the end of the backward (bias_grads_deferred)
        part = _defer_part(nws, x.device)
        S = ctypes.c_int32(0)
        L.call("ldm_conv_backward_weight_defer", byref(desc), x.data_ptr(), dy.data_ptr(), dw.data_ptr(),
               int(accumulate), ctypes.c_void_p(part), code, ctypes.byref(S), stream_handle())
        if S.value > 0:
            _BIAS_DEFER[-1].append(L.WgradRedJob(part, dw.data_ptr(), S.value, dw.numel(), int(accumulate)))
        return dw
    ws = scratch("wgrad", nws, x.device)
    L.call("ldm_conv_backward_weight_dt", byref(desc), x.data_ptr(), dy.data_ptr(), dw.data_ptr(), int(accumulate),
           ws.data_ptr(), code, stream_handle())
    return dw


def act_backward(dy, act, act_out=None, pre_act=None, need_dv=True, need_bias=False, need_bcast=False, db_out=None):
    """(dv, dbias, dbcast) of y = act(v) (+bcast[b,c]) (+skip) for NCHW dy; db_out (contiguous [C]) receives
    dbias in place of a new tensor.  dy and act_out may be 16-bit maps (one 16-bit type); dv is stored like dy."""
    st = T16.get(dy.dtype) or (T16.get(act_out.dtype) if act_out is not None else None) or 0
    dy, dyh = in16(dy, st)
    if act_out is not None:
        act_out, ah = in16(act_out, st)
    else:
        ah = False
    B, C = dy.shape[0], dy.shape[1]
    HW = dy.numel() // max(1, B * C)
    dv = (dy if act == "none" else torch.empty_like(dy)) if need_dv else None
    if db_out is not None:
        assert db_out.is_contiguous() and db_out.numel() == C and db_out.dtype == torch.float32
    db = (db_out if db_out is not None else torch.empty(C, device=dy.device, dtype=torch.float32)) \
        if need_bias else None
    dbc = torch.empty((B, C), device=dy.device, dtype=torch.float32) if need_bcast else None
    if act == "none" and not need_bias and not need_bcast:
        return dv, None, None
    code = L.ACT[act] | st_code(st, x16=ah, dy16=dyh, dx16=dyh and dv is not None)
    if _BIAS_DEFER and need_bias and not need_bcast and HW > 16:
        # the bias gradient's finalize waits for the end of the backward (bias_grads_deferred)
        lib = L.load()
        part = _defer_part(int(lib.ldm_act_partial_floats(B, C, HW)), dy.device)
        q = ctypes.c_int32(0)
        L.call("ldm_act_backward_defer", dy.data_ptr(), _p(act_out), _p(None if pre_act is None else f32c(pre_act)),
               code, B, C, HW, _p(dv) if act != "none" else None, _p(db), ctypes.c_void_p(part),
               ctypes.byref(q), stream_handle())
        if q.value > 0:
            _BIAS_DEFER[-1].append(L.ActFinJob(part, db.data_ptr(), B, C, q.value, 0))
        return dv, db, dbc
    ws = reduce_workspace(B, C, HW, dy.device) if (need_bias or need_bcast) else None
    L.call("ldm_act_backward", dy.data_ptr(), _p(act_out), _p(None if pre_act is None else f32c(pre_act)), code, B,
           C, HW, _p(dv) if act != "none" else None, _p(db), _p(dbc), _p(ws), stream_handle())
    return dv, db, dbc


_BIAS_DEFER = []     # job lists of the open bias_grads_deferred blocks
_DEFER_ARENA = {}    # device -> [chunks, cursor]: the deferred partials' storage, reused step after step


def _defer_part(nfloats, device):
    """Device address of nfloats floats of the deferral arena: chunks allocated on first use and kept (a captured
    step records their addresses; every step takes them in the same order, so the eager warm-up sizes them)."""
    ent = _DEFER_ARENA.setdefault(str(device), {"chunks": [], "ci": 0, "off": 0})
    need = (int(nfloats) + 63) // 64 * 64
    while True:
        if ent["ci"] < len(ent["chunks"]):
            ch = ent["chunks"][ent["ci"]]
            if ent["off"] + need <= ch.numel():
                ptr = ch.data_ptr() + ent["off"] * 4
                ent["off"] += need
                return ptr
            ent["ci"] += 1
            ent["off"] = 0
            continue
        ent["chunks"].append(torch.empty(max(need, 1 << 20), device=device, dtype=torch.float32))


class bias_grads_deferred:
    """with bias_grads_deferred(): loss.backward() -- the convs' bias gradients (ldm_act_backward's per-channel sums,
    and the BatchNorm dx sums that stand for them, batchnorm_backward(dx_sum=True)) are finalized at the end of the
    block, one launch for all of them (ldm_act_finalize_many), and so are the weight gradients' split-K reductions
    (conv_backward_weight: ldm_wgrad_reduce_many), on the current stream
    (which the autograd engine has synchronised with the backward's leaf streams by then).  Only where nothing reads a
    bias gradient before the block ends: LDMTrainer's step without a gradient all-reduce (its post-accumulate hooks
    would read it early).  Bitwise the immediate finalize."""

    def __init__(self, enabled=True):
        self.enabled = bool(enabled)

    def __enter__(self):
        if self.enabled:
            _BIAS_DEFER.append([])
            for ent in _DEFER_ARENA.values():
                ent["ci"], ent["off"] = 0, 0
        return self

    def __exit__(self, *exc):
        if not self.enabled:
            return False
        jobs = _BIAS_DEFER.pop()
        if jobs and exc[0] is None:
            red = [j for j in jobs if isinstance(j, L.WgradRedJob)]
            fin = [j for j in jobs if isinstance(j, L.ActFinJob)]
            if red:
                arr = (L.WgradRedJob * len(red))(*red)
                L.call("ldm_wgrad_reduce_many", ctypes.cast(arr, ctypes.c_void_p), len(red), stream_handle())
            if fin:
                arr = (L.ActFinJob * len(fin))(*fin)
                L.call("ldm_act_finalize_many", ctypes.cast(arr, ctypes.c_void_p), len(fin), stream_handle())
        return False


def reduce_workspace(B, C, HW, device):
    """Scratch for the sliced per-channel reductions (reduce.hip)."""
    return scratch("reduce", L.load().ldm_reduce_workspace_floats(B, C, HW), device)


class _Sync:
    """A resolved SyncBatchNorm target: `pg` is the process group (None = the default group)."""

    def __init__(self, pg):
        self.pg = pg


def _sync_group(group):
    """The group a SyncBatchNorm-marked module reduces over as a _Sync, or None when the statistics stay
    local (sync off, no process group, or a group of one rank).  group=True means the default group.  An
    object with an `ldm_allreduce_sum(t)` method stands in for a process group (it sums t in place over its
    ranks): the captured-step tests simulate a world-2 SyncBatchNorm with one on a single GPU."""
    import torch.distributed as dist
    if hasattr(group, "ldm_allreduce_sum"):
        return _Sync(group)
    if group is False or group is None or not dist.is_available() or not dist.is_initialized():
        return None
    g = None if group is True else group
    return _Sync(g) if dist.get_world_size(g) > 1 else None


def _allreduce_sum(t, group):
    if hasattr(group, "ldm_allreduce_sum"):
        group.ldm_allreduce_sum(t)
        return
    import torch.distributed as dist
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)


def batchnorm_backward(dy, y, x, save_mean, save_invstd, weight, act, need_dx=True, need_w=True, need_b=True,
                       sync=False, bias=None, dx_sum=False):
    """Train-mode BN backward.  sync: SyncBatchNorm over the default group (True) or a given group.  The
    per-rank sums and the per-rank element count travel in ONE fp64 all-reduce of 2C+1 values; the apply
    stage reads the global count on the device (reduce.hip), so there is no host synchronisation.  For act
    none / relu the output y is not read (the ReLU mask is re-evaluated from x, weight and bias)."""
    # 16-bit maps (one 16-bit type): dy, x, y as stored; dx stored like x (the gradient of the BN input)
    st = T16.get(dy.dtype) or T16.get(x.dtype) or 0
    dy, dyh = in16(dy, st)
    x, xh = in16(x, st)
    B, C = dy.shape[0], dy.shape[1]
    HW = max(1, math.prod(dy.shape[2:]))
    dx = torch.empty(dy.shape, device=dy.device, dtype=x.dtype) if need_dx else None
    dw = torch.empty(C, device=dy.device, dtype=torch.float32) if need_w else None
    db = torch.empty(C, device=dy.device, dtype=torch.float32) if need_b else None
    ws = reduce_workspace(B, C, HW, dy.device)
    yh = False
    if act in ("none", "relu"):
        y = None
    elif y is not None:
        y, yh = in16(y, st)
    code = L.ACT[act] | st_code(st, x16=xh, y16=yh, dy16=dyh, dx16=xh and need_dx)
    pg = _sync_group(sync)
    if pg is None:
        if dx_sum and dx is not None:
            # + the per-channel sum of dx (the bias gradient of the conv that produced x), from the apply pass
            # itself: attached to dx for that conv's backward (functional._conv_backward)
            dxs = torch.empty(C, device=dy.device, dtype=torch.float32)
            if _BIAS_DEFER:   # the sum's finalize waits for the end of the backward (bias_grads_deferred)
                lib = L.load()
                part = _defer_part(int(lib.ldm_bn_dxsum_partial_floats(B, C, HW)), dy.device)
                P = ctypes.c_int32(0)
                L.call("ldm_batchnorm_backward_dxsum_defer", dy.data_ptr(), _p(y), x.data_ptr(), save_mean.data_ptr(),
                       save_invstd.data_ptr(), _p(weight), _p(bias), code, B, C, HW, dx.data_ptr(), _p(dw), _p(db),
                       dxs.data_ptr(), ctypes.c_void_p(part), ctypes.byref(P), ws.data_ptr(), stream_handle())
                _BIAS_DEFER[-1].append(L.ActFinJob(part, dxs.data_ptr(), B, C, P.value, 1))
            else:
                L.call("ldm_batchnorm_backward_dxsum", dy.data_ptr(), _p(y), x.data_ptr(), save_mean.data_ptr(),
                       save_invstd.data_ptr(), _p(weight), _p(bias), code, B, C, HW, dx.data_ptr(), _p(dw), _p(db),
                       dxs.data_ptr(), ws.data_ptr(), stream_handle())
            dx._ldm_chan_sum = dxs
            return dx, dw, db
        L.call("ldm_batchnorm_backward", dy.data_ptr(), _p(y), x.data_ptr(), save_mean.data_ptr(),
               save_invstd.data_ptr(), _p(weight), _p(bias), code, B, C, HW, _p(dx), _p(dw), _p(db),
               ws.data_ptr(), stream_handle())
        return dx, dw, db
    # SyncBatchNorm: local sums (+ local count) -> all-reduce -> dx with the global count (parameter
    # grads stay local, as in torch.nn.SyncBatchNorm)
    sums = torch.empty(2 * C + 1, device=dy.device, dtype=torch.float64)
    L.call("ldm_batchnorm_backward_reduce", _p(dy if B else None), _p(y if B else None), _p(x if B else None),
           save_mean.data_ptr(), save_invstd.data_ptr(), _p(weight), _p(bias), code, B, C, HW,
           sums.data_ptr(), _p(dw), _p(db), ws.data_ptr(), stream_handle())
    _allreduce_sum(sums, pg.pg)
    if dx is not None and B:
        L.call("ldm_batchnorm_backward_apply", dy.data_ptr(), _p(y), x.data_ptr(), save_mean.data_ptr(),
               save_invstd.data_ptr(), _p(weight), _p(bias), code, B, C, HW, sums.data_ptr(), -1.0,
               dx.data_ptr(), stream_handle())
    return dx, dw, db


def attention_backward(q, kv, dout, heads):
    q, kv, dout = f32c(q), f32c(kv), f32c(dout)
    B, E, Lq = q.shape
    S = kv.shape[2]
    dq = torch.empty_like(q)
    dkv = torch.empty_like(kv)
    scale = float(math.sqrt(1.0 / float(E // heads)))
    L.call("ldm_attention_backward", q.data_ptr(), kv.data_ptr(), dout.data_ptr(), dq.data_ptr(), dkv.data_ptr(), B, E,
           heads, Lq, S, scale, stream_handle())
    return dq, dkv


def batchnorm_train_(x, weight, bias, running_mean, running_var, momentum, eps, act="none", save=False, sync=False,
                     out=None):
    """Train-mode BatchNorm2d (+activation), in place on x, or from x into `out` when given; updates running
    stats like nn.BatchNorm2d."""
    require_device(x, dtype=None)
    require_device(weight, bias, running_mean, running_var)
    assert x.is_contiguous() and (x.dtype == torch.float32 or x.dtype in T16)
    y = x if out is None else out
    assert y.is_contiguous() and y.shape == x.shape and (y.dtype == torch.float32 or y.dtype in T16)
    st = T16.get(x.dtype) or T16.get(y.dtype) or 0
    assert x.dtype in (torch.float32, TORCH16.get(st)) and y.dtype in (torch.float32, TORCH16.get(st)), \
        "batchnorm: one 16-bit storage type per call"
    B, C, H, W = x.shape
    sm = si = None
    if save:
        sm = torch.empty(C, device=x.device, dtype=torch.float32)
        si = torch.empty(C, device=x.device, dtype=torch.float32)
    ws = reduce_workspace(B, C, H * W, x.device)
    # inside an autocast region the BN output is rounded like the 16-bit output of the reference's BatchNorm on
    # a 16-bit conv output (LDM_ACT_ROUND_*: the activation code's high bits)
    rdt = autocast_out(autocast_dt())
    act_code = L.ACT[act] | (((rdt & 0xff) << 8) if rdt & L.DT_ROUND_OUT else 0) | \
        st_code(st, x16=x.dtype != torch.float32, y16=y.dtype != torch.float32)
    pg = _sync_group(sync)
    if pg is None:
        L.call("ldm_batchnorm_train_out", x.data_ptr(), y.data_ptr(), B, C, H * W, _p(weight), _p(bias),
               _p(running_mean), _p(running_var), float(momentum), float(eps), act_code, _p(sm), _p(si),
               ws.data_ptr(), stream_handle())
    else:
        # SyncBatchNorm (torch.nn.SyncBatchNorm semantics): fp64 (sum x, sum x^2, count) all-reduced over the
        # group in one collective, normalised with the global batch statistics (the global count is read on
        # the device); running stats use the global unbiased variance.  An empty local shard (B == 0) still
        # joins the collective with zero sums and updates its running statistics like every other rank.
        stats = torch.empty(2 * C + 1, device=x.device, dtype=torch.float64)
        xp = x.data_ptr() if B else None
        yp = y.data_ptr() if B else None
        L.call("ldm_batchnorm_stats_code", xp, st_code(st, x16=x.dtype != torch.float32), B, C, H * W,
               stats.data_ptr(), ws.data_ptr(), stream_handle())
        _allreduce_sum(stats, pg.pg)
        L.call("ldm_batchnorm_apply_out", xp, yp, B, C, H * W, stats.data_ptr(), -1.0, _p(weight), _p(bias),
               _p(running_mean), _p(running_var), float(momentum), float(eps), act_code, _p(sm), _p(si),
               stream_handle())
    return (sm, si) if save else None


def activation(x, act, inplace=False):
    require_device(x, dtype=None)   # (a 16-bit map is read through an fp32 copy)
    x = f32c(x)
    y = x if inplace else torch.empty_like(x)
    L.call("ldm_activation", x.data_ptr(), y.data_ptr(), x.numel(), L.ACT[act], stream_handle())
    return y


def batchnorm_eval(x, weight, bias, running_mean, running_var, eps, act="none"):
    require_device(x, dtype=None)
    require_device(weight, bias, running_mean, running_var)
    x = f32c(x)
    y = torch.empty_like(x)
    B, C = x.shape[0], x.shape[1]
    HW = x.numel() // max(1, B * C)
    L.call("ldm_batchnorm_eval", x.data_ptr(), y.data_ptr(), B, C, HW, _p(weight), _p(bias), _p(running_mean),
           _p(running_var), float(eps), L.ACT[act], stream_handle())
    return y


_LOSS_WS = {}


def loss_forward(kind, a, b=None):
    """kind 0: mean((a-b)^2); kind 1: mean(0.5*(a^2-1-log(a^2+1e-8))).  Returns a 0-dim device tensor."""
    require_device(a, b, dtype=None)
    a = f32c(a)
    if b is not None:
        b = f32c(b)
        if b.shape != a.shape:
            raise RuntimeError(f"loss: shape mismatch {tuple(a.shape)} vs {tuple(b.shape)}")
    key = (str(a.device), _stream_key(a.device))
    ws = _LOSS_WS.get(key)
    if ws is None:
        ws = torch.empty(512, device=a.device, dtype=torch.float64)
        _LOSS_WS[key] = ws
    out = torch.empty((), device=a.device, dtype=torch.float32)
    L.call("ldm_loss_forward", kind, a.data_ptr(), _p(b), a.numel(), ws.data_ptr(), out.data_ptr(), stream_handle())
    return out


def loss_backward(kind, a, b, grad_out, need_a=True, need_b=False):
    a = f32c(a)
    b = None if b is None else f32c(b)
    g = f32c(grad_out.reshape(()).to(a.device))
    ga = torch.empty_like(a) if need_a else None
    gb = torch.empty_like(a) if (need_b and b is not None) else None
    L.call("ldm_loss_backward", kind, a.data_ptr(), _p(b), a.numel(), g.data_ptr(), _p(ga), _p(gb), stream_handle())
    return ga, gb


def _t_arg(t, device):
    if not t.is_cuda:
        t = t.to(device)
    t_is_float = 0 if t.dtype in (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8) else 1
    t = t.to(torch.int64 if t_is_float == 0 else torch.float32).reshape(-1).contiguous()
    return t, t_is_float


def sinusoid_embed(t, dim, device):
    t, is_f = _t_arg(t, device)
    out = torch.empty((t.shape[0], dim), device=device, dtype=torch.float32)
    L.call("ldm_sinusoid_embed", t.data_ptr(), is_f, t.shape[0], dim, sinusoid_freqs(dim, device).data_ptr(),
           out.data_ptr(), stream_handle())
    return out


# ------------------------------------------------------------------------------------------------
# time MLP, attention, scheduler
# ------------------------------------------------------------------------------------------------
_FREQ_CACHE = {}


def sinusoid_freqs(dim, device):
    """exp(arange(half) * -(ln(1e4)/(half-1))) computed exactly as model.py:241-243 (host constant)."""
    key = (dim, str(device))
    f = _FREQ_CACHE.get(key)
    if f is None:
        half = dim // 2
        e = math.log(10000) / (half - 1)
        f = torch.exp(torch.arange(half) * -e).to(torch.float32).to(device)
        _FREQ_CACHE[key] = f
    return f


def time_mlp(t, w1, b1, w2, b2):
    require_device(w1, b1, w2, b2)
    dim = w1.shape[0]
    t, t_is_float = _t_arg(t, w1.device)
    out = torch.empty((t.shape[0], dim), device=w1.device, dtype=torch.float32)
    L.call("ldm_time_mlp_forward", t.data_ptr(), t_is_float, t.shape[0], dim, sinusoid_freqs(dim, w1.device).data_ptr(),
           w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(), out.data_ptr(), stream_handle())
    return out


def attention_core(q, kv, heads):
    """q [B,E,L], kv [B,2E,S] -> [B,E,L] (softmax((q*sqrt(1/d))^T k) v per head)."""
    require_device(q, kv, dtype=None)
    q, kv = f32c(q), f32c(kv)
    B, E, Lq = q.shape
    S = kv.shape[2]
    out = torch.empty_like(q)
    scale = float(math.sqrt(1.0 / float(E // heads)))
    L.call("ldm_attention_core", q.data_ptr(), kv.data_ptr(), out.data_ptr(), B, E, heads, Lq, S, scale,
           stream_handle())
    return out


def attention_uses_flash(E, heads, Lq, S):
    """True when the KV-tiled kernels (flash.hip) carry the attention: L or S beyond the LDS-resident
    instances of ldm_attention_core (64 tokens)."""
    return max(Lq, S) > 64 and bool(L.load().ldm_attention_flash_supported(int(E), int(heads)))


def attention_forward_lse(q, kv, heads):
    """q [B,E,L], kv [B,2E,S] -> (out [B,E,L], lse [B,heads,L]) on the KV-tiled online-softmax kernel."""
    require_device(q, kv, dtype=None)
    q, kv = f32c(q), f32c(kv)
    B, E, Lq = q.shape
    S = kv.shape[2]
    out = torch.empty_like(q)
    lse = torch.empty((B, heads, Lq), device=q.device, dtype=torch.float32)
    scale = float(math.sqrt(1.0 / float(E // heads)))
    L.call("ldm_attention_forward_lse", q.data_ptr(), kv.data_ptr(), out.data_ptr(), lse.data_ptr(), B, E, heads, Lq, S,
           scale, stream_handle())
    return out, lse


def attention_backward_flash(q, kv, out, lse, dout, heads):
    q, kv, out, dout = f32c(q), f32c(kv), f32c(out), f32c(dout)
    B, E, Lq = q.shape
    S = kv.shape[2]
    dq = torch.empty_like(q)
    dkv = torch.empty_like(kv)
    delta = torch.empty((B, heads, Lq), device=q.device, dtype=torch.float32)
    scale = float(math.sqrt(1.0 / float(E // heads)))
    L.call("ldm_attention_backward_flash", q.data_ptr(), kv.data_ptr(), out.data_ptr(), lse.data_ptr(), dout.data_ptr(),
           dq.data_ptr(), dkv.data_ptr(), delta.data_ptr(), B, E, heads, Lq, S, scale, stream_handle())
    return dq, dkv


_COEF_CACHE = IdCache()


def alpha_bar_coef_table(alpha_bar, device):
    """[T,2] float32 {sqrt(ab), sqrt(1-ab)} on `device`: the exact fp32 values torch.sqrt gives for the
    reference's expressions (model.py:113, :124, :449-452).  Host constant, cached per buffer version."""
    per = _COEF_CACHE.get(alpha_bar)
    key = (alpha_bar._version, str(device))
    if per is None or per[0] != key:
        ab = alpha_bar.detach().to("cpu", torch.float32)
        tab = torch.stack([torch.sqrt(ab), torch.sqrt(1 - ab)], dim=1).contiguous().to(device)
        per = (key, tab)
        _COEF_CACHE[alpha_bar] = per
    return per[1]


def q_sample(x0, eps, coef_table, t):
    require_device(x0, eps, dtype=None)
    require_device(coef_table)
    t = t.to(x0.device, torch.int64).contiguous()
    x0 = f32c(x0)
    eps = f32c(eps)
    zt = torch.empty_like(x0)
    B = x0.shape[0]
    L.call("ldm_q_sample", x0.data_ptr(), eps.data_ptr(), coef_table.data_ptr(), coef_table.shape[0], t.data_ptr(),
           zt.data_ptr(), B, x0.numel() // B, stream_handle())
    return zt


def predict_start(zt, eps, coef_table, t):
    require_device(zt, eps, dtype=None)
    require_device(coef_table)
    t = t.to(zt.device, torch.int64).contiguous()
    zt = f32c(zt)
    eps = f32c(eps)
    x0 = torch.empty_like(zt)
    B = zt.shape[0]
    L.call("ldm_predict_start", zt.data_ptr(), eps.data_ptr(), coef_table.data_ptr(), coef_table.shape[0],
           t.data_ptr(), x0.data_ptr(), B, zt.numel() // B, stream_handle())
    return x0


def sched_backward(kind, g, coef_table, t, need_a=True, need_b=True):
    g = f32c(g)
    t = t.to(g.device, torch.int64).contiguous()
    ga = torch.empty_like(g) if need_a else None
    gb = torch.empty_like(g) if need_b else None
    B = g.shape[0]
    L.call("ldm_sched_backward", kind, g.data_ptr(), coef_table.data_ptr(), coef_table.shape[0], t.data_ptr(),
           _p(ga), _p(gb), B, g.numel() // B, stream_handle())
    return ga, gb


def ddim_step_(x, eps, coef4, eta, x0_log=None, eps_log=None):
    require_device(x, eps, coef4, x0_log, eps_log)
    L.call("ldm_ddim_step", x.data_ptr(), eps.data_ptr(), coef4.data_ptr(), float(eta), _p(x0_log), _p(eps_log),
           x.numel(), stream_handle())
    return x


# ------------------------------------------------------------------------------------------------
# data formats either side of the path (dataio.hip): 8-bit mel PNG pixels <-> dB, ToTensor
# ------------------------------------------------------------------------------------------------
def mel_quantize(db, max_db=80):
    """uint8 pixels of the reference's mel PNG (audio_processor.py:55-73) from a log-mel dB tensor."""
    require_device(db)
    db = f32c(db)
    out = torch.empty(db.shape, device=db.device, dtype=torch.uint8)
    L.call("ldm_mel_quantize", db.data_ptr(), out.data_ptr(), db.numel(), float(max_db), stream_handle())
    return out


def mel_dequantize(u8, max_db=80):
    """log-mel dB from the 8-bit pixels (audio_processor.py:91-93)."""
    require_device(u8, dtype=torch.uint8)
    if u8.dtype != torch.uint8:
        raise RuntimeError("mel_dequantize: expects uint8 pixels")
    u8 = u8.contiguous()
    out = torch.empty(u8.shape, device=u8.device, dtype=torch.float32)
    L.call("ldm_mel_dequantize", u8.data_ptr(), out.data_ptr(), u8.numel(), float(max_db), stream_handle())
    return out


def u8_to_unit(u8):
    """The [0,1] fp32 tensor torchvision's ToTensor makes of 8-bit pixels (u8 / 255)."""
    require_device(u8, dtype=torch.uint8)
    if u8.dtype != torch.uint8:
        raise RuntimeError("u8_to_unit: expects uint8 pixels")
    u8 = u8.contiguous()
    out = torch.empty(u8.shape, device=u8.device, dtype=torch.float32)
    L.call("ldm_u8_to_unit", u8.data_ptr(), out.data_ptr(), u8.numel(), stream_handle())
    return out


# ---- VGGish feature / style loss pieces (features.hip; reference loss.py:52-101) ---------------------------
def maxpool2x2(x):
    """nn.MaxPool2d(kernel_size=2, stride=2) on NCHW fp32 (floor mode)."""
    require_device(x, dtype=None, what="maxpool2x2")
    x = f32c(x)
    B, C, H, W = x.shape
    y = torch.empty((B, C, H // 2, W // 2), device=x.device, dtype=torch.float32)
    L.call("ldm_maxpool2x2", x.data_ptr(), y.data_ptr(), B, C, H, W, stream_handle())
    return y


def std_mse_accumulate(p, t, acc, scale, eps=1e-8, out=None):
    """acc (fp64 [1], device) += scale * mse(p / (std(p) + eps), t / (std(t) + eps)), std per sample over
    dims 1.. (unbiased, torch.std(dim=[1,2,3])); out (fp32 0-dim, optional) = acc.  One pass over p, t."""
    require_device(p, t, what="std_mse")
    p, t = f32c(p), f32c(t)
    if p.shape != t.shape:
        raise RuntimeError(f"std_mse: shape mismatch {tuple(p.shape)} vs {tuple(t.shape)}")
    B = p.shape[0]
    n = p.numel() // B
    mom = torch.empty((B, 5), device=p.device, dtype=torch.float64)
    ws = scratch("std_mse", L.load().ldm_std_mse_workspace_floats(B, n), p.device)
    L.call("ldm_std_mse_moments", p.data_ptr(), t.data_ptr(), B, n, mom.data_ptr(), ws.data_ptr(), stream_handle())
    L.call("ldm_std_mse_accumulate", mom.data_ptr(), B, n, float(eps), float(scale), acc.data_ptr(), _p(out),
           stream_handle())
    return mom
