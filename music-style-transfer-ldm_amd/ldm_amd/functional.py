"""Autograd-aware functional layer over ops.py.

Every function here computes on the HIP path.  When autograd needs a graph (grad mode on and an input
requires grad) the call is wrapped in a torch.autograd.Function whose backward runs the matching HIP
backward kernels (ldm_amd.backward); a missing backward raises instead of silently detaching.
"""
import contextlib
import os

import torch

from . import _lib as L
from . import ops

_BACKWARD = {}   # name -> callable(ctx, *grad_outputs) registered by ldm_amd.backward
STATS = {"conv_bias_from_bn": 0}   # conv backwards that took their bias gradient from the BN's dx sum (tests)


def register_backward(name):
    def deco(fn):
        _BACKWARD[name] = fn
        return fn
    return deco


def _needs_grad(*ts):
    if not torch.is_grad_enabled():
        return False
    return any(isinstance(t, torch.Tensor) and t.requires_grad for t in ts)


class _HipOp(torch.autograd.Function):
    """Generic wrapper: forward = fwd(ctx_dict, *tensors); backward dispatched by name."""

    @staticmethod
    def forward(ctx, name, fwd, nin, *args):
        tensors = args[:nin]
        store = {"grad": True}
        out = fwd(store, *tensors)
        ctx.name = name
        ctx.store = store
        ctx.nin = nin
        saved = store.pop("saved", ())
        ctx.save_for_backward(*saved)
        return out

    @staticmethod
    def backward(ctx, *grads):
        fn = _BACKWARD.get(ctx.name)
        if fn is None:
            raise NotImplementedError(f"music-style-transfer-ldm_amd: backward of '{ctx.name}' has no HIP kernel yet")
        gin = fn(ctx, *grads)
        return (None, None, None) + tuple(gin)


def hip_apply(name, fwd, *tensors):
    """Run fwd(store, *tensors) on the HIP path; build an autograd node only if needed."""
    if _needs_grad(*tensors):
        return _HipOp.apply(name, fwd, len(tensors), *tensors)
    return fwd({"grad": False}, *tensors)


# ------------------------------------------------------------------------------------------------
def _conv_desc(x, w, cfg):
    if cfg["transposed"]:
        cout, kh, kw = w.shape[1], w.shape[2], w.shape[3]
    else:
        cout, kh, kw = w.shape[0], w.shape[2], w.shape[3]
    return ops.make_desc(x.shape[0], x.shape[1], x.shape[2], x.shape[3], cout, kh, kw, cfg["stride"],
                         cfg["padding"], cfg["output_padding"], cfg["transposed"])


def conv(x, weight, bias, *, stride, padding, transposed=False, output_padding=0, act="none", bcast=None,
         skip=None, bn_eval=None, wkey=None):
    """act(BN_eval(conv(x,w)+b)) + bcast + skip, differentiable in x, weight, bias, bcast, skip.

    wkey = (owner_parameter, tag) caches the packed weight of a parameter slice against the parameter."""
    cfg = dict(stride=stride, padding=padding, transposed=transposed, output_padding=output_padding, act=act)

    def fwd(store, x_, w_, b_, bc_, sk_):
        aout = None
        if store["grad"] and act != "none" and (bc_ is not None or sk_ is not None):
            d = _conv_desc(x_, w_, cfg)
            aout = torch.empty((d.B, d.Cout, d.Hout, d.Wout), device=x_.device, dtype=torch.float32)
        dt = ops.autocast_dt()
        # the large maps of an autocast region stored in 16 bits, as ATen's (ops.store16_dtype)
        d = _conv_desc(x_, w_, cfg)
        odt = ops.store16_dtype(d.B * d.Cout * d.Hout * d.Wout, dt)
        y = ops.conv_forward(x_, w_, b_, bn=bn_eval, bcast=bc_, skip=sk_, wkey=wkey, act_out=aout, dtype=dt,
                             out_dtype=odt, **cfg)
        store["dtype"] = dt      # the backward convs run at the forward's autocast precision
        store["round"] = bool(ops.autocast_out(dt) & L.DT_ROUND_OUT)   # ... and output semantics
        store["cfg"] = cfg
        store["bn"] = bn_eval
        store["wkey"] = wkey
        store["saved"] = (x_, w_, y if aout is None else aout)
        store["bc_shape"] = None if bc_ is None else bc_.shape
        return y

    return hip_apply("conv", fwd, x, weight, bias, bcast, skip)


@register_backward("conv")
def _conv_backward(ctx, gy):
    """conv/convT backward: epilogue (act, bias, bcast, skip, eval-BN scale) -> dgrad on the dual
    descriptor -> wgrad (fixed-order split-K)."""
    x, w, a = ctx.saved_tensors
    cfg, bn = ctx.store["cfg"], ctx.store["bn"]
    nx, nw, nb, nbc, nsk = ctx.needs_input_grad[3:8]
    act = cfg["act"]
    if act == "gelu":
        raise NotImplementedError("conv backward with a fused GELU epilogue (apply GELU as its own op)")
    # a train-mode BatchNorm's backward (its input is this conv's output) may have summed the gradient per channel
    # as it wrote it (ops.batchnorm_backward dx_sum): that sum IS this conv's bias gradient
    chan_sum = getattr(gy, "_ldm_chan_sum", None)
    gy = gy.contiguous()   # (a 16-bit map's gradient stays 16-bit: the kernels below read it as stored)
    need_v = nx or nw or nb
    if act == "none" and bn is None and not nbc and chan_sum is not None:
        gv, gb, gbc = gy, (chan_sum if nb else None), None
        STATS["conv_bias_from_bn"] += 1
    else:
        gv, gb, gbc = ops.act_backward(gy, act, act_out=a, need_dv=need_v, need_bias=nb and bn is None,
                                       need_bcast=nbc)
    if bn is not None and need_v:
        g_, _b, _m, var, eps = bn
        zero = torch.zeros_like(var)
        gv = ops.batchnorm_eval(gv, g_, zero, zero, var, eps, "none")     # gv * gamma * invstd
        if nb:
            _, gb, _ = ops.act_backward(gv, "none", need_dv=False, need_bias=True)
    desc = _conv_desc(x, w, cfg)
    dt = ctx.store.get("dtype", 0)
    gx = ops.conv_backward_data(gv, w, desc, ctx.store["wkey"], dtype=dt, round_out=ctx.store.get("round", False),
                                out_dtype=x.dtype) if nx else None
    gw = ops.conv_backward_weight(x, gv, desc, dtype=dt) if nw else None
    if gbc is not None:
        gbc = gbc.reshape(ctx.store["bc_shape"])
    return gx, gw, gb, gbc, (gy if nsk else None)


def in_proj(q_nchw, kv_nchw, ipw, ipb):
    """(Wq q + bq, Wkv kv + bkv) of nn.MultiheadAttention's packed in-projection (in_proj_weight [3E, E],
    rows q | k | v) as two 1x1 convs under ONE autograd node: its backward writes the two row blocks of
    dW and db straight into one [3E, E] / [3E] gradient (per-slice nodes would zero-fill, copy and add
    the full tensor twice per call)."""
    E = ipw.shape[1]

    def fwd(store, q_, kv_, w_, b_):
        dt = ops.autocast_dt()
        wq, wkv = w_[:E].view(E, E, 1, 1), w_[E:].view(2 * E, E, 1, 1)
        q = ops.conv_forward(q_, wq, b_[:E], stride=1, padding=0, wkey=(ipw, "q"), dtype=dt)
        kv = ops.conv_forward(kv_, wkv, b_[E:], stride=1, padding=0, wkey=(ipw, "kv"), dtype=dt)
        store["dtype"] = dt
        store["round"] = bool(ops.autocast_out(dt) & L.DT_ROUND_OUT)
        store["owner"] = ipw        # the packed-weight caches are keyed on the parameter itself
        store["saved"] = (q_, kv_, w_)
        return q, kv

    return hip_apply("in_proj", fwd, q_nchw, kv_nchw, ipw, ipb)


@register_backward("in_proj")
def _in_proj_backward(ctx, gq, gkv):
    q_in, kv_in, w = ctx.saved_tensors
    nq, nkv, nw, nb = ctx.needs_input_grad[3:7]
    E = w.shape[1]
    dt, owner = ctx.store["dtype"], ctx.store["owner"]
    gw = torch.empty_like(w) if nw else None
    gb = torch.empty((3 * E,), device=w.device, dtype=torch.float32) if nb else None
    grads = []
    for x, g, lo, hi, tag, nx in ((q_in, gq, 0, E, "q", nq), (kv_in, gkv, E, 3 * E, "kv", nkv)):
        g = ops.f32c(g)
        desc = _conv_desc(x, w[lo:hi].view(hi - lo, E, 1, 1), dict(transposed=False, stride=1, padding=0,
                                                                  output_padding=0))
        if nb:
            ops.act_backward(g, "none", need_dv=False, need_bias=True, db_out=gb[lo:hi])
        grads.append(ops.conv_backward_data(g, w[lo:hi].view(hi - lo, E, 1, 1), desc, (owner, tag), dtype=dt,
                                            round_out=ctx.store.get("round", False)) if nx else None)
        if nw:
            ops.conv_backward_weight(x, g, desc, dw=gw[lo:hi].view(hi - lo, E, 1, 1), dtype=dt)
    return grads[0], grads[1], gw, gb


def linear(x, weight, bias, act="none"):
    """y = act(x W^T + b) for x [..., in]: a 1x1 conv over N = prod(leading dims) 'pixels'."""
    lead = x.shape[:-1]
    n = 1
    for s in lead:
        n *= s
    x4 = x.reshape(n, x.shape[-1], 1, 1)
    y = conv(x4, weight.view(weight.shape[0], weight.shape[1], 1, 1), bias, stride=1, padding=0, act=act,
             wkey=(weight, "lin"))     # pack cached against the parameter, not against this step's view
    return y.reshape(*lead, weight.shape[0])


def activation(x, act):
    def fwd(store, x_):
        y = ops.activation(x_, act)
        store["act"] = act
        store["saved"] = (x_, y)
        return y

    return hip_apply("activation", fwd, x)


def _as_nc(t):
    """[N, C, ...] view for the per-channel kernels (a 1-D tensor is one channel)."""
    if t.dim() >= 2:
        return t.reshape(t.shape[0], t.shape[1], -1)
    return t.reshape(1, 1, -1)


@register_backward("activation")
def _activation_backward(ctx, gy):
    x, y = ctx.saved_tensors
    act = ctx.store["act"]
    dv, _, _ = ops.act_backward(_as_nc(ops.f32c(gy)), act, act_out=_as_nc(y),
                                pre_act=_as_nc(ops.f32c(x)) if act == "gelu" else None)
    return (dv.reshape(x.shape),)


_SYNC_OVERRIDE = []   # stack of group overrides pushed by ldm_amd.dist.batchnorm_sync


def sync_group_for(m):
    """SyncBatchNorm group of module m: the innermost batchnorm_sync(...) override, else the module's mark
    (convert_sync_batchnorm), else False (local statistics)."""
    if _SYNC_OVERRIDE:
        return _SYNC_OVERRIDE[-1]
    return getattr(m, "ldm_sync_group", False)


_BN_COUNT_DEFER = []   # stack of lists collecting num_batches_tracked counters (bn_counts_deferred)


@contextlib.contextmanager
def bn_counts_deferred():
    """Within the block, training-mode BatchNorms with a momentum collect their num_batches_tracked counters
    instead of bumping each with its own one-element add kernel; on exit they are all bumped by one
    torch._foreach_add_ (the train step's five BN layers: 5 launches -> 1).  The counters are read only by the
    cumulative-average form (momentum None), which keeps the immediate add."""
    _BN_COUNT_DEFER.append([])
    try:
        yield
    finally:
        counters = _BN_COUNT_DEFER.pop()
        if counters:
            torch._foreach_add_(counters, 1)


def batchnorm(x, bn_module, act="none"):
    """nn.BatchNorm2d semantics (train: batch stats + running update; eval: running stats) + act."""
    m = bn_module
    use_batch = m.training or not m.track_running_stats
    if not use_batch:
        def fwd_eval(store, x_, w_, b_):
            y = ops.batchnorm_eval(x_, w_, b_, m.running_mean, m.running_var, m.eps, act)
            store["saved"] = (x_, w_, y)
            store["bn"] = (m.running_mean, m.running_var, m.eps, act)
            return y
        return hip_apply("batchnorm_eval", fwd_eval, x, m.weight, m.bias)

    momentum = m.momentum
    if m.training and m.track_running_stats:
        if momentum is None:
            m.num_batches_tracked.add_(1)
            momentum = 1.0 / float(m.num_batches_tracked.item())
        elif _BN_COUNT_DEFER:
            _BN_COUNT_DEFER[-1].append(m.num_batches_tracked)   # bumped by the enclosing bn_counts_deferred()
        else:
            m.num_batches_tracked.add_(1)
    rm = m.running_mean if (m.training and m.track_running_stats) else None
    rv = m.running_var if (m.training and m.track_running_stats) else None

    # SyncBatchNorm only for a module in training mode (torch.nn.SyncBatchNorm semantics: eval-mode use of
    # batch statistics, track_running_stats=False, stays local); the group comes from
    # ldm_amd.dist.convert_sync_batchnorm or an enclosing ldm_amd.dist.batchnorm_sync(...) block.
    sync = sync_group_for(m) if m.training else False

    def fwd_train(store, x_, w_, b_):
        # a 16-bit input map (16-bit storage) gives a 16-bit output, as ATen's BatchNorm under autocast
        xc = x_.contiguous() if x_.dtype in ops.T16 else ops.f32c(x_)
        y = torch.empty_like(xc)
        sm, si = ops.batchnorm_train_(xc, w_, b_, rm, rv, momentum if momentum is not None else 0.0, m.eps,
                                      act, save=True, sync=sync, out=y)
        store["saved"] = (x_, w_, b_, sm, si, y)
        store["act"] = act
        store["sync"] = sync
        return y

    return hip_apply("batchnorm_train", fwd_train, x, m.weight, m.bias)


@register_backward("batchnorm_train")
def _bn_train_backward(ctx, gy):
    x, w, b, sm, si, y = ctx.saved_tensors
    nx, nw, nb = ctx.needs_input_grad[3:6]
    dx, dw, db = ops.batchnorm_backward(gy, y, x, sm, si, w, ctx.store["act"], need_dx=nx,
                                        need_w=nw and w is not None, need_b=nb and b is not None,
                                        sync=ctx.store.get("sync", False), bias=b,
                                        dx_sum=os.environ.get("LDM_AMD_BN_DXSUM", "1") != "0")
    return dx, dw, db


def time_mlp(t, w1, b1, w2, b2):
    def fwd(store, w1_, b1_, w2_, b2_):
        return ops.time_mlp(t, w1_, b1_, w2_, b2_)

    return hip_apply("time_mlp", fwd, w1, b1, w2, b2)


def q_sample(x0, eps, coef_table, t):
    def fwd(store, x0_, eps_):
        store["sched"] = (coef_table, t)
        return ops.q_sample(x0_, eps_, coef_table, t)

    return hip_apply("q_sample", fwd, x0, eps)


def predict_start(zt, eps, coef_table, t):
    def fwd(store, zt_, eps_):
        store["sched"] = (coef_table, t)
        return ops.predict_start(zt_, eps_, coef_table, t)

    return hip_apply("predict_start", fwd, zt, eps)


def _sched_bw(kind):
    def bw(ctx, g):
        tab, t = ctx.store["sched"]
        return ops.sched_backward(kind, g, tab, t, ctx.needs_input_grad[3], ctx.needs_input_grad[4])
    return bw


register_backward("q_sample")(_sched_bw(0))
register_backward("predict_start")(_sched_bw(1))


def mse_loss(a, b):
    def fwd(store, a_, b_):
        store["saved"] = (a_, b_)
        return ops.loss_forward(0, a_, b_)

    return hip_apply("mse_loss", fwd, a, b)


def kl_loss(z):
    def fwd(store, z_):
        store["saved"] = (z_,)
        return ops.loss_forward(1, z_)

    return hip_apply("kl_loss", fwd, z)


@register_backward("mse_loss")
def _mse_backward(ctx, g):
    a, b = ctx.saved_tensors
    ga, gb = ops.loss_backward(0, a, b, g, ctx.needs_input_grad[3], ctx.needs_input_grad[4])
    return ga, gb


@register_backward("kl_loss")
def _kl_backward(ctx, g):
    (z,) = ctx.saved_tensors
    gz, _ = ops.loss_backward(1, z, None, g, True, False)
    return (gz,)


def attention_core(q, kv, heads):
    def fwd(store, q_, kv_):
        store["heads"] = heads
        if store["grad"] and ops.attention_uses_flash(q_.shape[1], heads, q_.shape[2], kv_.shape[2]):
            # wide maps: the KV-tiled kernels, whose backward needs the output and the per-query log-sum-exp
            out, lse = ops.attention_forward_lse(q_, kv_, heads)
            store["saved"] = (q_, kv_, out, lse)
            return out
        out = ops.attention_core(q_, kv_, heads)
        store["saved"] = (q_, kv_)
        return out

    return hip_apply("attention_core", fwd, q, kv)


@register_backward("attention_core")
def _attention_backward(ctx, gout):
    saved = ctx.saved_tensors
    if len(saved) == 4:
        q, kv, out, lse = saved
        return ops.attention_backward_flash(q, kv, out, lse, gout, ctx.store["heads"])
    q, kv = saved
    dq, dkv = ops.attention_backward(q, kv, gout, ctx.store["heads"])
    return dq, dkv
