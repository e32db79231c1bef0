"""UNet engine: binds a UNet module's parameters to the C ABI's ldm_unet_weights and runs the whole
denoiser (ldm_unet_forward) or the whole reverse loop (ldm_ddim_sample) in one C call each; the
reverse loop is replayed from a captured hipGraph (torch.cuda.CUDAGraph on the same stream).

Host side only: it owns workspaces (torch allocations) and caches, never computes.
"""
import ctypes

import torch

from . import _lib as L
from . import ops

byref = ctypes.byref

_CONV_NAMES = ("enc1", "enc2", "enc3", "enc4", "bottleneck", "dec4", "dec3", "dec2", "dec1")


class UNetEngine:
    """Runs `unet` (a models.model.UNet: reference parameter names / shapes) through libldm_amd."""

    def __init__(self, unet):
        self.unet = unet
        self._bound = {}      # shape key -> (key of param versions, UNetWeights, keepalive)
        self._ws = {}         # (shape key, device) -> workspace tensor
        self._graphs = {}

    # -------------------------------------------------------------------------------------------
    def shape(self, B, C, H, W):
        return L.UNetShape(B, C, H, W, self.unet.num_filters)

    def _params(self):
        u = self.unet
        ps = []
        for n in _CONV_NAMES:
            m = getattr(u, n)
            ps += [m.weight, m.bias]
        for ca in (u.cross_attention2, u.cross_attention1):
            a = ca.multihead_attn
            ps += [a.in_proj_weight, a.in_proj_bias, a.out_proj.weight, a.out_proj.bias]
        tm = u.time_mlp
        ps += [tm[1].weight, tm[1].bias, tm[3].weight, tm[3].bias]
        return ps

    def weights(self, shape):
        """UNetWeights for this shape, re-packing only the parameters whose _version moved."""
        skey = (shape.B, shape.C, shape.H, shape.W, shape.nf)
        params = self._params()
        for p in params:
            ops.require_device(p, what="UNet parameter")
            if not p.is_contiguous():
                raise RuntimeError("UNet parameters must be contiguous")
        vkey = tuple(p._version for p in params) + tuple(p.data_ptr() for p in params) + \
            tuple(sorted(ops._PLAN_OVERRIDE.items()))
        hit = self._bound.get(skey)
        if hit is not None and hit[0] == vkey:
            return hit[1]
        w = L.UNetWeights()
        L.call("ldm_unet_make_plans", byref(shape), byref(w))
        keep = []
        u = self.unet

        def desc(layer):
            d = L.ConvDesc()
            L.call("ldm_unet_layer_desc", byref(shape), layer, byref(d))
            return d

        def bind(layer, weight4d, owner, tag, plan_slot):
            d = desc(layer)
            forced = ops._PLAN_OVERRIDE.get(d.key())
            if forced is not None:
                plan = ops.get_plan(d)
                plan_slot[0] = plan
            else:
                plan = plan_slot[0]
            buf = ops.packed_weight(weight4d, d, plan, owner=owner, tag=tag)
            keep.append(buf)
            return buf.data_ptr()

        for i, n in enumerate(_CONV_NAMES):
            m = getattr(u, n)
            slot = [w.conv_plan[i]]
            w.conv_w[i] = bind(i, m.weight, m.weight, None, slot)
            w.conv_plan[i] = slot[0]
            w.conv_b[i] = m.bias.data_ptr()
        for j, ca in enumerate((u.cross_attention2, u.cross_attention1)):
            a = ca.multihead_attn
            E = a.embed_dim
            ipw, ipb = a.in_proj_weight, a.in_proj_bias
            base = 9 + 3 * j
            slot = [w.ca_plan_q[j]]
            w.ca_wq[j] = bind(base, ipw[:E].view(E, E, 1, 1), ipw, "q", slot)
            w.ca_plan_q[j] = slot[0]
            slot = [w.ca_plan_kv[j]]
            w.ca_wkv[j] = bind(base + 1, ipw[E:].view(2 * E, E, 1, 1), ipw, "kv", slot)
            w.ca_plan_kv[j] = slot[0]
            slot = [w.ca_plan_o[j]]
            w.ca_wo[j] = bind(base + 2, a.out_proj.weight.view(E, E, 1, 1), a.out_proj.weight, "o", slot)
            w.ca_plan_o[j] = slot[0]
            w.ca_bq[j] = ipb.data_ptr()
            w.ca_bkv[j] = ipb.data_ptr() + E * 4
            w.ca_bo[j] = a.out_proj.bias.data_ptr()
        tm = u.time_mlp
        freqs = ops.sinusoid_freqs(tm[1].weight.shape[0], tm[1].weight.device)
        keep.append(freqs)
        w.t_freqs = freqs.data_ptr()
        w.t_w1, w.t_b1 = tm[1].weight.data_ptr(), tm[1].bias.data_ptr()
        w.t_w2, w.t_b2 = tm[3].weight.data_ptr(), tm[3].bias.data_ptr()
        w._keep = keep
        self._bound[skey] = (vkey, w)
        return w

    def workspace(self, shape, device, nsteps=0):
        n = L.load().ldm_ddim_workspace_floats(byref(shape), int(nsteps))
        if n <= 0:
            raise RuntimeError("ldm_ddim_workspace_floats failed")
        key = (shape.B, shape.C, shape.H, shape.W, shape.nf, str(device))
        ws = self._ws.get(key)
        if ws is None or ws.numel() < n:
            ws = torch.empty(int(n), device=device, dtype=torch.float32)
            self._ws[key] = ws
        return ws

    # -------------------------------------------------------------------------------------------
    def forward(self, z, t, s5, s6, out=None):
        ops.require_device(z, s5, s6)
        z, s5, s6 = ops.f32c(z), ops.f32c(s5), ops.f32c(s6)
        B, C, H, W = z.shape
        shape = self.shape(B, C, H, W)
        if tuple(s5.shape) != (B, 256, H // 4, W // 4) or tuple(s6.shape) != (B, 512, H // 8, W // 8):
            raise RuntimeError(f"UNet: style maps must be s5 [B,256,H/4,W/4], s6 [B,512,H/8,W/8] for z {tuple(z.shape)}; "
                               f"got {tuple(s5.shape)}, {tuple(s6.shape)}")
        if t.numel() == 1 and B > 1:
            t = t.reshape(1).expand(B)
        t_dev, t_is_float = ops._t_arg(t, z.device)
        if t_dev.shape[0] != B:
            raise RuntimeError("UNet: t must have one entry per sample")
        w = self.weights(shape)
        ws = self.workspace(shape, z.device)
        y = out if out is not None else torch.empty_like(z)
        L.call("ldm_unet_forward", byref(shape), byref(w), z.data_ptr(), t_dev.data_ptr(), t_is_float, s5.data_ptr(),
               s6.data_ptr(), y.data_ptr(), ws.data_ptr(), ops.stream_handle())
        return y

    def ddim_loop(self, x, s5, s6, t_table, coef_table, eta, x0_logs=None, eps_logs=None):
        """In-place reverse loop on x ([B,C,H,W] contiguous fp32).  t_table [n,B] int64, coef [n,4] (device)."""
        B, C, H, W = x.shape
        shape = self.shape(B, C, H, W)
        w = self.weights(shape)
        n = t_table.shape[0]
        ws = self.workspace(shape, x.device, n)
        L.call("ldm_ddim_sample", byref(shape), byref(w), x.data_ptr(), s5.data_ptr(), s6.data_ptr(),
               t_table.data_ptr(), coef_table.data_ptr(), n, float(eta), ops._p(x0_logs), ops._p(eps_logs),
               ws.data_ptr(), ops.stream_handle())
        return x


class GraphedDDIM:
    """A captured reverse loop with static buffers: replay() re-runs all n steps from x_init."""

    def __init__(self, engine, x_init, s5, s6, t_table, coef_table, eta, logs=True):
        self.engine = engine
        dev = x_init.device
        self.x_init = x_init.contiguous().clone()
        self.x = torch.empty_like(self.x_init)
        self.s5 = s5.contiguous().clone()
        self.s6 = s6.contiguous().clone()
        self.t_table = t_table.to(dev).contiguous()
        self.coef = coef_table.to(dev).contiguous()
        n = self.t_table.shape[0]
        self.x0_logs = torch.empty((n,) + tuple(x_init.shape), device=dev) if logs else None
        self.eps_logs = torch.empty((n,) + tuple(x_init.shape), device=dev) if logs else None
        self.eta = float(eta)
        # warm-up (packs weights, allocates workspace) outside capture
        self.x.copy_(self.x_init)
        engine.ddim_loop(self.x, self.s5, self.s6, self.t_table, self.coef, self.eta, self.x0_logs, self.eps_logs)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.x.copy_(self.x_init)
            engine.ddim_loop(self.x, self.s5, self.s6, self.t_table, self.coef, self.eta, self.x0_logs, self.eps_logs)

    def replay(self):
        self.graph.replay()
        return self.x
