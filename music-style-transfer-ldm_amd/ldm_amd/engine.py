"""UNet engine: binds a UNet module's parameters to the C ABI's ldm_unet_weights and runs the whole
denoiser (ldm_unet_forward) or the whole reverse loop (ldm_ddim_sample) in one C call each; the
reverse loop is replayed from a captured hipGraph (torch.cuda.CUDAGraph on the same stream).

Host side only: it owns workspaces (torch allocations) and caches, never computes.
"""
import ctypes
import os

import torch

from . import _lib as L
from . import ops
from .graphs import capture

byref = ctypes.byref

_CONV_NAMES = ("enc1", "enc2", "enc3", "enc4", "bottleneck", "dec4", "dec3", "dec2", "dec1")


class UNetEngine:
    """Runs `unet` (a models.model.UNet: reference parameter names / shapes) through libldm_amd."""

    def __init__(self, unet, fold=None, step=None, dtype=None):
        self.unet = unet
        # Operand precision of the step kernels (ldm_capi.h LDM_DT_*): None follows the caller's
        # torch.autocast("cuda") region (fp16 / bf16 operands, fp32 accumulation and sampler state) or
        # LDM_AMD_STEP_DTYPE; "fp32" / "fp16" / "bf16" pins it.
        self.dtype = dtype
        # Re-associated cross-attentions in the reverse loop (ldm_capi.h use_fold); LDM_AMD_FOLD=0 turns
        # it off (A/B timing, parity of the literal form).
        self.fold = (os.environ.get("LDM_AMD_FOLD", "1") != "0") if fold is None else bool(fold)
        # Step kernels for the folded reverse loop (ldm_capi.h use_step): 1 or 2 (default, or True) the
        # register-direct kernels (uconv.hip; 2 selected the LDS-staged kernels of rounds 2-5, removed in round 6);
        # 0 conv.hip's general kernel (LDM_AMD_STEP, A/B timing).  Built for the LDM's latent 32 / 64 filters.
        if step is None:
            step = int(os.environ.get("LDM_AMD_STEP", "2"))
        self.step = 2 if step is True else (0 if step is False else int(step))
        if self.step not in (0, 1, 2):
            raise ValueError(f"step must be 0, 1 or 2, got {step!r}")
        self._bound = {}      # shape key -> (key of param versions, UNetWeights, keepalive)
        self._ws = {}         # (shape key, device) -> workspace tensor
        self._graphs = {}

    _DT = {"fp32": 0, "f32": 0, "float32": 0, "fp16": 1, "f16": 1, "float16": 1, "bf16": 2, "bfloat16": 2}

    def step_dtype(self):
        """LDM_DT_* the reverse loop's step kernels run at (see __init__)."""
        if self.dtype is not None:
            return self._DT[str(self.dtype).replace("torch.", "")]
        env = os.environ.get("LDM_AMD_STEP_DTYPE")
        if env:
            return self._DT[env]
        if torch.is_autocast_enabled("cuda"):
            dt = torch.get_autocast_dtype("cuda")
            return 1 if dt == torch.float16 else (2 if dt == torch.bfloat16 else 0)
        return 0

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

    @staticmethod
    def supports(channels):
        """The fused engine keeps the UNet's activations NHWC, which its MFMA conv instances need 8-aligned
        channel counts for (enc1's input, dec1's output); other latent widths (UNet(1, 1) on a raw mel, the
        VAE's default latent_dim=4) run the per-layer path (UNet._layerwise, NCHW kernels)."""
        return channels % 8 == 0 and channels >= 16

    @staticmethod
    def fold_applies(shape):
        """The folded cross-attentions re-associate the scores' contraction from d to E per head: that pays
        while the key count S stays below ~E/3 (the saved Q projection is L*E*E, the extra score work
        (heads-1)*L*S*E), and its LDS-resident instances cover S <= 64 (CA2) / 32 (CA1).  Wider latents (mels
        beyond 512 frames) run the literal loop with the KV-tiled attention (flash.hip)."""
        return shape.H * shape.W <= 1024

    def weights(self, shape):
        """UNetWeights for this shape, re-packing only the parameters whose _version moved."""
        skey = (shape.B, shape.C, shape.H, shape.W, shape.nf)
        params = self._params()
        for p in params:
            ops.require_device(p, what="UNet parameter")
            if not p.is_contiguous():
                raise RuntimeError("UNet parameters must be contiguous")
        vkey = tuple(p._version for p in params) + tuple(p.data_ptr() for p in params) + \
            tuple(sorted(ops._PLAN_OVERRIDE.items())) + (self.fold, self.step, self.step_dtype() if self.step else 0)
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
        folded = {}
        if self.fold and self.fold_applies(shape):
            # enc4 o out_proj(CA2) and bottleneck o out_proj(CA1), packed with those layers' plans
            for j, (layer, conv, ca) in enumerate(((3, u.enc4, u.cross_attention2), (4, u.bottleneck, u.cross_attention1))):
                a = ca.multihead_attn
                d = desc(layer)
                wf = torch.empty_like(conv.weight)
                pb = torch.empty((d.Cout, d.Hout, d.Wout), device=conv.weight.device, dtype=torch.float32)
                L.call("ldm_fold_conv_proj", byref(d), conv.weight.data_ptr(), conv.bias.data_ptr(),
                       a.out_proj.weight.data_ptr(), a.out_proj.bias.data_ptr(), a.embed_dim, wf.data_ptr(),
                       pb.data_ptr(), ops.stream_handle())
                buf = ops.packed_weight(wf, d, w.conv_plan[layer])
                keep += [wf, pb, buf]
                w.fold_w[j] = buf.data_ptr()
                w.fold_pb[j] = pb.data_ptr()
                w.ca_wq_raw[j] = a.in_proj_weight.data_ptr()
                folded[layer] = (wf, pb)
            w.use_fold = 1
            if self.step and shape.C == 32 and shape.nf == 64:
                lib = L.load()
                sdt = self.step_dtype()
                for i, n in enumerate(_CONV_NAMES):
                    src = folded[i][0] if i in folded else getattr(u, n).weight.detach()
                    src = ops.f32c(src)
                    # 16-bit operands read a 16-bit pack (half the floats of storage)
                    nfl = int(lib.ldm_step_packed_floats(i)) // (2 if sdt else 1)
                    buf = torch.empty(nfl, device=src.device, dtype=torch.float32)
                    L.call("ldm_step_pack_weight_dt", i, sdt, src.data_ptr(), buf.data_ptr(), ops.stream_handle())
                    keep += [src, buf]
                    w.step_w[i] = buf.data_ptr()
                for j, layer in enumerate((3, 4)):
                    pbt = folded[layer][1].permute(1, 2, 0).contiguous()     # [Hout, Wout, Cout]
                    keep.append(pbt)
                    w.step_pb[j] = pbt.data_ptr()
                w.use_step = self.step
                w.step_dtype = sdt
                # the bottleneck's fold unpacked: U (CA1's values folded into it) is formed from it once per loop
                w.step_bneck_w = folded[4][0].data_ptr()
        tm = u.time_mlp
        freqs = ops.sinusoid_freqs(tm[1].weight.shape[0], tm[1].weight.device)
        keep.append(freqs)
        w.t_freqs = freqs.data_ptr()
        w.t_w1, w.t_b1 = tm[1].weight.data_ptr(), tm[1].bias.data_ptr()
        w.t_w2, w.t_b2 = tm[3].weight.data_ptr(), tm[3].bias.data_ptr()
        w._keep = keep
        self._bound[skey] = (vkey, w)
        return w

    def workspace(self, shape, device, nsteps=0, slot=0):
        """Workspace for this shape and its bound plans; `slot` separates concurrently running sub-batch
        chains.  Zero-filled on allocation: it carries the split-K tile counters (ldm_capi.h)."""
        w = self.weights(shape)
        n = L.load().ldm_ddim_workspace_floats(byref(shape), byref(w), int(nsteps))
        if n <= 0:
            raise RuntimeError("ldm_ddim_workspace_floats failed")
        key = (shape.B, shape.C, shape.H, shape.W, shape.nf, str(device), slot)
        ws = self._ws.get(key)
        if ws is None or ws.numel() < n:
            ws = torch.zeros(int(n), device=device, dtype=torch.float32)
            self._ws[key] = ws
        return ws

    def side_streams(self, device, k):
        key = ("streams", str(device))
        ss = self._graphs.get(key, [])
        while len(ss) < k:
            ss.append(torch.cuda.Stream(device=device))
        self._graphs[key] = ss
        return ss[:k]

    @staticmethod
    def split_plan(t_table, B, split):
        """[(lo, hi, t_sub)] for `split` contiguous sub-batches; t_sub = t_table[:, lo:hi] made contiguous
        (prepared once, outside any timed / captured region, by GraphedDDIM)."""
        split = max(1, min(int(split), B))
        out = []
        for k in range(split):
            lo, hi = B * k // split, B * (k + 1) // split
            out.append((lo, hi, t_table[:, lo:hi].contiguous()))
        return out

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

    def _ddim_call(self, x, s5, s6, t_table, coef_table, eta, x0_logs, eps_logs, log_stride, slot):
        B, C, H, W = x.shape
        shape = self.shape(B, C, H, W)
        w = self.weights(shape)
        n = t_table.shape[0]
        ws = self.workspace(shape, x.device, n, slot)
        L.call("ldm_ddim_sample", byref(shape), byref(w), x.data_ptr(), s5.data_ptr(), s6.data_ptr(),
               t_table.data_ptr(), coef_table.data_ptr(), n, float(eta), ops._p(x0_logs), ops._p(eps_logs),
               int(log_stride), ws.data_ptr(), ops.stream_handle())

    def ddim_loop(self, x, s5, s6, t_table, coef_table, eta, x0_logs=None, eps_logs=None, split=1, plan=None):
        """In-place reverse loop on x ([B,C,H,W] contiguous fp32).  t_table [n,B] int64, coef [n,4] (device).

        split > 1 runs the batch as that many independent sub-batch chains, each on its own stream
        (forked from and joined back into the current stream, so it also works under graph capture).
        The path is per-sample, so the result is the same up to fp32 summation order (a sub-batch
        size may get a conv plan that splits K differently); the chains' launch and memory latencies
        overlap each other's work."""
        B = x.shape[0]
        if plan is None:
            plan = self.split_plan(t_table, B, split) if split > 1 else None
        if not plan or len(plan) == 1:
            self._ddim_call(x, s5, s6, t_table, coef_table, eta, x0_logs, eps_logs, 0, 0)
            return x
        per_step = x[0].numel() * B
        main = torch.cuda.current_stream(x.device)
        streams = self.side_streams(x.device, len(plan))
        C, H, W = x.shape[1:]
        for k, (lo, hi, t_sub) in enumerate(plan):   # bind / pack / allocate on the main stream first
            shape = self.shape(hi - lo, C, H, W)
            self.weights(shape)
            self.workspace(shape, x.device, t_table.shape[0], k)
        for k, (lo, hi, t_sub) in enumerate(plan):
            st = streams[k]
            st.wait_stream(main)
            if not torch.cuda.is_current_stream_capturing():
                t_sub.record_stream(st)
            with torch.cuda.stream(st):
                self._ddim_call(x[lo:hi], s5[lo:hi], s6[lo:hi], t_sub, coef_table, eta,
                                None if x0_logs is None else x0_logs[0, lo:hi],
                                None if eps_logs is None else eps_logs[0, lo:hi], per_step, k)
        for st in streams:
            main.wait_stream(st)
        return x


class GraphedDDIM:
    """A captured reverse loop with static buffers: replay() re-runs all n steps from x_init."""

    def __init__(self, engine, x_init, s5, s6, t_table, coef_table, eta, logs=True, split=1):
        self.engine = engine
        self.split = split
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
        # static sub-batch timestep tables, made once outside the captured region
        self.plan = engine.split_plan(self.t_table, x_init.shape[0], split) if split > 1 else None
        # warm-up (packs weights, allocates workspaces) outside capture
        self.x.copy_(self.x_init)
        self.engine.ddim_loop(self.x, self.s5, self.s6, self.t_table, self.coef, self.eta, self.x0_logs,
                              self.eps_logs, plan=self.plan)
        torch.cuda.synchronize()
        if not self.plan:
            self.graphs = [torch.cuda.CUDAGraph()]
            self.streams = None
            with capture(self.graphs[0]):
                self.x.copy_(self.x_init)
                self.engine.ddim_loop(self.x, self.s5, self.s6, self.t_table, self.coef, self.eta, self.x0_logs,
                                      self.eps_logs)
            return
        # One graph per sub-batch chain, each replayed on its own stream: a single graph's parallel
        # branches are executed one after another, separate graphs on separate streams (hardware
        # queues) run concurrently.
        self.streams = engine.side_streams(dev, len(self.plan))
        self.graphs = []
        per_step = self.x[0].numel() * self.x.shape[0]
        for k, (lo, hi, t_sub) in enumerate(self.plan):
            g = torch.cuda.CUDAGraph()
            with capture(g, stream=self.streams[k]):
                self.x[lo:hi].copy_(self.x_init[lo:hi])
                engine._ddim_call(self.x[lo:hi], self.s5[lo:hi], self.s6[lo:hi], t_sub, self.coef, self.eta,
                                  None if self.x0_logs is None else self.x0_logs[0, lo:hi],
                                  None if self.eps_logs is None else self.eps_logs[0, lo:hi], per_step, k)
            self.graphs.append(g)

    def replay(self):
        if self.streams is None:
            self.graphs[0].replay()
            return self.x
        main = torch.cuda.current_stream()
        for st, g in zip(self.streams, self.graphs):
            st.wait_stream(main)
            with torch.cuda.stream(st):
                g.replay()
        for st in self.streams:
            main.wait_stream(st)
        return self.x
