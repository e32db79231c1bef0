"""Per-phase timeline of the conv kernel from a diagnostic build (-DLDM_DIAG=4): block entry / end
wall clock (s_memrealtime, 100 MHz) and shader-clock stamps (s_memtime) after the prologue, after the
K loop and after the split-K LDS barrier.  Runs every UNet layer once at config-2 shape.

    LDM_AMD_LIB=.../libldm_amd_diag4.so python tools/stamp_probe.py
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "music-style-transfer-ldm_amd"))

import torch  # noqa: E402
from ldm_amd import _lib as L  # noqa: E402


def main():
    import models.model as M
    dev = torch.device("cuda:0")
    ldm = M.LDM(32, pretrained_path="").to(dev).eval()
    eng = M.engine_for(ldm.unet)
    shape = eng.shape(8, 32, 16, 64)
    w = eng.weights(shape)
    lib = L.load()
    lib.ldm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    names = ["enc1", "enc2", "enc3", "enc4", "bottleneck", "dec4", "dec3", "dec2", "dec1",
             "ca2.q", "ca2.kv", "ca2.out", "ca1.q", "ca1.kv", "ca1.out"]
    plans = list(w.conv_plan) + [w.ca_plan_q[0], w.ca_plan_kv[0], w.ca_plan_o[0],
                                 w.ca_plan_q[1], w.ca_plan_kv[1], w.ca_plan_o[1]]
    wptr = list(w.conv_w) + [w.ca_wq[0], w.ca_wkv[0], w.ca_wo[0], w.ca_wq[1], w.ca_wkv[1], w.ca_wo[1]]
    bptr = list(w.conv_b) + [w.ca_bq[0], w.ca_bkv[0], w.ca_bo[0], w.ca_bq[1], w.ca_bkv[1], w.ca_bo[1]]
    st = torch.cuda.current_stream()
    print(f"{'layer':12s} {'plan':10s} {'blocks':>6s} {'wall_us':>8s} {'skew_us':>8s} {'blk_us':>7s} "
          f"{'pre_us':>7s} {'ld0+epi':>8s} {'loop_cyc':>9s} {'red_cyc':>8s} {'clk_GHz':>7s} {'mfma/w':>6s}")
    for i, name in enumerate(names):
        d = L.ConvDesc()
        L.call("ldm_unet_layer_desc", ctypes.byref(shape), i, ctypes.byref(d))
        x = torch.randn(d.B, d.Cin, d.Hin, d.Win, device=dev)
        y = torch.empty(d.B, d.Cout, d.Hout, d.Wout, device=dev)
        ep = L.Epilogue()
        ep.bias = bptr[i]
        ep.act = 1 if i < 8 else 0
        plan = plans[i]
        ws = torch.zeros(max(1, int(plan.ws_floats)), device=dev)
        args = (ctypes.byref(d), ctypes.byref(plan), x.data_ptr(), wptr[i], ctypes.byref(ep), y.data_ptr(),
                ws.data_ptr(), st.cuda_stream)
        for _ in range(5):
            L.check(lib.ldm_conv_forward_ws(*args), name)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        L.check(lib.ldm_conv_forward_ws(*args), name)
        e1.record(st)
        torch.cuda.synchronize()
        if plan.kind == 0:
            print(f"{name:12s} direct  {e0.elapsed_time(e1) * 1e3:8.2f}")
            continue
        tile = 32 if plan.kind == 1 else 16
        bm, bn = tile * plan.tm, tile * plan.tn
        nph = 4 if d.transposed and d.stride == 2 else 1
        nq = d.B * (d.Hin * d.Win if nph == 4 else d.Hout * d.Wout)
        nblk = ((nq + bn - 1) // bn) * ((d.Cout + bm - 1) // bm) * nph * plan.ks
        buf = np.zeros((nblk, 6), dtype=np.uint64)
        assert lib.ldm_debug_stamps(buf.ctypes.data, nblk) == 0
        rt0, rt5 = buf[:, 0].astype(np.float64), buf[:, 5].astype(np.float64)
        c1, c2, c3, c4 = (buf[:, k].astype(np.float64) for k in (1, 2, 3, 4))
        blk_us = (rt5 - rt0) * 0.01
        clk = 2.1   # GHz, measured 1.9-2.2 under this load (s_memtime vs s_memrealtime)
        # MFMAs per wave (ideal): chunks of the slowest phase / wk, x 4 x tm x tn
        taps = d.kh * d.kw if nph == 1 else max(1, (d.kh * d.kw + 3) // 4)
        ck = 8 if plan.kind == 1 else 16
        mf = -(-(taps * d.Cin // ck) // (plan.wk * plan.ks)) * 4 * plan.tm * plan.tn
        post = (c4 - c1) / (clk * 1e3)
        print(f"{name:12s} {str(plan.key()):10s} {nblk:6d} "
              f"{e0.elapsed_time(e1) * 1e3:8.2f} {(rt0.max() - rt0.min()) * 0.01:8.2f} {np.median(blk_us):7.2f} "
              f"{np.median(blk_us - post):7.2f} {np.median(c2 - c1):8.0f} {np.median(c3 - c2):9.0f} "
              f"{np.median(c4 - c3):8.0f} {clk:7.2f} {mf:6d}")


if __name__ == "__main__":
    main()
