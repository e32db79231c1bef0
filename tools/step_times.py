"""Per-layer graph-timed durations of the step kernels (csrc/uconv.hip) at the sampling shape, and the
whole 49-iteration reverse loop with the step kernels on and off.

    python tools/step_times.py [--shape 8x16x64] [--reps 50]
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "music-style-transfer-ldm_amd"))

import torch  # noqa: E402

LAYERS = [(32, 64, 0), (64, 128, 1), (128, 256, 1), (256, 512, 1), (512, 512, 0), (512, 256, 2), (256, 128, 2),
          (128, 64, 2), (64, 32, 0)]
DIV = [1, 1, 2, 4, 8, 8, 4, 2, 1]
NAMES = ["enc1", "enc2", "enc3", "enc4", "bottleneck", "dec4", "dec3", "dec2"]


def graph_us(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    g.replay()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="8x16x64")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--stamps", action="store_true", help="per-block phase stamps (needs a UCONV_DIAG=4 build, tools/step_diag.sh)")
    ap.add_argument("--no-loop", action="store_true")
    ap.add_argument("--layers", default=None, help="comma list of layer indices (default all)")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "fp16", "bf16"],
                    help="operand precision of the step kernels (config 5: fp16)")
    ap.add_argument("--loop-only", default=None, help="comma list of use_step values: only time the loop")
    args = ap.parse_args()
    B, H, W = (int(v) for v in args.shape.split("x"))
    from ldm_amd import _lib as L
    dev = torch.device("cuda:0")
    lib = L.load()
    tot = 0.0
    sel = None if args.layers is None else {int(v) for v in args.layers.split(",")}
    for layer, name in enumerate(NAMES if args.loop_only is None else []):
        if sel is not None and layer not in sel:
            continue
        Cin, Cout, mode = LAYERS[layer]
        Hin, Win = H // DIV[layer], W // DIV[layer]
        Hout, Wout = (Hin, Win) if mode == 0 else ((Hin // 2, Win // 2) if mode == 1 else (2 * Hin, 2 * Win))
        x = torch.randn(B, Hin, Win, Cin, device=dev)
        w = torch.randn((Cin, Cout, 3, 3) if mode == 2 else (Cout, Cin, 3, 3), device=dev) * 0.05
        packed = torch.empty(int(lib.ldm_step_packed_floats(layer)), device=dev)
        dt = {"fp32": 0, "fp16": 1, "bf16": 2}[args.dtype]
        L.call("ldm_step_pack_weight_dt", layer, dt, w.data_ptr(), packed.data_ptr(), torch.cuda.current_stream().cuda_stream)
        bias = torch.randn((Hout * Wout * Cout) if layer in (3, 4) else Cout, device=dev)
        bc = torch.randn(B, Cout, device=dev)
        sk = torch.randn(B, Hout, Wout, Cout, device=dev)
        y = torch.empty(B, Hout, Wout, Cout, device=dev)

        # the split-K forms run with a workspace, as the loop runs them (ldm_step_layer_forms)
        nws = int(lib.ldm_step_workspace_floats(B, H, W))
        ws = torch.zeros(max(nws, 1), device=dev)

        def run():
            bcp = bc.data_ptr() if layer == 1 else None
            skp = sk.data_ptr() if mode == 2 else None
            stp = torch.cuda.current_stream().cuda_stream
            rc = lib.ldm_step_conv_ws(layer, B, H, W, x.data_ptr(), packed.data_ptr(), bias.data_ptr(), bcp, skp,
                                      y.data_ptr(), dt, ws.data_ptr(), stp)
            assert rc == 0

        us = graph_us(run, args.reps)
        fl = 2.0 * B * Cout * Hout * Wout * Cin * (9 if mode < 2 else 2.25)
        tot += us
        extra = ""
        if args.stamps:
            import numpy as np
            lib.ldm_debug_uconv_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
            graph_us(run, 10)          # stamps of the last launch of a 10-launch graph chain (warm)
            torch.cuda.synchronize()
            buf = np.zeros((4096, 5), dtype=np.uint64)
            assert lib.ldm_debug_uconv_stamps(buf.ctypes.data, 4096) == 0
            nb = int((buf[:, 0] > 0).sum())
            b = buf[:nb].astype(np.float64)
            clk = 2.1e3   # cycles per us (s_memtime), nominal under load
            blk = (b[:, 4] - b[:, 0]) * 0.01
            loop = (b[:, 2] - b[:, 1]) / clk
            red = (b[:, 3] - b[:, 2]) / clk
            span = (b[:, 4].max() - b[:, 0].min()) * 0.01
            skew = (b[:, 0].max() - b[:, 0].min()) * 0.01
            st0 = (b[:, 0] - b[:, 0].min()) * 0.01
            pct = np.percentile(st0, [10, 50, 90])
            extra = (f" | blocks {nb} span {span:5.2f} start p10/50/90 {pct[0]:4.2f}/{pct[1]:4.2f}/{pct[2]:4.2f} "
                     f"skew {skew:5.2f} blk {np.median(blk):5.2f} "
                     f"(max {blk.max():5.2f}) loop {np.median(loop):5.2f} red {np.median(red):5.2f} "
                     f"other {np.median(blk - loop - red):5.2f} us")
        print(f"{name:12s} {us:8.2f} us {fl / us / 1e6:8.1f} TF/s{extra}", flush=True)
    print(f"{'sum(8)':12s} {tot:8.2f} us", os.environ.get("LDM_AMD_LIB", ""))
    if args.no_loop:
        return

    import models.model as M
    from ldm_amd.engine import GraphedDDIM, UNetEngine
    torch.manual_seed(0)
    ldm = M.LDM(32, pretrained_path="").to(dev).eval()
    g = torch.Generator().manual_seed(1)
    style = torch.rand(B, 1, 8 * H, 8 * W, generator=g).to(dev)
    z = torch.randn((B, 32, H, W), generator=g).to(dev)
    times = torch.linspace(199, 0, 50).long()
    coefs = ldm.noise_scheduler.reverse_coefs(times).to(dev)
    tt = times[:-1].view(-1, 1).expand(-1, B).contiguous().to(dev)
    with torch.no_grad():
        emb = ldm.style_encoder(style)
        for step in ((0, 1, 2) if args.loop_only is None else [int(v) for v in args.loop_only.split(",")]):
            eng = UNetEngine(ldm.unet, fold=True, step=step)
            gd = GraphedDDIM(eng, z, emb["s5"], emb["s6"], tt, coefs, 0.0, logs=True)
            for _ in range(3):
                gd.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                gd.replay()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 20
            print(f"loop step={step}: {dt * 1e3:.3f} ms per 49 iterations = {dt / 49 * 1e6:.2f} us/iter, "
                  f"{49 / dt:.0f} steps/s", flush=True)


if __name__ == "__main__":
    main()
