"""Run one UNet layer's kernel (or a no-op kernel) back to back, for rocprofv3 counter passes and
launch-floor calibration.

    python tools/prof_layer.py --layer 4 --reps 200            # bottleneck conv at B=8, 16x64 latent
    python tools/prof_layer.py --layer attn2 --reps 200
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "music-style-transfer-ldm_amd"))

import torch  # noqa: E402
from ldm_amd import _lib as L, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", default="4")
    ap.add_argument("--shape", default="8x16x64")
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    B, H, W = (int(v) for v in args.shape.split("x"))
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    shape = L.UNetShape(B, 32, H, W, 64)
    if args.layer == "noop":   # launch floor: a 1-element elementwise kernel, back to back
        t1 = torch.zeros(1, device=dev)
        fn = lambda: ops.activation(t1, "relu", inplace=True)  # noqa: E731
    elif args.layer.startswith("attn"):
        E, Lt = (256, H * W // 16) if args.layer == "attn2" else (512, H * W // 64)
        q = torch.randn(B, E, Lt, device=dev)
        kv = torch.randn(B, 2 * E, Lt, device=dev)
        fn = lambda: ops.attention_core(q, kv, 4)  # noqa: E731
    else:
        d = L.ConvDesc()
        L.call("ldm_unet_layer_desc", ctypes.byref(shape), int(args.layer), ctypes.byref(d))
        plan = ops.get_plan(d)
        wshape = (d.Cin, d.Cout, d.kh, d.kw) if d.transposed else (d.Cout, d.Cin, d.kh, d.kw)
        w = torch.randn(wshape, device=dev) * 0.05
        wb = ops.packed_weight(w, d, plan)
        x = torch.randn(d.B, d.Cin, d.Hin, d.Win, device=dev)
        y = torch.empty(d.B, d.Cout, d.Hout, d.Wout, device=dev)
        ep = L.Epilogue()
        ep.act = 1
        lib = L.load()
        ws = torch.zeros(max(1, int(plan.ws_floats)), device=dev)
        a = (ctypes.byref(d), ctypes.byref(plan), x.data_ptr(), wb.data_ptr(), ctypes.byref(ep), y.data_ptr(),
             ws.data_ptr(), st.cuda_stream)
        fn = lambda: lib.ldm_conv_forward_ws(*a[:-1], torch.cuda.current_stream().cuda_stream)  # noqa: E731
        print("plan", plan.key(), "desc", d.key())
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(args.reps):
        fn()
    e1.record(st)
    e1.synchronize()
    print(f"layer {args.layer}: {e0.elapsed_time(e1) * 1e3 / args.reps:.2f} us/launch (eager)")
    # the same chain replayed from a hipGraph: device-side cost per launch in a dependent chain
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(args.reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0.record(st)
    g.replay()
    e1.record(st)
    e1.synchronize()
    print(f"layer {args.layer}: {e0.elapsed_time(e1) * 1e3 / args.reps:.2f} us/launch (graph)")


if __name__ == "__main__":
    main()
