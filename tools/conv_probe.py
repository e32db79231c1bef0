"""Decompose conv kernel time into a fixed cost and a per-K slope: time the bottleneck-like geometry
(M = Cout, N = B*H*W output columns) for several Cin and plans, graph-replayed back to back.

    python tools/conv_probe.py --cout 512 --hw 2x8 --cins 16,64,128,256,512 --plans 2114,1118,2118
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "music-style-transfer-ldm_amd"))

import torch  # noqa: E402
from ldm_amd import _lib as L, ops  # noqa: E402


def graph_us(fn, reps=200):
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(reps):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(5):
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cout", type=int, default=512)
    ap.add_argument("--hw", default="2x8")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--cins", default="16,64,128,256,512")
    ap.add_argument("--plans", default="")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    H, W = (int(v) for v in args.hw.split("x"))
    dev = torch.device("cuda:0")
    res = {}
    for cin in (int(c) for c in args.cins.split(",")):
        d = ops.make_desc(args.batch, cin, H, W, args.cout, args.k, args.k, 1, args.k // 2)
        x = torch.randn(args.batch, cin, H, W, device=dev)
        w = torch.randn(args.cout, cin, args.k, args.k, device=dev) * 0.05
        y = torch.empty(args.batch, args.cout, d.Hout, d.Wout, device=dev)
        plans = [tuple(int(c) for c in p) for p in args.plans.split(",") if p] or \
            [(k, tm, tn, wk) for k in (1, 2) for tm in (1, 2) for tn in (1, 2) for wk in (1, 2, 4, 8, 16)]
        for pl in plans:
            p = L.ConvPlan()
            if L.load().ldm_conv_make_plan_forced(ctypes.byref(d), *pl, ctypes.byref(p)) != 0:
                continue
            wb = torch.empty(int(p.packed_floats), device=dev)
            L.call("ldm_conv_pack_weight", ctypes.byref(d), ctypes.byref(p), w.data_ptr(), wb.data_ptr(),
                   ops.stream_handle())
            ep = L.Epilogue()
            ep.act = 1

            def fn(d=d, p=p, x=x, wb=wb, ep=ep, y=y):
                L.load().ldm_conv_forward(ctypes.byref(d), ctypes.byref(p), x.data_ptr(), wb.data_ptr(),
                                          ctypes.byref(ep), y.data_ptr(), torch.cuda.current_stream().cuda_stream)
            us = graph_us(fn)
            flops = 2.0 * args.batch * d.Hout * d.Wout * args.cout * cin * args.k * args.k
            res.setdefault("".join(map(str, pl)), {})[cin] = round(us, 3)
            print(f"cin={cin:4d} plan={pl} {us:8.3f} us  {flops / us / 1e6:7.2f} TF/s", flush=True)
    # noop floor
    t1 = torch.zeros(1, device=dev)
    res["noop"] = round(graph_us(lambda: ops.activation(t1, "relu", inplace=True)), 3)
    print("noop", res["noop"])
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
