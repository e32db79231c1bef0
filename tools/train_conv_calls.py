"""Every conv forward / data-gradient / weight-gradient call of one config-3 train step (bench.py's train line:
B = 32, bf16 autocast, 16-bit storage of the large maps), re-run alone with the step's own tensors and timed
(CUDA events, 20 reps), sorted by time: which layer calls the step's conv time goes to.

    python tools/train_conv_calls.py [--batch 32]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "music-style-transfer-ldm_amd")]

import torch  # noqa: E402


def time_us(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    import models.model as M
    from ldm_amd import ops
    from models.train import LDMTrainer
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    ldm = M.LDM(32, pretrained_path="").to(dev).train()
    tr = LDMTrainer(ldm, None, dev, lr=1e-4)
    tr.autocast_dtype = torch.bfloat16
    B = a.batch
    g = torch.Generator().manual_seed(11)
    content = torch.rand(B, 1, 128, 512, generator=g).to(dev)
    style = torch.rand(B, 1, 128, 512, generator=g).to(dev)
    for _ in range(2):
        tr.train_step(content, style)
    calls = []
    fwd, dgrad, wgrad = ops.conv_forward, ops.conv_backward_data, ops.conv_backward_weight

    def rec_fwd(*args, **kw):
        calls.append(("fwd", args, dict(kw)))
        return fwd(*args, **kw)

    def rec_dgrad(*args, **kw):
        calls.append(("dgrad", args, dict(kw)))
        return dgrad(*args, **kw)

    def rec_wgrad(*args, **kw):
        calls.append(("wgrad", args, dict(kw)))
        return wgrad(*args, **kw)

    ops.conv_forward, ops.conv_backward_data, ops.conv_backward_weight = rec_fwd, rec_dgrad, rec_wgrad
    try:
        tr.train_step(content, style)
        torch.cuda.synchronize()
    finally:
        ops.conv_forward, ops.conv_backward_data, ops.conv_backward_weight = fwd, dgrad, wgrad
    rows = []
    for kind, args, kw in calls:
        if kind == "fwd":
            x, w = args[0], args[1]
            kw2 = dict(kw)
            kw2.pop("out", None)
            kw2.pop("act_out", None)
            fn = lambda: fwd(*args, **kw2)  # noqa: E731
            d = ops.make_desc(x.shape[0], x.shape[1], x.shape[2], x.shape[3],
                              w.shape[1] if kw.get("transposed") else w.shape[0], w.shape[2], w.shape[3],
                              kw.get("stride", 1), kw.get("padding", 1), kw.get("output_padding", 0),
                              kw.get("transposed", False))
            xs = x
        elif kind == "dgrad":
            d = args[2]
            xs = args[0]
            fn = lambda: dgrad(*args, **kw)  # noqa: E731
        else:
            d = args[2]
            xs = args[0]
            fn = lambda: wgrad(*args, **kw)  # noqa: E731
        us = time_us(fn)
        taps = d.kh * d.kw / (4.0 if d.transposed else 1.0)
        flops = 2.0 * d.B * d.Cout * d.Hout * d.Wout * d.Cin * taps if not d.transposed else \
            2.0 * d.B * d.Cout * d.Hout * d.Wout * d.Cin * d.kh * d.kw / 4.0
        rows.append((us, kind, f"B{d.B} {d.Cin}->{d.Cout} {d.Hin}x{d.Win}->{d.Hout}x{d.Wout} k{d.kh} s{d.stride}"
                                f"{' T' if d.transposed else ''}", str(xs.dtype).replace("torch.", ""), flops))
    rows.sort(key=lambda r: -r[0])
    tot = sum(r[0] for r in rows)
    for us, kind, desc, dt, fl in rows:
        print(f"{us:8.1f} us  {kind:5s}  {desc:40s}  x {dt:8s}  {fl / us / 1e6:7.1f} TF/s")
    print(f"total {tot:.1f} us over {len(rows)} calls")


if __name__ == "__main__":
    main()
