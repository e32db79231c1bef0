"""One train-step conv call in a loop (for rocprofv3 --pmc passes on its kernel): a B = 32 bf16 layer of the
train step with 16-bit input storage, as the step calls it.

    python tools/one_conv.py <fwd|dgrad|wgrad> <Cin> <H> <W> <Cout> <k> <stride> [T] [--reps N]
e.g. python tools/one_conv.py fwd 64 64 256 128 3 2          (the VAE / style encoder's 64 -> 128 layer)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "music-style-transfer-ldm_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=("fwd", "dgrad", "wgrad"))
    ap.add_argument("cin", type=int)
    ap.add_argument("h", type=int)
    ap.add_argument("w", type=int)
    ap.add_argument("cout", type=int)
    ap.add_argument("k", type=int)
    ap.add_argument("stride", type=int)
    ap.add_argument("t", nargs="?", default="")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--maps32", action="store_true", help="fp32 storage of the maps (the UNet's small layers)")
    ap.add_argument("--x32", action="store_true", help="fp32 input map, 16-bit output (the encoders' first layers)")
    a = ap.parse_args()
    from ldm_amd import ops
    dev = torch.device("cuda:0")
    tr = a.t == "T"
    B, k, s = a.batch, a.k, a.stride
    p, op = 1, 0
    desc = ops.make_desc(B, a.cin, a.h, a.w, a.cout, k, k, s, p, op, tr)
    dt = 2
    mt = torch.float32 if a.maps32 else torch.bfloat16
    x = (torch.rand(B, a.cin, a.h, a.w, device=dev) - 0.5).to(torch.float32 if a.x32 else mt)
    w = torch.randn((a.cin, a.cout, k, k) if tr else (a.cout, a.cin, k, k), device=dev) * 0.05
    dy = (torch.rand(B, a.cout, desc.Hout, desc.Wout, device=dev) - 0.5).to(mt)
    if a.kind == "fwd":
        fn = lambda: ops.conv_forward(x, w, None, stride=s, padding=p, transposed=tr, output_padding=op, dtype=dt,  # noqa
                                      out_dtype=mt)
    elif a.kind == "dgrad":
        fn = lambda: ops.conv_backward_data(dy, w, desc, dtype=dt, out_dtype=mt)  # noqa
    else:
        fn = lambda: ops.conv_backward_weight(x, dy, desc, dtype=dt)  # noqa
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{a.kind} {a.cin}->{a.cout} {a.h}x{a.w} k{k} s{s}{' T' if tr else ''}: {e0.elapsed_time(e1) * 1e3 / a.reps:.1f} us")


if __name__ == "__main__":
    main()
