"""Time the train step's VALU convolutions (Cin = 1 first layers, the 64 -> 1 output convT and its data gradient)
in isolation at B = 32 with the 16-bit map storage the train step uses; reports GB/s of the stored bytes.  The
event times include the Python wrapper's host cost; run it under `rocprofv3 --kernel-trace --stats` for the
kernels' own durations (profiles/r04/valu_convs).
python tools/time_valu16.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "music-style-transfer-ldm_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402

from ldm_amd import ops  # noqa: E402
from time_wgrad import time_ms  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    dt, T16 = 2, torch.bfloat16
    x = torch.rand(32, 1, 128, 512, device=dev)
    w1 = torch.randn(64, 1, 3, 3, device=dev) * 0.3
    b1 = torch.randn(64, device=dev) * 0.1
    y = ops.conv_forward(x, w1, b1, stride=2, padding=1, dtype=dt, out_dtype=T16)
    t = time_ms(lambda: ops.conv_forward(x, w1, b1, stride=2, padding=1, dtype=dt, out_dtype=T16))
    byts = x.numel() * 4 + y.numel() * 2
    print(f"enc1 k3s2 1->64 fwd (bf16 out)      {t * 1e3:7.1f} us  {byts / t / 1e6:6.0f} GB/s", flush=True)
    h = torch.rand(32, 64, 64, 256, device=dev).to(T16)
    w2 = torch.randn(64, 1, 4, 4, device=dev) * 0.2
    b2 = torch.randn(1, device=dev) * 0.1
    o = ops.conv_forward(h, w2, b2, stride=2, padding=1, transposed=True, act="tanh", dtype=dt)
    t = time_ms(lambda: ops.conv_forward(h, w2, b2, stride=2, padding=1, transposed=True, act="tanh", dtype=dt))
    byts = h.numel() * 2 + o.numel() * 4
    print(f"dec3 convT k4 64->1 fwd (bf16 in)   {t * 1e3:7.1f} us  {byts / t / 1e6:6.0f} GB/s", flush=True)
    d2 = ops.make_desc(32, 64, 64, 256, 1, 4, 4, 2, 1, 0, True)
    r = torch.randn_like(o)
    g = ops.conv_backward_data(r, w2, d2, dtype=dt, out_dtype=T16)
    t = time_ms(lambda: ops.conv_backward_data(r, w2, d2, dtype=dt, out_dtype=T16))
    byts = r.numel() * 4 + g.numel() * 2
    print(f"dec3 dgrad (Cin = 1 k4, bf16 out)   {t * 1e3:7.1f} us  {byts / t / 1e6:6.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
