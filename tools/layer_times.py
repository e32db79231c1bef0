"""Per-layer graph-timed kernel durations of the UNet at a given shape (bench.time_layers), as a table.
    [LDM_AMD_LIB=...variant.so] python tools/layer_times.py [--shape 8x16x64]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "music-style-transfer-ldm_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="8x16x64")
    args = ap.parse_args()
    B, H, W = (int(v) for v in args.shape.split("x"))
    import models.model as M
    dev = torch.device("cuda:0")
    ldm = M.LDM(32, pretrained_path="").to(dev).eval()
    eng = M.engine_for(ldm.unet)
    with torch.no_grad():
        kt = bench.time_layers(eng, eng.shape(B, 32, H, W), dev)
    tot = 0.0
    for k, v in kt.items():
        print(f"{k:12s} {v['us']:8.2f} us {v['tflops']:7.1f} TF  {v.get('plan', '')}")
        tot += v["us"]
    print(f"{'sum':12s} {tot:8.2f} us", os.environ.get("LDM_AMD_LIB", "default lib"))


if __name__ == "__main__":
    main()
