"""Wall time of VGGishFeatureLoss on the HIP path at the train step's shape (B=32, 1x128x512, both sides
in one batch of 64) under torch.autocast(bf16) and in fp32; recipe weights.  python tools/time_vggish.py"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "music-style-transfer-ldm_amd"), os.path.join(ROOT, "tests", "golden")]
import recipe  # noqa: E402
from models.loss import VGGishFeatureLoss, vggish_features  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    feats = vggish_features()
    recipe.fill_module(feats, seed=800)
    loss = VGGishFeatureLoss(feats.to(dev))
    p = torch.rand(32, 1, 128, 512, device=dev)
    t = torch.rand(32, 1, 128, 512, device=dev)
    flops = 2 * 32 * 2 * sum(m.weight.numel() * (128 * 512) // (4 ** k)
                             for k, m in zip((0, 1, 2, 2, 3, 3), [m for m in feats if isinstance(m, torch.nn.Conv2d)]))
    for name, ctx in (("bf16", lambda: torch.autocast("cuda", dtype=torch.bfloat16)), ("fp32", torch.no_grad)):
        with ctx():
            for _ in range(2):
                loss(p, t)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                v = loss(p, t)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / 5 * 1e3
        print(f"vggish {name}: {ms:.2f} ms per call (B=32 pred + target), {flops / ms / 1e9:.1f} TFLOP/s, loss {v.item():.6f}")


if __name__ == "__main__":
    main()
