"""Autotune the conv plans of every UNet layer (and VAE / style-encoder convs) for the given latent
shapes on the current GPU; writes music-style-transfer-ldm_amd/tuned_plans.json.

    python tools/tune_unet.py --shapes 8x16x64 1x16x64 2x16x16
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "music-style-transfer-ldm_amd"))

import torch  # noqa: E402
from ldm_amd import _lib as L, autotune, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="+", default=["8x16x64"])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--dump", default=None, help="write every candidate's median time (us) as JSON here")
    ap.add_argument("--out", default=None, help="tuned-plan file (default: the package's tuned_plans.json)")
    args = ap.parse_args()
    table = {}
    dev = torch.device("cuda:0")
    ops.clear_plan_overrides()
    results = {}
    for s in args.shapes:
        B, H, W = (int(v) for v in s.split("x"))
        shape = L.UNetShape(B, 32, H, W, 64)
        for layer in range(15):
            d = L.ConvDesc()
            L.call("ldm_unet_layer_desc", ctypes.byref(shape), layer, ctypes.byref(d))
            if d.key() in results:
                continue
            best, med = autotune.tune_desc(d, dev, rounds=args.rounds, verbose=True)
            results[d.key()] = best
            table[",".join(map(str, d.key()))] = {",".join(map(str, c)): round(t, 3) for c, t in sorted(med.items(),
                                                                                                 key=lambda kv: kv[1])}
    out = args.out or autotune.TUNED_PATH
    autotune.save_tuned(results, path=out, meta={"device": torch.cuda.get_device_name(0)})
    print("saved", len(results), "plans to", out)
    if args.dump:
        import json
        with open(args.dump, "w") as f:
            json.dump(table, f, indent=1)


if __name__ == "__main__":
    main()
