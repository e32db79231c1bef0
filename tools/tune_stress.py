"""Autotune the conv plans of shape S (bench.py --workload stress: UNet(1, 1) on the raw [B,1,128,512] mel) on the
current GPU and merge them into music-style-transfer-ldm_amd/tuned_plans.json.

The descriptors are the ones one eager UNet forward at that shape asks ops.get_plan for (recorded, not
re-derived); each is timed over every valid (kind, tm, tn, wk, ks) instance by ldm_amd.autotune (hipGraph chains,
interleaved rounds, median), the heuristic plan among them.

    python tools/tune_stress.py [--batch 1] [--dump gpurun_out/tune_stress.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "music-style-transfer-ldm_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from ldm_amd import autotune, ops  # noqa: E402


def stress_descs(batch, dev):
    """Descriptors (by key) of the general conv path in one UNet(1, 1) forward at shape S."""
    import models.model as M
    unet = M.UNet(1, 1, 64).to(dev).eval()
    g = torch.Generator().manual_seed(1)
    x = torch.randn((batch, 1, 128, 512), generator=g).to(dev)
    emb = {"s5": torch.rand((batch, 256, 32, 128), generator=g).to(dev),
           "s6": torch.rand((batch, 512, 16, 64), generator=g).to(dev)}
    t = torch.full((batch,), 500, dtype=torch.long, device=dev)
    seen = {}
    orig = ops.get_plan

    def rec(desc, force=None):
        seen.setdefault(desc.key(), desc)
        return orig(desc, force)

    ops.get_plan = rec
    try:
        with torch.no_grad():
            unet(x, t, emb)
        torch.cuda.synchronize()
    finally:
        ops.get_plan = orig
    return seen


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--dump", default=None, help="write every candidate's median time (us) as JSON here")
    ap.add_argument("--out", default=None, help="tuned-plan file (default: the package's tuned_plans.json)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    descs = stress_descs(args.batch, dev)
    print(len(descs), "descriptors", flush=True)
    results, table = {}, {}
    for key, d in descs.items():
        best, med = autotune.tune_desc(d, dev, rounds=args.rounds, verbose=True)
        default = tuple(ops.get_plan(d).key()) if key not in ops._PLAN_OVERRIDE else None
        results[key] = best
        table[",".join(map(str, key))] = {",".join(map(str, c)): round(v, 3)
                                          for c, v in sorted(med.items(), key=lambda kv: kv[1])}
        print("  default", default, flush=True)
    out = args.out or autotune.TUNED_PATH
    autotune.save_tuned(results, path=out, meta={"device": torch.cuda.get_device_name(0)})
    print("saved", len(results), "plans to", out)
    if args.dump:
        with open(args.dump, "w") as f:
            json.dump(table, f, indent=1)


if __name__ == "__main__":
    main()
