"""Autotune the conv plans the train step uses (configs 3/4: VAE encode, style encoder, UNet, VAE decode,
forward and data-gradient convs at batch 32 on 1x128x512 mels); merges them into tuned_plans.json.

    python tools/tune_train.py [--batch 32] [--rounds 2]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "music-style-transfer-ldm_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from ldm_amd import _lib as L, autotune, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import models.model as M
    from models.train import LDMTrainer
    dev = torch.device("cuda:0")
    seen = {}
    orig = ops.get_plan

    def rec(desc, force=None):
        seen.setdefault(desc.key(), L.ConvDesc(*[getattr(desc, f) for f, _ in L.ConvDesc._fields_]))
        return orig(desc, force)
    ops.get_plan = rec
    torch.manual_seed(0)
    ldm = M.LDM(32, pretrained_path="").to(dev)
    trainer = LDMTrainer(ldm, None, dev, lr=1e-4)
    ldm.train()
    g = torch.Generator().manual_seed(11)
    B = args.batch
    content = torch.rand(B, 1, 128, 512, generator=g).to(dev)
    style = torch.rand(B, 1, 128, 512, generator=g).to(dev)
    trainer.train_step(content, style)
    torch.cuda.synchronize()
    ops.get_plan = orig
    print(f"{len(seen)} conv descriptors in the train step", flush=True)
    results = {}
    t0 = time.time()
    for key, d in seen.items():
        default = tuple(ops.get_plan(d).key())
        cands = autotune.candidates(d, min_waves=256, max_waves=1 << 22)
        if default not in cands:
            cands.append(default)            # the heuristic plan competes too
        if len(cands) < 2:
            continue
        w_shape = (d.Cin, d.Cout, d.kh, d.kw) if d.transposed else (d.Cout, d.Cin, d.kh, d.kw)
        w = torch.randn(w_shape, device=dev) * 0.05
        x = torch.randn(d.B, d.Cin, d.Hin, d.Win, device=dev)
        y = torch.empty(d.B, d.Cout, d.Hout, d.Wout, device=dev)
        times = {c: [] for c in cands}
        for _ in range(args.rounds):
            for c in cands:
                times[c].append(autotune.time_plan(d, c, x, w, y, reps=10))
        med = {c: sorted(v)[len(v) // 2] for c, v in times.items()}
        best = min(med, key=med.get)
        if best != default:
            results[key] = best
        print(key, "best", best, f"{med[best]:.2f}us", "default", default, f"{med[default]:.2f}us",
              f"({len(cands)} plans, {time.time() - t0:.1f}s)", flush=True)
    out = args.out or autotune.TUNED_PATH
    autotune.save_tuned(results, path=out, meta={"device": torch.cuda.get_device_name(0)})
    print("saved", len(results), "plans to", out)


if __name__ == "__main__":
    main()
