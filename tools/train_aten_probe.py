"""Where the ATen device kernels of the train step come from (fills, adds, copies that never reached a HIP
kernel of ours): one eager bf16 config-3 step (bench.py's train line, B = 32) under torch.profiler with Python
stacks; prints every aten op that launched a device kernel, grouped by op and innermost package frame.

    python tools/train_aten_probe.py [--batch 32] [--steps 1]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "music-style-transfer-ldm_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=1)
    a = ap.parse_args()
    import models.model as M
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
    for _ in range(3):
        tr.train_step(content, style)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(a.steps):
            tr.train_step(content, style)
        torch.cuda.synchronize()
    # every aten op on device tensors in one step, with its innermost package frames (TorchDispatchMode: the
    # autograd engine carries the mode into its device thread, so the backward's own accumulations show up)
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    seen = collections.Counter()

    class Log(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = str(func.overloadpacket.__name__)
            if name in ("add_", "add", "copy_", "fill_", "zero_", "mul", "mul_", "sum", "cat", "clone",
                        "_to_copy", "zeros_like", "ones_like", "div", "sub", "reciprocal", "_local_scalar_dense",
                        "normal_", "random_", "stack", "index_put_", "masked_fill_", "where"):
                fr = [f"{f.filename.split('music-style-transfer-ldm_amd/')[-1]}:{f.lineno}:{f.name}"
                      for f in traceback.extract_stack()[:-1] if "music-style-transfer-ldm_amd" in f.filename]
                shp = [tuple(t.shape) for t in args if isinstance(t, torch.Tensor)][:2]
                seen[(name, str(shp), " <- ".join(reversed(fr[-3:])) or "(autograd engine)")] += 1
            return func(*args, **(kwargs or {}))

    with Log():
        tr.train_step(content, style)
        torch.cuda.synchronize()
    for (name, shp, where), n in sorted(seen.items(), key=lambda kv: -kv[1]):
        print(f"DISPATCH {n:3d} {name:20s} {shp:40s} {where}")
    groups = collections.Counter()
    times = collections.Counter()
    for ev in prof.events():
        if not ev.name.startswith("aten::") or ev.device_type != torch.autograd.DeviceType.CPU:
            continue
        dt = getattr(ev, "self_device_time_total", None)
        if dt is None:
            dt = getattr(ev, "self_cuda_time_total", 0)
        if dt <= 0:
            continue
        if ev.name in ("aten::empty", "aten::empty_strided", "aten::as_strided", "aten::view", "aten::reshape"):
            continue
        frames = [f for f in (ev.stack or []) if "music-style-transfer-ldm_amd" in f or "tools/" in f]
        where = " <- ".join(f.split("music-style-transfer-ldm_amd/")[-1] for f in frames[:3]) or "(no package frame)"
        groups[(ev.name, where)] += 1
        times[(ev.name, where)] += dt
    for (name, where), n in sorted(groups.items(), key=lambda kv: -kv[1]):
        print(f"{n / a.steps:6.1f}/step {times[(name, where)] / a.steps:8.1f} us  {name:28s} {where}")
    # the same ops with their Python stacks (innermost package frames), from the profiler's stack grouping
    want = ("aten::add_", "aten::copy_", "aten::mul", "aten::fill_", "aten::add", "aten::zero_", "aten::sum",
            "aten::cat", "aten::reciprocal", "aten::_local_scalar_dense", "aten::normal_", "aten::random_")
    for row in prof.key_averages(group_by_stack_n=12):
        if row.key not in want:
            continue
        st = [f for f in row.stack if "music-style-transfer-ldm_amd" in f or "site-packages/torch" not in f]
        print(f"--- {row.key} x{row.count / a.steps:.1f}/step")
        for f in st[:8]:
            print("      ", f.split("repo/")[-1])


if __name__ == "__main__":
    main()
