"""How much of a train step is host time?  Times LDMTrainer.train_step at B=32 bf16 three ways:
wall per step, host enqueue time up to the loss .item() syncs (optimizer step included), and the
python-side time of the forward and of backward() alone.   python tools/host_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "music-style-transfer-ldm_amd")]
import torch  # noqa: E402

import models.model as M  # noqa: E402
import models.train as TR  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    ldm = M.LDM(32, pretrained_path="").to(dev)
    tr = TR.LDMTrainer(ldm, None, dev, lr=1e-4)
    tr.autocast_dtype = torch.bfloat16
    ldm.train()
    B = 32
    content = torch.rand(B, 1, 128, 512, device=dev)
    style = torch.rand(B, 1, 128, 512, device=dev)
    for _ in range(3):
        tr.train_step(content, style)
    torch.cuda.synchronize()
    marks = {}
    orig_backward = torch.Tensor.backward

    def bw(self, *a, **k):
        t0 = time.perf_counter()
        r = orig_backward(self, *a, **k)
        marks["backward_host"] = marks.get("backward_host", 0) + time.perf_counter() - t0
        return r
    orig_step = tr.scaler.step

    def st(*a, **k):
        t0 = time.perf_counter()
        r = orig_step(*a, **k)
        marks["opt_host"] = marks.get("opt_host", 0) + time.perf_counter() - t0
        marks["enqueued"] = marks.get("enqueued", 0) + time.perf_counter() - marks["t_start"]
        return r
    torch.Tensor.backward = bw
    tr.scaler.step = st
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        marks["t_start"] = time.perf_counter()
        tr.train_step(content, style)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n
    torch.Tensor.backward = orig_backward
    print(f"wall {wall * 1e3:.3f} ms/step; host to end of optimizer step {marks['enqueued'] / n * 1e3:.3f} ms; "
          f"backward() host {marks['backward_host'] / n * 1e3:.3f} ms; scaler.step host {marks['opt_host'] / n * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
