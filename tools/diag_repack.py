"""Diagnostic: one graphed LDMTrainer run (B, precision, batched re-pack) per process.
python tools/diag_repack.py <B> <fp32|fp16|bf16> <0|1>"""
import faulthandler
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests", "golden"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "music-style-transfer-ldm_amd"))
faulthandler.enable()
if os.environ.get("SEGV_BT"):
    import ctypes
    ctypes.CDLL(os.path.join(os.path.dirname(__file__), "libsegv_bt.so")).segv_bt_install()
import torch  # noqa: E402

import recipe  # noqa: E402


class _ZeroFeat(torch.nn.Module):
    def forward(self, a, b):
        return torch.zeros((), device=a.device)


def main():
    B, prec, batched = int(sys.argv[1]), sys.argv[2], sys.argv[3] == "1"
    import models.model as M
    import models.train as TR
    cuda = torch.device("cuda:0")
    m = M.LDM(32, pretrained_path="")
    recipe.fill_module(m, seed=710)
    m.feature_loss_net = _ZeroFeat()
    m = m.to(cuda).train()
    tr = TR.LDMTrainer(m, [], cuda, lr=1e-3)
    tr.autocast_enabled = prec != "fp32"
    tr.autocast_dtype = {"fp16": torch.float16, "bf16": torch.bfloat16}.get(prec)
    tr.batched_repack = batched
    tr.graph_step = True
    content = torch.from_numpy(recipe.uniform01((B, 1, 128, 128), 1)).to(cuda)
    style = torch.from_numpy(recipe.uniform01((B, 1, 128, 128), 2)).to(cuda)
    t = torch.tensor([17, 160] * (B // 2), device=cuda)
    noise = torch.from_numpy(recipe.normal((B, 32, 16, 16), 3)).to(cuda)
    for i in range(4):
        print(f"step {i} ...", flush=True)
        print(tr.train_step(content, style, t=t, noise=noise), flush=True)
        if i == 1 and os.environ.get("LIVE_GRAPH"):
            import gc
            gc.collect()
            live = [o for o in gc.get_objects() if isinstance(o, torch.Tensor) and o.grad_fn is not None]
            print("live tensors with grad_fn after step 1:", len(live), flush=True)
            for o in live[:8]:
                refs = [type(r).__name__ for r in gc.get_referrers(o)]
                print("  ", tuple(o.shape), type(o.grad_fn).__name__, refs[:6], flush=True)
    print("ok", B, prec, batched, flush=True)


main()
