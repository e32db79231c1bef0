"""Round 4's weight-gradient side stream in isolation (the variant that segfaulted in capture_end,
gpurun_out/r4wg*/): a two-branch autograd graph (one branch's forward on a side stream S, as graphs.branch runs
the style encoder) whose backward nodes each fork ONE shared stream W from the node's current stream (S or the
origin M), allocate their weight-gradient output on W, and join W back before returning it to autograd
(which steals it as the leaf's .grad).  Captured with torch.cuda.graph in the given mode, replayed, checked
against the eager step.

    python tools/capture_wgrad_repro.py <thread_local|global> <join: 1|0> [flags]

join=0 leaves the per-node join out (W's work reaches the origin only through later forks).  flags (one word,
any of): n = no side-stream branch S in the forward (every node on the origin stream); p = the weight gradient
written into a buffer allocated before the capture (no allocation on W during the capture); s = a separate
fork stream per node instead of one shared W.
"""
import sys

import torch

MODE = sys.argv[1] if len(sys.argv) > 1 else "thread_local"
JOIN = len(sys.argv) < 3 or sys.argv[2] != "0"
FLAGS = sys.argv[3] if len(sys.argv) > 3 else ""
dev = torch.device("cuda:0")
W_STREAM = torch.cuda.Stream(device=dev)
S_STREAM = torch.cuda.Stream(device=dev)
W_PER_NODE = [torch.cuda.Stream(device=dev) for _ in range(4)]
GW_BUF = {}


class Lin(torch.autograd.Function):
    """y = x @ w; backward: dx on the current stream, dw on W (allocated there)."""

    @staticmethod
    def forward(ctx, x, w, i):
        ctx.save_for_backward(x, w)
        ctx.i = i
        return x @ w

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        cur = torch.cuda.current_stream(dev)
        ws = W_PER_NODE[ctx.i] if "s" in FLAGS else W_STREAM
        ws.wait_stream(cur)
        with torch.cuda.stream(ws):
            if "p" in FLAGS:
                gw = torch.matmul(x.t(), gy, out=GW_BUF[ctx.i])
            else:
                gw = x.t() @ gy
        gx = gy @ w.t()
        if JOIN:
            cur.wait_stream(ws)
        return gx, gw, None


def step(params, xa, xb):
    for p in params:
        p.grad = None
    m = torch.cuda.current_stream(dev)
    side = m if "n" in FLAGS else S_STREAM
    side.wait_stream(m)
    with torch.cuda.stream(side):
        hb = torch.relu(Lin.apply(xb, params[0], 0))
        hb = Lin.apply(hb, params[1], 1)
    ha = torch.relu(Lin.apply(xa, params[2], 2))
    m.wait_stream(side)
    out = Lin.apply(ha + hb, params[3], 3)
    loss = (out * out).mean()
    loss.backward()
    if not JOIN:
        for w in [W_STREAM] + W_PER_NODE:
            m.wait_stream(w)
    return loss.detach()


def main():
    torch.manual_seed(0)
    params = [torch.randn(64, 64, device=dev, requires_grad=True) * 1 for _ in range(4)]
    params = [p.detach().requires_grad_(True) for p in params]
    xa = torch.randn(128, 64, device=dev)
    xb = torch.randn(128, 64, device=dev)
    for i in range(4):
        GW_BUF[i] = torch.empty(64, 64, device=dev)
    ref = step(params, xa, xb)
    ref_g = [p.grad.clone() for p in params]
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode=MODE):
        out = step(params, xa, xb)
        print(f"[{MODE} join={int(JOIN)} flags={FLAGS}] body captured; ending capture", flush=True)
    print(f"[{MODE} join={int(JOIN)} flags={FLAGS}] capture_end returned", flush=True)
    g.replay()
    torch.cuda.synchronize()
    ok = torch.allclose(out, ref) and all(torch.allclose(p.grad, r) for p, r in zip(params, ref_g))
    print(f"[{MODE} join={int(JOIN)} flags={FLAGS}] replay ok={ok}", flush=True)
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
