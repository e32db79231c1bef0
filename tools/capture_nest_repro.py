"""Nested fork inside a hipGraph capture, without autograd: the capture's origin stream M forks S, S forks W
(from the main thread, or from a second thread: `worker`), W joins S, S joins M, the capture ends.  Isolates
what tools/capture_wgrad_repro.py found (a fork from a branch stream in the backward crashes capture_end; a fork
from the origin stream does not).

    python tools/capture_nest_repro.py <main|worker> <thread_local|global> [depth: 1|2]

depth 1 = the nested fork (M -> S -> W); depth 2 = W forked from M instead (M -> S, M -> W, both joined): the
control.
"""
import sys
import threading

import torch

WHERE = sys.argv[1] if len(sys.argv) > 1 else "main"
MODE = sys.argv[2] if len(sys.argv) > 2 else "thread_local"
NESTED = len(sys.argv) < 4 or sys.argv[3] != "2"
dev = torch.device("cuda:0")
S = torch.cuda.Stream(device=dev)
W = torch.cuda.Stream(device=dev)


def main():
    x = torch.ones(4096, device=dev)
    y = torch.zeros(4096, device=dev)
    z = torch.zeros(4096, device=dev)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    err = []

    def nested(parent):
        try:
            W.wait_stream(parent)
            with torch.cuda.stream(W):
                z.add_(x, alpha=3.0)
            parent.wait_stream(W)
        except Exception as e:   # noqa: BLE001
            err.append(repr(e))

    tag = f"[{WHERE} {MODE} {'nested' if NESTED else 'flat'}]"
    with torch.cuda.graph(g, capture_error_mode=MODE):
        m = torch.cuda.current_stream()
        x.add_(1.0)
        S.wait_stream(m)
        with torch.cuda.stream(S):
            y.add_(x, alpha=2.0)
        parent = S if NESTED else m
        if WHERE == "main":
            nested(parent)
        else:
            t = threading.Thread(target=nested, args=(parent,))
            t.start()
            t.join()
        m.wait_stream(S)
        print(f"{tag} body done, errors={err}; ending capture", flush=True)
    print(f"{tag} capture_end returned", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(f"{tag} replay: x={x[0].item()} y={y[0].item()} z={z[0].item()}", flush=True)


if __name__ == "__main__":
    main()
