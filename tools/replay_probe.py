"""Does torch.cuda.CUDAGraph.replay() block the host / serialize streams on this ROCm build?"""
import time

import torch


def main():
    dev = torch.device("cuda:0")
    x = torch.randn(4096, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    gs = []
    for st in (s1, s2):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            y = x
            for _ in range(200):
                y = torch.sin(y)
        gs.append(g)
    torch.cuda.synchronize()
    for g in gs:
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gs[0].replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"one replay: host call {1e3 * (t1 - t0):.3f} ms, until done {1e3 * (t2 - t0):.3f} ms")
    main_s = torch.cuda.current_stream()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for st, g in zip((s1, s2), gs):
        st.wait_stream(main_s)
        with torch.cuda.stream(st):
            g.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"two replays on two streams: host {1e3 * (t1 - t0):.3f} ms, until done {1e3 * (t2 - t0):.3f} ms")
    print("torch", torch.__version__, "hip", torch.version.hip)


if __name__ == "__main__":
    main()
