"""Which side-stream fork / join pattern inside a hipGraph capture does the runtime survive?

Round 4's weight-gradient side stream (LDM_AMD_WGRAD_STREAM, removed) segfaulted in torch's capture_end
(gpurun_out/r4wg*/).  That variant was the only one in which a stream that was NOT yet part of the capture
entered it from the autograd engine's device thread (a fork inside a backward node), while the capture had been
begun on the main thread in the thread-local mode.  The shipped branch streams (graphs.branch) always enter
the capture from the capturing thread.  This probe isolates that difference:

    python tools/capture_fork_repro.py <fork_thread: main|worker> <mode: thread_local|global> [join: 1|0]

captures on stream M in the main thread; a fresh side stream W waits on M from `fork_thread`, runs one op,
and (join=1) M waits on W; then the capture ends, is replayed and the result is checked.  Run each case in
its own process (a segfault ends it): tools/gpu_capture_fork.sh.
"""
import sys
import threading

import torch


def main():
    where, mode = sys.argv[1], sys.argv[2]
    do_join = len(sys.argv) < 4 or sys.argv[3] != "0"
    dev = torch.device("cuda:0")
    x = torch.zeros(1024, device=dev)
    y = torch.zeros(1024, device=dev)
    side = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    err = []

    def fork_body(main_stream):
        try:
            side.wait_stream(main_stream)
            with torch.cuda.stream(side):
                y.add_(x, alpha=2.0)
            if do_join:
                main_stream.wait_stream(side)
        except Exception as e:   # noqa: BLE001 - reported below
            err.append(repr(e))

    with torch.cuda.graph(g, capture_error_mode=mode):
        m = torch.cuda.current_stream()
        x.add_(1.0)
        if where == "main":
            fork_body(m)
        else:
            t = threading.Thread(target=fork_body, args=(m,))
            t.start()
            t.join()
        with torch.cuda.stream(m):
            x.mul_(3.0)
        print(f"[{where} {mode} join={int(do_join)}] body done, errors={err}; ending capture", flush=True)
    print(f"[{where} {mode} join={int(do_join)}] capture_end returned", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(f"[{where} {mode} join={int(do_join)}] replay ok: x={x[0].item()} y={y[0].item()}", flush=True)


if __name__ == "__main__":
    main()
