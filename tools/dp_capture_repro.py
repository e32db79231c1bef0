"""Reproduce (or rule out) the round-3 abort of the RCCL-captured DP train step, without the model.

Hypothesis: ProcessGroupNCCL's watchdog thread polls the HIP end-events of EAGER collectives still on its work
list (it retires a completed work only on its next pass, every ~100 ms).  If the main thread is inside a
`torch.cuda.graph` capture in the default *global* capture mode at that moment, the runtime refuses the event
query from the other thread; WorkNCCL rethrows, the watchdog thread dies and, with
TORCH_NCCL_ASYNC_ERROR_HANDLING=3 (the default), the process aborts — from a thread with no Python frame, some
time after the capture, e.g. while the main thread replays.

    python tools/dp_capture_repro.py thread_local|global

world-1 'nccl' over env:// (TCPStore, as bench.py), one eager all-reduce, then a >= 0.5 s capture that starts
right after it, then replays.  Prints REPRO_OK on success.
"""
import os
import sys
import time

import torch
import torch.distributed as tdist


def main(mode):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    tdist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    x = torch.ones(1 << 20, device=dev)
    y = torch.zeros_like(x)
    for it in range(3):
        w = tdist.all_reduce(x, async_op=True)       # eager: enqueued on the watchdog's work list
        w.wait()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        t0 = time.time()
        with torch.cuda.graph(g, capture_error_mode=mode):
            while time.time() - t0 < 0.5:          # span several watchdog passes
                for _ in range(50):
                    y.add_(x)
                time.sleep(0.01)
            cw = tdist.all_reduce(y, async_op=True)   # a captured collective, as GradAllReduce records
            cw.wait()
        for _ in range(20):
            g.replay()
        torch.cuda.synchronize()
        time.sleep(0.3)
        print(f"iter {it}: capture+replay ok ({mode})", flush=True)
    tdist.destroy_process_group()
    print("REPRO_OK", flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "thread_local")
