"""hipGraph capture for the LDM path (the reverse loop, the train step, the autotuner's timing chains).

Every capture here runs in the *thread-local* capture mode.  torch.cuda.graph's default is the global mode,
in which, while one thread captures, every OTHER thread of the process is refused potentially unsafe runtime
calls — hipEventQuery among them.  With a 'nccl' (RCCL) process group alive, ProcessGroupNCCL's watchdog
thread polls the end events of the eager collectives on its work list (a completed work leaves the list only
at the watchdog's next pass, ~100 ms later).  A data-parallel train step captured right after its eager
warm-up steps (whose bucketed all-reduces are still listed), or a sampler captured right after a barrier,
therefore raced the watchdog: when a pass fell inside the capture window the event query failed,
WorkNCCL rethrew, the watchdog thread died and, with TORCH_NCCL_ASYNC_ERROR_HANDLING=3 (the default), took
the process down from a thread with no Python frame — after the capture, e.g. during the first replays
(round 3's intermittent abort).  In thread-local mode only the capturing thread is
restricted, which is all the capture needs: nothing on this path calls the runtime from another thread.
"""
import torch

CAPTURE_MODE = "thread_local"


def capture(graph, stream=None, pool=None):
    """Context manager: capture into `graph` (torch.cuda.CUDAGraph) on `stream`, thread-local mode."""
    return torch.cuda.graph(graph, pool=pool, stream=stream, capture_error_mode=CAPTURE_MODE)
