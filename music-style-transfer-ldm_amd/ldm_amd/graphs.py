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
restricted.  Note that the backward of a captured train step runs on autograd's device worker thread, not on the
capturing thread: in thread-local mode that thread is not checked for unsafe calls (a hidden synchronisation or
legacy-stream call in a backward function would run at capture time and be missing from the replays instead of
failing the capture).  The guard for that is tests/test_gpu_train.py's capture of the whole train step in the
global mode (LDM_AMD_CAPTURE_MODE=global; no RCCL watchdog is alive there), which must succeed and replay
equal to the eager step.

Side streams (branch(), the pool of prepare_streams) are recorded per capture: capture() joins every pool
stream that took part in the capture back into the origin stream before the capture ends, so no captured work
is left outside the graph's sink whatever order autograd ran the branches in.

Only the capture's ORIGIN stream forks.  A fork from a stream that is itself a forked capture stream (origin M
forks S, S forks W; W joins S, S joins M) segfaults the HIP runtime in hipStreamEndCapture on ROCm 7.2, from the
capturing thread alone, without autograd (tools/capture_nest_repro.py; the same pattern inside a backward,
tools/capture_wgrad_repro.py): that was round 4's crash of the per-conv weight-gradient side stream, whose
backward nodes of the style-encoder branch forked from the branch stream.  branch() therefore runs its block in
place when the current stream is a capture stream other than the origin.
"""
import contextlib
import os

import torch

CAPTURE_MODE = "thread_local"


def capture_mode():
    """The capture mode of capture(): thread_local, or LDM_AMD_CAPTURE_MODE (global / relaxed / thread_local)."""
    return os.environ.get("LDM_AMD_CAPTURE_MODE", CAPTURE_MODE)


_CAPTURES = []   # per capture in progress: (origin stream, set of pool streams that joined it)


def quiesce_collectives():
    """Before a capture: wait until the default process group's watchdog has retired every eager collective still
    on its work list (ProcessGroup._wait_for_pending_works; a no-op without an initialised group or for a backend
    without it).  A capture that started while the list still held eager works could have the watchdog query their
    events inside the capture window: round 3's abort, and in round 6 an abort in capture_end once the train step
    stopped waiting on the host every step (its eager warm-up steps' all-reduces reached the capture sooner)."""
    try:
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            return
        dist.distributed_c10d._get_default_group()._wait_for_pending_works()
    except Exception:
        pass


@contextlib.contextmanager
def capture(graph, stream=None, pool=None):
    """Context manager: capture into `graph` (torch.cuda.CUDAGraph) on `stream` (capture_mode()).  Before the
    capture ends, the origin stream waits on every branch stream that forked from it during the capture.  Before it
    starts, the device is synchronised and the process group's pending eager collectives retired
    (quiesce_collectives)."""
    if not _CAPTURES:
        torch.cuda.synchronize()
        quiesce_collectives()
    with torch.cuda.graph(graph, pool=pool, stream=stream, capture_error_mode=capture_mode()):
        origin = torch.cuda.current_stream()
        rec = (origin, {})
        _CAPTURES.append(rec)
        ok = False
        try:
            yield
            ok = True
        finally:
            _CAPTURES.pop()
            # joined whether or not the body succeeded: an unjoined fork would make the capture's end raise
            # hipErrorStreamCaptureUnjoined and hide the body's own exception
            for side in rec[1].values():
                try:
                    origin.wait_stream(side)
                except Exception:
                    if ok:
                        raise


def captured_side_streams():
    """The branch streams recorded by the innermost capture in progress (for tests / assertions)."""
    return list(_CAPTURES[-1][1].values()) if _CAPTURES else []


_BRANCH_STREAMS = {}


def _stream_switch(device, var, default):
    """An env switch for the side-stream forms: "1" on, "0" off, unset: `default` ("capture": only while the
    current stream is capturing a hipGraph).  Measured (profiles/r04/branch_streams): the replayed train step
    runs the DAG's independent branches concurrently (4.96 -> 4.70 ms with the style-encoder branch), while an
    eager step pays more in host-side stream bookkeeping than it gains (5.87 -> 6.97 ms)."""
    if torch.device(device).type != "cuda":
        return False
    v = os.environ.get(var, default)
    if v == "capture":
        return torch.cuda.is_current_stream_capturing()
    return v != "0"


def branch_streams_enabled(device):
    """Independent branches of the train step on their own streams (LDM_AMD_BRANCH_STREAMS)."""
    return _stream_switch(device, "LDM_AMD_BRANCH_STREAMS", "capture")


_POOL_SIZE = 8


def prepare_streams(device):
    """Create the side-stream pool of `device` (outside any capture: a stream is never created while a graph
    is being captured)."""
    key = str(torch.device(device))
    if key not in _BRANCH_STREAMS:
        _BRANCH_STREAMS[key] = ([torch.cuda.Stream(device=torch.device(device)) for _ in range(_POOL_SIZE)], {})


def branch_stream(device, name):
    """The side stream of branch `name` on `device` (a fixed stream of the pool per name), or None when the
    pool does not exist yet and the current stream is capturing, or the pool is used up."""
    key = str(torch.device(device))
    if key not in _BRANCH_STREAMS:
        if torch.cuda.is_current_stream_capturing():
            return None
        prepare_streams(device)
    pool, names = _BRANCH_STREAMS[key]
    i = names.get(name)
    if i is None:
        if len(names) >= len(pool):
            return None
        i = names[name] = len(names)
    return pool[i]


@contextlib.contextmanager
def branch(device, name):
    """Run the block on the side stream `name`, forked from the current stream: the block's work may overlap
    what the current stream does next, until join() (or a consumer on another stream, which the autograd
    engine orders after it).  Inside a graph capture the fork and the join become graph edges.  Yields the
    stream to pass to join(); with branch streams off the block runs in place and join() does nothing."""
    if not branch_streams_enabled(device):
        yield None
        return
    main = torch.cuda.current_stream(torch.device(device))
    capturing = torch.cuda.is_current_stream_capturing()
    if capturing and _CAPTURES and main.cuda_stream != _CAPTURES[-1][0].cuda_stream:
        yield None          # never fork from a forked capture stream (the runtime crashes at capture end)
        return
    side = branch_stream(device, name)
    if side is None or side.cuda_stream == main.cuda_stream:
        yield None
        return
    side.wait_stream(main)
    if _CAPTURES and capturing:
        _CAPTURES[-1][1][side.cuda_stream] = side
    with torch.cuda.stream(side):
        yield side


def join(side, device):
    """The current stream waits for everything queued on `side` so far.  Tensors a branch made and the current
    stream reads afterwards need no record_stream: their blocks return to the branch's pool when freed, and
    the branch's next allocation comes after its next fork, i.e. after a wait on the current stream."""
    if side is None:
        return
    torch.cuda.current_stream(torch.device(device)).wait_stream(side)
