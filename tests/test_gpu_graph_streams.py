"""Branch streams inside a hipGraph capture (ldm_amd/graphs.py).

A fork from a stream that is itself a forked capture stream segfaults the HIP runtime in hipStreamEndCapture
(ROCm 7.2; tools/capture_nest_repro.py): round 4's weight-gradient side stream did exactly that
from the style-encoder branch.  graphs.branch() forks only from the capture's origin stream and runs a nested
branch in place; capture() joins every branch stream before the capture ends.  Reference context: the captured
train step, /root/reference/models/train.py:163-208."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_nested_branch_runs_in_place_and_replays(cuda, monkeypatch):
    from ldm_amd import graphs as G
    monkeypatch.setenv("LDM_AMD_BRANCH_STREAMS", "capture")
    G.prepare_streams(cuda)
    x = torch.ones(4096, device=cuda)
    y = torch.zeros(4096, device=cuda)
    z = torch.zeros(4096, device=cuda)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    seen = {}
    with G.capture(g):
        origin = torch.cuda.current_stream()
        x.add_(1.0)
        with G.branch(cuda, "outer") as s1:
            seen["outer"] = s1
            y.add_(x, alpha=2.0)
            with G.branch(cuda, "inner") as s2:       # would fork from the branch stream: runs in place
                seen["inner"] = s2
                z.add_(y, alpha=3.0)
        seen["recorded"] = [s.cuda_stream for s in G.captured_side_streams()]
        # no join(s1): capture() must join the outer branch itself before the capture ends
    assert seen["outer"] is not None and seen["outer"].cuda_stream != origin.cuda_stream
    assert seen["inner"] is None
    assert seen["recorded"] == [seen["outer"].cuda_stream]
    x.fill_(1.0), y.zero_(), z.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert float(x[0]) == 2.0 and float(y[0]) == 4.0 and float(z[0]) == 12.0


def test_branch_outside_capture_is_in_place_by_default(cuda, monkeypatch):
    from ldm_amd import graphs as G
    monkeypatch.setenv("LDM_AMD_BRANCH_STREAMS", "capture")
    with G.branch(cuda, "outer") as s:
        assert s is None
