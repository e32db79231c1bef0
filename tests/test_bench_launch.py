"""CPU: bench.py as its own N-rank launcher (`bench.py --gpus N` without torchrun).

launch_ranks() drives a stub worker over gloo here; the same function starts the real bench ranks (RCCL) on a
node.  The refusal paths are checked on the real script: with fewer visible HIP devices than --gpus (this
container has none) it exits non-zero before any GPU call, and a --gpus / WORLD_SIZE mismatch is refused
instead of running one rank."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")

STUB = r'''
import os, sys, torch, torch.distributed as dist
dist.init_process_group("gloo")                     # env:// rendezvous from the launcher's variables
r, w = dist.get_rank(), dist.get_world_size()
t = torch.tensor([float(r + 1)])
dist.all_reduce(t)
assert int(os.environ["RANK"]) == r and int(os.environ["LOCAL_RANK"]) == r and os.environ["MASTER_ADDR"] == "127.0.0.1"
with open(os.path.join(sys.argv[1], f"rank{r}.txt"), "w") as f:
    f.write(f"{r} {w} {int(t.item())}")
dist.destroy_process_group()
if len(sys.argv) > 2 and int(sys.argv[2]) == r:
    sys.exit(7)
'''


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


@pytest.mark.parametrize("n", [2, 3])
def test_launch_ranks_stub_gloo(tmp_path, n):
    bench = _bench()
    stub = tmp_path / "stub.py"
    stub.write_text(STUB)
    env = {k: v for k, v in os.environ.items() if k not in ("MASTER_PORT", "WORLD_SIZE", "RANK", "LOCAL_RANK")}
    rc = bench.launch_ranks(n, [sys.executable, str(stub), str(tmp_path)], env=env)
    assert rc == 0
    got = sorted((tmp_path / f"rank{r}.txt").read_text() for r in range(n))
    assert got == [f"{r} {n} {n * (n + 1) // 2}" for r in range(n)]


def test_launch_ranks_reports_failing_rank(tmp_path):
    bench = _bench()
    stub = tmp_path / "stub.py"
    stub.write_text(STUB)
    env = {k: v for k, v in os.environ.items() if k not in ("MASTER_PORT", "WORLD_SIZE", "RANK", "LOCAL_RANK")}
    rc = bench.launch_ranks(2, [sys.executable, str(stub), str(tmp_path), "1"], env=env, grace_s=5.0)
    assert rc == 7


def _run_bench(args, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=300)


def test_bench_gpus2_refuses_without_devices():
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("two or more HIP devices visible")
    p = _run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert p.returncode != 0
    assert "HIP device(s) visible" in p.stderr, p.stderr[-2000:]


def test_bench_world_mismatch_refused():
    p = _run_bench(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE=1" in p.stderr, p.stderr[-2000:]
