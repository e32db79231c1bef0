"""Per-layer plan autotuner for the implicit-GEMM conv kernel.

For a conv descriptor, every valid (kind, tm, tn, wk) instance is timed with HIP events on the current
stream (same process, interleaved rounds, median) and the fastest is recorded.  Results persist in
tuned_plans.json next to the package (committed, so a fresh GPU box starts tuned) and are applied
through ops._PLAN_OVERRIDE, which both the per-layer path and the fused UNet engine honour.
"""
import ctypes
import json
import os

import torch

from . import _lib as L
from . import ops
from .graphs import capture

TUNED_PATH = os.path.join(L.PKG_ROOT, "tuned_plans.json")


def _tiles(desc, kind, tm, tn):
    tile = 32 if kind == 1 else 16
    bm, bn = tile * tm, tile * tn
    ph = 4 if desc.transposed and desc.stride == 2 else 1
    nq = desc.B * (desc.Hin * desc.Win if ph == 4 else desc.Hout * desc.Wout)
    return -(-desc.Cout // bm) * -(-nq // bn) * ph


def candidates(desc, min_waves=256, max_waves=16384):
    """Valid (kind, tm, tn, wk, ks) plans whose grid holds between min_waves and max_waves waves."""
    out = []
    if desc.Cout <= 64 and desc.layout == 0:
        out.append((0, 1, 1, 1, 1))
    for kind in (1, 2):
        for tm in (1, 2):
            for tn in (1, 2):
                tiles = _tiles(desc, kind, tm, tn)
                for wk in (1, 2, 4, 8):
                    bal = (-1, -2, -4) if (desc.transposed and desc.stride == 2) else ()
                    for ks in (1, 2, 4, 8, 16) + bal:
                        if not min_waves <= tiles * wk * (abs(ks) * (9 if ks < 0 else 4)) // 4 <= max_waves:
                            continue
                        p = L.ConvPlan()
                        rc = L.load().ldm_conv_make_plan_forced(ctypes.byref(desc), kind, tm, tn, wk, ks,
                                                                ctypes.byref(p))
                        if rc == 0:
                            out.append((kind, tm, tn, wk, ks))
    return out


def time_plan(desc, cand, x, w, y, reps=30):
    plan = ops.get_plan(desc, force=cand)
    wbuf = ops.packed_weight(w, desc, plan, owner=w, tag=("tune", cand))
    ep = L.Epilogue()
    ep.act = 1
    st = torch.cuda.current_stream()
    lib = L.load()
    ws = torch.zeros(max(1, int(plan.ws_floats)), device=x.device)
    args = (ctypes.byref(desc), ctypes.byref(plan), x.data_ptr(), wbuf.data_ptr(), ctypes.byref(ep), y.data_ptr(),
            ws.data_ptr(), st.cuda_stream)
    for _ in range(3):
        L.check(lib.ldm_conv_forward_ws(*args), "tune")
    torch.cuda.synchronize()
    # reps dependent launches captured in one hipGraph and replayed: device time per launch including
    # the kernel boundary, without the host launch cost that dominates eager timing of short kernels
    cap = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with capture(g, stream=cap):
        a2 = args[:-1] + (cap.cuda_stream,)
        for _ in range(reps):
            lib.ldm_conv_forward_ws(*a2)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    g.replay()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def tune_desc(desc, device, rounds=3, verbose=False):
    w_shape = (desc.Cin, desc.Cout, desc.kh, desc.kw) if desc.transposed else (desc.Cout, desc.Cin, desc.kh, desc.kw)
    w = torch.randn(w_shape, device=device) * 0.05
    x = torch.randn(desc.B, desc.Cin, desc.Hin, desc.Win, device=device)
    y = torch.empty(desc.B, desc.Cout, desc.Hout, desc.Wout, device=device)
    cands = candidates(desc)
    times = {c: [] for c in cands}
    for _ in range(rounds):
        for c in cands:
            times[c].append(time_plan(desc, c, x, w, y))
    med = {c: sorted(v)[len(v) // 2] for c, v in times.items()}
    best = min(med, key=med.get)
    if verbose:
        print(desc.key(), "best", best, f"{med[best]:.2f}us", "default",
              f"{med.get(tuple(ops.get_plan(desc).key()), float('nan')):.2f}us")
    return best, med


def load_tuned(path=TUNED_PATH):
    if not os.path.exists(path):
        return 0
    with open(path) as f:
        tab = json.load(f)
    n = 0
    for k, v in tab.get("plans", {}).items():
        ops._PLAN_OVERRIDE[tuple(int(s) for s in k.split(","))] = tuple(v) + (1,) * (5 - len(v))
        n += 1
    return n


def save_tuned(results, path=TUNED_PATH, meta=None):
    tab = {"plans": {}, "meta": meta or {}}
    if os.path.exists(path):
        with open(path) as f:
            tab = json.load(f)
        tab.setdefault("plans", {})
    for key, best in results.items():
        tab["plans"][",".join(str(int(s)) for s in key)] = list(best)
    with open(path, "w") as f:
        json.dump(tab, f, indent=1, sort_keys=True)
