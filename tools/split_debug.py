"""Debug: which outputs / counters of a split-K launch are left unwritten / nonzero."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "music-style-transfer-ldm_amd"))
import torch  # noqa: E402
from ldm_amd import _lib as L, ops  # noqa: E402

dev = torch.device("cuda:0")
for (B, Cin, H, W, Cout, k, s, tr, pl) in [(8, 512, 2, 8, 256, 3, 2, True, (1, 1, 1, 4, 4)),
                                           (8, 512, 2, 8, 512, 3, 1, False, (1, 1, 1, 4, 4)),
                                           (8, 512, 2, 8, 256, 3, 2, True, (1, 1, 1, 1, 2))]:
    desc = ops.make_desc(B, Cin, H, W, Cout, k, k, s, 1, 1 if tr else 0, tr)
    plan = ops.get_plan(desc, force=pl)
    w = torch.randn((Cin, Cout, k, k) if tr else (Cout, Cin, k, k), device=dev) * 0.05
    wb = ops.packed_weight(w, desc, plan)
    x = torch.randn(B, Cin, H, W, device=dev)
    y = torch.full((B, Cout, desc.Hout, desc.Wout), float("nan"), device=dev)
    ws = torch.zeros(int(plan.ws_floats), device=dev)
    L.call("ldm_conv_forward_ws", ctypes.byref(desc), ctypes.byref(plan), x.data_ptr(), wb.data_ptr(), None,
           y.data_ptr(), ws.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    bad = torch.isnan(y)
    tile = 32
    nph = 4 if tr else 1
    nq = B * (H * W if tr else desc.Hout * desc.Wout)
    ntiles = -(-Cout // tile) * -(-nq // tile) * nph
    cnt = ws[:ntiles].view(torch.int32).cpu()
    print(desc.key(), pl, "unwritten", int(bad.sum()), "of", y.numel(), "nonzero counters", int((cnt != 0).sum()),
          "of", ntiles, "values", sorted(set(cnt.tolist()))[:10])
    if bad.any():
        idx = bad.nonzero()
        print("  unwritten b:", sorted(set(idx[:, 0].tolist())), "c range", int(idx[:, 1].min()), int(idx[:, 1].max()),
              "oy", sorted(set(idx[:, 2].tolist())), "ox", sorted(set(idx[:, 3].tolist()))[:20])
        # parity classes
        par = sorted(set(((idx[:, 2] % 2) * 2 + idx[:, 3] % 2).tolist()))
        print("  phases", par)
    y2 = ops.conv_forward(x, w, None, stride=s, padding=1, transposed=tr, output_padding=1 if tr else 0,
                          plan=ops.get_plan(desc, force=(2, 1, 1, 1, 1)))
    ok = ~bad
    print("  max err on written", float((y[ok] - y2[ok]).abs().max()))
