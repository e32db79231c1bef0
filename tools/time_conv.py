"""Time the 16-bit forward and data-gradient convolutions of the train step's large-plane layers (B = 32,
1x128x512 mels) with the plan the train step picks (tiled kind 3 where it applies).
python tools/time_conv.py [bf16|fp16]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "music-style-transfer-ldm_amd")]
import torch  # noqa: E402

from ldm_amd import ops  # noqa: E402
from time_wgrad import LAYERS, time_ms  # noqa: E402

EXTRA = [("vae_dec3 convT k4 64->1", 32, 64, 64, 256, 1, 4, 2, 1, 0, True),
         ("vae_enc1 k3s2 1->64", 32, 1, 128, 512, 64, 3, 2, 1, 0, False),
         ("style_enc5 k3s2 256->256", 32, 256, 8, 32, 256, 3, 2, 1, 0, False)]


def main():
    dt = 1 if (len(sys.argv) > 1 and sys.argv[1] == "fp16") else 2
    dev = torch.device("cuda:0")
    tot = 0.0
    for name, B, Cin, H, W, Cout, k, s, p, op, tr in LAYERS + EXTRA:
        desc = ops.make_desc(B, Cin, H, W, Cout, k, k, s, p, op, tr)
        x = torch.randn(B, Cin, H, W, device=dev)
        w = torch.randn((Cin, Cout, k, k) if tr else (Cout, Cin, k, k), device=dev) * 0.05
        y = ops.conv_forward(x, w, None, stride=s, padding=p, transposed=tr, output_padding=op, dtype=dt)
        dy = torch.randn_like(y)
        flops = 2.0 * B * Cin * Cout * k * k * (H * W if tr else desc.Hout * desc.Wout)
        byts = 4.0 * (x.numel() + y.numel())
        tf = ops.time_ms if hasattr(ops, "time_ms") else None
        t_f = time_ms(lambda: ops.conv_forward(x, w, None, stride=s, padding=p, transposed=tr, output_padding=op,
                                               dtype=dt, out=y))
        t_d = time_ms(lambda: ops.conv_backward_data(dy, w, desc, dtype=dt))
        pf = ops.tiled_plan(desc, dt) or ops.get_plan(desc)
        pd = ops.tiled_plan(ops.dual_desc(desc), dt) or ops.get_plan(ops.dual_desc(desc))
        tot += t_f + t_d
        print(f"{name:28s} fwd {t_f * 1e3:7.1f} us ({flops / t_f / 1e9:6.1f} TF/s, {byts / t_f / 1e6:6.0f} GB/s, kind {pf.kind})"
              f"  dgrad {t_d * 1e3:7.1f} us ({flops / t_d / 1e9:6.1f} TF/s, kind {pd.kind})", flush=True)
        del tf
    print(f"total fwd+dgrad {tot * 1e3:.1f} us")


if __name__ == "__main__":
    main()
