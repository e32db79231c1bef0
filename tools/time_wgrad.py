"""Time the 16-bit weight gradient of the train step's large-plane layers (B = 32, 1x128x512 mels):
the double-rate form (wgrad_lp_kernel) against the tap-shared form (LDM_WGRAD_LP=0).
python tools/time_wgrad.py [bf16|fp16]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "music-style-transfer-ldm_amd")]
import torch  # noqa: E402

from ldm_amd import ops  # noqa: E402

# (name, B, Cin, H, W, Cout, k, s, p, op, transposed)
LAYERS = [
    ("vae_enc2 k3s2 64->128", 32, 64, 64, 256, 128, 3, 2, 1, 0, False),
    ("vae_enc3 k3s2 128->32", 32, 128, 32, 128, 32, 3, 2, 1, 0, False),
    ("vae_dec1 convT k4 32->128", 32, 32, 16, 64, 128, 4, 2, 1, 0, True),
    ("vae_dec2 convT k4 128->64", 32, 128, 32, 128, 64, 4, 2, 1, 0, True),
    ("style_enc2 k3s2 64->128", 32, 64, 64, 256, 128, 3, 2, 1, 0, False),
    ("style_enc3 k3s2 128->256", 32, 128, 32, 128, 256, 3, 2, 1, 0, False),
    ("style_enc4 k3s2 256->256", 32, 256, 16, 64, 256, 3, 2, 1, 0, False),
    ("unet_enc1 k3s1 32->64", 32, 32, 16, 64, 64, 3, 1, 1, 0, False),
    ("unet_dec1 k3s1 64->32", 32, 64, 16, 64, 32, 3, 1, 1, 0, False),
]


def time_ms(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    dt = 1 if (len(sys.argv) > 1 and sys.argv[1] == "fp16") else 2
    dev = torch.device("cuda:0")
    tot = {"lp": 0.0, "ts": 0.0}
    for name, B, Cin, H, W, Cout, k, s, p, op, tr in LAYERS:
        desc = ops.make_desc(B, Cin, H, W, Cout, k, k, s, p, op, tr)
        x = torch.randn(B, Cin, H, W, device=dev)
        Ho = (H - 1) * s - 2 * p + k + op if tr else (H + 2 * p - k) // s + 1
        Wo = (W - 1) * s - 2 * p + k + op if tr else (W + 2 * p - k) // s + 1
        dy = torch.randn(B, Cout, Ho, Wo, device=dev)
        flops = 2.0 * B * Cin * Cout * k * k * (H * W if tr else Ho * Wo)
        res = {}
        for form in ("lp", "ts"):
            os.environ["LDM_WGRAD_LP"] = "1" if form == "lp" else "0"
            res[form] = time_ms(lambda: ops.conv_backward_weight(x, dy, desc, dtype=dt))
            tot[form] += res[form]
        a = ops.conv_backward_weight(x, dy, desc, dtype=dt)
        os.environ["LDM_WGRAD_LP"] = "1"
        b = ops.conv_backward_weight(x, dy, desc, dtype=dt)
        err = float((a - b).abs().max() / b.abs().max())
        print(f"{name:28s} lp {res['lp'] * 1e3:8.1f} us ({flops / res['lp'] / 1e9:7.1f} TF/s)   "
              f"tap-shared {res['ts'] * 1e3:8.1f} us   rel diff {err:.1e}", flush=True)
    print(f"total lp {tot['lp'] * 1e3:.1f} us, tap-shared {tot['ts'] * 1e3:.1f} us")


if __name__ == "__main__":
    main()
