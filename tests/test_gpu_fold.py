"""The reverse loop's folded cross-attention, kernel by kernel (csrc/misc.hip).

ldm_attention_fold_keys: kf [B,heads,S,E] = scale * Wq_h^T K_h and bf [B,heads,S] = scale * bq_h^T K_h (fp64
sums, one rounding), at the reverse loop's key counts and others (S % 4 == 0: four keys per thread with the
bias as an extra column; S = 10: the one-output-per-thread kernel); ldm_attention_folded: z [B,L,E] -> softmax((Wq z + bq) * scale)^T K) V, token-major, against float64
torch of the unfolded attention (model.py:140-153, nn.MultiheadAttention's Q in-projection + score product).
"""
import numpy as np
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu


def npy(t):
    return t.detach().double().cpu().numpy()


@pytest.mark.parametrize("B,E,S", [(8, 256, 64), (8, 512, 16), (2, 256, 12), (3, 512, 40), (2, 256, 10)])
def test_fold_keys_vs_float64(cuda, B, E, S):
    from ldm_amd import _lib as L
    heads, d = 4, E // 4
    g = torch.Generator().manual_seed(E + S + B)
    kv = torch.randn(B, 2 * E, S, generator=g)
    wq = torch.randn(E, E, generator=g) / E ** 0.5
    bq = torch.randn(E, generator=g) * 0.1
    scale = float(np.sqrt(1.0 / d))
    kvd, wqd, bqd = kv.to(cuda), wq.to(cuda), bq.to(cuda)
    kf = torch.full((B, heads, S, E), float("nan"), device=cuda)
    bf = torch.full((B, heads, S), float("nan"), device=cuda)
    L.call("ldm_attention_fold_keys", kvd.data_ptr(), wqd.data_ptr(), bqd.data_ptr(), B, E, heads, S, scale,
           kf.data_ptr(), bf.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    K = kv.double()[:, :E].view(B, heads, d, S)              # K_h [d, S]
    W = wq.double().view(heads, d, E)                         # Wq_h [d, E]
    kf_ref = scale * torch.einsum("hce,bhcs->bhse", W, K)
    bf_ref = scale * torch.einsum("hc,bhcs->bhs", bq.double().view(heads, d), K)
    assert rel_err(npy(kf), kf_ref.numpy()) < 1e-6
    assert rel_err(npy(bf), bf_ref.numpy()) < 1e-6


@pytest.mark.parametrize("B,E,L,S", [(8, 256, 64, 64), (8, 512, 16, 16), (2, 256, 16, 16)])
def test_folded_attention_vs_float64(cuda, B, E, L, S):
    from ldm_amd import _lib as L_
    heads, d = 4, E // 4
    g = torch.Generator().manual_seed(7 * E + L)
    z = torch.randn(B, L, E, generator=g)
    kv = torch.randn(B, 2 * E, S, generator=g)
    wq = torch.randn(E, E, generator=g) / E ** 0.5
    bq = torch.randn(E, generator=g) * 0.1
    scale = float(np.sqrt(1.0 / d))
    st = torch.cuda.current_stream().cuda_stream
    zd, kvd, wqd, bqd = z.to(cuda), kv.to(cuda), wq.to(cuda), bq.to(cuda)
    kf = torch.empty((B, heads, S, E), device=cuda)
    bf = torch.empty((B, heads, S), device=cuda)
    out = torch.full((B, L, E), float("nan"), device=cuda)
    L_.call("ldm_attention_fold_keys", kvd.data_ptr(), wqd.data_ptr(), bqd.data_ptr(), B, E, heads, S, scale,
            kf.data_ptr(), bf.data_ptr(), st)
    L_.call("ldm_attention_folded", zd.data_ptr(), kvd.data_ptr(), kf.data_ptr(), bf.data_ptr(), out.data_ptr(), B, E,
            heads, L, S, st)
    torch.cuda.synchronize()
    q = torch.einsum("oe,ble->blo", wq.double(), z.double()) + bq.double()    # [B, L, E]
    qh = q.view(B, L, heads, d).permute(0, 2, 1, 3)                            # [B, h, L, d]
    K = kv.double()[:, :E].view(B, heads, d, S)
    V = kv.double()[:, E:].view(B, heads, d, S)
    p = torch.softmax(torch.einsum("bhld,bhds->bhls", qh * scale, K), dim=-1)
    o = torch.einsum("bhls,bhds->bhld", p, V).permute(0, 2, 1, 3).reshape(B, L, E)
    assert rel_err(npy(out), o.numpy()) < 1e-5
