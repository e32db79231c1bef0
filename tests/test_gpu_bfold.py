"""The reverse loop's bottleneck on CA1's folded values (csrc/bfold.hip; reference model.py:214-217 = CA1 ->
bottleneck conv -> ReLU) against float64 of the literal order: the folded attention's probabilities, the values
folded into the (out-projection-folded) bottleneck weights, and the per-step contraction, on random operands at
the canonical 2 x 8 plane.  Tolerance: max |y - y64| <= 1e-5 max |y64| (fp32 against float64; the north_star
bound is 1e-4).  The end-to-end loop with the fold is pinned by tests/test_gpu_bench_config.py (the bench object
against the oracle)."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_err

pytestmark = pytest.mark.gpu


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def _operands(B, seed):
    g = torch.Generator().manual_seed(seed)
    z4 = torch.rand(B, 16, 512, generator=g)                          # token-major (NHWC on the 2 x 8 plane)
    kf = torch.randn(B, 4, 16, 512, generator=g) * 0.05
    bf = torch.randn(B, 4, 16, generator=g) * 0.1
    kv = torch.randn(B, 1024, 16, generator=g)
    wf = torch.randn(512, 512, 3, 3, generator=g) / np.sqrt(4608.0)
    pb = torch.randn(16, 512, generator=g) * 0.1                      # position-major bias [l][co]
    return z4, kf, bf, kv, wf, pb


def _reference64(z4, kf, bf, kv, wf, pb):
    z, kf, bf, kv, wf, pb = (t.double() for t in (z4, kf, bf, kv, wf, pb))
    B = z.shape[0]
    scores = torch.einsum("ble,bhse->bhls", z, kf) + bf[:, :, None, :]
    p = torch.softmax(scores, dim=-1)                                 # [B, 4, 16, 16]
    v = kv[:, 512:, :].reshape(B, 4, 128, 16)                         # V[b, h, d, s]
    a = torch.einsum("bhls,bhds->blhd", p, v).reshape(B, 16, 512)    # concat_h P_h V_h, token-major
    x = a.permute(0, 2, 1).reshape(B, 512, 2, 8)
    y = F.conv2d(x, wf, padding=1) + pb.t().reshape(1, 512, 2, 8)
    return p, torch.relu(y).permute(0, 2, 3, 1).reshape(B, 16, 512)


@pytest.mark.parametrize("B", [1, 3, 8])
def test_bneck_fold_matches_float64(cuda, B):
    from ldm_amd import _lib as L
    ops = _operands(B, 100 + B)
    p64, y64 = _reference64(*ops)
    z4, kf, bf, kv, wf, pb = (t.to(cuda).contiguous() for t in ops)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = torch.empty(B, 4, 16, 16, device=cuda)
    u = torch.empty(B, 512, 576, device=cuda)
    y = torch.empty(B, 16, 512, device=cuda)
    L.call("ldm_attention_folded_probs", _ptr(z4), _ptr(kf), _ptr(bf), _ptr(p), B, 512, 4, 16, 16, st)
    L.call("ldm_bneck_fold_values", _ptr(wf), _ptr(kv), _ptr(u), B, st)
    L.call("ldm_bneck_pv", _ptr(u), _ptr(p), _ptr(pb), _ptr(y), B, 0, st)
    torch.cuda.synchronize()
    assert rel_err(p.cpu().numpy(), p64.numpy()) < 1e-5
    # U against float64 of its definition
    v = ops[3].double()[:, 512:, :].reshape(B, 4, 128, 16)
    w = ops[4].double().reshape(512, 4, 128, 9)
    u64 = torch.einsum("ohdt,bhds->bohts", w, v).permute(0, 1, 3, 2, 4).reshape(B, 512, 576)
    assert rel_err(u.cpu().numpy(), u64.numpy()) < 1e-5
    err = rel_err(y.cpu().numpy(), y64.numpy())
    print(f"B={B}: bottleneck on folded values vs float64 {err:.2e}")
    assert err < 1e-5
    # bitwise rerun (fixed-order sums)
    y2 = torch.empty_like(y)
    L.call("ldm_bneck_pv", _ptr(u), _ptr(p), _ptr(pb), _ptr(y2), B, 0, st)
    torch.cuda.synchronize()
    assert torch.equal(y, y2)


@pytest.mark.parametrize("dt,t16", [(1, torch.float16), (2, torch.bfloat16)])
def test_bneck_pv_rounds_output_to_16_bits(cuda, dt, t16):
    """Inside autocast (a 16-bit sampling loop) the bottleneck output is rounded to the region's type, as the
    reference's autocast conv returns a 16-bit tensor (the relu of a rounded value is exactly representable)."""
    from ldm_amd import _lib as L
    B = 2
    z4, kf, bf, kv, wf, pb = (t.to(cuda).contiguous() for t in _operands(B, 7))
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = torch.empty(B, 4, 16, 16, device=cuda)
    u = torch.empty(B, 512, 576, device=cuda)
    y32 = torch.empty(B, 16, 512, device=cuda)
    y16 = torch.empty(B, 16, 512, device=cuda)
    L.call("ldm_attention_folded_probs", _ptr(z4), _ptr(kf), _ptr(bf), _ptr(p), B, 512, 4, 16, 16, st)
    L.call("ldm_bneck_fold_values", _ptr(wf), _ptr(kv), _ptr(u), B, st)
    L.call("ldm_bneck_pv", _ptr(u), _ptr(p), _ptr(pb), _ptr(y32), B, 0, st)
    L.call("ldm_bneck_pv", _ptr(u), _ptr(p), _ptr(pb), _ptr(y16), B, dt, st)
    torch.cuda.synchronize()
    assert torch.equal(y16, y16.to(t16).float())
    assert rel_err(y16.cpu().numpy(), y32.cpu().numpy()) < (1e-3 if dt == 1 else 8e-3)


def test_bneck_fold_applies_at_the_bench_shape():
    from ldm_amd import _lib as L
    lib = L.load()
    assert lib.ldm_bneck_fold_supported(8, 16, 64) == 1
    assert lib.ldm_bneck_fold_supported(9, 16, 64) == 0       # U would outgrow W'
    assert lib.ldm_bneck_fold_supported(8, 16, 128) == 0      # not the 2 x 8 plane


@pytest.mark.parametrize("B", [1, 8])
def test_ca1_probs_kernel_matches_float64(cuda, B):
    """The reverse loop's CA1 probabilities kernel (ca1_probs_kernel) against float64 and against the generic
    attention kernel's probabilities-only instance."""
    from ldm_amd import _lib as L
    ops = _operands(B, 300 + B)
    p64, _ = _reference64(*ops)
    z4, kf, bf, kv, wf, pb = (t.to(cuda).contiguous() for t in ops)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = torch.empty(B, 4, 16, 16, device=cuda)
    p2 = torch.empty(B, 4, 16, 16, device=cuda)
    L.call("ldm_ca1_probs", _ptr(z4), _ptr(kf), _ptr(bf), _ptr(p), B, st)
    L.call("ldm_attention_folded_probs", _ptr(z4), _ptr(kf), _ptr(bf), _ptr(p2), B, 512, 4, 16, 16, st)
    torch.cuda.synchronize()
    assert rel_err(p.cpu().numpy(), p64.numpy()) < 1e-5
    assert rel_err(p.cpu().numpy(), p2.cpu().numpy()) < 1e-6
