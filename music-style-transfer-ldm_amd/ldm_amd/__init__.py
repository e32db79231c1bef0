"""ldm_amd — MI355X-native (gfx950) kernels of the latent-diffusion hot path behind a C ABI
(include/ldm_capi.h, libldm_amd.so), plus the host-side runtime that binds torch tensors to it."""
from . import _lib, ops  # noqa: F401
from .autotune import load_tuned as _load_tuned

_load_tuned()
