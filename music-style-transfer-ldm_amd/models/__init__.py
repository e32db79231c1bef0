"""Drop-in replacement for the reference's `models` package (config / model / loss / train) whose
hot path runs on hand-written HIP kernels for MI355X (libldm_amd.so)."""
from . import _pathfix  # noqa: F401
