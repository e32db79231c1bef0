"""CPU: the C-ABI library loads, exports every entry point include/ldm_capi.h declares, and the ctypes
mirrors of its structs have the C layout (checked against a gcc-compiled probe of the header)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ldm_capi.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ldm_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_every_declared_symbol():
    from ldm_amd import _lib
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.ldm_capi_version() == 1


def test_ctypes_signature_table_matches_header():
    from ldm_amd import _lib
    assert set(_lib.SIGNATURES) == set(header_functions())


def test_struct_layout_matches_c(tmp_path):
    from ldm_amd import _lib as L
    probe = tmp_path / "probe.c"
    probe.write_text(f'#include "{HEADER}"\n#include <stdio.h>\n#include <stddef.h>\n'
                     "int main(void){printf(\"%zu %zu %zu %zu %zu %zu %zu\\n\", sizeof(ldm_conv_desc), "
                     "sizeof(ldm_epilogue), sizeof(ldm_conv_plan), sizeof(ldm_unet_shape), sizeof(ldm_unet_weights), "
                     "offsetof(ldm_unet_weights, ca_wq), offsetof(ldm_unet_weights, t_freqs)); return 0;}\n")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", str(probe), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = [ctypes.sizeof(L.ConvDesc), ctypes.sizeof(L.Epilogue), ctypes.sizeof(L.ConvPlan),
            ctypes.sizeof(L.UNetShape), ctypes.sizeof(L.UNetWeights), L.UNetWeights.ca_wq.offset,
            L.UNetWeights.t_freqs.offset]
    assert got == want


def test_errors_are_reported_not_crashes():
    from ldm_amd import _lib as L
    d = L.ConvDesc(1, 8, 4, 4, 8, 5, 5, 3, 3, 1, 1, 0, 0)   # wrong Hout
    p = L.ConvPlan()
    with pytest.raises(L.LDMError, match="output size"):
        L.call("ldm_conv_make_plan", ctypes.byref(d), ctypes.byref(p))
