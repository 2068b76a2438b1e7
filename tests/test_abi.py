"""CPU-side checks of the C ABI boundary: the library loads and exports every declared symbol."""
import os
import re
import subprocess

import numpy as np
from zonos_vibes_amd import _lib
from zonos_vibes_amd import synthetic as syn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "zonos_hip.h")


def declared_symbols(header=HEADER):
    src = open(header).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(zmi_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_binding_table():
    assert declared_symbols() == _lib.EXPORTED


def test_library_exports_only_declared_symbols():
    """Every exported zmi_ symbol is declared in the header (no undeclared or leftover diagnostic entry points)."""
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert set(re.findall(r"\s[TW]\s+(zmi_\w+)", out)) <= set(declared_symbols())


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\s[TW]\s+(zmi_\w+)", out))
    assert set(declared_symbols()) <= exported


def test_library_is_gfx950_code_object():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_struct_layouts():
    import ctypes
    assert ctypes.sizeof(_lib.Sampling) == 48
    assert ctypes.sizeof(_lib.GemvArgs) % 8 == 0


def test_synthetic_stream_is_reproducible():
    sp = syn.Spec("t", (4, 8), "bf16", 0.5, 1.0)
    a = syn.materialize_np(sp, 3)
    b = syn.materialize_np(sp, 3)
    assert a.dtype == np.uint16 and (a == b).all()
    v = syn.bf16_bits_to_f32(a)
    assert 0.49 < v.min() and v.max() < 1.51
    # chunked generation equals one-shot generation
    key = syn.tensor_key(0, "x")
    full = syn.uniform_f32(key, 1000, 1.0)
    part = np.concatenate([syn.uniform_f32(key, 300, 1.0), syn.uniform_f32(key, 700, 1.0, start=300)])
    assert (full == part).all()
