"""The C ABI library: built for gfx950, loads, exports every symbol the header
declares, host-side hashing matches hashlib (no GPU compute calls here)."""
import ctypes
import os
import re
import subprocess

import pytest

from das_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "das_mi355x.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(das_\w+)\(", src, re.M)))


def test_header_and_binding_agree():
    assert header_functions() == sorted(_lib.exported_symbols())


def test_library_exports_every_symbol():
    L = _lib.lib()
    for name in header_functions():
        assert hasattr(L, name), name


def test_library_has_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", _lib.LIB_PATH],
                         capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_host_md5_matches_reference_vectors(golden):
    hv = golden("hash_vectors.json")
    for s, h in hv["md5"]:
        assert _lib.digest_to_hex(_lib.md5_digest(s)) == h
    for parts, h in hv["composite"]:
        if all(len(p) == 32 for p in parts):
            d = [_lib.hex_to_digest(p) for p in parts]
            assert _lib.digest_to_hex(_lib.composite_digest(d)) == h


def test_expression_hasher_api(golden):
    from das_amd.expression_hasher import ExpressionHasher as EH
    hv = golden("hash_vectors.json")
    for t, n, h in hv["terminal"]:
        assert EH.terminal_hash(t, n) == h
    for parts, h in hv["composite"]:
        assert EH.composite_hash(parts) == h
    assert EH.composite_hash("x") == "x"
    # upper-case hex elements are joined as written (expression_hasher.py:33)
    import hashlib
    up = ["AF12F10F9AE2002A1607BA0B47BA8407", "bdfe4e7a431f73386f37c6448afe5840"]
    assert EH.composite_hash(up) == hashlib.md5(" ".join(up).encode()).hexdigest()
    with pytest.raises(ValueError):
        EH.composite_hash(3)
