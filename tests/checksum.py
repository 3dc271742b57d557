"""Order-independent answer checksum (test infrastructure).

The reference's answer is a *set* of assignments, each identified by its
var -> handle mapping (pattern_matcher.py:41-51, 370-384, 741-748).  At
BASELINE sizes no host copy of the rows is practical, so the full-size parity
tests compare, next to the row count, this checksum of the device answer
(das_table_checksum, das_amd/csrc/checksum.hip) with the same function
computed from the generator's own arrays:

    g(v, h)  = splitmix64(d64(h) ^ salt(v)) | 1
    row      = prod over the row's (variable, handle) pairs of g   (mod 2^64)
    checksum = sum over rows of row                                 (mod 2^64)

d64(h) = the handle's first 8 digest bytes as a little-endian integer;
salt(v) = the first 8 bytes of md5("das-var:" + name), little-endian.  The
product makes a row's value independent of column order; because it is a
product, the checksum of a join factors into per-key sums (the closed forms
below compute joins and cross products without enumerating them), while
swapping values between rows changes it.

Three equivalent implementations: pure Python ints (`row_value`, pinned
against oracle row sets in tests/test_closed_forms.py), numpy uint64 arrays
(`g_np`), torch int64 tensors on the GPU (`g_torch`, wrapping arithmetic).
"""
import functools
import hashlib

import numpy as np

M64 = (1 << 64) - 1
C1, C2 = 0xBF58476D1CE4E5B9, 0x94D049BB133111EB


@functools.lru_cache(maxsize=None)
def var_salt(name):
    return int.from_bytes(hashlib.md5(b"das-var:" + name.encode()).digest()[:8], "little")


def d64_hex(handle):
    return int.from_bytes(bytes.fromhex(handle)[:8], "little")


def d64_text(text):
    """d64 of the atom whose hashed string is `text` (a node "Type name")."""
    return int.from_bytes(hashlib.md5(text.encode()).digest()[:8], "little")


# -- pure Python ------------------------------------------------------------
def mix64(z):
    z = ((z ^ (z >> 30)) * C1) & M64
    z = ((z ^ (z >> 27)) * C2) & M64
    return z ^ (z >> 31)


def g(name, d64):
    return mix64(d64 ^ var_salt(name)) | 1


def row_value(mapping):
    """mapping: {variable name: handle} (an OrderedAssignment.mapping)."""
    h = 1
    for v, handle in mapping.items():
        h = (h * g(v, d64_hex(handle))) & M64
    return h


def rows_checksum(mappings):
    return sum(row_value(m) for m in mappings) & M64


# -- numpy (uint64 arithmetic wraps) -----------------------------------------
def mix64_np(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(C1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(C2)
    return z ^ (z >> np.uint64(31))


def g_np(name, d64):
    """g over an array of d64 values."""
    return mix64_np(np.asarray(d64, dtype=np.uint64) ^ np.uint64(var_salt(name))) | np.uint64(1)


def sum_np(x):
    return int(np.sum(np.asarray(x, dtype=np.uint64), dtype=np.uint64))


def prod_np(*xs):
    out = np.uint64(1)
    with np.errstate(over="ignore"):
        for x in xs:
            out = out * np.asarray(x, dtype=np.uint64)
    return out


def group_sum_np(keys, vals, n):
    """out[k] = sum of vals where keys == k (mod 2^64), k < n."""
    out = np.zeros(n, dtype=np.uint64)
    np.add.at(out, np.asarray(keys, dtype=np.int64), np.asarray(vals, dtype=np.uint64))
    return out


# -- torch (int64 arithmetic wraps; logical shifts by masking) ---------------
def _s64(x):
    return x - (1 << 64) if x >= (1 << 63) else x


def mix64_torch(z):
    z = z ^ ((z >> 30) & ((1 << 34) - 1))
    z = z * _s64(C1)
    z = z ^ ((z >> 27) & ((1 << 37) - 1))
    z = z * _s64(C2)
    return z ^ ((z >> 31) & ((1 << 33) - 1))


def g_torch(name, d64):
    """d64: int64 tensor (the digest words reinterpreted)."""
    return mix64_torch(d64 ^ _s64(var_salt(name))) | 1


def sum_torch(x):
    return int(x.sum().item()) & M64


def d64_from_words_torch(words):
    """(n, 4) int32/uint32 little-endian digest words -> int64 d64."""
    import torch
    w = words.to(torch.int64) & 0xFFFFFFFF
    return w[:, 0] | (w[:, 1] << 32)


# -- the device answer --------------------------------------------------------
def answer_checksum(ans):
    """(checksum, rows) of a PatternMatchingAnswer evaluated on a HipDB:
    das_table_checksum over each of its ordered tables."""
    from das_amd.pattern_matcher import pattern_matcher as pm
    total, rows = 0, 0
    db = ans._db
    if db is None:
        return 0, 0
    for t in db.rel_local_tables(ans._relation()):
        s, bad = t.checksum([var_salt(pm._var_name(v)) for v in t.vars])
        assert bad == 0, "table holds values that are not atom ids"
        total = (total + s) & M64
        rows += t.nrows
    return total, rows
