"""Host-side synthetic-input helpers (CPU)."""
import numpy as np

from das_amd import synthetic


def test_numbered_leaves_equal_python_strings():
    for n in (0, 1, 9, 10, 11, 99, 100, 1234):
        buf, off = synthetic.numbered_leaves("Concept n", n)
        got = [bytes(buf[int(off[i]):int(off[i + 1])]).decode() for i in range(n)]
        assert got == [f"Concept n{i}" for i in range(n)]
        assert off[0] == 0 and len(off) == n + 1


def test_numbered_leaves_match_build_arrays_layout():
    arrays, _ = synthetic.build_arrays(["T0"], [("Concept", "n", 123)], [])
    buf, off = synthetic.numbered_leaves("Concept n", 123)
    nt = len(arrays.type_names)
    base = int(arrays.leaf_off[nt])
    assert np.array_equal(arrays.leaf_bytes[base:], buf)
    assert np.array_equal(arrays.leaf_off[nt:] - base, off)
