"""The C builder of answer objects (das_amd._assign, csrc/pyassign.c) against
the Python classes' own assign() / freeze() (pattern_matcher.py:73-262):
same mapping / symbols / values / variables / frozen / hash, same set, and
str(set) formatting identical to the interpreter's.  CPU only: the tables are
host doubles with the das_table fetch surface."""
import numpy as np
import pytest

from das_amd.pattern_matcher import pattern_matcher as pm

pytest.importorskip("das_amd._assign")


class _T:
    def __init__(self, kind, vars_, cols):
        self.kind, self.vars, self.cols, self.members = kind, tuple(vars_), cols, None
        self.nrows = cols.shape[1]

    def fetch(self, row0=0, nrows=None):
        n = self.nrows - row0 if nrows is None else min(nrows, self.nrows - row0)
        return self.cols[:, row0:row0 + n].copy()


class _DB:
    def rel_local_tables(self, rel):
        return rel

    def hex_of(self, ids):
        return ["%032x" % (int(i) * 2654435761 % (1 << 128)) for i in np.asarray(ids).ravel()]


def _both(tables, limit=None):
    fast = pm._materialize(_DB(), tables, limit)
    saved = pm._assign
    pm._assign = None
    try:
        slow = pm._materialize(_DB(), tables, limit)
    finally:
        pm._assign = saved
    return fast, slow


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 6])
def test_ordered_objects_equal_python_built(k):
    rng = np.random.default_rng(k)
    cols = rng.integers(0, 300, size=(k, 3000)).astype(np.uint32)
    cols = np.unique(cols.T, axis=0).T.copy()
    vs = [pm._vid(f"$o{k}_{i}") for i in range(k)]
    fast, slow = _both([_T(0, vs, cols)])
    assert len(fast) == len(slow) == cols.shape[1]
    assert fast == slow
    by_hash = {a.hash: a for a in slow}
    for a in fast:
        b = by_hash[a.hash]
        assert type(a) is pm.OrderedAssignment
        assert (a.mapping, a.values, a.variables, a.frozen) == (b.mapping, b.values, b.variables, b.frozen)
        assert repr(a) == repr(b)
    assert pm._assign.format_set(fast, pm.OrderedAssignment) == str(fast)


@pytest.mark.parametrize("k", [2, 3])
def test_unordered_objects_equal_python_built(k):
    rng = np.random.default_rng(10 + k)
    cols = np.sort(rng.choice(500, size=(2000, k), replace=True), axis=1)
    cols = cols[np.all(np.diff(cols, axis=1) > 0, axis=1)].T.astype(np.uint32).copy()   # distinct values per row
    cols = np.unique(cols.T, axis=0).T.copy()
    vs = sorted(pm._vid(f"$u{k}_{i}") for i in range(k))
    fast, slow = _both([_T(1, vs, cols)])
    assert fast == slow and len(fast) == cols.shape[1]
    by_hash = {a.hash: a for a in slow}
    for a in fast:
        b = by_hash[a.hash]
        assert type(a) is pm.UnorderedAssignment
        assert (a.symbols, a.values, a.variables, a.frozen) == (b.symbols, b.values, b.variables, b.frozen)
    assert pm._assign.format_set(fast, pm.OrderedAssignment) == str(fast)


def test_two_tables_one_set_and_limit():
    rng = np.random.default_rng(3)
    a = _T(0, [pm._vid("$x"), pm._vid("$y")], rng.integers(0, 50, size=(2, 400)).astype(np.uint32))
    b = _T(0, [pm._vid("$x")], np.arange(30, dtype=np.uint32)[None, :].copy())
    fast, slow = _both([a, b])
    assert fast == slow
    lim_fast, lim_slow = _both([a, b], limit=420)
    assert lim_fast == lim_slow and len(lim_fast) <= 420
    assert pm._assign.format_set(set(), pm.OrderedAssignment) == "set()"


def test_sparse_ids_recoded():
    """Few values over a wide id range: re-coded, no id-sized lookup table."""
    cols = np.array([[5, 100_000_000, 7, 3_000_000_000], [9, 9, 200_000_001, 11]], dtype=np.uint32)
    t = _T(0, [pm._vid("$s1"), pm._vid("$s2")], cols)
    fast, slow = _both([t])
    assert fast == slow and len(fast) == 4
    assert {tuple(sorted(a.mapping.items())) for a in fast} == {tuple(sorted(a.mapping.items())) for a in slow}
