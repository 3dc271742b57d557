"""Pattern index P_{a,p} (index.hip) row order: for every named type, arity
a <= 3 and position p, the type's rows sorted by (t_p, the other targets in
position order, link id) -- the `patterns:` key families of
canonical_parser.py:148-176 with each key's links ordered so an anchored
range comes out sorted by its first free target.  The packed-key build (one
stable sort per type segment, two stages when the key exceeds 64 bits) must
equal the permutation build (DAS_PIDX_PERM=1) row for row, and P_{a,p>0}
derived from P_{a,0} (the default: a stable sort on t_p alone) the full-key
sort of each (DAS_PIDX_DERIVE=0)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _kb(name):
    from das_amd import loader, synthetic
    if name == "powerlaw":
        return synthetic.powerlaw_kb(300, 6000, link_types=4, seed=3)
    if name == "bio":
        return synthetic.bio_kb(300, 60, 4000, 200)
    b = loader.AtomBuilder()
    n = [b.terminal("Concept", f"c{i}", True) for i in range(40)]
    rng = np.random.default_rng(8)
    ls = []
    for i in range(600):
        ar = int(rng.integers(1, 4))
        tg = [n[int(x)] for x in rng.integers(0, 40, ar)]
        if ls and rng.random() < 0.3:
            tg[int(rng.integers(0, ar))] = ls[int(rng.integers(0, len(ls)))]   # nested link target
        ls.append(b.expr(f"R{int(rng.integers(0, 3))}", tg))
    return b.finish()


def _p_rows(ctx, n_types):
    """{(type, arity, p): rows (link, t0..) in P_{a,p} order} and the T_a rows."""
    out = {}
    for ar in (1, 2, 3):
        for ty in range(n_types):
            t = ctx.scan_link(ar, ty, [], list(range(ar)), ar, True, emit_link=True)
            T = t.fetch()
            t.free()
            if not T.shape[1]:
                continue
            out[(ty, ar, "T")] = T
            for p in range(ar):
                t = ctx.scan_link(ar, ty, [], list(range(ar)), ar, True, emit_link=True, order_pos=p)
                out[(ty, ar, p)] = t.fetch()
                t.free()
    return out


@pytest.mark.parametrize("kb", ["powerlaw", "bio", "nested"])
def test_gpu_pattern_index_order(kb, monkeypatch):
    from das_amd.database.hip_db import HipDB
    arrays = _kb(kb)
    got = {}
    for mode in ("packed", "two", "perm", "noderive"):
        monkeypatch.setenv("DAS_PIDX_PERM", "1" if mode == "perm" else "0")
        monkeypatch.setenv("DAS_PIDX_TWO", "1" if mode == "two" else "0")
        monkeypatch.setenv("DAS_PIDX_DERIVE", "0" if mode == "noderive" else "1")
        db = HipDB(device=0)
        db.load_arrays(arrays)
        got[mode] = _p_rows(db.ctx, db.stats().n_types)
    rows = got["packed"]
    assert any(k[1] == 3 for k in rows) or kb == "bio"
    for key, P in rows.items():
        if key[2] == "T":
            continue
        ty, ar, p = key
        T = rows[(ty, ar, "T")]               # columns: link, t0 .. t_{a-1}
        assert P.shape == T.shape, key
        others = [1 + q for q in range(ar) if q != p]
        # np.lexsort: last key is the primary one
        order = np.lexsort([T[0]] + [T[c] for c in reversed(others)] + [T[1 + p]])
        assert np.array_equal(P, T[:, order]), key
        for mode in ("two", "perm", "noderive"):
            assert np.array_equal(got[mode][key], P), (mode, key)
