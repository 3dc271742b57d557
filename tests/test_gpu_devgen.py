"""Device-resident build input (das_build_index_ex + das_synth_powerlaw_links):
the configs 4-5 KB generated in HBM indexes exactly like the same arrays
handed over from the host, and the generator is split-invariant."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ctx():
    import torch
    from das_amd import _lib
    return _lib.Context(0, torch.cuda.current_stream().cuda_stream)


def test_gpu_synth_split_invariant_and_in_range():
    import torch
    from das_amd import synthetic
    ctx = _ctx()
    n_nodes, n_links = 5000, 40_000
    whole = synthetic.powerlaw_kb_device(ctx, n_nodes, n_links)
    parts = [synthetic.powerlaw_kb_device(ctx, n_nodes, n_links, first=a, count=b - a)
             for a, b in ((0, 13_001), (13_001, 28_000), (28_000, 40_000))]
    torch.cuda.synchronize()
    h = whole.to_host()
    n2 = int(n_links * 0.7)
    assert list(whole.level_off) == [0, n2, n_links]
    ch2 = h.expr_child[:3 * n2].reshape(-1, 3)
    ch3 = h.expr_child[3 * n2:].reshape(-1, 4)
    nt = len(h.type_names)
    for ch in (ch2, ch3):
        assert ch[:, 0].max() < 4
        assert ch[:, 1:].min() >= nt and ch[:, 1:].max() < nt + n_nodes
    # Zipf(1.1): node 0 is the most frequent target by far
    cnt = np.bincount(ch2[:, 1:].reshape(-1) - nt, minlength=n_nodes)
    assert cnt.argmax() == 0 and cnt[0] > 5 * cnt[100]
    # the concatenated split equals the whole, row for row
    r2 = np.concatenate([p.to_host().expr_child[:3 * int(p.level_off[1])].reshape(-1, 3) for p in parts])
    r3 = np.concatenate([p.to_host().expr_child[3 * int(p.level_off[1]):].reshape(-1, 4) for p in parts])
    assert np.array_equal(r2, ch2) and np.array_equal(r3, ch3)


def _answer_set(db, q):
    from das_amd.pattern_matcher import pattern_matcher as pm
    ans = pm.PatternMatchingAnswer()
    q.matched(db, ans)
    return {frozenset(a.mapping.items()) for a in ans.assignments}


def test_gpu_device_build_equals_host_build():
    import torch
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    from das_amd.pattern_matcher import pattern_matcher as pm
    db_d = HipDB(device=0)
    arrays = synthetic.powerlaw_kb_device(db_d.ctx, 3000, 30_000)
    db_d.load_arrays(arrays)
    db_h = HipDB(device=0)
    db_h.load_arrays(arrays.to_host())
    torch.cuda.synchronize()
    sd, sh = db_d.stats(), db_h.stats()
    for f in ("n_atoms", "n_nodes", "n_links", "n_types", "n_ctypes"):
        assert getattr(sd, f) == getattr(sh, f), f
    assert list(db_d.count_atoms()) == list(db_h.count_atoms())
    # handles: md5 of the reference's strings (expression_hasher.py:9-35)
    md5 = lambda s: hashlib.md5(s.encode()).hexdigest()  # noqa: E731
    h = arrays.to_host()
    row = h.expr_child[:3]
    names = [h.node_name(int(x)) for x in row[1:]]
    link = md5(" ".join([md5(f"T{int(row[0])}")] + [md5(f"Concept {n}") for n in names]))
    assert db_d.get_link_handle(f"T{int(row[0])}", [md5(f"Concept {n}") for n in names]) == link
    assert db_d.link_exists(f"T{int(row[0])}", [md5(f"Concept {n}") for n in names])
    V, L, N = pm.Variable, pm.Link, pm.Node
    queries = [
        L("T0", [V("V1"), V("V2")], True),
        L("T1", [V("V1"), N("Concept", "n0")], True),
        L("T2", [V("V1"), V("V2"), V("V3")], True),
        pm.And([L("T0", [V("V1"), N("Concept", "n0")], True), L("T1", [V("V1"), V("V2")], True),
                L("T2", [V("V2"), N("Concept", "n1")], True), L("T3", [V("V2"), N("Concept", "n0")], True)]),
        pm.And([L("T0", [V("V1"), N("Concept", "n0")], True), L("T1", [V("V1"), V("V2")], True)]),
    ]
    for q in queries:
        assert _answer_set(db_d, q) == _answer_set(db_h, q)


def test_gpu_device_build_remote_links():
    """own=(lo, hi): links outside the range are directory-only (kind 3):
    same atoms, pattern rows only for the owned links."""
    import torch
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    from das_amd.pattern_matcher import pattern_matcher as pm
    n_nodes, n_links = 2000, 20_000
    db_all = HipDB(device=0)
    full = synthetic.powerlaw_kb_device(db_all.ctx, n_nodes, n_links)
    db_all.load_arrays(full)
    db_a, db_b = HipDB(device=0), HipDB(device=0)
    db_a.load_arrays(synthetic.powerlaw_kb_device(db_a.ctx, n_nodes, n_links, own=(0, 9000)))
    db_b.load_arrays(synthetic.powerlaw_kb_device(db_b.ctx, n_nodes, n_links, own=(9000, n_links)))
    torch.cuda.synchronize()
    assert db_a.stats().n_atoms == db_b.stats().n_atoms == db_all.stats().n_atoms
    V = pm.Variable
    for t in ("T0", "T3"):
        q = pm.Link(t, [V("V1"), V("V2"), V("V3")], True)
        a, b, w = _answer_set(db_a, q), _answer_set(db_b, q), _answer_set(db_all, q)
        assert a | b == w            # an atom both shards generate is indexed by both
