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


def _indexed_links(db):
    """Handles of the links this shard indexes (pattern rows: T_a by type)."""
    out = set()
    for t in db.arrays.type_names:
        tid = db.type_id.get(t)
        for tab in db.ctx.scan_type(tid) if tid is not None else []:
            if tab is not None and tab.nrows:
                out.update(db.hex_of(tab.fetch()[0]))
    return out


@pytest.mark.parametrize("world", [2, 3])
def test_gpu_device_build_handle_sharded(world):
    """shard=(rank, world) on a Zipf KB dense in duplicate links (hub pairs
    are generated many times): every rank holds the same directory, each
    distinct link is indexed on exactly the rank its handle names
    (int(handle[:8], 16) % world), and the shards' answers union to the
    single build's (canonical_parser.py:132-183: one index entry per handle)."""
    import torch
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    from das_amd.parallel import handle_owner
    from das_amd.pattern_matcher import pattern_matcher as pm
    n_nodes, n_links = 300, 20_000
    db_all = HipDB(device=0)
    db_all.load_arrays(synthetic.powerlaw_kb_device(db_all.ctx, n_nodes, n_links))
    full = _indexed_links(db_all)
    assert len(full) < n_links - 1000               # many generated duplicates collapse
    shards = []
    for r in range(world):
        db = HipDB(device=0)
        db.load_arrays(synthetic.powerlaw_kb_device(db.ctx, n_nodes, n_links, shard=(r, world)))
        shards.append(db)
    torch.cuda.synchronize()
    seen = {}
    for r, db in enumerate(shards):
        assert db.stats().n_atoms == db_all.stats().n_atoms
        links = _indexed_links(db)
        assert all(handle_owner(h, world) == r for h in links)
        for h in links:
            seen[h] = seen.get(h, 0) + 1
    assert seen == {h: 1 for h in full}
    V = pm.Variable
    for t in ("T0", "T3"):
        for q in (pm.Link(t, [V("V1"), V("V2"), V("V3")], True), pm.Link(t, [V("V1"), V("V2")], True)):
            parts = [_answer_set(db, q) for db in shards]
            w = _answer_set(db_all, q)
            assert set().union(*parts) == w
            assert sum(len(p) for p in parts) == len(w)       # disjoint


@pytest.mark.parametrize("world", [2, 3])
def test_gpu_exchange_build_indexes_each_link_once(world):
    """Config 4 at N GPUs (bench.py --workload build): each rank generates a
    range, hashes it (das_hash_owners), groups rows by owner
    (das_partition_rows) and sends them to the owners (here an in-process
    all-to-all); each rank builds what it received.  The shards' indexed
    links are disjoint, owned by handle, and union to the single build."""
    import torch
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    from das_amd.parallel import handle_owner, regroup_by_owner
    n_nodes, n_links = 400, 30_000
    db_all = HipDB(device=0)
    db_all.load_arrays(synthetic.powerlaw_kb_device(db_all.ctx, n_nodes, n_links))
    full = _indexed_links(db_all)
    sent = {}                                        # (src, arity group) -> (rows, counts)

    def make_exchange(src, box):
        def ex(rows, counts):
            box.append((rows.clone(), counts.copy()))
            return rows[:0]                          # filled in after every rank has sent
        return ex
    boxes = []
    for r in range(world):
        ctx_db = HipDB(device=0)
        lo, hi = n_links * r // world, n_links * (r + 1) // world
        part = synthetic.powerlaw_kb_device(ctx_db.ctx, n_nodes, n_links, first=lo, count=hi - lo)
        box = []
        regroup_by_owner(ctx_db.ctx, part, world, make_exchange(r, box))
        boxes.append(box)
        leaves = (part.leaf_bytes, part.leaf_off, part.leaf_kind, part.leaf_ctype, part.leaf_type_id,
                  part.name_start)
        names = part.type_names
        sent[r] = box
    seen = {}
    for dst in range(world):
        recv = []
        for g in range(2):
            chunks = []
            for src in range(world):
                rows, counts = boxes[src][g]
                off = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
                chunks.append(rows[int(off[dst]):int(off[dst + 1])])
            recv.append(torch.cat(chunks).reshape(-1))
        db = HipDB(device=0)
        db.load_arrays(synthetic.device_arrays(leaves, names, recv[0], recv[1]))
        links = _indexed_links(db)
        assert all(handle_owner(h, world) == dst for h in links)
        for h in links:
            seen[h] = seen.get(h, 0) + 1
    assert seen == {h: 1 for h in full}
    # grouping is stable and complete: every sent row's owner is its group
    rows, counts = boxes[0][0]
    assert int(counts.sum()) == rows.shape[0]


@pytest.mark.parametrize("onesweep", ["1", "0", "0-part", "0-part48"])
def test_gpu_large_build_sort_paths_agree(onesweep, monkeypatch):
    """A build whose sorts exceed 2^20 keys runs the onesweep passes (one
    histogram read up front, decoupled look-back per tile); with
    DAS_ONESWEEP=0 the per-pass histogram sort; "0-part" also sorts the
    digests on their top 40 bits and orders the runs sharing a prefix
    afterwards, and writes local2id through the partitioned scatter (both the
    default from 2^22 entries).  Same
    atoms, ids, links and answers either way, and the same as a small-sort
    reference build of the host copy checked against hashlib handles."""
    import torch
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    from das_amd.pattern_matcher import pattern_matcher as pm
    monkeypatch.setenv("DAS_ONESWEEP", onesweep[0])
    monkeypatch.setenv("DAS_L2I_PART", "1" if "part" in onesweep else "0")
    monkeypatch.setenv("DAS_DIGEST_PREFIX", "1" if "part" in onesweep else "0")
    # part48: a 16-bit prefix -- nearly every run holds several digests (LDS
    # run sorts), the hub links' duplicate runs exceed the LDS size (radix)
    if onesweep.endswith("48"):
        monkeypatch.setenv("DAS_DIGEST_PREFIX_SHIFT", "48")
    else:
        monkeypatch.delenv("DAS_DIGEST_PREFIX_SHIFT", raising=False)
    n_nodes, n_links = 1 << 18, 3 << 20
    db = HipDB(device=0)
    arrays = synthetic.powerlaw_kb_device(db.ctx, n_nodes, n_links)
    db.load_arrays(arrays)
    torch.cuda.synchronize()
    st = db.stats()
    dig, cat, ar, ty, nl = db._host_mirror()
    from das_amd import _lib
    hexes = _lib.digests_to_hex(dig)
    # ids in handle order inside each type segment's buckets, every handle distinct
    assert len(set(hexes)) == len(hexes) == st.n_atoms
    # sampled handles equal hashlib's (expression_hasher.py:9-35)
    h = arrays.to_host()
    md5 = lambda s: hashlib.md5(s.encode()).hexdigest()  # noqa: E731
    rng = np.random.default_rng(5)
    for j in rng.integers(0, n_links, 200):
        ch = h.children(int(j))
        names = [h.node_name(int(x)) for x in ch[1:]]
        tname = h.type_names[int(ch[0])]
        link = md5(" ".join([md5(tname)] + [md5(f"Concept {n}") for n in names]))
        assert db.link_exists(tname, [md5(f"Concept {n}") for n in names])
        assert db.get_link_handle(tname, [md5(f"Concept {n}") for n in names]) == link
    V = pm.Variable
    q = pm.And([pm.Link("T0", [V("V1"), pm.Node("Concept", "n0")], True), pm.Link("T1", [V("V1"), V("V2")], True)])
    ans = pm.PatternMatchingAnswer()
    q.matched(db, ans)
    # the same answer count on both sort paths (pinned by the closed form below)
    ch2 = h.expr_child[:3 * int(h.level_off[1])].reshape(-1, 3).astype(np.int64)
    nt = len(h.type_names)
    t0 = {tuple(r) for r in ch2[(ch2[:, 0] == 0) & (ch2[:, 2] == nt)][:, 1:]}
    v1 = {a for a, _ in t0}
    t1 = {tuple(r) for r in ch2[ch2[:, 0] == 1][:, 1:]}
    assert ans.count() == sum(1 for a, _ in t1 if a in v1)
