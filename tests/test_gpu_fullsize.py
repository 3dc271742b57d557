"""Parity at BASELINE.json's full sizes through size-independent properties:
the bench workloads' binding counts (config 2 bio at 20 M Member links,
config 5 hub at 10^9 links generated in HBM) against closed-form counts (numpy / torch)
from the generator's own arrays (distinct-pair joins as degree sums), so a
wrong row anywhere in a 10^7-10^8-row join changes the count -- and, next to
every count, an order-independent checksum of the answer's rows
(tests/checksum.py: das_table_checksum on the device against the same
function's closed form over the generator's arrays), so a wrong answer with
the right count fails too (pattern_matcher.py:41-51, 741-748)."""
import numpy as np
import pytest

from tests import checksum as CK

pytestmark = pytest.mark.gpu


def _pairs(arrays, type_name):
    """Distinct (t0, t1) leaf-index pairs of the arity-2 links of one type."""
    tid = arrays.type_id[type_name]
    off = arrays.expr_off
    out = []
    for g in range(len(arrays.level_off) - 1):
        b, e = int(arrays.level_off[g]), int(arrays.level_off[g + 1])
        if e <= b or int(off[b + 1] - off[b]) != 3:
            continue
        ch = arrays.expr_child[int(off[b]):int(off[e])].reshape(e - b, 3).astype(np.int64)
        ch = ch[ch[:, 0] == tid]
        out.append(ch[:, 1:])
    p = np.concatenate(out)
    return np.unique(p[:, 0] * (1 << 32) + p[:, 1])


def _count(db, spec):
    """(rows, checksum) of the device answer."""
    import bench
    from das_amd.pattern_matcher import pattern_matcher as pm
    ans = pm.PatternMatchingAnswer()
    bench.build_expr(pm, spec).matched(db, ans)
    ck, rows = CK.answer_checksum(ans)
    assert rows == ans.count()
    return rows, ck


def _count_many(db, specs):
    """(rows, checksum) of each answer of ONE pm.matched_many batch -- the
    bench step's call (das_plan_execute_many with its default side-stream
    chains, deferred Or unions and plans nested in read-back waits)."""
    import bench
    from das_amd.pattern_matcher import pattern_matcher as pm
    out = []
    for _, ans in pm.matched_many(db, [bench.build_expr(pm, s) for s in specs]):
        ck, rows = CK.answer_checksum(ans)
        assert rows == ans.count()
        out.append((rows, ck))
    return out


def _leaf_d64(arrays, n):
    """d64 (tests/checksum.py) of leaves 0 .. n-1 by hashlib over their strings."""
    return np.array([CK.d64_text(arrays.leaf_string(i)) for i in range(n)], dtype=np.uint64)


@pytest.fixture(scope="module")
def bio20m():
    """The bench's bio KB (bio_full_kb at 20 M Member links), indexed once
    for the module's bio tests, prefetched as bench.py's leg is."""
    import gc
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    arrays = synthetic.bio_full_kb(200_000, 50_000, 20_000_000, 100_000)
    db = HipDB(device=0)
    db.load_arrays(arrays)
    db.prefetch()
    yield db, arrays, _bio_base(arrays, 200_000, 50_000)
    del db, arrays
    gc.collect()


def _bio_base(arrays, n_genes, n_bps):
    """Anchor-independent parts of the bio closed forms."""
    base = len(arrays.type_names)                     # leaf index of gene 0; bps follow the genes
    m = _pairs(arrays, "Member")
    inh = _pairs(arrays, "Inheritance")
    D = _leaf_d64(arrays, arrays.n_leaf)
    return {"n_genes": n_genes, "n_bps": n_bps, "base": base, "m": m, "inh": inh, "D": D}


def _bio_want(arrays, B, anchor):
    """(rows, checksum) of bench.bio_specs(anchor=anchor)'s Q1-Q6 by closed form."""
    n_genes, n_bps, base, m, inh, D = (B[k] for k in ("n_genes", "n_bps", "base", "m", "inh", "D"))
    mg, mb = m >> 32, m & 0xFFFFFFFF
    rng = np.random.default_rng(17 + 7919 * anchor)
    ga, gb = (int(x) for x in rng.choice(np.arange(n_genes), 2, replace=False))   # bench.bio_specs' anchors
    bp0 = base + n_genes
    nl = base + n_genes + n_bps + 10_000                # every node index below the Concept blocks
    gdeg = np.bincount(mg, minlength=nl)
    outdeg = np.bincount(inh >> 32, minlength=nl)
    G = lambda v, x: CK.g_np(v, D[x])  # noqa: E731
    gsum = lambda k, v, n=nl: CK.group_sum_np(k, v, n)  # noqa: E731
    in_nl = mb < nl
    s_inh = gsum(inh >> 32, G("V_p", inh & 0xFFFFFFFF))               # per V_bp: sum over its parents
    s_mem = gsum(mb[in_nl], G("V_g", mg[in_nl]))                      # per V_bp: sum over its genes
    both = np.flatnonzero((s_inh != 0) | (s_mem != 0))
    inter = np.intersect1d(mb[mg == base + ga], mb[mg == base + gb])
    s0 = np.zeros(nl, dtype=bool)
    s0[mg[mb == bp0]] = True
    q4 = s0[mg] & in_nl
    want = {
        "Q1 Member(Vg,Vbp)": (len(m), CK.sum_np(CK.prod_np(G("V_g", mg), G("V_bp", mb)))),
        "Q2 Member*Inheritance": (int(outdeg[mb[in_nl]].sum()),
                                  CK.sum_np(CK.prod_np(s_mem[both], G("V_bp", both), s_inh[both]))),
        "Q3 same_biological_process (QUERY_1)": (len(inter), CK.sum_np(G("V_BiologicalProcess", inter))),
        "Q4 hub join": (int(gdeg[mg[mb == bp0]].sum()), CK.sum_np(CK.prod_np(G("V_g", mg[q4]), G("V_bp", mb[q4])))),
    }
    want.update(_query23_counts(arrays, n_genes, n_bps, base, ga, gb, m, inh, D=D))
    return want


def test_gpu_bio_fullsize_counts(bio20m, monkeypatch):
    """The bench's bio KB (bio_full_kb at 20 M Member links): Q1-Q4 against
    closed forms; the reference's QUERY_2 / QUERY_3 (Q5 / Q6) as one native
    plan call and through the per-operator path (same counts)."""
    import bench
    db, arrays, B = bio20m
    specs = dict(bench.bio_specs(np.arange(B["n_genes"])))
    want = _bio_want(arrays, B, 0)
    for name, spec in specs.items():
        assert _count(db, spec) == want[name], name
    # QUERY_2 / QUERY_3 through the per-operator fold as well (same answers)
    monkeypatch.setenv("DAS_PLAN", "0")
    for name in ("Q5 same_or_inherited_biological_process (QUERY_2)", "Q6 linked_reactome_uniprot (QUERY_3)"):
        assert _count(db, specs[name]) == want[name], name


def test_gpu_bio_fullsize_batched_step(bio20m):
    """bench.py's bio step exactly as timed: Q1-Q6 in ONE pm.matched_many
    call (das_plan_execute_many, default DAS_PLAN_NEST / DAS_DEFER /
    DAS_CHAIN_SIDE: plans nested in Q2's and Q6's long read-back waits on
    the plan side stream), over three gene anchors, then all three anchors'
    queries in one batch -- (count, checksum) per query against the closed
    forms (pattern_matcher.py:41-51, 705-748)."""
    import bench
    db, arrays, B = bio20m
    every, wants = [], []
    for anchor in (1, 2, 3):
        named = bench.bio_specs(np.arange(B["n_genes"]), anchor=anchor)
        want = _bio_want(arrays, B, anchor)
        got = _count_many(db, [q for _, q in named])
        for (name, _), g in zip(named, got):
            assert g == want[name], (anchor, name, g, want[name])
        every += [q for _, q in named]
        wants += [want[name] for name, _ in named]
    assert _count_many(db, every) == wants


def _query23_counts(arrays, n_genes, n_bps, base, ga, gb, m, inh, n_up=5000, n_r=1000, n_loc=40, D=None):
    """Closed forms of scripts/benchmark.py QUERY_2 / QUERY_3 (bench Q5 / Q6)
    over the generator's distinct link pairs, following the reference fold
    (pattern_matcher.py:491-500, 644-687, 705-748): (rows, checksum) per
    query.  The anchors' intermediate results are asserted non-empty, so
    reset-on-empty never applies.  D: d64 per leaf (_leaf_d64)."""
    from das_amd import synthetic
    _, off = synthetic.bio_nodes(n_genes, n_bps, n_up, n_r, n_loc)
    rng_of = lambda k, n: (base + off[k], base + off[k] + n)  # noqa: E731
    inside = lambda x, r: (x >= r[0]) & (x < r[1])  # noqa: E731
    G_, BP = rng_of("g", n_genes), rng_of("bp", n_bps)
    UP, R = rng_of("up", n_up), rng_of("r", n_r)
    concept = [rng_of(k, n) for k, n in (("upname", n_up), ("rname", n_r), ("loc", n_loc))]
    is_concept = lambda x: np.logical_or.reduce([inside(x, r) for r in concept])  # noqa: E731
    nl = arrays.n_leaf
    if D is None:
        D = _leaf_d64(arrays, nl)
    G = lambda v, x: CK.g_np(v, D[np.asarray(x, dtype=np.int64)])  # noqa: E731
    mg, mb = m >> 32, m & 0xFFFFFFFF
    A = set(mb[mg == base + ga].tolist())                  # Member(ga, V1)
    B = set(mb[mg == base + gb].tolist())                  # Member(gb, V2)
    # QUERY_2 = And[Member(ga,V1), Or[And[Member(gb,V2), InhT(V2,V3), InhT(V1,V3)], Member(gb,V1)]]
    ic, ip = inh >> 32, inh & 0xFFFFFFFF
    sel = inside(ic, BP) & inside(ip, BP)                  # template Inheritance(BP, BP)
    ic, ip = ic[sel], ip[sel]
    by_parent = {}
    for c, p in zip(ic.tolist(), ip.tolist()):
        by_parent.setdefault(p, []).append(c)
    inner1 = [(c, p) for c, p in zip(ic.tolist(), ip.tolist()) if c in B]         # (V2, V3)
    assert A and B and inner1
    inner = {(v1, v2, v3) for v2, v3 in inner1 for v1 in by_parent[v3]}          # (V1, V2, V3)
    rows3 = np.array(sorted(r for r in inner if r[0] in A), dtype=np.int64).reshape(-1, 3)
    ab = np.array(sorted(A & B), dtype=np.int64)
    ck2 = (CK.sum_np(CK.prod_np(G("V1_BiologicalProcess", rows3[:, 0]), G("V2_BiologicalProcess", rows3[:, 1]),
                                G("V3_BiologicalProcess", rows3[:, 2])))
           + CK.sum_np(G("V1_BiologicalProcess", ab))) & CK.M64
    q2 = len(rows3) + len(ab)
    # QUERY_3: same_bp x MemberT(Up, BP) x ListT(Up, .) x ListT(Up, .) x ListT(Reactome, Concept)
    S = A & B
    up = m[inside(mg, UP) & inside(mb, BP)]
    up = up[np.isin(up & 0xFFFFFFFF, np.array(sorted(S), dtype=np.int64))]
    ups, upb = up >> 32, up & 0xFFFFFFFF
    lst = _pairs(arrays, "List")
    la, lb = lst >> 32, lst & 0xFFFFFFFF
    lu = inside(la, UP) & is_concept(lb)
    nl_up = np.bincount(la[lu], minlength=int(UP[1]))
    j = int((nl_up[ups] ** 2).sum())
    lr = inside(la, R) & is_concept(lb)
    assert S and len(ups) and j and lr.sum()
    # rows (bp, up, c1, c2, r, c3): per (up, bp) the List sums of V_UniprotName
    # and V_Location over up's Concept lists, times the Reactome lists' sum
    sn = CK.group_sum_np(la[lu], G("V_UniprotName", lb[lu]), nl)
    sl = CK.group_sum_np(la[lu], G("V_Location", lb[lu]), nl)
    left = CK.sum_np(CK.prod_np(G("V_BiologicalProcess", upb), G("V_Uniprot", ups), sn[ups], sl[ups]))
    right = CK.sum_np(CK.prod_np(G("V_Reactome", la[lr]), G("V_ReactomeName", lb[lr])))
    ck3 = int(CK.prod_np(np.uint64(left), np.uint64(right)))
    return {"Q5 same_or_inherited_biological_process (QUERY_2)": (q2, ck2),
            "Q6 linked_reactome_uniprot (QUERY_3)": (j * int(lr.sum()), ck3)}


def _dev_pairs(arrays, k):
    """Distinct (t0, t1) leaf-index pairs (as t0 << 32 | t1, int64 on the GPU)
    of the arity-2 links of type T<k> in a device-generated KB."""
    import torch
    c2 = int(arrays.level_off[1])
    ch = arrays.expr_child[:3 * c2].view(-1, 3)
    sel = ch[:, 0] == k
    key = (ch[sel, 1].to(torch.int64) << 32) | ch[sel, 2].to(torch.int64)
    return torch.unique(key)


N_NODES, N_LINKS = 1 << 27, 1_000_000_000


@pytest.fixture(scope="module")
def kb1g():
    """The 10^9-link power-law KB of configs 4 / 5, generated in HBM and
    indexed ONCE for the module's tests (the generator's arrays are kept for
    the closed forms)."""
    import gc
    import torch
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    db = HipDB(device=0)
    arrays = synthetic.powerlaw_kb_device(db.ctx, N_NODES, N_LINKS)
    db.load_arrays(arrays)
    yield db, arrays
    del db, arrays
    gc.collect()
    torch.cuda.empty_cache()


def test_gpu_hub_fullsize_counts(kb1g):
    """Config 5 at BASELINE size (10^9 links generated in HBM): the bench's
    hub queries against semi-join closed forms over the generator's arrays."""
    import bench
    import torch
    db, arrays = kb1g
    n_nodes = N_NODES
    base = len(arrays.type_names)
    h0, h1 = base, base + 1
    pairs = {k: _dev_pairs(arrays, k) for k in range(4)}
    src = {k: (p >> 32) for k, p in pairs.items()}
    dst = {k: (p & 0xFFFFFFFF) for k, p in pairs.items()}

    def member(k, h):
        m = torch.zeros(base + n_nodes, dtype=torch.bool, device="cuda")
        m[src[k][dst[k] == h]] = True
        return m
    s1 = member(0, h0)
    s23 = member(2, h1) & member(3, h0)
    in1 = s1[src[1]]
    keep4 = in1 & s23[dst[1]]
    D = _dev_leaf_d64(db, arrays)
    ck = lambda sel: CK.sum_torch(CK.g_torch("V1", D[src[1][sel]]) * CK.g_torch("V2", D[dst[1][sel]]))  # noqa: E731
    want = {
        "H4 T0(V1,h0) T1(V1,V2) T2(V2,h1) T3(V2,h0)": (int(keep4.sum()), ck(keep4)),
        "H2 T0(V1,h0) T1(V1,V2)": (int(in1.sum()), ck(in1)),
    }
    assert want["H4 T0(V1,h0) T1(V1,V2) T2(V2,h1) T3(V2,h0)"][0] > 10_000_000
    del pairs, src, dst, s1, s23, in1, keep4
    for name, spec in bench.hub_specs():
        assert _count(db, spec) == want[name], name
    # bench.py's hub step as timed: H4 and H2 in ONE das_plan_execute_many
    # batch -- H2 nested in H4's filtered-walk read-back wait at 10^9 links
    # (plan side stream, second read-back slot), three times
    named = bench.hub_specs()
    for rep in range(3):
        assert _count_many(db, [q for _, q in named]) == [want[name] for name, _ in named], rep


def _dev_leaf_d64(db, arrays):
    """d64 (tests/checksum.py) of every leaf of a device-generated KB: the
    leaf strings hashed on the GPU (das_hash_strings_dev, the MD5 kernel
    test_gpu_md5_kernel_matches_hashlib pins), 1000 sampled against hashlib."""
    import torch
    from das_amd import _lib
    n = int(arrays.n_leaf)
    dev = torch.device("cuda:0")
    b = torch.from_numpy(np.asarray(arrays.leaf_bytes, dtype=np.uint8)).to(dev)
    o = torch.from_numpy(np.asarray(arrays.leaf_off).view(np.int64)).to(dev)
    words = torch.empty((n, 4), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    _lib.check(_lib.lib().das_hash_strings_dev(db.ctx.h, b.data_ptr(), o.data_ptr(), n, words.data_ptr()), db.ctx.h)
    torch.cuda.synchronize()
    del b, o
    D = CK.d64_from_words_torch(words)
    del words
    for i in np.random.default_rng(5).integers(0, n, 1000).tolist() + [0, n - 1]:
        assert (int(D[i]) & CK.M64) == CK.d64_text(arrays.leaf_string(i)), i
    return D


def test_gpu_build_fullsize_incoming_sets(kb1g):
    """Config 4 at BASELINE size (10^9 links generated in HBM): the incoming
    CSR (`incomming_set:<target>`, canonical_parser.py:141-143) of nodes
    sampled across the Zipf ranks equals what the generator's arrays imply --
    one entry per (distinct link, position) holding the node -- comes out
    sorted by link id, and every listed link targets the node."""
    import torch
    db, arrays = kb1g
    n_nodes, n_links = N_NODES, N_LINKS
    base = len(arrays.type_names)
    c2 = int(arrays.level_off[1])
    ch2 = arrays.expr_child[:3 * c2].view(-1, 3)
    ch3 = arrays.expr_child[3 * c2:].view(-1, 4)
    for rank in (3, 10, 100, 1000, 100_000, 10_000_000, n_nodes - 1):
        x = base + rank
        want = 0
        for ch in (ch2, ch3):
            rows = ch[(ch[:, 1:] == x).any(dim=1)]
            if rows.shape[0]:
                rows = torch.unique(rows, dim=0)               # one atom per distinct link
                want += int((rows[:, 1:] == x).sum())
        nid = int(db.ids_of([db.get_node_handle("Concept", f"n{rank}")])[0])
        assert nid >= 0, rank
        got = db.ctx.incoming(nid)
        assert got.shape[0] == want, (rank, got.shape[0], want)
        assert np.all(got[1:] >= got[:-1]), rank                # sorted by link id
        for lid in got[np.linspace(0, len(got) - 1, min(len(got), 200)).astype(np.int64)] if len(got) else []:
            assert nid in db.ctx.link_targets(int(lid)), (rank, int(lid))
    # handles at 10^9 links: ~10^3 sampled links and nodes equal hashlib's
    # (expression_hasher.py:9-35) and resolve to indexed atoms
    import hashlib
    md5 = lambda t: hashlib.md5(t.encode()).hexdigest()  # noqa: E731
    rng = np.random.default_rng(11)
    names = arrays.type_names
    for j in rng.integers(0, n_links, 1000):
        row = (ch2[int(j)] if j < c2 else ch3[int(j) - c2]).cpu().numpy()
        tn = names[int(row[0])]
        targets = [md5(f"Concept n{int(x) - base}") for x in row[1:]]
        h = md5(" ".join([md5(tn)] + targets))
        assert db.get_link_handle(tn, targets) == h
        assert db.link_exists(tn, targets), (int(j), h)
    for r in rng.integers(0, n_nodes, 1000):
        h = md5(f"Concept n{int(r)}")
        assert db.get_node_handle("Concept", f"n{int(r)}") == h and db.node_exists("Concept", f"n{int(r)}")


def _exec_rows(arrays):
    """(schema, key, value) leaf-index rows of the arity-3 Execution links (with repeats)."""
    off = arrays.expr_off
    out = []
    for g in range(len(arrays.level_off) - 1):
        b, e = int(arrays.level_off[g]), int(arrays.level_off[g + 1])
        if e <= b or int(off[b + 1] - off[b]) != 4:
            continue
        out.append(arrays.expr_child[int(off[b]):int(off[e])].reshape(e - b, 4)[:, 1:].astype(np.int64))
    return np.concatenate(out)


def _flybase_counts(arrays, gene, do_terms):
    """Closed forms of bench.flybase_specs (QueryFlyBase.ipynb cells 5-9) for
    one gene anchor, from the generator's distinct Execution rows: And folds
    as joins (pattern_matcher.py:705-748; every running result is asserted
    non-empty, so reset-on-empty never applies), Not as the anti-join of
    check_negation, Or as a union of distinct bindings.  (rows, checksum)
    per query; the checksum's per-key sums follow the same loops."""
    strs = arrays.leaf_strings()
    names = {s: i for i, s in enumerate(strs)}
    leaf = lambda t, n: names[f"{t} {n}"]  # noqa: E731
    d64 = {}

    def G(v, x):
        d = d64.get(x)
        if d is None:
            d = d64[x] = CK.d64_text(strs[x])
        return CK.g(v, d)
    M = CK.M64
    rows = _exec_rows(arrays)
    s = lambda n: leaf("Schema", "Schema:" + n)  # noqa: E731
    tab = {k: np.unique(rows[rows[:, 0] == s(n)][:, 1:], axis=0) for k, n in (
        ("uniq", "gene_uniquename"), ("rec", "gene_map_table_recombination_loc"),
        ("cyto", "gene_map_table_cytogenetic_loc"), ("do", "disease_model_annotations_DO_term"))}
    fb = leaf("Verbatim", f"FBgn{gene:07d}")

    def by(t, col):
        d = {}
        for a, b in tab[t].tolist():
            d.setdefault((a, b)[col], []).append((a, b)[1 - col])
        return d
    rec_by_val, uniq_by_val = by("rec", 1), by("uniq", 1)
    # per v2: (number of uniquename keys v with value v2, sum of g(var, v))
    u_sum = {}

    def uniq_of(v2, var):
        k = (v2, var)
        if k not in u_sum:
            us = uniq_by_val.get(v2, ())
            u_sum[k] = (len(us), sum(G(var, u) for u in us) & M)
        return u_sum[k]
    out = {}
    for name, t in (("F5 same recombination_loc", "rec"), ("F6 same cytogenetic_loc", "cyto")):
        r1 = set(tab[t][tab[t][:, 0] == fb][:, 1].tolist())
        t_by_val = by(t, 1)
        assert r1
        n = ck = 0
        for v1 in r1:
            for v2 in t_by_val.get(v1, ()):
                c, su = uniq_of(v2, "v3")
                n += c
                ck = (ck + G("v1", v1) * G("v2", v2) * su) & M
        out[name] = (n, ck)
    r1 = set(tab["rec"][tab["rec"][:, 0] == fb][:, 1].tolist())
    c_fb = set(tab["cyto"][tab["cyto"][:, 0] == fb][:, 1].tolist())
    cyto = set(map(tuple, tab["cyto"].tolist()))
    n = ck = 0
    for v1 in r1:
        for v2 in rec_by_val.get(v1, ()):
            c, su = uniq_of(v2, "v4")
            v3s = [v3 for v3 in c_fb if (v2, v3) not in cyto]
            n += c * len(v3s)
            s3 = sum(G("v3", v3) for v3 in v3s) & M
            ck = (ck + G("v1", v1) * G("v2", v2) * s3 * su) & M
    out["F7 same recomb, different cyto"] = (n, ck)
    terms = [leaf("Verbatim", d) for d in (do_terms or ["DOID:0"]) if f"Verbatim {d}" in names]
    v1s = set(tab["do"][np.isin(tab["do"][:, 1], terms)][:, 0].tolist())
    out["F9 DO-term Or"] = (len(v1s), sum(G("v1", v) for v in v1s) & M)
    rec_by_key = by("rec", 0)
    r_sum = {}
    n = ck = 0
    for v3, v2 in tab["uniq"].tolist():
        vs = rec_by_key.get(v2, ())
        if not vs:
            continue
        if v2 not in r_sum:
            r_sum[v2] = sum(G("v1", v) for v in vs) & M
        n += len(vs)
        ck = (ck + G("v3", v3) * G("v2", v2) * r_sum[v2]) & M
    out["FJ uniquename x recombination_loc"] = (n, ck)
    return out


def test_gpu_flybase_fullsize_counts():
    """Config 3 at bench size (flybase_kb: 300 k genes, 60 schemas, 26.7 M
    Execution links): the five FlyBase query shapes at two of the bench's gene
    anchors against closed forms over the generator's rows."""
    import bench
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    arrays = synthetic.flybase_kb(300_000, 60, 450_000)
    db = HipDB(device=0)
    db.load_arrays(arrays)
    db.prefetch()                        # anchors resolved through the host node directory (bench.py's path)
    assert db._node_dir is not None and len(db._node_dir) > 600_000          # every node (genes, FB ids, values)
    every, wants = [], []
    for gene in (7, 7 + 7919):
        do_terms = synthetic.flybase_do_terms(arrays, gene=gene)
        want = _flybase_counts(arrays, gene, do_terms)
        named = bench.flybase_specs(gene, do_terms)
        for name, spec in named:
            assert _count(db, spec) == want[name], (gene, name)
        # bench.py's step as timed: the five queries in one
        # das_plan_execute_many batch (grid chains on side streams launched in
        # the other plans' read-back waits, F9's union deferred)
        assert _count_many(db, [q for _, q in named]) == [want[name] for name, _ in named], gene
        every += [q for _, q in named]
        wants += [want[name] for name, _ in named]
    assert _count_many(db, every) == wants
    # fresh anchors straight into a batch (no one-by-one run before it: the
    # anchors' key ranges and shapes first seen inside the batch)
    for gene in (7 + 2 * 7919, 7 + 3 * 7919):
        do_terms = synthetic.flybase_do_terms(arrays, gene=gene)
        named = bench.flybase_specs(gene, do_terms)
        want = _flybase_counts(arrays, gene, do_terms)
        assert _count_many(db, [q for _, q in named]) == [want[name] for name, _ in named], gene
