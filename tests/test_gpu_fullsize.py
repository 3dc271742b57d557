"""Parity at BASELINE.json's full sizes through size-independent properties:
the bench workloads' binding counts (config 2 bio at 20 M Member links,
config 5 hub at 3 M links) against closed-form counts computed with numpy
from the generator's own arrays (distinct-pair joins as degree sums), so a
wrong row anywhere in a 10^7-10^8-row join changes the count."""
import numpy as np
import pytest

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
    import bench
    from das_amd.pattern_matcher import pattern_matcher as pm
    ans = pm.PatternMatchingAnswer()
    bench.build_expr(pm, spec).matched(db, ans)
    return ans.count()


def test_gpu_bio_fullsize_counts():
    import bench
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    n_genes, n_bps = 200_000, 50_000
    arrays = synthetic.bio_kb(n_genes, n_bps, 20_000_000, 100_000)
    db = HipDB(device=0)
    db.load_arrays(arrays)
    base = len(arrays.type_names)                     # leaf index of gene 0; bps follow the genes
    m = _pairs(arrays, "Member")
    mg, mb = m >> 32, m & 0xFFFFFFFF
    inh = _pairs(arrays, "Inheritance")
    outdeg = np.bincount(inh >> 32, minlength=base + n_genes + n_bps)
    gdeg = np.bincount(mg, minlength=base + n_genes)
    specs = dict(bench.bio_specs(np.arange(n_genes)))
    rng = np.random.default_rng(17)
    ga, gb = (int(x) for x in rng.choice(np.arange(n_genes), 2, replace=False))   # bench.bio_specs' anchors
    bp0 = base + n_genes
    want = {
        "Q1 Member(Vg,Vbp)": len(m),
        "Q2 Member*Inheritance": int(outdeg[mb].sum()),
        "Q3 same_biological_process": len(np.intersect1d(mb[mg == base + ga], mb[mg == base + gb])),
        "Q4 hub join": int(gdeg[mg[mb == bp0]].sum()),
    }
    for name, spec in specs.items():
        assert _count(db, spec) == want[name], name


def test_gpu_hub_fullsize_counts():
    import bench
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    n_nodes = 1 << 21
    arrays = synthetic.powerlaw_kb(n_nodes, 3_000_000, link_types=4)
    db = HipDB(device=0)
    db.load_arrays(arrays)
    base = len(arrays.type_names)
    t = _pairs(arrays, "T0")
    src, dst = t >> 32, t & 0xFFFFFFFF
    outdeg = np.bincount(src, minlength=base + n_nodes)
    h0, h1 = base, base + 1
    v1 = src[dst == h0]
    is_v1 = np.zeros(base + n_nodes, bool)
    is_v1[v1] = True
    is_v2 = np.zeros(base + n_nodes, bool)
    is_v2[src[dst == h1]] = True
    mid = is_v1[src] & is_v2[dst]                    # T(V1,V2) with T(V1,h0) and T(V2,h1)
    want = {
        "H4 T(V1,h0) T(V1,V2) T(V2,h1) T(V2,V3)": int(outdeg[dst[mid]].sum()),
        "H2 T(V1,h0) T(V1,V2)": int(outdeg[v1].sum()),
    }
    for name, spec in bench.hub_specs():
        assert _count(db, spec) == want[name], name
