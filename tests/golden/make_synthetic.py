"""Inputs for the reference-answered synthetic fixtures (TEST INFRASTRUCTURE).

Step 1 of tests/golden/generate.sh, run with this repo's interpreter (numpy):
writes the canonical MeTTa text of small seeded instances of the config 2-5
generators (das_amd.synthetic) and their query lists to the scratch
directory, plus `synthetic_specs.json`.  Step 2 (make_golden.py synthetic,
conda Python 3.9 with PLY) loads each text through the reference's own
CanonicalParser and answers every query with the reference pattern_matcher,
writing tests/golden/kb_<name>.json.  tests/test_gpu_golden.py regenerates
the same text (checked by its sha256) and replays the queries on the GPU.

Query sets per KB:
  bio_full   bench.py Q1-Q4; scripts/benchmark.py QUERY_1-3
             (_same_biological_process, _same_or_inherited_biological_process,
             _linked_reactome_uniprot, benchmark.py:89-128); random shapes
  flybase    bench.py F5/F6/F7/F9/FJ (QueryFlyBase.ipynb cells 5-9) at
             several gene anchors
  powerlaw   random Link / And / Or / Not shapes, 2-4 clauses, arity 2-3
  hub        bench.py H4 / H2 (config 5) and the unanchored 4-clause chain
Entries with "no_overload": true are answered with the reference's
CONFIG['no_overload'] = True (pattern_matcher.py:16-19, :98).
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from das_amd import synthetic  # noqa: E402

SCRATCH = os.environ.get("DAS_GOLDEN_SCRATCH", "/tmp/das_golden")


def V(n):
    return ["Var", n]


def TV(n, t):
    return ["TVar", n, t]


def N(t, n):
    return ["Node", t, n]


def L(t, *targets, ordered=True):
    return ["Link", t, ordered, list(targets)]


def T(t, *tvars, ordered=True):
    return ["Template", t, ordered, list(tvars)]


# ---------------------------------------------------------------- generators
# (name, generator call, kwargs) -- the test side calls the same function
KBS = {
    "bio_full": ("bio_full_kb", dict(n_genes=120, n_bps=60, n_member=1500, n_inh=120, n_uniprot=80,
                                     n_up_member=400, n_reactome=25, n_context=200, n_loc=6, seed=31)),
    "flybase": ("flybase_kb", dict(n_genes=150, n_schema=6, rows_per_schema=300, n_loc=20, n_do=15, seed=32)),
    "powerlaw": ("powerlaw_kb", dict(n_nodes=300, n_links=3000, link_types=3, seed=33)),
    "hub": ("powerlaw_kb", dict(n_nodes=150, n_links=4000, link_types=4, seed=34)),
}


def make_arrays(name):
    fn, kw = KBS[name]
    return getattr(synthetic, fn)(**kw)


def text_of(name):
    return synthetic.to_canonical(make_arrays(name))


# ------------------------------------------------------------------- queries
def benchmark_queries(genes):
    """scripts/benchmark.py:40-128 query layouts (restated as specs)."""
    g = [N("Gene", x) for x in genes]
    member = lambda a, b: L("Member", a, b)  # noqa: E731
    member_t = lambda a, b: T("Member", a, b)  # noqa: E731
    inh_t = lambda a, b: T("Inheritance", a, b)  # noqa: E731
    list_t = lambda a, b: T("List", a, b)  # noqa: E731

    def evaluation(p, va, vb):
        return L("Evaluation", N("Predicate", p), list_t(va, vb))

    def context(va, vb, vc):
        return L("Context", member_t(va, vb), evaluation("has_location", va, vc))

    def same_bp(gs):
        return ["And", [member(x, V("V_BiologicalProcess")) for x in gs]]
    q1 = same_bp(g)
    v1, v2 = V("V1_BiologicalProcess"), V("V2_BiologicalProcess")
    tv1, tv2, tv3 = (TV(f"V{i}_BiologicalProcess", "BiologicalProcess") for i in (1, 2, 3))
    q2 = ["And", [member(g[0], v1),
                  ["Or", [["And", [member(g[1], v2), inh_t(tv2, tv3), inh_t(tv1, tv3)]],
                          member(g[1], v1)]]]]
    b1, up, re_, rn, loc, un = (TV("V_BiologicalProcess", "BiologicalProcess"), TV("V_Uniprot", "Uniprot"),
                                TV("V_Reactome", "Reactome"), TV("V_ReactomeName", "Concept"),
                                TV("V_Location", "Concept"), TV("V_UniprotName", "Concept"))
    q3 = ["And", [same_bp(g), member_t(up, b1), evaluation("has_name", up, un), context(up, re_, loc),
                  evaluation("has_name", re_, rn)]]
    return [q1, q2, q3]


def bench_bio_queries(ga, gb):
    g = lambda i: N("Gene", f"g{i}")  # noqa: E731
    bp = lambda i: N("BiologicalProcess", f"bp{i}")  # noqa: E731
    return [L("Member", V("V_g"), V("V_bp")),
            ["And", [L("Member", V("V_g"), V("V_bp")), L("Inheritance", V("V_bp"), V("V_p"))]],
            ["And", [L("Member", g(ga), V("V_bp")), L("Member", g(gb), V("V_bp"))]],
            ["And", [L("Member", V("V_g"), bp(0)), L("Member", V("V_g"), V("V_bp"))]]]


def random_queries(rng, types, nodes, n, arity3=False):
    """Ordered Link / And / Or / Not shapes over the given link types and
    (type, name) nodes; 2-4 clauses, shared and unshared variables."""
    def node():
        t, nm = nodes[rng.integers(len(nodes))]
        return N(t, nm)

    def lk(*targets):
        return L(types[rng.integers(len(types))], *targets)
    shapes = [
        lambda: lk(V("A"), node()),
        lambda: lk(node(), V("A")),
        lambda: lk(V("A"), V("B")),
        lambda: ["And", [lk(V("A"), V("B")), lk(V("B"), V("C"))]],
        lambda: ["And", [lk(node(), V("B")), lk(V("A"), V("B"))]],
        lambda: ["And", [lk(V("A"), V("B")), ["Not", lk(V("A"), node())]]],
        lambda: ["And", [lk(V("A"), node()), lk(V("A"), V("B")), ["Not", lk(V("B"), node())]]],
        lambda: ["Or", [lk(V("A"), node()), lk(V("A"), node())]],
        lambda: ["Or", [lk(V("A"), node()), ["Not", lk(V("A"), node())]]],
        lambda: ["And", [lk(V("A"), V("B")), lk(V("A"), V("C")), lk(V("C"), V("D"))]],
        lambda: ["And", [lk(V("A"), node()), lk(V("B"), node()), lk(V("A"), V("B"))]],
        lambda: ["And", [["Or", [lk(V("A"), node()), lk(V("A"), node())]], lk(V("A"), V("B"))]],
        lambda: ["And", [lk(V("A"), V("A"))]],
        lambda: ["And", [lk(V("A"), node()), lk(V("A"), node()), lk(V("B"), node())]],
    ]
    if arity3:
        shapes += [lambda: lk(V("A"), node(), V("B")),
                   lambda: ["And", [lk(V("A"), V("B"), V("C")), lk(V("C"), V("D"))]],
                   lambda: ["And", [lk(node(), V("B"), V("C")), ["Not", lk(V("B"), V("C"), node())]]]]
    return [shapes[int(rng.integers(len(shapes)))]() for _ in range(n)]


def queries_of(name, arrays):
    rng = np.random.default_rng(7)
    out = []
    if name == "bio_full":
        out += bench_bio_queries(3, 5)
        out += bench_bio_queries(10, 11)[2:]
        # gene pairs sharing a process (the benchmark samples random genes)
        for genes in (["g3", "g5"], ["g1", "g2"], ["g0", "g7", "g9"]):
            out += benchmark_queries(genes)
        out += random_queries(rng, ["Member", "Inheritance"],
                              [("Gene", f"g{i}") for i in range(0, 120, 7)] +
                              [("BiologicalProcess", f"bp{i}") for i in range(0, 60, 3)], 30)
        out += [T("Member", TV("A", "Uniprot"), TV("B", "BiologicalProcess")),
                T("List", TV("A", "Uniprot"), TV("B", "Concept")),
                L("Context", T("Member", TV("A", "Uniprot"), TV("B", "Reactome")),
                  L("Evaluation", N("Predicate", "has_location"),
                    T("List", TV("A", "Uniprot"), TV("C", "Concept")))),
                ["And", [L("Evaluation", N("Predicate", "has_name"), V("L")), L("List", V("U"), V("Nm"))]],
                ["And", [L("List", V("U"), N("Concept", "loc0")), L("Member", V("U"), V("R"))]]]
    elif name == "flybase":
        sys.path.insert(0, ROOT)
        import bench
        for gene in (0, 7, 42, 149):
            out += [q for _, q in bench.flybase_specs(gene, synthetic.flybase_do_terms(arrays, gene))]
    elif name == "powerlaw":
        out += random_queries(rng, ["T0", "T1", "T2"], [("Concept", f"n{i}") for i in
                                                          list(range(6)) + list(range(20, 300, 23))], 60,
                              arity3=True)
    elif name == "hub":
        import bench
        out += [q for _, q in bench.hub_specs()]
        n = lambda i: N("Concept", f"n{i}")  # noqa: E731
        out += [["And", [L("T0", V("V1"), n(0)), L("T0", V("V1"), V("V2")), L("T0", V("V2"), n(1)),
                         L("T0", V("V2"), V("V3"))]],
                ["And", [L("T1", n(0), V("V1")), L("T2", V("V1"), V("V2")), L("T3", V("V2"), n(0))]]]
    return out


def no_overload_picks(queries):
    """A few ordered join shapes re-answered under CONFIG['no_overload']."""
    picks = [q for q in queries if q[0] == "And" and all(t[0] == "Link" and t[2] for t in q[1])]
    return [dict(query=q, no_overload=True) for q in picks[:8]]


def main():
    os.makedirs(SCRATCH, exist_ok=True)
    specs = []
    for name in (sys.argv[1:] or list(KBS)):
        arrays = make_arrays(name)
        text = synthetic.to_canonical(arrays)
        path = os.path.join(SCRATCH, f"{name}.metta")
        with open(path, "w") as f:
            f.write(text)
        qs = queries_of(name, arrays)
        entries = [dict(query=q) for q in qs] + no_overload_picks(qs)
        fn, kw = KBS[name]
        specs.append({"name": name, "path": path, "queries": entries,
                      "generator": {"function": f"das_amd.synthetic.{fn}", "kwargs": kw},
                      "text_sha256": hashlib.sha256(text.encode()).hexdigest()})
        print(f"{name}: {arrays.n_expr} expressions, {len(entries)} queries, {len(text)} B", file=sys.stderr)
    with open(os.path.join(SCRATCH, "synthetic_specs.json"), "w") as f:
        json.dump(specs, f)


if __name__ == "__main__":
    main()
