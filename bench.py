"""bench.py — DAS query hot path on MI355X: bindings/s + HBM roofline.

Headline (BASELINE.json configs[1], the config the metric is quoted on that
fits one GPU): a seeded synthetic gene-level KB in scripts/benchmark.py's shape
(Member(Gene, BiologicalProcess) with Zipf(1.1) process popularity,
Inheritance(BP, BP)); the real bio_atomspace dump is not available offline.
One step = one pass of the query batch below through the reference API
(`expr.matched(db, answer)`), single-Link and 2-clause And queries:

  Q1 Member(V_g, V_bp)                                  full single-link scan
  Q2 And[Member(V_g, V_bp), Inheritance(V_bp, V_p)]     2-clause join
  Q3 And[Member(g_a, V_bp), Member(g_b, V_bp)]          _same_biological_process
  Q4 And[Member(V_g, bp_hub), Member(V_g, V_bp)]        hub join

value = distinct bindings produced by all ranks / wall time (answers counted
on the device, no Python object materialisation).  Multi-GPU: Member links
live on their gene's rank, Inheritance links on their handle's owner; And
joins are placed by cost (co-located / broadcast / all-to-all exchange,
das_amd/parallel.py); per-rank KB size is fixed (weak scaling).

The default run (`--workload all`) then measures the other configurations
one after another in the same process and adds their lines under
"workloads" (each with its own roofline, kernel table and CPU baseline):
  flybase  config 3: FlyBase-shaped Execution(Schema, key, value) KB, the
           QueryFlyBase.ipynb And / And+Not / Or query shapes, a fresh gene
           anchor per step (fixed KB, links sharded by handle: strong scaling)
  hub      config 5: 10^9-link power-law KB generated in HBM, 4-clause And
           on the top-degree hub nodes
  build    config 4: bulk ExpressionHasher + interning + pattern / template /
           incoming CSR build of the 10^9-link KB; value = links indexed per
           second of device time (at N GPUs: hash-owner regrouping + RCCL
           all-to-all + per-shard build)
`--workload X` runs one of them alone (the line is then X's own);
`--workload load` measures the canonical MeTTa reader -> device index path.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
# --batch -1: how a workload's timed step submits its queries -- the faster
# mode in round 6's same-process pairs (the other is timed beside it, fresh
# anchors): bio one by one 1.57-1.64 ms vs batched 1.67-1.73 (the batch's
# up-front lowering leaves the GPU idle, and its nested plans contend with the
# cross product; profiles/r6_bio_step_split.json); FlyBase batched 0.21-0.25 vs
# 0.25-0.32 (chains on side streams launched in the other plans' waits); hub
# batched 0.77-0.79 vs 0.84 (H2's expansion beside H4's latency-bound walk)
BATCH_DEFAULT = {"bio": 0, "flybase": 1, "hub": 1}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="all", choices=["all", "bio", "flybase", "hub", "build", "load",
                                                          "getlinks"])
    ap.add_argument("--legs", default="auto",
                    help="with --workload all: comma list of the extra workloads (auto: flybase,hub,build,getlinks "
                         "on one GPU; build at N > 1)")
    ap.add_argument("--leg-cpu-seconds", type=float, default=8.0,
                    help="CPU-baseline budget of each extra workload of --workload all")
    ap.add_argument("--build-warmup", default="full", choices=["full", "small"],
                    help="config 4 warm-up build: the same input (default; the timed build then reuses every "
                         "device block) or a 10^4-link KB")
    ap.add_argument("--batch", type=int, default=-1, choices=[-1, 0, 1],
                    help="1: a step's queries in one das_plan_execute_many call (pm.matched_many); 0: "
                         "query.matched(db, answer) one by one, the reference's call pattern; -1 (default): per "
                         "workload, the faster of the two as measured (BATCH_DEFAULT); the other is timed too")
    ap.add_argument("--events", default="dominant", choices=["dominant", "all", "none"],
                    help="timed-step HIP events: around the dominant kernel only, around every kernel scope, or none "
                         "(A/B of the events' own cost; the roofline then comes from the profiled warmup step)")
    # bio (config 2)
    ap.add_argument("--genes", type=int, default=200_000)
    ap.add_argument("--bps", type=int, default=50_000)
    ap.add_argument("--members", type=int, default=20_000_000)
    ap.add_argument("--inheritance", type=int, default=100_000)
    # flybase (config 3): ~27.9M links like the notebook KB (SimplePatternMiner.ipynb:19)
    ap.add_argument("--fb-genes", type=int, default=300_000)
    ap.add_argument("--fb-schema", type=int, default=60)
    ap.add_argument("--fb-rows", type=int, default=450_000)
    ap.add_argument("--gl-steps", type=int, default=3, help="getlinks: seed walks timed (at most --steps)")
    ap.add_argument("--gl-pattern-s", type=float, default=10.0,
                    help="getlinks: seconds of pattern counts per walk (the sample's first links)")
    # hub (config 5): H4's output grows ~ links^1.6 (Zipf hubs): 3M links -> ~4.3e8 bindings
    ap.add_argument("--hub-links", type=int, default=1_000_000_000)
    ap.add_argument("--hub-nodes", type=int, default=1 << 27)
    # build (config 4)
    ap.add_argument("--links", type=int, default=1_000_000_000)
    ap.add_argument("--nodes", type=int, default=1 << 27)
    ap.add_argument("--gen", default="device", choices=["device", "host"],
                    help="build/hub input: generated in HBM (default) or by numpy on the host")
    # load (canonical text): ~100 B a line
    ap.add_argument("--load-genes", type=int, default=200_000)
    ap.add_argument("--load-rows", type=int, default=200_000)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-materialise", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="no per-query timings and no join-probe variants after the timed steps (profiling runs: "
                         "the timed steps' launches are then the process's last ones)")
    ap.add_argument("--materialise-cap", type=int, default=2_000_000,
                    help="largest answer whose Python objects the materialisation-inclusive figure builds")
    ap.add_argument("--cprofile", default=None, help="write a host-side cProfile of 3 extra steps here")
    ap.add_argument("--detail", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="file for the full record (kernel tables, join variants, materialisation); the last stdout "
                         "line is the compact <= 4 KB summary")
    return ap.parse_args()


# ---------------------------------------------------------------------------
# workloads: KB + queries (the same spec drives the oracle's CPU baseline)
# ---------------------------------------------------------------------------
def _V(n):
    return ["Var", n]


def _L(t, *targets):
    return ["Link", t, True, list(targets)]


def _TV(n, t):
    return ["TVar", n, t]


def _T(t, *targets):
    return ["Template", t, True, list(targets)]


def reference_benchmark_specs(ga, gb):
    """scripts/benchmark.py:89-128 QUERY_1-3 on one gene pair (Q3, Q5, Q6)."""
    g = lambda i: ["Node", "Gene", f"g{i}"]  # noqa: E731
    member = lambda a, b: _L("Member", a, b)  # noqa: E731
    same_bp = ["And", [member(g(ga), _V("V_BiologicalProcess")), member(g(gb), _V("V_BiologicalProcess"))]]
    bpt = lambda n: _TV(n, "BiologicalProcess")  # noqa: E731
    same_or_inherited = ["And", [
        member(g(ga), _V("V1_BiologicalProcess")),
        ["Or", [["And", [member(g(gb), _V("V2_BiologicalProcess")),
                         _T("Inheritance", bpt("V2_BiologicalProcess"), bpt("V3_BiologicalProcess")),
                         _T("Inheritance", bpt("V1_BiologicalProcess"), bpt("V3_BiologicalProcess"))]],
                member(g(gb), _V("V1_BiologicalProcess"))]]]]
    up, r = _TV("V_Uniprot", "Uniprot"), _TV("V_Reactome", "Reactome")
    evaluation = lambda p, a, b: _L("Evaluation", ["Node", "Predicate", p], _T("List", a, b))  # noqa: E731
    reactome = ["And", [
        same_bp,
        _T("Member", up, _TV("V_BiologicalProcess", "BiologicalProcess")),
        evaluation("has_name", up, _TV("V_UniprotName", "Concept")),
        _L("Context", _T("Member", up, r), evaluation("has_location", up, _TV("V_Location", "Concept"))),
        evaluation("has_name", r, _TV("V_ReactomeName", "Concept"))]]
    return same_bp, same_or_inherited, reactome


def bio_specs(rank_genes, seed=17, anchor=0):
    """Q1-Q6; `anchor` picks the gene pair of the reference's own queries
    (each timed step uses its own, so no step replays an anchored lookup of
    an earlier one)."""
    import numpy as np
    rng = np.random.default_rng(seed + 7919 * anchor)
    ga, gb = (int(x) for x in rng.choice(rank_genes, 2, replace=False))
    bp = lambda i: ["Node", "BiologicalProcess", f"bp{i}"]  # noqa: E731
    q1, q2, q3 = reference_benchmark_specs(ga, gb)
    return [
        ("Q1 Member(Vg,Vbp)", _L("Member", _V("V_g"), _V("V_bp"))),
        ("Q2 Member*Inheritance", ["And", [_L("Member", _V("V_g"), _V("V_bp")),
                                           _L("Inheritance", _V("V_bp"), _V("V_p"))]]),
        ("Q3 same_biological_process (QUERY_1)", q1),
        ("Q4 hub join", ["And", [_L("Member", _V("V_g"), bp(0)), _L("Member", _V("V_g"), _V("V_bp"))]]),
        ("Q5 same_or_inherited_biological_process (QUERY_2)", q2),
        ("Q6 linked_reactome_uniprot (QUERY_3)", q3),
    ]


def flybase_specs(gene=7, do_terms=()):
    """QueryFlyBase.ipynb cells 5, 6, 7 and 9 (and the full uniquename x
    recombination_loc join the notebook's loops walk), on one gene's FB id."""
    s = lambda n: ["Node", "Schema", "Schema:" + n]  # noqa: E731
    fb = ["Node", "Verbatim", f"FBgn{gene:07d}"]
    E = lambda *t: _L("Execution", *t)  # noqa: E731
    rec, cyto, uniq, do = (s("gene_map_table_recombination_loc"), s("gene_map_table_cytogenetic_loc"),
                           s("gene_uniquename"), s("disease_model_annotations_DO_term"))
    v = _V
    specs = [
        ("F5 same recombination_loc", ["And", [E(rec, fb, v("v1")), E(rec, v("v2"), v("v1")), E(uniq, v("v3"), v("v2"))]]),
        ("F6 same cytogenetic_loc", ["And", [E(cyto, fb, v("v1")), E(cyto, v("v2"), v("v1")), E(uniq, v("v3"), v("v2"))]]),
        ("F7 same recomb, different cyto", ["And", [E(rec, fb, v("v1")), E(rec, v("v2"), v("v1")), E(cyto, fb, v("v3")),
                                                   ["Not", E(cyto, v("v2"), v("v3"))], E(uniq, v("v4"), v("v2"))]]),
        ("F9 DO-term Or", ["Or", [E(do, v("v1"), ["Node", "Verbatim", d]) for d in do_terms] or
                           [E(do, v("v1"), ["Node", "Verbatim", "DOID:0"])]]),
        ("FJ uniquename x recombination_loc", ["And", [E(uniq, v("v3"), v("v2")), E(rec, v("v2"), v("v1"))]]),
    ]
    return specs


def hub_specs():
    """Config 5: 4-clause And anchored on the two highest-degree nodes (Zipf
    ranks 0 and 1), one link type per clause, and its 2-clause prefix (the
    skewed hub join itself: every T1 link out of a T0-neighbour of h0).  At
    10^9 links an unanchored last clause (T(V2, V3)) would expand through hub
    out-degrees to ~10^14 rows, so the 4-clause And closes on the hubs."""
    n = lambda i: ["Node", "Concept", f"n{i}"]  # noqa: E731
    return [
        ("H4 T0(V1,h0) T1(V1,V2) T2(V2,h1) T3(V2,h0)",
         ["And", [_L("T0", _V("V1"), n(0)), _L("T1", _V("V1"), _V("V2")), _L("T2", _V("V2"), n(1)),
                  _L("T3", _V("V2"), n(0))]]),
        ("H2 T0(V1,h0) T1(V1,V2)", ["And", [_L("T0", _V("V1"), n(0)), _L("T1", _V("V1"), _V("V2"))]]),
    ]


# ---------------------------------------------------------------------------
# the DBInterface surface behind the reference's only published timings
# (notebooks/SimplePatternMiner.ipynb): a halo walk of get_links(None, None,
# template) + get_link_targets around a seed node, then pattern counting
# len(get_links(type, None, template)) over a sample of the walked links
# ---------------------------------------------------------------------------
W_ = "*"


def _halo_templates(h):
    """SimplePatternMiner.ipynb cell 6 (:395-401)."""
    return [[h, W_], [W_, h], [h, W_, W_], [W_, h, W_], [W_, W_, h]]


def _pattern_templates(link_type, targets):
    """build_patterns' templates per link (cell 5, arity 2 / 3)."""
    if len(targets) == 2:
        return [[link_type, W_, targets[1]], [link_type, targets[0], W_]]
    if len(targets) == 3:
        t0, t1, t2 = targets
        return [[link_type, W_, t1, t2], [link_type, t0, W_, t2], [link_type, t0, t1, W_],
                [link_type, W_, W_, t2], [link_type, W_, t1, W_], [link_type, t0, W_, W_]]
    return []


def miner_walk(api, seeds, rng, link_rate=0.01, max_pattern_links=2000, halo_length=2,
               max_level_nodes=1000, max_level_links=50_000, progress=None, pattern_budget_s=None):
    """SimplePatternMiner.ipynb cells 6 and 9 through the facade API `api`
    (get_links / get_link_targets / get_link_type / get_node_type /
    get_node_name): the halo walk (level by level, every template around
    every node handle, get_link_targets of every link found) and
    build_patterns' counts over the level-0 links plus a `link_rate` sample
    of the deeper ones.  Returns per phase: seconds, calls, links.

    A FlyBase schema or predicate node sits in millions of links, so a
    level expands at most `max_level_nodes` node handles and follows the
    targets of at most `max_level_links` links (in handle order, so every
    backend walks the same links); a level that hit a bound says so
    ("bounded").  `pattern_budget_s` ends the pattern counts after that many
    seconds (a count over a schema node materialises ~10^6 handles)."""
    node_handles = sorted(set(seeds))[:max_level_nodes]
    levels, halo = [], []
    for lv in range(halo_length):
        t0 = time.perf_counter()
        new_nodes, level_links, n_queries, bounded, rows = set(), set(), 0, False, 0
        t_log = t0
        for k, h in enumerate(node_handles):
            if progress and time.perf_counter() - t_log > 30:
                t_log = time.perf_counter()
                progress(f"halo level {lv}: node {k} of {len(node_handles)}, {n_queries} queries")
            for tpl in _halo_templates(h):
                found = sorted(set(api.get_links(None, None, tpl)))
                rows += len(found)
                n_queries += 1                                    # the notebook's count (:411-413):
                for link in found:                                # get_links + one per link found
                    if link not in level_links and len(level_links) >= max_level_links:
                        bounded = True
                        break
                    n_queries += 1
                    level_links.add(link)
                    new_nodes.update(api.get_link_targets(link))
        bounded = bounded or len(new_nodes) > max_level_nodes
        halo.append({"s": time.perf_counter() - t0, "queries": n_queries, "links": len(level_links),
                     "nodes": len(node_handles), "bounded": bounded, "rows": rows})
        if progress:
            progress(f"halo level {lv}: {len(node_handles)} nodes, {n_queries} queries, {len(level_links)} links")
        levels.append(level_links)
        node_handles = sorted(new_nodes)[:max_level_nodes]
    sample = sorted(levels[0])
    for lv in levels[1:]:
        sample += [link for link in sorted(lv) if rng.random() < link_rate][:max_pattern_links]
    t0 = time.perf_counter()
    calls, counted, done, t_log = 0, 0, 0, t0
    for link in sample:
        now = time.perf_counter()
        if pattern_budget_s is not None and now - t0 > pattern_budget_s:
            break
        if progress and now - t_log > 30:
            t_log = now
            progress(f"pattern counts: {done} of {len(sample)} links, {calls} get_links")
        done += 1
        targets = api.get_link_targets(link)
        link_type = api.get_link_type(link)
        for tpl in _pattern_templates(link_type, targets):
            try:                                                  # build_pattern_from_template
                for t in tpl[1:]:
                    if t != W_:
                        api.get_node_type(t)
                        api.get_node_name(t)
            except Exception:
                continue
            counted += len(api.get_links(tpl[0], None, tpl[1:]))
            calls += 1
    if progress:
        progress(f"pattern counts: {done} links, {calls} get_links, {counted} matched")
    return {"halo": halo, "pattern": {"s": time.perf_counter() - t0, "links": done, "get_links": calls,
                                      "matched": counted, "sampled": len(sample)}}


class OracleFacade:
    """The facade calls miner_walk makes, over the oracle's DB-path
    restatement (distributed_atom_space.py:259-296 over RedisMongoDB)."""

    def __init__(self, odb):
        self.db = odb

    def get_links(self, link_type, target_types=None, targets=None):
        link_type = W_ if link_type is None else link_type
        if target_types is not None and link_type != W_:
            ans = self.db.get_matched_type_template([link_type, *target_types])
        elif targets is not None:
            ans = self.db.get_matched_links(link_type, targets)
        else:
            ans = self.db.get_matched_type(link_type)
        return [a if isinstance(a, str) else a[0] for a in ans]

    def __getattr__(self, name):
        return getattr(self.db, name)


def build_expr(pm, spec):
    k = spec[0]
    if k == "Node":
        return pm.Node(spec[1], spec[2])
    if k == "Var":
        return pm.Variable(spec[1])
    if k == "TVar":
        return pm.TypedVariable(spec[1], spec[2])
    if k == "Template":
        return pm.LinkTemplate(spec[1], [build_expr(pm, t) for t in spec[3]], spec[2])
    if k == "Link":
        return pm.Link(spec[1], [build_expr(pm, t) for t in spec[3]], spec[2])
    if k == "Not":
        return pm.Not(build_expr(pm, spec[1]))
    return (pm.And if k == "And" else pm.Or)([build_expr(pm, t) for t in spec[1]])


def make_kb(args, rank, world, db):
    """(AtomArrays for this rank, specs_of(step) -> query specs, config dict,
    scaling).  Anchored queries take a different anchor every step."""
    import numpy as np
    from das_amd import parallel, synthetic
    if args.workload == "bio":
        if world == 1:
            arrays = synthetic.bio_full_kb(args.genes, args.bps, args.members, args.inheritance)
            rank_genes = np.arange(args.genes)
        else:
            arrays, rank_genes = parallel.bio_shard(args.genes, args.bps, args.members, args.inheritance, rank, world)
        cfg = {"workload": "config2 bio gene-level KB (+ annotation layouts): single-Link + 2-clause And (Q1-Q4) "
                           "+ scripts/benchmark.py QUERY_1-3 (Q3, Q5, Q6)",
               "genes_per_rank": int(len(rank_genes)), "bps": args.bps, "member_links_per_rank": args.members,
               "inheritance_links": args.inheritance}
        if world == 1:
            return arrays, lambda i: bio_specs(rank_genes, anchor=i), cfg, "weak"

        def specs(i):
            # the same expressions on every rank (each is one collective plan):
            # Q1 / Q2 / Q4 over every rank's Member links, and one instance of
            # the anchored QUERY_1-3 per rank, on a gene pair of that rank's
            # range (bio_shard: the same Member rows as the 1-GPU KB's genes, so
            # each instance answers as at 1 GPU; gathered plans are evaluated
            # by one rank each, round robin)
            out = [q for q in bio_specs(np.arange(args.genes), anchor=i) if q[0][:2] in ("Q1", "Q2", "Q4")]
            for r in range(world):
                out += [(f"{name} @rank{r}", q)
                        for name, q in bio_specs(np.arange(r * args.genes, (r + 1) * args.genes), anchor=i)
                        if name[:2] in ("Q3", "Q5", "Q6")]
            return out
        cfg["anchored_instances"] = "QUERY_1-3 (Q3, Q5, Q6) once per rank per step, each on its rank's genes"
        return arrays, specs, cfg, "weak"
    if args.workload == "flybase":
        arrays = synthetic.flybase_kb(args.fb_genes, args.fb_schema, args.fb_rows)
        # one gene anchor per step; each gene's DO terms (cell 9 builds its Or
        # from them), read off the arrays
        n = args.warmup + args.steps + 2
        genes = [(7 + 7919 * i) % args.fb_genes for i in range(n)]
        do_terms = {g: synthetic.flybase_do_terms(arrays, gene=g) for g in genes}
        arrays = parallel.shard_arrays(arrays, rank, world)
        cfg = {"workload": "config3 FlyBase-shaped Execution KB: QueryFlyBase.ipynb And/And+Not/Or shapes",
               "links": int(arrays.n_expr), "genes": args.fb_genes, "schemas": args.fb_schema,
               "anchors": "a different gene per step"}
        return arrays, lambda i: flybase_specs(genes[i % n], do_terms[genes[i % n]]), cfg, "strong"
    if args.gen == "device":
        # every rank generates the whole KB as its atom directory and indexes
        # the links whose handle it owns (das_build_index_sharded)
        arrays = synthetic.powerlaw_kb_device(db.ctx, args.hub_nodes, args.hub_links, link_types=4,
                                              shard=(rank, world), device=db.ctx.device)
    else:
        arrays = synthetic.powerlaw_kb(args.hub_nodes, args.hub_links, link_types=4)
        arrays = parallel.shard_arrays(arrays, rank, world)
    cfg = {"workload": "config5 power-law hypergraph: 4-clause And on hub nodes",
           "links": args.hub_links, "nodes": args.hub_nodes, "link_types": 4, "arity": "70% 2 / 30% 3",
           "generated": args.gen}
    return arrays, lambda i: hub_specs(), cfg, "strong"


def cpu_cores():
    """Host cores this process may use: the affinity set, capped by
    OMP_NUM_THREADS (the GPU box exports its CPU share there; nproc and
    os.cpu_count() show the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, cap) if cap > 0 else n)


def _cpu_sample(workload, args_d):
    """(AtomArrays, query specs, description) of the bounded CPU sample of a
    workload: the same generators and query shapes at reduced scale."""
    from das_amd import synthetic
    a = argparse.Namespace(**args_d)
    if workload == "bio":
        scale = 1000
        genes, bps = max(a.genes // scale, 50), max(a.bps // scale, 20)
        members, inh = max(a.members // scale, 500), max(a.inheritance // scale, 40)
        arrays = synthetic.bio_full_kb(genes, bps, members, inh, n_uniprot=max(5000 // scale, 20),
                                       n_up_member=max(50_000 // scale, 100), n_reactome=max(1000 // scale, 10),
                                       n_context=max(20_000 // scale, 40))
        specs = [s for k in range(8) for _, s in bio_specs(range(1, genes), anchor=k)]
        what = f"bio_full_kb(genes={genes}, bps={bps}, members={members}, inheritance={inh}) = 1/{scale} of the GPU workload"
    elif workload == "flybase":
        scale = 1000
        arrays = synthetic.flybase_kb(max(a.fb_genes // scale, 100), max(a.fb_schema // 10, 4),
                                      max(a.fb_rows // scale, 200), n_loc=50, n_do=40)
        specs = [s for g in range(0, 96, 3) for _, s in flybase_specs(g, synthetic.flybase_do_terms(arrays, gene=g))]
        what = f"flybase_kb at 1/{scale} of the GPU workload, 32 gene anchors"
    else:
        scale = max(a.hub_links // 30_000, 1)      # ~30 k links: a few oracle passes in the budget
        arrays = synthetic.powerlaw_kb(max(a.hub_nodes // scale, 200), max(a.hub_links // scale, 2000),
                                       link_types=4)
        specs = [s for _, s in hub_specs()]
        what = f"powerlaw_kb at 1/{scale} of the GPU workload"
    return arrays, specs, what


def _cpu_query_worker(job):
    """One process of the CPU baseline: evaluates whole queries, one at a
    time, round-robin from its offset, until the budget is spent.  fast:
    the oracle's And fold joins by hash on the shared variables (FAST_JOIN);
    else the reference's nested loop (pattern_matcher.py:732-738)."""
    workload, args_d, wid, budget, fast = job
    from oracle import das_oracle as O
    O.FAST_JOIN = bool(fast)
    arrays, specs, _ = _cpu_sample(workload, args_d)
    db = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    total, done, i = 0, 0, wid
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget:
        total += O.evaluate(specs[i % len(specs)], db).get("n", 0)
        done += 1
        i += 1
    return total, done, time.perf_counter() - t0


def _cpu_build_worker(job):
    """One process of the build CPU baseline: the oracle's ExpressionHasher
    + key-value index restatement (canonical_parser.py:132-183) over its own
    seeded power-law sample, repeated until the budget is spent."""
    wid, n_links, n_nodes, budget = job
    from das_amd import synthetic
    from oracle import das_oracle as O
    arrays = synthetic.powerlaw_kb(n_nodes, n_links, link_types=4, seed=1000 + wid)
    links, reps = 0, 0
    t0 = time.perf_counter()
    while True:
        kb = O.KB.from_arrays(arrays)         # md5 handles + composite types of every atom
        O.keyspace_lines(kb)                  # outgoing / incoming / pattern / template / name families
        links += len(kb.links)
        reps += 1
        if time.perf_counter() - t0 > budget:
            break
    return links, reps, time.perf_counter() - t0


def _calibration(join="nested"):
    """The oracle's time over the reference's on the reference-answered
    fixtures, for the And join the baseline ran (tools/calibrate_cpu.py)."""
    path = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        c = json.load(f)
    r = (c.get("joins") or {}).get(join) or {}
    return {"oracle_over_reference_time": r.get("ratio_all"), "join": join,
            "source": "profiles/cpu_calibration.json", "how": c.get("what")}


def _pool_map(fn, jobs):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")       # fresh interpreters: nothing of this process's GPU state
    with ctx.Pool(len(jobs)) as pool:
        return pool.map(fn, jobs)


def cpu_baseline(args, budget_s, fast=False):
    """The oracle on a bounded sample of the same workload, one process per
    host core, each evaluating whole queries one at a time (SURVEY.md
    §8d(ii)).  Default: the oracle's And fold as the reference's nested loop
    over both sides' assignments (FAST_JOIN = False; pattern_matcher.py:
    732-738), i.e. the reference's complexity -- its time against the
    reference's own on the reference-answered fixtures is the calibration
    (profiles/cpu_calibration.json, "nested").  fast: the oracle's hash join
    on the shared variables (same rows), reported apart as cpu_fast."""
    cores = cpu_cores()
    args_d = vars(args)
    _, specs, what = _cpu_sample(args.workload, args_d)
    t0 = time.perf_counter()
    res = _pool_map(_cpu_query_worker, [(args.workload, args_d, w, budget_s, fast) for w in range(cores)])
    wall = time.perf_counter() - t0
    total = sum(r[0] for r in res)
    done = sum(r[1] for r in res)
    span = max(r[2] for r in res)
    join = ("hash join on the shared variables (oracle FAST_JOIN=True, not the reference's complexity)" if fast
            else "nested-loop And (oracle FAST_JOIN=False, the reference's complexity)")
    return {"value": total / span, "unit": "bindings/s", "cores": cores, "kind": "port",
            "join": "hash" if fast else "nested",
            "sample": f"oracle, {join}, on {what}; {len(specs)} query instances, "
                      f"{cores} processes x one whole query at a time, {done} queries in {span:.1f} s "
                      f"({wall:.1f} s with interpreter start-up)",
            "calibration": _calibration("hash" if fast else "nested")}


def cpu_baseline_build(args, budget_s):
    cores = cpu_cores()
    n_links, n_nodes = 20_000, 4_000
    t0 = time.perf_counter()
    res = _pool_map(_cpu_build_worker, [(w, n_links, n_nodes, budget_s) for w in range(cores)])
    span = max(r[2] for r in res)
    links = sum(r[0] for r in res)
    return {"value": links / span, "unit": "links/s", "cores": cores, "kind": "port",
            "sample": f"oracle ExpressionHasher + key-value index restatement (KB.from_arrays + keyspace_lines) "
                      f"of powerlaw_kb({n_nodes} nodes, {n_links} links) per process, {cores} processes, "
                      f"{sum(r[1] for r in res)} builds in {span:.1f} s ({time.perf_counter() - t0:.1f} s wall)"}


def roofline_of(stats, workload="bio", name=None):
    """Dominant single-kernel scope ("k_*", one template instantiation) of
    the timed region -> roofline; multi-launch phases (join_build,
    incoming_csr, ...) are reported under "kernels" but are not a kernel's
    roofline.  achieved = algorithmic bytes per launch / mean launch time."""
    single = {k: v for k, v in stats.items() if k.startswith("k_")}
    if not single:
        return None
    if name is None or name not in single:
        name = max(single.items(), key=lambda kv: kv[1]["ms"])[0]
    st = single[name]
    achieved = st["bytes"] / (st["ms"] * 1e-3) / 1e9 if st["ms"] > 0 else 0.0
    traffic = None
    # per-kernel HBM bytes from this workload's rocprofv3 PMC passes (tools/profile_bench.sh)
    pmc = os.path.join(ROOT, "profiles", f"pmc_traffic_{workload}.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get(name, {}).get("bytes_per_launch")
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": name,
            "avg_launch_us": round(st["ms"] * 1e3 / max(st["launches"], 1), 2), "launches": st["launches"],
            "algorithmic_bytes_per_launch": st["bytes"] / max(st["launches"], 1)}


def kernels_of(stats):
    """Per scope: total ms, launches, mean launch us, algorithmic GB/s."""
    return {k: {"ms": round(v["ms"], 3), "launches": v["launches"],
                "avg_us": round(v["ms"] * 1e3 / max(v["launches"], 1), 2),
                "GBps": round(v["bytes"] / max(v["ms"], 1e-9) / 1e6, 1)}
            for k, v in sorted(stats.items(), key=lambda kv: -kv[1]["ms"])}


# ---------------------------------------------------------------------------
# config 4: bulk index build
# ---------------------------------------------------------------------------
def _sync_max(dist, values, device):
    """Element-wise max over ranks of a few floats (rank timings)."""
    import torch
    if not dist:
        return [float(v) for v in values]
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


def _sync_sum(dist, values, device):
    import torch
    if not dist:
        return [float(v) for v in values]
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return [float(x) for x in t.tolist()]


def build_algorithmic_bytes(n_links, frac_arity2=0.7):
    """SURVEY.md §8d config-4 algorithmic bytes: hash (arity*16 + 16) in + 16
    out per link, CSR 2*arity*4 + 4 per link."""
    n2 = int(n_links * frac_arity2)
    n3 = n_links - n2
    return n2 * (2 * 16 + 16 + 16 + 2 * 2 * 4 + 4) + n3 * (3 * 16 + 16 + 16 + 2 * 3 * 4 + 4)


def run_build(args, rank, world, dist, local_rank, backend="nccl"):
    """Config 4.  One GPU: the device build of the whole generated KB.  N GPUs:
    rank r generates the global link range [r L / N, (r+1) L / N) in HBM; the
    timed region hashes it (das_hash_owners), groups the rows by the owner of
    their handles (das_partition_rows), sends them to the owners with one RCCL
    all-to-all per arity and builds the shard it received -- links
    hash-partitioned by handle, each distinct link indexed on exactly one GPU.
    Inputs are resident in HBM when the timing starts; the host leaf strings'
    upload is input hand-over and is not timed (reported as wall_incl_upload_s)."""
    import torch
    from das_amd import parallel, synthetic
    from das_amd.database.hip_db import HipDB
    dev = torch.device("cuda", local_rank)
    t0 = time.perf_counter()
    db = HipDB(device=local_rank)
    log(f"generating {args.links} links ({args.gen})")
    if args.gen == "device":
        lo, hi = args.links * rank // world, args.links * (rank + 1) // world
        arrays = synthetic.powerlaw_kb_device(db.ctx, args.nodes, args.links, link_types=4, first=lo,
                                              count=hi - lo, device=local_rank)
    else:
        arrays = synthetic.powerlaw_kb(args.nodes, args.links, link_types=4)
        arrays = parallel.partition_arrays(arrays, rank, world)      # independent shards: strong scaling
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    # warm-up build: code objects and pools, and at N = 1 the same input, its
    # blocks all kept by the caching allocator (DAS_BUILD_KEEP_GB), so the
    # timed build maps no new device memory -- a fresh multi-GB hipMalloc in
    # the timed region stalled 1.4-1.9 s in ~1 of 3 processes (DAS_ALLOC_TRACE,
    # profiles/r5_build_alloc_stall.txt); --build-warmup small: round 4's
    # 10^4-link warm-up
    # (the warm-up build is also the cold one: its wall time, driver
    # allocations included, is reported as cold_build_ms; the timed build then
    # runs as any rebuild does -- its idle blocks returned at its end, after
    # its last kernel -- with the warm-up's blocks to reuse)
    keep_env = os.environ.get("DAS_BUILD_KEEP_GB")
    full_warm = args.build_warmup == "full" and world == 1
    t_cold = time.perf_counter()
    if full_warm:
        os.environ["DAS_BUILD_KEEP_GB"] = "100000"
        db.load_arrays(arrays)
    else:
        db.load_arrays(synthetic.powerlaw_kb(1000, 10000, link_types=4))
    torch.cuda.synchronize()
    cold_ms = (time.perf_counter() - t_cold) * 1e3
    if full_warm:
        if keep_env is None:
            os.environ.pop("DAS_BUILD_KEEP_GB", None)
        else:
            os.environ["DAS_BUILD_KEEP_GB"] = keep_env
    db.ctx.prof_reset()
    db.ctx.prof_enable(True)
    if dist:
        dist.barrier()
    log("building")
    t1 = time.perf_counter()
    ex_ms = 0.0
    if world > 1 and args.gen == "device":
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ex = parallel.rccl_exchange(dist, cpu_staging=(backend != "nccl"))

        def timed_ex(rows, counts):
            ev[0].record()
            out = ex(rows, counts)
            ev[1].record()
            ev[1].synchronize()
            nonlocal ex_ms
            ex_ms += ev[0].elapsed_time(ev[1])
            return out
        arrays = parallel.regroup_by_owner(db.ctx, arrays, world, timed_ex)
    db.load_arrays(arrays)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t1
    db.ctx.prof_enable(False)
    stats = db.ctx.prof_stats()
    # device time of the timed region: owner hashing + row grouping + the
    # all-to-all + the build (each measured by events on the stream)
    dev_ms = stats.get("build_device", {}).get("ms", wall * 1e3) + stats.get("hash_owners", {}).get("ms", 0.0) + \
        stats.get("partition_rows", {}).get("ms", 0.0) + ex_ms
    st = db.stats()
    local_links = int(st.n_links)
    dev_ms, wall = _sync_max(dist, [dev_ms, wall], dev if backend == "nccl" else "cpu")
    links = int(_sync_sum(dist, [local_links], dev if backend == "nccl" else "cpu")[0])
    # MD5 blocks hashed: a message of L bytes takes
    # ceil((L + 9) / 64) blocks; a composite message is K 32-hex handles joined
    # by spaces (33 K - 1 bytes), a terminal one its "Type name" string; a
    # link hashes two composites (its handle and its composite type)
    import numpy as np
    leaf_len = np.diff(arrays.leaf_off.astype(np.int64))
    blocks_leaf = int(((leaf_len + 9 + 63) // 64).sum())
    if getattr(arrays, "expr_on_device", False):
        nch = arrays.expr_off[1:] - arrays.expr_off[:-1]
        blocks_expr = 2 * int(((33 * nch - 1 + 9 + 63) // 64).sum().item())
        del nch
    else:
        nch = np.diff(arrays.expr_off.astype(np.int64))
        blocks_expr = 2 * int(((33 * nch - 1 + 9 + 63) // 64).sum())
    out = None
    if rank == 0:
        hash_ks = {k: v for k, v in stats.items() if k.startswith("k_hash_group")}
        hms = sum(v["ms"] for v in hash_ks.values())
        hl = stats.get("k_hash_strings", {"ms": 0, "bytes": 0, "launches": 0})
        # §8d algorithmic bytes of the whole build, all links (per GPU: / N)
        algo = build_algorithmic_bytes(args.links)
        achieved = algo / (dev_ms * 1e-3) / 1e9
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            log("cpu baseline")
            cpu = cpu_baseline_build(args, args.cpu_baseline_seconds)
        out = {"metric": "links indexed/s (bulk ExpressionHasher + intern + pattern/template/incoming CSR build)",
               "value": args.links / (dev_ms * 1e-3), "unit": "links/s", "n_gpus": world, "steps": 1, "warmup": 1,
               "ms_per_step": dev_ms, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
               "dtype": "u32",
               "data": "synthetic power-law hypergraph, Zipf(1.1) targets, " + (
                   "generated in HBM (das_synth_powerlaw_links)" if args.gen == "device" else "generated on the host"),
               "config": {"workload": "config4 bulk ExpressionHasher + IncomingSet CSR build", "links": args.links,
                          "nodes": args.nodes, "link_types": 4, "arity": "70% 2 / 30% 3",
                          "distinct_links_indexed": links,
                          "warmup_build": ("same input, its device blocks kept for the timed build (a rebuild: "
                                           "no driver allocation; it returns its idle blocks at its end)")
                          if full_warm else "10^4-link KB",
                          "parallelism": (f"links hash-partitioned by handle x{world}: generated in ranges, "
                                          "regrouped on their owners by RCCL all-to-all" if world > 1 else "1 GPU")},
               # the build's roofline is SURVEY.md §8d's: algorithmic bytes of
               # hash + CSR over all links / device time of the whole build (sort
               # passes, scratch and intern traffic count against it)
               "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS * world,
                            "unit": "GB/s", "frac": round(achieved / (HBM_PEAK_GBS * world), 4), "traffic": None,
                            "kernel": "whole build (SURVEY.md §8d bytes)",
                            "bytes_per_link": "hash (arity*16+16) in + 16 out, CSR 2*arity*4 + 4",
                            "algorithmic_bytes": algo},
               "dominant_kernel": roofline_of(stats, "build"),
               "cpu_baseline": cpu,
               "exchange_ms": round(ex_ms, 3) if world > 1 else None,
               "hash": {"ms": round(hms, 3), "md5_blocks_per_s": (blocks_leaf + blocks_expr) / max((hms + hl["ms"]) * 1e-3, 1e-12),
                        "md5_blocks": blocks_leaf + blocks_expr, "terminal_ms": round(hl["ms"], 3),
                        "valu": md5_valu(hash_ks)},
               "kernels": kernels_of(stats), "wall_incl_upload_s": round(wall, 3), "host_generate_s": round(t_gen, 2),
               "cold_build_ms": round(cold_ms, 1) if full_warm else None,
               "atoms": int(st.n_atoms), "device_bytes": int(st.device_bytes)}
    del db, arrays
    return out


VALU_PEAK_WAVE_INSTR = 256 * 4 * 2.4e9 / 2   # CUs x SIMDs x clock / 2 cycles per wave64 VALU op (MI355X_MICROARCH.md)


def md5_valu(hash_ks):
    """k_hash_group<K> against the VALU issue peak: wave instructions issued
    (static per-thread VALU count of the kernel, profiles/md5_isa.json from
    tools/isa_count.py, x expressions / 64) over the launch time."""
    path = os.path.join(ROOT, "profiles", "md5_isa.json")
    if not os.path.exists(path) or not hash_ks:
        return None
    with open(path) as f:
        isa = json.load(f)["kernels"]
    out = {}
    for k, v in hash_ks.items():
        if k not in isa or v["ms"] <= 0:
            continue
        # bytes scope = expressions * (36 K + 44): recover the expression count
        kk = int(k[k.index("<") + 1:-1])
        n_expr = v["bytes"] / (36.0 * kk + 44.0)
        wi = n_expr / 64.0 * isa[k]["valu"]
        rate = wi / (v["ms"] * 1e-3)
        out[k] = {"valu_per_expr": isa[k]["valu"], "wave_instr_per_s": rate, "peak": VALU_PEAK_WAVE_INSTR,
                  "frac": round(rate / VALU_PEAK_WAVE_INSTR, 4)}
    return out


def materialised_rate(pm, db, qs, cap):
    """Bindings/s including Python object materialisation (the reference's
    answer is a set of Assignment objects, distributed_atom_space.py:298-321):
    each query of one step is evaluated, then its answer's Assignment objects
    are built -- all of them, or the first `cap` rows when the answer is
    larger (the query's device time is then prorated to that slice).  Also
    returns str(set) formatting of the within-cap answers (the facade's
    DistributedAtomSpace.query output)."""
    from das_amd.distributed_atom_space import _format_assignments
    rows_all, t_all, per = 0, 0.0, {}
    fmt_rows, fmt_t = 0, 0.0
    for name, q in qs:
        t0 = time.perf_counter()
        ans = pm.PatternMatchingAnswer()
        q.matched(db, ans)
        c = ans.count()
        t1 = time.perf_counter()
        if c > cap:
            objs = pm._materialize(db, ans._relation(), limit=cap)
        else:
            objs = ans.assignments
        t2 = time.perf_counter()
        n = len(objs)
        if c <= cap and n:
            t3 = time.perf_counter()
            _format_assignments(objs)
            fmt_t += time.perf_counter() - t3
            fmt_rows += n
        tq = (t1 - t0) * (n / c if c else 1.0)
        per[name] = {"bindings": c, "materialised": n, "query_s": round(t1 - t0, 5), "objects_s": round(t2 - t1, 5),
                     "objects_per_s": round(n / (t2 - t1), 1) if t2 > t1 and n else None,
                     "sliced": c > cap}
        rows_all += n
        t_all += tq + (t2 - t1)
        del objs, ans
    return {"value": rows_all / t_all if t_all > 0 else None, "unit": "bindings/s", "bindings": rows_all,
            "seconds": round(t_all, 4), "cap": cap, "queries": per,
            "format_str_set_per_s": round(fmt_rows / fmt_t, 1) if fmt_t > 0 else None,
            "how": "matched() + answer.assignments (C builder of the Assignment objects); answers above `cap` rows: "
                   "the first `cap` rows, query time prorated"}


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def run_load(args, rank, world, local_rank):
    import numpy as np
    import torch
    from das_amd import _lib, synthetic
    from das_amd.database.hip_db import HipDB
    if world > 1 and rank != 0:
        return                      # host parse: one replica is the measurement
    log("generating the canonical text")
    arrays = synthetic.flybase_kb(args.load_genes, 20, args.load_rows)
    text = synthetic.to_canonical(arrays).encode()
    n_lines = text.count(b"\n")
    threads = int(os.environ.get("OMP_NUM_THREADS", "16"))
    db = HipDB(device=local_rank)
    db.load_arrays(_lib.parse_canonical(text[:200000].rsplit(b"\n", 1)[0] + b"\n", threads))   # warm-up
    torch.cuda.synchronize()
    db.ctx.prof_reset()
    db.ctx.prof_enable(True)
    log(f"parsing {len(text) / 1e6:.0f} MB ({n_lines} lines) on {threads} threads")
    t0 = time.perf_counter()
    parsed = _lib.parse_canonical(text, threads)
    t1 = time.perf_counter()
    db.load_arrays(parsed)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    db.ctx.prof_enable(False)
    stats = db.ctx.prof_stats()
    links = int(db.stats().n_links)
    out = {"metric": "links loaded/s (canonical MeTTa text -> native reader -> device index)",
           "value": links / (t2 - t0), "unit": "links/s", "n_gpus": 1, "steps": 1, "warmup": 1,
           "ms_per_step": (t2 - t0) * 1e3, "higher_is_better": True, "scaling": "replicas only",
           "vs_baseline": None, "dtype": "u8",
           "data": "synthetic FlyBase-shaped canonical text (flybase_kb -> to_canonical)",
           "config": {"workload": "canonical load: CanonicalParser.parse + index build", "bytes": len(text),
                      "lines": n_lines, "host_threads": threads},
           "parse_s": round(t1 - t0, 3), "parse_MBps": round(len(text) / (t1 - t0) / 1e6, 1),
           "index_s": round(t2 - t1, 3), "kernels": kernels_of(stats), "roofline": roofline_of(stats, "load"),
           "cpu_baseline": None, "atoms": int(db.stats().n_atoms)}
    if not args.no_cpu_baseline:
        # the oracle's CanonicalParser restatement (parse + md5 of every atom), one core
        from das_amd import loader
        from oracle import das_oracle as O
        small = synthetic.to_canonical(synthetic.flybase_kb(4000, 20, 4000))
        t = time.perf_counter()
        reps = 0
        while True:
            kb = O.KB.from_arrays(loader.parse_canonical(small).finish())
            reps += 1
            if time.perf_counter() - t > args.cpu_baseline_seconds:
                break
        dt = time.perf_counter() - t
        n = len(kb.links)
        out["cpu_baseline"] = {"value": n * reps / dt, "unit": "links/s", "cores": 1, "kind": "port",
                               "sample": f"loader.parse_canonical + oracle md5 hashing of a {len(small)} B "
                                         f"FlyBase-shaped text ({n} links), {reps} passes in {dt:.1f} s"}
    emit(out, args.detail)


def _miner_totals(runs):
    """queries, seconds of the halo walks and pattern counts of miner_walk runs."""
    hq = sum(h["queries"] for r in runs for h in r["halo"])
    hs = sum(h["s"] for r in runs for h in r["halo"])
    pc = sum(r["pattern"]["get_links"] for r in runs)
    ps = sum(r["pattern"]["s"] for r in runs)
    pl = sum(r["pattern"]["links"] for r in runs)
    hr = sum(h.get("rows", 0) for r in runs for h in r["halo"])
    hg = sum(h["nodes"] * 5 for r in runs for h in r["halo"])         # get_links calls (5 templates per node)
    pm_ = sum(r["pattern"]["matched"] for r in runs)
    return {"halo_queries": hq, "halo_s": hs, "halo_ms_per_query": 1e3 * hs / max(hq, 1),
            # per returned row: answers differ in size between the GPU KB and the
            # CPU's 1/300 sample (a hub's pattern key holds ~10^5 rows at full size)
            "halo_rows_per_get_links": hr / max(hg, 1), "halo_us_per_row": 1e6 * hs / max(hr, 1),
            "pattern_rows_per_get_links": pm_ / max(pc, 1), "pattern_us_per_row": 1e6 * ps / max(pm_, 1),
            "level_ms_per_query": [round(1e3 * sum(r["halo"][k]["s"] for r in runs) /
                                         max(sum(r["halo"][k]["queries"] for r in runs), 1), 5)
                                   for k in range(len(runs[0]["halo"]))] if runs else [],
            "pattern_get_links": pc, "pattern_s": ps, "pattern_ms_per_get_links": 1e3 * ps / max(pc, 1),
            # the notebook's own formula: elapsed / (8 x links) (SimplePatternMiner.ipynb:283)
            "pattern_ms_per_notebook_query": 1e3 * ps / max(8 * pl, 1)}


def _gl_cpu_worker(job):
    """CPU baseline of the getlinks leg: miner_walk over the oracle's DB-path
    restatement (dict-backed pattern / template / outgoing families, the
    reference's Redis + Mongo minus the network) on a scaled FlyBase KB."""
    genes, schemas, rows, budget = job
    import numpy as np
    from das_amd import synthetic
    from oracle import das_oracle as O
    arrays = synthetic.flybase_kb(genes, schemas, rows)
    api = OracleFacade(O.RedisMongoSemantics(O.KB.from_arrays(arrays)))
    rng = np.random.default_rng(5)
    runs, i = [], 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget:
        runs.append(miner_walk(api, [O.terminal_hash("gene", f"g{(7 + 7919 * i) % genes}")], rng))
        i += 1
    return runs


def run_getlinks(args, rank, world, local_rank):
    """The DBInterface query surface on the FlyBase-shaped KB (config 3's
    generator at the notebook's size, SimplePatternMiner.ipynb:19): per step
    one seed gene's halo walk (get_links(None, None, template) x 5 templates
    per node, get_link_targets per link, two levels) and build_patterns'
    pattern counts over the walked links -- the calls the reference's only
    published timings measure (2.289 / 0.097-0.131 ms per query, 74-104 ms per
    pattern count).  Host-driven single lookups: one replica
    is the measurement at N GPUs."""
    import numpy as np
    import torch
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    from das_amd.distributed_atom_space import DistributedAtomSpace
    from das_amd.expression_hasher import ExpressionHasher as EH
    if world > 1 and rank != 0:
        return None
    log("generating the FlyBase-shaped KB (getlinks)")
    arrays = synthetic.flybase_kb(args.fb_genes, args.fb_schema, args.fb_rows)
    db = HipDB(device=local_rank)
    db.load_arrays(arrays)
    t_pre = time.perf_counter()
    db.prefetch()                       # host copies of per-atom metadata + outgoing sets (redis_mongo_db.py:89-127)
    t_pre = time.perf_counter() - t_pre
    das = DistributedAtomSpace(db=db)
    steps = max(1, min(args.steps, args.gl_steps))
    seed = lambda i: EH.terminal_hash("gene", f"g{(7 + 7919 * i) % args.fb_genes}")  # noqa: E731
    rng = np.random.default_rng(5)
    log("getlinks warmup walk")
    for i in range(args.warmup and 1):
        miner_walk(das, [seed(1000 + i)], rng, progress=log, pattern_budget_s=args.gl_pattern_s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    runs = []
    for i in range(steps):
        runs.append(miner_walk(das, [seed(i)], rng, progress=log, pattern_budget_s=args.gl_pattern_s))
        log(f"getlinks walk {i}: {sum(h['queries'] for h in runs[-1]['halo'])} queries")
    elapsed = time.perf_counter() - t0
    tot = _miner_totals(runs)
    cpu = None
    if not args.no_cpu_baseline:
        log("cpu baseline (getlinks)")
        scale = 300                     # the oracle's pure-Python KB build: ~20 s at 1/300
        g, r = max(args.fb_genes // scale, 100), max(args.fb_rows // scale, 200)
        cruns = _pool_map(_gl_cpu_worker, [(g, args.fb_schema, r, args.cpu_baseline_seconds)])[0]
        ct = _miner_totals(cruns)
        cpu = {"value": ct["halo_queries"] / max(ct["halo_s"], 1e-9), "unit": "queries/s", "cores": 1,
               "kind": "port",
               "sample": f"miner_walk over the oracle's dict-backed DB-path restatement (no network) on "
                         f"flybase_kb({g} genes, {args.fb_schema} schemas, {r} rows) = 1/{scale} of the GPU KB, "
                         f"{len(cruns)} seeds, one process",
               "halo_ms_per_query": round(ct["halo_ms_per_query"], 5),
               "pattern_ms_per_get_links": round(ct["pattern_ms_per_get_links"], 5),
               "rows": {k: round(ct[k], 4) for k in ("halo_rows_per_get_links", "halo_us_per_row",
                                                     "pattern_rows_per_get_links", "pattern_us_per_row")}}
    if cpu is not None:
        # the two sides answer different KB sizes: rows per get_links and
        # microseconds per returned row, side by side
        cpu["rows_per_get_links"] = {"cpu_halo": round(ct["halo_rows_per_get_links"], 2),
                                     "gpu_halo": round(tot["halo_rows_per_get_links"], 2),
                                     "cpu_pattern": round(ct["pattern_rows_per_get_links"], 1),
                                     "gpu_pattern": round(tot["pattern_rows_per_get_links"], 1)}
        cpu["us_per_row"] = {"cpu_halo": round(ct["halo_us_per_row"], 4), "gpu_halo": round(tot["halo_us_per_row"], 4),
                             "cpu_pattern": round(ct["pattern_us_per_row"], 4),
                             "gpu_pattern": round(tot["pattern_us_per_row"], 4)}
    lat = {"halo_ms_per_query": round(tot["halo_ms_per_query"], 5), "level_ms_per_query": tot["level_ms_per_query"],
           "pattern_ms_per_get_links": round(tot["pattern_ms_per_get_links"], 5),
           "pattern_ms_per_notebook_query": round(tot["pattern_ms_per_notebook_query"], 5),
           "rows": {k: round(tot[k], 4) for k in ("halo_rows_per_get_links", "halo_us_per_row",
                                                  "pattern_rows_per_get_links", "pattern_us_per_row")},
           "published_ms_per_query": {"halo_level1": 2.289, "halo_level2": [0.097, 0.131],
                                      "pattern_count": [74, 104]}}
    out = {"metric": "DBInterface lookups/s (SimplePatternMiner halo walk: get_links + get_link_targets)",
           "value": tot["halo_queries"] / max(tot["halo_s"], 1e-9), "unit": "queries/s", "n_gpus": 1,
           "steps": steps, "warmup": 1, "ms_per_step": elapsed * 1e3 / steps, "higher_is_better": True,
           "scaling": "replicas only", "vs_baseline": None, "dtype": "u32",
           "data": "synthetic FlyBase-shaped KB (flybase_kb; the notebook's FlyBase dump needs a network fetch)",
           "config": {"workload": "DBInterface surface: SimplePatternMiner.ipynb halo walk + pattern counts",
                      "links": int(db.stats().n_links), "seeds": "one gene node per step",
                      "prefetch_s": round(t_pre, 3)},
           "roofline": None, "step_roofline": None, "cpu_baseline": cpu, "latency": lat,
           "walks": [{"halo": [{k: (round(v, 4) if isinstance(v, float) else v) for k, v in h.items()}
                               for h in r["halo"]],
                      "pattern": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r["pattern"].items()}}
                     for r in runs]}
    del das, db, arrays
    return out


# kernel scopes that are scratch, not algorithmic bytes (sort
# passes and count -> offset scans count against the fraction)
# (k_chunk_compact moves the filtered expansion's chunk runs out of its
# scratch: the walk already counts those outputs once)
_SCRATCH = ("k_radix", "k_scan_tiles", "k_scan_reduce", "k_scan_single", "k_bounds_u32", "k_chunk_compact")


def step_roofline(stats, ms_per_step, world, steps=1):
    """Step-level roofline: the algorithmic bytes of every kernel one step
    launches (each kernel's own inputs read once + outputs written once; sort
    passes and prefix-scan scratch excluded) over the whole step time --
    launch gaps, host work and small kernels count against it."""
    b = sum(v["bytes"] for k, v in stats.items() if k.startswith("k_") and not k.startswith(_SCRATCH)) / steps
    if ms_per_step <= 0:
        return None
    achieved = b / (ms_per_step * 1e-3) / 1e9
    peak = HBM_PEAK_GBS * world
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": peak, "unit": "GB/s",
            "frac": round(achieved / peak, 4), "algorithmic_bytes_per_step": b,
            "note": "sum of the step's per-kernel algorithmic bytes (k_* scopes of one profiled step, sort/scan "
                    "scratch excluded) / ms_per_step"}


def verify_steps(batched, single, names, dist, stage):
    """Per timed step: the answer size of each query as the step computed it
    (one das_plan_execute_many batch) against matched() one query at a time
    on the same query set; summed over ranks at N > 1.  Raises on any
    difference -- the bench's numbers are only reported for steps whose
    answers the one-by-one path confirms."""
    import numpy as np
    a = np.array(batched, dtype=np.float64)
    b = np.array(single, dtype=np.float64)
    if dist:
        a = np.array(_sync_sum(dist, a.ravel().tolist(), stage)).reshape(a.shape)
        b = np.array(_sync_sum(dist, b.ravel().tolist(), stage)).reshape(b.shape)
    bad = [(s, names[s][q], int(a[s, q]), int(b[s, q])) for s, q in zip(*np.nonzero(a != b))]
    if bad:
        raise AssertionError(f"batched step answers differ from matched() one by one (step, query, batched, "
                             f"single): {bad[:8]}")
    return {"steps": len(batched), "queries_per_step": len(names[0]) if names else 0,
            "bindings_checked": int(a.sum()), "how": "each timed step's per-query answer sizes (and so its total) "
                                                      "equal matched() one query at a time on the same query set"}


def run_query(args, workload, rank, world, dist, local_rank, backend):
    """One query workload (bio / flybase / hub): KB, warmup, K timed steps
    between barriers, max over ranks.  Returns rank 0's JSON dict."""
    import torch
    from das_amd.database.hip_db import HipDB
    from das_amd.pattern_matcher import pattern_matcher as pm
    args = argparse.Namespace(**dict(vars(args), workload=workload))
    if args.batch < 0:
        args.batch = BATCH_DEFAULT.get(workload, 1)
    t_build = time.perf_counter()
    log(f"generating {workload} KB")
    # one non-null stream shared by torch (collectives, staging buffers) and
    # the native context: exchanges are then ordered on the stream, with no
    # host synchronisation around each collective (parallel.HipLocal)
    torch.cuda.set_stream(torch.cuda.Stream(device=local_rank))
    db = HipDB(device=local_rank)
    arrays, specs, cfg, scaling = make_kb(args, rank, world, db)
    log(f"building the device index ({arrays.n_expr} expressions)")
    db.load_arrays(arrays)
    # the reference's loader ends with db.prefetch() (distributed_atom_space.py:
    # 138-168, redis_mongo_db.py:89-127): host copies of the node directory and
    # per-atom metadata, up to HipDB.PREFETCH_MAX_ATOMS (part of the load, untimed)
    db.prefetch()
    if getattr(arrays, "expr_on_device", False):
        arrays.drop_expr()          # device-generated input: free it once indexed
    del arrays
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t_build
    # one query set per step: anchored queries change their anchor every step
    n_sets = args.warmup + args.steps + 1
    # (and args.steps more, fresh anchors for the matched()-per-query timing)
    qsets = [[(name, build_expr(pm, s)) for name, s in specs(i)] for i in range(n_sets + args.steps)]
    stage_dev = torch.device("cuda", local_rank) if backend == "nccl" else "cpu"
    engine = None
    if world > 1:
        from das_amd import parallel
        # bio_shard places a gene's Member links on the gene's rank
        spec = {"Member": 0} if workload == "bio" else None
        engine = parallel.ShardedMatcher(db, dist, cpu_staging=(backend != "nccl"), partition_spec=spec)

        def run(q):
            return engine.count(q)
    else:
        def run(q):
            ans = pm.PatternMatchingAnswer()
            q.matched(db, ans)
            return ans.count()

    # Q2's launches are tagged inside the timed steps (das_prof_tag_plan:
    # Q2's own launches inside the batch, not those of the plans and chains
    # that run in its read-back waits): its And join's fraction is then the
    # in-step one, apart from QUERY_2 / QUERY_3's launches of the same kernel
    # instantiation.  The step is the same batch with or without the tag.
    tag_q2 = [False]

    def step(i, batch=None):
        """One pass over query set i -> the answer size of each query."""
        if engine is not None:
            if batch is False:
                return [run(q) for _, q in qsets[i]]
            # the step's queries share their collectives (ShardedMatcher.count_many)
            return list(engine.count_many([q for _, q in qsets[i]]))
        names = [name for name, _ in qsets[i]]
        q2 = next((k for k, name in enumerate(names) if name.startswith("Q2")), None) if tag_q2[0] else None
        if args.batch if batch is None else batch:
            # the step's queries in one das_plan_execute_many call
            # (pm.matched_many: a fused chain's GPU time overlaps the host
            # work of the next query)
            return [a.count() for _, a in pm.matched_many(db, [q for _, q in qsets[i]],
                                                           tag=None if q2 is None else (q2, "Q2"))]
        out = []
        for k, (name, q) in enumerate(qsets[i]):
            if k == q2:
                db.ctx.prof_tag("Q2")
            out.append(run(q))
            if k == q2:
                db.ctx.prof_tag(None)
        return out

    # the KB's host arrays, query objects and caches are long-lived: moved to
    # the collector's permanent generation, a full collection during the
    # timed steps walks only what a step allocates (a multi-ms pause there
    # added up to ~0.3 ms per bio step; DAS_BENCH_GC_FREEZE=0 off)
    import gc
    if os.environ.get("DAS_BENCH_GC_FREEZE") != "0":
        gc.collect()
        gc.freeze()
    log("warmup")
    # the warmup steps record every kernel scope (the "kernels" table); the
    # timed steps record events only around the dominant kernel, whose
    # roofline is then measured live without two event records per launch
    # of every other kernel (--events all: every scope in the timed steps too)
    for i in range(args.warmup):
        if i == args.warmup - 1:           # the last (warm) warmup step is the one profiled
            db.ctx.prof_reset()
            db.ctx.prof_enable(True)
        step(i)
    db.ctx.prof_enable(False)
    warm_stats = db.ctx.prof_stats()
    dominant = roofline_of(warm_stats, workload) if args.events == "dominant" else None
    per_query = {name: run(q) for name, q in qsets[args.warmup]}          # one by one: matched() per query
    if world > 1:
        # the answer's size: each rank counts the bindings it holds
        stage = torch.device("cuda", local_rank) if backend == "nccl" else "cpu"
        per_query = dict(zip(per_query, (int(x) for x in _sync_sum(dist, list(per_query.values()), stage))))
    # per-query wall time (the warm query set of the first timed step, 5 runs each)
    per_query_ms, per_query_ops = {}, {}
    from das_amd import _lib as _L
    for name, q in ([] if args.no_extras else qsets[args.warmup]):
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        c0 = _L.counters()
        t_q = time.perf_counter()
        for _ in range(5):
            run(q)
        torch.cuda.synchronize()
        per_query_ms[name] = round((time.perf_counter() - t_q) * 1e3 / 5, 4)
        c1 = _L.counters()
        # kernel scopes launched and host read-backs waited on, per query
        per_query_ops[name] = [round((c1[0] - c0[0]) / 5, 1), round((c1[1] - c0[1]) / 5, 1)]
    join_k = None

    def q2_only(i):
        # the And join of Q2 (Member x Inheritance) alone: its launch is then
        # the only one of its kernel in the measurement (QUERY_2 / QUERY_3
        # launch small ones of the same instantiations)
        return sum(run(q) for name, q in qsets[i] if name.startswith("Q2"))

    def q2_join_kernel():
        # the expansion kernel Q2's join runs as (the direct join's
        # k_dj_write<2,1> with Member as probe; with the reverse index join,
        # Inheritance rows expanding Member's P_{2,1} ranges: k_dj_write_bal<2,1>)
        db.ctx.prof_reset()
        db.ctx.prof_enable(True)
        q2_only(0)
        torch.cuda.synchronize()
        db.ctx.prof_enable(False)
        st = {k: v for k, v in db.ctx.prof_stats().items() if k.startswith("k_dj_write")}
        return max(st, key=lambda k: st[k]["ms"]) if st else None
    if workload == "bio" and world == 1 and not args.no_extras and dominant:
        join_k = q2_join_kernel()
    db.ctx.prof_reset()
    db.ctx.prof_only("|".join(k for k in ((dominant or {}).get("kernel"), join_k) if k) or None)
    tag_q2[0] = join_k is not None and args.events != "none"
    db.ctx.prof_enable(args.events != "none")
    db.ctx.prof_mark(1)                  # kernel-trace bracket of the timed steps (tools/step_split.py)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    coll0 = engine.sdb.plan_stats["collectives"] if engine else 0
    t0 = time.perf_counter()
    log("timed steps")
    step_counts = []
    for i in range(args.steps):
        step_counts.append(step(args.warmup + i))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    db.ctx.prof_mark(2)
    bindings = sum(sum(c) for c in step_counts)
    coll_per_step = (engine.sdb.plan_stats["collectives"] - coll0) / args.steps if engine else 0
    db.ctx.prof_enable(False)
    db.ctx.prof_only(None)
    tag_q2[0] = False
    stats = db.ctx.prof_stats()
    # Q2's And join inside the timed steps (one launch per step)
    and_join = roofline_of(stats, workload, join_k + "@Q2") if join_k and join_k + "@Q2" in stats else None
    if and_join:
        and_join["note"] = "Q2's And join launches inside the timed steps (das_prof_tag)"
    stats = {k: v for k, v in stats.items() if "@" not in k}
    # every timed step's answers against the same query set evaluated the
    # other way (untimed): batched steps against matched() one query at a
    # time, one-by-one steps against one das_plan_execute_many batch -- the
    # per-query answer sizes and so the step's total must be equal
    other = not args.batch
    check = verify_steps(step_counts, [step(args.warmup + i, batch=other) for i in range(args.steps)],
                         [[name for name, _ in qsets[args.warmup + i]] for i in range(args.steps)], dist, stage_dev)
    check["against"] = "pm.matched_many batches" if other else "matched() one query at a time"
    # the other submission mode, timed over query sets no earlier step used:
    # matched() per query is the reference's call pattern
    # (scripts/benchmark.py:231-239, QueryFlyBase.ipynb cells 5-9)
    other_ms = None
    if engine is None and not args.no_extras:
        for i in range(2):                         # the extra sets' shapes warm (no new anchors timed cold)
            step(args.warmup + i, batch=other)
        torch.cuda.synchronize()
        tm = time.perf_counter()
        for i in range(args.steps):
            step(n_sets + i, batch=other)
        torch.cuda.synchronize()
        other_ms = (time.perf_counter() - tm) * 1e3 / args.steps
    if args.cprofile and rank == 0:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for i in range(3):
            step(i)
        pr.disable()
        with open(args.cprofile, "w") as f:
            pstats.Stats(pr, stream=f).sort_stats("tottime").print_stats(40)
    variants = None
    if join_k is not None:
        # Q2's And join alone: the default (reverse index join: the 10^5
        # Inheritance rows expand their Member ranges of P_{2,1}), and the
        # direct join of round 3 (the 2*10^7 Member rows as probe, read from
        # the index HBM-cold, warmed by the count pass, or copied first)
        variants = {}
        for vname, env in (("default (Inheritance rows index-join Member's P_{2,1}), Q2 only", {}),
                           ("direct join, views, count pass warms the probe, Q2 only", {"DAS_REV_IJ": "0"}),
                           ("direct join, views, no warming (HBM-cold probe), Q2 only",
                            {"DAS_REV_IJ": "0", "DAS_DJ_WARM": "0"}),
                           ("direct join, large probes copied (MALL-warm), Q2 only",
                            {"DAS_REV_IJ": "0", "DAS_SCAN_VIEWS": "2"})):
            fn = q2_only if vname.endswith("Q2 only") else step
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                for i in range(2):
                    fn(i)
                vk = q2_join_kernel()               # this variant's expansion kernel
                db.ctx.prof_reset()
                db.ctx.prof_only(vk)
                db.ctx.prof_enable(True)
                torch.cuda.synchronize()
                tv = time.perf_counter()
                for i in range(5):
                    fn((args.warmup + i) % n_sets)
                torch.cuda.synchronize()
                tv = (time.perf_counter() - tv) * 1e3 / 5
                db.ctx.prof_enable(False)
                db.ctx.prof_only(None)
                variants[vname] = {"env": env, ("ms_per_query" if fn is q2_only else "ms_per_step"): round(tv, 4),
                                   "roofline": roofline_of(db.ctx.prof_stats(), workload, vk)}
            finally:
                for k, v in saved.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
    stage = stage_dev
    elapsed = _sync_max(dist, [elapsed], stage)[0]
    bindings = _sync_sum(dist, [bindings], stage)[0]
    value = bindings / elapsed
    ms_per_step = elapsed * 1e3 / args.steps
    incl = None
    if world == 1 and not args.no_materialise:
        incl = materialised_rate(pm, db, qsets[n_sets - 1], args.materialise_cap)
    out = None
    if rank == 0:
        cpu = cpu_fast = None
        if world == 1 and not args.no_cpu_baseline:
            log("cpu baseline")
            cpu = cpu_baseline(args, args.cpu_baseline_seconds)
            # the oracle's hash-join fold beside it (not the reference's complexity)
            cpu_fast = cpu_baseline(args, max(args.cpu_baseline_seconds / 3, 2.0), fast=True)
        data = {"bio": "synthetic (seeded bio_kb in scripts/benchmark.py shape; bio_atomspace dump unavailable offline)",
                "flybase": "synthetic FlyBase-shaped KB (flybase2metta Execution layout; the FlyBase dump needs a "
                           "network fetch)",
                "hub": "synthetic power-law hypergraph (powerlaw_kb, Zipf(1.1) targets)"}[workload]
        cfg = dict(cfg, bindings_per_step=per_query, parallelism=f"links sharded x{world}")
        # how a step submits its queries: one das_plan_execute_many call
        # (pm.matched_many; Q2's own launches tagged inside it), or one
        # matched() per query; N > 1: ShardedMatcher.count_many
        cfg["step_calls"] = ("ShardedMatcher.count_many" if world > 1 else
                             "pm.matched_many (das_plan_execute_many)" if args.batch else "matched() per query")
        cfg["step_check"] = check
        cfg["query_ms_rank0"] = per_query_ms
        cfg["query_launches_readbacks_rank0"] = per_query_ops
        out = {
            "metric": "pattern matches/sec (bindings/s) + % HBM roofline",
            "value": value, "unit": "bindings/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": scaling,
            "vs_baseline": None, "dtype": "u32", "data": data, "config": cfg,
            "roofline": roofline_of(stats, workload, dominant["kernel"] if dominant else None),
            "step_roofline": step_roofline(warm_stats if dominant else stats, ms_per_step, world,
                                           1 if dominant else args.steps),
            "cpu_baseline": cpu,
            "cpu_fast": cpu_fast,
            # latency-bound workloads: per query, its wall us and the kernel
            # scopes / host read-backs it takes (FlyBase: launches and waits,
            # not bytes, bound it)
            "latency": {name.split(" ")[0]: {"us": round(per_query_ms[name] * 1e3, 1),
                                             "launches": per_query_ops[name][0],
                                             "readbacks": per_query_ops[name][1]}
                        for name in per_query_ms} or None,
            "incl_materialisation": incl,
            "kernels": kernels_of(warm_stats if dominant else stats),
            "kernels_from": "last warmup step (every scope)" if dominant else "timed steps (every scope)",
            "build_s": round(t_build, 2),
            # both submission modes: the timed one's ms_per_step and the other
            # timed beside it on fresh anchors (matched() per query = the
            # reference's call pattern)
            "step_ms_matched": round(ms_per_step, 4) if not args.batch else
            (None if other_ms is None else round(other_ms, 4)),
            "step_ms_batched": round(ms_per_step, 4) if args.batch else
            (None if other_ms is None else round(other_ms, 4)),
        }
        if world > 1:
            out["sharded_plan_stats"] = dict(engine.sdb.plan_stats)
            out["collectives_per_step"] = round(coll_per_step, 2)
        if variants:
            out["join_probe_variants"] = variants
        if and_join:
            out["and_join_q2_in_step"] = and_join
    gc.unfreeze()
    del engine, qsets, db
    return out


# ---------------------------------------------------------------------------
# output: one compact JSON line last on stdout (the driver parses it from a
# bounded stdout tail), the full record in a detail file
# ---------------------------------------------------------------------------
LINE_MAX_BYTES = 4096
HEAD_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
             "vs_baseline", "dtype", "data")


def _r(x, nd=4):
    return round(x, nd) if isinstance(x, float) else x


def _compact_roofline(r, full=True):
    if not r:
        return None
    keys = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "avg_launch_us") if full else \
        ("kernel", "frac", "achieved")
    out = {k: _r(r.get(k)) for k in keys if k in r}
    if full and isinstance(out.get("traffic"), float):
        out["traffic"] = int(out["traffic"])
    return out


def _compact_cpu(c, full=True):
    if not c:
        return None
    if not full:
        return {k: (_r(c.get(k), 1) if k == "value" else c.get(k))
                for k in ("value", "join", "rows_per_get_links", "us_per_row") if k in c}
    out = {k: _r(c.get(k), 1) for k in ("value", "unit", "cores", "kind", "join") if k in c}
    out["sample"] = (c.get("sample") or "")[:240]
    return out


def _compact_leg(d):
    if "error" in d:
        return {"error": str(d["error"])[:200]}
    out = {k: _r(d.get(k)) for k in ("value", "unit", "ms_per_step") if k in d}
    if (d.get("config") or {}).get("step_calls"):
        out["step_calls"] = d["config"]["step_calls"]
    out["roofline"] = _compact_roofline(d.get("roofline"), full=False)
    sr = d.get("step_roofline")
    out["step_roofline"] = {"frac": sr.get("frac")} if sr else None
    out["cpu_baseline"] = _compact_cpu(d.get("cpu_baseline"), full=False)
    if d.get("cpu_fast"):
        out["cpu_fast"] = _compact_cpu(d.get("cpu_fast"), full=False)
    for k in ("step_ms_matched", "step_ms_batched", "cold_build_ms", "latency", "summary",
              "collectives_per_step"):   # latency legs: per-query us, launches / read-backs
        if d.get(k) is not None:
            out[k] = d[k]
    if isinstance(out.get("latency"), dict) and "rows" in out["latency"]:
        # (getlinks: the per-row figures are in cpu_baseline, beside the CPU's)
        out["latency"] = {k: v for k, v in out["latency"].items() if k not in ("rows", "level_ms_per_query")}
    return out


def compact_line(full):
    """The ONE JSON line bench.py ends its stdout with: the headline's
    contract keys, its roofline / step_roofline / cpu_baseline, and per extra
    workload only value, unit, ms_per_step, roofline {kernel, frac, achieved},
    step_roofline.frac and cpu_baseline.value (plus a latency leg's compact
    summary).  Kernel tables, join variants and materialisation detail stay in
    the detail file.  Guaranteed <= LINE_MAX_BYTES: optional parts are
    dropped, largest first, if a record ever grows past it."""
    line = {k: _r(full.get(k)) for k in HEAD_KEYS if k in full}
    cfg = full.get("config") or {}
    line["config"] = {k: cfg[k] for k in ("workload", "parallelism", "step_calls") if k in cfg}
    line["roofline"] = _compact_roofline(full.get("roofline"))
    line["step_roofline"] = _compact_roofline(full.get("step_roofline"))
    line["cpu_baseline"] = _compact_cpu(full.get("cpu_baseline"))
    if full.get("cpu_fast"):
        line["cpu_fast"] = _compact_cpu(full.get("cpu_fast"), full=False)
    for k in ("step_ms_matched", "step_ms_batched", "box", "latency", "summary", "collectives_per_step"):
        if full.get(k) is not None:
            line[k] = full[k]
    if isinstance(line.get("box"), dict):
        line["box"] = {k: v for k, v in line["box"].items() if k != "how"}
    jv = full.get("join_probe_variants") or {}
    ins = full.get("and_join_q2_in_step")
    if jv or ins:
        # Q2's And join (the north_star And-join target): its launch inside
        # the timed steps (kernel, fraction, us); beside it Q2 run alone five
        # times back to back (its P_{2,1} ranges may stay MALL-warm) and the
        # round-3 direct join HBM-cold
        d0 = next(iter(jv.values())) if jv else {}
        cold = next((v for k, v in jv.items() if "HBM-cold" in k), None)
        rf = d0.get("roofline") or {}
        src = ins or rf
        line["and_join_q2"] = {"kernel": (src.get("kernel") or "").split("@")[0] or None, "frac": src.get("frac"),
                               "us": src.get("avg_launch_us"), "in_step": ins is not None,
                               "q2_alone_frac": rf.get("frac"), "query_ms": d0.get("ms_per_query"),
                               "direct_cold_frac": ((cold or {}).get("roofline") or {}).get("frac")}
    if full.get("workloads"):
        line["workloads"] = {w: _compact_leg(d) for w, d in full["workloads"].items()}
    line["detail"] = full.get("detail_file")
    s = json.dumps(line, separators=(",", ":"))
    # never exceed the bound: shed the optional parts, then shorten the strings
    for drop in (("workloads", "summary"), ("and_join_q2",), ("workloads", "latency"), ("summary",), ("latency",),
                 ("data",)):
        if len(s.encode()) <= LINE_MAX_BYTES:
            break
        if len(drop) == 2:
            for leg in (line.get("workloads") or {}).values():
                leg.pop(drop[1], None)
        else:
            line.pop(drop[0], None)
        s = json.dumps(line, separators=(",", ":"))
    if len(s.encode()) > LINE_MAX_BYTES and line.get("cpu_baseline"):
        line["cpu_baseline"]["sample"] = line["cpu_baseline"]["sample"][:60]
        s = json.dumps(line, separators=(",", ":"))
    return s


def emit(full, detail_path):
    """Write the full record to `detail_path` (and a one-line-per-leg summary
    to stderr), then print the compact line as the LAST stdout line."""
    if detail_path:
        try:
            os.makedirs(os.path.dirname(os.path.abspath(detail_path)), exist_ok=True)
            with open(detail_path, "w") as f:
                json.dump(full, f)
            full["detail_file"] = os.path.relpath(os.path.abspath(detail_path), ROOT)
        except OSError as e:
            log(f"detail file not written: {e}")
    for name, d in [("headline", full)] + list((full.get("workloads") or {}).items()):
        r = d.get("roofline") or {}
        log(f"{name}: value {d.get('value')} {d.get('unit')} ms/step {d.get('ms_per_step')} "
            f"roofline {r.get('kernel')} {r.get('frac')}")
    sys.stdout.flush()
    print(compact_line(full), flush=True)


def _free_device():
    import gc
    import torch
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    # DAS_BENCH_SAME_DEVICE=1 + DAS_DIST_BACKEND=gloo rehearse N ranks on one GPU
    if os.environ.get("DAS_BENCH_SAME_DEVICE") == "1":
        local_rank = 0
    backend = os.environ.get("DAS_DIST_BACKEND", "nccl")
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    if args.workload == "load":
        run_load(args, rank, world, local_rank)
        if dist:
            dist.destroy_process_group()
        return
    if args.workload == "all":
        head = "bio"
        legs = args.legs.split(",") if args.legs != "auto" else (["flybase", "hub", "build", "getlinks"]
                                                                 if world == 1 else ["build"])
        legs = [w for w in legs if w]
    else:
        head, legs = args.workload, []

    def run_leg(w, a):
        if w == "build":
            return run_build(a, rank, world, dist, local_rank, backend)
        if w == "getlinks":
            return run_getlinks(a, rank, world, local_rank)
        return run_query(a, w, rank, world, dist, local_rank, backend)

    t_head = time.perf_counter()
    # the build leg runs first, in HBM no earlier leg has used: device memory
    # a leg frees is cleared by the driver before it can be mapped again, and a
    # 10^9-link build allocating ~87 GB after the hub leg's KB stalled on that
    # (2.47 s vs 0.85 s on one box, round 3)
    order = (["build"] if "build" in legs else []) + [head] + [w for w in legs if w != "build"]
    extra = {}
    line = None
    for w in order:
        if w == head:
            line = run_leg(head, args)
            _free_device()
            continue
        t_leg = time.perf_counter()
        a = argparse.Namespace(**dict(vars(args), cpu_baseline_seconds=args.leg_cpu_seconds))
        if w == "flybase":
            # a latency-bound step of ~0.25 ms: more untimed warmup steps (the
            # side streams' blocks, pinned pools, shape caches) and more timed
            # ones against scheduling noise -- milliseconds either way
            a.warmup, a.steps = max(args.warmup, 20), max(args.steps, 60)
        try:
            r = run_leg(w, a)
        except Exception as e:            # one leg failing must not lose the headline line
            log(f"workload {w} failed: {type(e).__name__}: {e}")
            r = {"error": f"{type(e).__name__}: {e}"}
        if rank == 0 and r is not None:
            r["leg_wall_s"] = round(time.perf_counter() - t_leg, 1)
            extra[w] = r
        _free_device()
    # the card's 16-byte nontemporal store ceiling (k_cartesian's pattern),
    # measured after the legs: write-bound fractions move with the card
    box = None
    try:
        from das_amd.database.hip_db import HipDB
        probe = HipDB(device=local_rank)
        gbps = probe.ctx.box_store_bw(4 << 30, 5)
        box = {"store16_nt_GBps": round(gbps, 1), "store16_nt_frac": round(gbps / HBM_PEAK_GBS, 4),
               "how": "das_box_store_bw: 4 GiB as six columns of nontemporal dwordx4 stores, 5 launches"}
        del probe
    except Exception as e:                  # the line is still written
        box = {"error": f"{type(e).__name__}: {e}"[:200]}
    if rank == 0:
        if line is not None:
            line["box"] = box
        if extra:
            line["workloads"] = extra
            line["headline_wall_s"] = round(time.perf_counter() - t_head, 1)
        emit(line, args.detail)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
