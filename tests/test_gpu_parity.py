"""GPU parity: the HIP path (through the C ABI) against the reference's golden
outputs and the CPU oracle, bit-exact (handles, binding sets)."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import das_oracle as O
from tests.util import build, canon, record, record_many, same

pytestmark = pytest.mark.gpu

DATA = os.path.join(os.path.dirname(__file__), "golden", "data")
KB_FIXTURES = ["kb_animals.json", "kb_toy_mining.json", "kb_stub_like.json"]


def _hipdb(arrays, tuple_targets=False):
    from das_amd.database.hip_db import HipDB
    db = HipDB(device=0, tuple_targets=tuple_targets)
    db.load_arrays(arrays)
    return db


# oracle answers shared by the parametrisations of one KB + query list (the
# variants differ only in the device path; the oracle reads no DAS_* switch)
_WANT = {}


def _wants(key, odb, qs):
    w = _WANT.get(key)
    if w is None:
        w = _WANT[key] = [O.evaluate(q, odb) for q in qs]
    return w


def _fixture_db(golden, name, tuple_targets=False):
    from das_amd import loader
    d = golden(name)
    return d, _hipdb(loader.from_tables(d["nodes"], d["links"]).finish(), tuple_targets)


# ----------------------------------------------------------------- hashing

def test_gpu_md5_kernel_matches_hashlib(golden):
    import torch
    from das_amd import _lib
    hv = golden("hash_vectors.json")
    strings = [s.encode("utf-8") for s, _ in hv["md5"]]
    off = np.zeros(len(strings) + 1, dtype=np.uint64)
    np.cumsum([len(s) for s in strings], out=off[1:])
    dev = torch.device("cuda:0")
    b = torch.from_numpy(np.frombuffer(b"".join(strings), dtype=np.uint8).copy()).to(dev)
    o = torch.from_numpy(off.view(np.int64).copy()).to(dev)
    out = torch.zeros((len(strings), 4), dtype=torch.int32, device=dev)
    ctx = _lib.Context(0, torch.cuda.current_stream().cuda_stream)
    _lib.check(_lib.lib().das_hash_strings_dev(ctx.h, b.data_ptr(), o.data_ptr(), len(strings), out.data_ptr()), ctx.h)
    torch.cuda.synchronize()
    got = _lib.digests_to_hex(out.cpu().numpy().view(np.uint32))
    assert got == [h for _, h in hv["md5"]]


@pytest.mark.parametrize("k", [2, 3, 4, 5])
def test_gpu_composite_kernel_matches_hashlib(k):
    import torch
    from das_amd import _lib
    rng = np.random.default_rng(k)
    n = 5000
    elems = rng.integers(0, 2**32, size=(n * k, 4), dtype=np.uint64).astype(np.uint32)
    dev = torch.device("cuda:0")
    e = torch.from_numpy(elems.view(np.int32)).to(dev)
    out = torch.zeros((n, 4), dtype=torch.int32, device=dev)
    ctx = _lib.Context(0, torch.cuda.current_stream().cuda_stream)
    _lib.check(_lib.lib().das_hash_fixed_dev(ctx.h, e.data_ptr(), k, n, out.data_ptr()), ctx.h)
    torch.cuda.synchronize()
    got = _lib.digests_to_hex(out.cpu().numpy().view(np.uint32))
    hx = _lib.digests_to_hex(elems)
    for i in range(0, n, 97):
        assert got[i] == O.composite_hash(hx[i * k:(i + 1) * k])


# ------------------------------------------------------------ index build

@pytest.mark.parametrize("degree", ["1", "0"])
@pytest.mark.parametrize("fixture", KB_FIXTURES)
def test_gpu_index_reproduces_reference_atoms(golden, fixture, degree, monkeypatch):
    monkeypatch.setenv("DAS_DEGREE_ORDER", degree)
    d, db = _fixture_db(golden, fixture)
    assert list(db.count_atoms()) == d["count_atoms"]
    dig, cat, ar, ty, nl = db._host_mirror()
    from das_amd import _lib
    hexes = _lib.digests_to_hex(dig)
    assert len(set(hexes)) == len(hexes)
    named = [int(ty[i]) if cat[i] in (1, 2) else 1 << 32 for i in range(len(hexes))]
    assert named == sorted(named)                                  # ids clustered by named type
    # inside a type: atoms referenced more often first (power-of-two bucket of
    # the link-target references, exact below 2^22 of them), then handle order;
    # DAS_DEGREE_ORDER=0: handle order only
    refs = {}
    for l in d["links"]:
        for t in l[2]:
            refs[t] = refs.get(t, 0) + 1
    bucket = lambda h: -int(np.floor(np.log2(refs.get(h, 0) + 1))) if degree == "1" else 0  # noqa: E731
    for t in set(named):
        grp = [h for h, k in zip(hexes, named) if k == t]
        assert grp == sorted(grp, key=lambda h: (bucket(h), h))
    assert db.ids_of(hexes).tolist() == list(range(len(hexes)))
    nodes = sorted([h, db.arrays.type_names[int(ty[i])], db.arrays.node_name(int(nl[i]))]
                   for i, h in enumerate(hexes) if cat[i] == 1)
    assert nodes == sorted(d["nodes"])
    links = {}
    for i, h in enumerate(hexes):
        if cat[i] == 2:
            links[h] = [db.arrays.type_names[int(ty[i])], db.get_link_targets(h)]
    assert {l[0]: [l[1], l[2]] for l in d["links"]} == links


def test_gpu_loader_files_match_reference_handles(golden):
    from das_amd import loader
    with open(os.path.join(DATA, "animals.metta")) as f:
        db = _hipdb(loader.parse_metta(f.read()).finish())
    d = golden("kb_animals.json")
    assert list(db.count_atoms()) == d["count_atoms"]
    assert sorted(db.get_all_nodes("Concept")) == sorted(n[0] for n in d["nodes"])
    assert db.get_node_handle("Concept", "human") == "af12f10f9ae2002a1607ba0b47ba8407"
    assert db.link_exists("Inheritance", ["af12f10f9ae2002a1607ba0b47ba8407", "bdfe4e7a431f73386f37c6448afe5840"])


def test_gpu_index_probes(golden):
    d, db = _fixture_db(golden, "kb_animals.json")
    for p in d["index"]:
        if p["kind"] == "links":
            r = db.get_matched_links(*p["args"])
        elif p["kind"] == "template":
            r = db.get_matched_type_template(p["args"])
        else:
            r = db.get_matched_type(p["args"])
        assert sorted(x if isinstance(x, str) else x[0] for x in r) == p["handles"], p["args"]


@pytest.mark.parametrize("tuple_targets", [False, True])
def test_gpu_answer_rows_formatting(tuple_targets, monkeypatch):
    """get_matched_links / get_matched_type_template / get_matched_type rows
    (handle, targets) against the oracle's DB path, through the per-id cache
    path, the C formatter (_assign.hex_pairs: HEX_DIRECT=0) from one device
    gather, and the C formatter from the prefetched host mirror."""
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    arrays = synthetic.bio_kb(300, 120, 3000, seed=4)
    db = HipDB(device=0, tuple_targets=tuple_targets)
    db.load_arrays(arrays)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    bp = O.terminal_hash("BiologicalProcess", "bp3")
    fmt = tuple if tuple_targets else list
    norm = lambda rows: sorted((h, fmt(tg)) for h, tg in rows)  # noqa: E731
    calls = [("get_matched_links", ("Member", ["*", "*"])), ("get_matched_links", ("Member", ["*", bp])),
             ("get_matched_type_template", (["Member", "Gene", "BiologicalProcess"],)),
             ("get_matched_type", ("Inheritance",))]
    want = [norm(getattr(odb, f)(*a)) for f, a in calls]
    assert len(want[0]) > 1000
    for mode in ("cache", "c-gather", "c-mirror"):
        monkeypatch.setattr(HipDB, "HEX_DIRECT", 1 << 30 if mode == "cache" else 0)
        if mode == "c-mirror":
            db.prefetch()
        for (f, a), w in zip(calls, want):
            got = getattr(db, f)(*a)
            assert all(isinstance(tg, fmt) for _, tg in got), (mode, f)
            assert norm(got) == w, (mode, f, a)
    # a link of a C-formatted answer resolves from the seeded handle cache
    h, tg = db.get_matched_links("Member", ["*", bp])[0]
    assert db.get_link_targets(h) == list(tg)


# ----------------------------------------------------------------- queries

@pytest.mark.parametrize("fixture", KB_FIXTURES)
def test_gpu_queries_match_reference(golden, fixture):
    """Reference DB path semantics (tuple targets): every answer bit-exact."""
    d, db = _fixture_db(golden, fixture, tuple_targets=True)
    bad = []
    for q in d["queries"]:
        got = record(q["query"], db)
        if not same(got, q):
            bad.append((q["query"], got, {k: q.get(k) for k in ("error", "matched", "negation", "n")}))
    assert not bad, bad


@pytest.mark.parametrize("fixture", KB_FIXTURES)
def test_gpu_queries_list_targets_match_oracle(golden, fixture):
    d, db = _fixture_db(golden, fixture, tuple_targets=False)
    odb = O.RedisMongoSemantics(O.KB.from_tables(d["nodes"], d["links"]), tuple_targets=False)
    for q in d["queries"]:
        want = O.evaluate(q["query"], odb)
        got = record(q["query"], db)
        assert same(got, want), (q["query"], got, want)


def _random_queries(rng, arrays, n):
    """Ordered single-link, 2/3-clause And, Not, Or over the KB's types/nodes."""
    types = [t for t in arrays.type_names if t not in ("Gene", "BiologicalProcess", "Concept", "Schema",
                                                       "Verbatim")]
    node_leaves = [i for i in range(arrays.n_leaf) if arrays.leaf_kind[i] == 1]
    qs = []
    V = lambda x: ["Var", x]  # noqa: E731

    def node():
        i = node_leaves[rng.integers(len(node_leaves))]
        s = arrays.leaf_string(i)
        t, n = s.split(" ", 1)
        return ["Node", t, n]

    def link(a, b):
        return ["Link", types[rng.integers(len(types))], True, [a, b]]
    for _ in range(n):
        k = rng.integers(9)
        if k == 6:      # Not term on variables the result binds only partly: no row is covered
            qs.append(["And", [link(V("A"), node()), link(V("A"), V("B")), ["Not", link(V("B"), V("C"))]]])
            continue
        if k == 7:      # Not term on both bound variables, reversed (anti index join, two lookups)
            qs.append(["And", [link(V("A"), V("B")), ["Not", link(V("B"), V("A"))]]])
            continue
        if k == 8:      # Not term on an unbound variable only
            qs.append(["And", [link(V("A"), V("B")), ["Not", link(V("C"), node())]]])
            continue
        if k == 0:
            qs.append(link(V("A"), node()))
        elif k == 1:
            qs.append(["And", [link(V("A"), V("B")), link(V("B"), V("C"))]])
        elif k == 2:
            qs.append(["And", [link(node(), V("B")), link(V("A"), V("B"))]])
        elif k == 3:
            qs.append(["And", [link(V("A"), V("B")), ["Not", link(V("A"), node())]]])
        elif k == 4:
            qs.append(["Or", [link(V("A"), node()), link(V("A"), node())]])
        else:
            qs.append(["And", [link(V("A"), V("B")), link(V("A"), V("C")), link(V("C"), V("D"))]])
    return qs


@pytest.mark.parametrize("sets", ["hash", "sort", "host"])
@pytest.mark.parametrize("gen", ["bio", "powerlaw"])
def test_gpu_synthetic_matches_oracle(gen, sets, monkeypatch):
    """Random Link / And / Or / Not queries; Or's dedup and Not's anti-join
    through the row hash sets and through the sort-based path (which also
    turns the semi-join off, so one-variable And terms take the direct join);
    "host": the per-operator path instead of the native plan."""
    from das_amd import synthetic
    if sets == "host":
        monkeypatch.setenv("DAS_PLAN", "0")
    if sets == "sort":
        monkeypatch.setenv("DAS_SET_SORT", "1")
        monkeypatch.setenv("DAS_SEMI_JOIN", "0")
    if gen == "bio":
        arrays = synthetic.bio_kb(300, 120, 3000, seed=7)
    else:
        arrays = synthetic.powerlaw_kb(400, 4000, link_types=2, seed=7)
        arrays.type_names  # arity-3 links exist too
    db = _hipdb(arrays)
    okb = O.KB.from_arrays(arrays)
    odb = O.RedisMongoSemantics(okb)
    assert db.count_atoms() == odb.count_atoms()
    rng = np.random.default_rng(11)
    qs = _random_queries(rng, arrays, 40)
    for q, want in zip(qs, _wants(("synthetic", gen), odb, qs)):
        got = record(q, db)
        assert same(got, want), (q, got["n"] if "n" in got else got, want.get("n"))


def test_gpu_facade_readme_examples():
    from das_amd.distributed_atom_space import DistributedAtomSpace
    from das_amd.pattern_matcher.pattern_matcher import And, Link, Node, Not, Or, PatternMatchingAnswer, Variable
    das = DistributedAtomSpace()
    das.load_knowledge_base(os.path.join(DATA, "animals.metta"))
    assert das.count_atoms() == (14, 26)
    assert das.get_node("Concept", "human") == "af12f10f9ae2002a1607ba0b47ba8407"
    inh = lambda a, b: Link("Inheritance", [a, b], True)  # noqa: E731
    out = das.query(Link("Inheritance", [Node("Concept", "human"), Variable("$2")], True))
    assert out == "{{'$2': 'bdfe4e7a431f73386f37c6448afe5840'}}"
    ans = PatternMatchingAnswer()
    assert And([inh(Variable("$1"), Variable("$2")), inh(Variable("$2"), Variable("$3"))]).matched(das.db, ans)
    assert len(ans.assignments) == 7
    ans = PatternMatchingAnswer()
    q = Or([And([inh(Variable("$1"), Variable("$2")), inh(Variable("$2"), Variable("$3")),
                 Not(inh(Variable("$1"), Node("Concept", "mammal")))]),
            inh(Node("Concept", "human"), Variable("$2"))])
    assert q.matched(das.db, ans) and len(ans.assignments) == 4
    # the service's query string (scripts/service_regression_test.sh:52-59) through _parse_query
    from das_amd.service import _parse_query
    assert das.query(_parse_query("Node n1 Concept human, Link Inheritance n1 $2")) == \
        "{{'$2': 'bdfe4e7a431f73386f37c6448afe5840'}}"
    q = _parse_query("Node m Concept mammal, Link Inheritance $1 $2, Link Inheritance $2 $3, AND, "
                     "Link Inheritance $1 m, NOT, AND")
    ans = PatternMatchingAnswer()
    assert q.matched(das.db, ans) and len(ans.assignments) == 3        # service/README.md:316-337
    assert sorted(das.get_links("Inheritance", None, ["*", "bdfe4e7a431f73386f37c6448afe5840"])) == sorted(
        das.db.get_matched_links("Inheritance", ["*", "bdfe4e7a431f73386f37c6448afe5840"]) and
        [h for h, _ in das.db.get_matched_links("Inheritance", ["*", "bdfe4e7a431f73386f37c6448afe5840"])])


def _sharded_kb(kind):
    """(AtomArrays, queries) of a two-rank sharded GPU test: the bio KB, and
    the hub / FlyBase shapes of configs 5 / 3 (Zipf KBs dense in duplicates)."""
    from das_amd import synthetic
    from tests.golden import make_synthetic as MS
    from tests.test_parallel_gloo import _fly_queries, _hub_queries, _queries
    if kind in ("default", "heavy", "small", "default_owner", "small_batch"):
        return synthetic.bio_kb(60, 25, 600, 80, seed=3), _queries()
    if kind in ("hub", "hub_small", "hub_exchange"):
        return MS.make_arrays("hub"), _hub_queries()
    if kind.startswith("bio_full"):
        # scripts/benchmark.py QUERY_1-3 (LinkTemplate leaves, template-target
        # Links, the nested Context link, the unconstrained last term's cross join)
        arrays = MS.make_arrays("bio_full")
        qs = []
        for genes in (["g3", "g5"], ["g1", "g2"]):
            qs += MS.benchmark_queries(genes)
        return arrays, qs
    return MS.make_arrays("flybase"), _fly_queries()


# mode -> environment of the two ranks: "heavy" folds operator by operator
# with the heavy-hitter split (no sharded native plan); "*small" lowers the
# gathered-term threshold so terms stay split on the shards (index joins
# through each shard's index, the fold's emptiness checks, fallbacks)
_SHARD_ENV = {"heavy": {"DAS_SHARDED_PLAN": "0", "DAS_JOIN_PLACEMENT": "exchange", "DAS_HEAVY_FRAC": "0.05"},
              "hub": {"DAS_JOIN_PLACEMENT": "exchange", "DAS_HEAVY_FRAC": "0.05"},
              "small": {"DAS_SHARD_SMALL": "40"}, "small_batch": {"DAS_SHARD_SMALL": "40"},
              "hub_small": {"DAS_SHARD_SMALL": "30"},
              # large terms over a gather budget scaled to the test KB: the
              # planner folds them with the all-to-all exchange (no forcing)
              "hub_exchange": {"DAS_SHARD_SMALL": "30", "DAS_SHARD_GATHER_BUDGET": "2000"}}


def _sharded_worker(rank, world, port, out_path, mode):
    import os as _os
    import torch
    import torch.distributed as dist
    _os.environ.update(_SHARD_ENV.get(mode, {}))
    _os.environ["MASTER_ADDR"] = "127.0.0.1"
    _os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from das_amd.database.hip_db import HipDB
    from das_amd.parallel import HipLocal, ShardedDB, shard_arrays
    from das_amd.pattern_matcher import pattern_matcher as pm
    from tests.test_gpu_devgen import _indexed_links
    arrays, queries = _sharded_kb(mode)
    # the whole KB is every rank's directory; links indexed by their handle's owner
    db = HipDB(device=0)
    db.load_arrays(shard_arrays(arrays, rank, world))
    sdb = ShardedDB(HipLocal(db, cpu_staging=True), dist)
    res = []
    if mode.endswith("_batch"):
        # every query at once: their sharded plans share one estimate
        # exchange, one gather and one outcome all-reduce (plan_many); the
        # ones that fall back are folded operator by operator
        exprs = [build(q) for q in queries]
        answers = [pm.PatternMatchingAnswer() for _ in exprs]
        c0 = sdb.plan_stats["collectives"]
        sdb._tops = {id(e) for e in exprs}
        got = sdb.plan_many(list(zip(exprs, answers)))
        sdb._tops = set()
        batch_coll = sdb.plan_stats["collectives"] - c0
        for e, a, m in zip(exprs, answers, got):
            if m is None:
                sdb._no_plan, sdb._top = {id(e)}, e
                a = pm.PatternMatchingAnswer()
                try:
                    m = e.matched(sdb, a)
                except AttributeError as err:
                    res.append({"error": type(err).__name__})
                    continue
                finally:
                    sdb._no_plan, sdb._top = set(), None
            rows = sorted(json.dumps(canon(x), sort_keys=True) for x in a.assignments)
            res.append({"matched": bool(m), "negation": a.negation, "n": a.count(), "rows": rows,
                        "local": sdb.rel_local_count(a._relation()), "native": 1, "collectives": 0})
        sdb.plan_stats["batch_collectives"] = batch_coll
        sdb.plan_stats["batch_fallbacks"] = sum(1 for m in got if m is None)
        queries = []
    for q in queries:
        ans = pm.PatternMatchingAnswer()
        st0 = dict(sdb.plan_stats)
        e = build(q)
        if mode.endswith("_owner"):
            sdb._top = e                      # as ShardedMatcher.count: gathered plans evaluated by one owner
        try:
            m = e.matched(sdb, ans)
        except AttributeError as e:
            res.append({"error": type(e).__name__})
            continue
        sdb._top = None
        st1 = dict(sdb.plan_stats)
        n = ans.count()
        rows = sorted(json.dumps(canon(a), sort_keys=True) for a in ans.assignments)
        res.append({"matched": bool(m), "negation": ans.negation, "n": n, "rows": rows,
                    "local": sdb.rel_local_count(ans._relation()),
                    "native": st1["native"] - st0["native"], "collectives": st1["collectives"] - st0["collectives"]})
    res.append(sorted(_indexed_links(db)))
    res.append(sdb.plan_stats)
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["default", "heavy", "small", "hub", "hub_small", "hub_exchange", "flybase",
                                  "flybase_owner", "default_owner", "bio_full", "bio_full_owner",
                                  "flybase_batch", "bio_full_batch", "small_batch"])
def test_gpu_sharded_two_ranks_one_gpu(mode):
    """The multi-GPU path with two ranks sharing cuda:0 over gloo, against the
    single-process oracle: handle-sharded builds (each link indexed on exactly
    one rank), sharded native plans (gathered terms + one split term read
    through each shard's index, das_plan_execute_sharded) and the
    operator-by-operator fold with exchanges and the heavy-hitter split;
    bio, the hub 4-clause And (config 5) and the FlyBase And / Not / Or
    shapes (config 3).  FlyBase queries take <= 3 collectives each."""
    import socket
    import tempfile
    import torch.multiprocessing as mp
    from das_amd.parallel import handle_owner
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    # three ranks where the exchange must pay: at two, broadcasting the
    # smaller side of a join never moves more rows than the exchange
    world = 3 if mode == "hub_exchange" else 2
    arrays, queries = _sharded_kb(mode)
    okb = O.KB.from_arrays(arrays)
    odb = O.RedisMongoSemantics(okb)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res")
        mp.spawn(_sharded_worker, args=(world, port, out, mode), nprocs=world, join=True)
        per_rank = [json.load(open(f"{out}.{r}")) for r in range(world)]
    stats = per_rank[0][-1]
    if mode == "heavy":
        assert stats["heavy"] > 0 and stats["native"] == 0, stats
    elif mode == "hub_exchange":
        # the default planner took the exchange for the two large terms
        assert stats["exchange"] > 0 and stats.get("split_fold", 0) > 0, stats
    else:
        assert stats["native"] > 0, stats
    if mode in ("small", "hub_small"):
        # some queries keep terms split across the shards and still verify
        assert any(r.get("native") and r.get("collectives") == 3 for r in per_rank[0][:-2]), per_rank[0][:-2]
    indexed = [set(per_rank[r][-2]) for r in range(world)]
    assert sum(len(x) for x in indexed) == len(set().union(*indexed))           # disjoint
    assert set().union(*indexed) == set(okb.links)
    assert all(handle_owner(h, world) == r for r in range(world) for h in indexed[r])
    for qi, q in enumerate(queries):
        want = O.evaluate(q, odb)
        if "error" in want:
            assert all(per_rank[r][qi] == {"error": want["error"]} for r in range(world)), q
            continue
        want_rows = sorted(json.dumps(r, sort_keys=True) for r in want["rows"])
        assert sum(per_rank[r][qi]["local"] for r in range(world)) == want["n"], q
        for r in range(world):
            got = per_rank[r][qi]
            assert (got["matched"], got["negation"], got["n"]) == (want["matched"], want["negation"], want["n"]), q
            assert got["rows"] == want_rows, q
        if mode.startswith("flybase") and not mode.endswith("_batch"):
            got = per_rank[0][qi]
            assert got["native"] == 1 and got["collectives"] <= 3, (q, got["native"], got["collectives"])
    if mode.endswith("_batch"):
        # the whole query list's sharded plans: at most 3 collectives together
        assert stats["batch_collectives"] <= 3, stats
        if mode.startswith("flybase"):
            assert stats["batch_fallbacks"] == 0, stats
    if mode in ("flybase", "flybase_owner"):
        # the second gene's queries reuse the first's leaf sizes (shape cache):
        # no estimate exchange, 2 collectives each
        assert stats["size_cache"] > 0, stats
        assert any(per_rank[0][qi]["collectives"] == 2 for qi in range(len(queries))), per_rank[0][:-2]
    if mode.endswith("_owner"):
        # wholly gathered top-level plans were evaluated by one rank each, in turn
        owners = [[r for r in range(world) if per_rank[r][qi].get("local")] for qi in range(len(queries))]
        assert any(o == [1] for o in owners) and any(o == [0] for o in owners), owners


def _surface_gpu_worker(rank, world, port, out_path):
    import os as _os
    import torch
    import torch.distributed as dist
    _os.environ["MASTER_ADDR"] = "127.0.0.1"
    _os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    from das_amd.distributed_atom_space import DistributedAtomSpace
    from das_amd.parallel import HipLocal, ShardedDB, shard_arrays
    from tests.test_parallel_gloo import _call, _canon_pairs, _surface_calls
    arrays = synthetic.bio_kb(60, 25, 600, 80, seed=3)
    db = HipDB(device=0)
    db.load_arrays(shard_arrays(arrays, rank, world))
    sdb = ShardedDB(HipLocal(db, cpu_staging=True), dist)
    kb = O.KB.from_arrays(arrays)
    res = [_canon_pairs(_call(sdb, c)) for c in _surface_calls(kb)]
    # the facade's get_links over the sharded DB (distributed_atom_space.py:259-284)
    das = DistributedAtomSpace.__new__(DistributedAtomSpace)
    das.db = sdb
    res.append(sorted(das.get_links("Member", None, ["*", "*"])))
    res.append(sorted(das.get_links("Inheritance", ["BiologicalProcess", "BiologicalProcess"])))
    res.append(sorted(das.get_links("Inheritance")))
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


def test_gpu_sharded_dbinterface_surface():
    """ShardedDB's get_matched_links / get_matched_type_template /
    get_matched_type and the facade's get_links with two ranks sharing
    cuda:0, each rank indexing only the links its handles own: every rank
    returns the single-process DB-path answer (oracle) -- the reference's
    DBInterface over a sharded Redis Cluster (redis_mongo_db.py:235-279)."""
    import socket
    import tempfile
    import torch.multiprocessing as mp
    from das_amd import synthetic
    from tests.test_parallel_gloo import _call, _canon_pairs, _surface_calls
    arrays = synthetic.bio_kb(60, 25, 600, 80, seed=3)
    kb = O.KB.from_arrays(arrays)
    odb = O.RedisMongoSemantics(kb)
    want = [_canon_pairs(_call(odb, c)) for c in _surface_calls(kb)]
    want += [sorted(h for h, _ in odb.get_matched_links("Member", ["*", "*"])),
             sorted(h for h, _ in odb.get_matched_type_template(["Inheritance", "BiologicalProcess",
                                                                 "BiologicalProcess"])),
             sorted(h for h, _ in odb.get_matched_type("Inheritance"))]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res")
        mp.spawn(_surface_gpu_worker, args=(2, port, out), nprocs=2, join=True)
        per_rank = [json.load(open(f"{out}.{r}")) for r in range(2)]
    for r in range(2):
        for i, (g, w) in enumerate(zip(per_rank[r], want)):
            assert g == w, (r, i, len(g), len(w))


def _composite_queries(rng, arrays, n):
    """Similarity / Set (unordered) terms mixed with Inheritance: every
    Assignment.join / check_negation kind pair of pattern_matcher.py:105-362."""
    node_leaves = [i for i in range(arrays.n_leaf) if arrays.leaf_kind[i] == 1]
    V = lambda x: ["Var", x]  # noqa: E731

    def node():
        t, nm = arrays.leaf_string(node_leaves[rng.integers(len(node_leaves))]).split(" ", 1)
        return ["Node", t, nm]

    inh = lambda a, b: ["Link", "Inheritance", True, [a, b]]  # noqa: E731
    sim = lambda a, b: ["Link", "Similarity", False, [a, b]]  # noqa: E731
    st = lambda a, b, c: ["Link", "Set", False, [a, b, c]]  # noqa: E731
    shapes = [
        lambda: sim(V("A"), V("B")),
        lambda: sim(node(), V("A")),
        lambda: ["And", [sim(V("A"), V("B")), inh(V("A"), V("C"))]],
        lambda: ["And", [inh(V("A"), V("B")), sim(V("A"), V("B"))]],
        lambda: ["And", [inh(V("A"), V("B")), inh(V("B"), V("C")), sim(V("A"), V("C"))]],
        lambda: ["And", [sim(V("A"), V("B")), sim(V("B"), V("C"))]],
        lambda: ["And", [sim(V("A"), V("B")), sim(V("A"), V("B"))]],
        lambda: ["And", [sim(V("A"), V("B")), sim(V("B"), V("C")), inh(V("A"), V("C"))]],
        lambda: ["And", [st(V("A"), V("B"), V("C")), sim(V("A"), V("B"))]],
        lambda: ["And", [st(V("A"), V("B"), V("C")), inh(V("A"), V("B"))]],
        lambda: ["And", [sim(V("A"), V("B")), ["Not", inh(V("A"), V("B"))]]],
        lambda: ["And", [inh(V("A"), V("B")), ["Not", sim(V("A"), V("B"))]]],
        lambda: ["And", [sim(V("A"), V("B")), ["Not", sim(V("A"), node())]]],
        lambda: ["And", [sim(V("A"), V("B")), inh(V("B"), V("C")), ["Not", inh(V("A"), node())]]],
        lambda: ["And", [st(V("A"), V("B"), V("C")), ["Not", sim(V("A"), V("B"))]]],
        lambda: ["Or", [inh(V("A"), node()), sim(V("A"), V("B"))]],
        lambda: ["Or", [["And", [sim(V("A"), V("B")), sim(V("A"), V("B"))]], sim(V("A"), V("B"))]],
        lambda: ["Or", [["And", [sim(V("A"), V("B")), inh(V("A"), V("B"))]], ["Not", inh(V("A"), node())]]],
        lambda: ["And", [["Or", [inh(V("A"), node()), sim(V("A"), V("B"))]], inh(V("A"), V("B"))]],
        lambda: ["And", [sim(V("A"), V("B")), ["Template", "Similarity", False,
                                                [["TVar", "A", "Concept"], ["TVar", "C", "Concept"]]]]],
    ]
    qs = [s() for s in shapes]
    qs += [shapes[rng.integers(len(shapes))]() for _ in range(n)]
    return qs


@pytest.mark.parametrize("tuple_targets", [False, True])
def test_gpu_composite_algebra_matches_oracle(tuple_targets):
    """Unordered / Composite assignments (pattern_matcher.py:158-368) on the
    GPU against the oracle, on a mixed ordered/unordered KB."""
    from das_amd import synthetic
    arrays = synthetic.similarity_kb(n_nodes=40, n_inh=300, n_sim=150, n_set=60, seed=5)
    db = _hipdb(arrays, tuple_targets=tuple_targets)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays), tuple_targets=tuple_targets)
    rng = np.random.default_rng(23)
    for q in _composite_queries(rng, arrays, 20):
        want = O.evaluate(q, odb)
        got = record(q, db)
        assert same(got, want), (q, got, {k: want.get(k) for k in ("error", "matched", "negation", "n")})


@pytest.mark.parametrize("force", ["0", "1", "", "sparse", "dense"])
def test_gpu_hub_join_expansion(force, monkeypatch):
    """A hub key whose probe unit owns > 64K outputs (config 5 skew): the
    output-balanced expansion, the per-unit expansion (forced) and the
    automatic choice all equal the oracle; "sparse" / "dense" force the
    direct join's build side through the in-place (lo, cnt) descriptors
    (k_lc_count / k_lc_base / k_lc_scatter) or the histogram + scan."""
    from das_amd import synthetic
    monkeypatch.delenv("DAS_DJ_BALANCED", raising=False)
    monkeypatch.delenv("DAS_DJ_BUILD", raising=False)
    if force in ("sparse", "dense"):
        monkeypatch.setenv("DAS_DJ_BUILD", force)
    elif force:
        monkeypatch.setenv("DAS_DJ_BALANCED", force)
    n = 1200
    rng = np.random.default_rng(4)
    hub = 0
    src = np.concatenate([np.arange(1, 301), rng.integers(1, n, 500)])           # 300 rows -> hub
    dst = np.concatenate([np.full(300, hub), rng.integers(1, n, 500)])
    src2 = np.concatenate([np.full(300, hub), rng.integers(1, n, 400)])          # hub -> 300 rows
    dst2 = np.concatenate([np.arange(301, 601), rng.integers(1, n, 400)])
    arrays, _ = synthetic.build_arrays(["T"], [("Concept", "n", n)],
                                       [("T", np.stack([src, dst], 1)), ("T", np.stack([src2, dst2], 1))])
    db = _hipdb(arrays)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    V = lambda x: ["Var", x]  # noqa: E731
    t = lambda a, b: ["Link", "T", True, [a, b]]  # noqa: E731
    for q in [["And", [t(V("A"), V("B")), t(V("B"), V("C"))]],
              ["And", [t(V("A"), ["Node", "Concept", "n0"]), t(V("X"), V("A")), t(["Node", "Concept", "n0"], V("Y"))]]]:
        want = O.evaluate(q, odb)
        got = record(q, db)
        assert same(got, want), (q, got.get("n"), want.get("n"))


def _assert_same_rows(got, want, what=""):
    """got == want for long row lists, reported by counts and the first
    difference (pytest's own diff of 10^7-row lists runs for minutes)."""
    if got == want:
        return
    i = next((k for k, (a, b) in enumerate(zip(got, want)) if a != b), min(len(got), len(want)))
    raise AssertionError(f"{what}: {len(got)} rows, want {len(want)}; first difference at {i}: "
                         f"{got[i] if i < len(got) else None} vs {want[i] if i < len(want) else None}")


def _np_join_rows(pa, pk, qk, qb):
    """The natural join of P(a, k) and Q(k, b) with multiplicities, as (a, k, b)
    uint64 columns (any order) -- numpy, for joins of 10^7+ rows."""
    pk, qk = np.asarray(pk, dtype=np.int64), np.asarray(qk, dtype=np.int64)
    order = np.argsort(qk, kind="stable")
    qk_s, qb_s = qk[order], np.asarray(qb, dtype=np.uint64)[order]
    nk = int(max(pk.max(initial=0), qk.max(initial=0))) + 1
    cnt = np.bincount(qk_s, minlength=nk)
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    c = cnt[pk]
    a = np.repeat(np.asarray(pa, dtype=np.uint64), c)
    k = np.repeat(pk.astype(np.uint64), c)
    first = np.repeat(start[pk], c)
    within = np.arange(int(c.sum()), dtype=np.int64) - np.repeat(np.cumsum(c) - c, c)
    b = qb_s[first + within]
    return a, k, b


def _packed_rows(cols, widths):
    """Rows of uint64 columns as one sorted uint64 array (fields side by side
    at the given bit widths, 64 in all at most): a multiset compared by one
    np.sort instead of a lexsort of every column."""
    key = np.zeros(len(cols[0]), dtype=np.uint64)
    for c, w in zip(cols, widths):
        c = np.asarray(c, dtype=np.uint64)
        assert c.size == 0 or int(c.max()) < (1 << w)
        key = (key << np.uint64(w)) | c
    key.sort()
    return key


def _assert_same_join(got, want):
    """got: (3, n) device join output columns (a, k, b); want: _np_join_rows --
    the same rows with the same multiplicities."""
    assert len(got[0]) == len(want[0]), (len(got[0]), len(want[0]))
    widths = [max(1, int(max(int(np.max(x, initial=0)), int(np.max(y, initial=0)))).bit_length())
              for x, y in zip(got, want)]
    if sum(widths) > 64:                                  # (not in these tests: every field fits)
        g = [np.asarray(x, dtype=np.uint64) for x in got]
        og, ow = np.lexsort((g[2], g[1], g[0])), np.lexsort((want[2], want[1], want[0]))
        for x, y in zip(g, want):
            assert np.array_equal(x[og], np.asarray(y)[ow])
        return
    bad = np.flatnonzero(_packed_rows(got, widths) != _packed_rows(want, widths))
    assert bad.size == 0, f"first difference at sorted row {bad[0]}"


@pytest.mark.parametrize("search", ["0", "1", "0-vec1", "0-vec0"])
@pytest.mark.parametrize("shape", ["sparse", "fanout2", "skew", "wide"])
def test_gpu_direct_join_owner_lanes(shape, search, monkeypatch):
    """das_join of two-column tables on one key through the direct-address
    join, whose expansions find each output's owner lane per round of 64
    outputs (owner_of_round: ballot fast path / LDS row + DPP max; search=1:
    the ds_bpermute binary search): lanes without outputs, fan-out ~2, skewed
    keys (the output-balanced expansion) and a wide fan-out, against a numpy
    join with multiplicities.  The 16-byte paths of 256-output blocks: both
    (default), the single-row run path only (vec1), none (vec0)."""
    monkeypatch.setenv("DAS_OWNER_SEARCH", search[0])
    monkeypatch.setenv("DAS_DJ_VEC", search[-1] if "vec" in search else "")
    from das_amd import _lib, synthetic
    db = _hipdb(synthetic.powerlaw_kb(100, 500, link_types=2, seed=3))
    rng = np.random.default_rng({"sparse": 1, "fanout2": 2, "skew": 3, "wide": 4}[shape])
    nk = 5000
    if shape == "sparse":
        pk, qk = rng.integers(0, nk, 60000), rng.integers(0, nk, 300)
    elif shape == "fanout2":
        pk, qk = rng.integers(0, nk, 60000), rng.integers(0, nk, 2 * nk)
    elif shape == "skew":
        pk = np.where(rng.random(60000) < 0.3, 7, rng.integers(0, nk, 60000))
        qk = np.concatenate([np.full(3000, 7), rng.integers(0, nk, 3000)])
    else:
        pk, qk = rng.integers(0, 50, 3000), rng.integers(0, 50, 4000)
    pa = rng.integers(0, 1 << 20, len(pk)).astype(np.uint32)
    qb = rng.integers(0, 1 << 20, len(qk)).astype(np.uint32)
    P = db.ctx.table_from_host(_lib.TABLE_ORDERED, [0, 1], np.stack([pa, pk.astype(np.uint32)]))
    Q = db.ctx.table_from_host(_lib.TABLE_ORDERED, [1, 2], np.stack([qk.astype(np.uint32), qb]))
    P.set_bounds([0, 0], [(1 << 20) - 1, nk])
    Q.set_bounds([0, 0], [nk, (1 << 20) - 1])
    got = db.ctx.join(P, Q).fetch()
    want = _np_join_rows(pa, pk, qk, qb)
    assert len(want[0]) > 1000
    _assert_same_join(got, want)


@pytest.mark.parametrize("count_pub", ["1", "0"])
@pytest.mark.parametrize("zlc", ["1", "0"])
def test_gpu_sparse_build_slots_cleared_between_joins(zlc, count_pub, monkeypatch):
    """The sparse direct-join build writes its (lo, cnt) slots into the
    context's descriptor array and clears them after the expansion (DAS_ZLC=1,
    default; 0: a fresh array per join): five joins in a row on one context,
    over overlapping and growing key ranges (build keys in sorted order or
    not), each against a numpy join with multiplicities.  With the reused array, a
    join that unwinds between writing its slots and clearing them
    (DAS_TEST_ZLC_THROW) must not leave them for the next join (advisor r4).
    count_pub: the expansion's per-unit counts and their offsets scan in one
    launch (k_dj_count_pub, the last block scans and publishes; default) or
    two (DAS_COUNT_PUB=0)."""
    monkeypatch.setenv("DAS_DJ_BUILD", "sparse")
    monkeypatch.setenv("DAS_ZLC", zlc)
    monkeypatch.setenv("DAS_COUNT_PUB", count_pub)
    from das_amd import _lib, synthetic
    db = _hipdb(synthetic.powerlaw_kb(100, 500, link_types=2, seed=3))
    rng = np.random.default_rng(11)
    for nk, nq, srt in ((20000, 300, False), (20000, 500, True), (90000, 800, False), (5000, 200, False),
                        (90000, 1000, True), (90000, 20000, False)):
        pk = rng.integers(0, nk, 30000)
        qk = rng.integers(0, nk, nq)
        if srt:
            qk = np.sort(qk)
        pa = rng.integers(0, 1 << 20, len(pk)).astype(np.uint32)
        qb = rng.integers(0, 1 << 20, len(qk)).astype(np.uint32)
        P = db.ctx.table_from_host(_lib.TABLE_ORDERED, [0, 1], np.stack([pa, pk.astype(np.uint32)]))
        Q = db.ctx.table_from_host(_lib.TABLE_ORDERED, [1, 2], np.stack([qk.astype(np.uint32), qb]))
        P.set_bounds([0, 0], [(1 << 20) - 1, nk])
        Q.set_bounds([0, 0], [nk, (1 << 20) - 1])
        if zlc == "1" and nk == 90000 and not srt:
            monkeypatch.setenv("DAS_TEST_ZLC_THROW", "1")
            with pytest.raises(Exception, match="DAS_TEST_ZLC_THROW"):
                db.ctx.join(P, Q)
            monkeypatch.delenv("DAS_TEST_ZLC_THROW")
        got = db.ctx.join(P, Q).fetch()
        by = {}
        for k, b in zip(qk.tolist(), qb.tolist()):
            by.setdefault(k, []).append(b)
        want = sorted((a, k, b) for a, k in zip(pa.tolist(), pk.tolist()) for b in by.get(k, ()))
        _assert_same_rows(sorted(zip(*[c.tolist() for c in got])), want, (nk, nq, srt))


@pytest.mark.parametrize("guard", ["1", "0"])
@pytest.mark.parametrize("build", ["", "sparse", "dense"])
@pytest.mark.parametrize("probe_rows", [5000, 40000])
def test_gpu_key_join_duplicate_build_keys(probe_rows, build, guard, monkeypatch):
    """das_join of a two-column probe with a one-column build side: distinct
    build keys take the key-set filter (semi_join, the duplicate-key guard
    riding on the compaction's count read-back -- DAS_SMALL_GUARD=1, the
    one-launch compaction below kSmallScan = 16384 rows -- or read first, 0);
    repeated build keys void the filter and the direct join counts each
    repeat (dense or sparse build side).  Against a numpy join with
    multiplicities."""
    monkeypatch.setenv("DAS_SMALL_GUARD", guard)
    if build:
        monkeypatch.setenv("DAS_DJ_BUILD", build)
    else:
        monkeypatch.delenv("DAS_DJ_BUILD", raising=False)
    from das_amd import _lib
    from das_amd.database.hip_db import HipDB
    from das_amd import synthetic
    db = _hipdb(synthetic.powerlaw_kb(100, 500, link_types=2, seed=3))
    rng = np.random.default_rng(probe_rows)
    key_lo = 1 << 20 if build == "sparse" else 100
    pa = rng.integers(0, 1000, probe_rows).astype(np.uint32)
    pb = (key_lo + rng.integers(0, 70000 if build == "sparse" else 3000, probe_rows)).astype(np.uint32)
    P = db.ctx.table_from_host(_lib.TABLE_ORDERED, [0, 1], np.stack([pa, pb]))
    P.set_bounds([0, key_lo], [999, key_lo + 70000])
    for dup in (False, True):
        q = np.unique(pb[rng.integers(0, probe_rows, 300)])
        if dup:
            q = np.concatenate([q, q[::3]])                    # every third key twice
        Q = db.ctx.table_from_host(_lib.TABLE_ORDERED, [1], q[None, :].astype(np.uint32))
        Q.set_bounds([int(q.min())], [int(q.max())])
        got = db.ctx.join(P, Q).fetch()
        mult = dict(zip(*np.unique(q, return_counts=True)))
        want = sorted((int(a), int(b)) for a, b in zip(pa, pb) for _ in range(mult.get(b, 0)))
        assert sorted(zip(got[0].tolist(), got[1].tolist())) == want, (dup, len(want), got.shape)


@pytest.mark.parametrize("fixture", KB_FIXTURES)
def test_gpu_incoming_sets(golden, fixture):
    """incomming_set:<target> (canonical_parser.py:141-143): the links whose
    targets contain each atom, from the device incoming CSR."""
    d, db = _fixture_db(golden, fixture)
    want = {}
    for h, t, targets, _ in d["links"]:
        for x in targets:
            want.setdefault(x, set()).add(h)
    atoms = [n[0] for n in d["nodes"]] + [l[0] for l in d["links"]]
    for h in atoms:
        got = db.get_incoming_links(h)
        assert len(got) == len(set(got))
        assert set(got) == want.get(h, set()), h


def test_gpu_incoming_sets_synthetic():
    from das_amd import synthetic
    arrays = synthetic.powerlaw_kb(300, 3000, link_types=3, seed=2)
    db = _hipdb(arrays)
    kb = O.KB.from_arrays(arrays)
    want = {}
    for h, (t, targets, *_rest) in kb.links.items():
        for x in targets:
            want.setdefault(x, set()).add(h)
    for h in list(kb.nodes)[:300] + list(kb.links)[:200]:
        assert set(db.get_incoming_links(h)) == want.get(h, set()), h


@pytest.mark.parametrize("sets", ["hash", "sort"])
def test_gpu_flybase_queries_match_oracle(sets, monkeypatch):
    """Config 3: the QueryFlyBase.ipynb And / And+Not / Or shapes (bench.py
    --workload flybase) on a small FlyBase-shaped KB, every gene anchor;
    set operations through hash sets and through sorting."""
    import bench
    if sets == "sort":
        monkeypatch.setenv("DAS_SET_SORT", "1")
    from das_amd import synthetic
    arrays = synthetic.flybase_kb(200, 6, 400, n_loc=20, n_do=15, seed=3)
    db = _hipdb(arrays)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    for gene in (0, 7, 50, 199):
        for name, q in bench.flybase_specs(gene, synthetic.flybase_do_terms(arrays, gene)):
            want = O.evaluate(q, odb)
            got = record(q, db)
            assert same(got, want), (name, gene, got.get("n"), want.get("n"))


@pytest.mark.parametrize("semi", ["1", "0"])
def test_gpu_hub_four_clause_matches_oracle(semi, monkeypatch):
    """Config 5: the 4-clause hub And of bench.py --workload hub; the
    one-variable hub clauses through the key-bitmap semi-join (1) and the
    direct join (0)."""
    import bench
    from das_amd import synthetic
    monkeypatch.setenv("DAS_SEMI_JOIN", semi)
    arrays = synthetic.powerlaw_kb(200, 4000, link_types=4, seed=5)
    db = _hipdb(arrays)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    n = lambda i: ["Node", "Concept", f"n{i}"]  # noqa: E731
    V = bench._V
    # plus the unanchored 4-clause chain (hub out-degree expansion in the last clause)
    chain = ("T0(V1,h0) T0(V1,V2) T0(V2,h1) T0(V2,V3)",
             ["And", [bench._L("T0", V("V1"), n(0)), bench._L("T0", V("V1"), V("V2")),
                      bench._L("T0", V("V2"), n(1)), bench._L("T0", V("V2"), V("V3"))]])
    for name, q in bench.hub_specs() + [chain]:
        want = O.evaluate(q, odb)
        got = record(q, db)
        assert want.get("n", 0) > 0, name
        assert same(got, want), (name, got.get("n"), want.get("n"))


@pytest.mark.parametrize("multi", ["1", "1-twopass", "1-local", "1-unstaged", "1-atomic", "1-capped", "0"])
def test_gpu_semi_join_multi_matches_oracle(multi, monkeypatch):
    """Runs of one-variable hub clauses on one variable (T2(V2,a), T3(V2,b),
    ...) folded by ONE filter with the intersection of their key sets
    (semi_join_multi, forced below its size floor with DAS_SEMI_MULTI=1)
    against the term-by-term fold (0).  Random anchors make some
    intersections empty: then the plan executor folds term by term, which
    keeps And's reset-on-empty rule (pattern_matcher.py:725-729) -- a
    running result emptied by T2 is replaced by T3's rows."""
    import bench
    from das_amd import synthetic
    monkeypatch.setenv("DAS_SEMI_MULTI", multi[0])
    # the filtered expansion in one pass with LDS flag tiles (unsorted) ...
    monkeypatch.setenv("DAS_FILT_FUSED", "0" if multi in ("1-twopass", "1-local", "1-unstaged", "1-atomic") else "1")
    # ... as one walk writing chunk-locally + a compaction -- the kept rows
    # staged in LDS (k_dj_filt_staged, default), or stored lane by lane
    # (k_dj_filt<2>, DAS_FILT_STAGED=0), or placed by one atomic per chunk
    # (=atomic, no compaction) -- or as a flag pass and a second walk
    monkeypatch.setenv("DAS_FILT_LOCAL", "0" if multi == "1-twopass" else "1")
    monkeypatch.setenv("DAS_FILT_STAGED", {"1-unstaged": "0", "1-atomic": "atomic"}.get(multi, "1"))
    # ... and the one walk's scratch over its budget: the two passes instead
    if multi == "1-capped":
        monkeypatch.setenv("DAS_FILT_SCRATCH_MAX", "0")
    else:
        monkeypatch.delenv("DAS_FILT_SCRATCH_MAX", raising=False)
    arrays = synthetic.powerlaw_kb(200, 4000, link_types=4, seed=5)
    db = _hipdb(arrays)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    n = lambda i: ["Node", "Concept", f"n{i}"]  # noqa: E731
    V, L = bench._V, bench._L
    rng = np.random.default_rng(33)
    specs = [q for _, q in bench.hub_specs()]
    specs.append(["And", [L("T0", V("V1"), n(0)), L("T1", V("V1"), V("V2")), L("T2", V("V2"), n(1)),
                          L("T3", V("V2"), n(0)), L("T0", V("V2"), n(2))]])
    # one filter term after the index-joined term, then a term on the filtered variable
    specs.append(["And", [L("T0", V("V1"), n(0)), L("T0", V("V1"), V("V2")), L("T0", V("V2"), n(1)),
                          L("T0", V("V2"), V("V3"))]])
    # a filter term whose key set misses every joined row: term-by-term fold (reset-on-empty)
    specs.append(["And", [L("T0", V("V1"), n(0)), L("T1", V("V1"), V("V2")), L("T2", V("V2"), n(132)),
                          L("T3", V("V2"), n(0))]])
    for _ in range(24):
        a, b, c = (int(x) for x in rng.integers(0, 200, 3))
        t = [f"T{int(x)}" for x in rng.integers(0, 4, 4)]
        run = [L(t[1], V("V2"), n(a)), L(t[2], V("V2"), n(b))]
        if rng.random() < 0.4:
            run.append(L(t[3], n(c), V("V2")))
        specs.append(["And", [L(t[0], V("V1"), n(int(rng.integers(0, 4)))), L("T1", V("V1"), V("V2"))] + run])
    nonempty = 0
    for q in specs:
        want = O.evaluate(q, odb)
        got = record(q, db)
        assert same(got, want), (q, got.get("n"), want.get("n"))
        nonempty += want.get("n", 0) > 0
    assert nonempty >= 4


@pytest.mark.parametrize("fused", ["1", "0"])
def test_gpu_chain_large_index_join_stage(fused, monkeypatch):
    """Fused single-launch And (k_chain) whose index-join stages probe more
    rows than one LDS prefix (kIjSmall = 2048): the chain ends after the
    last stage it completed and the host continues the And operator by
    operator (the partial-chain path); against the oracle and the
    per-operator path (DAS_FUSED=0)."""
    from das_amd import loader
    monkeypatch.setenv("DAS_FUSED", fused)
    rng = np.random.default_rng(12)
    b = loader.AtomBuilder()
    hub = b.terminal("Concept", "hub", True)
    xs = [b.terminal("Concept", f"x{i}", True) for i in range(2100)]
    ys = [b.terminal("Concept", f"y{i}", True) for i in range(300)]
    for x in xs:
        b.expr("Rel", [hub, x])
        for y in rng.choice(len(ys), int(rng.integers(1, 3)), replace=False):
            b.expr("Rel2", [x, ys[int(y)]])
    for y in ys[:150]:
        b.expr("Rel3", [y, xs[int(rng.integers(0, 2100))]])
    arrays = b.finish()
    db = _hipdb(arrays)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    V = lambda x: ["Var", x]  # noqa: E731
    h = ["Node", "Concept", "hub"]
    for q in (["And", [["Link", "Rel", True, [h, V("A")]], ["Link", "Rel2", True, [V("A"), V("B")]]]],
              ["And", [["Link", "Rel", True, [h, V("A")]], ["Link", "Rel2", True, [V("A"), V("B")]],
                       ["Link", "Rel3", True, [V("B"), V("C")]]]],
              ["And", [["Link", "Rel", True, [h, V("A")]], ["Link", "Rel2", True, [V("A"), V("B")]],
                       ["Not", ["Link", "Rel3", True, [V("B"), V("A")]]]]]):
        key = json.dumps(q)
        if key not in _CHAIN_WANT:                        # the oracle's nested loop: once per query
            _CHAIN_WANT[key] = O.evaluate(q, odb)
        want = _CHAIN_WANT[key]
        got = record(q, db)
        assert want.get("n", 0) > 1000                 # (stage inputs: 2100 and ~3150 rows)
        assert same(got, want), (q, got.get("n"), want.get("n"))


_CHAIN_WANT = {}


def test_gpu_grid_chain_matches_per_operator(monkeypatch):
    """The grid form of the fused And (k_chain_grid, DAS_CHAIN_GRID=1): a
    grounded scan feeding an index join whose output every workgroup expands a
    slice of, then row-local stages -- index joins, a cross join with a
    scanned term, an anti index join -- against the per-operator path
    (DAS_FUSED=0) and, where it is cheap, the oracle.  Also: a running result
    empty on every workgroup after the partition (reset-on-empty: redone
    operator by operator), a segment overflowing after the partition (one
    workgroup's rows fan out past kGridSeg = 4096: redone), and the automatic
    choice (DAS_CHAIN_GRID unset)."""
    from das_amd import loader
    rng = np.random.default_rng(5)
    b = loader.AtomBuilder()
    C = lambda n: b.terminal("Concept", n, True)  # noqa: E731
    hub = C("hub")
    xs = [C(f"x{i}") for i in range(50)]
    ys = [C(f"y{i}") for i in range(4000)]
    zs = [C(f"z{i}") for i in range(6000)]
    ws = [C(f"w{i}") for i in range(3)]
    for x in xs:
        b.expr("Rel", [hub, x])
    for y in range(3000):                              # x0 is a hub of Rel2; the others link a few ys
        b.expr("Rel2", [xs[0], ys[y]])
    for i in range(1, 50):
        for y in rng.choice(4000, 5, replace=False):
            b.expr("Rel2", [xs[i], ys[int(y)]])
    for y in range(4000):
        b.expr("Rel3", [ys[y], zs[int(rng.integers(0, 6000))]])
    for z in range(5000):                              # ys[7] fans out past a segment
        b.expr("Rel6", [ys[7], zs[z]])
    for w in ws[:2]:
        b.expr("Rel4", [hub, w])
    for y in rng.choice(4000, 1500, replace=False):
        b.expr("Rel5", [ys[int(y)], ws[int(rng.integers(0, 2))]])
    for z in range(20):
        b.expr("Rel7", [zs[z], zs[z + 1]])             # keys no B reaches
    arrays = b.finish()
    db = _hipdb(arrays)
    V = lambda x: ["Var", x]  # noqa: E731
    h = ["Node", "Concept", "hub"]
    L = lambda t, *a: ["Link", t, True, list(a)]  # noqa: E731
    qs = [["And", [L("Rel", h, V("A")), L("Rel2", V("A"), V("B"))]],
          ["And", [L("Rel", h, V("A")), L("Rel2", V("A"), V("B")), L("Rel3", V("B"), V("C"))]],
          ["And", [L("Rel", h, V("A")), L("Rel2", V("A"), V("B")), L("Rel4", h, V("W")),
                   ["Not", L("Rel5", V("B"), V("W"))], L("Rel3", V("B"), V("C"))]],
          ["And", [L("Rel", h, V("A")), L("Rel2", V("A"), V("B")), L("Rel7", V("B"), V("C")),
                   L("Rel3", V("B"), V("D"))]],
          ["And", [L("Rel", h, V("A")), L("Rel2", V("A"), V("B")), L("Rel6", V("B"), V("C"))]]]
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    wants = []
    for i, q in enumerate(qs):
        monkeypatch.setenv("DAS_FUSED", "0")
        want = record(q, db)
        wants.append(want)
        if i == 0:
            assert same(want, O.evaluate(q, odb))
        for grid in ("1", None):
            monkeypatch.setenv("DAS_FUSED", "1")
            if grid:
                monkeypatch.setenv("DAS_CHAIN_GRID", grid)
            else:
                monkeypatch.delenv("DAS_CHAIN_GRID", raising=False)
            got = record(q, db)
            assert same(got, want), (i, grid, got.get("n"), want.get("n"))
        assert want.get("n", 0) > 1000 or i == 3, (i, want.get("n"))
    # a first term larger than a segment (Rel6: 5000 rows > kGridSeg) before
    # an index join: the grid partitions the scan itself (DAS_CHAIN_PSCAN=1;
    # 0, the default: scan + direct join); a join empty on every workgroup, a first term
    # with no row at all
    monkeypatch.delenv("DAS_CHAIN_GRID", raising=False)
    ps = [["And", [L("Rel6", V("B"), V("C")), L("Rel7", V("C"), V("D"))]],
          ["And", [L("Rel6", V("B"), V("C")), L("Rel3", V("D"), V("C"))]],
          ["And", [L("Rel6", V("B"), V("C")), L("Rel4", V("C"), V("D"))]],
          ["And", [L("Rel6", ["Node", "Concept", "y8"], V("C")), L("Rel7", V("C"), V("D"))]]]
    for i, q in enumerate(ps):
        monkeypatch.setenv("DAS_FUSED", "0")
        want = record(q, db)
        monkeypatch.setenv("DAS_FUSED", "1")
        for pscan in ("1", "0"):
            monkeypatch.setenv("DAS_CHAIN_PSCAN", pscan)
            got = record(q, db)
            assert same(got, want), ("pscan", i, pscan, got.get("n"), want.get("n"))
        if i < 2:
            assert want["n"] > 0, i
    monkeypatch.setenv("DAS_CHAIN_PSCAN", "1")
    for i, (g, w) in enumerate(zip(record_many(ps, db), [record(q, db) for q in ps])):
        assert same(g, w), ("pscan batch", i)
    monkeypatch.delenv("DAS_CHAIN_PSCAN", raising=False)
    # the same Ands as one batch (das_plan_execute_many): grid chains in
    # flight together, the redo and reset-on-empty ones evaluated again
    for grid in ("1", None):
        if grid:
            monkeypatch.setenv("DAS_CHAIN_GRID", grid)
        else:
            monkeypatch.delenv("DAS_CHAIN_GRID", raising=False)
        for i, (g, w) in enumerate(zip(record_many(qs, db), wants)):
            assert same(g, w), (i, grid, g.get("n"), w.get("n"))


@pytest.mark.parametrize("defer", ["1", "0", "1-nomirror"])
def test_gpu_plan_execute_many_matches_one_by_one(defer, monkeypatch):
    """das_plan_execute_many (pm.matched_many, bench.py's step): each answer
    equals the expression evaluated alone -- FlyBase And / And+Not / Or
    shapes on several anchors (fused chains launched first, read back last),
    grid chains including a redo (a segment overflow) and a reset-on-empty,
    a failing term, a Not root, and an And the chain answers only in part;
    DAS_DEFER=0 runs every plan in turn.  1-nomirror: no host mirror of the
    pattern keys (DAS_HOST_KEY_MIRROR=0, the path of P_{a,p} above 2^24
    keys), and the batch runs first, so the chains the wait hook compiles
    resolve their anchored key ranges through a device read-back of their
    own while the outer plan's read-back is pending (PubLevel)."""
    import bench
    from das_amd import synthetic
    monkeypatch.setenv("DAS_DEFER", defer[0])
    if defer.endswith("nomirror"):
        monkeypatch.setenv("DAS_HOST_KEY_MIRROR", "0")
    arrays = synthetic.flybase_kb(200, 6, 400, n_loc=20, n_do=15, seed=3)
    db = _hipdb(arrays)
    qs = []
    for gene in (0, 7, 50, 199, 10 ** 6):
        qs += [q for _, q in bench.flybase_specs(gene, synthetic.flybase_do_terms(arrays, gene))]
    qs.append(["Not", qs[0][1][0]])
    qs = qs + qs[:3]                                    # the same plan twice in one batch
    if defer.endswith("nomirror"):
        got = record_many(qs, db)                       # key ranges not cached yet
        want = [record(q, db) for q in qs]
    else:
        want = [record(q, db) for q in qs]
        got = record_many(qs, db)
    for i, (g, w) in enumerate(zip(got, want)):
        assert same(g, w), (i, g.get("n"), w.get("n"))
    assert any(w["n"] for w in want) and any(not w["matched"] for w in want)
    # more deferrable chains than pooled slots (kPubPool = 16): the rest in turn
    big = [q for q in qs if q[0] == "And"] * 3
    assert len(big) > 16
    got = record_many(big, db)
    for i, g in enumerate(got):
        assert same(g, record(big[i], db)), i


@pytest.mark.parametrize("mode", ["nest", "split", "plain", "nest-nomirror"])
def test_gpu_plan_execute_many_heavy_lead(mode, monkeypatch):
    """das_plan_execute_many's other plans.  nest (the default, here at every
    read-back wait: DAS_PLAN_NEST_MIN=0): the pending plans run whole inside
    a plan's wait, on the plan side stream with their own read-back slot.
    split (DAS_PLAN_SIDE=1, any lead heavier than the rest): from the second
    batch on, the plan whose shape launched the most bytes first, the rest
    after it on the side stream.  plain: all in order.  Bio Q1-Q6 and hub
    H4 / H2 shapes over fresh anchors, three batches each, every answer equal
    to its one-by-one evaluation."""
    import bench
    from das_amd import synthetic
    monkeypatch.setenv("DAS_PLAN_SPLIT_MIN", "0")
    monkeypatch.setenv("DAS_PLAN_NEST_MIN", "0")
    monkeypatch.setenv("DAS_PLAN_SIDE", "1" if mode == "split" else "0")
    monkeypatch.setenv("DAS_PLAN_NEST", "1" if mode.startswith("nest") else "0")
    nomirror = mode.endswith("nomirror")
    if nomirror:                                        # key ranges by device read-backs
        monkeypatch.setenv("DAS_HOST_KEY_MIRROR", "0")
    arrays = synthetic.bio_kb(300, 60, 4000, 200, seed=4)
    db = _hipdb(arrays)
    for rep in range(3):
        qs = [q for _, q in bench.bio_specs(np.arange(300), anchor=rep)]
        got = record_many(qs, db) if nomirror else None
        want = [record(q, db) for q in qs]
        for i, (g, w) in enumerate(zip(got or record_many(qs, db), want)):
            assert same(g, w), ("bio", rep, i, g.get("n"), w.get("n"))
    arrays = synthetic.powerlaw_kb(3000, 300000, link_types=4, seed=21)
    db = _hipdb(arrays)
    qs = [q for _, q in bench.hub_specs()]
    got = record_many(qs, db) if nomirror else None
    want = [record(q, db) for q in qs]
    for rep in range(3):
        for i, (g, w) in enumerate(zip(got if (got and rep == 0) else record_many(qs, db), want)):
            assert same(g, w), ("hub", rep, i, g.get("n"), w.get("n"))


def test_gpu_native_canonical_load_matches_oracle():
    """Canonical text -> native reader (canonical.cpp) -> device index: the
    queries answer as the oracle over the Python reader's atoms; nested
    expressions and repeated terminals included."""
    from das_amd import loader, synthetic
    from das_amd.database.hip_db import HipDB
    arrays = synthetic.powerlaw_kb(150, 1500, link_types=3, seed=9)
    text = synthetic.to_canonical(arrays)
    text += '(T0 "Concept n1" (T1 "Concept n2" "Concept n3"))\n(T2 (T1 "Concept n2" "Concept n3") "Concept n1")\n'
    db = HipDB(device=0)
    db.load_canonical(text)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(loader.parse_canonical(text).finish()))
    assert db.count_atoms() == odb.count_atoms()
    rng = np.random.default_rng(21)
    for q in _random_queries(rng, arrays, 30):
        want = O.evaluate(q, odb)
        got = record(q, db)
        assert same(got, want), (q, got.get("n"), want.get("n"))


def test_gpu_facade_canonical_file(golden):
    """DistributedAtomSpace.load_canonical_knowledge_base on the reference's
    canonical sample (stored in tests/golden/data): the stored counts."""
    from das_amd.distributed_atom_space import DistributedAtomSpace
    das = DistributedAtomSpace()
    das.load_canonical_knowledge_base(os.path.join(os.path.dirname(__file__), "golden", "data",
                                                   "canonical_toy-example-mining.metta"))
    d = golden("kb_toy_mining.json")
    assert das.count_atoms() == (len(d["nodes"]), len(d["links"]))


def _read_lines(path):
    with open(path) as f:
        return [l.rstrip("\n") for l in f if l.strip()]


def test_gpu_keyspace_export_matches_reference_files(tmp_path):
    """das_export_keyspace on the canonical toy KB reproduces, byte for byte
    (after the reference's own sort), the key-value files the reference's
    CanonicalParser wrote (tests/golden/kv_toy_mining, make_golden.py)."""
    from das_amd.database.hip_db import HipDB
    db = HipDB(device=0)
    with open(os.path.join(DATA, "canonical_toy-example-mining.metta")) as f:
        db.load_canonical(f.read())
    counts = db.export_keyspace(str(tmp_path))
    base = os.path.join(os.path.dirname(__file__), "golden", "kv_toy_mining")
    for name, n in counts.items():
        got = _read_lines(tmp_path / f"{name}.txt")
        assert got == sorted(got), name                      # written in bytewise order
        assert got == sorted(_read_lines(os.path.join(base, f"{name}.txt"))), name
        assert n == len(got)


@pytest.mark.parametrize("gen", ["powerlaw", "nested"])
def test_gpu_keyspace_export_matches_oracle(gen, tmp_path):
    """Arity 1-4 links, nested links, repeated targets: the export equals the
    oracle's restatement of the reference's key-value files."""
    from das_amd import loader, synthetic
    from das_amd.database.hip_db import HipDB
    if gen == "powerlaw":
        arrays = synthetic.powerlaw_kb(120, 900, link_types=3, seed=4)
    else:
        b = loader.AtomBuilder()
        n = [b.terminal("Concept", f"c{i}", True) for i in range(6)]
        l1 = b.expr("List", [n[0], n[1]])
        b.expr("Evaluation", [n[2], l1])
        b.expr("Set", [n[3]])
        b.expr("List", [n[0], n[1], n[2], n[3]])
        b.expr("Inheritance", [n[4], n[4]])
        b.expr("Member", [b.expr("List", [n[5], l1, n[5]]), n[1], n[2]])
        arrays = b.finish()
    db = _hipdb(arrays)
    db.export_keyspace(str(tmp_path))
    want = O.keyspace_lines(O.KB.from_arrays(arrays))
    for name, lines in want.items():
        assert _read_lines(tmp_path / f"{name}.txt") == lines, name


# ------------------------------------------------------------ index join

@pytest.mark.parametrize("mode", ["1", "1-bsearch", "1-ranged", "1-rank", "0", "rev"])
@pytest.mark.parametrize("gen", ["bio", "powerlaw", "flybase"])
def test_gpu_index_join_forced_matches_oracle(gen, mode, monkeypatch):
    """And with das_index_join forced on every eligible term (1: keys found
    through the dense per-type key directory; 1-bsearch: by binary search
    over the unique keys) and never (0): the same answers as the oracle,
    incl. grounded-prefix terms (FlyBase Execution(Schema s, V, V)), hub
    keys and empty joins that fall back to the scan path (reset-on-empty).
    1-ranged: grounded-key terms searched within the (type, t_q = v) rows of
    P_{a,q} (ranged mode) wherever the shape allows it; the other modes
    never take it.  rev: unfused, an And's second Link term index-joined
    into the first term's index at every size (DAS_REV_IJ=1).  1-rank: keys
    found through the rank directory (bit per id + word prefixes) at every
    key span (DAS_KEY_RANK=1; by default only spans of >= 2^20 ids)."""
    import bench
    from das_amd import synthetic
    monkeypatch.setenv("DAS_INDEX_JOIN", "" if mode == "rev" else mode[0])
    monkeypatch.setenv("DAS_KEY_RANK", "1" if mode == "1-rank" else "")
    monkeypatch.setenv("DAS_REV_IJ", "1" if mode == "rev" else "")
    if mode == "rev":
        monkeypatch.setenv("DAS_FUSED", "0")
    monkeypatch.setenv("DAS_IJ_RANGED", "1" if mode == "1-ranged" else "0")
    if mode == "1-bsearch":
        monkeypatch.setenv("DAS_NO_KEY_DIR", "1")
    if gen == "bio":
        arrays = synthetic.bio_kb(300, 120, 3000, seed=8)
    elif gen == "powerlaw":
        arrays = synthetic.powerlaw_kb(400, 6000, link_types=4, seed=8)
    else:
        arrays = synthetic.flybase_kb(200, 6, 400, n_loc=20, n_do=15, seed=3)
    db = _hipdb(arrays)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    rng = np.random.default_rng(23)
    qs = [] if gen == "flybase" else _random_queries(rng, arrays, 40)
    if gen == "flybase":
        for gene in (0, 7, 11):
            qs += [q for _, q in bench.flybase_specs(gene, synthetic.flybase_do_terms(arrays, gene))]
    if gen == "powerlaw":
        qs += [q for _, q in bench.hub_specs()]
    if gen == "bio":
        qs += [q for _, q in bench.bio_specs(np.arange(300))]
    for q, want in zip(qs, _wants(("index_join", gen), odb, qs)):
        got = record(q, db)
        assert same(got, want), (q, got.get("n"), want.get("n"))


@pytest.mark.parametrize("gen", ["bio", "powerlaw"])
def test_gpu_no_overload_matches_oracle(gen):
    """CONFIG['no_overload'] = True (pattern_matcher.py:16-19, :98): distinct
    variables of an ordered assignment take distinct values, in scans and
    in joins; random shapes against the oracle under the same flag."""
    from das_amd import synthetic
    from das_amd.pattern_matcher import pattern_matcher as pm
    if gen == "bio":
        arrays = synthetic.bio_kb(200, 60, 2500, seed=12)
    else:
        arrays = synthetic.powerlaw_kb(150, 3000, link_types=2, seed=12)
    db = _hipdb(arrays)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    rng = np.random.default_rng(5)
    pm.CONFIG["no_overload"] = O.CONFIG["no_overload"] = True
    try:
        for q in _random_queries(rng, arrays, 30):
            want = O.evaluate(q, odb)
            got = record(q, db)
            assert same(got, want), (q, got.get("n"), want.get("n"))
    finally:
        pm.CONFIG["no_overload"] = O.CONFIG["no_overload"] = False


@pytest.mark.parametrize("views", ["1", "2"])
@pytest.mark.parametrize("gen", ["bio", "powerlaw"])
def test_gpu_scan_views_match_oracle(gen, views, monkeypatch):
    """DAS_SCAN_VIEWS=1 (default): predicate-free scans inside a plan are views
    of the index rows (no copy); 2: only scans up to 2^20 rows are.  The
    answers, including single-Link ones whose view leaves the plan as a copy,
    equal the oracle's."""
    from das_amd import synthetic
    monkeypatch.setenv("DAS_SCAN_VIEWS", views)
    arrays = synthetic.bio_kb(300, 60, 4000, 200) if gen == "bio" else \
        synthetic.powerlaw_kb(200, 4000, link_types=4, seed=5)
    db = _hipdb(arrays)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    rng = np.random.default_rng(3)
    qs = _random_queries(rng, arrays, 30)
    wants = _wants(("scan_views", gen), odb, qs)             # the oracle once for both settings
    for q, want in zip(qs, wants):
        got = record(q, db)
        assert same(got, want), (q, got.get("n"), want.get("n"))


def test_gpu_ij_mid_matches_multi_launch(monkeypatch):
    """Index joins of mid-size probes (kIjSmall < rows <= kIjMid) in one
    multi-workgroup launch writing the waves' outputs in completion order
    (k_ij_mid) give the same answer sets as the multi-launch ordered path
    (DAS_IJ_MID=0, checked against the oracle by the tests above; the
    oracle's nested-loop And is too slow at these sizes): the Member scan
    (~8000 rows) joined through Inheritance's pattern index, and FlyBase
    chains whose middle result outgrows the fused chain.  The oracle itself
    covers k_ij_mid at 3000-row probes in test_gpu_index_join_forced_*[bio]."""
    import bench
    from das_amd import synthetic
    monkeypatch.setenv("DAS_INDEX_JOIN", "1")
    V, L = bench._V, bench._L
    cases = []
    arrays = synthetic.bio_kb(600, 200, 8000, 400, seed=12)
    cases.append((arrays, [
        ["And", [L("Member", V("G"), V("B")), L("Inheritance", V("B"), V("P"))]],
        ["And", [L("Member", V("G"), V("B")), L("Inheritance", V("P"), V("B"))]],
        ["And", [L("Member", V("G"), V("B")), L("Member", V("G2"), V("B")), L("Inheritance", V("B"), V("P"))]]]))
    arrays = synthetic.flybase_kb(6000, 6, 6000, n_loc=3, n_do=15, seed=5)
    qs = []
    for gene in (0, 7):
        qs += [q for name, q in bench.flybase_specs(gene, synthetic.flybase_do_terms(arrays, gene))
               if name[:2] in ("F5", "F6", "F7")]
    cases.append((arrays, qs))
    # hub keys: a wave owning more than kIjMidWave outputs, or more outputs
    # than the speculative table, sends the join down the balanced path
    arrays = synthetic.powerlaw_kb(3000, 300000, link_types=4, seed=21)
    cases.append((arrays, [q for _, q in bench.hub_specs()]))
    for arrays, qs in cases:
        db = _hipdb(arrays)
        for q in qs:
            monkeypatch.setenv("DAS_IJ_MID", "1")
            got = record(q, db)
            monkeypatch.setenv("DAS_IJ_MID", "0")
            want = record(q, db)
            assert same(got, want), (q, got.get("n"), want.get("n"))


@pytest.mark.parametrize("bits", ["1", "0"])
def test_gpu_union_of_scans_matches_oracle(bits, monkeypatch):
    """Or of anchored one-column scans above the fused chain's size (FlyBase
    cell 9's DO-term Or over hot terms: thousands of rows, genes repeated
    across terms): the one-launch bitmap union (k_union_first, unsorted) and
    the count / write / hash-dedup path (DAS_UNION_BITS=0) against the
    oracle; the queries run back to back, twice."""
    import bench
    from das_amd import synthetic
    monkeypatch.setenv("DAS_UNION_BITS", bits)
    arrays = synthetic.flybase_kb(3000, 5, 500, n_loc=10, n_do=4, seed=9)
    db = _hipdb(arrays)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    E, V = (lambda *t: bench._L("Execution", *t)), bench._V
    do = ["Node", "Schema", "Schema:disease_model_annotations_DO_term"]
    qs = [["Or", [E(do, V("v1"), ["Node", "Verbatim", f"DOID:{d}"]) for d in ds]]
          for ds in ((0, 1), (0, 1, 2, 3), (3, 2), (0, 0))]
    qs.append(["Or", [E(do, V("v1"), ["Node", "Verbatim", "DOID:0"]), E(do, V("v1"), ["Node", "Verbatim", "nope"])]])
    wants = _wants(("union_bits",), odb, qs)
    for _ in range(2):
        for q, want in zip(qs, wants):
            got = record(q, db)
            assert same(got, want), (q, got.get("n"), want.get("n"))


def test_gpu_miner_walk_matches_oracle():
    """The DBInterface calls SimplePatternMiner.ipynb makes (bench.py's
    getlinks leg: halo walk of get_links(None, None, template) +
    get_link_targets, build_patterns' get_links counts), through the facade
    over HipDB before and after prefetch() (host metadata mirrors), against
    the same walk over the oracle: same queries, links and matched counts."""
    import bench
    from das_amd import synthetic
    from das_amd.distributed_atom_space import DistributedAtomSpace
    arrays = synthetic.flybase_kb(400, 10, 600, n_loc=30, n_do=40)
    db = _hipdb(arrays)
    das = DistributedAtomSpace(db=db)
    api = bench.OracleFacade(O.RedisMongoSemantics(O.KB.from_arrays(arrays)))
    seeds = [[O.terminal_hash("gene", f"g{g}")] for g in (0, 7, 123)]
    seeds.append([O.terminal_hash("Verbatim", "FBgn0000042"), O.terminal_hash("Verbatim", "loc3")])

    def strip(r):
        return [(h["queries"], h["links"], h["nodes"]) for h in r["halo"]], \
            (r["pattern"]["links"], r["pattern"]["get_links"], r["pattern"]["matched"])
    for prefetched in (False, True):
        if prefetched:
            db.prefetch()
        for s in seeds:
            got = bench.miner_walk(das, s, np.random.default_rng(1), link_rate=0.2)
            want = bench.miner_walk(api, s, np.random.default_rng(1), link_rate=0.2)
            assert strip(got) == strip(want), (s, prefetched)
            assert got["halo"][1]["links"] > 0
            # the bench's per-level bounds (hub schema nodes): same links walked
            kw = dict(link_rate=0.2, max_level_nodes=5, max_level_links=40)
            got = bench.miner_walk(das, s, np.random.default_rng(1), **kw)
            want = bench.miner_walk(api, s, np.random.default_rng(1), **kw)
            assert strip(got) == strip(want), (s, prefetched, "bounded")
            assert got["halo"][1]["links"] <= 40 and got["halo"][1]["nodes"] <= 5
    # per-link metadata after prefetch equals the device path's
    link = sorted(api.get_links(None, None, ["*", seeds[1][0], "*"]))[0]
    assert das.get_link_targets(link) == api.get_link_targets(link)
    assert das.get_link_type(link) == "Execution"
    assert das.get_node_name(seeds[1][0]) == "g7" and das.get_node_type(seeds[1][0]) == "gene"


def test_gpu_table_checksum_matches_oracle_rows():
    """das_table_checksum (the full-size tests' set checksum) over the device
    answers of the bench's bio and FlyBase queries on small instances equals
    tests/checksum.py's function over the oracle's row sets."""
    import bench
    from das_amd import synthetic
    from tests import checksum as CK
    from das_amd.pattern_matcher import pattern_matcher as pm
    ng = 300
    cases = [(synthetic.bio_full_kb(ng, 80, 6000, 300, n_uniprot=60, n_up_member=800, n_reactome=15,
                                    n_context=300, n_loc=8), bench.bio_specs(np.arange(ng)))]
    fa = synthetic.flybase_kb(300, 8, 400, n_loc=20, n_do=30)
    cases.append((fa, bench.flybase_specs(7, synthetic.flybase_do_terms(fa, gene=7))))
    for arrays, specs in cases:
        db = _hipdb(arrays)
        odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
        for name, spec in specs:
            want = O.evaluate(spec, odb)
            ans = pm.PatternMatchingAnswer()
            bench.build_expr(pm, spec).matched(db, ans)
            got = CK.answer_checksum(ans)
            assert got[1] == want["n"], name
            assert got[0] == CK.rows_checksum(dict(r[1]) for r in want["rows"]), name


@pytest.mark.parametrize("ranged", ["1", "0"])
def test_gpu_ranged_index_join_long_ranges(ranged, monkeypatch):
    """Index joins whose grounded key holds a long row range (the ranged
    mode's interpolation window, narrow_eq): probe values below, above and
    between the range's keys, keys with runs longer than the 32-value
    window, repeated probe values, and keys at both ends of the range --
    against the oracle, ranged mode forced (1) and off (0)."""
    from das_amd import loader
    monkeypatch.setenv("DAS_IJ_RANGED", ranged)
    monkeypatch.setenv("DAS_INDEX_JOIN", "1")
    rng = np.random.default_rng(21)
    b = loader.AtomBuilder()
    C = lambda n: b.terminal("Concept", n, True)  # noqa: E731
    sch = C("schema")
    other = C("other")
    ks = [C(f"k{i}") for i in range(3000)]
    vs = [C(f"v{i}") for i in range(50)]
    probes = [C(f"p{i}") for i in range(40)]
    for i in range(3000):
        if i % 7 == 3:
            continue                                   # keys absent from the range
        reps = 120 if i in (0, 1500, 2999) else (40 if i % 97 == 0 else 1 + i % 3)
        for r in range(reps):
            b.expr("Exec", [sch, ks[i], vs[(i + r) % 50]])
        b.expr("Exec", [other, ks[i], vs[i % 50]])
    for p in probes:
        for k in rng.choice(3000, 30, replace=False).tolist() + [0, 1500, 2999, 3, 97]:
            b.expr("Has", [p, ks[int(k)]])
    arrays = b.finish()
    db = _hipdb(arrays)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    V = lambda x: ["Var", x]  # noqa: E731
    L = lambda t, *a: ["Link", t, True, list(a)]  # noqa: E731
    s = ["Node", "Concept", "schema"]
    for pi in (0, 7, 39):
        p = ["Node", "Concept", f"p{pi}"]
        q = ["And", [L("Has", p, V("K")), L("Exec", s, V("K"), V("W"))]]
        want = O.evaluate(q, odb)
        got = record(q, db)
        assert want.get("n", 0) > 100
        assert same(got, want), (pi, got.get("n"), want.get("n"))
