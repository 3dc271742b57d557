"""Multi-rank evaluation (das_amd/parallel.py) on CPU: world_size 2 over gloo.

The exchange logic (which rows go where, all-to-all / all-gather sequences,
global emptiness, global dedup) is the product code; each rank's local engine
here is a CPU test double with HipLocal's surface, built on the oracle's
DB-path semantics over the rank's own link partition.  Answers must equal the
single-process oracle over the whole KB."""
import json
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from das_amd.parallel import handle_owner
from oracle import das_oracle as O

ORDERED, UNORDERED, COMPOSITE = 0, 1, 2


class NTable:
    def __init__(self, kind, vars_, rows, members=None):
        self.kind = kind
        self.vars = tuple(vars_)
        self.members = tuple(members) if kind == COMPOSITE else None
        self.rows = np.asarray(rows, dtype=np.uint32).reshape(-1, len(vars_))

    @property
    def nrows(self):
        return self.rows.shape[0]

    @property
    def schema(self):
        return (self.kind, self.vars, self.members)

    def fetch(self):
        return self.rows.T.copy()


# ---- composite rows <-> the oracle's row model (ints as variables and values)
def _parts(t):
    """(ordered var list or None, [member var lists]) of a table schema."""
    if t.kind == ORDERED:
        return list(t.vars), []
    if t.kind == UNORDERED:
        return None, [list(t.vars)]
    o = [v for v, m in zip(t.vars, t.members) if m < 0]
    mem = {}
    for v, m in zip(t.vars, t.members):
        if m >= 0:
            mem.setdefault(m, []).append(v)
    return (o or None), [mem[m] for m in sorted(mem)]


def _to_oracle(t, r):
    r = [int(x) for x in r]
    if t.kind == ORDERED:
        return O.o_row(dict(zip(t.vars, r)))
    if t.kind == UNORDERED:
        return O.u_row(t.vars, r)
    o, mems = _parts(t)
    k = len(o) if o else 0
    orow = O.o_row(dict(zip(o, r[:k]))) if o else None
    us = []
    for mv in mems:
        us.append(O.u_row(mv, r[k:k + len(mv)]))
        k += len(mv)
    return ("C", orow, us)


def _join_schema(a, b):
    """Output schema of the CompositeAssignment join (composite.hip)."""
    if a.kind == ORDERED or (a.kind == UNORDERED and b.kind == COMPOSITE):
        x, y = b, a
    else:
        x, y = a, b
    xo, xm = _parts(x)
    yo, ym = _parts(y)
    o = set(xo or [])
    if y.kind != UNORDERED and not (xo and not yo):
        o |= set(yo or [])
    mems = xm + (ym if y.kind != ORDERED else [])
    vars_ = sorted(o) + [v for m in mems for v in m]
    members = [-1] * len(o) + [i for i, m in enumerate(mems) for _ in m]
    return vars_, members


def _from_oracle(vars_, members, rows):
    out = []
    for r in rows:
        vals = dict(r[1][1]) if r[1] is not None else {}
        line = [vals[v] for v, m in zip(vars_, members) if m < 0]
        for u in r[2]:
            line += list(u[2])
        out.append(line)
    return NTable(COMPOSITE, vars_, np.array(out, np.uint32).reshape(-1, len(vars_)), members)


class NRel:
    def __init__(self, tables):
        self.tables = [t for t in tables if t.nrows]
        self._global = None


class NumpyLocal:
    """CPU double of parallel.HipLocal: global atom directory, local links."""

    tuple_targets = False

    def __init__(self, kb_full, rank, world, by_target=None, local_kb=None):
        """by_target {link type: position}: those links live on the rank that
        owns the atom at that position (hash of its handle), the rest by the
        link's own handle -- the layout ShardedDB's partition_spec describes.
        local_kb: this rank's links given directly (parallel.shard_arrays)."""
        handles = set(kb_full.nodes) | set(kb_full.links)
        for _, (_, tg, _) in kb_full.links.items():
            handles.update(tg)
        self.hexes = sorted(handles)
        self.id_of = {h: i for i, h in enumerate(self.hexes)}
        local = O.KB()
        local.nodes = dict(kb_full.nodes)
        by_target = by_target or {}

        def owner(h, v):
            key = v[1][by_target[v[0]]] if v[0] in by_target else h
            return handle_owner(key, world)
        local.links = {h: v for h, v in kb_full.links.items() if owner(h, v) == rank} if local_kb is None \
            else dict(local_kb.links)
        self.odb = O.RedisMongoSemantics(local)
        self.full = O.RedisMongoSemantics(kb_full)

    # DBInterface bits the matcher / ShardedDB use
    def node_exists(self, t, n):
        return self.full.node_exists(t, n)

    def link_exists(self, t, tg):
        return self.full.link_exists(t, tg)

    def get_node_handle(self, t, n):
        return self.full.get_node_handle(t, n)

    def get_link_handle(self, t, tg):
        return self.full.get_link_handle(t, tg)

    def count_atoms(self):
        return (len(self.odb.kb.nodes), len(self.odb.kb.links))

    def hex_of(self, ids):
        return [self.hexes[int(i)] for i in np.asarray(ids).ravel()]

    def rel_local_tables(self, rel):
        return rel.tables

    # the DBInterface pattern / template families (ShardedDB gathers the
    # (link, targets) id rows of every rank's own links)
    def get_matched_links(self, link_type, targets):
        return self.full.get_matched_links(link_type, targets)

    def _pair_table(self, pairs, arity):
        rows = [[self.id_of[h]] + [self.id_of[x] for x in tg] for h, tg in pairs if len(tg) == arity]
        return NTable(ORDERED, [-1] + list(range(arity)), np.array(rows, np.uint32).reshape(-1, arity + 1))

    def matched_links_table(self, link_type, targets):
        return self._pair_table(self.odb.get_matched_links(link_type, targets), len(targets))

    def matched_template_table(self, template):
        return self._pair_table(self.odb.get_matched_type_template(template), len(template) - 1)

    def matched_type_tables(self, link_type):
        pairs = self.odb.get_matched_type(link_type)
        return {a: self._pair_table(pairs, a) for a in sorted({len(tg) for _, tg in pairs})}

    # scans (oracle semantics, local links only)
    def match_link(self, link_type, handles, var_ids, ordered, no_overload=False, order_var=None):
        from das_amd.pattern_matcher.pattern_matcher import _var_name
        pairs = self.odb.get_matched_links(link_type, handles)
        names = [v for v in var_ids if v is not None]
        rows = set()
        for _, targets in pairs:
            if ordered:
                m = {}
                ok = True
                for v, h in zip(var_ids, targets):
                    if v is None:
                        continue
                    if v in m and m[v] != h:
                        ok = False
                        break
                    m[v] = h
                if ok:
                    rows.add(tuple(self.id_of[m[v]] for v in sorted(m)))
            else:
                rem = list(targets)
                for h in handles:
                    if h != "*":
                        rem.remove(h)
                if len(set(rem)) == len(rem):
                    rows.add(tuple(sorted(self.id_of[h] for h in rem)))
        vars_ = sorted(set(names)) if ordered else sorted(names)
        return NRel([NTable(ORDERED if ordered else UNORDERED, vars_, sorted(rows))])

    def match_template(self, link_type, target_types, var_ids, ordered, no_overload=False):
        pairs = self.odb.get_matched_type_template([link_type, *target_types])
        rows = set()
        for _, targets in pairs:
            if ordered:
                m = {}
                ok = True
                for v, h in zip(var_ids, targets):
                    if v in m and m[v] != h:
                        ok = False
                        break
                    m[v] = h
                if ok:
                    rows.add(tuple(self.id_of[m[v]] for v in sorted(m)))
            elif len(set(targets)) == len(targets):
                rows.add(tuple(sorted(self.id_of[h] for h in targets)))
        vars_ = sorted(set(var_ids)) if ordered else sorted(var_ids)
        return NRel([NTable(ORDERED if ordered else UNORDERED, vars_, sorted(rows))])

    # table ops
    def empty_table(self, kind, vars_, members=None):
        return NTable(kind, vars_, np.zeros((0, len(vars_)), np.uint32), members)

    def partition(self, t, key_vars, nparts):
        cols = [t.vars.index(v) for v in key_vars] if key_vars else list(range(len(t.vars)))
        h = np.zeros(t.nrows, dtype=np.uint64)
        for c in cols:
            h = h * np.uint64(1000003) + t.rows[:, c].astype(np.uint64)
        dest = (h % np.uint64(nparts)).astype(np.int64)
        order = np.argsort(dest, kind="stable")
        counts = np.bincount(dest, minlength=nparts).astype(np.uint64)
        return NTable(t.kind, t.vars, t.rows[order], t.members), counts

    def dedup(self, t):
        if t.nrows == 0:
            return t
        return NTable(t.kind, t.vars, np.unique(t.rows, axis=0))

    def concat(self, ts):
        return NTable(ts[0].kind, ts[0].vars, np.concatenate([t.rows for t in ts]), ts[0].members)

    def set_dedup(self, ts):
        seen, out = set(), []
        for t in ts:
            keep = []
            for r in t.rows:
                k = O.ident(_to_oracle(t, r))
                if k not in seen:
                    seen.add(k)
                    keep.append(r)
            out.append(NTable(t.kind, t.vars, np.array(keep, np.uint32).reshape(-1, len(t.vars)), t.members))
        return out

    def set_minus(self, a, b):
        gone = {O.ident(_to_oracle(t, r)) for t in b for r in t.rows}
        return [NTable(t.kind, t.vars, np.array([r for r in t.rows if O.ident(_to_oracle(t, r)) not in gone],
                                                np.uint32).reshape(-1, len(t.vars)), t.members) for t in a]

    def slice(self, t, lo, hi):
        return NTable(t.kind, t.vars, t.rows[lo:hi], t.members)

    def gather_rows(self, t, idx):
        return NTable(t.kind, t.vars, t.rows[np.asarray(idx, dtype=np.int64)], t.members)

    def gather_ranges(self, t, begin, end):
        idx = [np.arange(int(b), int(e)) for b, e in zip(begin, end)]
        return self.gather_rows(t, np.concatenate(idx) if idx else np.zeros(0, np.int64))

    def join(self, a, b, no_overload=False):
        if a.kind != ORDERED or b.kind != ORDERED:
            vars_, members = _join_schema(a, b)
            rb = [_to_oracle(b, r) for r in b.rows]
            out = [j for r in a.rows for y in rb for j in [O.join(_to_oracle(a, r), y)] if j is not None]
            return _from_oracle(vars_, members, out)
        shared = sorted(set(a.vars) & set(b.vars))
        uni = sorted(set(a.vars) | set(b.vars))
        idx = {}
        for r in b.rows:
            idx.setdefault(tuple(r[b.vars.index(v)] for v in shared), []).append(r)
        out = []
        for r in a.rows:
            for s in idx.get(tuple(r[a.vars.index(v)] for v in shared), []):
                m = {v: r[a.vars.index(v)] for v in a.vars}
                m.update({v: s[b.vars.index(v)] for v in b.vars})
                out.append([m[v] for v in uni])
        return NTable(ORDERED, uni, np.array(out, np.uint32).reshape(-1, len(uni)))

    def antijoin(self, a, t):
        if a.kind != ORDERED or t.kind != ORDERED:
            rt = [_to_oracle(t, r) for r in t.rows]
            keep = [r for r in a.rows if all(O.check_negation(_to_oracle(a, r), x) for x in rt)]
            return NTable(a.kind, a.vars, np.array(keep, np.uint32).reshape(-1, len(a.vars)), a.members)
        if not set(t.vars) <= set(a.vars):
            return a
        bad = {tuple(r) for r in t.rows}
        keep = [r for r in a.rows if tuple(r[a.vars.index(v)] for v in t.vars) not in bad]
        return NTable(a.kind, a.vars, np.array(keep, np.uint32).reshape(-1, len(a.vars)))

    # collective staging (CPU tensors for gloo)
    def xfer_tensor(self, arr):
        return torch.from_numpy(np.ascontiguousarray(arr))

    def xfer_numpy(self, t):
        return t.numpy()

    def rows_buffer(self, n, ncols):
        return torch.zeros((max(n, 0), max(ncols, 1)), dtype=torch.int32)

    def rows_out(self, t):
        return torch.from_numpy(t.rows.astype(np.int32).reshape(-1, max(len(t.vars), 1)).copy())

    def rows_pad(self, buf, width, ncols):
        out = self.rows_buffer(width, ncols)
        out[:buf.shape[0]] = buf
        return out

    def rows_in(self, kind, vars_, buf, n, members=None):
        return NTable(kind, vars_, buf[:n].numpy().astype(np.uint32).reshape(-1, len(vars_)), members)

    def rows_in_many(self, kind, vars_, bufs, counts, members=None):
        parts = [b[:c].numpy() for b, c in zip(bufs, counts)]
        return NTable(kind, vars_, np.concatenate(parts).astype(np.uint32).reshape(-1, len(vars_)), members)


def _queries():
    V = lambda n: ["Var", n]  # noqa: E731
    m = lambda a, b: ["Link", "Member", True, [a, b]]  # noqa: E731
    i = lambda a, b: ["Link", "Inheritance", True, [a, b]]  # noqa: E731
    g = lambda k: ["Node", "Gene", f"g{k}"]  # noqa: E731
    bp = lambda k: ["Node", "BiologicalProcess", f"bp{k}"]  # noqa: E731
    return [
        m(V("G"), V("B")),
        m(V("G"), bp(0)),
        ["And", [m(V("G"), V("B")), i(V("B"), V("P"))]],
        ["And", [m(g(3), V("B")), m(g(5), V("B"))]],
        ["And", [m(V("G"), bp(0)), m(V("G"), V("B"))]],
        ["And", [m(V("G"), V("B")), ["Not", m(V("G"), bp(1))]]],
        ["Or", [m(V("G"), bp(0)), m(V("G"), bp(2))]],
        ["Or", [i(V("B"), V("P")), ["Not", i(V("B"), bp(0))]]],
        # Or with a Not of the positive term's own schema: rel_minus must
        # subtract (pattern_matcher.py:681, term_answer - or_answer)
        ["Or", [m(V("G"), bp(0)), ["Not", m(V("G"), bp(1))]]],
        ["Or", [m(V("G"), bp(0)), m(V("G"), bp(2)), ["Not", m(V("G"), bp(0))]]],
        ["And", [i(V("A"), V("B")), i(V("B"), V("C")), i(V("C"), V("D"))]],
        ["And", [m(g(7), V("B")), i(V("X"), V("Y"))]],           # no shared variable
        ["Link", "*", True, [V("X"), bp(0)]],                     # global dedup path
        ["Template", "Inheritance", True, [["TVar", "A", "BiologicalProcess"], ["TVar", "B", "BiologicalProcess"]]],
    ]


def _composite_queries():
    """Similarity / Set terms: the CompositeAssignment exchange paths."""
    V = lambda n: ["Var", n]  # noqa: E731
    c = lambda k: ["Node", "Concept", f"c{k}"]  # noqa: E731
    inh = lambda a, b: ["Link", "Inheritance", True, [a, b]]  # noqa: E731
    sim = lambda a, b: ["Link", "Similarity", False, [a, b]]  # noqa: E731
    st = lambda a, b, d: ["Link", "Set", False, [a, b, d]]  # noqa: E731
    return [
        sim(V("A"), V("B")),
        sim(c(0), V("A")),
        ["And", [inh(V("A"), V("B")), sim(V("A"), V("B"))]],
        ["And", [sim(V("A"), V("B")), sim(V("B"), V("C"))]],
        ["And", [sim(V("A"), V("B")), sim(V("A"), V("B"))]],
        ["And", [inh(V("A"), V("B")), inh(V("B"), V("C")), sim(V("A"), V("C"))]],
        ["And", [st(V("A"), V("B"), V("C")), sim(V("A"), V("B"))]],
        ["And", [sim(V("A"), V("B")), ["Not", inh(V("A"), V("B"))]]],
        ["And", [inh(V("A"), V("B")), ["Not", sim(V("A"), V("B"))]]],
        ["Or", [inh(V("A"), c(1)), sim(V("A"), V("B"))]],
        ["Or", [["And", [sim(V("A"), V("B")), inh(V("A"), V("B"))]], ["Not", inh(V("A"), c(0))]]],
        ["And", [sim(V("A"), V("B")), sim(V("A"), V("C")), ["Not", st(V("A"), V("B"), V("C"))]]],
    ]


def _fly_queries():
    import bench
    from das_amd import synthetic
    from tests.golden import make_synthetic as MS
    arrays = MS.make_arrays("flybase")
    return [q for g in (0, 42) for _, q in bench.flybase_specs(g, synthetic.flybase_do_terms(arrays, g))]


def _hub_queries():
    import bench
    V = lambda n: ["Var", n]  # noqa: E731
    n = lambda i: ["Node", "Concept", f"n{i}"]  # noqa: E731
    L = lambda t, a, b: ["Link", t, True, [a, b]]  # noqa: E731
    return [q for _, q in bench.hub_specs()] + [
        ["And", [L("T0", V("V1"), n(0)), L("T0", V("V1"), V("V2")), L("T0", V("V2"), n(1))]],
        ["And", [L("T1", V("V1"), V("V2")), L("T1", V("V2"), n(0)), ["Not", L("T2", V("V1"), n(1))]]],
        # two large unanchored terms on the hub keys (config 5's skewed exchange)
        ["And", [L("T1", V("V1"), V("V2")), L("T2", V("V2"), V("V3"))]],
        # the open 4-clause chain of SURVEY.md §8d config 5
        ["And", [L("T0", V("V1"), n(0)), L("T1", V("V1"), V("V2")), L("T2", V("V2"), n(1)),
                 L("T3", V("V2"), V("V3"))]]]


# kind -> (DAS_JOIN_PLACEMENT, DAS_HEAVY_FRAC)
_ENV = {"bio_exchange": ("exchange", ""), "bio_broadcast": ("broadcast", ""), "bio_heavy": ("exchange", "0.05"),
        "hub": ("exchange", "0.05"), "flybase": ("exchange", "0.2")}


def _kb(kind):
    from das_amd import synthetic
    if kind in ("bio", "bio_part", "bio_exchange", "bio_broadcast", "bio_heavy"):
        return O.KB.from_arrays(synthetic.bio_kb(60, 25, 600, 80, seed=3)), _queries()
    if kind == "flybase":
        from tests.golden import make_synthetic as MS
        return O.KB.from_arrays(MS.make_arrays("flybase")), _fly_queries()
    if kind == "hub":
        from tests.golden import make_synthetic as MS
        return O.KB.from_arrays(MS.make_arrays("hub")), _hub_queries()
    return O.KB.from_arrays(synthetic.similarity_kb(n_nodes=20, n_inh=90, n_sim=45, n_set=20, seed=9)), \
        _composite_queries()


def _worker(rank, world, port, out_path, kind):
    place, heavy = _ENV.get(kind, ("", ""))
    os.environ["DAS_JOIN_PLACEMENT"] = place
    if heavy:
        os.environ["DAS_HEAVY_FRAC"] = heavy
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from das_amd.parallel import ShardedDB
    from tests.util import build, canon
    from das_amd.pattern_matcher import pattern_matcher as pm
    kb, queries = _kb(kind)
    spec = {"Member": 0} if kind == "bio_part" else None
    # links by their handle's owner (the bench's layout, parallel.shard_arrays)
    sdb = ShardedDB(NumpyLocal(kb, rank, world, by_target=spec), dist, partition_spec=spec)
    res = []
    for q in queries:
        ans = pm.PatternMatchingAnswer()
        try:
            m = build(q).matched(sdb, ans)
        except AttributeError as e:
            res.append({"error": type(e).__name__})
            continue
        rows = sorted(json.dumps(canon(a), sort_keys=True) for a in ans.assignments)
        res.append({"matched": bool(m), "negation": ans.negation, "n": ans.count(), "rows": rows,
                    "local": sdb.rel_local_count(ans._relation())})
    res.append(sdb.plan_stats)
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2])
@pytest.mark.parametrize("kind", ["bio", "bio_part", "bio_exchange", "bio_broadcast", "bio_heavy", "hub",
                                  "flybase", "composite"])
def test_sharded_matcher_equals_single_process_oracle(world, kind):
    kb, queries = _kb(kind)
    odb = O.RedisMongoSemantics(kb)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res")
        mp.spawn(_worker, args=(world, _free_port(), out, kind), nprocs=world, join=True)
        per_rank = [json.load(open(f"{out}.{r}")) for r in range(world)]
    stats = per_rank[0][-1]
    if kind == "bio_part":
        assert stats["colocated"] > 0 and stats["broadcast"] > 0, stats    # both placements exercised
    if kind in ("bio_exchange", "bio_broadcast"):
        assert stats[kind[4:]] > 0 and stats["colocated"] == 0, stats
    if _ENV.get(kind, ("", ""))[1]:
        assert stats["heavy"] > 0, stats                                  # skewed buckets split
    for qi, q in enumerate(queries):
        want = O.evaluate(q, odb)
        if "error" in want:
            assert all(per_rank[r][qi] == {"error": want["error"]} for r in range(world)), q
            continue
        want_rows = sorted(json.dumps(r, sort_keys=True) for r in want["rows"])
        locals_ = 0
        for r in range(world):
            got = per_rank[r][qi]
            assert got["matched"] == want["matched"] and got["negation"] == want["negation"], q
            assert got["n"] == want["n"], (q, got["n"], want["n"])
            assert got["rows"] == want_rows, q
            locals_ += got["local"]
        assert locals_ == want["n"], (q, locals_, want["n"])      # partitions are disjoint


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", ["bio_full", "hub"])
def test_partition_arrays_build_union_equals_single_build(world, name):
    """Config 4 at N GPUs: each rank indexes only its partition_arrays shard.
    The shards' key-value families (outgoing / incoming sets, pattern and
    template keys, names -- canonical_parser.py:119-183) must union to the
    single build's, and every link (nested ones too) is indexed on exactly
    one rank: the one its handle names."""
    from das_amd.parallel import partition_arrays
    from tests.golden import make_synthetic as MS
    full_kb = O.KB.from_arrays(MS.make_arrays(name))
    full = O.keyspace_lines(full_kb)
    union = {k: set() for k in full}
    owners = {}
    for r in range(world):
        kb = O.KB.from_arrays(partition_arrays(MS.make_arrays(name), r, world))
        for k, lines in O.keyspace_lines(kb).items():
            union[k] |= set(lines)
        for h in kb.links:
            owners[h] = owners.get(h, 0) + 1
            assert handle_owner(h, world) == r
    for k in full:
        assert union[k] == set(full[k]), k
    assert owners == {h: 1 for h in full_kb.links}


def _surface_calls(kb):
    """get_matched_links / get_matched_type_template / get_matched_type calls
    (DistributedAtomSpace.get_links' three branches, distributed_atom_space.py:259-284)."""
    node = sorted(kb.nodes)
    return [("links", "Member", ["*", "*"]), ("links", "Member", ["*", node[3]]), ("links", "*", [node[5], "*"]),
            ("links", "Inheritance", ["*", "*"]), ("links", "Member", [node[1], node[2]]),
            ("links", "Nope", ["*", "*"]),
            ("template", ["Member", "Gene", "BiologicalProcess"]), ("template", ["Inheritance"]),
            ("template", ["Inheritance", "BiologicalProcess", "BiologicalProcess"]),
            ("type", "Member"), ("type", "Inheritance"), ("type", "Nope")]


def _call(db, c):
    if c[0] == "links":
        return db.get_matched_links(c[1], c[2])
    if c[0] == "template":
        return db.get_matched_type_template(c[1])
    return db.get_matched_type(c[1])


def _canon_pairs(x):
    return sorted(json.dumps(p if isinstance(p, str) else [p[0], list(p[1])]) for p in x)


def _surface_worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from das_amd.parallel import ShardedDB
    kb, _ = _kb("bio")
    sdb = ShardedDB(NumpyLocal(kb, rank, world), dist)
    res = [_canon_pairs(_call(sdb, c)) for c in _surface_calls(kb)]
    res.append(sdb.plan_stats["collectives"])
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


def test_sharded_dbinterface_surface_equals_single_process():
    """ShardedDB.get_matched_links / get_matched_type_template /
    get_matched_type over two ranks, each holding only its own links' index
    rows: every rank returns the single-process DB-path answer (the reference
    serves these from a sharded Redis Cluster, redis_mongo_db.py:235-279)."""
    kb, _ = _kb("bio")
    odb = O.RedisMongoSemantics(kb)
    want = [_canon_pairs(_call(odb, c)) for c in _surface_calls(kb)]
    assert any(len(w) > 10 for w in want)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res")
        mp.spawn(_surface_worker, args=(2, _free_port(), out), nprocs=2, join=True)
        per_rank = [json.load(open(f"{out}.{r}")) for r in range(2)]
    for r in range(2):
        assert per_rank[r][:-1] == want
        assert per_rank[r][-1] > 0                      # the rows came through collectives
