"""Multi-GPU query evaluation: links hash-partitioned across ranks, binding
tables exchanged with all-to-all only where a join needs co-location.

Layout.  Every rank holds the *atom directory* of the whole KB
(all handles -> global ids, outgoing sets), so ids agree across ranks and
node/link existence needs no collective; the *pattern index* rows (T_a, C_a,
P_{a,p}) of a link live only on its owner shard.  The reference's only
"distribution" is Redis Cluster key sharding plus one Mongo
(das/distributed_atom_space.py:48-61); there is no counterpart of this
exchange in the reference.

Relational algebra of pattern_matcher over sharded relations:
  scan        local (each rank scans its own links); rows of different links
              are distinct, so no exchange unless the scan can duplicate
              bindings ('*' type, repeated variable, unordered sets) -> global
              dedup (repartition by every column)
  join        repartition both sides by hash(shared variables) (all-to-all),
              local join; no shared variable -> all-gather the smaller side
  antijoin    repartition by hash(forbidden variables)
  union/minus repartition by hash(all columns), local dedup / antijoin
  nonempty    all-reduce of local row counts (so control flow is identical
              on every rank and every rank issues the same collectives)

The collectives go through torch.distributed ("nccl" = RCCL on ROCm, over
xGMI; "gloo" in the CPU tests).  `local` is a HipDB (or, in tests, a CPU
double with the same surface).
"""
import gc
import os

import numpy as np

from .database.db_interface import UNORDERED_LINK_TYPES, WILDCARD
from .database.hip_db import RelationalDB

L_MAXCOLS = 16                              # columns of a binding table (das_internal.h kMaxCols)

ORDERED, UNORDERED, COMPOSITE = 0, 1, 2


def _part(t):
    """How a local table's rows are spread over ranks: ("atom", var) = by the
    owner of that variable's atom (partition_spec), ("hash", vars) = by
    hash(vars) after an exchange, None = unknown."""
    return getattr(t, "part", None)


def _with_part(t, part):
    try:
        t.part = part
    except AttributeError:
        pass
    return t


def _members(t):
    return getattr(t, "members", None)


def _has_o(t):
    if t.kind == ORDERED:
        return True
    return t.kind == COMPOSITE and any(m < 0 for m in t.members)


def _join_raises(ta, tb):
    """The reference's AttributeError for a pair of non-empty relations
    (pattern_matcher.py:106 via CompositeAssignment.join :348-349): the
    absorbing composite has an ordered part and the other composite has none."""
    if ta.kind == ORDERED or (ta.kind == UNORDERED and tb.kind == COMPOSITE):
        x, y = tb, ta
    else:
        x, y = ta, tb
    return y.kind == COMPOSITE and not _has_o(y) and _has_o(x)


def _antijoin_raises(t, f):
    """check_negation against a composite negation (:117, :359-360)."""
    return f.kind == COMPOSITE and t.kind != UNORDERED


class DRel:
    """A sharded relation: one local table per schema, empty tables kept so the
    schema list (and so the collective sequence) is the same on every rank."""

    __slots__ = ("tables", "_global")

    def __init__(self, tables):
        self.tables = list(tables)
        self._global = None


class ShardedDB(RelationalDB):

    def __init__(self, local, dist, group=None, partition_spec=None):
        """partition_spec: {link type: target position} for link types whose
        links are placed on the rank that owns the atom at that position (one
        owner function for every listed type, e.g. bio_shard's gene ranges).
        Scans of those types are then known to be partitioned by the variable
        at that position, and joins on it need no exchange."""
        self.local = local
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.tuple_targets = local.tuple_targets
        self.spec = dict(partition_spec or {})
        # join placements taken; native = expressions evaluated by one sharded
        # native plan (fallback: its check failed), collectives issued
        self.plan_stats = {"colocated": 0, "broadcast": 0, "exchange": 0, "heavy": 0, "native": 0,
                           "native_fallback": 0, "collectives": 0, "size_cache": 0}
        # leaf sizes of sharded plans known without an exchange (generation,
        # exact sizes by leaf words, upper bounds by leaf shape)
        self._size_gen = None
        self._exact_sizes = {}
        self._shape_sizes = {}
        # DAS_JOIN_PLACEMENT=exchange|broadcast forces one placement (tests)
        self.force = os.environ.get("DAS_JOIN_PLACEMENT", "")
        # the top-level expression of the current ShardedMatcher call, and the
        # round-robin owner of the next wholly gathered top-level plan
        self._top = None
        self._tops = set()          # ids of the top-level expressions of a batch (ShardedMatcher.count_many)
        self._no_plan = set()       # ids of batch expressions that fell back: the operator fold
        self._gather_seq = 0
        # a key bucket is heavy when its rows (both sides) exceed this fraction
        # of one rank's fair share of the join's rows (DAS_HEAVY_FRAC, tests)
        self.heavy_frac = float(os.environ.get("DAS_HEAVY_FRAC", "1.0"))

    # ------------------------------------------------------------ collectives
    @property
    def pattern_black_list(self):
        """The local engine's load-time pattern black list (HipDB.load_arrays)."""
        return self.local.pattern_black_list

    @pattern_black_list.setter
    def pattern_black_list(self, value):
        self.local.pattern_black_list = list(value)

    def _allreduce_sum(self, values):
        t = self.local.xfer_tensor(np.asarray(values, dtype=np.int64))
        self.dist.all_reduce(t, group=self.group)
        self.plan_stats["collectives"] += 1
        return self.local.xfer_numpy(t)

    def _allgather_i64(self, values):
        """[world, len(values)] int64 of every rank's `values` (one collective)."""
        t = self.local.xfer_tensor(np.asarray(values, dtype=np.int64))
        out = self.local.xfer_tensor(np.zeros(self.world * t.numel(), dtype=np.int64))
        self.dist.all_gather_into_tensor(out, t, group=self.group)
        self.plan_stats["collectives"] += 1
        return self.local.xfer_numpy(out).reshape(self.world, -1)

    def _exchange(self, table, key_vars):
        """Repartition `table` by hash(key_vars) (every column if empty)."""
        if self.world == 1:
            return table
        key = tuple(sorted(key_vars)) if key_vars else ("*",)        # "*": every column
        if _part(table) == ("hash", key):
            return table                                   # already placed by this key
        return _with_part(self._exchange_rows(table, list(key) if key_vars else []), ("hash", key))

    def _exchange_rows(self, table, key_vars):
        part, counts = self.local.partition(table, list(key_vars), self.world)
        return self._send_grouped(table, part, counts)

    def _send_grouped(self, table, part, counts):
        """All-to-all of `part` (the rows of `table` grouped by destination
        rank, counts[d] rows for rank d): sizes first, then the rows."""
        send_counts = self.local.xfer_tensor(counts.astype(np.int64))
        recv_counts = self.local.xfer_tensor(np.zeros(self.world, dtype=np.int64))
        self.dist.all_to_all_single(recv_counts, send_counts, group=self.group)
        self.plan_stats["collectives"] += 2
        rc = self.local.xfer_numpy(recv_counts).tolist()
        ncols = len(table.vars)
        send = self.local.rows_out(part)
        recv = self.local.rows_buffer(int(sum(rc)), ncols)
        self.dist.all_to_all_single(recv, send, output_split_sizes=rc, input_split_sizes=counts.tolist(),
                                    group=self.group)
        return self.local.rows_in(table.kind, table.vars, recv, int(sum(rc)), _members(table))

    def _gather_all(self, table):
        """Every rank gets the whole relation (all-gather of row blocks)."""
        if self.world == 1:
            return table
        n = self._allgather_counts(table.nrows)
        ncols = len(table.vars)
        send = self.local.rows_out(table)
        width = int(max(n)) if len(n) else 0
        padded = self.local.rows_pad(send, width, ncols)
        outs = [self.local.rows_buffer(width, ncols) for _ in range(self.world)]
        self.dist.all_gather(outs, padded, group=self.group)
        self.plan_stats["collectives"] += 1
        return self.local.rows_in_many(table.kind, table.vars, outs, [int(x) for x in n], _members(table))

    def _rank_slice(self, table):
        """This rank's share of a table every rank holds identically."""
        if self.world == 1:
            return table
        lo = table.nrows * self.rank // self.world
        hi = table.nrows * (self.rank + 1) // self.world
        return self.local.slice(table, lo, hi)

    def _allgather_counts(self, n):
        t = self.local.xfer_tensor(np.array([n], dtype=np.int64))
        outs = [self.local.xfer_tensor(np.zeros(1, dtype=np.int64)) for _ in range(self.world)]
        self.dist.all_gather(outs, t, group=self.group)
        self.plan_stats["collectives"] += 1
        return np.array([int(self.local.xfer_numpy(o)[0]) for o in outs], dtype=np.int64)

    # ----------------------------------------------------- DBInterface (global)
    def node_exists(self, node_type, node_name):
        return self.local.node_exists(node_type, node_name)

    def link_exists(self, link_type, targets):
        return self.local.link_exists(link_type, targets)

    def get_node_handle(self, node_type, node_name):
        return self.local.get_node_handle(node_type, node_name)

    def get_link_handle(self, link_type, targets):
        return self.local.get_link_handle(link_type, targets)

    def get_link_targets(self, handle):
        return self.local.get_link_targets(handle)

    def is_ordered(self, handle):
        return self.local.is_ordered(handle)

    # The pattern / template families of a sharded KB: each shard holds the
    # index rows of the links it owns, so a lookup scans every shard's rows of
    # the key and gathers them -- the reference reads the same families from
    # a Redis Cluster whose key slots are spread over nodes
    # (redis_mongo_db.py:235-279, distributed_atom_space.py:48-61, 259-284).
    # Every rank calls these together (SPMD) and every rank gets the whole
    # answer, sorted by link id (the reference returns a Redis set: no order).
    def _gather_pairs(self, tables):
        """{arity: local (link, t0..t_{a-1}) table or None} -> [(handle,
        targets)] of every shard's rows.  The arities present anywhere are
        agreed first (one all-reduce), then one all-gather per arity present."""
        have = np.zeros(9, dtype=np.int64)
        for a, t in tables.items():
            if t is not None:
                have[a] = t.nrows
        got = self._allreduce_sum(have) if self.world > 1 else have
        out = []
        fmt = tuple if self.tuple_targets else list
        for a in range(9):
            if int(got[a]) == 0:
                continue
            t = tables.get(a)
            if t is None:
                t = self.local.empty_table(ORDERED, [-1] + list(range(a)))
            cols = self._gather_all(t).fetch()
            if cols.shape[1] == 0:
                continue
            cols = cols[:, np.argsort(cols[0], kind="stable")]
            links = self.local.hex_of(cols[0])
            tg = [self.local.hex_of(cols[1 + k]) for k in range(a)]
            enabled = gc.isenabled()
            gc.disable()                     # one container per row (HipDB._pairs)
            try:
                out += list(zip(links, map(fmt, zip(*tg))))
            finally:
                if enabled:
                    gc.enable()
        return out

    def get_matched_links(self, link_type, target_handles):
        """redis_mongo_db.py:235-252 over every shard: a grounded key is a
        directory lookup (every shard holds the whole atom directory); a key
        with a wildcard gathers every shard's rows of the pattern key."""
        if link_type != WILDCARD and WILDCARD not in target_handles:
            return self.local.get_matched_links(link_type, target_handles)
        t = self.local.matched_links_table(link_type, list(target_handles))
        return self._gather_pairs({len(target_handles): t})

    def get_all_nodes(self, node_type, names=False):
        return self.local.get_all_nodes(node_type, names)

    def get_matched_type_template(self, template):
        """redis_mongo_db.py:269-275 over every shard (templates:<ctype>)."""
        if len(template) == 1:
            return self.get_matched_type(template[0])
        t = self.local.matched_template_table(list(template))
        return self._gather_pairs({len(template) - 1: t})

    def get_matched_type(self, link_type):
        """redis_mongo_db.py:277-279 over every shard (templates:<type>)."""
        tables = self.local.matched_type_tables(link_type)
        return self._gather_pairs({a: tables.get(a) for a in range(9)})

    def get_node_name(self, node_handle):
        return self.local.get_node_name(node_handle)

    def get_matched_node_name(self, node_type, substring):
        return self.local.get_matched_node_name(node_type, substring)

    def count_atoms(self):
        nodes, links = self.local.count_atoms()
        return (nodes, int(self._allreduce_sum([links])[0]))

    def hex_of(self, ids):
        return self.local.hex_of(ids)

    def prefetch_handles(self, handles):
        if hasattr(self.local, "prefetch_handles"):
            self.local.prefetch_handles(handles)

    # ------------------------------------------------------- matcher entries
    @staticmethod
    def _schema(var_ids, ordered):
        names = [v for v in var_ids if v is not None]
        return (ORDERED if ordered else UNORDERED), tuple(sorted(set(names)) if ordered else sorted(names))

    def _ensure(self, rel, kind, vars_):
        tables = self.local.rel_local_tables(rel)
        if tables:
            return tables[0]
        return self.local.empty_table(kind, list(vars_))

    def match_link(self, link_type, handles, var_ids, ordered, no_overload=False, order_var=None):
        kind, vars_ = self._schema(var_ids, ordered)
        names = [v for v in var_ids if v is not None]
        if not ordered and len(set(names)) != len(names):
            return DRel([])
        t = self._ensure(self.local.match_link(link_type, handles, var_ids, ordered, no_overload, order_var=order_var),
                         kind, vars_)
        dup = link_type == WILDCARD or len(set(names)) != len(names) or not ordered or \
            link_type in UNORDERED_LINK_TYPES
        if dup:
            t = _with_part(self.local.dedup(self._exchange(t, [])), ("hash", ("*",)))
        elif link_type in self.spec and self.spec[link_type] < len(var_ids) and \
                var_ids[self.spec[link_type]] is not None:
            t = _with_part(t, ("atom", var_ids[self.spec[link_type]]))
        return DRel([t])

    def match_template(self, link_type, target_types, var_ids, ordered, no_overload=False):
        kind = ORDERED if ordered else UNORDERED
        vars_ = tuple(sorted(set(var_ids))) if ordered else tuple(sorted(var_ids))
        if not ordered and len(set(var_ids)) != len(var_ids):
            return DRel([])
        t = self._ensure(self.local.match_template(link_type, target_types, var_ids, ordered, no_overload),
                         kind, vars_)
        if not ordered or len(set(var_ids)) != len(var_ids):
            t = self.local.dedup(self._exchange(t, []))
        return DRel([t])

    # ------------------------------------------------- sharded native plans
    # A term whose rows over all shards exceed SMALL (DAS_SHARD_SMALL) stays
    # split (read from each shard's index); smaller terms are gathered to
    # every shard.
    SMALL = 1 << 22
    GATHER_LIMIT = 1 << 26              # rows gathered per query at most (else the per-operator path)
    GATHER_BUDGET = 1 << 28             # bytes of large terms gathered at most (else the per-operator fold)

    def plan_sharded(self, expr, answer):
        """Evaluates `expr` as ONE das_plan_execute_sharded call per GPU, or
        returns None (the caller then folds it operator by operator).

        Shapes: a single Link, an And of Links / grounded terms / Not(Link),
        an Or of Links (each Link ordered, its rows distinct).  Every Link's
        index rows are estimated on each shard and all-gathered (collective
        1); an And keeps its one large term -- or several, when
        partition_spec places them all by the same variable -- split across
        shards, read through each shard's index (scan, index join, filtered
        expansion), and gathers every other term to every shard in one
        all-gather (collective 2).  The fold assumes the split running result
        non-empty where it tests it; the final all-reduce of the result rows
        and of those tests' outcomes (collective 3) confirms it, or the
        expression falls back (pattern_matcher.py:705-748 semantics either way).
        One expression of plan_many."""
        return self.plan_many([(expr, answer)])[0]

    def plan_many(self, items):
        """plan_sharded for several independent expressions at once -- a
        step's queries -- with their collectives shared: ONE estimate
        all-gather for every leaf no cache settles, ONE all-to-all carrying
        every expression's gathered terms (to every shard, or to the owner
        of a wholly gathered top-level plan), ONE all-reduce of every
        expression's outcome (result rows, schema / overflow flags, the
        split running results' non-empty tests).  items: (expr, answer)
        pairs; returns each expression's matched() or None (that expression
        falls back to the operator fold, on every shard alike).  Every shard
        takes the same decisions in the same order from collective results
        only, so every shard issues the same collectives."""
        res = [None] * len(items)
        sts = []
        for k, (expr, answer) in enumerate(items):
            st = None if id(expr) in self._no_plan else self._plan_prepare(expr, answer)
            if st is not None:
                st["k"] = k
                sts.append(st)
        if not sts:
            return res
        self._plan_sizes([st for st in sts if st["leaves_sized"]])            # collective 1 (or none)
        ready = []
        for st in sts:
            if self._plan_place(st):
                ready.append(st)
        self._plan_gather([st for st in ready if st["gathered"]])             # collective 2 (or none)
        vecs = []
        for st in ready:
            self._plan_evaluate(st)
            if st.get("vec") is not None:
                vecs.append(st)
        if vecs:                                                              # collective 3 (or none)
            got = self._allreduce_sum(np.concatenate([st["vec"] for st in vecs]))
            o = 0
            for st in vecs:
                m = len(st["vec"])
                st["got"] = got[o:o + m]
                o += m
        for st in ready:
            res[st["k"]] = self._plan_finish(st)
        return res

    def _plan_prepare(self, expr, answer):
        """Phase 1 (local): the lowered plan and its shape; None when it is
        not a sharded native plan."""
        from .pattern_matcher import pattern_matcher as pm
        from . import _lib as L
        db = getattr(self.local, "db", None)
        if db is None or not hasattr(db, "ctx") or os.environ.get("DAS_SHARDED_PLAN") == "0" or answer.negation:
            return None
        no_overload = bool(pm.CONFIG['no_overload'])
        key = (db.generation, no_overload)
        cached = getattr(expr, '_plan', None)
        if cached is None or cached[0] != key:
            cached = (key, pm._lower(expr, db, no_overload))
            expr._plan = cached
        nodes = cached[1]
        if nodes is None:
            return None
        W = L.PLAN_WORDS
        n = len(nodes) // W
        rec = nodes.reshape(n, W)
        op = rec[:, 0]
        leaves = [i for i in range(n) if op[i] in (L.PLAN_LINK, L.PLAN_TEMPLATE)]
        # A tree whose leaves are all gathered evaluates identically on every
        # shard (any shape).  Terms can stay split only under a root And (or
        # Link) whose children are leaves: LINK / CONST / TEMPLATE / NOT LINK.
        pos, neg = [], []
        flat = op[0] == L.PLAN_LINK
        if op[0] == L.PLAN_LINK:
            pos = [0]
        elif op[0] == L.PLAN_AND:
            i, flat = 1, True
            for _ in range(int(rec[0, 1])):
                if op[i] == L.PLAN_NOT and i + 1 < n and op[i + 1] in (L.PLAN_LINK, L.PLAN_TEMPLATE):
                    neg.append(i + 1)
                    i += 2
                elif op[i] in (L.PLAN_LINK, L.PLAN_CONST, L.PLAN_TEMPLATE):
                    pos.append(i)
                    i += 1
                else:
                    flat = False
                    break
            flat = flat and i == n
        single = op[0] == L.PLAN_LINK and not rec[0, 3]
        if op[0] == L.PLAN_LINK and not single:
            return None                                  # one '*'-type / repeated-variable Link: host fold
        st = {"expr": expr, "answer": answer, "db": db, "ctx": db.ctx, "nodes": nodes, "n": n, "rec": rec,
              "op": op, "leaves": leaves, "pos": pos, "neg": neg, "flat": flat, "single": single,
              "no_overload": no_overload, "top": expr is self._top or id(expr) in self._tops,
              "gathered": [], "local": []}
        st["leaves_sized"] = not single and bool(leaves)
        if single:
            st["local"] = [0]
        return st

    def _plan_sizes(self, sts):
        """Phase 2: (G, M) per leaf of every plan -- its rows over all shards and
        on the largest one.  Exact from the estimate exchange (one all-gather
        of every shard's das_plan_estimates, with its das_plan_bounds riding
        along, for every plan at once), or -- when every leaf of a plan was
        seen before -- from the caches that exchange fills: a leaf's exact
        sizes by its words (a term that repeats, e.g. FlyBase's unanchored
        E(rec, V2, V1)), else its shape's upper bounds (a fresh anchor of a
        known shape); then the plan needs no exchange.  Bounds only raise
        gather slot sizes and split decisions, never the answer.  The caches
        fill from collective results, so every shard holds the same."""
        if not sts:
            return
        db = sts[0]["db"]
        if self._size_gen != db.generation:
            self._size_gen = db.generation
            self._exact_sizes, self._shape_sizes = {}, {}
        small = int(os.environ.get("DAS_SHARD_SMALL", self.SMALL))
        miss = []
        for st in sts:
            rec, leaves = st["rec"], st["leaves"]
            st["keys"] = [rec[i].tobytes() for i in leaves]
            st["skeys"] = [self._shape_key(rec[i]) for i in leaves]
            G, M = {}, {}
            hit_all = os.environ.get("DAS_SHARD_SIZE_CACHE") != "0"
            if hit_all:
                for i, k, sk in zip(leaves, st["keys"], st["skeys"]):
                    hit = self._exact_sizes.get(k)
                    if hit is None:
                        # a shape bound only where it settles the leaf as small
                        # (gathered); a large bound (a hub key somewhere) needs
                        # the exact sizes for the split decision
                        hit = self._shape_sizes.get(sk)
                        if hit is not None and hit[0] > small:
                            hit = None
                    if hit is None:
                        hit_all = False
                        break
                    G[i], M[i] = hit
            st["G"], st["M"] = G, M
            if hit_all:
                self.plan_stats["size_cache"] += 1
            else:
                miss.append(st)
        if not miss:
            return
        parts = []
        for st in miss:
            ctx, nodes, n, leaves = st["ctx"], st["nodes"], st["n"], st["leaves"]
            b = ctx.plan_bounds(nodes, n)[leaves]
            parts.append(np.concatenate([ctx.plan_estimates(nodes, n)[leaves].astype(np.int64),
                                         np.where(b == np.uint64(2 ** 64 - 1), -1, b.astype(np.int64))]))
        got = self._allgather_i64(np.concatenate(parts))
        if len(self._exact_sizes) > self.SIZE_CACHE:
            self._exact_sizes.clear()
        if len(self._shape_sizes) > self.SIZE_CACHE:
            self._shape_sizes.clear()
        o = 0
        for st in miss:
            nl = len(st["leaves"])
            est, bnd = got[:, o:o + nl], got[:, o + nl:o + 2 * nl]
            o += 2 * nl
            for j, i in enumerate(st["leaves"]):
                st["G"][i], st["M"][i] = int(est[:, j].sum()), int(est[:, j].max())
                self._exact_sizes[st["keys"][j]] = (st["G"][i], st["M"][i])
                if (bnd[:, j] >= 0).all():
                    self._shape_sizes[st["skeys"][j]] = (int(bnd[:, j].sum()), int(bnd[:, j].max()))

    def _plan_place(self, st):
        """Phase 3 (local, from the sizes): which terms stay split, which are
        gathered, and the owner of a wholly gathered top-level plan; False
        when the plan does not apply (every shard decides alike)."""
        from . import _lib as L
        rec, op, leaves, pos = st["rec"], st["op"], st["leaves"], st["pos"]
        db, ctx = st["db"], st["ctx"]
        if not st["single"] and leaves:
            G = st["G"]
            local = []
            if st["flat"]:
                small = int(os.environ.get("DAS_SHARD_SMALL", self.SMALL))
                # split candidates: Links whose rows are distinct across shards
                big = [i for i in pos if op[i] == L.PLAN_LINK and not rec[i, 3] and G[i] > small]
                if len(big) > 1:
                    # several large terms: all stay split when partition_spec
                    # places them by one variable (co-located joins), else the
                    # largest does and the others are gathered -- unless
                    # gathering them would move more than the budget's bytes:
                    # then the operator-by-operator fold joins them where they
                    # are, placing each join by cost (broadcast of a small side,
                    # or the all-to-all exchange by the shared variables with
                    # the heavy-hitter split, _join_shared)
                    pv = {self._placement_var(db, rec[i]) for i in big}
                    if len(pv) == 1 and None not in pv:
                        local = big
                    else:
                        top = max(big, key=lambda i: G[i])
                        moved = sum(4 * int(rec[i, L.PLAN_SCAN]) * G[i] * (self.world - 1) for i in big if i != top)
                        if moved > int(os.environ.get("DAS_SHARD_GATHER_BUDGET", self.GATHER_BUDGET)):
                            self.plan_stats["split_fold"] = self.plan_stats.get("split_fold", 0) + 1
                            return False
                        local = [top]
                else:
                    local = big
            gathered = [i for i in leaves if i not in local]
            if sum(G[i] for i in gathered) > self.GATHER_LIMIT:
                return False
            st["local"], st["gathered"] = local, gathered
        # a wholly gathered top-level expression is evaluated by ONE shard
        # (round robin over such plans, the same on every shard): its inputs
        # go to that shard only, the others skip the native call and take
        # the answer's size, flags and table schemas from the all-reduce
        st["owner"] = None
        if not st["local"] and st["top"] and self.world > 1 and os.environ.get("DAS_GATHERED_OWNER") != "0":
            st["owner"] = self._gather_seq % self.world
            self._gather_seq += 1
        # gathered terms: this shard's rows, all-gathered into every shard --
        # or sent to the owner only; a term whose rows may repeat ('*' type,
        # repeated variable) is deduplicated after
        st["tables"] = [ctx.scan_words(st["nodes"], i) for i in st["gathered"]]
        st["caps"] = [st["M"][i] for i in st["gathered"]]
        st["inputs"] = []
        return True

    def _plan_gather(self, sts):
        """Phase 4: every plan's gathered terms in ONE all-to-all: a plan's
        block (per table a header of row count and column bounds, then its
        rows in a slot of its largest estimate, row-major) goes to every shard,
        or to its owner only.  A table with more rows than its slot (an
        estimate below the rows) is sent as the count OVER with no rows: the
        receivers' plan falls back -- on every shard alike for an all-gathered
        plan; an owner's plan carries the fallback in its all-reduce."""
        if not sts:
            return
        import torch
        loc = self.local
        gpu = loc.gpu
        lay = []                                  # per plan: (H, offsets, width) of its block
        for st in sts:
            tables = st["tables"]
            H = sum(1 + 2 * len(t.vars) for t in tables)
            offs, off = [], H
            for c, t in zip(st["caps"], tables):
                offs.append(off)
                off += int(c) * max(len(t.vars), 1)
            lay.append((H, offs, off))
        dests = [[d for d in range(self.world) if st["owner"] is None or st["owner"] == d] for st in sts]
        # the send buffer: for each destination, the blocks of the plans it
        # receives, in plan order (the same layout on every shard)
        send_sizes = [sum(lay[j][2] for j in range(len(sts)) if d in dests[j]) for d in range(self.world)]
        blk = torch.zeros(sum(send_sizes), dtype=torch.int32, device=gpu)
        base = {}
        o = 0
        for d in range(self.world):
            for j in range(len(sts)):
                if d in dests[j]:
                    base[(j, d)] = o
                    o += lay[j][2]
        if not loc.stream_ordered:
            torch.cuda.current_stream().synchronize()
        for j, st in enumerate(sts):
            H, offs, width = lay[j]
            hdr = []
            over = []
            for t, c in zip(st["tables"], st["caps"]):
                ov = t.nrows > int(c)
                over.append(ov)
                lo, hi = t.bounds()
                hdr += [self.OVER if ov else t.nrows] + list(lo) + list(hi)
            h = torch.from_numpy(np.array(hdr, dtype=np.uint32).view(np.int32)).to(gpu)
            # one shard's block, then copied to each further destination
            d0 = dests[j][0]
            b0 = base[(j, d0)]
            blk[b0:b0 + H] = h
            for t, tof, ov in zip(st["tables"], offs, over):
                if t.nrows and not ov:
                    loc.db.ctx.export_rows(t, blk.data_ptr() + 4 * (b0 + tof))
            if not loc.stream_ordered:
                loc.db.ctx.sync()
            for d in dests[j][1:]:
                bd = base[(j, d)]
                blk[bd:bd + width] = blk[b0:b0 + width]
        if not loc.stream_ordered:
            loc.db.ctx.sync()
        stage = blk if loc.dev == gpu else blk.cpu()
        mine = [j for j in range(len(sts)) if self.rank in dests[j]]
        per_src = sum(lay[j][2] for j in mine)
        out = torch.empty(self.world * per_src, dtype=torch.int32, device=stage.device)
        self.dist.all_to_all_single(out, stage, output_split_sizes=[per_src] * self.world,
                                    input_split_sizes=send_sizes, group=self.group)
        self.plan_stats["collectives"] += 1
        out_dev = out.to(gpu)
        # the headers of the blocks this shard received, in one copy to the host
        hcols, o = [], 0
        for j in mine:
            hcols += range(o, o + lay[j][0])
            o += lay[j][2]
        heads_all = (out.view(self.world, per_src)[:, torch.tensor(hcols, dtype=torch.long, device=out.device)]
                     .cpu().numpy().view(np.uint32)) if hcols else None
        if not loc.stream_ordered:
            torch.cuda.current_stream().synchronize()
        o = 0
        ho = 0
        for j in mine:
            st = sts[j]
            H, offs, width = lay[j]
            heads = heads_all[:, ho:ho + H]
            ho += H
            tables = st["tables"]
            cnt_cols = np.cumsum([0] + [1 + 2 * len(t.vars) for t in tables[:-1]])
            if (heads[:, cnt_cols] == self.OVER).any():
                self.plan_stats["gather_overflow"] = self.plan_stats.get("gather_overflow", 0) + 1
                st["inputs"] = None
                o += width
                continue
            result = []
            h = 0
            for t, tof in zip(tables, offs):
                k = len(t.vars)
                cnt = heads[:, h].astype(np.int64)
                lo = heads[:, h + 1:h + 1 + k]
                hi = heads[:, h + 1 + k:h + 1 + 2 * k]
                h += 1 + 2 * k
                parts = [loc.db.ctx.import_rows(t.kind, list(t.vars), out_dev.data_ptr() + 4 * (r * per_src + o + tof),
                                                int(cnt[r]), t.members) for r in range(self.world) if cnt[r]]
                g = parts[0] if len(parts) == 1 else (loc.db.ctx.concat(parts) if parts else
                                                      loc.db.ctx.import_rows(t.kind, list(t.vars), None, 0, t.members))
                has = cnt > 0
                if has.any() and k:
                    g.set_bounds(lo[has].min(axis=0), hi[has].max(axis=0))
                result.append(g)
            st["inputs"] = result
            o += width
        for j, st in enumerate(sts):
            if j not in mine:
                st["inputs"] = "elsewhere"
        if not loc.stream_ordered:
            loc.db.ctx.sync()
        del out_dev

    def _plan_evaluate(self, st):
        """Phase 5 (local): the native call where this shard evaluates the
        plan, and the vector this plan adds to the shared all-reduce (None
        when it needs none)."""
        from . import _lib as L
        ctx, rec, op, n = st["ctx"], st["rec"], st["op"], st["n"]
        st["vec"] = None
        inputs = st["inputs"]
        if inputs is not None and inputs != "elsewhere":
            inputs = [ctx.dedup(t) if rec[i, 3] and t.nrows else t for i, t in zip(st["gathered"], inputs)]
        words = st["nodes"].copy().reshape(n, L.PLAN_WORDS)
        for slot, i in enumerate(st["gathered"]):
            words[i, 0] = L.PLAN_INPUT
            words[i, 2] = slot
        words = words.reshape(-1)
        st["tables"] = None
        if st["owner"] is not None:
            # an owner-evaluated plan: the owner evaluates, every shard learns
            # the answer's size, flags and table schemas
            K, Wd = self.OWNER_TABLES, 2 + 2 * L_MAXCOLS
            vec = np.zeros(5 + K * Wd, dtype=np.int64)
            st["out"] = []
            if self.rank == st["owner"] and inputs is None:
                vec[4] = 1
            elif self.rank == st["owner"]:
                matched, negation, out, _ = ctx.plan_execute_sharded(words, n, inputs, st["no_overload"])
                vec[0] = sum(t.nrows for t in out)
                vec[1], vec[2], vec[3] = int(matched), int(negation), len(out)
                self._describe(out[:K], vec[5:])
                st["out"] = out
            st["vec"] = vec
            return
        if inputs is None:
            st["fallback"] = True                        # an estimate below the rows: the operator fold
            return
        matched, negation, out, checks = ctx.plan_execute_sharded(words, n, inputs, st["no_overload"])
        st["matched"], st["negation"], st["out"], st["checks"] = matched, negation, out, checks
        if st["local"]:
            # the tested running results must hold rows on some shard: after
            # each positive term from the first split one up to (not
            # including) the last, whose emptiness is just the answer's
            single, pos = st["single"], st["pos"]
            first = min(pos.index(i) for i in st["local"]) if not single else 0
            need = list(range(first, len(checks) - 1)) if not single else []
            # one ordered table per shard, the And's schema (sorted variable
            # ids of its positive terms), even where this shard has no rows:
            # later collectives over the relation pair tables up by position
            s0 = L.PLAN_SCAN
            vars_ = sorted({int(np.int32(rec[i, s0 + 10 + p])) for i in (pos if not single else [0])
                            if op[i] == L.PLAN_LINK for p in range(int(rec[i, s0]))
                            if int(np.int32(rec[i, s0 + 10 + p])) >= 0})
            out = [t for t in out if t.nrows]
            bad = int(len(out) > 1 or any(t.kind != L.TABLE_ORDERED or list(t.vars) != vars_ for t in out))
            if not out:
                out = [self.local.empty_table(L.TABLE_ORDERED, vars_)]
            st["out"] = out
            st["vec"] = np.array([sum(t.nrows for t in out), bad] + [int(checks[j]) for j in need], dtype=np.int64)

    def _plan_finish(self, st):
        """Phase 6: the answer from the shared all-reduce (or, for a plan every
        shard evaluated whole, shard 0's tables); None = fall back."""
        from . import _lib as L
        answer = st["answer"]
        if st.get("fallback"):
            return None
        if st["owner"] is not None:
            got, owner = st["got"], st["owner"]
            if int(got[4]):
                self.plan_stats["native_fallback"] += 1
                return None
            K, Wd = self.OWNER_TABLES, 2 + 2 * L_MAXCOLS
            out = st["out"]
            nt = int(got[3])
            if nt > K:
                # more schemas than the vector describes: a second all-reduce with all of them
                big = np.zeros(nt * Wd, dtype=np.int64)
                if self.rank == owner:
                    self._describe(out, big)
                big = self._allreduce_sum(big)
                if self.rank != owner:
                    out = self._schemas(big, nt)
            elif self.rank != owner:
                out = self._schemas(got[5:], nt)
            rel = DRel(out)
            rel._global = int(got[0])
            self.plan_stats["native"] += 1
            answer._set(self, rel)
            answer.negation = bool(got[2])
            return bool(got[1])
        matched, negation, out = st["matched"], st["negation"], st["out"]
        if not st["local"]:
            # every shard holds the whole answer: shard 0 keeps it
            total = sum(t.nrows for t in out)
            if self.rank != 0:
                out = [self.local.empty_table(t.kind, list(t.vars), t.members) for t in out]
            rel = DRel(out)
            rel._global = total
        else:
            got = st["got"]
            if int(got[1]) or any(int(x) == 0 for x in got[2:]):
                self.plan_stats["native_fallback"] += 1
                return None
            rel = DRel(out)
            rel._global = int(got[0])
            if matched:
                matched = rel._global > 0
        self.plan_stats["native"] += 1
        answer._set(self, rel)
        answer.negation = negation
        return matched

    SIZE_CACHE = 1 << 12                    # leaf sizes kept per kind

    @staticmethod
    def _shape_key(words):
        """A leaf record with its grounded targets masked (scan and index-join
        target words, include/das_mi355x.h das_plan_node_t): its query shape."""
        from . import _lib as L
        w = np.array(words, dtype=np.uint32)
        for base in (L.PLAN_SCAN, 28):
            t = w[base + 2:base + 10]
            t[t != np.uint32(L.DAS_NONE)] = 0xFFFFFFFE
        return w.tobytes()

    OWNER_TABLES = 16                       # answer tables an owner-evaluated plan describes

    @staticmethod
    def _describe(tables, v):
        """An owner-evaluated answer's table schemas into its all-reduce
        vector: kind, variables, composite members per table."""
        W = 2 + 2 * L_MAXCOLS
        for i, t in enumerate(tables):
            d = v[i * W:(i + 1) * W]
            d[0], d[1] = int(t.kind), len(t.vars)
            d[2:2 + len(t.vars)] = [int(x) + 1 for x in t.vars]          # +1: 0 = unused
            mem = list(t.members) if t.members is not None else []
            d[2 + L_MAXCOLS:2 + L_MAXCOLS + len(mem)] = [int(x) + 2 for x in mem]

    def _schemas(self, v, nt):
        """Empty tables of the schemas an owner described."""
        from . import _lib as L
        W = 2 + 2 * L_MAXCOLS
        res = []
        for i in range(nt):
            d = v[i * W:(i + 1) * W]
            kind, nv = int(d[0]), int(d[1])
            vars_ = [int(x) - 1 for x in d[2:2 + nv]]
            mem = [int(x) - 2 for x in d[2 + L_MAXCOLS:2 + L_MAXCOLS + nv]] if kind == L.TABLE_COMPOSITE else None
            res.append(self.local.empty_table(kind, vars_, mem))
        return res

    def _placement_var(self, db, words):
        """The variable that places this Link term's rows (partition_spec:
        links of its type live on the owner of the atom at a position), or None."""
        from . import _lib as L
        s0 = L.PLAN_SCAN
        tid = int(words[s0 + 1])
        name = next((t for t, i in db.type_id.items() if i == tid), None)
        p = self.spec.get(name)
        if p is None or p >= int(words[s0]):
            return None
        v = int(np.int32(words[s0 + 10 + p]))
        return v if v >= 0 else None

    def get_link_type(self, link_handle):
        return self.local.get_link_type(link_handle)

    def get_node_type(self, node_handle):
        return self.local.get_node_type(node_handle)

    def get_atom_as_dict(self, handle, arity=-1):
        return self.local.get_atom_as_dict(handle, arity)

    def get_atom_as_deep_representation(self, handle, arity=-1):
        return self.local.get_atom_as_deep_representation(handle, arity)

    OVER = 0xFFFFFFFF                     # _plan_gather header: rows over the slot

    # ------------------------------------------------------- relation algebra
    def rel_empty(self):
        return DRel([])

    def _global_rows(self, rel):
        if rel._global is None:
            rel._global = int(self._allreduce_sum([sum(t.nrows for t in rel.tables)])[0])
        return rel._global

    def rel_nonempty(self, rel):
        return self._global_rows(rel) > 0

    def rel_count(self, rel):
        return self._global_rows(rel)

    def rel_local_count(self, rel):
        return sum(t.nrows for t in rel.tables)

    def rel_local_tables(self, rel):
        return [self._gather_all(t) for t in rel.tables]

    def _group(self, tables):
        g = {}
        for t in tables:
            g.setdefault((t.kind, tuple(t.vars), _members(t)), []).append(t)
        return g

    def rel_normalize(self, rel):
        if any(t.kind == COMPOSITE for t in rel.tables):
            # composite identities cross schemas (XOR, :279-286): replicate,
            # dedup identically on every rank, keep this rank's share
            merged = [ts[0] if len(ts) == 1 else self.local.concat(ts) for ts in self._group(rel.tables).values()]
            full = [self._gather_all(t) for t in merged]
            return DRel([self._rank_slice(t) for t in self.local.set_dedup(full)])
        out = []
        for _, ts in self._group(rel.tables).items():
            if len(ts) == 1:
                out.append(ts[0])
            else:
                out.append(self.local.dedup(self._exchange(self.local.concat(ts), [])))
        return DRel(out)

    def rel_union(self, a, b):
        return self.rel_normalize(DRel(a.tables + b.tables))

    def rel_join(self, a, b):
        from .pattern_matcher.pattern_matcher import CONFIG
        out = []
        for ta in a.tables:
            for tb in b.tables:
                if ta.kind != ORDERED or tb.kind != ORDERED:
                    # CompositeAssignment algebra: no equality key in general;
                    # replicate the smaller side, keep the operand order
                    na, nb = (int(x) for x in self._allreduce_sum([ta.nrows, tb.nrows]))
                    if na and nb and _join_raises(ta, tb):
                        raise AttributeError("'NoneType' object has no attribute 'frozen'")
                    if na <= nb:
                        out.append(self.local.join(self._gather_all(ta), tb, CONFIG['no_overload']))
                    else:
                        out.append(self.local.join(ta, self._gather_all(tb), CONFIG['no_overload']))
                    continue
                shared = sorted(set(ta.vars) & set(tb.vars))
                if shared:
                    out.append(self._join_shared(ta, tb, shared, CONFIG['no_overload']))
                else:
                    na = self._allreduce_sum([ta.nrows])[0]
                    nb = self._allreduce_sum([tb.nrows])[0]
                    if na <= nb:
                        out.append(self.local.join(self._gather_all(ta), tb, CONFIG['no_overload']))
                    else:
                        out.append(self.local.join(ta, self._gather_all(tb), CONFIG['no_overload']))
        return DRel(out)

    def _join_shared(self, ta, tb, shared, no_overload):
        """Ordered equi-join on `shared`, placed by cost:
        * both sides partitioned by the same atom variable in `shared`
          (partition_spec) or by the same hash key: join where the rows are;
        * one side small (its rows x world < both sides' rows): replicate it
          to every rank, leave the large side in place (SURVEY §8e's
          broadcast of heavy / small relations);
        * otherwise repartition both by hash(shared) (all-to-all)."""
        pa, pb = _part(ta), _part(tb)
        if not self.force and pa is not None and pa == pb and ((pa[0] == "atom" and pa[1] in shared) or
                                            (pa[0] == "hash" and set(pa[1]) <= set(shared))):
            self.plan_stats["colocated"] += 1
            return _with_part(self.local.join(ta, tb, no_overload), pa)
        wa, wb = (int(x) for x in self._allreduce_sum([ta.nrows * max(len(ta.vars), 1),
                                                       tb.nrows * max(len(tb.vars), 1)]))
        if self.force == "broadcast" or (not self.force and min(wa, wb) * self.world < wa + wb):
            self.plan_stats["broadcast"] += 1
            if wa <= wb:
                return _with_part(self.local.join(self._gather_all(ta), tb, no_overload), pb)
            return _with_part(self.local.join(ta, self._gather_all(tb), no_overload), pa)
        key = tuple(shared)
        self.plan_stats["exchange"] += 1
        skewed = self._join_skewed(ta, tb, shared, no_overload)
        if skewed is not None:
            return skewed
        return _with_part(self.local.join(self._exchange(ta, shared), self._exchange(tb, shared), no_overload),
                          ("hash", key))

    HEAVY_BUCKETS = 4096

    def _join_skewed(self, ta, tb, shared, no_overload):
        """Heavy-hitter handling of an exchanged join (SURVEY §8e, config 5's
        hub keys): both sides are bucketed by hash(shared) and the global
        bucket histogram is all-reduced.  A bucket holding more than
        heavy_frac x (join rows / world) is heavy: hashing it would send all
        its rows to one rank.  In a heavy bucket the side with more rows stays
        where it is (split across ranks) and the other side is all-gathered
        to every rank; light buckets take the usual all-to-all.  Returns None
        when no bucket is heavy."""
        nb = self.HEAVY_BUCKETS
        pa, ca = self.local.partition(ta, list(shared), nb)
        pb, cb = self.local.partition(tb, list(shared), nb)
        g = self._allreduce_sum(np.concatenate([ca.astype(np.int64), cb.astype(np.int64)]))
        ga, gb = g[:nb], g[nb:]
        load = ga + gb
        fair = max(load.sum() / self.world, 1)
        heavy = (load > self.heavy_frac * fair) & (ga > 0) & (gb > 0)
        offa = np.concatenate([[0], np.cumsum(ca.astype(np.int64))])
        offb = np.concatenate([[0], np.cumsum(cb.astype(np.int64))])
        if not heavy.any():
            if nb % self.world:
                return None
            # no heavy bucket: the usual exchange, from these bucket runs (the
            # partition hash is the exchange's: bucket b goes to rank b % world)
            # instead of partitioning both sides again
            key = tuple(shared)

            def grouped(t, p, c, off):
                ks = [np.arange(d, nb, self.world) for d in range(self.world)]
                counts = np.array([int(c[k].astype(np.int64).sum()) for k in ks], dtype=np.int64)
                order = np.concatenate(ks)
                keep = off[order + 1] > off[order]
                rows = self.local.gather_ranges(p, off[order][keep], off[order + 1][keep])
                return _with_part(self._send_grouped(t, rows, counts), ("hash", key))
            return _with_part(self.local.join(grouped(ta, pa, ca, offa), grouped(tb, pb, cb, offb), no_overload),
                              ("hash", key))
        self.plan_stats["heavy"] += 1
        a_stays = heavy & (ga >= gb)                      # a split in place, b gathered
        b_stays = heavy & ~a_stays

        def rows(t, off, mask):
            # the rows of the selected buckets (runs of the partitioned
            # table), gathered on the device from their row ranges
            ks = np.nonzero(mask)[0]
            keep = off[ks + 1] > off[ks]
            return self.local.gather_ranges(t, off[ks][keep], off[ks + 1][keep])
        light = ~heavy
        a_light, b_light = rows(pa, offa, light), rows(pb, offb, light)
        out = [self.local.join(self._exchange(a_light, shared), self._exchange(b_light, shared), no_overload),
               self.local.join(rows(pa, offa, a_stays), self._gather_all(rows(pb, offb, a_stays)), no_overload),
               self.local.join(self._gather_all(rows(pa, offa, b_stays)), rows(pb, offb, b_stays), no_overload)]
        out = [t for t in out if t.nrows]
        if not out:
            none = np.zeros(nb, dtype=bool)
            return self.local.join(rows(pa, offa, none), rows(pb, offb, none), no_overload)
        return _with_part(out[0] if len(out) == 1 else self.local.concat(out), None)

    def rel_antijoin(self, rel, forbidden):
        tables = rel.tables
        for f in forbidden.tables:
            nxt = []
            for t in tables:
                if t.kind != ORDERED or f.kind != ORDERED:
                    nt, nf = (int(x) for x in self._allreduce_sum([t.nrows, f.nrows]))
                    if nt and nf and _antijoin_raises(t, f):
                        raise AttributeError("'CompositeAssignment' object has no attribute "
                                             + ("'is_covered_by_ordered'" if t.kind == ORDERED
                                                else "'unordered_assignments'"))
                    nxt.append(self.local.antijoin(t, self._gather_all(f)) if nf else t)
                    continue
                if set(f.vars) <= set(t.vars):
                    key = sorted(f.vars)
                    wt, wf = (int(x) for x in self._allreduce_sum([t.nrows * max(len(t.vars), 1),
                                                                   f.nrows * max(len(f.vars), 1)]))
                    if self.force != "exchange" and wf * self.world < wt + wf:   # small forbidden set: replicate it
                        nxt.append(_with_part(self.local.antijoin(t, self._gather_all(f)), _part(t)))
                    else:
                        nxt.append(_with_part(self.local.antijoin(self._exchange(t, key), self._exchange(f, key)),
                                              ("hash", tuple(key))))
                else:
                    nxt.append(t)
            tables = nxt
        return DRel(tables)

    def rel_minus(self, a, b):
        if any(t.kind == COMPOSITE for t in a.tables + b.tables):
            if not a.tables or not b.tables:
                return DRel(a.tables)
            fa = [self._gather_all(t) for t in a.tables]
            fb = [self._gather_all(t) for t in b.tables]
            return DRel([self._rank_slice(t) for t in self.local.set_minus(fa, fb)])
        groups = self._group(b.tables)
        out = []
        for t in a.tables:
            fs = groups.get((t.kind, tuple(t.vars), _members(t)), [])
            if fs:
                t = self._exchange(t, [])
                for f in fs:
                    t = self.local.antijoin(t, self._exchange(f, []))
            out.append(t)
        return DRel(out)


# ---------------------------------------------------------------------------
# The GPU local engine surface ShardedDB needs (HipDB + torch buffers)
# ---------------------------------------------------------------------------
class HipLocal:
    """Adapts a HipDB for ShardedDB: device tables, torch CUDA staging buffers
    for the RCCL collectives."""

    def __init__(self, db, cpu_staging=False):
        """cpu_staging: collective buffers on the host (gloo backend; used to
        rehearse several ranks on one GPU).  Default: device buffers (RCCL).
        When the context runs on torch's current stream (HipDB's default),
        staging copies and collectives are ordered by the stream itself: no
        host synchronisation around them."""
        import torch
        self.db = db
        self.torch = torch
        self.gpu = torch.device("cuda", torch.cuda.current_device())
        self.dev = torch.device("cpu") if cpu_staging else self.gpu
        self.tuple_targets = db.tuple_targets
        # (the null stream does not count: the context then runs on a stream
        # of its own)
        self.stream_ordered = (not cpu_staging and bool(db.stream) and
                               db.stream == torch.cuda.current_stream().cuda_stream)

    @property
    def pattern_black_list(self):
        """The local index's load-time pattern black list (HipDB.load_arrays)."""
        return self.db.pattern_black_list

    @pattern_black_list.setter
    def pattern_black_list(self, value):
        self.db.pattern_black_list = list(value)

    def __getattr__(self, name):     # DBInterface passthrough
        return getattr(self.db, name)

    def rel_local_tables(self, rel):
        return rel.tables

    def empty_table(self, kind, vars_, members=None):
        return self.db.ctx.import_rows(kind, vars_, None, 0, members)

    def partition(self, t, key_vars, nparts):
        return self.db.ctx.partition(t, key_vars, nparts)

    def dedup(self, t):
        return self.db.ctx.dedup(t)

    def concat(self, ts):
        return self.db.ctx.concat(ts)

    def join(self, a, b, no_overload):
        return self.db.ctx.join(a, b, no_overload)

    def antijoin(self, a, t):
        return self.db.ctx.antijoin(a, t)

    def set_dedup(self, ts):
        return self.db.ctx.set_dedup(ts)

    def set_minus(self, a, b):
        return self.db.ctx.set_minus(a, b)

    def slice(self, t, lo, hi):
        return self.db.ctx.gather_ranges(t, [lo], [hi])

    def gather_rows(self, t, idx):
        return self.db.ctx.gather(t, idx)

    def gather_ranges(self, t, begin, end):
        return self.db.ctx.gather_ranges(t, begin, end)

    def xfer_tensor(self, arr):
        return self.torch.from_numpy(np.ascontiguousarray(arr)).to(self.dev)

    def xfer_numpy(self, t):
        return t.cpu().numpy()

    def rows_buffer(self, n, ncols):
        return self.torch.empty((max(n, 0), max(ncols, 1)), dtype=self.torch.int32, device=self.dev)

    def rows_out(self, t):
        buf = self.torch.empty((t.nrows, max(len(t.vars), 1)), dtype=self.torch.int32, device=self.gpu)
        if self.stream_ordered:
            # one stream: the allocation, the export and the collective that
            # reads the buffer are ordered without the host
            if t.nrows:
                self.db.ctx.export_rows(t, buf.data_ptr())
            return buf
        # torch's allocation must be ready before the ctx stream writes it, and
        # the ctx stream (its own, when torch runs on the null stream) must be
        # done before torch / the collective reads it
        self.torch.cuda.current_stream().synchronize()
        if t.nrows:
            self.db.ctx.export_rows(t, buf.data_ptr())
        self.db.ctx.sync()
        return buf if self.dev == self.gpu else buf.cpu()

    def rows_pad(self, buf, width, ncols):
        if buf.shape[0] == width:
            return buf
        out = self.rows_buffer(width, ncols)
        out[:buf.shape[0]] = buf
        return out

    def rows_in(self, kind, vars_, buf, n, members=None):
        buf = buf.to(self.gpu).contiguous()
        if self.stream_ordered:
            # the import kernel follows the collective on the stream; torch's
            # caching allocator does not reuse `buf` before work queued on the
            # stream that uses it has run
            return self.db.ctx.import_rows(kind, list(vars_), buf.data_ptr() if n else None, n, members)
        self.torch.cuda.current_stream().synchronize()     # copy / collective landed
        t = self.db.ctx.import_rows(kind, list(vars_), buf.data_ptr() if n else None, n, members)
        self.db.ctx.sync()                                  # before `buf` can be freed / reused
        return t

    def rows_in_many(self, kind, vars_, bufs, counts, members=None):
        parts = [b[:c] for b, c in zip(bufs, counts)]
        cat = self.torch.cat(parts) if parts else self.rows_buffer(0, len(vars_))
        return self.rows_in(kind, vars_, cat, int(sum(counts)), members)


class ShardedMatcher:
    """bench.py helper: evaluates one expression on the sharded DB and returns
    the number of distinct bindings held by this rank (sum over ranks = the
    answer's size)."""

    def __init__(self, db, dist, cpu_staging=False, partition_spec=None):
        self.sdb = ShardedDB(HipLocal(db, cpu_staging), dist, partition_spec=partition_spec)

    def count(self, expr):
        from .pattern_matcher.pattern_matcher import PatternMatchingAnswer
        ans = PatternMatchingAnswer()
        self.sdb._top = expr
        try:
            expr.matched(self.sdb, ans)
        finally:
            self.sdb._top = None
        return self.sdb.rel_local_count(ans._relation()) if ans._rel is not None else 0

    def count_many(self, exprs):
        """count() of a step's independent expressions, their sharded plans
        sharing one estimate exchange, one gather and one outcome all-reduce
        (ShardedDB.plan_many); an expression whose plan falls back is then
        folded operator by operator, on every shard alike."""
        from .pattern_matcher.pattern_matcher import PatternMatchingAnswer
        sdb = self.sdb
        answers = [PatternMatchingAnswer() for _ in exprs]
        sdb._tops = {id(e) for e in exprs}
        try:
            res = sdb.plan_many(list(zip(exprs, answers)))
        finally:
            sdb._tops = set()
        out = []
        for e, a, r in zip(exprs, answers, res):
            if r is None:
                sdb._no_plan = {id(e)}
                sdb._top = e
                try:
                    a = PatternMatchingAnswer()
                    e.matched(sdb, a)
                finally:
                    sdb._no_plan = set()
                    sdb._top = None
            out.append(sdb.rel_local_count(a._relation()) if a._rel is not None else 0)
        return out


# ---------------------------------------------------------------------------
# Sharded synthetic KB for the benchmark (every rank builds the directory of
# the whole KB; index rows only for the links it owns)
# ---------------------------------------------------------------------------

def handle_owner(handle, world):
    """Shard that owns a handle (links hash-partitioned by handle, SURVEY.md
    §8e): int(handle[:8], 16) % world -- das_amd/csrc/common.h handle_owner."""
    return int(handle[:8], 16) % world if world > 1 else 0


def host_owners(arrays, world, exprs=None):
    """Owner shard of expressions' handles, hashed on the host (hashlib md5,
    expression_hasher.py:9-35): the restatement of das_hash_owners for small
    KBs and the CPU tests.  exprs: the expression indices wanted (default all;
    their contained expressions are hashed too)."""
    import hashlib
    nl, ne = arrays.n_leaf, arrays.n_expr
    off = arrays.expr_off.astype(np.int64)
    child = arrays.expr_child.astype(np.int64)
    want = np.arange(ne) if exprs is None else np.asarray(exprs, dtype=np.int64)
    memo = {}

    def h(u):
        r = memo.get(u)
        if r is None:
            if u < nl:
                r = hashlib.md5(bytes(arrays.leaf_bytes[int(arrays.leaf_off[u]):int(arrays.leaf_off[u + 1])])).hexdigest()
            else:
                j = u - nl
                ch = [h(int(c)) for c in child[off[j]:off[j + 1]]]
                r = ch[0] if len(ch) == 1 else hashlib.md5(" ".join(ch).encode()).hexdigest()
            memo[u] = r
        return r
    return np.array([handle_owner(h(nl + int(j)), world) for j in want], dtype=np.int64)


def bio_shard(n_genes, n_bps, n_members, n_inh, rank, world, seed=20250209):
    """Weak scaling of the gene-level KB (synthetic.bio_full_kb's layouts):
    rank r owns the Member links of its own n_genes genes (gene range
    r*n_genes.., placed by gene: partition_spec {"Member": 0}); Inheritance
    and the annotation layouts (Uniprot / Reactome Member, List, Evaluation,
    Context) are the same on every rank and indexed by their handle's owner.
    Every rank's Member block is drawn from the same random stream as
    bio_full_kb's (shifted by r*n_genes), so at world 1 the KB IS
    bio_full_kb(n_genes, n_bps, n_members, n_inh) and rank r's genes answer
    the anchored queries exactly as the 1-GPU KB's genes do (bench.py's
    per-rank QUERY_1-3 instances: equal work per rank).
    Returns (AtomArrays for this rank, this rank's gene ids)."""
    from . import synthetic
    total_genes = n_genes * world
    nodes, off = synthetic.bio_nodes(total_genes, n_bps)
    blocks = []
    rest_rng = None
    for r in range(world):
        rng = np.random.default_rng(seed)
        genes = r * n_genes + rng.integers(0, n_genes, n_members)
        bps = synthetic.zipf_indices(rng, n_bps, n_members)
        if rest_rng is None:
            rest_rng = rng                    # bio_full_kb's stream continues with Inheritance
        blocks.append(("Member", np.stack([off["g"] + genes, off["bp"] + bps], 1),
                       np.full(n_members, 1 if r == rank or world == 1 else 3, np.uint8)))
    rng = rest_rng
    child = rng.integers(1, n_bps, n_inh)
    parent = (rng.random(n_inh) * child).astype(np.int64)
    BY_HANDLE = 4                        # placeholder kind: owner decided from the handle below
    rest = [("Inheritance", np.stack([off["bp"] + child, off["bp"] + parent], 1))]
    rest += synthetic.bio_annotation_blocks(rng, off, n_bps, base=len(blocks) + 1)
    blocks += [(t, ch, np.full(len(ch), BY_HANDLE, np.uint8)) for t, ch in rest]
    arrays = synthetic.build_nested(synthetic.BIO_TYPES, nodes, blocks)
    kinds = arrays.expr_kind.copy()
    idx = np.nonzero(kinds == BY_HANDLE)[0]
    kinds[idx] = 1
    if world > 1:
        kinds[idx[host_owners(arrays, world, idx) != rank]] = 3
    arrays.expr_kind = kinds
    return arrays, np.arange(rank * n_genes, (rank + 1) * n_genes)


def shard_arrays(arrays, rank, world):
    """Query layout of a fixed KB over `world` GPUs (strong scaling): every
    rank loads the whole KB as its atom directory (ids agree across ranks) and
    indexes only the links whose handle it owns (handle_owner); the build does
    the split (das_build_index_sharded), so every copy of one handle --
    repeated expressions, nested children -- lands on one rank."""
    arrays.shard = (rank, world) if world > 1 else None
    return arrays


def partition_arrays(arrays, rank, world, owners=None):
    """Independent shards for the bulk build (config 4 at N GPUs, host-side
    input): rank r indexes only the links whose handle it owns (handle_owner;
    `owners` = per-expression owner if already known, else hashed on the
    host), keeps the expressions those links contain so their handles hash,
    and every leaf.  A contained link owned by another rank stays
    directory-only (kind 3): each link is indexed on exactly one rank.  Atom
    ids are then local to the shard (the reference's sharded Redis keys, not
    the replicated directory ShardedDB queries need)."""
    from .loader import AtomArrays
    if world == 1:
        return arrays
    nl, ne = arrays.n_leaf, arrays.n_expr
    off = arrays.expr_off.astype(np.int64)
    child = arrays.expr_child.astype(np.int64)
    keep = np.zeros(ne, dtype=bool)
    groups = [(int(arrays.level_off[g]), int(arrays.level_off[g + 1])) for g in range(len(arrays.level_off) - 1)]
    own = (host_owners(arrays, world) if owners is None else np.asarray(owners)) == rank
    for b, e in groups:
        if e <= b:
            continue
        keep[b:e] = own[b:e] & (arrays.expr_kind[b:e] == 1)
    for b, e in reversed(groups):          # parents before children: close over nesting
        if e <= b:
            continue
        k = int(off[b + 1] - off[b])
        ch = child[off[b]:off[e]].reshape(e - b, k)[keep[b:e]]
        sub = ch[ch >= nl] - nl
        keep[sub] = True
    kinds = arrays.expr_kind.copy()
    kinds[(kinds == 1) & ~own] = 3
    newpos = np.cumsum(keep) - 1
    nch = np.diff(off)[keep]
    expr_off = np.zeros(int(keep.sum()) + 1, dtype=np.uint64)
    np.cumsum(nch, out=expr_off[1:])
    parts = []
    for b, e in groups:
        if e <= b:
            continue
        k = int(off[b + 1] - off[b])
        parts.append(child[off[b]:off[e]].reshape(e - b, k)[keep[b:e]].reshape(-1))
    ch = np.concatenate(parts) if parts else np.zeros(0, np.int64)
    ch = np.where(ch >= nl, nl + newpos[np.maximum(ch - nl, 0)], ch)
    level_off = [0]
    for b, e in groups:
        level_off.append(level_off[-1] + int(keep[b:e].sum()))
    return AtomArrays(arrays.leaf_bytes, arrays.leaf_off, arrays.leaf_kind, arrays.leaf_ctype, arrays.leaf_type_id,
                      arrays.name_start, expr_off, ch.astype(np.uint32), kinds[keep],
                      arrays.expr_ctype_leaf[keep], np.array(level_off, dtype=np.uint64), arrays.type_names)


# ---------------------------------------------------------------------------
# Config 4 at N GPUs from device-generated ranges: links regrouped on the
# owners of their handles before the per-shard build
# ---------------------------------------------------------------------------

def regroup_by_owner(ctx, arrays, world, exchange):
    """`arrays`: this rank's generated range of a flat two-level KB
    (synthetic.device_arrays: arity-2 rows then arity-3 rows, node leaves
    only).  Every link's handle is hashed on the device (das_hash_owners), the
    rows are grouped by owner (das_partition_rows) and handed to
    `exchange(rows (n, K) int32 tensor, counts) -> received rows (m, K)`,
    the all-to-all (rccl_exchange below; tests pass an in-process stand-in).
    Returns the DeviceAtomArrays of the received rows: all owned here, so a
    plain build indexes each distinct link on exactly one rank.  Duplicates
    of one handle generated on several ranks all arrive at its owner and
    intern to one atom there."""
    import torch
    from . import synthetic
    ne = arrays.n_expr
    owner = torch.empty(max(ne, 1), dtype=torch.uint8, device=arrays.expr_child.device)
    ctx.hash_owners(arrays, world, owner)
    lv = [int(x) for x in arrays.level_off]
    assert len(lv) == 3, "regroup_by_owner: expected the arity-2 / arity-3 groups of a flat KB"
    c2, c3 = lv[1], lv[2] - lv[1]
    out = []
    for b, n, K, base in ((0, c2, 3, 0), (c2, c3, 4, 3 * c2)):
        rows = arrays.expr_child[base:base + n * K]
        grouped = torch.empty_like(rows)
        counts = ctx.partition_rows(rows, n, K, owner[b:b + n], world, grouped) if n else \
            np.zeros(world, dtype=np.uint64)
        out.append(exchange(grouped.reshape(-1, K), counts))
    leaves = (arrays.leaf_bytes, arrays.leaf_off, arrays.leaf_kind, arrays.leaf_ctype, arrays.leaf_type_id,
              arrays.name_start)
    return synthetic.device_arrays(leaves, arrays.type_names, out[0].reshape(-1), out[1].reshape(-1))


def rccl_exchange(dist, group=None, cpu_staging=False):
    """exchange() for regroup_by_owner over torch.distributed: split sizes
    first, then one all_to_all_single of the rows (RCCL over xGMI with device
    tensors; gloo with cpu_staging)."""
    import torch

    def ex(rows, counts):
        dev = rows.device
        stage = torch.device("cpu") if cpu_staging else dev
        sc = torch.from_numpy(counts.astype(np.int64)).to(stage)
        rc = torch.empty_like(sc)
        dist.all_to_all_single(rc, sc, group=group)
        rcl = [int(x) for x in rc.tolist()]
        recv = torch.empty((sum(rcl), rows.shape[1]), dtype=rows.dtype, device=stage)
        dist.all_to_all_single(recv, rows.to(stage), output_split_sizes=rcl,
                               input_split_sizes=[int(x) for x in counts], group=group)
        return recv.to(dev)
    return ex
