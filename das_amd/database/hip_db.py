"""HipDB — the DBInterface backed by the MI355X HBM index.

Drop-in for the reference's production adapter `RedisMongoDB`
(das/database/redis_mongo_db.py:49-335): the same methods, argument meaning,
return formats and exceptions, with the Redis pattern/template sets and the
Mongo collections replaced by the device index that `das_build_index` builds
(include/das_mi355x.h).  Method docstrings cite the reference method each one
replaces.

Two extra, non-reference entry points feed the pattern matcher without
materialising Python tuples: `match_link` and `match_template` return device
binding tables (`Relation`).
"""
import gc
import itertools
import os
import re
from typing import Any, List, Tuple

import numpy as np

from .. import _lib
try:
    from .. import _assign as _hex          # C handle formatting of large answers (csrc/pyassign.c)
except ImportError:                         # pragma: no cover - built with the library
    _hex = None
from .. import loader as _loader
from ..expression_hasher import ExpressionHasher
from .db_interface import UNORDERED_LINK_TYPES, WILDCARD, DBInterface

# one token per index load of any HipDB in the process: a lowered plan cached on
# an expression names the load it was lowered against (ids are per load)
_LOADS = itertools.count(1)


class Relation:
    """A set of assignments held on the GPU: device tables, one per schema
    (kind, variable ids).  Rows of one table are distinct."""

    __slots__ = ("tables", "_global")

    def __init__(self, tables=()):
        self.tables = [t for t in tables if t is not None and t.nrows > 0]
        self._global = None

    @property
    def nrows(self):
        return sum(t.nrows for t in self.tables)

    def __bool__(self):
        return self.nrows > 0

    def __len__(self):
        return self.nrows


class RelationalDB(DBInterface):
    """A DBInterface whose pattern-matcher entry points return device
    relations, plus the relation algebra the matcher folds them with."""

    tuple_targets = False

    def rel_empty(self):
        return Relation()

    def rel_nonempty(self, rel) -> bool:
        return bool(rel)

    def rel_count(self, rel) -> int:
        return rel.nrows

    def rel_local_tables(self, rel):
        return rel.tables

    def prefetch_handles(self, handles) -> None:
        """Resolves handles an expression is about to test, in one batch
        (no reference counterpart: RedisMongoDB.prefetch caches types only)."""


def _group(tables):
    g = {}
    for t in tables:
        g.setdefault(t.schema, []).append(t)
    return g


def _has_composite(tables):
    return any(t.kind == _lib.TABLE_COMPOSITE for t in tables)


def _reference_pattern_keys(type_hash, elements):
    """The `keys` list of canonical_parser.py:145-175 for one link, as
    (type hash or '*', element or '*', ...) tuples: [*, e...] for every
    arity, every mask with >= 1 wildcard for arities 1-3."""
    keys = [(WILDCARD, *elements)]
    a = len(elements)
    if 1 <= a <= 3:
        for mask in range(1, 1 << (a + 1)):
            keys.append(tuple([WILDCARD if mask & 1 else type_hash] +
                              [WILDCARD if mask >> (i + 1) & 1 else e for i, e in enumerate(elements)]))
    return keys


def _stale_entries(order, black_list):
    """The reference's stale pattern entries (canonical_parser.py:144-178):
    walking `order` (loader.canonical_pattern_order), a blacklisted link is
    written under the keys of the last link that was not -- {key: {handle:
    targets}} -- and one before any such link raises UnboundLocalError, as
    the reference's load does."""
    stale, keys = {}, None
    for h, t, elements in order:
        if t not in black_list:
            keys = _reference_pattern_keys(ExpressionHasher.named_type_hash(t), elements)
            continue
        if keys is None:
            raise UnboundLocalError("local variable 'keys' referenced before assignment")
        for k in keys:
            stale.setdefault(k, {})[h] = tuple(elements)
    return stale


class HipDB(RelationalDB):

    PREFETCH_MAX_ATOMS = 1 << 26            # host mirrors of prefetch() up to this many atoms
    HEX_DIRECT = 4096                       # hex_of: larger id arrays skip the per-id cache
    SEED_MAX = 1 << 16                      # _pairs: answers up to this size seed the handle cache

    def __init__(self, device: int = 0, stream=None, tuple_targets: bool = False,
                 stale_pattern_keys: bool = False):
        """`tuple_targets=True` reproduces the reference DB path exactly,
        including returning targets as tuples from get_matched_links, which
        makes `Link._assign_variables` raise AttributeError for unordered links
        with a grounded target.  The default returns lists (the
        semantics StubDB and service/README.md:356-363 show).

        `stale_pattern_keys=True` reproduces what the reference's canonical
        loader does with a non-empty `pattern_black_list`
        (canonical_parser.py:144-180): its pattern-key loop never resets
        `keys` for a blacklisted link, so that link is written under the
        PREVIOUS link's pattern keys in load order (links_1, links_2, links_n
        collections, first occurrence in parse order), and a blacklisted first
        link raises UnboundLocalError.  load_canonical then records those
        stale entries and every pattern-key answer includes them (a Link
        query hitting one binds the stale link's own targets, and raises
        AssertionError when their count differs: _assign_variables :467).
        Default: the intended semantics -- a blacklisted type's links get no
        pattern keys at all.  (The MettaYacc loader walks a Python set
        there, parser_threads.py:185-219: no order to reproduce.)"""
        if stream is None:
            try:
                import torch
                if torch.cuda.is_available():
                    torch.cuda.set_device(device)
                    stream = torch.cuda.current_stream(device).cuda_stream
            except ImportError:
                stream = None
        self.ctx = _lib.Context(device, stream)
        self.stream = stream
        self.tuple_targets = tuple_targets
        self.arrays = None
        self.type_id = {}
        self._hex_cache = {}
        self._handle_cache = {}
        self._node_handles = {}
        self._plan_records = {}
        self.generation = 0
        self.shard = None
        self._mirror = None
        self._hstore = None
        self._outgoing = None
        self._node_dir = None
        self.pattern_black_list = []
        self.stale_pattern_keys = stale_pattern_keys
        self._stale = None              # stale_pattern_keys: pattern key -> {link handle: targets}

    def __repr__(self):
        return "<HipDB>"

    # ------------------------------------------------------------------ load
    def load_arrays(self, arrays: "_loader.AtomArrays", shard=None):
        """Hash + intern + index every atom on the GPU (replaces the Mongo
        insert / key-value files / Redis SADD of canonical_parser.py:111-240).
        shard=(rank, world) (default: `arrays.shard`, set by
        parallel.shard_arrays): the whole KB is this rank's atom directory, and
        only the links whose handle `rank` owns get pattern-index rows."""
        self.generation = next(_LOADS)      # invalidates lowered query plans (unique across HipDBs)
        self._plan_records = {}
        self.shard = shard if shard is not None else getattr(arrays, "shard", None)
        # pattern_black_list is read at load time, as the reference's loaders
        # read it (distributed_atom_space.py:346, 409)
        self.ctx.set_pattern_black_list(self.pattern_black_list)
        self.ctx.build_index(arrays, self.shard)
        self.arrays = arrays
        self.type_id = dict(arrays.type_id)
        self._hex_cache = {}
        self._handle_cache = {}
        self._mirror = None
        self._hstore = None
        self._outgoing = None
        self._node_dir = None
        self._stale = None

    def load_metta(self, texts):
        self.load_arrays(_loader.parse_metta(texts).finish())

    def load_canonical(self, texts):
        """Canonical MeTTa through the native reader (das_parse_canonical).
        With stale_pattern_keys and a non-empty pattern_black_list, the
        reference loader's stale pattern entries are recorded (see __init__)."""
        stale = self.stale_from_canonical(texts)
        self.load_arrays(_lib.parse_canonical(texts))
        self._stale = stale

    def save_parsed(self, path):
        """The loaded KB's parsed atom arrays, pattern_black_list and (with
        stale_pattern_keys) the stale entries to one .npz, so a later
        load_parsed rebuilds the device index without the parser -- what the
        reference's kept key-value files do for its loader
        (canonical_parser.py:28-29, 235, 317-319)."""
        if self.arrays is None:
            raise ValueError("nothing loaded")
        stale = [[list(k), {h: list(t) for h, t in v.items()}] for k, v in (self._stale or {}).items()]
        self.arrays.save(path, {"pattern_black_list": list(self.pattern_black_list), "stale": stale})

    def load_parsed(self, path):
        """Rebuilds the index from save_parsed's file (the black list it was
        loaded with included); returns the AtomArrays."""
        arrays, extra = _loader.AtomArrays.load(path)
        self.pattern_black_list = list(extra.get("pattern_black_list", []))
        self.load_arrays(arrays)
        self._stale = {tuple(k): {h: tuple(t) for h, t in v.items()} for k, v in extra.get("stale", [])} or None
        return arrays

    def stale_from_canonical(self, texts):
        """stale_pattern_keys with a non-empty pattern_black_list: the stale
        entries the reference's loader would write for this canonical text
        (raises UnboundLocalError where its load does); else None."""
        if not (self.stale_pattern_keys and self.pattern_black_list):
            return None
        return _stale_entries(_loader.canonical_pattern_order(texts), set(self.pattern_black_list)) or None

    # ----------------------------------------- stale_pattern_keys (compat)
    def stale_values(self, link_type, target_handles):
        """{link handle: targets} the reference's loader wrote under this
        pattern key for blacklisted links (stale_pattern_keys), or None."""
        if not self._stale:
            return None
        th = WILDCARD if link_type == WILDCARD else ExpressionHasher.named_type_hash(link_type)
        hs = sorted(target_handles) if link_type in UNORDERED_LINK_TYPES else list(target_handles)
        return self._stale.get((th, *hs))

    def _stale_union(self, rel, link_type, handles, var_ids, ordered, no_overload, extra):
        """match_link's answer with the stale entries of its key added, each
        through Link._assign_variables (pattern_matcher.py:466-489) as the
        reference evaluates every value of the key."""
        arity = len(handles)
        for tg in extra.values():
            if len(tg) != arity:
                raise AssertionError(f"link_targets = {list(tg)} self.targets = {handles}")
        grounded = [h for h, v in zip(handles, var_ids) if v is None]
        if not ordered and grounded and self.tuple_targets:
            raise AttributeError("'tuple' object has no attribute 'remove'")
        rows = []
        for tg in extra.values():
            if ordered:
                m, vals, ok = {}, set(), True
                for v, h in zip(var_ids, tg):
                    if v is None:
                        continue
                    if v in m:
                        ok = m[v] == h
                    elif no_overload and h in vals:
                        ok = False
                    else:
                        m[v] = h
                        vals.add(h)
                    if not ok:
                        break
                if ok:
                    rows.append(m)
            else:
                left = list(tg)
                for h in grounded:
                    left.remove(h)                      # ValueError when absent, as list.remove
                names = [v for v in var_ids if v is not None]
                assert len(names) == len(left)
                if len(set(names)) == len(names) and len(set(left)) == len(left):
                    rows.append((names, left))           # UnorderedAssignment.freeze: counts agree
        if not rows:
            return rel
        old = [t for t in rel.tables if t.nrows]
        if ordered:
            vars_ = list(old[0].vars) if old else list(dict.fromkeys(v for v in var_ids if v is not None))
            ids = {h: i for h, i in zip(*self._ids_for([h for r in rows for h in r.values()]))}
            cols = [[ids[r[v]] for r in rows] for v in vars_]
            kind = _lib.TABLE_ORDERED
        else:
            vars_ = list(old[0].vars) if old else sorted(set(rows[0][0]))
            ids = {h: i for h, i in zip(*self._ids_for([h for _, left in rows for h in left]))}
            vals = [sorted(ids[h] for h in left) for _, left in rows]
            cols = [list(c) for c in zip(*vals)]
            kind = _lib.TABLE_UNORDERED
        t = self.ctx.table_from_host(kind, vars_, np.array(cols, dtype=np.uint32).reshape(len(vars_), len(rows)))
        merged = self.ctx.concat(old + [t]) if old else t
        return Relation([self.ctx.dedup(merged)])

    def _ids_for(self, handles):
        hs = list(dict.fromkeys(handles))
        return hs, self.ids_of(hs).tolist()

    def touches_stale(self, expr) -> bool:
        """Whether evaluating `expr` reads a pattern key that holds stale
        entries (the plan executor then steps aside: the per-operator path
        adds them at each Link)."""
        if not self._stale:
            return False
        k = getattr(expr, '_k', None)
        if k in ('a', 'o'):
            return any(self.touches_stale(t) for t in expr.terms)
        if k == 'x':
            return self.touches_stale(expr.term)
        if k == 'l':
            if any(self.touches_stale(t) for t in expr.targets):
                return True
            hs = [t.get_handle(self) for t in expr.targets]
            return None not in hs and WILDCARD in hs and self.stale_values(expr.atom_type, hs) is not None
        return False

    def clear(self):
        b = _loader.AtomBuilder()
        self.load_arrays(b.finish())

    def stats(self):
        return self.ctx.stats()

    def export_keyspace(self, directory):
        """Writes the Redis key-value files of the reference's loader
        (outgoing_set / incomming_set / patterns / templates / names,
        canonical_parser.py:119-183) for the loaded KB into `directory`."""
        os.makedirs(directory, exist_ok=True)
        return self.ctx.export_keyspace(directory)

    # --------------------------------------------------------------- helpers
    def _resolve(self, handles):
        """handle -> (id, category, arity) through a host cache of the device
        index (handles are immutable once the index is built).  After
        prefetch() every node handle is in a host directory: a fresh query
        anchor resolves without a device round trip."""
        nd = self._node_dir
        if nd is not None:
            for h in handles:
                if h not in self._handle_cache:
                    i = nd.get(h)
                    if i is not None:
                        self._handle_cache[h] = (i, 1, 0)
        miss = [h for h in dict.fromkeys(handles) if h not in self._handle_cache]
        if miss and all(type(h) is str and len(h) == 32 for h in miss):
            try:
                ids, cat, ar = self.ctx.lookup_hex(miss)
            except ValueError:          # not hex: the per-handle path below sorts it out
                pass
            else:
                for h, i, c, a in zip(miss, ids, cat, ar):
                    self._handle_cache[h] = (i, c, a)
                miss = []
        if miss:
            good = []
            for h in miss:
                try:
                    good.append((h, _lib.hex_to_digest(h)))
                except ValueError:
                    self._handle_cache[h] = (-1, 0, 0)
            if good:
                ids, cat, ar, _ = self.ctx.lookup(np.stack([d for _, d in good]))
                for (h, _), i, c, a in zip(good, ids.tolist(), cat.tolist(), ar.tolist()):
                    self._handle_cache[h] = (i, c, a)
        return [self._handle_cache[h] for h in handles]

    def prefetch_handles(self, handles) -> None:
        self._resolve(list(handles))

    def ids_of(self, handles: List[str]) -> np.ndarray:
        if not handles:
            return np.zeros(0, dtype=np.int64)
        return np.array([r[0] for r in self._resolve(handles)], dtype=np.int64)

    def _lookup(self, handle):
        r = self._handle_cache.get(handle)
        return r if r is not None else self._resolve([handle])[0]

    def hex_of(self, ids) -> List[str]:
        if len(ids) <= 16:
            # a few ids (one link's targets): the cache, no numpy set ops
            hc = self._hex_cache
            out = [hc.get(int(i)) for i in ids]
            if None not in out:
                return out
        ids = np.asarray(ids, dtype=np.uint32).ravel()
        if ids.size == 0:
            return []
        if _hex is not None and self._mirror is not None:
            # digests on the host (prefetch): every handle formatted in C,
            # once per atom (the store keeps the str objects made so far)
            if self._hstore is None:
                self._hstore = [None] * len(self._mirror[0])
            return _hex.hex_list(self._mirror[0], ids, ids.size, self._hstore)
        if ids.size > self.HEX_DIRECT:
            # a large answer: its digests straight from the mirror (prefetch)
            # or one device gather, formatted in one pass (no per-id cache work)
            if _hex is not None:
                if self._mirror is not None:
                    return _hex.hex_list(self._mirror[0], ids, ids.size)
                return _hex.hex_list(np.ascontiguousarray(self.ctx.atoms_info(ids)[0]), None, ids.size)
            dig = self._mirror[0][ids] if self._mirror is not None else self.ctx.atoms_info(ids)[0]
            return _lib.digests_to_hex(dig)
        uniq = np.unique(ids)
        missing = [int(i) for i in uniq if int(i) not in self._hex_cache]
        if missing:
            dig, _, _, _, _ = self.ctx.atoms_info(np.array(missing, dtype=np.uint32))
            for i, h in zip(missing, _lib.digests_to_hex(dig)):
                self._hex_cache[i] = h
        return [self._hex_cache[int(i)] for i in ids]

    def _host_mirror(self):
        """Host copy of per-atom category/type/name leaf (metadata calls only)."""
        if self._mirror is None:
            n = int(self.ctx.stats().n_atoms)
            ids = np.arange(n, dtype=np.uint32)
            dig, cat, ar, ty, nl = self.ctx.atoms_info(ids)
            self._mirror = (dig, cat, ar, ty, nl)
        return self._mirror

    def _atom_type_ok(self, name):
        return name in self.type_id

    def _exists(self, handle, arity):
        """_retrieve_mongo_document(handle, arity) is not None (redis_mongo_db.py:129-145)."""
        aid, cat, ar = self._lookup(handle)
        if aid < 0:
            return False
        if arity == 0:
            return cat == 1
        if cat not in (2, 3):          # 3: a link whose index rows live on another shard
            return False
        if arity == 1:
            return ar == 1
        if arity == 2:
            return ar == 2
        return ar not in (1, 2)

    def _fmt_targets(self, targets):
        return tuple(targets) if self.tuple_targets else list(targets)

    # ------------------------------------------------- DBInterface (reference)
    def node_exists(self, node_type: str, node_name: str) -> bool:
        """redis_mongo_db.py:204-208"""
        return self._exists(self.get_node_handle(node_type, node_name), 0)

    def link_exists(self, link_type: str, target_handles: List[str]) -> bool:
        """redis_mongo_db.py:210-213 (no sorting for unordered types, as the reference)"""
        h = ExpressionHasher.expression_hash(ExpressionHasher.named_type_hash(link_type), target_handles)
        return self._exists(h, len(target_handles))

    def get_node_handle(self, node_type: str, node_name: str) -> str:
        """redis_mongo_db.py:215-216 (memoised: a query names few nodes, often again)"""
        key = (node_type, node_name)
        h = self._node_handles.get(key)
        if h is None:
            if len(self._node_handles) > (1 << 20):
                self._node_handles.clear()
            h = self._node_handles[key] = ExpressionHasher.terminal_hash(node_type, node_name)
        return h

    def get_link_handle(self, link_type: str, target_handles: List[str]) -> str:
        """redis_mongo_db.py:218-220"""
        return ExpressionHasher.expression_hash(ExpressionHasher.named_type_hash(link_type), target_handles)

    def get_link_targets(self, link_handle: str) -> List[str]:
        """redis_mongo_db.py:222-227: the outgoing set.  Redis returns a set, so
        order and repeats are not preserved there; here the stored order is
        returned (a superset of what the reference guarantees).  After
        prefetch() the host copy of the outgoing CSR answers it."""
        aid, cat, _ = self._lookup(link_handle)
        if aid < 0 or cat not in (2, 3):
            raise ValueError(f"Invalid handle: {link_handle}")
        if self._outgoing is not None:
            off, tgt = self._outgoing
            return self.hex_of(tgt[int(off[aid]):int(off[aid + 1])])
        return self.hex_of(self.ctx.link_targets(aid))

    def get_incoming_links(self, atom_handle: str) -> List[str]:
        """The `incomming_set:<handle>` index family (canonical_parser.py:141-143,
        parser_threads.py:155-159; no reference DBInterface method reads it):
        every link whose targets contain the atom.  Redis returns a set; here
        the handles come sorted by link id."""
        aid, cat, _ = self._lookup(atom_handle)
        if aid < 0:
            raise ValueError(f"Invalid handle: {atom_handle}")
        return list(dict.fromkeys(self.hex_of(self.ctx.incoming(aid))))   # a set, as SADD builds it

    def is_ordered(self, link_handle: str) -> bool:
        """redis_mongo_db.py:229-233"""
        aid, cat, _ = self._lookup(link_handle)
        if aid < 0 or cat != 2:
            raise ValueError(f"Invalid handle: {link_handle}")
        return True

    def get_matched_links(self, link_type: str, target_handles: List[str]):
        """redis_mongo_db.py:235-252: grounded -> [handle] / []; otherwise the
        pattern key (sorted targets for Similarity/Set) -> [(handle, targets)]."""
        if link_type != WILDCARD and WILDCARD not in target_handles:
            h = self.get_link_handle(link_type, target_handles)
            return [h] if self._exists(h, len(target_handles)) else []
        t = self.matched_links_table(link_type, target_handles)
        out = self._pairs(t, len(target_handles)) if t is not None else []
        extra = self.stale_values(link_type, target_handles)
        if extra:
            out = list(out) + [(h, tuple(tg) if self.tuple_targets else list(tg)) for h, tg in extra.items()]
        return out

    # the (link, t0 .. t_{a-1}) id rows behind get_matched_links /
    # get_matched_type_template / get_matched_type, before formatting (a
    # sharded DB gathers these from every shard, parallel.ShardedDB)
    def matched_links_table(self, link_type, target_handles):
        """Rows of the pattern key (link_type, target_handles) with at least
        one wildcard; None when the key cannot match (unknown type / target)."""
        if link_type in UNORDERED_LINK_TYPES:
            target_handles = sorted(target_handles)
        arity = len(target_handles)
        ttype = self._type_or_empty(link_type)
        if ttype is False:
            return None
        tids = self._target_ids(target_handles)
        if tids is None:
            return None
        return self.ctx.scan_link(arity, ttype, tids, list(range(arity)), 0, True, False, True)

    def matched_template_table(self, template):
        """Rows of templates:<composite type of `template`> (len >= 2); None
        when no link has that composite type."""
        ct, _ = self._template_ctype(template)
        if ct < 0:
            return None
        arity = len(template) - 1
        return self.ctx.scan_template(ct, arity, list(range(arity)), True, False, True)

    def matched_type_tables(self, link_type):
        """{arity: rows} of templates:<named_type_hash(link_type)>."""
        tid = self.type_id.get(link_type)
        if tid is None:
            return {}
        return {a: t for a, t in enumerate(self.ctx.scan_type(tid)) if t is not None}

    def _pairs(self, t, arity):
        cols = t.fetch()
        n = cols.shape[1]
        if n == 0:
            return []
        # one container per row: with the collector on, every 700 of them start
        # a collection that walks the handle cache and the caller's live
        # objects (~1 us per row at 10^6 cached handles instead of ~0.15)
        enabled = gc.isenabled()
        gc.disable()
        try:
            if n > self.HEX_DIRECT and _hex is not None:
                # every handle str written in C (_assign.hex_pairs), from the
                # mirror or from one device gather of the answer's digests
                cols = np.ascontiguousarray(cols)
                if self._mirror is not None:
                    out = _hex.hex_pairs(self._mirror[0], cols, arity + 1, n, self.tuple_targets)
                else:
                    dig = np.ascontiguousarray(self.ctx.atoms_info(cols.ravel())[0])
                    out = _hex.hex_pairs(dig, None, arity + 1, n, self.tuple_targets)
                links = None
            else:
                links = self.hex_of(cols[0])
                tg = [self.hex_of(cols[1 + k]) for k in range(arity)]
                out = list(zip(links, zip(*tg) if self.tuple_targets else map(list, zip(*tg))))
            # the links of a pattern answer are indexed here (category 2): a
            # caller's next get_link_targets / link lookups of them (the
            # SimplePatternMiner halo walk) need no device lookup
            self._seed(links if links is not None else out, cols[0], arity)
            return out
        finally:
            if enabled:
                gc.enable()

    def _seed(self, strs, ids, arity):
        """The links of a pattern answer are indexed here (category 2): a
        caller's next get_link_targets / link lookups of them (the
        SimplePatternMiner halo walk) need no device lookup.  strs: handle
        strs or (handle, targets) pairs, ids: their atom ids."""
        hc = self._handle_cache
        if len(hc) > (1 << 23):
            hc.clear()
        if len(strs) > self.SEED_MAX:
            return
        if _hex is not None:
            _hex.seed(hc, strs, np.ascontiguousarray(ids, dtype=np.uint32), arity)
            return
        for h, i in zip(strs, np.asarray(ids).tolist()):
            if not isinstance(h, str):
                h = h[0]
            if h not in hc:
                hc[h] = (i, 2, arity)

    def get_matched_link_handles(self, link_type: str, target_handles: List[str]) -> List[str]:
        """[h for h, _ in get_matched_links(link_type, target_handles)]
        without building the target lists: what the facade's get_links
        returns in its default HANDLE format (distributed_atom_space.py:
        259-284), e.g. SimplePatternMiner's len(get_links(...)) counts."""
        if link_type != WILDCARD and WILDCARD not in target_handles:
            return self.get_matched_links(link_type, target_handles)
        if self._stale and self.stale_values(link_type, target_handles):
            return [h for h, _ in self.get_matched_links(link_type, target_handles)]
        t = self.matched_links_table(link_type, target_handles)
        if t is None or t.nrows == 0:
            return []
        ids = np.ascontiguousarray(t.fetch()[0])
        enabled = gc.isenabled()
        gc.disable()
        try:
            links = self.hex_of(ids)
            self._seed(links, ids, len(target_handles))
            return links
        finally:
            if enabled:
                gc.enable()

    def get_all_nodes(self, node_type: str, names: bool = False) -> List[str]:
        """redis_mongo_db.py:254-267"""
        tid = self.type_id.get(node_type)
        if tid is None:
            return []
        dig, cat, _, ty, nl = self._host_mirror()
        sel = np.nonzero((cat == 1) & (ty == tid))[0]
        if names:
            return [self.arrays.node_name(int(nl[i])) for i in sel]
        return _lib.digests_to_hex(dig[sel]) if sel.size else []

    def _template_ctype(self, template):
        hashed = []
        for t in template:
            if not isinstance(t, str):
                raise TypeError("sequence item: expected str instance, list found")
            hashed.append(_lib.md5_digest(t))
        if len(hashed) == 1:
            return None, hashed[0]
        return self.ctx.ctype_lookup(_lib.composite_digest(hashed)), None

    def get_matched_type_template(self, template: List[Any]) -> List[str]:
        """redis_mongo_db.py:269-275 (templates:<composite_type_hash>)"""
        if len(template) == 1:
            self._template_ctype(template)          # the reference's TypeError for a non-str element
            return self.get_matched_type(template[0])
        t = self.matched_template_table(template)
        return self._pairs(t, len(template) - 1) if t is not None else []

    def get_matched_type(self, link_type: str) -> List[str]:
        """redis_mongo_db.py:277-279 (templates:<named_type_hash>)"""
        out = []
        for a, t in self.matched_type_tables(link_type).items():
            out += self._pairs(t, a)
        return out

    def get_node_name(self, node_handle: str) -> str:
        """redis_mongo_db.py:281-285 (names:<handle>)"""
        aid, cat, _ = self._lookup(node_handle)
        if aid < 0 or cat != 1:
            raise ValueError(f"Invalid handle: {node_handle}")
        if self._mirror is not None:
            return self.arrays.node_name(int(self._mirror[4][aid]))
        _, _, _, _, nl = self.ctx.atoms_info(np.array([aid], dtype=np.uint32))
        return self.arrays.node_name(int(nl[0]))

    def get_matched_node_name(self, node_type: str, substring: str) -> str:
        """redis_mongo_db.py:287-293 (Mongo $regex on names of that type)"""
        tid = self.type_id.get(node_type)
        if tid is None:
            return []
        dig, cat, _, ty, nl = self._host_mirror()
        sel = np.nonzero((cat == 1) & (ty == tid))[0]
        rx = re.compile(substring)
        hits = [i for i in sel if rx.search(self.arrays.node_name(int(nl[i])))]
        return _lib.digests_to_hex(dig[hits]) if hits else []

    def get_atom_as_dict(self, handle, arity=-1) -> dict:
        """redis_mongo_db.py:297-311"""
        aid, cat, ar = self._lookup(handle)
        if aid < 0 or cat == 0:
            return {}
        _, _, _, ty, nl = self.ctx.atoms_info(np.array([aid], dtype=np.uint32))
        tname = self.arrays.type_names[int(ty[0])]
        if cat == 1:
            return {"handle": handle, "type": tname, "name": self.arrays.node_name(int(nl[0]))}
        targets = self.hex_of(self.ctx.link_targets(aid))
        return {"handle": handle, "type": tname, "template": self._template_of(aid), "targets": targets}

    def _template_of(self, aid):
        _, cat, _, ty, _ = self.ctx.atoms_info(np.array([aid], dtype=np.uint32))
        tname = self.arrays.type_names[int(ty[0])]
        if cat[0] != 2:
            return tname
        return [tname] + [self._template_of(int(x)) for x in self.ctx.link_targets(aid)]

    def get_atom_as_deep_representation(self, handle: str, arity=-1) -> str:
        """redis_mongo_db.py:187-199, 313-314"""
        aid, cat, _ = self._lookup(handle)
        if aid < 0:
            raise ValueError(f"Invalid handle: {handle}")
        return self._deep(aid)

    def _deep(self, aid):
        _, cat, _, ty, nl = self.ctx.atoms_info(np.array([aid], dtype=np.uint32))
        tname = self.arrays.type_names[int(ty[0])] if ty[0] != _lib.DAS_NONE else None
        if cat[0] == 1:
            return {"type": tname, "name": self.arrays.node_name(int(nl[0]))}
        return {"type": tname, "targets": [self._deep(int(x)) for x in self.ctx.link_targets(aid)]}

    def _type_of(self, aid):
        if self._mirror is not None:
            return self.arrays.type_names[int(self._mirror[3][aid])]
        _, _, _, ty, _ = self.ctx.atoms_info(np.array([aid], dtype=np.uint32))
        return self.arrays.type_names[int(ty[0])]

    def get_link_type(self, link_handle: str) -> str:
        aid, cat, _ = self._lookup(link_handle)
        if aid < 0 or cat not in (2, 3):
            raise KeyError(link_handle)
        return self._type_of(aid)

    def get_node_type(self, node_handle: str) -> str:
        aid, cat, _ = self._lookup(node_handle)
        if aid < 0 or cat != 1:
            raise KeyError(node_handle)
        return self._type_of(aid)

    def count_atoms(self) -> Tuple[int, int]:
        """redis_mongo_db.py:330-335"""
        st = self.ctx.stats()
        return (int(st.n_nodes), int(st.n_links))

    def prefetch(self) -> None:
        """redis_mongo_db.py:89-127 caches the node / link type documents in
        host memory for the per-atom metadata calls; here the index is
        resident in HBM, and prefetch copies the per-atom metadata (handle,
        category, arity, type, name leaf) and the outgoing CSR to the host, so
        get_link_targets / get_link_type / get_node_type / get_node_name are
        host lookups instead of a device round trip each (the
        SimplePatternMiner.ipynb halo walk calls get_link_targets per link),
        and a host directory of the node handles lets a query's fresh node
        anchors resolve without a device lookup.  KBs above
        PREFETCH_MAX_ATOMS atoms keep every call on the device."""
        st = self.ctx.stats()
        if int(st.n_atoms) > self.PREFETCH_MAX_ATOMS:
            return                          # (a 10^9-link KB: the device index answers every call)
        dig, cat, _, _, _ = self._host_mirror()
        if self._node_dir is None:
            sel = np.nonzero(cat == 1)[0]
            self._node_dir = dict(zip(_lib.digests_to_hex(dig[sel]), sel.tolist())) if sel.size else {}
        if self._outgoing is None:
            self._outgoing = self.ctx.outgoing_csr()

    # ------------------------------------------------ matcher entry points
    def _type_or_empty(self, link_type):
        """type id, None for '*', False for a type the KB never saw (no match)."""
        if link_type == WILDCARD:
            return None
        tid = self.type_id.get(link_type)
        return False if tid is None else tid

    def _target_ids(self, handles):
        """ids for grounded handles (DAS_NONE for '*'); None if one is unknown."""
        cache = self._handle_cache
        miss = [h for h in handles if h != WILDCARD and h not in cache]
        if miss:
            self._resolve(miss)
        out = []
        for h in handles:
            if h == WILDCARD:
                out.append(_lib.DAS_NONE)
                continue
            i = cache[h][0]
            if i < 0:
                return None
            out.append(i)
        return out

    def match_link(self, link_type, handles, var_ids, ordered, no_overload=False, order_var=None):
        """Link.matched's wildcard branch fused with _assign_variables
        (pattern_matcher.py:515-535 over redis_mongo_db.py:235-252).
        handles: reference-order target handles ('*' for variables);
        var_ids: variable id per position in the Link's own target order;
        order_var: the variable the caller will join on -- a typed scan then
        returns its rows sorted by it (same answer, join-friendly order)."""
        spec = self.link_scan_spec(link_type, handles, var_ids, ordered, no_overload, order_var)
        rel = Relation()
        if spec is not None:
            args, dedup = spec
            t = self.ctx.scan_link(*args)
            if dedup:
                t = self.ctx.dedup(t)
            rel = Relation([t])
        extra = self.stale_values(link_type, handles)
        if extra:
            rel = self._stale_union(rel, link_type, handles, var_ids, ordered, no_overload, extra)
        return rel

    def link_scan_spec(self, link_type, handles, var_ids, ordered, no_overload=False, order_var=None):
        """(scan_link arguments, dedup) of match_link; None when the scan
        matches nothing (unknown type or target, repeated unordered variable)."""
        if link_type in UNORDERED_LINK_TYPES:
            order = sorted(range(len(handles)), key=lambda i: handles[i])
            key_handles = [handles[i] for i in order]
        else:
            key_handles = list(handles)
        arity = len(handles)
        ttype = self._type_or_empty(link_type)
        tids = self._target_ids(key_handles)
        if ttype is False or tids is None or arity == 0 or arity > 8:
            return None
        names = [v for v in var_ids if v is not None]
        repeated = len(set(names)) != len(names)
        if ordered:
            var = [v if v is not None else -1 for v in var_ids]
            order_pos = -1
            if order_var is not None and order_var in var and link_type not in UNORDERED_LINK_TYPES:
                order_pos = var.index(order_var)
            args = (arity, ttype, tids, var, 0, True, no_overload, False, order_pos)
        else:
            if repeated:
                return None             # UnorderedAssignment.assign rejects a repeat (:196-197)
            args = (arity, ttype, tids, names, len(names), False, no_overload, False, -1)
        # rows are distinct links of one type unless a '*' type, a repeated
        # variable, an unordered value set or the sorted-key quirk of ordered
        # Similarity/Set queries can make two links bind the same values
        dedup = ttype is None or repeated or not ordered or link_type in UNORDERED_LINK_TYPES
        return args, dedup

    def match_template(self, link_type, target_types, var_ids, ordered, no_overload=False):
        """LinkTemplate.matched (pattern_matcher.py:603-614) over
        get_matched_type_template (redis_mongo_db.py:269-275)."""
        ct, named = self._template_ctype([link_type, *target_types])
        if named is not None:
            if self.get_matched_type(link_type):
                raise AssertionError("LinkTemplate without targets matched links with targets")
            return Relation()
        if ct < 0:
            return Relation()
        if not ordered and len(set(var_ids)) != len(var_ids):
            return Relation()
        t = self.ctx.scan_template(ct, len(target_types), list(var_ids), ordered, no_overload)
        if not ordered or len(set(var_ids)) != len(var_ids):
            t = self.ctx.dedup(t)
        return Relation([t])

    # ------------------------------------------------ relation algebra (1 GPU)
    def rel_normalize(self, rel):
        """One table per schema, rows distinct (Python set semantics).  A
        composite row can equal a row of another schema (XOR identity,
        pattern_matcher.py:279-286), so relations holding composites are
        deduplicated across all their tables by canonical identity."""
        if _has_composite(rel.tables):
            groups = _group(rel.tables)
            merged = [ts[0] if len(ts) == 1 else self.ctx.concat(ts) for ts in groups.values()]
            return Relation(self.ctx.set_dedup(merged))
        out = []
        for schema, ts in _group(rel.tables).items():
            out.append(ts[0] if len(ts) == 1 else self.ctx.dedup(self.ctx.concat(ts)))
        return Relation(out)

    def rel_union(self, a, b):
        return self.rel_normalize(Relation(a.tables + b.tables))

    def rel_join(self, a, b):
        """And's join step (pattern_matcher.py:732-738) for every schema pair."""
        from ..pattern_matcher.pattern_matcher import CONFIG
        out = []
        for ta in a.tables:
            for tb in b.tables:
                # ordered x ordered: natural join; any unordered operand: the
                # CompositeAssignment algebra (:203-209, :316-351) on the GPU
                out.append(self.ctx.join(ta, tb, CONFIG['no_overload']))
        return Relation(out)

    def index_join_spec(self, link_type, handles, var_ids):
        """(arity, type id, target ids, variables) of das_index_join for one
        ordered Link term, or None when the index join cannot apply."""
        if link_type in UNORDERED_LINK_TYPES:
            return None
        ttype = self._type_or_empty(link_type)
        if ttype is None or ttype is False:
            return None
        tids = self._target_ids(list(handles))
        if tids is None:
            return None
        return len(handles), ttype, tids, [v if v is not None else -1 for v in var_ids]

    def rel_index_join(self, acc, link_type, handles, var_ids):
        """And's join of the running relation with one ordered Link term
        through the pattern index (das_index_join): the rows of
        rel_join(acc, match_link(...)) without scanning the term.  None when
        it does not apply to every table of acc (the caller scans + joins)."""
        if not acc.tables:
            return None
        spec = self.index_join_spec(link_type, handles, var_ids)
        if spec is None:
            return None
        out = []
        for t in acc.tables:
            if t.kind != _lib.TABLE_ORDERED:
                return None
            r = self.ctx.index_join(t, *spec)
            if r is None:
                return None
            out.append(r)
        return Relation(out)

    def rel_antijoin(self, rel, forbidden):
        """check_negation of every row against every forbidden row (:741-746)."""
        tables = rel.tables
        for f in forbidden.tables:
            nxt = []
            for t in tables:
                nxt.append(self.ctx.antijoin(t, f))
            tables = nxt
        return Relation(tables)

    def rel_minus(self, a, b):
        """Set difference a - b by identity (same kind and variables, equal
        values; canonical identity when composites are involved)."""
        if _has_composite(a.tables) or _has_composite(b.tables):
            if not a.tables or not b.tables:
                return Relation(a.tables)
            return Relation(self.ctx.set_minus(a.tables, b.tables))
        groups = _group(b.tables)
        out = []
        for t in a.tables:
            for f in groups.get(t.schema, []):
                t = self.ctx.antijoin(t, f)
            out.append(t)
        return Relation(out)
