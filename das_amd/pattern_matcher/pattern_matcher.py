"""Pattern matcher with the reference's API (das/pattern_matcher/pattern_matcher.py).

Same classes, constructor signatures and `matched(db, answer) -> bool`
contract; `answer.assignments` is the reference's set of `Assignment`
objects.  Evaluation is different: every term produces a *device* binding
relation (HipDB.match_link / match_template -> scan kernels), `And` folds
them with GPU natural joins and anti-joins, `Or` with GPU union/dedup and set
difference.  Python `Assignment` objects are only built when a caller reads
`answer.assignments`.

Semantics kept from the reference: reset-on-empty in
And (:725-729), skipped empty terms (:717-719), negated terms collected as a
forbidden set (:720-724, :741-746), Or with Not terms = And(negated) minus the
positive union with negation=True (:674-683), top-level Not flips the flag
(:627-631), `_typed_variable_matched` last-writer-wins (:491-500).

All assignment kinds are evaluated on the GPU: ordered natural joins, and
for unordered (Similarity/Set) operands the reference's Unordered /
CompositeAssignment algebra (:158-368: containment / coverage /
compatibility checks, XOR set identity), das_amd/csrc/composite.hip.
"""
import gc
import os
import struct
from abc import ABC, abstractmethod
from collections import Counter
from copy import deepcopy
from enum import Enum, auto
from functools import cmp_to_key
from typing import Dict, FrozenSet, List, Optional, Set, Union

import numpy as np

from .. import _lib
from ..database.db_interface import UNORDERED_LINK_TYPES, WILDCARD, DBInterface
from ..database.hip_db import HipDB, Relation, RelationalDB

DEBUG_AND = False
DEBUG_OR = False
DEBUG_NOT = False
DEBUG_LINK = False
DEBUG_LINK_TEMPLATE = False

CONFIG = {
    'no_overload': False,   # distinct variables must take distinct values (ordered)
}


class CompatibilityStatus(int, Enum):
    INCOMPATIBLE = auto()
    NO_COVERING = auto()
    FIRST_COVERS_SECOND = auto()
    SECOND_COVERS_FIRST = auto()
    EQUAL = auto()


# ---------------------------------------------------------------------------
# variable ids (device tables carry small integer variable ids)
# ---------------------------------------------------------------------------
_VAR_ID: Dict[str, int] = {}
_VAR_NAME: List[str] = []


def _vid(name: str) -> int:
    v = _VAR_ID.get(name)
    if v is None:
        v = len(_VAR_NAME)
        _VAR_ID[name] = v
        _VAR_NAME.append(name)
    return v


def _var_name(v: int) -> str:
    return _VAR_NAME[v]


# ---------------------------------------------------------------------------
# Assignments: the reference's value objects (identity = hash equality)
# ---------------------------------------------------------------------------
class Assignment(ABC):

    def __init__(self):
        self.variables: Union[Set[str], FrozenSet] = set()
        self.hash: int = 0
        self.frozen = False

    def __hash__(self) -> int:
        assert self.hash
        return self.hash

    def __eq__(self, other) -> bool:
        assert self.hash and other.hash
        return self.hash == other.hash

    def __lt__(self, other) -> bool:
        assert self.hash and other.hash
        return self.hash < other.hash

    def freeze(self) -> bool:
        if self.frozen:
            return False
        self.frozen = True
        self.variables = frozenset(self.variables)
        return True

    @abstractmethod
    def assign(self, variable: str, value: str) -> bool: ...

    @abstractmethod
    def join(self, other: 'Assignment') -> 'Assignment': ...

    @abstractmethod
    def check_negation(self, negation: 'Assignment') -> bool: ...


def _bad_assign(variable, value, frozen):
    if variable is None or value is None or frozen:
        raise ValueError(f'Invalid assignment: variable = {variable} value = {value} frozen = {frozen}')


class OrderedAssignment(Assignment):

    def __init__(self):
        super().__init__()
        self.mapping: Dict[str, str] = {}
        self.values: Union[Set[str], FrozenSet] = set()

    def __repr__(self):
        return repr(self.mapping)

    def freeze(self):
        assert super().freeze()
        self.values = frozenset(self.values)
        self.hash = hash(frozenset(self.mapping.items()))
        return True

    def assign(self, variable: str, value: str) -> bool:
        _bad_assign(variable, value, self.frozen)
        if variable in self.variables:
            return self.mapping[variable] == value
        if CONFIG['no_overload'] and value in self.values:
            return False
        self.variables.add(variable)
        self.values.add(value)
        self.mapping[variable] = value
        return True

    def evaluate_compatibility(self, other) -> CompatibilityStatus:
        assert other is not None
        if self.hash == other.hash:
            return CompatibilityStatus.EQUAL
        if any(self.mapping[v] != other.mapping[v] for v in self.variables & other.variables):
            return CompatibilityStatus.INCOMPATIBLE
        if other.variables < self.variables:
            return CompatibilityStatus.FIRST_COVERS_SECOND
        if self.variables < other.variables:
            return CompatibilityStatus.SECOND_COVERS_FIRST
        return CompatibilityStatus.NO_COVERING

    def compatible(self, other) -> bool:
        return self.evaluate_compatibility(other) != CompatibilityStatus.INCOMPATIBLE

    def _join_ordered(self, other):
        status = self.evaluate_compatibility(other)
        if status == CompatibilityStatus.INCOMPATIBLE:
            return None
        if status in (CompatibilityStatus.EQUAL, CompatibilityStatus.FIRST_COVERS_SECOND):
            return self
        if status == CompatibilityStatus.SECOND_COVERS_FIRST:
            return other
        merged = OrderedAssignment()
        for var, val in list(self.mapping.items()) + list(other.mapping.items()):
            if not merged.assign(var, val):
                return None
        merged.freeze()
        return merged

    def join(self, other: Assignment) -> Assignment:
        assert self.frozen and other.frozen
        return self._join_ordered(other) if isinstance(other, OrderedAssignment) else other.join(self)

    def check_negation(self, negation: Assignment) -> bool:
        if isinstance(negation, OrderedAssignment):
            return self.evaluate_compatibility(negation) not in (
                CompatibilityStatus.EQUAL, CompatibilityStatus.FIRST_COVERS_SECOND)
        return not negation.is_covered_by_ordered(self)


class UnorderedAssignment(Assignment):

    def __init__(self):
        super().__init__()
        self.symbols: Dict[str, int] = {}
        self.values: Dict[str, int] = {}

    def __repr__(self):
        syms = [s for s, c in self.symbols.items() for _ in range(c)]
        vals = [v for v, c in self.values.items() for _ in range(c)]
        return '*' + repr(dict(zip(syms, vals)))

    def freeze(self):
        assert super().freeze()
        if sorted(self.symbols.values()) != sorted(self.values.values()):
            return False
        self.hash = hash((hash(frozenset(self.symbols.items())), hash(frozenset(self.values.items()))))
        return True

    def assign(self, variable: str, value: str) -> bool:
        _bad_assign(variable, value, self.frozen)
        if variable in self.variables:
            return False
        self.symbols[variable] = self.symbols.get(variable, 0) + 1
        self.values[value] = self.values.get(value, 0) + 1
        self.variables.add(variable)
        return True

    def join(self, other: Assignment) -> Assignment:
        assert self.frozen and other.frozen
        if isinstance(other, CompositeAssignment):
            return other.join(self)
        return CompositeAssignment(self).join(other)

    def check_negation(self, negation: Assignment) -> bool:
        if isinstance(negation, OrderedAssignment):
            return not self.contains_ordered(negation)
        if isinstance(negation, UnorderedAssignment):
            return not self.contains_unordered(negation)
        return all(not self.contains_unordered(u) for u in negation.unordered_mappings)

    def contains_ordered(self, ordered_assignment) -> bool:
        if not set(ordered_assignment.mapping) <= set(self.variables):
            return False
        need = Counter(ordered_assignment.mapping.values())
        return all(self.values.get(v, 0) >= c for v, c in need.items())

    def is_covered_by_ordered(self, ordered_assignment) -> bool:
        sym = Counter(self.symbols)
        val = Counter(self.values)
        sym.subtract(Counter(ordered_assignment.mapping.keys()))
        val.subtract(Counter(ordered_assignment.mapping.values()))
        return all(c <= 0 for c in sym.values()) and all(c <= 0 for c in val.values())

    def contains_unordered(self, unordered_assignment) -> bool:
        return all(self.symbols.get(s, 0) >= c for s, c in unordered_assignment.symbols.items()) and \
            all(self.values.get(v, 0) >= c for v, c in unordered_assignment.values.items())

    def compatible(self, other) -> bool:
        common_syms = set(self.variables) & set(other.variables)
        common_vals = set(self.values) & set(other.values)
        s_self = sum(self.symbols[s] for s in common_syms)
        s_other = sum(other.symbols[s] for s in common_syms)
        v_self = sum(self.values[v] for v in common_vals)
        v_other = sum(other.values[v] for v in common_vals)
        return v_other >= s_self and v_self >= s_other


class CompositeAssignment(Assignment):

    def __init__(self, assignment: UnorderedAssignment):
        super().__init__()
        self.unordered_mappings: List[UnorderedAssignment] = [assignment]
        self.ordered_mapping: Optional[OrderedAssignment] = None
        self.variables = deepcopy(assignment.variables)
        assert self._freeze()

    def __repr__(self):
        return f'Ordered = {self.ordered_mapping} | Unordered = {self.unordered_mappings}'

    def _freeze(self):
        assert super().freeze()
        self._recompute_hash()
        return True

    def freeze(self):
        assert False

    def assign(self, variable: str, value: str) -> bool:
        assert False

    def _recompute_hash(self) -> None:
        h = self.ordered_mapping.hash if self.ordered_mapping else 1
        for u in self.unordered_mappings:
            h ^= u.hash
        self.hash = h

    def _viable(self) -> bool:
        if not self.ordered_mapping:
            return bool(self.unordered_mappings)
        return all(u.contains_ordered(self.ordered_mapping) or u.is_covered_by_ordered(self.ordered_mapping)
                   for u in self.unordered_mappings)

    def _add_ordered_mapping(self, other: OrderedAssignment) -> bool:
        if self.ordered_mapping is None:
            self.ordered_mapping = other
        else:
            self.ordered_mapping = self.ordered_mapping.join(other)
            if self.ordered_mapping is None:
                return False
        if not self._viable():
            return False
        self._recompute_hash()
        return True

    def _add_unordered_mapping(self, u) -> bool:
        if self.ordered_mapping and not u.contains_ordered(self.ordered_mapping):
            return False
        if not all(x.compatible(u) for x in self.unordered_mappings):
            return False
        self.unordered_mappings.append(u)
        self._recompute_hash()
        return True

    def join(self, other: Assignment) -> Assignment:
        assert self.frozen and other.frozen
        out = deepcopy(self)
        if isinstance(other, OrderedAssignment):
            ok = out._add_ordered_mapping(other)
        elif isinstance(other, UnorderedAssignment):
            ok = out._add_unordered_mapping(other)
        else:
            ok = out._add_ordered_mapping(other.ordered_mapping) and \
                all(out._add_unordered_mapping(u) for u in other.unordered_mappings)
        return out if ok else None

    def check_negation(self, negation: Assignment) -> bool:
        if isinstance(negation, OrderedAssignment):
            return all(not u.contains_ordered(negation) for u in self.unordered_mappings)
        if isinstance(negation, UnorderedAssignment):
            return all(not u.contains_unordered(negation) for u in self.unordered_mappings)
        raise AttributeError("'CompositeAssignment' object has no attribute 'unordered_assignments'")

    def contains_ordered(self, ordered_assignment) -> bool:
        return all(u.contains_ordered(ordered_assignment) for u in self.unordered_mappings)

    def contains_unordered(self, unordered_assignment) -> bool:
        return all(u.contains_unordered(unordered_assignment) for u in self.unordered_mappings)


# ---------------------------------------------------------------------------
# Relational evaluation: the DB owns the device relation algebra
# (HipDB on one GPU, parallel.ShardedDB across ranks)
# ---------------------------------------------------------------------------

def _hip(db):
    if not isinstance(db, RelationalDB):
        raise TypeError(f"das_amd evaluates patterns on the MI355X index; got {db!r} (use HipDB)")
    return db


# ---------------------------------------------------------------------------
# Whole-expression plans: an And / Or / Not tree of ordered, flat Links is
# lowered once per (expression, index) to das_plan_node_t records and folded
# by das_plan_execute in a single native call (das_amd/csrc/plan.hip restates
# the And / Or / Not rules below).  Anything else -- unordered links,
# templates, nested link targets, sharded DBs -- takes the per-operator path.
# ---------------------------------------------------------------------------


class _Unsupported(Exception):
    pass


_RECORD = struct.Struct("<51I")
_WORDS = 51


def _node_record(op, nchild=0, value=0, spec=None, ij=None):
    """One das_plan_node_t as 204 bytes (51 u32 words, include/das_mi355x.h)."""
    words = [op, nchild, value, 0, 0] + [0] * 46
    if spec is not None:
        args, dedup = spec
        words[3] = 1 if dedup else 0
        words[5:28] = _scan_words(*args)
    if ij is not None:
        words[4] = 1
        words[28:51] = _scan_words(ij[0], ij[1], ij[2], ij[3], 0, True)
    return _RECORD.pack(*[w & 0xFFFFFFFF for w in words])


def _scan_words(arity, type_id, targets, var, n_vars, ordered, no_overload=False, emit_link=False, order_pos=-1):
    """das_link_scan_t as 23 words (field order of include/das_mi355x.h)."""
    t = list(targets) + [_lib.DAS_NONE] * (8 - len(targets))
    v = list(var) + [-1] * (8 - len(var))
    return [arity, _lib.DAS_NONE if type_id is None else type_id] + t + v + \
        [n_vars, 1 if ordered else 0, 1 if no_overload else 0, 1 if emit_link else 0, order_pos]


_HEADERS = {}


def _header(op, nchild=0, value=0):
    key = (op, nchild, value)
    r = _HEADERS.get(key)
    if r is None:
        r = _HEADERS[key] = _node_record(op, nchild, value)
    return r


def _link_signature(link):
    """What a Link's plan record depends on besides the index: its type,
    targets (variable names / node type and name) and join-order hint."""
    sig = [link.atom_type, getattr(link, '_order_var', None)]
    for t in link.targets:
        k = t._k
        if k == 'v':
            sig.append(t.name)
        elif k == 'n':
            sig.append((t.atom_type, t.name))
        else:
            raise _Unsupported()          # LinkTemplate / nested Link / typed targets
    return tuple(sig)


def _link_record(link, db, no_overload):
    """Link.matched (pattern_matcher.py:502-538) as one plan record: every
    target matched (node_exists), link_exists when nothing is a wildcard,
    else the match_link scan (+ the index-join form And may use)."""
    if not all(t.matched(db, None) for t in link.targets):
        return _header(_lib.PLAN_CONST, 0, 0)
    handles = [t.get_handle(db) for t in link.targets]
    if WILDCARD not in handles:
        return _header(_lib.PLAN_CONST, 0, 1 if db.link_exists(link.atom_type, handles) else 0)
    var_ids = [_vid(t.name) if t._k == 'v' else None for t in link.targets]
    hint = getattr(link, '_order_var', None)
    spec = db.link_scan_spec(link.atom_type, handles, var_ids, True, no_overload,
                             _vid(hint) if hint is not None else None)
    if spec is None:
        return _header(_lib.PLAN_CONST, 0, 0)
    ij = None if no_overload else db.index_join_spec(link.atom_type, handles, var_ids)
    return _node_record(_lib.PLAN_LINK, 0, 0, spec, ij)


def _template_record(tmpl, db, no_overload):
    """LinkTemplate.matched (pattern_matcher.py:603-614 over
    get_matched_type_template, redis_mongo_db.py:269-275) as one TEMPLATE
    record: the composite type's links, every target a typed variable."""
    ct, named = db._template_ctype([tmpl.link_type, *[v.type for v in tmpl.targets]])
    if named is not None:
        raise _Unsupported()                  # a template without targets (match_template's assertion case)
    if ct < 0:
        return _header(_lib.PLAN_CONST, 0, 0)
    var_ids = [_vid(v.name) for v in tmpl.targets]
    words = [_lib.PLAN_TEMPLATE, 0, 0, 1 if len(set(var_ids)) != len(var_ids) else 0, 0] + [0] * 46
    words[5:28] = _scan_words(len(var_ids), ct, [], var_ids, 0, True, no_overload)
    return _RECORD.pack(*[w & 0xFFFFFFFF for w in words])


def _walk(expr, out, links, root=True):
    """Prefix-order skeleton of `expr`: header records and Link slots."""
    k = expr._k
    if k == 'a' or k == 'o':
        if not expr.terms:
            out.append(_header(_lib.PLAN_CONST, 0, 0))
            return
        if k == 'a' and not getattr(expr, '_planned', False):
            expr._plan_orders()
            expr._planned = True
        out.append(_header(_lib.PLAN_AND if k == 'a' else _lib.PLAN_OR, len(expr.terms)))
        for t in expr.terms:
            _walk(t, out, links, False)
    elif k == 'x':
        out.append(_header(_lib.PLAN_NOT, 1))
        _walk(expr.term, out, links, False)
    elif k == 'l':
        if any(t._k == 't' for t in expr.targets):
            # Link._typed_variable_matched (:491-500); at the root its answer
            # after a failing target is observable: the host path keeps that
            if root:
                raise _Unsupported()
            if any(t._k in ('v', 'tv') for t in expr.targets):
                out.append(_header(_lib.PLAN_CONST, 0, 0))
                return
            out.append(_header(_lib.PLAN_TVM, len(expr.targets)))
            for t in expr.targets:
                _walk(t, out, links, False)
            return
        if not expr.ordered:
            raise _Unsupported()
        links.append((len(out), expr, _link_signature(expr)))
        out.append(None)
    elif k == 't':
        if not expr.ordered or root:
            raise _Unsupported()
        links.append((len(out), expr, ('t', expr.link_type, tuple((v.name, v.type) for v in expr.targets))))
        out.append(None)
    elif k == 'n' or k == 'v':
        links.append((len(out), expr, None))
        out.append(None)
    else:
        raise _Unsupported()


class _NoShape(Exception):
    pass


def _shape(expr, nodes):
    """Structure key of `expr` with its nodes' names left out (the nodes are
    appended to `nodes` in walk order).  Raises _NoShape for what a
    parameterised plan cannot carry: a Link whose targets are all grounded
    (its record is link_exists of those very handles) and the unordered link
    types (their scan keys are sorted by handle)."""
    k = expr._k
    if k == 'n':
        nodes.append(expr)
        return expr.atom_type
    if k == 'v':
        return ('v', expr.name)
    if k == 'tv':
        return ('tv', expr.name, expr.type)
    if k == 'l':
        if expr.atom_type in UNORDERED_LINK_TYPES or all(t._k == 'n' for t in expr.targets):
            raise _NoShape()
        return ('l', expr.atom_type, expr.ordered, tuple([_shape(t, nodes) for t in expr.targets]))
    if k == 't':
        return ('t', expr.link_type, expr.ordered, tuple([(v.name, v.type) for v in expr.targets]))
    if k == 'x':
        return ('x', _shape(expr.term, nodes))
    if k == 'a' or k == 'o':
        return (k, tuple([_shape(t, nodes) for t in expr.terms]))
    raise _NoShape()


def _node_ids(db, nodes):
    """Atom ids of `nodes` (one batched lookup), or None if one is not a node
    of the KB (its term's record would then be a constant)."""
    hs = [n.get_handle(db) for n in nodes]
    out = []
    for aid, cat, _ in db._resolve(hs):
        if aid < 0 or cat != 1:
            return None
        out.append(aid)
    return out


_UNORDERED = frozenset(UNORDERED_LINK_TYPES)


def _lower(expr, db, no_overload):
    """The das_plan_node_t array (51 u32 words per node) of `expr`, or None.

    A query shape seen before (the same tree with other node names, e.g. a
    fresh gene anchor) is answered from the shape cache: its words with each
    node's atom id patched into the scan / index-join target slots it
    occupies -- one batched handle lookup, no re-lowering.  Otherwise Link
    records are cached per (index, signature), so a repeated query re-lowers
    only the links whose anchors changed; their handles are resolved in one
    batched lookup."""
    shapes = db.__dict__.setdefault('_plan_shapes', {})
    if shapes and _assign is not None and hasattr(_assign, "plan_words"):
        # the shape-cache hit below, in C (das_amd/csrc/pyassign.c plan_words);
        # None: take the Python path
        nh, hc = getattr(db, "_node_handles", None), getattr(db, "_handle_cache", None)
        if type(nh) is dict and type(hc) is dict:
            w = _assign.plan_words(expr, shapes, no_overload, nh, hc, getattr(db, "_node_dir", None),
                                   _UNORDERED, db.get_node_handle)
            if w is not None:
                return w
    nodes = []
    try:
        skey = (no_overload, _shape(expr, nodes))
    except _NoShape:
        skey = None
    if skey is not None:
        hit = shapes.get(skey)
        if hit is not None:
            ids = _node_ids(db, nodes) if nodes else []
            if ids is not None:
                words, patches = hit
                w = words.copy()
                for wi, k in patches:
                    w[wi] = ids[k]
                return w
    out, links = [], []
    try:
        _walk(expr, out, links)
    except _Unsupported:
        return None
    cache = db.__dict__.setdefault('_plan_records', {})
    if len(cache) > (1 << 16):
        cache.clear()
    todo = []
    for pos, e, sig in links:
        if sig is not None:
            r = cache.get((no_overload, sig))
            if r is not None:
                out[pos] = r
                continue
        todo.append((pos, e, sig))
    if todo:
        try:
            _resolve(todo, out, cache, db, no_overload)
        except _Unsupported:
            return None
    words = np.frombuffer(b"".join(out), dtype=np.uint32)
    if skey is not None and (not nodes or _node_ids(db, nodes) is not None):
        # every node exists: each Link record's grounded targets are these
        # nodes' ids at fixed word offsets (scan targets at 7 + p, the index
        # join's at 30 + p; include/das_mi355x.h das_plan_node_t)
        ordinal = {id(n): i for i, n in enumerate(nodes)}
        patches = []
        for pos, e, _ in links:
            if e._k != 'l':
                continue
            base = _WORDS * pos
            if int(words[base]) != _lib.PLAN_LINK:
                continue
            for p, t in enumerate(e.targets):
                if t._k == 'n':
                    patches.append((base + 7 + p, ordinal[id(t)]))
                    if int(words[base + 4]):
                        patches.append((base + 30 + p, ordinal[id(t)]))
        if len(shapes) > (1 << 12):
            shapes.clear()
        shapes[skey] = (words, patches)
    return words


def _resolve(todo, out, cache, db, no_overload):
    """Records of the leaves _lower found no cached record for."""
    if todo:
        nodes = [t for _, e, _ in todo for t in (e.targets if e._k == 'l' else [e] if e._k == 'n' else [])
                 if t._k == 'n']
        if nodes:
            db.prefetch_handles([n.get_handle(db) for n in nodes])
        for pos, e, sig in todo:
            if e._k == 'n':
                out[pos] = _header(_lib.PLAN_CONST, 0, 1 if e.matched(db, None) else 0)
            elif e._k == 'v':
                out[pos] = _header(_lib.PLAN_CONST, 0, 1)
            elif e._k == 't':
                out[pos] = cache[(no_overload, sig)] = _template_record(e, db, no_overload)
            else:
                out[pos] = cache[(no_overload, sig)] = _link_record(e, db, no_overload)


def _try_plan(expr, db, answer):
    """Evaluates `expr` with one das_plan_execute call when it can; returns
    its matched() result, or None for the per-operator path."""
    if os.environ.get("DAS_PLAN") == "0" or answer.negation:
        return None
    if type(db) is not HipDB:
        # a sharded DB (das_amd.parallel.ShardedDB) plans across its GPUs
        sharded = getattr(db, "plan_sharded", None)
        return sharded(expr, answer) if sharded is not None else None
    if db._stale and db.touches_stale(expr):
        return None                             # stale_pattern_keys: the per-operator path adds them
    no_overload = bool(CONFIG['no_overload'])
    key = (db.generation, no_overload)          # generation: unique per load, any HipDB
    cached = getattr(expr, '_plan', None)
    if cached is None or cached[0] != key:
        cached = (key, _lower(expr, db, no_overload))
        expr._plan = cached
    nodes = cached[1]
    if nodes is None:
        return None
    matched, negation, tables = db.ctx.plan_execute(nodes, len(nodes) // 51, no_overload)
    answer._set(db, Relation(tables))
    answer.negation = negation
    return matched


def matched_many(db, exprs, tag=None):
    """[(matched, answer)] of independent expressions, each as
    `expr.matched(db, answer)` with a fresh PatternMatchingAnswer would give.
    On one HipDB the plannable ones go to ONE das_plan_execute_many call (the
    GPU runs an expression's fused chain while the host prepares the next);
    the rest, and every expression on other DBs, are evaluated one by one.
    tag = (index, name): the kernel scopes of exprs[index] are recorded as
    "<scope>@<name>" (das_prof_tag_plan; bench.py's in-step And join)."""
    res = [None] * len(exprs)
    batch = []
    if type(db) is HipDB and os.environ.get("DAS_PLAN") != "0":
        no_overload = bool(CONFIG['no_overload'])
        key = (db.generation, no_overload)
        for i, e in enumerate(exprs):
            # the operators whose matched() tries a whole-expression plan
            # first, with its prelude (And.matched / Or.matched / Not.matched)
            # (a root Link is one LINK / CONST plan node: Link.matched's scan
            # or link_exists, :502-538 -- batched too, e.g. bench Q1)
            if type(e) is Link:
                if not e.ordered:
                    continue
            elif type(e) not in (And, Or, Not) or (type(e) is not Not and not e.terms):
                continue
            if db._stale and db.touches_stale(e):
                continue
            cached = getattr(e, '_plan', None)
            if cached is None or cached[0] != key:
                cached = (key, _lower(e, db, no_overload))
                e._plan = cached
            if cached[1] is not None:
                batch.append((i, cached[1]))
        if batch:
            at = next((k for k, (i, _) in enumerate(batch) if tag and i == tag[0]), None)
            if at is not None:
                db.ctx.prof_tag_plan(at, tag[1])
            try:
                outs = db.ctx.plan_execute_many([(w, len(w) // _WORDS) for _, w in batch], no_overload)
            finally:
                if at is not None:
                    db.ctx.prof_tag_plan(None)
            for (i, _), (matched, negation, tables) in zip(batch, outs):
                ans = PatternMatchingAnswer()
                ans._set(db, Relation(tables))
                ans.negation = negation
                res[i] = (matched, ans)
    for i, e in enumerate(exprs):
        if res[i] is None:
            ans = PatternMatchingAnswer()
            tagged = tag is not None and i == tag[0] and type(db) is HipDB
            if tagged:
                db.ctx.prof_tag(tag[1])
            try:
                res[i] = (e.matched(db, ans), ans)
            finally:
                if tagged:
                    db.ctx.prof_tag(None)
    return res


# ---------------------------------------------------------------------------
# Answers
# ---------------------------------------------------------------------------
class PatternMatchingAnswer:

    def __init__(self):
        self._rel: Optional[Relation] = None
        self._db: Optional[HipDB] = None
        self._py = None
        self.negation: bool = False

    def __repr__(self):
        s = 'NOT\n' if self.negation else ''
        for a in self.assignments:
            s += str(a) + '\n'
        return s

    def _set(self, db, rel):
        self._db = db
        self._rel = rel
        self._py = None

    def _relation(self):
        if self._py is not None and self._rel is None:
            if self._py:
                raise NotImplementedError("host-built assignments cannot feed the device matcher")
            return Relation()
        return self._rel if self._rel is not None else Relation()

    def __len__(self):
        return len(self.assignments)

    @property
    def assignments(self):
        if self._py is None:
            self._py = _materialize(self._db, self._rel)
        return self._py

    @assignments.setter
    def assignments(self, value):
        self._py = set(value)
        self._rel = None

    def count(self) -> int:
        """Number of distinct assignments, without building Python objects
        (summed over ranks for a sharded DB)."""
        if self._py is not None and self._rel is None:
            return len(self._py)
        if self._db is None:
            return 0
        return self._db.rel_count(self._relation())


try:
    from .. import _assign          # C builder of the answer's Assignment objects (csrc/pyassign.c)
except ImportError:                 # not built: the same objects through assign() / freeze() below
    _assign = None


def _handle_strings(db, fetched):
    """One handle string per distinct atom id of the fetched tables: (lut,
    strs, fetched') with strs[lut[v]] = the 32-hex handle of value v of the
    (possibly re-coded) columns in fetched'.  Dense id ranges index a lookup
    table directly; a few values over a wide id range are re-coded to their
    rank among the distinct ids (no id-sized allocation)."""
    parts = [c.ravel() for _, c in fetched if c.size]
    if not parts:
        return np.zeros(1, np.uint32), [], fetched
    total = sum(p.size for p in parts)
    hi = int(max(int(p.max()) for p in parts))
    if hi < (1 << 27) and 8 * total >= hi:
        present = np.zeros(hi + 1, dtype=bool)
        for p in parts:
            present[p] = True
        ids = np.flatnonzero(present).astype(np.uint32)
        lut = np.zeros(hi + 1, dtype=np.uint32)
        lut[ids] = np.arange(ids.size, dtype=np.uint32)
        return lut, list(db.hex_of(ids)), fetched
    ids = np.unique(np.concatenate(parts))
    recoded = [(t, np.searchsorted(ids, c).astype(np.uint32)) for t, c in fetched]
    return np.arange(ids.size, dtype=np.uint32), list(db.hex_of(ids)), recoded


def _materialize(db, rel, limit=None):
    """answer.assignments: the reference's set of Assignment objects for the
    device relation (lazy: built when a caller reads it).  `limit`: only the
    first `limit` rows (bench.py's materialisation rate on large answers)."""
    out = set()
    if rel is None or not rel:
        return out
    fetched = []
    for t in db.rel_local_tables(rel):
        if limit is not None:
            if limit <= 0:
                break
            fetched.append((t, t.fetch(0, limit)))
            limit -= fetched[-1][1].shape[1]
        else:
            fetched.append((t, t.fetch()))
    fast = _assign is not None and all(t.kind != _lib.TABLE_COMPOSITE for t, _ in fetched)
    if fast:
        lut, strs, fetched = _handle_strings(db, fetched)
        # the objects hold strings and frozensets only (no reference cycles):
        # the cyclic collector's passes over millions of young objects would
        # cost more than building them
        gc_on = gc.isenabled()
        gc.disable()
        try:
            for t, cols in fetched:
                if not t.nrows:
                    continue
                names = tuple(_var_name(v) for v in t.vars)
                cls, kind = (OrderedAssignment, 0) if t.kind == _lib.TABLE_ORDERED else (UnorderedAssignment, 1)
                _assign.add_rows(out, cls, kind, names, np.ascontiguousarray(cols, np.uint32), lut, strs)
        finally:
            if gc_on:
                gc.enable()
        return out
    for t, cols in fetched:
        names = [_var_name(v) for v in t.vars]
        hexcols = [db.hex_of(c) for c in cols]
        if t.kind == _lib.TABLE_COMPOSITE:
            o_cols = [k for k, m in enumerate(t.members) if m < 0]
            m_cols = {}
            for k, m in enumerate(t.members):
                if m >= 0:
                    m_cols.setdefault(m, []).append(k)
        for i in range(cols.shape[1] if cols.ndim == 2 else 0):
            if t.kind == _lib.TABLE_ORDERED:
                a = _ordered(names, hexcols, range(len(names)), i)
            elif t.kind == _lib.TABLE_UNORDERED:
                a = _unordered(names, hexcols, range(len(names)), i)
            else:
                us = [_unordered(names, hexcols, m_cols[m], i) for m in sorted(m_cols)]
                a = CompositeAssignment(us[0])
                a.unordered_mappings = us
                a.ordered_mapping = _ordered(names, hexcols, o_cols, i) if o_cols else None
                a._recompute_hash()
            out.add(a)
    return out


def _ordered(names, hexcols, cols, i):
    a = OrderedAssignment()
    for k in cols:
        a.assign(names[k], hexcols[k][i])
    a.freeze()
    return a


def _unordered(names, hexcols, cols, i):
    a = UnorderedAssignment()
    for k in cols:
        a.assign(names[k], hexcols[k][i])
    a.freeze()
    return a


# ---------------------------------------------------------------------------
# Expressions
# ---------------------------------------------------------------------------
class LogicalExpression(ABC):
    # class tag for the hot lowering / planning walks (isinstance through
    # ABCMeta costs ~0.5 us per call): 'n' Node, 'l' Link, 'v' Variable,
    # 'tv' TypedVariable, 't' LinkTemplate, 'a' And, 'o' Or, 'x' Not
    _k = ''

    @abstractmethod
    def matched(self, db: DBInterface, answer: PatternMatchingAnswer) -> bool: ...

    def __repr__(self):
        return '<LogicalExpression>'


class Atom(LogicalExpression, ABC):

    def __init__(self, atom_type: str):
        self.atom_type = atom_type
        self.handle = None

    def __repr__(self):
        return f'{self.atom_type}'

    @abstractmethod
    def get_handle(self, db: DBInterface) -> str: ...


class Node(Atom):
    _k = 'n'

    def __init__(self, node_type: str, node_name: str):
        super().__init__(node_type)
        self.name = node_name

    def __repr__(self):
        return f'<{super().__repr__()}: {self.name}>'

    def get_handle(self, db: DBInterface) -> str:
        if not self.handle:
            self.handle = db.get_node_handle(self.atom_type, self.name)
        return self.handle

    def matched(self, db: DBInterface, answer: PatternMatchingAnswer) -> bool:
        return db.node_exists(self.atom_type, self.name)


def _variables_last(t1, t2):
    """Link.__init__'s comparator for unordered links (pattern_matcher.py:442-448)."""
    if isinstance(t1, Variable):
        return 1
    if isinstance(t2, Variable):
        return -1
    return 0


class Link(Atom):
    _k = 'l'

    def __init__(self, link_type: str, targets: List[Atom], ordered: bool):
        assert not any(isinstance(target, TypedVariable) for target in targets)
        super().__init__(link_type)
        self.ordered = ordered
        self.targets = targets if ordered else sorted(targets, key=cmp_to_key(_variables_last))

    def __repr__(self):
        return f'<{super().__repr__()}: {self.targets}>'

    def get_handle(self, db: DBInterface) -> str:
        if not self.handle:
            hs = [t.get_handle(db) for t in self.targets]
            if any(h is None for h in hs):
                return None
            self.handle = db.get_link_handle(self.atom_type, hs)
        return self.handle

    def _typed_variable_matched(self, db, answer) -> bool:
        if any(isinstance(t, Variable) for t in self.targets):
            return False
        return all(t.matched(db, answer) for t in self.targets)

    def matched(self, db: DBInterface, answer: PatternMatchingAnswer) -> bool:
        db = _hip(db)
        if any(isinstance(t, LinkTemplate) for t in self.targets):
            return self._typed_variable_matched(db, answer)
        if not all(t.matched(db, answer) for t in self.targets):
            return False
        handles = [t.get_handle(db) for t in self.targets]
        if WILDCARD not in handles:
            return db.link_exists(self.atom_type, handles)
        var_ids = [_vid(t.name) if isinstance(t, Variable) else None for t in self.targets]
        hint = getattr(self, '_order_var', None)
        if hint is not None:
            rel = db.match_link(self.atom_type, handles, var_ids, self.ordered, CONFIG['no_overload'],
                                order_var=_vid(hint))
        else:
            rel = db.match_link(self.atom_type, handles, var_ids, self.ordered, CONFIG['no_overload'])
        found = db.rel_nonempty(rel)
        if db.tuple_targets and not self.ordered and found and any(v is None for v in var_ids):
            # reference DB path: list.remove on a tuple (pattern_matcher.py:484)
            raise AttributeError("'tuple' object has no attribute 'remove'")
        answer._set(db, rel)
        return found


    def _index_join(self, db, acc):
        """rel_join(acc, this term's relation) through the pattern index, or
        None when the shape does not allow it (And.matched scans instead)."""
        if not self.ordered or CONFIG['no_overload'] or not hasattr(db, 'rel_index_join'):
            return None
        if getattr(db, '_stale', None) and db.touches_stale(self):
            return None                         # the scan adds the stale entries (HipDB.match_link)
        if not all(isinstance(t, Variable) or type(t) is Node for t in self.targets):
            return None
        if any(isinstance(t, TypedVariable) for t in self.targets):
            return None
        handles = [t.get_handle(db) for t in self.targets]
        var_ids = [_vid(t.name) if isinstance(t, Variable) else None for t in self.targets]
        return db.rel_index_join(acc, self.atom_type, handles, var_ids)


class Variable(Atom):
    _k = 'v'

    def __init__(self, variable_name: str):
        super().__init__('ANY')
        self.name = variable_name

    def __repr__(self):
        return f'{self.name}'

    def get_handle(self, db: DBInterface) -> str:
        return WILDCARD

    def matched(self, db: DBInterface, answer: PatternMatchingAnswer) -> bool:
        return True


class TypedVariable(Variable):
    _k = 'tv'

    def __init__(self, variable_name: str, variable_type: str):
        super().__init__(variable_name)
        self.type = variable_type

    def __repr__(self):
        return f'{self.name}: {self.type}'


class LinkTemplate(LogicalExpression):
    _k = 't'

    def __init__(self, link_type: str, targets: List[TypedVariable], ordered: bool):
        assert all(isinstance(target, TypedVariable) for target in targets)
        self.link_type = link_type
        self.targets = targets
        self.ordered = ordered
        self.handle = None

    def __repr__(self):
        return f'<{self.link_type}: {self.targets}>'

    def matched(self, db: DBInterface, answer: PatternMatchingAnswer) -> bool:
        db = _hip(db)
        rel = db.match_template(self.link_type, [v.type for v in self.targets],
                                [_vid(v.name) for v in self.targets], self.ordered, CONFIG['no_overload'])
        answer._set(db, rel)
        return db.rel_nonempty(rel)


class Not(LogicalExpression):
    _k = 'x'

    def __init__(self, term: LogicalExpression):
        self.term = term

    def __repr__(self):
        return f'NOT({self.term})'

    def matched(self, db: DBInterface, answer: PatternMatchingAnswer) -> bool:
        r = _try_plan(self, db, answer)
        if r is not None:
            return r
        self.term.matched(db, answer)
        answer.negation = not answer.negation
        return True


def _nodes_of(expr, out):
    k = expr._k
    if k == 'n':
        out.append(expr)
    elif k == 'l':
        for t in expr.targets:
            _nodes_of(t, out)
    elif k == 'x':
        _nodes_of(expr.term, out)
    elif k == 'a' or k == 'o':
        for t in expr.terms:
            _nodes_of(t, out)
    return out


def _prefetch(expr, db):
    """One batched handle lookup for every grounded node under an And / Or
    (instead of one device round trip per node_exists)."""
    nodes = getattr(expr, '_nodes', None)
    if nodes is None:
        nodes = expr._nodes = _nodes_of(expr, [])
    if nodes:
        db.prefetch_handles([n.get_handle(db) for n in nodes])


class Or(LogicalExpression):
    _k = 'o'

    def __init__(self, terms: List[LogicalExpression]):
        self.terms = terms

    def __repr__(self):
        return f'OR({self.terms})'

    def matched(self, db: DBInterface, answer: PatternMatchingAnswer) -> bool:
        db = _hip(db)
        if not self.terms:
            return False
        r = _try_plan(self, db, answer)
        if r is not None:
            return r
        _prefetch(self, db)
        union = None
        any_matched = False
        negated = [t for t in self.terms if isinstance(t, Not)]
        for term in self.terms:
            if isinstance(term, Not):
                continue
            sub = PatternMatchingAnswer()
            if not term.matched(db, sub):
                continue
            any_matched = True
            rel = sub._relation()
            if db.rel_nonempty(rel):
                union = rel if union is None else db.rel_union(union, rel)
        union = union if union is not None else db.rel_empty()
        if negated:
            sub = PatternMatchingAnswer()
            And([t.term for t in negated]).matched(db, sub)
            answer._set(db, db.rel_minus(sub._relation(), union))
            answer.negation = True
        else:
            answer._set(db, union)
        return any_matched


class And(LogicalExpression):
    _k = 'a'

    def __init__(self, terms: List[LogicalExpression]):
        self.terms = terms

    def __repr__(self):
        return f'AND({self.terms})'

    def post_process(self, assignment) -> Assignment:
        return assignment

    def _plan_orders(self):
        """Scan-order hints: each positive Link term is asked for its rows
        sorted by its first variable that another term also binds (the join
        key), so joins probe sorted keys.  Answers are unchanged."""
        def names(t):
            return [x.name for x in t.targets if x._k == 'v' or x._k == 'tv'] if t._k == 'l' else []
        vs = [set(names(t)) for t in self.terms]
        for i, t in enumerate(self.terms):
            if t._k != 'l':
                continue
            others = set().union(*(v for j, v in enumerate(vs) if j != i)) if len(vs) > 1 else set()
            t._order_var = next((n for n in names(t) if n in others), None)

    def matched(self, db: DBInterface, answer: PatternMatchingAnswer) -> bool:
        db = _hip(db)
        if not self.terms:
            return False
        # (the scan-order hints: _walk sets them when it lowers the And, and a
        # query shape seen before needs none)
        r = _try_plan(self, db, answer)
        if r is not None:
            return r
        if not getattr(self, '_planned', False):
            self._plan_orders()
            self._planned = True
        _prefetch(self, db)
        acc = None
        forbidden = []
        for term in self.terms:
            if acc is not None and isinstance(term, Link) and db.rel_nonempty(acc):
                # index join (das_index_join): the term's rows are looked up
                # from the running result's keys instead of scanned; an empty
                # result takes the scan path, which tells a failing term
                # (And -> False) from an empty join (reset-on-empty)
                rel = term._index_join(db, acc)
                if rel is not None and db.rel_nonempty(rel):
                    acc = rel
                    continue
            sub = PatternMatchingAnswer()
            if not term.matched(db, sub):
                return False
            rel = sub._relation()
            if not db.rel_nonempty(rel):
                continue
            if sub.negation:
                forbidden.append(rel)
                continue
            # reset-on-empty (pattern_matcher.py:725-729): an empty running
            # result takes the next term's assignments as they are
            acc = rel if acc is None or not db.rel_nonempty(acc) else db.rel_join(acc, rel)
        if acc is None:
            acc = db.rel_empty()
        for f in forbidden:
            if db.rel_nonempty(acc):
                acc = db.rel_antijoin(acc, f)
        acc = db.rel_normalize(acc)
        answer._set(db, acc)
        return db.rel_nonempty(acc)
