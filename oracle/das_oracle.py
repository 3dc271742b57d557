"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference (tanksha/das @ 2025-02-09) for the query hot
path: the handle function, the DB-path index semantics and the pattern-matcher
evaluation.  It exists to CHECK the MI355X product (`das_amd/`); only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import it.
The product never imports, links or executes anything under `oracle/`.

Parity pinning: every function here is checked against golden fixtures that
were produced by running the reference itself in the build container
(`tests/golden/make_golden.py`: reference MettaYacc / CanonicalParser loaders +
RedisMongoDB adapter over in-memory Redis/Mongo stand-ins, and the reference
StubDB), and against the known-answer handles printed in the reference
(`scripts/service_regression_test.sh:34,43`, `service/README.md:290-378`).

Data model (a restatement, not the reference's class hierarchy):
  * an ordered row      ("O", ((var, val), ...))             sorted items
  * an unordered row    ("U", frozenset(vars), (val, ...))     sorted values
  * a composite row     ("C", O-row | None, [U-row, ...])      member order kept
Rows are hashable by `ident()` which reproduces what the reference's
`Assignment.__hash__`/`__eq__` treat as equal (pattern_matcher.py:41-51, 89,
190, 279-286, 307-314).
"""
import hashlib
import json
import re
from collections import Counter
from functools import cmp_to_key

WILDCARD = "*"                                   # db_interface.py:4
UNORDERED_LINK_TYPES = ["Similarity", "Set"]     # db_interface.py:5
CONFIG = {"no_overload": False}                  # pattern_matcher.py:16-19


# ---------------------------------------------------------------------------
# Handles — expression_hasher.py:9-35 (hashlib.md5 is the reference's own dep)
# ---------------------------------------------------------------------------

def md5hex(text):
    return hashlib.md5(text.encode("utf-8")).hexdigest()


def named_type_hash(name):
    return md5hex(name)


def terminal_hash(named_type, name):
    return md5hex(" ".join([named_type, name]))


def composite_hash(base):
    if isinstance(base, str):
        return base
    if len(base) == 1:
        return base[0]
    return md5hex(" ".join(base))     # TypeError for nested lists, as the reference


def expression_hash(type_hash, elements):
    return composite_hash([type_hash, *elements])


# ---------------------------------------------------------------------------
# KB: what the reference stores (Mongo docs).  Built either from golden atom
# tables or from loader arrays (das_amd.loader.AtomArrays layout) by hashing.
# ---------------------------------------------------------------------------

class KB:
    def __init__(self):
        self.nodes = {}      # handle -> (type, name)
        self.links = {}      # handle -> (type, [targets], composite_type_hash)

    @classmethod
    def from_tables(cls, nodes, links):
        kb = cls()
        for h, t, n in nodes:
            kb.nodes[h] = (t, n)
        for h, t, targets, ct in links:
            kb.links[h] = (t, list(targets), ct)
        return kb

    @classmethod
    def from_arrays(cls, arrays):
        """Hash an AtomArrays bundle the reference way (canonical_parser.py:242-305,
        base_yacc.py:83-161): leaves are md5(string); an expression's handle is
        composite_hash([md5(type), child handles...]) and its composite type is
        composite_hash([child composite types...])."""
        kb = cls()
        leaf_hash = [md5hex(s) for s in arrays.leaf_strings()]
        n_leaf = len(leaf_hash)
        ctype_leaf = arrays.leaf_ctype
        h = leaf_hash + [None] * arrays.n_expr
        ct = [leaf_hash[ctype_leaf[i]] for i in range(n_leaf)] + [None] * arrays.n_expr
        order = sorted(range(arrays.n_expr), key=lambda j: arrays.expr_level[j])
        for j in order:
            ch = arrays.children(j)
            h[n_leaf + j] = composite_hash([h[c] for c in ch])
            if arrays.expr_ctype_leaf[j] >= 0:
                ct[n_leaf + j] = leaf_hash[arrays.expr_ctype_leaf[j]]
            else:
                ct[n_leaf + j] = composite_hash([ct[c] for c in ch])
        for i in range(n_leaf):
            if arrays.leaf_kind[i] == 1:
                kb.nodes[h[i]] = (arrays.leaf_string(arrays.leaf_ctype[i]), arrays.node_name(i))
        for j in range(arrays.n_expr):
            if arrays.expr_kind[j] == 1:
                ch = arrays.children(j)
                kb.links.setdefault(h[n_leaf + j], (arrays.leaf_string(ch[0]), [h[c] for c in ch[1:]],
                                                     ct[n_leaf + j]))
        return kb

    def node_table(self):
        return sorted([h, t, n] for h, (t, n) in self.nodes.items())

    def link_table(self):
        return sorted([h, t, list(tg), ct] for h, (t, tg, ct) in self.links.items())


# ---------------------------------------------------------------------------
# DB-path semantics — redis_mongo_db.py:204-279 over the index families of
# canonical_parser.py:132-183 / parser_threads.py:171-253.
# ---------------------------------------------------------------------------

def _pattern_keys(type_hash, elements):
    """Pattern-key families, as tuples instead of md5(" ".join(...))."""
    keys = {(WILDCARD, *elements)}
    arity = len(elements)
    if 1 <= arity <= 3:
        for mask in range(1 << (arity + 1)):
            key = [WILDCARD if mask & 1 else type_hash]
            key += [WILDCARD if mask >> (i + 1) & 1 else e for i, e in enumerate(elements)]
            if mask != 0:
                keys.add(tuple(key))
    return keys


def keyspace_lines(kb):
    """The key-value files CanonicalParser writes before populating Redis
    (canonical_parser.py:119-183 via key_value_file.py:8-16), as sorted line
    lists: outgoing / incoming sets, patterns (the reference's key list per
    arity, including the [*, e...] key it appends twice for arities 1-3),
    templates (composite type hash and named type hash) and names."""
    out = {"outgoing_set": [], "incomming_set": [], "patterns": [], "templates": [], "names": []}
    for h, (t, targets, ct) in kb.links.items():
        for x in targets:                                     # :139-143
            out["outgoing_set"].append(f"{h}\t{x}")
            out["incomming_set"].append(f"{x}\t{h}")
        th = named_type_hash(t)
        arity = len(targets)
        keys = [[WILDCARD, *targets]]                         # :145
        if 1 <= arity <= 3:                                   # :146-175, every mask with >= 1 wildcard
            for mask in range(1, 1 << (arity + 1)):
                keys.append([WILDCARD if mask & 1 else th] +
                            [WILDCARD if mask >> (i + 1) & 1 else e for i, e in enumerate(targets)])
        value = "\t".join([h, *targets])
        for k in keys:                                        # :176-177
            out["patterns"].append(f"{composite_hash(k)}\t{value}")
        out["templates"].append(f"{ct}\t{value}")            # :179-180
        out["templates"].append(f"{th}\t{value}")
    for h, (_, name) in kb.nodes.items():                     # :119-121
        out["names"].append(f"{h}\t{name}")
    return {k: sorted(v) for k, v in out.items()}


class RedisMongoSemantics:
    """Restatement of RedisMongoDB over an in-memory KB."""

    def __init__(self, kb, pattern_black_list=(), tuple_targets=False, stale_key_order=None):
        """pattern_black_list: named types whose links get no pattern keys
        (the intent of canonical_parser.py:144 / parser_threads.py:185).
        stale_key_order: the link handles in the order the reference's
        pattern-key loop walks them -- the loop never resets `keys` for a
        blacklisted link, so it is written under the previous link's keys
        (canonical_parser.py:177-178, parser_threads.py:218-219), and a
        blacklisted first link raises UnboundLocalError; given the order,
        this restates that behaviour exactly."""
        self.kb = kb
        self.tuple_targets = tuple_targets
        self.patterns = {}
        self.templates = {}
        self.collection = {}
        for h, (t, targets, ct) in kb.links.items():
            a = len(targets)
            self.collection[h] = "1" if a == 1 else ("2" if a == 2 else "N")
            value = (h, tuple(targets))
            if stale_key_order is None and t not in pattern_black_list:
                for k in _pattern_keys(named_type_hash(t), targets):
                    self.patterns.setdefault(k, set()).add(value)
            self.templates.setdefault(ct, set()).add(value)
            self.templates.setdefault(named_type_hash(t), set()).add(value)
        if stale_key_order is not None:
            keys = None
            for h in stale_key_order:
                t, targets, _ = kb.links[h]
                if t not in pattern_black_list:
                    keys = _pattern_keys(named_type_hash(t), targets)
                elif keys is None:
                    raise UnboundLocalError("local variable 'keys' referenced before assignment")
                for k in keys:
                    self.patterns.setdefault(k, set()).add((h, tuple(targets)))

    def _fmt(self, values):
        if self.tuple_targets:
            return [(h, tuple(t)) for h, t in values]
        return [(h, list(t)) for h, t in values]

    def _exists(self, handle, arity):
        if arity == 0:
            return handle in self.kb.nodes
        want = "1" if arity == 1 else ("2" if arity == 2 else "N")
        return self.collection.get(handle) == want

    def node_exists(self, node_type, node_name):
        return terminal_hash(node_type, node_name) in self.kb.nodes

    def link_exists(self, link_type, targets):
        return self._exists(expression_hash(named_type_hash(link_type), targets), len(targets))

    def get_node_handle(self, node_type, node_name):
        return terminal_hash(node_type, node_name)

    def get_link_handle(self, link_type, targets):
        return expression_hash(named_type_hash(link_type), targets)

    def get_matched_links(self, link_type, targets):
        if link_type != WILDCARD and WILDCARD not in targets:
            h = self.get_link_handle(link_type, targets)
            return [h] if self._exists(h, len(targets)) else []
        type_hash = WILDCARD if link_type == WILDCARD else named_type_hash(link_type)
        if link_type in UNORDERED_LINK_TYPES:
            targets = sorted(targets)
        return self._fmt(self.patterns.get((type_hash, *targets), ()))

    def get_matched_type_template(self, template):
        hashed = [named_type_hash(t) if isinstance(t, str) else t for t in template]
        return self._fmt(self.templates.get(composite_hash(hashed), ()))

    def get_matched_type(self, link_type):
        return self._fmt(self.templates.get(named_type_hash(link_type), ()))

    def count_atoms(self):
        return (len(self.kb.nodes), len(self.kb.links))

    # per-atom metadata (the calls SimplePatternMiner.ipynb makes per link)
    def get_link_targets(self, link_handle):
        """redis_mongo_db.py:222-227 (`outgoing_set:<handle>`; Redis returns a
        set, the stored order is returned here)."""
        v = self.kb.links.get(link_handle)
        if v is None:
            raise ValueError(f"Invalid handle: {link_handle}")
        return list(v[1])

    def get_link_type(self, link_handle):
        """redis_mongo_db.py:316-321 (link_type_cache: KeyError when absent)."""
        return self.kb.links[link_handle][0]

    def get_node_type(self, node_handle):
        """redis_mongo_db.py:323-328 (node_type_cache)."""
        return self.kb.nodes[node_handle][0]

    def get_node_name(self, node_handle):
        """redis_mongo_db.py:281-285 (`names:<handle>`)."""
        v = self.kb.nodes.get(node_handle)
        if v is None:
            raise ValueError(f"Invalid handle: {node_handle}")
        return v[1]


class StubSemantics:
    """Restatement of StubDB (stub_db.py:8-188): readable handles, membership
    matching for Similarity/Set, every arity indexed."""

    def __init__(self, nodes, links):
        self.all_nodes = list(nodes)
        self.all_links = [list(l) for l in links]
        self.template_index = {}
        for link in self.all_links:
            key = [link[0]] + [self._split(t)[0] for t in link[1:]]
            self.template_index.setdefault(str(key), []).append(
                [self._link_handle(link[0], link[1:]), link[1:]])

    @staticmethod
    def _split(h):
        v = re.split("[<: >]", h)
        return (v[1], v[3])

    @staticmethod
    def _link_handle(t, targets):
        targets = list(targets)
        if t in ("Similarity", "Set"):
            targets.sort()
        return f"<{t}: {targets}>"

    def node_exists(self, t, n):
        return f"<{t}: {n}>" in self.all_nodes

    def link_exists(self, t, targets):
        h = self._link_handle(t, targets)
        return any(self._link_handle(l[0], l[1:]) == h for l in self.all_links)

    def get_node_handle(self, t, n):
        h = f"<{t}: {n}>"
        return h if h in self.all_nodes else None

    def get_link_handle(self, t, targets):
        for link in self.all_links:
            if link[0] == t and len(targets) == len(link) - 1:
                if t == "Similarity":
                    if all(x in targets for x in link[1:]):
                        return self._link_handle(t, link[1:])
                elif t == "Inheritance":
                    if all(targets[i] == link[i + 1] for i in range(len(targets))):
                        return self._link_handle(t, targets)
                else:
                    raise ValueError(f"Invalid link type: {t}")
        return None

    def get_matched_links(self, t, targets):
        out = []
        for link in self.all_links:
            if len(targets) != len(link) - 1 or link[0] != t:
                continue
            if t in ("Similarity", "Set"):
                if all(x == WILDCARD or x in link[1:] for x in targets):
                    out.append([self._link_handle(t, link[1:]), link[1:]])
            elif t in ("Inheritance", "List"):
                if all(targets[i] in (WILDCARD, link[i + 1]) for i in range(len(targets))):
                    out.append([self._link_handle(t, link[1:]), link[1:]])
            else:
                raise ValueError(f"Invalid link type: {t}")
        return out

    def get_matched_type_template(self, template):
        assert len(template) == 3
        return [[h, list(tg)] for h, tg in self.template_index.get(str(template), [])]


# ---------------------------------------------------------------------------
# Assignment algebra — pattern_matcher.py:31-368, restated over tuples.
# ---------------------------------------------------------------------------

def o_row(mapping):
    return ("O", tuple(sorted(mapping.items())))


def u_row(vars_, values):
    return ("U", frozenset(vars_), tuple(sorted(values)))


def ident(row):
    """Set identity (pattern_matcher.py:41-51): what two equal-hash rows share."""
    if row[0] in ("O", "U"):
        return row
    _, o, us = row
    parity = Counter(us)
    odd = frozenset(u for u, c in parity.items() if c % 2)
    if o is not None and not odd:
        return o
    return ("C", None if o is None else o[1], odd)


def canon_json(row):
    """The canonical identity in the golden-fixture JSON layout."""
    i = ident(row)
    if i[0] == "O":
        return ["O", [list(x) for x in i[1]]]
    if i[0] == "U":
        return ["U", sorted(i[1]), list(i[2])]
    o = None if i[1] is None else [list(x) for x in i[1]]
    members = sorted(json.dumps(["U", sorted(u[1]), list(u[2])]) for u in i[2])
    return ["C", o, [json.loads(m) for m in members]]


class RowSet:
    """Python-set semantics keyed by ident(): the first inserted row is kept."""

    def __init__(self, rows=()):
        self.d = {}
        for r in rows:
            self.add(r)

    def add(self, r):
        self.d.setdefault(ident(r), r)

    def update(self, rows):
        for r in rows:
            self.add(r)

    def __iter__(self):
        return iter(list(self.d.values()))

    def __len__(self):
        return len(self.d)

    def __bool__(self):
        return bool(self.d)

    def minus(self, other):
        return RowSet(r for k, r in self.d.items() if k not in other.d)


EQUAL, INCOMPATIBLE, FIRST_COVERS_SECOND, SECOND_COVERS_FIRST, NO_COVERING = range(5)


def _o_compat(a, b):      # evaluate_compatibility, pattern_matcher.py:141-153
    if a[1] == b[1]:
        return EQUAL
    ma, mb = dict(a[1]), dict(b[1])
    for v in set(ma) & set(mb):
        if ma[v] != mb[v]:
            return INCOMPATIBLE
    if set(mb) < set(ma):
        return FIRST_COVERS_SECOND
    if set(ma) < set(mb):
        return SECOND_COVERS_FIRST
    return NO_COVERING


def _o_join(a, b):        # _join_ordered, pattern_matcher.py:119-139
    s = _o_compat(a, b)
    if s == INCOMPATIBLE:
        return None
    if s in (EQUAL, FIRST_COVERS_SECOND):
        return a
    if s == SECOND_COVERS_FIRST:
        return b
    merged = {}
    values = set()
    for var, val in list(a[1]) + list(b[1]):
        if var in merged:
            if merged[var] != val:
                return None
            continue
        if CONFIG["no_overload"] and val in values:
            return None
        merged[var] = val
        values.add(val)
    return o_row(merged)


def _u_contains_o(u, o):          # contains_ordered, :219-228
    cnt = Counter()
    for var, val in o[1]:
        if var not in u[1]:
            return False
        cnt[val] += 1
    have = Counter(u[2])
    return all(have[v] >= c for v, c in cnt.items())


def _u_covered_by_o(u, o):        # is_covered_by_ordered, :230-235
    sym = Counter({v: 1 for v in u[1]})
    val = Counter(u[2])
    for var, value in o[1]:
        sym[var] -= 1
        val[value] -= 1
    return all(c <= 0 for c in sym.values()) and all(c <= 0 for c in val.values())


def _u_contains_u(a, b):          # contains_unordered, :238-245
    if not b[1] <= a[1]:
        return False
    have = Counter(a[2])
    return all(have[v] >= c for v, c in Counter(b[2]).items())


def _u_compatible(a, b):          # compatible, :247-262 (all counts are 1)
    nsym = len(a[1] & b[1])
    nval = len(set(a[2]) & set(b[2]))
    return nval >= nsym


def _c_add_ordered(o_cur, us, o_new):      # _add_ordered_mapping, :316-327
    if o_new is None and o_cur is not None:
        raise AttributeError("'NoneType' object has no attribute 'frozen'")
    o = o_new if o_cur is None else _o_join(o_cur, o_new)
    if o_cur is not None and o is None:
        return None
    if o is None:
        return (None,) if us else None      # viability with no ordered mapping
    for u in us:
        if not _u_contains_o(u, o) and not _u_covered_by_o(u, o):
            return None
    return (o,)


def _c_add_unordered(o, us, u):            # _add_unordered_mapping, :329-336
    if o is not None and not _u_contains_o(u, o):
        return False
    if any(not _u_compatible(x, u) for x in us):
        return False
    us.append(u)
    return True


def _c_join(c, other):                     # CompositeAssignment.join, :341-351
    o, us = c[1], list(c[2])
    if other[0] == "O":
        r = _c_add_ordered(o, us, other)
        return None if r is None else ("C", r[0], us)
    if other[0] == "U":
        return ("C", o, us) if _c_add_unordered(o, us, other) else None
    r = _c_add_ordered(o, us, other[1])
    if r is None:
        return None
    o = r[0]
    for u in other[2]:
        if not _c_add_unordered(o, us, u):
            return None
    return ("C", o, us)


def join(a, b):
    """a.join(b) — OrderedAssignment.join :105-110, UnorderedAssignment.join
    :203-209, CompositeAssignment.join :341-351."""
    if a[0] == "O":
        if b[0] == "O":
            return _o_join(a, b)
        return join(b, a)
    if a[0] == "U":
        if b[0] == "C":
            return join(b, a)
        return _c_join(("C", None, [a]), b)
    return _c_join(a, b)


FAST_JOIN = True            # tests: False = the nested loop everywhere


def _ordered_hash_join(acc, rows):
    """The And fold's nested loop (:732-738) for ordered rows of one variable
    set per side: only pairs agreeing on the shared variables can join
    (_o_compat is INCOMPATIBLE otherwise, and join() returns None), so each
    row of `acc` is joined with the rows of `rows` that carry its shared
    values.  The same joined rows -- as a list in another order; the fold
    keeps only their set and their emptiness -- at the cost of the output
    instead of |acc| x |rows|.  None: not that case (the caller loops)."""
    if CONFIG["no_overload"] or not FAST_JOIN:
        return None
    rows = list(rows)
    if not acc or not rows or any(r[0] != "O" for r in acc) or any(r[0] != "O" for r in rows):
        return None
    va = {tuple(v for v, _ in r[1]) for r in acc}
    vb = {tuple(v for v, _ in r[1]) for r in rows}
    if len(va) != 1 or len(vb) != 1:
        return None
    shared = sorted(set(next(iter(va))) & set(next(iter(vb))))
    index = {}
    for b in rows:
        m = dict(b[1])
        index.setdefault(tuple(m[v] for v in shared), []).append(b)
    out = []
    for a in acc:
        m = dict(a[1])
        for b in index.get(tuple(m[v] for v in shared), ()):
            j = _o_join(a, b)
            if j is not None:
                out.append(j)
    return out


def _ordered_nested_join(acc, rows):
    """The And fold's nested loop (:732-738) itself -- every (acc, rows) pair
    evaluated, the reference's complexity -- for ordered rows, with each row's
    mapping dict and variable set built once per fold, as the reference's
    OrderedAssignment holds them from freeze() on (:58-70, 141-153): the
    pair's work is then the reference's evaluate_compatibility / _join_ordered
    (:119-153).  Same rows as join() per pair.  None: not that case."""
    if CONFIG["no_overload"]:
        return None
    rows = list(rows)
    if any(r[0] != "O" for r in acc) or any(r[0] != "O" for r in rows):
        return None
    pa = [(a, dict(a[1]), frozenset(a1 for a1, _ in a[1])) for a in acc]
    pb = [(b, dict(b[1]), frozenset(b1 for b1, _ in b[1])) for b in rows]
    out = []
    for a, ma, sa in pa:
        for b, mb, sb in pb:
            if a[1] == b[1]:                      # EQUAL
                out.append(a)
                continue
            ok = True
            for v in sa & sb:
                if ma[v] != mb[v]:                # INCOMPATIBLE
                    ok = False
                    break
            if not ok:
                continue
            if sb < sa:                           # FIRST_COVERS_SECOND
                out.append(a)
            elif sa < sb:                         # SECOND_COVERS_FIRST
                out.append(b)
            else:                                 # NO_COVERING: merged mapping
                m = dict(ma)
                m.update(mb)
                out.append(o_row(m))
    return out


def check_negation(a, tabu):
    """a.check_negation(tabu) — :112-117, :211-217, :353-362."""
    if a[0] == "O":
        if tabu[0] == "O":
            return _o_compat(a, tabu) not in (EQUAL, FIRST_COVERS_SECOND)
        if tabu[0] == "U":
            return not _u_covered_by_o(tabu, a)
        raise AttributeError("'CompositeAssignment' object has no attribute 'is_covered_by_ordered'")
    if a[0] == "U":
        if tabu[0] == "O":
            return not _u_contains_o(a, tabu)
        if tabu[0] == "U":
            return not _u_contains_u(a, tabu)
        return all(not _u_contains_u(a, u) for u in tabu[2])
    if tabu[0] == "O":
        return all(not _u_contains_o(u, tabu) for u in a[2])
    if tabu[0] == "U":
        return all(not _u_contains_u(u, tabu) for u in a[2])
    raise AttributeError("'CompositeAssignment' object has no attribute 'unordered_assignments'")


# ---------------------------------------------------------------------------
# Expression evaluation — pattern_matcher.py:386-748, over JSON query specs:
#   ["Node", type, name] ["Var", name] ["TVar", name, type]
#   ["Link", type, ordered, [targets]] ["Template", type, ordered, [tvars]]
#   ["Not", term] ["And", [terms]] ["Or", [terms]]
# ---------------------------------------------------------------------------

class Answer:
    def __init__(self):
        self.rows = RowSet()
        self.negation = False


def _is_var(spec):
    return spec[0] in ("Var", "TVar")


def _link_targets(spec):
    """Link.__init__ :439-453: unordered targets stable-sorted, variables last."""
    def cmp(t1, t2):
        if _is_var(t1):
            return 1
        if _is_var(t2):
            return -1
        return 0
    targets = spec[3]
    return list(targets) if spec[2] else sorted(targets, key=cmp_to_key(cmp))


def handle_of(spec, db):
    if spec[0] == "Node":
        return db.get_node_handle(spec[1], spec[2])
    if _is_var(spec):
        return WILDCARD
    if spec[0] == "Link":
        hs = [handle_of(t, db) for t in _link_targets(spec)]
        if any(h is None for h in hs):
            return None
        return db.get_link_handle(spec[1], hs)
    raise AttributeError(f"{spec[0]} has no handle")


def _assign_link(spec, targets_q, db, link_targets):
    """Link._assign_variables :466-489."""
    assert len(link_targets) == len(targets_q)
    if spec[2]:
        mapping, values = {}, set()
        for atom, h in zip(targets_q, link_targets):
            if _is_var(atom):
                name = atom[1]
                if name in mapping:
                    if mapping[name] != h:
                        return None
                else:
                    if CONFIG["no_overload"] and h in values:
                        return None
                    mapping[name] = h
                    values.add(h)
        return o_row(mapping)
    remaining = link_targets
    to_match = []
    for atom in targets_q:
        if _is_var(atom):
            to_match.append(atom)
        else:
            remaining.remove(handle_of(atom, db))   # AttributeError on tuples (A7)
    assert len(to_match) == len(remaining)
    names = [a[1] for a in to_match]
    if len(set(names)) != len(names):
        return None
    if len(set(remaining)) != len(remaining):
        return None
    return u_row(names, remaining)


def _assign_template(spec, link_targets):
    """LinkTemplate._assign_variables :591-601."""
    assert len(link_targets) == len(spec[3])
    names = [v[1] for v in spec[3]]
    if spec[2]:
        mapping, values = {}, set()
        for name, h in zip(names, link_targets):
            if name in mapping:
                if mapping[name] != h:
                    return None
            else:
                if CONFIG["no_overload"] and h in values:
                    return None
                mapping[name] = h
                values.add(h)
        return o_row(mapping)
    if len(set(names)) != len(names) or len(set(link_targets)) != len(link_targets):
        return None
    return u_row(names, link_targets)


def matched(spec, db, answer):
    kind = spec[0]
    if kind == "Node":                                       # :431-432
        return db.node_exists(spec[1], spec[2])
    if kind in ("Var", "TVar"):                              # :555-556, 573-574
        return True
    if kind == "Link":                                       # :502-538
        targets = _link_targets(spec)
        if any(t[0] == "Template" for t in targets):         # :491-500
            for t in targets:
                if _is_var(t):
                    return False
            return all(matched(t, db, answer) for t in targets)
        if not all(matched(t, db, answer) for t in targets):
            return False
        handles = [handle_of(t, db) for t in targets]
        if WILDCARD in handles:
            answer.rows = RowSet()
            for link, link_targets in db.get_matched_links(spec[1], handles):
                row = _assign_link(spec, targets, db, link_targets)
                if row is not None:
                    answer.rows.add(row)
            return bool(answer.rows)
        return db.link_exists(spec[1], handles)
    if kind == "Template":                                   # :603-614
        found = db.get_matched_type_template([spec[1], *[v[2] for v in spec[3]]])
        answer.rows = RowSet()
        for link, link_targets in found:
            row = _assign_template(spec, link_targets)
            if row is not None:
                answer.rows.add(row)
        return bool(answer.rows)
    if kind == "Not":                                        # :627-631
        matched(spec[1], db, answer)
        answer.negation = not answer.negation
        return True
    if kind == "Or":                                         # :644-687
        terms = spec[1]
        if not terms:
            return False
        union = None
        or_matched = False
        negative = []
        for term in terms:
            if term[0] == "Not":
                negative.append(term)
                continue
            sub = Answer()
            if not matched(term, db, sub):
                continue
            or_matched = True
            if not sub.rows:
                continue
            if not union:
                union = sub.rows
                continue
            union.update(sub.rows)
        union = union or RowSet()
        if negative:
            sub = Answer()
            matched(["And", [t[1] for t in negative]], db, sub)
            answer.rows = sub.rows.minus(union)
            answer.negation = True
        else:
            answer.rows = union
        return or_matched
    if kind == "And":                                        # :705-748
        terms = spec[1]
        if not terms:
            return False
        acc = []          # list semantics inside And (:732-738)
        forbidden = RowSet()
        for term in terms:
            sub = Answer()
            if not matched(term, db, sub):
                return False
            if not sub.rows:
                continue
            if sub.negation:
                forbidden.update(sub.rows)
                continue
            if not acc:
                acc = list(sub.rows)
                continue
            fast = _ordered_hash_join(acc, sub.rows) if FAST_JOIN else _ordered_nested_join(acc, sub.rows)
            acc = fast if fast is not None else \
                [j for a in acc for b in sub.rows for j in [join(a, b)] if j is not None]
        result = RowSet()
        for a in acc:
            if all(check_negation(a, t) for t in forbidden):
                result.add(a)
        answer.rows = result
        return bool(result)
    raise ValueError(f"unknown expression {kind}")


def evaluate(spec, db):
    """Returns the golden-fixture style record for one query."""
    ans = Answer()
    try:
        m = matched(spec, db, ans)
    except (AttributeError, ValueError, TypeError, AssertionError) as e:
        return {"error": type(e).__name__}
    rows = sorted(json.dumps(canon_json(r), sort_keys=True) for r in ans.rows)
    return {"matched": bool(m), "negation": ans.negation, "n": len(ans.rows),
            "rows": [json.loads(r) for r in rows],
            "sha256": hashlib.sha256("\n".join(rows).encode()).hexdigest()}
