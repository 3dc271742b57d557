"""Host-side ingestion: MeTTa text -> AtomArrays (the das_atoms_t layout).

Parsing is host work; what it hands the GPU is the
expression DAG: string leaves (type names, terminals) and expressions whose
first child is the link type.  Hashing, interning and every index are built
on the device (`das_build_index`).  Two readers reproduce the reference's two
loaders:

* `parse_metta`      general MeTTa with deferred typedef resolution, as
                     MettaYacc/BaseYacc (das/base_yacc.py:83-161,
                     das/metta_yacc.py:38-172): nodes are the terminals that
                     appear inside expressions; a symbol used as a target is
                     its typedef expression (md5(":"), md5(name), md5(type)).
* `parse_canonical`  one expression per line, typed terminals "Type name", as
                     CanonicalParser (das/canonical_parser.py:242-365): nodes
                     are the terminals declared by `(: "name" Type)` lines.
"""
import json
import re

import numpy as np

NONE = 0xFFFFFFFF
LEAF_TYPE, LEAF_NODE, LEAF_OTHER = 0, 1, 2
EXPR_LINK, EXPR_TYPEDEF = 1, 2
BASIC_TYPE = "Type"          # metta_lex.py:4
TYPEDEF_MARK = ":"


class AtomArrays:
    """Flat arrays in the das_atoms_t layout (include/das_mi355x.h)."""

    def __init__(self, leaf_bytes, leaf_off, leaf_kind, leaf_ctype, leaf_type_id, name_start,
                 expr_off, expr_child, expr_kind, expr_ctype_leaf, level_off, type_names):
        self.leaf_bytes = np.ascontiguousarray(leaf_bytes, dtype=np.uint8)
        self.leaf_off = np.ascontiguousarray(leaf_off, dtype=np.uint64)
        self.leaf_kind = np.ascontiguousarray(leaf_kind, dtype=np.uint8)
        self.leaf_ctype = np.ascontiguousarray(leaf_ctype, dtype=np.uint32)
        self.leaf_type_id = np.ascontiguousarray(leaf_type_id, dtype=np.uint32)
        self.name_start = np.ascontiguousarray(name_start, dtype=np.uint32)
        self.expr_off = np.ascontiguousarray(expr_off, dtype=np.uint64)
        self.expr_child = np.ascontiguousarray(expr_child, dtype=np.uint32)
        self.expr_kind = np.ascontiguousarray(expr_kind, dtype=np.uint8)
        self.expr_ctype_leaf = np.ascontiguousarray(expr_ctype_leaf, dtype=np.int32)
        self.level_off = np.ascontiguousarray(level_off, dtype=np.uint64)
        self.type_names = list(type_names)
        self.type_id = {n: i for i, n in enumerate(self.type_names)}

    @property
    def n_leaf(self):
        return len(self.leaf_off) - 1

    @property
    def n_expr(self):
        return len(self.expr_off) - 1

    # --- accessors used by tests / the oracle -------------------------------
    @property
    def expr_level(self):
        lv = np.zeros(self.n_expr, dtype=np.int64)
        for g in range(len(self.level_off) - 1):
            lv[int(self.level_off[g]):int(self.level_off[g + 1])] = g
        return lv

    def leaf_string(self, i):
        return bytes(self.leaf_bytes[int(self.leaf_off[i]):int(self.leaf_off[i + 1])]).decode("utf-8")

    def leaf_strings(self):
        return [self.leaf_string(i) for i in range(self.n_leaf)]

    def node_name(self, i):
        b = int(self.leaf_off[i]) + int(self.name_start[i])
        return bytes(self.leaf_bytes[b:int(self.leaf_off[i + 1])]).decode("utf-8")

    def children(self, j):
        return [int(x) for x in self.expr_child[int(self.expr_off[j]):int(self.expr_off[j + 1])]]

    # --- resume without the parser ------------------------------------------
    _FIELDS = ("leaf_bytes", "leaf_off", "leaf_kind", "leaf_ctype", "leaf_type_id", "name_start", "expr_off",
               "expr_child", "expr_kind", "expr_ctype_leaf", "level_off")

    def save(self, path, extra=None):
        """The parsed KB as one uncompressed .npz (plain arrays, no pickles):
        the analogue of the reference loader's kept key-value files, which
        let a later load skip the parser (canonical_parser.py:28-29, 235,
        317-319).  `extra`: a JSON-serialisable dict stored beside them."""
        meta = {"format": "das_amd.AtomArrays/1", "type_names": self.type_names, "extra": extra or {}}
        fields = {k: getattr(self, k) for k in self._FIELDS}
        fields["meta_json"] = np.frombuffer(json.dumps(meta).encode("utf-8"), dtype=np.uint8)
        with open(path, "wb") as f:
            np.savez(f, **fields)

    @classmethod
    def load(cls, path, mmap=False):
        """(AtomArrays, extra) from save(); allow_pickle stays off."""
        with np.load(path, allow_pickle=False, mmap_mode="r" if mmap else None) as z:
            meta = json.loads(bytes(z["meta_json"]).decode("utf-8"))
            if meta.get("format") != "das_amd.AtomArrays/1":
                raise ValueError(f"{path}: not a saved das_amd KB")
            a = cls(*[z[k] for k in cls._FIELDS], meta["type_names"])
        return a, meta.get("extra", {})


class AtomBuilder:
    """Incremental builder; `finish()` groups expressions by (level, arity)."""

    def __init__(self):
        self.leaf_index = {}
        self.leaf_str = []
        self.leaf_kind = []
        self.leaf_ctype = []
        self.name_start = []
        self.type_names = []
        self.type_of_leaf = {}
        self.e_children = []      # child refs: leaf i -> i, expr j -> -(j + 1)
        self.e_kind = []
        self.e_ctype_leaf = []
        self.e_level = []

    def type_leaf(self, name):
        i = self.leaf_index.get(name)
        if i is None:
            i = len(self.leaf_str)
            self.leaf_index[name] = i
            self.leaf_str.append(name)
            self.leaf_kind.append(LEAF_TYPE)
            self.leaf_ctype.append(i)
            self.name_start.append(0)
        if i not in self.type_of_leaf:
            if self.leaf_kind[i] != LEAF_TYPE:
                raise ValueError(f"'{name}' is both a terminal string and a type name")
            self.type_of_leaf[i] = len(self.type_names)
            self.type_names.append(name)
        return i

    def terminal(self, named_type, name, node):
        """Leaf hashed as terminal_hash(named_type, name) (expression_hasher.py:17-19)."""
        t = self.type_leaf(named_type)
        s = " ".join([named_type, name])
        i = self.leaf_index.get(s)
        if i is None:
            i = len(self.leaf_str)
            self.leaf_index[s] = i
            self.leaf_str.append(s)
            self.leaf_kind.append(LEAF_NODE if node else LEAF_OTHER)
            self.leaf_ctype.append(t)
            self.name_start.append(len(named_type.encode("utf-8")) + 1)
        elif node and self.leaf_kind[i] == LEAF_OTHER:
            self.leaf_kind[i] = LEAF_NODE
        return i

    def expr(self, type_name, children, kind=EXPR_LINK, ctype_leaf=-1):
        """children: refs returned by terminal()/expr()/type_leaf(); returns a ref."""
        t = self.type_leaf(type_name)
        refs = [t] + list(children)
        lv = 1 + max([self.e_level[-r - 1] if r < 0 else 0 for r in refs])
        self.e_children.append(refs)
        self.e_kind.append(kind)
        self.e_ctype_leaf.append(ctype_leaf)
        self.e_level.append(lv)
        return -len(self.e_children)

    def typedef_expr(self, name, type_name):
        """The typedef atom (: name type) — expression_hash(md5(':'), [md5(name), md5(type)])
        (canonical_parser.py:48-59, base_yacc.py:108-130).  Used as a target it is
        the symbol's handle; its composite type is md5(name) (base_yacc.py:147-161)."""
        n = self.type_leaf(name)
        t = self.type_leaf(type_name)
        return self.expr(TYPEDEF_MARK, [n, t], kind=EXPR_TYPEDEF, ctype_leaf=n)

    def finish(self):
        n_leaf = len(self.leaf_str)
        n_expr = len(self.e_children)
        enc = [s.encode("utf-8") for s in self.leaf_str]
        lens = np.array([len(b) for b in enc], dtype=np.uint64)
        leaf_off = np.zeros(n_leaf + 1, dtype=np.uint64)
        np.cumsum(lens, out=leaf_off[1:])
        leaf_bytes = np.frombuffer(b"".join(enc), dtype=np.uint8) if n_leaf else np.zeros(0, np.uint8)
        leaf_type_id = np.full(n_leaf, NONE, dtype=np.uint32)
        for i, tid in self.type_of_leaf.items():
            leaf_type_id[i] = tid
        # group expressions by (level, number of children)
        nch = np.array([len(c) for c in self.e_children], dtype=np.int64)
        lev = np.array(self.e_level, dtype=np.int64)
        order = np.lexsort((np.arange(n_expr), nch, lev)) if n_expr else np.zeros(0, np.int64)
        newpos = np.empty(n_expr, dtype=np.int64)
        newpos[order] = np.arange(n_expr)
        expr_off = np.zeros(n_expr + 1, dtype=np.uint64)
        np.cumsum(nch[order], out=expr_off[1:])
        child = np.empty(int(expr_off[-1]) if n_expr else 0, dtype=np.uint32)
        pos = 0
        for j in order:
            for r in self.e_children[j]:
                child[pos] = r if r >= 0 else n_leaf + newpos[-r - 1]
                pos += 1
        kinds = np.array(self.e_kind, dtype=np.uint8)[order] if n_expr else np.zeros(0, np.uint8)
        ctl = np.array(self.e_ctype_leaf, dtype=np.int32)[order] if n_expr else np.zeros(0, np.int32)
        groups = [0]
        for k in range(1, n_expr):
            a, b = order[k - 1], order[k]
            if lev[a] != lev[b] or nch[a] != nch[b]:
                groups.append(k)
        groups.append(n_expr)
        if n_expr == 0:
            groups = [0]
        self._newpos = newpos
        return AtomArrays(leaf_bytes, leaf_off, np.array(self.leaf_kind, np.uint8),
                          np.array(self.leaf_ctype, np.uint32), leaf_type_id,
                          np.array(self.name_start, np.uint32), expr_off, child, kinds, ctl,
                          np.array(groups, dtype=np.uint64), self.type_names)

    def unified(self, ref):
        """Unified index (after finish()) of a builder ref."""
        return ref if ref >= 0 else len(self.leaf_str) + int(self._newpos[-ref - 1])


# ---------------------------------------------------------------------------
# General MeTTa (MettaYacc semantics)
# ---------------------------------------------------------------------------
_TOKEN = re.compile(r'\s*(?:(\()|(\))|(:)|"([^"]+)"|([^\W0-9]\w*)|(\S))')


def _tokens(text):
    pos = 0
    n = len(text)
    while pos < n:
        m = _TOKEN.match(text, pos)
        if not m or m.end() == pos:
            break
        pos = m.end()
        if m.group(1):
            yield ("(", None)
        elif m.group(2):
            yield (")", None)
        elif m.group(3):
            yield (":", None)
        elif m.group(4) is not None:
            yield ("T", m.group(4))
        elif m.group(5) is not None:
            yield ("S", m.group(5))
        elif m.group(6) is not None:
            if m.group(6).strip():
                raise SyntaxError(f"illegal character {m.group(6)!r} (metta_lex.py:58-63)")


def _read_sexprs(text):
    stack = [[]]
    for kind, val in _tokens(text):
        if kind == "(":
            stack.append([])
        elif kind == ")":
            if len(stack) < 2:
                raise SyntaxError("unbalanced ')'")
            e = stack.pop()
            stack[-1].append(("E", e))
        else:
            stack[-1].append((kind, val))
    if len(stack) != 1:
        raise SyntaxError("unbalanced '('")
    return stack[0]


def parse_metta(texts, builder=None):
    """MeTTa source(s) -> AtomBuilder, MettaYacc semantics."""
    if isinstance(texts, str):
        texts = [texts]
    b = builder or AtomBuilder()
    tops = []
    named_types = {BASIC_TYPE: BASIC_TYPE}
    typedefs = []
    for text in texts:
        for item in _read_sexprs(text):
            if item[0] != "E":
                raise SyntaxError("top level must be expressions")
            body = item[1]
            if body and body[0][0] == ":":
                if len(body) != 3 or body[1][0] not in ("S", "T") or body[2][0] != "S":
                    raise SyntaxError(f"bad typedef {body}")
                named_types[body[1][1]] = body[2][1]
                typedefs.append((body[1][1], body[2][1]))
            else:
                tops.append(body)
    symbol_ref = {}

    def sym(name):
        if name not in named_types:
            raise NameError(f"undefined symbol {name} (UndefinedSymbolError, exceptions.py:19-22)")
        r = symbol_ref.get(name)
        if r is None:
            r = b.typedef_expr(name, named_types[name])
            symbol_ref[name] = r
        return r

    def build(body):
        if not body:
            raise SyntaxError("empty expression")
        head = body[0]
        if head[0] != "S":
            raise NotImplementedError("only symbol-headed expressions are typed (base_yacc.py:101-105)")
        if head[1] not in named_types:
            raise NameError(f"undefined symbol {head[1]}")
        kids = []
        for kind, val in body[1:]:
            if kind == "E":
                if val and val[0][0] == ":":
                    raise SyntaxError("nested type definition (metta_yacc.py:145-156)")
                kids.append(build(val))
            elif kind == "T":
                if val not in named_types:
                    raise NameError(f"undefined terminal {val}")
                kids.append(b.terminal(named_types[val], val, node=True))
            elif kind == "S":
                kids.append(sym(val))
            else:
                raise SyntaxError(f"unexpected token {kind}")
        return b.expr(head[1], kids)

    for body in tops:
        build(body)
    return b


# ---------------------------------------------------------------------------
# Canonical MeTTa (CanonicalParser semantics)
# ---------------------------------------------------------------------------

def _canonical_expression(line, b):
    stack = []            # refs, or ("sym", name) for raw symbols
    cur = []
    i, n = 0, len(line)
    while i < n:
        c = line[i]
        if c == '"':
            # closing quote: the first '"' not preceded by a backslash (canonical_parser.py:287)
            j = i + 1
            while j < n and not (line[j] == '"' and line[j - 1] != "\\"):
                j += 1
            if j >= n:
                raise SyntaxError(f"unterminated string: {line[:80]}")
            parts = line[i + 1:j].split()
            stype, name = parts[0], " ".join(parts[1:])
            stack.append(b.terminal(stype, name, node=False))
            i = j + 1
            continue
        if c == "(":
            stack.append("(")
        elif c == " ":
            if cur:
                stack.append(("sym", "".join(cur)))
                cur = []
        elif c == ")":
            if cur:
                stack.append(("sym", "".join(cur)))
                cur = []
            items = []
            while stack and stack[-1] != "(":
                items.append(stack.pop())
            stack.pop()
            items.reverse()
            if not items or not isinstance(items[0], tuple):
                raise NotImplementedError("canonical expression without a type symbol")
            kids = []
            for x in items[1:]:
                if isinstance(x, tuple):
                    raise NotImplementedError("bare symbols as link targets (canonical_parser.py:253-261)")
                kids.append(x)
            stack.append(b.expr(items[0][1], kids))
        else:
            cur.append(c)
        i += 1
    if len(stack) != 1:
        raise SyntaxError(f"unbalanced canonical line: {line[:80]}")


_LINE_BREAK = re.compile(r"\r\n|\r|\n")


def parse_canonical(texts, builder=None):
    """Canonical MeTTa -> AtomBuilder (canonical_parser.py:315-365)."""
    if isinstance(texts, str):
        texts = [texts]
    b = builder or AtomBuilder()
    for text in texts:
        state = 0
        for raw in _LINE_BREAK.split(text):      # universal newlines, as `for line in file`
            line = raw.strip()
            if not line:
                continue
            words = line.split()
            if state == 0:
                if words[0] != "(:":
                    raise SyntaxError(f"expected a typedef: {line[:80]}")
                if words[1].startswith('"'):
                    state = 1
                else:
                    b.type_leaf(words[1])
                    b.type_leaf(words[-1].rstrip(")"))
            if state == 1:
                if words[0] == "(:":
                    name = " ".join(words[1:-1]).strip('"')
                    b.terminal(words[-1].rstrip(")"), name, node=True)
                    continue
                state = 2
            if state == 2:
                if words[0] == "(:" or not line.startswith("(") or not line.endswith(")"):
                    raise SyntaxError(f"bad canonical expression line: {line[:80]}")
                _canonical_expression(line, b)
    return b


class _OrderRecorder:
    """AtomBuilder stand-in for _canonical_expression: handles instead of
    refs, and every link in the order CanonicalParser._add_expression sees
    it (post-order: a nested link before the link holding it)."""

    def __init__(self):
        from .expression_hasher import ExpressionHasher
        self.eh = ExpressionHasher
        self.links = []

    def terminal(self, stype, name, node=False):
        return self.eh.terminal_hash(stype, name)

    def expr(self, type_name, kids):
        h = self.eh.expression_hash(self.eh.named_type_hash(type_name), kids)
        self.links.append((h, type_name, list(kids)))
        return h


def canonical_pattern_order(texts):
    """The links of canonical MeTTa text in the order the reference's
    pattern-key loop walks them (canonical_parser.py:132-183): collection
    links_1, then links_2, then links_n (_populate_mongo_links :185-206),
    each in insertion order -- the first occurrence of each handle in parse
    order (_add_expression :77-93 is called as an expression closes,
    _mongo_insert_many :95-110 drops repeats).  [(handle, named_type,
    [element handles])]."""
    if isinstance(texts, str):
        texts = [texts]
    rec = _OrderRecorder()
    for text in texts:
        state = 0
        for raw in _LINE_BREAK.split(text):
            line = raw.strip()
            if not line:
                continue
            words = line.split()
            if state == 0 and words[0] == "(:" and not words[1].startswith('"'):
                continue
            if words[0] == "(:":
                state = 1
                continue
            state = 2
            _canonical_expression(line, rec)
    seen, by_arity = set(), ([], [], [])
    for h, t, kids in rec.links:
        if h in seen:
            continue
        seen.add(h)
        by_arity[0 if len(kids) == 1 else 1 if len(kids) == 2 else 2].append((h, t, kids))
    return by_arity[0] + by_arity[1] + by_arity[2]


def _nesting_levels(p):
    """1 + the deepest expression child, per expression (groups are children-first)."""
    lev = np.zeros(p.n_expr, dtype=np.int64)
    for g in range(len(p.level_off) - 1):
        b, e = int(p.level_off[g]), int(p.level_off[g + 1])
        if e <= b:
            continue
        k = int(p.expr_off[b + 1] - p.expr_off[b])
        ch = p.expr_child[int(p.expr_off[b]):int(p.expr_off[e])].reshape(e - b, k).astype(np.int64)
        sub = np.where(ch >= p.n_leaf, lev[np.maximum(ch - p.n_leaf, 0)], 0)
        lev[b:e] = 1 + sub.max(axis=1)
    return lev


def concat_arrays(parts):
    """One AtomArrays from several (e.g. the native canonical reader's output
    and a MeTTa builder's): leaves are appended (the device interns repeats by
    digest), named types are merged by name, expression groups are re-formed
    by (level, number of children) keeping each part's order."""
    parts = [p for p in parts if p is not None]
    if len(parts) == 1:
        return parts[0]
    names, tid = [], {}
    leaf_bytes, leaf_off, leaf_kind, leaf_ctype, leaf_type_id, name_start = [], [], [], [], [], []
    e_child, e_nch, e_level, e_kind, e_ctl, e_part_pos = [], [], [], [], [], []
    leaf_base, byte_base = 0, 0
    total_leaf = sum(p.n_leaf for p in parts)
    expr_base = 0
    for p in parts:
        remap = np.array([tid.setdefault(n, len(tid)) for n in p.type_names], dtype=np.uint32)
        names = sorted(tid, key=tid.get)
        ltid = p.leaf_type_id.copy()
        m = ltid != NONE
        ltid[m] = remap[ltid[m]]
        leaf_bytes.append(p.leaf_bytes)
        leaf_off.append(p.leaf_off[:-1] + np.uint64(byte_base))
        leaf_kind.append(p.leaf_kind)
        leaf_ctype.append(p.leaf_ctype + np.uint32(leaf_base))
        leaf_type_id.append(ltid)
        name_start.append(p.name_start)
        nch = np.diff(p.expr_off.astype(np.int64))
        lev = _nesting_levels(p)
        ch = p.expr_child.astype(np.int64)
        is_expr = ch >= p.n_leaf
        ch = np.where(is_expr, ch - p.n_leaf + total_leaf + expr_base, ch + leaf_base)
        e_child.append(ch)
        e_nch.append(nch)
        e_level.append(lev)
        e_kind.append(p.expr_kind)
        ctl = p.expr_ctype_leaf.astype(np.int64)
        e_ctl.append(np.where(ctl >= 0, ctl + leaf_base, -1))
        leaf_base += p.n_leaf
        byte_base += int(p.leaf_off[-1])
        expr_base += p.n_expr
    nch = np.concatenate(e_nch)
    lev = np.concatenate(e_level)
    n_expr = len(nch)
    order = np.lexsort((np.arange(n_expr), nch, lev))
    newpos = np.empty(n_expr, dtype=np.int64)
    newpos[order] = np.arange(n_expr)
    old_off = np.zeros(n_expr + 1, dtype=np.int64)
    np.cumsum(nch, out=old_off[1:])
    ch = np.concatenate(e_child)
    ch = np.where(ch >= total_leaf, newpos[np.maximum(ch - total_leaf, 0)] + total_leaf, ch)
    expr_off = np.zeros(n_expr + 1, dtype=np.uint64)
    np.cumsum(nch[order], out=expr_off[1:])
    idx = np.concatenate([np.arange(old_off[j], old_off[j + 1]) for j in order]) if n_expr else np.zeros(0, np.int64)
    groups = [0]
    for k in range(1, n_expr):
        a, b = order[k - 1], order[k]
        if lev[a] != lev[b] or nch[a] != nch[b]:
            groups.append(k)
    if n_expr:
        groups.append(n_expr)
    off = np.concatenate(leaf_off + [np.array([byte_base], dtype=np.uint64)])
    return AtomArrays(np.concatenate(leaf_bytes), off, np.concatenate(leaf_kind), np.concatenate(leaf_ctype),
                      np.concatenate(leaf_type_id), np.concatenate(name_start), expr_off,
                      ch[idx].astype(np.uint32), np.concatenate(e_kind)[order],
                      np.concatenate(e_ctl)[order].astype(np.int32), np.array(groups, dtype=np.uint64), names)


# ---------------------------------------------------------------------------
# From stored-atom tables (golden fixtures: what the reference put in Mongo)
# ---------------------------------------------------------------------------

def from_tables(nodes, links):
    """nodes: [handle, type, name]; links: [handle, type, [target handles], ctype].
    Rebuilds the DAG; the GPU then recomputes every handle."""
    b = AtomBuilder()
    ref = {}
    for h, t, name in nodes:
        ref[h] = b.terminal(t, name, node=True)
    pending = {h: (t, tg) for h, t, tg, _ in links}

    def make(h, depth=0):
        if h in ref:
            return ref[h]
        if h not in pending or depth > 10000:
            raise KeyError(f"target {h} is neither a stored node nor a stored link")
        t, tg = pending[h]
        r = b.expr(t, [make(x, depth + 1) for x in tg])
        ref[h] = r
        return r

    for h, _, _, _ in links:
        make(h)
    return b
