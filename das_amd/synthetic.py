"""Seeded synthetic knowledge bases in the shapes the reference benchmarks
(no network: the bio_atomspace and FlyBase dumps are not available, SURVEY.md
§8d).  Generators emit AtomArrays directly (vectorised numpy), so 10^7-10^9
links do not go through a text parser.

* `bio_kb`      config 2: gene-level KB of scripts/benchmark.py:89-138 —
                Member(Gene, BiologicalProcess) with Zipf(1.1) process
                popularity, Inheritance(BP, BP) hierarchy.
* `flybase_kb`  config 3: Execution(Schema, pk, value) arity-3 rows
                (flybase2metta/sql_reader.py:297-302).
* `powerlaw_kb` configs 4-5: arity 2-3 links over Zipf(1.1) node popularity.
"""
import numpy as np

from .loader import AtomArrays, LEAF_NODE, LEAF_TYPE, NONE

SEED = 20250209


def zipf_indices(rng, n_items, size, s=1.1):
    """Zipf(s)-distributed indices in [0, n_items) (inverse-CDF over ranks)."""
    ranks = np.arange(1, n_items + 1, dtype=np.float64)
    p = ranks ** (-s)
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    u = rng.random(size)
    return np.minimum(np.searchsorted(cdf, u), n_items - 1).astype(np.int64)


def build_arrays(type_names, node_blocks, link_blocks):
    """node_blocks: [(type_name, prefix, count)] -> node g of block b is the
    terminal "type prefix<g>"; global node index = block offset + g.
    link_blocks: [(type_name, children int array (n, k)[, expr kinds (n,)])] of
    global node indices; kind 1 = local link, 3 = link owned by another shard.
    Returns AtomArrays plus the per-block node offsets."""
    types = list(type_names)
    tid = {t: i for i, t in enumerate(types)}
    for t, _, _ in node_blocks:
        if t not in tid:
            tid[t] = len(types)
            types.append(t)
    for blk in link_blocks:
        t = blk[0]
        if t not in tid:
            tid[t] = len(types)
            types.append(t)
    n_types = len(types)
    # leaves: the type names, then the nodes
    strings = [t.encode() for t in types]
    node_off = []
    node_ctype, name_start = [], []
    n_nodes = 0
    for t, prefix, count in node_blocks:
        node_off.append(n_types + n_nodes)
        strings.extend(f"{t} {prefix}{i}".encode() for i in range(count))
        node_ctype.append(np.full(count, tid[t], dtype=np.uint32))
        name_start.append(np.full(count, len(t.encode()) + 1, np.uint32))
        n_nodes += count
    return _finish_arrays(types, tid, strings, n_types, n_nodes, node_ctype, name_start, link_blocks), node_off


def _finish_arrays(types, tid, strings, n_types, n_nodes, node_ctype, name_start, link_blocks):
    n_leaf = n_types + n_nodes
    lens = np.fromiter((len(s) for s in strings), dtype=np.uint64, count=n_leaf)
    leaf_off = np.zeros(n_leaf + 1, dtype=np.uint64)
    np.cumsum(lens, out=leaf_off[1:])
    leaf_bytes = np.frombuffer(b"".join(strings), dtype=np.uint8)
    leaf_kind = np.concatenate([np.full(n_types, LEAF_TYPE, np.uint8), np.full(n_nodes, LEAF_NODE, np.uint8)])
    leaf_ctype = np.concatenate([np.arange(n_types, dtype=np.uint32)] + node_ctype) if n_nodes else \
        np.arange(n_types, dtype=np.uint32)
    leaf_type_id = np.concatenate([np.arange(n_types, dtype=np.uint32), np.full(n_nodes, NONE, np.uint32)])
    name_start = np.concatenate([np.zeros(n_types, np.uint32)] + list(name_start))
    # expressions: one group per arity (all at level 1)
    by_k, kinds_k = {}, {}
    for blk in link_blocks:
        t, ch = blk[0], np.asarray(blk[1], dtype=np.int64)
        kinds = np.asarray(blk[2], np.uint8) if len(blk) > 2 else np.ones(ch.shape[0], np.uint8)
        k = ch.shape[1] + 1
        full = np.concatenate([np.full((ch.shape[0], 1), tid[t], np.int64), ch + n_types], axis=1)
        by_k.setdefault(k, []).append(full)
        kinds_k.setdefault(k, []).append(kinds)
    childs, groups, nchs, ekinds = [], [0], [], []
    total = 0
    for k in sorted(by_k):
        blk = np.concatenate(by_k[k])
        childs.append(blk.reshape(-1).astype(np.uint32))
        nchs.append(np.full(blk.shape[0], k, np.uint64))
        ekinds.append(np.concatenate(kinds_k[k]))
        total += blk.shape[0]
        groups.append(total)
    n_expr = total
    nch = np.concatenate(nchs) if nchs else np.zeros(0, np.uint64)
    expr_off = np.zeros(n_expr + 1, dtype=np.uint64)
    np.cumsum(nch, out=expr_off[1:])
    expr_child = np.concatenate(childs) if childs else np.zeros(0, np.uint32)
    expr_kind = np.concatenate(ekinds) if ekinds else np.zeros(0, np.uint8)
    return AtomArrays(leaf_bytes, leaf_off, leaf_kind, leaf_ctype, leaf_type_id, name_start, expr_off,
                      expr_child, expr_kind, np.full(n_expr, -1, np.int32),
                      np.array(groups, np.uint64), types)


def build_arrays_named(type_names, node_lists, link_blocks):
    """build_arrays with explicit node names: node_lists = [(type, [names])]."""
    types = list(type_names)
    tid = {t: i for i, t in enumerate(types)}
    for t, _ in node_lists:
        if t not in tid:
            tid[t] = len(types)
            types.append(t)
    for blk in link_blocks:
        if blk[0] not in tid:
            tid[blk[0]] = len(types)
            types.append(blk[0])
    n_types = len(types)
    strings = [t.encode() for t in types]
    node_ctype, name_start = [], []
    n_nodes = 0
    for t, names in node_lists:
        strings.extend(f"{t} {n}".encode() for n in names)
        node_ctype.append(np.full(len(names), tid[t], dtype=np.uint32))
        name_start.append(np.full(len(names), len(t.encode()) + 1, np.uint32))
        n_nodes += len(names)
    return _finish_arrays(types, tid, strings, n_types, n_nodes, node_ctype, name_start, link_blocks)


def bio_kb(n_genes=20000, n_bps=10000, n_member=1_000_000, n_inh=None, seed=SEED):
    """Config 2 stand-in: Member(Gene, BP), Inheritance(BP, BP)."""
    rng = np.random.default_rng(seed)
    n_inh = n_inh if n_inh is not None else 2 * n_bps
    genes = rng.integers(0, n_genes, n_member)
    bps = zipf_indices(rng, n_bps, n_member)
    child = rng.integers(1, n_bps, n_inh)
    parent = (rng.random(n_inh) * child).astype(np.int64)      # parents have lower index
    arrays, off = build_arrays(
        ["Member", "Inheritance"],
        [("Gene", "g", n_genes), ("BiologicalProcess", "bp", n_bps)],
        [("Member", np.stack([genes, n_genes + bps], 1)),
         ("Inheritance", np.stack([n_genes + child, n_genes + parent], 1))])
    return arrays


def expr_ref(block, rows):
    """Child reference to rows of an earlier link block (build_nested)."""
    return -(1 + (np.int64(block) << np.int64(32)) + np.asarray(rows, dtype=np.int64))


def build_nested(type_names, node_blocks, link_blocks):
    """build_arrays for nested expressions: link block children are global
    node indices (>= 0) or expr_ref(b, row) references to rows of an earlier
    block b; a node block (type, [names], n) names its nodes explicitly; a
    link block (type, children[, expr kinds]).
    Expressions are grouped by (nesting level, arity) as the
    AtomArrays layout requires, each block keeping its row order."""
    types = list(type_names)
    tid = {t: i for i, t in enumerate(types)}
    for t, _, _ in node_blocks:
        tid.setdefault(t, len(tid))
    for blk in link_blocks:
        tid.setdefault(blk[0], len(tid))
    types = sorted(tid, key=tid.get)
    n_types = len(types)
    strings = [t.encode() for t in types]
    node_ctype, name_start, n_nodes = [], [], 0
    for t, prefix, count in node_blocks:
        names = prefix if isinstance(prefix, list) else [f"{prefix}{i}" for i in range(count)]
        strings.extend(f"{t} {n}".encode() for n in names)
        node_ctype.append(np.full(len(names), tid[t], dtype=np.uint32))
        name_start.append(np.full(len(names), len(t.encode()) + 1, np.uint32))
        n_nodes += len(names)
    n_leaf = n_types + n_nodes
    # nesting level and arity of every block
    level, chs = [], []
    for blk in link_blocks:
        ch = np.asarray(blk[1], dtype=np.int64)
        refs = -(ch[ch < 0] + 1) >> np.int64(32)
        level.append(1 + max([level[int(b)] for b in np.unique(refs)], default=0))
        chs.append(ch)
    key = sorted(range(len(link_blocks)), key=lambda b: (level[b], chs[b].shape[1], b))
    start, total = {}, 0
    for b in key:
        start[b] = total
        total += chs[b].shape[0]
    childs, nchs, groups, prev = [], [], [0], None
    kinds = []
    run = 0
    for b in key:
        blk = link_blocks[b]
        kinds.append(np.asarray(blk[2], np.uint8) if len(blk) > 2 else np.ones(chs[b].shape[0], np.uint8))
        ch = chs[b]
        neg = ch < 0
        r = -(ch[neg] + 1)
        src, row = r >> np.int64(32), r & np.int64(0xFFFFFFFF)
        out = ch + n_types
        out[neg] = n_leaf + np.array([start[int(s)] for s in src], dtype=np.int64) + row
        full = np.concatenate([np.full((ch.shape[0], 1), tid[link_blocks[b][0]], np.int64), out], axis=1)
        g = (level[b], ch.shape[1])
        if prev is not None and g != prev:
            groups.append(run)
        prev = g
        run += ch.shape[0]
        childs.append(full.reshape(-1).astype(np.uint32))
        nchs.append(np.full(ch.shape[0], ch.shape[1] + 1, np.uint64))
    groups.append(run)
    lens = np.fromiter((len(s) for s in strings), dtype=np.uint64, count=n_leaf)
    leaf_off = np.zeros(n_leaf + 1, dtype=np.uint64)
    np.cumsum(lens, out=leaf_off[1:])
    nch = np.concatenate(nchs)
    expr_off = np.zeros(total + 1, dtype=np.uint64)
    np.cumsum(nch, out=expr_off[1:])
    return AtomArrays(np.frombuffer(b"".join(strings), dtype=np.uint8), leaf_off,
                      np.concatenate([np.full(n_types, LEAF_TYPE, np.uint8), np.full(n_nodes, LEAF_NODE, np.uint8)]),
                      np.concatenate([np.arange(n_types, dtype=np.uint32)] + node_ctype),
                      np.concatenate([np.arange(n_types, dtype=np.uint32), np.full(n_nodes, NONE, np.uint32)]),
                      np.concatenate([np.zeros(n_types, np.uint32)] + name_start),
                      expr_off, np.concatenate(childs), np.concatenate(kinds), np.full(total, -1, np.int32),
                      np.array(groups, np.uint64), types)


BIO_TYPES = ["Member", "Inheritance", "List", "Evaluation", "Context"]


def bio_nodes(n_genes, n_bps, n_uniprot=5000, n_reactome=1000, n_loc=40):
    """Node blocks of the gene-level KB and each block's first node index."""
    nodes = [("Gene", "g", n_genes), ("BiologicalProcess", "bp", n_bps), ("Uniprot", "up", n_uniprot),
             ("Reactome", "r", n_reactome), ("Concept", "upname", n_uniprot), ("Concept", "rname", n_reactome),
             ("Concept", "loc", n_loc), ("Predicate", ["has_name"], 1), ("Predicate", ["has_location"], 1)]
    off, o = {}, 0
    for t, p, c in nodes:
        off[p if isinstance(p, str) else p[0]] = o
        o += c
    return nodes, off


def bio_annotation_blocks(rng, off, n_bps, n_uniprot=5000, n_up_member=50_000, n_reactome=1000, n_context=20_000,
                          n_loc=40, base=0):
    """The annotation-service layouts (data/annotation_service/*.metta) around
    the gene-level core, as link blocks; `base` = index of the first of them
    in the caller's block list (nested children reference blocks by index):
      Member(Uniprot, BiologicalProcess)                      Zipf(1.1)
      Evaluation(has_name, List(Uniprot, Concept name))       one per protein
      Evaluation(has_name, List(Reactome, Concept name))      one per pathway
      Context(Member(Uniprot, Reactome),
              Evaluation(has_location, List(Uniprot, Concept location)))"""
    up_m = rng.integers(0, n_uniprot, n_up_member)
    up_bp = zipf_indices(rng, n_bps, n_up_member)
    ctx_up = rng.integers(0, n_uniprot, n_context)
    ctx_r = zipf_indices(rng, n_reactome, n_context)
    ctx_loc = zipf_indices(rng, n_loc, n_context)
    ups, rs = np.arange(n_uniprot), np.arange(n_reactome)
    name_pred = lambda n: np.full(n, off["has_name"], np.int64)  # noqa: E731
    B = lambda k: base + k  # noqa: E731
    return [
        ("Member", np.stack([off["up"] + up_m, off["bp"] + up_bp], 1)),                  # 0
        ("List", np.stack([off["up"] + ups, off["upname"] + ups], 1)),                   # 1
        ("List", np.stack([off["r"] + rs, off["rname"] + rs], 1)),                       # 2
        ("Member", np.stack([off["up"] + ctx_up, off["r"] + ctx_r], 1)),                 # 3
        ("List", np.stack([off["up"] + ctx_up, off["loc"] + ctx_loc], 1)),               # 4
        ("Evaluation", np.stack([name_pred(n_uniprot), expr_ref(B(1), ups)], 1)),        # 5
        ("Evaluation", np.stack([name_pred(n_reactome), expr_ref(B(2), rs)], 1)),        # 6
        ("Evaluation", np.stack([np.full(n_context, off["has_location"], np.int64),
                                 expr_ref(B(4), np.arange(n_context))], 1)),             # 7
        ("Context", np.stack([expr_ref(B(3), np.arange(n_context)), expr_ref(B(7), np.arange(n_context))], 1)),
    ]


def bio_full_kb(n_genes=20000, n_bps=10000, n_member=1_000_000, n_inh=None, n_uniprot=5000,
                n_up_member=50_000, n_reactome=1000, n_context=20_000, n_loc=40, seed=SEED):
    """The gene-level KB scripts/benchmark.py's three query layouts need
    (benchmark.py:40-128), with the annotation-service file shapes
    (data/annotation_service/*.metta):
      Member(Gene, BiologicalProcess)           Zipf(1.1) process popularity
      Inheritance(BP, BP)                       parents have lower index
      + bio_annotation_blocks (Uniprot / Reactome Member, List, Evaluation, Context)
    Nodes: g<i>, bp<i>, up<i>, r<i>, upname<i>, rname<i>, loc<i>, and the
    predicates has_name / has_location.  The Member(Gene) and Inheritance
    links are bio_kb's with the same arguments."""
    rng = np.random.default_rng(seed)
    n_inh = n_inh if n_inh is not None else 2 * n_bps
    nodes, off = bio_nodes(n_genes, n_bps, n_uniprot, n_reactome, n_loc)
    genes = rng.integers(0, n_genes, n_member)
    bps = zipf_indices(rng, n_bps, n_member)
    child = rng.integers(1, n_bps, n_inh)
    parent = (rng.random(n_inh) * child).astype(np.int64)
    blocks = [
        ("Member", np.stack([off["g"] + genes, off["bp"] + bps], 1)),
        ("Inheritance", np.stack([off["bp"] + child, off["bp"] + parent], 1)),
    ] + bio_annotation_blocks(rng, off, n_bps, n_uniprot, n_up_member, n_reactome, n_context, n_loc, base=2)
    return build_nested(BIO_TYPES, nodes, blocks)


def flybase_kb(n_genes=200_000, n_schema=60, rows_per_schema=400_000, n_loc=5_000, n_do=2_000,
               seed=SEED):
    """Config 3: FlyBase-shaped canonical KB in flybase2metta's
    Execution(Schema s, key, value) layout (sql_reader.py:297-302), arity 3.
    Genes have a pk node and an FB id (Verbatim); the tables QueryFlyBase.ipynb
    queries are present with their semantics, the rest are filler tables
    keyed by FB id with Zipf(1.1) values:
      Schema:gene_uniquename                     (gene pk, FB id)
      Schema:gene_map_table_recombination_loc    (FB id, location)
      Schema:gene_map_table_cytogenetic_loc      (FB id, cyto location)
      Schema:disease_model_annotations_DO_term   (FB id, DO term), ~2 per gene
    Node names: "FBgn%07d" (Verbatim), "g%d" (gene), "loc%d"/"cyto%d"/"DOID:%d"."""
    rng = np.random.default_rng(seed)
    named = ["Schema:gene_uniquename", "Schema:gene_map_table_recombination_loc",
             "Schema:gene_map_table_cytogenetic_loc", "Schema:disease_model_annotations_DO_term"]
    n_fill = max(n_schema - len(named), 0)
    n_val = max(rows_per_schema // 4, 1000)
    # node blocks (global index = block offset + i)
    blocks = [("Schema", "Schema:fill", 0), ("gene", "g", n_genes), ("Verbatim", "FBgn", n_genes),
              ("Verbatim", "loc", n_loc), ("Verbatim", "cyto", n_loc), ("Verbatim", "DOID:", n_do),
              ("Verbatim", "val", n_val)]
    off = {}
    o = 0
    for t, p, c in blocks:
        off[p] = o
        o += c
    schema_names = named + [f"Schema:table{i}_col" for i in range(n_fill)]
    genes = np.arange(n_genes)
    fb = off["FBgn"] + genes
    links = []

    def ex(si, a, b):
        links.append(np.stack([np.full(len(a), si, np.int64), a, b], 1))
    ex(0, off["g"] + genes, fb)
    ex(1, fb, off["loc"] + zipf_indices(rng, n_loc, n_genes))
    ex(2, fb, off["cyto"] + zipf_indices(rng, n_loc, n_genes))
    k = 2 * n_genes
    ex(3, fb[rng.integers(0, n_genes, k)], off["DOID:"] + zipf_indices(rng, n_do, k))
    for i in range(n_fill):
        ex(len(named) + i, fb[rng.integers(0, n_genes, rows_per_schema)],
           off["val"] + zipf_indices(rng, n_val, rows_per_schema))
    ch = np.concatenate(links)
    # schema nodes go first as their own block: shift every other index
    n_s = len(schema_names)
    ch[:, 1:] += n_s
    arrays = build_arrays_named(["Execution"], [("Schema", schema_names)] +
                                [(t, [f"{p}{i}" if p != "FBgn" else f"FBgn{i:07d}" for i in range(c)])
                                 for t, p, c in blocks[1:]],
                                [("Execution", ch)])
    return arrays


def to_canonical(arrays):
    """Canonical MeTTa text of an AtomArrays KB (the format CanonicalParser
    reads, canonical_parser.py:315-365): typedefs, declared terminals (the
    node leaves), then one line per top-level expression."""
    nl, ne = arrays.n_leaf, arrays.n_expr
    off, ch = arrays.expr_off, arrays.expr_child
    leaf = [bytes(arrays.leaf_bytes[int(arrays.leaf_off[i]):int(arrays.leaf_off[i + 1])]).decode()
            for i in range(nl)]
    out = [f"(: {t} Type)" for t in arrays.type_names]
    for i in range(nl):
        if arrays.leaf_kind[i] == LEAF_NODE:
            ns = int(arrays.name_start[i])
            out.append(f'(: "{leaf[i][ns:]}" {leaf[i][:ns - 1]})')
    nested = np.zeros(ne, dtype=bool)
    kids = ch[ch >= nl].astype(np.int64) - nl
    nested[kids[:]] = True
    # every expression's first child is its type leaf, except those whose
    # parent marks them as nested (they print inline)

    def render(j):
        c = ch[int(off[j]):int(off[j + 1])]
        parts = [leaf[int(c[0])]]
        for x in c[1:]:
            x = int(x)
            parts.append(render(x - nl) if x >= nl else f'"{leaf[x]}"')
        return "(" + " ".join(parts) + ")"

    for j in range(ne):
        if not nested[j] and arrays.expr_kind[j] != 2:
            out.append(render(j))
    return "\n".join(out) + "\n"


def _leaf_name(arrays, i):
    a, b = int(arrays.leaf_off[i]), int(arrays.leaf_off[i + 1])
    return bytes(arrays.leaf_bytes[a + int(arrays.name_start[i]):b]).decode()


def flybase_do_terms(arrays, gene=7):
    """DO terms of one gene in a flybase_kb (QueryFlyBase.ipynb cell 9 builds
    its Or over them), read back from the arrays."""
    want_s, want_g = "Schema:disease_model_annotations_DO_term", f"FBgn{gene:07d}"
    off = arrays.expr_off
    out = []
    for g in range(len(arrays.level_off) - 1):
        b, e = int(arrays.level_off[g]), int(arrays.level_off[g + 1])
        if e <= b or int(off[b + 1] - off[b]) != 4:
            continue
        ch = arrays.expr_child[int(off[b]):int(off[e])].reshape(e - b, 4)
        s_leaf = g_leaf = None
        for i in np.unique(ch[:, 1]):
            if _leaf_name(arrays, i) == want_s:
                s_leaf = i
        if s_leaf is None:
            continue
        rows = ch[ch[:, 1] == s_leaf]
        for i in np.unique(rows[:, 2]):
            if _leaf_name(arrays, i) == want_g:
                g_leaf = i
        if g_leaf is not None:
            out = sorted({_leaf_name(arrays, i) for i in rows[rows[:, 2] == g_leaf][:, 3]})
    return out


def powerlaw_kb(n_nodes=1 << 16, n_links=1 << 20, frac_arity2=0.7, link_types=4, seed=SEED):
    """Configs 4-5 shape: Zipf(1.1) targets, 70% arity 2 / 30% arity 3, 4 link types."""
    rng = np.random.default_rng(seed)
    n2 = int(n_links * frac_arity2)
    n3 = n_links - n2
    blocks = []
    names = [f"T{i}" for i in range(link_types)]
    t2 = rng.integers(0, link_types, n2)
    t3 = rng.integers(0, link_types, n3)
    a2 = zipf_indices(rng, n_nodes, (n2, 2))
    a3 = zipf_indices(rng, n_nodes, (n3, 3))
    for i, nm in enumerate(names):
        blocks.append((nm, a2[t2 == i]))
        blocks.append((nm, a3[t3 == i]))
    arrays, off = build_arrays(names, [("Concept", "n", n_nodes)], blocks)
    return arrays


def similarity_kb(n_nodes=300, n_inh=1200, n_sim=600, n_set=200, seed=SEED):
    """Mixed ordered / unordered KB for the Composite-assignment algebra:
    Inheritance(a, b) ordered; Similarity(a, b) and Set(a, b, c) unordered
    (stored in both directions for Similarity, as data/samples/animals.metta
    does), Zipf(1.1) endpoints so joins meet on hubs."""
    rng = np.random.default_rng(seed)
    inh = zipf_indices(rng, n_nodes, (n_inh, 2))
    sim = zipf_indices(rng, n_nodes, (n_sim, 2))
    sim = np.concatenate([sim, sim[:, ::-1]])
    st = zipf_indices(rng, n_nodes, (n_set, 3))
    arrays, off = build_arrays(
        ["Inheritance", "Similarity", "Set"],
        [("Concept", "c", n_nodes)],
        [("Inheritance", inh), ("Similarity", sim), ("Set", st)])
    return arrays


def numbered_leaves(prefix, n):
    """Leaf bytes + offsets of the n strings prefix + str(i), i = 0..n-1
    (native host generator: 2^27 strings in well under a second)."""
    from ._lib import numbered_strings
    return numbered_strings(prefix, n)


class DeviceAtomArrays(AtomArrays):
    """AtomArrays whose expression arrays (expr_off / expr_child / expr_kind /
    expr_ctype_leaf) are torch tensors resident on a GPU; the leaves stay on
    the host (node names are read back from them).  `HipDB.load_arrays`
    builds it through das_build_index_ex(DAS_BUILD_EXPR_ON_DEVICE)."""
    expr_on_device = True

    def __init__(self, leaf_bytes, leaf_off, leaf_kind, leaf_ctype, leaf_type_id, name_start,
                 expr_off, expr_child, expr_kind, expr_ctype_leaf, level_off, type_names):
        super().__init__(leaf_bytes, leaf_off, leaf_kind, leaf_ctype, leaf_type_id, name_start,
                         np.zeros(1, np.uint64), np.zeros(0, np.uint32), np.zeros(0, np.uint8),
                         np.zeros(0, np.int32), level_off, type_names)
        self.expr_off, self.expr_child, self.expr_kind, self.expr_ctype_leaf = \
            expr_off, expr_child, expr_kind, expr_ctype_leaf

    @property
    def n_expr(self):
        return int(self.expr_off.numel()) - 1

    def drop_expr(self):
        """Frees the device expression arrays once the index is built (the
        index keeps everything queries need; leaves stay for node names)."""
        import torch
        dev = self.expr_off.device
        self._n_expr = self.n_expr
        self.expr_off = torch.zeros(1, dtype=torch.int64, device=dev)
        self.expr_child = torch.zeros(0, dtype=torch.int32, device=dev)
        self.expr_kind = torch.zeros(0, dtype=torch.uint8, device=dev)
        self.expr_ctype_leaf = torch.zeros(0, dtype=torch.int32, device=dev)

    def to_host(self):
        """The same KB as host AtomArrays (tests: host-input build parity)."""
        return AtomArrays(self.leaf_bytes, self.leaf_off, self.leaf_kind, self.leaf_ctype, self.leaf_type_id,
                          self.name_start, self.expr_off.cpu().numpy().view(np.uint64),
                          self.expr_child.cpu().numpy().view(np.uint32), self.expr_kind.cpu().numpy(),
                          self.expr_ctype_leaf.cpu().numpy(), self.level_off, self.type_names)


def powerlaw_leaves(n_nodes, link_types):
    """Host leaf arrays of the configs 4-5 KB: type names T0..T{k-1}, Concept,
    then the node terminals "Concept n<i>"."""
    names = [f"T{i}" for i in range(link_types)] + ["Concept"]
    n_types = len(names)
    nb, noff = numbered_leaves("Concept n", n_nodes)
    tb = [t.encode() for t in names]
    tlen = np.array([len(t) for t in tb], dtype=np.uint64)
    leaf_bytes = np.concatenate([np.frombuffer(b"".join(tb), np.uint8), nb])
    leaf_off = np.concatenate([np.concatenate([[0], np.cumsum(tlen)]).astype(np.uint64),
                               noff[1:] + np.uint64(tlen.sum())])
    leaf_kind = np.concatenate([np.full(n_types, LEAF_TYPE, np.uint8), np.full(n_nodes, LEAF_NODE, np.uint8)])
    leaf_ctype = np.concatenate([np.arange(n_types, dtype=np.uint32), np.full(n_nodes, n_types - 1, np.uint32)])
    leaf_type_id = np.concatenate([np.arange(n_types, dtype=np.uint32), np.full(n_nodes, NONE, np.uint32)])
    name_start = np.concatenate([np.zeros(n_types, np.uint32), np.full(n_nodes, len("Concept") + 1, np.uint32)])
    return (leaf_bytes, leaf_off, leaf_kind, leaf_ctype, leaf_type_id, name_start), names


def device_arrays(leaves, names, child2, child3, shard=None):
    """DeviceAtomArrays over host leaves and device link rows: child2 = flat
    int32 tensor of arity-2 rows (type leaf + 2 node leaves, 3 words each),
    child3 of arity-3 rows (4 words each)."""
    import torch
    dev = child2.device
    c2, c3 = child2.numel() // 3, child3.numel() // 4
    child = torch.cat([child2.reshape(-1), child3.reshape(-1)]) if c3 else child2.reshape(-1)
    ne = c2 + c3
    eoff = torch.empty(ne + 1, dtype=torch.int64, device=dev)
    eoff[:c2 + 1] = torch.arange(c2 + 1, dtype=torch.int64, device=dev) * 3
    if c3:
        eoff[c2 + 1:] = 3 * c2 + torch.arange(1, c3 + 1, dtype=torch.int64, device=dev) * 4
    kind = torch.ones(ne, dtype=torch.uint8, device=dev)
    ctl = torch.full((ne,), -1, dtype=torch.int32, device=dev)
    level_off = np.array([0, c2, ne], dtype=np.uint64)
    out = DeviceAtomArrays(*leaves, eoff, child, kind, ctl, level_off, names)
    out.shard = shard if shard is not None and shard[1] > 1 else None
    return out


def powerlaw_kb_device(ctx, n_nodes, n_links, frac_arity2=0.7, link_types=4, seed=SEED, s=1.1,
                       first=0, count=None, shard=None, device=0):
    """Configs 4-5 shape generated on the GPU (das_synth_powerlaw_links):
    global links 0 .. n2-1 have arity 2, n2 .. n_links-1 arity 3 (n2 =
    frac_arity2 * n_links); link i's type and Zipf(s) targets are a hash of
    (seed, i).  This call materialises links [first, first+count).
    shard=(rank, world): the multi-GPU query layout (parallel.shard_arrays) --
    the build indexes only the links whose handle `rank` owns.
    Nodes are the terminals "Concept n<i>"; link types T0..T{link_types-1}."""
    import torch
    count = n_links - first if count is None else count
    end = first + count
    n2 = int(n_links * frac_arity2)
    r2 = (min(max(first, 0), n2), min(end, n2))
    r3 = (max(first, n2), max(end, n2))
    c2, c3 = r2[1] - r2[0], r3[1] - r3[0]
    leaves, names = powerlaw_leaves(n_nodes, link_types)
    n_types = len(names)
    dev = torch.device("cuda", device)
    child2 = torch.empty(3 * c2, dtype=torch.int32, device=dev)
    child3 = torch.empty(4 * c3, dtype=torch.int32, device=dev)
    if c2:
        ctx.synth_powerlaw_links(child2, r2[0], c2, 3, link_types, 0, n_types, n_nodes, s, seed)
    if c3:
        ctx.synth_powerlaw_links(child3, r3[0], c3, 4, link_types, 0, n_types, n_nodes, s, seed)
    return device_arrays(leaves, names, child2, child3, shard)
