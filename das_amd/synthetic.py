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
    node_ctype = []
    n_nodes = 0
    for t, prefix, count in node_blocks:
        node_off.append(n_types + n_nodes)
        strings.extend(f"{t} {prefix}{i}".encode() for i in range(count))
        node_ctype.append(np.full(count, tid[t], dtype=np.uint32))
        n_nodes += count
    n_leaf = n_types + n_nodes
    lens = np.fromiter((len(s) for s in strings), dtype=np.uint64, count=n_leaf)
    leaf_off = np.zeros(n_leaf + 1, dtype=np.uint64)
    np.cumsum(lens, out=leaf_off[1:])
    leaf_bytes = np.frombuffer(b"".join(strings), dtype=np.uint8)
    leaf_kind = np.concatenate([np.full(n_types, LEAF_TYPE, np.uint8), np.full(n_nodes, LEAF_NODE, np.uint8)])
    leaf_ctype = np.concatenate([np.arange(n_types, dtype=np.uint32)] + node_ctype) if n_nodes else \
        np.arange(n_types, dtype=np.uint32)
    leaf_type_id = np.concatenate([np.arange(n_types, dtype=np.uint32), np.full(n_nodes, NONE, np.uint32)])
    name_start = np.concatenate([np.zeros(n_types, np.uint32)] +
                                [np.full(c, len(t.encode()) + 1 + 0, np.uint32) for t, _, c in node_blocks])
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
    arrays = AtomArrays(leaf_bytes, leaf_off, leaf_kind, leaf_ctype, leaf_type_id, name_start, expr_off,
                        expr_child, expr_kind, np.full(n_expr, -1, np.int32),
                        np.array(groups, np.uint64), types)
    return arrays, node_off


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


def flybase_kb(n_rows=100_000, n_schema=60, n_pk=200_000, n_values=50_000, seed=SEED):
    """Config 3 shape: Execution(Schema s, Concept pk, Verbatim value), Zipf values."""
    rng = np.random.default_rng(seed)
    s = rng.integers(0, n_schema, n_rows)
    pk = rng.integers(0, n_pk, n_rows)
    v = zipf_indices(rng, n_values, n_rows)
    arrays, off = build_arrays(
        ["Execution"],
        [("Schema", "s", n_schema), ("Concept", "pk", n_pk), ("Verbatim", "v", n_values)],
        [("Execution", np.stack([s, n_schema + pk, n_schema + n_pk + v], 1))])
    return arrays


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
