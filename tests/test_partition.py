"""Link sharding helpers of das_amd.parallel (host code): handle-owner
partitions are disjoint, cover the KB, and keep nested links whole."""
import numpy as np

from das_amd import loader, parallel, synthetic
from oracle import das_oracle as O


def _nested():
    b = loader.AtomBuilder()
    n = [b.terminal("Concept", f"c{i}", True) for i in range(6)]
    l1 = b.expr("List", [n[0], n[1]])
    b.expr("Evaluation", [n[2], l1])
    b.expr("Evaluation", [n[3], l1])
    b.expr("Member", [b.expr("List", [n[5], l1, n[5]]), n[1], n[2]])
    return b.finish()


def test_partition_arrays_cover_and_disjoint():
    for arrays in (synthetic.powerlaw_kb(300, 3000, link_types=3, seed=2), _nested()):
        full = O.KB.from_arrays(arrays).links
        parts = [O.KB.from_arrays(parallel.partition_arrays(arrays, r, 3)).links for r in range(3)]
        union = {}
        for p in parts:
            union.update(p)
        assert union == full
        # top-level links land on exactly one shard (nested ones follow their parents)
        tops = [set(p) for p in parts]
        nested_handles = {t for (_, tg, _) in full.values() for t in tg if t in full}
        for i in range(3):
            for j in range(i + 1, 3):
                assert not ((tops[i] & tops[j]) - nested_handles)


def test_host_owners_are_handle_owners():
    """parallel.host_owners = int(handle[:8], 16) % world of each expression's
    reference handle (the device's das_hash_owners, common.h handle_owner)."""
    for arrays in (synthetic.powerlaw_kb(200, 1000, link_types=2, seed=3), _nested()):
        kb_hex = _expr_handles(arrays)
        for world in (2, 3, 8):
            got = parallel.host_owners(arrays, world)
            assert got.tolist() == [int(h[:8], 16) % world for h in kb_hex]


def _expr_handles(arrays):
    leaf = [O.md5hex(s) for s in arrays.leaf_strings()]
    h = leaf + [None] * arrays.n_expr
    for j in sorted(range(arrays.n_expr), key=lambda j: arrays.expr_level[j]):
        h[arrays.n_leaf + j] = O.composite_hash([h[c] for c in arrays.children(j)])
    return h[arrays.n_leaf:]


def test_shard_arrays_declares_the_handle_split():
    arrays = synthetic.powerlaw_kb(200, 1000, link_types=2, seed=3)
    kinds = arrays.expr_kind.copy()
    a = parallel.shard_arrays(arrays, 1, 2)
    assert a.shard == (1, 2) and np.array_equal(a.expr_kind, kinds)     # the build splits by handle
