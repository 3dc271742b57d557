"""Link sharding helpers of das_amd.parallel (host code): content-hash
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


def test_shard_arrays_marks_remote_links():
    arrays = synthetic.powerlaw_kb(200, 1000, link_types=2, seed=3)
    kinds = [parallel.shard_arrays(synthetic.powerlaw_kb(200, 1000, link_types=2, seed=3), r, 2).expr_kind
             for r in range(2)]
    local = [(k == 1) for k in kinds]
    assert not np.any(local[0] & local[1])
    assert np.all(local[0] | local[1] | (arrays.expr_kind != 1))
