"""The full-size closed forms of tests/test_gpu_fullsize.py pinned against
the oracle on small instances of the same generator (CPU): scripts/benchmark.py
QUERY_2 / QUERY_3 (bench Q5 / Q6) counts and answer checksums
(tests/checksum.py) from the generator's distinct link pairs equal the
oracle's nested-loop evaluation of the reference fold, and the checksum
function itself behaves as a set checksum should."""
import numpy as np
import pytest

from oracle import das_oracle as O
from tests import checksum as CK


def _oracle_ck(rec):
    """(rows, checksum) of an oracle record's ordered rows."""
    assert all(r[0] == "O" for r in rec["rows"])
    return rec["n"], CK.rows_checksum(dict(r[1]) for r in rec["rows"])


def test_checksum_function_properties():
    """Order independence, column-order independence, sensitivity to a swap
    of values between rows, and the three implementations agreeing."""
    import hashlib
    rng = np.random.default_rng(3)
    hx = [hashlib.md5(str(i).encode()).hexdigest() for i in range(50)]
    rows = [{"A": hx[rng.integers(50)], "B": hx[rng.integers(50)]} for _ in range(40)]
    base = CK.rows_checksum(rows)
    assert CK.rows_checksum(rows[::-1]) == base
    assert CK.rows_checksum([{"B": r["B"], "A": r["A"]} for r in rows]) == base
    swapped = [dict(r) for r in rows]
    swapped[0]["B"], swapped[1]["B"] = rows[1]["B"], rows[0]["B"]
    if rows[0]["B"] != rows[1]["B"] and rows[0]["A"] != rows[1]["A"]:
        assert CK.rows_checksum(swapped) != base
    renamed = [{"A": r["A"], "C": r["B"]} for r in rows]
    assert CK.rows_checksum(renamed) != base
    # numpy and torch forms
    da = np.array([CK.d64_hex(r["A"]) for r in rows], dtype=np.uint64)
    db_ = np.array([CK.d64_hex(r["B"]) for r in rows], dtype=np.uint64)
    assert CK.sum_np(CK.prod_np(CK.g_np("A", da), CK.g_np("B", db_))) == base
    import torch
    ta, tb = torch.from_numpy(da.view(np.int64)), torch.from_numpy(db_.view(np.int64))
    assert CK.sum_torch(CK.g_torch("A", ta) * CK.g_torch("B", tb)) == base
    # a cross product's checksum is the product of the sides' checksums
    left = [{"A": h} for h in hx[:7]]
    right = [{"B": h} for h in hx[7:12]]
    cross = [{**a, **b} for a in left for b in right]
    assert CK.rows_checksum(cross) == (CK.rows_checksum(left) * CK.rows_checksum(right)) & CK.M64


@pytest.mark.parametrize("anchor", [0, 1, 2])
def test_query23_closed_forms_match_oracle(anchor):
    import bench
    from das_amd import synthetic
    from tests.test_gpu_fullsize import _pairs, _query23_counts
    ng, nb = 300, 80
    arrays = synthetic.bio_full_kb(ng, nb, 6000, 300, n_uniprot=60, n_up_member=800, n_reactome=15, n_context=300,
                                   n_loc=8)
    base = len(arrays.type_names)
    specs = dict(bench.bio_specs(np.arange(ng), anchor=anchor))
    rng = np.random.default_rng(17 + 7919 * anchor)        # bench.bio_specs' anchors
    ga, gb = (int(x) for x in rng.choice(np.arange(ng), 2, replace=False))
    want = _query23_counts(arrays, ng, nb, base, ga, gb, _pairs(arrays, "Member"), _pairs(arrays, "Inheritance"),
                           n_up=60, n_r=15, n_loc=8)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    for name, n in want.items():
        assert _oracle_ck(O.evaluate(specs[name], odb)) == n, name


@pytest.mark.parametrize("gene", [0, 7, 42])
def test_flybase_closed_forms_match_oracle(gene):
    import bench
    from das_amd import synthetic
    from tests.test_gpu_fullsize import _flybase_counts
    arrays = synthetic.flybase_kb(300, 8, 400, n_loc=20, n_do=30)
    do_terms = synthetic.flybase_do_terms(arrays, gene=gene)
    want = _flybase_counts(arrays, gene, do_terms)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    for name, spec in bench.flybase_specs(gene, do_terms):
        assert _oracle_ck(O.evaluate(spec, odb)) == want[name], name
