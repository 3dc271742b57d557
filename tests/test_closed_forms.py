"""The full-size closed forms of tests/test_gpu_fullsize.py pinned against
the oracle on small instances of the same generator (CPU): scripts/benchmark.py
QUERY_2 / QUERY_3 (bench Q5 / Q6) counts from the generator's distinct link
pairs equal the oracle's nested-loop evaluation of the reference fold."""
import numpy as np
import pytest

from oracle import das_oracle as O


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
        assert O.evaluate(specs[name], odb)["n"] == n, name


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
        assert O.evaluate(spec, odb)["n"] == want[name], name
