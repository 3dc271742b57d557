"""Lowered-plan caching and the plan executor's answer-table capacity.

* An expression object caches its lowered das_plan_node_t records keyed by the
  index load they were lowered against.  Reused across two HipDBs (loaded
  with different KBs, the second possibly at the first one's address) it must
  re-lower, never replay the other index's atom / type ids.
* An Or of many Links with different variable sets has one answer table per
  schema; past the binding's first capacity guess (64) the call is repeated
  with the capacity the library reports, instead of failing."""
import gc

import pytest

from oracle import das_oracle as O
from tests.util import build, record, same

pytestmark = pytest.mark.gpu


def _db(arrays):
    from das_amd.database.hip_db import HipDB
    db = HipDB(device=0)
    db.load_arrays(arrays)
    return db


def _member_inh():
    V = lambda x: ["Var", x]  # noqa: E731
    return ["And", [["Link", "Member", True, [V("G"), V("B")]], ["Link", "Inheritance", True, [V("B"), V("P")]]]]


def test_gpu_expression_reused_across_dbs():
    from das_amd import synthetic
    from das_amd.pattern_matcher import pattern_matcher as pm
    spec = _member_inh()
    expr = build(spec)
    kbs = [synthetic.bio_kb(50, 20, 400, 40, seed=1), synthetic.bio_kb(90, 35, 700, 70, seed=2)]
    wants = [O.evaluate(spec, O.RedisMongoSemantics(O.KB.from_arrays(a))) for a in kbs]
    tokens = set()
    for k in (0, 1, 0, 1):
        db = _db(kbs[k])
        tokens.add(db.generation)
        ans = pm.PatternMatchingAnswer()
        m = expr.matched(db, ans)            # the same object every time: its plan cache is reused
        assert m == wants[k]["matched"]
        assert ans.count() == wants[k]["n"]
        assert same(record(spec, db), wants[k])
        del ans, db
        gc.collect()                         # the next HipDB may reuse this one's address
    assert len(tokens) == 4                  # one load token per load, across instances


def test_gpu_plan_more_answer_schemas_than_first_capacity():
    """Or of 80 single-Link terms, each binding its own variable: 80 schemas."""
    from das_amd import synthetic
    arrays = synthetic.bio_kb(40, 15, 300, 30, seed=4)
    db = _db(arrays)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    terms = [["Link", "Member", True, [["Node", "Gene", f"g{i % 40}"], ["Var", f"V{i}"]]] for i in range(80)]
    spec = ["Or", terms]
    want = O.evaluate(spec, odb)
    got = record(spec, db)
    assert same(got, want), (got, want.get("n"))
    assert want["n"] > 64


def test_gpu_shape_cache_patches_anchor_ids():
    """A query shape lowered once is reused for other anchors (the same tree
    with other node names): its words with the new nodes' ids patched in must
    equal a from-scratch lowering of the new expression, and the answers the
    oracle's -- including anchors that are no node of the KB (the constant
    records of the full lowering) and a Not term sharing the anchor node."""
    import bench
    from das_amd import synthetic
    from das_amd.pattern_matcher import pattern_matcher as pm
    arrays = synthetic.flybase_kb(400, 8, 1500, n_loc=30, n_do=20, seed=3)
    db = _db(arrays)
    odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    genes = [7, 11, 7, 250, 399, 3, 10**6]          # 10**6: FBgn id absent from the KB
    for g in genes:
        for name, spec in bench.flybase_specs(g, synthetic.flybase_do_terms(arrays, gene=g) if g < 400 else ()):
            e1, e2 = build(spec), build(spec)
            hit = pm._lower(e1, db, False)            # the shape cache, after the first gene
            db.__dict__.pop('_plan_shapes', None)
            db.__dict__.pop('_plan_records', None)
            full = pm._lower(e2, db, False)           # from scratch
            assert (hit is None) == (full is None), name
            if full is not None:
                assert hit.tobytes() == full.tobytes(), (name, g)
            want = O.evaluate(spec, odb)
            assert same(record(spec, db), want), (name, g)
