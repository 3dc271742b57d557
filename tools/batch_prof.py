"""Host / GPU split of the batched FlyBase step (bench.py --workload flybase
--batch 1): per fresh-anchor step, the Python lowering of the 5 queries, the
das_plan_execute_many call and the answer counts, plus one DAS_TRACE
timeline of the native call (run with DAS_TRACE=1 to get it on stderr)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from das_amd import synthetic  # noqa: E402
from das_amd.database.hip_db import HipDB  # noqa: E402
from das_amd.pattern_matcher import pattern_matcher as pm  # noqa: E402

arrays = synthetic.flybase_kb(300_000, 60, 450_000)
db = HipDB(device=0)
db.load_arrays(arrays)
db.prefetch()
genes = [(7 + 7919 * i) % 300_000 for i in range(80)]
sets = [[bench.build_expr(pm, s) for _, s in bench.flybase_specs(g, synthetic.flybase_do_terms(arrays, gene=g))]
        for g in genes]
no = bool(pm.CONFIG['no_overload'])
trace = os.environ.get("DAS_TRACE") is not None
tl, tx, tc, tw = [], [], [], []
for k, qs in enumerate(sets):
    t0 = time.perf_counter()
    words = []
    for e in qs:
        if type(e) is pm.And and not getattr(e, '_planned', False):
            e._plan_orders()
            e._planned = True
        w = pm._lower(e, db, no)
        e._plan = ((db.generation, no), w)
        words.append((w, len(w) // 51))
    t1 = time.perf_counter()
    outs = db.ctx.plan_execute_many(words, no)
    t2 = time.perf_counter()
    n = sum(t.nrows for _, _, ts in outs for t in ts)
    t3 = time.perf_counter()
    # the whole bench step on the next anchor set (lowering included)
    if k + 1 < len(sets):
        pass
    if k >= 10:
        tl.append(t1 - t0)
        tx.append(t2 - t1)
        tc.append(t3 - t2)
    if trace and k == len(sets) - 1:
        break
for k, qs in enumerate(sets[-20:]):
    t0 = time.perf_counter()
    sum(a.count() for _, a in pm.matched_many(db, qs))
    tw.append(time.perf_counter() - t0)
med = lambda v: sorted(v)[len(v) // 2] * 1e6  # noqa: E731
print({"lower_us": round(med(tl), 1), "execute_many_us": round(med(tx), 1), "count_us": round(med(tc), 1),
       "matched_many_step_us (warm anchors)": round(med(tw), 1)})

if os.environ.get("BP_CPROFILE"):
    import cProfile
    import pstats
    fresh = [[bench.build_expr(pm, s) for _, s in bench.flybase_specs(g, synthetic.flybase_do_terms(arrays, gene=g))]
             for g in [(11 + 104729 * i) % 300_000 for i in range(200)]]
    pr = cProfile.Profile()
    pr.enable()
    for qs in fresh:
        for e in qs:
            if type(e) is pm.And and not getattr(e, '_planned', False):
                e._plan_orders()
                e._planned = True
            pm._lower(e, db, no)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
