"""FJ (uniquename x recombination_loc) on the bench's FlyBase KB: its lowered
plan records (op, index_join, scan rows per node) and one evaluation; run
with DAS_TRACE=1 for the host timeline on stderr."""
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
spec = dict(bench.flybase_specs(7, synthetic.flybase_do_terms(arrays, gene=7)))["FJ uniquename x recombination_loc"]
e = bench.build_expr(pm, spec)
w = pm._lower(e, db, False)
n = len(w) // 51
rows = db.ctx.plan_estimates(w, n) if hasattr(db.ctx, "plan_estimates") else None
for i in range(n):
    r = w[51 * i: 51 * (i + 1)]
    print("node", i, "op", int(r[0]), "words0-8", [int(x) for x in r[:9]], "rows", None if rows is None else int(rows[i]))
for _ in range(3):
    a = pm.PatternMatchingAnswer()
    e.matched(db, a)
t0 = time.perf_counter()
a = pm.PatternMatchingAnswer()
e.matched(db, a)
print("FJ", a.count(), "rows", (time.perf_counter() - t0) * 1e6, "us")
