"""Runs one FlyBase query shape (argv[1], e.g. FJ) over fresh gene anchors,
for rocprofv3 --kernel-trace: per-query wall vs its kernels' GPU time."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from das_amd import synthetic  # noqa: E402
from das_amd.database.hip_db import HipDB  # noqa: E402
from das_amd.pattern_matcher import pattern_matcher as pm  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "FJ"
arrays = synthetic.flybase_kb(300_000, 60, 450_000)
db = HipDB(device=0)
db.load_arrays(arrays)
db.prefetch()
genes = [(7 + 7919 * i) % 300_000 for i in range(40)]
qs = [e for g in genes for n, e in
      [(n, bench.build_expr(pm, s)) for n, s in bench.flybase_specs(g, synthetic.flybase_do_terms(arrays, gene=g))]
      if n.startswith(which)]
for e in qs[:10]:
    a = pm.PatternMatchingAnswer()
    e.matched(db, a)
    a.count()
t0 = time.perf_counter()
for e in qs[10:]:
    a = pm.PatternMatchingAnswer()
    e.matched(db, a)
    a.count()
print(f"{which}: {(time.perf_counter() - t0) * 1e6 / len(qs[10:]):.1f} us per query over {len(qs[10:])}", flush=True)
