"""Per-query wall us over the bench's FlyBase steps (a fresh gene anchor per
step, bench.py make_kb), under DAS_CHAIN_GRID=0 / auto: which anchors cost
what.  Run on the GPU box."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from das_amd import _lib, synthetic  # noqa: E402
from das_amd.database.hip_db import HipDB  # noqa: E402
from das_amd.pattern_matcher import pattern_matcher as pm  # noqa: E402

arrays = synthetic.flybase_kb(300_000, 60, 450_000)
db = HipDB(device=0)
db.load_arrays(arrays)
db.prefetch()
n = 27
genes = [(7 + 7919 * i) % 300_000 for i in range(n)]
for mode in sys.argv[1:] or ["0", "auto"]:
    if mode == "auto":
        os.environ.pop("DAS_CHAIN_GRID", None)
    else:
        os.environ["DAS_CHAIN_GRID"] = mode
    tot = {}
    for i, g in enumerate(genes):
        row = []
        for name, spec in bench.flybase_specs(g, synthetic.flybase_do_terms(arrays, gene=g)):
            e = bench.build_expr(pm, spec)
            c0 = _lib.counters()
            t0 = time.perf_counter()
            a = pm.PatternMatchingAnswer()
            e.matched(db, a)
            k = a.count()
            us = (time.perf_counter() - t0) * 1e6
            c1 = _lib.counters()
            q = name.split()[0]
            if i >= 5:
                tot[q] = tot.get(q, 0) + us
            row.append(f"{q} {us:6.1f}us {k:7d}r {c1[0]-c0[0]:2d}L {c1[1]-c0[1]}R")
        print(f"mode {mode} gene {g:6d}: " + " | ".join(row), flush=True)
    print(f"mode {mode} mean over steps 5..: " + ", ".join(f"{q} {v / (n - 5):.1f}" for q, v in tot.items()),
          f"sum {sum(tot.values()) / (n - 5):.1f} us", flush=True)
