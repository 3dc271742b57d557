"""cProfile of fresh-anchor FlyBase queries (host side of a cold anchor)."""
import cProfile
import os
import pstats
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
genes = [(7 + 7919 * i) % 300_000 for i in range(60)]
sets = [[(n, bench.build_expr(pm, s)) for n, s in bench.flybase_specs(g, synthetic.flybase_do_terms(arrays, gene=g))]
        for g in genes]


def run(qs, which):
    out = {}
    for name, e in qs:
        if which and not name.startswith(which):
            continue
        t0 = time.perf_counter()
        a = pm.PatternMatchingAnswer()
        e.matched(db, a)
        a.count()
        out[name.split()[0]] = (time.perf_counter() - t0) * 1e6
    return out


for qs in sets[:5]:
    run(qs, None)
tot = {}
for qs in sets[5:30]:
    for k, v in run(qs, None).items():
        tot[k] = tot.get(k, 0) + v
print("all five per step:", {k: round(v / 25, 1) for k, v in tot.items()}, round(sum(tot.values()) / 25, 1))
tot = {}
for qs in sets[30:45]:
    for k, v in run(qs, "F5").items():
        tot[k] = tot.get(k, 0) + v
print("F5 alone per step:", {k: round(v / 15, 1) for k, v in tot.items()})
pr = cProfile.Profile()
pr.enable()
for qs in sets[45:60]:
    run(qs, None)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25); pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
