"""Host profile of the FlyBase step through the reference's call pattern
(one expr.matched(db, answer) per query, QueryFlyBase.ipynb cells 5-9):
wall per query shape, a cProfile of 40 steps, and with DAS_TRACE=1 the native
timeline of one step's calls on stderr.  Run on the GPU box:

    python tools/fb_matched_profile.py > out.txt 2> trace.txt
"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
from das_amd import synthetic  # noqa: E402
from das_amd.database.hip_db import HipDB  # noqa: E402
from das_amd.pattern_matcher import pattern_matcher as pm  # noqa: E402

torch.cuda.set_stream(torch.cuda.Stream(device=0))
db = HipDB(device=0)
arrays = synthetic.flybase_kb(300_000, 60, 450_000)
db.load_arrays(arrays)
db.prefetch()
genes = [(7 + 7919 * i) % 300_000 for i in range(200)]
sets = [[(n, bench.build_expr(pm, q)) for n, q in bench.flybase_specs(g, synthetic.flybase_do_terms(arrays, g))]
        for g in genes]


def step(qs):
    n = 0
    for _, q in qs:
        a = pm.PatternMatchingAnswer()
        q.matched(db, a)
        n += a.count()
    return n


for qs in sets[:40]:
    step(qs)
torch.cuda.synchronize()
per = {}
for qs in sets[40:120]:
    for name, q in qs:
        t0 = time.perf_counter()
        a = pm.PatternMatchingAnswer()
        q.matched(db, a)
        a.count()
        per.setdefault(name.split()[0], []).append(time.perf_counter() - t0)
print("per query median us:", {k: round(sorted(v)[len(v) // 2] * 1e6, 1) for k, v in per.items()})
t0 = time.perf_counter()
for qs in sets[120:160]:
    step(qs)
torch.cuda.synchronize()
print("step ms (matched one by one):", round((time.perf_counter() - t0) * 1e3 / 40, 4))
t0 = time.perf_counter()
for qs in sets[120:160]:
    pm.matched_many(db, [q for _, q in qs])
torch.cuda.synchronize()
print("step ms (matched_many):", round((time.perf_counter() - t0) * 1e3 / 40, 4))
pr = cProfile.Profile()
pr.enable()
for qs in sets[160:200]:
    step(qs)
pr.disable()
pstats.Stats(pr, stream=sys.stdout).sort_stats("tottime").print_stats(25)
