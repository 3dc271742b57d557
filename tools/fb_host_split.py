"""Host split of one FlyBase query through matched() (the reference's call
pattern): the whole call, the lowering alone (`pattern_matcher._lower`, a
shape-cache hit), and the native call alone (`Context.plan_execute` on the
lowered words, ctypes included), medians over fresh anchors.  GPU box:

    python tools/fb_host_split.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
from das_amd import synthetic  # noqa: E402
from das_amd.database.hip_db import HipDB  # noqa: E402
from das_amd.pattern_matcher import pattern_matcher as pm  # noqa: E402
from das_amd import _lib  # noqa: E402
from das_amd.database.hip_db import Relation  # noqa: E402

torch.cuda.set_stream(torch.cuda.Stream(device=0))
db = HipDB(device=0)
arrays = synthetic.flybase_kb(300_000, 60, 450_000)
db.load_arrays(arrays)
db.prefetch()
genes = [(7 + 7919 * i) % 300_000 for i in range(300)]


def sets(lo, hi):
    return [[(n, bench.build_expr(pm, q)) for n, q in bench.flybase_specs(g, synthetic.flybase_do_terms(arrays, g))]
            for g in genes[lo:hi]]


def med(v):
    return round(sorted(v)[len(v) // 2] * 1e6, 1)


for qs in sets(0, 40):
    for _, q in qs:
        q.matched(db, pm.PatternMatchingAnswer())
torch.cuda.synchronize()
full, low, ex, cnt = {}, {}, {}, {}
for qs in sets(40, 140):
    for name, q in qs:
        k = name.split()[0]
        t0 = time.perf_counter()
        a = pm.PatternMatchingAnswer()
        q.matched(db, a)
        a.count()
        full.setdefault(k, []).append(time.perf_counter() - t0)
for qs in sets(140, 240):
    for name, q in qs:
        k = name.split()[0]
        t0 = time.perf_counter()
        w = pm._lower(q, db, False)
        low.setdefault(k, []).append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        m, neg, tabs = db.ctx.plan_execute(w, len(w) // 51, False)
        ex.setdefault(k, []).append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        a = pm.PatternMatchingAnswer()
        a._set(db, Relation(tabs))
        a.count()
        cnt.setdefault(k, []).append(time.perf_counter() - t0)
print("median us per query: matched()", {k: med(v) for k, v in full.items()})
print("  _lower (shape-cache hit)", {k: med(v) for k, v in low.items()})
print("  ctx.plan_execute (native + ctypes)", {k: med(v) for k, v in ex.items()})
print("  answer + count", {k: med(v) for k, v in cnt.items()})
ctypes_calls = []
for _ in range(200):
    t0 = time.perf_counter()
    _lib.counters()
    ctypes_calls.append(time.perf_counter() - t0)
print("  one trivial ctypes call (das_counters)", med(ctypes_calls))
