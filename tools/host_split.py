"""Where a fresh-anchor FlyBase query spends its host time (run on the GPU
box): wall time of Expression.matched + answer.count(), split into the
Python lowering (pattern_matcher._lower), the native call
(Context.plan_execute) and the rest; medians over fresh gene anchors.

    python tools/host_split.py [--anchors 24]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genes", type=int, default=300_000)
    ap.add_argument("--schema", type=int, default=60)
    ap.add_argument("--rows", type=int, default=450_000)
    ap.add_argument("--anchors", type=int, default=24)
    args = ap.parse_args()
    import torch
    import bench
    from das_amd import _lib, synthetic
    from das_amd.database.hip_db import HipDB
    from das_amd.pattern_matcher import pattern_matcher as pm
    arrays = synthetic.flybase_kb(args.genes, args.schema, args.rows)
    db = HipDB(device=0)
    db.load_arrays(arrays)
    torch.cuda.synchronize()
    acc = {"lower": 0.0, "native": 0.0}
    real_lower, real_exec = pm._lower, _lib.Context.plan_execute

    def lower(*a, **k):
        t0 = time.perf_counter()
        try:
            return real_lower(*a, **k)
        finally:
            acc["lower"] += time.perf_counter() - t0

    def execute(self, *a, **k):
        t0 = time.perf_counter()
        try:
            return real_exec(self, *a, **k)
        finally:
            acc["native"] += time.perf_counter() - t0
    pm._lower, _lib.Context.plan_execute = lower, execute
    res = {}
    for rnd, genes in (("warm-up", [5 + 7919 * i for i in range(4)]),
                       ("fresh", [13 + 7919 * i for i in range(args.anchors)])):
        specs = [bench.flybase_specs(g, synthetic.flybase_do_terms(arrays, g)) for g in genes]
        qs = [[(n, bench.build_expr(pm, s)) for n, s in sp] for sp in specs]
        rows = {}
        for step in qs:
            for name, q in step:
                acc["lower"] = acc["native"] = 0.0
                t0 = time.perf_counter()
                a = pm.PatternMatchingAnswer()
                q.matched(db, a)
                a.count()
                wall = time.perf_counter() - t0
                rows.setdefault(name, []).append((wall, acc["lower"], acc["native"]))
        if rnd == "fresh":
            for name, v in rows.items():
                med = lambda i: sorted(x[i] for x in v)[len(v) // 2] * 1e6  # noqa: E731
                res[name] = {"wall_us": round(med(0), 1), "lower_us": round(med(1), 1),
                             "native_us": round(med(2), 1),
                             "rest_us": round(med(0) - med(1) - med(2), 1)}
            res["step_us (sum of medians)"] = round(sum(r["wall_us"] for r in res.values()), 1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
