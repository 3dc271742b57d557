"""Per-query latency of the native plan path (das_plan_execute) against the
per-operator host path on the FlyBase-shaped KB (run on the GPU box):
fresh query objects every repetition (lowering included) and reused ones.

    python tools/plan_ab.py [--genes 300000] [--reps 30]
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
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--kernels", action="store_true", help="also: per-query kernel scopes (plan path, one run each)")
    args = ap.parse_args()
    import torch
    import bench
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    from das_amd.pattern_matcher import pattern_matcher as pm
    arrays = synthetic.flybase_kb(args.genes, args.schema, args.rows)
    genes = [7 + 7919 * i for i in range(8)]
    do = {g: synthetic.flybase_do_terms(arrays, g) for g in genes}
    db = HipDB(device=0)
    db.load_arrays(arrays)
    torch.cuda.synchronize()
    out = {}
    for mode in ("1", "0", "1", "0"):
        os.environ["DAS_PLAN"] = mode
        res = {}
        for fresh in (True, False):
            specs = [bench.flybase_specs(g, do[g]) for g in genes]
            qs0 = [[(n, bench.build_expr(pm, s)) for n, s in sp] for sp in specs]
            for k in range(len(qs0[0])):
                name = qs0[0][k][0]
                ts = []
                for r in range(args.reps):
                    sp = specs[r % len(genes)]
                    q = bench.build_expr(pm, sp[k][1]) if fresh else qs0[r % len(genes)][k][1]
                    t0 = time.perf_counter()
                    a = pm.PatternMatchingAnswer()
                    q.matched(db, a)
                    a.count()
                    ts.append(time.perf_counter() - t0)
                ts.sort()
                res[f"{name} {'fresh' if fresh else 'reused'}"] = round(ts[len(ts) // 2] * 1e6, 1)
        out[f"plan={mode}"] = res if f"plan={mode}" not in out else {k: [out[f'plan={mode}'][k], v] for k, v in res.items()}
    if args.kernels:
        os.environ["DAS_PLAN"] = "1"
        specs = bench.flybase_specs(genes[1], do[genes[1]])
        for name, s in specs:
            q = bench.build_expr(pm, s)
            a = pm.PatternMatchingAnswer()
            q.matched(db, a)                      # warm
            q = bench.build_expr(pm, bench.flybase_specs(genes[2], do[genes[2]])[[n for n, _ in specs].index(name)][1])
            db.ctx.prof_reset()
            db.ctx.prof_enable(True)
            a = pm.PatternMatchingAnswer()
            q.matched(db, a)
            n = a.count()
            db.ctx.prof_enable(False)
            st = db.ctx.prof_stats()
            out[f"kernels {name} (n={n})"] = {k: [v["launches"], round(v["ms"] * 1e3, 1)]
                                             for k, v in sorted(st.items(), key=lambda kv: -kv[1]["ms"])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
