"""Host timeline of the native plan path for the FlyBase shapes (run on the
GPU box with DAS_TRACE=1): each query is run warm on one anchor, then once on
a fresh anchor; das_plan_execute prints its marks (kernel scopes, read-back
waits, plan nodes, microseconds from the call's start) to stderr.

    DAS_TRACE=1 python tools/trace_plan.py [--genes 300000] 2> trace.txt
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genes", type=int, default=300_000)
    ap.add_argument("--schema", type=int, default=60)
    ap.add_argument("--rows", type=int, default=450_000)
    ap.add_argument("--workload", choices=("flybase", "bio"), default="flybase",
                    help="bio: bench.py's Q1-Q6 on its bio_full KB (20 M Member links), warm and on a fresh gene pair")
    ap.add_argument("--cprofile", default=None, help="also: cProfile of 20 fresh anchors x 5 queries into this file")
    args = ap.parse_args()
    import torch
    import bench
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    from das_amd.pattern_matcher import pattern_matcher as pm
    if args.workload == "bio":
        arrays = synthetic.bio_full_kb(200_000, 50_000, 20_000_000, 100_000)
        db = HipDB(device=0)
        db.load_arrays(arrays)
        torch.cuda.synchronize()
        for anchor, tag in ((0, "warm-up"), (0, "warm"), (5, "fresh anchor")):
            for name, spec in bench.bio_specs(range(1, 200_000), anchor=anchor):
                q = bench.build_expr(pm, spec)
                print(f"[trace] === {name} ({tag})", file=sys.stderr, flush=True)
                t0 = time.perf_counter()
                a = pm.PatternMatchingAnswer()
                q.matched(db, a)
                n = a.count()
                dt = (time.perf_counter() - t0) * 1e6
                print(f"[trace] === {name} ({tag}): {dt:.1f} us wall, {n} bindings", file=sys.stderr, flush=True)
        return
    arrays = synthetic.flybase_kb(args.genes, args.schema, args.rows)
    db = HipDB(device=0)
    db.load_arrays(arrays)
    torch.cuda.synchronize()
    warm = 7
    # a fresh anchor with several DO terms (F9's Or has one term per term)
    fresh = next(g for g in range(7 + 7919 * 3, args.genes, 7919) if len(synthetic.flybase_do_terms(arrays, g)) >= 3)
    for gene, tag in ((warm, "warm-up"), (warm, "warm"), (fresh, "fresh anchor")):
        for name, spec in bench.flybase_specs(gene, synthetic.flybase_do_terms(arrays, gene)):
            q = bench.build_expr(pm, spec)
            print(f"[trace] === {name} ({tag})", file=sys.stderr, flush=True)
            t0 = time.perf_counter()
            a = pm.PatternMatchingAnswer()
            q.matched(db, a)
            n = a.count()
            dt = (time.perf_counter() - t0) * 1e6
            print(f"[trace] === {name} ({tag}): {dt:.1f} us wall, {n} bindings", file=sys.stderr, flush=True)
    if args.cprofile:
        import cProfile
        import pstats
        genes = [11 + 7919 * i for i in range(20)]
        qs = [bench.build_expr(pm, s) for g in genes
              for _, s in bench.flybase_specs(g, synthetic.flybase_do_terms(arrays, g))]
        pr = cProfile.Profile()
        t0 = time.perf_counter()
        pr.enable()
        for q in qs:
            a = pm.PatternMatchingAnswer()
            q.matched(db, a)
            a.count()
        pr.disable()
        dt = time.perf_counter() - t0
        with open(args.cprofile, "w") as f:
            f.write(f"{len(qs)} fresh-anchor queries in {dt * 1e3:.2f} ms ({dt * 1e6 / len(qs):.1f} us each)\n")
            pstats.Stats(pr, stream=f).sort_stats("tottime").print_stats(45)


if __name__ == "__main__":
    main()
