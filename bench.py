"""bench.py — DAS query hot path on MI355X: bindings/s + HBM roofline.

Workload (BASELINE.json configs[1], the config the metric is quoted on that
fits one GPU): a seeded synthetic gene-level KB in scripts/benchmark.py's
shape (Member(Gene, BiologicalProcess) with Zipf(1.1) process popularity,
Inheritance(BP, BP)); the real bio_atomspace dump is not available offline.
One step = one pass of the query batch below through the reference API
(`expr.matched(db, answer)`), single-Link and 2-clause And queries:

  Q1 Member(V_g, V_bp)                                  full single-link scan
  Q2 And[Member(V_g, V_bp), Inheritance(V_bp, V_p)]     2-clause join
  Q3 And[Member(g_a, V_bp), Member(g_b, V_bp)]          _same_biological_process
  Q4 And[Member(V_g, bp_hub), Member(V_g, V_bp)]        hub join

value = distinct bindings produced by all ranks / wall time (answers counted
on the device, no Python object materialisation).  Multi-GPU: links are
partitioned across ranks (Member by gene range, Inheritance by content hash)
and And joins repartition both binding tables by the join key with an RCCL
all-to-all (das_amd/parallel.py); per-rank KB size is fixed (weak scaling).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--genes", type=int, default=200_000)
    ap.add_argument("--bps", type=int, default=50_000)
    ap.add_argument("--members", type=int, default=20_000_000)
    ap.add_argument("--inheritance", type=int, default=100_000)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cprofile", default=None, help="write a host-side cProfile of 3 extra steps here")
    return ap.parse_args()


def queries(pm, rank_genes, n_bps, seed):
    import numpy as np
    rng = np.random.default_rng(seed)
    V = pm.Variable
    g = lambda i: pm.Node("Gene", f"g{i}")  # noqa: E731
    bp = lambda i: pm.Node("BiologicalProcess", f"bp{i}")  # noqa: E731
    member = lambda a, b: pm.Link("Member", [a, b], True)  # noqa: E731
    inh = lambda a, b: pm.Link("Inheritance", [a, b], True)  # noqa: E731
    ga, gb = (int(x) for x in rng.choice(rank_genes, 2, replace=False))
    return [
        ("Q1 Member(Vg,Vbp)", member(V("V_g"), V("V_bp"))),
        ("Q2 Member*Inheritance", pm.And([member(V("V_g"), V("V_bp")), inh(V("V_bp"), V("V_p"))])),
        ("Q3 same_biological_process", pm.And([member(g(ga), V("V_bp")), member(g(gb), V("V_bp"))])),
        ("Q4 hub join", pm.And([member(V("V_g"), bp(0)), member(V("V_g"), V("V_bp"))])),
    ]


def cpu_baseline(args, budget_s):
    """The oracle (CPU restatement keeping the reference's nested-loop join
    complexity) on a bounded sample of the same workload, one core."""
    from das_amd import synthetic
    from oracle import das_oracle as O
    scale = 1000
    genes, bps = max(args.genes // scale, 50), max(args.bps // scale, 20)
    members, inh = max(args.members // scale, 500), max(args.inheritance // scale, 40)
    arrays = synthetic.bio_kb(genes, bps, members, inh)
    db = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
    V = lambda n: ["Var", n]  # noqa: E731
    member = lambda a, b: ["Link", "Member", True, [a, b]]  # noqa: E731
    inh_l = lambda a, b: ["Link", "Inheritance", True, [a, b]]  # noqa: E731
    specs = [member(V("V_g"), V("V_bp")),
             ["And", [member(V("V_g"), V("V_bp")), inh_l(V("V_bp"), V("V_p"))]],
             ["And", [member(["Node", "Gene", "g1"], V("V_bp")), member(["Node", "Gene", "g2"], V("V_bp"))]],
             ["And", [member(V("V_g"), ["Node", "BiologicalProcess", "bp0"]), member(V("V_g"), V("V_bp"))]]]
    total, t0, passes = 0, time.perf_counter(), 0
    while True:
        for s in specs:
            total += O.evaluate(s, db).get("n", 0)
        passes += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": total / dt, "unit": "bindings/s", "cores": 1, "kind": "port",
            "sample": f"oracle (nested-loop And, reference complexity) on bio_kb(genes={genes}, bps={bps}, "
                      f"members={members}, inheritance={inh}) = 1/{scale} of the GPU workload, Q1-Q4, "
                      f"{passes} passes in {dt:.1f} s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    # DAS_BENCH_SAME_DEVICE=1 + DAS_DIST_BACKEND=gloo rehearse N ranks on one GPU
    if os.environ.get("DAS_BENCH_SAME_DEVICE") == "1":
        local_rank = 0
    backend = os.environ.get("DAS_DIST_BACKEND", "nccl")
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    from das_amd.pattern_matcher import pattern_matcher as pm

    # ---- knowledge base (per-rank partition for N > 1) ----
    t_build = time.perf_counter()
    if world == 1:
        arrays = synthetic.bio_kb(args.genes, args.bps, args.members, args.inheritance)
        rank_genes = np.arange(args.genes)
    else:
        from das_amd import parallel
        arrays, rank_genes = parallel.bio_shard(args.genes, args.bps, args.members, args.inheritance, rank, world)
    db = HipDB(device=local_rank)
    db.load_arrays(arrays)
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t_build
    qs = queries(pm, rank_genes, args.bps, seed=17)
    if world > 1:
        from das_amd import parallel
        engine = parallel.ShardedMatcher(db, dist, cpu_staging=(backend != "nccl"))

        def run(q):
            return engine.count(q)
    else:
        def run(q):
            ans = pm.PatternMatchingAnswer()
            q.matched(db, ans)
            return ans.count()

    def step():
        return sum(run(q) for _, q in qs)

    for _ in range(args.warmup):
        step()
    per_query = {name: run(q) for name, q in qs}
    db.ctx.prof_reset()
    db.ctx.prof_enable(True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bindings = 0
    for _ in range(args.steps):
        bindings += step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    db.ctx.prof_enable(False)
    stats = db.ctx.prof_stats()
    if args.cprofile and rank == 0:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(3):
            step()
        pr.disable()
        with open(args.cprofile, "w") as f:
            pstats.Stats(pr, stream=f).sort_stats("tottime").print_stats(40)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        b = torch.tensor([bindings], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(b)
        bindings = float(b.item())
    value = bindings / elapsed

    # dominant kernel of the timed region -> roofline
    # single-kernel scopes only ("k_*"); multi-launch phases such as join_build
    # are reported under "kernels" but are not a kernel's roofline
    single = {k: v for k, v in stats.items() if k.startswith("k_")}
    dom = max(single.items(), key=lambda kv: kv[1]["ms"]) if single else None
    roofline = None
    if dom:
        name, st = dom
        achieved = st["bytes"] / (st["ms"] * 1e-3) / 1e9 if st["ms"] > 0 else 0.0
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                traffic = json.load(f).get(name, {}).get("bytes_per_launch")
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": name,
                    "avg_launch_us": round(st["ms"] * 1e3 / max(st["launches"], 1), 2),
                    "algorithmic_bytes_per_launch": st["bytes"] / max(st["launches"], 1)}
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args, args.cpu_baseline_seconds)
        out = {
            "metric": "pattern matches/sec (bindings/s) + % HBM roofline",
            "value": value, "unit": "bindings/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (seeded bio_kb in scripts/benchmark.py shape; bio_atomspace dump unavailable offline)",
            "config": {"workload": "config2 bio gene-level KB: single-Link + 2-clause And (Q1-Q4)",
                       "genes_per_rank": int(len(rank_genes)), "bps": args.bps,
                       "member_links_per_rank": args.members, "inheritance_links": args.inheritance,
                       "bindings_per_step_rank0": per_query, "parallelism": f"links sharded x{world}"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "kernels": {k: {"ms": round(v["ms"], 3), "launches": v["launches"],
                            "GBps": round(v["bytes"] / max(v["ms"], 1e-9) / 1e6, 1)} for k, v in stats.items()},
            "build_s": round(t_build, 2),
        }
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
