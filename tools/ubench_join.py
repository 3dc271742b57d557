"""Join-kernel microbenchmark (run on the GPU box): direct-address join of a
large probe table against a small build table, for several probe-key
distributions, with the library's per-kernel HIP-event timings.

    python tools/ubench_join.py [--np 13500000] [--nb 100000] [--range 50000]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from das_amd import _lib  # noqa: E402
from das_amd.synthetic import zipf_indices  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--np", type=int, default=13_500_000)
    ap.add_argument("--nb", type=int, default=100_000)
    ap.add_argument("--range", type=int, default=50_000)
    ap.add_argument("--genes", type=int, default=200_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--unique-build", action="store_true", help="build keys distinct (semi-join shape)")
    args = ap.parse_args()
    import torch
    torch.cuda.init()
    ctx = _lib.Context(0, None)
    rng = np.random.default_rng(1)
    R, G = args.range, args.genes
    zipf = zipf_indices(rng, R, args.np).astype(np.uint32)
    keys = {"zipf": zipf, "uniform": rng.integers(0, R, args.np).astype(np.uint32), "zipf_sorted": np.sort(zipf)}
    genes = (R + rng.integers(0, G, args.np)).astype(np.uint32)
    if args.unique_build:
        bk = rng.permutation(R)[:min(args.nb, R)].astype(np.uint32)
    else:
        bk = rng.integers(0, R, args.nb).astype(np.uint32)
    bp = rng.integers(0, R, bk.shape[0]).astype(np.uint32)
    Q = ctx.table_from_host(_lib.TABLE_ORDERED, [1, 2], np.stack([bk, bp]))
    Q.set_bounds([0, 0], [R - 1, R - 1])
    out = {}
    for name, k in keys.items():
        P = ctx.table_from_host(_lib.TABLE_ORDERED, [0, 1], np.stack([genes, k]))
        P.set_bounds([R, 0], [R + G - 1, R - 1])
        ctx.join(P, Q).free()                       # warm-up
        ctx.prof_reset()
        ctx.prof_enable(True)
        n = 0
        for _ in range(args.reps):
            t = ctx.join(P, Q)
            n = t.nrows
            t.free()
        ctx.prof_enable(False)
        st = ctx.prof_stats()
        out[name] = {"out_rows": n, **{kn: {"us": round(v["ms"] * 1e3 / max(v["launches"], 1), 1),
                                            "GBps": round(v["bytes"] / max(v["ms"], 1e-9) / 1e6, 1)}
                                       for kn, v in st.items()}}
        P.free()
    print(json.dumps({"args": vars(args), "variant": os.environ.get("DAS_DJ_VARIANT", "0"), "results": out}))


if __name__ == "__main__":
    main()
