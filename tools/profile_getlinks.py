"""cProfile of bench.py's getlinks leg (one seed walk on the FlyBase-shaped KB):
where the host time of get_links / get_link_targets goes.

    python tools/profile_getlinks.py [out.txt]
"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import bench
    from das_amd import synthetic
    from das_amd.database.hip_db import HipDB
    from das_amd.distributed_atom_space import DistributedAtomSpace
    from das_amd.expression_hasher import ExpressionHasher as EH
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/profile_getlinks.txt"
    arrays = synthetic.flybase_kb(300_000, 60, 450_000)
    db = HipDB(device=0)
    db.load_arrays(arrays)
    db.prefetch()
    das = DistributedAtomSpace(db=db)
    seed = [EH.terminal_hash("gene", "g7")]
    bench.miner_walk(das, seed, np.random.default_rng(5), pattern_budget_s=3, progress=print)
    pr = cProfile.Profile()
    t = time.perf_counter()
    pr.enable()
    r = bench.miner_walk(das, seed, np.random.default_rng(5), pattern_budget_s=5, progress=print)
    pr.disable()
    print("walk", time.perf_counter() - t, r["pattern"])
    with open(out, "w") as f:
        f.write(f"{r}\n")
        pstats.Stats(pr, stream=f).sort_stats("tottime").print_stats(35)
        pstats.Stats(pr, stream=f).sort_stats("cumtime").print_stats(35)


if __name__ == "__main__":
    main()
