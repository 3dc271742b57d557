"""DAS_TRACE timeline of one batched bio step (Q3-Q6 through
pm.matched_many, as bench.py's step submits them) and the step's wall time
with and without the heavy-lead split; run on the GPU box with DAS_TRACE=1
for the timeline on stderr."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from das_amd.database.hip_db import HipDB  # noqa: E402
from das_amd.pattern_matcher import pattern_matcher as pm  # noqa: E402

sys.argv = [sys.argv[0]]
args = bench.parse()
torch.cuda.set_stream(torch.cuda.Stream(device=0))
db = HipDB(device=0)
arrays, specs, cfg, _ = bench.make_kb(bench.argparse.Namespace(**dict(vars(args), workload="bio")), 0, 1, db)
db.load_arrays(arrays)
db.prefetch()
sets = [[bench.build_expr(pm, s) for name, s in specs(i) if not name.startswith(("Q1", "Q2"))] for i in range(30)]
for qs in sets[:10]:
    pm.matched_many(db, qs)
torch.cuda.synchronize()
ts = []
for qs in sets[10:29]:
    t0 = time.perf_counter()
    pm.matched_many(db, qs)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
print("batched Q3-Q6 step ms (median)", round(sorted(ts)[len(ts) // 2] * 1e3, 3), flush=True)
pm.matched_many(db, sets[29])
torch.cuda.synchronize()
