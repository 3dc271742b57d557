"""Host timeline (DAS_TRACE=1) of the FlyBase queries under the one-workgroup
and the grid chain (DAS_CHAIN_GRID), plus wall us per query: where a fused
And's time goes.  Run on the GPU box: python tools/chain_diag.py [genes...]"""
import os
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
genes = [int(g) for g in sys.argv[1:]] or [7]
for gene in genes:
    specs = bench.flybase_specs(gene, synthetic.flybase_do_terms(arrays, gene=gene))
    for mode in ("0", "1"):
        os.environ["DAS_CHAIN_GRID"] = mode
        for name, spec in specs:
            e = bench.build_expr(pm, spec)
            for _ in range(3):
                a = pm.PatternMatchingAnswer()
                e.matched(db, a)
                a.count()
            t0 = time.perf_counter()
            for _ in range(10):
                a = pm.PatternMatchingAnswer()
                e.matched(db, a)
                n = a.count()
            us = (time.perf_counter() - t0) * 1e5
            print(f"gene {gene} grid {mode} {name.split()[0]}: {us:.1f} us, {n} rows", flush=True)
            if name.split()[0] in ("F5", "F6", "F7"):
                os.environ["DAS_TRACE"] = "1"
                a = pm.PatternMatchingAnswer()
                e.matched(db, a)
                a.count()
                os.environ.pop("DAS_TRACE")
