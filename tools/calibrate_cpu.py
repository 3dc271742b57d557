"""CPU-baseline calibration: the oracle's query time
against the reference's own, on the same KBs and queries, in one container.

The reference cannot travel to the GPU box, so bench.py times the oracle (a
restatement that keeps the reference's nested-loop `And`) on the box's host
cores.  This script runs the oracle over every query of the reference-answered
fixtures (tests/golden/kb_{bio_full,flybase,powerlaw,hub}.json, whose
`ref_seconds` are the reference's matched() wall times measured in this
container by make_golden.py) and writes the per-fixture time ratio to
profiles/cpu_calibration.json; bench.py reports it beside its cpu_baseline.

    python tools/calibrate_cpu.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from das_amd import loader  # noqa: E402
from oracle import das_oracle as O  # noqa: E402
from tests.golden import make_synthetic as MS  # noqa: E402


def _ratios(fast):
    """Per fixture: the oracle's matched() time (And fold joined as the
    reference's nested loop, or by hash when `fast`) over the reference's."""
    O.FAST_JOIN = fast
    out, tot_o, tot_r = {}, 0.0, 0.0
    for name in ("bio_full", "flybase", "powerlaw", "hub"):
        with open(os.path.join(ROOT, "tests", "golden", f"kb_{name}.json")) as f:
            d = json.load(f)
        db = O.RedisMongoSemantics(O.KB.from_arrays(loader.parse_canonical(MS.text_of(name)).finish()),
                                   tuple_targets=True)
        t_o = t_r = 0.0
        n = 0
        for q in d["queries"]:
            if "ref_seconds" not in q:
                continue
            O.CONFIG["no_overload"] = bool(q.get("no_overload"))
            t0 = time.perf_counter()
            O.evaluate(q["query"], db)
            t_o += time.perf_counter() - t0
            O.CONFIG["no_overload"] = False
            t_r += q["ref_seconds"]
            n += q.get("n", 0)
        out[name] = {"queries": len(d["queries"]), "bindings": n, "oracle_s": round(t_o, 4),
                     "reference_s": round(t_r, 4), "ratio": round(t_o / t_r, 4)}
        tot_o += t_o
        tot_r += t_r
    return {"fixtures": out, "ratio_all": round(tot_o / tot_r, 4)}


def main():
    out = {"what": "oracle matched() time / reference matched() time, same KB and queries, one core each, "
                   "build container (nproc = %d); nested: the oracle's And fold as the reference's nested loop "
                   "(FAST_JOIN=False, what bench.py's cpu_baseline runs), hash: joined by hash on the shared "
                   "variables (FAST_JOIN=True, bench.py's cpu_fast)" % os.cpu_count(),
           "joins": {"nested": _ratios(False), "hash": _ratios(True)}}
    path = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
