"""One-screen summary of a bench.py JSON line (headline + legs):
    python tools/bench_summary.py gpurun_out/r3_bench_all.json"""
import json
import sys


def show(d, name):
    r = d.get("roofline") or {}
    sr = d.get("step_roofline") or {}
    print(f"{name}: {d.get('value', 0):.4g} {d.get('unit')}  {d.get('ms_per_step', 0):.4f} ms/step  "
          f"roofline {r.get('kernel')} {r.get('frac')}  step_frac {sr.get('frac')}")
    q = (d.get("config") or {}).get("query_ms_rank0")
    if q:
        print("   query ms:", {k.split(' ')[0]: v for k, v in q.items()})
    ks = d.get("kernels") or {}
    print("   kernels:", {k: (v.get("avg_us"), v.get("launches")) for k, v in list(ks.items())[:7]})
    inc = d.get("incl_materialisation")
    if inc:
        print(f"   incl_materialisation {inc.get('value', 0):.4g} bindings/s")


d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
show(d, "headline")
for k, v in (d.get("workloads") or {}).items():
    show(v, k)
for k, v in (d.get("join_probe_variants") or {}).items():
    print("  join variant", k, v.get("ms_per_step") or v.get("ms_per_query"), (v.get("roofline") or {}).get("frac"))
