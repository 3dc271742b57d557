"""Compares a 1-GPU bench line with the same bench at N ranks (bench.py
--gpus N, e.g. the 2-ranks-on-one-GPU gloo rehearsal) on the same sizes:

* bio (weak scaling): each rank's QUERY_1-3 instance ("Q3 ... @rank r")
  answers exactly as at 1 GPU; Q1 / Q2 / Q4 grow with the gene Member rows
  (every rank's are the 1-GPU rows on its own gene range) while the shared
  annotation-layout Member links count once, so they lie in (1, N] x the
  1-GPU answer (reported with the ratio);
* flybase / hub (strong scaling, one KB): every answer size is the 1-GPU one;
* build: the distinct links indexed over all ranks equal 1 GPU's.

    python tools/rehearse_check.py <1gpu.json> <Nranks.json> [out.json]
"""
import json
import sys


def load(path):
    with open(path) as f:
        return json.loads([l for l in f if l.startswith("{")][-1])


def sizes(line):
    c = line.get("config", {})
    return c.get("bindings_per_step") or c.get("bindings_per_step_rank0") or {}


def check_bio(a, b, n):
    out, ok = {}, True
    qa = sizes(a)
    for name, v in sizes(b).items():
        base = name.split(" @rank")[0]
        want = qa.get(base)
        if want is None:
            continue
        if " @rank" in name:
            good = v == want
            out[name] = {"1gpu": want, "n_ranks": v, "expected": want, "ok": good}
        else:
            good = want < v <= n * want
            out[name] = {"1gpu": want, "n_ranks": v, "ratio": round(v / max(want, 1), 4), "ok": good}
        ok &= good
    return ok, out


def check_equal(a, b):
    out, ok = {}, True
    qa = sizes(a)
    for name, v in sizes(b).items():
        out[name] = {"1gpu": qa.get(name), "n_ranks": v, "ok": qa.get(name) == v}
        ok &= qa.get(name) == v
    return ok, out


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    n = int(b.get("n_gpus", 2))
    res = {"n_ranks": n}
    legs = [("headline", a, b)] + [(w, a.get("workloads", {}).get(w), b.get("workloads", {}).get(w))
                                   for w in b.get("workloads", {})]
    allok = True
    for w, la, lb in legs:
        if not la or not lb or "error" in lb:
            continue
        wl = (lb.get("config") or {}).get("workload", "")
        if wl.startswith("config2"):
            ok, d = check_bio(la, lb, n)
        elif wl.startswith("config4"):
            x, y = la["config"]["distinct_links_indexed"], lb["config"]["distinct_links_indexed"]
            ok, d = x == y, {"distinct_links_indexed": {"1gpu": x, "n_ranks": y}}
        else:
            ok, d = check_equal(la, lb)
        res[w] = {"ok": ok, "queries": d, "ms_per_step_1gpu": la.get("ms_per_step"),
                  "ms_per_step_n_ranks": lb.get("ms_per_step"), "sharded_plan_stats": lb.get("sharded_plan_stats")}
        allok &= ok
    res["ok"] = allok
    s = json.dumps(res, indent=1)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(s + "\n")
    print(s)
    sys.exit(0 if allok else 1)


if __name__ == "__main__":
    main()
