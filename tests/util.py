"""Helpers shared by the tests: canonical forms of product answers, query
specs -> das_amd expression objects."""
import hashlib
import json

from das_amd.pattern_matcher import pattern_matcher as pm


def build(spec):
    kind = spec[0]
    if kind == "Node":
        return pm.Node(spec[1], spec[2])
    if kind == "Var":
        return pm.Variable(spec[1])
    if kind == "TVar":
        return pm.TypedVariable(spec[1], spec[2])
    if kind == "Link":
        return pm.Link(spec[1], [build(t) for t in spec[3]], spec[2])
    if kind == "Template":
        return pm.LinkTemplate(spec[1], [build(t) for t in spec[3]], spec[2])
    if kind == "Not":
        return pm.Not(build(spec[1]))
    if kind == "And":
        return pm.And([build(t) for t in spec[1]])
    if kind == "Or":
        return pm.Or([build(t) for t in spec[1]])
    raise ValueError(spec)


def canon(a):
    """Canonical identity in the golden-fixture layout (oracle.canon_json)."""
    if isinstance(a, pm.OrderedAssignment):
        return ["O", [list(x) for x in sorted(a.mapping.items())]]
    if isinstance(a, pm.UnorderedAssignment):
        vals = [k for k, c in a.values.items() for _ in range(c)]
        return ["U", sorted(a.symbols.keys()), sorted(vals)]
    if isinstance(a, pm.CompositeAssignment):
        parity = {}
        for u in a.unordered_mappings:
            k = json.dumps(canon(u))
            parity[k] = parity.get(k, 0) + 1
        odd = sorted(k for k, c in parity.items() if c % 2)
        o = a.ordered_mapping
        if o is not None and not odd:
            return canon(o)
        return ["C", None if o is None else [list(x) for x in sorted(o.mapping.items())],
                [json.loads(k) for k in odd]]
    raise TypeError(type(a))


def record(expr_spec, db):
    """Evaluate on the product; same record layout as the golden fixtures."""
    ans = pm.PatternMatchingAnswer()
    try:
        m = build(expr_spec).matched(db, ans)
    except NotImplementedError:
        raise
    except (AttributeError, ValueError, TypeError, AssertionError) as e:
        return {"error": type(e).__name__}
    rows = sorted(json.dumps(canon(a), sort_keys=True) for a in ans.assignments)
    return {"matched": bool(m), "negation": ans.negation, "n": len(ans.assignments),
            "sha256": hashlib.sha256("\n".join(rows).encode()).hexdigest(),
            "count": ans.count()}


def _rec(m, ans):
    rows = sorted(json.dumps(canon(a), sort_keys=True) for a in ans.assignments)
    return {"matched": bool(m), "negation": ans.negation, "n": len(ans.assignments),
            "sha256": hashlib.sha256("\n".join(rows).encode()).hexdigest(),
            "count": ans.count()}


def record_many(expr_specs, db):
    """record() of each spec, the batch evaluated by pm.matched_many (one
    das_plan_execute_many call on a HipDB)."""
    return [_rec(m, ans) for m, ans in pm.matched_many(db, [build(s) for s in expr_specs])]


def same(got, want):
    if want.get("error") or got.get("error"):
        return got.get("error") == want.get("error")
    # the device count (what bench.py reports) must equal the materialised set
    if "count" in got and got["count"] != got["n"]:
        return False
    return all(got[k] == want[k] for k in ("matched", "negation", "n", "sha256"))


def uses_composite(spec):
    """True if the reference would build a CompositeAssignment or check an
    unordered negation: an unordered Link/Template inside a multi-term And/Or."""
    def has_unordered(s):
        if s[0] in ("Link", "Template"):
            return (not s[2]) or any(has_unordered(t) for t in s[3] if isinstance(t, list))
        if s[0] == "Not":
            return has_unordered(s[1])
        if s[0] in ("And", "Or"):
            return any(has_unordered(t) for t in s[1])
        return False

    def walk(s):
        if s[0] in ("And", "Or"):
            if s[0] == "And" and len(s[1]) > 1 and has_unordered(s):
                return True
            return any(walk(t) for t in s[1])
        if s[0] == "Not":
            return walk(s[1])
        return False
    return walk(spec)
