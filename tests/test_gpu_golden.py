"""GPU parity against the reference's own answers on the config 2-5 shapes
(tests/golden/kb_{bio_full,flybase,powerlaw,hub}.json, written by running the
reference here: make_synthetic.py + make_golden.py).  The KB text is
regenerated from the seeded generator (its sha256 must equal the one the
reference loaded), read by the native canonical reader, hashed and indexed
on the GPU, and every query is replayed through the reference API on the
HIP path: scripts/benchmark.py QUERY_1-3 (nested And / Or / LinkTemplate
targets inside Context / Evaluation), bench.py's bio / FlyBase / hub query
batches, random shapes, and CONFIG['no_overload'] = True entries."""
import hashlib
import json

import pytest

from tests.golden import make_synthetic as MS
from tests.util import record, same

pytestmark = pytest.mark.gpu

FIXTURES = ["bio_full", "flybase", "powerlaw", "hub"]


def _table_sha(rows):
    return hashlib.sha256("\n".join(json.dumps(r) for r in sorted(rows)).encode()).hexdigest()


def _atom_tables(db):
    """What the reference stored in Mongo (make_golden.atom_table), read back
    from the device index: nodes (handle, type, name); links (handle, type,
    targets, composite type hash)."""
    from das_amd.expression_hasher import ExpressionHasher as EH
    nodes, links = [], {}
    for t in db.arrays.type_names:
        hs = db.get_all_nodes(t)
        nodes += [[h, t, n] for h, n in zip(hs, db.get_all_nodes(t, names=True))]
        for h, targets in db.get_matched_type(t):
            links[h] = (t, list(targets))
    ctype = {h: EH.named_type_hash(t) for h, t, _ in nodes}

    def ct(h):
        if h not in ctype:
            t, targets = links[h]
            ctype[h] = EH.composite_hash([EH.named_type_hash(t)] + [ct(x) for x in targets])
        return ctype[h]
    return nodes, [[h, t, tg, ct(h)] for h, (t, tg) in links.items()]


@pytest.mark.parametrize("plan", ["1", "1-unfused", "1-multi", "1-sparse", "1-dense", "1-rev", "1-grid", "0"])
@pytest.mark.parametrize("name", FIXTURES)
def test_gpu_matches_reference_on_synthetic(golden, name, plan, monkeypatch):
    """plan 1: And / Or / Not trees folded natively (das_plan_execute), small
    Ands fused into one launch; 1-unfused: the same without the fused chain;
    1-multi: Ors of Link scans always through the multi-segment scan +
    dedup; 1-sparse / 1-dense: every direct join's build side through the
    in-place (lo, cnt) descriptors / the histogram + scan (the default picks
    by size, and these KBs are below the sparse floor); 1-rev: unfused, an
    And's second Link term index-joined into the first term's index at every
    size (DAS_REV_IJ=1); 1-grid: every fused And the grid chain can take
    through it (DAS_CHAIN_GRID=1); plan 0: the per-operator host path."""
    monkeypatch.setenv("DAS_PLAN", plan[0])
    monkeypatch.setenv("DAS_FUSED", "0" if plan in ("1-unfused", "1-rev") else "1")
    monkeypatch.setenv("DAS_REV_IJ", "1" if plan == "1-rev" else "")
    monkeypatch.setenv("DAS_UNION_MULTI", "1" if plan == "1-multi" else "0")
    if plan == "1-grid":
        monkeypatch.setenv("DAS_CHAIN_GRID", "1")
    else:
        monkeypatch.delenv("DAS_CHAIN_GRID", raising=False)
    if plan in ("1-sparse", "1-dense"):
        monkeypatch.setenv("DAS_DJ_BUILD", plan[2:])
    else:
        monkeypatch.delenv("DAS_DJ_BUILD", raising=False)
    from das_amd.database.hip_db import HipDB
    from das_amd.pattern_matcher import pattern_matcher as pm
    d = golden(f"kb_{name}.json")
    text = MS.text_of(name)
    assert hashlib.sha256(text.encode()).hexdigest() == d["text_sha256"]
    db = HipDB(device=0, tuple_targets=True)
    db.load_canonical(text)
    assert list(db.count_atoms()) == d["count_atoms"]
    nodes, links = _atom_tables(db)
    assert _table_sha(nodes) == d["nodes_sha256"]
    assert _table_sha(links) == d["links_sha256"]
    bad = []
    for q in d["queries"]:
        pm.CONFIG["no_overload"] = bool(q.get("no_overload"))
        try:
            got = record(q["query"], db)
        finally:
            pm.CONFIG["no_overload"] = False
        if not same(got, q):
            bad.append((q["query"], q.get("no_overload"), got.get("n", got), q.get("n", q.get("error"))))
    assert not bad, bad
    if plan[0] == "1":
        # scripts/benchmark.py QUERY_2 / QUERY_3 (ordered LinkTemplate terms,
        # Links with template targets inside And / Or) take the native plan
        from tests.util import build
        tq = [q["query"] for q in d["queries"] if _has_ordered_templates_below_root(q["query"])]
        assert tq or name != "bio_full"
        for spec in tq:
            e = build(spec)
            e.matched(db, pm.PatternMatchingAnswer())
            assert getattr(e, "_plan", (None, None))[1] is not None, spec


def _has_ordered_templates_below_root(spec):
    def templates(s):
        if not isinstance(s, list) or not s:
            return []
        if s[0] == "Template":
            return [s]
        if s[0] == "Link":
            return [t for x in s[3] for t in templates(x)]
        if s[0] == "Not":
            return templates(s[1])
        if s[0] in ("And", "Or"):
            return [t for x in s[1] for t in templates(x)]
        return []
    ts = templates(spec)
    return spec[0] in ("And", "Or") and bool(ts) and all(t[2] for t in ts)


@pytest.mark.parametrize("plan", ["1", "0", "many"])
def test_gpu_pattern_black_list_reference_mode(golden, plan, monkeypatch, tmp_path):
    """HipDB(stale_pattern_keys=True): the reference canonical loader's own
    pattern_black_list behaviour (canonical_parser.py:144-180, stale `keys`),
    for EVERY canonical-loader case of kb_blacklist.json -- every query and
    every index probe equals the reference's recorded answer (including the
    queries the stale entries touch and their AssertionErrors), and a
    blacklisted first link fails the load with UnboundLocalError.  plan: 1 =
    one query at a time (plans where no stale key is touched), 0 = the
    per-operator path, many = the queries in one pm.matched_many batch; then
    the same through the facade (load_canonical_knowledge_base)."""
    import os
    from das_amd.database.hip_db import HipDB
    from das_amd.distributed_atom_space import DistributedAtomSpace
    from tests.util import record_many
    monkeypatch.setenv("DAS_PLAN", "0" if plan == "0" else "1")
    d = golden("kb_blacklist.json")
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data")
    checked = touched = probes = failed_loads = 0
    for case in d["cases"]:
        if case["loader"] != "canonical":
            continue
        if case["source"] == "inline":
            text = d["canonical_text"]
        else:
            with open(os.path.join(here, os.path.basename(case["source"]))) as f:
                text = f.read()
        db = HipDB(device=0, tuple_targets=True, stale_pattern_keys=True)
        db.pattern_black_list = list(case["black_list"])
        if case.get("load_error"):
            with pytest.raises(UnboundLocalError):
                db.load_canonical(text)
            failed_loads += 1
            continue
        db.load_canonical(text)
        assert list(db.count_atoms()) == case["count_atoms"]
        qs = [q["query"] for q in case["queries"]]
        got = record_many(qs, db) if plan == "many" else [record(q, db) for q in qs]
        for q, g in zip(case["queries"], got):
            assert same(g, q), (case["black_list"], q["query"], g, {k: q.get(k) for k in ("n", "error")})
            checked += 1
        touched += sum(1 for q in qs if db.touches_stale(_build(q)))
        for p in case.get("index") or []:
            args = p["args"]
            try:
                if p["kind"] == "links":
                    r = db.get_matched_links(*args)
                elif p["kind"] == "template":
                    r = db.get_matched_type_template(args)
                else:
                    r = db.get_matched_type(args)
            except (ValueError, AssertionError, AttributeError, KeyError) as e:
                assert p.get("error") == type(e).__name__, (case["black_list"], p)
                continue
            assert "error" not in p, (case["black_list"], p)
            assert sorted(x if isinstance(x, str) else x[0] for x in r) == p["handles"], (case["black_list"], p)
            probes += 1
        # the facade: DistributedAtomSpace(stale_pattern_keys=True)
        f = tmp_path / "kb.metta"
        f.write_text(text)
        das = DistributedAtomSpace(tuple_targets=True, stale_pattern_keys=True)
        das.pattern_black_list = list(case["black_list"])
        das.load_canonical_knowledge_base(str(f))
        for p in case.get("index") or []:
            if p["kind"] == "links" and "error" not in p:
                assert sorted(das.db.get_matched_links(*p["args"]), key=str) == \
                    sorted(db.get_matched_links(*p["args"]), key=str)
    assert failed_loads >= 2 and checked >= 70 and touched > 0 and probes >= 60, (failed_loads, checked, touched, probes)


def test_gpu_resume_saved_kb(golden, tmp_path):
    """save_parsed_knowledge_base / load_parsed_knowledge_base (the resume
    without the parser, as the reference loader reuses its key-value files):
    a KB reloaded from the saved file answers every reference-recorded query
    of kb_bio_full.json and equals the first load's atom tables; a
    stale_pattern_keys KB keeps its black list and its stale entries (every
    query of a kb_blacklist.json canonical case the stale keys touch); a
    transaction after the resume adds to the resumed KB."""
    import os
    from das_amd.distributed_atom_space import DistributedAtomSpace
    from das_amd.database.hip_db import HipDB
    d = golden("kb_bio_full.json")
    f = tmp_path / "bio.metta"
    f.write_text(MS.text_of("bio_full"))
    das = DistributedAtomSpace(tuple_targets=True)
    das.load_canonical_knowledge_base(str(f))
    saved = tmp_path / "bio.npz"
    das.save_parsed_knowledge_base(str(saved))
    das2 = DistributedAtomSpace(tuple_targets=True)
    das2.load_parsed_knowledge_base(str(saved))
    assert list(das2.count_atoms()) == d["count_atoms"]
    assert _atom_tables(das2.db) == _atom_tables(das.db)
    bad = [q["query"] for q in d["queries"] if not q.get("no_overload") and not same(record(q["query"], das2.db), q)]
    assert not bad, bad
    n0, l0 = das2.count_atoms()
    tr = das2.open_transaction()
    for line in ("(: Concept Type)", "(: Inheritance Type)", '(: "resumed_a" Concept)', '(: "resumed_b" Concept)',
                 '(Inheritance "resumed_a" "resumed_b")'):
        tr.add(line)
    das2.commit_transaction(tr)
    assert tuple(das2.count_atoms()) == (n0 + 2, l0 + 1)
    # stale_pattern_keys: the black list and the stale entries travel
    b = golden("kb_blacklist.json")
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data")
    done = 0
    for case in b["cases"]:
        if case["loader"] != "canonical" or case.get("load_error") or not case["black_list"]:
            continue
        if case["source"] == "inline":
            text = b["canonical_text"]
        else:
            with open(os.path.join(here, os.path.basename(case["source"]))) as fh:
                text = fh.read()
        db = HipDB(device=0, tuple_targets=True, stale_pattern_keys=True)
        db.pattern_black_list = list(case["black_list"])
        db.load_canonical(text)
        p = tmp_path / f"bl{done}.npz"
        db.save_parsed(str(p))
        db2 = HipDB(device=0, tuple_targets=True, stale_pattern_keys=True)
        db2.load_parsed(str(p))
        assert db2.pattern_black_list == list(case["black_list"]) and db2._stale == db._stale
        for q in case["queries"]:
            assert same(record(q["query"], db2), q), (case["black_list"], q["query"])
        done += 1
    assert done >= 2


def _build(spec):
    from tests.util import build
    return build(spec)


@pytest.mark.parametrize("plan", ["1", "0"])
def test_gpu_pattern_black_list(golden, plan, monkeypatch):
    """pattern_black_list (kb_blacklist.json, reference-run with non-empty
    black lists, both loaders): the product follows the intended semantics --
    a black-listed type's links get no pattern keys (typed and '*' Link
    queries with a wildcard never return them) and keep their template keys
    (canonical_parser.py:144, 179-180; parser_threads.py:185) -- i.e. the
    oracle without the reference's stale-key bug.  Every query and index probe
    equals that oracle, and every query the bug does not touch equals the
    reference's own answer (tests/test_oracle.py pins the bug's restatement
    against the same fixture)."""
    import os
    from oracle import das_oracle as O
    from das_amd import _lib, loader
    from das_amd.database.hip_db import HipDB
    from das_amd.distributed_atom_space import DistributedAtomSpace
    monkeypatch.setenv("DAS_PLAN", plan)
    d = golden("kb_blacklist.json")
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data")
    checked = reference_equal = 0
    for case in d["cases"]:
        if case.get("load_error"):
            continue
        bl = case["black_list"]
        db = HipDB(device=0, tuple_targets=True)
        db.pattern_black_list = list(bl)
        if case["loader"] == "metta":
            with open(os.path.join(here, os.path.basename(case["source"]))) as f:
                db.load_arrays(loader.parse_metta([f.read()]).finish())
        else:
            db.load_arrays(_lib.parse_canonical([d["canonical_text"]]))
        kb = O.KB.from_tables(case["nodes"], case["links"])
        want_db = O.RedisMongoSemantics(kb, bl, tuple_targets=True)
        stale_db = O.RedisMongoSemantics(kb, bl, tuple_targets=True, stale_key_order=case["pattern_order"])
        assert list(db.count_atoms()) == case["count_atoms"]
        for q in case["queries"]:
            want = O.evaluate(q["query"], want_db)
            got = record(q["query"], db)
            assert same(got, want), (bl, q["query"])
            checked += 1
            if want == O.evaluate(q["query"], stale_db):
                assert same(got, q), (bl, q["query"])
                reference_equal += 1
        for p in case.get("index") or []:
            args = p["args"]
            if p["kind"] == "links":
                r, w = db.get_matched_links(*args), want_db.get_matched_links(*args)
            elif p["kind"] == "template":
                r, w = db.get_matched_type_template(args), want_db.get_matched_type_template(args)
            else:
                r, w = db.get_matched_type(args), want_db.get_matched_type(args)
            key = lambda xs: sorted(x if isinstance(x, str) else x[0] for x in xs)  # noqa: E731
            assert key(r) == key(w), (bl, p)
    assert checked > 100 and reference_equal > checked // 2
    # through the facade: the attribute the reference's loaders read
    das = DistributedAtomSpace()
    das.pattern_black_list = ["Similarity"]
    p = os.path.join(here, "animals.metta")
    das.load_knowledge_base(p)
    assert das.get_links("Similarity", None, ["*", "*"]) == []
    assert len(das.get_links("Similarity", ["Concept", "Concept"])) == 14
    assert sorted(das.get_links("*", None, ["*", "*"])) == sorted(das.get_links("Inheritance", None, ["*", "*"]))
    assert len(das.get_links("Inheritance", None, ["*", "*"])) == 12
