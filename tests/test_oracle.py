"""The CPU oracle against the reference's own outputs (golden fixtures made by
running the reference here, tests/golden/make_golden.py) and the handles the
reference prints (scripts/service_regression_test.sh, service/README.md)."""
import hashlib

import pytest

from oracle import das_oracle as O

KB_FIXTURES = ["kb_animals.json", "kb_toy_mining.json", "kb_stub_like.json"]

# Appendix C of SURVEY.md; printed by the reference at
# scripts/service_regression_test.sh:34,43 and service/README.md:290-378
KNOWN = {
    ("Concept", "human"): "af12f10f9ae2002a1607ba0b47ba8407",
    ("Concept", "mammal"): "bdfe4e7a431f73386f37c6448afe5840",
    ("Concept", "monkey"): "1cdffc6b0b89ff41d68bec237481d1e1",
    ("Concept", "chimp"): "5b34c54bee150c04f9fa584b899dc030",
    ("Concept", "snake"): "c1db9b517073e51eb7ef6fed608ec204",
    ("Concept", "earthworm"): "bb34ce95f161a6b37ff54b3d4c817857",
    ("Concept", "rhino"): "99d18c702e813b07260baf577c60c455",
    ("Concept", "triceratops"): "d03e59654221c1e8fcda404fd5c8d6cb",
    ("Concept", "vine"): "b94941d8cd1c0ee4ad3dd3dcab52b964",
    ("Concept", "ent"): "4e8e26e3276af8a5c2ac2cc2dc95c6d2",
    ("Concept", "animal"): "0a32b476852eeb954979b87f5f6cb7af",
    ("Concept", "reptile"): "b99ae727c787f1b13b452fd4c9ce1b9a",
    ("Concept", "dinosaur"): "08126b066d32ee37743e255a2558cccd",
}
INH_HUMAN_MAMMAL = "c93e1e758c53912638438e2a7d7f7b7f"


def test_known_handles():
    for (t, n), h in KNOWN.items():
        assert O.terminal_hash(t, n) == h
    assert O.expression_hash(O.named_type_hash("Inheritance"),
                             [KNOWN[("Concept", "human")], KNOWN[("Concept", "mammal")]]) == INH_HUMAN_MAMMAL


def test_hash_vectors(golden):
    hv = golden("hash_vectors.json")
    for s, h in hv["md5"]:
        assert O.md5hex(s) == h
    for parts, h in hv["composite"]:
        assert O.composite_hash(parts) == h
    for t, n, h in hv["terminal"]:
        assert O.terminal_hash(t, n) == h


def _check(rec, want):
    if want.get("error"):
        return rec.get("error") == want["error"]
    return rec.get("error") is None and all(rec[k] == want[k] for k in ("matched", "negation", "n", "sha256"))


@pytest.mark.parametrize("fixture", KB_FIXTURES)
def test_oracle_matches_reference_db_path(golden, fixture):
    d = golden(fixture)
    kb = O.KB.from_tables(d["nodes"], d["links"])
    db = O.RedisMongoSemantics(kb, tuple_targets=True)
    assert list(db.count_atoms()) == d["count_atoms"]
    bad = [q["query"] for q in d["queries"] if not _check(O.evaluate(q["query"], db), q)]
    assert not bad, bad


@pytest.mark.parametrize("fixture", KB_FIXTURES)
def test_oracle_list_targets_agree_where_reference_succeeds(golden, fixture):
    d = golden(fixture)
    db = O.RedisMongoSemantics(O.KB.from_tables(d["nodes"], d["links"]), tuple_targets=False)
    for q in d["queries"]:
        if not q.get("error"):
            assert _check(O.evaluate(q["query"], db), q), q["query"]


def test_oracle_index_probes(golden):
    d = golden("kb_animals.json")
    db = O.RedisMongoSemantics(O.KB.from_tables(d["nodes"], d["links"]))
    for p in d["index"]:
        if p["kind"] == "links":
            r = db.get_matched_links(*p["args"])
        elif p["kind"] == "template":
            r = db.get_matched_type_template(p["args"])
        else:
            r = db.get_matched_type(p["args"])
        assert sorted(x if isinstance(x, str) else x[0] for x in r) == p["handles"], p["args"]


def test_oracle_matches_reference_stubdb(golden):
    d = golden("stubdb.json")
    db = O.StubSemantics(d["nodes"], d["links"])
    bad = [q["query"] for q in d["queries"] if not _check(O.evaluate(q["query"], db), q)]
    assert not bad, bad


def test_readme_examples(golden):
    """service/README.md:286-378 answer sizes (query strings -> expressions)."""
    d = golden("kb_animals.json")
    db = O.RedisMongoSemantics(O.KB.from_tables(d["nodes"], d["links"]))
    V = lambda n: ["Var", n]  # noqa: E731
    inh = lambda a, b: ["Link", "Inheritance", True, [a, b]]  # noqa: E731
    mammal, human = ["Node", "Concept", "mammal"], ["Node", "Concept", "human"]
    q1 = ["And", [inh(V("$1"), V("$2")), inh(V("$2"), V("$3"))]]
    q2 = ["And", [["Not", inh(V("$1"), mammal)], inh(V("$1"), V("$2")), inh(V("$2"), V("$3"))]]
    q3 = ["Or", [["And", [inh(V("$1"), V("$2")), inh(V("$2"), V("$3")), ["Not", inh(V("$1"), mammal)]]],
                 inh(human, V("$2"))]]
    assert O.evaluate(q1, db)["n"] == 7
    assert O.evaluate(q2, db)["n"] == 3
    assert O.evaluate(q3, db)["n"] == 4
    assert O.evaluate(["Link", "Similarity", False, [V("$1"), V("$2")]], db)["n"] == 7


def test_oracle_keyspace_matches_reference_files(golden):
    """keyspace_lines restates the key-value files the reference's
    CanonicalParser wrote for the toy-mining KB (tests/golden/kv_toy_mining)."""
    import os
    d = golden("kb_toy_mining.json")
    kb = O.KB.from_tables(d["nodes"], d["links"])
    got = O.keyspace_lines(kb)
    base = os.path.join(os.path.dirname(__file__), "golden", "kv_toy_mining")
    for name, lines in got.items():
        with open(os.path.join(base, f"{name}.txt")) as f:
            want = sorted(l.rstrip("\n") for l in f if l.strip())
        assert lines == want, name


def _probe(db, p):
    if p["kind"] == "links":
        r = db.get_matched_links(*p["args"])
    elif p["kind"] == "template":
        r = db.get_matched_type_template(p["args"])
    else:
        r = db.get_matched_type(p["args"])
    return sorted(x if isinstance(x, str) else x[0] for x in r)


def test_oracle_blacklist_stale_keys_reproduce_reference(golden):
    """pattern_black_list as the reference actually behaves
    (kb_blacklist.json, reference-run): given the order its pattern-key loop
    walked the links, the oracle's stale-key restatement answers every query
    and index probe as the reference did, and raises where the reference's
    load failed (a blacklisted first link: UnboundLocalError; in the MettaYacc
    loader it kills the pattern thread and the load then asserts)."""
    d = golden("kb_blacklist.json")
    assert len(d["cases"]) >= 5
    for case in d["cases"]:
        kb = O.KB.from_tables(case["nodes"], case["links"])
        bl = case["black_list"]
        order = case["pattern_order"]
        assert sorted(order) == sorted(x[0] for x in case["links"])
        if case.get("load_error"):
            with pytest.raises(UnboundLocalError):
                O.RedisMongoSemantics(kb, bl, tuple_targets=True, stale_key_order=order)
            continue
        db = O.RedisMongoSemantics(kb, bl, tuple_targets=True, stale_key_order=order)
        assert list(db.count_atoms()) == case["count_atoms"]
        bad = [q["query"] for q in case["queries"] if not _check(O.evaluate(q["query"], db), q)]
        assert not bad, (bl, bad)
        for p in case.get("index") or []:
            if "error" not in p:
                assert _probe(db, p) == p["handles"], (bl, p["args"])


def test_oracle_blacklist_intended_vs_reference(golden):
    """The intended semantics (blacklisted links get no pattern keys, template
    keys kept) -- what das_amd follows -- agree with the reference on every
    query the stale keys do not touch; the ones they touch are counted (the
    fixture must show the reference's behaviour on some)."""
    d = golden("kb_blacklist.json")
    touched = untouched = 0
    for case in d["cases"]:
        if case.get("load_error"):
            continue
        kb = O.KB.from_tables(case["nodes"], case["links"])
        bl = case["black_list"]
        stale = O.RedisMongoSemantics(kb, bl, tuple_targets=True, stale_key_order=case["pattern_order"])
        want = O.RedisMongoSemantics(kb, bl, tuple_targets=True)
        for q in case["queries"]:
            a, b = O.evaluate(q["query"], stale), O.evaluate(q["query"], want)
            if a == b:
                untouched += 1
                assert _check(b, q), q["query"]
            else:
                touched += 1
    assert touched > 0 and untouched > touched, (touched, untouched)


def test_oracle_hash_join_equals_nested_loop(monkeypatch):
    """The oracle's And fold joins ordered rows of one variable set through a
    hash on the shared variables (FAST_JOIN): the same answers as the
    reference's nested loop (pattern_matcher.py:732-738) on random And / Not /
    Or queries over small bio and power-law KBs, incl. reset-on-empty Ands."""
    import numpy as np
    from das_amd import synthetic
    from tests.test_gpu_parity import _random_queries
    for arrays, seed in ((synthetic.bio_kb(60, 12, 300, 20), 1), (synthetic.powerlaw_kb(60, 500, link_types=3, seed=4), 2)):
        odb = O.RedisMongoSemantics(O.KB.from_arrays(arrays))
        qs = _random_queries(np.random.default_rng(seed), arrays, 40)
        monkeypatch.setattr(O, "FAST_JOIN", True)
        fast = [O.evaluate(q, odb) for q in qs]
        monkeypatch.setattr(O, "FAST_JOIN", False)
        slow = [O.evaluate(q, odb) for q in qs]
        assert fast == slow
        assert any(r.get("n") for r in slow)
        # the nested loop with per-row mappings (bench.py's cpu_baseline)
        # against join() per pair
        monkeypatch.setattr(O, "_ordered_nested_join", lambda acc, rows: None)
        assert [O.evaluate(q, odb) for q in qs] == slow
        monkeypatch.undo()


def test_stale_pattern_keys_host_restatement_matches_fixture(golden):
    """HipDB(stale_pattern_keys=True)'s host side, for every canonical-loader
    case of kb_blacklist.json (reference-run): the reference's pattern-loop
    order recomputed from the canonical text (loader.canonical_pattern_order:
    links_1 / links_2 / links_n, first occurrence in parse order) equals the
    order the fixture recorded, the stale entries it derives equal the
    oracle's (pinned against the reference's answers above), and a
    blacklisted first link raises UnboundLocalError as the reference's load."""
    import os
    from das_amd import loader
    from das_amd.database import hip_db
    d = golden("kb_blacklist.json")
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data")
    n = 0
    for case in d["cases"]:
        if case["loader"] != "canonical":
            continue
        if case["source"] == "inline":
            text = d["canonical_text"]
        else:
            with open(os.path.join(here, os.path.basename(case["source"]))) as f:
                text = f.read()
        order = loader.canonical_pattern_order(text)
        assert [h for h, _, _ in order] == case["pattern_order"]
        bl = set(case["black_list"])
        if case.get("load_error"):
            with pytest.raises(UnboundLocalError):
                hip_db._stale_entries(order, bl)
            n += 1
            continue
        stale = hip_db._stale_entries(order, bl)
        kb = O.KB.from_tables(case["nodes"], case["links"])
        odb = O.RedisMongoSemantics(kb, case["black_list"], tuple_targets=True, stale_key_order=case["pattern_order"])
        want = {}
        for k, vals in odb.patterns.items():
            for h, tg in vals:
                if kb.links[h][0] in bl:
                    want.setdefault(k, {})[h] = tuple(tg)
        assert stale == want and stale
        n += 1
    assert n >= 4
