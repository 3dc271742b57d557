"""The oracle pinned on the config 2-5 shapes: small seeded instances of the
synthetic generators (bio_full / flybase / powerlaw / hub), loaded and
answered by the reference itself in the build container
(tests/golden/make_synthetic.py + make_golden.py synthetic).  Each fixture
holds the generator call, the sha256 of the canonical text, the sha256 of
the atom tables the reference stored, and every query's answer set."""
import hashlib
import json

import pytest

from oracle import das_oracle as O
from tests.golden import make_synthetic as MS

FIXTURES = ["bio_full", "flybase", "powerlaw", "hub"]


def table_sha(rows):
    return hashlib.sha256("\n".join(json.dumps(r) for r in rows).encode()).hexdigest()


def oracle_record(entry, db):
    O.CONFIG["no_overload"] = bool(entry.get("no_overload"))
    try:
        return O.evaluate(entry["query"], db)
    finally:
        O.CONFIG["no_overload"] = False


def check(rec, want):
    if want.get("error"):
        return rec.get("error") == want["error"]
    return rec.get("error") is None and all(rec[k] == want[k] for k in ("matched", "negation", "n", "sha256"))


@pytest.mark.parametrize("name", FIXTURES)
def test_generator_text_is_the_one_the_reference_loaded(golden, name):
    d = golden(f"kb_{name}.json")
    assert d["source"] == {"function": f"das_amd.synthetic.{MS.KBS[name][0]}", "kwargs": MS.KBS[name][1]}
    assert hashlib.sha256(MS.text_of(name).encode()).hexdigest() == d["text_sha256"]


@pytest.mark.parametrize("name", FIXTURES)
def test_oracle_matches_reference_on_synthetic(golden, name):
    from das_amd import loader
    d = golden(f"kb_{name}.json")
    kb = O.KB.from_arrays(loader.parse_canonical(MS.text_of(name)).finish())
    assert [len(kb.nodes), len(kb.links)] == d["count_atoms"]
    assert table_sha(kb.node_table()) == d["nodes_sha256"]
    assert table_sha(kb.link_table()) == d["links_sha256"]
    db = O.RedisMongoSemantics(kb, tuple_targets=True)
    bad = [(q["query"], q.get("no_overload")) for q in d["queries"]
           if q.get("ref_seconds", 0) < 1.0 and not check(oracle_record(q, db), q)]
    assert not bad, bad
