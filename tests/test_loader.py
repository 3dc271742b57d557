"""Host ingestion: the loader's DAG, hashed the reference way by the oracle,
reproduces exactly the atoms the reference stored (handles, types, targets,
composite types).  The GPU recomputes the same handles in test_gpu_parity."""
import os

from das_amd import loader
from oracle import das_oracle as O

DATA = os.path.join(os.path.dirname(__file__), "golden", "data")


def _tables_equal(kb, d):
    assert kb.node_table() == sorted(d["nodes"])
    assert kb.link_table() == sorted(d["links"])


def test_metta_loader_animals(golden):
    with open(os.path.join(DATA, "animals.metta")) as f:
        arrays = loader.parse_metta(f.read()).finish()
    _tables_equal(O.KB.from_arrays(arrays), golden("kb_animals.json"))


def test_canonical_loader_toy_mining(golden):
    with open(os.path.join(DATA, "canonical_toy-example-mining.metta")) as f:
        arrays = loader.parse_canonical(f.read()).finish()
    _tables_equal(O.KB.from_arrays(arrays), golden("kb_toy_mining.json"))


def test_metta_loader_nested_stub_like(golden):
    import importlib.util
    spec = importlib.util.spec_from_file_location("mg", os.path.join(os.path.dirname(__file__), "golden",
                                                                      "make_golden.py"))
    # only the inline KB text is needed; read it without importing the reference
    src = open(spec.origin).read()
    start = src.index('STUB_LIKE_METTA = """') + len('STUB_LIKE_METTA = """')
    head = src[start:src.index('"""', start)]
    names = ["human", "monkey", "chimp", "snake", "earthworm", "rhino", "triceratops", "vine", "ent",
             "mammal", "animal", "reptile", "dinosaur", "plant"]
    rest_start = src.index('"plant"]) + """', start) + len('"plant"]) + """')
    rest = src[rest_start:src.index('"""', rest_start)]
    text = head + "\n".join(f'(: "{n}" Concept)' for n in names) + rest
    arrays = loader.parse_metta(text).finish()
    _tables_equal(O.KB.from_arrays(arrays), golden("kb_stub_like.json"))


def test_from_tables_roundtrip(golden):
    d = golden("kb_stub_like.json")
    arrays = loader.from_tables(d["nodes"], d["links"]).finish()
    _tables_equal(O.KB.from_arrays(arrays), d)


def test_levels_are_grouped_by_arity():
    b = loader.AtomBuilder()
    a = b.terminal("Concept", "a", True)
    c = b.terminal("Concept", "c", True)
    l1 = b.expr("Inheritance", [a, c])
    b.expr("List", [l1, a, c])
    b.expr("Set", [a])
    arr = b.finish()
    for g in range(len(arr.level_off) - 1):
        s, e = int(arr.level_off[g]), int(arr.level_off[g + 1])
        ks = {int(arr.expr_off[j + 1] - arr.expr_off[j]) for j in range(s, e)}
        assert len(ks) == 1


def test_saved_kb_roundtrip(golden, tmp_path):
    """AtomArrays.save / load (the resume-without-parser file): every array,
    the type names and the extra metadata come back unchanged, through plain
    np.load (allow_pickle off), and the reloaded arrays still hash to the
    atoms the reference stored."""
    import numpy as np
    with open(os.path.join(DATA, "animals.metta")) as f:
        arrays = loader.parse_metta(f.read()).finish()
    p = tmp_path / "kb.npz"
    arrays.save(p, {"pattern_black_list": ["Similarity"], "stale": [[["a", "b"], {"h": ["x", "y"]}]]})
    back, extra = loader.AtomArrays.load(p)
    for k in loader.AtomArrays._FIELDS:
        a, b = getattr(arrays, k), getattr(back, k)
        assert a.dtype == b.dtype and np.array_equal(a, b), k
    assert back.type_names == arrays.type_names and back.type_id == arrays.type_id
    assert extra == {"pattern_black_list": ["Similarity"], "stale": [[["a", "b"], {"h": ["x", "y"]}]]}
    _tables_equal(O.KB.from_arrays(back), golden("kb_animals.json"))
    bad = tmp_path / "bad.npz"
    np.savez(bad, meta_json=np.frombuffer(b'{"format": "other"}', dtype=np.uint8))
    import pytest
    with pytest.raises(ValueError):
        loader.AtomArrays.load(bad)
