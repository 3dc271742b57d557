"""Native canonical MeTTa reader (das_parse_canonical, canonical.cpp) against
the reference's stored atoms and against the Python restatement
(loader.parse_canonical, CanonicalParser semantics canonical_parser.py:242-365).
Host code only: runs without a GPU."""
import os

import numpy as np
import pytest

from das_amd import _lib, loader
from oracle import das_oracle as O

DATA = os.path.join(os.path.dirname(__file__), "golden", "data")


def _tables(arrays):
    kb = O.KB.from_arrays(arrays)
    return kb.node_table(), kb.link_table()


def test_native_canonical_toy_mining(golden):
    with open(os.path.join(DATA, "canonical_toy-example-mining.metta")) as f:
        text = f.read()
    nodes, links = _tables(_lib.parse_canonical(text))
    d = golden("kb_toy_mining.json")
    assert nodes == sorted(d["nodes"])
    assert links == sorted(d["links"])


def _random_canonical(rng, n_nodes=60, n_lines=400, ws=False):
    types = ["Concept", "Predicate", "Schema"]
    links = ["Inheritance", "Similarity", "Evaluation", "List", "Execution"]
    out = [f"(: {t} Type)" for t in types + links]
    names = []
    for i in range(n_nodes):
        t = types[i % len(types)]
        nm = f"n{i}" if i % 7 else f"multi word  name {i}"
        names.append((t, " ".join(nm.split())))
        out.append(f'(: "{nm}" {t})')

    def term():
        t, nm = names[rng.integers(len(names))]
        if ws and rng.random() < 0.3:
            nm = nm.replace(" ", "  \t ")
        return f'"{t} {nm}"'

    def expr(depth):
        k = int(rng.integers(1, 4))
        kids = [expr(depth + 1) if depth < 2 and rng.random() < 0.25 else term() for _ in range(k)]
        return f"({links[rng.integers(len(links))]} " + " ".join(kids) + ")"

    for _ in range(n_lines):
        line = expr(0)
        if ws and rng.random() < 0.2:
            line = "  \t" + line + " \t "
        out.append(line)
    return out


@pytest.mark.parametrize("chunk", ["", "97"])
@pytest.mark.parametrize("seed", [1, 2])
def test_native_matches_python_reader(seed, chunk, monkeypatch):
    """Same stored atoms (handles, types, targets, composite types) as the
    Python reader, with nesting, multi-word names, whitespace runs and, for
    chunk=97, hundreds of parse chunks merged."""
    if chunk:
        monkeypatch.setenv("DAS_PARSE_CHUNK_BYTES", chunk)
    rng = np.random.default_rng(seed)
    lines = _random_canonical(rng, ws=True)
    sep = ["\n", "\r\n", "\r"][seed % 3]
    text = sep.join(lines) + sep
    want = _tables(loader.parse_canonical(text).finish())
    got = _tables(_lib.parse_canonical(text, threads=4))
    assert got == want


def test_native_thread_and_chunk_invariance(monkeypatch):
    rng = np.random.default_rng(5)
    text = "\n".join(_random_canonical(rng, n_lines=800))
    a = _lib.parse_canonical(text, threads=1)
    monkeypatch.setenv("DAS_PARSE_CHUNK_BYTES", "301")
    b = _lib.parse_canonical(text, threads=8)
    for f in ("leaf_bytes", "leaf_off", "leaf_kind", "leaf_ctype", "leaf_type_id", "name_start", "expr_off",
              "expr_child", "expr_kind", "expr_ctype_leaf", "level_off"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    assert a.type_names == b.type_names


def test_native_escaped_quote_and_multiple_files():
    t1 = '(: Concept Type)\n(: "a" Concept)\n(Inheritance "Concept a \\"q\\" b" "Concept a")\n'
    t2 = '(: Concept Type)\n(: "z" Concept)\n(Similarity "Concept z" "Concept a")\n'
    want = _tables(loader.parse_canonical([t1, t2]).finish())
    got = _tables(_lib.parse_canonical([t1, t2]))
    assert got == want
    names = {n[2] for n in got[0]}
    assert names == {"a", "z"}
    assert len(got[1]) == 2


@pytest.mark.parametrize("text", [
    '(: Concept Type)\n(Inheritance "Concept a" "Concept b")\n',                    # no terminal section
    '(: Concept Type)\n(: "a" Concept)\n(Inheritance "Concept a")\n(: "b" Concept)\n',  # typedef after expressions
    '(: Concept Type)\n(: "a" Concept)\n(Inheritance "Concept a"\n',               # unbalanced
    '(: Concept Type)\n(: "a" Concept)\n(Inheritance "Concept a)\n',               # unterminated string
    '(: Concept Type Extra)\n(: "a" Concept)\n',                                     # typedef word count
])
def test_native_syntax_errors_raise_assertion(text):
    with pytest.raises(AssertionError, match="line"):
        _lib.parse_canonical(text)


def test_native_flybase_shape_roundtrip():
    """A FlyBase-shaped canonical dump (Execution(Schema, key, value) rows,
    flybase2metta sql_reader.py:297-302) written from flybase_kb, read back by
    the native reader: the same atoms as the generator's arrays."""
    from das_amd import synthetic
    arrays = synthetic.flybase_kb(60, 5, 80, n_loc=10, n_do=8)
    text = synthetic.to_canonical(arrays)
    got = _tables(_lib.parse_canonical(text))
    want = _tables(arrays)
    assert got == want


def test_concat_arrays_matches_one_builder():
    """Facade path: native canonical output + MeTTa builder output, concatenated
    (loader.concat_arrays), store the same atoms as one Python builder over both."""
    with open(os.path.join(DATA, "canonical_toy-example-mining.metta")) as f:
        canon = f.read()
    with open(os.path.join(DATA, "animals.metta")) as f:
        metta = f.read()
    nested = ('(: Concept Type)\n(: "p" Concept)\n(: "q" Concept)\n'
              '(Evaluation "Concept p" (List "Concept p" (Set "Concept q")))\n(List "Concept q" "Concept p")\n')
    b = loader.AtomBuilder()
    loader.parse_canonical([canon, nested], b)
    loader.parse_metta([metta], b)
    want = _tables(b.finish())
    got = _tables(loader.concat_arrays([_lib.parse_canonical([canon, nested]),
                                        loader.parse_metta([metta]).finish()]))
    assert got == want
