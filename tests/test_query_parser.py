"""The service's query mini-language (service/server.py:34-81) -> the
pattern_matcher expression tree, and its None / IndexError cases."""
import pytest

from das_amd.pattern_matcher.pattern_matcher import And, Link, Node, Not, Or, Variable
from das_amd.service import _parse_query


def shape(e):
    if isinstance(e, Node):
        return ("Node", e.atom_type, e.name)
    if isinstance(e, Variable):
        return ("Var", e.name)
    if isinstance(e, Link):
        return ("Link", e.atom_type, e.ordered, tuple(shape(t) for t in e.targets))
    if isinstance(e, Not):
        return ("Not", shape(e.term))
    kind = "And" if isinstance(e, And) else "Or"
    return (kind, tuple(shape(t) for t in e.terms))


def test_service_regression_query():
    # scripts/service_regression_test.sh:52
    q = _parse_query("Node n1 Concept human, Link Inheritance n1 $2")
    assert shape(q) == ("Link", "Inheritance", True, (("Node", "Concept", "human"), ("Var", "$2")))


def test_postfix_and_or_not():
    q = _parse_query("Node n1 Concept mammal, Node n2 Concept plant, Link Inheritance $1 $2, "
                     "Link Inheritance $2 $3, AND, Link Inheritance $1 n1, NOT, AND")
    inh = lambda a, b: ("Link", "Inheritance", True, (a, b))  # noqa: E731
    V = lambda n: ("Var", n)  # noqa: E731
    assert shape(q) == ("And", (("And", (inh(V("$1"), V("$2")), inh(V("$2"), V("$3")))),
                                ("Not", inh(V("$1"), ("Node", "Concept", "mammal")))))
    q = _parse_query("Node h Concept human, Link Similarity $1 h, Link Similarity h $2, OR")
    # unordered: non-variables first (Link.__init__, pattern_matcher.py:439-453)
    assert shape(q) == ("Or", (("Link", "Similarity", False, (("Node", "Concept", "human"), ("Var", "$1"))),
                               ("Link", "Similarity", False, (("Node", "Concept", "human"), ("Var", "$2")))))


@pytest.mark.parametrize("text", [
    "Node n1 Concept",                                  # Node chunk needs 4 words
    "Link Inheritance",                                 # Link chunk needs >= 3 words
    "Link Inheritance n9 $1",                           # unknown node alias
    "AND",                                              # operator on an empty stack
    "Link Inheritance $1 $2, Link Inheritance $2 $3",   # two terms left
    "Node n1 Concept a, Link Inheritance n1 $1, Node n2 Concept b",   # Node after the node section
    "Link Inheritance $1 $2, XOR",                      # unknown operator
])
def test_invalid_queries_return_none(text):
    assert _parse_query(text) is None


def test_empty_chunk_raises_like_the_reference():
    with pytest.raises(IndexError):
        _parse_query("Link Inheritance $1 $2, ")
