"""Golden-vector generator (TEST INFRASTRUCTURE, runs only in the build container).

Imports the read-only reference (tanksha/das @ /root/reference) with in-memory
stand-ins for Redis and MongoDB, loads small knowledge bases through the
reference's own loaders (MettaYacc `load_knowledge_base`, `CanonicalParser`
`load_canonical_knowledge_base`), runs query expressions through the
reference `pattern_matcher` against the reference `RedisMongoDB` adapter, and
writes canonicalised answers as JSON fixtures under tests/golden/.

Nothing here is imported by the product (`das_amd/`).  The fakes below are our
own code: they implement only the handful of redis-py / pymongo calls the
reference adapter makes (`sadd`, `smembers`, `flushall`; `insert_many`,
`find`, `find_one`, `count_documents`, `estimated_document_count`).

Run with the conda interpreter (it has ply 3.11, the reference's pinned PLY):
    PYTHONDONTWRITEBYTECODE=1 /opt/conda/bin/python3.9 tests/golden/make_golden.py
(`tests/golden/generate.sh` does this, after writing the synthetic KB files.)
"""
import hashlib
import json
import os
import re
import sys
import types

REF = os.environ.get("DAS_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
SCRATCH = os.environ.get("DAS_GOLDEN_SCRATCH", "/tmp/das_golden")

# ----------------------------------------------------------------------------
# In-memory Redis / Mongo stand-ins (only what the reference adapter calls)
# ----------------------------------------------------------------------------


class FakeRedis:
    def __init__(self, *a, **kw):
        self.sets = {}

    def sadd(self, key, *values):
        s = self.sets.setdefault(key, set())
        for v in values:
            s.add(v if isinstance(v, bytes) else str(v).encode())
        return len(values)

    def smembers(self, key):
        return set(self.sets.get(key, set()))

    def flushall(self):
        self.sets.clear()


def _install_fake_redis():
    redis_mod = types.ModuleType("redis")
    redis_mod.Redis = FakeRedis
    cluster = types.ModuleType("redis.cluster")
    cluster.RedisCluster = FakeRedis
    redis_mod.cluster = cluster
    sys.modules["redis"] = redis_mod
    sys.modules["redis.cluster"] = cluster


class FakeCollection:
    def __init__(self):
        self.docs = {}

    def insert_many(self, docs, ordered=True):
        dup = 0
        for d in docs:
            if d["_id"] in self.docs:
                dup += 1
                continue
            self.docs[d["_id"]] = dict(d)
        if dup:
            raise Exception(f"duplicate key ({dup})")

    def _match(self, d, flt):
        for k, v in (flt or {}).items():
            if isinstance(v, dict) and "$regex" in v:
                if k not in d or re.search(v["$regex"], d[k]) is None:
                    return False
            elif d.get(k, None) != v:
                return False
        return True

    def find(self, flt=None):
        if flt and list(flt.keys()) == ["_id"]:
            d = self.docs.get(flt["_id"])
            return iter([d] if d is not None else [])
        return iter([d for d in self.docs.values() if self._match(d, flt)])

    def find_one(self, flt=None):
        for d in self.find(flt):
            return d
        return None

    def count_documents(self, flt):
        return sum(1 for _ in self.find(flt))

    def estimated_document_count(self):
        return len(self.docs)


class FakeMongo:
    def __init__(self):
        self.cols = {}

    def get_collection(self, name):
        return self.cols.setdefault(str(getattr(name, "value", name)), FakeCollection())

    def __getitem__(self, name):
        return self.get_collection(name)

    def collection_names(self):
        return list(self.cols.keys())

    def drop_collection(self, name):
        self.cols.pop(name, None)


# ----------------------------------------------------------------------------
# Reference import
# ----------------------------------------------------------------------------

_install_fake_redis()
sys.path.insert(0, REF)
os.makedirs(SCRATCH, exist_ok=True)
import das.canonical_parser as canonical_parser_mod  # noqa: E402
import das.parser_threads as parser_threads_mod  # noqa: E402

canonical_parser_mod.TMP_DIR = SCRATCH
from das.database.redis_mongo_db import RedisMongoDB  # noqa: E402
from das.distributed_atom_space import DistributedAtomSpace  # noqa: E402
from das.expression_hasher import ExpressionHasher  # noqa: E402
from das.pattern_matcher import pattern_matcher as pm  # noqa: E402


def new_das():
    das = object.__new__(DistributedAtomSpace)
    das.database_name = "das"
    das.mongo_db = FakeMongo()
    das.redis = FakeRedis()
    das.db = RedisMongoDB(das.redis, das.mongo_db)
    das.db.prefetch()
    das.pattern_black_list = []
    return das


def _patch_shared_tmp():
    orig = parser_threads_mod.SharedData.__init__

    def init(self):
        orig(self)
        self.temporary_file_name = {k: os.path.join(SCRATCH, os.path.basename(v))
                                    for k, v in self.temporary_file_name.items()}
    parser_threads_mod.SharedData.__init__ = init


_patch_shared_tmp()
# the MettaYacc loader sleeps 10 s between files to dodge PLY's thread-unsafe
# start-up; a scratch harness loads one file at a time instead.
import das.distributed_atom_space as das_mod  # noqa: E402
das_mod.sleep = lambda s: None


def load_metta(paths, black_list=()):
    das = new_das()
    das.pattern_black_list = list(black_list)
    for p in paths:
        das.load_knowledge_base(p)
    return das


def load_canonical(path, black_list=()):
    das = new_das()
    das.pattern_black_list = list(black_list)
    das.load_canonical_knowledge_base(path)
    das.db.prefetch()
    return das


# ----------------------------------------------------------------------------
# Query specs (JSON) -> reference objects
# ----------------------------------------------------------------------------


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
    """Canonical identity of an Assignment (what the reference set dedups on).

    Ordered: the mapping.  Unordered: (variable set, value multiset).
    Composite: ordered mapping (or none) + the unordered members that occur an
    odd number of times (their hashes are XOR-folded, so pairs cancel,
    pattern_matcher.py:279-286, 307-314).  A composite whose unordered members
    all cancel and that has an ordered mapping has the ordered mapping's hash,
    so it is the same set element as that ordered assignment.
    """
    if isinstance(a, pm.OrderedAssignment):
        return ["O", sorted(a.mapping.items())]
    if isinstance(a, pm.UnorderedAssignment):
        vals = []
        for k, c in a.values.items():
            vals += [k] * c
        return ["U", sorted(a.symbols.keys()), sorted(vals)]
    if isinstance(a, pm.CompositeAssignment):
        members = {}
        for u in a.unordered_mappings:
            key = json.dumps(canon(u))
            members[key] = members.get(key, 0) ^ 1
        odd = sorted(k for k, v in members.items() if v)
        if a.ordered_mapping is not None and not odd:
            return ["O", sorted(a.ordered_mapping.mapping.items())]
        ordered = sorted(a.ordered_mapping.mapping.items()) if a.ordered_mapping is not None else None
        return ["C", ordered, [json.loads(k) for k in odd]]
    raise TypeError(type(a))


def answer_record(db, spec, inline_limit=400, no_overload=False):
    import time
    expr = build(spec)
    answer = pm.PatternMatchingAnswer()
    rec = {"query": spec}
    if no_overload:
        rec["no_overload"] = True
    pm.CONFIG["no_overload"] = no_overload          # pattern_matcher.py:16-19
    t0 = time.perf_counter()
    try:
        matched = expr.matched(db, answer)
    except Exception as e:  # reference raises (A7 tuple targets, composite negation ...)
        rec["error"] = type(e).__name__
        return rec
    finally:
        pm.CONFIG["no_overload"] = False
    # reference matched() wall time in this container (CPU-baseline calibration)
    rec["ref_seconds"] = round(time.perf_counter() - t0, 6)
    rows = sorted(json.dumps(canon(a), sort_keys=True) for a in answer.assignments)
    rec["matched"] = bool(matched)
    rec["negation"] = bool(answer.negation)
    rec["n"] = len(answer.assignments)
    rec["n_distinct_canon"] = len(set(rows))
    rec["sha256"] = hashlib.sha256("\n".join(rows).encode()).hexdigest()
    if len(rows) <= inline_limit:
        rec["rows"] = [json.loads(r) for r in rows]
    return rec


def atom_table(das):
    """Every node and link the reference stored (handle, type, name/targets)."""
    db = das.db
    nodes = []
    for d in db.mongo_nodes_collection.find():
        nodes.append([d["_id"], d["named_type"], d["name"]])
    links = []
    for tag in ["1", "2", "N"]:
        for d in db.mongo_link_collection[tag].find():
            links.append([d["_id"], d["named_type"], db._get_mongo_document_keys(d),
                          d["composite_type_hash"]])
    return sorted(nodes), sorted(links)


def index_counts(das, probes):
    db = das.db
    out = []
    for kind, args in probes:
        try:
            if kind == "links":
                r = db.get_matched_links(*args)
            elif kind == "template":
                r = db.get_matched_type_template(args)
            elif kind == "type":
                r = db.get_matched_type(args)
            else:
                raise ValueError(kind)
            hs = sorted(x if isinstance(x, str) else x[0] for x in r)
            out.append({"kind": kind, "args": args, "n": len(r), "handles": hs})
        except Exception as e:
            out.append({"kind": kind, "args": args, "error": type(e).__name__})
    return out


# ----------------------------------------------------------------------------
# Query sets
# ----------------------------------------------------------------------------

def N(t, n):
    return ["Node", t, n]


def V(n):
    return ["Var", n]


def L(t, targets, ordered=True):
    return ["Link", t, ordered, targets]


def C(n):
    return N("Concept", n)


def animals_queries():
    q = []
    human, mammal, animal, chimp, monkey = C("human"), C("mammal"), C("animal"), C("chimp"), C("monkey")
    snake, earthworm, ent, plant = C("snake"), C("earthworm"), C("ent"), C("plant")
    dino, rept, trice = C("dinosaur"), C("reptile"), C("triceratops")
    # nodes / grounded links (scripts/regression.py:30-75)
    q += [human, C("blah"), N("blah", "human")]
    q += [L("Inheritance", [human, mammal]), L("Similarity", [human, mammal], False),
          L("Similarity", [snake, earthworm], False), L("Similarity", [earthworm, snake], False),
          L("Inheritance", [mammal, human]), L("blah", [human, mammal]),
          L("Similarity", [snake], False), L("Similarity", [C("blah"), snake], False)]
    # nested grounded / nested variable links
    l1, l2 = L("Inheritance", [dino, rept]), L("Inheritance", [trice, dino])
    q += [L("List", [l1, l2]), L("Set", [l1, l2], False), L("List", [l1, V("V1")]),
          L("List", [L("Inheritance", [V("V1"), rept]), V("V2")])]
    # single links with variables (regression.py:76-99)
    q += [L("Inheritance", [V("V1"), mammal]), L("Inheritance", [V("V1"), V("V2")]),
          L("Inheritance", [V("V1"), V("V1")]), L("Inheritance", [V("V2"), V("V1")]),
          L("Inheritance", [mammal, V("V1")]), L("Inheritance", [animal, V("V1")]),
          L("Similarity", [V("V1"), V("V2")], False), L("Similarity", [human, V("V1")], False),
          L("Similarity", [V("V1"), human], False), L("Similarity", [V("V1"), V("V1")], False),
          L("Similarity", [V("V1"), V("V2")], True), L("Similarity", [human, V("V1")], True),
          L("Similarity", [V("V1"), human], True),
          L("*", [V("V1"), mammal]), L("*", [human, V("V1")]), L("*", [V("V1"), V("V2")]),
          L("*", [human, mammal]),
          L("Inheritance", [V("V1")]), L("Inheritance", [V("V1"), V("V2"), V("V3")]),
          L("Inheritance", [V("V1"), C("blah")])]
    # templates
    q += [["Template", "Inheritance", True, [["TVar", "V1", "Concept"], ["TVar", "V2", "Concept"]]],
          ["Template", "Similarity", True, [["TVar", "V1", "Concept"], ["TVar", "V2", "Concept"]]],
          ["Template", "Similarity", False, [["TVar", "V1", "Concept"], ["TVar", "V2", "Concept"]]],
          ["Template", "Inheritance", True, [["TVar", "V1", "Concept"], ["TVar", "V1", "Concept"]]],
          ["Template", "Inheritance", True, [["TVar", "V1", "Concept"], ["TVar", "V2", "blah"]]]]
    inh12 = L("Inheritance", [V("V1"), V("V2")])
    inh23 = L("Inheritance", [V("V2"), V("V3")])
    # Not / And / Or (regression.py:100-160, service/README.md:286-378)
    q += [["Not", L("Inheritance", [human, mammal])], ["Not", L("Inheritance", [V("V1"), mammal])],
          ["Not", L("Inheritance", [V("V1"), human])]]
    q += [["And", [inh12, inh23]],
          ["And", [inh12, L("Similarity", [V("V1"), V("V2")], False)]],
          ["And", [L("Inheritance", [V("V1"), V("V3")]), L("Inheritance", [V("V2"), V("V3")]),
                   L("Similarity", [V("V1"), V("V2")], False)]],
          ["And", [L("Inheritance", [V("V1"), V("V3")]), L("Inheritance", [V("V2"), V("V3")]),
                   ["Not", L("Similarity", [V("V1"), V("V2")], False)]]],
          ["And", [inh12, inh23, ["Not", L("Inheritance", [V("V1"), mammal])]]],
          ["And", [["Not", L("Inheritance", [V("V1"), mammal])], inh12, inh23]],
          ["And", [inh12, ["Not", L("Inheritance", [V("V1"), V("V2")])]]],
          ["And", [inh12, ["Not", L("Inheritance", [V("V2"), mammal])]]],
          ["And", [inh12, ["Not", L("Inheritance", [V("V4"), mammal])]]],
          ["And", [L("Inheritance", [V("V1"), mammal]), L("Inheritance", [V("V2"), animal])]],
          ["And", [L("Inheritance", [V("V1"), mammal]), L("Inheritance", [V("V1"), C("plant")]),
                   L("Similarity", [V("V2"), V("V3")], False)]],
          ["And", [L("Inheritance", [human, mammal]), L("Inheritance", [V("V1"), mammal])]],
          ["And", [L("Inheritance", [mammal, human]), L("Inheritance", [V("V1"), mammal])]],
          ["And", [L("Inheritance", [V("V1"), mammal]), L("Inheritance", [V("V1"), mammal])]],
          ["And", [L("Inheritance", [V("V1"), V("V2")]), L("Inheritance", [V("V2"), V("V3")]),
                   L("Inheritance", [V("V3"), V("V4")])]],
          ["And", [L("Inheritance", [V("V1"), V("V2")]), L("Inheritance", [V("V3"), V("V4")])]],
          ["And", [["Template", "Inheritance", True, [["TVar", "V1", "Concept"], ["TVar", "V2", "Concept"]]],
                   L("Inheritance", [V("V2"), animal])]],
          ["And", [L("Inheritance", [V("V1"), V("V2")]), L("Similarity", [V("V1"), V("V3")], True)]]]
    q += [["Or", [L("Inheritance", [V("V1"), mammal]), L("Inheritance", [V("V1"), animal])]],
          ["Or", [L("Inheritance", [V("V1"), mammal]), L("Inheritance", [V("V2"), animal])]],
          ["Or", [["And", [inh12, inh23, ["Not", L("Inheritance", [V("V1"), mammal])]]],
                  L("Inheritance", [human, V("V2")])]],
          ["Or", [L("Similarity", [V("V1"), human], False), L("Similarity", [V("V1"), snake], False)]],
          ["Or", [inh12, ["Not", L("Inheritance", [V("V1"), mammal])]]],
          ["Or", [["Not", L("Inheritance", [V("V1"), mammal])]]],
          ["Or", [L("Inheritance", [human, mammal]), L("Inheritance", [V("V1"), plant])]],
          ["Or", [L("Inheritance", [mammal, human]), L("Inheritance", [V("V1"), C("blah")])]],
          ["And", [["Or", [L("Inheritance", [V("V1"), mammal]), L("Inheritance", [V("V1"), plant])]],
                   L("Similarity", [V("V1"), V("V2")], True)]],
          ["Not", ["Not", L("Inheritance", [V("V1"), mammal])]]]
    # unordered / composite joins (pattern_matcher_test.py:393-625 shapes)
    sim = L("Similarity", [V("V1"), V("V2")], False)
    q += [["And", [sim, L("Similarity", [V("V2"), V("V3")], False)]],
          ["And", [sim, inh12]], ["And", [inh12, sim]],
          ["And", [sim, ["Not", inh12]]],
          ["And", [L("Similarity", [V("V1"), V("V2")], False), L("Inheritance", [V("V1"), V("V3")])]],
          ["And", [sim, sim]]]
    return q


def toy_mining_queries():
    human, man, woman = C("human"), C("man"), C("woman")
    q = [L("Inheritance", [V("V1"), human]), L("Inheritance", [V("V1"), V("V2")]),
         ["And", [L("Inheritance", [V("V1"), human]), L("Inheritance", [V("V1"), man])]],
         ["And", [L("Inheritance", [V("V1"), human]), L("Inheritance", [V("V1"), V("V2")])]],
         ["And", [L("Inheritance", [V("V1"), human]), ["Not", L("Inheritance", [V("V1"), woman])]]],
         ["And", [L("Inheritance", [V("V1"), V("V2")]), L("Inheritance", [V("V1"), V("V3")]),
                  ["Not", L("Inheritance", [V("V1"), C("ugly")])]]],
         ["Or", [L("Inheritance", [V("V1"), man]), L("Inheritance", [V("V1"), woman])]],
         ["Template", "Inheritance", True, [["TVar", "V1", "Concept"], ["TVar", "V2", "Concept"]]]]
    return q


def stub_like_queries():
    human, ent, monkey, chimp, mammal = C("human"), C("ent"), C("monkey"), C("chimp"), C("mammal")
    dino, rept, trice = C("dinosaur"), C("reptile"), C("triceratops")
    l1, l2 = L("Inheritance", [dino, rept]), L("Inheritance", [trice, dino])
    return [
        L("List", [human, ent, V("V1"), V("V2")]),
        L("Set", [human, ent, V("V1"), V("V2")], False),
        L("List", [human, ent, monkey, chimp]),
        L("Set", [human, ent, monkey, chimp], False),
        L("List", [human, V("V1"), V("V2")]),
        L("List", [V("V1"), V("V2"), V("V3")]),
        L("List", [V("V1"), monkey, V("V2")]),
        L("List", [V("V1"), V("V2")]),
        L("Set", [V("V1"), V("V2")], False),
        L("List", [l1, V("V1")]),
        L("Set", [l1, V("V1")], False),
        L("Set", [V("V1"), l1], False),
        L("List", [l1, l2]),
        L("Set", [l1, l2], False),
        L("Set", [l2, l1], False),
        L("*", [V("V1"), V("V2"), V("V3")]),
        L("*", [human, V("V1"), V("V2")]),
        ["And", [L("List", [V("V1"), V("V2"), V("V3")]), L("Inheritance", [V("V2"), mammal])]],
        ["And", [L("List", [V("V1"), V("V2"), V("V3")]), L("List", [V("V3"), V("V2"), V("V1")])]],
        ["And", [L("List", [V("V1"), V("V2"), V("V3")]), L("Inheritance", [V("V1"), V("V4")]),
                 ["Not", L("Inheritance", [V("V3"), mammal])]]],
        ["Template", "List", True, [["TVar", "V1", "Concept"], ["TVar", "V2", "Concept"], ["TVar", "V3", "Concept"]]],
        ["Template", "Set", False, [["TVar", "V1", "Concept"], ["TVar", "V2", "Concept"], ["TVar", "V3", "Concept"]]],
        ["Link", "Evaluation", True, [N("Predicate", "has"), ["Template", "List", True,
                                                               [["TVar", "V1", "Concept"], ["TVar", "V2", "Concept"]]]]],
    ]


STUB_LIKE_METTA = """(: Similarity Type)
(: Concept Type)
(: Inheritance Type)
(: List Type)
(: Set Type)
(: Evaluation Type)
(: Predicate Type)
(: "has" Predicate)
""" + "\n".join(f'(: "{n}" Concept)' for n in [
    "human", "monkey", "chimp", "snake", "earthworm", "rhino", "triceratops", "vine", "ent",
    "mammal", "animal", "reptile", "dinosaur", "plant"]) + """
(Similarity "human" "monkey")
(Similarity "human" "chimp")
(Similarity "chimp" "monkey")
(Inheritance "human" "mammal")
(Inheritance "monkey" "mammal")
(Inheritance "chimp" "mammal")
(Inheritance "mammal" "animal")
(Inheritance "dinosaur" "reptile")
(Inheritance "triceratops" "dinosaur")
(List (Inheritance "dinosaur" "reptile") (Inheritance "triceratops" "dinosaur"))
(Set (Inheritance "dinosaur" "reptile") (Inheritance "triceratops" "dinosaur"))
(List "human" "ent" "monkey" "chimp")
(List "human" "mammal" "triceratops" "vine")
(List "human" "monkey" "chimp")
(List "chimp" "monkey" "human")
(List "triceratops" "ent" "monkey")
(List "human" "human" "human")
(Set "triceratops" "vine" "monkey" "snake")
(Set "human" "ent" "monkey" "chimp")
(Set "human" "monkey" "chimp")
(Set "chimp" "human" "monkey")
(List "human" "mammal")
(Evaluation "has" (List "human" "mammal"))
(Evaluation "has" (List "chimp" "monkey"))
"""


def animals_probes(das):
    h = lambda n: das.db.get_node_handle("Concept", n)  # noqa: E731
    P = []
    for t in ["Inheritance", "Similarity", "*", "blah"]:
        for targets in [["*", "*"], ["*", h("mammal")], [h("mammal"), "*"], ["*", h("animal")],
                        [h("human"), "*"], ["*", h("human")], [h("monkey"), h("human")],
                        [h("human"), h("monkey")], [h("chimp"), h("mammal")], ["*"], ["*", "*", "*"]]:
            P.append(("links", [t, targets]))
    for tpl in [["Inheritance", "Concept", "Concept"], ["Similarity", "Concept", "Concept"],
                ["Inheritance", "Concept", "blah"], ["Similarity", "blah", "Concept"]]:
        P.append(("template", tpl))
    for t in ["Inheritance", "Similarity", "blah"]:
        P.append(("type", t))
    return P


def write(name, obj):
    path = os.path.join(HERE, name)
    with open(path, "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", path)


def kb_fixture(name, das, queries, probes=None, source=None, table_limit=(2000, 4000)):
    """queries: specs, or {"query": spec, "no_overload": bool} entries."""
    nodes, links = atom_table(das)
    db = das.db
    entries = [q if isinstance(q, dict) else {"query": q} for q in queries]
    out = {
        "kb": name,
        "source": source,
        "count_atoms": list(das.count_atoms()),
        "nodes": nodes if len(nodes) <= table_limit[0] else None,
        "links": links if len(links) <= table_limit[1] else None,
        "nodes_sha256": hashlib.sha256("\n".join(json.dumps(n) for n in nodes).encode()).hexdigest(),
        "links_sha256": hashlib.sha256("\n".join(json.dumps(l) for l in links).encode()).hexdigest(),
        "queries": [answer_record(db, e["query"], no_overload=e.get("no_overload", False)) for e in entries],
    }
    if probes is not None:
        out["index"] = index_counts(das, probes)
    return out


def hash_vectors():
    """Known-answer vectors for the ExpressionHasher (expression_hasher.py:9-35)."""
    import random
    rnd = random.Random(20250209)
    strings = ["", "a", "Concept", "Concept human", "Type", ":", "*", "Similarity",
               "x" * 55, "y" * 56, "z" * 63, "w" * 64, "v" * 119, "u" * 120, "t" * 200,
               "Concept 2-LTR circle formation", "café über", "中文 \U0001F600"]
    for _ in range(40):
        n = rnd.randint(0, 300)
        strings.append("".join(chr(rnd.randint(32, 126)) for _ in range(n)))
    strings.append("".join(chr(rnd.randint(0x80, 0x7FF)) for _ in range(70)))
    md5 = [[s, ExpressionHasher._compute_hash(s)] for s in strings]
    comp = []
    for k in [1, 2, 3, 4, 5, 8]:
        for _ in range(4):
            parts = [hashlib.md5(str(rnd.random()).encode()).hexdigest() for _ in range(k)]
            comp.append([parts, ExpressionHasher.composite_hash(parts)])
    comp.append([["*", "*", hashlib.md5(b"q").hexdigest()],
                 ExpressionHasher.composite_hash(["*", "*", hashlib.md5(b"q").hexdigest()])])
    term = [[t, n, ExpressionHasher.terminal_hash(t, n)] for t, n in
            [("Concept", "human"), ("Concept", "mammal"), ("Gene", "FBgn0000001"), ("Concept", "a b  c")]]
    return {"md5": md5, "composite": comp, "terminal": term}


def stubdb_fixture():
    """Reference StubDB (stub_db.py:91-188) + reference matcher: the
    pattern_matcher_test.py query shapes, answered by the reference itself."""
    from das.database.stub_db import StubDB
    db = StubDB()
    sim = L("Similarity", [V("V1"), V("V2")], False)
    set4 = L("Set", [V("V1"), V("V2"), V("V3"), V("V4")], False)
    inh = L("Inheritance", [V("V1"), V("V2")])
    human, mammal, animal, chimp, monkey, ent = C("human"), C("mammal"), C("animal"), C("chimp"), C("monkey"), C("ent")
    snake, earthworm, vine = C("snake"), C("earthworm"), C("vine")
    dino, rept, trice = C("dinosaur"), C("reptile"), C("triceratops")
    l1, l2 = L("Inheritance", [dino, rept]), L("Inheritance", [trice, dino])
    qs = [
        C("mammal"), C("blah"), N("blah", "mammal"),
        L("Inheritance", [human, mammal]), L("Similarity", [human, mammal], False),
        L("Inheritance", [mammal, human]),
        L("Similarity", [snake, earthworm], False), L("Similarity", [earthworm, snake], False),
        L("Similarity", [earthworm, vine], False), L("Similarity", [vine, snake], False),
        L("Similarity", [vine], False), L("Similarity", [C("blah"), snake, vine], False),
        L("List", [l1, l2]), L("List", [l2, l1]), L("Set", [l1, l2], False), L("Set", [l2, l1], False),
        L("Inheritance", [V("V1"), mammal]), L("Inheritance", [V("V1"), V("V2")]),
        L("Inheritance", [V("V1"), V("V1")]), L("Inheritance", [mammal, V("V1")]),
        L("Inheritance", [animal, V("V1")]), sim,
        L("Similarity", [human, V("V1")], False), L("Similarity", [V("V1"), human], False),
        L("List", [human, ent, V("V1"), V("V2")]), L("List", [human, V("V1"), V("V2"), ent]),
        L("Set", [human, ent, V("V1"), V("V2")], False), L("Set", [human, V("V1"), V("V2"), ent], False),
        L("Set", [ent, V("V1"), V("V2"), human], False), L("Set", [monkey, V("V1"), V("V2"), chimp], False),
        ["And", [inh, sim]],
        ["And", [L("Inheritance", [V("V1"), V("V3")]), L("Inheritance", [V("V2"), V("V3")]), sim]],
        ["And", [L("Inheritance", [V("V1"), V("V3")]), L("Inheritance", [V("V2"), V("V3")]), ["Not", sim]]],
        ["And", [set4, sim]], ["And", [sim, set4]],
        ["And", [set4, ["Not", sim]]],
        ["And", [["Not", L("Similarity", [V("V1"), V("V2")], True)], set4]],
        ["And", [set4, inh]], ["And", [inh, set4]],
        ["And", [set4, ["Not", inh]]], ["And", [["Not", inh], set4]],
        ["And", [set4, ["Not", inh], sim]], ["And", [["Not", inh], sim, set4]],
        ["Template", "Inheritance", True, [["TVar", "V1", "Concept"], ["TVar", "V2", "Concept"]]],
        ["Template", "Similarity", True, [["TVar", "V1", "Concept"], ["TVar", "V2", "Concept"]]],
        ["And", [sim, L("Similarity", [V("V2"), V("V3")], False)]],
        ["Or", [L("Inheritance", [V("V1"), mammal]), sim]],
        ["And", [["Or", [L("Inheritance", [V("V1"), mammal]), sim]], inh]],
    ]
    return {"kb": "stubdb", "links": db.all_links, "nodes": db.all_nodes,
            "queries": [answer_record(db, q) for q in qs]}


# A canonical KB whose link types interleave (canonical_parser.py:132-183
# walks links_1, links_2, links_N in insertion order), for the
# pattern_black_list fixture: a blacklisted type's links follow links of
# every other type, arity 2 and 3.
BLACKLIST_CANONICAL = "\n".join(
    ["(: Concept Type)", "(: Inheritance Type)", "(: Similarity Type)", "(: List Type)", "(: Evaluation Type)",
     "(: Predicate Type)", '(: "has" Predicate)']
    + [f'(: "c{i}" Concept)' for i in range(12)]
    + [f'(Inheritance "Concept c{a}" "Concept c{b}")' if k % 4 == 0 else
       f'(Similarity "Concept c{a}" "Concept c{b}")' if k % 4 == 1 else
       f'(List "Concept c{a}" "Concept c{b}" "Concept c{(a + b) % 12}")' if k % 4 == 2 else
       f'(Evaluation "Predicate has" (List "Concept c{a}" "Concept c{b}"))'
       for k, (a, b) in enumerate((i % 12, (5 * i + 3 + i // 12) % 12) for i in range(60))]) + "\n"


def blacklist_queries():
    c = [C(f"c{i}") for i in range(12)]
    q = []
    for t in ("Inheritance", "Similarity", "List", "Evaluation", "*"):
        q += [L(t, [V("V1"), V("V2")]), L(t, [c[0], V("V1")]), L(t, [V("V1"), c[3]]),
              L(t, [V("V1"), V("V2"), V("V3")]), L(t, [c[1], V("V1"), V("V2")]),
              ["Template", t, True, [["TVar", "V1", "Concept"], ["TVar", "V2", "Concept"]]]]
    q += [L("Similarity", [V("V1"), V("V2")], False), L("Similarity", [c[0], V("V1")], False),
          ["And", [L("Inheritance", [V("V1"), V("V2")]), L("Similarity", [V("V2"), V("V3")])]],
          ["And", [L("Inheritance", [V("V1"), V("V2")]), ["Not", L("Similarity", [V("V1"), V("V2")])]]],
          ["Or", [L("Inheritance", [V("V1"), c[3]]), L("Similarity", [V("V1"), c[3]])]],
          L("Similarity", [c[0], c[3]]), L("Inheritance", [c[0], c[3]])]
    return q


def blacklist_probes(das):
    h = lambda n: das.db.get_node_handle("Concept", n)  # noqa: E731
    P = []
    for t in ["Inheritance", "Similarity", "List", "Evaluation", "*"]:
        for targets in [["*", "*"], [h("c0"), "*"], ["*", h("c3")], ["*", "*", "*"], [h("c1"), "*", "*"]]:
            P.append(("links", [t, targets]))
        P.append(("type", t))
    for tpl in [["Inheritance", "Concept", "Concept"], ["Similarity", "Concept", "Concept"],
                ["List", "Concept", "Concept", "Concept"]]:
        P.append(("template", tpl))
    return P


_PATTERN_ORDER = []


def _record_pattern_order():
    """The order BuildPatternsThread (parser_threads.py:181-219) walks the
    MettaYacc loader's links, recorded before it runs (read only)."""
    orig = parser_threads_mod.BuildPatternsThread.run

    def run(self):
        _PATTERN_ORDER.append([e.hash_code for e in self.shared_data.regular_expressions_list])
        orig(self)
    parser_threads_mod.BuildPatternsThread.run = run


_record_pattern_order()


def blacklist_fixture():
    """pattern_black_list (distributed_atom_space.py:38, 346, 409): the
    reference's loaders skip the pattern-key family of a blacklisted link
    (canonical_parser.py:144, parser_threads.py:185) -- but `keys` is not
    reset, so the link is written under the previous link's keys
    (canonical_parser.py:177-178, parser_threads.py:218-219), or the load
    fails when no earlier link set them.  Recorded for both loaders."""
    out = {"cases": []}
    p = os.path.join(SCRATCH, "blacklist.metta")
    with open(p, "w") as f:
        f.write(BLACKLIST_CANONICAL)
    cases = [("metta", os.path.join(REF, "data/samples/animals.metta"), ["Similarity"], animals_queries, animals_probes),
             ("metta", os.path.join(REF, "data/samples/animals.metta"), ["Inheritance"], animals_queries, animals_probes),
             ("canonical", p, ["Similarity"], blacklist_queries, blacklist_probes),
             ("canonical", p, ["Similarity", "Evaluation"], blacklist_queries, blacklist_probes),
             ("canonical", p, ["Inheritance"], blacklist_queries, blacklist_probes),
             ("canonical", os.path.join(REF, "data/samples/canonical_toy-example-mining.metta"), ["Inheritance"],
              toy_mining_queries, None)]
    for loader, path, bl, queries, probes in cases:
        rec = {"loader": loader, "black_list": bl,
               "source": "inline" if path == p else os.path.relpath(path, REF)}
        _PATTERN_ORDER.clear()
        das = new_das()
        das.pattern_black_list = list(bl)
        try:
            if loader == "metta":
                das.load_knowledge_base(path)
            else:
                das.load_canonical_knowledge_base(path)
                das.db.prefetch()
        except Exception as e:
            rec["load_error"] = type(e).__name__
        # the links in the order the pattern-key loop walked them
        # (canonical_parser.py:136-137: links_1, links_2, links_N collections in
        # insertion order; parser_threads.py:183: regular_expressions_list)
        if loader == "metta":
            rec["pattern_order"] = [h for order in _PATTERN_ORDER for h in order]
        else:
            rec["pattern_order"] = [d["_id"] for tag in ["1", "2", "N"]
                                    for d in das.db.mongo_link_collection[tag].find()]
        if "load_error" not in rec:
            rec.update(kb_fixture("blacklist", das, queries(), probes(das) if probes else None, rec["source"]))
        else:
            nodes, links = atom_table(das)
            rec["nodes"], rec["links"] = nodes, links
        out["cases"].append(rec)
    out["canonical_text"] = BLACKLIST_CANONICAL
    return out


def main():
    which = sys.argv[1:] or ["hash", "stubdb", "animals", "toy_mining", "stub_like", "synthetic"]
    if "hash" in which:
        write("hash_vectors.json", hash_vectors())
    if "stubdb" in which:
        write("stubdb.json", stubdb_fixture())
    if "animals" in which:
        das = load_metta([os.path.join(REF, "data/samples/animals.metta")])
        write("kb_animals.json", kb_fixture("animals", das, animals_queries(), animals_probes(das),
                                            "data/samples/animals.metta"))
    if "toy_mining" in which:
        das = load_canonical(os.path.join(REF, "data/samples/canonical_toy-example-mining.metta"))
        write("kb_toy_mining.json", kb_fixture("toy_mining", das, toy_mining_queries(), None,
                                               "data/samples/canonical_toy-example-mining.metta"))
    if "kv_toy_mining" in which:
        # the key-value files CanonicalParser writes before populating Redis
        # (canonical_parser.py:132-183, key_value_file.py:8-16), sorted by the
        # reference's own `sort` call: the byte-level target of das_export_keyspace
        load_canonical(os.path.join(REF, "data/samples/canonical_toy-example-mining.metta"))
        out_dir = os.path.join(HERE, "kv_toy_mining")
        os.makedirs(out_dir, exist_ok=True)
        for name in ("outgoing_set", "incomming_set", "patterns", "templates", "names"):
            with open(os.path.join(SCRATCH, f"parser_{name}.txt")) as f:
                lines = sorted(l.rstrip("\n") for l in f if l.strip())
            with open(os.path.join(out_dir, f"{name}.txt"), "w") as f:
                f.write("".join(l + "\n" for l in lines))
    if "blacklist" in which:
        write("kb_blacklist.json", blacklist_fixture())
    if "stub_like" in which:
        p = os.path.join(SCRATCH, "stub_like.metta")
        with open(p, "w") as f:
            f.write(STUB_LIKE_METTA)
        das = load_metta([p])
        write("kb_stub_like.json", kb_fixture("stub_like", das, stub_like_queries(), None, "inline"))
    if "synthetic" in which:
        spec_path = os.path.join(SCRATCH, "synthetic_specs.json")
        if os.path.exists(spec_path):
            with open(spec_path) as f:
                specs = json.load(f)
            for s in specs:
                das = load_canonical(s["path"])
                fx = kb_fixture(s["name"], das, s["queries"], None, s["generator"], table_limit=(0, 0))
                fx["text_sha256"] = s["text_sha256"]
                write(f"kb_{s['name']}.json", fx)


if __name__ == "__main__":
    main()
