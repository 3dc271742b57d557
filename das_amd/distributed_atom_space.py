"""DistributedAtomSpace facade with the reference's API
(das/distributed_atom_space.py:26-415).

The reference connects to Redis + MongoDB from environment variables; this
facade owns a `HipDB` on one MI355X instead (`device=` / `DAS_DEVICE`).  Query
evaluation, output formats and the loader entry points keep the reference's
names and behaviour.
"""
import json
import os
from enum import Enum, auto
from typing import Dict, List, Tuple, Union

from . import _lib
from . import loader as _loader
from .database.db_interface import WILDCARD
from .database.hip_db import HipDB
from .pattern_matcher.pattern_matcher import LogicalExpression, PatternMatchingAnswer
from .transaction import Transaction


class QueryOutputFormat(int, Enum):
    HANDLE = auto()
    ATOM_INFO = auto()
    JSON = auto()


def _format_assignments(assignments) -> str:
    """str(set of assignments) (distributed_atom_space.py:308), with each
    OrderedAssignment's repr(mapping) taken in C (das_amd._assign.format_set)
    instead of through its Python __repr__."""
    from .pattern_matcher import pattern_matcher as _pm
    if _pm._assign is None:
        return str(assignments)
    return _pm._assign.format_set(assignments, _pm.OrderedAssignment)


class DistributedAtomSpace:

    def __init__(self, **kwargs):
        self.database_name = kwargs.get("database_name", "das")
        device = int(kwargs.get("device", os.environ.get("DAS_DEVICE", 0)))
        # db: an existing DBInterface (a HipDB, or a parallel.ShardedDB over
        # one process per GPU); default: a HipDB on `device`
        # stale_pattern_keys: the reference canonical loader's pattern keys
        # under a non-empty pattern_black_list, bug for bug (HipDB)
        self.db = kwargs.get("db") or HipDB(device=device, tuple_targets=kwargs.get("tuple_targets", False),
                                            stale_pattern_keys=kwargs.get("stale_pattern_keys", False))
        self.pattern_black_list = []
        self._metta_sources = []
        self._canonical_sources = []
        self._parsed = None          # arrays resumed by load_parsed_knowledge_base

    # -- loading -------------------------------------------------------------
    def _get_file_list(self, source):
        """distributed_atom_space.py:81-99"""
        answer = []
        if os.path.isfile(source):
            answer.append(source)
        elif os.path.isdir(source):
            for file_name in os.listdir(source):
                path = "/".join([source, file_name])
                if os.path.exists(path):
                    answer.append(path)
        else:
            raise ValueError(f"Invalid knowledge base path: {source}")
        answer = [f for f in answer if f.endswith(".metta") or f.endswith(".scm")]
        if len(answer) == 0:
            raise ValueError(f"No MeTTa files found in {source}")
        return answer

    def _rebuild(self):
        # canonical files through the native reader (canonical.cpp), general
        # MeTTa through the Python MettaYacc restatement, one device index
        # the loaders honour pattern_black_list (distributed_atom_space.py:346, 409)
        self.db.pattern_black_list = list(self.pattern_black_list)
        parts = [self._parsed] if self._parsed is not None else []
        stale = None
        if self._canonical_sources:
            if not self._metta_sources and hasattr(self.db, "stale_from_canonical"):
                stale = self.db.stale_from_canonical(self._canonical_sources)
            parts.append(_lib.parse_canonical(self._canonical_sources))
        if self._metta_sources or not parts:
            parts.append(_loader.parse_metta(self._metta_sources).finish())
        if self._parsed is not None and (self._canonical_sources or self._metta_sources):
            stale = None        # stale entries are recorded for canonical-only loads
        self.db.load_arrays(_loader.concat_arrays(parts))
        if stale:
            self.db._stale = stale

    def load_knowledge_base(self, source):
        """distributed_atom_space.py:336-363 (general MeTTa)."""
        for f in self._get_file_list(source):
            with open(f) as fh:
                self._metta_sources.append(fh.read())
        self._rebuild()

    def load_canonical_knowledge_base(self, source):
        """distributed_atom_space.py:365-414 (canonical MeTTa)."""
        for f in sorted(self._get_file_list(source), reverse=True):
            with open(f) as fh:
                self._canonical_sources.append(fh.read())
        self._rebuild()

    def save_parsed_knowledge_base(self, path):
        """The loaded KB, parsed, to one .npz (HipDB.save_parsed): a later
        load_parsed_knowledge_base skips the parser, as the reference's
        loader does when it reuses its key-value files
        (canonical_parser.py:28-29, 317-319)."""
        self.db.save_parsed(path)

    def load_parsed_knowledge_base(self, path):
        """Replaces the KB with a saved one (its pattern_black_list
        included); later loads and transactions add to it."""
        self._metta_sources = []
        self._canonical_sources = []
        self._parsed = self.db.load_parsed(path)
        self.pattern_black_list = list(self.db.pattern_black_list)

    def open_transaction(self) -> Transaction:
        return Transaction()

    def commit_transaction(self, transaction: Transaction) -> None:
        """distributed_atom_space.py:326-334: parse the transaction's MeTTa with
        the knowledge already loaded, then rebuild the device index."""
        self._metta_sources.append(transaction.metta_string)
        self._rebuild()

    def clear_database(self):
        self._metta_sources = []
        self._canonical_sources = []
        self._parsed = None
        self.db.clear()

    # -- API -----------------------------------------------------------------
    def count_atoms(self) -> Tuple[int, int]:
        return self.db.count_atoms()

    def get_atom(self, handle: str, output_format: QueryOutputFormat = QueryOutputFormat.HANDLE):
        if output_format == QueryOutputFormat.HANDLE or not handle:
            atom = self.db.get_atom_as_dict(handle)
            return atom["handle"] if atom else ""
        if output_format == QueryOutputFormat.ATOM_INFO:
            return self.db.get_atom_as_dict(handle)
        if output_format == QueryOutputFormat.JSON:
            return json.dumps(self.db.get_atom_as_deep_representation(handle), sort_keys=False, indent=4)
        raise ValueError(f"Invalid output format: '{output_format}'")

    def get_node(self, node_type: str, node_name: str, output_format: QueryOutputFormat = QueryOutputFormat.HANDLE):
        node_handle = self.db.get_node_handle(node_type, node_name)
        if output_format == QueryOutputFormat.HANDLE or node_handle is None:
            return node_handle
        if output_format == QueryOutputFormat.ATOM_INFO:
            return self.db.get_atom_as_dict(node_handle)
        if output_format == QueryOutputFormat.JSON:
            return json.dumps(self.db.get_atom_as_deep_representation(node_handle), sort_keys=False, indent=4)
        raise ValueError(f"Invalid output format: '{output_format}'")

    def get_nodes(self, node_type: str, node_name: str = None, output_format=QueryOutputFormat.HANDLE):
        if node_name is not None:
            answer = [self.db.get_node_handle(node_type, node_name)]
        else:
            answer = self.db.get_all_nodes(node_type)
        if output_format == QueryOutputFormat.HANDLE or not answer:
            return answer
        if output_format == QueryOutputFormat.ATOM_INFO:
            return [self.db.get_atom_as_dict(h) for h in answer]
        if output_format == QueryOutputFormat.JSON:
            return json.dumps([self.db.get_atom_as_deep_representation(h) for h in answer], sort_keys=False, indent=4)
        raise ValueError(f"Invalid output format: '{output_format}'")

    def get_link(self, link_type: str, targets: List[str] = None, output_format=QueryOutputFormat.HANDLE):
        link_handle = self.db.get_link_handle(link_type, targets)
        if link_handle is None or output_format == QueryOutputFormat.HANDLE:
            return link_handle
        if output_format == QueryOutputFormat.ATOM_INFO:
            return self.db.get_atom_as_dict(link_handle, len(targets))
        if output_format == QueryOutputFormat.JSON:
            return json.dumps(self.db.get_atom_as_deep_representation(link_handle, len(targets)),
                              sort_keys=False, indent=4)
        raise ValueError(f"Invalid output format: '{output_format}'")

    def get_links(self, link_type: str, target_types: str = None, targets: List[str] = None,
                  output_format: QueryOutputFormat = QueryOutputFormat.HANDLE):
        """distributed_atom_space.py:259-284"""
        if link_type is None:
            link_type = WILDCARD
        if target_types is not None and link_type != WILDCARD:
            db_answer = self.db.get_matched_type_template([link_type, *target_types])
        elif targets is not None and output_format == QueryOutputFormat.HANDLE and \
                hasattr(self.db, "get_matched_link_handles"):
            # the handles alone: no (link, targets) rows built only to be dropped
            return self.db.get_matched_link_handles(link_type, targets)
        elif targets is not None:
            db_answer = self.db.get_matched_links(link_type, targets)
        elif link_type != WILDCARD:
            db_answer = self.db.get_matched_type(link_type)
        else:
            raise ValueError("Invalid parameters")
        if output_format == QueryOutputFormat.HANDLE:
            if not db_answer:
                return []
            return db_answer if isinstance(db_answer[0], str) else [h for h, _ in db_answer]
        if output_format == QueryOutputFormat.ATOM_INFO:
            return [self.db.get_atom_as_dict(a if isinstance(a, str) else a[0]) for a in db_answer]
        if output_format == QueryOutputFormat.JSON:
            return json.dumps([self.db.get_atom_as_deep_representation(a if isinstance(a, str) else a[0])
                               for a in db_answer], sort_keys=False, indent=4)
        raise ValueError(f"Invalid output format: '{output_format}'")

    def get_link_type(self, link_handle: str) -> str:
        return self.db.get_link_type(link_handle)

    def get_link_targets(self, link_handle: str) -> List[str]:
        return self.db.get_link_targets(link_handle)

    def get_node_type(self, node_handle: str) -> str:
        return self.db.get_node_type(node_handle)

    def get_node_name(self, node_handle: str) -> str:
        return self.db.get_node_name(node_handle)

    def query(self, query: LogicalExpression, output_format: QueryOutputFormat = QueryOutputFormat.HANDLE) -> str:
        """distributed_atom_space.py:298-321"""
        query_answer = PatternMatchingAnswer()
        matched = query.matched(self.db, query_answer)
        tag_not = ""
        mapping = ""
        if matched:
            if query_answer.negation:
                tag_not = "NOT "
            if output_format == QueryOutputFormat.HANDLE:
                mapping = _format_assignments(query_answer.assignments)
            elif output_format in (QueryOutputFormat.ATOM_INFO, QueryOutputFormat.JSON):
                # the reference calls .items() on a set here and raises
                # (distributed_atom_space.py:312-318); kept as-is.
                query_answer.assignments.items()
            else:
                raise ValueError(f"Invalid output format: '{output_format}'")
        return f"{tag_not}{mapping}"
