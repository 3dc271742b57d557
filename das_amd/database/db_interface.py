"""The reference's DB plugin surface (das/database/db_interface.py:4-71).

`HipDB` (das_amd/database/hip_db.py) is the MI355X implementation.  The
constants and method names are the reference's, so callers written against
`DBInterface` keep working after the import swap.
"""
from abc import ABC, abstractmethod
from typing import Any, List

WILDCARD = "*"
UNORDERED_LINK_TYPES = ["Similarity", "Set"]


class DBInterface(ABC):

    def __repr__(self):
        return "<DBInterface>"

    @abstractmethod
    def node_exists(self, node_type: str, node_name: str) -> bool: ...

    @abstractmethod
    def link_exists(self, link_type: str, targets: List[str]) -> bool: ...

    @abstractmethod
    def get_node_handle(self, node_type: str, node_name: str) -> str: ...

    @abstractmethod
    def get_link_handle(self, link_type: str, target_handles: List[str]) -> str: ...

    @abstractmethod
    def get_link_targets(self, handle: str) -> List[str]: ...

    @abstractmethod
    def is_ordered(self, handle: str) -> bool: ...

    @abstractmethod
    def get_matched_links(self, link_type: str, target_handles: List[str]): ...

    @abstractmethod
    def get_all_nodes(self, node_type: str, names: bool = False) -> List[str]: ...

    @abstractmethod
    def get_matched_type_template(self, template: List[Any]) -> List[str]: ...

    @abstractmethod
    def get_matched_type(self, link_named_type: str): ...

    @abstractmethod
    def get_node_name(self, node_handle: str) -> str: ...

    @abstractmethod
    def get_matched_node_name(self, node_type: str, substring: str) -> str: ...

    def get_atom_as_dict(self, handle: str, arity: int):
        pass

    def get_atom_as_deep_representation(self, handle: str, arity: int):
        pass

    def count_atoms(self):
        pass
