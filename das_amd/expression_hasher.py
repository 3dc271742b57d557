"""ExpressionHasher with the reference's API (das/expression_hasher.py:4-35).

Single handles (query planning, facade calls: a handful per query) are
computed on the host with hashlib's MD5, the function the reference itself
calls; bulk hashing of a knowledge base runs on the GPU inside
`das_build_index` (one message per lane, das_amd/csrc/hash.hip).
"""
import hashlib
from typing import Any, List


class ExpressionHasher:

    compound_separator = " "

    @staticmethod
    def _compute_hash(text: str) -> str:
        return hashlib.md5(text.encode("utf-8")).hexdigest()

    @staticmethod
    def named_type_hash(name: str) -> str:
        return ExpressionHasher._compute_hash(name)

    @staticmethod
    def terminal_hash(named_type: str, terminal_name: str) -> str:
        return ExpressionHasher._compute_hash(ExpressionHasher.compound_separator.join([named_type, terminal_name]))

    @staticmethod
    def expression_hash(named_type_hash: str, elements: List[str]) -> str:
        return ExpressionHasher.composite_hash([named_type_hash, *elements])

    @staticmethod
    def composite_hash(hash_base: Any) -> str:
        if isinstance(hash_base, str):
            return hash_base
        if isinstance(hash_base, list):
            if len(hash_base) == 1:
                return hash_base[0]
            return ExpressionHasher._compute_hash(ExpressionHasher.compound_separator.join(hash_base))
        raise ValueError(f"Invalid base to compute composite hash: {type(hash_base)}: {hash_base}")
