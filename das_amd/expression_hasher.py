"""ExpressionHasher with the reference's API (das/expression_hasher.py:4-35).

Single handles (query planning, facade calls) are computed by the native
library's host MD5; bulk hashing of a knowledge base runs on the GPU inside
`das_build_index` (one message per lane, das_amd/csrc/hash.hip).
"""
import re
from typing import Any, List

from . import _lib

_HANDLE = re.compile(r"[0-9a-f]{32}")


class ExpressionHasher:

    compound_separator = " "

    @staticmethod
    def _compute_hash(text: str) -> str:
        return _lib.digest_to_hex(_lib.md5_digest(text))

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
            # digest fast path only for lowercase-hex handles: their hex
            # re-encoding is the text the reference joins (:33); anything else
            # (upper case hex, the '*' of pattern keys) is hashed as given
            if all(isinstance(h, str) and _HANDLE.fullmatch(h) for h in hash_base):
                digests = [_lib.hex_to_digest(h) for h in hash_base]
                return _lib.digest_to_hex(_lib.composite_digest(digests))
            return ExpressionHasher._compute_hash(ExpressionHasher.compound_separator.join(hash_base))
        raise ValueError(f"Invalid base to compute composite hash: {type(hash_base)}: {hash_base}")
