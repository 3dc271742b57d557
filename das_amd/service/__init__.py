"""Caller side of the gRPC service (service/server.py): the query-string
mini-language that the service's `query` RPC evaluates through
`DistributedAtomSpace.query`.  The gRPC transport itself is out of scope."""
from .query_parser import _parse_query, parse_query  # noqa: F401
