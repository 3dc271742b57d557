"""das_amd — MI355X-native query hot path of DAS (Distributed Atom Space).

Drop-in for tanksha/das's `DistributedAtomSpace` / `pattern_matcher` /
`DBInterface` surface, backed by hand-written HIP kernels for gfx950
(das_amd/csrc) behind the C ABI in include/das_mi355x.h.
"""
__version__ = "0.1.0"
