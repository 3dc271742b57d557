"""ctypes binding of libdas_mi355x.so (include/das_mi355x.h).

The product path has no CPU fallback: if the shared library is missing or no
gfx950 device is present, importing works but every call that needs the GPU
raises `DasNativeError` (or `ImportError` for a missing library) loudly.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DAS_MI355X_LIB", os.path.join(_HERE, "libdas_mi355x.so"))

DAS_NONE = 0xFFFFFFFF
TABLE_ORDERED = 0
TABLE_UNORDERED = 1
TABLE_COMPOSITE = 2

ERR_INVALID, ERR_HIP, ERR_NOT_BUILT, ERR_UNSUPPORTED, ERR_INTERNAL, ERR_ATTRIBUTE = -1, -2, -3, -4, -5, -6
ERR_SYNTAX = -7


class DasNativeError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[das_mi355x {code}] {msg}")
        self.code = code


class das_atoms_t(C.Structure):
    _fields_ = [
        ("n_leaf", C.c_uint64),
        ("leaf_bytes", C.c_void_p),
        ("leaf_off", C.c_void_p),
        ("leaf_kind", C.c_void_p),
        ("leaf_ctype", C.c_void_p),
        ("leaf_type_id", C.c_void_p),
        ("n_expr", C.c_uint64),
        ("expr_off", C.c_void_p),
        ("expr_child", C.c_void_p),
        ("expr_kind", C.c_void_p),
        ("expr_ctype_leaf", C.c_void_p),
        ("n_levels", C.c_uint32),
        ("level_off", C.c_void_p),
        ("n_types", C.c_uint32),
    ]


class das_index_stats_t(C.Structure):
    _fields_ = [
        ("n_atoms", C.c_uint64), ("n_nodes", C.c_uint64), ("n_links", C.c_uint64),
        ("n_types", C.c_uint64), ("n_ctypes", C.c_uint64), ("device_bytes", C.c_uint64),
        ("links_by_arity", C.c_uint64 * 9),
    ]


class das_link_scan_t(C.Structure):
    _fields_ = [
        ("arity", C.c_uint32), ("type_id", C.c_uint32), ("target", C.c_uint32 * 8),
        ("var", C.c_int32 * 8), ("n_vars", C.c_uint32), ("ordered", C.c_uint32),
        ("no_overload", C.c_uint32), ("emit_link", C.c_uint32), ("order_pos", C.c_int32),
    ]


class das_template_scan_t(C.Structure):
    _fields_ = [
        ("ctype_id", C.c_uint32), ("arity", C.c_uint32), ("var", C.c_int32 * 8),
        ("ordered", C.c_uint32), ("no_overload", C.c_uint32), ("emit_link", C.c_uint32),
    ]


class das_plan_node_t(C.Structure):
    _fields_ = [
        ("op", C.c_int32), ("nchild", C.c_uint32), ("value", C.c_uint32), ("dedup", C.c_uint32),
        ("index_join", C.c_uint32), ("scan", das_link_scan_t), ("ij", das_link_scan_t),
    ]


PLAN_LINK, PLAN_CONST, PLAN_NOT, PLAN_AND, PLAN_OR, PLAN_INPUT, PLAN_TEMPLATE, PLAN_TVM = 1, 2, 3, 4, 5, 6, 7, 8
PLAN_WORDS = 51                   # u32 words per das_plan_node_t
PLAN_SCAN = 5                     # word offset of its `scan` (das_link_scan_t)

P = C.c_void_p
DAS_BUILD_EXPR_ON_DEVICE = 1
U32P = C.POINTER(C.c_uint32)

# name -> (restype, argtypes); every function returns int status unless noted.
_SIGS = {
    "das_version": (C.c_int, []),
    "das_ctx_create": (C.c_int, [C.c_int, P, C.POINTER(P)]),
    "das_ctx_destroy": (C.c_int, [P]),
    "das_last_error": (C.c_char_p, [P]),
    "das_ctx_sync": (C.c_int, [P]),
    "das_md5": (C.c_int, [P, C.c_uint64, P]),
    "das_composite_digest": (C.c_int, [P, C.c_uint32, P]),
    "das_hash_strings_dev": (C.c_int, [P, P, P, C.c_uint64, P]),
    "das_hash_fixed_dev": (C.c_int, [P, P, C.c_uint32, C.c_uint64, P]),
    "das_build_index": (C.c_int, [P, C.POINTER(das_atoms_t)]),
    "das_build_index_ex": (C.c_int, [P, C.POINTER(das_atoms_t), C.c_uint32]),
    "das_build_index_sharded": (C.c_int, [P, C.POINTER(das_atoms_t), C.c_uint32, C.c_uint32, C.c_uint32]),
    "das_hash_owners": (C.c_int, [P, C.POINTER(das_atoms_t), C.c_uint32, C.c_uint32, P]),
    "das_partition_rows": (C.c_int, [P, P, C.c_uint64, C.c_uint32, P, C.c_uint32, P, P]),
    "das_numbered_strings": (C.c_int, [C.c_char_p, C.c_uint64, C.c_uint64, C.c_uint64, P, P]),
    "das_synth_powerlaw_links": (C.c_int, [P, P, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32,
                                           C.c_uint32, C.c_uint64, C.c_double, C.c_uint64]),
    "das_index_stats": (C.c_int, [P, C.POINTER(das_index_stats_t)]),
    "das_lookup": (C.c_int, [P, P, C.c_uint64, P, P, P, P]),
    "das_atoms_info": (C.c_int, [P, P, C.c_uint64, P, P, P, P, P]),
    "das_link_targets": (C.c_int, [P, C.c_uint32, P, C.c_uint32, P]),
    "das_ctype_lookup": (C.c_int, [P, P, P]),
    "das_incoming": (C.c_int, [P, C.c_uint32, P, C.c_uint64, P]),
    "das_export_outgoing": (C.c_int, [P, P, P, P, P]),
    "das_counters": (C.c_int, [P]),
    "das_scan_link": (C.c_int, [P, C.POINTER(das_link_scan_t), C.POINTER(P)]),
    "das_scan_template": (C.c_int, [P, C.POINTER(das_template_scan_t), C.POINTER(P)]),
    "das_scan_type": (C.c_int, [P, C.c_uint32, P]),
    "das_join": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(P)]),
    "das_antijoin": (C.c_int, [P, P, P, C.POINTER(P)]),
    "das_index_join": (C.c_int, [P, P, C.POINTER(das_link_scan_t), C.POINTER(P)]),
    "das_dedup": (C.c_int, [P, P, C.POINTER(P)]),
    "das_concat": (C.c_int, [P, P, C.c_uint32, C.POINTER(P)]),
    "das_set_dedup": (C.c_int, [P, P, C.c_uint32, P]),
    "das_set_minus": (C.c_int, [P, P, C.c_uint32, P, C.c_uint32, P]),
    "das_table_members": (C.c_int, [P, P]),
    "das_table_set_bounds": (C.c_int, [P, P, P]),
    "das_table_get_bounds": (C.c_int, [P, P, P]),
    "das_table_checksum": (C.c_int, [P, P, P, P]),
    "das_set_pattern_black_list": (C.c_int, [P, P, C.c_uint32]),
    "das_table_info": (C.c_int, [P, P, P, P, P]),
    "das_table_fetch": (C.c_int, [P, P, C.c_uint64, C.c_uint64, P]),
    "das_table_column": (C.c_int, [P, C.c_int32, P]),
    "das_table_from_host": (C.c_int, [P, C.c_int32, C.c_int32, P, P, P, C.c_uint64, C.POINTER(P)]),
    "das_table_free": (C.c_int, [P]),
    "das_partition": (C.c_int, [P, P, P, C.c_uint32, C.c_uint32, C.POINTER(P), P]),
    "das_table_gather": (C.c_int, [P, P, P, C.c_uint64, C.POINTER(P)]),
    "das_table_gather_ranges": (C.c_int, [P, P, P, P, C.c_uint32, C.POINTER(P)]),
    "das_table_export_rows": (C.c_int, [P, P, P]),
    "das_table_import_rows": (C.c_int, [P, C.c_int32, C.c_int32, P, P, P, C.c_uint64, C.POINTER(P)]),
    "das_parse_canonical": (C.c_int, [P, P, C.c_uint32, C.c_uint32, C.POINTER(P)]),
    "das_export_keyspace": (C.c_int, [P, C.c_char_p, P]),
    "das_parsed_atoms": (C.c_int, [P, C.POINTER(das_atoms_t), C.POINTER(P)]),
    "das_parsed_type_name": (C.c_int, [P, C.c_uint32, C.POINTER(C.c_char_p), C.POINTER(C.c_uint64)]),
    "das_parsed_free": (C.c_int, [P]),
    "das_plan_execute": (C.c_int, [P, C.POINTER(das_plan_node_t), C.c_uint32, C.c_uint32, P, C.c_uint32,
                                   C.POINTER(C.c_uint32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "das_plan_execute_many": (C.c_int, [P, C.c_uint32, P, P, C.c_uint32, P, C.c_uint32, P, P, P, P]),
    "das_plan_execute_info": (C.c_int, [P, P, C.c_uint32, C.c_uint32, P, C.c_uint32, P, P, P, P]),
    "das_plan_execute_sharded": (C.c_int, [P, C.POINTER(das_plan_node_t), C.c_uint32, C.c_uint32, P, C.c_uint32, P,
                                           C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_int32),
                                           C.POINTER(C.c_int32), P, C.c_uint32, C.POINTER(C.c_uint32)]),
    "das_plan_estimates": (C.c_int, [P, C.POINTER(das_plan_node_t), C.c_uint32, P]),
    "das_plan_bounds": (C.c_int, [P, C.POINTER(das_plan_node_t), C.c_uint32, P]),
    "das_prof_enable": (C.c_int, [P, C.c_int]),
    "das_prof_only": (C.c_int, [P, C.c_char_p]),
    "das_prof_tag": (C.c_int, [P, C.c_char_p]),
    "das_prof_tag_plan": (C.c_int, [P, C.c_uint32, C.c_char_p]),
    "das_box_store_bw": (C.c_int, [P, C.c_uint64, C.c_uint32, P]),
    "das_prof_mark": (C.c_int, [P, C.c_uint32]),
    "das_prof_reset": (C.c_int, [P]),
    "das_prof_read": (C.c_int, [P, C.c_char_p, P, P, P]),
    "das_prof_names": (C.c_int, [P, P, C.c_uint64]),
}

_lib = None


def lib():
    """The loaded shared library (raises ImportError if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libdas_mi355x.so not found at {LIB_PATH}: run __graft_entry__.build() "
                              "(hipcc --offload-arch=gfx950); there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGS)


def check(rc, ctx=None):
    if rc != 0:
        msg = lib().das_last_error(ctx)
        msg = msg.decode(errors="replace") if msg else ""
        if rc == ERR_INVALID:
            raise ValueError(msg)
        if rc == ERR_UNSUPPORTED:
            raise NotImplementedError(msg)
        if rc == ERR_ATTRIBUTE:
            raise AttributeError(msg)
        if rc == ERR_SYNTAX:
            raise AssertionError(msg)
        raise DasNativeError(rc, msg)


def ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


# ---------------------------------------------------------------------------
# canonical MeTTa reader (host C++, canonical.cpp)
# ---------------------------------------------------------------------------

def parse_canonical(texts, threads=0):
    """Canonical MeTTa text(s) -> loader.AtomArrays through das_parse_canonical
    (CanonicalParser.parse, canonical_parser.py:242-365).  Each text is one
    file with its own typedef / terminal / expression sections."""
    from .loader import AtomArrays
    if isinstance(texts, (str, bytes)):
        texts = [texts]
    bufs = [t.encode("utf-8") if isinstance(t, str) else bytes(t) for t in texts]
    n = len(bufs)
    arr = (C.c_char_p * max(n, 1))(*bufs)
    lens = np.array([len(b) for b in bufs] or [0], dtype=np.uint64)
    h = P()
    check(lib().das_parse_canonical(C.cast(arr, P), ptr(lens), n, int(threads), C.byref(h)))
    try:
        a = das_atoms_t()
        ns = P()
        check(lib().das_parsed_atoms(h, C.byref(a), C.byref(ns)))

        def take(p, count, dt):
            if not count:
                return np.zeros(0, dtype=dt)
            addr = p.value if isinstance(p, P) else p
            buf = (C.c_char * (count * np.dtype(dt).itemsize)).from_address(addr)
            return np.frombuffer(buf, dtype=dt).copy()

        nl, ne, ng = int(a.n_leaf), int(a.n_expr), int(a.n_levels)
        leaf_off = take(a.leaf_off, nl + 1, np.uint64)
        expr_off = take(a.expr_off, ne + 1, np.uint64)
        names = []
        for i in range(int(a.n_types)):
            sp, ln = C.c_char_p(), C.c_uint64()
            check(lib().das_parsed_type_name(h, i, C.byref(sp), C.byref(ln)))
            names.append(C.string_at(sp, ln.value).decode("utf-8"))
        return AtomArrays(take(a.leaf_bytes, int(leaf_off[-1]), np.uint8), leaf_off,
                          take(a.leaf_kind, nl, np.uint8), take(a.leaf_ctype, nl, np.uint32),
                          take(a.leaf_type_id, nl, np.uint32), take(ns, nl, np.uint32), expr_off,
                          take(a.expr_child, int(expr_off[-1]), np.uint32), take(a.expr_kind, ne, np.uint8),
                          take(a.expr_ctype_leaf, ne, np.int32), take(a.level_off, ng + 1, np.uint64), names)
    finally:
        lib().das_parsed_free(h)


def numbered_strings(prefix, n, first=0):
    """(bytes u8 array, n+1 u64 offsets) of prefix + str(first + i), i < n
    (das_numbered_strings: multi-threaded host C++)."""
    pre = prefix.encode()
    last = first + max(n - 1, 0)
    cap = n * (len(pre) + len(str(last)))
    out = np.empty(max(cap, 1), dtype=np.uint8)
    off = np.empty(n + 1, dtype=np.uint64)
    check(lib().das_numbered_strings(pre, len(pre), first, n, ptr(out), ptr(off)))
    return out[:int(off[-1])], off


# ---------------------------------------------------------------------------
# host hashing helpers (query planning); bulk hashing happens on the GPU
# ---------------------------------------------------------------------------

def md5_digest(text):
    b = text.encode("utf-8") if isinstance(text, str) else bytes(text)
    buf = C.create_string_buffer(b, len(b)) if b else None
    out = np.zeros(4, dtype=np.uint32)
    check(lib().das_md5(buf, len(b), ptr(out)))
    return out


def composite_digest(digests):
    d = np.ascontiguousarray(np.asarray(digests, dtype=np.uint32).reshape(-1, 4))
    out = np.zeros(4, dtype=np.uint32)
    check(lib().das_composite_digest(ptr(d), d.shape[0], ptr(out)))
    return out


def digest_to_hex(d):
    return np.asarray(d, dtype="<u4").tobytes().hex()


def counters():
    """(kernel launches, host read-backs) since the library loaded (das_counters)."""
    out = (C.c_uint64 * 2)()
    check(lib().das_counters(out))
    return int(out[0]), int(out[1])


def digests_to_hex(arr):
    """(n,4) uint32 little-endian words -> list of 32-char hex handles."""
    raw = np.ascontiguousarray(np.asarray(arr, dtype="<u4")).tobytes()
    h = raw.hex()
    return [h[i:i + 32] for i in range(0, len(h), 32)]


def hex_to_digest(h):
    if not isinstance(h, str) or len(h) != 32:
        raise ValueError(f"Invalid handle: {h}")
    try:
        return np.frombuffer(bytes.fromhex(h), dtype="<u4").astype(np.uint32)
    except ValueError:
        raise ValueError(f"Invalid handle: {h}")


class Table:
    """Owning wrapper of a das_table_t* (a device binding table)."""

    __slots__ = ("ctx", "h", "kind", "vars", "members", "nrows", "part")

    def __init__(self, ctx, handle, info=None):
        self.ctx = ctx
        self.h = handle
        self.part = None          # multi-GPU: how the rows are spread over ranks (das_amd.parallel)
        if info is not None and info[0] != TABLE_COMPOSITE:
            # (kind, ncols, nrows, 0, vars[16]) as das_plan_execute_many reports them
            self.kind, self.nrows = info[0], info[2]
            self.vars = tuple(info[4:4 + info[1]])
            self.members = None
            return
        kind = C.c_int32()
        ncols = C.c_int32()
        vars_ = (C.c_int32 * 16)()
        nrows = C.c_uint64()
        check(lib().das_table_info(handle, C.byref(kind), C.byref(ncols), vars_, C.byref(nrows)))
        self.kind = kind.value
        self.vars = tuple(vars_[i] for i in range(ncols.value))
        self.nrows = nrows.value
        if self.kind == TABLE_COMPOSITE:
            mem = (C.c_int32 * 16)()
            check(lib().das_table_members(handle, mem))
            self.members = tuple(mem[i] for i in range(ncols.value))
        else:
            self.members = None

    @property
    def schema(self):
        return (self.kind, self.vars, self.members)

    def set_bounds(self, lo, hi):
        k = len(self.vars)
        a = (C.c_uint32 * max(k, 1))(*[int(x) for x in lo])
        b = (C.c_uint32 * max(k, 1))(*[int(x) for x in hi])
        check(lib().das_table_set_bounds(self.h, a, b))

    def bounds(self):
        """(lo, hi) lists of the inclusive per-column value bounds."""
        k = len(self.vars)
        lo, hi = (C.c_uint32 * max(k, 1))(), (C.c_uint32 * max(k, 1))()
        check(lib().das_table_get_bounds(self.h, lo, hi))
        return [lo[i] for i in range(k)], [hi[i] for i in range(k)]

    def fetch(self, row0=0, nrows=None):
        """Rows [row0, row0 + nrows) (default: all) as a (ncols, n) host array."""
        n = self.nrows - row0 if nrows is None else min(nrows, self.nrows - row0)
        n, k = max(n, 0), len(self.vars)
        out = np.empty((k, n), dtype=np.uint32)
        if n and k:
            check(lib().das_table_fetch(self.ctx.h, self.h, row0, n, ptr(out)), self.ctx.h)
        return out

    def checksum(self, salts):
        """(sum, bad) of das_table_checksum with one 64-bit salt per column."""
        s = np.asarray([int(x) & ((1 << 64) - 1) for x in salts], dtype=np.uint64)
        assert len(s) == len(self.vars)
        out = np.zeros(2, dtype=np.uint64)
        check(lib().das_table_checksum(self.ctx.h, self.h, ptr(s), ptr(out)), self.ctx.h)
        return int(out[0]), int(out[1])

    def free(self):
        if self.h is not None:
            lib().das_table_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Context:
    """A device context: one HBM index + the stream every kernel runs on."""

    def __init__(self, device=0, stream=None):
        h = P()
        check(lib().das_ctx_create(int(device), stream, C.byref(h)))
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            lib().das_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _table(self, fn, *args):
        out = P()
        check(fn(self.h, *args, C.byref(out)), self.h)
        return Table(self, out)

    @staticmethod
    def _atoms(a):
        """(das_atoms_t, build flags, buffers to keep alive) of host AtomArrays
        or of a KB whose expression arrays are device tensors (`expr_on_device`)."""
        dev = bool(getattr(a, "expr_on_device", False))
        eptr = (lambda t: C.c_void_p(t.data_ptr())) if dev else ptr
        keep = [a.leaf_bytes, a.leaf_off, a.leaf_kind, a.leaf_ctype, a.leaf_type_id, a.expr_off,
                a.expr_child, a.expr_kind, a.expr_ctype_leaf, a.level_off]
        s = das_atoms_t(
            n_leaf=a.n_leaf, leaf_bytes=ptr(a.leaf_bytes), leaf_off=ptr(a.leaf_off), leaf_kind=ptr(a.leaf_kind),
            leaf_ctype=ptr(a.leaf_ctype), leaf_type_id=ptr(a.leaf_type_id), n_expr=a.n_expr,
            expr_off=eptr(a.expr_off), expr_child=eptr(a.expr_child), expr_kind=eptr(a.expr_kind),
            expr_ctype_leaf=eptr(a.expr_ctype_leaf), n_levels=len(a.level_off) - 1, level_off=ptr(a.level_off),
            n_types=len(a.type_names))
        return s, (DAS_BUILD_EXPR_ON_DEVICE if dev else 0), keep

    def set_pattern_black_list(self, type_names):
        """Named types whose links the next build gives no pattern keys
        (das_set_pattern_black_list; md5 of each name = named_type_hash)."""
        import hashlib
        names = sorted(set(type_names or ()))
        d = np.frombuffer(b"".join(hashlib.md5(n.encode()).digest() for n in names), dtype="<u4").copy()
        check(lib().das_set_pattern_black_list(self.h, ptr(d) if len(names) else None, len(names)), self.h)

    def build_index(self, arrays, shard=None):
        """Host arrays (das_build_index), or a KB whose expression arrays are
        device tensors (`arrays.expr_on_device`, das_build_index_ex).
        shard=(rank, world): links hash-partitioned by handle, this context
        indexing the links whose handles `rank` owns (das_build_index_sharded)."""
        s, flags, keep = self._atoms(arrays)
        if shard is not None and shard[1] > 1:
            check(lib().das_build_index_sharded(self.h, C.byref(s), flags, int(shard[0]), int(shard[1])), self.h)
        elif flags:
            check(lib().das_build_index_ex(self.h, C.byref(s), flags), self.h)
        else:
            check(lib().das_build_index(self.h, C.byref(s)), self.h)
        del keep

    def hash_owners(self, arrays, world, d_owner):
        """Owner shard of every expression's handle into device u8 tensor d_owner."""
        s, flags, keep = self._atoms(arrays)
        check(lib().das_hash_owners(self.h, C.byref(s), flags, int(world), C.c_void_p(d_owner.data_ptr())), self.h)
        del keep

    def partition_rows(self, rows, n, k, owner, world, out):
        """n rows of k u32 (device tensor) regrouped by device u8 `owner` into
        `out`; returns the per-owner row counts."""
        counts = np.zeros(world, dtype=np.uint64)
        check(lib().das_partition_rows(self.h, C.c_void_p(rows.data_ptr()), int(n), int(k),
                                       C.c_void_p(owner.data_ptr()), int(world), C.c_void_p(out.data_ptr()),
                                       ptr(counts)), self.h)
        return counts

    def synth_powerlaw_links(self, d_child, first, n, k, n_link_types, type_leaf0, node_leaf0, n_nodes,
                             s=1.1, seed=0):
        """Fills device buffer `d_child` (a u32/i32 tensor of n*k) with links
        [first, first+n) of the counter-hashed Zipf hypergraph."""
        check(lib().das_synth_powerlaw_links(self.h, C.c_void_p(d_child.data_ptr()), first, n, k, n_link_types,
                                             type_leaf0, node_leaf0, n_nodes, s, seed), self.h)

    def export_keyspace(self, directory):
        """Redis key-space files of the index (das_export_keyspace) -> line counts."""
        counts = np.zeros(5, dtype=np.uint64)
        check(lib().das_export_keyspace(self.h, str(directory).encode(), ptr(counts)), self.h)
        return dict(zip(("outgoing_set", "incomming_set", "patterns", "templates", "names"),
                        (int(x) for x in counts)))

    def stats(self):
        st = das_index_stats_t()
        check(lib().das_index_stats(self.h, C.byref(st)), self.h)
        return st

    def lookup(self, digests):
        d = np.ascontiguousarray(np.asarray(digests, dtype=np.uint32).reshape(-1, 4))
        n = d.shape[0]
        ids = np.zeros(n, dtype=np.int64)
        cat = np.zeros(n, dtype=np.uint8)
        ar = np.zeros(n, dtype=np.uint32)
        ty = np.zeros(n, dtype=np.uint32)
        if n:
            check(lib().das_lookup(self.h, ptr(d), n, ptr(ids), ptr(cat), ptr(ar), ptr(ty)), self.h)
        return ids, cat, ar, ty

    def lookup_hex(self, hexes):
        """Handle strings -> (ids, categories, arities) as lists: lookup()
        without numpy, for the few handles of one query."""
        n = len(hexes)
        buf = (C.c_uint32 * (4 * n)).from_buffer_copy(bytes.fromhex("".join(hexes)))
        ids, cat = (C.c_int64 * n)(), (C.c_uint8 * n)()
        ar, ty = (C.c_uint32 * n)(), (C.c_uint32 * n)()
        check(lib().das_lookup(self.h, buf, n, ids, cat, ar, ty), self.h)
        return list(ids), list(cat), list(ar)

    def atoms_info(self, ids):
        ids = np.ascontiguousarray(np.asarray(ids, dtype=np.uint32))
        n = ids.shape[0]
        dig = np.zeros((n, 4), dtype=np.uint32)
        cat = np.zeros(n, dtype=np.uint8)
        ar = np.zeros(n, dtype=np.uint32)
        ty = np.zeros(n, dtype=np.uint32)
        nl = np.zeros(n, dtype=np.uint32)
        if n:
            check(lib().das_atoms_info(self.h, ptr(ids), n, ptr(dig), ptr(cat), ptr(ar), ptr(ty), ptr(nl)), self.h)
        return dig, cat, ar, ty, nl

    def link_targets(self, atom_id):
        buf = np.zeros(64, dtype=np.uint32)
        n = C.c_uint32()
        check(lib().das_link_targets(self.h, int(atom_id), ptr(buf), 64, C.byref(n)), self.h)
        return buf[:n.value].copy()

    def outgoing_csr(self):
        """(tgt_off u64[n_atoms + 1], tgt u32[...]) host copies of the outgoing CSR."""
        n_off, n_tgt = C.c_uint64(), C.c_uint64()
        check(lib().das_export_outgoing(self.h, None, None, C.byref(n_off), C.byref(n_tgt)), self.h)
        off = np.empty(n_off.value, dtype=np.uint64)
        tgt = np.empty(max(n_tgt.value, 1), dtype=np.uint32)
        check(lib().das_export_outgoing(self.h, ptr(off), ptr(tgt), C.byref(n_off), C.byref(n_tgt)), self.h)
        return off, tgt[:n_tgt.value]

    def incoming(self, atom_id):
        n = C.c_uint64()
        check(lib().das_incoming(self.h, int(atom_id), None, 0, C.byref(n)), self.h)
        out = np.zeros(max(n.value, 1), dtype=np.uint32)
        if n.value:
            check(lib().das_incoming(self.h, int(atom_id), ptr(out), n.value, C.byref(n)), self.h)
        return out[:n.value]

    def ctype_lookup(self, digest):
        d = np.ascontiguousarray(np.asarray(digest, dtype=np.uint32))
        out = C.c_int64()
        check(lib().das_ctype_lookup(self.h, ptr(d), C.byref(out)), self.h)
        return out.value

    def plan_execute(self, words, n_nodes, no_overload=False):
        """das_plan_execute over n_nodes das_plan_node_t records given as a
        u32 array (51 words each) -> (matched, negation, [Table])."""
        cap = 16
        nodes = words.__array_interface__["data"][0]
        while True:
            out = (P * cap)()
            n_out, matched, neg = C.c_uint32(), C.c_int32(), C.c_int32()
            info = (C.c_int64 * (20 * cap))()
            rc = lib().das_plan_execute_info(self.h, nodes, n_nodes, 1 if no_overload else 0, out, cap,
                                             C.byref(n_out), C.byref(matched), C.byref(neg), info)
            if rc == ERR_INVALID and n_out.value > cap:
                cap = n_out.value          # more answer schemas than slots: run again with room for all
                continue
            check(rc, self.h)
            k = n_out.value
            return bool(matched.value), bool(neg.value), [Table(self, out[i], info[20 * i:20 * i + 20])
                                                          for i in range(k)]

    def plan_execute_many(self, plans, no_overload=False):
        """das_plan_execute_many over [(words, n_nodes)] -> one (matched,
        negation, [Table]) per plan, each as plan_execute's on it alone."""
        m = len(plans)
        if m == 0:
            return []
        ptrs = (P * m)(*[w.ctypes.data for w, _ in plans])
        ns = np.array([k for _, k in plans], dtype=np.uint32)
        cap = 8 * m
        while True:
            out = (P * cap)()
            n_out = np.zeros(m, dtype=np.uint32)
            matched = np.zeros(m, dtype=np.int32)
            neg = np.zeros(m, dtype=np.int32)
            info = np.zeros((cap, 20), dtype=np.int64)
            rc = lib().das_plan_execute_many(self.h, m, ptrs, ptr(ns), 1 if no_overload else 0, out, cap, ptr(n_out),
                                             ptr(matched), ptr(neg), ptr(info))
            if rc == ERR_INVALID and int(n_out.sum()) > cap:
                cap = int(n_out.sum())
                continue
            check(rc, self.h)
            res, k = [], 0
            inf = info.tolist()
            for i in range(m):
                j = int(n_out[i])
                res.append((bool(matched[i]), bool(neg[i]), [Table(self, out[k + q], inf[k + q]) for q in range(j)]))
                k += j
            return res

    def plan_execute_sharded(self, words, n_nodes, inputs, no_overload=False):
        """das_plan_execute_sharded: (matched, negation, [Table], checks)."""
        nodes = C.cast(words.ctypes.data, C.POINTER(das_plan_node_t))
        ins = (P * max(len(inputs), 1))(*[t.h for t in inputs])
        cap, ccap = 64, max(64, n_nodes)
        while True:
            out = (P * cap)()
            ck = np.zeros(ccap, dtype=np.uint8)
            n_out, matched, neg, n_ck = C.c_uint32(), C.c_int32(), C.c_int32(), C.c_uint32()
            rc = lib().das_plan_execute_sharded(self.h, nodes, n_nodes, 1 if no_overload else 0, ins, len(inputs),
                                                out, cap, C.byref(n_out), C.byref(matched), C.byref(neg), ptr(ck),
                                                ccap, C.byref(n_ck))
            if rc == ERR_INVALID and (n_out.value > cap or n_ck.value > ccap):
                cap, ccap = max(cap, n_out.value), max(ccap, n_ck.value)
                continue
            check(rc, self.h)
            return (bool(matched.value), bool(neg.value), [Table(self, out[i]) for i in range(n_out.value)],
                    ck[:n_ck.value].copy())

    def plan_estimates(self, words, n_nodes):
        """Index rows each LINK node's scan would read on this GPU (u64 per node)."""
        out = np.zeros(max(n_nodes, 1), dtype=np.uint64)
        nodes = C.cast(words.ctypes.data, C.POINTER(das_plan_node_t))
        check(lib().das_plan_estimates(self.h, nodes, n_nodes, ptr(out)), self.h)
        return out[:n_nodes]

    def plan_bounds(self, words, n_nodes):
        """Per node, an upper bound of plan_estimates over its shape (u64; 2^64-1 unknown)."""
        out = np.zeros(max(n_nodes, 1), dtype=np.uint64)
        nodes = C.cast(words.ctypes.data, C.POINTER(das_plan_node_t))
        check(lib().das_plan_bounds(self.h, nodes, n_nodes, ptr(out)), self.h)
        return out[:n_nodes]

    def scan_words(self, words, node):
        """The rows of plan leaf `node` on this GPU: das_scan_link of a LINK
        record's scan, das_scan_template of a TEMPLATE record's."""
        base = PLAN_WORDS * node
        if int(words[base]) == PLAN_TEMPLATE:
            w = words[base + PLAN_SCAN:base + PLAN_SCAN + 23]
            return self.scan_template(int(w[1]), int(w[0]), [int(np.int32(v)) for v in w[10:10 + int(w[0])]],
                                      bool(w[19]), bool(w[20]))
        q = C.cast(words.ctypes.data + 4 * (base + PLAN_SCAN), C.POINTER(das_link_scan_t))
        return self._table(lib().das_scan_link, q)

    @staticmethod
    def link_scan_struct(q, arity, type_id, targets, var, n_vars, ordered, no_overload=False, emit_link=False,
                         order_pos=-1):
        """Fills a das_link_scan_t (scan_link's argument layout)."""
        q.order_pos = order_pos
        q.arity = arity
        q.type_id = DAS_NONE if type_id is None else type_id
        for i in range(8):
            q.target[i] = targets[i] if i < len(targets) else DAS_NONE
            q.var[i] = var[i] if i < len(var) else -1
        q.n_vars = n_vars
        q.ordered = 1 if ordered else 0
        q.no_overload = 1 if no_overload else 0
        q.emit_link = 1 if emit_link else 0
        return q

    def scan_link(self, arity, type_id, targets, var, n_vars, ordered, no_overload=False, emit_link=False,
                  order_pos=-1):
        q = das_link_scan_t()
        q.order_pos = order_pos
        q.arity = arity
        q.type_id = DAS_NONE if type_id is None else type_id
        for i in range(8):
            q.target[i] = targets[i] if i < len(targets) else DAS_NONE
            q.var[i] = var[i] if i < len(var) else -1
        q.n_vars = n_vars
        q.ordered = 1 if ordered else 0
        q.no_overload = 1 if no_overload else 0
        q.emit_link = 1 if emit_link else 0
        return self._table(lib().das_scan_link, C.byref(q))

    def index_join(self, a, arity, type_id, targets, var):
        """das_index_join: join(a, scan_link(ordered q)) through P_{a,p};
        None when it does not apply (the caller scans and joins)."""
        q = das_link_scan_t()
        q.order_pos = -1
        q.arity = arity
        q.type_id = DAS_NONE if type_id is None else type_id
        for i in range(8):
            q.target[i] = targets[i] if i < len(targets) else DAS_NONE
            q.var[i] = var[i] if i < len(var) else -1
        q.ordered = 1
        out = P()
        check(lib().das_index_join(self.h, a.h, C.byref(q), C.byref(out)), self.h)
        return Table(self, out) if out.value else None

    def scan_template(self, ctype_id, arity, var, ordered, no_overload=False, emit_link=False):
        q = das_template_scan_t()
        q.ctype_id = ctype_id
        q.arity = arity
        for i in range(8):
            q.var[i] = var[i] if i < len(var) else -1
        q.ordered = 1 if ordered else 0
        q.no_overload = 1 if no_overload else 0
        q.emit_link = 1 if emit_link else 0
        return self._table(lib().das_scan_template, C.byref(q))

    def scan_type(self, type_id):
        arr = (P * 9)()
        check(lib().das_scan_type(self.h, int(type_id), arr), self.h)
        return [Table(self, arr[a]) if arr[a] else None for a in range(9)]

    def join(self, a, b, no_overload=False):
        return self._table(lib().das_join, a.h, b.h, 1 if no_overload else 0)

    def antijoin(self, a, t):
        return self._table(lib().das_antijoin, a.h, t.h)

    def dedup(self, a):
        return self._table(lib().das_dedup, a.h)

    def concat(self, tables):
        arr = (P * len(tables))(*[t.h for t in tables])
        return self._table(lib().das_concat, arr, len(tables))

    def set_dedup(self, tables):
        """Python-set identity across tables of any kinds: first occurrence kept."""
        arr = (P * len(tables))(*[t.h for t in tables])
        out = (P * len(tables))()
        check(lib().das_set_dedup(self.h, arr, len(tables), out), self.h)
        return [Table(self, out[i]) for i in range(len(tables))]

    def set_minus(self, a, b):
        """Rows of each table of `a` whose identity is in no table of `b`."""
        aa = (P * max(len(a), 1))(*[t.h for t in a])
        bb = (P * max(len(b), 1))(*[t.h for t in b])
        out = (P * max(len(a), 1))()
        check(lib().das_set_minus(self.h, aa, len(a), bb, len(b), out), self.h)
        return [Table(self, out[i]) for i in range(len(a))]

    def table_from_host(self, kind, vars_, cols, members=None):
        cols = np.ascontiguousarray(np.asarray(cols, dtype=np.uint32))
        v = (C.c_int32 * max(len(vars_), 1))(*vars_)
        m = (C.c_int32 * max(len(vars_), 1))(*members) if members is not None else None
        n = cols.shape[1] if cols.ndim == 2 else 0
        return self._table(lib().das_table_from_host, kind, len(vars_), v, m, ptr(cols), n)

    def partition(self, t, key_vars, nparts):
        kv = (C.c_int32 * max(len(key_vars), 1))(*key_vars)
        counts = np.zeros(nparts, dtype=np.uint64)
        out = P()
        check(lib().das_partition(self.h, t.h, kv, len(key_vars), nparts, C.byref(out), ptr(counts)), self.h)
        return Table(self, out), counts

    def gather(self, t, idx):
        """Rows idx (host indices) of table t as a new table."""
        idx = np.ascontiguousarray(np.asarray(idx, dtype=np.uint32))
        return self._table(lib().das_table_gather, t.h, ptr(idx), idx.shape[0])

    def gather_ranges(self, t, begin, end):
        """Rows [begin[i], end[i]) of table t, in range order, as a new table."""
        b = np.ascontiguousarray(np.asarray(begin, dtype=np.uint64))
        e = np.ascontiguousarray(np.asarray(end, dtype=np.uint64))
        return self._table(lib().das_table_gather_ranges, t.h, ptr(b), ptr(e), b.shape[0])

    def export_rows(self, t, dptr):
        check(lib().das_table_export_rows(self.h, t.h, dptr), self.h)

    def import_rows(self, kind, vars_, dptr, nrows, members=None):
        v = (C.c_int32 * max(len(vars_), 1))(*vars_)
        m = (C.c_int32 * max(len(vars_), 1))(*members) if members is not None else None
        return self._table(lib().das_table_import_rows, kind, len(vars_), v, m, dptr, nrows)

    def prof_enable(self, on=True):
        check(lib().das_prof_enable(self.h, 1 if on else 0), self.h)

    def prof_reset(self):
        check(lib().das_prof_reset(self.h), self.h)

    def prof_only(self, name=None):
        """Record events only for scopes named `name` (None: every scope)."""
        check(lib().das_prof_only(self.h, name.encode() if name else None), self.h)

    def prof_tag(self, tag=None):
        """Name the scopes recorded from now on "<scope>@<tag>" (None: untagged)."""
        check(lib().das_prof_tag(self.h, tag.encode() if tag else None), self.h)

    def box_store_bw(self, nbytes=4 << 30, reps=5):
        """GB/s of the card's 16-byte nontemporal stores (das_box_store_bw)."""
        g = C.c_double()
        check(lib().das_box_store_bw(self.h, int(nbytes), int(reps), C.byref(g)), self.h)
        return g.value

    def prof_mark(self, mark_id):
        """A k_prof_mark launch on the context stream (kernel-trace bracket)."""
        check(lib().das_prof_mark(self.h, int(mark_id)), self.h)

    def prof_tag_plan(self, plan=None, tag=None):
        """Tag the launches of plan `plan` of each following plan_execute_many
        batch "<scope>@<tag>" (None: untag)."""
        on = plan is not None and tag
        check(lib().das_prof_tag_plan(self.h, int(plan) if on else 0xFFFFFFFF, tag.encode() if on else None), self.h)

    def prof_stats(self):
        buf = C.create_string_buffer(1 << 16)
        check(lib().das_prof_names(self.h, buf, len(buf)), self.h)
        out = {}
        for name in buf.value.decode().split("\n"):
            if not name:
                continue
            ms, n, b = C.c_double(), C.c_uint64(), C.c_double()
            check(lib().das_prof_read(self.h, name.encode(), C.byref(ms), C.byref(n), C.byref(b)), self.h)
            out[name] = {"ms": ms.value, "launches": n.value, "bytes": b.value}
        return out

    def sync(self):
        check(lib().das_ctx_sync(self.h), self.h)
