// extern "C" boundary (include/das_mi355x.h).  Every entry point catches
// das::Error / std::exception and returns a status; the message is kept per
// context for das_last_error.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "canonical.h"
#include "das_internal.h"
#include "md5.h"

using das::Ctx;
using das::Digest;
using das::Error;
using das::Table;

struct das_ctx {
  Ctx c;
};
struct das_table {
  Table t;
};
struct das_parsed {
  std::unique_ptr<das::Parsed> p;
};

namespace {

thread_local std::string g_err;   // errors without a context

int fail(das_ctx_t* ctx, int code, const std::string& msg) {
  if (ctx) ctx->c.err = msg;
  g_err = msg;
  return code;
}

// DAS_SYNC_CHECK=1: synchronise after every entry point so an asynchronous
// kernel fault is reported by the call that launched it (debug builds of a run).
bool sync_check() {
  static const bool on = [] {
    const char* e = std::getenv("DAS_SYNC_CHECK");
    return e && e[0] == '1';
  }();
  return on;
}

// DAS_HOST_TRACE=1: one stderr line per entry point with its host time (us),
// to attribute host-side gaps between kernels.
bool host_trace() {
  static const bool on = [] {
    const char* e = std::getenv("DAS_HOST_TRACE");
    return e && e[0] == '1';
  }();
  return on;
}

struct HostTrace {
  const char* fn;
  std::chrono::steady_clock::time_point t0;
  explicit HostTrace(const char* f) : fn(f) {
    if (host_trace()) t0 = std::chrono::steady_clock::now();
  }
  ~HostTrace() {
    if (!host_trace()) return;
    const auto t1 = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[das] %-26s %12.1f %8.1f\n", fn,
                 std::chrono::duration<double, std::micro>(t0.time_since_epoch()).count(),
                 std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
};

// The context a C-ABI call runs for, visible to KScope for its duration.
struct ActiveCtx {
  das::Ctx* prev;
  explicit ActiveCtx(das::Ctx* c) : prev(das::active_ctx()) { das::active_ctx() = c; }
  ~ActiveCtx() { das::active_ctx() = prev; }
};

template <typename F>
int guarded(das_ctx_t* ctx, F&& f, const char* fn = __builtin_FUNCTION()) {
  HostTrace tr(fn);
  try {
    if (ctx) {
      std::lock_guard<std::mutex> lk(ctx->c.mu);
      ActiveCtx act(&ctx->c);
      int cur = -1;
      if (hipGetDevice(&cur) != hipSuccess || cur != ctx->c.device) DAS_HIP(hipSetDevice(ctx->c.device));
      f();
      if (sync_check()) {
        DAS_HIP(hipStreamSynchronize(ctx->c.s));
        DAS_HIP(hipGetLastError());
      }
    } else {
      f();
    }
    return DAS_OK;
  } catch (const Error& e) {
    return fail(ctx, e.code, e.what());
  } catch (const std::exception& e) {
    return fail(ctx, DAS_ERR_INTERNAL, e.what());
  } catch (...) {
    return fail(ctx, DAS_ERR_INTERNAL, "unknown error");
  }
}

// Schema of an imported table: composite member ids run 0, 1, .. in column
// order after the ordered (-1) columns, each member's variables sorted.
void check_schema(int32_t kind, int32_t ncols, const int32_t* vars, const int32_t* member) {
  DAS_CHECK(kind >= DAS_TABLE_ORDERED && kind <= DAS_TABLE_COMPOSITE, das::DAS_E_INVALID, "bad table kind");
  DAS_CHECK(ncols >= 0 && ncols <= das::kMaxCols, das::DAS_E_UNSUPPORTED, "too many columns");
  if (kind != DAS_TABLE_COMPOSITE) return;
  DAS_CHECK(member != nullptr, das::DAS_E_INVALID, "composite table without member ids");
  int32_t prev = -1;
  for (int c = 0; c < ncols; ++c) {
    DAS_CHECK(member[c] == prev || member[c] == prev + 1, das::DAS_E_INVALID, "composite member ids out of order");
    if (c > 0 && member[c] == member[c - 1])
      DAS_CHECK(vars[c] > vars[c - 1], das::DAS_E_INVALID, "composite member variables not sorted");
    prev = member[c];
  }
}

das_table_t* wrap(std::unique_ptr<Table> t) {
  // das_table holds a Table; take over every field and the device buffer
  auto* w = new das_table;
  w->t = *t;
  t->data = nullptr;
  return w;
}

__global__ void k_atom_info(const uint32_t* ids, uint64_t n, const Digest* dig, const uint8_t* cat,
                            const uint32_t* arity, const uint32_t* type, const uint32_t* name_leaf, Digest* o_dig,
                            uint8_t* o_cat, uint32_t* o_arity, uint32_t* o_type, uint32_t* o_name) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t id = ids[i];
    if (o_dig) o_dig[i] = dig[id];
    if (o_cat) o_cat[i] = cat[id];
    if (o_arity) o_arity[i] = arity[id];
    if (o_type) o_type[i] = type[id];
    if (o_name) o_name[i] = name_leaf[id];
  }
}

}  // namespace

extern "C" {

int das_version(void) { return 1; }

int das_ctx_create(int device, void* stream, das_ctx_t** out) {
  if (!out) return fail(nullptr, DAS_ERR_INVALID, "null out");
  das_ctx_t* ctx = nullptr;
  int rc = guarded(nullptr, [&] {
    int n = 0;
    DAS_HIP(hipGetDeviceCount(&n));
    DAS_CHECK(device >= 0 && device < n, das::DAS_E_INVALID, "no such HIP device");
    DAS_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    DAS_HIP(hipGetDeviceProperties(&prop, device));
    DAS_CHECK(std::strncmp(prop.gcnArchName, "gfx950", 6) == 0, das::DAS_E_UNSUPPORTED,
              std::string("this build targets gfx950 (MI355X), device is ") + prop.gcnArchName);
    // keep freed stream-ordered allocations in the pool: the query operators
    // allocate per call, and returning memory to the OS at each sync costs more
    // than the kernels on small queries
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
      uint64_t keep = ~0ull;
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
    ctx = new das_ctx_t;
    ctx->c.device = device;
    if (stream) {
      ctx->c.s = (hipStream_t)stream;
    } else {
      // a blocking stream: ordered against work on the legacy null stream
      // (torch's default stream), so torch-side copies into buffers the
      // library reads, and reads of buffers it wrote, need no extra fences
      DAS_HIP(hipStreamCreateWithFlags(&ctx->c.s, hipStreamDefault));
      ctx->c.own_stream = true;
    }
  });
  if (rc) {
    delete ctx;
    return rc;
  }
  *out = ctx;
  return DAS_OK;
}

int das_ctx_destroy(das_ctx_t* ctx) {
  if (!ctx) return DAS_OK;
  int rc = guarded(ctx, [&] {
    DAS_HIP(hipStreamSynchronize(ctx->c.s));
    das::prof_collect(ctx->c);
    for (hipEvent_t e : ctx->c.ev_pool) (void)hipEventDestroy(e);
    ctx->c.ev_pool.clear();
    das::free_index(ctx->c.idx);
    ctx->c.zlc.release();                 // back to the cache while the stream still exists
    das::cache_release_stream(ctx->c.s);
    for (auto& z : ctx->c.zlc_side) z.release();
    for (hipStream_t& ss : ctx->c.side)
      if (ss) {
        DAS_HIP(hipStreamSynchronize(ss));
        das::cache_release_stream(ss);
        DAS_HIP(hipStreamDestroy(ss));
        ss = nullptr;
      }
    if (ctx->c.gsc_pool) {
      (void)hipFree(ctx->c.gsc_pool);
      ctx->c.gsc_pool = nullptr;
    }
    for (hipEvent_t e : ctx->c.side_ev) (void)hipEventDestroy(e);
    ctx->c.side_ev.clear();
    if (ctx->c.own_stream) DAS_HIP(hipStreamDestroy(ctx->c.s));
  });
  delete ctx;
  return rc;
}

const char* das_last_error(const das_ctx_t* ctx) { return ctx ? ctx->c.err.c_str() : g_err.c_str(); }

int das_counters(uint64_t out[2]) {
  if (!out) return fail(nullptr, DAS_ERR_INVALID, "null out");
  das::read_counters(out);
  return DAS_OK;
}

int das_ctx_sync(das_ctx_t* ctx) {
  return guarded(ctx, [&] { DAS_HIP(hipStreamSynchronize(ctx->c.s)); });
}

int das_md5(const uint8_t* bytes, uint64_t n, uint32_t out[4]) {
  das::md5::digest_bytes(bytes, n, out);
  return DAS_OK;
}

int das_composite_digest(const uint32_t* digests, uint32_t k, uint32_t out[4]) {
  if (k == 0) return fail(nullptr, DAS_ERR_INVALID, "composite of nothing");
  if (k == 1) {
    std::memcpy(out, digests, 16);
    return DAS_OK;
  }
  std::string msg;
  msg.reserve(33 * k);
  for (uint32_t i = 0; i < k; ++i) {
    char hex[32];
    das::md5::to_hex(digests + 4 * i, hex);
    if (i) msg.push_back(' ');
    msg.append(hex, 32);
  }
  das::md5::digest_bytes((const uint8_t*)msg.data(), msg.size(), out);
  return DAS_OK;
}

int das_hash_strings_dev(das_ctx_t* ctx, const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint32_t* d_out) {
  return guarded(ctx, [&] { das::hash_strings(d_bytes, d_off, n, dig_s((Digest*)d_out), ctx->c.s); });
}

int das_hash_fixed_dev(das_ctx_t* ctx, const uint32_t* d_elems, uint32_t k, uint64_t n, uint32_t* d_out) {
  return guarded(ctx, [&] { das::hash_fixed((const Digest*)d_elems, k, n, (Digest*)d_out, ctx->c.s); });
}

int das_parse_canonical(const char* const* texts, const uint64_t* lens, uint32_t n_texts, uint32_t n_threads,
                        das_parsed_t** out) {
  return guarded(nullptr, [&] {
    DAS_CHECK(out && (n_texts == 0 || (texts && lens)), das::DAS_E_INVALID, "null argument");
    auto p = das::parse_canonical(texts, lens, n_texts, n_threads);
    *out = new das_parsed{std::move(p)};
  });
}

int das_parsed_atoms(const das_parsed_t* p, das_atoms_t* a, const uint32_t** name_start) {
  return guarded(nullptr, [&] {
    DAS_CHECK(p && a, das::DAS_E_INVALID, "null argument");
    const das::Parsed& x = *p->p;
    a->n_leaf = x.leaf_kind.size();
    a->leaf_bytes = x.leaf_bytes.data();
    a->leaf_off = x.leaf_off.data();
    a->leaf_kind = x.leaf_kind.data();
    a->leaf_ctype = x.leaf_ctype.data();
    a->leaf_type_id = x.leaf_type_id.data();
    a->n_expr = x.expr_kind.size();
    a->expr_off = x.expr_off.data();
    a->expr_child = x.expr_child.data();
    a->expr_kind = x.expr_kind.data();
    a->expr_ctype_leaf = x.expr_ctype_leaf.data();
    a->n_levels = (uint32_t)(x.level_off.size() - 1);
    a->level_off = x.level_off.data();
    a->n_types = (uint32_t)x.type_names.size();
    if (name_start) *name_start = x.name_start.data();
  });
}

int das_parsed_type_name(const das_parsed_t* p, uint32_t type_id, const char** name, uint64_t* len) {
  return guarded(nullptr, [&] {
    DAS_CHECK(p && name && len, das::DAS_E_INVALID, "null argument");
    DAS_CHECK(type_id < p->p->type_names.size(), das::DAS_E_INVALID, "type id out of range");
    *name = p->p->type_names[type_id].data();
    *len = p->p->type_names[type_id].size();
  });
}

int das_parsed_free(das_parsed_t* p) {
  delete p;
  return DAS_OK;
}

int das_export_keyspace(das_ctx_t* ctx, const char* dir, uint64_t counts[5]) {
  return guarded(ctx, [&] {
    DAS_CHECK(dir, das::DAS_E_INVALID, "null directory");
    const das::ExportCounts n = das::export_keyspace(ctx->c, dir);
    if (counts) {
      counts[0] = n.outgoing;
      counts[1] = n.incoming;
      counts[2] = n.patterns;
      counts[3] = n.templates;
      counts[4] = n.names;
    }
  });
}

// A build keeps every freed scratch block in the caching allocator (best-fit
// reuse, no budget) and, when it ends, returns the idle ones to the driver --
// all of them by default, or down to DAS_BUILD_KEEP_GB (the largest kept):
// bench.py's build leg keeps everything from a same-input warm-up build, so
// the timed build maps no new device memory (a fresh multi-GB hipMalloc there
// stalled 1.4-1.9 s in ~1 of 3 processes, profiles/r5_build_alloc_stall.txt).
struct BuildHold {
  BuildHold() { das::cache_hold(true); }
  ~BuildHold() {
    das::cache_hold(false);
    const char* k = std::getenv("DAS_BUILD_KEEP_GB");
    das::cache_trim_to(k ? (size_t)(std::atof(k) * 1e9) : 0);
  }
};

int das_build_index(das_ctx_t* ctx, const das_atoms_t* atoms) {
  if (!ctx || !atoms) return fail(ctx, DAS_ERR_INVALID, "null argument");
  return guarded(ctx, [&] {
    BuildHold hold;
    das::build_index(ctx->c, *atoms, 0);
  });
}

int das_build_index_ex(das_ctx_t* ctx, const das_atoms_t* atoms, uint32_t flags) {
  if (!ctx || !atoms) return fail(ctx, DAS_ERR_INVALID, "null argument");
  if (flags & ~DAS_BUILD_EXPR_ON_DEVICE) return fail(ctx, DAS_ERR_INVALID, "unknown build flags");
  return guarded(ctx, [&] {
    BuildHold hold;
    das::build_index(ctx->c, *atoms, flags);
  });
}

int das_build_index_sharded(das_ctx_t* ctx, const das_atoms_t* atoms, uint32_t flags, uint32_t rank,
                            uint32_t world) {
  if (!ctx || !atoms) return fail(ctx, DAS_ERR_INVALID, "null argument");
  if (flags & ~DAS_BUILD_EXPR_ON_DEVICE) return fail(ctx, DAS_ERR_INVALID, "unknown build flags");
  return guarded(ctx, [&] {
    BuildHold hold;
    das::build_index(ctx->c, *atoms, flags, rank, world);
  });
}

int das_hash_owners(das_ctx_t* ctx, const das_atoms_t* atoms, uint32_t flags, uint32_t world, uint8_t* d_owner) {
  if (!ctx || !atoms || (atoms->n_expr && !d_owner)) return fail(ctx, DAS_ERR_INVALID, "null argument");
  if (flags & ~DAS_BUILD_EXPR_ON_DEVICE) return fail(ctx, DAS_ERR_INVALID, "unknown build flags");
  return guarded(ctx, [&] { das::hash_owners(ctx->c, *atoms, flags, world, d_owner); });
}

int das_partition_rows(das_ctx_t* ctx, const uint32_t* d_rows, uint64_t n, uint32_t K, const uint8_t* d_owner,
                       uint32_t world, uint32_t* d_out, uint64_t* counts) {
  if (!ctx || !counts || (n && (!d_rows || !d_owner || !d_out))) return fail(ctx, DAS_ERR_INVALID, "null argument");
  return guarded(ctx, [&] { das::partition_rows(ctx->c, d_rows, n, K, d_owner, world, d_out, counts); });
}

int das_numbered_strings(const char* prefix, uint64_t plen, uint64_t first, uint64_t n, uint8_t* out,
                         uint64_t* off) {
  if ((plen && !prefix) || !off || (n && !out)) return fail(nullptr, DAS_ERR_INVALID, "null argument");
  return guarded(nullptr, [&] { das::numbered_strings(prefix, plen, first, n, out, off); });
}

int das_synth_powerlaw_links(das_ctx_t* ctx, uint32_t* d_child, uint64_t first, uint64_t n, uint32_t K,
                             uint32_t n_link_types, uint32_t type_leaf0, uint32_t node_leaf0, uint64_t n_nodes,
                             double s, uint64_t seed) {
  if (!ctx || (n && !d_child)) return fail(ctx, DAS_ERR_INVALID, "null argument");
  return guarded(ctx, [&] {
    das::synth_powerlaw_links(d_child, first, n, K, n_link_types, type_leaf0, node_leaf0, n_nodes, s, seed,
                              ctx->c.s);
  });
}

int das_index_stats(das_ctx_t* ctx, das_index_stats_t* out) {
  return guarded(ctx, [&] {
    const das::Index& x = ctx->c.idx;
    std::memset(out, 0, sizeof(*out));
    out->n_atoms = x.n_atoms;
    out->n_nodes = x.n_nodes;
    out->n_links = x.n_links;
    out->n_types = x.n_types;
    out->n_ctypes = x.ctype_digest.size();
    out->device_bytes = x.device_bytes;
    for (int a = 1; a <= das::kMaxArity; ++a) out->links_by_arity[a] = x.ttab[a].rows;
  });
}

int das_lookup(das_ctx_t* ctx, const uint32_t* digests, uint64_t n, int64_t* ids, uint8_t* cat, uint32_t* arity,
               uint32_t* type) {
  bool done = false;
  int rc = guarded(ctx, [&] {
    done = das::lookup_small(ctx->c, (const Digest*)digests, n, ids, cat, arity, type);
    if (!done) das::lookup_digests(ctx->c, (const Digest*)digests, n, ids);
  });
  if (rc || done || (!cat && !arity && !type)) return rc;
  std::vector<uint32_t> valid;
  std::vector<uint64_t> where;
  for (uint64_t i = 0; i < n; ++i) {
    if (cat) cat[i] = 0;
    if (arity) arity[i] = 0;
    if (type) type[i] = das::kNone;
    if (ids[i] >= 0) { valid.push_back((uint32_t)ids[i]); where.push_back(i); }
  }
  if (valid.empty()) return DAS_OK;
  std::vector<uint8_t> c(valid.size());
  std::vector<uint32_t> a(valid.size()), t(valid.size());
  rc = das_atoms_info(ctx, valid.data(), valid.size(), nullptr, c.data(), a.data(), t.data(), nullptr);
  if (rc) return rc;
  for (size_t k = 0; k < valid.size(); ++k) {
    if (cat) cat[where[k]] = c[k];
    if (arity) arity[where[k]] = a[k];
    if (type) type[where[k]] = t[k];
  }
  return DAS_OK;
}

int das_atoms_info(das_ctx_t* ctx, const uint32_t* ids, uint64_t n, uint32_t* digests, uint8_t* cat, uint32_t* arity,
                   uint32_t* type, uint32_t* name_leaf) {
  return guarded(ctx, [&] {
    const das::Index& x = ctx->c.idx;
    DAS_CHECK(x.built, das::DAS_E_NOT_BUILT, "index not built");
    if (!n) return;
    for (uint64_t i = 0; i < n; ++i) DAS_CHECK(ids[i] < x.n_atoms, das::DAS_E_INVALID, "atom id out of range");
    hipStream_t s = ctx->c.s;
    das::DBuf<uint32_t> d_ids(n, s);
    DAS_HIP(hipMemcpyAsync(d_ids.p, ids, 4 * n, hipMemcpyHostToDevice, s));
    das::DBuf<Digest> dg(digests ? n : 0, s);
    das::DBuf<uint8_t> dc(cat ? n : 0, s);
    das::DBuf<uint32_t> da(arity ? n : 0, s), dt(type ? n : 0, s), dn(name_leaf ? n : 0, s);
    hipLaunchKernelGGL(k_atom_info, dim3(das::grid_for(n, 256)), dim3(256), 0, s, (const uint32_t*)d_ids.p, n,
                       (const Digest*)x.digest, (const uint8_t*)x.cat, (const uint32_t*)x.arity,
                       (const uint32_t*)x.type, (const uint32_t*)x.name_leaf, dg.p, dc.p, da.p, dt.p, dn.p);
    DAS_HIP(hipGetLastError());
    if (digests) DAS_HIP(hipMemcpyAsync(digests, dg.p, 16 * n, hipMemcpyDeviceToHost, s));
    if (cat) DAS_HIP(hipMemcpyAsync(cat, dc.p, n, hipMemcpyDeviceToHost, s));
    if (arity) DAS_HIP(hipMemcpyAsync(arity, da.p, 4 * n, hipMemcpyDeviceToHost, s));
    if (type) DAS_HIP(hipMemcpyAsync(type, dt.p, 4 * n, hipMemcpyDeviceToHost, s));
    if (name_leaf) DAS_HIP(hipMemcpyAsync(name_leaf, dn.p, 4 * n, hipMemcpyDeviceToHost, s));
    DAS_HIP(hipStreamSynchronize(s));
  });
}

int das_link_targets(das_ctx_t* ctx, uint32_t id, uint32_t* out, uint32_t cap, uint32_t* n) {
  return guarded(ctx, [&] {
    const das::Index& x = ctx->c.idx;
    DAS_CHECK(x.built, das::DAS_E_NOT_BUILT, "index not built");
    DAS_CHECK(id < x.n_atoms, das::DAS_E_INVALID, "atom id out of range");
    uint64_t off[2];
    DAS_HIP(hipMemcpyAsync(off, x.tgt_off + id, 16, hipMemcpyDeviceToHost, ctx->c.s));
    DAS_HIP(hipStreamSynchronize(ctx->c.s));
    const uint64_t k = off[1] - off[0];
    *n = (uint32_t)k;
    DAS_CHECK(k <= cap, das::DAS_E_INVALID, "target buffer too small");
    if (k) {
      DAS_HIP(hipMemcpyAsync(out, x.tgt + off[0], 4 * k, hipMemcpyDeviceToHost, ctx->c.s));
      DAS_HIP(hipStreamSynchronize(ctx->c.s));
    }
  });
}

int das_export_outgoing(das_ctx_t* ctx, uint64_t* off, uint32_t* tgt, uint64_t* n_off, uint64_t* n_tgt) {
  return guarded(ctx, [&] {
    const das::Index& x = ctx->c.idx;
    DAS_CHECK(x.built, das::DAS_E_NOT_BUILT, "index not built");
    DAS_CHECK(n_off && n_tgt, das::DAS_E_INVALID, "null size argument");
    uint64_t total = 0;
    DAS_HIP(hipMemcpyAsync(&total, x.tgt_off + x.n_atoms, 8, hipMemcpyDeviceToHost, ctx->c.s));
    DAS_HIP(hipStreamSynchronize(ctx->c.s));
    *n_off = x.n_atoms + 1;
    *n_tgt = total;
    if (!off && !tgt) return;
    DAS_CHECK(off && tgt, das::DAS_E_INVALID, "null buffer");
    DAS_HIP(hipMemcpyAsync(off, x.tgt_off, 8 * (x.n_atoms + 1), hipMemcpyDeviceToHost, ctx->c.s));
    if (total) DAS_HIP(hipMemcpyAsync(tgt, x.tgt, 4 * total, hipMemcpyDeviceToHost, ctx->c.s));
    DAS_HIP(hipStreamSynchronize(ctx->c.s));
  });
}

int das_incoming(das_ctx_t* ctx, uint32_t id, uint32_t* out, uint64_t cap, uint64_t* n) {
  return guarded(ctx, [&] {
    const das::Index& idx = ctx->c.idx;
    DAS_CHECK(idx.built, das::DAS_E_NOT_BUILT, "index not built");
    DAS_CHECK(id < idx.n_atoms, das::DAS_E_INVALID, "atom id out of range");
    uint32_t be[2];
    DAS_HIP(hipMemcpyAsync(be, idx.in_off + id, 8, hipMemcpyDeviceToHost, ctx->c.s));
    DAS_HIP(hipStreamSynchronize(ctx->c.s));
    *n = be[1] - be[0];
    const uint64_t m = std::min<uint64_t>(*n, cap);
    if (m) {
      DAS_HIP(hipMemcpyAsync(out, idx.in_link + be[0], 4 * m, hipMemcpyDeviceToHost, ctx->c.s));
      DAS_HIP(hipStreamSynchronize(ctx->c.s));
    }
  });
}

int das_ctype_lookup(das_ctx_t* ctx, const uint32_t digest[4], int64_t* ctype_id) {
  return guarded(ctx, [&] {
    const auto& v = ctx->c.idx.ctype_digest;
    Digest q{{digest[0], digest[1], digest[2], digest[3]}};
    auto it = std::lower_bound(v.begin(), v.end(), q, [](const Digest& a, const Digest& b) {
      return a.hi() < b.hi() || (a.hi() == b.hi() && a.lo() < b.lo());
    });
    *ctype_id = (it != v.end() && it->hi() == q.hi() && it->lo() == q.lo()) ? (int64_t)(it - v.begin()) : -1;
  });
}

int das_scan_link(das_ctx_t* ctx, const das_link_scan_t* q, das_table_t** out) {
  return guarded(ctx, [&] { *out = wrap(das::scan_link(ctx->c, *q)); });
}

int das_scan_template(das_ctx_t* ctx, const das_template_scan_t* q, das_table_t** out) {
  return guarded(ctx, [&] { *out = wrap(das::scan_template(ctx->c, *q)); });
}

int das_scan_type(das_ctx_t* ctx, uint32_t type_id, das_table_t** out9) {
  return guarded(ctx, [&] {
    for (int a = 0; a <= 8; ++a) out9[a] = nullptr;
    const das::Index& x = ctx->c.idx;
    DAS_CHECK(x.built, das::DAS_E_NOT_BUILT, "index not built");
    if (type_id >= x.n_types) return;
    for (int a = 1; a <= das::kMaxArity; ++a) {
      const das::RowTable& rt = x.ttab[a];
      if (!rt.rows) continue;
      const uint64_t b = x.type_off[a][type_id], e = x.type_off[a][type_id + 1];
      if (e <= b) continue;
      int32_t vars[das::kMaxCols];
      for (int k = 0; k <= a; ++k) vars[k] = k - 1;
      auto t = das::new_table(ctx->c, DAS_TABLE_ORDERED, a + 1, vars, e - b);
      t->nrows = e - b;
      for (int k = 0; k <= a; ++k)
        das::copy_dev(t->col(k), rt.col(k) + b, 4 * (e - b), ctx->c.s);
      out9[a] = wrap(std::move(t));
    }
  });
}

int das_join(das_ctx_t* ctx, const das_table_t* a, const das_table_t* b, uint32_t no_overload, das_table_t** out) {
  return guarded(ctx, [&] { *out = wrap(das::join(ctx->c, a->t, b->t, (int)no_overload)); });
}

int das_index_join(das_ctx_t* ctx, const das_table_t* a, const das_link_scan_t* q, das_table_t** out) {
  if (!ctx || !a || !q || !out) return fail(ctx, DAS_ERR_INVALID, "null argument");
  return guarded(ctx, [&] {
    auto t = das::index_join(ctx->c, a->t, *q);
    *out = t ? wrap(std::move(t)) : nullptr;
  });
}

int das_antijoin(das_ctx_t* ctx, const das_table_t* a, const das_table_t* t, das_table_t** out) {
  return guarded(ctx, [&] { *out = wrap(das::antijoin(ctx->c, a->t, t->t)); });
}

int das_dedup(das_ctx_t* ctx, const das_table_t* a, das_table_t** out) {
  return guarded(ctx, [&] { *out = wrap(das::dedup(ctx->c, a->t)); });
}

int das_concat(das_ctx_t* ctx, const das_table_t* const* ts, uint32_t n, das_table_t** out) {
  return guarded(ctx, [&] {
    std::vector<const Table*> v(n);
    for (uint32_t i = 0; i < n; ++i) v[i] = &ts[i]->t;
    *out = wrap(das::concat(ctx->c, v.data(), (int)n));
  });
}

int das_table_info(const das_table_t* t, int32_t* kind, int32_t* ncols, int32_t* vars, uint64_t* nrows) {
  if (!t) return fail(nullptr, DAS_ERR_INVALID, "null table");
  if (kind) *kind = t->t.kind;
  if (ncols) *ncols = t->t.ncols;
  if (vars) std::memcpy(vars, t->t.vars, sizeof(int32_t) * t->t.ncols);
  if (nrows) *nrows = t->t.nrows;
  return DAS_OK;
}

int das_table_fetch(das_ctx_t* ctx, const das_table_t* t, uint64_t row0, uint64_t nrows, uint32_t* out) {
  return guarded(ctx, [&] {
    DAS_CHECK(row0 + nrows <= t->t.nrows, das::DAS_E_INVALID, "fetch out of range");
    for (int c = 0; c < t->t.ncols; ++c)
      if (nrows)
        DAS_HIP(hipMemcpyAsync(out + (uint64_t)c * nrows, t->t.col(c) + row0, 4 * nrows, hipMemcpyDeviceToHost,
                               ctx->c.s));
    DAS_HIP(hipStreamSynchronize(ctx->c.s));
  });
}

int das_table_column(const das_table_t* t, int32_t c, uint32_t** dptr) {
  if (!t || c < 0 || c >= t->t.ncols) return fail(nullptr, DAS_ERR_INVALID, "bad column");
  *dptr = t->t.col(c);
  return DAS_OK;
}

int das_table_from_host(das_ctx_t* ctx, int32_t kind, int32_t ncols, const int32_t* vars, const int32_t* member,
                        const uint32_t* cols, uint64_t nrows, das_table_t** out) {
  return guarded(ctx, [&] {
    check_schema(kind, ncols, vars, member);
    auto t = das::new_table(ctx->c, kind, ncols, vars, nrows, member);
    t->nrows = nrows;
    for (int c = 0; c < ncols; ++c)
      if (nrows) DAS_HIP(hipMemcpyAsync(t->col(c), cols + (uint64_t)c * nrows, 4 * nrows, hipMemcpyHostToDevice, ctx->c.s));
    DAS_HIP(hipStreamSynchronize(ctx->c.s));
    *out = wrap(std::move(t));
  });
}

int das_table_free(das_table_t* t) {
  delete t;
  return DAS_OK;
}

int das_partition(das_ctx_t* ctx, const das_table_t* t, const int32_t* key_vars, uint32_t nkey, uint32_t nparts,
                  das_table_t** out, uint64_t* counts) {
  return guarded(ctx, [&] { *out = wrap(das::partition(ctx->c, t->t, key_vars, nkey, nparts, counts)); });
}

int das_table_gather(das_ctx_t* ctx, const das_table_t* t, const uint32_t* idx, uint64_t n, das_table_t** out) {
  return guarded(ctx, [&] {
    for (uint64_t i = 0; i < n; ++i) DAS_CHECK(idx[i] < t->t.nrows, das::DAS_E_INVALID, "gather index out of range");
    das::DBuf<uint32_t> d(n ? n : 1, ctx->c.s);
    if (n) DAS_HIP(hipMemcpyAsync(d.p, idx, 4 * n, hipMemcpyHostToDevice, ctx->c.s));
    *out = wrap(das::gather_table(ctx->c, t->t, d.p, n));
    DAS_HIP(hipStreamSynchronize(ctx->c.s));      // `idx` is caller memory
  });
}

int das_table_gather_ranges(das_ctx_t* ctx, const das_table_t* t, const uint64_t* begin, const uint64_t* end,
                            uint32_t n_ranges, das_table_t** out) {
  if (!ctx || !t || !out || (n_ranges && (!begin || !end))) return fail(ctx, DAS_ERR_INVALID, "null argument");
  return guarded(ctx, [&] { *out = wrap(das::gather_ranges(ctx->c, t->t, begin, end, n_ranges)); });
}

int das_table_export_rows(das_ctx_t* ctx, const das_table_t* t, uint32_t* d_dst) {
  return guarded(ctx, [&] { das::export_rows(ctx->c, t->t, d_dst); });
}

int das_table_import_rows(das_ctx_t* ctx, int32_t kind, int32_t ncols, const int32_t* vars, const int32_t* member,
                          const uint32_t* d_src, uint64_t nrows, das_table_t** out) {
  return guarded(ctx, [&] {
    check_schema(kind, ncols, vars, member);
    *out = wrap(das::import_rows(ctx->c, kind, ncols, vars, member, d_src, nrows));
  });
}

int das_table_set_bounds(das_table_t* t, const uint32_t* lo, const uint32_t* hi) {
  if (!t) return fail(nullptr, DAS_ERR_INVALID, "null table");
  for (int c = 0; c < t->t.ncols; ++c) {
    t->t.lo[c] = lo ? lo[c] : 0u;
    t->t.hi[c] = hi ? hi[c] : 0xFFFFFFFFu;
  }
  return DAS_OK;
}

int das_set_pattern_black_list(das_ctx_t* ctx, const uint32_t* type_digests, uint32_t n) {
  return guarded(ctx, [&] {
    DAS_CHECK(n == 0 || type_digests, das::DAS_E_INVALID, "null digests");
    ctx->c.black_list.assign(reinterpret_cast<const das::Digest*>(type_digests),
                             reinterpret_cast<const das::Digest*>(type_digests) + n);
  });
}

int das_table_checksum(das_ctx_t* ctx, const das_table_t* t, const uint64_t* salt, uint64_t out[2]) {
  return guarded(ctx, [&] {
    DAS_CHECK(t && salt && out, das::DAS_E_INVALID, "null argument");
    das::table_checksum(ctx->c, t->t, salt, out);
  });
}

int das_box_store_bw(das_ctx_t* ctx, uint64_t bytes, uint32_t reps, double* gbps) {
  return guarded(ctx, [&] {
    DAS_CHECK(gbps, das::DAS_E_INVALID, "null argument");
    *gbps = das::box_store_bw(ctx->c, bytes, reps);
  });
}

int das_prof_mark(das_ctx_t* ctx, uint32_t id) {
  return guarded(ctx, [&] { das::prof_mark(ctx->c, id); });
}

int das_table_get_bounds(const das_table_t* t, uint32_t* lo, uint32_t* hi) {
  if (!t || !lo || !hi) return fail(nullptr, DAS_ERR_INVALID, "null argument");
  for (int c = 0; c < t->t.ncols; ++c) {
    lo[c] = t->t.lo[c];
    hi[c] = t->t.hi[c];
  }
  return DAS_OK;
}

int das_table_members(const das_table_t* t, int32_t* member) {
  if (!t) return fail(nullptr, DAS_ERR_INVALID, "null table");
  for (int c = 0; c < t->t.ncols; ++c) member[c] = t->t.kind == DAS_TABLE_COMPOSITE ? t->t.member[c]
                                                 : t->t.kind == DAS_TABLE_UNORDERED ? 0 : -1;
  return DAS_OK;
}

int das_set_dedup(das_ctx_t* ctx, const das_table_t* const* ts, uint32_t n, das_table_t** out) {
  return guarded(ctx, [&] {
    std::vector<const Table*> v(n);
    for (uint32_t i = 0; i < n; ++i) v[i] = &ts[i]->t;
    auto r = das::set_dedup(ctx->c, v.data(), (int)n);
    for (uint32_t i = 0; i < n; ++i) out[i] = wrap(std::move(r[i]));
  });
}

int das_set_minus(das_ctx_t* ctx, const das_table_t* const* a, uint32_t na, const das_table_t* const* b, uint32_t nb,
                  das_table_t** out) {
  return guarded(ctx, [&] {
    std::vector<const Table*> va(na), vb(nb);
    for (uint32_t i = 0; i < na; ++i) va[i] = &a[i]->t;
    for (uint32_t i = 0; i < nb; ++i) vb[i] = &b[i]->t;
    auto r = das::set_minus(ctx->c, va.data(), (int)na, vb.data(), (int)nb);
    for (uint32_t i = 0; i < na; ++i) out[i] = wrap(std::move(r[i]));
  });
}

int das_plan_execute_info(das_ctx_t* ctx, const das_plan_node_t* nodes, uint32_t n, uint32_t no_overload,
                          das_table_t** out, uint32_t cap, uint32_t* n_out, int32_t* matched, int32_t* negation,
                          int64_t* info) {
  if (!ctx || !nodes || !n_out || !matched || !negation || (cap && !out)) return fail(ctx, DAS_ERR_INVALID, "null argument");
  return guarded(ctx, [&] {
    auto r = das::plan_execute(ctx->c, nodes, n, (int)no_overload);
    *n_out = (uint32_t)r.tables.size();     // on overflow: the capacity the caller needs
    DAS_CHECK(r.tables.size() <= cap, das::DAS_E_INVALID, "plan: more answer tables than `cap`");
    for (size_t i = 0; i < r.tables.size(); ++i) {
      if (info) {
        // what das_table_info reports (das_plan_execute_many's layout)
        int64_t* f = info + 20 * i;
        const auto& t = *r.tables[i];
        f[0] = t.kind;
        f[1] = t.ncols;
        f[2] = (int64_t)t.nrows;
        f[3] = 0;
        for (int k = 0; k < 16; ++k) f[4 + k] = k < t.ncols ? t.vars[k] : 0;
      }
      out[i] = wrap(std::move(r.tables[i]));
    }
    *matched = r.matched ? 1 : 0;
    *negation = r.negation ? 1 : 0;
  });
}

int das_plan_execute(das_ctx_t* ctx, const das_plan_node_t* nodes, uint32_t n, uint32_t no_overload,
                     das_table_t** out, uint32_t cap, uint32_t* n_out, int32_t* matched, int32_t* negation) {
  return das_plan_execute_info(ctx, nodes, n, no_overload, out, cap, n_out, matched, negation, nullptr);
}

int das_plan_execute_many(das_ctx_t* ctx, uint32_t n_plans, const das_plan_node_t* const* nodes, const uint32_t* n,
                          uint32_t no_overload, das_table_t** out, uint32_t cap, uint32_t* n_out, int32_t* matched,
                          int32_t* negation, int64_t* info) {
  if (!ctx || (n_plans && (!nodes || !n || !n_out || !matched || !negation)) || (cap && !out))
    return fail(ctx, DAS_ERR_INVALID, "null argument");
  return guarded(ctx, [&] {
    auto rs = das::plan_execute_many(ctx->c, nodes, n, n_plans, (int)no_overload);
    uint64_t total = 0;
    for (auto& r : rs) total += r.tables.size();
    for (uint32_t i = 0; i < n_plans; ++i) n_out[i] = (uint32_t)rs[i].tables.size();
    // on overflow every answer is dropped; n_out says the room each needs
    DAS_CHECK(total <= cap, das::DAS_E_INVALID, "plans: more answer tables than `cap`");
    uint64_t k = 0;
    for (uint32_t i = 0; i < n_plans; ++i) {
      for (auto& t : rs[i].tables) {
        if (info) {
          // what das_table_info reports, so the caller needs no call per table
          int64_t* f = info + 20 * k;
          f[0] = t->kind;
          f[1] = t->ncols;
          f[2] = (int64_t)t->nrows;
          f[3] = 0;
          for (int c = 0; c < 16; ++c) f[4 + c] = c < t->ncols ? t->vars[c] : 0;
        }
        out[k++] = wrap(std::move(t));
      }
      matched[i] = rs[i].matched ? 1 : 0;
      negation[i] = rs[i].negation ? 1 : 0;
    }
  });
}

int das_plan_execute_sharded(das_ctx_t* ctx, const das_plan_node_t* nodes, uint32_t n, uint32_t no_overload,
                             const das_table_t* const* inputs, uint32_t n_inputs, das_table_t** out, uint32_t cap,
                             uint32_t* n_out, int32_t* matched, int32_t* negation, uint8_t* checks,
                             uint32_t checks_cap, uint32_t* n_checks) {
  if (!ctx || !nodes || !n_out || !matched || !negation || !n_checks || (n_inputs && !inputs))
    return fail(ctx, DAS_ERR_INVALID, "null argument");
  return guarded(ctx, [&] {
    std::vector<const das::Table*> in(n_inputs);
    for (uint32_t i = 0; i < n_inputs; ++i) in[i] = inputs[i] ? &inputs[i]->t : nullptr;
    std::vector<uint8_t> ck;
    auto r = das::plan_execute_sharded(ctx->c, nodes, n, (int)no_overload, in, ck);
    *n_out = (uint32_t)r.tables.size();
    *n_checks = (uint32_t)ck.size();
    DAS_CHECK(r.tables.size() <= cap && ck.size() <= checks_cap, das::DAS_E_INVALID,
              "plan: more answer tables or checks than their capacity");
    for (size_t i = 0; i < r.tables.size(); ++i) out[i] = wrap(std::move(r.tables[i]));
    for (size_t i = 0; i < ck.size(); ++i) checks[i] = ck[i];
    *matched = r.matched ? 1 : 0;
    *negation = r.negation ? 1 : 0;
  });
}

int das_plan_estimates(das_ctx_t* ctx, const das_plan_node_t* nodes, uint32_t n, uint64_t* rows) {
  if (!ctx || (n && (!nodes || !rows))) return fail(ctx, DAS_ERR_INVALID, "null argument");
  return guarded(ctx, [&] {
    DAS_CHECK(ctx->c.idx.built, das::DAS_E_NOT_BUILT, "index not built");
    const das::Index& idx = ctx->c.idx;
    for (uint32_t i = 0; i < n; ++i) {
      const das_plan_node_t& x = nodes[i];
      if (x.op == DAS_PLAN_LINK || x.op == DAS_PLAN_INPUT)
        rows[i] = das::scan_estimate(ctx->c, x.scan);
      else if (x.op == DAS_PLAN_TEMPLATE && x.scan.type_id < idx.ctype_range.size())
        rows[i] = idx.ctype_range[x.scan.type_id].end - idx.ctype_range[x.scan.type_id].begin;
      else
        rows[i] = 0;
    }
  });
}

int das_plan_bounds(das_ctx_t* ctx, const das_plan_node_t* nodes, uint32_t n, uint64_t* rows) {
  if (!ctx || (n && (!nodes || !rows))) return fail(ctx, DAS_ERR_INVALID, "null argument");
  return guarded(ctx, [&] {
    DAS_CHECK(ctx->c.idx.built, das::DAS_E_NOT_BUILT, "index not built");
    const das::Index& idx = ctx->c.idx;
    for (uint32_t i = 0; i < n; ++i) {
      const das_plan_node_t& x = nodes[i];
      if (x.op == DAS_PLAN_LINK || x.op == DAS_PLAN_INPUT)
        rows[i] = das::scan_bound(ctx->c, x.scan);
      else if (x.op == DAS_PLAN_TEMPLATE && x.scan.type_id < idx.ctype_range.size())
        rows[i] = idx.ctype_range[x.scan.type_id].end - idx.ctype_range[x.scan.type_id].begin;
      else
        rows[i] = 0;
    }
  });
}

int das_prof_enable(das_ctx_t* ctx, int on) {
  return guarded(ctx, [&] {
    das::prof_collect(ctx->c);
    ctx->c.prof = on != 0;
  });
}

int das_prof_only(das_ctx_t* ctx, const char* name) {
  return guarded(ctx, [&] {
    das::prof_collect(ctx->c);
    ctx->c.prof_only = name ? name : "";
  });
}

int das_prof_tag(das_ctx_t* ctx, const char* tag) {
  return guarded(ctx, [&] { ctx->c.prof_tag = tag ? tag : ""; });
}

int das_prof_tag_plan(das_ctx_t* ctx, uint32_t plan, const char* tag) {
  return guarded(ctx, [&] {
    ctx->c.tag_plan = tag && tag[0] ? plan : ~0u;
    ctx->c.tag_plan_name = tag ? tag : "";
  });
}

int das_prof_reset(das_ctx_t* ctx) {
  return guarded(ctx, [&] {
    das::prof_collect(ctx->c);
    ctx->c.kstats.clear();
  });
}

int das_prof_read(das_ctx_t* ctx, const char* name, double* ms, uint64_t* launches, double* bytes) {
  return guarded(ctx, [&] {
    das::prof_collect(ctx->c);
    auto it = ctx->c.kstats.find(name);
    das::KStat z;
    const das::KStat& k = it == ctx->c.kstats.end() ? z : it->second;
    *ms = k.ms;
    *launches = k.launches;
    *bytes = k.bytes;
  });
}

int das_prof_names(das_ctx_t* ctx, char* buf, uint64_t cap) {
  return guarded(ctx, [&] {
    das::prof_collect(ctx->c);
    std::string all;
    for (auto& kv : ctx->c.kstats) all += kv.first + "\n";
    DAS_CHECK(all.size() + 1 <= cap, das::DAS_E_INVALID, "buffer too small");
    std::memcpy(buf, all.c_str(), all.size() + 1);
  });
}

}  // extern "C"

namespace das {
Ctx*& active_ctx() {
  thread_local Ctx* c = nullptr;
  return c;
}

namespace {
std::atomic<uint64_t> g_launches{0}, g_readbacks{0};
}  // namespace
void count_launch() { g_launches.fetch_add(1, std::memory_order_relaxed); }
void count_readback() { g_readbacks.fetch_add(1, std::memory_order_relaxed); }
void read_counters(uint64_t out[2]) {
  out[0] = g_launches.load(std::memory_order_relaxed);
  out[1] = g_readbacks.load(std::memory_order_relaxed);
}

void launch_gate(Ctx& c, double algorithmic_bytes) {
  if (!c.gate_s || algorithmic_bytes < c.gate_min) return;
  hipEvent_t e = c.fence_event(2 * kPubPool + 3);
  DAS_HIP(hipEventRecord(e, c.gate_s));
  DAS_HIP(hipStreamWaitEvent(c.s, e, 0));
  c.gate_s = nullptr;                                  // once per nested plan
}

KScope::KScope(const char* name, double algorithmic_bytes) {
  Ctx* c = active_ctx();
  if (c && c->gate_s) launch_gate(*c, algorithmic_bytes);
  if (c && c->prof) {
    impl = new ProfScope(*c, name, algorithmic_bytes);      // (counts the launch)
  } else {
    count_launch();
    if (trace_on()) trace_mark("kernel", std::string(name) + " " + std::to_string((uint64_t)algorithmic_bytes) + " B");
  }
}

namespace {
struct TraceEv {
  const char* what;
  std::string name;
  double us;
};
thread_local std::vector<TraceEv> t_trace;
double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

bool trace_on() {
  static const bool on = std::getenv("DAS_TRACE") != nullptr;
  return on;
}
void trace_mark(const char* what, const std::string& name) {
  if (trace_on()) t_trace.push_back({what, name, now_us()});
}
void trace_dump(const char* title) {
  if (!trace_on() || t_trace.empty()) return;
  const double t0 = t_trace.front().us;
  std::fprintf(stderr, "[trace] %s\n", title);
  for (auto& e : t_trace) std::fprintf(stderr, "[trace] %9.1f %s %s\n", e.us - t0, e.what, e.name.c_str());
  t_trace.clear();
}
KScope::~KScope() { delete static_cast<ProfScope*>(impl); }

void prof_add_bytes(Ctx& c, const std::string& name, double bytes) {
  const std::string tagged = c.prof_tag.empty() ? name : name + "@" + c.prof_tag;
  for (auto it = c.pending.rbegin(); it != c.pending.rend(); ++it)
    if (it->name == tagged) {
      it->bytes += bytes;
      return;
    }
}

void prof_collect(Ctx& c) {
  if (c.pending.empty()) return;
  DAS_HIP(hipStreamSynchronize(c.s));
  for (auto& p : c.pending) {
    float ms = 0;
    DAS_HIP(hipEventElapsedTime(&ms, p.a, p.b));
    KStat& k = c.kstats[p.name];
    k.ms += ms;
    k.bytes += p.bytes;
    k.launches += 1;
    c.ev_pool.push_back(p.a);
    c.ev_pool.push_back(p.b);
  }
  c.pending.clear();
}
}  // namespace das
