// Internal types of the DAS MI355X library: the HBM-resident atom index and
// device binding tables.  Layout rationale is in DESIGN.md §3.
#pragma once
#include <array>
#include <map>
#include <unordered_map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/das_mi355x.h"
#include "common.h"
#include "prims.h"

namespace das {

constexpr int kMaxArity = 8;      // index tables exist for arity 1..kMaxArity
constexpr int kMaxPosArity = 3;   // per-position (pattern) index: arity 1..3, as the reference
constexpr int kMaxCols = 16;      // columns in a binding table
constexpr int kTypeBits = 24;     // named types < 2^24 (P-index key = type << 32 | target)

// External category codes (das_lookup): a remote link is an atom of the global
// id space whose index rows live on another shard (multi-GPU).
enum AtomCat : uint8_t { CAT_OTHER = 0, CAT_NODE = 1, CAT_LINK = 2, CAT_LINK_REMOTE = 3 };
// Priority when several loader entries share a digest (a local link wins).
enum CatPrio : uint8_t { PRIO_OTHER = 0, PRIO_NODE = 1, PRIO_REMOTE = 2, PRIO_LINK = 3 };
__host__ __device__ inline uint8_t cat_of_prio(uint32_t p) {
  return p == PRIO_LINK ? CAT_LINK : p == PRIO_REMOTE ? CAT_LINK_REMOTE : p == PRIO_NODE ? CAT_NODE : CAT_OTHER;
}

// Rows (link id, t0 .. t_{a-1}) stored column-major: column c at data + c*rows.
struct RowTable {
  int arity = 0;
  uint64_t rows = 0;
  uint64_t ld = 0;                 // column stride: rows rounded up to 64 (16-byte aligned columns)
  uint32_t* data = nullptr;
  uint32_t* col(int c) const { return data + (uint64_t)c * ld; }
};
inline uint64_t col_stride(uint64_t rows) { return (rows + 63) & ~63ull; }

// P_{a,p}: RowTable sorted by (type, t_p, the other targets in position
// order, link id) + unique (type, t_p) keys -> row offsets.
struct PosIndex {
  RowTable t;
  uint64_t nkeys = 0;
  uint64_t* ukey = nullptr;   // sorted unique (type << 32 | t_p)
  uint64_t* uoff = nullptr;   // nkeys + 1 row offsets
  // Dense key directory per type (index joins): dir[ty][t - dir_lo[ty]] =
  // the index of key (ty, t) in ukey, or kNone; built where the type's t_p
  // span is at most 2x its key count, or 16x up to 2^28 ids.
  std::vector<uint32_t*> dir;
  std::vector<uint32_t> dir_lo, dir_n;
  // Otherwise a bucket directory: bucket b = (t - dir_lo) >> bshift holds
  // the keys ukey[bdir[ty][b] .. bdir[ty][b + 1]) (~2 per bucket), searched
  // in place of the whole type's keys (index joins of sparse key ranges).
  std::vector<uint32_t*> bdir;
  std::vector<uint32_t> bshift, bn;
  // Rank directory (in place of a dense one over >= 2^20 ids): one bit per
  // id of the span (rbits, 64-bit words) and each word's count of earlier
  // set bits (rpre); key (ty, t) is ukey[rklo + rpre[w] + popc(bits below
  // t's bit)] -- 1.5 bits per id instead of 32, so a probe's directory lines
  // are shared with its neighbours and the directory stays MALL-resident.
  std::vector<uint64_t*> rbits;
  std::vector<uint32_t*> rpre;
  std::vector<uint64_t> rklo;
  // host mirror of ukey / uoff (nkeys <= kHostKeyMirror), else empty
  std::vector<uint64_t> h_ukey, h_uoff;
};
constexpr uint64_t kHostKeyMirror = 1ull << 24;   // keys per P_{a,p} mirrored on the host (256 MB at most)
// the mirror's key limit for the next build: kHostKeyMirror, or
// DAS_HOST_KEY_MIRROR (tests: 0 = no mirror, every anchored key range is
// resolved on the device through a read-back)
uint64_t host_key_mirror_max();
constexpr uint64_t kHostNodeMirror = 1ull << 24;  // nodes mirrored on the host (384 MB at most)

struct CtypeRange {
  uint32_t arity;
  uint64_t begin, end;        // rows of ctab[arity]
};

struct Index {
  bool built = false;
  hipStream_t stream = nullptr;  // stream the index arrays were allocated on (caching allocator)
  uint64_t n_atoms = 0, n_nodes = 0, n_links = 0, n_types = 0;
  Digest* digest = nullptr;    // [n_atoms] by id (ids clustered by named type)
  uint32_t* by_digest = nullptr; // [n_atoms] ids in handle (digest) order
  uint8_t* cat = nullptr;      // [n_atoms]
  uint32_t* type = nullptr;    // [n_atoms] named type id (kNone for CAT_OTHER)
  uint32_t* arity = nullptr;   // [n_atoms]
  uint64_t* tgt_off = nullptr; // [n_atoms + 1]
  uint32_t* in_off = nullptr;  // [n_atoms + 1] incoming CSR offsets
  uint32_t* in_link = nullptr; // [in_total] links containing each atom, by (target, link id)
  uint64_t in_total = 0;
  uint32_t* tgt = nullptr;     // [sum arity]
  uint32_t* ctype = nullptr;   // [n_atoms] composite-type id of links, kNone otherwise
  uint32_t* name_leaf = nullptr; // [n_atoms] loader leaf index of nodes (kNone otherwise)
  // T_a: links of arity a sorted by (type, id);   C_a: by (ctype, id)
  std::array<RowTable, kMaxArity + 1> ttab{};
  std::array<RowTable, kMaxArity + 1> ctab{};
  std::array<std::array<PosIndex, kMaxPosArity>, kMaxPosArity + 1> pidx{};
  std::array<std::vector<uint64_t>, kMaxArity + 1> type_off;   // host: n_types + 1 per arity
  // host: id bounds of T_a column c over links of named type t, at
  // [(t * (a + 1) + c) * 2 + {0: min, 1: max}]; gbound: same over all types.
  // Ids are clustered by named type, so a variable bound at a position of a
  // typed link has a tight id range (direct-address joins size their
  // offsets array from it without a device round trip).
  std::array<std::vector<uint32_t>, kMaxArity + 1> tbound, gbound;
  std::vector<Digest> ctype_digest;                            // host: sorted ctype digests
  std::vector<Digest> type_digest;                             // host: md5(type name) per named type
  // host: 1 = the named type is in the pattern black list the build was
  // given (its links get no pattern keys, canonical_parser.py:144 /
  // parser_threads.py:185; template keys are kept)
  std::vector<uint8_t> no_pattern;
  bool no_pattern_any = false;
  bool blocked(uint32_t ty) const { return ty < no_pattern.size() && no_pattern[ty]; }
  std::vector<uint32_t> type_name_len;                         // host: bytes of each type name
  std::vector<CtypeRange> ctype_range;                         // host
  // host mirror of the nodes in handle order (n_nodes <= kHostNodeMirror):
  // digest, id and named type -- an anchored query resolves its grounded
  // nodes without a device round trip
  std::vector<Digest> h_node_dig;
  std::vector<uint32_t> h_node_id, h_node_type;
  std::vector<void*> owned;                                    // device allocations
  std::map<std::array<uint64_t, 4>, std::pair<uint64_t, uint64_t>> range_cache;   // P lookups
  uint64_t device_bytes = 0;
};

struct Table {
  int kind = DAS_TABLE_ORDERED;
  int ncols = 0;
  int sorted_col = -1;              // rows ascending by this column (-1: no known order)
  int32_t vars[kMaxCols] = {0};
  int32_t member[kMaxCols] = {0};   // DAS_TABLE_COMPOSITE: -1 ordered column, else member index
  // host-known value bounds per column (inclusive); [0, kNone] = unknown
  uint32_t lo[kMaxCols] = {0};
  uint32_t hi[kMaxCols] = {kNone, kNone, kNone, kNone, kNone, kNone, kNone, kNone,
                           kNone, kNone, kNone, kNone, kNone, kNone, kNone, kNone};
  uint64_t nrows = 0, cap = 0;
  uint32_t* data = nullptr;   // ncols columns of `cap` u32 each
  hipStream_t s = nullptr;
  bool view = false;          // data points into an index table (not owned; plan-internal only)
  uint32_t* col(int c) const { return data + (uint64_t)c * cap; }
  ~Table() {
    if (data && !view) cache_free(data);
  }
};

// Per-kernel timing with HIP events on the ctx stream (das_prof_*): what
// bench.py's roofline figures are computed from.
struct KStat {
  double ms = 0, bytes = 0;
  uint64_t launches = 0;
};
struct PendingEv {
  std::string name;
  hipEvent_t a, b;
  double bytes;
};

struct Ctx {
  bool prof = false;
  // while a plan evaluates (das_plan_execute): a predicate-free scan whose
  // columns are consecutive index columns returns a view of them instead of
  // a copy (2: scans up to kViewRows rows, 1: all, 0: none); views are
  // materialised before a table leaves the plan
  int scan_views = 0;
  std::string prof_only;             // non-empty: only scopes of these names ('|'-separated) record events
  std::string prof_tag;              // non-empty: recorded scopes are named "<scope>@<tag>" (one query's launches)
  uint32_t tag_plan = ~0u;           // das_plan_execute_many: the plan whose launches carry tag_plan_name
  std::string tag_plan_name;
  // a plan nested in another's read-back wait (das_plan_execute_many): its
  // first kernel of >= gate_min algorithmic bytes waits for the work launched
  // on gate_s (the outer plan's stream) so far -- latency-bound stages
  // overlap, two HBM-bound floods do not (launch_gate)
  hipStream_t gate_s = nullptr;
  double gate_min = 0;
  bool prof_selected(const std::string& name) const {
    if (prof_only.empty()) return true;
    size_t b = 0;
    while (b <= prof_only.size()) {
      size_t e = prof_only.find('|', b);
      if (e == std::string::npos) e = prof_only.size();
      if (prof_only.compare(b, e - b, name) == 0) return true;
      b = e + 1;
    }
    return false;
  }
  std::vector<PendingEv> pending;
  std::vector<hipEvent_t> ev_pool;   // recycled timing events (creation is not cheap on ROCm)
  // timing only: no system-scope fence when the event is recorded -- a default
  // event writes back and invalidates the caches there, which the next
  // kernels pay for (DAS_PROF_FENCE=1: default events, A/B)
  hipEvent_t take_event() {
    if (ev_pool.empty()) {
      hipEvent_t e;
      const char* f = std::getenv("DAS_PROF_FENCE");
      if (f && f[0] == '1') DAS_HIP(hipEventCreate(&e));
      else DAS_HIP(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
      return e;
    }
    hipEvent_t e = ev_pool.back();
    ev_pool.pop_back();
    return e;
  }
  std::map<std::string, KStat> kstats;
  int device = 0;
  hipStream_t s = nullptr;
  bool own_stream = false;
  std::string err;
  std::mutex mu;
  Index idx;
  HostScalar scratch;
  // (lo, cnt) descriptor array of the sparse direct-join build, all-zero
  // between joins (direct_join clears the slots it wrote)
  DBuf<uint2> zlc;
  // pattern black list for the next index build: md5 of each type name
  std::vector<Digest> black_list;
  // side streams for fused chains in flight together (das_plan_execute_many),
  // each with two fence events per pooled run (created on first use)
  static constexpr int kSide = 4;                     // 0..2: chains; 3: the batch's other plans
  static constexpr int kChainSides = 3, kPlanSide = 3;
  hipStream_t side[kSide] = {};
  DBuf<uint2> zlc_side[kSide];                        // the sparse-join scratch of each side stream
  DBuf<uint2>& zlc_of(hipStream_t st) {
    for (int i = 0; i < kSide; ++i)
      if (side[i] && st == side[i]) return zlc_side[i];
    return zlc;
  }
  // algorithmic bytes launched per query shape in its last batch (the batch's
  // order: the heaviest plan first, on the context's stream)
  std::unordered_map<uint64_t, double> plan_bytes;
  std::vector<hipEvent_t> side_ev;
  hipStream_t side_stream(int i) {
    if (!side[i]) {
      // the batch's other plans (kPlanSide) run beside the lead plan's long
      // kernels: their queue gets the highest dispatch priority
      // (DAS_PLAN_PRIO=0: default priority, A/B)
      // (DAS_CHAIN_PRIO=1: the chains' side streams too, A/B)
      int lo = 0, hi = 0;
      const char* pp = std::getenv("DAS_PLAN_PRIO");
      const char* cp = std::getenv("DAS_CHAIN_PRIO");
      const bool high = i == kPlanSide ? !(pp && pp[0] == '0') : (cp && cp[0] == '1');
      if (high && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess)
        DAS_HIP(hipStreamCreateWithPriority(&side[i], hipStreamNonBlocking, hi));
      else
        DAS_HIP(hipStreamCreateWithFlags(&side[i], hipStreamNonBlocking));
    }
    return side[i];
  }
  // zeroed grid-chain counter blocks, one per pooled chain of a batch (the
  // grid kernel leaves its block zero again)
  static constexpr uint32_t kGscBlock = 64;               // words per block (>= the kernel's kGscWords)
  uint32_t* gsc_pool = nullptr;
  // blocks 0 .. kPubPool-1: a batch's pooled chains; kPubPool + level: the
  // one-at-a-time chain of each read-back level (fused_and)
  static constexpr uint32_t kGscBlocks = 18;
  uint32_t* gsc_block(uint32_t k) {
    if (!gsc_pool) {
      DAS_HIP(hipMalloc((void**)&gsc_pool, 4ull * kGscBlock * kGscBlocks));
      DAS_HIP(hipMemset(gsc_pool, 0, 4ull * kGscBlock * kGscBlocks));
    }
    return gsc_pool + (uint64_t)kGscBlock * (k % kGscBlocks);
  }
  hipEvent_t fence_event(uint32_t i) {
    while (side_ev.size() <= i) {
      hipEvent_t e;
      DAS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      side_ev.push_back(e);
    }
    return side_ev[i];
  }
  // loader-side host copies kept for metadata calls
  std::vector<uint8_t> leaf_bytes;
  std::vector<uint64_t> leaf_off;
};

// Scope names are the kernel's name as rocprofv3 reports it, shortened the
// way tools/pmc_traffic.py shortens it (namespaces dropped, integer template
// arguments kept, unsigned int/long -> u32/u64), e.g. "k_dj_write<2,1,u32>",
// so every launch size and time pairs with its rocprof row.
// Host timeline (DAS_TRACE=1, tools): marks on a monotonic microsecond clock
// -- kernel scopes, read-back waits, plan nodes -- printed to stderr by
// das_plan_execute.
bool trace_on();
void trace_mark(const char* what, const std::string& name = std::string());
// process-wide counts of kernel scopes entered and of host read-backs waited
// on (das_counters; bench.py reports them per query for latency-bound legs)
void count_launch();
// algorithmic bytes of the kernel scopes this thread entered (a plan's
// weight, das_plan_execute_many)
inline double& launched_bytes() {
  thread_local double b = 0;
  return b;
}
void count_readback();
void read_counters(uint64_t out[2]);
void trace_dump(const char* title);

void launch_gate(Ctx& c, double algorithmic_bytes);
struct ProfScope {
  Ctx& c;
  std::string name;
  double bytes;
  hipEvent_t a = nullptr, b = nullptr;
  ProfScope(Ctx& ctx, std::string n, double algorithmic_bytes) : c(ctx), name(std::move(n)), bytes(algorithmic_bytes) {
    if (c.gate_s) launch_gate(c, algorithmic_bytes);
    count_launch();
    launched_bytes() += algorithmic_bytes;
    if (trace_on()) trace_mark("kernel", name + " " + std::to_string((uint64_t)algorithmic_bytes) + " B");
    if (!c.prof || !c.prof_selected(name)) return;
    if (!c.prof_tag.empty()) name += "@" + c.prof_tag;
    a = c.take_event();
    b = c.take_event();
    DAS_HIP(hipEventRecord(a, c.s));
  }
  ~ProfScope() {
    if (!c.prof || !a) return;
    (void)hipEventRecord(b, c.s);
    c.pending.push_back(PendingEv{name, a, b, bytes});
  }
};
void prof_collect(Ctx& c);
// Adds algorithmic bytes to the latest recorded launch of scope `name` (bytes
// known only after the kernel: e.g. the outputs a filter kept).
void prof_add_bytes(Ctx& c, const std::string& name, double bytes);
// The context whose C-ABI call runs on this thread (KScope's target).
Ctx*& active_ctx();

// hash.hip
void hash_strings(const uint8_t* bytes, const uint64_t* off, uint64_t n, DigS out, hipStream_t s);
void hash_group(DigS table, DigS ctab, const uint32_t* child, const uint64_t* child_off,
                const int32_t* ctype_leaf, uint64_t n_leaf, uint64_t begin, uint64_t n, uint32_t K,
                hipStream_t s, uint32_t* etype = nullptr);   // etype: each expression's type leaf (nullable)
void hash_fixed(const Digest* elems, uint32_t k, uint64_t n, Digest* out, hipStream_t s);

// index.hip
// shard_rank / shard_world > 1: a link (expr kind 1 or 3) gets pattern-index
// rows iff handle_owner(its digest, world) == rank, else it is directory-only
// (links hash-partitioned by handle); world 1: kinds as given.
void build_index(Ctx& c, const das_atoms_t& a, uint32_t flags, uint32_t shard_rank = 0, uint32_t shard_world = 1);
// Owning shard of every expression's handle (hashes leaves and expressions as
// the build does, step 1); d_owner: n_expr device bytes.
void hash_owners(Ctx& c, const das_atoms_t& a, uint32_t flags, uint32_t world, uint8_t* d_owner);
// Rows (K u32 each) regrouped by owner, stable inside an owner; counts[world].
void partition_rows(Ctx& c, const uint32_t* d_rows, uint64_t n, uint32_t K, const uint8_t* d_owner, uint32_t world,
                    uint32_t* d_out, uint64_t* counts);
void numbered_strings(const char* prefix, uint64_t plen, uint64_t first, uint64_t n, uint8_t* out, uint64_t* off);
void synth_powerlaw_links(uint32_t* d_child, uint64_t first, uint64_t n, uint32_t K, uint32_t n_link_types,
                          uint32_t type_leaf0, uint32_t node_leaf0, uint64_t n_nodes, double s, uint64_t seed,
                          hipStream_t st);
void free_index(Index& idx);
void lookup_digests(Ctx& c, const Digest* h_digests, uint64_t n, int64_t* h_ids);
// ids + category / arity / type of up to 4096 handles in one pinned round
// trip (false: batch too large, use lookup_digests + das_atoms_info)
bool lookup_small(Ctx& c, const Digest* h_digests, uint64_t n, int64_t* h_ids, uint8_t* cat, uint32_t* arity,
                  uint32_t* type);

// Column pointers of a table (kernel argument by value).
struct ColSet {
  const uint32_t* c[kMaxCols];
  int n;
};

// query.hip
ColSet cols_of(const Table& t);
void sort_perm(const ColSet& cs, uint64_t n, uint32_t* perm, int bits, hipStream_t s);
int id_bits(const Ctx& c);
std::unique_ptr<Table> gather_table(Ctx& c, const Table& a, const uint32_t* idx, uint64_t m);
// rows [begin[i], end[i]) of `a` for every range i, in range order (host arrays)
std::unique_ptr<Table> gather_ranges(Ctx& c, const Table& a, const uint64_t* begin, const uint64_t* end,
                                     uint32_t n_ranges);
std::unique_ptr<Table> compact_table(Ctx& c, const Table& a, const uint32_t* keep);
// lo/cnt per probe row: the equal range of its key in the sorted build keys
void join_ranges(Ctx& c, const ColSet& probe, uint64_t np, const ColSet& build_sorted, uint64_t nb, uint32_t* lo,
                 uint32_t* cnt);
std::unique_ptr<Table> scan_link(Ctx& c, const das_link_scan_t& q);
std::unique_ptr<Table> scan_template(Ctx& c, const das_template_scan_t& q);
std::unique_ptr<Table> join(Ctx& c, const Table& a, const Table& b, int flags);
// rows of p whose value of the one shared variable lies in EVERY qs[i]'s key
// set (each qs[i] one column, distinct keys); nullptr when not applicable
std::unique_ptr<Table> semi_join_multi(Ctx& c, const Table& p, const std::vector<const Table*>& qs);
// index_join(a, q) restricted to the rows whose fresh variable fvar lies in
// every qs[i]'s key set, filtered during the expansion; nullptr: not applicable
std::unique_ptr<Table> index_join_filtered(Ctx& c, const Table& a, const das_link_scan_t& q, int32_t fvar,
                                           const std::vector<const Table*>& qs);
std::unique_ptr<Table> index_join(Ctx& c, const Table& a, const das_link_scan_t& q);   // nullptr: not applicable
// rows of a whose link (q's grounded targets + a's values of q's variables)
// does not exist; nullptr when a does not bind every variable position
std::unique_ptr<Table> anti_index_join(Ctx& c, const Table& a, const das_link_scan_t& q);
std::unique_ptr<Table> antijoin(Ctx& c, const Table& a, const Table& t);
std::unique_ptr<Table> dedup(Ctx& c, const Table& a);
std::unique_ptr<Table> concat(Ctx& c, const Table* const* ts, int n);
std::unique_ptr<Table> new_table(Ctx& c, int kind, int ncols, const int32_t* vars, uint64_t cap,
                                 const int32_t* member = nullptr);
// Same schema and column bounds as `a` (a subset of its rows will be stored).
inline std::unique_ptr<Table> new_table_like(Ctx& c, const Table& a, uint64_t cap) {
  auto t = new_table(c, a.kind, a.ncols, a.vars, cap, a.member);
  t->sorted_col = a.sorted_col;
  for (int k = 0; k < a.ncols; ++k) {
    t->lo[k] = a.lo[k];
    t->hi[k] = a.hi[k];
  }
  return t;
}
std::unique_ptr<Table> partition(Ctx& c, const Table& t, const int32_t* key_vars, uint32_t nkey, uint32_t nparts,
                                 uint64_t* counts);
void export_rows(Ctx& c, const Table& t, uint32_t* dst);
// Order-independent checksum of an ordered table (checksum.hip): out[0] = sum
// over rows of the product over columns of g(salt[c], digest), out[1] = values
// that are not atom ids.
void table_checksum(Ctx& c, const Table& t, const uint64_t* salt, uint64_t out[2]);
double box_store_bw(Ctx& c, uint64_t bytes, uint32_t reps);
void prof_mark(Ctx& c, uint32_t id);
std::unique_ptr<Table> import_rows(Ctx& c, int kind, int ncols, const int32_t* vars, const int32_t* member,
                                   const uint32_t* src, uint64_t n);

// plan.hip: whole-expression evaluation (das_plan_execute)
struct PlanOutput {
  bool matched = false, negation = false;
  std::vector<std::unique_ptr<Table>> tables;
};
PlanOutput plan_execute(Ctx& c, const das_plan_node_t* nodes, uint32_t n, int no_overload);
// Several independent plans in one call (das_plan_execute_many): each result
// equals plan_execute's on that plan alone.  Plans whose root And one fused
// chain answers are launched first, without waiting; the other plans run
// while the chains do; the chains' outcomes are read back last.
std::vector<PlanOutput> plan_execute_many(Ctx& c, const das_plan_node_t* const* nodes, const uint32_t* n,
                                          uint32_t n_plans, int no_overload);
// Sharded evaluation (das_plan_execute_sharded): INPUT leaves are the
// caller's tables (replicated relations), LINK leaves scan / index-join this
// shard's index (partial relations, whose emptiness is assumed, not tested);
// `checks` gets one bit per positive term of the top-level And: the local
// running result is non-empty after that term.
PlanOutput plan_execute_sharded(Ctx& c, const das_plan_node_t* nodes, uint32_t n, int no_overload,
                                const std::vector<const Table*>& inputs, std::vector<uint8_t>& checks);
// Rows a das_scan_link would read (its index ranges; an upper bound of its output).
uint64_t scan_estimate(Ctx& c, const das_link_scan_t& q);
// An upper bound of scan_estimate over every choice of the scan's grounded
// targets (its shape): the largest key range of its type at a grounded
// position; the exact estimate when nothing is grounded; ~0 when unknown.
uint64_t scan_bound(Ctx& c, const das_link_scan_t& q);
// query.hip: an And of ordered Links (terms) and Not(Link) filters (anti)
// evaluated by one single-workgroup launch when its running result stays
// small.  0: not taken (the caller evaluates it operator by operator);
// 1: evaluated -- `matched`, and the result table when matched; 2: partial
// -- `out` is the (non-empty) running result after the first *consumed
// terms, no Not filter applied: the caller continues the And from there.
int fused_and(Ctx& c, const std::vector<const das_plan_node_t*>& terms,
              const std::vector<const das_plan_node_t*>& anti, int no_overload, bool& matched,
              std::unique_ptr<Table>& out, uint32_t* consumed);
// query.hip: an Or of ordered Links with one schema (no Not terms): the
// scans and the union's dedup in one launch.  0: not taken; 1: evaluated.
// The fused And of a whole And operator launched without waiting for its
// outcome (das_plan_execute_many): null when fused_and would not fuse every
// term and Not filter of it; `k` picks the pooled read-back slot and
// descriptor buffer (pub_reserve_pool), which stay the run's until
// fused_and_finish.  fused_and_finish: 1 = answered (matched / out as
// fused_and's), 0 = evaluate the And another way (a grid chain's redo, a
// chain that stopped early).
struct ChainRun;
struct ChainRunDel {
  void operator()(ChainRun* r) const;
};
using ChainRunPtr = std::unique_ptr<ChainRun, ChainRunDel>;
// side >= 0: compiled and launched on side stream `side` (its tables from
// that stream's blocks), which first waits for `fence_in` (recorded on the
// context's stream when the batch began) if *waited is false
ChainRunPtr fused_and_launch(Ctx& c, const std::vector<const das_plan_node_t*>& terms,
                             const std::vector<const das_plan_node_t*>& anti, int no_overload, uint32_t k,
                             int side = -1, hipEvent_t fence_in = nullptr, bool* waited = nullptr);
int fused_and_finish(Ctx& c, ChainRun& r, bool& matched, std::unique_ptr<Table>& out);
// false when fused_and_launch would surely return null (a first term too
// large for the one-workgroup chain): host checks only, nothing allocated
bool fused_and_viable(Ctx& c, const std::vector<const das_plan_node_t*>& terms,
                      const std::vector<const das_plan_node_t*>& anti, int no_overload);
// An Or of one-column scans launched as one bitmap union (k_union_first)
// without waiting for its size (das_plan_execute_many): fused_or with
// `defer` launches and returns 2 when that path applies (0 otherwise,
// nothing launched); fused_or_finish reads the size back (1: answered, 0:
// evaluate the Or another way).
struct UnionRun {
  std::unique_ptr<Table> res;
  DBuf<uint32_t> own;                                 // bitmap + counters
  PubSlot ps{};
  uint32_t ulo = 0, uhi = 0, pool = 0;
  hipStream_t ls = nullptr;
  int fence = -1;
  bool waited = false;
  ~UnionRun() {
    if (ls && !waited) (void)hipStreamSynchronize(ls);   // dropped before its read-back
  }
};
int fused_or(Ctx& c, const std::vector<const das_plan_node_t*>& terms, int no_overload, bool& matched,
             std::unique_ptr<Table>& out, struct UnionRun* defer = nullptr);
std::unique_ptr<UnionRun> fused_or_launch(Ctx& c, const std::vector<const das_plan_node_t*>& terms, int no_overload,
                                          uint32_t k, int side, hipEvent_t fence_in, bool* waited);
int fused_or_finish(Ctx& c, UnionRun& u, bool& matched, std::unique_ptr<Table>& out);

// export.hip: Redis key-space files (canonical_parser.py:119-183)
struct ExportCounts {
  uint64_t outgoing = 0, incoming = 0, patterns = 0, templates = 0, names = 0;
};
ExportCounts export_keyspace(Ctx& c, const std::string& dir);

// composite.hip: Unordered / Composite assignment algebra (pattern_matcher.py:158-368)
std::unique_ptr<Table> theta_join(Ctx& c, const Table& a, const Table& b, int no_overload);
std::unique_ptr<Table> theta_antijoin(Ctx& c, const Table& a, const Table& t);
std::vector<std::unique_ptr<Table>> set_dedup(Ctx& c, const Table* const* ts, int n);
std::vector<std::unique_ptr<Table>> set_minus(Ctx& c, const Table* const* a, int na, const Table* const* b, int nb);

}  // namespace das
