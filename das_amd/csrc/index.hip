// HBM index build: hashing, handle interning and the CSR-style tables the
// query operators read.  Replaces the reference's load path
//   CanonicalParser.parse/_add_* + Mongo insert_many         canonical_parser.py:48-124, 185-206
//   _build_key_value_files + sort(1) + Redis SADD              canonical_parser.py:132-240
// (same families as parser_threads.py:141-253 for the MettaYacc loader).
//
// Layout:
//   atoms        sorted by digest (== sorted hex handle): id order == handle order
//   T_a          links of arity a, rows (link, t0..t_{a-1}) sorted by (type, id)
//   C_a          same rows sorted by (composite type, id)       -> templates:*
//   P_{a,p}      same rows sorted by (type, t_p, id), a <= 3     -> patterns:* with a
//                grounded target at p (unique (type<<32|t_p) keys + row offsets), and
//                typed all-wildcard scans whose output must come sorted by t_p
//   tgt_off/tgt  outgoing sets (stored target order)
// Pattern keys with only wildcard targets are served by T_a (typed) or all of
// T_a ('*' type); a '*' type with grounded targets by one key range of P_{a,p}
// per named type.  This covers exactly the families the reference writes for arity
// 1..3 (canonical_parser.py:148-176); arity >= 4 only has [*, e0..en].
#include <cstring>
#include <map>
#include <mutex>
#include <optional>
#include "das_internal.h"
#include "md5.h"

namespace das {

__global__ void k_iota(uint32_t* p, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)i;
}
__global__ void k_gather_u32(const uint32_t* src, const uint32_t* idx, uint32_t* dst, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[idx[i]];
}

__global__ void k_copy_u32(uint32_t* dst, const uint32_t* src, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}
__global__ void k_fill_u32(uint32_t* dst, uint32_t v, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = v;
}
__global__ void k_copy_u128(uint4* dst, const uint4* src, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

namespace {
// Scalar read-backs (output sizes) without the runtime's blocking wait: a
// one-wave kernel copies up to 8 words into fine-grained pinned host memory
// with system-scope stores, then releases a sequence number; the host spins
// on it.  hipStreamSynchronize's wake-up after a short kernel costs tens of
// microseconds, which is most of a small join.  The spin polls the stream
// every 256 rounds so a faulting kernel is reported instead of waited on.
struct PubArgs {
  const uint32_t* p[8];
  uint32_t n;
};

__global__ void k_publish(PubArgs a, uint32_t* slot, uint32_t seq) {
  const uint32_t i = threadIdx.x;
  if (i < a.n) __hip_atomic_store(&slot[i], *a.p[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __threadfence_system();
  __syncthreads();
  if (i == 0) __hip_atomic_store(&slot[15], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Slot {
  uint32_t* p = nullptr;
  uint32_t seq = 0;
  Slot() {
    DAS_HIP(hipHostMalloc((void**)&p, 64, hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(p, 0, 64);
  }
  ~Slot() { if (p) (void)hipHostFree(p); }
};
// level 1: a plan nested in another's read-back wait (das_plan_execute_many)
// has its own slot and staging buffer, so the outer wait's sequence and
// request stay untouched
thread_local int t_pub_level = 0;

Slot& slot() {
  thread_local Slot s[2];
  return s[t_pub_level];
}

}  // namespace

PubLevel::PubLevel() {
  DAS_CHECK(t_pub_level == 0, DAS_E_INTERNAL, "read-back level: nested twice");
  t_pub_level = 1;
}
PubLevel::~PubLevel() { t_pub_level = 0; }
int pub_level() { return t_pub_level; }

uint8_t* pinned_stage(uint64_t bytes) {
  struct Stage {
    uint8_t* p = nullptr;
    uint64_t cap = 0;
    ~Stage() { if (p) (void)hipHostFree(p); }
  };
  thread_local Stage sts[2];
  Stage& st = sts[t_pub_level];
  if (bytes > st.cap) {
    if (st.p) DAS_HIP(hipHostFree(st.p));
    st.cap = std::max<uint64_t>(bytes, 1 << 16);
    DAS_HIP(hipHostMalloc((void**)&st.p, st.cap, hipHostMallocCoherent | hipHostMallocMapped));
  }
  return st.p;
}

PubSlot pub_reserve() {
  Slot& sl = slot();
  const uint32_t seq = ++sl.seq ? sl.seq : ++sl.seq;      // never 0 (the initial value)
  return PubSlot{sl.p, seq};
}

PubSlot pub_reserve_pool(uint32_t k) {
  DAS_CHECK(k < kPubPool, DAS_E_INTERNAL, "read-back pool: bad slot");
  thread_local std::unique_ptr<Slot> pool[kPubPool];
  if (!pool[k]) pool[k] = std::make_unique<Slot>();
  Slot& sl = *pool[k];
  const uint32_t seq = ++sl.seq ? sl.seq : ++sl.seq;
  return PubSlot{sl.p, seq};
}

uint8_t* pinned_stage_pool(uint32_t k, uint64_t bytes) {
  DAS_CHECK(k < kPubPool, DAS_E_INTERNAL, "staging pool: bad buffer");
  struct Stage {
    uint8_t* p = nullptr;
    uint64_t cap = 0;
    ~Stage() { if (p) (void)hipHostFree(p); }
  };
  thread_local Stage pool[kPubPool];
  Stage& st = pool[k];
  if (bytes > st.cap) {
    if (st.p) DAS_HIP(hipHostFree(st.p));
    st.p = nullptr;
    st.cap = std::max<uint64_t>(bytes, 1 << 14);
    DAS_HIP(hipHostMalloc((void**)&st.p, st.cap, hipHostMallocCoherent | hipHostMallocMapped));
  }
  return st.p;
}

namespace {
thread_local WaitHook* t_wait_hook = nullptr;
thread_local double t_wait_mark = 0;           // launched_bytes() when the last wait ended
}

void set_wait_hook(WaitHook* hook) { t_wait_hook = hook; }
double bytes_since_wait() { return launched_bytes() - t_wait_mark; }

void pub_wait(const PubSlot& ps, hipStream_t s, uint32_t* out, uint32_t n) {
  count_readback();
  if (t_wait_hook && *t_wait_hook && __atomic_load_n(&ps.p[15], __ATOMIC_ACQUIRE) != ps.seq) {
    WaitHook* h = t_wait_hook;
    t_wait_hook = nullptr;                       // no nested call from inside the hook
    trace_mark("wait hook");
    const bool done = (*h)([&] { return __atomic_load_n(&ps.p[15], __ATOMIC_ACQUIRE) == ps.seq; });
    t_wait_hook = done ? nullptr : h;
  }
  trace_mark("wait");
  for (uint64_t it = 1;; ++it) {
    if (__atomic_load_n(&ps.p[15], __ATOMIC_ACQUIRE) == ps.seq) break;
    if ((it & 255) == 0) {
      const hipError_t e = hipStreamQuery(s);
      if (e == hipSuccess) {
        if (__atomic_load_n(&ps.p[15], __ATOMIC_ACQUIRE) == ps.seq) break;
        DAS_HIP(hipStreamSynchronize(s));
        DAS_CHECK(__atomic_load_n(&ps.p[15], __ATOMIC_ACQUIRE) == ps.seq, DAS_E_INTERNAL, "read-back slot not written");
        break;
      }
      if (e != hipErrorNotReady) DAS_HIP(e);
    }
    __builtin_ia32_pause();
  }
  for (uint32_t i = 0; i < n; ++i) out[i] = __atomic_load_n(&ps.p[i], __ATOMIC_RELAXED);
  t_wait_mark = launched_bytes();
  trace_mark("woke");
}

ScanCtr& scan_ctr(hipStream_t s) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, ScanCtr> m;
  int dev = 0;
  DAS_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(mu);
  auto it = m.find({dev, s});
  if (it != m.end()) return it->second;
  ScanCtr c{nullptr, 0};
  DAS_HIP(hipMalloc((void**)&c.p, 64));
  DAS_HIP(hipMemsetAsync(c.p, 0, 64, s));
  return m.emplace(std::make_pair(dev, s), c).first->second;
}

namespace {
void read_words(const PubArgs& a, hipStream_t s, uint32_t* out) {
  const PubSlot ps = pub_reserve();
  hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, s, a, ps.p, ps.seq);
  DAS_HIP(hipGetLastError());
  pub_wait(ps, s, out, a.n);
}
}  // namespace

uint64_t read_u64(const uint64_t* d, hipStream_t s) {
  PubArgs a{};
  a.p[0] = reinterpret_cast<const uint32_t*>(d);
  a.p[1] = a.p[0] + 1;
  a.n = 2;
  uint32_t w[2];
  read_words(a, s, w);
  return (uint64_t)w[0] | ((uint64_t)w[1] << 32);
}
void read_u64x2(const uint64_t* d, hipStream_t s, uint64_t out[2]) {
  PubArgs a{};
  for (int i = 0; i < 4; ++i) a.p[i] = reinterpret_cast<const uint32_t*>(d) + i;
  a.n = 4;
  uint32_t w[4];
  read_words(a, s, w);
  out[0] = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  out[1] = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
}
uint32_t read_u32(const uint32_t* d, hipStream_t s) {
  PubArgs a{};
  a.p[0] = d;
  a.n = 1;
  uint32_t w;
  read_words(a, s, &w);
  return w;
}
void read_u32x2(const uint32_t* d0, const uint32_t* d1, hipStream_t s, uint32_t out[2]) {
  PubArgs a{};
  a.p[0] = d0;
  a.p[1] = d1;
  a.n = 2;
  read_words(a, s, out);
}

namespace {

template <typename T>
T* dalloc(Index& idx, uint64_t count) {
  T* p = nullptr;
  if (!count) count = 1;
  p = (T*)cache_alloc(sizeof(T) * count, idx.stream);   // best-fit from the build's freed scratch
  idx.owned.push_back(p);
  idx.device_bytes += sizeof(T) * count;
  return p;
}

template <typename T>
DBuf<T> upload(const T* h, uint64_t n, hipStream_t s) {
  DBuf<T> d(n ? n : 1, s);
  if (n) DAS_HIP(hipMemcpyAsync(d.p, h, sizeof(T) * n, hipMemcpyHostToDevice, s));
  return d;
}

__global__ void k_leaf_ctype(DigS dig, const uint32_t* leaf_ctype, DigS ct, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    ct[i] = dig[leaf_ctype[i]];
}

// flag/catl over unified indices: nodes, links, and anything a link targets.
// world > 1: a link's category comes from its handle's owner (indexed here iff
// handle_owner == rank), so every copy of one handle agrees on every shard.
__global__ void k_init_cat(const uint8_t* leaf_kind, const uint8_t* expr_kind, DigS dig, uint64_t n_leaf,
                           uint64_t n_expr, uint32_t rank, uint32_t world, uint8_t* catl, uint32_t* flag) {
  const uint64_t n = n_leaf + n_expr;
  for (uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; u < n; u += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t c = PRIO_OTHER;
    uint32_t f = 0;
    if (u < n_leaf) {
      if (leaf_kind[u] == 1) { c = PRIO_NODE; f = 1; }
    } else {
      const uint8_t k = expr_kind[u - n_leaf];
      if (k == 1 || k == 3) {
        const bool own = world > 1 ? handle_owner(dig[u], world) == rank : k == 1;
        c = own ? PRIO_LINK : PRIO_REMOTE;
        f = 1;
      }
    }
    catl[u] = c;
    flag[u] = f;
  }
}

__global__ void k_expr_owner(DigS dig, uint64_t n_leaf, uint64_t n_expr, uint32_t world, uint8_t* owner) {
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n_expr; j += (uint64_t)gridDim.x * blockDim.x)
    owner[j] = (uint8_t)handle_owner(dig[n_leaf + j], world);
}

// partition_rows: per-block owner histograms (block-major), then a stable
// scatter.  One wave's rows go out in lane order per owner (ballot prefix),
// waves of a block in order through an LDS running count.
constexpr int kPartMaxWorld = 64;
__global__ void __launch_bounds__(256) k_owner_hist(const uint8_t* owner, uint64_t n, uint32_t world, uint64_t per_block,
                                                    uint32_t* hist) {
  __shared__ uint32_t h[kPartMaxWorld];
  for (uint32_t w = threadIdx.x; w < world; w += blockDim.x) h[w] = 0;
  __syncthreads();
  const uint64_t b = blockIdx.x * per_block, e = b + per_block < n ? b + per_block : n;
  for (uint64_t i = b + threadIdx.x; i < e; i += blockDim.x) atomicAdd(&h[owner[i]], 1u);
  __syncthreads();
  for (uint32_t w = threadIdx.x; w < world; w += blockDim.x) hist[(uint64_t)w * gridDim.x + blockIdx.x] = h[w];
}

__global__ void __launch_bounds__(256) k_owner_scatter(const uint32_t* rows, const uint8_t* owner, uint64_t n,
                                                       uint32_t K, uint32_t world, uint64_t per_block,
                                                       const uint32_t* off, uint32_t* out) {
  __shared__ uint32_t base[kPartMaxWorld];
  for (uint32_t w = threadIdx.x; w < world; w += blockDim.x) base[w] = off[(uint64_t)w * gridDim.x + blockIdx.x];
  __syncthreads();
  const uint64_t b = blockIdx.x * per_block, e = b + per_block < n ? b + per_block : n;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (uint64_t t = b; t < e; t += blockDim.x) {
    const uint64_t i = t + threadIdx.x;
    const uint32_t o = i < e ? owner[i] : 0xFFu;
    // waves of the block take their turn so rows stay in input order
    for (uint32_t wv = 0; wv < blockDim.x / 64; ++wv) {
      if (wv == wave) {
        for (uint32_t w = 0; w < world; ++w) {
          const uint64_t m = __ballot(o == w);
          if (!m) continue;
          if (o == w) {
            const uint64_t dst = (uint64_t)base[w] + __popcll(m & ((1ull << lane) - 1));
            for (uint32_t k = 0; k < K; ++k) out[dst * K + k] = rows[i * K + k];
          }
          if (lane == 0) base[w] += (uint32_t)__popcll(m);
        }
      }
      __syncthreads();
    }
  }
}

__global__ void k_mark_targets(const uint8_t* expr_kind, const uint64_t* off, const uint32_t* child, uint64_t n_expr,
                               uint32_t* flag) {
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n_expr; j += (uint64_t)gridDim.x * blockDim.x) {
    if (expr_kind[j] != 1 && expr_kind[j] != 3) continue;
    // (read first: nodes and links are flagged by k_init_cat already, and a
    // hub's flag line would otherwise take ~10^8 stores)
    for (uint64_t k = off[j] + 1; k < off[j + 1]; ++k)
      if (!flag[child[k]]) flag[child[k]] = 1;
  }
}

// Compaction: out[scan[i]] = i for flagged i.
__global__ void k_compact_index(const uint32_t* flag, const uint32_t* scan, uint64_t n, uint32_t* out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (flag[i]) out[scan[i]] = (uint32_t)i;
}

__global__ void k_digest_key(DigS dig, const uint32_t* idx, uint64_t n, uint64_t* key, bool hi) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const Digest d = dig[idx[i]];
    key[i] = hi ? d.hi() : d.lo();
  }
}

// Counts adjacent entries whose 64-bit high halves tie but whose digests differ
// (then the hi-only sort is not a full 128-bit order and we redo it).
__global__ void k_hi_ties(DigS dig, const uint32_t* idx, uint64_t n, uint32_t* bad) {
  for (uint64_t i = 1 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const Digest a = dig[idx[i - 1]], b = dig[idx[i]];
    if (a.hi() == b.hi() && a.lo() != b.lo()) atomicAdd(bad, 1u);
  }
}

// Adjacent sorted keys that agree on bits [shift, 64) but differ below: the
// prefix-only sort did not fully order them.
__global__ void k_prefix_ties(const uint64_t* key, uint64_t n, int shift, uint32_t* bad) {
  uint32_t b = 0;
  for (uint64_t i = 1 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t x = key[i - 1], y = key[i];
    b |= (x >> shift) == (y >> shift) && x != y;
  }
  if (__ballot(b) && __lane_id() == 0) atomicOr(bad, 1u);
}

// Same checks on the sorted high halves: only adjacent entries whose high
// halves tie gather their digests (duplicate atoms and hi collisions).
// The digest sort's key with the entry's category priority (2 bits) in place
// of the high half's two lowest bits: equal digests stay adjacent (ordered by
// category inside their run); entries whose keys agree above those bits but
// whose digests differ are caught by k_prio_ties (then the exact sort runs).
__global__ void k_digest_key_prio(DigS dig, const uint32_t* idx, const uint8_t* prio, uint64_t n,
                                  uint64_t* key) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t u = idx[i];
    key[i] = (dig[u].hi() & ~3ull) | (uint64_t)(prio[u] & 3u);
  }
}
__global__ void k_prio_ties(const uint64_t* key, DigS dig, const uint32_t* idx, uint64_t n, uint32_t* bad) {
  uint32_t b = 0;
  for (uint64_t i = 1 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if ((key[i] >> 2) == (key[i - 1] >> 2)) {
      const Digest a = dig[idx[i - 1]], c = dig[idx[i]];
      b |= a.hi() != c.hi() || a.lo() != c.lo();
    }
  if (__ballot(b) && __lane_id() == 0) atomicOr(bad, 1u);
}
// tie-free category-carrying keys: a run starts where the digest bits change
__global__ void k_first_flags_prio(const uint64_t* key, uint64_t n, uint32_t* first) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    first[i] = i == 0 || (key[i] >> 2) != (key[i - 1] >> 2);
}

__global__ void k_hi_ties_key(const uint64_t* key, DigS dig, const uint32_t* idx, uint64_t n, uint32_t* bad) {
  uint32_t b = 0;
  for (uint64_t i = 1 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (key[i] == key[i - 1]) b |= dig[idx[i - 1]].lo() != dig[idx[i]].lo();
  if (__ballot(b) && __lane_id() == 0) atomicOr(bad, 1u);
}
__global__ void k_first_flags_key(const uint64_t* key, DigS dig, const uint32_t* idx, uint64_t n,
                                  uint32_t* first) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t f = 1;
    if (i > 0 && key[i] == key[i - 1]) f = dig[idx[i - 1]].lo() != dig[idx[i]].lo();
    first[i] = f;
  }
}

__global__ void k_first_flags(DigS dig, const uint32_t* idx, uint64_t n, uint32_t* first) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t f = 1;
    if (i > 0) {
      const Digest a = dig[idx[i - 1]], b = dig[idx[i]];
      f = (a.w[0] != b.w[0]) | (a.w[1] != b.w[1]) | (a.w[2] != b.w[2]) | (a.w[3] != b.w[3]);
    }
    first[i] = f;
  }
}

// id = inclusive run index; catmax = max category over the run; rep = the
// smallest unified index of that category.  Runs are digest-sorted, so ids
// are sequential in i; a run of one (the common case) is settled here with
// plain stores, longer runs (duplicate atoms) with atomics plus k_pick_rep.
// A hub node's run spans hundreds of millions of entries, so same-address
// atomics would serialise: lanes of one run first reduce inside the wave
// (a run is contiguous in i), the run's last lane in the wave issues the
// atomic, and only when a plain load says the stored value would change.
__device__ __forceinline__ bool wave_run_tail(uint32_t id) {
  const uint32_t nid = __shfl_down(id, 1, 64);
  return __lane_id() == 63 || nid != id;
}

// local2id != nullptr: local2id[u] = id (a 4-byte random scatter per entry);
// else ids[i] = id in sorted order, scattered later window by window
// (scatter_partitioned: the random writes land in a MALL-sized window at a time)
__global__ void __launch_bounds__(256) k_assign_ids(const uint32_t* idx, const uint32_t* first, const uint32_t* scan,
                                                    uint64_t n, const uint8_t* catl, const uint64_t* pkey,
                                                    uint32_t* local2id, uint32_t* ids, uint32_t* catmax, uint32_t* rep,
                                                    uint8_t* cat_sorted) {
  const int lane = __lane_id();
  for (uint64_t base = blockIdx.x * (uint64_t)blockDim.x; base < n; base += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = base + threadIdx.x;           // block-uniform trip count: the whole wave shuffles
    const bool act = i < n;
    uint32_t id = kNone, m = 0;
    bool single = true;
    if (act) {
      id = scan[i] + first[i] - 1;
      const uint32_t u = idx[i];
      const uint8_t c = pkey ? (uint8_t)(pkey[i] & 3u) : catl[u];   // pkey: the category rode in the sort key
      if (local2id) local2id[u] = id;
      else ids[i] = id;
      cat_sorted[i] = c;
      single = first[i] && (i + 1 == n || first[i + 1]);
      if (single) {
        catmax[id] = c;
        rep[id] = u;
      }
      m = c;
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {               // segmented max over equal ids
      const uint32_t om = __shfl_up(m, d, 64), oid = __shfl_up(id, d, 64);
      if (lane >= d && oid == id) m = om > m ? om : m;
    }
    const bool tail = wave_run_tail(id);             // every lane shuffles, outside the branch
    if (act && !single && tail && catmax[id] < m) atomicMax(&catmax[id], m);
  }
}

__global__ void __launch_bounds__(256) k_pick_rep(const uint32_t* idx, const uint32_t* first, const uint32_t* scan,
                                                  uint64_t n, const uint8_t* cat_sorted, const uint32_t* catmax,
                                                  uint32_t* rep) {
  const int lane = __lane_id();
  for (uint64_t base = blockIdx.x * (uint64_t)blockDim.x; base < n; base += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = base + threadIdx.x;
    const bool act = i < n;
    uint32_t id = kNone, mn = kNone;
    bool single = true;
    if (act) {
      id = scan[i] + first[i] - 1;
      single = first[i] && (i + 1 == n || first[i + 1]);   // singleton: settled by k_assign_ids
      if (!single && (uint32_t)cat_sorted[i] == catmax[id]) mn = idx[i];
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {               // segmented min over equal ids
      const uint32_t om = __shfl_up(mn, d, 64), oid = __shfl_up(id, d, 64);
      if (lane >= d && oid == id) mn = om < mn ? om : mn;
    }
    const bool tail = wave_run_tail(id);
    if (act && !single && mn != kNone && tail && mn < rep[id]) atomicMin(&rep[id], mn);
  }
}

// every run must have found its representative (a miss would send later
// gathers to index kNone): flagged here and reported as an error instead
__global__ void k_rep_missing(const uint32_t* rep, uint64_t n, uint32_t* bad) {
  uint32_t miss = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    miss |= rep[i] == kNone;
  if (__ballot(miss) && __lane_id() == 0) atomicOr(bad, 1u);
}

// dst[key[i]] = val[i] over (key, val) pairs grouped by the key's top bits:
// consecutive waves write into one key window at a time, so the random 4-byte
// stores merge in the L2 / MALL before they reach HBM
__global__ void k_scatter_pairs(const uint32_t* __restrict__ key, const uint32_t* __restrict__ val, uint64_t n,
                                uint32_t* __restrict__ dst) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[key[i]] = val[i];
}

// named-type cluster key of a temp (digest-order) id; kNone types last
__global__ void k_temp_type(uint64_t n_atoms, const uint32_t* rep, const uint32_t* catmax, uint64_t n_leaf,
                            const uint32_t* leaf_ctype, const uint32_t* leaf_type_id, const uint32_t* etype,
                            uint32_t n_types, uint32_t degree_bits, uint32_t* key) {
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n_atoms; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t u = rep[t];
    uint32_t ty = kNone;
    if (u < n_leaf) {
      ty = leaf_type_id[leaf_ctype[u]];
    } else if (catmax[t] == PRIO_LINK || catmax[t] == PRIO_REMOTE) {
      ty = leaf_type_id[etype[u - n_leaf]];
    }
    const uint32_t k = ty == kNone ? n_types : ty;
    // degree_bits = 5: (type, 31) -- the bucket of an atom with no sampled
    // reference; k_run_bucket lowers it for the referenced ones
    key[t] = degree_bits ? (k << 5) | 31u : k;
  }
}

// References to each unified index from link expressions (kinds 1 and 3:
// every rank of a sharded KB holds all of them, so all ranks count alike),
// counted without same-address atomics (a hub is referenced 10^8 times):
// every stride-th link writes its targets into fixed slots (kNone padding),
// the slots are radix-sorted, and each run of equal targets adds its length
// once (one atomic per run end and per run start).
__global__ void k_ref_sample(const uint8_t* expr_kind, const uint64_t* off, const uint32_t* child, uint64_t n_expr,
                             uint64_t stride, uint64_t n_samp, uint32_t* slots) {
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < n_samp; s += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t j = s * stride;
    uint32_t* o = slots + s * kMaxArity;
    uint32_t k = 0;
    if (j < n_expr && (expr_kind[j] == 1 || expr_kind[j] == 3)) {
      const uint64_t b = off[j] + 1, e = off[j + 1];
      for (uint64_t c = b; c < e && k < (uint32_t)kMaxArity; ++c) o[k++] = child[c];
    }
    for (; k < (uint32_t)kMaxArity; ++k) o[k] = kNone;
  }
}
// after k_temp_type: each sampled run's atom (temp id through local2id) takes
// the bucket 31 - floor(log2(count + 1)) in its key's low 5 bits; copies of
// one atom keep the largest count (atomicMin: deterministic)
__global__ void k_run_bucket(const uint32_t* key, uint64_t n, const uint32_t* cnt, const uint32_t* local2id,
                             uint32_t* tkey) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t u = key[i];
    if (u == kNone || (i + 1 < n && key[i + 1] == u)) continue;    // run ends only
    const uint32_t t = local2id[u];
    if (t == kNone) continue;
    atomicMin(&tkey[t], (tkey[t] & ~31u) | (uint32_t)__clz((int)(cnt[u] + 1u)));
  }
}
__global__ void k_run_count(const uint32_t* key, uint64_t n, uint32_t* cnt) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t k = key[i];
    if (k == kNone) continue;
    if (i == 0 || key[i - 1] != k) atomicSub(&cnt[k], (uint32_t)i);
    if (i + 1 == n || key[i + 1] != k) atomicAdd(&cnt[k], (uint32_t)(i + 1));
  }
}

// host node mirror: nodes in by_digest (handle) order
__global__ void k_node_flags(uint64_t n, const uint32_t* by_digest, const uint8_t* cat, uint32_t* flag) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    flag[i] = cat[by_digest[i]] == CAT_NODE ? 1u : 0u;
}
__global__ void k_node_pack(uint64_t n, const uint32_t* by_digest, const uint8_t* cat, const uint32_t* pos,
                            const Digest* dig, const uint32_t* type, Digest* o_dig, uint32_t* o_id, uint32_t* o_type) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t id = by_digest[i];
    if (cat[id] != CAT_NODE) continue;
    const uint32_t o = pos[i];
    o_dig[o] = dig[id];
    o_id[o] = id;
    o_type[o] = type[id];
  }
}

// final id f <- temp perm[f]; by_digest[temp] = f
__global__ void k_apply_perm(uint64_t n, const uint32_t* perm, const uint32_t* rep, const uint32_t* catmax,
                             uint32_t* rep2, uint32_t* cat2, uint32_t* by_digest) {
  for (uint64_t f = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; f < n; f += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t t = perm[f];
    rep2[f] = rep[t];
    cat2[f] = catmax[t];
    by_digest[t] = (uint32_t)f;
  }
}

__global__ void k_remap_local(uint64_t n, const uint32_t* by_digest, uint32_t* local2id) {
  for (uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; u < n; u += (uint64_t)gridDim.x * blockDim.x)
    if (local2id[u] != kNone) local2id[u] = by_digest[local2id[u]];
}

// tkey (non-null): the id-order sort keys, already in final id order -- each
// atom's named type is its key's high bits (k_temp_type looked it up once),
// so the type's two dependent gathers (expr_child[expr_off[j]], then the type
// table; leaf_ctype for nodes) are not repeated here
__global__ void k_fill_atoms(uint64_t n_atoms, const uint32_t* rep, const uint32_t* catmax, DigS dig,
                             DigS ct, uint64_t n_leaf, const uint32_t* leaf_ctype,
                             const uint32_t* leaf_type_id, const uint64_t* expr_off, const uint32_t* expr_child,
                             Digest* a_dig, uint8_t* a_cat, uint32_t* a_type, uint32_t* a_arity, Digest* a_ct,
                             uint32_t* a_name_leaf, const uint32_t* tkey, uint32_t tshift, uint32_t n_types,
                             uint64_t* a_eoff) {
  for (uint64_t id = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; id < n_atoms;
       id += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t u = rep[id];
    const uint8_t c = cat_of_prio(catmax[id]);
    a_dig[id] = dig[u];
    a_ct[id] = ct[u];
    a_cat[id] = c;
    uint32_t ty = kNone, ar = 0, nl = kNone;
    if (tkey) {
      const uint32_t k = tkey[id] >> tshift;
      ty = k == n_types ? kNone : k;
    }
    if (u < n_leaf) {
      if (!tkey) ty = leaf_type_id[leaf_ctype[u]];
      if (c == CAT_NODE) nl = u;
    } else {
      const uint64_t j = u - n_leaf;
      if (c == CAT_LINK || c == CAT_LINK_REMOTE) {
        const uint64_t b0 = expr_off[j];
        if (!tkey) ty = leaf_type_id[expr_child[b0]];
        ar = (uint32_t)(expr_off[j + 1] - b0 - 1);
        if (a_eoff) a_eoff[id] = b0;                   // k_fill_targets reads it in id order
      }
    }
    a_type[id] = ty;
    a_arity[id] = ar;
    a_name_leaf[id] = nl;
  }
}

// a_eoff[id]: the link's expression offset, written in id order by
// k_fill_atoms (no random expr_off gather through rep here); its targets
// are the expression's elements after the type, tgt_off[id + 1] - tgt_off[id]
// of them
__global__ void k_fill_targets(uint64_t n_atoms, const uint8_t* a_cat, const uint64_t* tgt_off,
                               const uint64_t* a_eoff, const uint32_t* expr_child, const uint32_t* local2id,
                               uint32_t* tgt) {
  for (uint64_t id = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; id < n_atoms;
       id += (uint64_t)gridDim.x * blockDim.x) {
    if (a_cat[id] != CAT_LINK && a_cat[id] != CAT_LINK_REMOTE) continue;
    const uint64_t b = a_eoff[id] + 1;
    const uint64_t o = tgt_off[id], m = tgt_off[id + 1] - o;
    for (uint64_t k = 0; k < m; ++k) tgt[o + k] = local2id[expr_child[b + k]];
  }
}

__global__ void k_link_flags(const uint8_t* cat, const uint32_t* arity, uint64_t n, uint32_t want_arity, uint32_t* f) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    f[i] = (cat[i] == CAT_LINK) && (want_arity == kNone || arity[i] == want_arity);
}

__global__ void k_arity_hist(const uint8_t* cat, const uint32_t* arity, uint64_t n, unsigned long long* h) {
  // per-thread counters for nodes and arities 0..kMaxArity (registers), one LDS
  // add per counter per thread, one global add per counter per block: the
  // same-address LDS atomics of a per-element histogram serialise a wave
  constexpr int NC = kMaxArity + 2;               // [0..kMaxArity] arities, [NC-1] nodes
  __shared__ unsigned int sh[64];
  if (threadIdx.x < 64) sh[threadIdx.x] = 0;
  __syncthreads();
  uint32_t cnt[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) cnt[k] = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t c = cat[i];
    if (c == CAT_NODE) { ++cnt[NC - 1]; continue; }
    if (c != CAT_LINK) continue;
    const uint32_t a = arity[i];
    if (a <= (uint32_t)kMaxArity) {
#pragma unroll
      for (int k = 0; k <= kMaxArity; ++k) cnt[k] += (a == (uint32_t)k);
    } else {
      atomicAdd(&sh[a > 62 ? 62 : a], 1u);        // rare: reported as unsupported by the caller
    }
  }
#pragma unroll
  for (int k = 0; k < NC - 1; ++k)
    if (cnt[k]) atomicAdd(&sh[k], cnt[k]);
  if (cnt[NC - 1]) atomicAdd(&sh[63], cnt[NC - 1]);
  __syncthreads();
  if (threadIdx.x < 64 && sh[threadIdx.x]) atomicAdd(&h[threadIdx.x], (unsigned long long)sh[threadIdx.x]);
}

__global__ void k_ct_key(const Digest* a_ct, const uint32_t* ids, uint64_t n, uint64_t* key, bool hi) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const Digest d = a_ct[ids[i]];
    key[i] = hi ? d.hi() : d.lo();
  }
}

__global__ void k_set_ctype(const uint32_t* ids, const uint32_t* first, const uint32_t* scan, uint64_t n,
                            uint32_t* a_ctype) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    a_ctype[ids[i]] = scan[i] + first[i] - 1;
}

__global__ void k_ct_unique(const Digest* a_ct, const uint32_t* ids, const uint32_t* first, const uint32_t* scan,
                            uint64_t n, Digest* out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (first[i]) out[scan[i]] = a_ct[ids[i]];
}

__global__ void k_u32_key(const uint32_t* src, const uint32_t* ids, uint64_t n, uint32_t* key) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    key[i] = src[ids[i]];
}

__global__ void k_pos_key(const uint32_t* type, const uint64_t* tgt_off, const uint32_t* tgt, const uint32_t* ids,
                          uint64_t n, uint32_t p, uint64_t* key) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t id = ids[i];
    key[i] = ((uint64_t)type[id] << 32) | (uint64_t)tgt[tgt_off[id] + p];
  }
}

// target q of each link in ids (the secondary key of P_{a,p})
__global__ void k_tgt_key(const uint64_t* tgt_off, const uint32_t* tgt, const uint32_t* ids, uint64_t n, uint32_t q,
                          uint32_t* key) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    key[i] = tgt[tgt_off[ids[i]] + q];
}

// rows: col 0 = link id, col 1+k = target k
__global__ void k_gather_rows(const uint32_t* ids, uint64_t R, uint64_t ld, uint32_t arity, const uint64_t* tgt_off,
                              const uint32_t* tgt, uint32_t* out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < R; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t id = ids[i];
    out[i] = id;
    const uint64_t o = tgt_off[id];
    for (uint32_t k = 0; k < arity; ++k) out[(uint64_t)(k + 1) * ld + i] = tgt[o + k];
  }
}

// P_{a,p} of one named type's segment [b, b + n) of T_a (rows sorted by
// (type, id)): the rows ordered by (t_p, the other targets in position
// order, id) through ONE stable sort of a packed key -- each field is the
// target minus the segment's column minimum (tbound), in bits_for(max - min)
// bits, t_p most significant -- with the link id (or the T row) as payload.
// The P table's columns then come back out of the key by a streaming unpack
// instead of gathers through a permutation into tgt_off / tgt.
struct PackKey {
  uint32_t n;                  // fields in the key
  uint32_t pos[3];             // target position of field k (k = 0 most significant)
  uint32_t lo[3];              // segment minimum of that column
  uint32_t sh[3];              // bit offset of field k in the key
  uint32_t bits[3];
};

// key of T row b + (rsel ? rsel[i] : i); val = the row's link id (rsel null) or keeps rsel
__global__ void k_pack_key(const uint32_t* __restrict__ T, uint64_t ld, uint64_t b, uint64_t n, PackKey f,
                           const uint32_t* __restrict__ rsel, uint64_t* __restrict__ key, uint32_t* __restrict__ val) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = b + (rsel ? rsel[i] : i);
    uint64_t k = 0;
    for (uint32_t j = 0; j < f.n; ++j) k |= (uint64_t)(T[(uint64_t)(1 + f.pos[j]) * ld + r] - f.lo[j]) << f.sh[j];
    key[i] = k;
    if (!rsel) val[i] = T[r];
  }
}

// stage 1 of a key wider than 64 bits (arity 3): the least significant
// target alone, payload = the row inside the segment
__global__ void k_pack_key32(const uint32_t* __restrict__ col, uint64_t b, uint64_t n, uint32_t lo,
                             uint32_t* __restrict__ key, uint32_t* __restrict__ row) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    key[i] = col[b + i] - lo;
    row[i] = (uint32_t)i;
  }
}

// P_{a,p} (p > 0) from P_{a,0}'s rows [b, b + n) of one type, which are in
// (t_0, .., t_{a-1}) order: key = (t_p - lo) << 32 | low, where low is the
// other target (arity 2) or the row's place in the segment (arity 3); val =
// the link id.  A stable sort on the high word alone then gives (t_p, the
// other targets in position order) -- P_{a,p}'s order -- in ~27-bit passes.
__global__ void k_derive_key(const uint32_t* __restrict__ P0, uint64_t ld, uint64_t b, uint64_t n, uint32_t ar,
                             uint32_t p, uint32_t lo, uint64_t* __restrict__ key, uint32_t* __restrict__ val) {
  const uint32_t q = p == 0 ? 1u : 0u;               // arity 2: the other position
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = b + i;
    const uint32_t low = ar == 2 ? P0[(uint64_t)(1 + q) * ld + r] : (uint32_t)i;
    key[i] = ((uint64_t)(P0[(uint64_t)(1 + p) * ld + r] - lo) << 32) | low;
    val[i] = P0[r];
  }
}

// sorted derive keys -> P_{a,p} rows [b, b + n); arity 3 reads its two other
// targets at P_{a,0} row b + low
__global__ void k_derive_unpack(const uint64_t* __restrict__ key, const uint32_t* __restrict__ val, uint64_t n,
                                uint32_t ar, uint32_t p, uint32_t lo, uint32_t ty, const uint32_t* __restrict__ P0,
                                uint64_t ld0, uint64_t b, uint32_t* __restrict__ out, uint64_t ld,
                                uint64_t* __restrict__ pk) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = key[i];
    const uint32_t tp = (uint32_t)(k >> 32) + lo, low = (uint32_t)k;
    const uint64_t o = b + i;
    out[o] = val[i];
    out[(uint64_t)(1 + p) * ld + o] = tp;
    if (ar == 2) {
      out[(uint64_t)(1 + (p == 0 ? 1u : 0u)) * ld + o] = low;
    } else {
      for (uint32_t q = 0; q < ar; ++q)
        if (q != p) out[(uint64_t)(1 + q) * ld + o] = P0[(uint64_t)(1 + q) * ld0 + b + low];
    }
    pk[o] = ((uint64_t)ty << 32) | tp;
  }
}

// sorted (key, val) -> P rows [ob, ob + n): id, the key's targets, and the
// target left out of the key (pos_rest, read at T row b + val; val is then a
// row, else the link id); pk = type << 32 | t_p for the key directory
__global__ void k_unpack_key(const uint64_t* __restrict__ key, const uint32_t* __restrict__ val, uint64_t n,
                             PackKey f, int32_t pos_rest, const uint32_t* __restrict__ T, uint64_t tld, uint64_t b,
                             uint32_t ty, uint32_t* __restrict__ out, uint64_t ld, uint64_t ob,
                             uint64_t* __restrict__ pk) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = key[i];
    const uint32_t v = val[i];
    uint32_t tp = 0;
    for (uint32_t j = 0; j < f.n; ++j) {
      const uint32_t t = (uint32_t)((k >> f.sh[j]) & ((1ull << f.bits[j]) - 1)) + f.lo[j];
      out[(uint64_t)(1 + f.pos[j]) * ld + ob + i] = t;
      if (j == 0) tp = t;
    }
    if (pos_rest >= 0) {
      const uint64_t r = b + v;
      out[ob + i] = T[r];
      out[(uint64_t)(1 + pos_rest) * ld + ob + i] = T[(uint64_t)(1 + pos_rest) * tld + r];
    } else {
      out[ob + i] = v;
    }
    pk[ob + i] = ((uint64_t)ty << 32) | tp;
  }
}

template <typename K>
__global__ void k_run_flags(const K* key, uint64_t n, uint32_t* f) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    f[i] = (i == 0) || key[i] != key[i - 1];
}

template <typename K>
__global__ void k_run_emit(const K* key, const uint32_t* f, const uint32_t* scan, uint64_t n, K* ukey, uint64_t* uoff) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (f[i]) {
      ukey[scan[i]] = key[i];
      uoff[scan[i]] = i;
    }
}

__global__ void k_lookup(const Digest* dig, const uint32_t* by_digest, uint64_t n_atoms, const Digest* q, uint64_t nq,
                         int64_t* out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nq; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t qh = q[i].hi(), ql = q[i].lo();
    uint64_t lo = 0, hi = n_atoms;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      const Digest d = dig[by_digest[mid]];
      const uint64_t dh = d.hi(), dl = d.lo();
      if (dh < qh || (dh == qh && dl < ql)) lo = mid + 1;
      else hi = mid;
    }
    int64_t r = -1;
    if (lo < n_atoms) {
      const uint32_t id = by_digest[lo];
      const Digest d = dig[id];
      if (d.hi() == qh && d.lo() == ql) r = (int64_t)id;
    }
    out[i] = r;
  }
}

struct WidenU32 {
  const uint32_t* a;
  uint64_t n;
  __device__ uint64_t operator()(uint64_t i) const { return i < n ? (uint64_t)a[i] : 0ull; }
  static std::string name() { return "WidenU32"; }
};

inline dim3 G(uint64_t n) { return dim3(grid_for(n, 256)); }
constexpr unsigned B = 256;

// Indices 0..n) of `flag` set -> compacted list (device) + count.
uint64_t compact_flags(const uint32_t* flag, uint64_t n, DBuf<uint32_t>& out, hipStream_t s) {
  if (!n) { out.alloc(1, s); return 0; }
  DBuf<uint32_t> scan(n, s);
  exclusive_scan<uint32_t>(flag, n, scan.p, s);
  uint32_t last[2];
  read_u32x2(scan.p + n - 1, flag + n - 1, s, last);
  const uint64_t m = (uint64_t)last[0] + last[1];
  out.alloc(m ? m : 1, s);
  KScope ks("k_compact_index", 8.0 * n + 4.0 * m);
  hipLaunchKernelGGL(k_compact_index, G(n), dim3(B), 0, s, flag, (const uint32_t*)scan.p, n, out.p);
  DAS_HIP(hipGetLastError());
  return m;
}

// link id of every outgoing-set entry: out[tgt_off[a] + k] = a
__global__ void k_owner_fill(const uint64_t* tgt_off, uint64_t n_atoms, uint32_t* out) {
  for (uint64_t a = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; a < n_atoms; a += (uint64_t)gridDim.x * blockDim.x)
    for (uint64_t i = tgt_off[a]; i < tgt_off[a + 1]; ++i) out[i] = (uint32_t)a;
}

// sorted keys in [0, n_keys) -> off[k] = first index with key >= k, k in [0, n_keys]
// (one binary search per k: runs of absent keys can be long)
// Two levels: the search first runs over every kBoundStep-th key (samp, a
// few MB that stay in L2 / MALL across the threads' searches), then inside
// one kBoundStep-key block -- ~8 cold loads per search instead of ~31.
constexpr uint64_t kBoundStep = 256;
__global__ void k_bound_sample(const uint32_t* key, uint64_t n, uint32_t* samp, uint64_t ns) {
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < ns; j += (uint64_t)gridDim.x * blockDim.x)
    samp[j] = key[j * kBoundStep];
}
__global__ void k_bounds_u32(const uint32_t* key, uint64_t n, uint32_t n_keys, uint32_t* off, const uint32_t* samp,
                             uint64_t ns) {
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k <= n_keys; k += (uint64_t)gridDim.x * blockDim.x) {
    // first sample >= k: the answer lies in ((j - 1) * step, j * step]
    uint64_t lo = 0, hi = ns;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (samp[mid] < k) lo = mid + 1; else hi = mid;
    }
    hi = lo < ns ? lo * kBoundStep : n;
    lo = lo ? (lo - 1) * kBoundStep + 1 : 0;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (key[mid] < k) lo = mid + 1; else hi = mid;
    }
    off[k] = (uint32_t)lo;
  }
}

// Column id bounds of rows [b, e) of a T_a table (one named type's segment):
// per-thread running min/max, wave + block reduction, one atomic per block
// and column (per-row or per-wave atomics on one address serialise).
__global__ void __launch_bounds__(256) k_seg_minmax(const uint32_t* data, uint64_t rows, uint32_t ncol, uint64_t b,
                                                    uint64_t e, uint32_t* bnd) {
  __shared__ uint32_t s_mn[4], s_mx[4];
  for (uint32_t c = 0; c < ncol; ++c) {
    const uint32_t* col = data + (uint64_t)c * rows;
    uint32_t mn = 0xFFFFFFFFu, mx = 0u;
    for (uint64_t r = b + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < e; r += (uint64_t)gridDim.x * blockDim.x) {
      const uint32_t v = col[r];
      mn = v < mn ? v : mn;
      mx = v > mx ? v : mx;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      mn = min(mn, (uint32_t)__shfl_xor(mn, d, 64));
      mx = max(mx, (uint32_t)__shfl_xor(mx, d, 64));
    }
    if (__lane_id() == 0) {
      s_mn[threadIdx.x >> 6] = mn;
      s_mx[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int w = 1; w < 4; ++w) {
        mn = min(mn, s_mn[w]);
        mx = max(mx, s_mx[w]);
      }
      atomicMin(&bnd[2 * c], mn);
      atomicMax(&bnd[2 * c + 1], mx);
    }
    __syncthreads();
  }
}

// tbound/gbound of T_a (type_off must already hold its per-type row offsets).
void col_bounds(Index& idx, const RowTable& t, uint64_t n_types, hipStream_t s) {
  const uint32_t ncol = (uint32_t)t.arity + 1;
  const uint64_t nb = n_types * ncol * 2;
  std::vector<uint32_t> h(nb);
  for (uint64_t k = 0; k < nb; k += 2) {
    h[k] = 0xFFFFFFFFu;
    h[k + 1] = 0u;
  }
  DBuf<uint32_t> d(nb ? nb : 1, s);
  if (nb) DAS_HIP(hipMemcpyAsync(d.p, h.data(), 4 * nb, hipMemcpyHostToDevice, s));
  const auto& to = idx.type_off[t.arity];
  for (uint64_t ty = 0; ty < n_types && ty + 1 < to.size(); ++ty) {
    const uint64_t b = to[ty], e = to[ty + 1];
    if (e <= b) continue;
    KScope ks("k_seg_minmax", 4.0 * ncol * (e - b));
    hipLaunchKernelGGL(k_seg_minmax, dim3(grid_for(e - b, 256, 1024)), dim3(256), 0, s, (const uint32_t*)t.data,
                       t.ld, ncol, b, e, d.p + ty * ncol * 2);
  }
  DAS_HIP(hipGetLastError());
  if (nb) DAS_HIP(hipMemcpyAsync(h.data(), d.p, 4 * nb, hipMemcpyDeviceToHost, s));
  DAS_HIP(hipStreamSynchronize(s));
  std::vector<uint32_t> g(ncol * 2);
  for (uint32_t c = 0; c < ncol; ++c) {
    g[2 * c] = 0xFFFFFFFFu;
    g[2 * c + 1] = 0u;
    for (uint64_t ty = 0; ty < n_types; ++ty) {
      g[2 * c] = std::min(g[2 * c], h[(ty * ncol + c) * 2]);
      g[2 * c + 1] = std::max(g[2 * c + 1], h[(ty * ncol + c) * 2 + 1]);
    }
  }
  idx.tbound[t.arity] = std::move(h);
  idx.gbound[t.arity] = std::move(g);
}

// dst[keys[i]] = vals[i] for keys < key_range, as one radix partition pass of
// the pairs by the keys' top 8 bits (LDS-staged scatter, contiguous runs per
// bucket) followed by an in-order scatter: each bucket's keys span
// key_range / 256 slots of dst, so the writes of the waves in flight share a
// window of a few MB instead of the whole array.  keys / vals are consumed.
void scatter_partitioned(uint32_t* keys, uint32_t* vals, uint64_t n, uint64_t key_range, uint32_t* dst,
                         hipStream_t s) {
  if (!n) return;
  DAS_CHECK(n < (1ull << 32), DAS_E_UNSUPPORTED, "scatter_partitioned: more than 2^32 pairs");
  const int bits = std::max(1, bits_for(key_range ? key_range - 1 : 0));
  // DAS_L2I_BITS=16 (A/B): two LSD passes on the keys' top 16 bits, so the
  // scatter's windows are key_range / 2^16 slots (L2-sized) instead of / 2^8:
  // k_scatter_pairs 29 -> 15 ms at 10^9 links, but the second pass costs as
  // much (build 650-658 vs 649-653 ms, one box), so one pass stays
  static const int pbits = std::getenv("DAS_L2I_BITS") && std::atoi(std::getenv("DAS_L2I_BITS")) == 16 ? 16 : 8;
  if (pbits == 16 && bits > 16) {
    radix_sort_pairs<uint32_t>(keys, vals, n, bits - 16, bits, s);
    KScope ks("k_scatter_pairs", 12.0 * n);
    hipLaunchKernelGGL(k_scatter_pairs, G(n), dim3(B), 0, s, (const uint32_t*)keys, (const uint32_t*)vals, n, dst);
    DAS_HIP(hipGetLastError());
    return;
  }
  const int shift = std::max(0, bits - 8);
  const uint32_t tiles = (uint32_t)((n + kSortTile - 1) / kSortTile);
  DBuf<uint32_t> hist((uint64_t)tiles * 256, s), offs((uint64_t)tiles * 256, s), k2(n, s), v2(n, s);
  {
    KScope ks("k_radix_hist<u32>", 4.0 * n);
    hipLaunchKernelGGL((k_radix_hist<uint32_t>), dim3(tiles), dim3(kSortBlock), 0, s, (const uint32_t*)keys, n, shift,
                       hist.p, tiles);
  }
  exclusive_scan<uint32_t>(hist.p, (uint64_t)tiles * 256, offs.p, s);
  {
    KScope ks("k_radix_scatter_lds<u32,true>", 16.0 * n);
    hipLaunchKernelGGL((k_radix_scatter_lds<uint32_t, true>), dim3(tiles), dim3(kSortBlock), 0, s, (const uint32_t*)keys,
                       (const uint32_t*)vals, k2.p, v2.p, n, shift, (const uint32_t*)hist.p, (const uint32_t*)offs.p,
                       tiles);
  }
  KScope ks("k_scatter_pairs", 12.0 * n);
  hipLaunchKernelGGL(k_scatter_pairs, G(n), dim3(B), 0, s, (const uint32_t*)k2.p, (const uint32_t*)v2.p, n, dst);
  DAS_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Digest sort on a key prefix.  Digests are uniform, so after an LSD sort on
// the keys' top 40 bits (5 passes instead of 8) the entries are grouped in
// runs of equal prefix that almost always hold one digest (its duplicates:
// ~10^-3 of the distinct digests share a 40-bit prefix at 10^9 entries).  A
// run holding several digests is put in order afterwards: descents inside a
// run are listed (k_prefix_descents), each run with a descent is located once
// (k_descent_runs, a wave walking to its ends), runs up to kRunSortMax entries
// are sorted in LDS by one block each (k_sort_runs_lds), longer ones by a
// radix sort of their low key bits.  The full key order results (equal keys,
// i.e. copies of one digest with one category, in any order: nothing
// downstream depends on their order).
// ---------------------------------------------------------------------------
constexpr int kPrefixShift = 24;                  // sorted bits [24, 64): 40 bits
constexpr uint32_t kMaxDescents = 1u << 22;
constexpr uint32_t kRunSortMax = 4096;

__global__ void k_prefix_descents(const uint64_t* __restrict__ key, uint64_t n, int shift, uint32_t* list,
                                  uint32_t* count, uint32_t cap) {
  for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x; b < n; b += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = b + threadIdx.x;        // block-uniform trip count: the wave ballots together
    bool d = false;
    if (i >= 1 && i < n) {
      const uint64_t a = key[i - 1], c = key[i];
      d = ((a ^ c) >> shift) == 0 && (a >> 2) > (c >> 2);
    }
    const uint64_t m = __ballot(d);
    if (!m) continue;
    uint32_t base = 0;
    if (__lane_id() == 0) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = __shfl(base, 0, 64);
    const uint32_t slot = base + (uint32_t)__popcll(m & __lanemask_lt());
    if (d && slot < cap) list[slot] = (uint32_t)i;
  }
}

// One wave per listed descent: the run [s, e) of equal prefix around it is
// emitted by the wave whose descent is the run's first (a wave that meets an
// earlier descent on its way left leaves the run to that one).
__global__ void k_descent_runs(const uint64_t* __restrict__ key, uint64_t n, int shift, const uint32_t* list,
                               uint32_t nd, uint2* runs, uint32_t* count) {
  const uint32_t lane = __lane_id();
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
  for (uint64_t w = blockIdx.x * (uint64_t)(blockDim.x / 64) + (threadIdx.x >> 6); w < nd; w += waves) {
    const uint64_t i = list[w];
    const uint64_t P = key[i] >> shift;
    // left: positions i-1, i-2, ... 64 per step
    int64_t s = -1;
    bool abort = false;
    for (int64_t j = (int64_t)i - 1; s < 0 && !abort; j -= 64) {
      const int64_t p = j - (int64_t)lane;
      bool in = false, desc = false;
      if (p >= 0) {
        const uint64_t kp = key[p];
        in = (kp >> shift) == P;
        if (in && p >= 1) {
          const uint64_t km = key[p - 1];
          desc = (km >> shift) == P && (km >> 2) > (kp >> 2);
        }
      }
      if (__ballot(desc)) abort = true;                  // an earlier descent of this run
      const uint64_t out = __ballot(!in);                // lanes past the run's start (or p < 0)
      if (out) s = j - (int64_t)__ffsll((long long)out) + 2;     // first lane out: p + 1
    }
    if (abort) continue;
    uint64_t e = 0;
    for (uint64_t j = i + 1; e == 0; j += 64) {
      const uint64_t p = j + lane;
      const bool in = p < n && (key[p] >> shift) == P;
      const uint64_t out = __ballot(!in);
      if (out) e = j + (uint64_t)__ffsll((long long)out) - 1;
    }
    if (lane == 0) {
      const uint32_t r = atomicAdd(count, 1u);
      runs[r] = make_uint2((uint32_t)s, (uint32_t)e);
    }
  }
}

// One block per run of at most kRunSortMax entries: bitonic sort of the
// (key, value) pairs in LDS by the whole key.
__global__ void __launch_bounds__(256) k_sort_runs_lds(uint64_t* key, uint32_t* val, const uint2* runs, uint32_t nr) {
  __shared__ uint64_t sk[kRunSortMax];
  __shared__ uint32_t sv[kRunSortMax];
  for (uint32_t r = blockIdx.x; r < nr; r += gridDim.x) {
    const uint2 run = runs[r];
    const uint32_t m = run.y - run.x;
    if (m > kRunSortMax) continue;                      // block-uniform: the host sorts it
    uint32_t np = 2;
    while (np < m) np <<= 1;
    for (uint32_t t = threadIdx.x; t < np; t += blockDim.x) {
      sk[t] = t < m ? key[run.x + t] : ~0ull;
      sv[t] = t < m ? val[run.x + t] : 0u;
    }
    __syncthreads();
    for (uint32_t k = 2; k <= np; k <<= 1) {
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        for (uint32_t t = threadIdx.x; t < np; t += blockDim.x) {
          const uint32_t o = t ^ j;
          if (o > t) {
            const bool up = (t & k) == 0;
            const uint64_t a = sk[t], b = sk[o];
            if ((a > b) == up) {
              sk[t] = b;
              sk[o] = a;
              const uint32_t x = sv[t];
              sv[t] = sv[o];
              sv[o] = x;
            }
          }
        }
        __syncthreads();
      }
    }
    for (uint32_t t = threadIdx.x; t < m; t += blockDim.x) {
      key[run.x + t] = sk[t];
      val[run.x + t] = sv[t];
    }
    __syncthreads();
  }
}

// After radix_sort_pairs(key, idx, n, shift, 64): order the runs of equal
// key >> shift that hold several keys.  false: too many descents to list
// (the caller sorts the remaining bits instead).
bool fix_prefix_runs(uint64_t* key, uint32_t* idx, uint64_t n, int shift, hipStream_t s) {
  DBuf<uint32_t> cnt(2, s), list(kMaxDescents, s);
  fill_dev(cnt.p, 0, 8, s);
  {
    KScope ks("k_prefix_descents", 8.0 * n);
    hipLaunchKernelGGL(k_prefix_descents, G(n), dim3(B), 0, s, (const uint64_t*)key, n, shift, list.p, cnt.p,
                       kMaxDescents);
    DAS_HIP(hipGetLastError());
  }
  const uint32_t nd = read_u32(cnt.p, s);
  if (nd == 0) return true;
  if (nd > kMaxDescents) return false;
  DBuf<uint2> runs(nd, s);
  hipLaunchKernelGGL(k_descent_runs, dim3(grid_for(nd, B / 64, 65535u)), dim3(B), 0, s, (const uint64_t*)key, n,
                     shift, (const uint32_t*)list.p, nd, runs.p, cnt.p + 1);
  DAS_HIP(hipGetLastError());
  const uint32_t nr = read_u32(cnt.p + 1, s);
  if (!nr) return true;
  {
    KScope ks("k_sort_runs_lds", 24.0 * nr);
    hipLaunchKernelGGL(k_sort_runs_lds, dim3(std::min<uint32_t>(nr, 65535u)), dim3(256), 0, s, key, idx,
                       (const uint2*)runs.p, nr);
    DAS_HIP(hipGetLastError());
  }
  std::vector<uint2> h(nr);
  DAS_HIP(hipMemcpyAsync(h.data(), runs.p, sizeof(uint2) * nr, hipMemcpyDeviceToHost, s));
  DAS_HIP(hipStreamSynchronize(s));
  for (const uint2& r : h)
    if (r.y - r.x > kRunSortMax) radix_sort_pairs<uint64_t>(key + r.x, idx + r.x, r.y - r.x, 0, shift, s);
  return true;
}

// Sorts idx[0..n) by the 128-bit digest dig[idx[i]] (hi-only fast path, exact
// fallback); key[i] = the high half of entry i's digest, sorted.  With
// `prio` (category per unified index) the fast path carries it in the key's
// two lowest bits and returns true: then key >> 2 separates digests and
// key & 3 is the entry's category.  false: exact order, key = high halves.
bool sort_by_digest(DigS dig, uint32_t* idx, uint64_t n, DBuf<uint64_t>& key, hipStream_t s,
                    const uint8_t* prio = nullptr) {
  key.alloc(n ? n : 1, s);
  if (n <= 1) {
    if (n) hipLaunchKernelGGL(k_digest_key, dim3(1), dim3(64), 0, s, dig, (const uint32_t*)idx, n, key.p, true);
    return false;
  }
  DBuf<uint32_t> bad(1, s);
  fill_dev(bad.p, 0, 4, s);
  if (prio) {
    {
      KScope ks("k_digest_key", 29.0 * n);         // index, gathered digest half, category, key out
      hipLaunchKernelGGL(k_digest_key_prio, G(n), dim3(B), 0, s, dig, (const uint32_t*)idx, prio, n, key.p);
    }
    // large sorts: the top 40 key bits, then the runs that hold several keys
    // (DAS_DIGEST_PREFIX=0: all 64 bits; =1: the prefix path at any size)
    const char* pe = std::getenv("DAS_DIGEST_PREFIX");
    const bool prefix = pe && pe[0] == '1' ? true : n >= (1ull << 22) && !(pe && pe[0] == '0');
    // (DAS_DIGEST_PREFIX_SHIFT: a shorter prefix, so that most runs need
    // ordering -- tests of the run fix-up)
    const char* ps = std::getenv("DAS_DIGEST_PREFIX_SHIFT");
    const int shift = ps ? std::max(2, std::min(56, std::atoi(ps))) : kPrefixShift;
    radix_sort_pairs<uint64_t>(key.p, idx, n, prefix ? shift : 0, 64, s);
    if (prefix && !fix_prefix_runs(key.p, idx, n, shift, s))
      radix_sort_pairs<uint64_t>(key.p, idx, n, 0, 64, s);
    {
      KScope ks("k_prio_ties", 8.0 * n);            // sorted keys; digests only where the digest bits tie
      hipLaunchKernelGGL(k_prio_ties, G(n), dim3(B), 0, s, (const uint64_t*)key.p, dig, (const uint32_t*)idx, n,
                         bad.p);
    }
    if (read_u32(bad.p, s) == 0) return true;
    fill_dev(bad.p, 0, 4, s);
  }
  {
    KScope ks("k_digest_key", 28.0 * n);           // index, gathered digest half (8 of 16 B), key out
    hipLaunchKernelGGL(k_digest_key, G(n), dim3(B), 0, s, dig, (const uint32_t*)idx, n, key.p, true);
  }
  radix_sort_pairs<uint64_t>(key.p, idx, n, 0, 64, s);
  {
    KScope ks("k_hi_ties_key", 8.0 * n);          // sorted keys; digests only where they tie
    hipLaunchKernelGGL(k_hi_ties_key, G(n), dim3(B), 0, s, (const uint64_t*)key.p, dig, (const uint32_t*)idx, n, bad.p);
  }
  if (read_u32(bad.p, s) == 0) return false;
  // exact: LSD over (lo, hi)
  hipLaunchKernelGGL(k_digest_key, G(n), dim3(B), 0, s, dig, (const uint32_t*)idx, n, key.p, false);
  radix_sort_pairs<uint64_t>(key.p, idx, n, 0, 64, s);
  hipLaunchKernelGGL(k_digest_key, G(n), dim3(B), 0, s, dig, (const uint32_t*)idx, n, key.p, true);
  radix_sort_pairs<uint64_t>(key.p, idx, n, 0, 64, s);
  return false;
}

// Run-length encoding of sorted keys: unique keys + n_runs+1 offsets (device).
template <typename K>
uint64_t rle(const K* key, uint64_t n, K** ukey, uint64_t** uoff, Index& idx, hipStream_t s) {
  DBuf<uint32_t> f(n ? n : 1, s), scan(n ? n : 1, s);
  uint64_t m = 0;
  const std::string tag = key_tag<K>();
  if (n) {
    KScope ks(("k_run_flags<" + tag + ">").c_str(), (sizeof(K) + 4.0) * n);
    hipLaunchKernelGGL((k_run_flags<K>), G(n), dim3(B), 0, s, key, n, f.p);
    exclusive_scan<uint32_t>(f.p, n, scan.p, s);
    m = (uint64_t)read_u32(scan.p + n - 1, s) + read_u32(f.p + n - 1, s);
  }
  *ukey = dalloc<K>(idx, m);
  *uoff = dalloc<uint64_t>(idx, m + 1);
  if (n) {
    KScope ks(("k_run_emit<" + tag + ">").c_str(), (sizeof(K) + 8.0) * n + (sizeof(K) + 8.0) * m);
    hipLaunchKernelGGL((k_run_emit<K>), G(n), dim3(B), 0, s, key, (const uint32_t*)f.p, (const uint32_t*)scan.p, n,
                       *ukey, *uoff);
    DAS_HIP(hipGetLastError());
  }
  DAS_HIP(hipMemcpyAsync(*uoff + m, &n, sizeof(uint64_t), hipMemcpyHostToDevice, s));
  DAS_HIP(hipStreamSynchronize(s));   // &n is a host stack value
  return m;
}

}  // namespace

namespace {
// Per type ty: first/last key index of (ty, *) in the sorted unique keys and
// their t_p values -> out[4 ty .. 4 ty + 3] = {klo, khi, tmin, tmax}.
__global__ void k_type_key_bounds(const uint64_t* ukey, uint64_t nkeys, uint32_t ntypes, uint64_t* out) {
  const uint32_t ty = blockIdx.x * blockDim.x + threadIdx.x;
  if (ty >= ntypes) return;
  uint64_t b[2];
  for (int e = 0; e < 2; ++e) {
    const uint64_t q = (uint64_t)(ty + e) << 32;
    uint64_t lo = 0, hi = nkeys;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (ukey[mid] < q) lo = mid + 1; else hi = mid;
    }
    b[e] = lo;
  }
  out[4 * ty] = b[0];
  out[4 * ty + 1] = b[1];
  out[4 * ty + 2] = b[1] > b[0] ? (uint32_t)ukey[b[0]] : 0;
  out[4 * ty + 3] = b[1] > b[0] ? (uint32_t)ukey[b[1] - 1] : 0;
}
__global__ void k_dir_scatter(const uint64_t* ukey, uint64_t klo, uint64_t n, uint32_t tlo, uint32_t* dir) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dir[(uint32_t)ukey[klo + i] - tlo] = (uint32_t)(klo + i);
}
// Bucket directory of one type's sorted keys ukey[klo, klo + n): bucket b =
// (t - tlo) >> shift; bdir[b] = the first key index of bucket >= b, for b in
// [0, nb] (bdir[nb] = klo + n).  Key i writes the buckets after its
// predecessor's up to its own: every slot is written exactly once.
__global__ void k_bdir_fill(const uint64_t* ukey, uint64_t klo, uint64_t n, uint32_t tlo, uint32_t shift,
                            uint32_t nb, uint32_t* bdir) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i <= n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t b1 = i < n ? ((uint32_t)ukey[klo + i] - tlo) >> shift : nb;
    const int64_t b0 = i == 0 ? -1 : (int64_t)(((uint32_t)ukey[klo + i - 1] - tlo) >> shift);
    for (int64_t b = b0 + 1; b <= (int64_t)b1; ++b) bdir[b] = (uint32_t)(klo + i);
  }
}
}  // namespace

void free_index(Index& idx) {
  for (void* p : idx.owned) cache_free(p);
  idx.owned.clear();
  idx = Index();
}

// rank directory: the bit of every key of ukey[klo, klo + n) (sorted, so
// neighbouring lanes mostly set bits of one word: one atomic per word run)
__global__ void k_rank_bits(const uint64_t* ukey, uint64_t klo, uint64_t n, uint32_t tmin, unsigned long long* bits) {
  for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x; b < n; b += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = b + threadIdx.x;             // block-uniform trip count: the whole wave shuffles
    const bool act = i < n;
    const uint32_t d = act ? (uint32_t)(ukey[klo + i] & 0xFFFFFFFFull) - tmin : 0u;
    const uint32_t w = act ? d >> 6 : 0xFFFFFFFFu;
    unsigned long long m = act ? 1ull << (d & 63) : 0ull;
    // OR the bits of the lanes sharing this lane's word (runs: sorted keys)
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
      const unsigned long long om = __shfl_down(m, s, 64);
      const uint32_t ow = __shfl_down(w, s, 64);
      if ((int)__lane_id() + s < 64 && ow == w) m |= om;
    }
    const uint32_t pw = __shfl_up(w, 1, 64);
    if (act && (__lane_id() == 0 || pw != w)) atomicOr(&bits[w], m);   // the run's first lane
  }
}
__global__ void k_rank_popc(const uint64_t* bits, uint64_t nw, uint32_t* pc) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * blockDim.x)
    pc[i] = (uint32_t)__popcll(bits[i]);
}

void build_key_dir(PosIndex& P, Index& idx, hipStream_t s) {
  const uint32_t nt = (uint32_t)idx.n_types;
  P.dir.assign(nt, nullptr);
  P.dir_lo.assign(nt, 0);
  P.dir_n.assign(nt, 0);
  P.bdir.assign(nt, nullptr);
  P.bshift.assign(nt, 0);
  P.bn.assign(nt, 0);
  P.rbits.assign(nt, nullptr);
  P.rpre.assign(nt, nullptr);
  P.rklo.assign(nt, 0);
  if (!P.nkeys || !nt || P.nkeys >= 0xFFFFFFFFull) return;
  DBuf<uint64_t> kb(4ull * nt, s);
  hipLaunchKernelGGL(k_type_key_bounds, dim3((nt + 63) / 64), dim3(64), 0, s, (const uint64_t*)P.ukey, P.nkeys, nt,
                     kb.p);
  DAS_HIP(hipGetLastError());
  std::vector<uint64_t> hb(4ull * nt);
  DAS_HIP(hipMemcpyAsync(hb.data(), kb.p, 32ull * nt, hipMemcpyDeviceToHost, s));
  DAS_HIP(hipStreamSynchronize(s));
  for (uint32_t ty = 0; ty < nt; ++ty) {
    const uint64_t klo = hb[4 * ty], khi = hb[4 * ty + 1], tmin = hb[4 * ty + 2], tmax = hb[4 * ty + 3];
    if (khi <= klo) continue;
    const uint64_t span = tmax - tmin + 1;
    // dense key ranges, and sparse ones up to 16 id slots per key (at most
    // 2^28 slots, 1 GiB): a probe's key is then ONE load instead of a binary
    // search over the type's keys (~24 dependent loads at 10^7 keys: config
    // 5's T1 holds ~1.7 10^7 first targets over 1.3 10^8 node ids)
    // (DAS_KEY_DIR_SPARSE=0: dense ranges only, the round-2/3 rule, for A/B)
    static const bool sparse = !(std::getenv("DAS_KEY_DIR_SPARSE") && std::getenv("DAS_KEY_DIR_SPARSE")[0] == '0');
    if (span > 2 * (khi - klo) + 4096 && (!sparse || span > 16 * (khi - klo) || span > (1ull << 28))) {
      // bucket directory: ~2 keys per bucket (DAS_KEY_BDIR=0: none, A/B)
      static const bool bd = !(std::getenv("DAS_KEY_BDIR") && std::getenv("DAS_KEY_BDIR")[0] == '0');
      if (!bd || khi - klo < 64) continue;
      uint32_t shift = 0;
      while ((span >> shift) > (khi - klo) / 2) ++shift;
      const uint32_t nb = (uint32_t)(((span - 1) >> shift) + 1);
      uint32_t* b = dalloc<uint32_t>(idx, (uint64_t)nb + 1);
      KScope ks("k_bdir_fill", 8.0 * (khi - klo) + 4.0 * nb);
      hipLaunchKernelGGL(k_bdir_fill, dim3(grid_for(khi - klo + 1, 256, 8192)), dim3(256), 0, s,
                         (const uint64_t*)P.ukey, klo, khi - klo, (uint32_t)tmin, shift, nb, b);
      DAS_HIP(hipGetLastError());
      P.bdir[ty] = b;
      P.bshift[ty] = shift;
      P.bn[ty] = nb;
      P.dir_lo[ty] = (uint32_t)tmin;
      continue;
    }
    // large spans: the rank directory (DAS_KEY_RANK=0: dense, A/B; =1 at any span)
    const char* rk = std::getenv("DAS_KEY_RANK");
    if (rk && rk[0] == '1' ? true : span >= (1ull << 20) && !(rk && rk[0] == '0')) {
      const uint64_t nw = (span + 63) / 64;
      uint64_t* rb = dalloc<uint64_t>(idx, nw);
      uint32_t* rp = dalloc<uint32_t>(idx, nw + 1);
      fill_dev(rb, 0, 8 * nw, s);
      {
        KScope ks("k_rank_bits", 8.0 * (khi - klo) + 8.0 * nw);
        hipLaunchKernelGGL(k_rank_bits, dim3(grid_for(khi - klo, 256, 8192)), dim3(256), 0, s,
                           (const uint64_t*)P.ukey, klo, khi - klo, (uint32_t)tmin, (unsigned long long*)rb);
      }
      {
        DBuf<uint32_t> pc(nw, s);
        KScope ks("k_rank_popc", 12.0 * nw);
        hipLaunchKernelGGL(k_rank_popc, dim3(grid_for(nw, 256, 8192)), dim3(256), 0, s, (const uint64_t*)rb, nw, pc.p);
        exclusive_scan<uint32_t>(pc.p, nw, rp, s);
      }
      DAS_HIP(hipGetLastError());
      P.rbits[ty] = rb;
      P.rpre[ty] = rp;
      P.rklo[ty] = klo;
      P.dir_lo[ty] = (uint32_t)tmin;
      P.dir_n[ty] = (uint32_t)span;
      continue;
    }
    uint32_t* d = dalloc<uint32_t>(idx, span);
    fill_dev(d, 0xFF, 4 * span, s);
    KScope ks("k_dir_scatter", 12.0 * (khi - klo));
    hipLaunchKernelGGL(k_dir_scatter, dim3(grid_for(khi - klo, 256, 8192)), dim3(256), 0, s, (const uint64_t*)P.ukey,
                       klo, khi - klo, (uint32_t)tmin, d);
    DAS_HIP(hipGetLastError());
    P.dir[ty] = d;
    P.dir_lo[ty] = (uint32_t)tmin;
    P.dir_n[ty] = (uint32_t)span;
  }
}

namespace {
__global__ void k_unsorted(const uint32_t* key, uint64_t n, uint32_t* bad) {
  uint32_t b = 0;
  for (uint64_t i = 1 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    b |= key[i] < key[i - 1];
  if (__ballot(b) && __lane_id() == 0) atomicOr(bad, 1u);
}
// keys[0..n) already non-decreasing (one read pass; a sort by them would be a no-op)
bool keys_sorted(const uint32_t* key, uint64_t n, hipStream_t s) {
  if (n <= 1) return true;
  DBuf<uint32_t> bad(1, s);
  fill_dev(bad.p, 0, 4, s);
  KScope ks("k_unsorted", 4.0 * n);
  hipLaunchKernelGGL(k_unsorted, G(n), dim3(B), 0, s, key, n, bad.p);
  DAS_HIP(hipGetLastError());
  return read_u32(bad.p, s) == 0;
}
// Step 1 of the build: md5 of every leaf string, composite_hash of every
// expression level by level (children first), and the composite types.
void hash_all(Ctx& c, const das_atoms_t& a, bool dev_expr, const uint8_t* d_bytes, const uint64_t* d_loff,
              const uint32_t* d_lct, const uint32_t* p_child, const uint64_t* p_eoff, const int32_t* p_ectl,
              DigS dig, DigS ct, uint32_t* etype = nullptr) {
  hipStream_t s = c.s;
  const uint64_t nl = a.n_leaf;
  {
    ProfScope ps(c, "k_hash_strings", (double)a.leaf_off[nl] + 8.0 * nl + 16.0 * nl);
    hash_strings(d_bytes, d_loff, nl, dig, s);
  }
  if (nl) {
    KScope ks("k_leaf_ctype", 36.0 * nl);
    hipLaunchKernelGGL(k_leaf_ctype, G(nl), dim3(B), 0, s, dig, d_lct, ct, nl);
  }
  for (uint32_t g = 0; g < a.n_levels; ++g) {
    const uint64_t b = a.level_off[g], e = a.level_off[g + 1];
    if (e <= b) continue;
    uint32_t K;
    if (dev_expr) {
      uint64_t o[2];
      read_u64x2(a.expr_off + b, s, o);
      K = (uint32_t)(o[1] - o[0]);
    } else {
      K = (uint32_t)(a.expr_off[b + 1] - a.expr_off[b]);
    }
    // per expression: K child ids, K child digests + ctypes, offset, ctype leaf, two digests out
    ProfScope ps(c, K <= 9 ? "k_hash_group<" + std::to_string(K) + ">" : std::string("k_hash_group_dyn"),
                 (double)(e - b) * (4.0 * K + 32.0 * K + 8.0 + 4.0 + 32.0));
    hash_group(dig, ct, p_child, p_eoff, p_ectl, nl, b, e - b, K, s, etype);
  }
}
}  // namespace

void hash_owners(Ctx& c, const das_atoms_t& a, uint32_t flags, uint32_t world, uint8_t* d_owner) {
  DAS_CHECK(world >= 1 && world <= 256, DAS_E_INVALID, "bad world size");
  const bool dev_expr = (flags & DAS_BUILD_EXPR_ON_DEVICE) != 0;
  hipStream_t s = c.s;
  const uint64_t nl = a.n_leaf, ne = a.n_expr, nu = nl + ne;
  DAS_CHECK(nu > 0 && nu < 0xFFFFFFF0ull, DAS_E_INVALID, "atom count out of range");
  if (!ne) return;
  const uint64_t n_child = dev_expr ? read_u64(a.expr_off + ne, s) : a.expr_off[ne];
  auto d_bytes = upload(a.leaf_bytes, a.leaf_off[nl], s);
  auto d_loff = upload(a.leaf_off, nl + 1, s);
  auto d_lct = upload(a.leaf_ctype, nl, s);
  DBuf<uint64_t> d_eoff;
  DBuf<uint32_t> d_child;
  DBuf<int32_t> d_ectl;
  if (!dev_expr) {
    d_eoff = upload(a.expr_off, ne + 1, s);
    d_child = upload(a.expr_child, n_child, s);
    d_ectl = upload(a.expr_ctype_leaf, ne, s);
  }
  ProfScope whole(c, "hash_owners", 0.0);
  DBuf<Digest> dc(2 * nu, s);                  // interleaved {digest, composite digest} per unified index
  const DigS dig{dc.p, 2}, ct{dc.p + 1, 2};
  hash_all(c, a, dev_expr, d_bytes.p, d_loff.p, d_lct.p, dev_expr ? a.expr_child : d_child.p,
           dev_expr ? a.expr_off : d_eoff.p, dev_expr ? a.expr_ctype_leaf : d_ectl.p, dig, ct);
  KScope ks("k_expr_owner", 17.0 * ne);
  hipLaunchKernelGGL(k_expr_owner, G(ne), dim3(B), 0, s, dig, nl, ne, world, d_owner);
  DAS_HIP(hipGetLastError());
}

void partition_rows(Ctx& c, const uint32_t* d_rows, uint64_t n, uint32_t K, const uint8_t* d_owner, uint32_t world,
                    uint32_t* d_out, uint64_t* counts) {
  DAS_CHECK(world >= 1 && world <= (uint32_t)kPartMaxWorld && K >= 1, DAS_E_INVALID, "partition_rows: bad sizes");
  hipStream_t s = c.s;
  for (uint32_t w = 0; w < world; ++w) counts[w] = 0;
  if (!n) return;
  ProfScope whole(c, "partition_rows", 0.0);
  const uint64_t per_block = 4096;
  const uint64_t nb = (n + per_block - 1) / per_block;
  DAS_CHECK(nb * world < (1ull << 31) && n < (1ull << 32), DAS_E_UNSUPPORTED, "partition_rows: too many rows");
  DBuf<uint32_t> hist(nb * world, s), off(nb * world, s);
  {
    KScope ks("k_owner_hist", 1.0 * n + 4.0 * nb * world);
    hipLaunchKernelGGL(k_owner_hist, dim3((unsigned)nb), dim3(256), 0, s, d_owner, n, world, per_block, hist.p);
  }
  exclusive_scan<uint32_t>(hist.p, nb * world, off.p, s);
  {
    KScope ks("k_owner_scatter", 1.0 * n + 8.0 * K * n);
    hipLaunchKernelGGL(k_owner_scatter, dim3((unsigned)nb), dim3(256), 0, s, d_rows, d_owner, n, K, world, per_block,
                       (const uint32_t*)off.p, d_out);
  }
  DAS_HIP(hipGetLastError());
  std::vector<uint32_t> starts(world + 1);
  for (uint32_t w = 0; w < world; ++w) starts[w] = read_u32(off.p + (uint64_t)w * nb, s);
  starts[world] = (uint32_t)n;
  for (uint32_t w = 0; w < world; ++w) counts[w] = starts[w + 1] - starts[w];
}

namespace {
}  // namespace

uint64_t host_key_mirror_max() {
  const char* e = std::getenv("DAS_HOST_KEY_MIRROR");
  return e ? std::strtoull(e, nullptr, 10) : kHostKeyMirror;
}

void build_index(Ctx& c, const das_atoms_t& a, uint32_t flags, uint32_t shard_rank, uint32_t shard_world) {
  DAS_CHECK(shard_world >= 1 && shard_rank < shard_world && shard_world <= 256, DAS_E_INVALID, "bad shard rank/world");
  // DAS_BUILD_EXPR_ON_DEVICE: expr_off / expr_child / expr_kind /
  // expr_ctype_leaf are device pointers (resident input, nothing uploaded)
  const bool dev_expr = (flags & DAS_BUILD_EXPR_ON_DEVICE) != 0;
  hipStream_t s = c.s;
  free_index(c.idx);
  Index& idx = c.idx;
  idx.stream = s;
  const uint64_t nl = a.n_leaf, ne = a.n_expr, nu = nl + ne;
  DAS_CHECK(nu > 0 && nu < 0xFFFFFFF0ull, DAS_E_INVALID, "atom count out of range");
  DAS_CHECK(a.n_types < (1u << kTypeBits), DAS_E_UNSUPPORTED, "too many named types");
  const uint64_t n_bytes = a.leaf_off[nl];
  const uint64_t n_child = dev_expr ? (ne ? read_u64(a.expr_off + ne, s) : 0) : a.expr_off[ne];

  // host copies for metadata (node names)
  c.leaf_bytes.assign(a.leaf_bytes, a.leaf_bytes + n_bytes);
  c.leaf_off.assign(a.leaf_off, a.leaf_off + nl + 1);
  // named types: md5(name) (named_type_hash, expression_hasher.py:13-14) and name length
  idx.type_digest.assign(a.n_types, Digest{});
  idx.type_name_len.assign(a.n_types, 0);
  for (uint64_t i = 0; i < nl; ++i) {
    const uint32_t t = a.leaf_type_id[i];
    if (t == kNone || t >= a.n_types) continue;
    const uint64_t b = a.leaf_off[i], e = a.leaf_off[i + 1];
    md5::digest_bytes(a.leaf_bytes + b, e - b, idx.type_digest[t].w);
    idx.type_name_len[t] = (uint32_t)(e - b);
  }
  // the pattern black list given for this build (das_set_pattern_black_list)
  idx.no_pattern.assign(a.n_types, 0);
  idx.no_pattern_any = false;
  for (uint32_t t = 0; t < a.n_types; ++t)
    for (const Digest& d : c.black_list)
      if (std::memcmp(d.w, idx.type_digest[t].w, 16) == 0) {
        idx.no_pattern[t] = 1;
        idx.no_pattern_any = true;
      }

  std::optional<ProfScope> up(std::in_place, c, "upload",
                              (double)n_bytes + 8.0 * nl + 13.0 * nl + (dev_expr ? 0.0 : 8.0 * ne + 4.0 * n_child + 5.0 * ne));
  auto d_bytes = upload(a.leaf_bytes, n_bytes, s);
  auto d_loff = upload(a.leaf_off, nl + 1, s);
  auto d_lkind = upload(a.leaf_kind, nl, s);
  auto d_lct = upload(a.leaf_ctype, nl, s);
  auto d_ltype = upload(a.leaf_type_id, nl, s);
  DBuf<uint64_t> d_eoff;
  DBuf<uint32_t> d_child;
  DBuf<uint8_t> d_ekind;
  DBuf<int32_t> d_ectl;
  if (!dev_expr) {
    d_eoff = upload(a.expr_off, ne + 1, s);
    d_child = upload(a.expr_child, n_child, s);
    d_ekind = upload(a.expr_kind, ne, s);
    d_ectl = upload(a.expr_ctype_leaf, ne, s);
  }
  const uint64_t* p_eoff = dev_expr ? a.expr_off : d_eoff.p;
  const uint32_t* p_child = dev_expr ? a.expr_child : d_child.p;
  const uint8_t* p_ekind = dev_expr ? a.expr_kind : d_ekind.p;
  const int32_t* p_ectl = dev_expr ? a.expr_ctype_leaf : d_ectl.p;
  up.reset();
  // device-side build (hash, intern, CSRs, index tables): config 4's timed region
  ProfScope whole(c, "build_device", 0.0);

  // 1. digests + composite types of every unified index
  // interleaved {digest, composite digest} records: the hash pass's child
  // gathers and k_fill_atoms' per-atom gathers read both from one line
  DBuf<Digest> dc(2 * nu, s);
  const DigS dig{dc.p, 2}, ct{dc.p + 1, 2};
  // each expression's type leaf, written in order by the hash pass (which
  // reads it anyway): k_temp_type's type lookup is one gather, not the two
  // dependent ones through expr_off / expr_child
  DBuf<uint32_t> etype(ne ? ne : 1, s);
  {
    ProfScope ph(c, "phase_hash", 0.0);
    hash_all(c, a, dev_expr, d_bytes.p, d_loff.p, d_lct.p, p_child, p_eoff, p_ectl, dig, ct, etype.p);
  }
  // (phase_* scopes: the build's steps as the bench's kernel table lists them)
  std::optional<ProfScope> phase(std::in_place, c, "phase_intern", 0.0);

  // 2. which unified indices are atoms (nodes, links, link targets)
  DBuf<uint8_t> catl(nu, s);
  DBuf<uint32_t> flag(nu, s);
  {
    KScope ks("k_init_cat", 1.0 * nu + 5.0 * nu);
    hipLaunchKernelGGL(k_init_cat, G(nu), dim3(B), 0, s, (const uint8_t*)d_lkind.p, (const uint8_t*)p_ekind,
                       dig, nl, ne, shard_rank, shard_world, catl.p, flag.p);
  }
  if (ne) {
    KScope ks("k_mark_targets", 9.0 * ne + 8.0 * n_child);
    hipLaunchKernelGGL(k_mark_targets, G(ne), dim3(B), 0, s, (const uint8_t*)p_ekind, (const uint64_t*)p_eoff,
                       (const uint32_t*)p_child, ne, flag.p);
  }
  DAS_HIP(hipGetLastError());
  DBuf<uint32_t> list;
  const uint64_t nc = compact_flags(flag.p, nu, list, s);
  flag.release();

  // 3. intern: sort by digest, one id per distinct digest
  DBuf<uint64_t> skey;
  const bool prio_key = sort_by_digest(dig, list.p, nc, skey, s, catl.p);
  DBuf<uint32_t> first(nc ? nc : 1, s), scan(nc ? nc : 1, s);
  uint64_t n_atoms = 0;
  if (nc) {
    if (prio_key) {
      KScope ks("k_first_flags_prio", 12.0 * nc);  // sorted keys in, flags out
      hipLaunchKernelGGL(k_first_flags_prio, G(nc), dim3(B), 0, s, (const uint64_t*)skey.p, nc, first.p);
    } else {
      KScope ks("k_first_flags_key", 12.0 * nc);   // sorted keys in, flags out; digests only where keys tie
      hipLaunchKernelGGL(k_first_flags_key, G(nc), dim3(B), 0, s, (const uint64_t*)skey.p, dig,
                         (const uint32_t*)list.p, nc, first.p);
    }
    exclusive_scan<uint32_t>(first.p, nc, scan.p, s);
    n_atoms = (uint64_t)read_u32(scan.p + nc - 1, s) + read_u32(first.p + nc - 1, s);
  }
  DBuf<uint32_t> local2id(nu, s), catmax(n_atoms ? n_atoms : 1, s), rep(n_atoms ? n_atoms : 1, s);
  fill_dev(local2id.p, 0xFF, 4 * nu, s);
  fill_dev(catmax.p, 0, 4 * catmax.n, s);
  fill_dev(rep.p, 0xFF, 4 * rep.n, s);
  // local2id by a partitioned scatter above 2^22 entries (DAS_L2I_PART=0: the
  // direct 4-byte random scatter, which wrote ~10x its bytes at 10^9 links;
  // =1: partitioned at every size, tests)
  const char* l2p = std::getenv("DAS_L2I_PART");
  const bool l2i_part = l2p && l2p[0] == '1' ? nc > 0 : nc >= (1ull << 22) && !(l2p && l2p[0] == '0');
  DBuf<uint32_t> ids(l2i_part ? nc : 0, s);
  if (nc) {
    DBuf<uint8_t> cs(nc, s);
    {
      // list, first, scan, catl in; local2id (or the ids in sorted order), sorted
      // category out; catmax + rep per atom
      KScope ks("k_assign_ids", (l2i_part ? 19.0 : 19.0) * nc + 8.0 * n_atoms);
      hipLaunchKernelGGL(k_assign_ids, G(nc), dim3(B), 0, s, (const uint32_t*)list.p, (const uint32_t*)first.p,
                         (const uint32_t*)scan.p, nc, (const uint8_t*)catl.p,
                         prio_key ? (const uint64_t*)skey.p : nullptr, l2i_part ? nullptr : local2id.p,
                         l2i_part ? ids.p : nullptr, catmax.p, rep.p, cs.p);
    }
    skey.release();
    {
      KScope ks("k_pick_rep", 13.0 * nc);
      hipLaunchKernelGGL(k_pick_rep, G(nc), dim3(B), 0, s, (const uint32_t*)list.p, (const uint32_t*)first.p,
                         (const uint32_t*)scan.p, nc, (const uint8_t*)cs.p, (const uint32_t*)catmax.p, rep.p);
    }
    DBuf<uint32_t> bad(1, s);
    fill_dev(bad.p, 0, 4, s);
    {
      KScope ks("k_rep_missing", 4.0 * n_atoms);
      hipLaunchKernelGGL(k_rep_missing, G(n_atoms), dim3(B), 0, s, (const uint32_t*)rep.p, n_atoms, bad.p);
    }
    DAS_HIP(hipGetLastError());
    DAS_CHECK(read_u32(bad.p, s) == 0, DAS_E_INTERNAL, "intern: a digest run has no representative");
  }
  first.release(); scan.release();
  if (l2i_part) scatter_partitioned(list.p, ids.p, nc, nu, local2id.p, s);     // after k_pick_rep read `list`
  ids.release(); list.release();

  phase.emplace(c, "phase_id_order", 0.0);
  // 3b. final ids clustered by named type, so a variable's bindings occupy a
  // compact id range (direct-address joins); inside a type, atoms referenced
  // more often come first (a power-of-two bucket of their reference count,
  // then digest order), so the hot keys of a power-law KB share a few cache
  // lines of any id-indexed bitmap or directory.  by_digest keeps the digest
  // order for handle lookups.  DAS_DEGREE_ORDER=0: digest order inside a type.
  // (the sorted id-order keys stay for k_fill_atoms: each atom's type)
  DBuf<uint32_t> tkey(n_atoms ? n_atoms : 1, s);
  uint32_t tshift = 0;
  {
    DBuf<uint32_t> perm(n_atoms ? n_atoms : 1, s);
    const char* dg = std::getenv("DAS_DEGREE_ORDER");
    const bool degree = !(dg && dg[0] == '0') && ne > 0;
    tshift = degree ? 5u : 0u;
    if (n_atoms) {
      DBuf<uint32_t> cnt, slots;
      uint64_t n_slots = 0;
      if (degree) {
        // every link below 2^22 targets, else every 64th link (the bucket only
        // orders; a hub stays a hub in any sample)
        const uint64_t stride = n_child < (1ull << 22) ? 1 : 64;
        const uint64_t n_samp = (ne + stride - 1) / stride;
        n_slots = n_samp * kMaxArity;
        cnt.alloc(nu, s);
        fill_dev(cnt.p, 0, 4 * nu, s);
        slots.alloc(n_slots, s);
        {
          KScope ks("k_ref_sample", 21.0 * n_samp + 4.0 * n_slots);
          hipLaunchKernelGGL(k_ref_sample, G(n_samp), dim3(B), 0, s, (const uint8_t*)p_ekind, (const uint64_t*)p_eoff,
                             (const uint32_t*)p_child, ne, stride, n_samp, slots.p);
        }
        radix_sort_pairs<uint32_t>(slots.p, nullptr, n_slots, 0, 32, s);
        {
          KScope ks("k_run_count", 8.0 * n_slots);
          hipLaunchKernelGGL(k_run_count, G(n_slots), dim3(B), 0, s, (const uint32_t*)slots.p, n_slots, cnt.p);
        }
        DAS_HIP(hipGetLastError());
      }
      {
        KScope ks("k_temp_type", 24.0 * n_atoms);    // rep, catmax, a type lookup, key out
        hipLaunchKernelGGL(k_temp_type, G(n_atoms), dim3(B), 0, s, n_atoms, (const uint32_t*)rep.p,
                           (const uint32_t*)catmax.p, nl, (const uint32_t*)d_lct.p, (const uint32_t*)d_ltype.p,
                           (const uint32_t*)etype.p, a.n_types, degree ? 5u : 0u, tkey.p);
        etype.release();
      }
      if (degree) {
        KScope ks("k_run_bucket", 8.0 * n_slots);
        hipLaunchKernelGGL(k_run_bucket, G(n_slots), dim3(B), 0, s, (const uint32_t*)slots.p, n_slots,
                           (const uint32_t*)cnt.p, (const uint32_t*)local2id.p, tkey.p);
        DAS_HIP(hipGetLastError());
        slots.release();
        cnt.release();
      }
      const int kbits = std::max(1, bits_for(a.n_types)) + (degree ? 5 : 0);
      iota(perm.p, n_atoms, s);
      radix_sort_pairs<uint32_t>(tkey.p, perm.p, n_atoms, 0, kbits, s);
    }
    idx.by_digest = dalloc<uint32_t>(idx, n_atoms);
    DBuf<uint32_t> rep2(n_atoms ? n_atoms : 1, s), cat2(n_atoms ? n_atoms : 1, s);
    if (n_atoms) {
      {
        KScope ks("k_apply_perm", 24.0 * n_atoms);
        hipLaunchKernelGGL(k_apply_perm, G(n_atoms), dim3(B), 0, s, n_atoms, (const uint32_t*)perm.p,
                           (const uint32_t*)rep.p, (const uint32_t*)catmax.p, rep2.p, cat2.p, idx.by_digest);
      }
      KScope ks("k_remap_local", 8.0 * nu + 4.0 * n_atoms);
      hipLaunchKernelGGL(k_remap_local, G(nu), dim3(B), 0, s, nu, (const uint32_t*)idx.by_digest, local2id.p);
      DAS_HIP(hipGetLastError());
    }
    rep = std::move(rep2);
    catmax = std::move(cat2);
  }

  phase.emplace(c, "phase_atom_arrays", 0.0);
  // 4. atom arrays (id order: named type, reference bucket, handle)
  idx.n_atoms = n_atoms;
  idx.n_types = a.n_types;
  idx.digest = dalloc<Digest>(idx, n_atoms);
  idx.cat = dalloc<uint8_t>(idx, n_atoms);
  idx.type = dalloc<uint32_t>(idx, n_atoms);
  idx.arity = dalloc<uint32_t>(idx, n_atoms);
  idx.tgt_off = dalloc<uint64_t>(idx, n_atoms + 1);
  idx.ctype = dalloc<uint32_t>(idx, n_atoms);
  idx.name_leaf = dalloc<uint32_t>(idx, n_atoms);
  DBuf<Digest> a_ct(n_atoms ? n_atoms : 1, s);
  DBuf<uint64_t> a_eoff(n_atoms ? n_atoms : 1, s);
  if (n_atoms) {
    // rep + catmax in, digest + ctype digest gathered, type lookup; digest,
    // cat, type, arity, ctype digest, name leaf out
    KScope ks("k_fill_atoms", 8.0 * n_atoms + 32.0 * n_atoms + 8.0 * n_atoms + 16.0 * n_atoms + 29.0 * n_atoms);
    hipLaunchKernelGGL(k_fill_atoms, G(n_atoms), dim3(B), 0, s, n_atoms, (const uint32_t*)rep.p,
                       (const uint32_t*)catmax.p, dig, ct, nl,
                       (const uint32_t*)d_lct.p, (const uint32_t*)d_ltype.p, (const uint64_t*)p_eoff,
                       (const uint32_t*)p_child, idx.digest, idx.cat, idx.type, idx.arity, a_ct.p, idx.name_leaf,
                       (const uint32_t*)tkey.p, tshift, (uint32_t)a.n_types, a_eoff.p);
    DAS_HIP(hipGetLastError());
  }
  tkey.release();
  fill_dev(idx.ctype, 0xFF, 4 * (n_atoms ? n_atoms : 1), s);
  // outgoing CSR
  {
    // widen arity to u64 for the scan (sum of arities may exceed 2^32 at 1B links)
    exclusive_scan_fn<uint64_t>(WidenU32{idx.arity, n_atoms}, n_atoms + 1, idx.tgt_off, s);
    const uint64_t total = read_u64(idx.tgt_off + n_atoms, s);
    idx.tgt = dalloc<uint32_t>(idx, total);
    KScope ks("k_fill_targets", 13.0 * n_atoms + 12.0 * total);     // per target: child in, id lookup, target out
    if (n_atoms)
      hipLaunchKernelGGL(k_fill_targets, G(n_atoms), dim3(B), 0, s, n_atoms, (const uint8_t*)idx.cat,
                         (const uint64_t*)idx.tgt_off, (const uint64_t*)a_eoff.p, (const uint32_t*)p_child,
                         (const uint32_t*)local2id.p, idx.tgt);
    DAS_HIP(hipGetLastError());
  }
  a_eoff.release();
  dc.release(); catl.release(); local2id.release(); catmax.release(); rep.release();
  d_child.release(); d_bytes.release();
  phase.reset();

  // incoming CSR (the reference's `incomming_set:<target>` family,
  // canonical_parser.py:141-143): every (target, link) pair of the outgoing
  // sets, sorted by target then link id; in_off by bucket bounds.
  {
    ProfScope ps(c, "incoming_csr", 0.0);
    const uint64_t total = read_u64(idx.tgt_off + n_atoms, s);
    DAS_CHECK(total < (1ull << 32), DAS_E_UNSUPPORTED, "incoming CSR: more than 2^32 link targets");
    idx.in_off = dalloc<uint32_t>(idx, n_atoms + 1);
    idx.in_link = dalloc<uint32_t>(idx, total);
    if (total) {
      DBuf<uint32_t> key(total, s);
      {
        KScope ks("k_owner_fill", 8.0 * n_atoms + 4.0 * total);
        hipLaunchKernelGGL(k_owner_fill, G(n_atoms), dim3(B), 0, s, (const uint64_t*)idx.tgt_off, n_atoms, idx.in_link);
      }
      copy_dev(key.p, idx.tgt, 4 * total, s);
      radix_sort_pairs<uint32_t>(key.p, idx.in_link, total, 0, std::max(1, bits_for(n_atoms ? n_atoms - 1 : 0)), s);
      const uint64_t ns = (total + kBoundStep - 1) / kBoundStep;
      DBuf<uint32_t> samp(ns, s);
      hipLaunchKernelGGL(k_bound_sample, G(ns), dim3(B), 0, s, (const uint32_t*)key.p, total, samp.p, ns);
      KScope ks("k_bounds_u32", 4.0 * total + 4.0 * (n_atoms + 1));
      hipLaunchKernelGGL(k_bounds_u32, G(n_atoms + 1), dim3(B), 0, s, (const uint32_t*)key.p, total,
                         (uint32_t)n_atoms, idx.in_off, (const uint32_t*)samp.p, ns);
    } else {
      fill_dev(idx.in_off, 0, 4 * (n_atoms + 1), s);
    }
    DAS_HIP(hipGetLastError());
    idx.in_total = total;
  }

  // 5. counts per arity, node count
  uint64_t links_of_arity[kMaxArity + 1] = {};
  {
    DBuf<unsigned long long> h(64, s);
    fill_dev(h.p, 0, 64 * 8, s);
    KScope ks("k_arity_hist", 5.0 * n_atoms);
    if (n_atoms) hipLaunchKernelGGL(k_arity_hist, dim3(grid_for(n_atoms, B, 2048)), dim3(B), 0, s, (const uint8_t*)idx.cat,
                                    (const uint32_t*)idx.arity, n_atoms, h.p);
    unsigned long long hh[64];
    DAS_HIP(hipMemcpyAsync(hh, h.p, sizeof(hh), hipMemcpyDeviceToHost, s));
    DAS_HIP(hipStreamSynchronize(s));
    for (int i = 0; i <= kMaxArity; ++i) links_of_arity[i] = hh[i];
    idx.n_nodes = hh[63];
    idx.n_links = 0;
    for (int i = 0; i < 63; ++i) idx.n_links += hh[i];
    for (int i = kMaxArity + 1; i < 63; ++i)
      DAS_CHECK(hh[i] == 0, DAS_E_UNSUPPORTED, "links with arity > 8 are not indexed by this build");
  }

  // 6. composite-type ids over links
  phase.emplace(c, "phase_ctypes", 0.0);
  uint64_t n_ctypes = 0;
  {
    DBuf<uint32_t> lf(n_atoms ? n_atoms : 1, s), lids;
    if (n_atoms) {
      KScope ks("k_link_flags", 9.0 * n_atoms);
      hipLaunchKernelGGL(k_link_flags, G(n_atoms), dim3(B), 0, s, (const uint8_t*)idx.cat,
                                    (const uint32_t*)idx.arity, n_atoms, kNone, lf.p);
    }
    const uint64_t nlk = compact_flags(lf.p, n_atoms, lids, s);
    if (nlk) {
      // sort link ids by ctype digest (hi, exact fallback)
      DBuf<uint64_t> key(nlk, s);
      {
        KScope ks("k_ct_key", 28.0 * nlk);
        hipLaunchKernelGGL(k_ct_key, G(nlk), dim3(B), 0, s, (const Digest*)a_ct.p, (const uint32_t*)lids.p, nlk, key.p, true);
      }
      // composite types are few: order by the top 16 bits of hi (2 passes, not
      // 8); exact unless two different hi values share those bits, or two
      // different digests share hi -- either sends us to the full sort
      radix_sort_pairs<uint64_t>(key.p, lids.p, nlk, 48, 64, s);
      DBuf<uint32_t> bad(1, s);
      fill_dev(bad.p, 0, 4, s);
      hipLaunchKernelGGL(k_prefix_ties, G(nlk), dim3(B), 0, s, (const uint64_t*)key.p, nlk, 48, bad.p);
      hipLaunchKernelGGL(k_hi_ties, G(nlk), dim3(B), 0, s, dig_s(a_ct.p), (const uint32_t*)lids.p, nlk, bad.p);
      if (read_u32(bad.p, s)) {
        hipLaunchKernelGGL(k_ct_key, G(nlk), dim3(B), 0, s, (const Digest*)a_ct.p, (const uint32_t*)lids.p, nlk, key.p, false);
        radix_sort_pairs<uint64_t>(key.p, lids.p, nlk, 0, 64, s);
        hipLaunchKernelGGL(k_ct_key, G(nlk), dim3(B), 0, s, (const Digest*)a_ct.p, (const uint32_t*)lids.p, nlk, key.p, true);
        radix_sort_pairs<uint64_t>(key.p, lids.p, nlk, 0, 64, s);
      }
      DBuf<uint32_t> f(nlk, s), sc(nlk, s);
      {
        KScope ks("k_first_flags", 24.0 * nlk);
        hipLaunchKernelGGL(k_first_flags, G(nlk), dim3(B), 0, s, dig_s(a_ct.p), (const uint32_t*)lids.p, nlk, f.p);
      }
      exclusive_scan<uint32_t>(f.p, nlk, sc.p, s);
      n_ctypes = (uint64_t)read_u32(sc.p + nlk - 1, s) + read_u32(f.p + nlk - 1, s);
      {
        KScope ks("k_set_ctype", 16.0 * nlk);
        hipLaunchKernelGGL(k_set_ctype, G(nlk), dim3(B), 0, s, (const uint32_t*)lids.p, (const uint32_t*)f.p,
                           (const uint32_t*)sc.p, nlk, idx.ctype);
      }
      DBuf<Digest> u(n_ctypes, s);
      hipLaunchKernelGGL(k_ct_unique, G(nlk), dim3(B), 0, s, (const Digest*)a_ct.p, (const uint32_t*)lids.p,
                         (const uint32_t*)f.p, (const uint32_t*)sc.p, nlk, u.p);
      idx.ctype_digest.resize(n_ctypes);
      DAS_HIP(hipMemcpyAsync(idx.ctype_digest.data(), u.p, sizeof(Digest) * n_ctypes, hipMemcpyDeviceToHost, s));
      DAS_HIP(hipStreamSynchronize(s));
      DAS_HIP(hipGetLastError());
    }
  }
  a_ct.release();
  idx.ctype_range.assign(n_ctypes, CtypeRange{0, 0, 0});

  // 7. per-arity tables
  phase.emplace(c, "phase_tables", 0.0);
  const uint64_t mirror_max = host_key_mirror_max();
  for (uint32_t ar = 1; ar <= (uint32_t)kMaxArity; ++ar) {
    if (!links_of_arity[ar]) continue;        // no link of this arity (step 5's counts): no flag pass
    DBuf<uint32_t> lf(n_atoms ? n_atoms : 1, s), ids;
    if (n_atoms) {
      KScope ks("k_link_flags", 9.0 * n_atoms);
      hipLaunchKernelGGL(k_link_flags, G(n_atoms), dim3(B), 0, s, (const uint8_t*)idx.cat,
                         (const uint32_t*)idx.arity, n_atoms, ar, lf.p);
    }
    const uint64_t R = compact_flags(lf.p, n_atoms, ids, s);
    lf.release();
    if (!R) continue;
    const int tbits = bits_for(a.n_types ? a.n_types - 1 : 0);
    // T_a by (type, id)
    {
      DBuf<uint32_t> key(R, s), perm(R, s);
      copy_dev(perm.p, ids.p, 4 * R, s);
      {
        KScope ks("k_u32_key", 12.0 * R);
        hipLaunchKernelGGL(k_u32_key, G(R), dim3(B), 0, s, (const uint32_t*)idx.type, (const uint32_t*)perm.p, R, key.p);
      }
      // no sort: final ids are clustered by named type (step 3b) and T_a
      // holds links only, so the arity's link ids in ascending order are
      // already in (type, id) order (a kNone type would sort last: none is a link)
      (void)tbits;
      RowTable& t = idx.ttab[ar];
      t.arity = (int)ar;
      t.rows = R;
      t.ld = col_stride(R);
      t.data = dalloc<uint32_t>(idx, (uint64_t)(ar + 1) * t.ld);
      {
        // id in, its target offset and targets gathered, (id, targets) row out
        KScope ks("k_gather_rows", 4.0 * R + 8.0 * R + 4.0 * ar * R + 4.0 * (ar + 1) * R);
        hipLaunchKernelGGL(k_gather_rows, G(R), dim3(B), 0, s, (const uint32_t*)perm.p, R, t.ld, ar,
                           (const uint64_t*)idx.tgt_off, (const uint32_t*)idx.tgt, t.data);
      }
      // host type offsets
      uint32_t* ukey; uint64_t* uoff;
      const uint64_t m = rle<uint32_t>(key.p, R, &ukey, &uoff, idx, s);
      std::vector<uint32_t> hk(m);
      std::vector<uint64_t> ho(m + 1);
      DAS_HIP(hipMemcpyAsync(hk.data(), ukey, 4 * m, hipMemcpyDeviceToHost, s));
      DAS_HIP(hipMemcpyAsync(ho.data(), uoff, 8 * (m + 1), hipMemcpyDeviceToHost, s));
      DAS_HIP(hipStreamSynchronize(s));
      auto& to = idx.type_off[ar];
      to.assign(a.n_types + 1, 0);
      // to[t] = first row with type >= t
      uint64_t r = 0;
      for (uint32_t ty = 0; ty <= a.n_types; ++ty) {
        while (r < m && hk[r] < ty) ++r;
        to[ty] = r < m ? ho[r] : R;
      }
      col_bounds(idx, t, a.n_types, s);
    }
    // C_a by (ctype, id)
    {
      DBuf<uint32_t> key(R, s), perm(R, s);
      copy_dev(perm.p, ids.p, 4 * R, s);
      {
        KScope ks("k_u32_key", 12.0 * R);
        hipLaunchKernelGGL(k_u32_key, G(R), dim3(B), 0, s, (const uint32_t*)idx.ctype, (const uint32_t*)perm.p, R, key.p);
      }
      const int cbits = bits_for(n_ctypes ? n_ctypes - 1 : 0);
      if (!keys_sorted(key.p, R, s)) radix_sort_pairs<uint32_t>(key.p, perm.p, R, 0, cbits > 0 ? cbits : 1, s);
      RowTable& t = idx.ctab[ar];
      t.arity = (int)ar;
      t.rows = R;
      t.ld = col_stride(R);
      t.data = dalloc<uint32_t>(idx, (uint64_t)(ar + 1) * t.ld);
      {
        // id in, its target offset and targets gathered, (id, targets) row out
        KScope ks("k_gather_rows", 4.0 * R + 8.0 * R + 4.0 * ar * R + 4.0 * (ar + 1) * R);
        hipLaunchKernelGGL(k_gather_rows, G(R), dim3(B), 0, s, (const uint32_t*)perm.p, R, t.ld, ar,
                           (const uint64_t*)idx.tgt_off, (const uint32_t*)idx.tgt, t.data);
      }
      uint32_t* ukey; uint64_t* uoff;
      const uint64_t m = rle<uint32_t>(key.p, R, &ukey, &uoff, idx, s);
      std::vector<uint32_t> hk(m);
      std::vector<uint64_t> ho(m + 1);
      DAS_HIP(hipMemcpyAsync(hk.data(), ukey, 4 * m, hipMemcpyDeviceToHost, s));
      DAS_HIP(hipMemcpyAsync(ho.data(), uoff, 8 * (m + 1), hipMemcpyDeviceToHost, s));
      DAS_HIP(hipStreamSynchronize(s));
      for (uint64_t r = 0; r < m; ++r) idx.ctype_range[hk[r]] = CtypeRange{ar, ho[r], ho[r + 1]};
    }
    // P_{a,p}
    const bool packed = !(std::getenv("DAS_PIDX_PERM") && std::getenv("DAS_PIDX_PERM")[0] == '1') &&
                        idx.type_off[ar].size() == a.n_types + 1 && idx.type_off[ar][a.n_types] == R;
    if (ar <= (uint32_t)kMaxPosArity && packed) {
      const RowTable& T = idx.ttab[ar];
      const auto& to = idx.type_off[ar];
      const auto& tb = idx.tbound[ar];
      const uint32_t ncol = ar + 1;
      for (uint32_t p = 0; p < ar; ++p) {
        PosIndex& P = idx.pidx[ar][p];
        P.t.arity = (int)ar;
        P.t.rows = R;
        P.t.ld = col_stride(R);
        P.t.data = dalloc<uint32_t>(idx, (uint64_t)(ar + 1) * P.t.ld);
        DBuf<uint64_t> pk(R, s);
        // p > 0: from P_{a,0}'s rows (DAS_PIDX_DERIVE=0: each P_{a,p} sorted
        // from the type table on its full key, A/B)
        const char* dv = std::getenv("DAS_PIDX_DERIVE");
        const bool derive = p > 0 && (ar == 2 || ar == 3) && !(dv && dv[0] == '0');
        const PosIndex& P0 = idx.pidx[ar][0];
        for (uint32_t ty = 0; ty < a.n_types && derive; ++ty) {
          const uint64_t b = to[ty], n = to[ty + 1] - to[ty];
          if (!n) continue;
          const uint32_t lo = tb[((uint64_t)ty * ncol + 1 + p) * 2];
          const uint32_t bits = (uint32_t)bits_for(tb[((uint64_t)ty * ncol + 1 + p) * 2 + 1] - lo);
          DAS_CHECK(n < (1ull << 32), DAS_E_UNSUPPORTED, "pattern index: a type segment of 2^32 links");
          DBuf<uint64_t> key(n, s);
          DBuf<uint32_t> val(n, s);
          {
            KScope ks("k_derive_key", 4.0 * (ar == 2 ? 3 : 2) * n + 12.0 * n);
            hipLaunchKernelGGL(k_derive_key, G(n), dim3(B), 0, s, (const uint32_t*)P0.t.data, P0.t.ld, b, n, ar, p, lo,
                               key.p, val.p);
          }
          if (bits) radix_sort_pairs<uint64_t>(key.p, val.p, n, 32, 32 + (int)bits, s);
          {
            KScope ks("k_derive_unpack", 12.0 * n + 4.0 * (ar + 1) * n + 8.0 * n + (ar == 3 ? 8.0 * n : 0.0));
            hipLaunchKernelGGL(k_derive_unpack, G(n), dim3(B), 0, s, (const uint64_t*)key.p, (const uint32_t*)val.p, n,
                               ar, p, lo, ty, (const uint32_t*)P0.t.data, P0.t.ld, b, P.t.data, P.t.ld, pk.p);
          }
          DAS_HIP(hipGetLastError());
        }
        for (uint32_t ty = 0; ty < a.n_types && !derive; ++ty) {
          const uint64_t b = to[ty], n = to[ty + 1] - to[ty];
          if (!n) continue;
          // fields: t_p, then the other positions in order
          uint32_t pos[3], nf = 0;
          pos[nf++] = p;
          for (uint32_t q = 0; q < ar; ++q)
            if (q != p) pos[nf++] = q;
          uint32_t lo[3], bits[3], total = 0;
          for (uint32_t j = 0; j < nf; ++j) {
            lo[j] = tb[((uint64_t)ty * ncol + 1 + pos[j]) * 2];
            bits[j] = (uint32_t)bits_for(tb[((uint64_t)ty * ncol + 1 + pos[j]) * 2 + 1] - lo[j]);
            total += bits[j];
          }
          // a key wider than 64 bits (arity 3): the last field is sorted
          // first on its own (LSD), the rest carry the segment row
          const bool force_two = std::getenv("DAS_PIDX_TWO") && std::getenv("DAS_PIDX_TWO")[0] == '1';
          const bool two = total > 64 || (nf == 3 && force_two);      // (tests: DAS_PIDX_TWO=1)
          PackKey f{};
          f.n = two ? nf - 1 : nf;
          uint32_t sh = 0;
          for (int j = (int)f.n - 1; j >= 0; --j) {
            f.pos[j] = pos[j];
            f.lo[j] = lo[j];
            f.bits[j] = bits[j];
            f.sh[j] = sh;
            sh += bits[j];
          }
          DBuf<uint64_t> key(n, s);
          DBuf<uint32_t> val(n, s);
          if (two) {
            DBuf<uint32_t> k32(n, s);
            {
              KScope ks("k_pack_key32", 12.0 * n);
              hipLaunchKernelGGL(k_pack_key32, G(n), dim3(B), 0, s, (const uint32_t*)T.col(1 + pos[nf - 1]), b, n,
                                 lo[nf - 1], k32.p, val.p);
            }
            radix_sort_pairs<uint32_t>(k32.p, val.p, n, 0, std::max(1u, bits[nf - 1]), s);
          }
          {
            // fields in, key (+ link id) out; stage 2 gathers its fields at the sorted rows
            KScope ks("k_pack_key", (two ? 12.0 : 12.0) * n + 4.0 * f.n * n);
            hipLaunchKernelGGL(k_pack_key, G(n), dim3(B), 0, s, (const uint32_t*)T.data, T.ld, b, n, f,
                               two ? (const uint32_t*)val.p : nullptr, key.p, val.p);
          }
          if (sh) radix_sort_pairs<uint64_t>(key.p, val.p, n, 0, (int)sh, s);
          {
            KScope ks("k_unpack_key", 12.0 * n + 4.0 * (ar + 1) * n + 8.0 * n);
            hipLaunchKernelGGL(k_unpack_key, G(n), dim3(B), 0, s, (const uint64_t*)key.p, (const uint32_t*)val.p, n,
                               f, two ? (int32_t)pos[nf - 1] : -1, (const uint32_t*)T.data, T.ld, b, ty, P.t.data,
                               P.t.ld, b, pk.p);
          }
          DAS_HIP(hipGetLastError());
        }
        P.nkeys = rle<uint64_t>(pk.p, R, &P.ukey, &P.uoff, idx, s);
        build_key_dir(P, idx, s);
        if (P.nkeys <= mirror_max) {
          P.h_ukey.resize(P.nkeys);
          P.h_uoff.resize(P.nkeys + 1);
          DAS_HIP(hipMemcpyAsync(P.h_ukey.data(), P.ukey, 8 * P.nkeys, hipMemcpyDeviceToHost, s));
          DAS_HIP(hipMemcpyAsync(P.h_uoff.data(), P.uoff, 8 * (P.nkeys + 1), hipMemcpyDeviceToHost, s));
          DAS_HIP(hipStreamSynchronize(s));
        }
      }
    } else if (ar <= (uint32_t)kMaxPosArity) {
      // permutation path (links of no named type present, or DAS_PIDX_PERM=1)
      for (uint32_t p = 0; p < ar; ++p) {
        DBuf<uint64_t> key(R, s);
        DBuf<uint32_t> perm(R, s);
        copy_dev(perm.p, ids.p, 4 * R, s);
        // secondary order by the other targets in position order (LSD: least
        // significant key first), so an anchored range of P_{a,p} comes out
        // sorted by its first non-grounded other target and can be a join's
        // build side without a sort
        for (int q = (int)ar - 1; q >= 0; --q) {
          if ((uint32_t)q == p) continue;
          DBuf<uint32_t> k2(R, s);
          {
            KScope ks("k_tgt_key", 20.0 * R);
            hipLaunchKernelGGL(k_tgt_key, G(R), dim3(B), 0, s, (const uint64_t*)idx.tgt_off, (const uint32_t*)idx.tgt,
                               (const uint32_t*)perm.p, R, (uint32_t)q, k2.p);
          }
          radix_sort_pairs<uint32_t>(k2.p, perm.p, R, 0, std::max(1, bits_for(n_atoms ? n_atoms - 1 : 0)), s);
        }
        {
          KScope ks("k_pos_key", 28.0 * R);
          hipLaunchKernelGGL(k_pos_key, G(R), dim3(B), 0, s, (const uint32_t*)idx.type, (const uint64_t*)idx.tgt_off,
                             (const uint32_t*)idx.tgt, (const uint32_t*)perm.p, R, p, key.p);
        }
        // (type, t_p, t_q, id): sort by t_p, then (stable) by type
        radix_sort_pairs<uint64_t>(key.p, perm.p, R, 0, std::max(1, bits_for(n_atoms ? n_atoms - 1 : 0)), s);
        radix_sort_pairs<uint64_t>(key.p, perm.p, R, 32, 32 + std::max(1, tbits), s);
        PosIndex& P = idx.pidx[ar][p];
        P.t.arity = (int)ar;
        P.t.rows = R;
        P.t.ld = col_stride(R);
        P.t.data = dalloc<uint32_t>(idx, (uint64_t)(ar + 1) * P.t.ld);
        {
          KScope ks("k_gather_rows", 4.0 * R + 8.0 * R + 4.0 * ar * R + 4.0 * (ar + 1) * R);
          hipLaunchKernelGGL(k_gather_rows, G(R), dim3(B), 0, s, (const uint32_t*)perm.p, R, P.t.ld, ar,
                             (const uint64_t*)idx.tgt_off, (const uint32_t*)idx.tgt, P.t.data);
        }
        P.nkeys = rle<uint64_t>(key.p, R, &P.ukey, &P.uoff, idx, s);
        build_key_dir(P, idx, s);
        if (P.nkeys <= mirror_max) {
          // host copy of the unique keys and offsets: an anchored scan finds
          // its key range without a device round trip
          P.h_ukey.resize(P.nkeys);
          P.h_uoff.resize(P.nkeys + 1);
          DAS_HIP(hipMemcpyAsync(P.h_ukey.data(), P.ukey, 8 * P.nkeys, hipMemcpyDeviceToHost, s));
          DAS_HIP(hipMemcpyAsync(P.h_uoff.data(), P.uoff, 8 * (P.nkeys + 1), hipMemcpyDeviceToHost, s));
          DAS_HIP(hipStreamSynchronize(s));
        }
      }
    }
    DAS_HIP(hipGetLastError());
  }
  phase.reset();
  idx.h_node_dig.clear();
  idx.h_node_id.clear();
  idx.h_node_type.clear();
  if (idx.n_nodes && idx.n_nodes <= kHostNodeMirror && idx.n_atoms < 0xFFFFFFFFull) {
    const uint64_t n = idx.n_atoms;
    DBuf<uint32_t> flag(n, s), pos(n + 1, s);
    {
      KScope ks("k_node_flags", 9.0 * n);
      hipLaunchKernelGGL(k_node_flags, G(n), dim3(B), 0, s, n, (const uint32_t*)idx.by_digest,
                         (const uint8_t*)idx.cat, flag.p);
    }
    const uint64_t nn = scan_total<uint32_t>(SpanIn<uint32_t>{flag.p}, n, pos.p, s);
    if (nn) {
      DBuf<Digest> od(nn, s);
      DBuf<uint32_t> oi(nn, s), ot(nn, s);
      {
        KScope ks("k_node_pack", 9.0 * n + 24.0 * nn);
        hipLaunchKernelGGL(k_node_pack, G(n), dim3(B), 0, s, n, (const uint32_t*)idx.by_digest,
                           (const uint8_t*)idx.cat, (const uint32_t*)pos.p, (const Digest*)idx.digest,
                           (const uint32_t*)idx.type, od.p, oi.p, ot.p);
      }
      idx.h_node_dig.resize(nn);
      idx.h_node_id.resize(nn);
      idx.h_node_type.resize(nn);
      DAS_HIP(hipMemcpyAsync(idx.h_node_dig.data(), od.p, sizeof(Digest) * nn, hipMemcpyDeviceToHost, s));
      DAS_HIP(hipMemcpyAsync(idx.h_node_id.data(), oi.p, 4 * nn, hipMemcpyDeviceToHost, s));
      DAS_HIP(hipMemcpyAsync(idx.h_node_type.data(), ot.p, 4 * nn, hipMemcpyDeviceToHost, s));
      DAS_HIP(hipStreamSynchronize(s));
    }
  }
  DAS_HIP(hipStreamSynchronize(s));
  idx.built = true;
}

namespace {
// Handle lookups through pinned staging (one workgroup; small batches):
// the request digests are read over the host mapping, each result is
// stored to the host with system scope, then the slot is released.
// out[2i] = id (-1: absent), out[2i + 1] = category | arity << 8 | type << 32
__global__ void __launch_bounds__(256) k_lookup_pub(const Digest* dig, const uint32_t* by_digest, const uint8_t* cat,
                                                    const uint32_t* arity, const uint32_t* type, uint64_t n_atoms,
                                                    const Digest* q, uint64_t nq, int64_t* out, uint32_t* slot,
                                                    uint32_t seq) {
  for (uint64_t i = threadIdx.x; i < nq; i += blockDim.x) {
    const uint64_t qh = q[i].hi(), ql = q[i].lo();
    uint64_t lo = 0, hi = n_atoms;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      const Digest d = dig[by_digest[mid]];
      const uint64_t dh = d.hi(), dl = d.lo();
      if (dh < qh || (dh == qh && dl < ql)) lo = mid + 1;
      else hi = mid;
    }
    int64_t r = -1, info = (int64_t)kNone << 32;
    if (lo < n_atoms) {
      const uint32_t id = by_digest[lo];
      const Digest d = dig[id];
      if (d.hi() == qh && d.lo() == ql) {
        r = (int64_t)id;
        info = (int64_t)((uint64_t)cat[id] | ((uint64_t)(arity[id] & 0xFFFFFFu) << 8) | ((uint64_t)type[id] << 32));
      }
    }
    __hip_atomic_store(&out[2 * i], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&out[2 * i + 1], info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(&slot[15], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace

bool lookup_small(Ctx& c, const Digest* h, uint64_t n, int64_t* out, uint8_t* cat, uint32_t* arity, uint32_t* type) {
  DAS_CHECK(c.idx.built, DAS_E_NOT_BUILT, "index not built");
  if (n > 4096) return false;
  if (!n) return true;
  {
    // every digest a node of the host mirror: answered on the host
    const auto& nd = c.idx.h_node_dig;
    auto less = [](const Digest& a, const Digest& b) {
      return a.hi() < b.hi() || (a.hi() == b.hi() && a.lo() < b.lo());
    };
    uint64_t i = 0;
    for (; i < n && !nd.empty(); ++i) {
      const size_t j = std::lower_bound(nd.begin(), nd.end(), h[i], less) - nd.begin();
      if (j == nd.size() || nd[j].hi() != h[i].hi() || nd[j].lo() != h[i].lo()) break;
      out[i] = c.idx.h_node_id[j];
      if (cat) cat[i] = CAT_NODE;
      if (arity) arity[i] = 0;
      if (type) type[i] = c.idx.h_node_type[j];
    }
    if (i == n) return true;
  }
  uint8_t* st = pinned_stage(n * (sizeof(Digest) + 16));
  Digest* q = reinterpret_cast<Digest*>(st);
  int64_t* r = reinterpret_cast<int64_t*>(st + n * sizeof(Digest));
  std::memcpy(q, h, n * sizeof(Digest));
  const Index& x = c.idx;
  const PubSlot ps = pub_reserve();
  hipLaunchKernelGGL(k_lookup_pub, dim3(1), dim3(256), 0, c.s, (const Digest*)x.digest, (const uint32_t*)x.by_digest,
                     (const uint8_t*)x.cat, (const uint32_t*)x.arity, (const uint32_t*)x.type, x.n_atoms,
                     (const Digest*)q, n, r, ps.p, ps.seq);
  DAS_HIP(hipGetLastError());
  pub_wait(ps, c.s, nullptr, 0);
  for (uint64_t i = 0; i < n; ++i) {
    out[i] = r[2 * i];
    const uint64_t info = (uint64_t)r[2 * i + 1];
    if (cat) cat[i] = (uint8_t)(info & 0xFF);
    if (arity) arity[i] = (uint32_t)((info >> 8) & 0xFFFFFF);
    if (type) type[i] = (uint32_t)(info >> 32);
  }
  return true;
}

void lookup_digests(Ctx& c, const Digest* h, uint64_t n, int64_t* out) {
  DAS_CHECK(c.idx.built, DAS_E_NOT_BUILT, "index not built");
  if (!n) return;
  auto q = upload(h, n, c.s);
  DBuf<int64_t> r(n, c.s);
  hipLaunchKernelGGL(k_lookup, G(n), dim3(B), 0, c.s, (const Digest*)c.idx.digest, (const uint32_t*)c.idx.by_digest,
                     c.idx.n_atoms, (const Digest*)q.p,
                     n, r.p);
  DAS_HIP(hipGetLastError());
  DAS_HIP(hipMemcpyAsync(out, r.p, 8 * n, hipMemcpyDeviceToHost, c.s));
  DAS_HIP(hipStreamSynchronize(c.s));
}

}  // namespace das
