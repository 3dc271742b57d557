// Query operators over the HBM index: Link / LinkTemplate scans with fused
// variable assignment, ordered natural join, anti-join, set dedup.
//
// Reference semantics (das/pattern_matcher/pattern_matcher.py):
//   scan      Link.matched :502-538 -> RedisMongoDB.get_matched_links
//             (redis_mongo_db.py:235-252) -> Link._assign_variables :466-489
//   template  LinkTemplate.matched :603-614 / _assign_variables :591-601
//   join      OrderedAssignment.join/_join_ordered/evaluate_compatibility
//             :105-153 == natural join on the shared variables
//   antijoin  And.matched :741-746 with OrderedAssignment.check_negation
//             :112-117 (a row is dropped iff a forbidden mapping is a subset)
//   dedup     Python set semantics of PatternMatchingAnswer.assignments
//
// Kernels are wave64 ballot/popcount compactions; counts go through a
// per-block two-pass (count -> scan -> write) so output order is the input
// order (deterministic) and no global atomics sit on the hot path.
#include <algorithm>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <optional>
#include <string>

#include "das_internal.h"

namespace das {

__global__ void k_compact_index_q(const uint32_t* flag, const uint32_t* scan, uint64_t n, uint32_t* out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (flag[i]) out[scan[i]] = (uint32_t)i;
}

namespace {

struct FlagIn {
  const uint32_t* a;
  uint64_t n;
  __device__ uint32_t operator()(uint64_t i) const { return i < n ? a[i] : 0u; }
};

struct WidenCnt {
  const uint32_t* a;
  uint64_t n;
  __device__ uint64_t operator()(uint64_t i) const { return i < n ? (uint64_t)a[i] : 0ull; }
};

constexpr unsigned B = 256;
constexpr int kChunkIters = 16;                 // rows per thread per block chunk
constexpr uint64_t kChunk = (uint64_t)B * kChunkIters;
inline dim3 G(uint64_t n) { return dim3(grid_for(n, B)); }

// ---------------------------------------------------------------------------
// Scan spec (device, by value)
// ---------------------------------------------------------------------------
struct ScanSpec {
  const uint32_t* col[kMaxArity + 1];  // col[0] = link id, col[1+k] = target k
  uint32_t arity;
  uint32_t fixed[kMaxArity];           // kNone = no filter
  int32_t outpos[kMaxCols];            // ordered: source position of out col (-1 link)
  uint32_t nout;
  uint32_t eq_a[kMaxArity], eq_b[kMaxArity], neq;
  uint32_t no_overload;
  uint32_t unordered;
  uint32_t upos[kMaxArity], nupos;     // unordered: wildcard positions
  uint32_t emit_link;
  uint32_t all_keep;                   // no predicate at all (pure projection)
};

__device__ __forceinline__ bool scan_keep(const ScanSpec& sp, uint64_t r) {
  if (sp.all_keep) return true;
  for (uint32_t p = 0; p < sp.arity; ++p)
    if (sp.fixed[p] != kNone && sp.col[1 + p][r] != sp.fixed[p]) return false;
  for (uint32_t e = 0; e < sp.neq; ++e)
    if (sp.col[1 + sp.eq_a[e]][r] != sp.col[1 + sp.eq_b[e]][r]) return false;
  if (sp.unordered) {
    for (uint32_t i = 0; i < sp.nupos; ++i)
      for (uint32_t j = i + 1; j < sp.nupos; ++j)
        if (sp.col[1 + sp.upos[i]][r] == sp.col[1 + sp.upos[j]][r]) return false;
  } else if (sp.no_overload) {
    const uint32_t base = sp.emit_link ? 1 : 0;
    for (uint32_t i = base; i < sp.nout; ++i)
      for (uint32_t j = i + 1; j < sp.nout; ++j)
        if (sp.col[1 + sp.outpos[i]][r] == sp.col[1 + sp.outpos[j]][r]) return false;
  }
  return true;
}

__device__ __forceinline__ void scan_emit(const ScanSpec& sp, uint64_t r, uint32_t* out, uint64_t cap, uint64_t pos) {
  if (!sp.unordered) {
    for (uint32_t c = 0; c < sp.nout; ++c) out[c * cap + pos] = sp.col[1 + sp.outpos[c]][r];
    return;
  }
  uint32_t c0 = 0;
  if (sp.emit_link) { out[pos] = sp.col[0][r]; c0 = 1; }
  uint32_t v[kMaxArity];
  for (uint32_t i = 0; i < sp.nupos; ++i) v[i] = sp.col[1 + sp.upos[i]][r];
  for (uint32_t i = 1; i < sp.nupos; ++i) {       // insertion sort, <= 8 values
    uint32_t x = v[i];
    int j = (int)i - 1;
    while (j >= 0 && v[j] > x) { v[j + 1] = v[j]; --j; }
    v[j + 1] = x;
  }
  for (uint32_t i = 0; i < sp.nupos; ++i) out[(c0 + i) * cap + pos] = v[i];
}

__global__ void __launch_bounds__(B) k_scan_count(ScanSpec sp, uint64_t begin, uint64_t end, uint32_t* chunk_cnt) {
  __shared__ uint32_t s_w[B / 64];
  const uint64_t cb = begin + (uint64_t)blockIdx.x * kChunk;
  uint32_t cnt = 0;
  for (int it = 0; it < kChunkIters; ++it) {
    const uint64_t r = cb + (uint64_t)it * B + threadIdx.x;
    if (r < end && scan_keep(sp, r)) ++cnt;
  }
  cnt = wave_reduce_sum(cnt);
  if (__lane_id() == 0) s_w[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) chunk_cnt[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

__global__ void __launch_bounds__(B) k_scan_write(ScanSpec sp, uint64_t begin, uint64_t end, const uint32_t* chunk_off,
                                                  uint32_t* out, uint64_t cap) {
  __shared__ uint32_t s_w[B / 64];
  __shared__ uint32_t s_run;
  const uint64_t cb = begin + (uint64_t)blockIdx.x * kChunk;
  const int wave = threadIdx.x >> 6;
  const uint64_t lt = __lanemask_lt();
  if (threadIdx.x == 0) s_run = chunk_off ? chunk_off[blockIdx.x] : (uint32_t)(cb - begin);
  __syncthreads();
  for (int it = 0; it < kChunkIters; ++it) {
    const uint64_t r = cb + (uint64_t)it * B + threadIdx.x;
    const bool keep = r < end && scan_keep(sp, r);
    const uint64_t m = __ballot(keep);
    if (__lane_id() == 0) s_w[wave] = __popcll(m);
    __syncthreads();
    uint32_t pos = s_run + __popcll(m & lt);
    for (int w = 0; w < wave; ++w) pos += s_w[w];
    if (keep) scan_emit(sp, r, out, cap, pos);
    __syncthreads();
    if (threadIdx.x == 0) s_run += s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
  }
}

// Several scans with one output schema in one pass (Or's union of Link
// terms): segment s = (spec, row range), its chunks numbered from chunk0;
// block b scans chunk b of the segment that holds it.  Specs by value.
constexpr int kMultiSeg = 6;
struct MultiScan {
  uint32_t nseg;
  struct Seg {
    ScanSpec sp;
    uint64_t begin, end, chunk0;
  } seg[kMultiSeg];
};

__device__ __forceinline__ const MultiScan::Seg& seg_of(const MultiScan& ms, uint32_t b) {
  uint32_t s = 0;
  while (s + 1 < ms.nseg && ms.seg[s + 1].chunk0 <= b) ++s;
  return ms.seg[s];
}

__global__ void __launch_bounds__(B) k_scan_count_multi(MultiScan ms, uint32_t* chunk_cnt) {
  __shared__ uint32_t s_w[B / 64];
  const MultiScan::Seg& sg = seg_of(ms, blockIdx.x);
  const uint64_t cb = sg.begin + (uint64_t)(blockIdx.x - sg.chunk0) * kChunk;
  uint32_t cnt = 0;
  for (int it = 0; it < kChunkIters; ++it) {
    const uint64_t r = cb + (uint64_t)it * B + threadIdx.x;
    if (r < sg.end && scan_keep(sg.sp, r)) ++cnt;
  }
  cnt = wave_reduce_sum(cnt);
  if (__lane_id() == 0) s_w[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) chunk_cnt[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

__global__ void __launch_bounds__(B) k_scan_write_multi(MultiScan ms, const uint32_t* chunk_off, uint32_t* out,
                                                        uint64_t cap) {
  __shared__ uint32_t s_w[B / 64];
  __shared__ uint32_t s_run;
  const MultiScan::Seg& sg = seg_of(ms, blockIdx.x);
  const uint64_t cb = sg.begin + (uint64_t)(blockIdx.x - sg.chunk0) * kChunk;
  const int wave = threadIdx.x >> 6;
  const uint64_t lt = __lanemask_lt();
  if (threadIdx.x == 0) s_run = chunk_off[blockIdx.x];
  __syncthreads();
  for (int it = 0; it < kChunkIters; ++it) {
    const uint64_t r = cb + (uint64_t)it * B + threadIdx.x;
    const bool keep = r < sg.end && scan_keep(sg.sp, r);
    const uint64_t m = __ballot(keep);
    if (__lane_id() == 0) s_w[wave] = __popcll(m);
    __syncthreads();
    uint32_t pos = s_run + __popcll(m & lt);
    for (int w = 0; w < wave; ++w) pos += s_w[w];
    if (keep) scan_emit(sg.sp, r, out, cap, pos);
    __syncthreads();
    if (threadIdx.x == 0) s_run += s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
  }
}

// Single-workgroup scan of a small range (an anchored key range): count,
// compaction and column writes in one launch, the row count published
// straight into the pinned read-back slot (one launch + one round trip where
// k_scan_count -> scan_total -> k_scan_write take three launches).  The
// output table is sized by the range (an upper bound of the kept rows).
constexpr int kSmallBlock = 1024;
constexpr uint64_t kSmallScan = 16384;

__device__ __forceinline__ void publish_u32(uint32_t* slot, uint32_t seq, uint32_t v) {
  __hip_atomic_store(&slot[0], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __threadfence_system();
  __hip_atomic_store(&slot[15], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Or of one-column scans (FlyBase's DO-term Or): the union's distinct values
// in ONE launch.  Each scanned row that passes its scan's predicate (the
// grounded targets outside the key range) tests and sets its value's bit in
// a bitmap over the column's host-known id range; the row that set it
// writes the value, at a position its block reserves with one atomic (output
// unsorted, one row per distinct value -- Python set semantics).  One row
// per thread (the segments are chunked by B rows, not kChunk): a block's
// load -> test-and-set -> reserve chain runs once, so the launch is as deep
// as one chain instead of kChunkIters of them (F9: 71 -> ~15 us).  ctr[0]:
// rows written, ctr[1]: blocks done, ctr[2]: values outside [lo, lo + range)
// (the host then takes the general path); the last block publishes ctr[0]
// and ctr[2].
__global__ void __launch_bounds__(B) k_union_first(MultiScan ms, uint32_t lo, uint32_t range,
                                                   uint32_t* __restrict__ bits, uint32_t* __restrict__ out,
                                                   uint32_t* __restrict__ ctr, uint32_t* slot, uint32_t seq) {
  __shared__ uint32_t s_w[B / 64];
  __shared__ uint32_t s_base;
  const MultiScan::Seg& sg = seg_of(ms, blockIdx.x);
  const uint64_t r = sg.begin + (uint64_t)(blockIdx.x - sg.chunk0) * B + threadIdx.x;
  const uint32_t* src = sg.sp.col[1 + sg.sp.outpos[0]];
  const int wave = threadIdx.x >> 6;
  uint32_t bad = 0;
  bool first = false;
  uint32_t v = 0;
  if (r < sg.end && scan_keep(sg.sp, r)) {
    v = src[r];
    const uint32_t d = v - lo;
    if (d < range) {
      const uint32_t m = 1u << (d & 31);
      first = (atomicOr(&bits[d >> 5], m) & m) == 0;
    } else {
      bad = 1;
    }
  }
  const uint64_t bal = __ballot(first);
  if (__lane_id() == 0) s_w[wave] = (uint32_t)__popcll(bal);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < B / 64; ++w) t += s_w[w];
    s_base = t ? atomicAdd(&ctr[0], t) : 0u;
  }
  __syncthreads();
  uint32_t pos = s_base + (uint32_t)__popcll(bal & __lanemask_lt());
  for (int w = 0; w < wave; ++w) pos += s_w[w];
  if (first) out[pos] = v;
  if (__ballot(bad) && __lane_id() == 0) atomicOr(&ctr[2], 1u);
  __syncthreads();
  // arrival without an agent-scope release (on gfx950 each one writes this
  // XCD's L2 back; one per block serialised ~2.5 us a block per XCD): the
  // rows are read by later launches only, the last block reads counters,
  // atomics performed at the coherence point once this thread's are done
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (atomicAdd(&ctr[1], 1u) == gridDim.x - 1)
      publish_u32(slot, seq, atomicAdd(&ctr[2], 0u) ? 0xFFFFFFFFu : atomicAdd(&ctr[0], 0u));
  }
}


__global__ void __launch_bounds__(kSmallBlock) k_scan_small(ScanSpec sp, uint64_t begin, uint64_t end, uint32_t* out,
                                                            uint64_t cap, uint32_t* slot, uint32_t seq) {
  constexpr int W = kSmallBlock / 64;
  __shared__ uint32_t s_w[W];
  __shared__ uint32_t s_run;
  const int wave = threadIdx.x >> 6;
  const uint64_t lt = __lanemask_lt();
  if (threadIdx.x == 0) s_run = 0;
  __syncthreads();
  for (uint64_t r0 = begin; r0 < end; r0 += kSmallBlock) {
    const uint64_t r = r0 + threadIdx.x;
    const bool keep = r < end && scan_keep(sp, r);
    const uint64_t m = __ballot(keep);
    if (__lane_id() == 0) s_w[wave] = __popcll(m);
    __syncthreads();
    uint32_t pos = s_run + __popcll(m & lt);
    for (int w = 0; w < wave; ++w) pos += s_w[w];
    if (keep) scan_emit(sp, r, out, cap, pos);
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (int w = 0; w < W; ++w) t += s_w[w];
      s_run += t;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) publish_u32(slot, seq, s_run);
}

// Pure projection (a scan with no predicate): out column c = source column
// outpos[c] over [begin, end).  Output columns are 16-byte aligned (table
// column strides are multiples of 64 rows); a source column is too when
// `begin` is a multiple of 4, then 16-byte lanes, two in flight per thread;
// otherwise 4-byte lanes, four in flight (each load instruction still covers
// 256 contiguous bytes per wave).
__global__ void __launch_bounds__(B) k_project(ScanSpec sp, uint64_t begin, uint64_t n, uint32_t* out, uint64_t cap) {
  const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint32_t c = 0; c < sp.nout; ++c) {
    const uint32_t* __restrict__ src = sp.col[1 + sp.outpos[c]] + begin;
    uint32_t* __restrict__ dst = out + c * cap;
    if (((((uintptr_t)src) | ((uintptr_t)dst)) & 15) == 0) {
      const uint64_t n4 = n >> 2;
      const uint4* s4 = reinterpret_cast<const uint4*>(src);
      uint4* d4 = reinterpret_cast<uint4*>(dst);
      uint64_t i = tid;
      for (; i + stride < n4; i += 2 * stride) {
        const uint4 a = s4[i], b = s4[i + stride];
        d4[i] = a;
        d4[i + stride] = b;
      }
      if (i < n4) d4[i] = s4[i];
      for (uint64_t j = (n4 << 2) + tid; j < n; j += stride) dst[j] = src[j];
    } else {
      uint64_t i = tid;
      for (; i + 3 * stride < n; i += 4 * stride) {
        const uint32_t a = src[i], b = src[i + stride], x = src[i + 2 * stride], y = src[i + 3 * stride];
        dst[i] = a;
        dst[i + stride] = b;
        dst[i + 2 * stride] = x;
        dst[i + 3 * stride] = y;
      }
      for (; i < n; i += stride) dst[i] = src[i];
    }
  }
}

// Range lookup in a P_{a,p} key array: [lower_bound(lo), lower_bound(hi)) -> rows.
// Key ranges through pinned staging (das_internal: pinned_stage): requests
// read over the host mapping, replies stored to the host, slot released.
__global__ void __launch_bounds__(256) k_key_ranges_pub(const uint64_t* ukey, const uint64_t* uoff, uint64_t nkeys,
                                                        const uint64_t* qlo, const uint64_t* qhi, uint32_t nq,
                                                        uint64_t* out, uint32_t* slot, uint32_t seq) {
  for (uint32_t i = threadIdx.x; i < 2 * nq; i += blockDim.x) {
    const uint64_t q = (i & 1) ? qhi[i >> 1] : qlo[i >> 1];
    uint64_t lo = 0, hi = nkeys;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (ukey[mid] < q) lo = mid + 1; else hi = mid;
    }
    __hip_atomic_store(&out[i], uoff[lo], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(&slot[15], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------
// Join / antijoin / dedup helpers
// ---------------------------------------------------------------------------

// Lexicographic compare of row i of A-cols against row j of B-cols.
__device__ __forceinline__ int cmp_rows(const ColSet& a, uint64_t i, const ColSet& b, uint64_t j) {
  for (int c = 0; c < a.n; ++c) {
    const uint32_t x = a.c[c][i], y = b.c[c][j];
    if (x != y) return x < y ? -1 : 1;
  }
  return 0;
}

__device__ __forceinline__ uint64_t lower_bound_rows(const ColSet& probe, uint64_t i, const ColSet& sorted, uint64_t n) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (cmp_rows(sorted, mid, probe, i) < 0) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ uint64_t upper_bound_rows(const ColSet& probe, uint64_t i, const ColSet& sorted, uint64_t n) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (cmp_rows(sorted, mid, probe, i) <= 0) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ void k_join_count(ColSet probe_key, uint64_t np, ColSet build_key, uint64_t nb, uint32_t* lo_out,
                             uint32_t* cnt) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < np; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t lo = lower_bound_rows(probe_key, i, build_key, nb);
    uint64_t hi = lo;
    if (lo < nb && cmp_rows(build_key, lo, probe_key, i) == 0) hi = upper_bound_rows(probe_key, i, build_key, nb);
    lo_out[i] = (uint32_t)lo;
    cnt[i] = (uint32_t)(hi - lo);
  }
}

// Output column sources: src[c] = (side, column) ; side 0 probe, 1 build
struct OutMap {
  const uint32_t* col[kMaxCols];
  uint8_t side[kMaxCols];
  int n;
};

__global__ void k_join_expand(const uint64_t* offs, uint64_t np, const uint32_t* lo, OutMap om, uint64_t total,
                              uint32_t* out, uint64_t cap) {
  for (uint64_t o = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; o < total; o += (uint64_t)gridDim.x * blockDim.x) {
    // i = upper_bound(offs, o) - 1
    uint64_t a = 0, b = np;
    while (a < b) {
      const uint64_t mid = (a + b) >> 1;
      if (offs[mid] <= o) a = mid + 1; else b = mid;
    }
    const uint64_t i = a - 1;
    const uint64_t j = lo[i] + (o - offs[i]);
    for (int c = 0; c < om.n; ++c) out[(uint64_t)c * cap + o] = om.side[c] ? om.col[c][j] : om.col[c][i];
  }
}

// Output o = (probe row o / nb, build row o % nb).  A thread writes four
// consecutive outputs per column as one 16-byte nontemporal store (columns
// are 64-row aligned, so a partial last quad stays inside the capacity); one
// division per thread: the grid stride S quads advances (i, j) by
// (4S / nb, 4S % nb) with a carry.  A pure write stream at ~6 TB/s on MI355X
// (4-byte stores: ~3.4 TB/s; tools/ubench/cart_bw.hip, profiles/archive/r3_cart_bw.txt).
// NC: output columns, specialised up to 6.
template <int NC>
__global__ void __launch_bounds__(B) k_cartesian(OutMap om, uint64_t np, uint64_t nb, uint64_t total, uint64_t sq,
                                                 uint64_t sr, uint32_t* out, uint64_t cap) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const int nc = NC > 0 ? NC : om.n;
  const uint64_t nq = (total + 3) >> 2;
  uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (q >= nq) return;
  uint64_t i = (q << 2) / nb, j = (q << 2) - i * nb;
  const uint32_t* col[kMaxCols];
  bool side[kMaxCols];
#pragma unroll
  for (int c = 0; c < (NC > 0 ? NC : kMaxCols); ++c) {
    if (c >= nc) break;
    col[c] = om.col[c];
    side[c] = om.side[c] != 0;
  }
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (; q < nq; q += stride) {
    uint64_t ii[4], jj[4];
    ii[0] = i;
    jj[0] = j;
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      ii[k] = ii[k - 1];
      jj[k] = jj[k - 1] + 1;
      if (jj[k] == nb) { jj[k] = 0; ++ii[k]; }
    }
#pragma unroll
    for (int c = 0; c < (NC > 0 ? NC : kMaxCols); ++c) {
      if (c >= nc) break;
      uint32_t v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = ii[k] < np ? (side[c] ? col[c][jj[k]] : col[c][ii[k]]) : 0u;
      __builtin_nontemporal_store(v4u{v[0], v[1], v[2], v[3]}, reinterpret_cast<v4u*>(out + (uint64_t)c * cap) + q);
    }
    i += sq;
    j += sr;
    if (j >= nb) { j -= nb; ++i; }
  }
}

// ---------------------------------------------------------------------------
// Row hash sets (Not / Or / dedup without sorting): open addressing, linear
// probing, slots hold row indices (kEmpty = free), insert-only so a slot
// never returns to free and every tuple owns exactly one slot.  Row equality
// compares the full tuples, so the result is exact whatever the hash.
// ---------------------------------------------------------------------------
constexpr uint32_t kEmpty = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t hs_mix(uint32_t h) {   // murmur3 finaliser
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t row_hash(const ColSet& k, uint64_t i) {
  uint32_t h = 0x2545f491u;
  for (int c = 0; c < k.n; ++c) h = hs_mix(h ^ (k.c[c][i] + 0x9e3779b9u * (uint32_t)(c + 1)));
  return h;
}
__device__ __forceinline__ bool rows_equal(const ColSet& a, uint64_t i, const ColSet& b, uint64_t j) {
  for (int c = 0; c < a.n; ++c)
    if (a.c[c][i] != b.c[c][j]) return false;
  return true;
}
__device__ __forceinline__ uint32_t slot_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Inserts rows [0, n); with `keep_min` the slot ends holding the smallest
// index of its tuple (the first occurrence).
__global__ void k_hset_insert(ColSet k, uint64_t n, uint32_t* tab, uint32_t mask, int keep_min) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t h = row_hash(k, i) & mask;
    for (uint32_t probe = 0; probe <= mask; ++probe, h = (h + 1) & mask) {
      uint32_t cur = slot_load(&tab[h]);
      if (cur == kEmpty) {
        cur = atomicCAS(&tab[h], kEmpty, (uint32_t)i);
        if (cur == kEmpty) break;
      }
      if (rows_equal(k, cur, k, i)) {
        if (keep_min) atomicMin(&tab[h], (uint32_t)i);
        break;
      }
    }
  }
}
// keep[i] = row i is its tuple's first occurrence
__global__ void k_hset_first(ColSet k, uint64_t n, const uint32_t* tab, uint32_t mask, uint32_t* keep) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t h = row_hash(k, i) & mask, f = 0;
    for (uint32_t probe = 0; probe <= mask; ++probe, h = (h + 1) & mask) {
      const uint32_t cur = tab[h];
      if (cur == kEmpty) break;                     // (unreachable: row i was inserted)
      if (rows_equal(k, cur, k, i)) { f = cur == (uint32_t)i; break; }
    }
    keep[i] = f;
  }
}
// keep[i] = probe row i (columns in the set's order) is NOT in the set of `t`
__global__ void k_hset_anti(ColSet a, uint64_t n, ColSet t, const uint32_t* tab, uint32_t mask, uint32_t* keep) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t h = row_hash(a, i) & mask, k = 1;
    for (uint32_t probe = 0; probe <= mask; ++probe, h = (h + 1) & mask) {
      const uint32_t cur = tab[h];
      if (cur == kEmpty) break;
      if (rows_equal(t, cur, a, i)) { k = 0; break; }
    }
    keep[i] = k;
  }
}

// keep[i] = 0 if a matching row exists in `sorted`
__global__ void k_anti_flags(ColSet probe, uint64_t np, ColSet sorted, uint64_t ns, uint32_t* keep) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < np; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t lo = lower_bound_rows(probe, i, sorted, ns);
    keep[i] = !(lo < ns && cmp_rows(sorted, lo, probe, i) == 0);
  }
}

__global__ void k_distinct_flags(ColSet sorted, uint64_t n, uint32_t* keep) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    keep[i] = (i == 0) || cmp_rows(sorted, i - 1, sorted, i) != 0;
}

// no_overload filter on join output: distinct vars must have distinct values
__global__ void k_overload_flags(ColSet t, uint64_t n, uint32_t* keep) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t k = 1;
    for (int a = 0; a < t.n && k; ++a)
      for (int b = a + 1; b < t.n; ++b)
        if (t.c[a][i] == t.c[b][i]) { k = 0; break; }
    keep[i] = k;
  }
}

__global__ void k_gather_cols(ColSet src, const uint32_t* idx, uint64_t n, uint32_t* out, uint64_t cap) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t r = idx[i];
    for (int c = 0; c < src.n; ++c) out[(uint64_t)c * cap + i] = src.c[c][r];
  }
}

// ---------------------------------------------------------------------------
// Direct-address join on one shared variable (atom ids are dense and the key
// column's id bounds are known on the host):
//   build  k_key_hist -> scan -> k_key_scatter (counting sort) -> k_pack_lc
//   probe  k_dj_count (per wave-unit output totals) -> scan -> k_dj_write
// ---------------------------------------------------------------------------
constexpr int kDjWaves = B / 64;

// min / max of a key column by ONE workgroup, published straight into the
// pinned read-back slot (words 0, 1; sequence in word 15)
__global__ void __launch_bounds__(1024) k_key_minmax_pub(const uint32_t* key, uint64_t n, uint32_t* slot, uint32_t seq) {
  __shared__ uint32_t s_lo[16], s_hi[16];
  uint32_t lo = 0xFFFFFFFFu, hi = 0;
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t k = key[i];
    lo = k < lo ? k : lo;
    hi = k > hi ? k : hi;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t a = __shfl_xor(lo, d, 64), b = __shfl_xor(hi, d, 64);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  if (__lane_id() == 0) {
    s_lo[threadIdx.x >> 6] = lo;
    s_hi[threadIdx.x >> 6] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
      lo = s_lo[w] < lo ? s_lo[w] : lo;
      hi = s_hi[w] > hi ? s_hi[w] : hi;
    }
    __hip_atomic_store(&slot[0], lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&slot[1], hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    __hip_atomic_store(&slot[15], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void __launch_bounds__(B) k_key_minmax(const uint32_t* key, uint64_t n, uint32_t* mm) {
  __shared__ uint32_t s_lo[kDjWaves], s_hi[kDjWaves];
  uint32_t lo = 0xFFFFFFFFu, hi = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t k = key[i];
    lo = k < lo ? k : lo;
    hi = k > hi ? k : hi;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t a = __shfl_xor(lo, d, 64), b = __shfl_xor(hi, d, 64);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  if (__lane_id() == 0) {
    s_lo[threadIdx.x >> 6] = lo;
    s_hi[threadIdx.x >> 6] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kDjWaves; ++w) {
      lo = s_lo[w] < lo ? s_lo[w] : lo;
      hi = s_hi[w] > hi ? s_hi[w] : hi;
    }
    atomicMin(&mm[0], lo);
    atomicMax(&mm[1], hi);
  }
}

// Keys outside [kmin, kmin + range) cannot occur (range = the key column's
// bound); they are skipped rather than written out of bounds.
__global__ void __launch_bounds__(B) k_key_hist(const uint32_t* key, uint64_t n, uint32_t kmin, uint32_t range,
                                                uint32_t* cnt) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x; i0 < n; i0 += stride) {   // wave-uniform trip count
    const uint64_t i = i0 + threadIdx.x;
    const uint32_t d = i < n ? key[i] - kmin : range;
    const bool act = d < range;
    wave_agg_atomic_inc(cnt, act ? d : 0u, act);
  }
}

// Sorted build keys: off[d] = first row whose key >= kmin + d, d in [0, range]
// (a binary search per d: gaps between present keys can be long).
__global__ void k_bucket_bounds(const uint32_t* key, uint64_t n, uint32_t kmin, uint32_t range, uint32_t* off) {
  for (uint64_t d = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; d <= range; d += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = kmin + d;
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if ((uint64_t)key[mid] < k) lo = mid + 1; else hi = mid;
    }
    off[d] = (uint32_t)lo;
  }
}

__global__ void __launch_bounds__(B) k_key_scatter(ColSet src, const uint32_t* key, uint64_t n, uint32_t kmin,
                                                   uint32_t range, uint32_t* cursor, uint32_t* out, uint64_t cap) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x; i0 < n; i0 += stride) {
    const uint64_t i = i0 + threadIdx.x;
    const uint32_t d = i < n ? key[i] - kmin : range;
    const bool act = d < range;
    const uint32_t pos = wave_agg_atomic_inc(cursor, act ? d : 0u, act);
    if (act)
      for (int c = 0; c < src.n; ++c) out[(uint64_t)c * cap + pos] = src.c[c][i];
  }
}

// (lo, cnt) of a key's bucket packed in one 8-byte entry: one gather per probe
// row instead of two (random 4-byte gathers are address-unit bound).
// Bucket descriptor of a key: (lo, cnt) in one 8-byte entry, one gather per
// probe row.
__global__ void k_pack_lc(const uint32_t* off, uint32_t range, uint2* lc) {
  for (uint64_t d = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; d < range; d += (uint64_t)gridDim.x * blockDim.x)
    lc[d] = make_uint2(off[d], off[d + 1] - off[d]);
}

// Sparse build keys over a wide slot range (bio QUERY_3: ~2*10^4 rows keyed
// by Member link ids over 1.4*10^7 slots): the (lo, cnt) descriptors are
// written straight into a zeroed lc array -- one 8-byte store stream per
// slot -- instead of a histogram, a scan, a copy and the packing of range+1
// offsets (~5x the slot bytes).  Counts by wave-aggregated atomics on
// lc[d].y (each row keeps its rank inside its key); sorted keys take their
// run start as lo, unsorted ones get a base per key from one atomic per wave
// (k_lc_base) and are scattered by (base + rank) (k_lc_scatter).
__global__ void __launch_bounds__(B) k_lc_count(const uint32_t* key, uint64_t n, uint32_t kmin, uint32_t range,
                                                uint2* lc, uint32_t* rank, int sorted) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x; i0 < n; i0 += stride) {   // wave-uniform trip count
    const uint64_t i = i0 + threadIdx.x;
    const uint32_t k = i < n ? key[i] : 0u;
    const uint32_t d = i < n ? k - kmin : range;
    const bool act = d < range;
    const uint32_t r = wave_agg_atomic_inc(reinterpret_cast<uint32_t*>(lc) + 1, act ? 2u * d : 0u, act);
    if (!act) continue;
    if (sorted) {
      if (i == 0 || key[i - 1] != k) lc[d].x = (uint32_t)i;
    } else {
      rank[i] = r;
    }
  }
}

__global__ void __launch_bounds__(B) k_lc_base(const uint32_t* key, const uint32_t* rank, uint64_t n, uint32_t kmin,
                                               uint32_t range, uint2* lc, uint32_t* total) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x; i0 < n; i0 += stride) {
    const uint64_t i = i0 + threadIdx.x;
    const uint32_t d = i < n ? key[i] - kmin : range;
    const uint32_t v = (d < range && rank[i] == 0u) ? lc[d].y : 0u;   // one row per key claims its run
    const uint32_t inc = wave_incl_sum_u32(v);
    const uint32_t sum = __shfl(inc, 63, 64);
    uint32_t base = 0;
    if (__lane_id() == 63 && sum) base = atomicAdd(total, sum);
    base = __shfl(base, 63, 64);
    if (v) lc[d].x = base + inc - v;
  }
}

// the slots k_lc_count / k_lc_base wrote (and the running base at lc[range])
// back to zero: the context's descriptor array stays all-zero between joins
__global__ void __launch_bounds__(B) k_lc_clear(const uint32_t* key, uint64_t n, uint32_t kmin, uint32_t range,
                                                uint2* lc) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t d = key[i] - kmin;
    if (d < range) lc[d] = make_uint2(0u, 0u);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) lc[range] = make_uint2(0u, 0u);
}

__global__ void __launch_bounds__(B) k_lc_scatter(ColSet src, const uint32_t* key, const uint32_t* rank, uint64_t n,
                                                  uint32_t kmin, uint32_t range, const uint2* lc, uint32_t* out,
                                                  uint64_t cap) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t d = key[i] - kmin;
    if (d >= range) continue;
    const uint64_t pos = (uint64_t)lc[d].x + rank[i];
    for (int c = 0; c < src.n; ++c) out[(uint64_t)c * cap + pos] = src.c[c][i];
  }
}

// Probe = wave units of kXRows consecutive probe rows (kXGroups groups of 64,
// one row per lane).  No LDS arrays and no block barriers: a unit's counts,
// prefix and expansion live in registers; each output chunk of 64 finds its
// owning row by a 6-step binary search over the lanes' prefixes
// (ds_bpermute), takes the probe values from the owner lane and gathers the
// build payload at (bucket lo + rank inside the bucket).  Stores are one
// coalesced 256-byte column segment per chunk.
#ifndef DAS_DJ_GROUPS
#define DAS_DJ_GROUPS 2
#endif
constexpr int kXGroups = DAS_DJ_GROUPS;
constexpr uint64_t kXRows = 64ull * kXGroups;
constexpr uint64_t kHeavyUnit = 1ull << 16;   // outputs above which a unit is expanded output-balanced

__device__ __forceinline__ uint32_t lane_get(uint32_t v, int src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}

// The owner lanes of one round of 64 consecutive outputs ob + lane (the max
// lane with pre <= o; pre non-decreasing over the lanes, cnt = each lane's
// outputs).  Wave-uniform fast path: when no lane's range starts inside the
// round (a skewed key's long run), its owner is the owner of ob for all 64
// outputs (*uni = true, two ballots).  Otherwise each lane whose range starts
// inside the round writes its id at that offset of the wave's 64-entry LDS row
// (the owner of ob at offset 0) and an inclusive DPP max over the row gives
// every output its owner: two LDS stores, one load and six VALU steps in place
// of six dependent ds_bpermute rounds.
__device__ __forceinline__ int owner_of_round(uint32_t ob, uint32_t pre, uint32_t cnt, uint32_t* row, int lane,
                                              bool* uni) {
  const uint64_t m0 = __ballot(pre <= ob);
  const int l0 = 63 - __clzll((long long)m0);
  const uint64_t m1 = __ballot(pre <= ob + 63u);
  if (63 - __clzll((long long)m1) == l0) {
    *uni = true;
    return l0;
  }
  *uni = false;
  // volatile: lanes exchange values through the row, which the compiler's
  // per-lane memory model would otherwise let it forward (a lane's load
  // replaced by its own earlier store, the load sunk under the branch of the
  // other store); one wave's LDS accesses complete in program order
  typedef __attribute__((address_space(3))) volatile uint32_t lds_u32;
  lds_u32* vr = (lds_u32*)row;
  vr[lane] = lane == 0 ? (uint32_t)l0 : 0u;
  if (cnt && pre > ob && pre - ob < 64u) vr[pre - ob] = (uint32_t)lane;
  return (int)wave_incl_max_u32(vr[lane]);
}

// Expands outputs [rs, re) of one 64-row group (relative to the group's first
// output, written at obase + o): output o belongs to the max lane l with
// pre[l] <= o and is build row ex[l] + (o - pre[l]).  kXUnroll rounds of 64
// outputs are resolved first and their build loads issued together, so a
// wave keeps several loads in flight instead of one load -> store round trip
// per 64 outputs.
#ifndef DAS_DJ_UNROLL
#define DAS_DJ_UNROLL 4
#endif
constexpr int kXUnroll = DAS_DJ_UNROLL;
// the 16-byte run and quad paths move one block of 4 outputs per lane (256 per
// wave) whatever the rounds' unroll is: their guard, advance and LDS row size
constexpr int kVecBlock = 256;
// largest descriptor array (slots) the context keeps zeroed between sparse joins
constexpr uint64_t kZlcMax = 1ull << 26;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));   // dword-aligned 16-byte load

// 16-byte output store, nontemporal in the instantiations for large outputs
// (>= 2^22 rows): with nontemporal stores in every join, bio QUERY_3's
// k_cartesian -- which reads a small join result once per output row -- ran
// 1221 instead of 928 us (profiles/r4_dj_vec_ab.jsonl); the 25 M-row Q2 join
// runs 64-72 us with them, 87 us with plain 16-byte stores.  A template
// parameter, not a run-time branch: the compiler sinks a nontemporal and a
// plain store of two branches into one plain store.
template <bool NT>
__device__ __forceinline__ void store16(uint32_t* p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
  else *reinterpret_cast<u32x4*>(p) = v;
}

template <int NP, int NB, typename T, int V = 1, bool NT = false>
__device__ __forceinline__ void expand_group(T rs, T re, T pre, uint32_t cnt, uint32_t ex, const uint32_t* pv,
                                             const uint32_t* const* bb, uint32_t* const* po, uint32_t* const* bo,
                                             uint64_t obase, int lane, uint32_t* row, int search) {
  // 32-bit groups: owner_of_round (unless DAS_OWNER_SEARCH=1); each lane's
  // ex - pre travels as one value (br = (ex - pre)[owner] + o)
  const bool fast = sizeof(T) == 4 && !(search & 1);
  (void)cnt;
  // Run path (not with DAS_DJ_VEC=0, search bit 1): 256 consecutive outputs of
  // ONE probe row -- a skewed key's run, an index join's P range -- are
  // consecutive build rows: each lane moves 4 of them per column with one
  // 16-byte load and one 16-byte nontemporal store (4-byte stores top out at
  // ~3.1-3.4 TB/s on this part, 16-byte ones reach ~7, k_cartesian), and
  // writes the probe values as 16-byte splats; 256 outputs of several probe
  // rows take the quad path below (not with DAS_DJ_VEC=1, search bit 2).
  // Needs 16-byte aligned output positions: a head of up to 3 outputs goes
  // through the rounds first.  `row`: the wave's 256-entry LDS row.
  const bool runs = fast && !(search & 2) && (re - rs) > (T)kVecBlock;
  const uint32_t exp = ex - (uint32_t)pre;
  const T head = runs ? (T)((4u - ((uint32_t)(obase + rs) & 3u)) & 3u) : (T)0;
  for (T o0 = rs; o0 < re;) {
    const T lim = (head && o0 == rs) ? rs + head : re;
    if (runs && lim == re && (re - o0) >= (T)kVecBlock) {
      const uint64_t m0 = __ballot((uint32_t)pre <= (uint32_t)o0);
      const int l0 = 63 - __clzll((long long)m0);
      const uint64_t m1 = __ballot((uint32_t)pre <= (uint32_t)o0 + 255u);
      if (63 - __clzll((long long)m1) == l0) {
        const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)exp, l0) + (uint32_t)o0 + 4u * (uint32_t)lane;
        const uint64_t op = obase + (uint64_t)o0 + 4ull * (uint64_t)lane;
        u32x4 bv4[NB > 0 ? NB : 1];
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const u32x4_a4 x = *reinterpret_cast<const u32x4_a4*>(bb[i] + b0);
          bv4[i] = u32x4{x.x, x.y, x.z, x.w};
        }
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)pv[i], l0);
          store16<NT>(po[i] + op, u32x4{v, v, v, v});
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) store16<NT>(bo[i] + op, bv4[i]);
        o0 += (T)kVecBlock;
        continue;
      }
      if (!(search & 4)) {
        // Quad path: the 256 outputs span several probe rows.  Lane `lane`
        // takes outputs o0 + 4 lane .. + 3: every probe row starting inside
        // the block writes its lane id at its start offset of the wave's
        // 256-entry LDS row (the owner of o0 at offset 0), and a max scan
        // over the row -- 4 entries per lane, then an inclusive DPP max over
        // the lanes -- gives each output its owner.  The build values are 4
        // dword gathers per column; every column is written with ONE 16-byte
        // nontemporal store per lane instead of four 4-byte ones.
        typedef __attribute__((address_space(3))) volatile uint32_t lds_u32;
        lds_u32* vr = (lds_u32*)row;
#pragma unroll
        for (int k = 0; k < 4; ++k) vr[4 * lane + k] = (lane == 0 && k == 0) ? (uint32_t)l0 : 0u;
        if (cnt && (uint32_t)pre > (uint32_t)o0 && (uint32_t)pre - (uint32_t)o0 < 256u)
          vr[(uint32_t)pre - (uint32_t)o0] = (uint32_t)lane;
        uint32_t m[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) m[k] = vr[4 * lane + k];
#pragma unroll
        for (int k = 1; k < 4; ++k) m[k] = m[k] > m[k - 1] ? m[k] : m[k - 1];
        const uint32_t incl = wave_incl_max_u32(m[3]);
        const uint32_t prev = (uint32_t)__shfl_up((int)incl, 1, 64);
        const uint32_t ex0 = lane ? prev : 0u;
        const uint32_t q0 = (uint32_t)o0 + 4u * (uint32_t)lane;
        const uint64_t op = obase + (uint64_t)q0;
        int own[4];
        uint32_t brk[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          own[k] = (int)(m[k] > ex0 ? m[k] : ex0);
          brk[k] = lane_get(exp, own[k]) + q0 + (uint32_t)k;
        }
        u32x4 bq[NB > 0 ? NB : 1];
#pragma unroll
        for (int i = 0; i < NB; ++i) bq[i] = u32x4{bb[i][brk[0]], bb[i][brk[1]], bb[i][brk[2]], bb[i][brk[3]]};
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          const u32x4 pq{lane_get(pv[i], own[0]), lane_get(pv[i], own[1]), lane_get(pv[i], own[2]),
                         lane_get(pv[i], own[3])};
          store16<NT>(po[i] + op, pq);
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) store16<NT>(bo[i] + op, bq[i]);
        o0 += (T)kVecBlock;
        continue;
      }
    }
    // rounds of this iteration that hold outputs (wave-uniform): a group of
    // 64 rows at fan-out ~2 fills 2 of the 4, and the owner searches of an
    // empty round would be a third of the kernel's LDS instructions
    const int nr = V == 0 ? kXUnroll : (lim - o0) >= (T)(64 * kXUnroll) ? kXUnroll : (int)((lim - o0 + 63) / 64);
    T o[kXUnroll];
    int l[kXUnroll];
    bool un[kXUnroll];
    uint32_t br[kXUnroll];
#pragma unroll
    for (int u = 0; u < kXUnroll; ++u) {
      o[u] = o0 + (T)(u * 64 + lane);
      l[u] = 0;
      un[u] = false;
      br[u] = 0;
      if (u >= nr) continue;
      if (fast) {
        const int ll = owner_of_round((uint32_t)(o0 + (T)(u * 64)), (uint32_t)pre, cnt, row, lane, &un[u]);
        l[u] = ll;
        br[u] = (un[u] ? (uint32_t)__builtin_amdgcn_readlane((int)exp, ll) : lane_get(exp, ll)) + (uint32_t)o[u];
        continue;
      }
      int ll = 0;                                            // owner: max lane with pre <= o
#pragma unroll
      for (int step = 32; step >= 1; step >>= 1) {
        const T pl = (T)__shfl(pre, ll + step, 64);
        if (ll + step < 64 && pl <= o[u]) ll += step;
      }
      l[u] = ll;
      br[u] = lane_get(ex, ll) + (uint32_t)(o[u] - (T)__shfl(pre, ll, 64));
    }
    uint32_t bv[kXUnroll][NB > 0 ? NB : 1];
#pragma unroll
    for (int u = 0; u < kXUnroll; ++u)
#pragma unroll
      for (int i = 0; i < NB; ++i) bv[u][i] = (u < nr && o[u] < lim) ? bb[i][br[u]] : 0u;
#pragma unroll
    for (int u = 0; u < kXUnroll; ++u) {
      if (u >= nr) continue;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const uint32_t v = un[u] ? (uint32_t)__builtin_amdgcn_readlane((int)pv[i], l[u]) : lane_get(pv[i], l[u]);
        if (o[u] < lim) po[i][obase + o[u]] = v;
      }
#pragma unroll
      for (int i = 0; i < NB; ++i)
        if (o[u] < lim) bo[i][obase + o[u]] = bv[u][i];
    }
    o0 = lim != re ? lim : o0 + (T)(64 * kXUnroll);
  }
}

// warm0 / warm1 (nullable): probe payload columns the expansion reads next;
// touched here so they arrive from the MALL, not cold HBM, when the probe is
// a view of index rows (no projection copy left them warm)
__global__ void __launch_bounds__(B) k_dj_count(const uint32_t* pkey, uint64_t np, uint32_t kmin, uint32_t range,
                                                const uint2* lc, uint64_t units, uint64_t* unit_tot,
                                                const uint32_t* warm0, const uint32_t* warm1) {
  const uint64_t waves = (uint64_t)gridDim.x * (B / 64);
  const int lane = __lane_id();
  for (uint64_t u = blockIdx.x * (uint64_t)(B / 64) + (threadIdx.x >> 6); u < units; u += waves) {
    const uint64_t r0 = u * kXRows;
    uint32_t d[kXGroups];
#pragma unroll
    for (int g = 0; g < kXGroups; ++g) {
      const uint64_t r = r0 + g * 64 + lane;
      d[g] = r < np ? pkey[r] - kmin : 0xFFFFFFFFu;       // wraps for keys below kmin
      if (warm0 && r < np) {
        const uint32_t w0 = warm0[r];
        asm volatile("" ::"v"(w0));
      }
      if (warm1 && r < np) {
        const uint32_t w1 = warm1[r];
        asm volatile("" ::"v"(w1));
      }
    }
    uint64_t acc = 0;
#pragma unroll
    for (int g = 0; g < kXGroups; ++g)
      if (d[g] < range) acc += lc[d[g]].y;
    acc = wave_reduce_sum(acc);
    if (lane == 0) unit_tot[u] = acc;      // the scan also yields the largest unit
  }
}

// k_dj_count + the count -> offsets scan in ONE launch for up to
// kCountPubUnits units: every block writes its units' counts through to the
// coherence point and arrives on a ticket; the last block scans the counts
// into unit_off (unit_off[units] = total) and publishes (total, largest unit)
// to the pinned read-back slot -- the scan launch and its launch gap are gone
// (bio QUERY_2 / QUERY_3 run five such joins per step)
constexpr uint64_t kCountPubUnits = 8192;
__global__ void __launch_bounds__(B) k_dj_count_pub(const uint32_t* pkey, uint64_t np, uint32_t kmin, uint32_t range,
                                                    const uint2* lc, uint64_t units, uint64_t* unit_tot,
                                                    const uint32_t* warm0, const uint32_t* warm1, uint64_t* unit_off,
                                                    unsigned long long* ctr, unsigned long long last, uint32_t* slot,
                                                    uint32_t seq) {
  __shared__ uint64_t s_sum[B / 64];
  __shared__ uint64_t s_mx[B / 64];
  __shared__ int s_last;
  const uint64_t waves = (uint64_t)gridDim.x * (B / 64);
  const int lane = __lane_id();
  for (uint64_t u = blockIdx.x * (uint64_t)(B / 64) + (threadIdx.x >> 6); u < units; u += waves) {
    const uint64_t r0 = u * kXRows;
    uint32_t d[kXGroups];
#pragma unroll
    for (int g = 0; g < kXGroups; ++g) {
      const uint64_t r = r0 + g * 64 + lane;
      d[g] = r < np ? pkey[r] - kmin : 0xFFFFFFFFu;
      if (warm0 && r < np) {
        const uint32_t w0 = warm0[r];
        asm volatile("" ::"v"(w0));
      }
      if (warm1 && r < np) {
        const uint32_t w1 = warm1[r];
        asm volatile("" ::"v"(w1));
      }
    }
    uint64_t acc = 0;
#pragma unroll
    for (int g = 0; g < kXGroups; ++g)
      if (d[g] < range) acc += lc[d[g]].y;
    acc = wave_reduce_sum(acc);
    if (lane == 0) __hip_atomic_store(&unit_tot[u], acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // (write-through arrivals: no agent-scope release per block)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) s_last = __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == last;
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  uint64_t total, mx;
  block_scan_loop<uint64_t>(SpanIn<uint64_t>{unit_tot}, units, unit_off, total, mx, s_sum, s_mx);
  if (threadIdx.x == 0) unit_off[units] = total;
  const uint32_t w[4] = {(uint32_t)total, (uint32_t)(total >> 32), (uint32_t)mx, (uint32_t)(mx >> 32)};
  pub_store(slot, seq, w, 4);
}

// Output columns of a direct join, split by side so the kernel is
// specialised on their counts (pointers stay in scalar registers).
struct JoinCols {
  const uint32_t* p[kMaxCols];   // probe-side source columns
  const uint32_t* b[kMaxCols];   // build-side source columns (rows of the sorted build table)
  int po[kMaxCols], bo[kMaxCols];  // their output column indices
  int np, nb;
  int search;                    // bit 0: owner lanes by the 6-step ds_bpermute search (DAS_OWNER_SEARCH=1, A/B);
                                 // bit 1: no 16-byte paths (DAS_DJ_VEC=0); bit 2: no quad path
                                 // (DAS_DJ_VEC=1); bit 3: no run path in the filtered walk (DAS_FILT_RUN=0)
};

// DAS_OWNER_SEARCH=1: the expansions find each output's owner lane by the
// binary search over the lanes' prefixes (round 3); default: owner_of_round.
// DAS_DJ_VEC=0 (bit 1): no 16-byte paths in expand_group; =1 (bit 2): the
// single-row run path only, no quad path (A/B).
inline int owner_search_env() {
  const char* e = std::getenv("DAS_OWNER_SEARCH");
  const char* v = std::getenv("DAS_DJ_VEC");
  const char* fr = std::getenv("DAS_FILT_RUN");
  return (e && e[0] == '1' ? 1 : 0) | (v && v[0] == '0' ? 2 : 0) | (v && v[0] == '1' ? 4 : 0) |
         (fr && fr[0] == '0' ? 8 : 0);
}

template <int NP, int NB, typename T, int V, bool NT = false>
__global__ void __launch_bounds__(B) k_dj_write(const uint32_t* __restrict__ pkey, uint64_t np, uint32_t kmin,
                                                uint32_t range, const uint2* __restrict__ lc, uint64_t units,
                                                const uint64_t* __restrict__ unit_off, JoinCols jc,
                                                uint32_t* __restrict__ out, uint64_t cap) {
  __shared__ uint32_t s_row[B / 64][kVecBlock];             // the wave's LDS row (owner_of_round, quad path)
  uint32_t* row = s_row[threadIdx.x >> 6];
  const uint64_t waves = (uint64_t)gridDim.x * (B / 64);
  const int lane = __lane_id();
  const uint32_t* pp[NP > 0 ? NP : 1];
  const uint32_t* bb[NB > 0 ? NB : 1];
  uint32_t* po[NP > 0 ? NP : 1];
  uint32_t* bo[NB > 0 ? NB : 1];
#pragma unroll
  for (int i = 0; i < NP; ++i) { pp[i] = jc.p[i]; po[i] = out + (uint64_t)jc.po[i] * cap; }
#pragma unroll
  for (int i = 0; i < NB; ++i) { bb[i] = jc.b[i]; bo[i] = out + (uint64_t)jc.bo[i] * cap; }
  for (uint64_t u = blockIdx.x * (uint64_t)(B / 64) + (threadIdx.x >> 6); u < units; u += waves) {
    const uint64_t r0 = u * kXRows;
    uint32_t d[kXGroups];
#pragma unroll
    for (int g = 0; g < kXGroups; ++g) {
      const uint64_t r = r0 + g * 64 + lane;
      d[g] = r < np ? pkey[r] - kmin : 0xFFFFFFFFu;
    }
    uint2 e[kXGroups];
#pragma unroll
    for (int g = 0; g < kXGroups; ++g) e[g] = d[g] < range ? lc[d[g]] : make_uint2(0u, 0u);
    uint32_t pv[kXGroups][NP > 0 ? NP : 1];                 // probe values of this lane's rows
#pragma unroll
    for (int g = 0; g < kXGroups; ++g) {
      const uint64_t r = r0 + g * 64 + lane;
#pragma unroll
      for (int i = 0; i < NP; ++i) pv[g][i] = r < np ? pp[i][r] : 0u;
    }
    uint64_t base = unit_off[u];
#pragma unroll
    for (int g = 0; g < kXGroups; ++g) {
      const T c = (T)e[g].y;
      const T inc = wave_inclusive_scan(c);
      const T tot = (T)__shfl(inc, 63, 64);
      const T pre = inc - c;                                 // this lane's first output
      expand_group<NP, NB, T, V, NT>((T)0, tot, pre, e[g].y, e[g].x, pv[g], bb, po, bo, base, lane, row, jc.search);
      base += tot;
    }
  }
}

// Skew-balanced variant (hub keys: one probe unit can own millions of
// outputs): waves own fixed OUTPUT chunks instead of probe units.  A wave
// finds the unit holding its first output by a 64-ary search over the unit
// offsets, then expands only the slice of each group that falls in its chunk.
constexpr uint64_t kBalChunk = 1024;

template <int NP, int NB, typename T, bool NT = false>
__global__ void __launch_bounds__(B) k_dj_write_bal(const uint32_t* __restrict__ pkey, uint64_t np, uint32_t kmin,
                                                    uint32_t range, const uint2* __restrict__ lc, uint64_t units,
                                                    const uint64_t* __restrict__ unit_off, JoinCols jc,
                                                    uint32_t* __restrict__ out, uint64_t cap, uint64_t total,
                                                    uint64_t chunk) {
  const uint64_t waves = (uint64_t)gridDim.x * (B / 64);
  const int lane = __lane_id();
  const uint32_t* pp[NP > 0 ? NP : 1];
  const uint32_t* bb[NB > 0 ? NB : 1];
  uint32_t* po[NP > 0 ? NP : 1];
  uint32_t* bo[NB > 0 ? NB : 1];
#pragma unroll
  for (int i = 0; i < NP; ++i) { pp[i] = jc.p[i]; po[i] = out + (uint64_t)jc.po[i] * cap; }
#pragma unroll
  for (int i = 0; i < NB; ++i) { bb[i] = jc.b[i]; bo[i] = out + (uint64_t)jc.bo[i] * cap; }
  __shared__ uint32_t s_row[B / 64][kVecBlock];             // the wave's LDS row (owner_of_round, quad path)
  uint32_t* row = s_row[threadIdx.x >> 6];
  const uint64_t chunks = (total + chunk - 1) / chunk;
  for (uint64_t w = blockIdx.x * (uint64_t)(B / 64) + (threadIdx.x >> 6); w < chunks; w += waves) {
    const uint64_t ob = w * chunk;
    const uint64_t oe = ob + chunk < total ? ob + chunk : total;
    // last unit with unit_off[u] <= ob   (unit_off[units] == total > ob)
    uint64_t lo = 0, hi = units;
    while (hi - lo > 1) {
      const uint64_t step = (hi - lo + 63) / 64;
      const uint64_t idx = lo + (uint64_t)lane * step;
      const bool ok = idx < hi && unit_off[idx] <= ob;
      const uint64_t m = __ballot(ok);
      const uint64_t nlo = lo + (uint64_t)(63 - __clzll((long long)m)) * step;
      hi = nlo + step < hi ? nlo + step : hi;
      lo = nlo;
    }
    for (uint64_t u = lo; u < units; ++u) {
      uint64_t base = unit_off[u];
      if (base >= oe) break;
      const uint64_t r0 = u * kXRows;
      uint2 e[kXGroups];
#pragma unroll
      for (int g = 0; g < kXGroups; ++g) {
        const uint64_t r = r0 + g * 64 + lane;
        const uint32_t d = r < np ? pkey[r] - kmin : 0xFFFFFFFFu;
        e[g] = d < range ? lc[d] : make_uint2(0u, 0u);
      }
#pragma unroll
      for (int g = 0; g < kXGroups; ++g) {
        const T c = (T)e[g].y;
        const T inc = wave_inclusive_scan(c);
        const T tot = (T)__shfl(inc, 63, 64);
        const T pre = inc - c;
        const uint64_t gb = base, ge = base + tot;
        base = ge;
        if (ge <= ob || gb >= oe) continue;
        const T rs = (T)((ob > gb ? ob : gb) - gb), re = (T)((oe < ge ? oe : ge) - gb);
        const uint64_t r = r0 + g * 64 + lane;
        uint32_t pv[NP > 0 ? NP : 1];
#pragma unroll
        for (int i = 0; i < NP; ++i) pv[i] = r < np ? pp[i][r] : 0u;
        expand_group<NP, NB, T, 1, NT>(rs, re, pre, (uint32_t)c, e[g].x, pv, bb, po, bo, gb, lane, row, jc.search);
      }
    }
  }
}

template <int NP, int NB>
void launch_dj_write(unsigned grid, hipStream_t s, const uint32_t* pkey, uint64_t np, uint32_t kmin, uint32_t range,
                     const uint2* lc, uint64_t units, const uint64_t* toff, const JoinCols& jc, uint32_t* out,
                     uint64_t cap, uint64_t total, bool balanced, double bytes) {
  const bool wide = total >= (1ull << 32) - (1ull << 16);
  static const int fixed = std::getenv("DAS_DJ_FIXED") && std::getenv("DAS_DJ_FIXED")[0] == '1';
  // 16-byte stores nontemporal for outputs of 2^22 rows or more (DAS_DJ_NT=1
  // always, 0 never); 64-bit-offset and fixed-round launches: plain
  static const char* nte = std::getenv("DAS_DJ_NT");
  const bool nt = !wide && (nte && nte[0] == '1' ? true : nte && nte[0] == '0' ? false : total >= (1ull << 22)) &&
                  (balanced || !fixed);
  // scope names = rocprof's names of the instantiation launched below
  KScope ks((std::string(balanced ? "k_dj_write_bal<" : "k_dj_write<") + std::to_string(NP) + "," +
             std::to_string(NB) + (wide ? ",u64" : ",u32") + (balanced ? "" : (fixed && !wide) ? ",0" : ",1") +
             (nt ? ",true>" : ",false>"))
                .c_str(), bytes);
  if (balanced) {
    // outputs per wave (DAS_BAL_CHUNK, A/B: 512 .. 8192, a multiple of 64)
    static const uint64_t chunk = [] {
      const char* e = std::getenv("DAS_BAL_CHUNK");
      const uint64_t v = e ? std::strtoull(e, nullptr, 10) : kBalChunk;
      return v >= 64 && v <= 8192 && v % 64 == 0 ? v : kBalChunk;
    }();
    const unsigned g = grid_for((total + chunk - 1) / chunk, B / 64, 65535u * 4u);
    if (wide)
      hipLaunchKernelGGL((k_dj_write_bal<NP, NB, uint64_t>), dim3(g), dim3(B), 0, s, pkey, np, kmin, range, lc, units,
                         toff, jc, out, cap, total, chunk);
    else if (nt)
      hipLaunchKernelGGL((k_dj_write_bal<NP, NB, uint32_t, true>), dim3(g), dim3(B), 0, s, pkey, np, kmin, range, lc,
                         units, toff, jc, out, cap, total, chunk);
    else
      hipLaunchKernelGGL((k_dj_write_bal<NP, NB, uint32_t, false>), dim3(g), dim3(B), 0, s, pkey, np, kmin, range, lc,
                         units, toff, jc, out, cap, total, chunk);
    return;
  }
  if (wide) {
    hipLaunchKernelGGL((k_dj_write<NP, NB, uint64_t, 1>), dim3(grid), dim3(B), 0, s, pkey, np, kmin, range, lc, units,
                       toff, jc, out, cap);
  } else if (fixed) {
    hipLaunchKernelGGL((k_dj_write<NP, NB, uint32_t, 0>), dim3(grid), dim3(B), 0, s, pkey, np, kmin, range, lc, units,
                       toff, jc, out, cap);
  } else if (nt) {
    hipLaunchKernelGGL((k_dj_write<NP, NB, uint32_t, 1, true>), dim3(grid), dim3(B), 0, s, pkey, np, kmin, range, lc,
                       units, toff, jc, out, cap);
  } else {
    hipLaunchKernelGGL((k_dj_write<NP, NB, uint32_t, 1, false>), dim3(grid), dim3(B), 0, s, pkey, np, kmin, range, lc,
                       units, toff, jc, out, cap);
  }
}

// dispatch on (probe cols, build cols); wide schemas use the 4 x 4 kernel in
// column slices
// bytes(np, nb): algorithmic bytes of a launch writing np probe and nb build columns
template <typename Bytes>
void dj_write(unsigned grid, hipStream_t s, const uint32_t* pkey, uint64_t np, uint32_t kmin, uint32_t range,
              const uint2* lc, uint64_t units, const uint64_t* toff, const JoinCols& jc, uint32_t* out, uint64_t cap,
              uint64_t total, bool balanced, const Bytes& bytes) {
  int pi = 0, bi = 0;
  do {
    JoinCols part{};
    part.search = owner_search_env();
    part.np = std::min(jc.np - pi, 4);
    part.nb = std::min(jc.nb - bi, 4);
    for (int i = 0; i < part.np; ++i) { part.p[i] = jc.p[pi + i]; part.po[i] = jc.po[pi + i]; }
    for (int i = 0; i < part.nb; ++i) { part.b[i] = jc.b[bi + i]; part.bo[i] = jc.bo[bi + i]; }
    pi += part.np;
    bi += part.nb;
#define DJ(NPV, NBV)                                                                                  \
  if (part.np == NPV && part.nb == NBV) {                                                             \
    launch_dj_write<NPV, NBV>(grid, s, pkey, np, kmin, range, lc, units, toff, part, out, cap, total, balanced,      \
                              bytes(part.np, part.nb));                                                            \
    continue;                                                                                         \
  }
    DJ(0, 1) DJ(0, 2) DJ(0, 3) DJ(0, 4)
    DJ(1, 0) DJ(1, 1) DJ(1, 2) DJ(1, 3) DJ(1, 4)
    DJ(2, 0) DJ(2, 1) DJ(2, 2) DJ(2, 3) DJ(2, 4)
    DJ(3, 0) DJ(3, 1) DJ(3, 2) DJ(3, 3) DJ(3, 4)
    DJ(4, 0) DJ(4, 1) DJ(4, 2) DJ(4, 3) DJ(4, 4)
#undef DJ
  } while (pi < jc.np || bi < jc.nb);
}

// ---------------------------------------------------------------------------
// Filtered expansion: a join whose fresh build column is then filtered by
// semi-join terms (T0(V1,h0) T1(V1,V2) | T2(V2,h1) T3(V2,h0) of the hub And:
// the key bitmap holds T2's and T3's keys).  The join's outputs are expanded
// virtually, in output-balanced chunks, twice: MODE 0 tests each output's
// build value against the bitmap (one flag byte per output, the chunk's kept
// count); MODE 1 writes only the kept outputs, in output order, at the
// chunk's scanned offset.  The unfiltered join is never materialised.
// MODE 2 (one walk): tests each output and writes the kept ones at the
// chunk's own slot range [w CH, w CH + kept) of a scratch table (cap = the
// virtual output count) with the chunk's kept count; k_chunk_compact then
// moves the chunk runs to their scanned offsets -- the outputs are walked and
// their build rows gathered once instead of twice, and no flag bytes go
// through HBM (no atomics: the order is the two-pass order).
// ---------------------------------------------------------------------------
struct FiltKey {
  const uint32_t* col;     // build column holding the filtered variable
  uint32_t lo, range;
  const uint32_t* bits;
  int bcol;                // its index among the join's build output columns
};

// NPC / NBC: the probe / build output column counts when specialised (the
// pointers then live in registers), -1 = read from jc at run time
// MODE 3 (MODE 2 staged): a chunk's kept outputs are collected in its wave's
// LDS rows (stage: NPC + NBC columns of CH) and leave as 16-byte stores to
// the chunk's scratch slots (+ its count, for k_chunk_compact) instead of
// each lane's scattered 4-byte stores; with `kept` set, at a place reserved
// by ONE atomic per chunk instead (no scratch, no compaction; unsorted).
template <int MODE, int NPC, int NBC, int CH, int XU>
__device__ __forceinline__ void dj_filt_body(const uint32_t* __restrict__ pkey, uint64_t np, uint32_t kmin,
                                             uint32_t range, const uint2* __restrict__ lc, uint64_t units,
                                             const uint64_t* __restrict__ unit_off, uint64_t total, FiltKey fk,
                                             uint8_t* __restrict__ fl, uint32_t* __restrict__ ccnt,
                                             const uint32_t* __restrict__ coff, const JoinCols& jc,
                                             uint32_t* __restrict__ out, uint64_t cap, uint64_t wlo, uint64_t whi,
                                             uint32_t* row, uint32_t* stage = nullptr,
                                             unsigned long long* kept = nullptr,
                                             const uint32_t* __restrict__ cunit = nullptr) {
  const uint64_t waves = (uint64_t)gridDim.x * (B / 64);
  const int lane = __lane_id();
  const uint64_t lt = __lanemask_lt();
  const int ncp = NPC >= 0 ? NPC : jc.np, ncb = NBC >= 0 ? NBC : jc.nb;
  const uint32_t* pp[4];
  const uint32_t* bp[4];
  uint32_t* po[4];
  uint32_t* bo[4];
  uint32_t* sp[4];                          // MODE 3: the LDS rows of the probe / build output columns
  uint32_t* sb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    pp[i] = i < ncp ? jc.p[i] : nullptr;
    bp[i] = i < ncb ? jc.b[i] : nullptr;
    po[i] = i < ncp && MODE >= 1 && MODE != 3 ? out + (uint64_t)jc.po[i] * cap : nullptr;
    bo[i] = i < ncb && MODE >= 1 && MODE != 3 ? out + (uint64_t)jc.bo[i] * cap : nullptr;
    sp[i] = i < ncp && MODE == 3 ? stage + (uint64_t)i * CH : nullptr;
    sb[i] = i < ncb && MODE == 3 ? stage + (uint64_t)(ncp + i) * CH : nullptr;
  }
  // chunks [wlo, whi) of the virtual outputs
  for (uint64_t w = wlo + blockIdx.x * (uint64_t)(B / 64) + (threadIdx.x >> 6); w < whi; w += waves) {
    const uint64_t ob = w * CH;
    const uint64_t oe = ob + CH < total ? ob + CH : total;
    uint64_t lo = 0, hi = units;                       // last unit with unit_off[u] <= ob
    if (cunit) {
      lo = cunit[w];                                   // (k_chunk_units: one load, no search)
      hi = lo + 1;
    }
    while (hi - lo > 1) {
      const uint64_t step = (hi - lo + 63) / 64;
      const uint64_t idx = lo + (uint64_t)lane * step;
      const bool ok = idx < hi && unit_off[idx] <= ob;
      const uint64_t m = __ballot(ok);
      const uint64_t nlo = lo + (uint64_t)(63 - __clzll((long long)m)) * step;
      hi = nlo + step < hi ? nlo + step : hi;
      lo = nlo;
    }
    uint32_t run = 0;                                  // kept outputs of this chunk so far
    const uint64_t obase = MODE == 1 ? (uint64_t)coff[w] : MODE == 2 ? (w - wlo) * CH : 0ull;   // (MODE 3: LDS row 0)
    for (uint64_t u = lo; u < units; ++u) {
      uint64_t base = unit_off[u];
      if (base >= oe) break;
      const uint64_t r0 = u * kXRows;
      uint2 e[kXGroups];
#pragma unroll
      for (int g = 0; g < kXGroups; ++g) {
        const uint64_t r = r0 + g * 64 + lane;
        // (pkey null: the probe rows' own (first, count), k_ij_lc's row ids
        // are the identity -- one load instead of two dependent ones)
        const uint32_t d = r < np ? (pkey ? pkey[r] - kmin : (uint32_t)r) : 0xFFFFFFFFu;
        e[g] = d < range ? lc[d] : make_uint2(0u, 0u);
      }
#pragma unroll
      for (int g = 0; g < kXGroups; ++g) {
        const uint32_t c = e[g].y;
        const uint32_t inc = wave_inclusive_scan(c);
        const uint32_t tot = (uint32_t)__shfl(inc, 63, 64);
        const uint32_t pre = inc - c;
        const uint64_t gb = base, ge = base + tot;
        base = ge;
        if (ge <= ob || gb >= oe) continue;
        const uint32_t rs = (uint32_t)((ob > gb ? ob : gb) - gb), re = (uint32_t)((oe < ge ? oe : ge) - gb);
        const uint64_t r = r0 + g * 64 + lane;
        uint32_t pv[4] = {0u, 0u, 0u, 0u};
        if (MODE >= 1) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (i < ncp) pv[i] = r < np ? pp[i][r] : 0u;
        }
        const uint32_t exp = e[g].x - pre;           // br = (ex - pre)[owner] + o
        // Run path (one walk, one build column -- the filtered one): 256
        // consecutive outputs of ONE probe row (a hub's run of P rows) are
        // consecutive build rows: each lane tests 4 of them with one 16-byte
        // load and 4 bitmap words, and the kept ones leave compacted by a
        // wave prefix sum -- instead of 4 rounds of owner lanes, 4-byte
        // gathers and ballots (DAS_DJ_VEC=0: off)
        const bool runs = MODE >= 2 && ncb == 1 && fk.bcol == 0 && !(jc.search & 10) && (re - rs) > 256u;
        for (uint32_t o0 = rs; o0 < re;) {
          if (runs && re - o0 >= 256u) {
            const uint64_t m0 = __ballot(pre <= o0);
            const int l0 = 63 - __clzll((long long)m0);
            const uint64_t m1 = __ballot(pre <= o0 + 255u);
            if (63 - __clzll((long long)m1) == l0) {
              const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)exp, l0) + o0 + 4u * (uint32_t)lane;
              const u32x4_a4 x = *reinterpret_cast<const u32x4_a4*>(fk.col + b0);
              const uint32_t v[4] = {x.x - fk.lo, x.y - fk.lo, x.z - fk.lo, x.w - fk.lo};
              uint32_t wd[4];
#pragma unroll
              for (int k = 0; k < 4; ++k) wd[k] = v[k] < fk.range ? fk.bits[v[k] >> 5] : 0u;
              bool f[4];
              uint32_t cnt = 0;
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                f[k] = v[k] < fk.range && ((wd[k] >> (v[k] & 31)) & 1u);
                cnt += f[k] ? 1u : 0u;
              }
              const uint32_t inc = wave_inclusive_scan(cnt);
              const uint32_t tot = (uint32_t)__shfl(inc, 63, 64);
              uint64_t pos = obase + run + (inc - cnt);
              uint32_t pvl[4];
#pragma unroll
              for (int i = 0; i < 4; ++i) pvl[i] = i < ncp ? (uint32_t)__builtin_amdgcn_readlane((int)pv[i], l0) : 0u;
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                if (!f[k]) continue;
                if constexpr (MODE == 3) {
#pragma unroll
                  for (int i = 0; i < 4; ++i)
                    if (i < ncp) sp[i][pos] = pvl[i];
                  sb[0][pos] = v[k] + fk.lo;
                } else {
#pragma unroll
                  for (int i = 0; i < 4; ++i)
                    if (i < ncp) po[i][pos] = pvl[i];
                  bo[0][pos] = v[k] + fk.lo;
                }
                ++pos;
              }
              run += tot;
              o0 += 256u;
              continue;
            }
          }
          const int nr = (re - o0) >= 64u * XU ? XU : (int)((re - o0 + 63) / 64);
          uint32_t o[XU], br[XU];
          int ll[XU];
          bool un[XU];
#pragma unroll
          for (int q = 0; q < XU; ++q) {
            o[q] = o0 + (uint32_t)(q * 64 + lane);
            ll[q] = 0;
            un[q] = false;
            br[q] = 0;
            if (q >= nr) continue;
            if (!(jc.search & 1)) {
              const int l = owner_of_round(o0 + (uint32_t)(q * 64), pre, c, row, lane, &un[q]);
              ll[q] = l;
              br[q] = (un[q] ? (uint32_t)__builtin_amdgcn_readlane((int)exp, l) : lane_get(exp, l)) + o[q];
              continue;
            }
            int l = 0;                                 // owner: max lane with pre <= o
#pragma unroll
            for (int st = 32; st >= 1; st >>= 1) {
              const uint32_t pl = (uint32_t)__shfl(pre, l + st, 64);
              if (l + st < 64 && pl <= o[q]) l += st;
            }
            ll[q] = l;
            br[q] = lane_get(e[g].x, l) + (o[q] - (uint32_t)__shfl(pre, l, 64));
          }
          if (MODE == 0) {
            uint32_t v[XU];
#pragma unroll
            for (int q = 0; q < XU; ++q) v[q] = (q < nr && o[q] < re) ? fk.col[br[q]] - fk.lo : 0xFFFFFFFFu;
            uint32_t wd[XU];
#pragma unroll
            for (int q = 0; q < XU; ++q) wd[q] = v[q] < fk.range ? fk.bits[v[q] >> 5] : 0u;
#pragma unroll
            for (int q = 0; q < XU; ++q) {
              if (q >= nr) continue;
              const bool f = v[q] < fk.range && ((wd[q] >> (v[q] & 31)) & 1u);
              if (o[q] < re) fl[gb + o[q]] = f ? 1 : 0;
              run += (uint32_t)__popcll(__ballot(f));
            }
          } else {
            bool f[XU];
            uint32_t v[XU];
            if constexpr (MODE == 1) {
#pragma unroll
              for (int q = 0; q < XU; ++q) f[q] = q < nr && o[q] < re && fl[gb + o[q]] != 0;
            } else {
#pragma unroll
              for (int q = 0; q < XU; ++q) v[q] = (q < nr && o[q] < re) ? fk.col[br[q]] - fk.lo : 0xFFFFFFFFu;
              uint32_t wd[XU];
#pragma unroll
              for (int q = 0; q < XU; ++q) wd[q] = v[q] < fk.range ? fk.bits[v[q] >> 5] : 0u;
#pragma unroll
              for (int q = 0; q < XU; ++q) f[q] = v[q] < fk.range && ((wd[q] >> (v[q] & 31)) & 1u);
            }
            // build columns of the kept outputs (MODE 2: the filtered column
            // is the value just tested, no second load)
            uint32_t bv[XU][4];
#pragma unroll
            for (int q = 0; q < XU; ++q)
#pragma unroll
              for (int i = 0; i < 4; ++i)
                bv[q][i] = (i < ncb && f[q]) ? (MODE >= 2 && i == fk.bcol ? v[q] + fk.lo : bp[i][br[q]]) : 0u;
#pragma unroll
            for (int q = 0; q < XU; ++q) {
              if (q >= nr) continue;
              const uint64_t m = __ballot(f[q]);
              const uint64_t pos = obase + run + __popcll(m & lt);
              run += (uint32_t)__popcll(m);
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                if (i >= ncp) break;
                const uint32_t x = un[q] ? (uint32_t)__builtin_amdgcn_readlane((int)pv[i], ll[q])
                                         : lane_get(pv[i], ll[q]);
                if (f[q]) {
                  if constexpr (MODE == 3) sp[i][pos] = x;
                  else po[i][pos] = x;
                }
              }
              if (f[q]) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                  if (i < ncb) {
                    if constexpr (MODE == 3) sb[i][pos] = bv[q][i];
                    else bo[i][pos] = bv[q][i];
                  }
              }
            }
          }
          o0 += 64u * XU;
        }
      }
    }
    if constexpr (MODE == 3) {
      // the chunk's kept rows, LDS -> the chunk's slots (or a reserved place)
      // of the output: a head of <= 3 rows aligns the destination, 16-byte
      // stores, a tail of <= 3
      if (!kept && lane == 0) ccnt[w] = run;
      if (run) {
        // (LDS writes and reads of one wave stay in program order; the
        // barrier keeps the compiler from moving them across each other)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        unsigned long long b = 0;
        if (kept && lane == 0) b = atomicAdd(kept, (unsigned long long)run);
        if (!kept) b = (unsigned long long)(w - wlo) * CH;
        const uint64_t base = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), 0) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, 0);
        const uint32_t h = (4u - (uint32_t)(base & 3u)) & 3u;
        const uint32_t head = h < run ? h : run;
        const uint32_t nq = (run - head) / 4u;
        const uint32_t t0 = head + 4u * nq;
        for (int k = 0; k < ncp + ncb; ++k) {
          const uint32_t* sc = stage + (uint64_t)k * CH;
          const int col = k < ncp ? jc.po[k] : jc.bo[k - ncp];
          uint32_t* dc = out + (uint64_t)col * cap + base;
          if ((uint32_t)lane < head) dc[lane] = sc[lane];
          if (head == 0) {
            // chunk slots (CH-aligned, the default): the LDS quads are 16-byte
            // aligned too -- one conflict-free ds_read_b128 per lane instead
            // of four dword reads 16 bytes apart (4-way bank conflicts)
            for (uint32_t q = (uint32_t)lane; q < nq; q += 64u)
              store16<true>(dc + 4u * q, *reinterpret_cast<const u32x4*>(sc + 4u * q));
          } else {
            for (uint32_t q = (uint32_t)lane; q < nq; q += 64u) {
              const uint32_t j = head + 4u * q;
              store16<true>(dc + j, u32x4{sc[j], sc[j + 1], sc[j + 2], sc[j + 3]});
            }
          }
          if (t0 + (uint32_t)lane < run) dc[t0 + lane] = sc[t0 + lane];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    } else if (MODE != 1 && lane == 0) {
      ccnt[w] = run;
    }
  }
}

template <int MODE, int NPC = -1, int NBC = -1, int CH = (int)kBalChunk, int XU = kXUnroll>
__global__ void __launch_bounds__(B) k_dj_filt(const uint32_t* __restrict__ pkey, uint64_t np, uint32_t kmin,
                                               uint32_t range, const uint2* __restrict__ lc, uint64_t units,
                                               const uint64_t* __restrict__ unit_off, uint64_t total, FiltKey fk,
                                               uint8_t* __restrict__ fl, uint32_t* __restrict__ ccnt,
                                               const uint32_t* __restrict__ coff, JoinCols jc,
                                               uint32_t* __restrict__ out, uint64_t cap, uint64_t wlo,
                                               uint64_t whi) {
  __shared__ uint32_t s_row[B / 64][64];                    // owner_of_round's row per wave
  dj_filt_body<MODE, NPC, NBC, CH, XU>(pkey, np, kmin, range, lc, units, unit_off, total, fk, fl, ccnt, coff, jc, out,
                                       cap, wlo, whi, s_row[threadIdx.x >> 6]);
}

// MODE 3: chunks of CH outputs, each wave's kept rows staged in LDS, then
// written to the chunk's slots [(w - wlo) CH, + ccnt[w]) of `out` (a scratch
// for k_chunk_compact), or -- kept non-null -- at a place reserved by one
// atomic on *kept (A/B: DAS_FILT_STAGED=atomic)
template <int NPC, int NBC, int CH>
__global__ void __launch_bounds__(B) k_dj_filt_staged(const uint32_t* __restrict__ pkey, uint64_t np, uint32_t kmin,
                                                      uint32_t range, const uint2* __restrict__ lc, uint64_t units,
                                                      const uint64_t* __restrict__ unit_off, uint64_t total,
                                                      FiltKey fk, JoinCols jc, uint32_t* __restrict__ out,
                                                      uint64_t cap, uint64_t wlo, uint64_t whi,
                                                      uint32_t* __restrict__ ccnt, unsigned long long* __restrict__ kept,
                                                      const uint32_t* __restrict__ cunit) {
  __shared__ uint32_t s_row[B / 64][64];
  __shared__ __attribute__((aligned(16))) uint32_t s_stage[B / 64][(NPC + NBC) * CH];
  dj_filt_body<3, NPC, NBC, CH, kXUnroll>(pkey, np, kmin, range, lc, units, unit_off, total, fk, nullptr, ccnt,
                                          nullptr, jc, out, cap, wlo, whi, s_row[threadIdx.x >> 6],
                                          s_stage[threadIdx.x >> 6], kept, cunit);
}

// For every CH-output chunk, the unit holding its first output (the last unit
// u with unit_off[u] <= w CH), one thread per chunk: the walk's per-chunk
// search (4 dependent rounds inside its latency chain) becomes one load
template <int CH>
__global__ void __launch_bounds__(B) k_chunk_units(const uint64_t* __restrict__ unit_off, uint64_t units,
                                                   uint64_t chunks, uint32_t* __restrict__ cunit) {
  for (uint64_t w = blockIdx.x * (uint64_t)B + threadIdx.x; w < chunks; w += (uint64_t)gridDim.x * B) {
    const uint64_t ob = w * CH;
    uint64_t lo = 0, hi = units;
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (unit_off[mid] <= ob) lo = mid;
      else hi = mid;
    }
    cunit[w] = (uint32_t)lo;
  }
}

// MODE 2's second step: chunk w's kept rows [(w - wlo) CH, + cnt[w]) of the
// scratch columns move to [off[w], off[w] + cnt[w]) of the output, one wave
// per chunk of [wlo, whi), every column (ncols <= kMaxCols).
template <int CH>
__global__ void __launch_bounds__(B) k_chunk_compact(const uint32_t* __restrict__ src, uint64_t scap,
                                                     const uint32_t* __restrict__ cnt,
                                                     const uint32_t* __restrict__ off, uint64_t wlo, uint64_t whi,
                                                     int ncols, uint32_t* __restrict__ dst, uint64_t dcap) {
  // 16-byte moves: a head of up to 3 rows aligns the destination, then each
  // lane moves 4 rows per dwordx4 load (dword-aligned) and nontemporal
  // dwordx4 store, then a tail of up to 3 rows (dcap is a multiple of 64)
  const uint64_t waves = (uint64_t)gridDim.x * (B / 64);
  const uint32_t lane = (uint32_t)__lane_id();
  for (uint64_t w = wlo + blockIdx.x * (uint64_t)(B / 64) + (threadIdx.x >> 6); w < whi; w += waves) {
    const uint32_t n = cnt[w];
    const uint64_t s0 = (w - wlo) * CH, d0 = off[w];
    const uint32_t h = (4u - (uint32_t)(d0 & 3u)) & 3u;
    const uint32_t head = h < n ? h : n;
    const uint32_t nq = (n - head) / 4u;
    const uint32_t t0 = head + 4u * nq;
    for (int k = 0; k < ncols; ++k) {
      const uint32_t* sc = src + (uint64_t)k * scap + s0;
      uint32_t* dc = dst + (uint64_t)k * dcap + d0;
      if (lane < head) dc[lane] = sc[lane];
      u32x4_a4 x[CH / 256];
#pragma unroll
      for (int j = 0; j < CH / 256; ++j) {
        const uint32_t q = (uint32_t)j * 64u + lane;
        if (q < nq) x[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_a4*>(sc + head + 4u * q));
      }
#pragma unroll
      for (int j = 0; j < CH / 256; ++j) {
        const uint32_t q = (uint32_t)j * 64u + lane;
        if (q < nq) store16<true>(dc + head + 4u * q, u32x4{x[j].x, x[j].y, x[j].z, x[j].w});
      }
      if (t0 + lane < n) dc[t0 + lane] = sc[t0 + lane];
    }
  }
}

// Single pass of the filtered expansion.  A block takes kFuseChunks 1024-output
// chunks per wave; pass A tests every output's build value against the key
// bitmap (flag bytes in LDS, kept count per chunk), ONE atomic per block
// reserves the block's kept outputs at the end of the output, pass B re-walks
// the chunks (probe rows, owner prefixes and build rows are cache-resident now)
// and writes the kept outputs in chunk order.  Blocks land in completion
// order, so the output is not sorted; no flag array goes through HBM and the
// virtual outputs are walked from HBM once.
constexpr int kFuseChunks = 4;
template <int NPC = -1, int NBC = -1>
__global__ void __launch_bounds__(B) k_dj_filt_fused(const uint32_t* __restrict__ pkey, uint64_t np, uint32_t kmin,
                                                     uint32_t range, const uint2* __restrict__ lc, uint64_t units,
                                                     const uint64_t* __restrict__ unit_off, uint64_t total,
                                                     FiltKey fk, JoinCols jc, uint32_t* __restrict__ out,
                                                     uint64_t cap, unsigned long long* __restrict__ kept) {
  __shared__ uint8_t sflag[B / 64][kFuseChunks][kBalChunk];
  __shared__ uint32_t s_cnt[B / 64];
  __shared__ unsigned long long s_base;
  const int lane = __lane_id();
  const int wv = threadIdx.x >> 6;
  const uint64_t lt = __lanemask_lt();
  const uint64_t chunks = (total + kBalChunk - 1) / kBalChunk;
  const uint64_t per_block = (uint64_t)(B / 64) * kFuseChunks;
  const int ncp = NPC >= 0 ? NPC : jc.np, ncb = NBC >= 0 ? NBC : jc.nb;
  const uint32_t* pp[4];
  const uint32_t* bp[4];
  uint32_t* po[4];
  uint32_t* bo[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    pp[i] = i < ncp ? jc.p[i] : nullptr;
    bp[i] = i < ncb ? jc.b[i] : nullptr;
    po[i] = i < ncp ? out + (uint64_t)jc.po[i] * cap : nullptr;
    bo[i] = i < ncb ? out + (uint64_t)jc.bo[i] * cap : nullptr;
  }
  // block-uniform trip count: every wave reaches the barriers
  for (uint64_t it = blockIdx.x; it * per_block < chunks; it += gridDim.x) {
    uint32_t cnt[kFuseChunks];
    uint64_t cbase[kFuseChunks];
    for (int pass = 0; pass < 2; ++pass) {
      if (pass == 1) {
        uint32_t tot = 0;
#pragma unroll
        for (int k = 0; k < kFuseChunks; ++k) tot += cnt[k];
        if (lane == 0) s_cnt[wv] = tot;
        __syncthreads();
        if (threadIdx.x == 0) {
          uint32_t all = 0;
          for (int w = 0; w < B / 64; ++w) all += s_cnt[w];
          s_base = all ? atomicAdd(kept, (unsigned long long)all) : 0ull;
        }
        __syncthreads();
        uint64_t o0 = s_base;
        for (int w = 0; w < wv; ++w) o0 += s_cnt[w];
#pragma unroll
        for (int k = 0; k < kFuseChunks; ++k) {
          cbase[k] = o0;
          o0 += cnt[k];
        }
      }
#pragma unroll
      for (int k = 0; k < kFuseChunks; ++k) {
        const uint64_t w = it * per_block + (uint64_t)wv * kFuseChunks + k;
        if (pass == 0) cnt[k] = 0;
        if (w >= chunks || (pass == 1 && !cnt[k])) continue;
        uint8_t* fl = sflag[wv][k];
        const uint64_t ob = w * kBalChunk;
        const uint64_t oe = ob + kBalChunk < total ? ob + kBalChunk : total;
        uint64_t ulo = 0, uhi = units;                 // last unit with unit_off[u] <= ob
        while (uhi - ulo > 1) {
          const uint64_t step = (uhi - ulo + 63) / 64;
          const uint64_t idx = ulo + (uint64_t)lane * step;
          const bool ok = idx < uhi && unit_off[idx] <= ob;
          const uint64_t m = __ballot(ok);
          const uint64_t nlo = ulo + (uint64_t)(63 - __clzll((long long)m)) * step;
          uhi = nlo + step < uhi ? nlo + step : uhi;
          ulo = nlo;
        }
        uint32_t run = 0;
        for (uint64_t u = ulo; u < units; ++u) {
          uint64_t base = unit_off[u];
          if (base >= oe) break;
          const uint64_t r0 = u * kXRows;
          uint2 e[kXGroups];
#pragma unroll
          for (int g = 0; g < kXGroups; ++g) {
            const uint64_t r = r0 + g * 64 + lane;
            const uint32_t d = r < np ? pkey[r] - kmin : 0xFFFFFFFFu;
            e[g] = d < range ? lc[d] : make_uint2(0u, 0u);
          }
#pragma unroll
          for (int g = 0; g < kXGroups; ++g) {
            const uint32_t c = e[g].y;
            const uint32_t inc = wave_inclusive_scan(c);
            const uint32_t tot = (uint32_t)__shfl(inc, 63, 64);
            const uint32_t pre = inc - c;
            const uint64_t gb = base, ge = base + tot;
            base = ge;
            if (ge <= ob || gb >= oe) continue;
            const uint32_t rs = (uint32_t)((ob > gb ? ob : gb) - gb), re = (uint32_t)((oe < ge ? oe : ge) - gb);
            const uint64_t r = r0 + g * 64 + lane;
            uint32_t pv[4] = {0u, 0u, 0u, 0u};
            if (pass == 1) {
#pragma unroll
              for (int i = 0; i < 4; ++i)
                if (i < ncp) pv[i] = r < np ? pp[i][r] : 0u;
            }
            for (uint32_t o0 = rs; o0 < re; o0 += 64 * kXUnroll) {
              const int nr = (re - o0) >= 64u * kXUnroll ? kXUnroll : (int)((re - o0 + 63) / 64);
              uint32_t o[kXUnroll], br[kXUnroll];
              int ll[kXUnroll];
#pragma unroll
              for (int q = 0; q < kXUnroll; ++q) {
                o[q] = o0 + (uint32_t)(q * 64 + lane);
                ll[q] = 0;
                br[q] = 0;
                if (q >= nr) continue;
                int l = 0;                             // owner: max lane with pre <= o
#pragma unroll
                for (int st = 32; st >= 1; st >>= 1) {
                  const uint32_t pl = (uint32_t)__shfl(pre, l + st, 64);
                  if (l + st < 64 && pl <= o[q]) l += st;
                }
                ll[q] = l;
                br[q] = lane_get(e[g].x, l) + (o[q] - (uint32_t)__shfl(pre, l, 64));
              }
              if (pass == 0) {
                uint32_t v[kXUnroll];
#pragma unroll
                for (int q = 0; q < kXUnroll; ++q) v[q] = (q < nr && o[q] < re) ? fk.col[br[q]] - fk.lo : 0xFFFFFFFFu;
                uint32_t wd[kXUnroll];
#pragma unroll
                for (int q = 0; q < kXUnroll; ++q) wd[q] = v[q] < fk.range ? fk.bits[v[q] >> 5] : 0u;
#pragma unroll
                for (int q = 0; q < kXUnroll; ++q) {
                  if (q >= nr) continue;
                  const bool f = v[q] < fk.range && ((wd[q] >> (v[q] & 31)) & 1u);
                  if (o[q] < re) fl[gb + o[q] - ob] = f ? 1 : 0;
                  run += (uint32_t)__popcll(__ballot(f));
                }
              } else {
                bool f[kXUnroll];
#pragma unroll
                for (int q = 0; q < kXUnroll; ++q) f[q] = q < nr && o[q] < re && fl[gb + o[q] - ob] != 0;
                uint32_t bv[kXUnroll][4];
#pragma unroll
                for (int q = 0; q < kXUnroll; ++q)
#pragma unroll
                  for (int i = 0; i < 4; ++i) bv[q][i] = (i < ncb && f[q]) ? bp[i][br[q]] : 0u;
#pragma unroll
                for (int q = 0; q < kXUnroll; ++q) {
                  if (q >= nr) continue;
                  const uint64_t m = __ballot(f[q]);
                  const uint64_t pos = cbase[k] + run + __popcll(m & lt);
                  run += (uint32_t)__popcll(m);
#pragma unroll
                  for (int i = 0; i < 4; ++i) {
                    if (i >= ncp) break;
                    const uint32_t x = lane_get(pv[i], ll[q]);
                    if (f[q]) po[i][pos] = x;
                  }
                  if (f[q]) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                      if (i < ncb) bo[i][pos] = bv[q][i];
                  }
                }
              }
            }
          }
        }
        if (pass == 0) cnt[k] = run;
      }
    }
    __syncthreads();                                   // LDS flags and counts reused next iteration
  }
}

}  // namespace

ColSet cols_of(const Table& t) {
  ColSet s{};
  s.n = t.ncols;
  for (int c = 0; c < t.ncols; ++c) s.c[c] = t.col(c);
  return s;
}

// perm sorted by the given columns (LSD, stable).
void sort_perm(const ColSet& cs, uint64_t n, uint32_t* perm, int bits, hipStream_t s) {
  iota(perm, n, s);
  if (n <= 1) return;
  DBuf<uint32_t> key(n, s);
  for (int c = cs.n - 1; c >= 0; --c) {
    gather_u32(cs.c[c], perm, key.p, n, s);
    radix_sort_pairs<uint32_t>(key.p, perm, n, 0, bits > 0 ? bits : 1, s);
  }
}

int id_bits(const Ctx& c) { return bits_for(c.idx.n_atoms ? c.idx.n_atoms - 1 : 0); }

// Gathers rows idx[0..m) of table `a` into a new table (same schema).
namespace {
// output row o -> the source row of the range holding it (prefix = exclusive
// range-length sums, n_ranges + 1 entries)
__global__ void k_gather_ranges(ColSet src, const uint64_t* prefix, const uint64_t* begin, uint32_t n_ranges,
                                uint64_t m, uint32_t* dst, uint64_t cap) {
  for (uint64_t o = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; o < m; o += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t lo = 0, hi = n_ranges;                  // last range with prefix[r] <= o
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (prefix[mid] <= o) lo = mid;
      else hi = mid;
    }
    const uint64_t r = begin[lo] + (o - prefix[lo]);
    for (int k = 0; k < src.n; ++k) dst[(uint64_t)k * cap + o] = src.c[k][r];
  }
}
}  // namespace

std::unique_ptr<Table> gather_ranges(Ctx& c, const Table& a, const uint64_t* begin, const uint64_t* end,
                                     uint32_t n_ranges) {
  std::vector<uint64_t> h(2 * (uint64_t)n_ranges + 1, 0);
  uint64_t m = 0;
  for (uint32_t i = 0; i < n_ranges; ++i) {
    DAS_CHECK(begin[i] <= end[i] && end[i] <= a.nrows, DAS_E_INVALID, "gather range outside the table");
    h[i] = m;                                        // prefix
    h[n_ranges + 1 + i] = begin[i];
    m += end[i] - begin[i];
  }
  h[n_ranges] = m;
  auto t = new_table_like(c, a, m);
  t->nrows = m;
  if (m && a.ncols) {
    DBuf<uint64_t> d(h.size(), c.s);
    // from pageable memory: the runtime stages it before returning, so no
    // later user of the pinned staging buffer can overwrite a copy the
    // stream has not reached yet
    DAS_HIP(hipMemcpyAsync(d.p, h.data(), 8 * h.size(), hipMemcpyHostToDevice, c.s));
    hipLaunchKernelGGL(k_gather_ranges, G(m), dim3(B), 0, c.s, cols_of(a), (const uint64_t*)d.p,
                       (const uint64_t*)d.p + n_ranges + 1, n_ranges, m, t->data, t->cap);
    DAS_HIP(hipGetLastError());
  }
  return t;
}

std::unique_ptr<Table> gather_table(Ctx& c, const Table& a, const uint32_t* idx, uint64_t m) {
  auto t = new_table_like(c, a, m);
  t->nrows = m;
  if (m && a.ncols) {
    hipLaunchKernelGGL(k_gather_cols, G(m), dim3(B), 0, c.s, cols_of(a), idx, m, t->data, t->cap);
    DAS_HIP(hipGetLastError());
  }
  return t;
}

// ---------------------------------------------------------------------------
// Stream compaction by a row predicate, order kept: per-tile counts -> scan
// of the tile counts (its total sizes the output; one read-back) -> each
// tile re-evaluates the predicate, ranks its rows with wave scans and writes
// the kept rows' columns straight to their slots.  No per-row scan or index
// array goes through HBM.
// ---------------------------------------------------------------------------
// The tile's predicates are evaluated for all kScanItems rounds at once, on
// clamped (always valid) row indices, so their loads are issued together
// instead of one dependent round trip per round.
template <typename Pred>
__device__ __forceinline__ uint32_t tile_flags(const Pred& pred, uint64_t base, uint64_t n) {
  bool f[kScanItems];
#pragma unroll
  for (int r = 0; r < kScanItems; ++r) {
    const uint64_t i = base + (uint64_t)r * kScanBlock + threadIdx.x;
    f[r] = pred(i < n ? i : n - 1) && i < n;
  }
  uint32_t bits = 0;
#pragma unroll
  for (int r = 0; r < kScanItems; ++r) bits |= (f[r] ? 1u : 0u) << r;
  return bits;
}

// Also stores each thread's kScanItems flags as one byte (n / 8 bytes in all),
// so the compaction pass reads the flags instead of re-evaluating the
// predicate (a semi-join's bitmap probe is random and L2-missing).
template <typename Pred>
__global__ void __launch_bounds__(kScanBlock) k_tile_count(Pred pred, uint64_t n, uint32_t* tcnt, uint8_t* fl) {
  static_assert(kScanItems <= 8, "one flag byte per thread");
  __shared__ uint32_t s[kScanBlock / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  const uint32_t bits = tile_flags(pred, base, n);
  fl[(uint64_t)blockIdx.x * kScanBlock + threadIdx.x] = (uint8_t)bits;
  uint32_t acc = __popc(bits);
  acc = wave_reduce_sum(acc);
  if (__lane_id() == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) tcnt[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

__global__ void __launch_bounds__(kScanBlock) k_compact_rows(const uint8_t* __restrict__ fl,
                                                             const uint32_t* __restrict__ toff, ColSet src,
                                                             uint32_t* __restrict__ out, uint64_t cap) {
  constexpr int W = kScanBlock / 64;
  __shared__ uint32_t s_wave[kScanItems][W];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  const int wave = threadIdx.x >> 6;
  const uint32_t bits = fl[(uint64_t)blockIdx.x * kScanBlock + threadIdx.x];
  uint32_t inc[kScanItems];
#pragma unroll
  for (int r = 0; r < kScanItems; ++r) {
    inc[r] = wave_incl_sum_u32((bits >> r) & 1u);
    if (__lane_id() == 63) s_wave[r][wave] = inc[r];
  }
  __syncthreads();
  uint32_t carry = toff[blockIdx.x], o[kScanItems];
#pragma unroll
  for (int r = 0; r < kScanItems; ++r) {
    uint32_t pre = carry, all = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      pre += w < wave ? s_wave[r][w] : 0u;
      all += s_wave[r][w];
    }
    o[r] = pre + inc[r] - 1;
    carry += all;
  }
  // column by column, the kept rows' loads of all rounds in flight together
  for (int k = 0; k < src.n; ++k) {
    const uint32_t* col = src.c[k];
    uint32_t v[kScanItems];
#pragma unroll
    for (int r = 0; r < kScanItems; ++r)
      v[r] = ((bits >> r) & 1u) ? col[base + (uint64_t)r * kScanBlock + threadIdx.x] : 0u;
#pragma unroll
    for (int r = 0; r < kScanItems; ++r)
      if ((bits >> r) & 1u) out[(uint64_t)k * cap + o[r]] = v[r];
  }
}

struct FlagPred {
  const uint32_t* keep;
  __device__ __forceinline__ bool operator()(uint64_t i) const { return keep[i] != 0; }
};

// Single-workgroup compaction of a small table (the result of an anchored
// query's filter): predicate, in-order ranks and column writes in one launch,
// the kept count published to the pinned slot.
template <typename Pred>
__global__ void __launch_bounds__(kSmallBlock) k_compact_small(Pred pred, uint64_t n, ColSet src, uint32_t* out,
                                                               uint64_t cap, uint32_t* slot, uint32_t seq,
                                                               const uint32_t* guard) {
  constexpr int W = kSmallBlock / 64;
  __shared__ uint32_t s_w[W];
  __shared__ uint32_t s_run;
  const int wave = threadIdx.x >> 6;
  const uint64_t lt = __lanemask_lt();
  if (guard && *guard) {                      // voided (block-uniform): the count says so
    if (threadIdx.x == 0) publish_u32(slot, seq, 0xFFFFFFFFu);
    return;
  }
  if (threadIdx.x == 0) s_run = 0;
  __syncthreads();
  for (uint64_t r0 = 0; r0 < n; r0 += kSmallBlock) {
    const uint64_t r = r0 + threadIdx.x;
    const bool keep = r < n && pred(r);
    const uint64_t m = __ballot(keep);
    if (__lane_id() == 0) s_w[wave] = __popcll(m);
    __syncthreads();
    uint32_t pos = s_run + __popcll(m & lt);
    for (int w = 0; w < wave; ++w) pos += s_w[w];
    if (keep)
      for (int k = 0; k < src.n; ++k) out[(uint64_t)k * cap + pos] = src.c[k][r];
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (int w = 0; w < W; ++w) t += s_w[w];
      s_run += t;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) publish_u32(slot, seq, s_run);
}

// Marks tile 0's count when *guard is set (a condition the host would
// otherwise read back before the count): the count's read-back then carries it.
__global__ void k_guard_count(uint32_t* tcnt, const uint32_t* guard) {
  if (threadIdx.x == 0 && *guard) tcnt[0] |= 0x80000000u;
}

// guard (optional): a device flag that voids the compaction (nullptr returned),
// checked with the count's read-back instead of a read-back of its own
template <typename Pred>
std::unique_ptr<Table> compact_pred(Ctx& c, const Table& a, Pred pred, const char* prof = nullptr,
                                    double pred_bytes = 4.0, const uint32_t* guard = nullptr) {
  const uint64_t n = a.nrows;
  if (!n) return gather_table(c, a, nullptr, 0);
  const char* sg = std::getenv("DAS_SMALL_GUARD");        // A/B: 0 = read the guard first
  const bool fused_guard = !(sg && sg[0] == '0');
  if (guard && (n >= (1ull << 31) || (n <= kSmallScan && !fused_guard))) {   // read it first
    if (read_u32(guard, c.s)) return nullptr;
    guard = nullptr;
  }
  if (n <= kSmallScan) {                          // one launch; the guard rides on its count
    auto t = new_table_like(c, a, n);
    const PubSlot ps = pub_reserve();
    hipLaunchKernelGGL((k_compact_small<Pred>), dim3(1), dim3(kSmallBlock), 0, c.s, pred, n, cols_of(a), t->data,
                       t->cap, ps.p, ps.seq, guard);
    DAS_HIP(hipGetLastError());
    uint32_t m = 0;
    pub_wait(ps, c.s, &m, 1);
    if (m == 0xFFFFFFFFu) return nullptr;
    t->nrows = m;
    return t;
  }
  const uint64_t tiles = (n + kScanTile - 1) / kScanTile;
  DAS_CHECK(tiles < (1ull << 31), DAS_E_UNSUPPORTED, "compaction: too many rows");
  DBuf<uint32_t> tcnt(tiles, c.s), toff(tiles + 1, c.s);
  DBuf<uint8_t> fl(tiles * kScanBlock, c.s);
  {
    std::optional<ProfScope> ps;
    if (prof) ps.emplace(c, prof, pred_bytes * n);
    hipLaunchKernelGGL((k_tile_count<Pred>), dim3((unsigned)tiles), dim3(kScanBlock), 0, c.s, pred, n, tcnt.p, fl.p);
    DAS_HIP(hipGetLastError());
  }
  if (guard) {
    hipLaunchKernelGGL(k_guard_count, dim3(1), dim3(64), 0, c.s, tcnt.p, guard);
    DAS_HIP(hipGetLastError());
  }
  uint64_t mx = 0;
  const uint64_t m = scan_total<uint32_t>(SpanIn<uint32_t>{tcnt.p}, tiles, toff.p, c.s, &mx);
  if (guard && mx >= 0x80000000ull) return nullptr;
  auto t = new_table_like(c, a, m);
  t->nrows = m;
  if (m && a.ncols) {
    std::optional<ProfScope> ps;
    if (prof) ps.emplace(c, "k_compact_rows", n / 8.0 + 8.0 * a.ncols * m);
    hipLaunchKernelGGL(k_compact_rows, dim3((unsigned)tiles), dim3(kScanBlock), 0, c.s, (const uint8_t*)fl.p,
                       (const uint32_t*)toff.p, cols_of(a), t->data, t->cap);
    DAS_HIP(hipGetLastError());
  }
  return t;
}

// keep flags -> compacted table
std::unique_ptr<Table> compact_table(Ctx& c, const Table& a, const uint32_t* keep) {
  return compact_pred(c, a, FlagPred{keep});
}

void join_ranges(Ctx& c, const ColSet& probe, uint64_t np, const ColSet& build_sorted, uint64_t nb, uint32_t* lo,
                 uint32_t* cnt) {
  if (!np) return;
  hipLaunchKernelGGL(k_join_count, G(np), dim3(B), 0, c.s, probe, np, build_sorted, nb, lo, cnt);
  DAS_HIP(hipGetLastError());
}

std::unique_ptr<Table> new_table(Ctx& c, int kind, int ncols, const int32_t* vars, uint64_t cap,
                                 const int32_t* member) {
  DAS_CHECK(ncols >= 0 && ncols <= kMaxCols, DAS_E_UNSUPPORTED, "too many columns in a binding table");
  auto t = std::make_unique<Table>();
  t->kind = kind;
  t->ncols = ncols;
  for (int i = 0; i < ncols; ++i) t->vars[i] = vars ? vars[i] : 0;
  for (int i = 0; i < ncols; ++i) t->member[i] = member ? member[i] : -1;
  for (int i = 0; i < ncols; ++i) {
    t->lo[i] = 0;
    t->hi[i] = kNone;
  }
  t->s = c.s;
  t->cap = col_stride(cap ? cap : 1);      // 16-byte aligned columns
  if (ncols) t->data = (uint32_t*)cache_alloc(4ull * ncols * t->cap, c.s);
  return t;
}

// ---------------------------------------------------------------------------
// Scans
// ---------------------------------------------------------------------------
namespace {

std::unique_ptr<Table> run_scan_rows(Ctx& c, ScanSpec& sp, uint64_t begin, uint64_t end, int kind, int ncols,
                                     const int32_t* vars);

// Bounds of a scan's output columns from the index's per-type column bounds
// (ordered: the source position; unordered: the union over wildcard positions).
void scan_bounds(const Index& idx, const ScanSpec& sp, uint32_t type_id, Table& t) {
  const uint32_t ar = sp.arity, ncol = ar + 1;
  auto src = [&](int col, uint32_t& lo, uint32_t& hi) {
    const auto& tb = idx.tbound[ar];
    const auto& gb = idx.gbound[ar];
    if (type_id != kNone && (uint64_t)(type_id + 1) * ncol * 2 <= tb.size()) {
      lo = tb[((uint64_t)type_id * ncol + col) * 2];
      hi = tb[((uint64_t)type_id * ncol + col) * 2 + 1];
    } else if ((uint64_t)col * 2 + 1 < gb.size()) {
      lo = gb[col * 2];
      hi = gb[col * 2 + 1];
    } else {
      lo = 0;
      hi = kNone;
    }
  };
  for (int k = 0; k < t.ncols; ++k) {
    if (!sp.unordered) {
      src(1 + sp.outpos[k], t.lo[k], t.hi[k]);
      continue;
    }
    if (sp.emit_link && k == 0) {
      src(0, t.lo[k], t.hi[k]);
      continue;
    }
    uint32_t lo = kNone, hi = 0;
    for (uint32_t i = 0; i < sp.nupos; ++i) {
      uint32_t l, h;
      src(1 + (int)sp.upos[i], l, h);
      lo = std::min(lo, l);
      hi = std::max(hi, h);
    }
    t.lo[k] = lo;
    t.hi[k] = hi;
  }
}

std::unique_ptr<Table> run_scan(Ctx& c, ScanSpec& sp, uint64_t begin, uint64_t end, int kind, int ncols,
                                const int32_t* vars, uint32_t type_id) {
  auto t = run_scan_rows(c, sp, begin, end, kind, ncols, vars);
  scan_bounds(c.idx, sp, type_id, *t);
  return t;
}

constexpr uint64_t kViewRows = 1ull << 20;   // scans views by default up to this size (Ctx::scan_views)

std::unique_ptr<Table> run_scan_rows(Ctx& c, ScanSpec& sp, uint64_t begin, uint64_t end, int kind, int ncols,
                                     const int32_t* vars) {
  const uint64_t n = end > begin ? end - begin : 0;
  if (!n) return new_table(c, kind, ncols, vars, 0);
  const uint64_t chunks = (n + kChunk - 1) / kChunk;
  DAS_CHECK(chunks < (1ull << 31), DAS_E_UNSUPPORTED, "scan range too large");
  if (sp.all_keep) {
    if (!sp.unordered && c.scan_views && (c.scan_views == 1 || n <= kViewRows) && sp.nout > 0 &&
        (int)sp.nout == ncols) {
      // consecutive source columns (stride = the index table's column
      // stride): the scan is a view of rows [begin, end) -- no copy
      const uint32_t* c0 = sp.col[1 + sp.outpos[0]];
      const int64_t st = sp.nout > 1 ? sp.col[1 + sp.outpos[1]] - c0 : (int64_t)n;
      bool ok = st >= (int64_t)n;
      for (uint32_t k = 1; k < sp.nout && ok; ++k) ok = sp.col[1 + sp.outpos[k]] == c0 + k * st;
      if (ok) {
        auto t = new_table(c, kind, 0, vars, 0);
        t->ncols = ncols;
        for (int i = 0; i < ncols; ++i) {
          t->vars[i] = vars[i];
          t->member[i] = -1;
          t->lo[i] = 0;
          t->hi[i] = kNone;
        }
        t->view = true;
        t->data = const_cast<uint32_t*>(c0) + begin;
        t->cap = (uint64_t)st;
        t->nrows = n;
        return t;
      }
    }
    auto t = new_table(c, kind, ncols, vars, n);
    t->nrows = n;
    if (!sp.unordered) {   // pure projection
      ProfScope ps(c, "k_project", 8.0 * sp.nout * n);
      hipLaunchKernelGGL(k_project, dim3(grid_for(n / 8 + 1, B, 8192)), dim3(B), 0, c.s, sp, begin, n, t->data, t->cap);
      DAS_HIP(hipGetLastError());
      return t;
    }
    ProfScope ps(c, "k_scan_write", 4.0 * n * (sp.arity + 1) + 4.0 * n * sp.nout);
    hipLaunchKernelGGL(k_scan_write, dim3((unsigned)chunks), dim3(B), 0, c.s, sp, begin, end, (const uint32_t*)nullptr,
                       t->data, t->cap);
    DAS_HIP(hipGetLastError());
    return t;
  }
  if (n <= kSmallScan) {
    auto t = new_table(c, kind, ncols, vars, n);
    const PubSlot ps = pub_reserve();
    {
      ProfScope pf(c, "k_scan_small", 4.0 * n * (sp.arity + 1) + 4.0 * n * sp.nout);
      hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(kSmallBlock), 0, c.s, sp, begin, end, t->data, t->cap, ps.p,
                         ps.seq);
      DAS_HIP(hipGetLastError());
    }
    uint32_t m = 0;
    pub_wait(ps, c.s, &m, 1);
    t->nrows = m;
    return t;
  }
  DBuf<uint32_t> cnt(chunks, c.s), off(chunks + 1, c.s);
  {
    ProfScope ps(c, "k_scan_count", 4.0 * n * sp.arity);
    hipLaunchKernelGGL(k_scan_count, dim3((unsigned)chunks), dim3(B), 0, c.s, sp, begin, end, cnt.p);
    DAS_HIP(hipGetLastError());
  }
  const uint64_t m = scan_total<uint32_t>(SpanIn<uint32_t>{cnt.p}, chunks, off.p, c.s);
  auto t = new_table(c, kind, ncols, vars, m);
  t->nrows = m;
  if (m) {
    ProfScope ps(c, "k_scan_write", 4.0 * n * (sp.arity + 1) + 4.0 * m * sp.nout);
    hipLaunchKernelGGL(k_scan_write, dim3((unsigned)chunks), dim3(B), 0, c.s, sp, begin, end, (const uint32_t*)off.p,
                       t->data, t->cap);
    DAS_HIP(hipGetLastError());
  }
  return t;
}

void set_cols(ScanSpec& sp, const RowTable& rt) {
  for (int k = 0; k <= rt.arity; ++k) sp.col[k] = rt.col(k);
  // ScanSpec reads col[1 + p]; col[0] is the link id
}

}  // namespace

namespace {
// A Link scan resolved on the host: the spec, the row range(s) of the index
// table it reads, the output schema and order (scan_link runs it; the fused
// small-And chain embeds it as a stage).
struct ScanPrep {
  ScanSpec sp{};
  int32_t vars[kMaxCols] = {0};
  int ncols = 0;
  int kind = DAS_TABLE_ORDERED;
  std::vector<std::pair<uint64_t, uint64_t>> ranges;
  int sorted_pos = -1;
  bool empty = false;
};

void scan_prepare(Ctx& c, const das_link_scan_t& q, ScanPrep& P) {
  Index& idx = c.idx;
  DAS_CHECK(idx.built, DAS_E_NOT_BUILT, "index not built");
  const uint32_t ar = q.arity;
  DAS_CHECK(ar <= 8, DAS_E_INVALID, "arity > 8");
  // output schema
  int32_t* vars = P.vars;
  int& ncols = P.ncols;
  ScanSpec& sp = P.sp;
  sp.arity = ar;
  sp.no_overload = q.no_overload;
  sp.emit_link = q.emit_link;
  sp.unordered = q.ordered ? 0 : 1;
  int& kind = P.kind;
  kind = q.ordered ? DAS_TABLE_ORDERED : DAS_TABLE_UNORDERED;
  bool any_wild = false;
  for (uint32_t p = 0; p < ar; ++p) {
    sp.fixed[p] = q.target[p];
    if (q.target[p] == kNone) any_wild = true;
  }
  if (q.emit_link) { vars[ncols] = -1; sp.outpos[ncols] = -1; ++ncols; }
  if (q.ordered) {
    // distinct variables in ascending id order; repeated ones -> equality constraints
    int32_t first_pos[64];
    for (int i = 0; i < 64; ++i) first_pos[i] = -1;
    std::vector<std::pair<int32_t, uint32_t>> vp;
    for (uint32_t p = 0; p < ar; ++p)
      if (q.var[p] >= 0) vp.push_back({q.var[p], p});
    std::sort(vp.begin(), vp.end());
    for (size_t i = 0; i < vp.size(); ++i) {
      if (i > 0 && vp[i].first == vp[i - 1].first) {
        sp.eq_a[sp.neq] = vp[i - 1].second;
        sp.eq_b[sp.neq] = vp[i].second;
        ++sp.neq;
        continue;
      }
      DAS_CHECK(ncols < kMaxCols, DAS_E_UNSUPPORTED, "too many variables");
      vars[ncols] = vp[i].first;
      sp.outpos[ncols] = (int32_t)vp[i].second;
      ++ncols;
    }
    sp.nout = ncols;
  } else {
    for (uint32_t p = 0; p < ar; ++p)
      if (q.target[p] == kNone) sp.upos[sp.nupos++] = p;
    std::vector<int32_t> vs(q.var, q.var + q.n_vars);
    std::sort(vs.begin(), vs.end());
    for (int32_t v : vs) vars[ncols++] = v;
    DAS_CHECK(sp.nupos == q.n_vars, DAS_E_INVALID, "unordered scan: variables != wildcard positions");
    sp.nout = ncols;
  }
  auto empty = [&]() { P.empty = true; };
  if (ar == 0 || ar > (uint32_t)kMaxArity || idx.ttab[ar].rows == 0) return empty();
  if (q.type_id != kNone && q.type_id >= idx.n_types) return empty();
  // a black-listed type has no pattern keys (canonical_parser.py:144)
  if (q.type_id != kNone && idx.blocked(q.type_id)) return empty();
  // Families the reference indexes (canonical_parser.py:144-178)
  if (ar > (uint32_t)kMaxPosArity) {
    if (q.type_id != kNone || any_wild) return empty();   // only [*, e0..en]
  }
  auto& ranges = P.ranges;                                // row ranges of rt to scan
  const RowTable* rt = nullptr;
  std::vector<uint32_t> grounded;
  for (uint32_t p = 0; p < ar; ++p)
    if (q.target[p] != kNone) grounded.push_back(p);
  int& sorted_pos = P.sorted_pos;                         // output comes sorted by this position
  if (grounded.empty() || ar > (uint32_t)kMaxPosArity) {
    const bool typed = q.type_id != kNone;
    if (typed && ar <= (uint32_t)kMaxPosArity && q.order_pos >= 0 && (uint32_t)q.order_pos < ar &&
        idx.pidx[ar][q.order_pos].t.rows == idx.ttab[ar].rows) {
      // P_{a,p} holds the type's rows sorted by t_p: same range, sorted output
      rt = &idx.pidx[ar][q.order_pos].t;
      sorted_pos = q.order_pos;
    } else {
      rt = &idx.ttab[ar];
    }
    if (typed) {
      ranges.push_back({idx.type_off[ar][q.type_id], idx.type_off[ar][q.type_id + 1]});
    } else if (!idx.no_pattern_any) {
      ranges.push_back({0, rt->rows});
    } else {
      // '*' keys hold no black-listed link: the type segments around them
      uint64_t b = 0;
      for (uint32_t ty = 0; ty < idx.n_types && ty + 1 < idx.type_off[ar].size(); ++ty) {
        if (!idx.blocked(ty)) continue;
        if (idx.type_off[ar][ty] > b) ranges.push_back({b, idx.type_off[ar][ty]});
        b = std::max(b, idx.type_off[ar][ty + 1]);
      }
      if (rt->rows > b) ranges.push_back({b, rt->rows});
      if (ranges.empty()) return empty();
    }
  } else {
    // the cheapest P_{a,p} among the grounded positions: its key range(s)
    // (one per named type for a '*' type)
    std::vector<uint32_t> types;
    if (q.type_id != kNone) types.push_back(q.type_id);
    else
      for (uint32_t ty = 0; ty < idx.n_types; ++ty)
        if (idx.type_off[ar][ty + 1] > idx.type_off[ar][ty] && !idx.blocked(ty)) types.push_back(ty);
    uint64_t best = ~0ull;
    for (uint32_t p : grounded) {
      const PosIndex& P = idx.pidx[ar][p];
      if (!P.nkeys || types.empty()) return empty();
      std::vector<std::pair<uint64_t, uint64_t>> rr;
      std::vector<uint64_t> qlo, qhi;
      uint64_t total = 0;
      for (uint32_t ty : types) {
        const uint64_t k = ((uint64_t)ty << 32) | q.target[p];
        if (!P.h_ukey.empty()) {
          // host mirror of the keys: one binary search, no cache to consult
          const size_t i = std::lower_bound(P.h_ukey.begin(), P.h_ukey.end(), k) - P.h_ukey.begin();
          const bool has = i < P.h_ukey.size() && P.h_ukey[i] == k;
          rr.push_back(has ? std::pair<uint64_t, uint64_t>{P.h_uoff[i], P.h_uoff[i + 1]} : std::pair<uint64_t, uint64_t>{0, 0});
          continue;
        }
        const std::array<uint64_t, 4> ck{ar, p, k, 0};
        auto hit = idx.range_cache.find(ck);
        if (hit != idx.range_cache.end()) {
          rr.push_back(hit->second);
        } else {
          qlo.push_back(k);
          qhi.push_back(k + 1);
          rr.push_back({~0ull, ~0ull});
        }
      }
      if (!qlo.empty()) {
        const uint32_t nq = (uint32_t)qlo.size();
        std::vector<uint64_t> hr(2 * nq);
        if (!P.h_ukey.empty() || P.nkeys == 0) {
          // host mirror of the keys: no device round trip
          for (uint32_t i = 0; i < 2 * nq; ++i) {
            const uint64_t q = (i & 1) ? qhi[i >> 1] : qlo[i >> 1];
            hr[i] = P.h_uoff[std::lower_bound(P.h_ukey.begin(), P.h_ukey.end(), q) - P.h_ukey.begin()];
          }
        } else {
          uint64_t* st = reinterpret_cast<uint64_t*>(pinned_stage(32ull * nq));
          std::memcpy(st, qlo.data(), 8 * nq);
          std::memcpy(st + nq, qhi.data(), 8 * nq);
          const PubSlot ps = pub_reserve();
          hipLaunchKernelGGL(k_key_ranges_pub, dim3(1), dim3(256), 0, c.s, (const uint64_t*)P.ukey,
                             (const uint64_t*)P.uoff, P.nkeys, (const uint64_t*)st, (const uint64_t*)st + nq, nq,
                             st + 2 * nq, ps.p, ps.seq);
          DAS_HIP(hipGetLastError());
          pub_wait(ps, c.s, nullptr, 0);
          std::memcpy(hr.data(), st + 2 * nq, 16 * nq);
        }
        if (idx.range_cache.size() > (1u << 20)) idx.range_cache.clear();
        uint32_t j = 0;
        for (size_t i = 0; i < rr.size(); ++i)
          if (rr[i].first == ~0ull) {
            rr[i] = {hr[2 * j], hr[2 * j + 1]};
            idx.range_cache[std::array<uint64_t, 4>{ar, p, qlo[j], 0}] = rr[i];
            ++j;
          }
      }
      for (auto& r : rr) total += r.second - r.first;
      if (total < best) {
        best = total;
        ranges.clear();
        for (auto& r : rr)
          if (r.second > r.first) ranges.push_back(r);
        rt = &P.t;
        // this position's filter is implied by the range
        for (uint32_t pp = 0; pp < ar; ++pp) sp.fixed[pp] = q.target[pp];
        sp.fixed[p] = kNone;
        // P_{a,p} rows are (type, t_p, other targets in position order, id):
        // one key range comes out sorted by the first other target that is
        // not grounded (the grounded ones before it are filtered to one value)
        sorted_pos = -1;
        if (ranges.size() == 1)
          for (uint32_t q2 = 0; q2 < ar; ++q2) {
            if (q2 == p || q.target[q2] != kNone) continue;
            sorted_pos = (int)q2;
            break;
          }
      }
      if (best == 0) return empty();
    }
  }
  DAS_CHECK(rt != nullptr, DAS_E_INTERNAL, "scan without a table");
  for (auto& r : ranges) DAS_CHECK(r.first <= r.second && r.second <= rt->rows, DAS_E_INTERNAL, "scan range outside its table");
  set_cols(sp, *rt);
  bool filt = false;
  for (uint32_t p = 0; p < ar; ++p) filt |= sp.fixed[p] != kNone;
  sp.all_keep = !filt && sp.neq == 0 && !(sp.unordered && sp.nupos > 1) && !(!sp.unordered && sp.no_overload && sp.nout > 1);
  if (ranges.empty()) return empty();
}
}  // namespace

// Largest key range of P_{a,p} among the keys of named type `type`: an upper
// bound of any single-key scan of that (type, position) whatever the key.
__global__ void k_type_max_run(const uint64_t* __restrict__ ukey, const uint64_t* __restrict__ uoff, uint64_t nkeys,
                               uint64_t klo, uint64_t khi, unsigned long long* out) {
  __shared__ uint64_t s_b[2];
  if (threadIdx.x < 2) {                         // this block's copy of the type's key bounds
    const uint64_t v = threadIdx.x ? khi : klo;
    uint64_t lo = 0, hi = nkeys;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (ukey[mid] < v) lo = mid + 1; else hi = mid;
    }
    s_b[threadIdx.x] = lo;
  }
  __syncthreads();
  uint64_t m = 0;
  for (uint64_t k = s_b[0] + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < s_b[1];
       k += (uint64_t)gridDim.x * blockDim.x)
    m = max(m, uoff[k + 1] - uoff[k]);
  for (int d = 32; d >= 1; d >>= 1) m = max(m, (uint64_t)__shfl_xor((unsigned long long)m, d, 64));
  if (__lane_id() == 0 && m) atomicMax(out, (unsigned long long)m);
}

uint64_t type_max_run(Ctx& c, uint32_t a, uint32_t p, uint32_t type) {
  Index& idx = c.idx;
  const std::array<uint64_t, 4> key{a, p, type, ~0ull};          // (range_cache: these never collide)
  auto it = idx.range_cache.find(key);
  if (it != idx.range_cache.end()) return it->second.first;
  const PosIndex& P = idx.pidx[a][p];
  const uint64_t klo = (uint64_t)type << 32, khi = (uint64_t)(type + 1) << 32;
  uint64_t m = 0;
  if (!P.h_ukey.empty() || P.nkeys == 0) {
    const uint64_t b = std::lower_bound(P.h_ukey.begin(), P.h_ukey.end(), klo) - P.h_ukey.begin();
    const uint64_t e = std::lower_bound(P.h_ukey.begin(), P.h_ukey.end(), khi) - P.h_ukey.begin();
    for (uint64_t k = b; k < e; ++k) m = std::max<uint64_t>(m, P.h_uoff[k + 1] - P.h_uoff[k]);
  } else {
    DBuf<unsigned long long> out(1, c.s);
    fill_dev(out.p, 0, 8, c.s);
    hipLaunchKernelGGL(k_type_max_run, dim3(grid_for(P.nkeys, B, 1024)), dim3(B), 0, c.s, (const uint64_t*)P.ukey,
                       (const uint64_t*)P.uoff, P.nkeys, klo, khi, out.p);
    DAS_HIP(hipGetLastError());
    m = read_u64(reinterpret_cast<const uint64_t*>(out.p), c.s);
  }
  idx.range_cache[key] = {m, 0};
  return m;
}

uint64_t scan_bound(Ctx& c, const das_link_scan_t& q) {
  const uint32_t ar = q.arity;
  bool grounded = false;
  for (uint32_t p = 0; p < ar && p < 8; ++p) grounded |= q.target[p] != kNone;
  if (!grounded) return scan_estimate(c, q);               // no anchor: the same rows every time
  if (ar == 0 || ar > (uint32_t)kMaxPosArity || q.type_id == kNone || q.type_id >= c.idx.n_types) return ~0ull;
  uint64_t best = ~0ull;
  for (uint32_t p = 0; p < ar; ++p)
    if (q.target[p] != kNone && c.idx.pidx[ar][p].nkeys) best = std::min(best, type_max_run(c, ar, p, q.type_id));
  return best;
}

uint64_t scan_estimate(Ctx& c, const das_link_scan_t& q) {
  ScanPrep P;
  scan_prepare(c, q, P);
  if (P.empty) return 0;
  uint64_t n = 0;
  for (auto& r : P.ranges) n += r.second - r.first;
  return n;
}

std::unique_ptr<Table> scan_link(Ctx& c, const das_link_scan_t& q) {
  ScanPrep P;
  scan_prepare(c, q, P);
  if (P.empty) return new_table(c, P.kind, P.ncols, P.vars, 0);
  ScanSpec& sp = P.sp;
  std::unique_ptr<Table> t;
  if (P.ranges.size() == 1) {
    t = run_scan(c, sp, P.ranges[0].first, P.ranges[0].second, P.kind, P.ncols, P.vars, q.type_id);
  } else {
    std::vector<std::unique_ptr<Table>> parts;
    std::vector<const Table*> pp;
    for (auto& r : P.ranges) {
      parts.push_back(run_scan(c, sp, r.first, r.second, P.kind, P.ncols, P.vars, q.type_id));
      pp.push_back(parts.back().get());
    }
    t = concat(c, pp.data(), (int)pp.size());
  }
  if (P.sorted_pos >= 0 && q.ordered)
    for (int k = 0; k < t->ncols; ++k)
      if (sp.outpos[k] == P.sorted_pos) t->sorted_col = k;
  return t;
}

std::unique_ptr<Table> scan_template(Ctx& c, const das_template_scan_t& q) {
  Index& idx = c.idx;
  DAS_CHECK(idx.built, DAS_E_NOT_BUILT, "index not built");
  DAS_CHECK(q.ctype_id < idx.ctype_range.size(), DAS_E_INVALID, "bad ctype id");
  const CtypeRange& cr = idx.ctype_range[q.ctype_id];
  DAS_CHECK(q.arity == cr.arity, DAS_E_INVALID, "template arity mismatch");
  ScanSpec sp{};
  sp.arity = cr.arity;
  for (uint32_t p = 0; p < cr.arity; ++p) sp.fixed[p] = kNone;
  sp.no_overload = q.no_overload;
  sp.emit_link = q.emit_link;
  sp.unordered = q.ordered ? 0 : 1;
  int32_t vars[kMaxCols];
  int ncols = 0;
  if (q.emit_link) { vars[ncols] = -1; sp.outpos[ncols] = -1; ++ncols; }
  if (q.ordered) {
    std::vector<std::pair<int32_t, uint32_t>> vp;
    for (uint32_t p = 0; p < cr.arity; ++p) vp.push_back({q.var[p], p});
    std::sort(vp.begin(), vp.end());
    for (size_t i = 0; i < vp.size(); ++i) {
      if (i > 0 && vp[i].first == vp[i - 1].first) {
        sp.eq_a[sp.neq] = vp[i - 1].second;
        sp.eq_b[sp.neq] = vp[i].second;
        ++sp.neq;
        continue;
      }
      vars[ncols] = vp[i].first;
      sp.outpos[ncols] = (int32_t)vp[i].second;
      ++ncols;
    }
  } else {
    std::vector<int32_t> vs(q.var, q.var + cr.arity);
    std::sort(vs.begin(), vs.end());
    for (int32_t v : vs) vars[ncols++] = v;
    for (uint32_t p = 0; p < cr.arity; ++p) sp.upos[sp.nupos++] = p;
  }
  sp.nout = ncols;
  const int kind = q.ordered ? DAS_TABLE_ORDERED : DAS_TABLE_UNORDERED;
  DAS_CHECK(cr.begin <= cr.end && cr.end <= idx.ctab[cr.arity].rows, DAS_E_INTERNAL, "template range outside its table");
  set_cols(sp, idx.ctab[cr.arity]);
  sp.all_keep = sp.neq == 0 && !(sp.unordered && sp.nupos > 1) && !(!sp.unordered && sp.no_overload && sp.nout > 1);
  return run_scan(c, sp, cr.begin, cr.end, kind, ncols, vars, kNone);
}

// ---------------------------------------------------------------------------
// Join, antijoin, dedup, concat
// ---------------------------------------------------------------------------
// Direct-address join on a single shared variable; nullptr if the build key
// range is too sparse for a dense offsets array (caller falls back to sort +
// binary search).
// Probe expansion shared by the direct-address join and the index join:
// probe row r matches the build rows lc[pkey[r] - kmin] = (first, count).
std::unique_ptr<Table> dj_expand(Ctx& c, const Table& P, const uint32_t* pkey, uint32_t kmin, uint64_t range,
                                 const uint2* lc, const JoinCols& jc, int nu, const int32_t* uni,
                                 double build_bytes) {
  const uint64_t units = (P.nrows + kXRows - 1) / kXRows;
  const unsigned grid = grid_for(units, B / 64, 65535u * 4u);
  DBuf<uint64_t> tot(units, c.s), toff(units + 1, c.s);
  bool fused = false;
  PubSlot ps_count{};
  {
    // a view's payload columns are read cold by the expansion: warm them here
    const uint32_t* w[2] = {nullptr, nullptr};
    int nw = 0;
    const char* wf = std::getenv("DAS_DJ_WARM");           // A/B: 0 = no warming
    if (P.view && !(wf && wf[0] == '0'))
      for (int i = 0; i < jc.np && nw < 2; ++i)
        if (jc.p[i] != pkey) w[nw++] = jc.p[i];
    // (DAS_COUNT_PUB=0: the count and the scan as two launches, A/B)
    const char* cpe = std::getenv("DAS_COUNT_PUB");
    fused = units <= kCountPubUnits && !(cpe && cpe[0] == '0');
    ProfScope ps(c, fused ? "k_dj_count_pub" : "k_dj_count", 4.0 * P.nrows);
    if (fused) {
      ScanCtr& ct = scan_ctr(c.s);
      ps_count = pub_reserve();
      hipLaunchKernelGGL(k_dj_count_pub, dim3(grid), dim3(B), 0, c.s, pkey, P.nrows, kmin, (uint32_t)range, lc, units,
                         tot.p, w[0], w[1], toff.p, ct.p, (unsigned long long)(ct.base + grid - 1), ps_count.p,
                         ps_count.seq);
      ct.base += grid;
    } else {
      hipLaunchKernelGGL(k_dj_count, dim3(grid), dim3(B), 0, c.s, pkey, P.nrows, kmin, (uint32_t)range,
                         lc, units, tot.p, w[0], w[1]);
    }
    DAS_HIP(hipGetLastError());
  }
  uint64_t tm[2];
  if (fused) {
    uint32_t wv[4];
    pub_wait(ps_count, c.s, wv, 4);
    tm[0] = (uint64_t)wv[0] | ((uint64_t)wv[1] << 32);
    tm[1] = (uint64_t)wv[2] | ((uint64_t)wv[3] << 32);
  } else {
    tm[0] = scan_total<uint64_t>(SpanIn<uint64_t>{tot.p}, units, toff.p, c.s, &tm[1]);   // toff[units] = total
  }
  const uint64_t total = tm[0];
  // a unit owning far more outputs than a wave should expand alone (hub
  // keys) -> output-balanced expansion
  const char* fb = std::getenv("DAS_DJ_BALANCED");        // tests: force either expansion
  // ... and so should a probe with a high fan-out everywhere (an index join
  // of 10^5 anchors x 10^2 links each): its few hundred waves would each
  // expand thousands of outputs while most of the chip idles
  const bool fanout = total >= (1ull << 14) && total / kBalChunk > 2 * units;
  const bool balanced = fb ? fb[0] == '1' : (tm[1] > kHeavyUnit || fanout);
  auto out = new_table(c, DAS_TABLE_ORDERED, nu, uni, total);
  out->nrows = total;
  if (total) {
    // algorithmic bytes: probe payload + build payload +
    // output, per launch (a schema wider than 4 + 4 columns is written by
    // several launches, each reading the key and its own columns)
    const bool one = jc.np <= 4 && jc.nb <= 4;
    // build_bytes < 0: -(bytes per output) -- an index join reads one P row per output
    if (build_bytes < 0) build_bytes = -build_bytes * (double)total;
    auto bytes = [&](int np, int nb) {
      if (one) return 4.0 * P.nrows * P.ncols + build_bytes + 4.0 * total * nu;
      return 4.0 * P.nrows * (np + 1) + (jc.nb ? build_bytes * nb / jc.nb : 0.0) + 4.0 * total * (np + nb);
    };
    dj_write(grid, c.s, pkey, P.nrows, kmin, (uint32_t)range, lc, units, (const uint64_t*)toff.p, jc,
             out->data, out->cap, total, balanced, bytes);
    DAS_HIP(hipGetLastError());
  }
  return out;
}

std::unique_ptr<Table> direct_join(Ctx& c, const Table& P, const Table& Q, int32_t var,
                                   const std::vector<int32_t>& uni) {
  auto colof = [](const Table& t, int32_t v) {
    for (int i = 0; i < t.ncols; ++i) if (t.vars[i] == v) return i;
    return -1;
  };
  const uint32_t* qkey = Q.col(colof(Q, var));
  const uint32_t* pkey = P.col(colof(P, var));
  uint32_t h[2] = {0u, (uint32_t)(c.idx.n_atoms ? c.idx.n_atoms - 1 : 0)};
  const int qk = colof(Q, var);
  if (Q.hi[qk] != kNone && Q.lo[qk] <= Q.hi[qk]) {
    // host-known bound of the key column (index column bounds): no round trip
    h[0] = Q.lo[qk];
    h[1] = Q.hi[qk];
  } else if (!c.idx.n_atoms || c.idx.n_atoms > std::max<uint64_t>(8 * Q.nrows, 1ull << 22)) {
    // large id space: bound the offsets array by the build keys' actual range
    // (one workgroup publishing both bounds for build sides up to 2^18 rows,
    // else atomics + a published read-back -- not a blit copy and a stream
    // synchronisation: ~15-20 us per join of bio QUERY_2 / QUERY_3, r4 trace)
    if (Q.nrows <= (1ull << 18)) {
      const PubSlot ps = pub_reserve();
      hipLaunchKernelGGL(k_key_minmax_pub, dim3(1), dim3(1024), 0, c.s, qkey, Q.nrows, ps.p, ps.seq);
      DAS_HIP(hipGetLastError());
      pub_wait(ps, c.s, h, 2);
    } else {
      DBuf<uint32_t> mm(2, c.s);
      fill_dev(mm.p, 0xFF, 4, c.s);
      fill_dev(mm.p + 1, 0, 4, c.s);
      hipLaunchKernelGGL(k_key_minmax, dim3(grid_for(Q.nrows, B, 512)), dim3(B), 0, c.s, qkey, Q.nrows, mm.p);
      DAS_HIP(hipGetLastError());
      read_u32x2(mm.p, mm.p + 1, c.s, h);
    }
  }
  const uint64_t range = (uint64_t)h[1] - h[0] + 1;
  // the key-slot arrays cost ~20 B per slot of streaming work; the sort-merge
  // alternative costs a log2(|Q|)-step random search per probe row, so a
  // slot range up to a few times either side's rows still pays (10^9-link
  // KBs: node ranges of 10^8 ids against 10^8-row probes).  (Small joins
  // over a wide range -- bio QUERY_3's 2*10^4-row sides keyed by Member link
  // ids over 1.4*10^7 slots -- measured no faster sorted: 2^22 instead of
  // 2^26 below, bio step 1.994 vs 1.964 ms, profiles/archive/r3_bio_range_floor_ab.json)
  if (range > std::max<uint64_t>(std::max<uint64_t>(8 * Q.nrows, 4 * P.nrows), 1ull << 26) ||
      range >= 0xFFFFFFFFull || Q.nrows >= 0xFFFFFFFFull)
    return nullptr;
  const uint32_t kmin = h[0];
  std::unique_ptr<Table> Qs;
  const Table* Qb = &Q;
  // the (lo, cnt) descriptor of every key slot; one more entry holds the
  // sparse build's running base.  The sparse build (fewer launches, ~8 B per
  // slot instead of ~36) takes at most 2^18 build rows: its bases come from
  // one atomic per wave on one counter
  DBuf<uint2> lc;
  auto expand = [&](const Table& Qb, const uint2* lcp) {
    const int nu = (int)uni.size();
    JoinCols jc{};
    for (int k = 0; k < nu; ++k) {
      const int ip = colof(P, uni[k]);
      if (ip >= 0) { jc.p[jc.np] = P.col(ip); jc.po[jc.np++] = k; }
      else { jc.b[jc.nb] = Qb.col(colof(Qb, uni[k])); jc.bo[jc.nb++] = k; }
    }
    return dj_expand(c, P, pkey, kmin, range, lcp, jc, nu, uni.data(), 4.0 * Q.nrows * Q.ncols);
  };
  const char* bm = std::getenv("DAS_DJ_BUILD");   // A/B, tests: "dense" never, "sparse" whenever it fits
  const bool sparse = range < (1ull << 31) &&
      (bm && !std::strcmp(bm, "sparse") ? true
       : bm && !std::strcmp(bm, "dense") ? false : range > 16 * Q.nrows && range >= (1ull << 16) && Q.nrows <= (1ull << 18));
  if (sparse) {
    // few build rows over a wide slot range: descriptors written in place --
    // into the context's descriptor array, which stays all-zero between joins
    // (the build's own slots are cleared after the expansion: 2*10^4 slot
    // writes instead of a 112 MB fill per bio QUERY_3 join; DAS_ZLC=0: a
    // fresh array filled per join, A/B)
    const bool srt = Q.sorted_col == qk;
    const char* zf = std::getenv("DAS_ZLC");
    // the context keeps the zeroed array for ranges up to 2^26 slots (512 MB);
    // a wider range takes a fresh array filled for this join
    const bool reuse = !(zf && zf[0] == '0') && range + 1 <= kZlcMax;
    // from the first slot write until the build's own slots are cleared
    // again, any unwind (an allocation or launch failure, an expansion
    // throwing) leaves slots set: the guard drops the context's array, so the
    // next join starts from a fresh one
    // (one array per stream the context launches on: a join on a side
    // stream must not see another stream's slots before their clear ran)
    DBuf<uint2>& zlc = c.zlc_of(c.s);
    struct ZlcGuard {
      DBuf<uint2>& z;
      bool armed;
      ~ZlcGuard() {
        if (armed) z.release();
      }
    } zg{zlc, false};
    uint2* lcp = nullptr;
    {
      const bool fresh = !reuse || zlc.n < range + 1;
      ProfScope ps(c, "join_build", (srt ? 4.0 : 8.0 + 8.0 * Q.ncols) * Q.nrows + (fresh ? 8.0 * range : 0.0));
      if (reuse) {
        if (zlc.n < range + 1) {
          zlc.alloc(std::min<uint64_t>(std::max<uint64_t>(range + 1, 2 * zlc.n), kZlcMax), c.s);
          fill_dev(zlc.p, 0, 8 * zlc.n, c.s);
        }
        lcp = zlc.p;
        zg.armed = true;
      } else {
        lc.alloc(range + 1, c.s);
        fill_dev(lc.p, 0, 8 * (range + 1), c.s);
        lcp = lc.p;
      }
      DBuf<uint32_t> rk(srt ? 1 : Q.nrows, c.s);
      hipLaunchKernelGGL(k_lc_count, G(Q.nrows), dim3(B), 0, c.s, qkey, Q.nrows, kmin, (uint32_t)range, lcp, rk.p,
                         srt ? 1 : 0);
      if (!srt) {
        hipLaunchKernelGGL(k_lc_base, G(Q.nrows), dim3(B), 0, c.s, qkey, rk.p, Q.nrows, kmin, (uint32_t)range, lcp,
                           reinterpret_cast<uint32_t*>(lcp + range));
        Qs = new_table_like(c, Q, Q.nrows);
        Qs->nrows = Q.nrows;
        hipLaunchKernelGGL(k_lc_scatter, G(Q.nrows), dim3(B), 0, c.s, cols_of(Q), qkey, rk.p, Q.nrows, kmin,
                           (uint32_t)range, lcp, Qs->data, Qs->cap);
        Qb = Qs.get();
      }
      DAS_HIP(hipGetLastError());
    }
    if (!reuse) return expand(*Qb, lcp);
    if (const char* t = std::getenv("DAS_TEST_ZLC_THROW"); t && t[0] == '1')   // tests: an unwind mid-join
      DAS_CHECK(false, DAS_E_INTERNAL, "DAS_TEST_ZLC_THROW");
    std::unique_ptr<Table> out = expand(*Qb, lcp);
    hipLaunchKernelGGL(k_lc_clear, G(Q.nrows), dim3(B), 0, c.s, qkey, Q.nrows, kmin, (uint32_t)range, lcp);
    DAS_HIP(hipGetLastError());
    zg.armed = false;
    return out;
  }
  lc.alloc(range + 1, c.s);
  // bucket offsets of the build side: already grouped by key when it comes
  // sorted (an order-aware scan), else a counting sort
  DBuf<uint32_t> off(range + 1, c.s);
  if (Q.sorted_col == qk && range <= 4 * Q.nrows) {
    ProfScope ps(c, "join_build", 4.0 * Q.nrows + 4.0 * range);
    hipLaunchKernelGGL(k_bucket_bounds, G(range + 1), dim3(B), 0, c.s, qkey, Q.nrows, kmin, (uint32_t)range, off.p);
    DAS_HIP(hipGetLastError());
  } else if (Q.sorted_col == qk) {
    // sparse keys over a wide range: a histogram + scan beats a binary
    // search per slot, and sorted rows need no scatter
    DBuf<uint32_t> cnt(range + 1, c.s);
    ProfScope ps(c, "join_build", 4.0 * Q.nrows + 8.0 * range);
    fill_dev(cnt.p, 0, 4 * (range + 1), c.s);
    hipLaunchKernelGGL(k_key_hist, G(Q.nrows), dim3(B), 0, c.s, qkey, Q.nrows, kmin, (uint32_t)range, cnt.p);
    exclusive_scan<uint32_t>(cnt.p, range + 1, off.p, c.s);
    DAS_HIP(hipGetLastError());
  } else {
    DBuf<uint32_t> cnt(range + 1, c.s);
    ProfScope ps(c, "join_build", 4.0 * Q.nrows * (Q.ncols + 1) + 8.0 * range);
    fill_dev(cnt.p, 0, 4 * (range + 1), c.s);
    hipLaunchKernelGGL(k_key_hist, G(Q.nrows), dim3(B), 0, c.s, qkey, Q.nrows, kmin, (uint32_t)range, cnt.p);
    exclusive_scan<uint32_t>(cnt.p, range + 1, off.p, c.s);
    copy_dev(cnt.p, off.p, 4 * (range + 1), c.s);
    Qs = new_table_like(c, Q, Q.nrows);
    Qs->nrows = Q.nrows;
    hipLaunchKernelGGL(k_key_scatter, G(Q.nrows), dim3(B), 0, c.s, cols_of(Q), qkey, Q.nrows, kmin, (uint32_t)range,
                       cnt.p, Qs->data, Qs->cap);
    DAS_HIP(hipGetLastError());
    Qb = Qs.get();
  }
  hipLaunchKernelGGL(k_pack_lc, dim3(grid_for(range, B, 2048)), dim3(B), 0, c.s, (const uint32_t*)off.p,
                     (uint32_t)range, lc.p);
  DAS_HIP(hipGetLastError());
  return expand(*Qb, lc.p);
}

// ---------------------------------------------------------------------------
// Index (nested-loop) join: And's join of a bound table A with a Link whose
// join variable sits at an indexed position p.  Instead of scanning the
// Link's whole type segment and joining, every row of A looks its key up in
// P_{a,p} (one binary search over the unique (type, t_p) keys) and expands
// that contiguous row range: the same rows as join(A, scan_link(q)) -- each
// range holds exactly the links of that type with t_p = key -- at a cost
// proportional to A and the output, not to the Link's type segment.
// ---------------------------------------------------------------------------
struct IjGround {
  const uint32_t* col[kMaxArity];   // P_{a,p} columns of grounded targets, in the table's secondary order
  uint32_t val[kMaxArity];
  const uint32_t* src[kMaxArity];   // per-row value column instead of val (anti index join), or nullptr
  int n;
};

// (first row, count) in P_{a,p} of the links with t_p = t (and the grounded
// prefix g): the key through the dense directory (one load) or a binary
// search, then an equal-range search per grounded prefix target.  Ranged
// mode (fixed): the rows of one grounded key (type, t_q = v) of P_{a,q},
// known on the host, narrowed by the targets in P_{a,q}'s secondary order --
// the probe's own value among them (g.src) -- a search over one small,
// cache-resident range instead of random key ranges of the whole table.
struct IjKeys {
  uint64_t thi;
  const uint64_t* ukey;
  const uint64_t* uoff;
  uint64_t nkeys;
  const uint32_t* dir;
  uint32_t dlo, dn;
  uint32_t flo, fhi;    // ranged mode: rows [flo, fhi)
  int fixed;
  const uint32_t* bdir; // bucket directory (no dense one): keys of bucket (t - dlo) >> bshift
  uint32_t bshift, bn;
  const uint64_t* rbits; // rank directory (in place of a dense one over dn ids): bits, word prefixes
  const uint32_t* rpre;
  uint64_t rklo;
};

// Index in ukey of key (type, t) through the dense directory (one load), the
// bucket directory (two adjacent loads + a search of ~2 keys) or a binary
// search over every key; false if absent.
__device__ __forceinline__ bool ij_key_index(uint32_t t, const IjKeys& kx, uint64_t& lo) {
  if (kx.rbits) {
    const uint32_t d = t - kx.dlo;
    if (d >= kx.dn) return false;
    const uint64_t w = kx.rbits[d >> 6];          // the word and its prefix: two independent loads
    const uint32_t p = kx.rpre[d >> 6];
    const uint64_t below = w & ((1ull << (d & 63)) - 1ull);
    lo = kx.rklo + p + (uint64_t)__popcll(below);
    return (w >> (d & 63)) & 1ull;
  }
  if (kx.dir) {
    const uint32_t d = t - kx.dlo;
    const uint32_t j = d < kx.dn ? kx.dir[d] : 0xFFFFFFFFu;
    lo = j;
    return j != 0xFFFFFFFFu;
  }
  const uint64_t k = kx.thi | t;
  uint64_t l = 0, h = kx.nkeys;
  if (kx.bdir) {
    const uint32_t b = (t - kx.dlo) >> kx.bshift;
    if (t < kx.dlo || b >= kx.bn) return false;
    l = kx.bdir[b];
    h = kx.bdir[b + 1];
  }
  while (l < h) {
    const uint64_t mid = (l + h) >> 1;
    if (kx.ukey[mid] < k) l = mid + 1; else h = mid;
  }
  lo = l;
  return lo < kx.nkeys && kx.ukey[lo] == k;
}

// [b, end) narrowed to the rows of col (sorted over the range) equal to v:
// the two bounds searched in lockstep (two independent load chains per
// step).  (An interpolation guess with the 32 values around it loaded in one
// round was slower on FlyBase FJ's 3*10^5 ranged probes, 91-96 vs 72-78 us
// per query: the binary steps over a 1.8 MB range hit L2, the windows' 128 B
// per probe did not.)
__device__ __forceinline__ void narrow_eq(const uint32_t* __restrict__ col, uint32_t& b, uint32_t& end, uint32_t v) {
  uint32_t l = b, h = end, l2 = b, h2 = end;
  while (l < h || l2 < h2) {
    if (l < h) { const uint32_t m = (l + h) >> 1; if (col[m] < v) l = m + 1; else h = m; }
    if (l2 < h2) { const uint32_t m = (l2 + h2) >> 1; if (col[m] <= v) l2 = m + 1; else h2 = m; }
  }
  b = l;
  end = l2;
}

__device__ __forceinline__ uint2 ij_lookup(uint32_t t, const IjKeys& kx, const IjGround& g, uint64_t row = 0) {
  uint64_t lo;
  bool hit;
  if (kx.fixed) {
    lo = 0;
    hit = kx.fhi > kx.flo;
  } else {
    hit = ij_key_index(t, kx, lo);
  }
  uint2 e = make_uint2(0u, 0u);
  if (hit) {
    uint32_t b = kx.fixed ? kx.flo : (uint32_t)kx.uoff[lo], end = kx.fixed ? kx.fhi : (uint32_t)kx.uoff[lo + 1];
    // targets that lead the range's secondary order: the rows equal to each
    // value form a sub-range; its two bounds are searched in lockstep (two
    // independent load chains per step)
    for (int j = 0; j < g.n && b < end; ++j)
      narrow_eq(g.col[j], b, end, g.src[j] ? g.src[j][row] : g.val[j]);
    if (end > b) e = make_uint2(b, end - b);
  }
  return e;
}

__global__ void __launch_bounds__(B) k_ij_lc(const uint32_t* __restrict__ key, uint64_t n, IjKeys kx, IjGround g,
                                             uint2* __restrict__ lc, uint32_t* __restrict__ rowid) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    lc[i] = ij_lookup(key[i], kx, g, i);
    rowid[i] = (uint32_t)i;
  }
}

__device__ __forceinline__ uint32_t mix32(uint32_t h) {   // murmur3 finaliser
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}

// Few probe rows are latency-bound (a key directory load, its offsets, then
// an equal-range search per grounded target: ~16 dependent loads per probe,
// one thread at a time).  With few probes a group of G lanes serves each
// probe and searches G+1-ary: one round of G loads and a ballot narrows a
// range G+1-fold, so a ~100-row range takes one round.
// First index in [lo, hi) whose value is >= v (strict = false) or > v
// (strict = true), hi if none, by the G lanes of a group (all with the same
// arguments): a G+1-ary search, one round of G loads per step.
template <int G>
__device__ __forceinline__ void group_bounds(const uint32_t* __restrict__ col, uint32_t& lo, uint32_t& hi,
                                             uint32_t v) {
  const uint32_t gl = __lane_id() & (G - 1);
  const uint64_t gmask = (G >= 64 ? ~0ull : ((1ull << (G & 63)) - 1)) << (__lane_id() & ~(uint32_t)(G - 1) & 63);
  const int gbase = (int)(__lane_id() & ~(uint32_t)(G - 1));
  // lower bound (>= v) over [a0, a1), upper bound (> v) over [b0, b1): lockstep
  uint32_t a0 = lo, a1 = hi, b0 = lo, b1 = hi;
  bool da = false, db = false;
  while (!(da && db)) {
    const uint32_t la = a1 - a0, lb = b1 - b0;
    // sample positions: the range itself when it fits the group, else G
    // evenly spaced interior points
    const uint32_t pa = la <= G ? a0 + gl : a0 + (uint32_t)(((uint64_t)(gl + 1) * la) / (G + 1));
    const uint32_t pb = lb <= G ? b0 + gl : b0 + (uint32_t)(((uint64_t)(gl + 1) * lb) / (G + 1));
    const bool ina = !da && (la > G || gl < la), inb = !db && (lb > G || gl < lb);
    const uint32_t xa = ina ? col[pa] : 0u, xb = inb ? col[pb] : 0u;
    const uint32_t ca = (uint32_t)__popcll((__ballot(ina && xa < v) & gmask) >> gbase);
    const uint32_t cb = (uint32_t)__popcll((__ballot(inb && xb <= v) & gmask) >> gbase);
    if (!da) {
      if (la <= G) {
        a0 += ca;
        da = true;
      } else {
        const uint32_t n0 = ca == 0 ? a0 : a0 + (uint32_t)(((uint64_t)ca * la) / (G + 1)) + 1;
        const uint32_t n1 = ca == G ? a1 : a0 + (uint32_t)(((uint64_t)(ca + 1) * la) / (G + 1));
        a0 = n0;
        a1 = n1;
        if (a0 >= a1) da = true;
      }
    }
    if (!db) {
      if (lb <= G) {
        b0 += cb;
        db = true;
      } else {
        const uint32_t n0 = cb == 0 ? b0 : b0 + (uint32_t)(((uint64_t)cb * lb) / (G + 1)) + 1;
        const uint32_t n1 = cb == G ? b1 : b0 + (uint32_t)(((uint64_t)(cb + 1) * lb) / (G + 1));
        b0 = n0;
        b1 = n1;
        if (b0 >= b1) db = true;
      }
    }
  }
  lo = a0;
  hi = b0;
}

// ij_lookup by the G lanes of a group (same arguments, same result).
template <int G>
__device__ __forceinline__ uint2 ij_lookup_group(uint32_t t, const IjKeys& kx, const IjGround& g, uint64_t row) {
  uint32_t b = 0, end = 0;
  if (kx.fixed) {
    b = kx.flo;
    end = kx.fhi;
  } else {
    uint64_t lo;
    bool hit;
    hit = ij_key_index(t, kx, lo);
    if (hit) {
      b = (uint32_t)kx.uoff[lo];
      end = (uint32_t)kx.uoff[lo + 1];
    }
  }
  for (int j = 0; j < g.n && b < end; ++j) {
    const uint32_t v = g.src[j] ? g.src[j][row] : g.val[j];
    group_bounds<G>(g.col[j], b, end, v);
  }
  return end > b ? make_uint2(b, end - b) : make_uint2(0u, 0u);
}

// Lookups of rows [0, nin) into s_lo / s_pre (x, y of ij_lookup), by groups
// of G lanes (G = 1: one row per thread).
template <int G>
__device__ __forceinline__ void lookups_into(const uint32_t* key, const IjKeys& kx, const IjGround& g, uint32_t nin,
                                             uint32_t* s_lo, uint32_t* s_pre, uint32_t base) {
  if (G == 1) {
    for (uint32_t r = threadIdx.x; r < nin; r += kSmallBlock) {
      const uint2 e = ij_lookup(key[base + r], kx, g, base + r);
      s_lo[r] = e.x;
      s_pre[r] = e.y;
    }
  } else {
    const uint32_t groups = kSmallBlock / G, gid = threadIdx.x / G;
    for (uint32_t r0 = 0; r0 < nin; r0 += groups) {      // uniform trip count: every lane of a group searches
      const uint32_t r = r0 + gid;
      const uint32_t rr = r < nin ? r : nin - 1;
      const uint2 e = ij_lookup_group<G>(key[base + rr], kx, g, base + rr);
      if (r < nin && (threadIdx.x & (G - 1)) == 0) {
        s_lo[r] = e.x;
        s_pre[r] = e.y;
      }
    }
  }
}

// rows [base, base + nin) of the probe; results at s_lo / s_pre [0, nin)
__device__ __forceinline__ void lookups_small(const uint32_t* key, const IjKeys& kx, const IjGround& g, uint32_t nin,
                                              uint32_t* s_lo, uint32_t* s_pre, uint32_t base = 0) {
  if (nin <= kSmallBlock / 64) lookups_into<64>(key, kx, g, nin, s_lo, s_pre, base);
  else if (nin <= kSmallBlock / 16) lookups_into<16>(key, kx, g, nin, s_lo, s_pre, base);
  else if (nin <= kSmallBlock / 4) lookups_into<4>(key, kx, g, nin, s_lo, s_pre, base);
  else lookups_into<1>(key, kx, g, nin, s_lo, s_pre, base);
}

// Single-workgroup index join of a small probe table: lookups, a block scan
// of the match counts, and -- when the total fits the output table the host
// allocated speculatively (`cap` rows) -- the expansion, each thread taking
// outputs o, o + 1024, ... and finding its probe row by a binary search over
// the LDS prefix; the total is published to the pinned slot either way (the
// host redoes a larger join through the multi-launch path).
constexpr uint32_t kIjSmall = 2048;
constexpr uint64_t kIjSmallCap = 32768;

__global__ void __launch_bounds__(kSmallBlock) k_ij_small(const uint32_t* __restrict__ key, uint32_t n, IjKeys kx,
                                                          IjGround g, JoinCols jc, uint32_t* __restrict__ out,
                                                          uint64_t cap, uint32_t* slot, uint32_t seq) {
  constexpr int W = kSmallBlock / 64;
  __shared__ uint32_t s_pre[kIjSmall + 1];
  __shared__ uint32_t s_lo[kIjSmall];
  __shared__ uint32_t s_w[W];
  lookups_small(key, kx, g, n, s_lo, s_pre);
  __syncthreads();
  // exclusive scan of s_pre[0..n): rows in rounds of 1024
  const int wave = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (uint32_t r0 = 0; r0 < n; r0 += kSmallBlock) {
    const uint32_t r = r0 + threadIdx.x;
    const uint32_t v = r < n ? s_pre[r] : 0u;
    const uint32_t inc = wave_incl_sum_u32(v);
    if (__lane_id() == 63) s_w[wave] = inc;
    __syncthreads();
    uint32_t pre = carry + inc - v, all = 0;
    for (int w = 0; w < W; ++w) {
      if (w < wave) pre += s_w[w];
      all += s_w[w];
    }
    __syncthreads();
    if (r < n) s_pre[r] = pre;
    carry += all;
    __syncthreads();
  }
  if (threadIdx.x == 0) s_pre[n] = carry;
  __syncthreads();
  const uint32_t total = carry;
  if ((uint64_t)total <= cap) {
    for (uint32_t o = threadIdx.x; o < total; o += kSmallBlock) {
      uint32_t l = 0, h = n;                       // last row r with s_pre[r] <= o
      while (h - l > 1) {
        const uint32_t m = (l + h) >> 1;
        if (s_pre[m] <= o) l = m; else h = m;
      }
      const uint32_t br = s_lo[l] + (o - s_pre[l]);
      for (int i = 0; i < jc.np; ++i) out[(uint64_t)jc.po[i] * cap + o] = jc.p[i][l];
      for (int i = 0; i < jc.nb; ++i) out[(uint64_t)jc.bo[i] * cap + o] = jc.b[i][br];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) publish_u32(slot, seq, total);
}

// Multi-workgroup index join of a mid-size probe (kIjSmall < rows <= kIjMid)
// in ONE launch and one read-back: a wave looks up its 64 probe rows, scans
// their match counts, reserves its outputs with one atomic and expands them
// (owner lane by a search over the lanes' prefixes), so waves land in
// completion order -- the output is unsorted.  The last block to finish
// publishes the total; outputs past the speculative capacity are not
// written (the host then takes the multi-launch path), nor are a wave's
// outputs past kIjMidWave (a hub key's expansion by one wave would
// serialise: ctr[2] is set and the total published as ~0, the host then
// takes the output-balanced path).
constexpr uint32_t kIjMid = 32768;
constexpr uint32_t kIjMidWave = 4096;

__global__ void __launch_bounds__(B) k_ij_mid(const uint32_t* __restrict__ key, uint32_t n, IjKeys kx, IjGround g,
                                              JoinCols jc, uint32_t* __restrict__ out, uint64_t cap,
                                              uint32_t* __restrict__ ctr, uint32_t* slot, uint32_t seq) {
  const int lane = __lane_id();
  const uint32_t r = blockIdx.x * B + threadIdx.x;
  const uint2 e = r < n ? ij_lookup(key[r], kx, g, r) : make_uint2(0u, 0u);
  const uint32_t inc = wave_incl_sum_u32(e.y);
  const uint32_t tot = (uint32_t)__shfl(inc, 63, 64);
  const uint32_t pre = inc - e.y;
  if (tot > kIjMidWave) {
    if (lane == 0) atomicOr(&ctr[2], 1u);
  }
  // one reservation per block (same-address atomics serialise): the block's
  // waves take consecutive slices in wave order
  __shared__ uint32_t s_tot[B / 64], s_base;
  const int wv = threadIdx.x >> 6;
  if (lane == 0) s_tot[wv] = tot <= kIjMidWave ? tot : 0u;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t all = 0;
    for (int w = 0; w < B / 64; ++w) all += s_tot[w];
    s_base = all ? atomicAdd(&ctr[0], all) : 0u;
  }
  __syncthreads();
  uint32_t base = s_base;
  for (int w = 0; w < wv; ++w) base += s_tot[w];
  if (tot && tot <= kIjMidWave && (uint64_t)base + tot <= cap) {
    uint32_t pv[kMaxCols];
#pragma unroll
    for (int i = 0; i < kMaxCols; ++i) pv[i] = i < jc.np && r < n ? jc.p[i][r] : 0u;
    for (uint32_t o0 = 0; o0 < tot; o0 += 64) {
      const uint32_t o = o0 + lane;
      int ll = 0;                                    // owner: max lane with pre <= o
#pragma unroll
      for (int step = 32; step >= 1; step >>= 1) {
        const uint32_t pl = (uint32_t)__shfl(pre, ll + step, 64);
        if (ll + step < 64 && pl <= o) ll += step;
      }
      const uint32_t br = lane_get(e.x, ll) + (o - (uint32_t)__shfl(pre, ll, 64));
#pragma unroll
      for (int i = 0; i < kMaxCols; ++i) {
        if (i >= jc.np) break;
        const uint32_t v = lane_get(pv[i], ll);
        if (o < tot) out[(uint64_t)jc.po[i] * cap + base + o] = v;
      }
      if (o < tot)
        for (int i = 0; i < jc.nb; ++i) out[(uint64_t)jc.bo[i] * cap + base + o] = jc.b[i][br];
    }
  }
  __syncthreads();
  // arrival without an agent-scope release (on gfx950 each one writes this
  // XCD's L2 back; one per block serialised ~2.5 us a block per XCD): the
  // rows are read by later launches only, the last block reads counters,
  // atomics performed at the coherence point once this thread's are done
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (atomicAdd(&ctr[1], 1u) == gridDim.x - 1)
      publish_u32(slot, seq, atomicAdd(&ctr[2], 0u) ? 0xFFFFFFFFu : atomicAdd(&ctr[0], 0u));
  }
}

// Anti index join: keep row r of A when the link whose targets are the
// grounded targets and A's values of the term's variables does NOT exist --
// And's negation filter (pattern_matcher.py:741-746) for a Not(Link) term
// whose variables A binds, without scanning the term.  One key lookup plus
// one binary search per other position (P_{a,p}'s secondary order).
__global__ void __launch_bounds__(B) k_anti_ij(const uint32_t* __restrict__ key, uint64_t n, IjKeys kx, IjGround g,
                                               uint32_t* __restrict__ keep) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    keep[i] = ij_lookup(key[i], kx, g, i).y == 0 ? 1u : 0u;
}

namespace {
int colof_t(const Table& t, int32_t v) {
  for (int i = 0; i < t.ncols; ++i) if (t.vars[i] == v) return i;
  return -1;
}

IjKeys ij_keys(const PosIndex& PI, uint32_t type_id) {
  static const bool no_dir = std::getenv("DAS_NO_KEY_DIR") != nullptr;
  const bool use_rank = type_id < PI.rbits.size() && PI.rbits[type_id] && !no_dir;
  const bool use_dir = !use_rank && type_id < PI.dir.size() && PI.dir[type_id] && !no_dir;
  const bool use_bdir = !use_rank && !use_dir && type_id < PI.bdir.size() && PI.bdir[type_id] && !no_dir;
  return IjKeys{(uint64_t)type_id << 32, (const uint64_t*)PI.ukey, (const uint64_t*)PI.uoff, PI.nkeys,
                use_dir ? PI.dir[type_id] : nullptr, use_dir || use_bdir || use_rank ? PI.dir_lo[type_id] : 0u,
                use_dir || use_rank ? PI.dir_n[type_id] : 0u, 0u, 0u, 0,
                use_bdir ? PI.bdir[type_id] : nullptr, use_bdir ? PI.bshift[type_id] : 0u,
                use_bdir ? PI.bn[type_id] : 0u,
                use_rank ? (const uint64_t*)PI.rbits[type_id] : nullptr,
                use_rank ? (const uint32_t*)PI.rpre[type_id] : nullptr, use_rank ? PI.rklo[type_id] : 0ull};
}

// Anti index join of A by a Not(Link) term, resolved on the host.
struct AntiPlan {
  IjKeys kx{};
  IjGround g{};
  const uint32_t* key = nullptr;
  bool keep_all = false;       // no link of that arity is indexed: nothing is forbidden
};

// false: the term does not reduce to a lookup per row of A (a variable of
// the term that A does not bind: the caller keeps A whole)
bool anti_prepare(Ctx& c, const Table& A, const das_link_scan_t& q, AntiPlan& pl) {
  Index& idx = c.idx;
  DAS_CHECK(idx.built, DAS_E_NOT_BUILT, "index not built");
  const uint32_t ar = q.arity;
  if (A.kind != DAS_TABLE_ORDERED || !q.ordered || q.emit_link || q.type_id == kNone || q.type_id >= idx.n_types ||
      idx.blocked(q.type_id) || ar == 0 || ar > (uint32_t)kMaxPosArity || A.nrows >= 0xFFFFFFFFull)
    return false;
  // every position grounded or bound by A (else the filter is not a lookup)
  int bp = -1;
  for (uint32_t p = 0; p < ar; ++p) {
    if (q.target[p] != kNone) continue;
    if (q.var[p] < 0 || colof_t(A, q.var[p]) < 0) return false;
    if (bp < 0) bp = (int)p;
  }
  if (bp < 0) return false;
  const PosIndex& PI = idx.pidx[ar][bp];
  if (PI.nkeys == 0) {
    pl.keep_all = true;
    return true;
  }
  for (uint32_t p = 0; p < ar; ++p) {
    if ((int)p == bp) continue;
    pl.g.col[pl.g.n] = PI.t.col(1 + (int)p);
    if (q.target[p] != kNone) {
      pl.g.val[pl.g.n] = q.target[p];
      pl.g.src[pl.g.n] = nullptr;
    } else {
      pl.g.src[pl.g.n] = A.col(colof_t(A, q.var[p]));
    }
    ++pl.g.n;
  }
  pl.kx = ij_keys(PI, q.type_id);
  pl.key = A.col(colof_t(A, q.var[bp]));
  return true;
}

// Index join of A with a Link term, resolved on the host.  `rows` = A's row
// count, or an upper bound of it (the fused chain), for the cost choices.
struct IjPlan {
  IjKeys kx{};
  IjGround g{};
  JoinCols jc{};
  const uint32_t* akey = nullptr;
  std::vector<int32_t> uni;
  uint32_t lo[kMaxCols] = {0}, hi[kMaxCols] = {0};
  bool empty = false;          // no output row possible
};

// false: not an index join of A (the caller scans the term and joins)
bool ij_prepare(Ctx& c, const Table& A, const das_link_scan_t& q, uint64_t rows, IjPlan& pl, bool dir_only = false) {
  Index& idx = c.idx;
  DAS_CHECK(idx.built, DAS_E_NOT_BUILT, "index not built");
  const uint32_t ar = q.arity;
  if (A.kind != DAS_TABLE_ORDERED || !q.ordered || q.emit_link || q.type_id == kNone || q.type_id >= idx.n_types ||
      idx.blocked(q.type_id) || ar == 0 || ar > (uint32_t)kMaxPosArity || rows >= 0xFFFFFFFFull)
    return false;
  // one bound position; every other position a fresh, distinct variable or
  // a grounded target that leads P_{a,p}'s secondary order
  int bp = -1;
  std::vector<std::pair<int32_t, uint32_t>> fresh;   // (var, position)
  for (uint32_t p = 0; p < ar; ++p) {
    if (q.target[p] != kNone) {
      if (q.var[p] >= 0) return false;
      continue;
    }
    if (q.var[p] < 0) return false;
    if (colof_t(A, q.var[p]) >= 0) {
      if (bp >= 0) return false;
      bp = (int)p;
    } else {
      for (auto& f : fresh) if (f.first == q.var[p]) return false;
      fresh.push_back({q.var[p], p});
    }
  }
  if (bp < 0) return false;
  const PosIndex& PI = idx.pidx[ar][bp];
  IjGround& g = pl.g;
  {
    bool prefix = true;                          // still inside the grounded prefix
    for (uint32_t p = 0; p < ar; ++p) {
      if ((int)p == bp) continue;
      if (q.target[p] != kNone) {
        if (!prefix) return false;               // a grounded target after a free one: rows not contiguous
        g.col[g.n] = PI.t.col(1 + (int)p);
        g.val[g.n++] = q.target[p];
      } else {
        prefix = false;
      }
    }
  }
  // cost: a search per row of A against a scan of the Link's type segment
  {
    const char* f = std::getenv("DAS_INDEX_JOIN");          // tests: 1 always, 0 never
    if (f && f[0] == '0') return false;
    const uint64_t seg = idx.type_off[ar].size() > q.type_id + 1
                             ? idx.type_off[ar][q.type_id + 1] - idx.type_off[ar][q.type_id] : 0;
    // (with grounded targets the scan reads one key range, of unknown size
    // here: index-join only small probes)
    const bool cheap = g.n == 0 ? 4 * rows <= seg : rows <= (1ull << 20);
    if (!(f && f[0] == '1') && !cheap) return false;
  }
  DAS_CHECK(PI.t.rows < 0xFFFFFFFFull, DAS_E_UNSUPPORTED, "index join: P table too large");
  // output schema: A's variables and the fresh ones, ascending
  std::vector<int32_t>& uni = pl.uni;
  uni.assign(A.vars, A.vars + A.ncols);
  for (auto& f : fresh) uni.push_back(f.first);
  std::sort(uni.begin(), uni.end());
  DAS_CHECK((int)uni.size() <= kMaxCols, DAS_E_UNSUPPORTED, "too many variables");
  const int nu = (int)uni.size();
  // output column bounds: A's columns, and the type's bounds for fresh ones
  {
    const uint32_t ncol = ar + 1;
    const auto& tb = idx.tbound[ar];
    for (int k = 0; k < nu; ++k) {
      const int ia = colof_t(A, uni[k]);
      if (ia >= 0) {
        pl.lo[k] = A.lo[ia];
        pl.hi[k] = A.hi[ia];
        continue;
      }
      pl.lo[k] = 0;
      pl.hi[k] = kNone;
      for (auto& f : fresh)
        if (f.first == uni[k] && (uint64_t)(q.type_id + 1) * ncol * 2 <= tb.size()) {
          pl.lo[k] = tb[((uint64_t)q.type_id * ncol + 1 + f.second) * 2];
          pl.hi[k] = tb[((uint64_t)q.type_id * ncol + 1 + f.second) * 2 + 1];
        }
    }
  }
  if (rows == 0 || PI.nkeys == 0) {
    pl.empty = true;
    return true;
  }
  const uint32_t* akey = pl.akey = A.col(colof_t(A, q.var[bp]));
  IjKeys& kx = pl.kx;
  kx = ij_keys(PI, q.type_id);
  const RowTable* T = &PI.t;                     // the table the expansion reads
  {
    // ranged mode: the rows of a grounded key (type, t_q = v) of P_{a,q},
    // when they are few (found in the host key mirror) and ordered by the
    // probe's position once the grounded targets before it are fixed
    const char* f = std::getenv("DAS_IJ_RANGED");          // tests: 1 whenever possible, 0 never
    uint64_t best = ~0ull;
    IjGround gb{};
    uint32_t blo = 0, bhi = 0, bq = 0;
    for (uint32_t qq = 0; qq < ar && !(f && f[0] == '0'); ++qq) {
      if (q.target[qq] == kNone) continue;
      const PosIndex& PQ = idx.pidx[ar][qq];
      if (PQ.h_ukey.empty() || PQ.t.rows >= 0xFFFFFFFFull) continue;
      IjGround gq{};
      bool stop = false, ok = true, probe = false;
      for (uint32_t r = 0; r < ar && ok; ++r) {
        if (r == qq) continue;
        if (q.target[r] != kNone) {
          if (stop) ok = false;
          gq.col[gq.n] = PQ.t.col(1 + (int)r);
          gq.val[gq.n] = q.target[r];
          gq.src[gq.n++] = nullptr;
        } else if ((int)r == bp) {
          if (stop) ok = false;
          gq.col[gq.n] = PQ.t.col(1 + (int)r);
          gq.src[gq.n++] = akey;
          probe = true;
        } else {
          stop = true;
        }
      }
      if (!ok || !probe) continue;
      const uint64_t k = ((uint64_t)q.type_id << 32) | q.target[qq];
      const size_t i = std::lower_bound(PQ.h_ukey.begin(), PQ.h_ukey.end(), k) - PQ.h_ukey.begin();
      const bool has = i < PQ.h_ukey.size() && PQ.h_ukey[i] == k;
      const uint64_t lo = has ? PQ.h_uoff[i] : 0, hi = has ? PQ.h_uoff[i + 1] : 0;
      if (hi - lo < best) {
        best = hi - lo;
        gb = gq;
        blo = (uint32_t)lo;
        bhi = (uint32_t)hi;
        bq = qq;
      }
    }
    // many probes against one long grounded key range: a binary search of
    // log2(range) steps per probe costs more than reading the range once as
    // the build side of a direct join (FlyBase FJ: 3*10^5 probes into the
    // 4.5*10^5 rows of one schema, 73-76 vs 64-65 us per query) -- not an
    // index join then (DAS_INDEX_JOIN=1 / DAS_IJ_RANGED=1 keep it)
    // (dir_only: the fused chain's probes after a partitioned scan -- the
    // key-directory lookup instead of that search, no scan)
    const char* fij = std::getenv("DAS_INDEX_JOIN");
    const bool long_range = best != ~0ull && best > 0 && rows > 4096 && !(f && f[0] == '1') &&
                            (double)rows * std::log2((double)best) > 2.0 * (double)best;
    if (long_range && !dir_only && !(fij && fij[0] == '1')) return false;
    const bool take = best != ~0ull && !(dir_only && long_range) &&
                      ((f && f[0] == '1') || (best <= (1ull << 22) && best <= 64ull * rows));
    if (take) {
      g = gb;
      kx.fixed = 1;
      kx.flo = blo;
      kx.fhi = bhi;
      T = &idx.pidx[ar][bq].t;
    }
  }
  JoinCols& jc = pl.jc;
  for (int k = 0; k < nu; ++k) {
    const int ia = colof_t(A, uni[k]);
    if (ia >= 0) { jc.p[jc.np] = A.col(ia); jc.po[jc.np++] = k; continue; }
    for (auto& f : fresh)
      if (f.first == uni[k]) { jc.b[jc.nb] = T->col(1 + (int)f.second); jc.bo[jc.nb++] = k; }
  }
  return true;
}
}  // namespace

std::unique_ptr<Table> anti_index_join(Ctx& c, const Table& A, const das_link_scan_t& q) {
  AntiPlan pl;
  if (!anti_prepare(c, A, q, pl)) return nullptr;
  if (A.nrows == 0) return new_table_like(c, A, 0);
  if (pl.keep_all) {
    DBuf<uint32_t> all(A.nrows, c.s);
    iota(all.p, A.nrows, c.s);
    return gather_table(c, A, all.p, A.nrows);
  }
  DBuf<uint32_t> keep(A.nrows, c.s);
  {
    ProfScope ps(c, "k_anti_ij", 4.0 * A.nrows * (q.arity + 1));
    hipLaunchKernelGGL(k_anti_ij, G(A.nrows), dim3(B), 0, c.s, pl.key, A.nrows, pl.kx, pl.g, keep.p);
    DAS_HIP(hipGetLastError());
  }
  return compact_table(c, A, keep.p);
}

std::unique_ptr<Table> index_join(Ctx& c, const Table& A, const das_link_scan_t& q) {
  IjPlan pl;
  if (!ij_prepare(c, A, q, A.nrows, pl)) return nullptr;
  const int nu = (int)pl.uni.size();
  std::unique_ptr<Table> out;
  bool unsorted = false;                         // k_ij_mid: waves land in completion order
  if (pl.empty) {
    out = new_table(c, DAS_TABLE_ORDERED, nu, pl.uni.data(), 0);
  } else {
    if (A.nrows <= kIjSmall) {
      // one launch when the output fits a speculative table
      auto t = new_table(c, DAS_TABLE_ORDERED, nu, pl.uni.data(), kIjSmallCap);
      const PubSlot ps = pub_reserve();
      {
        ProfScope pf(c, "k_ij_small", 16.0 * A.nrows + 4.0 * A.nrows * A.ncols);
        hipLaunchKernelGGL(k_ij_small, dim3(1), dim3(kSmallBlock), 0, c.s, pl.akey, (uint32_t)A.nrows, pl.kx, pl.g,
                           pl.jc, t->data, t->cap, ps.p, ps.seq);
        DAS_HIP(hipGetLastError());
      }
      uint32_t total = 0;
      pub_wait(ps, c.s, &total, 1);
      if (total <= t->cap) {
        t->nrows = total;
        out = std::move(t);
      }
    }
    if (!out && A.nrows > kIjSmall && A.nrows <= kIjMid) {
      const char* f = std::getenv("DAS_IJ_MID");                // A/B, tests: 0 never
      if (!(f && f[0] == '0')) {
        // one launch when the output fits a speculative table of 4 rows per probe row
        auto t = new_table(c, DAS_TABLE_ORDERED, nu, pl.uni.data(), std::max<uint64_t>(65536, 4 * A.nrows));
        DBuf<uint32_t> ctr(3, c.s);
        fill_dev(ctr.p, 0, 12, c.s);
        const PubSlot ps = pub_reserve();
        {
          ProfScope pf(c, "k_ij_mid", 16.0 * A.nrows + 4.0 * A.nrows * A.ncols);
          hipLaunchKernelGGL(k_ij_mid, dim3((unsigned)((A.nrows + B - 1) / B)), dim3(B), 0, c.s, pl.akey,
                             (uint32_t)A.nrows, pl.kx, pl.g, pl.jc, t->data, t->cap, ctr.p, ps.p, ps.seq);
          DAS_HIP(hipGetLastError());
        }
        uint32_t total = 0;
        pub_wait(ps, c.s, &total, 1);
        if (total != 0xFFFFFFFFu && total <= t->cap) {
          t->nrows = total;
          out = std::move(t);
          unsorted = true;
        }
      }
    }
    if (!out) {
      DBuf<uint2> lc(A.nrows, c.s);
      DBuf<uint32_t> rowid(A.nrows, c.s);
      {
        ProfScope ps(c, "k_ij_lc", 4.0 * A.nrows + 8.0 * A.nrows + 4.0 * A.nrows);
        hipLaunchKernelGGL(k_ij_lc, G(A.nrows), dim3(B), 0, c.s, pl.akey, A.nrows, pl.kx, pl.g, lc.p, rowid.p);
        DAS_HIP(hipGetLastError());
      }
      // build bytes: the P_{a,p} rows each output reads (4 B per fresh column;
      // every output is its own P row, so the expansion sizes them)
      out = dj_expand(c, A, rowid.p, 0u, A.nrows, lc.p, pl.jc, nu, pl.uni.data(), -4.0 * pl.jc.nb);
    }
  }
  out->sorted_col = A.sorted_col >= 0 && !unsorted ? colof_t(*out, A.vars[A.sorted_col]) : -1;
  for (int k = 0; k < nu; ++k) {
    out->lo[k] = pl.lo[k];
    out->hi[k] = pl.hi[k];
  }
  return out;
}

// ---------------------------------------------------------------------------
// Fused small And (das_plan_execute).  An anchored And of ordered Links --
// the FlyBase shapes: a grounded scan, index joins, a small cross join, anti
// index joins for its Not terms -- keeps its running result at a few rows,
// so each operator is one small launch and one read-back round trip.  Here
// the whole chain runs in ONE workgroup of ONE launch, with one read-back:
// the stages (compiled on the host from the same prepare steps as the
// per-operator path: scan_prepare, ij_prepare, anti_prepare) are read from
// pinned memory into LDS, each stage's row count stays in LDS, every
// intermediate table is allocated up front at a speculative capacity.
//
// A stage that cannot run here -- its input is too large for the LDS
// prefix, its output outgrows its table, or an index join comes out empty
// (And's reset-on-empty path, pattern_matcher.py:720-733) -- ends the chain
// at the last complete running result ("partial"): the caller continues the
// And from the next term operator by operator.  A scan term with no rows
// makes the And fail (:712-713), as on the host path.
//
// Lookups of few probe rows go through groups of lanes (lookups_small).
// ---------------------------------------------------------------------------
namespace {
constexpr int kChainStages = 8;
constexpr uint32_t kChainCap = 32768;                 // rows per speculative table
constexpr uint32_t kChainIjRows = kIjSmall;           // probe rows an index-join stage takes in the chain
constexpr uint64_t kChainJoinPairs = 1ull << 22;      // cross-join work bound (pairs)

enum : uint32_t { CH_SCAN = 1, CH_IJ = 2, CH_JOIN = 3, CH_ANTI = 4, CH_DEDUP = 5 };
constexpr uint32_t kChainHash = 2 * kIjSmall;         // LDS hash slots of the dedup stage (power of two)
constexpr uint32_t kChainNoStage = 0xFFFFFFFFu;
enum : uint32_t { CHS_OK = 0, CHS_EMPTY_SCAN = 1, CHS_PARTIAL = 2 };

struct ChainStage {
  uint32_t op, in, rel, cap;     // input stage (running result), scanned stage (JOIN), output capacity
  uint32_t done;                 // the running result is complete after this stage
  uint32_t append;               // SCAN: append to this stage's table (Or's union), or kChainNoStage
  uint32_t empty_ok;             // SCAN: no rows is not a failing term (Or)
  uint32_t begin, end;           // SCAN: row range of the index table
  uint32_t ld;                   // column stride of dst (0: cap); grid chain: cap is per workgroup
  uint32_t ncols;                // columns of dst
  uint32_t part;                 // grid chain: the partition index join (each workgroup expands a slice)
  uint32_t* dst;                 // output table (ncols columns of `cap` rows)
  const uint32_t* key;           // IJ / ANTI: the probe key column
  ScanSpec sp;                   // SCAN
  IjKeys kx;                     // IJ / ANTI
  IjGround g;
  JoinCols jc;                   // IJ: output columns; JOIN: p = columns of `in`, b = of `rel`
  uint32_t nsh;                  // JOIN: shared-variable column pairs
  const uint32_t* sha[kMaxCols];
  const uint32_t* shb[kMaxCols];
  uint32_t ncopy;                // ANTI: the input's columns, copied
  const uint32_t* copy[kMaxCols];
};
struct ChainDesc {
  uint32_t nstage;
  uint32_t seg;                  // grid chain: rows per workgroup segment of every stage table (0: one workgroup)
  uint32_t* fin;                 // grid chain: the final table (columns of fin_ld rows)
  uint64_t fin_ld;
  uint32_t* gsc;                 // grid chain: device counters (kGscWords, zeroed by k_chain_prep)
  ChainStage st[kChainStages];
};
// grid chain counters: per-stage global row counts, then the output cursor,
// the finished-workgroup count and the redo flag
constexpr uint32_t kGscOut = kChainStages, kGscDone = kChainStages + 1, kGscRedo = kChainStages + 2,
                   kGscWords = kChainStages + 4;
static_assert(kGscWords <= Ctx::kGscBlock, "pooled grid-chain counter block too small");
enum : uint32_t { CHS_REDO = 3 };

// Block-wide ordered compaction step: this thread's output position among
// the kept rows of the round (keep order = thread order); advances *run.
__device__ __forceinline__ uint32_t chain_rank(bool keep, uint32_t* s_w, uint32_t* run) {
  constexpr int W = kSmallBlock / 64;
  const int wave = threadIdx.x >> 6;
  const uint64_t m = __ballot(keep);
  if (__lane_id() == 0) s_w[wave] = __popcll(m);
  __syncthreads();
  uint32_t pos = *run + __popcll(m & __lanemask_lt());
  uint32_t all = 0;
  for (int w = 0; w < W; ++w) {
    if (w < wave) pos += s_w[w];
    all += s_w[w];
  }
  __syncthreads();
  if (threadIdx.x == 0) *run += all;
  __syncthreads();
  return pos;
}

// The stages, by one workgroup (GRID = false: the whole chain) or by each
// workgroup of a grid (GRID = true).  In the grid form every workgroup runs
// the stages before the partition index join itself (they are small: grounded
// scans and their joins), writing its own segment [w * seg, (w + 1) * seg) of
// every stage table; at the partition stage it expands only its slice of the
// outputs (output-balanced over the workgroups), and every later stage is
// row-local -- index joins, joins with a (replicated) scanned term, anti
// index joins -- on the rows the workgroup holds.  No workgroup waits for
// another: each appends its final rows to the output table at a cursor and
// the last one to finish publishes the total.  A failure before or at the
// partition is the same in every workgroup (the chain ends "partial" there,
// as the one-workgroup chain does); after it -- a segment outgrowing its
// capacity -- the whole chain is redone by the caller.
template <bool GRID>
__device__ __forceinline__ void chain_body(const uint32_t* __restrict__ hdesc, uint32_t nwords, uint32_t* slot,
                                           uint32_t seq, uint64_t* tstamp) {
  const bool stamp = tstamp && (!GRID || blockIdx.x == 0);
  const uint64_t t_start = wall_clock64();
  if (stamp && threadIdx.x == 0) tstamp[0] = t_start;
  constexpr int W = kSmallBlock / 64;
  __shared__ ChainDesc d;
  __shared__ uint32_t s_cnt[kChainStages];
  __shared__ uint32_t s_buf[kChainHash + 1];             // IJ prefix + ranges, or the dedup hash slots
  uint32_t* s_pre = s_buf;
  uint32_t* s_lo = s_buf + kIjSmall + 1;
  __shared__ uint32_t s_w[W];
  __shared__ uint32_t s_run, s_state, s_acc, s_parted, s_base;
  uint32_t* dw = reinterpret_cast<uint32_t*>(&d);
  for (uint32_t i = threadIdx.x; i < nwords; i += kSmallBlock) dw[i] = hdesc[i];
  if (threadIdx.x == 0) {
    s_state = CHS_OK;
    s_acc = 0;
    s_parted = 0;
  }
  __syncthreads();
  if (stamp && threadIdx.x == 0) tstamp[1] = wall_clock64();
  const uint32_t G = GRID ? gridDim.x : 1u, wg = GRID ? blockIdx.x : 0u;
  const uint64_t off = GRID ? (uint64_t)wg * d.seg : 0ull;   // this workgroup's rows of every stage table
  for (uint32_t si = 0; si < d.nstage && s_state == CHS_OK; ++si) {
    const ChainStage& st = d.st[si];
    const uint64_t ld = st.ld ? st.ld : st.cap;
    uint32_t* dst = st.dst + off;
    const bool parted = GRID && s_parted;          // rows are this workgroup's share (uniform)
    if (threadIdx.x == 0) s_run = 0;
    __syncthreads();
    uint32_t n = 0;
    bool ok = true;                // uniform: the stage produced its full result
    bool redo = false;             // grid, after the partition: a segment overflowed
    if (st.op == CH_SCAN) {
      const bool app = st.append != kChainNoStage;
      if (app && threadIdx.x == 0) s_run = s_cnt[st.append];
      __syncthreads();
      // grid, partitioned scan (the chain's first term, too large to
      // replicate): this workgroup's slice of the rows, then every later
      // stage is row-local
      const bool pscan = GRID && st.part;
      const uint64_t span = st.end - st.begin;
      const uint32_t sb = pscan ? st.begin + (uint32_t)(span * wg / G) : st.begin;
      const uint32_t se = pscan ? st.begin + (uint32_t)(span * (wg + 1) / G) : st.end;
      for (uint32_t r0 = sb; r0 < se; r0 += kSmallBlock) {
        const uint32_t r = r0 + threadIdx.x;
        const bool keep = r < se && scan_keep(st.sp, r);
        const uint32_t pos = chain_rank(keep, s_w, &s_run);
        if (keep)                                      // chain scans are ordered (no local sort buffer)
          for (uint32_t c = 0; c < st.sp.nout; ++c) dst[c * ld + pos] = st.sp.col[1 + st.sp.outpos[c]][r];
      }
      n = s_run;
      if (app) {
        if (threadIdx.x == 0) s_cnt[st.append] = n;
        n = 0;
      } else if (pscan) {
        // an empty slice is not a failing term: the last workgroup tells
        // from the stage's total (kGscOut publish below)
        if (threadIdx.x == 0) {
          if (n) atomicAdd(&d.gsc[si], n);            // (the last workgroup tests totals for zero only)
          s_parted = 1;
        }
      } else if (n == 0 && !st.empty_ok && threadIdx.x == 0) {
        s_state = CHS_EMPTY_SCAN;
      }
    } else if (st.op == CH_DEDUP) {
      // distinct rows of the input (Python set semantics of Or's union):
      // an LDS open-addressing set of row indices, full-row equality
      const uint32_t nin = s_cnt[st.in];
      if (nin > kChainHash / 2) {
        ok = false;
      } else {
        for (uint32_t i = threadIdx.x; i < kChainHash; i += kSmallBlock) s_buf[i] = 0u;
        __syncthreads();
        // this thread's rows r and r + kSmallBlock: first occurrences (two
        // flags in registers, no indexed local array)
        static_assert(kChainHash / 2 == 2 * kSmallBlock, "two rows per thread");
        bool first[2] = {false, false};
#pragma unroll
        for (uint32_t k = 0; k < 2; ++k) {
          const uint32_t r = threadIdx.x + k * kSmallBlock;
          if (r >= nin) continue;
          uint32_t h = 0x9e3779b9u;
          for (uint32_t c = 0; c < st.ncopy; ++c) h = mix32(h ^ (st.copy[c][off + r] + 0x7f4a7c15u * (c + 1)));
          for (uint32_t probe = h & (kChainHash - 1);; probe = (probe + 1) & (kChainHash - 1)) {
            const uint32_t cur = atomicCAS(&s_buf[probe], 0u, r + 1);
            if (cur == 0u) {
              first[k] = true;
              break;
            }
            bool same = true;
            for (uint32_t c = 0; c < st.ncopy && same; ++c) same = st.copy[c][off + cur - 1] == st.copy[c][off + r];
            if (same) break;
          }
        }
#pragma unroll
        for (uint32_t k = 0; k < 2; ++k) {
          const uint32_t r = k * kSmallBlock + threadIdx.x;
          if (k * kSmallBlock >= nin) break;
          const bool keep = r < nin && first[k];
          const uint32_t pos = chain_rank(keep, s_w, &s_run);
          if (keep)
            for (uint32_t c = 0; c < st.ncopy; ++c) dst[(uint64_t)c * ld + pos] = st.copy[c][off + r];
        }
        n = s_run;
      }
    } else if (st.op == CH_IJ) {
      // the probe in chunks of kIjSmall rows (the LDS prefix): lookups, a
      // block scan of the match counts, the chunk's outputs appended in
      // probe order.  Inputs above kChainIjRows end the one-workgroup chain
      // instead: one workgroup expanding them lost to the multi-workgroup
      // index join (FlyBase F5 / F7 at hub genes, profiles/r2_flybase_host_split.json);
      // the grid chain takes any input its segments hold
      const uint32_t nin = s_cnt[st.in];
      const int wave = threadIdx.x >> 6;
      const bool part = GRID && st.part;
      uint32_t outn = 0;
      if ((!parted && nin > kChainIjRows) || (part && nin > kIjSmall)) ok = false;
      for (uint32_t c0 = 0; c0 < nin && ok && !redo; c0 += kIjSmall) {
        const uint32_t cn = nin - c0 < kIjSmall ? nin - c0 : kIjSmall;
        lookups_small(st.key, st.kx, st.g, cn, s_lo, s_pre, (uint32_t)(off + c0));
        __syncthreads();
        // exclusive scan of s_pre[0..cn) in rounds of 1024
        uint32_t carry = 0;
        for (uint32_t r0 = 0; r0 < cn; r0 += kSmallBlock) {
          const uint32_t r = r0 + threadIdx.x;
          const uint32_t v = r < cn ? s_pre[r] : 0u;
          const uint32_t inc = wave_incl_sum_u32(v);
          if (__lane_id() == 63) s_w[wave] = inc;
          __syncthreads();
          uint32_t pre = carry + inc - v, all = 0;
          for (int w = 0; w < W; ++w) {
            if (w < wave) pre += s_w[w];
            all += s_w[w];
          }
          __syncthreads();
          if (r < cn) s_pre[r] = pre;
          carry += all;
          __syncthreads();
        }
        if (threadIdx.x == 0) s_pre[cn] = carry;
        __syncthreads();
        // the partition stage expands outputs [o_lo, o_hi) of the total only
        const uint32_t o_lo = part ? (uint32_t)(((uint64_t)carry * wg) / G) : 0u;
        const uint32_t o_hi = part ? (uint32_t)(((uint64_t)carry * (wg + 1)) / G) : carry;
        if (part && carry == 0) {
          ok = false;                                  // empty everywhere: the chain ends partial
        } else if ((uint64_t)outn + (o_hi - o_lo) > st.cap) {
          if (parted || part) redo = true; else ok = false;
        } else {
          for (uint32_t o = o_lo + threadIdx.x; o < o_hi; o += kSmallBlock) {
            uint32_t l = 0, h = cn;                    // last row r with s_pre[r] <= o
            while (h - l > 1) {
              const uint32_t m = (l + h) >> 1;
              if (s_pre[m] <= o) l = m; else h = m;
            }
            const uint32_t br = s_lo[l] + (o - s_pre[l]);
            const uint64_t w = outn + (o - o_lo);
            for (int i = 0; i < st.jc.np; ++i) dst[(uint64_t)st.jc.po[i] * ld + w] = st.jc.p[i][off + c0 + l];
            for (int i = 0; i < st.jc.nb; ++i) dst[(uint64_t)st.jc.bo[i] * ld + w] = st.jc.b[i][br];
          }
          outn += o_hi - o_lo;
        }
        __syncthreads();                               // s_lo / s_pre are reused by the next chunk
      }
      n = outn;
      if (n == 0 && !parted && !part) ok = false;      // one workgroup: And's reset-on-empty path
      if (part && ok && !redo && threadIdx.x == 0) s_parted = 1;
    } else if (st.op == CH_JOIN) {
      const uint32_t na = s_cnt[st.in], nb = s_cnt[st.rel];
      const uint64_t pairs = (uint64_t)na * nb;
      if (pairs > kChainJoinPairs) {
        if (parted) redo = true; else ok = false;
      } else {
        for (uint64_t k0 = 0; k0 < pairs; k0 += kSmallBlock) {
          const uint64_t k = k0 + threadIdx.x;
          const uint32_t i = k < pairs ? (uint32_t)(k / nb) : 0u, j = k < pairs ? (uint32_t)(k % nb) : 0u;
          bool keep = k < pairs;
          for (uint32_t x = 0; x < st.nsh && keep; ++x) keep = st.sha[x][off + i] == st.shb[x][off + j];
          const uint32_t pos = chain_rank(keep, s_w, &s_run);
          if (keep && pos < st.cap) {
            for (int c = 0; c < st.jc.np; ++c) dst[(uint64_t)st.jc.po[c] * ld + pos] = st.jc.p[c][off + i];
            for (int c = 0; c < st.jc.nb; ++c) dst[(uint64_t)st.jc.bo[c] * ld + pos] = st.jc.b[c][off + j];
          }
        }
        n = s_run;
        if (n > st.cap) {
          if (parted) redo = true; else ok = false;
        } else if (n == 0 && !parted) {
          ok = false;
        }
      }
    } else {   // CH_ANTI
      const uint32_t nin = s_cnt[st.in];
      if (nin <= kIjSmall) {
        lookups_small(st.key, st.kx, st.g, nin, s_lo, s_pre, (uint32_t)off);   // s_pre[r] = matches of row r's link (0 or 1)
        __syncthreads();
        for (uint32_t r0 = 0; r0 < nin; r0 += kSmallBlock) {
          const uint32_t r = r0 + threadIdx.x;
          const bool keep = r < nin && s_pre[r] == 0;
          const uint32_t pos = chain_rank(keep, s_w, &s_run);
          if (keep)
            for (uint32_t c = 0; c < st.ncopy; ++c) dst[(uint64_t)c * ld + pos] = st.copy[c][off + r];
        }
      } else {
        for (uint32_t r0 = 0; r0 < nin; r0 += kSmallBlock) {
          const uint32_t r = r0 + threadIdx.x;
          const bool keep = r < nin && ij_lookup(st.key[off + r], st.kx, st.g, off + r).y == 0;
          const uint32_t pos = chain_rank(keep, s_w, &s_run);
          if (keep)
            for (uint32_t c = 0; c < st.ncopy; ++c) dst[(uint64_t)c * ld + pos] = st.copy[c][off + r];
        }
      }
      n = s_run;
    }
    if (threadIdx.x == 0) {
      s_cnt[si] = n;
      if (redo) {
        s_state = CHS_REDO;
      } else if (!ok) {
        s_state = CHS_PARTIAL;
      } else if (st.done) {
        s_acc = si;
      }
      if (GRID && parted && ok && !redo && n) atomicAdd(&d.gsc[si], n);   // the stage's rows over all workgroups
      if (stamp) tstamp[2 + si] = wall_clock64();
    }
    __syncthreads();
  }
  if constexpr (GRID) {
    // the final rows of this workgroup go to the output table at a cursor;
    // the last workgroup to finish publishes
    const bool fin = s_state == CHS_OK;
    const ChainStage& sa = d.st[s_acc];
    const uint32_t n = fin ? s_cnt[s_acc] : 0u;
    if (threadIdx.x == 0) {
      if (s_state == CHS_REDO) atomicOr(&d.gsc[kGscRedo], 1u);
      s_base = n ? atomicAdd(&d.gsc[kGscOut], n) : 0u;
    }
    __syncthreads();
    if (n) {
      const uint64_t ld = sa.ld ? sa.ld : sa.cap;
      for (uint32_t c = 0; c < sa.ncols; ++c)
        for (uint32_t r = threadIdx.x; r < n; r += kSmallBlock)
          d.fin[c * d.fin_ld + s_base + r] = sa.dst[c * ld + off + r];
    }
    // No agent-scope fence here: on gfx950 each one writes this XCD's L2 back,
    // and 32 workgroups per XCD doing so in turn cost ~80 us per chain.  The
    // final rows are read by later launches (the kernel boundary makes them
    // visible); the last workgroup reads only counters, which are atomics
    // performed at the coherence point -- thread 0 waits for its own
    // atomics to complete before it arrives.
    __syncthreads();
    if (threadIdx.x == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // (an arrival in two levels, per wg % 8 group then global, measured no
      // faster: FlyBase step 0.229 / 0.233 vs 0.229 / 0.219 ms one-level)
      const uint32_t prev = __hip_atomic_fetch_add(&d.gsc[kGscDone], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_run = prev == G - 1 ? 1u : 0u;
    }
    __syncthreads();
    if (!s_run) return;
    // the last workgroup: every counter read at once (one lane a word, one
    // memory latency instead of a dependent load per stage), then left zero
    // for the next chain of a pooled counter block (no k_chain_prep launch)
    uint32_t* s_g = s_buf;
    if (threadIdx.x < kGscWords) {
      s_g[threadIdx.x] = __hip_atomic_load(&d.gsc[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&d.gsc[threadIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      if (tstamp) {                                  // DAS_TRACE: the last workgroup's start and finish
        tstamp[kChainStages + 2] = t_start;
        tstamp[kChainStages + 3] = wall_clock64();
      }
      // every workgroup's counters and rows are in: the outcome
      const uint32_t redo = s_g[kGscRedo];
      uint32_t empty = 0;                            // a positive stage after the partition with no row anywhere
      bool after = false;
      for (uint32_t si = 0; si < d.nstage; ++si) {
        if (after && d.st[si].op != CH_ANTI && d.st[si].op != CH_SCAN && d.st[si].done && s_g[si] == 0)
          empty |= 1u << si;
        after = after || d.st[si].part;
      }
      // a partitioned scan with no row on any workgroup: a failing term
      bool failed = false;
      for (uint32_t si = 0; si < d.nstage; ++si)
        if (d.st[si].op == CH_SCAN && d.st[si].part && d.st[si].append == kChainNoStage && !d.st[si].empty_ok &&
            s_g[si] == 0)
          failed = true;
      const uint32_t st = failed ? CHS_EMPTY_SCAN : redo ? CHS_REDO : s_state;   // before the partition every workgroup agrees
      const uint32_t total = st == CHS_OK ? s_g[kGscOut] : s_cnt[s_acc];
      __hip_atomic_store(&slot[0], st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&slot[1], total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&slot[2], s_acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&slot[3], empty, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __threadfence_system();
      __hip_atomic_store(&slot[15], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
  // every store of the chain is made visible before the host reads the
  // counts and (later, through other launches) the tables
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(&slot[0], s_state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&slot[1], s_cnt[s_acc], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&slot[2], s_acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    __hip_atomic_store(&slot[15], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void __launch_bounds__(kSmallBlock) k_chain(const uint32_t* __restrict__ hdesc, uint32_t nwords,
                                                       uint32_t* slot, uint32_t seq, uint64_t* tstamp) {
  chain_body<false>(hdesc, nwords, slot, seq, tstamp);
}

// one workgroup per CU; the descriptor is read from device memory (k_chain_prep)
__global__ void __launch_bounds__(kSmallBlock) k_chain_grid(const uint32_t* __restrict__ ddesc, uint32_t nwords,
                                                            uint32_t* slot, uint32_t seq, uint64_t* tstamp) {
  chain_body<true>(ddesc, nwords, slot, seq, tstamp);
}

// the grid chain's descriptor from pinned host memory into device memory
// (every workgroup then reads it from L2, not over PCIe) and its counters zeroed
// (the loads of one thread issued together: the host memory's latency paid once)
__global__ void __launch_bounds__(kSmallBlock) k_chain_prep(const uint32_t* __restrict__ hdesc, uint32_t nwords,
                                                            uint32_t* __restrict__ ddesc, uint32_t* __restrict__ gsc) {
  constexpr uint32_t kPer = (sizeof(ChainDesc) / 4 + kSmallBlock - 1) / kSmallBlock;
  uint32_t v[kPer];
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t i = threadIdx.x + k * kSmallBlock;
    v[k] = i < nwords ? hdesc[i] : 0u;
  }
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t i = threadIdx.x + k * kSmallBlock;
    if (i < nwords) ddesc[i] = v[k];
  }
  if (threadIdx.x < kGscWords) gsc[threadIdx.x] = 0u;
}

}  // namespace

// Rows per workgroup segment of the grid chain's stage tables, and whether an
// And's leading terms want the grid chain: a grounded scan (and scans joined
// to it) feeding an index join whose output can outgrow the one-workgroup
// chain -- bound = the scanned rows x the index join's largest key range
// (type_max_run, an upper bound whatever the grounded targets) -- e.g. the
// FlyBase F5 / F7 join on a recombination_loc shared by ~10^5 genes
// (DESIGN.md §5).  DAS_CHAIN_GRID: 0 never, 1 whenever the shape allows.
constexpr uint32_t kGridSeg = 4096;

uint32_t cu_count(Ctx& c) {
  static int n[64] = {0};
  int& v = n[c.device & 63];
  if (!v) DAS_HIP(hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, c.device));
  return (uint32_t)v;
}

// rows a partitioned first scan may have: half of the grid's segments (room
// for an index join's fan-out on each slice)
uint64_t part_scan_max(Ctx& c) { return (uint64_t)cu_count(c) * kGridSeg / 2; }

bool chain_grid_wanted(Ctx& c, const std::vector<const das_plan_node_t*>& terms, size_t n_anti, bool force) {
  if (terms.size() < 2) return false;
  std::vector<int32_t> vars;
  uint64_t bound = 1;
  for (size_t k = 0; k < terms.size(); ++k) {
    const das_plan_node_t* x = terms[k];
    if (x->op != DAS_PLAN_LINK || !x->scan.ordered || x->dedup) return false;
    if (k > 0 && x->index_join) {
      const das_link_scan_t& q = x->ij;
      int bp = -1;
      for (uint32_t p = 0; p < q.arity && p < 8; ++p)
        if (q.target[p] == kNone && q.var[p] >= 0 && std::find(vars.begin(), vars.end(), q.var[p]) != vars.end())
          bp = (int)p;
      if (bp >= 0 && q.type_id < c.idx.n_types && q.arity <= (uint32_t)kMaxPosArity) {
        if (bound > kIjSmall) return false;           // the partition's probe is every workgroup's
        bound *= std::max<uint64_t>(type_max_run(c, q.arity, (uint32_t)bp, q.type_id), 1);
        const bool more = k + 1 < terms.size() || n_anti > 0;
        return force || bound > kChainCap || (more && bound > kChainIjRows);
      }
    }
    ScanPrep P;
    scan_prepare(c, x->scan, P);
    if (P.empty || P.kind != DAS_TABLE_ORDERED || P.ranges.size() != 1) return false;
    const uint64_t r = P.ranges[0].second - P.ranges[0].first;
    // a first term too large to replicate, followed by an index join: the
    // grid can partition the scan itself (each workgroup a slice of its
    // rows).  Off unless DAS_CHAIN_PSCAN=1: on FlyBase FJ (3*10^5 probes, the
    // key-directory lookups of a 4.5*10^5-row schema) the chain took 61 us
    // on the GPU against 47 us for the scan + direct join, and the batched
    // step 0.250-0.268 vs 0.212-0.226 ms (profiles/r5_flybase_env_ab.txt)
    if (k == 0 && r > kGridSeg) {
      const char* ps = std::getenv("DAS_CHAIN_PSCAN");
      return ps && ps[0] == '1' && terms[1]->op == DAS_PLAN_LINK && terms[1]->index_join && r <= part_scan_max(c);
    }
    if (r > kGridSeg) return false;
    bound *= std::max<uint64_t>(r, 1);
    vars.insert(vars.end(), P.vars, P.vars + P.ncols);
  }
  return false;
}

// A compiled fused And (one-workgroup or grid chain) between its launch and
// the read-back of its outcome: fused_and runs compile -> launch -> finish in
// a row; das_plan_execute_many launches several before it waits for any.
struct ChainRun {
  ChainDesc d{};
  std::vector<std::unique_ptr<Table>> tabs;                  // one output table per stage
  std::vector<uint32_t> terms_done;                          // positive terms folded after each stage
  std::unique_ptr<Table> fin;                                // grid: the final rows
  DBuf<uint32_t> gsc, dd;                                    // grid: counters, device descriptor
  bool grid = false, complete = false;
  int acc = -1;
  PubSlot ps{};
  uint64_t* ts = nullptr;
  uint64_t bytes = 0;
  hipStream_t ls = nullptr;                                   // the stream it was launched on
  int fence = -1;                                             // side stream: its fence events (2k, 2k+1)
  bool waited = false;                                        // chain_finish read its outcome
  bool noprep = false;                                        // grid: pooled counters, descriptor read from pinned memory
};
// 1: compiled; 0: nothing to fuse; -1: the grid form does not apply
int chain_compile(Ctx& c, const std::vector<const das_plan_node_t*>& terms,
                  const std::vector<const das_plan_node_t*>& anti, bool grid, ChainRun& R, uint32_t* gsc_fixed = nullptr);
void chain_launch(Ctx& c, ChainRun& R, const PubSlot& ps, uint8_t* stage, int side = -1, uint32_t k = 0);
int chain_finish(Ctx& c, ChainRun& R, bool& matched, std::unique_ptr<Table>& out, uint32_t* consumed);

// whether fused_and applies, and the form it would take first (grid or not)
int fused_and_form(Ctx& c, const std::vector<const das_plan_node_t*>& terms,
                   const std::vector<const das_plan_node_t*>& anti, int no_overload) {
  const char* f = std::getenv("DAS_FUSED");                  // tests: 0 never
  if ((f && f[0] == '0') || no_overload || terms.empty()) return -1;
  const char* gm = std::getenv("DAS_CHAIN_GRID");
  const bool want_grid = !(gm && gm[0] == '0') && chain_grid_wanted(c, terms, anti.size(), gm && gm[0] == '1');
  if (trace_on()) trace_mark(want_grid ? "chain grid" : "chain one workgroup");
  return want_grid ? 1 : 0;
}

int fused_and(Ctx& c, const std::vector<const das_plan_node_t*>& terms,
              const std::vector<const das_plan_node_t*>& anti, int no_overload, bool& matched,
              std::unique_ptr<Table>& out, uint32_t* consumed) {
  const int form = fused_and_form(c, terms, anti, no_overload);
  if (form < 0) return 0;
  // One at a time (matched()), a grid chain takes its counters from this
  // read-back level's pooled block (zeroed; the grid's last workgroup leaves
  // it zero) and every workgroup reads the descriptor from the pinned stage:
  // no k_chain_prep launch -- FlyBase F5 / F6 / F7 46.7 / 39.4 / 56.8 vs
  // 50.2 / 43.7 / 61.4 us per query, the matched() step 0.236-0.251 vs
  // 0.257-0.280 ms (round 6, one box, 9 of 10 alternating pairs).
  // DAS_CHAIN_PREP1=1: the prep launch (fresh counters, the descriptor
  // copied to device memory once).
  const char* cp = std::getenv("DAS_CHAIN_PREP1");
  uint32_t* gsc = cp && cp[0] == '1' ? nullptr : c.gsc_block(kPubPool + (uint32_t)pub_level());
  for (int attempt = form == 1 ? 0 : 1; attempt < 2; ++attempt) {
    ChainRun R;
    const int r = chain_compile(c, terms, anti, attempt == 0, R, gsc);
    if (r < 0) continue;                                      // the grid form does not apply: one workgroup
    if (r == 0) return 0;
    // (the descriptor stages in this thread's pinned buffer, read by the
    // launches before the read-back returns)
    chain_launch(c, R, pub_reserve(), pinned_stage(((R.bytes + 63) & ~63ull) + 8 * (kChainStages + 4)));
    return chain_finish(c, R, matched, out, consumed);
  }
  return 0;
}

// gsc_fixed: a pooled, zeroed counter block (the grid kernel leaves it zero
// again), which lets the grid read its descriptor from the pinned buffer with
// no k_chain_prep launch; null: fresh counters zeroed by k_chain_prep
int chain_compile(Ctx& c, const std::vector<const das_plan_node_t*>& terms,
                  const std::vector<const das_plan_node_t*>& anti, bool grid, ChainRun& R, uint32_t* gsc_fixed) {
  Index& idx = c.idx;
  ChainDesc& d = R.d;
  R.grid = grid;
  const uint32_t G = grid ? cu_count(c) : 1u;
  const uint64_t gcap = (uint64_t)G * kGridSeg;              // grid: every stage table holds G segments
  std::vector<std::unique_ptr<Table>>& tabs = R.tabs;
  std::vector<uint32_t>& terms_done = R.terms_done;
  auto add = [&](uint32_t op) -> ChainStage* {
    if (d.nstage >= (uint32_t)kChainStages) return nullptr;
    ChainStage& st = d.st[d.nstage++];
    st.op = op;
    st.append = kChainNoStage;
    return &st;
  };
  // a stage's table: one workgroup -> `cap` rows; grid -> G segments of kGridSeg
  auto place = [&](ChainStage* st, Table& t) {
    st->cap = grid ? kGridSeg : (uint32_t)t.cap;
    st->ld = grid ? (uint32_t)t.cap : 0u;
    st->ncols = (uint32_t)t.ncols;
    st->dst = t.data;
  };
  bool parted = false;
  uint64_t scan_rows = 0;                                     // a partitioned first scan's rows
  // a chain ending early (too many stages) still folds the terms compiled so
  // far; the caller continues from there
  int& acc = R.acc;                                           // stage holding the running result
  uint32_t nterm = 0;
  bool all_terms = true;
  for (const das_plan_node_t* x : terms) {
    if (x->op != DAS_PLAN_LINK || !x->scan.ordered || x->dedup) { all_terms = false; break; }
    if (acc >= 0 && x->index_join) {
      IjPlan pl;
      const Table& A = *tabs[acc];
      // (after a partitioned scan each workgroup probes its slice: the
      // lookup through the key directory, never a search of one long range)
      const bool ijok = scan_rows ? ij_prepare(c, A, x->ij, scan_rows, pl, true) : ij_prepare(c, A, x->ij, kIjSmall, pl);
      if (trace_on()) trace_mark("prep ij_prepare");
      if (ijok) {
        if (pl.empty) { all_terms = false; break; }
        ChainStage* st = add(CH_IJ);
        if (!st) { all_terms = false; break; }
        auto t = new_table(c, DAS_TABLE_ORDERED, (int)pl.uni.size(), pl.uni.data(), grid ? gcap : kChainCap);
        if (trace_on()) trace_mark("prep new_table");
        for (size_t k = 0; k < pl.uni.size(); ++k) {
          t->lo[k] = pl.lo[k];
          t->hi[k] = pl.hi[k];
        }
        st->in = (uint32_t)acc;
        st->done = 1;
        place(st, *t);
        st->part = grid && !parted;
        parted = parted || grid;
        st->key = pl.akey;
        st->kx = pl.kx;
        st->g = pl.g;
        st->jc = pl.jc;
        tabs.push_back(std::move(t));
        terms_done.push_back(++nterm);
        acc = (int)d.nstage - 1;
        continue;
      }
    }
    ScanPrep P;
    scan_prepare(c, x->scan, P);
    if (trace_on()) trace_mark("prep scan_prepare");
    if (P.empty || P.kind != DAS_TABLE_ORDERED || P.ranges.size() != 1) { all_terms = false; break; }
    const uint64_t b = P.ranges[0].first, e = P.ranges[0].second;
    // grid: every workgroup scans it into its segment, or (the first term,
    // larger than a segment) each a slice of it
    const bool pscan = grid && acc < 0 && e - b > kGridSeg && e - b <= part_scan_max(c);
    if ((e - b > kSmallScan && !pscan) || e >= 0xFFFFFFFFull || d.nstage + (acc >= 0 ? 2 : 1) > (uint32_t)kChainStages) {
      all_terms = false;
      break;
    }
    if (grid && e - b > kGridSeg && !pscan) return -1;
    ChainStage* st = add(CH_SCAN);
    auto t = new_table(c, P.kind, P.ncols, P.vars, grid ? gcap : e - b);
    scan_bounds(idx, P.sp, x->scan.type_id, *t);
    if (trace_on()) trace_mark("prep scan table");
    st->sp = P.sp;
    st->begin = (uint32_t)b;
    st->end = (uint32_t)e;
    place(st, *t);
    st->done = acc < 0 ? 1 : 0;
    if (pscan) {
      st->part = 1;
      parted = true;
      scan_rows = e - b;
    }
    tabs.push_back(std::move(t));
    const int rel = (int)d.nstage - 1;
    if (acc < 0) {
      terms_done.push_back(++nterm);
      acc = rel;
      continue;
    }
    terms_done.push_back(nterm);
    // And's join of the running result with the scanned term (join(), the
    // natural join on the shared variables; a cross join when none)
    const Table& A = *tabs[acc];
    const Table& R = *tabs[rel];
    std::vector<int32_t> va(A.vars, A.vars + A.ncols), vb(R.vars, R.vars + R.ncols), shared, uni;
    std::set_intersection(va.begin(), va.end(), vb.begin(), vb.end(), std::back_inserter(shared));
    std::set_union(va.begin(), va.end(), vb.begin(), vb.end(), std::back_inserter(uni));
    DAS_CHECK((int)uni.size() <= kMaxCols, DAS_E_UNSUPPORTED, "too many variables");
    ChainStage* js = add(CH_JOIN);
    auto jt = new_table(c, DAS_TABLE_ORDERED, (int)uni.size(), uni.data(), grid ? gcap : kChainCap);
    js->in = (uint32_t)acc;
    js->rel = (uint32_t)rel;
    js->done = 1;
    place(js, *jt);
    for (int32_t v : shared) {
      js->sha[js->nsh] = A.col(colof_t(A, v));
      js->shb[js->nsh++] = R.col(colof_t(R, v));
    }
    for (int k = 0; k < (int)uni.size(); ++k) {
      const int ia = colof_t(A, uni[k]), ib = colof_t(R, uni[k]);
      uint32_t lo = 0, hi = kNone;
      if (ia >= 0) { lo = std::max(lo, A.lo[ia]); hi = std::min(hi, A.hi[ia]); }
      if (ib >= 0) { lo = std::max(lo, R.lo[ib]); hi = std::min(hi, R.hi[ib]); }
      jt->lo[k] = lo;
      jt->hi[k] = hi;
      if (ia >= 0) { js->jc.p[js->jc.np] = A.col(ia); js->jc.po[js->jc.np++] = k; }
      else { js->jc.b[js->jc.nb] = R.col(ib); js->jc.bo[js->jc.nb++] = k; }
    }
    tabs.push_back(std::move(jt));
    terms_done.push_back(++nterm);
    acc = (int)d.nstage - 1;
  }
  if (acc < 0) return 0;
  if (grid && !parted) return -1;                             // no index join to partition on
  const uint32_t n_anti_stage0 = d.nstage;
  bool anti_ok = all_terms;
  if (all_terms)
    for (const das_plan_node_t* x : anti) {
      AntiPlan ap;
      const Table& A = *tabs[acc];
      if (!anti_prepare(c, A, x->ij, ap) || ap.keep_all) continue;   // nothing forbidden / not a lookup: A whole
      ChainStage* st = add(CH_ANTI);
      if (!st) {                                                     // the caller applies them all
        d.nstage = n_anti_stage0;
        tabs.resize(n_anti_stage0);
        terms_done.resize(n_anti_stage0);
        acc = (int)n_anti_stage0 - 1;
        anti_ok = false;
        break;
      }
      auto t = new_table_like(c, A, A.cap);
      for (int k = 0; k < A.ncols; ++k) {
        t->lo[k] = A.lo[k];
        t->hi[k] = A.hi[k];
      }
      st->in = (uint32_t)acc;
      st->done = 1;
      place(st, *t);
      st->key = ap.key;
      st->kx = ap.kx;
      st->g = ap.g;
      st->ncopy = (uint32_t)A.ncols;
      for (int k = 0; k < A.ncols; ++k) st->copy[k] = A.col(k);
      tabs.push_back(std::move(t));
      terms_done.push_back(nterm);
      acc = (int)d.nstage - 1;
    }
  if (d.nstage < 2) return 0;                                 // one operator: nothing to fuse
  R.complete = all_terms && anti_ok;
  // grid: the final rows gather into one table; device copies of the
  // descriptor and the counters
  if (grid) {
    const Table& A = *tabs[acc];
    R.fin = new_table(c, DAS_TABLE_ORDERED, A.ncols, A.vars, gcap);
    for (int k = 0; k < A.ncols; ++k) {
      R.fin->lo[k] = A.lo[k];
      R.fin->hi[k] = A.hi[k];
    }
    if (!gsc_fixed) R.gsc.alloc(kGscWords, c.s);
    R.noprep = gsc_fixed != nullptr;
    d.seg = kGridSeg;
    d.fin = R.fin->data;
    d.fin_ld = R.fin->cap;
    d.gsc = gsc_fixed ? gsc_fixed : R.gsc.p;
  }
  // only the stages in use travel (the kernel copies them into LDS)
  R.bytes = offsetof(ChainDesc, st) + sizeof(ChainStage) * d.nstage;
  static_assert(sizeof(ChainStage) % 4 == 0 && offsetof(ChainDesc, st) % 4 == 0, "word copy");
  return 1;
}

// `stage`: pinned host memory of at least chain_stage_bytes(R) that stays
// untouched until chain_finish (the launches read the descriptor from it).
// fence >= 0: launched on a side stream (c.s points at it, fused_and_launch);
// fence event 2k + 1 marks its end, which chain_finish makes the context's
// stream wait for before any of its tables is read there.
void chain_launch(Ctx& c, ChainRun& R, const PubSlot& ps, uint8_t* stage, int side, uint32_t k) {
  if (side >= 0) R.fence = (int)k;
  R.ls = c.s;
  const ChainDesc& d = R.d;
  const uint64_t bytes = R.bytes;
  // (DAS_TRACE: stage timestamps of the device clock after the descriptors)
  const uint64_t tsoff = (bytes + 63) & ~63ull;
  uint8_t* hd = stage;
  std::memcpy(hd, &d, bytes);
  R.ts = trace_on() ? reinterpret_cast<uint64_t*>(hd + tsoff) : nullptr;
  if (R.ts) std::memset(R.ts, 0, 8 * (kChainStages + 4));
  // algorithmic bytes known up front: the scanned index rows
  double sbytes = 0;
  for (uint32_t i = 0; i < d.nstage; ++i)
    if (d.st[i].op == CH_SCAN) sbytes += 4.0 * (d.st[i].end - d.st[i].begin) * (d.st[i].sp.arity + 1);
  if (trace_on()) trace_mark("prep staged");
  R.ps = ps;
  if (R.grid && R.noprep) {
    // every workgroup copies the descriptor from the pinned buffer itself
    ProfScope pf(c, "k_chain_grid", sbytes);
    hipLaunchKernelGGL(k_chain_grid, dim3(cu_count(c)), dim3(kSmallBlock), 0, c.s, (const uint32_t*)hd,
                       (uint32_t)(bytes / 4), ps.p, ps.seq, R.ts);
    DAS_HIP(hipGetLastError());
  } else if (R.grid) {
    const uint32_t G = cu_count(c);
    R.dd.alloc(bytes / 4, c.s);
    {
      ProfScope pf(c, "k_chain_prep", 2.0 * bytes);
      hipLaunchKernelGGL(k_chain_prep, dim3(1), dim3(kSmallBlock), 0, c.s, (const uint32_t*)hd, (uint32_t)(bytes / 4),
                         R.dd.p, R.gsc.p);
      DAS_HIP(hipGetLastError());
    }
    ProfScope pf(c, "k_chain_grid", sbytes);
    hipLaunchKernelGGL(k_chain_grid, dim3(G), dim3(kSmallBlock), 0, c.s, (const uint32_t*)R.dd.p,
                       (uint32_t)(bytes / 4), ps.p, ps.seq, R.ts);
    DAS_HIP(hipGetLastError());
  } else {
    ProfScope pf(c, "k_chain", sbytes);
    hipLaunchKernelGGL(k_chain, dim3(1), dim3(kSmallBlock), 0, c.s, (const uint32_t*)hd, (uint32_t)(bytes / 4), ps.p,
                       ps.seq, R.ts);
    DAS_HIP(hipGetLastError());
  }
  if (R.fence >= 0) DAS_HIP(hipEventRecord(c.fence_event(2 * k + 1), c.s));
}

uint64_t chain_stage_bytes(const ChainRun& R) { return ((R.bytes + 63) & ~63ull) + 8 * (kChainStages + 4); }

int chain_finish(Ctx& c, ChainRun& R, bool& matched, std::unique_ptr<Table>& out, uint32_t* consumed) {
  const ChainDesc& d = R.d;
  const bool grid = R.grid, complete = R.complete;
  uint64_t* ts = R.ts;
  auto& tabs = R.tabs;
  uint32_t w[4] = {0, 0, 0, 0};
  pub_wait(R.ps, R.ls ? R.ls : c.s, w, 4);
  R.waited = true;
  if (R.fence >= 0) {
    DAS_HIP(hipStreamWaitEvent(c.s, c.fence_event(2 * R.fence + 1), 0));
    R.fence = -1;
  }
  if (ts) {
    static const char* const kOp[] = {"?", "scan", "ij", "join", "anti"};
    trace_mark("chain copy", std::to_string((ts[1] - ts[0]) / 100.0) + " us");
    for (uint32_t i = 0; i < d.nstage && ts[2 + i]; ++i)
      trace_mark("chain stage", std::string(kOp[d.st[i].op < 5 ? d.st[i].op : 0]) + " " +
                                    std::to_string((ts[2 + i] - (i ? ts[1 + i] : ts[1])) / 100.0) + " us");
    if (grid && ts[kChainStages + 3])
      trace_mark("chain grid last workgroup",
                 "started " + std::to_string(((int64_t)ts[kChainStages + 2] - (int64_t)ts[0]) / 100.0) +
                     " us after workgroup 0, published at " +
                     std::to_string(((int64_t)ts[kChainStages + 3] - (int64_t)ts[0]) / 100.0) + " us");
  }
  matched = false;
  out.reset();
  if (w[0] == CHS_EMPTY_SCAN) return 1;                       // a failing term: And is False
  // grid: a segment overflowed after the partition, or a running result was
  // empty on every workgroup (And's reset-on-empty path): the caller folds
  // the whole And operator by operator
  if (w[0] == CHS_REDO || (grid && w[0] == CHS_OK && w[3] != 0)) {
    if (trace_on()) trace_mark("chain grid redo");
    return 0;
  }
  DAS_CHECK(w[2] < d.nstage && d.st[w[2]].done, DAS_E_INTERNAL, "fused chain: bad running result");
  const uint32_t last = w[2];
  // algorithmic bytes known only now: the final rows (grid: written to a
  // workgroup segment, then gathered into the output table)
  if (w[0] == CHS_OK && c.prof)
    prof_add_bytes(c, grid ? "k_chain_grid" : "k_chain", (grid ? 12.0 : 4.0) * d.st[last].ncols * w[1]);
  if (grid && w[0] == CHS_OK) {
    DAS_CHECK(last == (uint32_t)R.acc, DAS_E_INTERNAL, "grid chain: bad running result");
    if (complete && w[1] == 0) return 1;                      // nothing left after the Not filters
    R.fin->nrows = w[1];
    if (complete) {
      matched = true;
      out = std::move(R.fin);
      return 1;
    }
    out = std::move(R.fin);
    *consumed = R.terms_done[last];
    return 2;
  }
  if (w[0] == CHS_OK && last == d.nstage - 1 && complete) {
    if (w[1] == 0) return 1;                                  // nothing left after the Not filters
    tabs[last]->nrows = w[1];
    matched = true;
    out = std::move(tabs[last]);
    return 1;
  }
  // partial: the running result after terms_done[last] positive terms, no
  // Not filter applied yet (anti stages never stop a chain); in the grid
  // form only at or before the partition, where every workgroup holds the
  // same rows (workgroup 0's segment is rows [0, n) of the table)
  if (d.st[last].op == CH_ANTI) return 0;                     // cannot happen (anti stages never stop); be safe
  tabs[last]->nrows = w[1];
  out = std::move(tabs[last]);
  *consumed = R.terms_done[last];
  return 2;
}

bool fused_and_viable(Ctx& c, const std::vector<const das_plan_node_t*>& terms,
                      const std::vector<const das_plan_node_t*>& anti, int no_overload) {
  const int form = fused_and_form(c, terms, anti, no_overload);
  if (form < 0) return false;
  if (form == 1) return true;
  // the one-workgroup chain scans its first term whole: not past kSmallScan rows
  const das_plan_node_t* x = terms[0];
  if (x->op != DAS_PLAN_LINK || !x->scan.ordered || x->dedup) return false;
  ScanPrep P;
  scan_prepare(c, x->scan, P);
  return !P.empty && P.kind == DAS_TABLE_ORDERED && P.ranges.size() == 1 &&
         P.ranges[0].second - P.ranges[0].first <= kSmallScan;
}

std::unique_ptr<UnionRun> fused_or_launch(Ctx& c, const std::vector<const das_plan_node_t*>& terms, int no_overload,
                                          uint32_t k, int side, hipEvent_t fence_in, bool* waited) {
  struct Swap {
    Ctx& c;
    hipStream_t old;
    ~Swap() { c.s = old; }
  } sw{c, c.s};
  if (side >= 0) {
    hipStream_t ss = c.side_stream(side);
    if (waited && !*waited) {
      DAS_HIP(hipStreamWaitEvent(ss, fence_in, 0));
      *waited = true;
    }
    c.s = ss;
  }
  auto u = std::make_unique<UnionRun>();
  u->pool = k;
  bool m = false;
  std::unique_ptr<Table> t;
  if (fused_or(c, terms, no_overload, m, t, u.get()) != 2) return nullptr;
  if (side >= 0) {
    DAS_HIP(hipEventRecord(c.fence_event(2 * k + 1), c.s));
    u->fence = (int)k;
  }
  return u;
}

int fused_or_finish(Ctx& c, UnionRun& u, bool& matched, std::unique_ptr<Table>& out) {
  uint32_t n = 0;
  pub_wait(u.ps, u.ls ? u.ls : c.s, &n, 1);
  u.waited = true;
  if (u.fence >= 0) {
    DAS_HIP(hipStreamWaitEvent(c.s, c.fence_event(2 * u.fence + 1), 0));
    u.fence = -1;
  }
  matched = false;
  out.reset();
  if (n == 0xFFFFFFFFu) return 0;                             // the union did not fit: the Or another way
  matched = n > 0;
  if (matched) {
    u.res->nrows = n;
    u.res->lo[0] = u.ulo;
    u.res->hi[0] = u.uhi;
    u.res->sorted_col = -1;
    out = std::move(u.res);
  }
  return 1;
}

void ChainRunDel::operator()(ChainRun* r) const {
  // a run dropped before its outcome was read (an error in another plan of
  // the batch): its kernels may still read its tables, its pinned descriptor
  // and its slot, which the next run of the same pool entry reuses
  if (r && r->ls && !r->waited) (void)hipStreamSynchronize(r->ls);
  delete r;
}

ChainRunPtr fused_and_launch(Ctx& c, const std::vector<const das_plan_node_t*>& terms,
                             const std::vector<const das_plan_node_t*>& anti, int no_overload, uint32_t k,
                             int side, hipEvent_t fence_in, bool* waited) {
  const int form = fused_and_form(c, terms, anti, no_overload);
  if (form < 0) return nullptr;
  // a side stream: the run's tables are that stream's blocks, so it needs no
  // ordering after the context's stream beyond the batch's first fence
  struct Swap {
    Ctx& c;
    hipStream_t old;
    ~Swap() { c.s = old; }
  } sw{c, c.s};
  if (side >= 0) {
    hipStream_t ss = c.side_stream(side);
    if (waited && !*waited) {
      DAS_HIP(hipStreamWaitEvent(ss, fence_in, 0));
      *waited = true;
    }
    c.s = ss;
  }
  // DAS_CHAIN_PREP=0: pooled zeroed counters and every workgroup reading the
  // descriptor from pinned memory, no k_chain_prep launch -- measured no
  // faster (FlyBase step 0.235 / 0.254 vs 0.230 / 0.234 ms with the prep,
  // profiles/r5_flybase_env_ab.txt), so the prep stays the default
  const char* fp = std::getenv("DAS_CHAIN_PREP");
  uint32_t* gsc = fp && fp[0] == '0' ? c.gsc_block(k) : nullptr;
  for (int attempt = form == 1 ? 0 : 1; attempt < 2; ++attempt) {
    ChainRunPtr R(new ChainRun);
    const int r = chain_compile(c, terms, anti, attempt == 0, *R, gsc);
    if (r < 0) continue;
    if (r == 0 || !R->complete) return nullptr;
    chain_launch(c, *R, pub_reserve_pool(k), pinned_stage_pool(k, chain_stage_bytes(*R)), side, k);
    return R;
  }
  return nullptr;
}

int fused_and_finish(Ctx& c, ChainRun& R, bool& matched, std::unique_ptr<Table>& out) {
  uint32_t consumed = 0;
  const int r = chain_finish(c, R, matched, out, &consumed);
  if (r == 1) return 1;
  matched = false;
  out.reset();
  return 0;
}

int fused_or(Ctx& c, const std::vector<const das_plan_node_t*>& terms, int no_overload, bool& matched,
             std::unique_ptr<Table>& out, UnionRun* defer) {
  const char* f = std::getenv("DAS_FUSED");                  // tests: 0 never
  if ((f && f[0] == '0') || no_overload || terms.size() < 2 || terms.size() + 1 > (size_t)kChainStages) return 0;
  Index& idx = c.idx;
  std::vector<ScanPrep> preps(terms.size());
  uint64_t total = 0;
  for (size_t i = 0; i < terms.size(); ++i) {
    const das_plan_node_t* x = terms[i];
    if (x->op != DAS_PLAN_LINK || !x->scan.ordered) return 0;
    ScanPrep& P = preps[i];
    scan_prepare(c, x->scan, P);
    if (P.kind != DAS_TABLE_ORDERED) return 0;
    if (i && (P.ncols != preps[0].ncols || !std::equal(P.vars, P.vars + P.ncols, preps[0].vars))) return 0;
    if (P.empty) continue;
    if (P.ranges.size() != 1) return 0;
    total += P.ranges[0].second - P.ranges[0].first;
  }
  if (total == 0) return 0;
  bool single = true;
  for (auto& P : preps) single = single && (P.empty || P.ranges.size() == 1);
  const char* fm = std::getenv("DAS_UNION_MULTI");            // tests: 1 = always the multi-launch form
  const bool multi = total > kChainHash / 2 || !single || (fm && fm[0] == '1');
  if (defer && !multi) return 0;                              // deferred: the union launch only
  if (multi) {
    // larger: every range of every term counted in one launch, written in
    // one, then one dedup of the concatenation
    MultiScan ms{};
    uint64_t chunks = 0;
    for (auto& P : preps) {
      if (P.empty) continue;
      for (auto& r : P.ranges) {
        if (r.second <= r.first) continue;
        if (ms.nseg == (uint32_t)kMultiSeg) return 0;
        MultiScan::Seg& sg = ms.seg[ms.nseg++];
        sg.sp = P.sp;
        sg.begin = r.first;
        sg.end = r.second;
        sg.chunk0 = chunks;
        chunks += (r.second - r.first + kChunk - 1) / kChunk;
      }
    }
    if (!ms.nseg || chunks >= (1ull << 31)) return 0;
    uint64_t scanned = 0;
    for (uint32_t i = 0; i < ms.nseg; ++i) scanned += ms.seg[i].end - ms.seg[i].begin;
    // the union's column bounds: the union of the terms' bounds
    uint32_t ulo[kMaxCols], uhi[kMaxCols];
    for (int k = 0; k < preps[0].ncols; ++k) {
      ulo[k] = kNone;
      uhi[k] = 0;
    }
    for (size_t i = 0; i < terms.size(); ++i) {
      if (preps[i].empty) continue;
      Table tb;
      tb.ncols = preps[i].ncols;
      scan_bounds(idx, preps[i].sp, terms[i]->scan.type_id, tb);
      for (int k = 0; k < preps[0].ncols; ++k) {
        ulo[k] = std::min(ulo[k], tb.lo[k]);
        uhi[k] = std::max(uhi[k], tb.hi[k]);
      }
    }
    {
      // one output column: bitmap union in one launch (k_union_first)
      bool proj = preps[0].ncols == 1 && uhi[0] != kNone && ulo[0] <= uhi[0] && uhi[0] - ulo[0] < (1u << 27) &&
                  scanned < 0xFFFFFFF0ull;
      for (uint32_t i = 0; i < ms.nseg && proj; ++i)
        proj = !ms.seg[i].sp.unordered && !ms.seg[i].sp.emit_link && ms.seg[i].sp.nout == 1;
      const char* fb = std::getenv("DAS_UNION_BITS");                // A/B, tests: 0 never
      // (its segments re-chunked by B rows: one row per thread)
      MultiScan ms1 = ms;
      uint64_t blocks = 0;
      for (uint32_t i = 0; i < ms1.nseg; ++i) {
        ms1.seg[i].chunk0 = blocks;
        blocks += (ms1.seg[i].end - ms1.seg[i].begin + B - 1) / B;
      }
      proj = proj && blocks < (1ull << 32) / B;                 // the dispatch grid counts work-items in 32 bits
      if (defer && !(proj && !(fb && fb[0] == '0'))) return 0;   // deferred: the union launch only
      if (proj && !(fb && fb[0] == '0')) {
        const uint32_t range = uhi[0] - ulo[0] + 1;
        auto res = new_table(c, DAS_TABLE_ORDERED, 1, preps[0].vars, scanned);
        // (a fresh, filled bitmap per union: a context-level all-zero bitmap
        // cleared after each union was slower -- the clear of ~10^5 set bits
        // ran behind the union on the stream, F9 40 -> 53-59 us)
        const uint64_t words = (range + 31) / 32;
        DBuf<uint32_t> own(words + 3, c.s);
        fill_dev(own.p, 0, 4 * (words + 3), c.s);
        uint32_t* bitsp = own.p;
        uint32_t* ctrp = bitsp + words;
        const PubSlot ps = defer ? pub_reserve_pool(defer->pool) : pub_reserve();
        {
          ProfScope pf(c, "k_union_first", 8.0 * scanned);
          hipLaunchKernelGGL(k_union_first, dim3((unsigned)blocks), dim3(B), 0, c.s, ms1, ulo[0], range, bitsp,
                             res->data, ctrp, ps.p, ps.seq);
          DAS_HIP(hipGetLastError());
        }
        if (defer) {
          defer->res = std::move(res);
          defer->own = std::move(own);
          defer->ps = ps;
          defer->ulo = ulo[0];
          defer->uhi = uhi[0];
          defer->ls = c.s;
          return 2;
        }
        uint32_t n = 0;
        pub_wait(ps, c.s, &n, 1);
        if (n != 0xFFFFFFFFu) {
          out.reset();
          matched = n > 0;
          if (matched) {
            res->nrows = n;
            res->lo[0] = ulo[0];
            res->hi[0] = uhi[0];
            res->sorted_col = -1;
            out = std::move(res);
          }
          return 1;
        }
      }
    }
    DBuf<uint32_t> cnt(chunks, c.s), off(chunks + 1, c.s);
    {
      ProfScope pf(c, "k_scan_count_multi", 4.0 * scanned * terms[0]->scan.arity);
      hipLaunchKernelGGL(k_scan_count_multi, dim3((unsigned)chunks), dim3(B), 0, c.s, ms, cnt.p);
      DAS_HIP(hipGetLastError());
    }
    const uint64_t m = scan_total<uint32_t>(SpanIn<uint32_t>{cnt.p}, chunks, off.p, c.s);
    matched = false;
    out.reset();
    if (!m) return 1;
    auto cat = new_table(c, DAS_TABLE_ORDERED, preps[0].ncols, preps[0].vars, m);
    cat->nrows = m;
    {
      ProfScope pf(c, "k_scan_write_multi", 4.0 * scanned * (terms[0]->scan.arity + 1) + 4.0 * m * cat->ncols);
      hipLaunchKernelGGL(k_scan_write_multi, dim3((unsigned)chunks), dim3(B), 0, c.s, ms, (const uint32_t*)off.p,
                         cat->data, cat->cap);
      DAS_HIP(hipGetLastError());
    }
    for (int k = 0; k < cat->ncols; ++k) {
      cat->lo[k] = ulo[k];
      cat->hi[k] = uhi[k];
    }
    out = dedup(c, *cat);
    matched = out->nrows > 0;
    if (!matched) out.reset();
    return 1;
  }
  ChainDesc d{};
  auto cat = new_table(c, DAS_TABLE_ORDERED, preps[0].ncols, preps[0].vars, total);
  auto res = new_table(c, DAS_TABLE_ORDERED, preps[0].ncols, preps[0].vars, total);
  // column bounds: the union of the terms' bounds
  for (int k = 0; k < res->ncols; ++k) {
    res->lo[k] = kNone;
    res->hi[k] = 0;
  }
  bool any = false;
  for (size_t i = 0; i < terms.size(); ++i) {
    ScanPrep& P = preps[i];
    if (P.empty) continue;
    Table tb;
    tb.ncols = P.ncols;
    scan_bounds(idx, P.sp, terms[i]->scan.type_id, tb);
    for (int k = 0; k < res->ncols; ++k) {
      res->lo[k] = std::min(res->lo[k], tb.lo[k]);
      res->hi[k] = std::max(res->hi[k], tb.hi[k]);
    }
    ChainStage& st = d.st[d.nstage++];
    st.op = CH_SCAN;
    st.sp = P.sp;
    st.begin = (uint32_t)P.ranges[0].first;
    st.end = (uint32_t)P.ranges[0].second;
    st.cap = (uint32_t)cat->cap;
    st.dst = cat->data;
    st.empty_ok = 1;
    st.append = any ? 0u : kChainNoStage;
    st.done = any ? 0u : 1u;
    any = true;
  }
  ChainStage& dd = d.st[d.nstage++];
  dd.op = CH_DEDUP;
  dd.in = 0;
  dd.done = 1;
  dd.cap = (uint32_t)res->cap;
  dd.dst = res->data;
  dd.ncopy = (uint32_t)cat->ncols;
  for (int k = 0; k < cat->ncols; ++k) dd.copy[k] = cat->col(k);
  const uint64_t bytes = offsetof(ChainDesc, st) + sizeof(ChainStage) * d.nstage;
  uint8_t* hd = pinned_stage(bytes);
  std::memcpy(hd, &d, bytes);
  const PubSlot ps = pub_reserve();
  {
    ProfScope pf(c, "k_chain", 4.0 * total * (terms[0]->scan.arity + 1));
    hipLaunchKernelGGL(k_chain, dim3(1), dim3(kSmallBlock), 0, c.s, (const uint32_t*)hd, (uint32_t)(bytes / 4), ps.p,
                       ps.seq, (uint64_t*)nullptr);
    DAS_HIP(hipGetLastError());
  }
  uint32_t w[3] = {0, 0, 0};
  pub_wait(ps, c.s, w, 3);
  DAS_CHECK(w[0] == CHS_OK && w[2] == d.nstage - 1, DAS_E_INTERNAL, "fused union: incomplete");
  matched = w[1] > 0;
  out.reset();
  if (matched) {
    res->nrows = w[1];
    out = std::move(res);
  }
  return 1;
}

// ---------------------------------------------------------------------------
// Semi-join: the build side Q holds only the join variable.  When its keys
// are distinct (a typed Link with one variable and grounded other targets:
// each row is a different link, e.g. T(V2, h1) of the hub And), the join is
// a filter of P by Q's key set -- one bit per id of the key range (16 MB for
// 2^27 ids, L2/MALL-resident) instead of offsets and (first, count) pairs per
// key slot and two random lookups per probe row.  Duplicate keys (a bit
// already set) are detected while the bits are set; then the caller takes
// the direct join (multiplicities matter).
// ---------------------------------------------------------------------------
__global__ void k_bits_set(const uint32_t* __restrict__ key, uint64_t n, uint32_t kmin, uint32_t range,
                           uint32_t* bits, uint32_t* dup) {
  uint32_t d = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t k = key[i] - kmin;
    if (k >= range) continue;
    const uint32_t m = 1u << (k & 31);
    if (atomicOr(&bits[k >> 5], m) & m) d = 1;
  }
  if (__ballot(d) && __lane_id() == 0) atomicOr(dup, 1u);
}
// Same for a SORTED key column: lanes of a wave whose keys share a bitmap
// word are contiguous, so a segmented OR scan (duplicates show up as bits
// already present) leaves one atomic per word segment -- hub keys sit in
// adjacent ids, and per-key atomics on their few words would serialise.
__global__ void k_bits_set_sorted(const uint32_t* __restrict__ key, uint64_t n, uint32_t kmin, uint32_t range,
                                  uint32_t* bits, uint32_t* dup) {
  const int lane = __lane_id();
  uint32_t d = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x; i0 < n; i0 += stride) {     // wave-uniform trip count
    const uint64_t i = i0 + threadIdx.x;
    const uint32_t k = i < n ? key[i] - kmin : 0xFFFFFFFFu;
    const bool act = k < range;
    const uint32_t w = act ? k >> 5 : 0xFFFFFFFFu;
    uint32_t m = act ? 1u << (k & 31) : 0u;
#pragma unroll
    for (int st = 1; st < 64; st <<= 1) {
      const uint32_t om = (uint32_t)__shfl_up(m, st, 64), ow = (uint32_t)__shfl_up(w, st, 64);
      if (lane >= st && ow == w && act) {
        if (om & (1u << (k & 31))) d = 1;              // another lane of the segment holds this key
        m |= om;
      }
    }
    const uint32_t nw = (uint32_t)__shfl_down(w, 1, 64);
    const bool tail = act && (lane == 63 || nw != w);
    if (tail && (atomicOr(&bits[w], m) & m)) d = 1;
  }
  if (__ballot(d) && __lane_id() == 0) atomicOr(dup, 1u);
}

struct BitsPred {
  const uint32_t* key;
  uint32_t kmin, range;
  const uint32_t* bits;
  __device__ __forceinline__ bool operator()(uint64_t i) const {
    const uint32_t k = key[i] - kmin;
    return k < range && ((bits[k >> 5] >> (k & 31)) & 1u);
  }
};

std::unique_ptr<Table> semi_join(Ctx& c, const Table& P, const Table& Q) {
  const char* f = std::getenv("DAS_SEMI_JOIN");           // tests: 0 never
  if (f && f[0] == '0') return nullptr;
  const int32_t var = Q.vars[0];
  int pk = -1;
  for (int i = 0; i < P.ncols; ++i) if (P.vars[i] == var) pk = i;
  if (pk < 0 || Q.nrows >= 0xFFFFFFFFull) return nullptr;
  uint32_t lo = Q.lo[0], hi = Q.hi[0];
  if (hi == kNone || lo > hi) {
    lo = 0;
    hi = (uint32_t)(c.idx.n_atoms ? c.idx.n_atoms - 1 : 0);
  }
  const uint64_t range = (uint64_t)hi - lo + 1;
  if (range > (1ull << 31)) return nullptr;
  const uint64_t words = (range + 31) / 32;
  DBuf<uint32_t> bits(words + 1, c.s);                     // + the duplicate flag
  fill_dev(bits.p, 0, 4 * (words + 1), c.s);
  {
    ProfScope ps(c, "join_build", 4.0 * Q.nrows + 4.0 * words);
    hipLaunchKernelGGL(k_bits_set, G(Q.nrows), dim3(B), 0, c.s, (const uint32_t*)Q.col(0), Q.nrows, lo, (uint32_t)range,
                       bits.p, bits.p + words);
    DAS_HIP(hipGetLastError());
  }
  // the probe is the compaction's predicate: no flag array; duplicate keys
  // (counts matter: nullptr, the caller joins) are read back with the count
  return compact_pred(c, P, BitsPred{(const uint32_t*)P.col(pk), lo, (uint32_t)range, (const uint32_t*)bits.p},
                      "k_tile_count<BitsPred>", 4.0, (const uint32_t*)bits.p + words);
}

// Several one-variable build sides on the same variable (consecutive terms of
// an And, e.g. T2(V2, h1), T3(V2, h0) of the hub query): their key sets are
// intersected as bitmaps first -- one set pass per term into its own bitmap
// (duplicates detected as in semi_join), one AND per extra term -- and P is
// filtered ONCE by the intersection, instead of one probe + compaction pass
// per term.  The bitmap spans the intersection of the columns' id bounds: a
// key outside it is in no intersection.  nullptr when a side does not fit
// (the caller joins term by term); the plan executor checks that the result
// is non-empty before taking it (And's reset-on-empty rule).
__global__ void k_bits_and(uint32_t* __restrict__ acc, const uint32_t* __restrict__ b, uint64_t words) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < words; i += (uint64_t)gridDim.x * blockDim.x)
    acc[i] &= b[i];
}

// The intersection of the key sets of Qs (one column each, variable `var`) as
// a bitmap over [lo, hi] (narrowed here to the Qs' bounds); false when a Q
// does not qualify, the range is too wide or a Q repeats a key.  lo > hi on
// return: the bounds are disjoint, no key is in every set.
bool key_bits(Ctx& c, const std::vector<const Table*>& Qs, int32_t var, uint64_t& lo, uint64_t& hi,
              DBuf<uint32_t>& acc) {
  auto clip = [&](uint32_t l, uint32_t h) {
    if (h == kNone || l > h) return;                       // unknown bound
    lo = std::max<uint64_t>(lo, l);
    hi = std::min<uint64_t>(hi, h);
  };
  for (const Table* Q : Qs) {
    if (Q->kind != DAS_TABLE_ORDERED || Q->ncols != 1 || Q->vars[0] != var || Q->nrows >= 0xFFFFFFFFull) return false;
    clip(Q->lo[0], Q->hi[0]);
  }
  if (lo > hi) return true;
  const uint64_t range = hi - lo + 1;
  if (range > (1ull << 31)) return false;
  const uint64_t words = (range + 31) / 32;
  acc.alloc(words + 1, c.s);                                // + the duplicate flag
  DBuf<uint32_t> one(Qs.size() > 1 ? words + 1 : 1, c.s);
  // every term's duplicate-key flag goes to acc[words]: one read-back at the end
  for (size_t i = 0; i < Qs.size(); ++i) {
    uint32_t* bits = i == 0 ? acc.p : one.p;
    fill_dev(bits, 0, 4 * (i == 0 ? words + 1 : words), c.s);
    {
      ProfScope ps(c, "join_build", 4.0 * Qs[i]->nrows + 4.0 * words);
      if (Qs[i]->sorted_col == 0)
        hipLaunchKernelGGL(k_bits_set_sorted, G(Qs[i]->nrows), dim3(B), 0, c.s, (const uint32_t*)Qs[i]->col(0),
                           Qs[i]->nrows, (uint32_t)lo, (uint32_t)range, bits, acc.p + words);
      else
        hipLaunchKernelGGL(k_bits_set, G(Qs[i]->nrows), dim3(B), 0, c.s, (const uint32_t*)Qs[i]->col(0),
                           Qs[i]->nrows, (uint32_t)lo, (uint32_t)range, bits, acc.p + words);
      DAS_HIP(hipGetLastError());
    }
    if (i) {
      KScope ks("k_bits_and", 12.0 * words);
      hipLaunchKernelGGL(k_bits_and, G(words), dim3(B), 0, c.s, acc.p, (const uint32_t*)one.p, words);
      DAS_HIP(hipGetLastError());
    }
  }
  return read_u32(acc.p + words, c.s) == 0;                  // duplicate keys: counts matter
}

std::unique_ptr<Table> semi_join_multi(Ctx& c, const Table& P, const std::vector<const Table*>& Qs) {
  if (Qs.empty() || P.kind != DAS_TABLE_ORDERED || !P.nrows) return nullptr;
  const int32_t var = Qs[0]->vars[0];
  int pk = -1;
  for (int i = 0; i < P.ncols; ++i) if (P.vars[i] == var) pk = i;
  if (pk < 0) return nullptr;
  uint64_t lo = 0, hi = c.idx.n_atoms ? c.idx.n_atoms - 1 : 0;
  if (P.hi[pk] != kNone && P.lo[pk] <= P.hi[pk]) {
    lo = P.lo[pk];
    hi = std::min<uint64_t>(hi, P.hi[pk]);
  }
  DBuf<uint32_t> acc;
  if (!key_bits(c, Qs, var, lo, hi, acc)) return nullptr;
  if (lo > hi) return new_table_like(c, P, 0);              // disjoint bounds: nothing passes
  const uint64_t range = hi - lo + 1;
  auto out = compact_pred(c, P, BitsPred{(const uint32_t*)P.col(pk), (uint32_t)lo, (uint32_t)range,
                                         (const uint32_t*)acc.p},
                          "k_tile_count<BitsPred>", 4.0);
  out->sorted_col = P.sorted_col;
  for (int k = 0; k < out->ncols; ++k) {
    out->lo[k] = P.lo[k];
    out->hi[k] = P.hi[k];
  }
  out->lo[pk] = (uint32_t)lo;
  out->hi[pk] = (uint32_t)hi;
  return out;
}

// index_join(A, q) followed by the semi-join of every Qs[i] on q's fresh
// variable fvar, with the join's outputs filtered while they are expanded
// (k_dj_filt) -- the unfiltered join is never written.  nullptr when it does
// not apply; the plan executor takes a non-empty result only.
std::unique_ptr<Table> index_join_filtered(Ctx& c, const Table& A, const das_link_scan_t& q, int32_t fvar,
                                           const std::vector<const Table*>& Qs) {
  IjPlan pl;
  if (Qs.empty() || !ij_prepare(c, A, q, A.nrows, pl) || pl.empty) return nullptr;
  pl.jc.search = owner_search_env();
  const JoinCols& jc = pl.jc;
  if (jc.np > 4 || jc.nb > 4) return nullptr;
  int fb = -1;
  for (int i = 0; i < jc.nb; ++i)
    if (pl.uni[jc.bo[i]] == fvar) fb = i;
  if (fb < 0) return nullptr;
  const int nu = (int)pl.uni.size();
  const int fo = jc.bo[fb];
  uint64_t lo = 0, hi = c.idx.n_atoms ? c.idx.n_atoms - 1 : 0;
  if (pl.hi[fo] != kNone && pl.lo[fo] <= pl.hi[fo]) {
    lo = pl.lo[fo];
    hi = std::min<uint64_t>(hi, pl.hi[fo]);
  }
  DBuf<uint32_t> bits;
  if (!key_bits(c, Qs, fvar, lo, hi, bits)) return nullptr;
  if (lo > hi) return new_table(c, DAS_TABLE_ORDERED, nu, pl.uni.data(), 0);
  DBuf<uint2> lc(A.nrows, c.s);
  DBuf<uint32_t> rowid(A.nrows, c.s);
  {
    ProfScope ps(c, "k_ij_lc", 4.0 * A.nrows + 8.0 * A.nrows + 4.0 * A.nrows);
    hipLaunchKernelGGL(k_ij_lc, G(A.nrows), dim3(B), 0, c.s, pl.akey, A.nrows, pl.kx, pl.g, lc.p, rowid.p);
    DAS_HIP(hipGetLastError());
  }
  const uint64_t units = (A.nrows + kXRows - 1) / kXRows;
  const unsigned grid = grid_for(units, B / 64, 65535u * 4u);
  DBuf<uint64_t> tot(units, c.s), toff(units + 1, c.s);
  {
    ProfScope ps(c, "k_dj_count", 4.0 * A.nrows);
    hipLaunchKernelGGL(k_dj_count, dim3(grid), dim3(B), 0, c.s, (const uint32_t*)rowid.p, A.nrows, 0u,
                       (uint32_t)A.nrows, (const uint2*)lc.p, units, tot.p, (const uint32_t*)nullptr,
                       (const uint32_t*)nullptr);
    DAS_HIP(hipGetLastError());
  }
  const uint64_t total = scan_total<uint64_t>(SpanIn<uint64_t>{tot.p}, units, toff.p, c.s);
  if (!total) return new_table(c, DAS_TABLE_ORDERED, nu, pl.uni.data(), 0);
  if (total >= (1ull << 32) - (1ull << 16)) return nullptr;
  const uint64_t chunks = (total + kBalChunk - 1) / kBalChunk;
  const unsigned fgrid = grid_for(chunks, B / 64, 65535u * 4u);
  const FiltKey fk{jc.b[fb], (uint32_t)lo, (uint32_t)(hi - lo + 1), (const uint32_t*)bits.p, fb};
  // DAS_FILT_FUSED=1: one pass, unsorted output, while the worst case (every
  // virtual output kept) fits the output buffer.  Off by default: at config 5
  // it ran 924 us against 337 + 296 us for the two ordered passes (round 3,
  // profiles/archive/r3_hub_filt_ab.json) -- the LDS flag tiles cut its occupancy
  const char* ff = std::getenv("DAS_FILT_FUSED");
  if (ff && ff[0] == '1' && (uint64_t)nu * total * 4 <= (16ull << 30)) {
    const unsigned ugrid = grid_for((chunks + (B / 64) * kFuseChunks - 1) / ((B / 64) * kFuseChunks), 1, 65535u * 4u);
    auto out = new_table(c, DAS_TABLE_ORDERED, nu, pl.uni.data(), total);
    DBuf<unsigned long long> kept(1, c.s);
    fill_dev(kept.p, 0, 8, c.s);
    const bool spec = (jc.np == 1 && jc.nb == 1) || (jc.np == 2 && jc.nb == 1) || (jc.np == 1 && jc.nb == 2);
    {
      // per probe row its row id, (first, count) and probe columns; per
      // output its build value and (kept) its build columns; kept outputs out
      ProfScope ps(c, spec ? "k_dj_filt_fused<" + std::to_string(jc.np) + "," + std::to_string(jc.nb) + ">"
                           : std::string("k_dj_filt_fused<-1,-1>"),
                   (12.0 + 4.0 * jc.np) * A.nrows + 4.0 * total);
#define FILT_F(NPV, NBV)                                                                                          \
  hipLaunchKernelGGL((k_dj_filt_fused<NPV, NBV>), dim3(ugrid), dim3(B), 0, c.s, (const uint32_t*)rowid.p, A.nrows, 0u, \
                     (uint32_t)A.nrows, (const uint2*)lc.p, units, (const uint64_t*)toff.p, total, fk, jc, out->data,  \
                     out->cap, kept.p)
      if (jc.np == 1 && jc.nb == 1) FILT_F(1, 1);
      else if (jc.np == 2 && jc.nb == 1) FILT_F(2, 1);
      else if (jc.np == 1 && jc.nb == 2) FILT_F(1, 2);
      else FILT_F(-1, -1);
#undef FILT_F
      DAS_HIP(hipGetLastError());
    }
    out->nrows = read_u64(reinterpret_cast<const uint64_t*>(kept.p), c.s);
    // the kept outputs' columns written (bytes known only now: charged to the scope's launch below)
    prof_add_bytes(c, spec ? "k_dj_filt_fused<" + std::to_string(jc.np) + "," + std::to_string(jc.nb) + ">"
                           : std::string("k_dj_filt_fused<-1,-1>"),
                   (4.0 * nu) * out->nrows);
    out->sorted_col = -1;                          // chunks land in completion order
    for (int k = 0; k < nu; ++k) {
      out->lo[k] = pl.lo[k];
      out->hi[k] = pl.hi[k];
    }
    out->lo[fo] = (uint32_t)lo;
    out->hi[fo] = (uint32_t)hi;
    return out;
  }
  // outputs per wave chunk of the two passes (DAS_FILT_CHUNK: 1024 / 2048 / 4096, A/B)
  static const int ch = [] {
    const char* e = std::getenv("DAS_FILT_CHUNK");
    const int v = e ? std::atoi(e) : 0;
    return v == 2048 || v == 4096 ? v : 1024;
  }();
  const uint64_t fchunks = (total + ch - 1) / ch;
  const unsigned fgrid2 = grid_for(fchunks, B / 64, 65535u * 4u);
  // one walk writing kept outputs chunk-locally (k_dj_filt<2>) + a
  // compaction of the chunk runs: config 5's H4 0.82 -> 0.71 ms against the
  // flag pass and a second walk (DAS_FILT_LOCAL=0, A/B;
  // profiles/archive/r3_hub_local_ab.json)
  const char* fle = std::getenv("DAS_FILT_LOCAL");
  const bool local = !(fle && fle[0] == '0');
  // its scratch holds every virtual output's columns (4 nu B each, against one
  // flag byte per output for the two passes): taken while that stays within
  // 16 GiB and half the device's free memory, and falls back to the two
  // passes when the allocation fails (DAS_FILT_SCRATCH_MAX caps it, tests)
  const uint64_t scr_bytes = (uint64_t)nu * total * 4;
  const char* sme = std::getenv("DAS_FILT_SCRATCH_MAX");
  const uint64_t scr_cap = sme ? std::strtoull(sme, nullptr, 10) : (16ull << 30);
  bool fits = local && ch == 1024 && scr_bytes <= scr_cap;
  if (fits && scr_bytes > (1ull << 30)) {
    size_t fr = 0, tot = 0;
    fits = hipMemGetInfo(&fr, &tot) == hipSuccess && scr_bytes <= fr / 2;
  }
  DBuf<uint32_t> scr;
  if (fits) {
    try {
      scr.alloc((uint64_t)nu * total, c.s);
    } catch (const Error&) {
      (void)hipGetLastError();
      fits = false;                                   // out of memory: the two passes below
    }
  }
  if (fits) {
    // The one walk stages each chunk's kept rows in its wave's LDS rows and
    // writes them to the chunk's slots of the scratch with 16-byte stores
    // (k_dj_filt_staged, 512-output chunks): the walk itself 429 -> 228 us at
    // config 5 (each lane's scattered 4-byte stores were the cost).
    // DAS_FILT_STAGED=0: the unstaged walk (k_dj_filt<2>, 1024-output chunks);
    // =atomic: the staged rows placed straight in the output by one atomic
    // per chunk, no scratch, no compaction -- 1,600 us: 1.2 * 10^5 atomics on
    // one address from 8 XCDs serialise (A/B record, output unsorted)
    const char* se = std::getenv("DAS_FILT_STAGED");
    const bool spec = (jc.np == 1 && jc.nb == 1) || (jc.np == 2 && jc.nb == 1) || (jc.np == 1 && jc.nb == 2);
    const bool staged = !(se && se[0] == '0') && spec && nu == jc.np + jc.nb;
    const bool atomic_place = staged && se && !std::strcmp(se, "atomic");
    const uint64_t sch = staged ? 512 : 1024;
    const uint64_t nch = (total + sch - 1) / sch;
    const unsigned sgrid = grid_for(nch, B / 64, 65535u * 4u);
    DBuf<uint32_t> ccnt(nch, c.s), coff(nch + 1, c.s);
    DBuf<unsigned long long> kept;
    std::unique_ptr<Table> direct_out;
    if (atomic_place) {
      direct_out = new_table(c, DAS_TABLE_ORDERED, nu, pl.uni.data(), total);
      kept.alloc(1, c.s);
      fill_dev(kept.p, 0, 8, c.s);
    }
    // the chunks' first units (DAS_FILT_CUNIT=0: the walk searches them)
    const char* cue = std::getenv("DAS_FILT_CUNIT");
    const bool cun = staged && !(cue && cue[0] == '0') && units < (1ull << 32);
    DBuf<uint32_t> cunit;
    if (cun) {
      cunit.alloc(nch, c.s);
      KScope ks("k_chunk_units", 4.0 * nch);
      hipLaunchKernelGGL(k_chunk_units<512>, G(nch), dim3(B), 0, c.s, (const uint64_t*)toff.p, units, nch, cunit.p);
      DAS_HIP(hipGetLastError());
    }
    const std::string nm = staged ? "k_dj_filt_staged<" + std::to_string(jc.np) + "," + std::to_string(jc.nb) + ",512>"
                           : spec ? "k_dj_filt<2," + std::to_string(jc.np) + "," + std::to_string(jc.nb) + ",1024,4>"
                                  : std::string("k_dj_filt<2,-1,-1,1024,4>");
    {
      // per probe row its row id, (first, count) and probe columns; per
      // output its build value (a P row); kept outputs' columns written
      ProfScope ps(c, nm, (12.0 + 4.0 * jc.np) * A.nrows + 4.0 * total);
#define FILT_S(NPV, NBV)                                                                                         \
  hipLaunchKernelGGL((k_dj_filt_staged<NPV, NBV, 512>), dim3(sgrid), dim3(B), 0, c.s, (const uint32_t*)nullptr,    \
                     A.nrows, 0u, (uint32_t)A.nrows, (const uint2*)lc.p, units, (const uint64_t*)toff.p, total, fk, \
                     jc, atomic_place ? direct_out->data : scr.p, atomic_place ? direct_out->cap : total, 0ull, nch, \
                     atomic_place ? (uint32_t*)nullptr : ccnt.p, atomic_place ? kept.p : nullptr, \
                     cun ? (const uint32_t*)cunit.p : nullptr)
#define FILT_L(NPV, NBV)                                                                                       \
  hipLaunchKernelGGL((k_dj_filt<2, NPV, NBV, 1024>), dim3(sgrid), dim3(B), 0, c.s, (const uint32_t*)rowid.p, A.nrows, \
                     0u, (uint32_t)A.nrows, (const uint2*)lc.p, units, (const uint64_t*)toff.p, total, fk,             \
                     (uint8_t*)nullptr, ccnt.p, (const uint32_t*)nullptr, jc, scr.p, total, 0ull, nch)
      if (staged) {
        if (jc.np == 1 && jc.nb == 1) FILT_S(1, 1);
        else if (jc.np == 2 && jc.nb == 1) FILT_S(2, 1);
        else FILT_S(1, 2);
      } else if (jc.np == 1 && jc.nb == 1) FILT_L(1, 1);
      else if (jc.np == 2 && jc.nb == 1) FILT_L(2, 1);
      else if (jc.np == 1 && jc.nb == 2) FILT_L(1, 2);
      else FILT_L(-1, -1);
#undef FILT_S
#undef FILT_L
      DAS_HIP(hipGetLastError());
    }
    auto finish = [&](std::unique_ptr<Table> out, int sorted) {
      out->sorted_col = sorted;
      for (int k = 0; k < nu; ++k) {
        out->lo[k] = pl.lo[k];
        out->hi[k] = pl.hi[k];
      }
      out->lo[fo] = (uint32_t)lo;
      out->hi[fo] = (uint32_t)hi;
      return out;
    };
    if (atomic_place) {
      const uint64_t m = read_u64(reinterpret_cast<const uint64_t*>(kept.p), c.s);
      prof_add_bytes(c, nm, 4.0 * nu * m);
      direct_out->nrows = m;
      return finish(std::move(direct_out), -1);               // chunks land in completion order
    }
    const uint64_t m = scan_total<uint32_t>(SpanIn<uint32_t>{ccnt.p}, nch, coff.p, c.s);
    prof_add_bytes(c, nm, 4.0 * nu * m);
    auto out = new_table(c, DAS_TABLE_ORDERED, nu, pl.uni.data(), m);
    out->nrows = m;
    if (m) {
      KScope ks(staged ? "k_chunk_compact<512>" : "k_chunk_compact<1024>", 8.0 * nu * m + 8.0 * nch);
      if (staged)
        hipLaunchKernelGGL(k_chunk_compact<512>, dim3(sgrid), dim3(B), 0, c.s, (const uint32_t*)scr.p, total,
                           (const uint32_t*)ccnt.p, (const uint32_t*)coff.p, 0ull, nch, nu, out->data, out->cap);
      else
        hipLaunchKernelGGL(k_chunk_compact<1024>, dim3(sgrid), dim3(B), 0, c.s, (const uint32_t*)scr.p, total,
                           (const uint32_t*)ccnt.p, (const uint32_t*)coff.p, 0ull, nch, nu, out->data, out->cap);
      DAS_HIP(hipGetLastError());
    }
    const int sorted = A.sorted_col >= 0 ? colof_t(*out, A.vars[A.sorted_col]) : -1;
    return finish(std::move(out), sorted);
  }
  DBuf<uint8_t> fl(total, c.s);
  DBuf<uint32_t> ccnt(fchunks, c.s), coff(fchunks + 1, c.s);
  {
    // per probe row its row id and (first, count); per output its build
    // value (a P row) and its flag byte
    // (xu: see DAS_FILT_UNROLL below; the scope names rocprof's instantiation)
    static const int xu0 = [] {
      const char* e = std::getenv("DAS_FILT_UNROLL");
      const int v = e ? std::atoi(e) : 0;
      return v == 8 || v == 16 ? v : 4;
    }();
    ProfScope ps(c, "k_dj_filt<0,-1,-1," + std::to_string(ch) + "," + std::to_string(ch == 1024 ? xu0 : 4) + ">",
                 12.0 * A.nrows + 5.0 * total);
#define FILT_0(CHV)                                                                                                \
  hipLaunchKernelGGL((k_dj_filt<0, -1, -1, CHV>), dim3(fgrid2), dim3(B), 0, c.s, (const uint32_t*)rowid.p, A.nrows,   \
                     0u, (uint32_t)A.nrows, (const uint2*)lc.p, units, (const uint64_t*)toff.p, total, fk, fl.p, ccnt.p, \
                     (const uint32_t*)nullptr, jc, (uint32_t*)nullptr, 0ull, 0ull, fchunks)
    // DAS_FILT_UNROLL (8 / 16): rounds of 64 outputs whose build values and
    // bitmap words are loaded together in the flag pass (A/B; default 4)
    static const int xu = [] {
      const char* e = std::getenv("DAS_FILT_UNROLL");
      const int v = e ? std::atoi(e) : 0;
      return v == 8 || v == 16 ? v : 4;
    }();
    if (ch == 2048) FILT_0(2048);
    else if (ch == 4096) FILT_0(4096);
    else if (xu == 8)
      hipLaunchKernelGGL((k_dj_filt<0, -1, -1, 1024, 8>), dim3(fgrid2), dim3(B), 0, c.s, (const uint32_t*)rowid.p,
                         A.nrows, 0u, (uint32_t)A.nrows, (const uint2*)lc.p, units, (const uint64_t*)toff.p, total, fk,
                         fl.p, ccnt.p, (const uint32_t*)nullptr, jc, (uint32_t*)nullptr, 0ull, 0ull, fchunks);
    else if (xu == 16)
      hipLaunchKernelGGL((k_dj_filt<0, -1, -1, 1024, 16>), dim3(fgrid2), dim3(B), 0, c.s, (const uint32_t*)rowid.p,
                         A.nrows, 0u, (uint32_t)A.nrows, (const uint2*)lc.p, units, (const uint64_t*)toff.p, total, fk,
                         fl.p, ccnt.p, (const uint32_t*)nullptr, jc, (uint32_t*)nullptr, 0ull, 0ull, fchunks);
    else FILT_0(1024);
#undef FILT_0
    DAS_HIP(hipGetLastError());
  }
  const uint64_t m = scan_total<uint32_t>(SpanIn<uint32_t>{ccnt.p}, fchunks, coff.p, c.s);
  auto out = new_table(c, DAS_TABLE_ORDERED, nu, pl.uni.data(), m);
  out->nrows = m;
  if (m) {
    // + the probe columns, the flags, the kept outputs' build rows and their columns out
    // (named as rocprof names the instantiation launched below)
    const bool spec = (jc.np == 1 && jc.nb == 1) || (jc.np == 2 && jc.nb == 1) || (jc.np == 1 && jc.nb == 2);
    const std::string chs4 = "," + std::to_string(ch) + ",4>";
    ProfScope ps(c, spec ? "k_dj_filt<1," + std::to_string(jc.np) + "," + std::to_string(jc.nb) + chs4
                         : "k_dj_filt<1,-1,-1" + chs4,
                 (12.0 + 4.0 * jc.np) * A.nrows + 1.0 * total + 4.0 * jc.nb * m + 4.0 * nu * m);
#define FILT_W(NPV, NBV, CHV)                                                                                  \
  hipLaunchKernelGGL((k_dj_filt<1, NPV, NBV, CHV>), dim3(fgrid2), dim3(B), 0, c.s, (const uint32_t*)rowid.p, A.nrows, \
                     0u, (uint32_t)A.nrows, (const uint2*)lc.p, units, (const uint64_t*)toff.p, total, fk, fl.p,      \
                     (uint32_t*)nullptr, (const uint32_t*)coff.p, jc, out->data, out->cap, 0ull, fchunks)
#define FILT_WC(CHV)                                    \
  if (jc.np == 1 && jc.nb == 1) FILT_W(1, 1, CHV);      \
  else if (jc.np == 2 && jc.nb == 1) FILT_W(2, 1, CHV); \
  else if (jc.np == 1 && jc.nb == 2) FILT_W(1, 2, CHV); \
  else FILT_W(-1, -1, CHV);
    if (ch == 2048) { FILT_WC(2048) }
    else if (ch == 4096) { FILT_WC(4096) }
    else { FILT_WC(1024) }
#undef FILT_WC
#undef FILT_W
    DAS_HIP(hipGetLastError());
  }
  out->sorted_col = A.sorted_col >= 0 ? colof_t(*out, A.vars[A.sorted_col]) : -1;
  for (int k = 0; k < nu; ++k) {
    out->lo[k] = pl.lo[k];
    out->hi[k] = pl.hi[k];
  }
  out->lo[fo] = (uint32_t)lo;
  out->hi[fo] = (uint32_t)hi;
  return out;
}

std::unique_ptr<Table> join(Ctx& c, const Table& A, const Table& Bt, int no_overload) {
  if (A.kind != DAS_TABLE_ORDERED || Bt.kind != DAS_TABLE_ORDERED) return theta_join(c, A, Bt, no_overload);
  // schemas
  std::vector<int32_t> va(A.vars, A.vars + A.ncols), vb(Bt.vars, Bt.vars + Bt.ncols), shared, uni;
  std::set_intersection(va.begin(), va.end(), vb.begin(), vb.end(), std::back_inserter(shared));
  std::set_union(va.begin(), va.end(), vb.begin(), vb.end(), std::back_inserter(uni));
  DAS_CHECK((int)uni.size() <= kMaxCols, DAS_E_UNSUPPORTED, "too many variables");
  auto colof = [](const Table& t, int32_t v) {
    for (int i = 0; i < t.ncols; ++i) if (t.vars[i] == v) return i;
    return -1;
  };
  const int nu = (int)uni.size();
  if (A.nrows == 0 || Bt.nrows == 0) return new_table(c, DAS_TABLE_ORDERED, nu, uni.data(), 0);
  // probe = larger side, build = smaller (sorted)
  const bool a_probe = A.nrows >= Bt.nrows;
  const Table& P = a_probe ? A : Bt;
  const Table& Q = a_probe ? Bt : A;
  std::unique_ptr<Table> out;
  if (shared.empty()) {
    const uint64_t total = P.nrows * Q.nrows;
    out = new_table(c, DAS_TABLE_ORDERED, nu, uni.data(), total);
    out->nrows = total;
    OutMap om{};
    om.n = nu;
    for (int k = 0; k < nu; ++k) {
      int ip = colof(P, uni[k]);
      if (ip >= 0) { om.col[k] = P.col(ip); om.side[k] = 0; }
      else { om.col[k] = Q.col(colof(Q, uni[k])); om.side[k] = 1; }
    }
    ProfScope ps(c, "k_cartesian<" + std::to_string(nu >= 2 && nu <= 6 ? nu : 0) + ">", 4.0 * nu * total);
    const unsigned cg = grid_for((total + 3) / 4, B);
    const uint64_t S = 4ull * cg * B, sq = S / Q.nrows, sr = S % Q.nrows;
    DAS_CHECK(out->cap % 4 == 0 && (reinterpret_cast<uintptr_t>(out->data) & 15) == 0, DAS_E_INTERNAL,
              "cartesian: output columns not 16-byte aligned");
    switch (nu) {
      case 2: hipLaunchKernelGGL(k_cartesian<2>, dim3(cg), dim3(B), 0, c.s, om, P.nrows, Q.nrows, total, sq, sr, out->data, out->cap); break;
      case 3: hipLaunchKernelGGL(k_cartesian<3>, dim3(cg), dim3(B), 0, c.s, om, P.nrows, Q.nrows, total, sq, sr, out->data, out->cap); break;
      case 4: hipLaunchKernelGGL(k_cartesian<4>, dim3(cg), dim3(B), 0, c.s, om, P.nrows, Q.nrows, total, sq, sr, out->data, out->cap); break;
      case 5: hipLaunchKernelGGL(k_cartesian<5>, dim3(cg), dim3(B), 0, c.s, om, P.nrows, Q.nrows, total, sq, sr, out->data, out->cap); break;
      case 6: hipLaunchKernelGGL(k_cartesian<6>, dim3(cg), dim3(B), 0, c.s, om, P.nrows, Q.nrows, total, sq, sr, out->data, out->cap); break;
      default: hipLaunchKernelGGL(k_cartesian<0>, dim3(cg), dim3(B), 0, c.s, om, P.nrows, Q.nrows, total, sq, sr, out->data, out->cap); break;
    }
    DAS_HIP(hipGetLastError());
  } else if (shared.size() == 1 && Q.ncols == 1 && (out = semi_join(c, P, Q))) {
    // key-set filter taken (the build side adds no columns)
  } else if (shared.size() == 1 && (out = direct_join(c, P, Q, shared[0], uni))) {
    // direct-address path taken
  } else {
    // sort build rows by the shared columns
    ColSet qk{};
    qk.n = (int)shared.size();
    for (int k = 0; k < qk.n; ++k) qk.c[k] = Q.col(colof(Q, shared[k]));
    DBuf<uint32_t> perm(Q.nrows, c.s);
    {
      ProfScope ps(c, "join_build_sort", 4.0 * Q.nrows * (Q.ncols + 2));
      sort_perm(qk, Q.nrows, perm.p, id_bits(c), c.s);
    }
    auto Qs = gather_table(c, Q, perm.p, Q.nrows);
    perm.release();
    ColSet qks{}, pk{};
    qks.n = pk.n = (int)shared.size();
    for (int k = 0; k < qks.n; ++k) {
      qks.c[k] = Qs->col(colof(*Qs, shared[k]));
      pk.c[k] = P.col(colof(P, shared[k]));
    }
    DBuf<uint32_t> lo(P.nrows, c.s), cnt(P.nrows, c.s);
    DBuf<uint64_t> offs(P.nrows + 1, c.s);
    {
      ProfScope ps(c, "k_join_count", 4.0 * P.nrows * (pk.n + 2));
      hipLaunchKernelGGL(k_join_count, G(P.nrows), dim3(B), 0, c.s, pk, P.nrows, qks, Qs->nrows, lo.p, cnt.p);
      DAS_HIP(hipGetLastError());
    }
    const uint64_t total = scan_total<uint64_t>(WidenCnt{cnt.p, P.nrows}, P.nrows, offs.p, c.s);
    out = new_table(c, DAS_TABLE_ORDERED, nu, uni.data(), total);
    out->nrows = total;
    if (total) {
      OutMap om{};
      om.n = nu;
      for (int k = 0; k < nu; ++k) {
        int ip = colof(P, uni[k]);
        if (ip >= 0) { om.col[k] = P.col(ip); om.side[k] = 0; }
        else { om.col[k] = Qs->col(colof(*Qs, uni[k])); om.side[k] = 1; }
      }
      // algorithmic: the join's output, |O| x 4 B x k_out
      ProfScope ps(c, "k_join_expand", 4.0 * nu * total);
      hipLaunchKernelGGL(k_join_expand, G(total), dim3(B), 0, c.s, (const uint64_t*)offs.p, P.nrows,
                         (const uint32_t*)lo.p, om, total, out->data, out->cap);
      DAS_HIP(hipGetLastError());
    }
  }
  // the output keeps the probe side's row order (direct, sort-merge and
  // cartesian joins all emit in probe order)
  {
    const Table& Pt = A.nrows >= Bt.nrows ? A : Bt;
    out->sorted_col = Pt.sorted_col >= 0 ? colof(*out, Pt.vars[Pt.sorted_col]) : -1;
  }
  // output column bounds: the source column's (both sides' intersection for a shared variable)
  for (int k = 0; k < out->ncols; ++k) {
    uint32_t lo = 0, hi = kNone;
    const int ia = colof(A, out->vars[k]), ib = colof(Bt, out->vars[k]);
    if (ia >= 0) { lo = std::max(lo, A.lo[ia]); hi = std::min(hi, A.hi[ia]); }
    if (ib >= 0) { lo = std::max(lo, Bt.lo[ib]); hi = std::min(hi, Bt.hi[ib]); }
    out->lo[k] = lo;
    out->hi[k] = hi;
  }
  if (no_overload && out->nrows) {
    // _join_ordered NO_COVERING path re-assigns every value (pattern_matcher.py:128-137);
    // covering joins return an operand unchanged.
    const bool a_sub = std::includes(vb.begin(), vb.end(), va.begin(), va.end());
    const bool b_sub = std::includes(va.begin(), va.end(), vb.begin(), vb.end());
    if (!a_sub && !b_sub) {
      DBuf<uint32_t> keep(out->nrows, c.s);
      hipLaunchKernelGGL(k_overload_flags, G(out->nrows), dim3(B), 0, c.s, cols_of(*out), out->nrows, keep.p);
      DAS_HIP(hipGetLastError());
      out = compact_table(c, *out, keep.p);
    }
  }
  return out;
}

// Hash sets below 2^26 rows (a table of <= 2^28 slots); DAS_SET_SORT=1 forces
// the sort-based path (tests cover both).
bool use_hash_set(uint64_t n) {
  const char* f = std::getenv("DAS_SET_SORT");
  return n <= (1ull << 26) && !(f && f[0] == '1');
}
uint32_t hset_mask(uint64_t n) {
  uint64_t m = 1024;
  while (m < 2 * n) m <<= 1;
  return (uint32_t)(m - 1);
}

std::unique_ptr<Table> antijoin(Ctx& c, const Table& A, const Table& T) {
  if (A.kind != DAS_TABLE_ORDERED || T.kind != DAS_TABLE_ORDERED) return theta_antijoin(c, A, T);
  std::vector<int32_t> va(A.vars, A.vars + A.ncols), vt(T.vars, T.vars + T.ncols);
  const bool covered = std::includes(va.begin(), va.end(), vt.begin(), vt.end());
  if (!covered || T.nrows == 0 || A.nrows == 0) {
    DBuf<uint32_t> idx(A.nrows ? A.nrows : 1, c.s);
    iota(idx.p, A.nrows, c.s);
    return gather_table(c, A, idx.p, A.nrows);
  }
  auto colof = [](const Table& t, int32_t v) {
    for (int i = 0; i < t.ncols; ++i) if (t.vars[i] == v) return i;
    return -1;
  };
  ColSet tk = cols_of(T);
  if (use_hash_set(T.nrows)) {
    ColSet ak{};
    ak.n = T.ncols;
    for (int k = 0; k < T.ncols; ++k) ak.c[k] = A.col(colof(A, T.vars[k]));
    const uint32_t mask = hset_mask(T.nrows);
    DBuf<uint32_t> tab((uint64_t)mask + 1, c.s), keep(A.nrows, c.s);
    fill_dev(tab.p, 0xFF, 4ull * (mask + 1), c.s);
    hipLaunchKernelGGL(k_hset_insert, G(T.nrows), dim3(B), 0, c.s, tk, T.nrows, tab.p, mask, 0);
    DAS_HIP(hipGetLastError());
    {
      ProfScope ps(c, "k_hset_anti", 4.0 * A.nrows * (T.ncols + 1));
      hipLaunchKernelGGL(k_hset_anti, G(A.nrows), dim3(B), 0, c.s, ak, A.nrows, tk, (const uint32_t*)tab.p, mask,
                         keep.p);
      DAS_HIP(hipGetLastError());
    }
    return compact_table(c, A, keep.p);
  }
  DBuf<uint32_t> perm(T.nrows, c.s);
  sort_perm(tk, T.nrows, perm.p, id_bits(c), c.s);
  auto Ts = gather_table(c, T, perm.p, T.nrows);
  ColSet tks = cols_of(*Ts), ak{};
  ak.n = T.ncols;
  for (int k = 0; k < T.ncols; ++k) ak.c[k] = A.col(A.kind == DAS_TABLE_ORDERED ? colof(A, T.vars[k]) : k);
  DBuf<uint32_t> keep(A.nrows, c.s);
  {
    ProfScope ps(c, "k_anti_flags", 4.0 * A.nrows * (T.ncols + 1));
    hipLaunchKernelGGL(k_anti_flags, G(A.nrows), dim3(B), 0, c.s, ak, A.nrows, tks, Ts->nrows, keep.p);
  }
  DAS_HIP(hipGetLastError());
  return compact_table(c, A, keep.p);
}

std::unique_ptr<Table> dedup(Ctx& c, const Table& A) {
  if (A.kind == DAS_TABLE_COMPOSITE) {
    const Table* one = &A;
    return std::move(set_dedup(c, &one, 1)[0]);
  }
  if (A.nrows <= 1) {
    DBuf<uint32_t> idx(A.nrows ? A.nrows : 1, c.s);
    iota(idx.p, A.nrows, c.s);
    return gather_table(c, A, idx.p, A.nrows);
  }
  if (use_hash_set(A.nrows)) {
    // first occurrences, in input order (the input's row order is kept)
    const uint32_t mask = hset_mask(A.nrows);
    DBuf<uint32_t> tab((uint64_t)mask + 1, c.s), keep(A.nrows, c.s);
    fill_dev(tab.p, 0xFF, 4ull * (mask + 1), c.s);
    hipLaunchKernelGGL(k_hset_insert, G(A.nrows), dim3(B), 0, c.s, cols_of(A), A.nrows, tab.p, mask, 1);
    DAS_HIP(hipGetLastError());
    {
      ProfScope ps(c, "k_hset_first", 4.0 * A.nrows * (A.ncols + 1));
      hipLaunchKernelGGL(k_hset_first, G(A.nrows), dim3(B), 0, c.s, cols_of(A), A.nrows, (const uint32_t*)tab.p, mask,
                         keep.p);
      DAS_HIP(hipGetLastError());
    }
    return compact_table(c, A, keep.p);
  }
  DBuf<uint32_t> perm(A.nrows, c.s);
  sort_perm(cols_of(A), A.nrows, perm.p, id_bits(c), c.s);
  auto S = gather_table(c, A, perm.p, A.nrows);
  S->sorted_col = A.ncols ? 0 : -1;
  DBuf<uint32_t> keep(A.nrows, c.s);
  hipLaunchKernelGGL(k_distinct_flags, G(A.nrows), dim3(B), 0, c.s, cols_of(*S), A.nrows, keep.p);
  DAS_HIP(hipGetLastError());
  return compact_table(c, *S, keep.p);
}

// ---------------------------------------------------------------------------
// Exchange helpers (multi-GPU): destination by key hash, row-major staging
// ---------------------------------------------------------------------------
namespace {
__global__ void k_dest(ColSet key, uint64_t n, uint32_t nparts, uint32_t* dest) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t h = 0x9e3779b9u;
    for (int c = 0; c < key.n; ++c) h = mix32(h ^ (key.c[c][i] + 0x7f4a7c15u * (uint32_t)(c + 1)));
    dest[i] = h % nparts;
  }
}
__global__ void k_rows_out(ColSet src, uint64_t n, uint32_t* dst) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    for (int c = 0; c < src.n; ++c) dst[i * src.n + c] = src.c[c][i];
}
__global__ void k_rows_in(const uint32_t* src, uint64_t n, int ncols, uint32_t* out, uint64_t cap) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    for (int c = 0; c < ncols; ++c) out[(uint64_t)c * cap + i] = src[i * ncols + c];
}
__global__ void k_dest_hist(const uint32_t* dest, uint64_t n, unsigned long long* cnt) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[dest[i]], 1ull);
}
}  // namespace

std::unique_ptr<Table> partition(Ctx& c, const Table& t, const int32_t* key_vars, uint32_t nkey, uint32_t nparts,
                                 uint64_t* counts) {
  DAS_CHECK(nparts >= 1 && nparts <= 4096, DAS_E_INVALID, "bad partition count");
  ColSet key{};
  if (nkey == 0) {
    key = cols_of(t);
  } else {
    key.n = (int)nkey;
    for (uint32_t k = 0; k < nkey; ++k) {
      int ci = -1;
      for (int i = 0; i < t.ncols; ++i) if (t.vars[i] == key_vars[k]) ci = i;
      DAS_CHECK(ci >= 0, DAS_E_INVALID, "partition key is not a column of the table");
      key.c[k] = t.col(ci);
    }
  }
  for (uint32_t d = 0; d < nparts; ++d) counts[d] = 0;
  if (t.nrows == 0) return gather_table(c, t, nullptr, 0);
  DBuf<uint32_t> dest(t.nrows, c.s), perm(t.nrows, c.s);
  DBuf<unsigned long long> h(nparts, c.s);
  fill_dev(h.p, 0, 8 * nparts, c.s);
  hipLaunchKernelGGL(k_dest, G(t.nrows), dim3(B), 0, c.s, key, t.nrows, nparts, dest.p);
  hipLaunchKernelGGL(k_dest_hist, G(t.nrows), dim3(B), 0, c.s, (const uint32_t*)dest.p, t.nrows, h.p);
  DAS_HIP(hipGetLastError());
  iota(perm.p, t.nrows, c.s);
  radix_sort_pairs<uint32_t>(dest.p, perm.p, t.nrows, 0, std::max(1, bits_for(nparts - 1)), c.s);
  std::vector<unsigned long long> hh(nparts);
  DAS_HIP(hipMemcpyAsync(hh.data(), h.p, 8 * nparts, hipMemcpyDeviceToHost, c.s));
  DAS_HIP(hipStreamSynchronize(c.s));
  for (uint32_t d = 0; d < nparts; ++d) counts[d] = hh[d];
  auto out = gather_table(c, t, perm.p, t.nrows);
  out->sorted_col = -1;
  return out;
}

void export_rows(Ctx& c, const Table& t, uint32_t* dst) {
  if (!t.nrows || !t.ncols) return;
  hipLaunchKernelGGL(k_rows_out, G(t.nrows), dim3(B), 0, c.s, cols_of(t), t.nrows, dst);
  DAS_HIP(hipGetLastError());
}

std::unique_ptr<Table> import_rows(Ctx& c, int kind, int ncols, const int32_t* vars, const int32_t* member,
                                   const uint32_t* src, uint64_t n) {
  auto t = new_table(c, kind, ncols, vars, n, member);
  t->nrows = n;
  if (n && ncols) {
    hipLaunchKernelGGL(k_rows_in, G(n), dim3(B), 0, c.s, src, n, ncols, t->data, t->cap);
    DAS_HIP(hipGetLastError());
  }
  return t;
}

std::unique_ptr<Table> concat(Ctx& c, const Table* const* ts, int n) {
  DAS_CHECK(n >= 1, DAS_E_INVALID, "concat of nothing");
  const Table& f = *ts[0];
  uint64_t total = 0;
  for (int i = 0; i < n; ++i) {
    DAS_CHECK(ts[i]->kind == f.kind && ts[i]->ncols == f.ncols, DAS_E_INVALID, "concat: schema mismatch");
    for (int k = 0; k < f.ncols; ++k)
      DAS_CHECK(ts[i]->vars[k] == f.vars[k] && ts[i]->member[k] == f.member[k], DAS_E_INVALID, "concat: schema mismatch");
    total += ts[i]->nrows;
  }
  auto t = new_table_like(c, f, total);
  t->nrows = total;
  if (n > 1) t->sorted_col = -1;
  for (int i = 1; i < n; ++i)
    for (int k = 0; k < f.ncols; ++k) {
      t->lo[k] = std::min(t->lo[k], ts[i]->lo[k]);
      t->hi[k] = std::max(t->hi[k], ts[i]->hi[k]);
    }
  uint64_t o = 0;
  for (int i = 0; i < n; ++i) {
    for (int k = 0; k < f.ncols; ++k)
      if (ts[i]->nrows)
        copy_dev(t->col(k) + o, ts[i]->col(k), 4 * ts[i]->nrows, c.s);
    o += ts[i]->nrows;
  }
  return t;
}

}  // namespace das
