// Device primitives shared by the index build and the query kernels:
// exclusive scan, stable LSD radix sort (pairs), gather/iota/compaction.
// All launches go on the caller's stream; nothing here synchronises except
// the explicit `read_scalar` helper.
#pragma once
#include <functional>
#include "common.h"

namespace das {

// ---------------------------------------------------------------------------
// Exclusive scan (wave-level shuffles, 2048 items per 256-thread block)
// ---------------------------------------------------------------------------
// Timing scope for one kernel launch below the context layer (sorts, scans,
// index build kernels): HIP events on the stream of the context whose C-ABI
// call is running on this thread, when its profiling is on (das_prof_*).
// Names follow ProfScope's convention (das_internal.h).
struct KScope {
  void* impl = nullptr;
  KScope(const char* name, double algorithmic_bytes);
  ~KScope();
  KScope(const KScope&) = delete;
  KScope& operator=(const KScope&) = delete;
};
template <typename K> constexpr const char* key_tag();
template <> constexpr const char* key_tag<uint32_t>() { return "u32"; }
template <> constexpr const char* key_tag<uint64_t>() { return "u64"; }

constexpr int kScanBlock = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanBlock * kScanItems;

// 32-bit wave scans on DPP lane moves (row_shr 1/2/4/8 inside 16-lane rows,
// then row_bcast 15/31 across rows): VALU-latency steps instead of
// ds_bpermute round trips.  Invalid source lanes read 0, the identity of
// both sum and unsigned max.
#define DAS_DPP(x, ctrl, rmask) \
  ((uint32_t)__builtin_amdgcn_update_dpp(0, (int)(x), (ctrl), (rmask), 0xf, false))

__device__ __forceinline__ uint32_t wave_incl_sum_u32(uint32_t x) {
  x += DAS_DPP(x, 0x111, 0xf);
  x += DAS_DPP(x, 0x112, 0xf);
  x += DAS_DPP(x, 0x114, 0xf);
  x += DAS_DPP(x, 0x118, 0xf);
  x += DAS_DPP(x, 0x142, 0xa);
  x += DAS_DPP(x, 0x143, 0xc);
  return x;
}

__device__ __forceinline__ uint32_t wave_incl_max_u32(uint32_t x) {
  x = max(x, DAS_DPP(x, 0x111, 0xf));
  x = max(x, DAS_DPP(x, 0x112, 0xf));
  x = max(x, DAS_DPP(x, 0x114, 0xf));
  x = max(x, DAS_DPP(x, 0x118, 0xf));
  x = max(x, DAS_DPP(x, 0x142, 0xa));
  x = max(x, DAS_DPP(x, 0x143, 0xc));
  return x;
}

template <typename T>
__device__ __forceinline__ T wave_inclusive_scan(T x) {
  if constexpr (sizeof(T) == 4) {
    return (T)wave_incl_sum_u32((uint32_t)x);
  } else {
    const int lane = __lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      T y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    return x;
  }
}

// One atomicAdd per lane on base[slot]; lanes sharing the first active lane's
// slot are merged into a single atomic (Zipf hubs put many equal keys in one
// wave).  Returns the lane's pre-increment value.  Call wave-uniformly.
__device__ __forceinline__ uint32_t wave_agg_atomic_inc(uint32_t* base, uint32_t slot, bool active) {
  const uint64_t act = __ballot(active);
  if (!act) return 0;
  const int lane = __lane_id();
  const int leader = __ffsll((unsigned long long)act) - 1;
  const uint32_t ls = __shfl(slot, leader, 64);
  const bool same = active && slot == ls;
  const uint64_t m = __ballot(same);
  uint32_t b = 0;
  if (lane == leader) b = atomicAdd(&base[ls], (uint32_t)__popcll(m));
  b = __shfl(b, leader, 64);
  if (same) return b + (uint32_t)__popcll(m & ((1ull << lane) - 1));
  return active ? atomicAdd(&base[slot], 1u) : 0u;
}

template <typename T>
__device__ __forceinline__ T wave_reduce_sum(T x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

// Per-tile sums.
template <typename T, typename In>
__global__ void __launch_bounds__(kScanBlock) k_scan_reduce(In in, uint64_t n, T* tile_sums) {
  __shared__ T s[kScanBlock / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  T acc = 0;
#pragma unroll
  for (int r = 0; r < kScanItems; ++r) {
    uint64_t i = base + (uint64_t)r * kScanBlock + threadIdx.x;
    if (i < n) acc += (T)in(i);
  }
  acc = wave_reduce_sum(acc);
  if (__lane_id() == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    T t = 0;
    for (int w = 0; w < kScanBlock / 64; ++w) t += s[w];
    tile_sums[blockIdx.x] = t;
  }
}

// Scan each tile with its (already scanned) tile offset.
template <typename T, typename In>
__global__ void __launch_bounds__(kScanBlock) k_scan_tiles(In in, uint64_t n, const T* tile_off, T* out) {
  constexpr int W = kScanBlock / 64;
  __shared__ T s_wave[kScanItems][W];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  const int wave = threadIdx.x >> 6;
  // every round's input loaded up front (one round trip, not one per round),
  // then all wave scans, one barrier, and the stores
  T x[kScanItems], inc[kScanItems];
#pragma unroll
  for (int r = 0; r < kScanItems; ++r) {
    const uint64_t i = base + (uint64_t)r * kScanBlock + threadIdx.x;
    x[r] = (i < n) ? (T)in(i) : (T)0;
  }
#pragma unroll
  for (int r = 0; r < kScanItems; ++r) {
    inc[r] = wave_inclusive_scan(x[r]);
    if (__lane_id() == 63) s_wave[r][wave] = inc[r];
  }
  __syncthreads();
  T carry = tile_off ? tile_off[blockIdx.x] : (T)0;
#pragma unroll
  for (int r = 0; r < kScanItems; ++r) {
    T pre = carry, all = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      pre += w < wave ? s_wave[r][w] : (T)0;
      all += s_wave[r][w];
    }
    const uint64_t i = base + (uint64_t)r * kScanBlock + threadIdx.x;
    if (i < n) out[i] = pre + inc[r] - x[r];
    carry += all;
  }
}

template <typename T>
struct PtrIn {
  const T* p;
  __device__ __forceinline__ T operator()(uint64_t i) const { return p[i]; }
  static std::string name() { return std::string("PtrIn<") + key_tag<T>() + ">"; }
};

// out[i] = sum_{j<i} in(j).  Returns nothing; total = out[n-1] + in(n-1).
template <typename T, typename In>
void exclusive_scan_fn(In in, uint64_t n, T* out, hipStream_t s) {
  if (n == 0) return;
  uint64_t tiles = (n + kScanTile - 1) / kScanTile;
  const std::string targs = std::string("<") + key_tag<T>() + "," + In::name() + ">";
  if (tiles == 1) {
    KScope ks(("k_scan_tiles" + targs).c_str(), 2.0 * sizeof(T) * n);
    hipLaunchKernelGGL((k_scan_tiles<T, In>), dim3(1), dim3(kScanBlock), 0, s, in, n, (const T*)nullptr, out);
    DAS_HIP(hipGetLastError());
    return;
  }
  DBuf<T> sums(tiles, s), offs(tiles, s);
  {
    KScope ks(("k_scan_reduce" + targs).c_str(), (double)sizeof(T) * n);
    hipLaunchKernelGGL((k_scan_reduce<T, In>), dim3((unsigned)tiles), dim3(kScanBlock), 0, s, in, n, sums.p);
  }
  DAS_HIP(hipGetLastError());
  exclusive_scan_fn<T>(PtrIn<T>{sums.p}, tiles, offs.p, s);
  KScope ks(("k_scan_tiles" + targs).c_str(), 2.0 * sizeof(T) * n);
  hipLaunchKernelGGL((k_scan_tiles<T, In>), dim3((unsigned)tiles), dim3(kScanBlock), 0, s, in, n,
                     (const T*)offs.p, out);
  DAS_HIP(hipGetLastError());
}

template <typename T>
void exclusive_scan(const T* in, uint64_t n, T* out, hipStream_t s) {
  exclusive_scan_fn<T>(PtrIn<T>{in}, n, out, s);
}

// ---------------------------------------------------------------------------
// Exclusive scan whose total reaches the host without extra launches.
// `scan_total` writes out[0..n] (out[n] = total) and returns {total, max of
// in()}: the reduce pass's last block to finish (an acq_rel ticket on a
// per-stream counter) scans the tile sums in place and publishes total and
// max straight into the pinned read-back slot, then the tile pass runs while
// the host spins.  Two launches and one round trip per count -> size step,
// where scan + copy + publish took five.
// ---------------------------------------------------------------------------
struct PubSlot {
  uint32_t* p;      // pinned, coherent host words 0..15 (15 = sequence)
  uint32_t seq;
};
PubSlot pub_reserve();
void pub_wait(const PubSlot& ps, hipStream_t s, uint32_t* out, uint32_t n);
// Host work to do while a read-back is outstanding: a pub_wait of this
// thread whose slot is not yet written calls the hook with a predicate "the
// slot is written" before it spins; the hook does work in pieces while the
// predicate is false and returns true once it has none left (it is then
// cleared) -- das_plan_execute_many compiles and launches its chains in the
// gaps where a synchronous plan waits for a size.  nullptr: none.
using WaitHook = std::function<bool(const std::function<bool()>& ready)>;
void set_wait_hook(WaitHook* hook);
// algorithmic bytes of the kernel scopes launched since this thread's last
// read-back wait ended: how long the wait now starting can be expected to be
double bytes_since_wait();
// While alive: pub_reserve / pinned_stage hand out this thread's second slot
// and staging buffer (a plan run inside another plan's read-back wait)
int pub_level();                 // 0, or 1 inside a PubLevel
struct PubLevel {
  PubLevel();
  ~PubLevel();
  PubLevel(const PubLevel&) = delete;
  PubLevel& operator=(const PubLevel&) = delete;
};
// Pinned, device-mapped staging memory for small request / reply calls
// (handle lookups, index key ranges): the host writes the request, one
// kernel reads it over the mapping and writes its reply back with
// system-scope stores before releasing a PubSlot; the host spins on the
// slot.  One launch per call, no runtime copies and no stream wait.  The
// buffer is this thread's, reused by its next call.
uint8_t* pinned_stage(uint64_t bytes);
// Read-back slot and staging buffer number k (k < kPubPool) of this thread,
// apart from the ones above: for launches in flight together whose read-backs
// are taken later (das_plan_execute_many's deferred chains)
constexpr uint32_t kPubPool = 16;
PubSlot pub_reserve_pool(uint32_t k);
uint8_t* pinned_stage_pool(uint32_t k, uint64_t bytes);
// Per-(device, stream) completion counter of the reduce pass; `base` = its
// value before the next launch (the host advances it by the launch's tiles).
struct ScanCtr {
  unsigned long long* p;
  uint64_t base;
};
ScanCtr& scan_ctr(hipStream_t s);

// Called by every thread of one block: lanes < n store w[lane], then the
// sequence number is released (system scope) after them.
__device__ __forceinline__ void pub_store(uint32_t* slot, uint32_t seq, const uint32_t* w, int n) {
  if ((int)threadIdx.x < n) __hip_atomic_store(&slot[threadIdx.x], w[threadIdx.x], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_SYSTEM);
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(&slot[15], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename T>
__device__ __forceinline__ void block_sum_max(T& sum, uint64_t& mx, T* s_sum, uint64_t* s_mx) {
  sum = wave_reduce_sum(sum);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) { const uint64_t o = __shfl_xor(mx, d, 64); mx = o > mx ? o : mx; }
  if (__lane_id() == 0) { s_sum[threadIdx.x >> 6] = sum; s_mx[threadIdx.x >> 6] = mx; }
  __syncthreads();
  sum = 0;
  mx = 0;
  for (int w = 0; w < kScanBlock / 64; ++w) { sum += s_sum[w]; mx = s_mx[w] > mx ? s_mx[w] : mx; }
  __syncthreads();
}

// One block scans rows [0, n) of `in` into out (block loop with carry),
// accumulating the max; used for n <= one tile and for the tile sums.  Each
// round takes kScanPre consecutive rows per thread, all loaded before the
// round's scan: one memory latency per 4096 rows instead of one per 256 (the
// last-block scans of the count / reduce kernels sit in a query's latency
// chain).  In place (out == in's array) is fine: a thread writes only the rows
// it loaded, after the round's loads.
constexpr int kScanPre = 16;
template <typename T, typename In>
__device__ __forceinline__ void block_scan_loop(In in, uint64_t n, T* out, T& total, uint64_t& mx, T* s_wave,
                                                uint64_t* s_mx) {
  const int wave = threadIdx.x >> 6;
  T carry = 0;
  uint64_t m = 0;
  for (uint64_t base = 0; base < n; base += (uint64_t)kScanBlock * kScanPre) {
    const uint64_t i0 = base + (uint64_t)threadIdx.x * kScanPre;
    T x[kScanPre];
#pragma unroll
    for (int k = 0; k < kScanPre; ++k) x[k] = i0 + k < n ? (T)in(i0 + k) : (T)0;
    T sum = 0;
#pragma unroll
    for (int k = 0; k < kScanPre; ++k) {
      m = (uint64_t)x[k] > m ? (uint64_t)x[k] : m;
      sum += x[k];
    }
    const T inc = wave_inclusive_scan(sum);
    if (__lane_id() == 63) s_wave[wave] = inc;
    __syncthreads();
    T pre = carry + inc - sum;
    for (int w = 0; w < wave; ++w) pre += s_wave[w];
    for (int w = 0; w < kScanBlock / 64; ++w) carry += s_wave[w];
#pragma unroll
    for (int k = 0; k < kScanPre; ++k) {
      if (i0 + k < n) out[i0 + k] = pre;
      pre += x[k];
    }
    __syncthreads();
  }
  T dummy = 0;
  block_sum_max(dummy, m, s_wave, s_mx);
  total = carry;
  mx = m;
}

template <typename T, typename In>
__global__ void __launch_bounds__(kScanBlock) k_scan_single_pub(In in, uint64_t n, T* out, uint32_t* slot,
                                                               uint32_t seq) {
  __shared__ T s_wave[kScanBlock / 64];
  __shared__ uint64_t s_mx[kScanBlock / 64];
  T total;
  uint64_t mx;
  block_scan_loop<T>(in, n, out, total, mx, s_wave, s_mx);
  if (threadIdx.x == 0) out[n] = total;
  const uint64_t t64 = (uint64_t)total;
  const uint32_t w[4] = {(uint32_t)t64, (uint32_t)(t64 >> 32), (uint32_t)mx, (uint32_t)(mx >> 32)};
  pub_store(slot, seq, w, 4);
}

template <typename T>
struct SpanIn {
  const T* p;
  __device__ __forceinline__ T operator()(uint64_t i) const { return p[i]; }
};

template <typename T, typename In>
__global__ void __launch_bounds__(kScanBlock) k_scan_reduce_pub(In in, uint64_t n, T* tsum, uint64_t* tmax,
                                                               uint64_t tiles, unsigned long long* ctr,
                                                               unsigned long long last, T* out, uint32_t* slot,
                                                               uint32_t seq) {
  __shared__ T s_sum[kScanBlock / 64];
  __shared__ uint64_t s_mx[kScanBlock / 64];
  __shared__ int s_last;
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  T acc = 0;
  uint64_t m = 0;
#pragma unroll
  for (int r = 0; r < kScanItems; ++r) {
    const uint64_t i = base + (uint64_t)r * kScanBlock + threadIdx.x;
    if (i < n) {
      const T x = (T)in(i);
      acc += x;
      m = (uint64_t)x > m ? (uint64_t)x : m;
    }
  }
  block_sum_max(acc, m, s_sum, s_mx);
  if (threadIdx.x == 0) {
    // the tile's sum and max written through to the coherence point (agent
    // scope atomic stores), drained, then the arrival: no agent-scope
    // release per block (on gfx950 each one writes this XCD's L2 back)
    __hip_atomic_store(&tsum[blockIdx.x], acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&tmax[blockIdx.x], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t = __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = t == last;
  }
  __syncthreads();
  if (!s_last) return;
  // the last block: an agent-scope acquire (this XCD's stale lines of the
  // other tiles' sums invalidated), then plain reads
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  T total;
  uint64_t mx;
  block_scan_loop<T>(SpanIn<T>{tsum}, tiles, tsum, total, mx, s_sum, s_mx);   // in place, element-wise
  uint64_t mx2 = 0;
  for (uint64_t i = threadIdx.x; i < tiles; i += kScanBlock) mx2 = tmax[i] > mx2 ? tmax[i] : mx2;
  T dummy = 0;
  block_sum_max(dummy, mx2, s_sum, s_mx);
  if (threadIdx.x == 0) out[n] = total;
  const uint64_t t64 = (uint64_t)total;
  const uint32_t w[4] = {(uint32_t)t64, (uint32_t)(t64 >> 32), (uint32_t)mx2, (uint32_t)(mx2 >> 32)};
  pub_store(slot, seq, w, 4);
}

template <typename In>
struct Bounded {
  In in;
  uint64_t n;
  __device__ __forceinline__ auto operator()(uint64_t i) const -> decltype(in(i)) { return i < n ? in(i) : 0; }
};

template <typename T, typename In>
__global__ void k_max_of(In in, uint64_t n, unsigned long long* mx) {
  uint64_t m = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    m = (uint64_t)in(i) > m ? (uint64_t)in(i) : m;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) { const uint64_t o = __shfl_xor(m, d, 64); m = o > m ? o : m; }
  if (__lane_id() == 0 && m) atomicMax(mx, (unsigned long long)m);
}

constexpr uint64_t kPubMaxTiles = 1024;   // tile sums the last block scans alone (4 block rounds)

// Per-tile sum and max (the multi-level path of scan_total).
template <typename T, typename In>
__global__ void __launch_bounds__(kScanBlock) k_scan_reduce_mx(In in, uint64_t n, T* tsum, uint64_t* tmax) {
  __shared__ T s_sum[kScanBlock / 64];
  __shared__ uint64_t s_mx[kScanBlock / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  T acc = 0;
  uint64_t m = 0;
#pragma unroll
  for (int r = 0; r < kScanItems; ++r) {
    const uint64_t i = base + (uint64_t)r * kScanBlock + threadIdx.x;
    if (i < n) {
      const T x = (T)in(i);
      acc += x;
      m = (uint64_t)x > m ? (uint64_t)x : m;
    }
  }
  block_sum_max(acc, m, s_sum, s_mx);
  if (threadIdx.x == 0) {
    tsum[blockIdx.x] = acc;
    tmax[blockIdx.x] = m;
  }
}

// Device-to-device copy of `bytes` (a multiple of 4) as a kernel: the
// runtime's copy path costs far more host time per call than a launch.
__global__ void k_copy_u32(uint32_t* dst, const uint32_t* src, uint64_t n);
__global__ void k_copy_u128(uint4* dst, const uint4* src, uint64_t n);
inline void copy_dev(void* dst, const void* src, uint64_t bytes, hipStream_t s) {
  if (!bytes) return;
  const bool wide = ((((uintptr_t)dst) | ((uintptr_t)src) | bytes) & 15) == 0;
  KScope ks(wide ? "k_copy_u128" : "k_copy_u32", 2.0 * bytes);
  if (wide) {
    const uint64_t n = bytes / 16;
    hipLaunchKernelGGL(k_copy_u128, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, (uint4*)dst, (const uint4*)src, n);
  } else {
    const uint64_t n = bytes / 4;
    hipLaunchKernelGGL(k_copy_u32, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, (uint32_t*)dst,
                       (const uint32_t*)src, n);
  }
  DAS_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Stable LSD radix sort of (key, u32 value) pairs, 8-bit digits.
// Upsweep: per-tile LDS histogram -> digit-major table -> exclusive scan.
// Downsweep: per 256-key round, lanes with equal digits are matched with
// 8 wave ballots (rank = popcount of lower peers), waves are prefixed through
// LDS, so the scatter keeps input order inside each digit (stable).
// ---------------------------------------------------------------------------
constexpr int kSortBlock = 256;
constexpr int kSortItems = 16;
constexpr int kSortTile = kSortBlock * kSortItems;

template <typename K>
__global__ void __launch_bounds__(kSortBlock) k_radix_hist(const K* keys, uint64_t n, int shift,
                                                          uint32_t* hist, uint32_t n_tiles) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
#pragma unroll 4
  for (int r = 0; r < kSortItems; ++r) {
    uint64_t i = base + (uint64_t)r * kSortBlock + threadIdx.x;
    if (i < n) atomicAdd(&h[(uint32_t)(keys[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[(uint64_t)threadIdx.x * n_tiles + blockIdx.x] = h[threadIdx.x];
}

template <typename K, bool kHasVals>
__global__ void __launch_bounds__(kSortBlock) k_radix_scatter(const K* kin, const uint32_t* vin, K* kout,
                                                             uint32_t* vout, uint64_t n, int shift,
                                                             const uint32_t* offs, uint32_t n_tiles) {
  __shared__ uint32_t s_base[256];
  __shared__ uint32_t s_cnt[kSortBlock / 64][256];
  const int tid = threadIdx.x, wave = tid >> 6;
  s_base[tid] = offs[(uint64_t)tid * n_tiles + blockIdx.x];
#pragma unroll
  for (int w = 0; w < kSortBlock / 64; ++w) s_cnt[w][tid] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
  const uint64_t lt = __lanemask_lt();
  for (int r = 0; r < kSortItems; ++r) {
    const uint64_t i = base + (uint64_t)r * kSortBlock + tid;
    const bool valid = i < n;
    K k = valid ? kin[i] : (K)0;
    uint32_t v = 0;
    if (kHasVals && valid) v = vin[i];
    const uint32_t d = (uint32_t)(k >> shift) & 255u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bb = __ballot(bit);
      peers &= bit ? bb : ~bb;
    }
    const uint32_t rank = __popcll(peers & lt);
    if (valid && rank == 0) s_cnt[wave][d] = __popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pos = s_base[d] + rank;
      for (int w = 0; w < wave; ++w) pos += s_cnt[w][d];
      kout[pos] = k;
      if (kHasVals) vout[pos] = v;
    }
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (int w = 0; w < kSortBlock / 64; ++w) {
      add += s_cnt[w][tid];
      s_cnt[w][tid] = 0;
    }
    s_base[tid] += add;
    __syncthreads();
  }
}

// LDS-staged scatter: the tile's keys are first placed in LDS in digit order
// (tile-local offsets from the tile's histogram), then written out by
// consecutive threads, so each digit's run of the tile (~16 keys at 256
// digits) leaves as one contiguous store instead of 64 lanes hitting up to
// 64 buckets per wave store.  Values follow in a second phase through the
// SAME LDS buffer (each item's tile position and each output slot's global
// position stay in registers), so a block holds one tile of keys, not keys
// plus values: twice the resident blocks for 64-bit keys.  Same stable order
// as k_radix_scatter.
template <typename K, bool kHasVals>
__global__ void __launch_bounds__(kSortBlock) k_radix_scatter_lds(const K* kin, const uint32_t* vin, K* kout,
                                                                 uint32_t* vout, uint64_t n, int shift,
                                                                 const uint32_t* hist, const uint32_t* offs,
                                                                 uint32_t n_tiles) {
  __shared__ K s_key[kSortTile];
  __shared__ uint32_t s_gbase[256], s_loff[256], s_run[256];
  __shared__ uint32_t s_cnt[kSortBlock / 64][256];
  __shared__ uint32_t s_wsum[kSortBlock / 64];
  const int tid = threadIdx.x, wave = tid >> 6;
  const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
  // keys (and values) of all rounds loaded up front
  K kr[kSortItems];
  uint32_t vr[kHasVals ? kSortItems : 1];
#pragma unroll
  for (int r = 0; r < kSortItems; ++r) {
    const uint64_t i = base + (uint64_t)r * kSortBlock + tid;
    kr[r] = i < n ? kin[i] : (K)0;
    if (kHasVals) vr[r] = i < n ? vin[i] : 0u;
  }
  {
    // tile-local exclusive offset of each digit (thread = digit)
    const uint32_t c = hist[(uint64_t)tid * n_tiles + blockIdx.x];
    const uint32_t inc = wave_incl_sum_u32(c);
    if (__lane_id() == 63) s_wsum[wave] = inc;
    s_gbase[tid] = offs[(uint64_t)tid * n_tiles + blockIdx.x];
    s_run[tid] = 0;
#pragma unroll
    for (int w = 0; w < kSortBlock / 64; ++w) s_cnt[w][tid] = 0;
    __syncthreads();
    uint32_t pre = inc - c;
    for (int w = 0; w < wave; ++w) pre += s_wsum[w];
    s_loff[tid] = pre;
    __syncthreads();
  }
  const uint64_t lt = __lanemask_lt();
  uint32_t lpos[kHasVals ? kSortItems : 1];             // tile position of this thread's item r
#pragma unroll
  for (int r = 0; r < kSortItems; ++r) {
    const uint64_t i = base + (uint64_t)r * kSortBlock + tid;
    const bool valid = i < n;
    const uint32_t d = (uint32_t)(kr[r] >> shift) & 255u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bb = __ballot(bit);
      peers &= bit ? bb : ~bb;
    }
    const uint32_t rank = __popcll(peers & lt);
    if (valid && rank == 0) s_cnt[wave][d] = __popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pos = s_loff[d] + s_run[d] + rank;
      for (int w = 0; w < wave; ++w) pos += s_cnt[w][d];
      s_key[pos] = kr[r];
      if (kHasVals) lpos[r] = pos;
    }
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (int w = 0; w < kSortBlock / 64; ++w) {
      add += s_cnt[w][tid];
      s_cnt[w][tid] = 0;
    }
    s_run[tid] += add;
    __syncthreads();
  }
  const uint32_t valid_n = (uint32_t)(n - base < (uint64_t)kSortTile ? n - base : (uint64_t)kSortTile);
  uint32_t gpos[kHasVals ? kSortItems : 1];             // global slot of tile position tid + k * kSortBlock
#pragma unroll
  for (int k = 0; k < kSortItems; ++k) {
    const uint32_t j = (uint32_t)tid + (uint32_t)k * kSortBlock;
    if (j < valid_n) {
      const K key = s_key[j];
      const uint32_t d = (uint32_t)(key >> shift) & 255u;
      const uint32_t g = s_gbase[d] + (j - s_loff[d]);    // < n < 2^32
      kout[g] = key;
      if (kHasVals) gpos[k] = g;
    }
  }
  if (kHasVals) {
    uint32_t* s_val = reinterpret_cast<uint32_t*>(s_key);
    __syncthreads();                                   // every key read out of the buffer
#pragma unroll
    for (int r = 0; r < kSortItems; ++r)
      if (base + (uint64_t)r * kSortBlock + tid < n) s_val[lpos[r]] = vr[r];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSortItems; ++k) {
      const uint32_t j = (uint32_t)tid + (uint32_t)k * kSortBlock;
      if (j < valid_n) vout[gpos[k]] = s_val[j];
    }
  }
}

// ---------------------------------------------------------------------------
// Onesweep passes (large sorts): the digit histograms of EVERY pass come from
// one read of the keys up front (k_radix_ghist); each pass is then a single
// kernel -- a block takes the next tile in launch order (atomic ticket),
// counts its digits in LDS, publishes the counts, and derives its tile offset
// per digit by looking back over the earlier tiles' published counts
// (decoupled look-back: a tile's inclusive prefix once known, else its own
// count and the look-back continues).  No per-pass histogram kernel, no
// tiles x 256 scan.  Earlier tiles were ticketed by blocks already running,
// so every wait ends; a wait longer than kLookbackSpin rounds sets an error
// flag instead of spinning on (the caller raises).
// ---------------------------------------------------------------------------
constexpr uint64_t kLbAgg = 1ull << 62, kLbInc = 2ull << 62, kLbMask = (1ull << 62) - 1;
constexpr uint32_t kLookbackSpin = 1u << 24;

template <typename K>
__global__ void __launch_bounds__(kSortBlock) k_radix_ghist(const K* keys, uint64_t n, int shift0, int npass,
                                                           uint32_t* ghist) {
  __shared__ uint32_t h[8][256];
  for (int p = 0; p < npass; ++p) h[p][threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t i = blockIdx.x * (uint64_t)kSortBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kSortBlock) {
    const K k = keys[i];
    for (int p = 0; p < npass; ++p) atomicAdd(&h[p][(uint32_t)(k >> (shift0 + 8 * p)) & 255u], 1u);
  }
  __syncthreads();
  for (int p = 0; p < npass; ++p)
    if (h[p][threadIdx.x]) atomicAdd(&ghist[p * 256 + threadIdx.x], h[p][threadIdx.x]);
}

template <typename K, bool kHasVals>
__global__ void __launch_bounds__(kSortBlock) k_radix_onesweep(const K* kin, const uint32_t* vin, K* kout,
                                                              uint32_t* vout, uint64_t n, int shift,
                                                              const uint32_t* ghist, uint64_t* status,
                                                              uint32_t* ticket, uint32_t* err) {
  __shared__ K s_key[kSortTile];
  __shared__ uint32_t s_gbase[256], s_loff[256], s_run[256], s_hist[256];
  __shared__ uint32_t s_cnt[kSortBlock / 64][256];
  __shared__ uint32_t s_wsum[kSortBlock / 64];
  __shared__ uint32_t s_tile;
  const int tid = threadIdx.x, wave = tid >> 6;
  if (tid == 0) s_tile = atomicAdd(ticket, 1u);
  s_hist[tid] = 0;
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint64_t base = (uint64_t)tile * kSortTile;
  K kr[kSortItems];
  uint32_t vr[kHasVals ? kSortItems : 1];
#pragma unroll
  for (int r = 0; r < kSortItems; ++r) {
    const uint64_t i = base + (uint64_t)r * kSortBlock + tid;
    kr[r] = i < n ? kin[i] : (K)0;
    if (kHasVals) vr[r] = i < n ? vin[i] : 0u;
    if (i < n) atomicAdd(&s_hist[(uint32_t)(kr[r] >> shift) & 255u], 1u);
  }
  __syncthreads();
  {
    // publish this tile's count of digit `tid`, then look back for the
    // earlier tiles' total (thread = digit)
    const uint32_t c = s_hist[tid];
    uint64_t* st = status + (uint64_t)tile * 256 + tid;
    __hip_atomic_store(st, (tile == 0 ? kLbInc : kLbAgg) | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t pre = 0;
    for (int64_t j = (int64_t)tile - 1; j >= 0;) {
      const uint64_t v = __hip_atomic_load(status + (uint64_t)j * 256 + tid, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      if (v & kLbInc) { pre += v & kLbMask; break; }
      if (v & kLbAgg) { pre += v & kLbMask; --j; continue; }
      uint32_t spins = 0;                              // tile j not published yet
      while (!(__hip_atomic_load(status + (uint64_t)j * 256 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &
               (kLbInc | kLbAgg))) {
        if (++spins > kLookbackSpin) { atomicOr(err, 1u); j = -1; break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (tile) __hip_atomic_store(st, kLbInc | (pre + c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // global base of digit `tid` = all smaller digits + earlier tiles' count of it
    uint32_t g = ghist[tid];
    const uint32_t ginc = wave_incl_sum_u32(g);
    if (__lane_id() == 63) s_wsum[wave] = ginc;
    const uint32_t linc = wave_incl_sum_u32(c);
    __syncthreads();
    uint32_t gpre = ginc - g, lpre = linc - c;
    for (int w = 0; w < wave; ++w) gpre += s_wsum[w];
    __syncthreads();
    if (__lane_id() == 63) s_wsum[wave] = linc;
    __syncthreads();
    for (int w = 0; w < wave; ++w) lpre += s_wsum[w];
    s_gbase[tid] = gpre + (uint32_t)pre;
    s_loff[tid] = lpre;
    s_run[tid] = 0;
#pragma unroll
    for (int w = 0; w < kSortBlock / 64; ++w) s_cnt[w][tid] = 0;
    __syncthreads();
  }
  const uint64_t lt = __lanemask_lt();
  uint32_t lpos[kHasVals ? kSortItems : 1];
#pragma unroll
  for (int r = 0; r < kSortItems; ++r) {
    const uint64_t i = base + (uint64_t)r * kSortBlock + tid;
    const bool valid = i < n;
    const uint32_t d = (uint32_t)(kr[r] >> shift) & 255u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bb = __ballot(bit);
      peers &= bit ? bb : ~bb;
    }
    const uint32_t rank = __popcll(peers & lt);
    if (valid && rank == 0) s_cnt[wave][d] = __popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pos = s_loff[d] + s_run[d] + rank;
      for (int w = 0; w < wave; ++w) pos += s_cnt[w][d];
      s_key[pos] = kr[r];
      if (kHasVals) lpos[r] = pos;
    }
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (int w = 0; w < kSortBlock / 64; ++w) {
      add += s_cnt[w][tid];
      s_cnt[w][tid] = 0;
    }
    s_run[tid] += add;
    __syncthreads();
  }
  const uint32_t valid_n = (uint32_t)(n - base < (uint64_t)kSortTile ? n - base : (uint64_t)kSortTile);
  uint32_t gpos[kHasVals ? kSortItems : 1];
#pragma unroll
  for (int k = 0; k < kSortItems; ++k) {
    const uint32_t j = (uint32_t)tid + (uint32_t)k * kSortBlock;
    if (j < valid_n) {
      const K key = s_key[j];
      const uint32_t d = (uint32_t)(key >> shift) & 255u;
      const uint32_t g = s_gbase[d] + (j - s_loff[d]);
      kout[g] = key;
      if (kHasVals) gpos[k] = g;
    }
  }
  if (kHasVals) {
    uint32_t* s_val = reinterpret_cast<uint32_t*>(s_key);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortItems; ++r)
      if (base + (uint64_t)r * kSortBlock + tid < n) s_val[lpos[r]] = vr[r];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSortItems; ++k) {
      const uint32_t j = (uint32_t)tid + (uint32_t)k * kSortBlock;
      if (j < valid_n) vout[gpos[k]] = s_val[j];
    }
  }
}

uint32_t read_u32(const uint32_t* d, hipStream_t s);
inline void fill_dev(void* dst, int byte, uint64_t bytes, hipStream_t s);

// Sorts keys[0..n) (and vals alongside, if given) by bits [begin_bit, end_bit).
// Result lands back in keys/vals.
template <typename K>
void radix_sort_pairs(K* keys, uint32_t* vals, uint64_t n, int begin_bit, int end_bit, hipStream_t s) {
  if (n <= 1 || end_bit <= begin_bit) return;
  // DAS_ONESWEEP=1: onesweep passes (measured slower at 10^9 keys: each
  // digit's look-back walks earlier tiles one dependent load at a time, so the
  // per-pass histogram kernels stay the default)
  const char* os_env = std::getenv("DAS_ONESWEEP");
  const bool onesweep = os_env && os_env[0] == '1';
  if (onesweep && n >= (1ull << 20)) {
    DAS_CHECK(n < (1ull << 32), DAS_E_UNSUPPORTED, "radix sort: more than 2^32 keys");
    const uint32_t tiles = (uint32_t)((n + kSortTile - 1) / kSortTile);
    const int npass = (end_bit - begin_bit + 7) / 8;
    DBuf<K> k2(n, s);
    DBuf<uint32_t> v2(vals ? n : 0, s);
    DBuf<uint32_t> ghist(256 * (uint64_t)npass, s), ctl(2 * (uint64_t)npass + 1, s);
    DBuf<uint64_t> status((uint64_t)tiles * 256, s);
    fill_dev(ghist.p, 0, 4 * 256 * (uint64_t)npass, s);
    fill_dev(ctl.p, 0, 4 * (2 * (uint64_t)npass + 1), s);
    const std::string tag = key_tag<K>();
    {
      KScope ks(("k_radix_ghist<" + tag + ">").c_str(), (double)n * sizeof(K));
      hipLaunchKernelGGL((k_radix_ghist<K>), dim3(grid_for(n, kSortBlock, 2048)), dim3(kSortBlock), 0, s,
                         (const K*)keys, n, begin_bit, npass, ghist.p);
      DAS_HIP(hipGetLastError());
    }
    const double kv = (double)n * (sizeof(K) + (vals ? 4.0 : 0.0));
    K* ka = keys; K* kb = k2.p;
    uint32_t* va = vals; uint32_t* vb = v2.p;
    for (int p = 0; p < npass; ++p) {
      fill_dev(status.p, 0, 8 * (uint64_t)tiles * 256, s);
      KScope ks(("k_radix_onesweep<" + tag + (vals ? ",true>" : ",false>")).c_str(), 2.0 * kv);
      if (vals)
        hipLaunchKernelGGL((k_radix_onesweep<K, true>), dim3(tiles), dim3(kSortBlock), 0, s, (const K*)ka,
                           (const uint32_t*)va, kb, vb, n, begin_bit + 8 * p, (const uint32_t*)ghist.p + 256 * p,
                           status.p, ctl.p + p, ctl.p + 2 * npass);
      else
        hipLaunchKernelGGL((k_radix_onesweep<K, false>), dim3(tiles), dim3(kSortBlock), 0, s, (const K*)ka,
                           (const uint32_t*)nullptr, kb, (uint32_t*)nullptr, n, begin_bit + 8 * p,
                           (const uint32_t*)ghist.p + 256 * p, status.p, ctl.p + p, ctl.p + 2 * npass);
      DAS_HIP(hipGetLastError());
      std::swap(ka, kb);
      std::swap(va, vb);
    }
    if (npass & 1) {
      copy_dev(keys, ka, sizeof(K) * n, s);
      if (vals) copy_dev(vals, va, sizeof(uint32_t) * n, s);
    }
    DAS_CHECK(read_u32(ctl.p + 2 * npass, s) == 0, DAS_E_INTERNAL, "radix sort: look-back wait exceeded its bound");
    return;
  }
  DAS_CHECK(n < (1ull << 32), DAS_E_UNSUPPORTED, "radix sort: more than 2^32 keys");
  const uint32_t tiles = (uint32_t)((n + kSortTile - 1) / kSortTile);
  DBuf<K> k2(n, s);
  DBuf<uint32_t> v2(vals ? n : 0, s);
  DBuf<uint32_t> hist((uint64_t)tiles * 256, s), offs((uint64_t)tiles * 256, s);
  K* ka = keys; K* kb = k2.p;
  uint32_t* va = vals; uint32_t* vb = v2.p;
  int passes = 0;
  const std::string tag = key_tag<K>();
  const double kv = (double)n * (sizeof(K) + (vals ? 4.0 : 0.0));    // one pass: keys (+ values) in and out
  for (int shift = begin_bit; shift < end_bit; shift += 8, ++passes) {
    {
      KScope ks(("k_radix_hist<" + tag + ">").c_str(), (double)n * sizeof(K));
      hipLaunchKernelGGL((k_radix_hist<K>), dim3(tiles), dim3(kSortBlock), 0, s, (const K*)ka, n, shift, hist.p, tiles);
    }
    DAS_HIP(hipGetLastError());
    exclusive_scan<uint32_t>(hist.p, (uint64_t)tiles * 256, offs.p, s);
    static const bool lds = !(std::getenv("DAS_SORT_LDS") && std::getenv("DAS_SORT_LDS")[0] == '0');
    KScope ks(((lds ? "k_radix_scatter_lds<" : "k_radix_scatter<") + tag + (vals ? ",true>" : ",false>")).c_str(),
              2.0 * kv);
    if (lds && vals)
      hipLaunchKernelGGL((k_radix_scatter_lds<K, true>), dim3(tiles), dim3(kSortBlock), 0, s, (const K*)ka,
                         (const uint32_t*)va, kb, vb, n, shift, (const uint32_t*)hist.p, (const uint32_t*)offs.p,
                         tiles);
    else if (lds)
      hipLaunchKernelGGL((k_radix_scatter_lds<K, false>), dim3(tiles), dim3(kSortBlock), 0, s, (const K*)ka,
                         (const uint32_t*)nullptr, kb, (uint32_t*)nullptr, n, shift, (const uint32_t*)hist.p,
                         (const uint32_t*)offs.p, tiles);
    else if (vals)
      hipLaunchKernelGGL((k_radix_scatter<K, true>), dim3(tiles), dim3(kSortBlock), 0, s, (const K*)ka,
                         (const uint32_t*)va, kb, vb, n, shift, (const uint32_t*)offs.p, tiles);
    else
      hipLaunchKernelGGL((k_radix_scatter<K, false>), dim3(tiles), dim3(kSortBlock), 0, s, (const K*)ka,
                         (const uint32_t*)nullptr, kb, (uint32_t*)nullptr, n, shift, (const uint32_t*)offs.p, tiles);
    DAS_HIP(hipGetLastError());
    std::swap(ka, kb);
    std::swap(va, vb);
  }
  if (passes & 1) {
    copy_dev(keys, ka, sizeof(K) * n, s);
    if (vals) copy_dev(vals, va, sizeof(uint32_t) * n, s);
  }
}

inline int bits_for(uint64_t max_value) {
  int b = 0;
  while (b < 64 && (max_value >> b) != 0) ++b;
  return b;
}

// ---------------------------------------------------------------------------
// Small element-wise helpers
// ---------------------------------------------------------------------------
__global__ void k_iota(uint32_t* p, uint64_t n);
__global__ void k_gather_u32(const uint32_t* src, const uint32_t* idx, uint32_t* dst, uint64_t n);

inline void iota(uint32_t* p, uint64_t n, hipStream_t s) {
  if (!n) return;
  KScope ks("k_iota", 4.0 * n);
  hipLaunchKernelGGL(k_iota, dim3(grid_for(n, 256)), dim3(256), 0, s, p, n);
  DAS_HIP(hipGetLastError());
}
inline void gather_u32(const uint32_t* src, const uint32_t* idx, uint32_t* dst, uint64_t n, hipStream_t s) {
  if (!n) return;
  KScope ks("k_gather_u32", 12.0 * n);
  hipLaunchKernelGGL(k_gather_u32, dim3(grid_for(n, 256)), dim3(256), 0, s, src, idx, dst, n);
  DAS_HIP(hipGetLastError());
}

// hipMemsetAsync replacement (a multiple of 4 bytes, every byte = `byte`): the
// runtime's fill path also costs far more host time than a launch.
__global__ void k_fill_u32(uint32_t* dst, uint32_t v, uint64_t n);
inline void fill_dev(void* dst, int byte, uint64_t bytes, hipStream_t s) {
  if (!bytes) return;
  const uint32_t b = (uint32_t)(byte & 0xFF);
  const uint64_t n = bytes / 4;
  KScope ks("k_fill_u32", (double)bytes);
  hipLaunchKernelGGL(k_fill_u32, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, (uint32_t*)dst,
                     b | (b << 8) | (b << 16) | (b << 24), n);
  DAS_HIP(hipGetLastError());
}

// Reads one device u64 (or u32) back to the host through pinned memory;
// synchronises the stream.
uint64_t read_u64(const uint64_t* d, hipStream_t s);
uint32_t read_u32(const uint32_t* d, hipStream_t s);
void read_u64x2(const uint64_t* d, hipStream_t s, uint64_t out[2]);   // d[0], d[1] in one round trip
void read_u32x2(const uint32_t* d0, const uint32_t* d1, hipStream_t s, uint32_t out[2]);

template <typename T, typename In>
uint64_t scan_total(In in, uint64_t n, T* out, hipStream_t s, uint64_t* max_out = nullptr) {
  const uint64_t tiles = (n + kScanTile - 1) / kScanTile;
  uint32_t w[4];
  if (tiles <= 1) {
    const PubSlot ps = pub_reserve();
    hipLaunchKernelGGL((k_scan_single_pub<T, In>), dim3(1), dim3(kScanBlock), 0, s, in, n, out, ps.p, ps.seq);
    DAS_HIP(hipGetLastError());
    pub_wait(ps, s, w, 4);
  } else if (tiles <= kPubMaxTiles) {
    DBuf<T> tsum(tiles, s);
    DBuf<uint64_t> tmax(tiles, s);
    ScanCtr& ct = scan_ctr(s);
    const PubSlot ps = pub_reserve();
    hipLaunchKernelGGL((k_scan_reduce_pub<T, In>), dim3((unsigned)tiles), dim3(kScanBlock), 0, s, in, n, tsum.p,
                       tmax.p, tiles, ct.p, (unsigned long long)(ct.base + tiles - 1), out, ps.p, ps.seq);
    DAS_HIP(hipGetLastError());
    ct.base += tiles;
    hipLaunchKernelGGL((k_scan_tiles<T, In>), dim3((unsigned)tiles), dim3(kScanBlock), 0, s, in, n,
                       (const T*)tsum.p, out);
    DAS_HIP(hipGetLastError());
    pub_wait(ps, s, w, 4);
  } else {
    // multi-level: tile sums (and maxima), scanned by this function, then
    // the tile pass; the total reaches the host through the inner scan
    DBuf<T> tsum(tiles, s), toff(tiles + 1, s);
    DBuf<uint64_t> tmax(tiles, s);
    hipLaunchKernelGGL((k_scan_reduce_mx<T, In>), dim3((unsigned)tiles), dim3(kScanBlock), 0, s, in, n, tsum.p,
                       tmax.p);
    DAS_HIP(hipGetLastError());
    uint64_t mx = 0;
    const uint64_t total = scan_total<T>(SpanIn<T>{tsum.p}, tiles, toff.p, s, nullptr);
    hipLaunchKernelGGL((k_scan_tiles<T, In>), dim3((unsigned)tiles), dim3(kScanBlock), 0, s, in, n,
                       (const T*)toff.p, out);
    DAS_HIP(hipGetLastError());
    copy_dev(out + n, toff.p + tiles, sizeof(T), s);
    if (max_out) {
      DBuf<uint64_t> tm(tiles + 1, s);
      scan_total<uint64_t>(SpanIn<uint64_t>{tmax.p}, tiles, tm.p, s, &mx);
    }
    w[0] = (uint32_t)total; w[1] = (uint32_t)(total >> 32);
    w[2] = (uint32_t)mx; w[3] = (uint32_t)(mx >> 32);
  }
  if (max_out) *max_out = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  return (uint64_t)w[0] | ((uint64_t)w[1] << 32);
}

}  // namespace das
