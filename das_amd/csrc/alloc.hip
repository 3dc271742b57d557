// Caching device allocator for query-time buffers.
//
// Every table and scratch buffer of a query lives on its context's stream, so
// a freed block can be handed to the next allocation on the same stream with
// no fence: stream order already puts the new work after the old.  Blocks are
// kept per (stream, size class) and only returned to the driver when the
// context's stream is destroyed or the cache exceeds its budget, so a query
// step performs no runtime allocation calls once warm (the runtime's own
// stream-ordered allocator costs microseconds per call and, under a step's
// mix of sizes, occasionally hundreds of microseconds).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace das {

namespace {

struct Cache {
  std::mutex mu;
  std::map<std::pair<hipStream_t, size_t>, std::vector<void*>> free_blocks;
  std::unordered_map<void*, std::pair<hipStream_t, size_t>> live;
  size_t cached_bytes = 0;
};

Cache& cache() {
  static Cache* c = new Cache();   // never destroyed: frees may arrive during exit
  return *c;
}

constexpr size_t kCacheBudget = 64ull << 30;   // cached (idle) bytes kept at most
constexpr size_t kBestFitMin = 64ull << 20;     // best-fit reuse from this block size up
std::atomic<int> g_hold{0};                     // > 0: keep every freed block (cache_hold)

// DAS_ALLOC_TRACE=1: one stderr line per driver allocation (size, host ms)
// and per out-of-memory fallback, to attribute host gaps in large builds.
bool alloc_trace() {
  static const bool on = [] {
    const char* e = std::getenv("DAS_ALLOC_TRACE");
    return e && e[0] == '1';
  }();
  return on;
}

hipError_t traced_malloc(void** p, size_t bytes, const char* what) {
  if (!alloc_trace()) return hipMalloc(p, bytes);
  const auto t0 = std::chrono::steady_clock::now();
  const hipError_t e = hipMalloc(p, bytes);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  size_t fr = 0, tot = 0;
  (void)hipMemGetInfo(&fr, &tot);
  std::fprintf(stderr, "[das alloc] %s %.3f GB %.3f ms%s (free %.1f GB, cached %.1f GB)\n", what, bytes / 1e9, ms,
               e == hipSuccess ? "" : " FAILED", fr / 1e9, cache().cached_bytes / 1e9);
  return e;
}

size_t size_class(size_t bytes) {
  if (bytes <= 256) return 256;
  if (bytes <= (1u << 20)) {                     // powers of two up to 1 MiB
    size_t c = 512;
    while (c < bytes) c <<= 1;
    return c;
  }
  const size_t g = bytes <= (64ull << 20) ? (1ull << 20) : (16ull << 20);
  return (bytes + g - 1) / g * g;                // 1 MiB / 16 MiB granules above
}

}  // namespace

void* cache_alloc(size_t bytes, hipStream_t s) {
  if (!bytes) return nullptr;
  const size_t cls = size_class(bytes);
  Cache& c = cache();
  {
    std::lock_guard<std::mutex> lk(c.mu);
    // exact class; large requests also take the smallest idle block below
    // twice their size (a 10^9-link build frees and re-requests tens of GB
    // in shifting sizes: every block handed back to the driver is cleared
    // before it can be mapped again, a multi-second stall per allocation)
    const size_t top = cls >= kBestFitMin ? 2 * cls : cls + 1;
    for (auto it = c.free_blocks.lower_bound({s, cls});
         it != c.free_blocks.end() && it->first.first == s && it->first.second < top; ++it) {
      if (it->second.empty()) continue;
      void* p = it->second.back();
      it->second.pop_back();
      c.cached_bytes -= it->first.second;
      c.live[p] = it->first;
      return p;
    }
  }
  void* p = nullptr;
  hipError_t e = traced_malloc(&p, cls, "cache");
  if (e != hipSuccess) {
    // out of memory with idle blocks cached: give back the largest ones
    // until the request fits, keep the rest cached (every hipFree of a large
    // block costs milliseconds: freeing the whole cache at once stalled a
    // 10^9-link build for ~1.4 s, round 5)
    (void)hipGetLastError();
    std::vector<std::pair<std::pair<hipStream_t, size_t>, void*>> idle;
    {
      std::lock_guard<std::mutex> lk(c.mu);
      for (auto& kv : c.free_blocks)
        for (void* q : kv.second) idle.push_back({kv.first, q});
      c.free_blocks.clear();
      c.cached_bytes = 0;
    }
    std::sort(idle.begin(), idle.end(), [](const auto& x, const auto& y) { return x.first.second > y.first.second; });
    DAS_HIP(hipDeviceSynchronize());
    if (alloc_trace()) std::fprintf(stderr, "[das alloc] OOM fallback: %zu idle blocks\n", idle.size());
    size_t k = 0, freed = 0;
    p = nullptr;
    for (; k < idle.size() && !p; ++k) {
      (void)hipFree(idle[k].second);
      freed += idle[k].first.second;
      if (freed >= cls && hipMalloc(&p, cls) != hipSuccess) {
        (void)hipGetLastError();
        p = nullptr;
      }
    }
    {
      std::lock_guard<std::mutex> lk(c.mu);
      for (size_t r = k; r < idle.size(); ++r) {
        c.free_blocks[idle[r].first].push_back(idle[r].second);
        c.cached_bytes += idle[r].first.second;
      }
    }
    if (!p) DAS_HIP(traced_malloc(&p, cls, "cache-retry"));
  }
  std::lock_guard<std::mutex> lk(c.mu);
  c.live[p] = {s, cls};
  return p;
}

void cache_free(void* p) {
  if (!p) return;
  Cache& c = cache();
  void* drop = nullptr;
  {
    std::lock_guard<std::mutex> lk(c.mu);
    auto it = c.live.find(p);
    if (it == c.live.end()) return;
    const auto key = it->second;
    c.live.erase(it);
    if (c.cached_bytes + key.second > kCacheBudget && g_hold.load() == 0) {
      drop = p;
    } else {
      c.free_blocks[key].push_back(p);
      c.cached_bytes += key.second;
    }
  }
  if (drop) {
    const auto t0 = std::chrono::steady_clock::now();
    (void)hipDeviceSynchronize();   // the block may still be in use by queued work
    (void)hipFree(drop);
    if (alloc_trace())
      std::fprintf(stderr, "[das alloc] drop (over budget) %.3f ms\n",
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  }
}

void cache_hold(bool on) { g_hold += on ? 1 : -1; }

void cache_trim() {
  Cache& c = cache();
  std::vector<void*> idle;
  {
    std::lock_guard<std::mutex> lk(c.mu);
    for (auto& kv : c.free_blocks) idle.insert(idle.end(), kv.second.begin(), kv.second.end());
    c.free_blocks.clear();
    c.cached_bytes = 0;
  }
  if (idle.empty()) return;
  (void)hipDeviceSynchronize();   // idle blocks may still be read by queued work
  for (void* q : idle) (void)hipFree(q);
}

void cache_trim_to(size_t keep) {
  Cache& c = cache();
  std::vector<std::pair<size_t, std::pair<std::pair<hipStream_t, size_t>, void*>>> idle;
  std::vector<void*> drop;
  {
    std::lock_guard<std::mutex> lk(c.mu);
    if (c.cached_bytes <= keep) return;
    for (auto& kv : c.free_blocks)
      for (void* q : kv.second) idle.push_back({kv.first.second, {kv.first, q}});
    // the smallest go first: the large ones are what the next build re-requests
    std::sort(idle.begin(), idle.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
    size_t cached = c.cached_bytes;
    for (auto& it : idle) {
      if (cached <= keep) break;
      auto& v = c.free_blocks[it.second.first];
      for (size_t i = 0; i < v.size(); ++i)
        if (v[i] == it.second.second) {
          v[i] = v.back();
          v.pop_back();
          break;
        }
      cached -= it.first;
      drop.push_back(it.second.second);
    }
    c.cached_bytes = cached;
  }
  if (drop.empty()) return;
  (void)hipDeviceSynchronize();   // idle blocks may still be read by queued work
  for (void* q : drop) (void)hipFree(q);
}

void cache_release_stream(hipStream_t s) {
  Cache& c = cache();
  std::vector<void*> idle;
  {
    std::lock_guard<std::mutex> lk(c.mu);
    for (auto it = c.free_blocks.begin(); it != c.free_blocks.end();) {
      if (it->first.first == s) {
        for (void* p : it->second) {
          idle.push_back(p);
          c.cached_bytes -= it->first.second;
        }
        it = c.free_blocks.erase(it);
      } else {
        ++it;
      }
    }
  }
  for (void* p : idle) (void)hipFree(p);
}

}  // namespace das
