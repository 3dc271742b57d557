// Shared host/device plumbing for the DAS MI355X library (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "status.h"

namespace das {

constexpr int kWave = 64;          // CDNA wavefront width

#define DAS_HIP(expr)                                                            \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess)                                                          \
      throw ::das::Error(::das::DAS_E_HIP, std::string(#expr) + ": " +             \
                                               hipGetErrorString(_e) + " at " +    \
                                               __FILE__ + ":" + std::to_string(__LINE__)); \
  } while (0)

inline unsigned grid_for(uint64_t n, unsigned block, unsigned cap = 65535u * 8u) {
  uint64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// Caching allocator (alloc.hip): blocks reused per (stream, size class).
void* cache_alloc(size_t bytes, hipStream_t s);
void cache_free(void* p);
void cache_release_stream(hipStream_t s);
void cache_trim();
// idle blocks returned to the driver, smallest first, until at most `keep` bytes stay cached
void cache_trim_to(size_t keep);
                       // returns every idle cached block to the driver
void cache_hold(bool on);                 // nested: while held, freed blocks stay cached (no budget)

// Stream-ordered device buffer from the caching allocator (ctx stream).
template <typename T>
struct DBuf {
  T* p = nullptr;
  uint64_t n = 0;
  hipStream_t s = nullptr;
  DBuf() = default;
  DBuf(uint64_t count, hipStream_t st) { alloc(count, st); }
  void alloc(uint64_t count, hipStream_t st) {
    release();
    s = st;
    n = count;
    if (count) p = (T*)cache_alloc(sizeof(T) * count, st);
  }
  void release() {
    if (p) cache_free(p);
    p = nullptr;
    n = 0;
  }
  T* release_ownership() {
    T* q = p;
    p = nullptr;
    n = 0;
    return q;
  }
  ~DBuf() { release(); }
  DBuf(const DBuf&) = delete;
  DBuf& operator=(const DBuf&) = delete;
  DBuf(DBuf&& o) noexcept { *this = std::move(o); }
  DBuf& operator=(DBuf&& o) noexcept {
    if (this != &o) {
      release();
      p = o.p; n = o.n; s = o.s;
      o.p = nullptr; o.n = 0;
    }
    return *this;
  }
  uint64_t bytes() const { return sizeof(T) * n; }
};

// Pinned host scratch for small D2H reads that the planner needs (row counts).
struct HostScalar {
  uint64_t* h = nullptr;
  HostScalar() { DAS_HIP(hipHostMalloc((void**)&h, sizeof(uint64_t) * 64, hipHostMallocDefault)); }
  ~HostScalar() { if (h) (void)hipHostFree(h); }
};

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// A 128-bit MD5 digest, stored as the four little-endian state words a..d
// (byte i of the digest is byte (i&3) of word i>>2).  `hi()/lo()` give the
// big-endian 64-bit halves, so (hi, lo) order == lexicographic order of the
// 32-char hex handle (the order Python's sorted() gives handles).
struct Digest {
  uint32_t w[4];
  __host__ __device__ uint64_t hi() const {
    return ((uint64_t)__builtin_bswap32(w[0]) << 32) | __builtin_bswap32(w[1]);
  }
  __host__ __device__ uint64_t lo() const {
    return ((uint64_t)__builtin_bswap32(w[2]) << 32) | __builtin_bswap32(w[3]);
  }
};
// A digest table with an element stride: 1 = a plain Digest[]; 2 = one half
// of the build's interleaved {digest, composite digest} records, so a random
// gather of both (a child's two digests in the hash pass, an atom's in
// k_fill_atoms) touches one 64-byte line instead of two.
struct DigS {
  Digest* p;
  uint32_t st;
  __host__ __device__ Digest& operator[](uint64_t i) const { return p[i * st]; }
};
inline DigS dig_s(const Digest* p, uint32_t st = 1) { return DigS{const_cast<Digest*>(p), st}; }

// Shard that owns a handle when links are hash-partitioned by handle across
// `world` GPUs: the handle's first 8 hex characters as a
// number (int(handle[:8], 16), the digest's first four bytes big-endian), mod
// world.  Every copy of one expression has one digest, so exactly one shard
// indexes it.
__host__ __device__ inline uint32_t handle_owner(const Digest& d, uint32_t world) {
  return world > 1 ? __builtin_bswap32(d.w[0]) % world : 0u;
}

}  // namespace das
