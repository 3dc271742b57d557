// Order-independent checksum of a binding table under the reference's
// assignment identity (pattern_matcher.py:41-51: an OrderedAssignment is its
// var -> handle mapping; PatternMatchingAnswer keeps a *set* of them,
// :370-384, 741-748).  Parity at BASELINE sizes compares this value with the
// same function computed from a generator's own arrays (tests/checksum.py), so a wrong row with the right row count is caught.
//
//   g(v, d)  = splitmix64_final(d64 ^ salt[v]) | 1     (odd, so products stay informative)
//   row(r)   = prod over columns c of g(var_c, digest(value_c))   mod 2^64
//   sum(T)   = sum over rows of row(r)                              mod 2^64
//
// d64 = the atom's first 8 digest bytes as a little-endian integer (the first
// 16 hex characters of its handle, byte-reversed); salt[v] is the caller's
// 64-bit key of variable v's name.  The product makes the row value
// independent of column order and lets a cross product or a join's
// checksum be computed as products of per-key sums (the closed forms).
#include "das_internal.h"

namespace das {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

struct CkCols {
  const uint32_t* col[kMaxCols];
  uint64_t salt[kMaxCols];
};

// out[0] += sum of row values, out[1] += values outside [0, n_atoms) (must stay 0)
template <int NC>
__global__ void __launch_bounds__(256) k_table_checksum(CkCols cc, int ncols, uint64_t nrows, const Digest* dig,
                                                        uint64_t n_atoms, unsigned long long* out) {
  uint64_t acc = 0, bad = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const int nc = NC > 0 ? NC : ncols;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrows; r += stride) {
    uint64_t h = 1;
#pragma unroll
    for (int c = 0; c < (NC > 0 ? NC : kMaxCols); ++c) {
      if (c >= nc) break;
      const uint32_t v = cc.col[c][r];
      uint64_t d = 0;
      if (v < n_atoms) {
        const uint2 w = *reinterpret_cast<const uint2*>(&dig[v].w[0]);
        d = (uint64_t)w.x | ((uint64_t)w.y << 32);
      } else {
        ++bad;
      }
      h *= mix64(d ^ cc.salt[c]) | 1ull;
    }
    acc += h;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    acc += (uint64_t)__shfl_xor((long long)acc, o, 64);
    bad += (uint64_t)__shfl_xor((long long)bad, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(out, (unsigned long long)acc);
    if (bad) atomicAdd(out + 1, (unsigned long long)bad);
  }
}

void table_checksum(Ctx& c, const Table& t, const uint64_t* salt, uint64_t out[2]) {
  DAS_CHECK(c.idx.built, DAS_E_NOT_BUILT, "checksum: no index");
  DAS_CHECK(t.kind == DAS_TABLE_ORDERED, DAS_E_UNSUPPORTED, "checksum: ordered tables only");
  DAS_CHECK(t.ncols >= 1 && t.ncols <= kMaxCols, DAS_E_INVALID, "checksum: bad column count");
  CkCols cc{};
  for (int i = 0; i < t.ncols; ++i) {
    cc.col[i] = t.col(i);
    cc.salt[i] = salt[i];
  }
  DBuf<unsigned long long> acc(2, c.s);
  DAS_HIP(hipMemsetAsync(acc.p, 0, 16, c.s));
  if (t.nrows) {
    const unsigned g = grid_for(t.nrows, 256, 8192);
    switch (t.ncols) {
      case 1: hipLaunchKernelGGL(k_table_checksum<1>, dim3(g), dim3(256), 0, c.s, cc, t.ncols, t.nrows, c.idx.digest, c.idx.n_atoms, acc.p); break;
      case 2: hipLaunchKernelGGL(k_table_checksum<2>, dim3(g), dim3(256), 0, c.s, cc, t.ncols, t.nrows, c.idx.digest, c.idx.n_atoms, acc.p); break;
      case 3: hipLaunchKernelGGL(k_table_checksum<3>, dim3(g), dim3(256), 0, c.s, cc, t.ncols, t.nrows, c.idx.digest, c.idx.n_atoms, acc.p); break;
      default: hipLaunchKernelGGL(k_table_checksum<0>, dim3(g), dim3(256), 0, c.s, cc, t.ncols, t.nrows, c.idx.digest, c.idx.n_atoms, acc.p); break;
    }
    DAS_HIP(hipGetLastError());
  }
  unsigned long long h[2];
  DAS_HIP(hipMemcpyAsync(h, acc.p, 16, hipMemcpyDeviceToHost, c.s));
  DAS_HIP(hipStreamSynchronize(c.s));
  out[0] = h[0];
  out[1] = h[1];
}

// ---- measurement: the box's 16-byte nontemporal store ceiling and trace marks
// (bench.py records them next to every run: the write-bound kernels'
// fractions move with the card, k_cartesian 0.73-0.87 over the same binary)
namespace {
// n4 uint4 per column over `ncol` columns, as k_cartesian writes them: one
// nontemporal dwordx4 store per lane, grid-stride
typedef uint32_t st_v4u __attribute__((ext_vector_type(4)));
__global__ void k_store16_nt(st_v4u* out, uint64_t n4, uint64_t cap4, int ncol) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x)
    for (int c = 0; c < ncol; ++c)
      __builtin_nontemporal_store(st_v4u{(uint32_t)i, (uint32_t)i + 1, (uint32_t)i + 2, (uint32_t)c}, &out[c * cap4 + i]);
}
__global__ void k_prof_mark(uint32_t* p, uint32_t id) {
  if (threadIdx.x == 0) p[0] = id;
}
}  // namespace

double box_store_bw(Ctx& c, uint64_t bytes, uint32_t reps) {
  DAS_CHECK(bytes >= (1u << 20) && reps >= 1, DAS_E_INVALID, "store probe: bytes >= 1 MiB, reps >= 1");
  const int ncol = 6;
  const uint64_t cap4 = (bytes / 16 / ncol + 63) & ~63ull;
  DBuf<st_v4u> buf(cap4 * ncol, c.s);
  const unsigned g = grid_for(cap4, 256);              // k_cartesian's launch: about one quad per thread and column
  hipEvent_t a = c.take_event(), b = c.take_event();
  hipLaunchKernelGGL(k_store16_nt, dim3(g), dim3(256), 0, c.s, buf.p, cap4, cap4, ncol);   // warm
  DAS_HIP(hipEventRecord(a, c.s));
  for (uint32_t r = 0; r < reps; ++r)
    hipLaunchKernelGGL(k_store16_nt, dim3(g), dim3(256), 0, c.s, buf.p, cap4, cap4, ncol);
  DAS_HIP(hipGetLastError());
  DAS_HIP(hipEventRecord(b, c.s));
  DAS_HIP(hipEventSynchronize(b));
  float ms = 0;
  DAS_HIP(hipEventElapsedTime(&ms, a, b));
  c.ev_pool.push_back(a);
  c.ev_pool.push_back(b);
  return 16.0 * cap4 * ncol * reps / (ms * 1e-3) / 1e9;
}

void prof_mark(Ctx& c, uint32_t id) {
  DBuf<uint32_t> m(1, c.s);
  hipLaunchKernelGGL(k_prof_mark, dim3(1), dim3(64), 0, c.s, m.p, id);
  DAS_HIP(hipGetLastError());
}

}  // namespace das
