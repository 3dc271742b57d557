// Device-side generator of the configs 4-5 synthetic hypergraph (SURVEY.md
// §8d: "1 B links; 70% arity 2 / 30% arity 3; 4 link types; Zipf(1.1)
// targets; seed fixed; generated on device").  Bench / test input only: it
// writes expression children in the das_atoms_t layout straight into HBM, so a
// 10^9-link build starts from resident input instead of a 30 GB host upload.
//
// Link i (global index) draws every field from a counter-based hash of
// (seed, i, field), so the KB is the same whatever range a rank generates:
// the union of the N per-rank ranges is the one-GPU KB.
#include <cstring>
#include <thread>
#include <vector>

#include "das_internal.h"

namespace das {

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {     // splitmix64 finaliser
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Zipf(s) rank in [0, n) by inverting the continuous power law x^-s on
// [1, n+1): x = (1 - u (1 - (n+1)^(1-s)))^(1/(1-s)), rank = floor(x) - 1.
__device__ __forceinline__ uint32_t zipf_rank(uint64_t h, double one_minus_s, double tail, uint64_t n) {
  const double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);
  const double x = pow(1.0 - u * tail, 1.0 / one_minus_s);
  uint64_t r = (uint64_t)x;
  r = r ? r - 1 : 0;
  return (uint32_t)(r < n ? r : n - 1);
}

// One link per lane; row = [type leaf, K-1 node leaves], written as K
// consecutive u32 (the expression layout of das_atoms_t.expr_child).
template <int K>
__global__ void __launch_bounds__(256) k_synth_links(uint32_t* __restrict__ child, uint64_t first, uint64_t n,
                                                     uint32_t n_link_types, uint32_t type_leaf0,
                                                     uint32_t node_leaf0, uint64_t n_nodes, double one_minus_s,
                                                     double tail, uint64_t seed) {
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = first + j;
    const uint64_t base = mix64(seed ^ mix64(i));
    uint32_t row[K];
    row[0] = type_leaf0 + (uint32_t)(mix64(base) % n_link_types);
#pragma unroll
    for (int q = 1; q < K; ++q) row[q] = node_leaf0 + zipf_rank(mix64(base + (uint64_t)q), one_minus_s, tail, n_nodes);
    uint32_t* o = child + j * K;
#pragma unroll
    for (int q = 0; q < K; ++q) o[q] = row[q];
  }
}

}  // namespace

void synth_powerlaw_links(uint32_t* d_child, uint64_t first, uint64_t n, uint32_t K, uint32_t n_link_types,
                          uint32_t type_leaf0, uint32_t node_leaf0, uint64_t n_nodes, double s, uint64_t seed,
                          hipStream_t st) {
  DAS_CHECK(n_link_types > 0 && n_nodes > 0 && n_nodes < 0xFFFFFFF0ull, DAS_E_INVALID, "synth: bad sizes");
  DAS_CHECK(s > 1.0, DAS_E_INVALID, "synth: Zipf exponent must exceed 1");
  if (!n) return;
  const double oms = 1.0 - s;
  const double tail = 1.0 - pow((double)n_nodes + 1.0, oms);
  const dim3 g(grid_for(n, 256, 8192)), b(256);
  switch (K) {
    case 3: hipLaunchKernelGGL(k_synth_links<3>, g, b, 0, st, d_child, first, n, n_link_types, type_leaf0, node_leaf0, n_nodes, oms, tail, seed); break;
    case 4: hipLaunchKernelGGL(k_synth_links<4>, g, b, 0, st, d_child, first, n, n_link_types, type_leaf0, node_leaf0, n_nodes, oms, tail, seed); break;
    default: throw Error(DAS_E_UNSUPPORTED, "synth: arity 2 or 3 only");
  }
  DAS_HIP(hipGetLastError());
}

// Host: the n strings prefix + decimal(first + i) packed back to back, with
// n + 1 offsets (the node leaves "Concept n<i>" of configs 4-5; 2^27 of them
// are ~2.4 GB, written by up to 16 host threads at memory speed).
void numbered_strings(const char* prefix, uint64_t plen, uint64_t first, uint64_t n, uint8_t* out, uint64_t* off) {
  auto digits = [](uint64_t v) {
    int d = 1;
    while (v >= 10) { v /= 10; ++d; }
    return d;
  };
  // offsets: closed form per digit-length run
  auto offset_of = [&](uint64_t i) {     // bytes before string i
    uint64_t total = i * plen, v = first, end = first + i, p = 10;
    int d = 1;
    while (v < end) {
      while (v >= p) { p *= 10; ++d; }
      const uint64_t run_end = end < p ? end : p;
      total += (run_end - v) * (uint64_t)d;
      v = run_end;
    }
    return total;
  };
  const unsigned T = n < (1u << 16) ? 1u : 16u;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      const uint64_t b = n * t / T, e = n * (t + 1) / T;
      uint64_t o = offset_of(b);
      char tmp[24];
      for (uint64_t i = b; i < e; ++i) {
        off[i] = o;
        std::memcpy(out + o, prefix, plen);
        o += plen;
        uint64_t v = first + i;
        const int d = digits(v);
        for (int k = d - 1; k >= 0; --k) { tmp[k] = (char)('0' + v % 10); v /= 10; }
        std::memcpy(out + o, tmp, d);
        o += d;
      }
      if (t == T - 1) off[n] = o;
    });
  for (auto& x : th) x.join();
  if (!n) off[0] = 0;
}

}  // namespace das
