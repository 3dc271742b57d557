// ExpressionHasher on the GPU: one message per lane, bit-exact MD5 hex handles.
//
//   leaves     md5(utf8 string)                       expression_hasher.py:13-19
//   composites md5(" ".join(hex(child digests)))      expression_hasher.py:22-35
//
// Composite messages are generated in registers: for K elements the message
// is 33K-1 bytes; every byte position is a compile-time constant once the
// block/word loops are unrolled for a given K, so building the 16 message
// words of a block is pure shift/select work on the K child digests (no
// division, no scratch).  Expressions arrive grouped by (nesting level, K) so
// a wavefront never diverges on K.
#include "das_internal.h"
#include "md5.h"

namespace das {

__global__ void __launch_bounds__(256) k_hash_strings(const uint8_t* __restrict__ bytes,
                                                      const uint64_t* __restrict__ off, uint64_t n,
                                                      DigS out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = off[i];
    const uint64_t len = off[i + 1] - b;
    const uint8_t* p = bytes + b;
    uint32_t st[4];
    md5::init(st);
    const uint64_t nblocks = (len + 9 + 63) / 64;
    for (uint64_t blk = 0; blk < nblocks; ++blk) {
      uint32_t M[16];
      const uint64_t base = blk * 64;
      if (base + 64 <= len) {
#pragma unroll
        for (int w = 0; w < 16; ++w) {
          const uint8_t* q = p + base + 4 * w;
          M[w] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
        }
      } else {
#pragma unroll
        for (int w = 0; w < 16; ++w) {
          uint32_t word = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint64_t pos = base + 4 * w + k;
            uint32_t byte = pos < len ? p[pos] : (pos == len ? 0x80u : 0u);
            word |= byte << (8 * k);
          }
          M[w] = word;
        }
        if (blk == nblocks - 1) {
          M[14] = (uint32_t)(len * 8);
          M[15] = (uint32_t)((len * 8) >> 32);
        }
      }
      md5::transform(st, M);
    }
    out[i] = Digest{{st[0], st[1], st[2], st[3]}};
  }
}

// Message byte at compile-time position POS of " ".join(hex(d_0..d_{K-1})).
template <int K>
__device__ __forceinline__ uint32_t comp_byte(const uint32_t (&d)[K][4], int pos) {
  constexpr int L = 33 * K - 1;
  if (pos < L) {
    const int e = pos / 33, o = pos - e * 33;
    if (o == 32) return 0x20u;
    return md5::hex_byte(d[e], (uint32_t)o);
  }
  return pos == L ? 0x80u : 0u;
}

template <int K>
__device__ __forceinline__ void md5_composite(const uint32_t (&d)[K][4], uint32_t st[4]) {
  constexpr int L = 33 * K - 1;
  constexpr int NB = (L + 9 + 63) / 64;
  md5::init(st);
#pragma unroll
  for (int blk = 0; blk < NB; ++blk) {
    uint32_t M[16];
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      const int pos = blk * 64 + 4 * w;
      M[w] = comp_byte<K>(d, pos) | (comp_byte<K>(d, pos + 1) << 8) | (comp_byte<K>(d, pos + 2) << 16) |
             (comp_byte<K>(d, pos + 3) << 24);
    }
    if (blk == NB - 1) {
      M[14] = (uint32_t)(L * 8);
      M[15] = 0;
    }
    md5::transform(st, M);
  }
}

// Generic K (> 9 elements): runtime byte loop, still one lane per message.
__device__ void md5_composite_dyn(DigS tab, const uint32_t* child, uint32_t K, uint32_t st[4]) {
  const uint64_t L = 33ull * K - 1;
  const uint64_t NB = (L + 9 + 63) / 64;
  md5::init(st);
  for (uint64_t blk = 0; blk < NB; ++blk) {
    uint32_t M[16];
    for (int w = 0; w < 16; ++w) {
      uint32_t word = 0;
      for (int k = 0; k < 4; ++k) {
        const uint64_t pos = blk * 64 + 4 * w + k;
        uint32_t byte;
        if (pos < L) {
          const uint64_t e = pos / 33, o = pos - e * 33;
          byte = (o == 32) ? 0x20u : md5::hex_byte(tab[child[e]].w, (uint32_t)o);
        } else {
          byte = pos == L ? 0x80u : 0u;
        }
        word |= byte << (8 * k);
      }
      M[w] = word;
    }
    if (blk == NB - 1) {
      M[14] = (uint32_t)(L * 8);
      M[15] = (uint32_t)((L * 8) >> 32);
    }
    md5::transform(st, M);
  }
}

// Expressions [begin, begin+n) of one (level, K) group.  `table` holds the
// digests of every unified index; out = table + n_leaf (written in place).
// When `ctab` is given, the composite type is computed from the children's
// composite types the same way (canonical_parser.py:276, base_yacc.py:92-98),
// unless `ctype_leaf[j] >= 0` (typedef used as a symbol: md5(name)).
template <int K>
__global__ void __launch_bounds__(256, K <= 6 ? 6 : 1) k_hash_group(DigS table, DigS ctab,
                                                    const uint32_t* __restrict__ child,
                                                    const uint64_t* __restrict__ child_off,
                                                    const int32_t* __restrict__ ctype_leaf, uint64_t n_leaf,
                                                    uint64_t begin, uint64_t n, uint32_t* __restrict__ etype) {
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t j = begin + t;
    const uint32_t* ch = child + child_off[j];
    if (etype) etype[j] = ch[0];                       // the expression's first element: its type leaf
    const int32_t cl = ctab.p && ctype_leaf ? ctype_leaf[j] : -1;
    // both digests of every child loaded up front: with the interleaved
    // records (DigS stride 2) they share a line, and the composite digests
    // are in registers when the second MD5 starts
    uint32_t d[K][4], cd[K][4];
#pragma unroll
    for (int e = 0; e < K; ++e) {
      const Digest x = table[ch[e]];
#pragma unroll
      for (int q = 0; q < 4; ++q) d[e][q] = x.w[q];
      if (ctab.p && cl < 0) {
        const Digest y = ctab[ch[e]];
#pragma unroll
        for (int q = 0; q < 4; ++q) cd[e][q] = y.w[q];
      }
    }
    uint32_t st[4];
    if (K == 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q) st[q] = d[0][q];
    } else {
      md5_composite<K>(d, st);
    }
    table[n_leaf + j] = Digest{{st[0], st[1], st[2], st[3]}};
    if (ctab.p) {
      if (cl >= 0) {
        ctab[n_leaf + j] = table[cl];
      } else {
#pragma unroll
        for (int e = 0; e < K; ++e)
#pragma unroll
          for (int q = 0; q < 4; ++q) d[e][q] = cd[e][q];
        if (K == 1) {
#pragma unroll
          for (int q = 0; q < 4; ++q) st[q] = d[0][q];
        } else {
          md5_composite<K>(d, st);
        }
        ctab[n_leaf + j] = Digest{{st[0], st[1], st[2], st[3]}};
      }
    }
  }
}

__global__ void k_hash_group_dyn(DigS table, DigS ctab, const uint32_t* child, const uint64_t* child_off,
                                 const int32_t* ctype_leaf, uint64_t n_leaf, uint64_t begin, uint64_t n,
                                 uint32_t* etype) {
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t j = begin + t;
    const uint32_t* ch = child + child_off[j];
    if (etype) etype[j] = ch[0];
    const uint32_t K = (uint32_t)(child_off[j + 1] - child_off[j]);
    uint32_t st[4];
    md5_composite_dyn(table, ch, K, st);
    table[n_leaf + j] = Digest{{st[0], st[1], st[2], st[3]}};
    if (ctab.p) {
      const int32_t cl = ctype_leaf ? ctype_leaf[j] : -1;
      if (cl >= 0) {
        ctab[n_leaf + j] = table[cl];
      } else {
        md5_composite_dyn(ctab, ch, K, st);
        ctab[n_leaf + j] = Digest{{st[0], st[1], st[2], st[3]}};
      }
    }
  }
}

// Bench/test entry: message i = elems[i*K .. i*K+K) laid out contiguously.
template <int K>
__global__ void __launch_bounds__(256) k_hash_fixed(const Digest* __restrict__ elems, uint64_t n,
                                                    Digest* __restrict__ out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t d[K][4];
#pragma unroll
    for (int e = 0; e < K; ++e) {
      const Digest x = elems[i * K + e];
#pragma unroll
      for (int q = 0; q < 4; ++q) d[e][q] = x.w[q];
    }
    uint32_t st[4];
    md5_composite<K>(d, st);
    out[i] = Digest{{st[0], st[1], st[2], st[3]}};
  }
}

void hash_strings(const uint8_t* bytes, const uint64_t* off, uint64_t n, DigS out, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_hash_strings, dim3(grid_for(n, 256, 256 * 64)), dim3(256), 0, s, bytes, off, n, out);
  DAS_HIP(hipGetLastError());
}

void hash_group(DigS table, DigS ctab, const uint32_t* child, const uint64_t* child_off,
                const int32_t* ctype_leaf, uint64_t n_leaf, uint64_t begin, uint64_t n, uint32_t K,
                hipStream_t s, uint32_t* etype) {
  if (!n) return;
  const dim3 g(grid_for(n, 256, 256 * 64)), b(256);
#define DAS_HG(KK)                                                                                  \
  case KK:                                                                                          \
    hipLaunchKernelGGL((k_hash_group<KK>), g, b, 0, s, table, ctab, child, child_off, ctype_leaf, \
                       n_leaf, begin, n, etype);                                                    \
    break;
  switch (K) {
    DAS_HG(1) DAS_HG(2) DAS_HG(3) DAS_HG(4) DAS_HG(5) DAS_HG(6) DAS_HG(7) DAS_HG(8) DAS_HG(9)
    default:
      hipLaunchKernelGGL(k_hash_group_dyn, g, b, 0, s, table, ctab, child, child_off, ctype_leaf, n_leaf, begin, n,
                         etype);
  }
#undef DAS_HG
  DAS_HIP(hipGetLastError());
}

void hash_fixed(const Digest* elems, uint32_t k, uint64_t n, Digest* out, hipStream_t s) {
  if (!n) return;
  const dim3 g(grid_for(n, 256, 256 * 64)), b(256);
  switch (k) {
    case 2: hipLaunchKernelGGL((k_hash_fixed<2>), g, b, 0, s, elems, n, out); break;
    case 3: hipLaunchKernelGGL((k_hash_fixed<3>), g, b, 0, s, elems, n, out); break;
    case 4: hipLaunchKernelGGL((k_hash_fixed<4>), g, b, 0, s, elems, n, out); break;
    case 5: hipLaunchKernelGGL((k_hash_fixed<5>), g, b, 0, s, elems, n, out); break;
    default: throw Error(DAS_E_UNSUPPORTED, "hash_fixed: k must be 2..5");
  }
  DAS_HIP(hipGetLastError());
}

}  // namespace das
