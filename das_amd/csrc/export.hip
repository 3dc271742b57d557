// Redis key-space export of the device index.
//
// Writes the five key-value files CanonicalParser builds before it fills
// Redis (canonical_parser.py:119-183, key_value_file.py:8-16):
//   outgoing_set.txt   link \t target          one line per target position
//   incomming_set.txt  target \t link          (the reference's spelling)
//   patterns.txt       key \t link \t targets  key = composite_hash([type|*, t_0|*, ...])
//   templates.txt      key \t link \t targets  key = composite type hash, and named type hash
//   names.txt          node \t name
// each sorted bytewise (what `sort` does in the C locale), so a file can be
// diffed byte for byte against the reference's.  Pattern lines reproduce the
// reference's key list exactly, including the key it lists twice for
// arities 1-3 ([*, e0, ...] is appended before the per-arity list, which
// contains it again) and the single [*, e0, ..., en] key of arity >= 4.
//
// The pattern keys are the expensive part (up to 16 MD5s of up to 131-byte
// messages per link): one link per lane, every key's message generated in
// registers with compile-time byte positions (the mask is a template
// argument), then the (key, link) lines are ordered with two stable device
// radix sorts on the big-endian high 64 bits of the key and link digests.
// Ties of those 64 bits between different digests are resolved on the host.
#include <algorithm>
#include <cstdio>
#include <string>

#include "das_internal.h"
#include "md5.h"

namespace das {

namespace {

template <int A, int M>
struct KeyShape {
  static constexpr int P = A + 1;                                  // parts: type, t_0 .. t_{A-1}
  static constexpr bool wild(int p) { return (M >> p) & 1; }
  static constexpr int len(int p) { return wild(p) ? 1 : 32; }
  static constexpr int total() {
    int l = P - 1;
    for (int p = 0; p < P; ++p) l += len(p);
    return l;
  }
  static constexpr int L = total();
  static constexpr int NB = (L + 9 + 63) / 64;
};

// message byte at compile-time position pos of " ".join(part_0 .. part_A)
template <int A, int M>
__device__ __forceinline__ uint32_t key_byte(const uint32_t (&d)[A + 1][4], int pos) {
  using S = KeyShape<A, M>;
  if (pos >= S::L) return pos == S::L ? 0x80u : 0u;
  int q = pos;
#pragma unroll
  for (int p = 0; p < S::P; ++p) {
    const int l = S::len(p);
    if (q < l) return S::wild(p) ? 0x2Au : md5::hex_byte(d[p], (uint32_t)q);
    q -= l;
    if (q == 0) return 0x20u;
    q -= 1;
  }
  return 0u;
}

template <int A, int M>
__device__ __forceinline__ void key_md5(const uint32_t (&d)[A + 1][4], uint32_t st[4]) {
  using S = KeyShape<A, M>;
  md5::init(st);
#pragma unroll
  for (int blk = 0; blk < S::NB; ++blk) {
    uint32_t W[16];
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      const int pos = blk * 64 + 4 * w;
      W[w] = key_byte<A, M>(d, pos) | (key_byte<A, M>(d, pos + 1) << 8) | (key_byte<A, M>(d, pos + 2) << 16) |
             (key_byte<A, M>(d, pos + 3) << 24);
    }
    if (blk == S::NB - 1) {
      W[14] = (uint32_t)(S::L * 8);
      W[15] = 0;
    }
    md5::transform(st, W);
  }
}

__device__ __forceinline__ uint64_t be_hi(const uint32_t w[4]) {
  return __builtin_bswap64((uint64_t)w[0] | ((uint64_t)w[1] << 32));
}

// The reference's key list per arity (canonical_parser.py:144-178); bit 0 =
// type wildcard, bit 1 + i = target i wildcard.
template <int A> struct Masks;
template <> struct Masks<1> { static constexpr int n = 4; };
template <> struct Masks<2> { static constexpr int n = 8; };
template <> struct Masks<3> { static constexpr int n = 16; };
template <int A> struct Masks { static constexpr int n = 1; };

template <int A, int M>
__device__ __forceinline__ void emit(const uint32_t (&d)[A + 1][4], uint64_t line, uint32_t link, uint64_t link_hi,
                                     Digest* kd, uint64_t* khi, uint64_t* shi, uint32_t* lid) {
  uint32_t st[4];
  key_md5<A, M>(d, st);
  kd[line] = Digest{{st[0], st[1], st[2], st[3]}};
  khi[line] = be_hi(st);
  shi[line] = link_hi;
  lid[line] = link;
}

template <int A>
__global__ void __launch_bounds__(256) k_pattern_lines(const uint32_t* __restrict__ rows, uint64_t ld, uint64_t n,
                                                       const Digest* __restrict__ dig,
                                                       const uint32_t* __restrict__ type,
                                                       const Digest* __restrict__ type_dig, Digest* kd,
                                                       uint64_t* khi, uint64_t* shi, uint32_t* lid) {
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t link = rows[r];
    uint32_t d[A + 1][4];
    const Digest td = type_dig[type[link]];
#pragma unroll
    for (int q = 0; q < 4; ++q) d[0][q] = td.w[q];
#pragma unroll
    for (int k = 0; k < A; ++k) {
      const Digest x = dig[rows[(uint64_t)(k + 1) * ld + r]];
#pragma unroll
      for (int q = 0; q < 4; ++q) d[k + 1][q] = x.w[q];
    }
    const uint64_t lh = be_hi(dig[link].w);
    const uint64_t base = r * Masks<A>::n;
    if constexpr (A == 1) {
      emit<1, 1>(d, base + 0, link, lh, kd, khi, shi, lid);
      emit<1, 2>(d, base + 1, link, lh, kd, khi, shi, lid);
      emit<1, 1>(d, base + 2, link, lh, kd, khi, shi, lid);
      emit<1, 3>(d, base + 3, link, lh, kd, khi, shi, lid);
    } else if constexpr (A == 2) {
      emit<2, 1>(d, base + 0, link, lh, kd, khi, shi, lid);
      emit<2, 4>(d, base + 1, link, lh, kd, khi, shi, lid);
      emit<2, 2>(d, base + 2, link, lh, kd, khi, shi, lid);
      emit<2, 6>(d, base + 3, link, lh, kd, khi, shi, lid);
      emit<2, 1>(d, base + 4, link, lh, kd, khi, shi, lid);
      emit<2, 5>(d, base + 5, link, lh, kd, khi, shi, lid);
      emit<2, 3>(d, base + 6, link, lh, kd, khi, shi, lid);
      emit<2, 7>(d, base + 7, link, lh, kd, khi, shi, lid);
    } else if constexpr (A == 3) {
      emit<3, 1>(d, base + 0, link, lh, kd, khi, shi, lid);
      emit<3, 1>(d, base + 1, link, lh, kd, khi, shi, lid);
      emit<3, 2>(d, base + 2, link, lh, kd, khi, shi, lid);
      emit<3, 3>(d, base + 3, link, lh, kd, khi, shi, lid);
      emit<3, 4>(d, base + 4, link, lh, kd, khi, shi, lid);
      emit<3, 5>(d, base + 5, link, lh, kd, khi, shi, lid);
      emit<3, 6>(d, base + 6, link, lh, kd, khi, shi, lid);
      emit<3, 7>(d, base + 7, link, lh, kd, khi, shi, lid);
      emit<3, 8>(d, base + 8, link, lh, kd, khi, shi, lid);
      emit<3, 9>(d, base + 9, link, lh, kd, khi, shi, lid);
      emit<3, 10>(d, base + 10, link, lh, kd, khi, shi, lid);
      emit<3, 11>(d, base + 11, link, lh, kd, khi, shi, lid);
      emit<3, 12>(d, base + 12, link, lh, kd, khi, shi, lid);
      emit<3, 13>(d, base + 13, link, lh, kd, khi, shi, lid);
      emit<3, 14>(d, base + 14, link, lh, kd, khi, shi, lid);
      emit<3, 15>(d, base + 15, link, lh, kd, khi, shi, lid);
    } else {
      emit<A, 1>(d, base, link, lh, kd, khi, shi, lid);
    }
  }
}

__global__ void k_gather_u64(const uint64_t* src, const uint32_t* idx, uint64_t* dst, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[idx[i]];
}

inline dim3 G(uint64_t n) { return dim3(grid_for(n, 256, 65535u * 4u)); }

// permutation ordering lines by (khi, shi); both arrays are consumed
void order_lines(uint64_t* khi, uint64_t* shi, uint64_t n, uint32_t* perm, hipStream_t s) {
  iota(perm, n, s);
  radix_sort_pairs<uint64_t>(shi, perm, n, 0, 64, s);
  DBuf<uint64_t> k2(n, s);
  hipLaunchKernelGGL(k_gather_u64, G(n), dim3(256), 0, s, (const uint64_t*)khi, (const uint32_t*)perm, k2.p, n);
  DAS_HIP(hipGetLastError());
  radix_sort_pairs<uint64_t>(k2.p, perm, n, 0, 64, s);
}

struct Hex {
  char s[33];
  explicit Hex(const Digest& d) {
    md5::to_hex(d.w, s);
    s[32] = 0;
  }
};

int cmp_digest(const Digest& a, const Digest& b) {
  for (int i = 0; i < 4; ++i) {
    const uint32_t x = __builtin_bswap32(a.w[i]), y = __builtin_bswap32(b.w[i]);
    if (x != y) return x < y ? -1 : 1;
  }
  return 0;
}

struct Writer {
  FILE* f;
  std::string buf;
  explicit Writer(const std::string& path) : f(std::fopen(path.c_str(), "wb")) {
    DAS_CHECK(f, DAS_E_INVALID, "cannot open " + path + " for writing");
    buf.reserve(1 << 22);
  }
  ~Writer() {
    flush();
    if (f) std::fclose(f);
  }
  void flush() {
    if (!buf.empty() && f) std::fwrite(buf.data(), 1, buf.size(), f);
    buf.clear();
  }
  void put(const Digest& d) { buf.append(Hex(d).s, 32); }
  void tab() { buf.push_back('\t'); }
  void end() {
    buf.push_back('\n');
    if (buf.size() > (1u << 22)) flush();
  }
};

// host-side line sets (the small families): sort by full (key, value) digests
struct Pair {
  Digest k, v;
  uint32_t link;
};

}  // namespace

ExportCounts export_keyspace(Ctx& c, const std::string& dir) {
  Index& idx = c.idx;
  DAS_CHECK(idx.built, DAS_E_NOT_BUILT, "index not built");
  hipStream_t s = c.s;
  const uint64_t na = idx.n_atoms;
  // host mirrors of what every line prints
  std::vector<Digest> dig(na);
  std::vector<uint8_t> cat(na);
  std::vector<uint32_t> type(na), ctype(na), name_leaf(na);
  std::vector<uint64_t> toff(na + 1);
  DAS_HIP(hipMemcpyAsync(dig.data(), idx.digest, 16 * na, hipMemcpyDeviceToHost, s));
  DAS_HIP(hipMemcpyAsync(cat.data(), idx.cat, na, hipMemcpyDeviceToHost, s));
  DAS_HIP(hipMemcpyAsync(type.data(), idx.type, 4 * na, hipMemcpyDeviceToHost, s));
  DAS_HIP(hipMemcpyAsync(ctype.data(), idx.ctype, 4 * na, hipMemcpyDeviceToHost, s));
  DAS_HIP(hipMemcpyAsync(name_leaf.data(), idx.name_leaf, 4 * na, hipMemcpyDeviceToHost, s));
  DAS_HIP(hipMemcpyAsync(toff.data(), idx.tgt_off, 8 * (na + 1), hipMemcpyDeviceToHost, s));
  DAS_HIP(hipStreamSynchronize(s));
  std::vector<uint32_t> tgt(toff[na]);
  if (!tgt.empty()) DAS_HIP(hipMemcpyAsync(tgt.data(), idx.tgt, 4 * tgt.size(), hipMemcpyDeviceToHost, s));
  DAS_HIP(hipStreamSynchronize(s));
  ExportCounts cnt{};
  auto link_value = [&](Writer& w, uint32_t link) {
    w.put(dig[link]);
    for (uint64_t k = toff[link]; k < toff[link + 1]; ++k) {
      w.tab();
      w.put(dig[tgt[k]]);
    }
  };
  auto by_kv = [](const Pair& a, const Pair& b) {
    const int x = cmp_digest(a.k, b.k);
    return x ? x < 0 : cmp_digest(a.v, b.v) < 0;
  };

  // outgoing / incoming sets (canonical_parser.py:139-143)
  {
    std::vector<Pair> out, in;
    for (uint64_t a = 0; a < na; ++a) {
      if (cat[a] != CAT_LINK) continue;
      for (uint64_t k = toff[a]; k < toff[a + 1]; ++k) {
        out.push_back({dig[a], dig[tgt[k]], 0});
        in.push_back({dig[tgt[k]], dig[a], 0});
      }
    }
    for (int pass = 0; pass < 2; ++pass) {
      auto& v = pass ? in : out;
      std::sort(v.begin(), v.end(), by_kv);
      Writer w(dir + (pass ? "/incomming_set.txt" : "/outgoing_set.txt"));
      for (auto& p : v) {
        w.put(p.k);
        w.tab();
        w.put(p.v);
        w.end();
      }
      (pass ? cnt.incoming : cnt.outgoing) = v.size();
    }
  }

  // templates: composite type hash and named type hash (canonical_parser.py:179-180)
  {
    std::vector<Pair> t;
    for (uint64_t a = 0; a < na; ++a) {
      if (cat[a] != CAT_LINK) continue;
      DAS_CHECK(ctype[a] < idx.ctype_digest.size() && type[a] < idx.type_digest.size(), DAS_E_INTERNAL,
                "link without composite / named type");
      t.push_back({idx.ctype_digest[ctype[a]], dig[a], (uint32_t)a});
      t.push_back({idx.type_digest[type[a]], dig[a], (uint32_t)a});
    }
    std::sort(t.begin(), t.end(), by_kv);
    Writer w(dir + "/templates.txt");
    for (auto& p : t) {
      w.put(p.k);
      w.tab();
      link_value(w, p.link);
      w.end();
    }
    cnt.templates = t.size();
  }

  // names: node handle and name (canonical_parser.py:119-121)
  {
    std::vector<Pair> nm;
    for (uint64_t a = 0; a < na; ++a)
      if (cat[a] == CAT_NODE) nm.push_back({dig[a], Digest{}, (uint32_t)a});
    std::sort(nm.begin(), nm.end(), [](const Pair& x, const Pair& y) { return cmp_digest(x.k, y.k) < 0; });
    Writer w(dir + "/names.txt");
    for (auto& p : nm) {
      w.put(p.k);
      w.tab();
      const uint32_t leaf = name_leaf[p.link];
      DAS_CHECK(leaf + 1 < c.leaf_off.size() && type[p.link] < idx.type_name_len.size(), DAS_E_INTERNAL,
                "node without a name leaf");
      const uint64_t b = c.leaf_off[leaf] + idx.type_name_len[type[p.link]] + 1, e = c.leaf_off[leaf + 1];
      w.buf.append(reinterpret_cast<const char*>(c.leaf_bytes.data()) + b, e - b);
      w.end();
    }
    cnt.names = nm.size();
  }

  // patterns: device-hashed keys, device-ordered lines
  {
    DBuf<Digest> type_dig(std::max<size_t>(idx.type_digest.size(), 1), s);
    if (!idx.type_digest.empty())
      DAS_HIP(hipMemcpyAsync(type_dig.p, idx.type_digest.data(), 16 * idx.type_digest.size(), hipMemcpyHostToDevice,
                             s));
    Writer w(dir + "/patterns.txt");
    // one line set per arity, merged on the host by key (each set is sorted)
    struct Set {
      std::vector<uint32_t> perm, lid;
      std::vector<Digest> kd;
      uint64_t pos = 0;
    };
    std::vector<Set> sets;
    for (int a = 1; a <= kMaxArity; ++a) {
      const RowTable& rt = idx.ttab[a];
      if (!rt.rows) continue;
      int L = a == 1 ? 4 : a == 2 ? 8 : a == 3 ? 16 : 1;
      const uint64_t n = rt.rows * (uint64_t)L;
      DBuf<Digest> kd(n, s);
      DBuf<uint64_t> khi(n, s), shi(n, s);
      DBuf<uint32_t> lid(n, s), perm(n, s);
#define DAS_PL(AA)                                                                                          \
  case AA:                                                                                                  \
    hipLaunchKernelGGL(k_pattern_lines<AA>, G(rt.rows), dim3(256), 0, s, (const uint32_t*)rt.data, rt.ld,  \
                       rt.rows, (const Digest*)idx.digest, (const uint32_t*)idx.type,                        \
                       (const Digest*)type_dig.p, kd.p, khi.p, shi.p, lid.p);                                \
    break;
      switch (a) { DAS_PL(1) DAS_PL(2) DAS_PL(3) DAS_PL(4) DAS_PL(5) DAS_PL(6) DAS_PL(7) DAS_PL(8) }
#undef DAS_PL
      DAS_HIP(hipGetLastError());
      order_lines(khi.p, shi.p, n, perm.p, s);
      Set st;
      st.perm.resize(n);
      st.lid.resize(n);
      st.kd.resize(n);
      DAS_HIP(hipMemcpyAsync(st.perm.data(), perm.p, 4 * n, hipMemcpyDeviceToHost, s));
      DAS_HIP(hipMemcpyAsync(st.lid.data(), lid.p, 4 * n, hipMemcpyDeviceToHost, s));
      DAS_HIP(hipMemcpyAsync(st.kd.data(), kd.p, 16 * n, hipMemcpyDeviceToHost, s));
      DAS_HIP(hipStreamSynchronize(s));
      // exact order inside runs whose 64-bit prefixes tie
      auto full_less = [&](uint32_t x, uint32_t y) {
        const int k = cmp_digest(st.kd[x], st.kd[y]);
        return k ? k < 0 : cmp_digest(dig[st.lid[x]], dig[st.lid[y]]) < 0;
      };
      for (uint64_t i = 0; i + 1 < n;) {
        uint64_t j = i + 1;
        auto hi = [&](uint32_t x) {
          return std::make_pair(__builtin_bswap64((uint64_t)st.kd[x].w[0] | ((uint64_t)st.kd[x].w[1] << 32)),
                                __builtin_bswap64((uint64_t)dig[st.lid[x]].w[0] | ((uint64_t)dig[st.lid[x]].w[1] << 32)));
        };
        const auto h0 = hi(st.perm[i]);
        while (j < n && hi(st.perm[j]) == h0) ++j;
        if (j - i > 1) std::stable_sort(st.perm.begin() + i, st.perm.begin() + j, full_less);
        i = j;
      }
      sets.push_back(std::move(st));
    }
    // k-way merge of the per-arity sets by (key, link)
    for (;;) {
      int best = -1;
      for (int k = 0; k < (int)sets.size(); ++k) {
        Set& x = sets[k];
        if (x.pos >= x.perm.size()) continue;
        if (best < 0) { best = k; continue; }
        Set& y = sets[best];
        const uint32_t a = x.perm[x.pos], b = y.perm[y.pos];
        int cmp = cmp_digest(x.kd[a], y.kd[b]);
        if (!cmp) cmp = cmp_digest(dig[x.lid[a]], dig[y.lid[b]]);
        if (cmp < 0) best = k;
      }
      if (best < 0) break;
      Set& x = sets[best];
      const uint32_t a = x.perm[x.pos++];
      w.put(x.kd[a]);
      w.tab();
      link_value(w, x.lid[a]);
      w.end();
      ++cnt.patterns;
    }
  }
  return cnt;
}

}  // namespace das
