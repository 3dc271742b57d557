// Unordered / Composite assignment algebra on the GPU.
//
// Reference (das/pattern_matcher/pattern_matcher.py):
//   UnorderedAssignment  :158-262  (multisets of symbols and values; identity
//                                   = (symbol set, value multiset))
//   CompositeAssignment  :264-368  (one optional ordered mapping + a list of
//                                   unordered members; hash = ordered.hash (or
//                                   1) XOR member hashes, :279-286, :307-314)
//   joins                 OrderedAssignment.join :105-110, Unordered.join
//                         :203-209, Composite.join :341-351 with
//                         _add_ordered_mapping :316-327 (+ _check_ordered_
//                         viability :290-305) and _add_unordered_mapping :329-336
//   negation              check_negation :112-117, :211-217, :353-362
//
// Device tables (DAS_TABLE_COMPOSITE): the ordered columns first (member -1,
// sorted by variable id), then every unordered member in join order, each as
// its sorted variable ids (vars[]) and sorted values (columns).  An
// UNORDERED table is one member; an ORDERED table is an ordered part only.
//
// A join involving an unordered operand has no equality key in general: its
// row-pair predicate is a conjunction of set-containment checks.  The host
// lowers the reference's method sequence for the two operand schemas into a
// short list of checks over the "pair row" (left columns, then right
// columns); the kernels evaluate it one wave per left row, lanes striding over
// the candidate right rows (all of them, or the equal range on the shared
// ordered variables when there are any), with ballot compaction so the output
// keeps the reference's nested-loop order.  Schema-level outcomes (a check
// that can never hold, the reference's AttributeErrors) are decided on the
// host.
//
// Set identity (the Python `set` of assignments) is exact: every row gets a
// canonical key — [is-unordered flag | ordered values | per member variable
// set: the member value tuples sorted, equal pairs cancelled (the XOR),
// padded] — laid out per class of tables with the same ordered variables, and
// dedup / difference run as a sort + adjacent compare over those keys.
#include <algorithm>
#include <map>

#include "das_internal.h"

namespace das {

namespace {

constexpr unsigned B = 256;
constexpr int kMaxUni = 2 * kMaxCols;     // pair-row columns
constexpr int kMaxChecks = 64;
constexpr int kMaxKeyCols = 64;

enum CheckOp : uint8_t {
  CK_EQ,          // v[o0] == v[o1]
  CK_DISTINCT,    // values at o[0..no) pairwise distinct (no_overload)
  CK_CONTAINS_O,  // member A contains ordered o[]: o values distinct, each in A  (contains_ordered :219-228)
  CK_COVERED,     // every value of member A is an ordered value o[]          (is_covered_by_ordered :230-235)
  CK_VIABLE,      // (k&1 && CONTAINS_O) || (k&2 && COVERED)                    (_check_ordered_viability)
  CK_COMPAT,      // |values(A) & values(B)| >= k                              (compatible :247-262)
  CK_CONTAINS_U,  // values(B) subset of values(A)                             (contains_unordered :238-245)
};

struct Check {
  uint8_t op = 0;
  uint8_t a0 = 0, aw = 0;   // member A columns [a0, a0 + aw) of the pair row
  uint8_t b0 = 0, bw = 0;   // member B
  uint8_t k = 0;
  uint8_t no = 0;
  uint8_t o[kMaxCols] = {};
};

struct Theta {
  const uint32_t* col[kMaxUni];
  int nl = 0, nr = 0;
  int nchk = 0;
  int any = 0;              // 0: pair kept iff every check holds; 1: "hit" iff some check holds
  int nout = 0;
  uint8_t out[kMaxCols];
  Check chk[kMaxChecks];
};

__device__ __forceinline__ bool in_vals(uint32_t x, const uint32_t* v, int b, int w) {
  for (int k = 0; k < w; ++k)
    if (v[b + k] == x) return true;
  return false;
}

__device__ bool contains_o(const Check& c, const uint32_t* v) {
  for (int a = 0; a < c.no; ++a) {
    const uint32_t x = v[c.o[a]];
    for (int b = 0; b < a; ++b)
      if (v[c.o[b]] == x) return false;          // count 2 > count 1 in a value set
    if (!in_vals(x, v, c.a0, c.aw)) return false;
  }
  return true;
}

__device__ bool covered(const Check& c, const uint32_t* v) {
  for (int k = 0; k < c.aw; ++k) {
    const uint32_t x = v[c.a0 + k];
    bool f = false;
    for (int a = 0; a < c.no && !f; ++a) f = v[c.o[a]] == x;
    if (!f) return false;
  }
  return true;
}

__device__ bool eval_check(const Check& c, const uint32_t* v) {
  switch (c.op) {
    case CK_EQ:
      return v[c.o[0]] == v[c.o[1]];
    case CK_DISTINCT:
      for (int a = 0; a < c.no; ++a)
        for (int b = a + 1; b < c.no; ++b)
          if (v[c.o[a]] == v[c.o[b]]) return false;
      return true;
    case CK_CONTAINS_O:
      return contains_o(c, v);
    case CK_COVERED:
      return covered(c, v);
    case CK_VIABLE:
      return ((c.k & 1) && contains_o(c, v)) || ((c.k & 2) && covered(c, v));
    case CK_COMPAT: {
      int n = 0;
      for (int k = 0; k < c.aw; ++k) n += in_vals(v[c.a0 + k], v, c.b0, c.bw) ? 1 : 0;
      return n >= c.k;
    }
    case CK_CONTAINS_U:
      for (int k = 0; k < c.bw; ++k)
        if (!in_vals(v[c.b0 + k], v, c.a0, c.aw)) return false;
      return true;
  }
  return false;
}

__device__ __forceinline__ bool eval_pair(const Theta& th, uint32_t* v, uint64_t j) {
  for (int k = 0; k < th.nr; ++k) v[th.nl + k] = th.col[th.nl + k][j];
  if (th.any) {
    for (int c = 0; c < th.nchk; ++c)
      if (eval_check(th.chk[c], v)) return true;
    return false;
  }
  for (int c = 0; c < th.nchk; ++c)
    if (!eval_check(th.chk[c], v)) return false;
  return true;
}

// Candidate right rows of left row i: [lo[i], lo[i] + cnt[i]) or all of them.
__device__ __forceinline__ void cand(const uint32_t* lo, const uint32_t* cnt, uint64_t nr, uint64_t i, uint64_t& b,
                                     uint64_t& e) {
  if (lo) {
    b = lo[i];
    e = b + cnt[i];
  } else {
    b = 0;
    e = nr;
  }
}

// One wave per left row (grid-stride over rows).
__global__ void __launch_bounds__(B) k_theta_count(Theta th, uint64_t nl, uint64_t nr, const uint32_t* lo,
                                                   const uint32_t* cnt, uint64_t* out_cnt) {
  uint32_t v[kMaxUni];
  const uint64_t waves = (uint64_t)gridDim.x * (B / 64);
  const int lane = __lane_id();
  for (uint64_t i = blockIdx.x * (uint64_t)(B / 64) + (threadIdx.x >> 6); i < nl; i += waves) {
    for (int k = 0; k < th.nl; ++k) v[k] = th.col[k][i];
    uint64_t b, e;
    cand(lo, cnt, nr, i, b, e);
    uint64_t n = 0;
    for (uint64_t j0 = b; j0 < e; j0 += 64) {
      const uint64_t j = j0 + lane;
      const bool keep = j < e && eval_pair(th, v, j);
      n += (uint64_t)__popcll(__ballot(keep));
    }
    if (lane == 0) out_cnt[i] = n;
  }
}

__global__ void __launch_bounds__(B) k_theta_write(Theta th, uint64_t nl, uint64_t nr, const uint32_t* lo,
                                                   const uint32_t* cnt, const uint64_t* off, uint32_t* out,
                                                   uint64_t cap) {
  uint32_t v[kMaxUni];
  const uint64_t waves = (uint64_t)gridDim.x * (B / 64);
  const int lane = __lane_id();
  const uint64_t lt = __lanemask_lt();
  for (uint64_t i = blockIdx.x * (uint64_t)(B / 64) + (threadIdx.x >> 6); i < nl; i += waves) {
    for (int k = 0; k < th.nl; ++k) v[k] = th.col[k][i];
    uint64_t b, e;
    cand(lo, cnt, nr, i, b, e);
    uint64_t pos = off[i];
    for (uint64_t j0 = b; j0 < e; j0 += 64) {
      const uint64_t j = j0 + lane;
      const bool keep = j < e && eval_pair(th, v, j);
      const uint64_t m = __ballot(keep);
      if (keep) {
        const uint64_t o = pos + (uint64_t)__popcll(m & lt);
        for (int c = 0; c < th.nout; ++c) out[(uint64_t)c * cap + o] = v[th.out[c]];
      }
      pos += (uint64_t)__popcll(m);
    }
  }
}

// keep[i] = no right row hits left row i.
__global__ void __launch_bounds__(B) k_theta_anti(Theta th, uint64_t nl, uint64_t nr, uint32_t* keep) {
  uint32_t v[kMaxUni];
  const uint64_t waves = (uint64_t)gridDim.x * (B / 64);
  const int lane = __lane_id();
  for (uint64_t i = blockIdx.x * (uint64_t)(B / 64) + (threadIdx.x >> 6); i < nl; i += waves) {
    for (int k = 0; k < th.nl; ++k) v[k] = th.col[k][i];
    bool hit = false;
    for (uint64_t j0 = 0; j0 < nr && !hit; j0 += 64) {
      const uint64_t j = j0 + lane;
      hit = __ballot(j < nr && eval_pair(th, v, j)) != 0;
    }
    if (lane == 0) keep[i] = hit ? 0u : 1u;
  }
}

// ---------------------------------------------------------------------------
// Schemas on the host
// ---------------------------------------------------------------------------
struct Member {
  int c0 = 0, w = 0;              // pair-row (or table) columns
  std::vector<int32_t> vars;      // sorted variable ids
};
struct Side {
  bool has_o = false;
  std::vector<int32_t> ovars;     // sorted
  std::vector<int> ocol;          // column of ovars[k]
  std::vector<Member> mem;
};

Side side_of(const Table& t, int base) {
  Side s;
  if (t.kind == DAS_TABLE_ORDERED) {
    s.has_o = true;
    for (int c = 0; c < t.ncols; ++c) {
      s.ovars.push_back(t.vars[c]);
      s.ocol.push_back(base + c);
    }
  } else if (t.kind == DAS_TABLE_UNORDERED) {
    Member m;
    m.c0 = base;
    m.w = t.ncols;
    m.vars.assign(t.vars, t.vars + t.ncols);
    s.mem.push_back(m);
  } else {
    int c = 0;
    for (; c < t.ncols && t.member[c] < 0; ++c) {
      s.ovars.push_back(t.vars[c]);
      s.ocol.push_back(base + c);
    }
    s.has_o = c > 0;
    while (c < t.ncols) {
      Member m;
      m.c0 = base + c;
      const int id = t.member[c];
      while (c < t.ncols && t.member[c] == id) {
        m.vars.push_back(t.vars[c]);
        ++c;
      }
      m.w = (int)m.vars.size();
      s.mem.push_back(m);
    }
  }
  return s;
}

bool subset(const std::vector<int32_t>& a, const std::vector<int32_t>& b) {   // a <= b, both sorted
  return std::includes(b.begin(), b.end(), a.begin(), a.end());
}
int n_common(const std::vector<int32_t>& a, const std::vector<int32_t>& b) {
  std::vector<int32_t> r;
  std::set_intersection(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(r));
  return (int)r.size();
}

struct Plan {
  Theta th{};
  bool never = false;             // a check that can never hold: empty result / nothing hit
  std::vector<std::pair<int, int>> eq;   // (left col, right col) equalities (candidate ranges)
  void add(const Check& c) {
    DAS_CHECK(th.nchk < kMaxChecks, DAS_E_UNSUPPORTED, "composite join: too many checks");
    th.chk[th.nchk++] = c;
  }
};

Check ck_member(uint8_t op, const Member& a, const std::vector<int>& ocols) {
  Check c;
  c.op = op;
  c.a0 = (uint8_t)a.c0;
  c.aw = (uint8_t)a.w;
  c.no = (uint8_t)ocols.size();
  for (size_t k = 0; k < ocols.size(); ++k) c.o[k] = (uint8_t)ocols[k];
  return c;
}

// Ordered part of a growing composite: sorted vars + pair-row columns.
struct OPart {
  bool has = false;
  std::vector<int32_t> vars;
  std::vector<int> col;
};

// _add_unordered_mapping (:329-336): contains_ordered against the current
// ordered part, compatible with every member so far; then append.
void add_unordered(Plan& p, const OPart& o, std::vector<Member>& mem, const Member& u) {
  if (o.has) {
    if (!subset(o.vars, u.vars)) p.never = true;
    else p.add(ck_member(CK_CONTAINS_O, u, o.col));
  }
  for (const Member& x : mem) {
    const int nsym = n_common(x.vars, u.vars);
    if (nsym == 0) continue;                   // nval >= 0 always holds
    Check c;
    c.op = CK_COMPAT;
    c.a0 = (uint8_t)x.c0;
    c.aw = (uint8_t)x.w;
    c.b0 = (uint8_t)u.c0;
    c.bw = (uint8_t)u.w;
    c.k = (uint8_t)nsym;
    p.add(c);
  }
  mem.push_back(u);
}

[[noreturn]] void attribute_error(const char* msg) { throw Error(DAS_E_ATTRIBUTE, msg); }

}  // namespace

// ---------------------------------------------------------------------------
// Join (And.matched :732-738 over the Assignment.join dispatch)
// ---------------------------------------------------------------------------
std::unique_ptr<Table> theta_join(Ctx& c, const Table& A, const Table& Bt, int no_overload) {
  DAS_CHECK(A.ncols + Bt.ncols <= kMaxUni, DAS_E_UNSUPPORTED, "composite join: too many columns");
  const Side sa = side_of(A, 0), sb = side_of(Bt, A.ncols);
  // dispatch: X is the composite that absorbs Y (:105-110, :203-209, :341-351)
  const Side *X, *Y;
  int ykind;
  if (A.kind == DAS_TABLE_ORDERED) { X = &sb; Y = &sa; ykind = DAS_TABLE_ORDERED; }
  else if (A.kind == DAS_TABLE_UNORDERED && Bt.kind == DAS_TABLE_COMPOSITE) { X = &sb; Y = &sa; ykind = DAS_TABLE_UNORDERED; }
  else { X = &sa; Y = &sb; ykind = Bt.kind; }
  Plan p;
  const char* raise = nullptr;
  OPart o;
  o.has = X->has_o;
  o.vars = X->ovars;
  o.col = X->ocol;
  std::vector<Member> mem = X->mem;
  if (ykind == DAS_TABLE_ORDERED || ykind == DAS_TABLE_COMPOSITE) {
    // _add_ordered_mapping (:316-327)
    if (!o.has) {
      o.has = Y->has_o;
      o.vars = Y->ovars;
      o.col = Y->ocol;
    } else if (!Y->has_o) {
      // OrderedAssignment.join(None) (:106): raised only once a pair is evaluated
      raise = "'NoneType' object has no attribute 'frozen'";
    } else {
      // OrderedAssignment._join_ordered (:119-139): equal shared values; the
      // NO_COVERING branch re-assigns every value (no_overload)
      std::map<int32_t, int> m;
      for (size_t k = 0; k < o.vars.size(); ++k) m[o.vars[k]] = o.col[k];
      for (size_t k = 0; k < Y->ovars.size(); ++k) {
        auto it = m.find(Y->ovars[k]);
        if (it != m.end()) {
          Check e;
          e.op = CK_EQ;
          e.no = 2;
          e.o[0] = (uint8_t)it->second;
          e.o[1] = (uint8_t)Y->ocol[k];
          p.add(e);
          const int l = it->second < A.ncols ? it->second : Y->ocol[k];
          const int r = it->second < A.ncols ? Y->ocol[k] : it->second;
          p.eq.push_back({l, r});
        } else {
          m[Y->ovars[k]] = Y->ocol[k];
        }
      }
      const bool cov = subset(o.vars, Y->ovars) || subset(Y->ovars, o.vars);
      o.vars.clear();
      o.col.clear();
      for (auto& kv : m) {
        o.vars.push_back(kv.first);
        o.col.push_back(kv.second);
      }
      if (no_overload && !cov) {
        Check d;
        d.op = CK_DISTINCT;
        d.no = (uint8_t)o.col.size();
        for (size_t k = 0; k < o.col.size(); ++k) d.o[k] = (uint8_t)o.col[k];
        p.add(d);
      }
    }
    // _check_ordered_viability (:290-305)
    if (o.has) {
      for (const Member& u : mem) {
        const bool can_contain = subset(o.vars, u.vars), can_cover = subset(u.vars, o.vars);
        if (!can_contain && !can_cover) { p.never = true; break; }
        Check v = ck_member(CK_VIABLE, u, o.col);
        v.k = (uint8_t)((can_contain ? 1 : 0) | (can_cover ? 2 : 0));
        p.add(v);
      }
    }
    if (ykind == DAS_TABLE_COMPOSITE)
      for (const Member& u : Y->mem) add_unordered(p, o, mem, u);   // _add_unordered_mappings
  } else {
    add_unordered(p, o, mem, Y->mem[0]);
  }
  // output schema: ordered part (sorted vars) then members in order
  int32_t vars[kMaxCols], member[kMaxCols];
  int nout = 0;
  DAS_CHECK(o.vars.size() + [&] { size_t w = 0; for (auto& u : mem) w += u.w; return w; }() <= (size_t)kMaxCols,
            DAS_E_UNSUPPORTED, "composite join: too many output columns");
  for (size_t k = 0; k < o.vars.size(); ++k) {
    vars[nout] = o.vars[k];
    member[nout] = -1;
    p.th.out[nout++] = (uint8_t)o.col[k];
  }
  for (size_t m = 0; m < mem.size(); ++m)
    for (int k = 0; k < mem[m].w; ++k) {
      vars[nout] = mem[m].vars[k];
      member[nout] = (int32_t)m;
      p.th.out[nout++] = (uint8_t)(mem[m].c0 + k);
    }
  p.th.nout = nout;
  if (A.nrows == 0 || Bt.nrows == 0) return new_table(c, DAS_TABLE_COMPOSITE, nout, vars, 0, member);
  if (raise) attribute_error(raise);
  if (p.never) return new_table(c, DAS_TABLE_COMPOSITE, nout, vars, 0, member);
  // candidate ranges on the shared ordered variables: sort the right side
  std::unique_ptr<Table> Bs;
  const Table* R = &Bt;
  DBuf<uint32_t> lo, cnt;
  if (!p.eq.empty()) {
    ColSet rk{}, lk{};
    rk.n = lk.n = (int)p.eq.size();
    for (int k = 0; k < rk.n; ++k) {
      lk.c[k] = A.col(p.eq[k].first);
      rk.c[k] = Bt.col(p.eq[k].second - A.ncols);
    }
    DBuf<uint32_t> perm(Bt.nrows, c.s);
    sort_perm(rk, Bt.nrows, perm.p, id_bits(c), c.s);
    Bs = gather_table(c, Bt, perm.p, Bt.nrows);
    R = Bs.get();
    for (int k = 0; k < rk.n; ++k) rk.c[k] = R->col(p.eq[k].second - A.ncols);
    lo.alloc(A.nrows, c.s);
    cnt.alloc(A.nrows, c.s);
    join_ranges(c, lk, A.nrows, rk, R->nrows, lo.p, cnt.p);
  }
  p.th.nl = A.ncols;
  p.th.nr = R->ncols;
  for (int k = 0; k < A.ncols; ++k) p.th.col[k] = A.col(k);
  for (int k = 0; k < R->ncols; ++k) p.th.col[A.ncols + k] = R->col(k);
  p.th.any = 0;
  const unsigned grid = grid_for(A.nrows, B / 64, 65535u * 4u);
  DBuf<uint64_t> n(A.nrows + 1, c.s), off(A.nrows + 1, c.s);
  {
    ProfScope ps(c, "k_theta_count", 4.0 * A.nrows * A.ncols + 4.0 * Bt.nrows * Bt.ncols);
    hipLaunchKernelGGL(k_theta_count, dim3(grid), dim3(B), 0, c.s, p.th, A.nrows, R->nrows, (const uint32_t*)lo.p,
                       (const uint32_t*)cnt.p, n.p);
    DAS_HIP(hipGetLastError());
  }
  const uint64_t total = scan_total<uint64_t>(SpanIn<uint64_t>{n.p}, A.nrows, off.p, c.s);
  auto out = new_table(c, DAS_TABLE_COMPOSITE, nout, vars, total, member);
  out->nrows = total;
  for (int k = 0; k < nout; ++k) {
    const int u = p.th.out[k];
    out->lo[k] = u < A.ncols ? A.lo[u] : Bt.lo[u - A.ncols];
    out->hi[k] = u < A.ncols ? A.hi[u] : Bt.hi[u - A.ncols];
  }
  if (total) {
    ProfScope ps(c, "k_theta_write", 4.0 * total * nout);
    hipLaunchKernelGGL(k_theta_write, dim3(grid), dim3(B), 0, c.s, p.th, A.nrows, R->nrows, (const uint32_t*)lo.p,
                       (const uint32_t*)cnt.p, (const uint64_t*)off.p, out->data, out->cap);
    DAS_HIP(hipGetLastError());
  }
  return out;
}

// ---------------------------------------------------------------------------
// Negation (And.matched :741-746): drop rows of A that some row of T hits
// ---------------------------------------------------------------------------
std::unique_ptr<Table> theta_antijoin(Ctx& c, const Table& A, const Table& T) {
  DAS_CHECK(A.ncols + T.ncols <= kMaxUni, DAS_E_UNSUPPORTED, "negation: too many columns");
  const Side sa = side_of(A, 0), st = side_of(T, A.ncols);
  // check_negation AttributeErrors (:117 on a composite negation, :359-360):
  // raised only once a row is actually checked
  if (A.nrows && T.nrows && T.kind == DAS_TABLE_COMPOSITE && A.kind != DAS_TABLE_UNORDERED)
    attribute_error(A.kind == DAS_TABLE_ORDERED ? "'CompositeAssignment' object has no attribute 'is_covered_by_ordered'"
                                                : "'CompositeAssignment' object has no attribute 'unordered_assignments'");
  Plan p;
  auto contains_u = [&](const Member& a, const Member& t) {
    if (!subset(t.vars, a.vars)) return;
    Check k;
    k.op = CK_CONTAINS_U;
    k.a0 = (uint8_t)a.c0;
    k.aw = (uint8_t)a.w;
    k.b0 = (uint8_t)t.c0;
    k.bw = (uint8_t)t.w;
    p.add(k);
  };
  if (A.kind == DAS_TABLE_ORDERED) {
    // OrderedAssignment.check_negation :112-117 -> negation.is_covered_by_ordered(self)
    if (T.kind == DAS_TABLE_UNORDERED && subset(st.mem[0].vars, sa.ovars))
      p.add(ck_member(CK_COVERED, st.mem[0], sa.ocol));
  } else if (A.kind == DAS_TABLE_UNORDERED) {
    // UnorderedAssignment.check_negation :211-217
    const Member& a = sa.mem[0];
    if (T.kind == DAS_TABLE_ORDERED) {
      if (subset(st.ovars, a.vars)) p.add(ck_member(CK_CONTAINS_O, a, st.ocol));
    } else {
      for (const Member& t : st.mem) contains_u(a, t);
    }
  } else {
    // CompositeAssignment.check_negation :353-362
    for (const Member& a : sa.mem) {
      if (T.kind == DAS_TABLE_ORDERED) {
        if (subset(st.ovars, a.vars)) p.add(ck_member(CK_CONTAINS_O, a, st.ocol));
      } else if (T.kind == DAS_TABLE_UNORDERED) {
        contains_u(a, st.mem[0]);
      }
    }
  }
  if (p.th.nchk == 0 || T.nrows == 0 || A.nrows == 0) {   // nothing can hit
    DBuf<uint32_t> idx(A.nrows ? A.nrows : 1, c.s);
    iota(idx.p, A.nrows, c.s);
    return gather_table(c, A, idx.p, A.nrows);
  }
  p.th.nl = A.ncols;
  p.th.nr = T.ncols;
  for (int k = 0; k < A.ncols; ++k) p.th.col[k] = A.col(k);
  for (int k = 0; k < T.ncols; ++k) p.th.col[A.ncols + k] = T.col(k);
  p.th.any = 1;
  DBuf<uint32_t> keep(A.nrows, c.s);
  {
    ProfScope ps(c, "k_theta_anti", 4.0 * A.nrows * A.ncols + 4.0 * T.nrows * T.ncols);
    hipLaunchKernelGGL(k_theta_anti, dim3(grid_for(A.nrows, B / 64, 65535u * 4u)), dim3(B), 0, c.s, p.th, A.nrows,
                       T.nrows, keep.p);
    DAS_HIP(hipGetLastError());
  }
  return compact_table(c, A, keep.p);
}

// ---------------------------------------------------------------------------
// Set identity: canonical keys, dedup, difference
// ---------------------------------------------------------------------------
namespace {

struct KeyGroup {               // one member variable set of a class
  std::vector<int32_t> vars;
  int cap = 0;                  // max members with these variables in one table
  int base = 0;                 // first key column
};

struct KeyClass {
  std::vector<int32_t> ovars;
  std::vector<KeyGroup> groups;  // sorted by vars
  int ncols = 0;
};

// Per table: where each key column comes from.
struct KeySpec {
  const uint32_t* col[kMaxCols];
  uint32_t flag;                  // 1 for a pure UnorderedAssignment
  int no;                         // ordered columns: table cols 0..no) -> key cols 1..no]
  int ng;
  struct G {
    int base, cap, w, n;          // key base col, capacity (tuples), tuple width, tuples in this table
    uint8_t src[8];               // first table column of each tuple
  } g[8];
};

std::vector<int32_t> ovars_of(const Table& t) {
  std::vector<int32_t> v;
  if (t.kind == DAS_TABLE_ORDERED) v.assign(t.vars, t.vars + t.ncols);
  else if (t.kind == DAS_TABLE_COMPOSITE)
    for (int c = 0; c < t.ncols && t.member[c] < 0; ++c) v.push_back(t.vars[c]);
  return v;
}

// canonical key of every row: flag | ordered values | per group: member value
// tuples sorted, equal pairs cancelled (XOR identity), padded with kNone
__global__ void __launch_bounds__(B) k_identity_key(KeySpec ks, uint64_t n, uint32_t* const* key, uint64_t kcap,
                                                    uint64_t row0) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = row0 + i;
    (void)kcap;
    key[0][r] = ks.flag;
    for (int k = 0; k < ks.no; ++k) key[1 + k][r] = ks.col[k][i];
    for (int g = 0; g < ks.ng; ++g) {
      const auto& G = ks.g[g];
      uint32_t t[8][8];
      int ord[8];
      for (int m = 0; m < G.n; ++m) {
        ord[m] = m;
        for (int k = 0; k < G.w; ++k) t[m][k] = ks.col[G.src[m] + k][i];
      }
      auto less = [&](int a, int b) {
        for (int k = 0; k < G.w; ++k)
          if (t[a][k] != t[b][k]) return t[a][k] < t[b][k];
        return false;
      };
      for (int m = 1; m < G.n; ++m) {          // insertion sort of tuple indices
        const int x = ord[m];
        int j = m - 1;
        while (j >= 0 && less(x, ord[j])) { ord[j + 1] = ord[j]; --j; }
        ord[j + 1] = x;
      }
      int st[8], top = 0;                      // cancel equal pairs (stack)
      for (int m = 0; m < G.n; ++m) {
        if (top > 0 && !less(st[top - 1], ord[m]) && !less(ord[m], st[top - 1])) --top;
        else st[top++] = ord[m];
      }
      for (int m = 0; m < G.cap; ++m)
        for (int k = 0; k < G.w; ++k) key[G.base + m * G.w + k][r] = m < top ? t[st[m]][k] : kNone;
    }
  }
}

struct WideCols {
  const uint32_t* c[kMaxKeyCols];
  int n;
};

__device__ __forceinline__ int cmp_wide(const WideCols& a, uint64_t i, const WideCols& b, uint64_t j) {
  for (int c = 0; c < a.n; ++c) {
    const uint32_t x = a.c[c][i], y = b.c[c][j];
    if (x != y) return x < y ? -1 : 1;
  }
  return 0;
}

// first[k] for the sorted order perm: keep the earliest input row of each key
__global__ void k_first_of_run(WideCols key, const uint32_t* perm, uint64_t n, uint32_t* keep) {
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x)
    keep[perm[k]] = (k == 0 || cmp_wide(key, perm[k - 1], key, perm[k]) != 0) ? 1u : 0u;
}

// keep[i] = key row i of `a` absent from the rows of `b` sorted by perm
__global__ void k_absent(WideCols a, uint64_t na, WideCols b, const uint32_t* perm, uint64_t nb, uint32_t* keep) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < na; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t lo = 0, hi = nb;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (cmp_wide(b, perm[mid], a, i) < 0) lo = mid + 1; else hi = mid;
    }
    keep[i] = (lo < nb && cmp_wide(b, perm[lo], a, i) == 0) ? 0u : 1u;
  }
}

// Groups tables into identity classes (equal ordered variable sets) and lays
// out the key columns of each class.
std::map<std::vector<int32_t>, KeyClass> classes_of(const std::vector<const Table*>& ts) {
  std::map<std::vector<int32_t>, KeyClass> cls;
  for (const Table* t : ts) {
    KeyClass& k = cls[ovars_of(*t)];
    k.ovars = ovars_of(*t);
    if (t->kind == DAS_TABLE_ORDERED) continue;
    const Side s = side_of(*t, 0);
    std::map<std::vector<int32_t>, int> cnt;
    for (const Member& m : s.mem) cnt[m.vars]++;
    for (auto& kv : cnt) {
      auto it = std::find_if(k.groups.begin(), k.groups.end(), [&](const KeyGroup& g) { return g.vars == kv.first; });
      if (it == k.groups.end()) {
        KeyGroup g;
        g.vars = kv.first;
        g.cap = kv.second;
        k.groups.push_back(g);
      } else {
        it->cap = std::max(it->cap, kv.second);
      }
    }
  }
  for (auto& kv : cls) {
    KeyClass& k = kv.second;
    std::sort(k.groups.begin(), k.groups.end(), [](const KeyGroup& a, const KeyGroup& b) { return a.vars < b.vars; });
    int col = 1 + (int)k.ovars.size();
    DAS_CHECK(k.groups.size() <= 8, DAS_E_UNSUPPORTED, "set identity: too many member variable sets");
    for (KeyGroup& g : k.groups) {
      DAS_CHECK(g.cap <= 8 && g.vars.size() <= 8, DAS_E_UNSUPPORTED, "set identity: member too wide");
      g.base = col;
      col += g.cap * (int)g.vars.size();
    }
    DAS_CHECK(col <= kMaxKeyCols, DAS_E_UNSUPPORTED, "set identity: key too wide");
    k.ncols = col;
  }
  return cls;
}

// Key columns of tables ts (all of class k) stacked: returns the key buffer.
DBuf<uint32_t> make_keys(Ctx& c, const KeyClass& k, const std::vector<const Table*>& ts, uint64_t total,
                         WideCols& wc) {
  DBuf<uint32_t> buf((uint64_t)k.ncols * (total ? total : 1), c.s);
  std::vector<uint32_t*> cols(k.ncols);
  for (int j = 0; j < k.ncols; ++j) cols[j] = buf.p + (uint64_t)j * total;
  DBuf<uint32_t*> dcols(k.ncols, c.s);
  DAS_HIP(hipMemcpyAsync(dcols.p, cols.data(), sizeof(uint32_t*) * k.ncols, hipMemcpyHostToDevice, c.s));
  uint64_t row0 = 0;
  for (const Table* t : ts) {
    KeySpec ks{};
    ks.flag = t->kind == DAS_TABLE_UNORDERED ? 1u : 0u;
    for (int j = 0; j < t->ncols; ++j) ks.col[j] = t->col(j);
    const Side s = side_of(*t, 0);
    ks.no = (int)s.ovars.size();
    ks.ng = (int)k.groups.size();
    for (int g = 0; g < ks.ng; ++g) {
      auto& G = ks.g[g];
      G.base = k.groups[g].base;
      G.cap = k.groups[g].cap;
      G.w = (int)k.groups[g].vars.size();
      G.n = 0;
      for (const Member& m : s.mem)
        if (m.vars == k.groups[g].vars) G.src[G.n++] = (uint8_t)m.c0;
    }
    if (t->nrows) {
      hipLaunchKernelGGL(k_identity_key, dim3(grid_for(t->nrows, B)), dim3(B), 0, c.s, ks, t->nrows,
                         (uint32_t* const*)dcols.p, total, row0);
      DAS_HIP(hipGetLastError());
    }
    row0 += t->nrows;
  }
  wc.n = k.ncols;
  for (int j = 0; j < k.ncols; ++j) wc.c[j] = cols[j];
  return buf;
}

// stable sort permutation of stacked key rows
void sort_keys(Ctx& c, const WideCols& wc, uint64_t n, uint32_t* perm) {
  iota(perm, n, c.s);
  if (n <= 1) return;
  DBuf<uint32_t> kk(n, c.s);
  for (int j = wc.n - 1; j >= 0; --j) {
    gather_u32(wc.c[j], perm, kk.p, n, c.s);
    radix_sort_pairs<uint32_t>(kk.p, perm, n, 0, 32, c.s);
  }
}

}  // namespace

std::vector<std::unique_ptr<Table>> set_dedup(Ctx& c, const Table* const* ts, int n) {
  std::vector<std::unique_ptr<Table>> out(n);
  std::vector<const Table*> all(ts, ts + n);
  auto cls = classes_of(all);
  for (auto& kv : cls) {
    std::vector<const Table*> mine;
    std::vector<int> idx;
    uint64_t total = 0;
    for (int i = 0; i < n; ++i)
      if (ovars_of(*ts[i]) == kv.first) {
        mine.push_back(ts[i]);
        idx.push_back(i);
        total += ts[i]->nrows;
      }
    WideCols wc{};
    DBuf<uint32_t> keys = make_keys(c, kv.second, mine, total, wc);
    DBuf<uint32_t> perm(total ? total : 1, c.s), keep(total ? total : 1, c.s);
    if (total) {
      sort_keys(c, wc, total, perm.p);
      hipLaunchKernelGGL(k_first_of_run, dim3(grid_for(total, B)), dim3(B), 0, c.s, wc, (const uint32_t*)perm.p,
                         total, keep.p);
      DAS_HIP(hipGetLastError());
    }
    uint64_t row0 = 0;
    for (size_t m = 0; m < mine.size(); ++m) {
      out[idx[m]] = compact_table(c, *mine[m], keep.p + row0);
      row0 += mine[m]->nrows;
    }
  }
  return out;
}

std::vector<std::unique_ptr<Table>> set_minus(Ctx& c, const Table* const* a, int na, const Table* const* b, int nb) {
  std::vector<std::unique_ptr<Table>> out(na);
  std::vector<const Table*> all(a, a + na);
  all.insert(all.end(), b, b + nb);
  auto cls = classes_of(all);
  for (auto& kv : cls) {
    std::vector<const Table*> ma, mb;
    std::vector<int> idx;
    uint64_t ta = 0, tb = 0;
    for (int i = 0; i < na; ++i)
      if (ovars_of(*a[i]) == kv.first) {
        ma.push_back(a[i]);
        idx.push_back(i);
        ta += a[i]->nrows;
      }
    if (ma.empty()) continue;
    for (int i = 0; i < nb; ++i)
      if (ovars_of(*b[i]) == kv.first) {
        mb.push_back(b[i]);
        tb += b[i]->nrows;
      }
    WideCols wa{}, wb{};
    DBuf<uint32_t> ka = make_keys(c, kv.second, ma, ta, wa);
    DBuf<uint32_t> kb = make_keys(c, kv.second, mb, tb, wb);
    DBuf<uint32_t> perm(tb ? tb : 1, c.s), keep(ta ? ta : 1, c.s);
    if (ta) {
      if (tb) sort_keys(c, wb, tb, perm.p);
      hipLaunchKernelGGL(k_absent, dim3(grid_for(ta, B)), dim3(B), 0, c.s, wa, ta, wb, (const uint32_t*)perm.p, tb,
                         keep.p);
      DAS_HIP(hipGetLastError());
    }
    uint64_t row0 = 0;
    for (size_t m = 0; m < ma.size(); ++m) {
      out[idx[m]] = compact_table(c, *ma[m], keep.p + row0);
      row0 += ma[m]->nrows;
    }
  }
  return out;
}

}  // namespace das
