// Whole-expression evaluation in one C-ABI call (das_plan_execute).
//
// The Python matcher (das_amd/pattern_matcher) lowers an And / Or / Not tree
// of ordered, flat Links into a prefix-order node array: grounded nodes and
// links are settled on the host (node_exists / link_exists become CONST
// terms), every Link with a variable is one das_link_scan_t.  This file folds
// that tree with the same rules as the Python classes -- which restate the
// reference's -- so a query costs one host call instead of one per operator:
//   And.matched  pattern_matcher.py:705-748  (failing term -> False; empty
//                term skipped; Not terms -> forbidden; reset-on-empty; index
//                join of a Link term against the running result; negation
//                filter; set semantics)
//   Or.matched   :644-687  (union of matched terms; Not terms -> And of their
//                inner terms minus the union, negation flag set)
//   Not.matched  :627-631
// Tables of one relation are kept one per schema, rows distinct, empty tables
// dropped (das_amd.database.hip_db.Relation).
#include <functional>
#include <memory>
#include <vector>

#include "das_internal.h"

namespace das {
namespace {

using TablePtr = std::unique_ptr<Table>;

struct Rel {
  std::vector<TablePtr> t;
  bool partial = false;     // sharded: this shard's part of a relation split across shards
  bool nonempty() const {
    for (auto& x : t)
      if (x->nrows) return true;
    return false;
  }
  void push(TablePtr x) {
    if (x && x->nrows) t.push_back(std::move(x));
  }
};

struct Res {
  bool matched = false;
  Rel rel;
  bool neg = false;
};

bool same_schema(const Table& a, const Table& b) {
  if (a.kind != b.kind || a.ncols != b.ncols) return false;
  for (int i = 0; i < a.ncols; ++i)
    if (a.vars[i] != b.vars[i] || (a.kind == DAS_TABLE_COMPOSITE && a.member[i] != b.member[i])) return false;
  return true;
}

struct Exec;
void split_and(const Exec& ex, const std::vector<uint32_t>& terms, std::vector<const das_plan_node_t*>& pos,
               std::vector<const das_plan_node_t*>& neg);

struct Exec {
  Ctx& c;
  const das_plan_node_t* nd;
  uint32_t n;
  int no_overload;
  // sharded mode (das_plan_execute_sharded): INPUT leaves, partial relations
  const std::vector<const Table*>* inputs = nullptr;
  std::vector<uint8_t>* checks = nullptr;
  bool sharded() const { return inputs != nullptr; }
  // Emptiness as the fold sees it.  A partial relation is assumed non-empty
  // (its global emptiness needs every shard); the caller verifies the
  // assumption afterwards from the `checks` bits of all shards.
  bool ne(const Rel& r) const { return (sharded() && r.partial) || r.nonempty(); }

  uint32_t next(uint32_t i) const {
    DAS_CHECK(i < n, DAS_E_INVALID, "plan: truncated node array");
    const das_plan_node_t& x = nd[i];
    if (x.op == DAS_PLAN_LINK || x.op == DAS_PLAN_CONST || x.op == DAS_PLAN_INPUT || x.op == DAS_PLAN_TEMPLATE)
      return i + 1;
    if (x.op == DAS_PLAN_NOT) return next(i + 1);
    DAS_CHECK(x.op == DAS_PLAN_AND || x.op == DAS_PLAN_OR || x.op == DAS_PLAN_TVM, DAS_E_INVALID,
              "plan: bad node op");
    uint32_t j = i + 1;
    for (uint32_t k = 0; k < x.nchild; ++k) j = next(j);
    return j;
  }

  std::vector<uint32_t> children(uint32_t i) const {
    std::vector<uint32_t> out;
    uint32_t j = i + 1;
    for (uint32_t k = 0; k < nd[i].nchild; ++k) {
      out.push_back(j);
      j = next(j);
    }
    return out;
  }

  // rel_normalize: one table per schema (first-seen order), rows distinct
  Rel normalize(Rel a) {
    std::vector<std::vector<TablePtr>> groups;
    for (auto& x : a.t) {
      bool put = false;
      for (auto& g : groups)
        if (same_schema(*g[0], *x)) {
          g.push_back(std::move(x));
          put = true;
          break;
        }
      if (!put) {
        groups.emplace_back();
        groups.back().push_back(std::move(x));
      }
    }
    Rel out;
    out.partial = a.partial;
    for (auto& g : groups) {
      if (g.size() == 1) {
        out.push(std::move(g[0]));
        continue;
      }
      std::vector<const Table*> ts;
      for (auto& x : g) ts.push_back(x.get());
      auto cat = concat(c, ts.data(), (int)ts.size());
      out.push(dedup(c, *cat));
    }
    return out;
  }

  Rel join_rel(const Rel& a, const Rel& b) {
    Rel out;
    out.partial = a.partial || b.partial;
    for (auto& ta : a.t)
      for (auto& tb : b.t) out.push(join(c, *ta, *tb, no_overload));
    return out;
  }

  Rel antijoin_rel(Rel r, const Rel& f) {
    for (auto& ft : f.t) {
      Rel nx;
      nx.partial = r.partial;
      for (auto& t : r.t) nx.push(antijoin(c, *t, *ft));
      r = std::move(nx);
    }
    return r;
  }

  Rel minus_rel(Rel a, const Rel& b) {
    Rel out;
    out.partial = a.partial;
    for (auto& t : a.t) {
      TablePtr cur = std::move(t);
      for (auto& f : b.t)
        if (cur && cur->nrows && same_schema(*cur, *f)) cur = antijoin(c, *cur, *f);
      out.push(std::move(cur));
    }
    return out;
  }

  Res eval(uint32_t i) {
    const das_plan_node_t& x = nd[i];
    static const char* const kOp[] = {"?", "LINK", "CONST", "NOT", "AND", "OR", "INPUT", "TEMPLATE", "TVM"};
    if (trace_on()) trace_mark("node", x.op <= 8 ? kOp[x.op] : "?");
    Res r;
    switch (x.op) {
      case DAS_PLAN_CONST:
        r.matched = x.value != 0;
        return r;
      case DAS_PLAN_LINK: {
        DAS_CHECK(x.scan.ordered, DAS_E_UNSUPPORTED, "plan: unordered Link terms take the host path");
        TablePtr t = scan_link(c, x.scan);
        if (x.dedup && t->nrows) t = dedup(c, *t);
        r.rel.push(std::move(t));
        r.rel.partial = sharded();        // this shard's links only
        r.matched = ne(r.rel);
        return r;
      }
      case DAS_PLAN_INPUT: {
        // a caller's table (e.g. a term's rows gathered from every shard):
        // read in place, never freed here
        DAS_CHECK(sharded() && x.value < inputs->size() && (*inputs)[x.value], DAS_E_INVALID,
                  "plan: INPUT leaf without a table");
        auto v = std::make_unique<Table>(*(*inputs)[x.value]);
        v->view = true;
        r.rel.push(std::move(v));
        r.matched = r.rel.nonempty();
        return r;
      }
      case DAS_PLAN_TEMPLATE: {
        // LinkTemplate.matched (:603-614): the links of one composite type,
        // every target a typed variable (scan_template)
        DAS_CHECK(!sharded(), DAS_E_UNSUPPORTED, "plan: LinkTemplate terms are not sharded");
        das_template_scan_t q{};
        q.ctype_id = x.scan.type_id;
        q.arity = x.scan.arity;
        for (int p = 0; p < 8; ++p) q.var[p] = x.scan.var[p];
        q.ordered = x.scan.ordered;
        q.no_overload = x.scan.no_overload;
        TablePtr t = scan_template(c, q);
        if (x.dedup && t->nrows) t = dedup(c, *t);
        r.rel.push(std::move(t));
        r.matched = r.rel.nonempty();
        return r;
      }
      case DAS_PLAN_TVM: {
        // Link._typed_variable_matched (:491-500): every target matched in
        // order on the same answer (all() stops at the first failure); the
        // answer is the last one a target wrote (a template, a nested Link)
        uint32_t j = i + 1;
        Rel last;
        for (uint32_t k = 0; k < x.nchild; ++k) {
          Res s = eval(j);
          if (!s.matched) return Res{};
          const int32_t o = nd[j].op;
          // (sharded: a gathered template / Link leaf arrives as an INPUT leaf)
          if (o == DAS_PLAN_TEMPLATE || o == DAS_PLAN_TVM || o == DAS_PLAN_LINK || o == DAS_PLAN_INPUT)
            last = std::move(s.rel);
          j = next(j);
        }
        r.rel = std::move(last);
        r.matched = true;
        return r;
      }
      case DAS_PLAN_NOT:
        r = eval(i + 1);
        r.neg = !r.neg;
        r.matched = true;
        return r;
      case DAS_PLAN_AND:
        return eval_and(children(i), i == 0);
      case DAS_PLAN_OR:
        return eval_or(children(i));
      default:
        throw Error(DAS_E_INVALID, "plan: bad node op");
    }
  }

  // The variable of a Link term with exactly one variable position and every
  // other target grounded (its scan is one column of distinct keys), or -1.
  int32_t one_var(uint32_t ti) const {
    const das_plan_node_t& x = nd[ti];
    // sharded: only a replicated (INPUT) term is a whole key set to filter by
    if (x.op != (sharded() ? DAS_PLAN_INPUT : DAS_PLAN_LINK) || !x.scan.ordered || x.scan.emit_link ||
        x.scan.type_id == kNone)
      return -1;
    int32_t v = -1;
    for (uint32_t p = 0; p < x.scan.arity && p < 8; ++p) {
      if (x.scan.target[p] != kNone) continue;
      if (x.scan.var[p] < 0 || v >= 0) return -1;
      v = x.scan.var[p];
    }
    return v;
  }

  // End (exclusive) of the run of terms from k that semi_join_multi can fold
  // at once: Link terms with one variable, the same one, bound by the running
  // result's single table of more than 2^20 rows (smaller results take the
  // index join term by term).  DAS_SEMI_MULTI=1 drops the size floor, 0
  // disables the run (tests).
  size_t semi_run(const std::vector<uint32_t>& terms, size_t k, const Rel& acc) const {
    const char* f = std::getenv("DAS_SEMI_MULTI");
    if ((f && f[0] == '0') || acc.t.size() != 1) return k;
    const Table& a = *acc.t[0];
    if (a.kind != DAS_TABLE_ORDERED || (!(f && f[0] == '1') && a.nrows <= (1ull << 20))) return k;
    const int32_t v = one_var(terms[k]);
    bool bound = false;
    for (int i = 0; i < a.ncols; ++i) bound |= a.vars[i] == v;
    if (v < 0 || !bound) return k;
    size_t e = k + 1;
    while (e < terms.size() && one_var(terms[e]) == v) ++e;
    return e;
  }

  // And's fold of one positive term into the running result; false when the
  // term fails the And (:712-713).
  // The And's first two positive Link terms when the second one's rows are
  // few against the first one's: instead of joining the first term's scan
  // (probe, e.g. 2*10^7 Member rows) with the second's rows (build), the
  // second's rows look their key up in the FIRST term's pattern index and
  // expand its contiguous row ranges (index_join): the first term's rows
  // without a partner are never read, and each output's fresh column comes
  // from a contiguous P row.  Same rows as the join (a two-term join is
  // symmetric, and an empty join empties acc either way), other row order.
  // DAS_REV_IJ=0 off, =1 without the 2^16-row floor (tests).
  TablePtr reverse_ij(int64_t t0, const Rel& acc, const Rel& s) {
    const char* f = std::getenv("DAS_REV_IJ");
    if (t0 < 0 || sharded() || (f && f[0] == '0')) return nullptr;
    const das_plan_node_t& a = nd[t0];
    if (a.op != DAS_PLAN_LINK || !a.index_join || a.dedup || acc.t.size() != 1 || s.t.size() != 1) return nullptr;
    const Table& big = *acc.t[0];
    const Table& small = *s.t[0];
    if (small.kind != DAS_TABLE_ORDERED || !small.nrows || 4 * small.nrows > big.nrows) return nullptr;
    if (!(f && f[0] == '1') && big.nrows < (1ull << 16)) return nullptr;
    return index_join(c, small, a.ij);
  }

  // acc_term: the Link term whose scan alone is acc (-1: acc is anything else)
  bool step(uint32_t ti, Rel& acc, bool& have, std::vector<Rel>& forbidden, int64_t& acc_term) {
    const das_plan_node_t& x = nd[ti];
    if (have && x.op == DAS_PLAN_LINK && x.index_join && ne(acc)) {
      // the term's rows looked up from the running result's keys; an empty
      // result takes the scan path, which tells a failing term (And ->
      // False) from an empty join (reset-on-empty)
      Rel r;
      r.partial = sharded();              // looked up in this shard's index
      bool ok = true;
      for (auto& t : acc.t) {
        auto j = index_join(c, *t, x.ij);
        if (!j) {
          ok = false;
          break;
        }
        r.push(std::move(j));
      }
      if (ok && ne(r)) {
        acc = std::move(r);
        acc_term = -1;
        return true;
      }
    }
    Res s = eval(ti);
    if (!s.matched) return false;
    if (!ne(s.rel)) return true;
    if (s.neg) {
      forbidden.push_back(std::move(s.rel));
      return true;
    }
    if (!have || !ne(acc)) {
      acc = std::move(s.rel);
      have = true;
      acc_term = x.op == DAS_PLAN_LINK ? (int64_t)ti : -1;
    } else {
      TablePtr r = reverse_ij(acc_term, acc, s.rel);
      if (r) {
        acc = Rel{};
        acc.push(std::move(r));
      } else {
        acc = join_rel(acc, s.rel);
      }
      acc_term = -1;
    }
    return true;
  }

  // End (exclusive) of the one-variable filter terms that follow the
  // index-joined Link term k on one of its fresh variables (*v), or k.  The
  // running result must have more than 4096 rows (DAS_SEMI_MULTI as above).
  size_t filt_run(const std::vector<uint32_t>& terms, size_t k, const Table& a, int32_t& v) const {
    const char* f = std::getenv("DAS_SEMI_MULTI");
    // DAS_FILT_EXPAND=0 (A/B): the join written out, then filtered by the
    // key-set intersection (semi_join_multi) instead of the filtered expansion
    const char* fx = std::getenv("DAS_FILT_EXPAND");
    if ((f && f[0] == '0') || (fx && fx[0] == '0') || a.kind != DAS_TABLE_ORDERED ||
        (!(f && f[0] == '1') && a.nrows <= 4096) || k + 1 >= terms.size())
      return k;
    v = one_var(terms[k + 1]);
    if (v < 0) return k;
    const das_link_scan_t& q = nd[terms[k]].ij;
    bool fresh = false;
    for (uint32_t p = 0; p < q.arity && p < 8; ++p) fresh |= q.target[p] == kNone && q.var[p] == v;
    for (int i = 0; i < a.ncols; ++i) fresh &= a.vars[i] != v;
    if (!fresh) return k;
    size_t e = k + 2;
    while (e < terms.size() && one_var(terms[e]) == v) ++e;
    return e;
  }

  Res eval_and(const std::vector<uint32_t>& terms, bool root = false) {
    Res out;
    if (terms.empty()) return out;
    Rel acc;
    bool have = false;
    std::vector<Rel> forbidden;
    std::vector<uint32_t> anti;        // Not(Link) terms applied as anti index joins
    uint32_t skip = 0;                 // positive terms the fused chain already folded into acc
    const bool top = checks && root;
    auto log = [&](size_t n_terms) {   // sharded: acc's local emptiness after each positive term
      if (top)
        for (size_t j = 0; j < n_terms; ++j) checks->push_back(acc.nonempty() ? 1 : 0);
    };
    if (!sharded()) {
      // the leading Link terms of the And (and its Not(Link) filters): one
      // fused launch while the running result stays small
      std::vector<const das_plan_node_t*> pos, neg;
      split_and(*this, terms, pos, neg);
      bool m = false;
      TablePtr t;
      const int r = fused_and(c, pos, neg, no_overload, m, t, &skip);
      if (r == 1) {
        out.matched = m;
        if (m) out.rel.push(std::move(t));
        return out;
      }
      if (r == 2) {
        // the chain folded the first `skip` Link terms: continue from there
        acc.push(std::move(t));
        have = true;
      } else {
        skip = 0;
      }
    }
    uint32_t seen = 0;                 // Link / other positive terms met so far
    int64_t acc_term = -1;             // step(): the Link term whose scan alone is acc
    for (size_t k = 0; k < terms.size(); ++k) {
      const uint32_t ti = terms[k];
      const das_plan_node_t& x = nd[ti];
      if (!sharded() && x.op == DAS_PLAN_NOT && nd[ti + 1].op == DAS_PLAN_LINK && nd[ti + 1].index_join) {
        // Not.matched is always True and its rows only ever filter the final
        // result (:720-724, :741-746): instead of scanning the term, each
        // result row's link is looked up in the index at the end
        anti.push_back(ti + 1);
        continue;
      }
      if (x.op == DAS_PLAN_NOT) {
        // a negated term: its rows join `forbidden` (no fold of acc)
        if (!step(ti, acc, have, forbidden, acc_term)) return Res{};
        continue;
      }
      if (seen++ < skip) continue;
      if (have && ne(acc)) {
        const size_t e = semi_run(terms, k, acc);
        if (e >= k + 2) {
          // consecutive one-variable terms on one variable of a large running
          // result: each term scanned (a failing term fails the And,
          // :712-713), then ONE filter by the intersection of their key sets
          std::vector<Rel> rs;
          for (size_t j = k; j < e; ++j) {
            Res s = eval(terms[j]);
            if (!s.matched) return Res{};
            rs.push_back(std::move(s.rel));
          }
          std::vector<const Table*> qs;
          for (auto& r : rs) qs.push_back(r.t[0].get());
          TablePtr f = semi_join_multi(c, *acc.t[0], qs);
          const bool part = acc.partial;
          if (f && (f->nrows || (sharded() && part))) {
            // non-empty: every prefix of the term-by-term fold is non-empty
            // too (the fold's rows project onto each prefix), so no
            // reset-on-empty step was skipped and the rows are the same
            acc = Rel{};
            acc.partial = part;
            acc.push(std::move(f));
          } else {
            for (auto& r : rs) acc = ne(acc) ? join_rel(acc, r) : std::move(r);
          }
          seen += (uint32_t)(e - k - 1);
          log(e - k);
          k = e - 1;
          acc_term = -1;
          continue;
        }
      }
      if (have && x.op == DAS_PLAN_LINK && x.index_join && acc.t.size() == 1 && acc.nonempty()) {
        int32_t v = -1;
        const size_t e = filt_run(terms, k, *acc.t[0], v);
        if (e >= k + 2) {
          // an index-joined term whose fresh variable the next one-variable
          // terms filter (the hub And's T1(V1,V2) | T2(V2,h1) T3(V2,h0)):
          // the filter terms are scanned (a failing term fails the And), and
          // the join is expanded with their key-set intersection applied
          std::vector<Rel> rs;
          for (size_t j = k + 1; j < e; ++j) {
            Res s = eval(terms[j]);
            if (!s.matched) return Res{};
            rs.push_back(std::move(s.rel));
          }
          std::vector<const Table*> qs;
          for (auto& r : rs) qs.push_back(r.t[0].get());
          TablePtr f = index_join_filtered(c, *acc.t[0], x.ij, v, qs);
          if (f && (f->nrows || sharded())) {
            // non-empty: no prefix of the term-by-term fold was empty (see
            // semi_join_multi above), so the rows are the fold's
            acc = Rel{};
            acc.partial = sharded();      // expanded through this shard's index
            acc.push(std::move(f));
          } else {
            if (!step(ti, acc, have, forbidden, acc_term)) return Res{};
            for (auto& r : rs) acc = ne(acc) ? join_rel(acc, r) : std::move(r);
          }
          seen += (uint32_t)(e - k - 1);
          log(e - k);
          k = e - 1;
          acc_term = -1;
          continue;
        }
      }
      if (!step(ti, acc, have, forbidden, acc_term)) return Res{};
      log(1);
    }
    for (auto& f : forbidden)
      if (acc.nonempty()) acc = antijoin_rel(std::move(acc), f);
    for (uint32_t li : anti) {
      if (!acc.nonempty()) break;
      Rel nx;
      for (auto& t : acc.t) {
        // a table that does not bind every variable of the term: no row is
        // covered by a negated row (check_negation, :112-117) -- kept whole
        auto r = anti_index_join(c, *t, nd[li].ij);
        nx.push(r ? std::move(r) : std::move(t));
      }
      acc = std::move(nx);
    }
    out.rel = normalize(std::move(acc));
    out.matched = out.rel.nonempty();
    return out;
  }

  Res eval_or(const std::vector<uint32_t>& terms) {
    Res out;
    if (terms.empty()) return out;
    if (!sharded()) {
      // an Or of Links of one schema: scans and union in one launch
      std::vector<const das_plan_node_t*> links;
      for (uint32_t ti : terms) links.push_back(&nd[ti]);
      bool m = false;
      TablePtr t;
      if (fused_or(c, links, no_overload, m, t)) {
        out.matched = m;
        if (m) out.rel.push(std::move(t));
        return out;
      }
    }
    Rel uni;
    bool any = false;
    std::vector<uint32_t> negated;
    for (uint32_t ti : terms) {
      if (nd[ti].op == DAS_PLAN_NOT) {
        negated.push_back(ti + 1);
        continue;
      }
      Res s = eval(ti);
      if (!s.matched) continue;
      any = true;
      // (the union is normalised once at the end: the same set as after
      // every term, one dedup per schema instead of one per term)
      for (auto& t : s.rel.t) uni.push(std::move(t));
    }
    uni = normalize(std::move(uni));
    if (!negated.empty()) {
      Res sub = eval_and(negated);
      out.rel = minus_rel(std::move(sub.rel), uni);
      out.neg = true;
    } else {
      out.rel = std::move(uni);
    }
    out.matched = any;
    return out;
  }
};

struct Views {                          // scans may return index views while plans run
  Ctx& c;
  explicit Views(Ctx& cc) : c(cc) {
    // default (1): every predicate-free scan of consecutive index columns
    // is a view.  2: views up to kViewRows rows only, larger probe sides
    // copied (the copy leaves them MALL-warm for the join that reads them
    // next: the join kernel runs at ~0.50 of the HBM peak instead of ~0.41,
    // but the bio step is ~4 % slower with the copies, profiles/r3_*).
    // 0: never.
    const char* f = std::getenv("DAS_SCAN_VIEWS");
    c.scan_views = f && f[0] == '2' ? 2 : f && f[0] == '0' ? 0 : 1;
  }
  ~Views() { c.scan_views = 0; }
};

// An And's terms as fused_and takes them: the Not(Link) terms that an anti
// index join applies, and the others (eval_and)
void split_and(const Exec& ex, const std::vector<uint32_t>& terms, std::vector<const das_plan_node_t*>& pos,
               std::vector<const das_plan_node_t*>& neg) {
  for (uint32_t ti : terms) {
    const das_plan_node_t& x = ex.nd[ti];
    if (x.op == DAS_PLAN_NOT && ex.nd[ti + 1].op == DAS_PLAN_LINK && ex.nd[ti + 1].index_join) neg.push_back(&ex.nd[ti + 1]);
    else pos.push_back(&x);
  }
}

// a plan's query shape: its node words with the scan / index-join targets
// left out (the anchors a fresh query changes; words 7..14 and 30..37 of
// each das_plan_node_t), FNV-1a
uint64_t shape_hash(const das_plan_node_t* nd, uint32_t n) {
  static_assert(sizeof(das_plan_node_t) == 51 * 4, "plan node layout");
  const uint32_t* w = reinterpret_cast<const uint32_t*>(nd);
  uint64_t h = 1469598103934665603ull;
  for (uint64_t i = 0; i < 51ull * n; ++i) {
    const uint32_t k = (uint32_t)(i % 51);
    if ((k >= 7 && k < 15) || (k >= 30 && k < 38)) continue;
    h = (h ^ w[i]) * 1099511628211ull;
  }
  return h;
}

// a plan's answer: a view must not outlive the index, so the caller gets a copy
PlanOutput output(Ctx& c, Res r) {
  PlanOutput out;
  out.matched = r.matched;
  out.negation = r.neg;
  for (auto& t : r.rel.t) {
    if (t->view) {
      auto m = new_table_like(c, *t, t->nrows);
      m->nrows = t->nrows;
      for (int k = 0; k < t->ncols; ++k) copy_dev(m->col(k), t->col(k), 4 * t->nrows, c.s);
      t = std::move(m);
    }
    out.tables.push_back(std::move(t));
  }
  return out;
}

}  // namespace

PlanOutput plan_execute_sharded(Ctx& c, const das_plan_node_t* nodes, uint32_t n, int no_overload,
                                const std::vector<const Table*>& inputs, std::vector<uint8_t>& checks) {
  DAS_CHECK(c.idx.built, DAS_E_NOT_BUILT, "index not built");
  DAS_CHECK(n > 0, DAS_E_INVALID, "plan: no nodes");
  Exec ex{c, nodes, n, no_overload};
  ex.inputs = &inputs;
  ex.checks = &checks;
  DAS_CHECK(ex.next(0) == n, DAS_E_INVALID, "plan: node array is not one expression tree");
  trace_mark("plan (sharded)");
  Res r = ex.eval(0);
  trace_mark("done");
  trace_dump("das_plan_execute_sharded");
  PlanOutput out;
  out.matched = r.matched;
  out.negation = r.neg;
  for (auto& t : r.rel.t) {
    if (t->view) {
      // an INPUT table is the caller's: the answer gets its own copy
      auto m = new_table_like(c, *t, t->nrows);
      m->nrows = t->nrows;
      for (int k = 0; k < t->ncols; ++k) copy_dev(m->col(k), t->col(k), 4 * t->nrows, c.s);
      t = std::move(m);
    }
    out.tables.push_back(std::move(t));
  }
  return out;
}

PlanOutput plan_execute(Ctx& c, const das_plan_node_t* nodes, uint32_t n, int no_overload) {
  DAS_CHECK(c.idx.built, DAS_E_NOT_BUILT, "index not built");
  DAS_CHECK(n > 0, DAS_E_INVALID, "plan: no nodes");
  Exec ex{c, nodes, n, no_overload};
  DAS_CHECK(ex.next(0) == n, DAS_E_INVALID, "plan: node array is not one expression tree");
  trace_mark("plan");
  Res r;
  {
    Views v(c);
    r = ex.eval(0);
  }
  trace_mark("done");
  trace_dump("das_plan_execute");
  return output(c, std::move(r));
}

std::vector<PlanOutput> plan_execute_many(Ctx& c, const das_plan_node_t* const* nodes, const uint32_t* n,
                                          uint32_t n_plans, int no_overload) {
  DAS_CHECK(c.idx.built, DAS_E_NOT_BUILT, "index not built");
  for (uint32_t i = 0; i < n_plans; ++i) {
    DAS_CHECK(nodes[i] && n[i] > 0, DAS_E_INVALID, "plan: no nodes");
    Exec ex{c, nodes[i], n[i], no_overload};
    DAS_CHECK(ex.next(0) == n[i], DAS_E_INVALID, "plan: node array is not one expression tree");
  }
  std::vector<PlanOutput> outs(n_plans);
  std::vector<ChainRunPtr> runs(n_plans);
  std::vector<std::unique_ptr<UnionRun>> uruns(n_plans);
  const char* f = std::getenv("DAS_DEFER");               // A/B: 0 = every plan in turn
  const bool defer = !(f && f[0] == '0');
  const char* fh = std::getenv("DAS_DEFER_HOOK");         // A/B: 0 = chains launched before the other plans
  const char* sd = std::getenv("DAS_CHAIN_SIDE");         // A/B: 0 = chains on the context's stream
  const bool side = !(sd && sd[0] == '0');
  trace_mark("plans");
  Views v(c);
  // root Ands are the chain candidates; a chain runs on a side stream (its
  // tables that stream's blocks), ordered after the context's stream once,
  // at this fence: blocks of earlier batches' answers were last read there
  std::vector<uint8_t> cand(n_plans, 0), tried(n_plans, 0);
  uint32_t n_cand = 0;
  // (root Ors: their one-launch bitmap union, likewise launched early and
  // read back last; DAS_DEFER_OR=0 off)
  const char* fo = std::getenv("DAS_DEFER_OR");
  const bool defer_or = !(fo && fo[0] == '0');
  for (uint32_t i = 0; i < n_plans && defer; ++i) {
    if (n_cand >= kPubPool) break;
    if (nodes[i][0].op == DAS_PLAN_OR && defer_or && nodes[i][0].nchild >= 2) {
      cand[i] = 1;
      ++n_cand;
      continue;
    }
    if (nodes[i][0].op != DAS_PLAN_AND) continue;
    Exec ex{c, nodes[i], n[i], no_overload};
    std::vector<const das_plan_node_t*> pos, neg;
    split_and(ex, ex.children(0), pos, neg);
    if (!fused_and_viable(c, pos, neg, no_overload)) continue;   // runs with the other plans
    cand[i] = 1;
    ++n_cand;
  }
  hipEvent_t fence_in = nullptr;
  bool waited[Ctx::kSide] = {};
  // DAS_PLAN_SIDE=1: the heaviest other plan first, the rest on a side
  // stream (below).  Off by default: no faster in the bench steps (bio
  // 1.443 / 1.486 vs 1.430 / 1.469 ms, hub 0.891 / 0.888 vs 0.894 / 0.892;
  // the lead's cross product holds the CUs and HBM the side plans need,
  // even from a highest-priority queue; profiles/r5_plan_side_ab.txt)
  const char* ps = std::getenv("DAS_PLAN_SIDE");
  const bool plan_side = ps && ps[0] == '1' && n_plans - n_cand > 1;
  // a plan nested in another's long read-back wait (below; DAS_PLAN_NEST=0 off)
  const char* pn = std::getenv("DAS_PLAN_NEST");
  const bool nest = !(pn && pn[0] == '0') && n_plans - n_cand > 1;
  const char* nm = std::getenv("DAS_PLAN_NEST_MIN");             // tests: 0 = at every wait
  const double nest_min = nm ? std::atof(nm) : (double)(128u << 20);
  const char* ng = std::getenv("DAS_NEST_GATE_MB");               // 0: no gate (A/B)
  const double gate_min = (ng ? std::atof(ng) : 1024.0) * (1 << 20);
  if ((n_cand && side) || plan_side || nest) {
    // side streams are ordered after the context's stream as it stands when
    // the batch begins (their blocks' last readers), never after this batch's
    // own launches there
    fence_in = c.fence_event(2 * kPubPool);
    DAS_HIP(hipEventRecord(fence_in, c.s));
  }
  // das_prof_tag_plan: plan c.tag_plan's own launches are named
  // "<scope>@<tag>" (restored on exit, so plans nested in its waits and the
  // hook's chains stay untagged: the hook clears the tag, below)
  struct TagScope {
    Ctx& c;
    std::string old;
    bool on;
    TagScope(Ctx& c_, uint32_t i) : c(c_), old(c_.prof_tag), on(i == c_.tag_plan) {
      if (on) c.prof_tag = c.tag_plan_name;
    }
    ~TagScope() { if (on) c.prof_tag = old; }
  };
  auto eval_plan = [&](uint32_t i) {
    TagScope ts(c, i);
    Exec ex{c, nodes[i], n[i], no_overload};
    return output(c, ex.eval(0));
  };
  uint32_t pooled = 0, next = 0;
  // compiles and launches the next candidates' chains while ready() is false
  // (every remaining one when it is null); true when none is left
  auto launch_some = [&](const std::function<bool()>* ready) {
    for (; next < n_plans; ++next) {
      const uint32_t i = next;
      if (!cand[i] || tried[i]) continue;
      if (ready && (*ready)()) return false;
      tried[i] = 1;
      TagScope ts(c, i);
      Exec ex{c, nodes[i], n[i], no_overload};
      const int sidx = side ? (int)(pooled % Ctx::kChainSides) : -1;
      if (nodes[i][0].op == DAS_PLAN_OR) {
        std::vector<const das_plan_node_t*> links;
        for (uint32_t ti : ex.children(0)) links.push_back(&nodes[i][ti]);
        uruns[i] = fused_or_launch(c, links, no_overload, pooled, sidx, fence_in, sidx >= 0 ? &waited[sidx] : nullptr);
        if (uruns[i]) ++pooled;
        continue;
      }
      std::vector<const das_plan_node_t*> pos, neg;
      split_and(ex, ex.children(0), pos, neg);
      runs[i] = fused_and_launch(c, pos, neg, no_overload, pooled, sidx, fence_in, sidx >= 0 ? &waited[sidx] : nullptr);
      if (runs[i]) ++pooled;
    }
    return true;
  };
  auto launch_all = [&] { launch_some(nullptr); };
  // 1. the other plans first; the chains are compiled and launched in the
  // gaps where those plans wait for a read-back (host time otherwise spent
  // spinning), the rest after them
  // the other plans in order (below), with `order` / `done` shared with the
  // hook: a plan whose read-back wait follows >= nest_min launched bytes (the
  // hub's filtered walk) hosts the next pending plans, run whole inside that
  // wait on the plan side stream with their own read-back slot (PubLevel),
  // while the awaited slot is unwritten -- the hub's H2 expansion, bound by
  // HBM writes, then runs beside H4's latency-bound walk
  std::vector<uint32_t> order;
  for (uint32_t i = 0; i < n_plans; ++i)
    if (!cand[i]) order.push_back(i);
  std::vector<uint8_t> done(n_plans, 0);
  size_t cur = 0;                                          // the plan the main loop is in
  bool on_side = false;
  auto to_side = [&]() {
    hipStream_t ss = c.side_stream(Ctx::kPlanSide);
    if (!waited[Ctx::kPlanSide]) {
      DAS_HIP(hipStreamWaitEvent(ss, fence_in, 0));
      waited[Ctx::kPlanSide] = true;
    }
    on_side = true;
    return ss;
  };
  struct Swap {
    Ctx& c;
    hipStream_t old;
    ~Swap() { c.s = old; }
  };
  auto nest_some = [&](const std::function<bool()>& ready) {
    if (!nest || bytes_since_wait() < nest_min) return;
    for (size_t j = cur + 1; j < order.size() && !ready(); ++j) {
      const uint32_t i = order[j];
      if (done[i]) continue;
      done[i] = 1;
      if (trace_on()) trace_mark("nested plan");
      PubLevel lv;
      Swap sw{c, c.s};
      c.s = to_side();
      // its first flood of >= gate_min bytes (bio QUERY_3's 6.6 GB cross
      // product) waits for the outer plan's launched kernels: running beside
      // an HBM-bound join it slowed both (a 50 us join took 330 us beside it)
      struct Ungate {
        Ctx& c;
        ~Ungate() { c.gate_s = nullptr; }
      } ug{c};
      c.gate_s = gate_min > 0 ? sw.old : nullptr;
      c.gate_min = gate_min;
      outs[i] = eval_plan(i);
    }
  };
  // 1. the other plans first; the chains are compiled and launched in the
  // gaps where those plans wait for a read-back (host time otherwise spent
  // spinning), the rest after them
  WaitHook hook = [&](const std::function<bool()>& ready) {
    // the waiting plan's tag does not cover what runs in its wait
    struct Untag {
      Ctx& c;
      std::string old;
      ~Untag() { c.prof_tag = old; }
    } ut{c, c.prof_tag};
    c.prof_tag.clear();
    bool chains_done;
    {
      // the chains' own read-backs (a key range resolved on the device by
      // scan_prepare, a non-pooled outcome slot) and staging go to the second
      // level: the awaited slot and its request buffer stay the outer plan's
      PubLevel lv;
      chains_done = launch_some(&ready);
    }
    if (chains_done) nest_some(ready);
    bool pending = false;
    for (size_t j = cur + 1; j < order.size() && nest; ++j) pending = pending || !done[order[j]];
    return chains_done && !pending;
  };
  const bool hooked = (n_cand && !(fh && fh[0] == '0')) || nest;
  if (!hooked) launch_all();
  struct Unhook {
    ~Unhook() { set_wait_hook(nullptr); }
  } uh;
  if (hooked) set_wait_hook(&hook);
  // (DAS_PLAN_SIDE=1: the heaviest plan by the algorithmic bytes its shape
  // launched last time first, on the context's stream, the rest after it on
  // the side stream -- measured no faster, off by default)
  std::vector<uint64_t> shape(n_plans, 0);
  for (uint32_t i : order) shape[i] = shape_hash(nodes[i], n[i]);
  auto weight = [&](uint32_t i) {
    auto it = c.plan_bytes.find(shape[i]);
    return it == c.plan_bytes.end() ? -1.0 : it->second;
  };
  if (plan_side)
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return weight(a) > weight(b); });
  double rest = 0;
  for (size_t j = 1; j < order.size(); ++j) rest += std::max(weight(order[j]), 0.0);
  const char* sm = std::getenv("DAS_PLAN_SPLIT_MIN");          // tests: 0 = any lead heavier than the rest
  const double split_min = sm ? std::atof(sm) : (double)(64u << 20);
  const bool split = plan_side && weight(order[0]) > std::max(rest, split_min) && weight(order[0]) >= 0;
  for (size_t j = 0; j < order.size(); ++j) {
    const uint32_t i = order[j];
    if (done[i]) continue;                                 // ran nested in an earlier plan's wait
    done[i] = 1;
    cur = j;
    Swap sw{c, c.s};
    if (split && j > 0) c.s = to_side();
    const double b0 = launched_bytes();
    outs[i] = eval_plan(i);
    c.plan_bytes[shape[i]] = launched_bytes() - b0;
    if (hooked) set_wait_hook(&hook);                      // (re-armed for the next plan's waits)
  }
  if (c.plan_bytes.size() > 4096) c.plan_bytes.clear();
  set_wait_hook(nullptr);
  launch_all();                                           // (no-op once the hook ran)
  // 2. candidates no chain / union launch answers, in turn
  for (uint32_t i = 0; i < n_plans; ++i) {
    if (!cand[i] || runs[i] || uruns[i]) continue;
    outs[i] = eval_plan(i);
  }
  // 3. the unions' and chains' outcomes (a redo: the plan evaluated in full)
  for (uint32_t i = 0; i < n_plans; ++i) {
    if (!uruns[i]) continue;
    bool m = false;
    TablePtr t;
    if (fused_or_finish(c, *uruns[i], m, t)) {
      outs[i].matched = m;
      if (m && t && t->nrows) outs[i].tables.push_back(std::move(t));
    } else {
      outs[i] = eval_plan(i);
    }
    uruns[i].reset();
  }
  for (uint32_t i = 0; i < n_plans; ++i) {
    if (!runs[i]) continue;
    bool m = false;
    TablePtr t;
    if (fused_and_finish(c, *runs[i], m, t)) {
      outs[i].matched = m;
      if (m && t && t->nrows) outs[i].tables.push_back(std::move(t));
    } else {
      outs[i] = eval_plan(i);
    }
    runs[i].reset();
  }
  // the side stream's answers are read on the context's stream from here on
  if (on_side) {
    DAS_HIP(hipEventRecord(c.fence_event(2 * kPubPool + 2), c.side_stream(Ctx::kPlanSide)));
    DAS_HIP(hipStreamWaitEvent(c.s, c.fence_event(2 * kPubPool + 2), 0));
  }
  trace_mark("done");
  trace_dump("das_plan_execute_many");
  return outs;
}

}  // namespace das
