// Canonical MeTTa reader (host, multi-threaded): text -> das_atoms_t arrays.
//
// Replaces CanonicalParser.parse / _parse_expression (canonical_parser.py:
// 242-365), the step before hashing.  The reference
// walks the file line by line in three states:
//   READING_TYPES      `(: Name Type)`          typedefs (3 words)
//   READING_TERMINALS  `(: "name words" Type)`  declared terminals (nodes)
//   READING_EXPRESSIONS `(Type <child> ...)`    one expression per line,
//                       children are "Type name" terminals or nested
//                       expressions; nested expressions are links too.
// The sections are contiguous, so the file is cut into line-aligned chunks,
// pass 1 finds the two section boundaries per text, pass 2 parses every chunk
// independently and a merge lays the chunks out in file order: type leaves
// first (first-appearance order), then each chunk's terminal leaves, then the
// expressions grouped by (nesting level, number of children) with file order
// inside a group.  That is the layout loader.AtomBuilder.finish produces,
// except that terminals are not de-duplicated on the host: the device interns
// every leaf by digest (das_build_index), so repeats cost bytes, not atoms.
//
// Differences from the reference, on inputs it does not handle either: an
// empty line is skipped (the reference raises IndexError), and a bare symbol
// in a child position is rejected (the reference hashes the raw symbol text
// as if it were a handle, canonical_parser.py:253-261).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "canonical.h"

namespace das {

namespace {

constexpr uint64_t kNoPos = ~0ull;
constexpr uint32_t kNoTypeInit = 0xFFFFFFFFu;
constexpr uint8_t kLeafType = 0, kLeafNode = 1, kLeafOther = 2;
uint64_t chunk_bytes() {        // DAS_PARSE_CHUNK_BYTES: tests force many small chunks
  const char* e = std::getenv("DAS_PARSE_CHUNK_BYTES");
  const uint64_t v = e ? std::strtoull(e, nullptr, 10) : 0;
  return v ? v : (4ull << 20);
}

// Python str.split()/strip() whitespace, UTF-8 encoded: returns the byte
// length of the whitespace character at p, 0 if there is none.
inline int ws_len(const char* p, const char* e) {
  const unsigned char c = (unsigned char)*p;
  if (c > 32 && c < 128) return 0;          // printable ASCII: the common case
  if (c == ' ' || (c >= 9 && c <= 13) || (c >= 28 && c <= 31)) return 1;
  if (c < 0xC2) return 0;
  const unsigned char c1 = p + 1 < e ? (unsigned char)p[1] : 0;
  if (c == 0xC2) return (c1 == 0x85 || c1 == 0xA0) ? 2 : 0;                    // U+0085, U+00A0
  const unsigned char c2 = p + 2 < e ? (unsigned char)p[2] : 0;
  if (c == 0xE1) return (c1 == 0x9A && c2 == 0x80) ? 3 : 0;                     // U+1680
  if (c == 0xE2) {
    if (c1 == 0x80 && ((c2 >= 0x80 && c2 <= 0x8A) || c2 == 0xA8 || c2 == 0xA9 || c2 == 0xAF)) return 3;
    if (c1 == 0x81 && c2 == 0x9F) return 3;                                     // U+205F
    return 0;
  }
  if (c == 0xE3) return (c1 == 0x80 && c2 == 0x80) ? 3 : 0;                     // U+3000
  return 0;
}

// whitespace-separated words of [b, e)
void split_words(const char* b, const char* e, std::vector<std::string_view>& out) {
  out.clear();
  const char* p = b;
  while (p < e) {
    int w;
    while (p < e && (w = ws_len(p, e)) > 0) p += w;
    if (p >= e) break;
    const char* s = p;
    while (p < e && ws_len(p, e) == 0) ++p;
    out.emplace_back(s, (size_t)(p - s));
  }
}

inline bool is_break(char c) { return c == '\n' || c == '\r'; }

struct Text {
  const char* p;
  uint64_t n;
  uint64_t first_terminal = kNoPos;   // first `(: "..."` line
  uint64_t first_expr = kNoPos;       // first line not starting with the word `(:`
  uint64_t last_decl = 0;             // last `(:` line (+1; 0 = none)
};

struct Chunk {
  uint32_t text;
  uint64_t b, e;                      // line-aligned byte range inside the text
  // pass 1
  uint64_t first_terminal = kNoPos, first_expr = kNoPos, last_decl = 0;
  // pass 2: local types (first-appearance order)
  std::unordered_map<std::string_view, uint32_t> tmap;
  std::vector<std::string_view> types;
  std::vector<uint32_t> tglobal;
  uint32_t recent[4] = {kNoTypeInit, kNoTypeInit, kNoTypeInit, kNoTypeInit};
  int recent_next = 0;
  // terminal leaves
  std::vector<char> tbytes;
  std::vector<uint64_t> toff{0};
  std::vector<uint8_t> tkind;
  std::vector<uint32_t> ttype, tname;
  // expressions (post-order: children before parents)
  std::vector<uint64_t> child;        // tagged refs, see ref_*()
  std::vector<uint64_t> e_child0;
  std::vector<uint32_t> e_nch, e_level, e_rank;
  std::unordered_map<uint64_t, uint32_t> key_count;   // (level << 32 | nch) -> count
  std::vector<uint64_t> e_key;
  uint64_t last_key = ~0ull;
  uint32_t* last_count = nullptr;
  std::string err;
  uint64_t err_pos = kNoPos;
};

constexpr uint32_t kNoType = 0xFFFFFFFFu;
uint32_t local_type_slow(Chunk& c, std::string_view name);

// child reference tags
constexpr uint64_t kTagType = 0, kTagLeaf = 1ull << 62, kTagExpr = 2ull << 62, kTagMask = 3ull << 62;

uint32_t local_type(Chunk& c, std::string_view name) {
  // consecutive lines mostly repeat the same few types: check the last hits
  for (int k = 0; k < 4; ++k) {
    const uint32_t t = c.recent[k];
    if (t != kNoType && c.types[t] == name) return t;
  }
  const uint32_t t = local_type_slow(c, name);
  c.recent[c.recent_next] = t;
  c.recent_next = (c.recent_next + 1) & 3;
  return t;
}

uint32_t local_type_slow(Chunk& c, std::string_view name) {
  auto it = c.tmap.find(name);
  if (it != c.tmap.end()) return it->second;
  const uint32_t id = (uint32_t)c.types.size();
  c.tmap.emplace(name, id);
  c.types.push_back(name);
  return id;
}

void add_terminal(Chunk& c, std::string_view stype, const std::vector<std::string_view>& words, size_t w0,
                  size_t w1, bool node, bool strip_quotes) {
  const uint32_t t = local_type(c, stype);
  const size_t start = c.tbytes.size();
  c.tbytes.insert(c.tbytes.end(), stype.begin(), stype.end());
  c.tbytes.push_back(' ');
  const size_t name0 = c.tbytes.size();
  for (size_t i = w0; i < w1; ++i) {
    if (i > w0) c.tbytes.push_back(' ');
    c.tbytes.insert(c.tbytes.end(), words[i].begin(), words[i].end());
  }
  if (strip_quotes) {            // " ".join(words).strip('"')
    size_t a = name0, z = c.tbytes.size();
    while (a < z && c.tbytes[a] == '"') ++a;
    while (z > a && c.tbytes[z - 1] == '"') --z;
    if (a > name0 || z < c.tbytes.size()) {
      std::memmove(c.tbytes.data() + name0, c.tbytes.data() + a, z - a);
      c.tbytes.resize(name0 + (z - a));
    }
  }
  (void)start;
  c.toff.push_back(c.tbytes.size());
  c.tkind.push_back(node ? kLeafNode : kLeafOther);
  c.ttype.push_back(t);
  c.tname.push_back((uint32_t)stype.size() + 1);
}

inline std::string_view rstrip_paren(std::string_view w) {
  while (!w.empty() && w.back() == ')') w.remove_suffix(1);
  return w;
}

struct Item {
  enum Kind : uint8_t { Open, Sym, Ref } kind;
  std::string_view sym;
  uint64_t ref;
  uint32_t level;
};

// _parse_expression (canonical_parser.py:242-305) over one stripped line.
bool parse_expression(Chunk& c, const char* b, const char* e, std::vector<Item>& st,
                      std::vector<std::string_view>& words) {
  st.clear();
  int state = 0;
  const char* sym = nullptr;       // start of the pending symbol
  const char* term = nullptr;      // start of the pending quoted terminal
  char prev = 0;
  auto fail = [&](const char* at, const char* msg) {
    c.err = msg;
    c.err_pos = (uint64_t)(at - b);
    return false;
  };
  for (const char* p = b; p < e; ++p) {
    const char ch = *p;
    if (state == 0) {
      if (ch == '(') {
        if (sym) return fail(p, "symbol directly followed by '('");
        st.push_back({Item::Open, {}, 0, 0});
      } else if (ch == ' ') {
        if (sym) {
          st.push_back({Item::Sym, std::string_view(sym, (size_t)(p - sym)), 0, 0});
          sym = nullptr;
        }
      } else if (ch == ')') {
        if (sym) return fail(p, "bare symbol as a link target");
        size_t k = st.size();
        while (k > 0 && st[k - 1].kind != Item::Open) --k;
        if (k == 0) return fail(p, "unbalanced ')'");
        const size_t first = k;            // items [first, st.size())
        if (first == st.size() || st[first].kind != Item::Sym)
          return fail(p, "expression without a type symbol");
        uint32_t level = 0;
        const uint64_t c0 = c.child.size();
        const uint32_t t = local_type(c, st[first].sym);
        c.child.push_back(kTagType | t);
        for (size_t i = first + 1; i < st.size(); ++i) {
          if (st[i].kind != Item::Ref) return fail(p, "bare symbol as a link target");
          c.child.push_back(st[i].ref);
          level = std::max(level, st[i].level);
        }
        const uint32_t nch = (uint32_t)(st.size() - first);
        level += 1;
        const uint64_t key = ((uint64_t)level << 32) | nch;
        if (key != c.last_key) {
          c.last_key = key;
          c.last_count = &c.key_count[key];   // unordered_map references stay valid on insert
        }
        const uint32_t rank = (*c.last_count)++;
        const uint64_t eid = c.e_nch.size();
        c.e_child0.push_back(c0);
        c.e_nch.push_back(nch);
        c.e_level.push_back(level);
        c.e_rank.push_back(rank);
        c.e_key.push_back(key);
        st.resize(first - 1);              // pop the items and the '('
        if (!st.empty()) st.push_back({Item::Ref, {}, kTagExpr | eid, level});
      } else if (ch == '"') {
        if (sym) return fail(p, "symbol directly followed by '\"'");
        state = 1;
        term = p + 1;
      } else if (!sym) {
        sym = p;
      }
    } else if (ch == '"' && prev != '\\') {
      split_words(term, p, words);
      if (words.empty()) return fail(p, "empty terminal");
      add_terminal(c, words[0], words, 1, words.size(), false, false);
      st.push_back({Item::Ref, {}, kTagLeaf | (uint64_t)(c.tkind.size() - 1), 0});
      state = 0;
    }
    prev = ch;
  }
  if (state != 0) return fail(e, "unterminated string");
  if (sym || !st.empty()) return fail(e, "unbalanced expression");
  return true;
}

// strip one line [b, e) of Python whitespace
inline void strip(const char*& b, const char*& e) {
  int w;
  while (b < e && (w = ws_len(b, e)) > 0) b += w;
  while (e > b) {
    // trailing whitespace: test the 1-3 byte encodings ending at e
    if (ws_len(e - 1, e) == 1) { --e; continue; }
    if (e - b >= 2 && ws_len(e - 2, e) == 2) { e -= 2; continue; }
    if (e - b >= 3 && ws_len(e - 3, e) == 3) { e -= 3; continue; }
    break;
  }
}

template <typename F>
void for_lines(const char* base, uint64_t b, uint64_t e, F&& f) {
  uint64_t i = b;
  while (i < e) {
    uint64_t j = i;
    while (j < e && !is_break(base[j])) ++j;
    const char* lb = base + i;
    const char* le = base + j;
    strip(lb, le);
    if (lb < le) f(i, lb, le);
    i = j + 1;
  }
}

inline bool starts_decl(const char* b, const char* e) {
  // first word == "(:"
  return e - b >= 2 && b[0] == '(' && b[1] == ':' && (e - b == 2 || ws_len(b + 2, e) > 0);
}

void pass1(Chunk& c, const Text& t) {
  for_lines(t.p, c.b, c.e, [&](uint64_t pos, const char* b, const char* e) {
    if (starts_decl(b, e)) {
      c.last_decl = pos + 1;
      if (c.first_terminal == kNoPos) {
        const char* q = b + 2;
        int w;
        while (q < e && (w = ws_len(q, e)) > 0) q += w;
        if (q < e && *q == '"') c.first_terminal = pos;
      }
    } else if (c.first_expr == kNoPos) {
      c.first_expr = pos;
    }
  });
}

void pass2(Chunk& c, const Text& t) {
  // capacity guesses from the chunk size (~60-100 bytes a line, 2-3 terminals)
  const uint64_t nb = c.e - c.b;
  c.tbytes.reserve(nb);
  c.toff.reserve(nb / 24);
  c.tkind.reserve(nb / 24);
  c.ttype.reserve(nb / 24);
  c.tname.reserve(nb / 24);
  c.child.reserve(nb / 16);
  for (auto* v : {&c.e_nch, &c.e_level, &c.e_rank}) v->reserve(nb / 48);
  c.e_child0.reserve(nb / 48);
  c.e_key.reserve(nb / 48);
  std::vector<std::string_view> words;
  std::vector<Item> st;
  for_lines(t.p, c.b, c.e, [&](uint64_t pos, const char* b, const char* e) {
    if (!c.err.empty()) return;
    if (pos < t.first_terminal) {                   // READING_TYPES
      split_words(b, e, words);
      if (words.size() != 3) {
        c.err = "typedef line must have 3 words";
        c.err_pos = pos;
        return;
      }
      local_type(c, words[1]);
      local_type(c, rstrip_paren(words[2]));
    } else if (pos < t.first_expr) {                // READING_TERMINALS
      split_words(b, e, words);
      add_terminal(c, rstrip_paren(words.back()), words, 1, words.size() > 1 ? words.size() - 1 : 1, true, true);
    } else {                                        // READING_EXPRESSIONS
      if (*b != '(' || e[-1] != ')') {
        c.err = "expression line must start with '(' and end with ')'";
        c.err_pos = pos;
        return;
      }
      if (!parse_expression(c, b, e, st, words)) c.err_pos = pos + c.err_pos;
    }
  });
}

template <typename F>
void parallel_for(size_t n, unsigned threads, F&& f) {
  std::atomic<size_t> next{0};
  auto work = [&] {
    for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
  };
  const unsigned nt = (unsigned)std::min<size_t>(threads, n);
  std::vector<std::thread> pool;
  for (unsigned k = 1; k < nt; ++k) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
}

uint64_t line_of(const Text& t, uint64_t pos) {
  uint64_t line = 1;
  for (uint64_t i = 0; i < pos && i < t.n; ++i)
    if (t.p[i] == '\n' || (t.p[i] == '\r' && !(i + 1 < t.n && t.p[i + 1] == '\n'))) ++line;
  return line;
}

}  // namespace

std::unique_ptr<Parsed> parse_canonical(const char* const* texts, const uint64_t* lens, uint32_t n_texts,
                                        unsigned threads) {
  if (!threads) threads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const bool trace = std::getenv("DAS_PARSE_TRACE") != nullptr;
  auto t0 = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!trace) return;
    const auto t1 = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[parse] %-8s %9.1f ms\n", what, std::chrono::duration<double, std::milli>(t1 - t0).count());
    t0 = t1;
  };
  std::vector<Text> tx(n_texts);
  std::vector<Chunk> chunks;
  for (uint32_t i = 0; i < n_texts; ++i) {
    tx[i].p = texts[i];
    tx[i].n = lens[i];
    // line-aligned cuts every ~kChunkBytes
    const uint64_t cb = chunk_bytes();
    uint64_t b = 0;
    while (b < lens[i]) {
      uint64_t e = std::min(lens[i], b + cb);
      while (e < lens[i] && !is_break(texts[i][e - 1])) ++e;
      Chunk c;
      c.text = i;
      c.b = b;
      c.e = e;
      chunks.push_back(std::move(c));
      b = e;
    }
  }
  parallel_for(chunks.size(), threads, [&](size_t k) { pass1(chunks[k], tx[chunks[k].text]); });
  lap("pass1");
  if (trace) std::fprintf(stderr, "[parse] %zu chunks, %u threads\n", chunks.size(), threads);
  for (auto& c : chunks) {
    Text& t = tx[c.text];
    t.first_terminal = std::min(t.first_terminal, c.first_terminal);
    t.first_expr = std::min(t.first_expr, c.first_expr);
    t.last_decl = std::max(t.last_decl, c.last_decl);
  }
  for (auto& t : tx) {
    // the reference's state checks (canonical_parser.py:336-363)
    if (t.first_expr != kNoPos) {
      DAS_CHECK(t.first_terminal < t.first_expr, DAS_E_SYNTAX,
                "line " + std::to_string(line_of(t, t.first_expr)) + ": expression before the terminal section");
      DAS_CHECK(t.last_decl <= t.first_expr, DAS_E_SYNTAX,
                "line " + std::to_string(line_of(t, t.last_decl - 1)) + ": '(:' line inside the expression section");
    }
  }
  parallel_for(chunks.size(), threads, [&](size_t k) { pass2(chunks[k], tx[chunks[k].text]); });
  lap("pass2");
  for (auto& c : chunks)
    DAS_CHECK(c.err.empty(), DAS_E_SYNTAX,
              "line " + std::to_string(line_of(tx[c.text], c.err_pos)) + ": " + c.err);

  // ---- merge: global types, leaves, expression groups ----
  auto out = std::make_unique<Parsed>();
  std::unordered_map<std::string_view, uint32_t> gtype;
  for (auto& c : chunks) {
    c.tglobal.resize(c.types.size());
    for (size_t i = 0; i < c.types.size(); ++i) {
      auto it = gtype.find(c.types[i]);
      if (it == gtype.end()) {
        const uint32_t g = (uint32_t)out->type_names.size();
        gtype.emplace(c.types[i], g);
        out->type_names.emplace_back(c.types[i]);
        c.tglobal[i] = g;
      } else {
        c.tglobal[i] = it->second;
      }
    }
  }
  const uint64_t n_types = out->type_names.size();
  std::vector<uint64_t> leaf_base(chunks.size()), byte_base(chunks.size());
  uint64_t n_leaf = n_types, n_bytes = 0;
  for (auto& s : out->type_names) n_bytes += s.size();
  for (size_t k = 0; k < chunks.size(); ++k) {
    leaf_base[k] = n_leaf;
    byte_base[k] = n_bytes;
    n_leaf += chunks[k].tkind.size();
    n_bytes += chunks[k].tbytes.size();
  }
  // expression groups ordered by (level, nch)
  std::map<uint64_t, uint64_t> gcount;
  for (auto& c : chunks)
    for (auto& kv : c.key_count) gcount[kv.first] += kv.second;
  std::unordered_map<uint64_t, uint64_t> gbase, cbase;   // first expression / first child slot of a group
  uint64_t n_expr = 0, n_child = 0;
  out->level_off.push_back(0);
  for (auto& kv : gcount) {
    gbase[kv.first] = n_expr;
    cbase[kv.first] = n_child;
    n_expr += kv.second;
    n_child += kv.second * (kv.first & 0xFFFFFFFFull);
    out->level_off.push_back(n_expr);
  }
  // per chunk offset of its first expression inside each group
  std::vector<std::unordered_map<uint64_t, uint64_t>> coff(chunks.size());
  {
    std::unordered_map<uint64_t, uint64_t> run;
    for (size_t k = 0; k < chunks.size(); ++k)
      for (auto& kv : chunks[k].key_count) {
        coff[k][kv.first] = run[kv.first];
        run[kv.first] += kv.second;
      }
  }
  out->leaf_bytes.resize(n_bytes);
  out->leaf_off.resize(n_leaf + 1);
  out->leaf_kind.resize(n_leaf);
  out->leaf_ctype.resize(n_leaf);
  out->leaf_type_id.resize(n_leaf);
  out->name_start.resize(n_leaf);
  out->expr_off.resize(n_expr + 1);
  out->expr_child.resize(n_child);
  out->expr_kind.assign(n_expr, 1);
  out->expr_ctype_leaf.assign(n_expr, -1);
  {
    uint64_t o = 0;
    for (uint64_t i = 0; i < n_types; ++i) {
      const std::string& s = out->type_names[i];
      std::memcpy(out->leaf_bytes.data() + o, s.data(), s.size());
      out->leaf_off[i] = o;
      o += s.size();
      out->leaf_kind[i] = kLeafType;
      out->leaf_ctype[i] = (uint32_t)i;
      out->leaf_type_id[i] = (uint32_t)i;
      out->name_start[i] = 0;
    }
    out->leaf_off[n_leaf] = n_bytes;
  }
  for (auto& kv : gcount) {
    const uint64_t g0 = gbase[kv.first], c0 = cbase[kv.first], nch = kv.first & 0xFFFFFFFFull;
    for (uint64_t j = 0; j < kv.second; ++j) out->expr_off[g0 + j] = c0 + j * nch;
  }
  out->expr_off[n_expr] = n_child;
  lap("merge");
  parallel_for(chunks.size(), threads, [&](size_t k) {
    Chunk& c = chunks[k];
    const uint64_t lb = leaf_base[k], bb = byte_base[k];
    if (!c.tbytes.empty()) std::memcpy(out->leaf_bytes.data() + bb, c.tbytes.data(), c.tbytes.size());
    for (size_t i = 0; i < c.tkind.size(); ++i) {
      out->leaf_off[lb + i] = bb + c.toff[i];
      out->leaf_kind[lb + i] = c.tkind[i];
      out->leaf_ctype[lb + i] = c.tglobal[c.ttype[i]];
      out->leaf_type_id[lb + i] = 0xFFFFFFFFu;
      out->name_start[lb + i] = c.tname[i];
    }
    std::vector<uint64_t> gpos(c.e_nch.size());
    for (size_t x = 0; x < c.e_nch.size(); ++x) {
      const uint64_t key = c.e_key[x];
      const uint64_t pos = gbase.at(key) + coff[k].at(key) + c.e_rank[x];
      gpos[x] = pos;
      uint32_t* dst = out->expr_child.data() + out->expr_off[pos];
      for (uint32_t j = 0; j < c.e_nch[x]; ++j) {
        const uint64_t r = c.child[c.e_child0[x] + j];
        const uint64_t v = r & ~kTagMask;
        switch (r & kTagMask) {
          case kTagType: dst[j] = c.tglobal[v]; break;
          case kTagLeaf: dst[j] = (uint32_t)(lb + v); break;
          default: dst[j] = (uint32_t)(n_leaf + gpos[v]); break;
        }
      }
    }
  });
  lap("write");
  DAS_CHECK(n_leaf + n_expr < 0xFFFFFFF0ull, DAS_E_UNSUPPORTED, "more than 2^32 parsed atoms");
  return out;
}

}  // namespace das
