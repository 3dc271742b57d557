// Sanitizer driver for the canonical MeTTa reader (das_amd/csrc/canonical.cpp).
//
// Built host-only by `make -C das_amd/csrc asan` / `tsan` (plain g++ with
// -fsanitize=address,undefined or -fsanitize=thread) and run by
// tests/test_sanitizers.py on CPU.  For every input file it parses the text
// with 1, 2, 3, 8 and 16 threads and with 4 MiB, 4 KiB and 97-byte chunks,
// and requires every run to produce the same arrays (thread and chunk
// invariance); then it parses all files at once as one multi-text call.
// Files named "bad_*" must be rejected with DAS_E_SYNTAX (the reference's
// assertion cases, canonical_parser.py:307-310).  Any sanitizer report makes
// the process exit non-zero.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../das_amd/csrc/canonical.h"

namespace {

uint64_t fnv(uint64_t h, const void* p, size_t n) {
  const unsigned char* b = (const unsigned char*)p;
  for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

template <typename T>
uint64_t fnv_vec(uint64_t h, const std::vector<T>& v) {
  const uint64_t n = v.size();
  h = fnv(h, &n, sizeof(n));
  return v.empty() ? h : fnv(h, v.data(), sizeof(T) * v.size());
}

uint64_t digest(const das::Parsed& p) {
  uint64_t h = 1469598103934665603ull;
  h = fnv_vec(h, p.leaf_bytes);
  h = fnv_vec(h, p.leaf_off);
  h = fnv_vec(h, p.leaf_kind);
  h = fnv_vec(h, p.leaf_ctype);
  h = fnv_vec(h, p.leaf_type_id);
  h = fnv_vec(h, p.name_start);
  h = fnv_vec(h, p.expr_off);
  h = fnv_vec(h, p.expr_child);
  h = fnv_vec(h, p.expr_kind);
  h = fnv_vec(h, p.expr_ctype_leaf);
  h = fnv_vec(h, p.level_off);
  for (auto& s : p.type_names) h = fnv(h, s.data(), s.size());
  return h;
}

std::string slurp(const char* path) {
  std::ifstream f(path, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

// parse -> (ok, status, digest)
struct Out {
  int status = 0;
  uint64_t h = 0;
  uint64_t n_expr = 0;
};

Out run(const std::vector<std::string>& texts, unsigned threads, const char* chunk) {
  setenv("DAS_PARSE_CHUNK_BYTES", chunk, 1);
  std::vector<const char*> ptrs;
  std::vector<uint64_t> lens;
  for (auto& t : texts) {
    ptrs.push_back(t.data());
    lens.push_back(t.size());
  }
  Out o;
  try {
    auto p = das::parse_canonical(ptrs.data(), lens.data(), (uint32_t)texts.size(), threads);
    o.h = digest(*p);
    o.n_expr = p->expr_kind.size();
  } catch (const das::Error& e) {
    o.status = e.code;
  }
  return o;
}

}  // namespace

int main(int argc, char** argv) {
  const unsigned threads[] = {1, 2, 3, 8, 16};
  const char* chunks[] = {"0", "4096", "97"};
  int failures = 0;
  std::vector<std::string> good;
  for (int i = 1; i < argc; ++i) {
    const std::string path = argv[i];
    const std::string base = path.substr(path.find_last_of('/') + 1);
    const bool bad = base.rfind("bad_", 0) == 0;
    const std::string text = slurp(argv[i]);
    Out ref = run({text}, 1, "0");
    for (unsigned t : threads)
      for (const char* c : chunks) {
        Out o = run({text}, t, c);
        const bool same = o.status == ref.status && o.h == ref.h;
        if (!same) {
          std::printf("MISMATCH %s threads=%u chunk=%s status=%d/%d\n", base.c_str(), t, c, o.status, ref.status);
          ++failures;
        }
      }
    if (bad && ref.status != das::DAS_E_SYNTAX) {
      std::printf("NOT REJECTED %s status=%d\n", base.c_str(), ref.status);
      ++failures;
    }
    if (!bad && ref.status != 0) {
      std::printf("REJECTED %s status=%d\n", base.c_str(), ref.status);
      ++failures;
    }
    if (!bad) good.push_back(text);
    std::printf("%s %s expressions=%llu digest=%016llx\n", bad ? "bad " : "file", base.c_str(),
                (unsigned long long)ref.n_expr, (unsigned long long)ref.h);
  }
  if (good.size() > 1) {
    Out ref = run(good, 1, "0");
    for (unsigned t : threads) {
      Out o = run(good, t, "4096");
      if (o.status != ref.status || o.h != ref.h) {
        std::printf("MISMATCH multi-text threads=%u\n", t);
        ++failures;
      }
    }
    std::printf("multi %zu texts expressions=%llu status=%d\n", good.size(), (unsigned long long)ref.n_expr,
                ref.status);
  }
  std::printf("%s\n", failures ? "FAILED" : "OK");
  return failures ? 1 : 0;
}
