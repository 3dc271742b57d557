// Canonical MeTTa reader (canonical.cpp): parsed atoms in the das_atoms_t layout.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "status.h"

namespace das {

struct Parsed {
  std::vector<uint8_t> leaf_bytes;
  std::vector<uint64_t> leaf_off;
  std::vector<uint8_t> leaf_kind;
  std::vector<uint32_t> leaf_ctype, leaf_type_id, name_start;
  std::vector<uint64_t> expr_off;
  std::vector<uint32_t> expr_child;
  std::vector<uint8_t> expr_kind;
  std::vector<int32_t> expr_ctype_leaf;
  std::vector<uint64_t> level_off;
  std::vector<std::string> type_names;
};

// Parses n_texts canonical files (each with its own types / terminals /
// expressions sections) on `threads` host threads (0 = up to 16).  Throws
// Error(DAS_E_SYNTAX) where the reference's _check asserts.
std::unique_ptr<Parsed> parse_canonical(const char* const* texts, const uint64_t* lens, uint32_t n_texts,
                                        unsigned threads);

}  // namespace das
