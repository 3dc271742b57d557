// Status codes and the error type every entry point maps to its C-ABI status.
// Host-only (no HIP headers): the canonical reader includes this alone, so it
// also builds with plain g++ for the sanitizer targets (Makefile: asan, tsan).
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>

namespace das {

constexpr uint32_t kNone = 0xFFFFFFFFu;

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

enum Status : int {
  DAS_S_OK = 0,
  DAS_E_INVALID = -1,     // bad argument / misuse          -> ValueError
  DAS_E_HIP = -2,         // HIP runtime failure            -> RuntimeError
  DAS_E_NOT_BUILT = -3,   // index not built                -> RuntimeError
  DAS_E_UNSUPPORTED = -4, // shape outside this build       -> NotImplementedError
  DAS_E_INTERNAL = -5,
  DAS_E_ATTRIBUTE = -6,   // the reference raises AttributeError here -> AttributeError
  DAS_E_SYNTAX = -7,      // malformed input where the reference asserts -> AssertionError
};

#define DAS_CHECK(cond, code, msg)                 \
  do {                                             \
    if (!(cond)) throw ::das::Error((code), (msg)); \
  } while (0)

}  // namespace das
