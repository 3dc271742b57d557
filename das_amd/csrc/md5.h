// MD5 (RFC 1321) for the DAS handle function, host + device.
//
// The reference computes every atom handle as
//   md5(utf8(text)).hexdigest()                       expression_hasher.py:9-10
// where text is "Type name" for a terminal (:17-19), the type name for a type
// (:13-14) and " ".join([type_hash, *child_handles]) for a link (:22-35, with
// composite_hash([x]) == x).  Child handles enter a parent's message as
// 32 lowercase hex chars, so a link message is 33*k-1 bytes for k elements
// (98 B = 2 MD5 blocks at arity 2, 131 B = 3 blocks at arity 3).
//
// On the device one lane owns one message: the 16 message words of each
// 64-byte block are generated in registers straight from the child digests
// (hex-encoded on the fly) so a link costs (k*16) B of digest reads and 16 B
// of digest write, nothing else.
#pragma once
#include <cstdint>
#include <hip/hip_runtime.h>

namespace das {
namespace md5 {

#define DAS_HD __host__ __device__ __forceinline__

DAS_HD uint32_t rotl(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }

#define DAS_MD5_STEP(f, a, b, c, d, k, s, t) \
  a = b + rotl(a + (f) + (k) + (t), s)

// One 64-byte block.  M = 16 little-endian message words.
DAS_HD void transform(uint32_t st[4], const uint32_t M[16]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
#define F1(x, y, z) (z ^ (x & (y ^ z)))
#define F2(x, y, z) (y ^ (z & (x ^ y)))
#define F3(x, y, z) (x ^ y ^ z)
#define F4(x, y, z) (y ^ (x | ~z))
  DAS_MD5_STEP(F1(b, c, d), a, b, c, d, M[0], 7, 0xd76aa478u);
  DAS_MD5_STEP(F1(a, b, c), d, a, b, c, M[1], 12, 0xe8c7b756u);
  DAS_MD5_STEP(F1(d, a, b), c, d, a, b, M[2], 17, 0x242070dbu);
  DAS_MD5_STEP(F1(c, d, a), b, c, d, a, M[3], 22, 0xc1bdceeeu);
  DAS_MD5_STEP(F1(b, c, d), a, b, c, d, M[4], 7, 0xf57c0fafu);
  DAS_MD5_STEP(F1(a, b, c), d, a, b, c, M[5], 12, 0x4787c62au);
  DAS_MD5_STEP(F1(d, a, b), c, d, a, b, M[6], 17, 0xa8304613u);
  DAS_MD5_STEP(F1(c, d, a), b, c, d, a, M[7], 22, 0xfd469501u);
  DAS_MD5_STEP(F1(b, c, d), a, b, c, d, M[8], 7, 0x698098d8u);
  DAS_MD5_STEP(F1(a, b, c), d, a, b, c, M[9], 12, 0x8b44f7afu);
  DAS_MD5_STEP(F1(d, a, b), c, d, a, b, M[10], 17, 0xffff5bb1u);
  DAS_MD5_STEP(F1(c, d, a), b, c, d, a, M[11], 22, 0x895cd7beu);
  DAS_MD5_STEP(F1(b, c, d), a, b, c, d, M[12], 7, 0x6b901122u);
  DAS_MD5_STEP(F1(a, b, c), d, a, b, c, M[13], 12, 0xfd987193u);
  DAS_MD5_STEP(F1(d, a, b), c, d, a, b, M[14], 17, 0xa679438eu);
  DAS_MD5_STEP(F1(c, d, a), b, c, d, a, M[15], 22, 0x49b40821u);
  DAS_MD5_STEP(F2(b, c, d), a, b, c, d, M[1], 5, 0xf61e2562u);
  DAS_MD5_STEP(F2(a, b, c), d, a, b, c, M[6], 9, 0xc040b340u);
  DAS_MD5_STEP(F2(d, a, b), c, d, a, b, M[11], 14, 0x265e5a51u);
  DAS_MD5_STEP(F2(c, d, a), b, c, d, a, M[0], 20, 0xe9b6c7aau);
  DAS_MD5_STEP(F2(b, c, d), a, b, c, d, M[5], 5, 0xd62f105du);
  DAS_MD5_STEP(F2(a, b, c), d, a, b, c, M[10], 9, 0x02441453u);
  DAS_MD5_STEP(F2(d, a, b), c, d, a, b, M[15], 14, 0xd8a1e681u);
  DAS_MD5_STEP(F2(c, d, a), b, c, d, a, M[4], 20, 0xe7d3fbc8u);
  DAS_MD5_STEP(F2(b, c, d), a, b, c, d, M[9], 5, 0x21e1cde6u);
  DAS_MD5_STEP(F2(a, b, c), d, a, b, c, M[14], 9, 0xc33707d6u);
  DAS_MD5_STEP(F2(d, a, b), c, d, a, b, M[3], 14, 0xf4d50d87u);
  DAS_MD5_STEP(F2(c, d, a), b, c, d, a, M[8], 20, 0x455a14edu);
  DAS_MD5_STEP(F2(b, c, d), a, b, c, d, M[13], 5, 0xa9e3e905u);
  DAS_MD5_STEP(F2(a, b, c), d, a, b, c, M[2], 9, 0xfcefa3f8u);
  DAS_MD5_STEP(F2(d, a, b), c, d, a, b, M[7], 14, 0x676f02d9u);
  DAS_MD5_STEP(F2(c, d, a), b, c, d, a, M[12], 20, 0x8d2a4c8au);
  DAS_MD5_STEP(F3(b, c, d), a, b, c, d, M[5], 4, 0xfffa3942u);
  DAS_MD5_STEP(F3(a, b, c), d, a, b, c, M[8], 11, 0x8771f681u);
  DAS_MD5_STEP(F3(d, a, b), c, d, a, b, M[11], 16, 0x6d9d6122u);
  DAS_MD5_STEP(F3(c, d, a), b, c, d, a, M[14], 23, 0xfde5380cu);
  DAS_MD5_STEP(F3(b, c, d), a, b, c, d, M[1], 4, 0xa4beea44u);
  DAS_MD5_STEP(F3(a, b, c), d, a, b, c, M[4], 11, 0x4bdecfa9u);
  DAS_MD5_STEP(F3(d, a, b), c, d, a, b, M[7], 16, 0xf6bb4b60u);
  DAS_MD5_STEP(F3(c, d, a), b, c, d, a, M[10], 23, 0xbebfbc70u);
  DAS_MD5_STEP(F3(b, c, d), a, b, c, d, M[13], 4, 0x289b7ec6u);
  DAS_MD5_STEP(F3(a, b, c), d, a, b, c, M[0], 11, 0xeaa127fau);
  DAS_MD5_STEP(F3(d, a, b), c, d, a, b, M[3], 16, 0xd4ef3085u);
  DAS_MD5_STEP(F3(c, d, a), b, c, d, a, M[6], 23, 0x04881d05u);
  DAS_MD5_STEP(F3(b, c, d), a, b, c, d, M[9], 4, 0xd9d4d039u);
  DAS_MD5_STEP(F3(a, b, c), d, a, b, c, M[12], 11, 0xe6db99e5u);
  DAS_MD5_STEP(F3(d, a, b), c, d, a, b, M[15], 16, 0x1fa27cf8u);
  DAS_MD5_STEP(F3(c, d, a), b, c, d, a, M[2], 23, 0xc4ac5665u);
  DAS_MD5_STEP(F4(b, c, d), a, b, c, d, M[0], 6, 0xf4292244u);
  DAS_MD5_STEP(F4(a, b, c), d, a, b, c, M[7], 10, 0x432aff97u);
  DAS_MD5_STEP(F4(d, a, b), c, d, a, b, M[14], 15, 0xab9423a7u);
  DAS_MD5_STEP(F4(c, d, a), b, c, d, a, M[5], 21, 0xfc93a039u);
  DAS_MD5_STEP(F4(b, c, d), a, b, c, d, M[12], 6, 0x655b59c3u);
  DAS_MD5_STEP(F4(a, b, c), d, a, b, c, M[3], 10, 0x8f0ccc92u);
  DAS_MD5_STEP(F4(d, a, b), c, d, a, b, M[10], 15, 0xffeff47du);
  DAS_MD5_STEP(F4(c, d, a), b, c, d, a, M[1], 21, 0x85845dd1u);
  DAS_MD5_STEP(F4(b, c, d), a, b, c, d, M[8], 6, 0x6fa87e4fu);
  DAS_MD5_STEP(F4(a, b, c), d, a, b, c, M[15], 10, 0xfe2ce6e0u);
  DAS_MD5_STEP(F4(d, a, b), c, d, a, b, M[6], 15, 0xa3014314u);
  DAS_MD5_STEP(F4(c, d, a), b, c, d, a, M[13], 21, 0x4e0811a1u);
  DAS_MD5_STEP(F4(b, c, d), a, b, c, d, M[4], 6, 0xf7537e82u);
  DAS_MD5_STEP(F4(a, b, c), d, a, b, c, M[11], 10, 0xbd3af235u);
  DAS_MD5_STEP(F4(d, a, b), c, d, a, b, M[2], 15, 0x2ad7d2bbu);
  DAS_MD5_STEP(F4(c, d, a), b, c, d, a, M[9], 21, 0xeb86d391u);
#undef F1
#undef F2
#undef F3
#undef F4
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
}

DAS_HD void init(uint32_t st[4]) {
  st[0] = 0x67452301u; st[1] = 0xefcdab89u; st[2] = 0x98badcfeu; st[3] = 0x10325476u;
}

// Lowercase hex char of nibble v.
DAS_HD uint32_t hexc(uint32_t v) { return v < 10 ? 0x30u + v : 0x57u + v; }

// Byte `j` (0..31) of the hex string of a digest given as 4 LE words.
DAS_HD uint32_t hex_byte(const uint32_t d[4], uint32_t j) {
  uint32_t byte = (d[j >> 3] >> (((j >> 1) & 3) * 8)) & 0xffu;
  return hexc((j & 1) ? (byte & 0xfu) : (byte >> 4));
}

// Four hex chars (2 digest bytes) packed little-endian into one word:
// chars 4q..4q+3 of the 32-char hex string.
DAS_HD uint32_t hex_word(const uint32_t d[4], uint32_t q) {
  uint32_t b0 = (d[q >> 1] >> ((q & 1) * 16)) & 0xffu;
  uint32_t b1 = (d[q >> 1] >> ((q & 1) * 16 + 8)) & 0xffu;
  return hexc(b0 >> 4) | (hexc(b0 & 0xfu) << 8) | (hexc(b1 >> 4) << 16) | (hexc(b1 & 0xfu) << 24);
}

// Host-side one-shot MD5 of a byte string (query planning; bulk work is on the GPU).
inline void digest_bytes(const uint8_t* p, uint64_t n, uint32_t out[4]) {
  uint32_t st[4];
  init(st);
  uint64_t full = n / 64;
  uint32_t M[16];
  for (uint64_t b = 0; b < full; ++b) {
    for (int i = 0; i < 16; ++i) {
      const uint8_t* q = p + b * 64 + i * 4;
      M[i] = q[0] | (q[1] << 8) | (q[2] << 16) | ((uint32_t)q[3] << 24);
    }
    transform(st, M);
  }
  uint8_t tail[128] = {0};
  uint64_t rem = n - full * 64;
  for (uint64_t i = 0; i < rem; ++i) tail[i] = p[full * 64 + i];
  tail[rem] = 0x80;
  uint64_t tl = (rem + 9 <= 64) ? 64 : 128;
  uint64_t bits = n * 8;
  for (int i = 0; i < 8; ++i) tail[tl - 8 + i] = (uint8_t)(bits >> (8 * i));
  for (uint64_t b = 0; b < tl / 64; ++b) {
    for (int i = 0; i < 16; ++i) {
      const uint8_t* q = tail + b * 64 + i * 4;
      M[i] = q[0] | (q[1] << 8) | (q[2] << 16) | ((uint32_t)q[3] << 24);
    }
    transform(st, M);
  }
  for (int i = 0; i < 4; ++i) out[i] = st[i];
}

inline void to_hex(const uint32_t d[4], char out[32]) {
  for (uint32_t j = 0; j < 32; ++j) out[j] = (char)hex_byte(d, j);
}

inline int from_hex(const char* s, uint32_t d[4]) {
  uint8_t b[16];
  for (int i = 0; i < 16; ++i) {
    int v = 0;
    for (int k = 0; k < 2; ++k) {
      char c = s[2 * i + k];
      int x;
      if (c >= '0' && c <= '9') x = c - '0';
      else if (c >= 'a' && c <= 'f') x = c - 'a' + 10;
      else return -1;
      v = v * 16 + x;
    }
    b[i] = (uint8_t)v;
  }
  for (int i = 0; i < 4; ++i)
    d[i] = b[4 * i] | (b[4 * i + 1] << 8) | (b[4 * i + 2] << 16) | ((uint32_t)b[4 * i + 3] << 24);
  return 0;
}

#undef DAS_HD
}  // namespace md5
}  // namespace das
