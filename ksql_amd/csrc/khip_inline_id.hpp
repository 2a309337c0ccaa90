// khip_inline_id.hpp — the inline id of a digit STRING key (khip_dict.hpp), from its bytes as
// little-endian words.  No HIP dependencies: tests/test_inline_ids.py compiles it on the host
// against a byte-by-byte restatement.
//
// A key of 0..17 ASCII digits → KID_INLINE | len << 57 | decimal value.  SWAR over 8-byte words:
// every byte a digit iff its high nibble is 3 and adding 6 keeps it so; eight digits → their value
// by three multiply-shift steps (pairs, quads, the word), fewer than eight shifted up first (the
// zero bytes shifted in are leading zero digits).
#pragma once
#include <cstdint>

#ifndef KHIP_HD
#if defined(__HIPCC__)
#define KHIP_HD __host__ __device__
#else
#define KHIP_HD
#endif
#endif

namespace khip {

constexpr int64_t KID_INLINE = (int64_t)1 << 62;
constexpr int KEY_INLINE_MAX = 17;

// The low m bytes of w (0 <= m <= 8) are digits?
KHIP_HD inline bool swar_digits(uint64_t w, int m) {
  const uint64_t keep = m >= 8 ? ~0ULL : ((1ULL << (8 * m)) - 1);
  const uint64_t x = (w & keep) | (0x3030303030303030ULL & ~keep);
  return (x & 0xF0F0F0F0F0F0F0F0ULL) == 0x3030303030303030ULL &&
         ((x + 0x0606060606060606ULL) & 0xF0F0F0F0F0F0F0F0ULL) == 0x3030303030303030ULL;
}

// The value of the m digits in the low bytes of w (first digit in byte 0), 1 <= m <= 8.
KHIP_HD inline uint64_t swar_value(uint64_t w, int m) {
  const uint64_t keep = m >= 8 ? ~0ULL : ((1ULL << (8 * m)) - 1);
  uint64_t x = ((w & keep) - (0x3030303030303030ULL & keep)) << (8 * (8 - m));  // low bytes: leading zeros
  x = (x * 10 + (x >> 8)) & 0x00FF00FF00FF00FFULL;               // byte pairs: d0 * 10 + d1
  x = (x * 100 + (x >> 16)) & 0x0000FFFF0000FFFFULL;             // quads
  return (x * 10000 + (x >> 32)) & 0xFFFFFFFFULL;                // the word
}

// w[0..2]: the key's first 24 bytes as words (zero past len).  True and *code when inline.
KHIP_HD inline bool inline_id_words(const uint64_t* w, int64_t len, int64_t* code) {
  if (len < 0 || len > KEY_INLINE_MAX) return false;
  const int L = (int)len;
  const int m0 = L < 8 ? L : 8, m1 = L < 8 ? 0 : (L < 16 ? L - 8 : 8), m2 = L - m0 - m1;
  if (!swar_digits(w[0], m0) || !swar_digits(w[1], m1) || !swar_digits(w[2], m2)) return false;
  uint64_t v = m0 ? swar_value(w[0], m0) : 0;
  if (m1) {
    uint64_t p = 1;
    for (int j = 0; j < m1; j++) p *= 10;
    v = v * p + swar_value(w[1], m1);
  }
  if (m2) v = v * 10 + ((w[2] & 0xFF) - 0x30);
  *code = KID_INLINE | ((int64_t)L << 57) | (int64_t)v;
  return true;
}

}  // namespace khip
