// Host check of khip_inline_id.hpp against a byte-by-byte restatement (tests/test_inline_ids.py).
#include <cstdio>
#include <cstring>
#include <random>
#include <string>

#include "khip_inline_id.hpp"

static bool ref(const std::string& s, int64_t* code) {
  if (s.size() > 17) return false;
  uint64_t v = 0;
  for (char c : s) {
    if (c < '0' || c > '9') return false;
    v = v * 10 + (uint64_t)(c - '0');
  }
  *code = khip::KID_INLINE | ((int64_t)s.size() << 57) | (int64_t)v;
  return true;
}

static bool swar(const std::string& s, int64_t* code) {
  uint64_t w[3] = {0, 0, 0};
  memcpy(w, s.data(), s.size() < 24 ? s.size() : 24);
  return khip::inline_id_words(w, (int64_t)s.size(), code);
}

int main() {
  std::mt19937_64 rng(7);
  const char alpha[] = "0123456789/:.-+ aZ\xff\x30\x39";
  long n = 0, bad = 0;
  auto check = [&](const std::string& s) {
    int64_t a = 0, b = 0;
    const bool ra = ref(s, &a), rb = swar(s, &b);
    n++;
    if (ra != rb || (ra && a != b)) {
      if (bad++ < 10) printf("MISMATCH len %zu '%s': ref %d %lld swar %d %lld\n", s.size(), s.c_str(), ra, (long long)a, rb, (long long)b);
    }
  };
  for (int len = 0; len <= 24; len++) {
    for (int t = 0; t < 20000; t++) {
      std::string s(len, '0');
      const bool digits = (t & 3) != 0;
      for (int j = 0; j < len; j++) s[j] = digits ? (char)('0' + rng() % 10) : alpha[rng() % (sizeof(alpha) - 1)];
      if (digits && len && (t & 7) == 1) s[rng() % len] = alpha[10 + rng() % 8];  // one non-digit
      check(s);
    }
    check(std::string(len, '9'));
    check(std::string(len, '0'));
  }
  printf("%ld cases, %ld mismatches\n", n, bad);
  return bad ? 1 : 0;
}
