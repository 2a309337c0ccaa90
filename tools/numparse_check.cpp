// CPU check of ksql_amd/csrc/khip_numparse.hpp (test infrastructure): reads lines
// "<kind> <text>" (kind d = Double.parseDouble, l = Long.parseLong, i = Integer.parseInt) and
// prints "ok <value bits or integer>" or "err".
#include <cstdio>
#include <cstring>
#include <string>
#include <iostream>
#include "../ksql_amd/csrc/khip_numparse.hpp"
int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    if (line.size() < 2) { std::puts("err"); continue; }
    const char k = line[0];
    const uint8_t* p = (const uint8_t*)line.data() + 2;
    const int64_t n = (int64_t)line.size() - 2;
    if (k == 'd' || k == 'j') {
      double d;
      const int st = khip::np::java_parse_double(p, n, &d, k == 'd', true);
      if (st != khip::np::PD_OK) { std::puts("err"); continue; }
      uint64_t b;
      memcpy(&b, &d, 8);
      std::printf("ok %llu\n", (unsigned long long)b);
    } else if (k == 'l') {
      int64_t v;
      if (!khip::np::java_parse_long(p, n, &v)) std::puts("err"); else std::printf("ok %lld\n", (long long)v);
    } else {
      int32_t v;
      if (!khip::np::java_parse_int(p, n, &v)) std::puts("err"); else std::printf("ok %d\n", v);
    }
  }
  return 0;
}
