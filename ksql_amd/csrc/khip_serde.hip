// khip_serde.hip — deserialization of Kafka record bytes into device columns (gfx950).
//
// Replaces, for the hot path's source topics, the per-record GenericKeySerDe / GenericRowSerDe
// deserializers (KAFKA, DELIMITED, JSON, AVRO; include/ksqldb_hip.h "deserialization") that box every
// record into a GenericKey / GenericRow before the aggregate or join sees it — the reference's
// documented bottleneck (ksqldb-benchmark/README.md:7-9).
//
// Layout: the raw batch is the consumer's view — concatenated key / value bytes with n + 1
// offsets and null bitmaps.  One thread decodes one record (records are tens to hundreds of
// bytes; neighbouring threads read neighbouring bytes, so the loads stay cache friendly); each
// wave assembles the validity bitmaps of its 64 records with ballots (one 8-byte store per
// bitmap).  Numbers are converted exactly as Java does (khip_numparse.hpp); the rare double
// with more than 19 significant digits whose rounding needs big-integer arithmetic is finished
// by a second kernel (k_serde_fix) over just those fields, so the decode kernel keeps a small
// stack.
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "khip_util.hpp"
#include "khip_numparse.hpp"
#include "khip_upper.inc"

namespace khip {

constexpr int SD_MAX_FIELDS = 32;
constexpr int SD_NAME_BYTES = 64;

struct SerdeParams {
  int32_t key_format, key_type, value_format, n_fields, delimiter, n_out;
  int32_t ftype[SD_MAX_FIELDS];
  int32_t fout[SD_MAX_FIELDS];
  int32_t name_len[SD_MAX_FIELDS];
  uint8_t name[SD_MAX_FIELDS][SD_NAME_BYTES];
  // AVRO: the writer schema's fields in order: type (KHIP_AVRO_*), union (0 plain, 1 [null, T],
  // 2 [T, null]) and the ksql field (column schema index) it lands in, or -1
  int32_t avro_id, avro_nw, avro_incompat;
  int8_t aw_type[SD_MAX_FIELDS], aw_union[SD_MAX_FIELDS], aw_field[SD_MAX_FIELDS];
};

struct SerdeOut {
  int64_t* key_i64;
  uint8_t* key_valid;
  uint8_t* row_valid;
  void* col[SD_MAX_FIELDS];
  uint8_t* col_valid[SD_MAX_FIELDS];
  unsigned long long* n_err;
  unsigned long long* n_fix;
  int64_t* fix;  // (row, out column, byte offset, length | json flag << 32) per deferred double
  int64_t fix_cap;
};

// a field's value as the decode loop found it
struct Tok {
  int32_t off, len;  // bytes (for strings: between the quotes)
  int8_t kind;       // -1 absent, 0 null, 1 number, 2 string, 3 literal (true / false), 4 object / array
  int8_t esc;        // string with escapes
};

__device__ __forceinline__ uint64_t be_load(const uint8_t* p, int n) {
  uint64_t v = 0;
  for (int i = 0; i < n; i++) v = v << 8 | p[i];
  return v;
}

// (int) d and (long) d in Java: NaN → 0, saturating.
__device__ __forceinline__ int64_t java_d2l(double d) {
  if (d != d) return 0;
  if (d >= 9.2233720368547758e18) return INT64_MAX;
  if (d <= -9.2233720368547758e18) return INT64_MIN;
  return (int64_t)d;
}
__device__ __forceinline__ int32_t java_d2i(double d) {
  if (d != d) return 0;
  if (d >= 2147483647.0) return INT32_MAX;
  if (d <= -2147483648.0) return INT32_MIN;
  return (int32_t)d;
}

// Avro binary varint (BinaryDecoder.readInt / readLong): at most maxb bytes (5 / 10), the last one
// without a continuation bit ("Invalid int / long encoding" otherwise); bits past 64 are dropped
// (readInt's past 32 by the caller's truncation); the zig-zag decoding is the caller's.
__device__ __forceinline__ bool avro_varint(const uint8_t* p, int64_t n, int64_t* j, int maxb, uint64_t* out) {
  uint64_t v = 0;
  for (int k = 0; k < maxb; k++) {
    if (*j >= n) return false;  // EOFException
    const uint8_t b = p[(*j)++];
    v |= (uint64_t)(b & 0x7F) << (7 * k);
    if (!(b & 0x80)) {
      *out = v;
      return true;
    }
  }
  return false;
}

__device__ __forceinline__ int64_t zz64(uint64_t v) { return (int64_t)(v >> 1) ^ -(int64_t)(v & 1); }
__device__ __forceinline__ int32_t zz32(uint32_t v) { return (int32_t)(v >> 1) ^ -(int32_t)(v & 1); }

__device__ __forceinline__ uint64_t le_load(const uint8_t* p, int n) {
  uint64_t v = 0;
  for (int i = n - 1; i >= 0; i--) v = v << 8 | p[i];
  return v;
}

__device__ __forceinline__ bool json_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

// Skip one JSON value starting at p[i] (i < n, not whitespace); returns the index after it or -1.
__device__ int64_t json_skip(const uint8_t* p, int64_t i, int64_t n, Tok* t) {
  const uint8_t c = p[i];
  if (c == '"') {
    int64_t j = i + 1;
    int esc = 0;
    while (j < n && p[j] != '"') {
      if (p[j] == '\\') {
        esc = 1;
        j++;
      }
      j++;
    }
    if (j >= n) return -1;
    t->kind = 2;
    t->off = (int32_t)(i + 1);
    t->len = (int32_t)(j - i - 1);
    t->esc = (int8_t)esc;
    return j + 1;
  }
  if (c == '{' || c == '[') {
    int depth = 0;
    int64_t j = i;
    for (; j < n; j++) {
      const uint8_t d = p[j];
      if (d == '"') {
        j++;
        while (j < n && p[j] != '"') j += p[j] == '\\' ? 2 : 1;
        if (j >= n) return -1;
      } else if (d == '{' || d == '[') {
        depth++;
      } else if (d == '}' || d == ']') {
        if (--depth == 0) break;
      }
    }
    if (j >= n) return -1;
    t->kind = 4;
    t->off = (int32_t)i;
    t->len = (int32_t)(j + 1 - i);
    return j + 1;
  }
  if (c == 'n' || c == 't' || c == 'f') {
    const char* lit = c == 'n' ? "null" : (c == 't' ? "true" : "false");
    const int L = c == 'f' ? 5 : 4;
    if (i + L > n) return -1;
    for (int k = 0; k < L; k++)
      if (p[i + k] != (uint8_t)lit[k]) return -1;
    t->kind = c == 'n' ? 0 : 3;
    t->off = (int32_t)i;
    t->len = L;
    return i + L;
  }
  // number: -?(0|[1-9]d*)(.d+)?([eE][+-]?d+)?  (Jackson's strict grammar)
  int64_t j = i;
  if (p[j] == '-') j++;
  if (j >= n || !np::is_digit(p[j])) return -1;
  if (p[j] == '0') {
    j++;
    if (j < n && np::is_digit(p[j])) return -1;  // leading zero
  } else {
    while (j < n && np::is_digit(p[j])) j++;
  }
  if (j < n && p[j] == '.') {
    j++;
    if (j >= n || !np::is_digit(p[j])) return -1;
    while (j < n && np::is_digit(p[j])) j++;
  }
  if (j < n && (p[j] == 'e' || p[j] == 'E')) {
    j++;
    if (j < n && (p[j] == '+' || p[j] == '-')) j++;
    if (j >= n || !np::is_digit(p[j])) return -1;
    while (j < n && np::is_digit(p[j])) j++;
  }
  t->kind = 1;
  t->off = (int32_t)i;
  t->len = (int32_t)(j - i);
  return j;
}

// Case-insensitive field names: Java's String.toUpperCase() (default, non-tr/az/lt locale: the
// full unconditional Unicode mapping, e.g. "straße" → "STRASSE", "ǆ" → "Ǆ"), through the table
// tools/gen_upper.py generates (khip_upper.inc: the non-ASCII code points that change).
__constant__ uint32_t kUpperDev[KHIP_UPPER_N * 4] = KHIP_UPPER_TABLE;
static const uint32_t kUpperHost[KHIP_UPPER_N * 4] = KHIP_UPPER_TABLE;

__host__ __device__ inline uint8_t up(uint8_t c) { return c >= 'a' && c <= 'z' ? c - 32 : c; }

// One UTF-8 code point at s[i..n): its length, or 0 when the bytes are not well-formed.
__host__ __device__ inline int utf8_dec(const uint8_t* s, int n, int i, uint32_t* cp) {
  const uint8_t c = s[i];
  int l = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC0 ? 2 : 0;
  if (!l || c >= 0xF8 || i + l > n) return 0;
  uint32_t v = c & (0x7F >> l);
  for (int k = 1; k < l; k++) {
    if ((s[i + k] & 0xC0) != 0x80) return 0;
    v = (v << 6) | (s[i + k] & 0x3F);
  }
  if ((l == 2 && v < 0x80) || (l == 3 && v < 0x800) || (l == 4 && (v < 0x10000 || v > 0x10FFFF))) return 0;
  if (v >= 0xD800 && v < 0xE000) return 0;
  *cp = v;
  return l;
}

__host__ __device__ inline int utf8_enc(uint32_t cp, uint8_t* o) {
  if (cp < 0x80) { o[0] = (uint8_t)cp; return 1; }
  if (cp < 0x800) { o[0] = (uint8_t)(0xC0 | (cp >> 6)); o[1] = (uint8_t)(0x80 | (cp & 0x3F)); return 2; }
  if (cp < 0x10000) {
    o[0] = (uint8_t)(0xE0 | (cp >> 12));
    o[1] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
    o[2] = (uint8_t)(0x80 | (cp & 0x3F));
    return 3;
  }
  o[0] = (uint8_t)(0xF0 | (cp >> 18));
  o[1] = (uint8_t)(0x80 | ((cp >> 12) & 0x3F));
  o[2] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
  o[3] = (uint8_t)(0x80 | (cp & 0x3F));
  return 4;
}

// Upper-case mapping of a non-ASCII code point: up to three code points (unused = 0).
__host__ __device__ inline void upper_cp(const uint32_t* tab, uint32_t cp, uint32_t m[3]) {
  int lo = 0, hi = KHIP_UPPER_N;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (tab[mid * 4] < cp) lo = mid + 1;
    else hi = mid;
  }
  if (lo < KHIP_UPPER_N && tab[lo * 4] == cp) {
    m[0] = tab[lo * 4 + 1];
    m[1] = tab[lo * 4 + 2];
    m[2] = tab[lo * 4 + 3];
  } else {
    m[0] = cp;
    m[1] = m[2] = 0;
  }
}

// toUpperCase(a) == b, byte for byte (a, b UTF-8; a malformed a matches nothing).
__host__ __device__ inline bool upper_equals(const uint32_t* tab, const uint8_t* a, int na, const uint8_t* b, int nb) {
  int j = 0;
  for (int i = 0; i < na;) {
    if (a[i] < 0x80) {
      if (j >= nb || b[j] != up(a[i])) return false;
      i++;
      j++;
      continue;
    }
    uint32_t cp, m[3];
    const int l = utf8_dec(a, na, i, &cp);
    if (!l) return false;
    i += l;
    upper_cp(tab, cp, m);
    for (int k = 0; k < 3 && (k == 0 || m[k]); k++) {
      uint8_t e[4];
      const int el = utf8_enc(m[k], e);
      for (int x = 0; x < el; x++, j++)
        if (j >= nb || b[j] != e[x]) return false;
    }
  }
  return j == nb;
}

static std::string upper_utf8_host(const char* s) {
  const int n = (int)strlen(s);
  const uint8_t* a = (const uint8_t*)s;
  std::string out;
  for (int i = 0; i < n;) {
    if (a[i] < 0x80) {
      out.push_back((char)up(a[i++]));
      continue;
    }
    uint32_t cp, m[3];
    const int l = utf8_dec(a, n, i, &cp);
    if (!l) {  // malformed: kept as is (matches no ksql field name upper-cased by Java)
      out.push_back((char)a[i++]);
      continue;
    }
    i += l;
    upper_cp(kUpperHost, cp, m);
    for (int k = 0; k < 3 && (k == 0 || m[k]); k++) {
      uint8_t e[4];
      out.append((const char*)e, (size_t)utf8_enc(m[k], e));
    }
  }
  return out;
}

__device__ __forceinline__ bool hex4(const uint8_t* p, int64_t n, int64_t i, uint32_t* u) {
  if (i + 4 > n) return false;
  uint32_t v = 0;
  for (int k = 0; k < 4; k++) {
    const uint8_t h = p[i + k];
    const int d = h >= '0' && h <= '9' ? h - '0' : (h >= 'a' && h <= 'f' ? h - 'a' + 10 : (h >= 'A' && h <= 'F' ? h - 'A' + 10 : -1));
    if (d < 0) return false;
    v = v * 16 + (uint32_t)d;
  }
  *u = v;
  return true;
}

// JSON string unescape into buf (cap bytes); false on a bad escape or overflow.
__device__ bool json_unescape(const uint8_t* p, int64_t n, uint8_t* buf, int cap, int* outn) {
  int m = 0;
  for (int64_t i = 0; i < n; i++) {
    uint32_t c = p[i];
    bool cp = false;  // c is a code point from a \\u escape (else one raw byte)
    if (c == '\\') {
      if (++i >= n) return false;
      switch (p[i]) {
        case '"': c = '"'; break;
        case '\\': c = '\\'; break;
        case '/': c = '/'; break;
        case 'b': c = 8; break;
        case 'f': c = 12; break;
        case 'n': c = 10; break;
        case 'r': c = 13; break;
        case 't': c = 9; break;
        case 'u': {
          uint32_t u;
          if (!hex4(p, n, i + 1, &u)) return false;
          i += 4;
          if (u >= 0xD800 && u < 0xDC00) {  // a surrogate pair → one supplementary code point
            uint32_t lo;
            if (i + 2 >= n || p[i + 1] != '\\' || p[i + 2] != 'u' || !hex4(p, n, i + 3, &lo) || lo < 0xDC00 ||
                lo >= 0xE000)
              return false;  // a lone surrogate (matches no UTF-8 name, forms no number)
            i += 6;
            u = 0x10000 + ((u - 0xD800) << 10) + (lo - 0xDC00);
          } else if (u >= 0xDC00 && u < 0xE000) {
            return false;
          }
          c = u;
          cp = true;
          break;
        }
        default: return false;
      }
    }
    if (!cp || c < 0x80) {
      if (m >= cap) return false;
      buf[m++] = (uint8_t)c;
    } else {  // \u escapes of non-ASCII code points, as UTF-8 (raw bytes >= 0x80 pass through above)
      uint8_t e[4];
      const int el = utf8_enc(c, e);
      if (m + el > cap) return false;
      for (int k = 0; k < el; k++) buf[m++] = e[k];
    }
  }
  *outn = m;
  return true;
}


// Jackson reads a JSON number token with a fraction or an exponent as a BigDecimal
// (USE_BIG_DECIMAL_FOR_FLOATS, KsqlJsonDeserializer.java:68-70); JsonSerdeUtils.toInteger /
// toLong (:95-121) then take intValue() / asLong(): the integer part truncated toward zero, its
// low 32 / 64 bits.  Computed exactly from the digits: D x 10^s with s >= 64 is a multiple of 2^64;
// s < 0 drops the last -s digits.  false: the token is not a number BigDecimal accepts (its
// exponent must fit an int).
__device__ bool json_bigdec_low64(const uint8_t* p, int64_t n, uint64_t* out) {
  int64_t k = 0;
  const bool neg = n > 0 && p[0] == '-';
  if (neg) k++;
  const int64_t i0 = k;
  while (k < n && p[k] >= '0' && p[k] <= '9') k++;
  const int64_t i1 = k;
  int64_t f0 = k, f1 = k;
  if (k < n && p[k] == '.') {
    f0 = ++k;
    while (k < n && p[k] >= '0' && p[k] <= '9') k++;
    f1 = k;
  }
  if (i1 == i0 && f1 == f0) return false;
  int64_t e = 0;
  if (k < n && (p[k] == 'e' || p[k] == 'E')) {
    k++;
    bool en = false;
    if (k < n && (p[k] == '+' || p[k] == '-')) en = p[k++] == '-';
    if (k >= n) return false;
    for (; k < n && p[k] >= '0' && p[k] <= '9'; k++) {
      e = e * 10 + (p[k] - '0');
      if (e > 0x7FFFFFFFLL) return false;  // BigDecimal: exponent overflow
    }
    if (en) e = -e;
  }
  if (k != n) return false;
  const int64_t nint = i1 - i0, nfrac = f1 - f0;
  const int64_t s = e - nfrac;  // value = D x 10^s, D = the int digits then the fraction digits
  const int64_t keep = s >= 0 ? nint + nfrac : nint + nfrac + s;
  uint64_t v = 0;
  for (int64_t j = 0; j < keep; j++) v = v * 10 + (uint64_t)(p[j < nint ? i0 + j : f0 + (j - nint)] - '0');
  if (s >= 64) v = 0;
  for (int64_t j = 0; j < s && j < 64; j++) v *= 10;
  *out = neg ? 0 - v : v;
  return true;
}

// A numeric field (raw text p[0..n), json: a JSON number token, else Java text) → column.
// Returns 0 ok, 1 error, 2 deferred (big-integer rounding).
__device__ int put_number(const SerdeParams& q, int f, const uint8_t* p, int64_t n, bool json_num, void* col,
                          int64_t row) {
  const int t = q.ftype[f];
  if (json_num) {
    bool is_int = true;
    for (int64_t k = 0; k < n; k++)
      if (p[k] == '.' || p[k] == 'e' || p[k] == 'E') is_int = false;
    if (is_int && t != KHIP_TYPE_DOUBLE) {  // intValue() / asLong(): the low 32 / 64 bits of the integer
      uint64_t v = 0;
      int64_t k = p[0] == '-' ? 1 : 0;
      for (; k < n; k++) v = v * 10 + (p[k] - '0');
      if (p[0] == '-') v = 0 - v;
      if (!col) return 0;
      if (t == KHIP_TYPE_INT32) ((int32_t*)col)[row] = (int32_t)(uint32_t)v;
      else ((int64_t*)col)[row] = (int64_t)v;
      return 0;
    }
    if (t != KHIP_TYPE_DOUBLE) {  // BigDecimal → intValue() / longValue()
      uint64_t v;
      if (!json_bigdec_low64(p, n, &v)) return 1;
      if (!col) return 0;
      if (t == KHIP_TYPE_INT32) ((int32_t*)col)[row] = (int32_t)(uint32_t)v;
      else ((int64_t*)col)[row] = (int64_t)v;
      return 0;
    }
    double d;
    const int st = np::java_parse_double(p, n, &d, false, false);
    if (st != np::PD_OK) return col || st == 1 ? st : 0;  // an unread field's exact rounding is moot
    if (!col) return 0;
    if (t == KHIP_TYPE_INT32) ((int32_t*)col)[row] = java_d2i(d);
    else if (t == KHIP_TYPE_INT64) ((int64_t*)col)[row] = java_d2l(d);
    else ((double*)col)[row] = d;
    return 0;
  }
  if (t == KHIP_TYPE_INT32) {
    int32_t v;
    if (!np::java_parse_int(p, n, &v)) return 1;
    if (col) ((int32_t*)col)[row] = v;
  } else if (t == KHIP_TYPE_INT64) {
    int64_t v;
    if (!np::java_parse_long(p, n, &v)) return 1;
    if (col) ((int64_t*)col)[row] = v;
  } else {
    double d;
    const int st = np::java_parse_double(p, n, &d, true, false);
    if (st != np::PD_OK) return col || st == 1 ? st : 0;
    if (col) ((double*)col)[row] = d;
  }
  return 0;
}

// Stage the bytes [b0, b1) of `base` (one wave's records: the offsets are monotone) into the
// wave's LDS buffer with dword loads (coalesced); the record parsers then read LDS instead of
// issuing one global byte load per character.  Returns false (nothing staged) when the range does
// not fit.  lds byte of global byte x = buf + (x - *shift).
template <int WORDS>
__device__ __forceinline__ bool stage_bytes(uint32_t* buf, const uint8_t* base, int64_t b0, int64_t b1, int lane,
                                            int64_t* shift) {
  const uintptr_t ua = ((uintptr_t)(base + b0)) & ~(uintptr_t)3;
  const uintptr_t ue = (uintptr_t)(base + b1);
  const int64_t words = (int64_t)((ue - ua + 3) >> 2);
  if (b1 <= b0 || words > WORDS) return false;
  for (int64_t x = lane; x < words; x += 64) {
    const uintptr_t a = ua + 4 * (uintptr_t)x;
    uint32_t w;
    if (a >= (uintptr_t)(base + b0) && a + 4 <= ue) {
      w = *(const uint32_t*)a;
    } else {  // the range's partial first / last dword: only its bytes inside [b0, b1)
      w = 0;
      for (int k = 0; k < 4; k++) {
        const uintptr_t ak = a + k;
        if (ak >= (uintptr_t)(base + b0) && ak < ue) w |= (uint32_t)(*(const uint8_t*)ak) << (8 * k);
      }
    }
    buf[x] = w;
  }
  *shift = (int64_t)(ua - (uintptr_t)base);
  return true;
}

constexpr int SERDE_VWORDS = 1024;  // 4 KB of value bytes per wave (64 records of <= 64 bytes)
constexpr int SERDE_KWORDS = 256;   // 1 KB of key bytes per wave

// MAXF: compile-time bound on the schema's field count: the JSON field-token arrays (private
// memory) shrink to the schema (4 for the common narrow schemas; 32 otherwise).
template <int MAXF>
__global__ __launch_bounds__(256) void k_serde_decode(SerdeParams q, int64_t n, const int64_t* __restrict__ koff,
                                                      const uint8_t* __restrict__ kbytes, const uint8_t* __restrict__ kval,
                                                      const int64_t* __restrict__ voff, const uint8_t* __restrict__ vbytes,
                                                      const uint8_t* __restrict__ vval, SerdeOut o) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ uint32_t vst[4][SERDE_VWORDS];
  __shared__ uint32_t kst[4][SERDE_KWORDS];
  const int64_t w0 = i - lane, wl = (n - 1 < w0 + 63) ? n - 1 : w0 + 63;
  int64_t vshift = 0, kshift = 0;
  bool vstaged = false, kstaged = false;
  if (w0 < n) {
    vstaged = stage_bytes<SERDE_VWORDS>(vst[wave], vbytes, voff[w0], voff[wl + 1], lane, &vshift);
    if (q.key_format != KHIP_FMT_NONE && kbytes)
      kstaged = stage_bytes<SERDE_KWORDS>(kst[wave], kbytes, koff[w0], koff[wl + 1], lane, &kshift);
  }
  __syncthreads();
  // byte x of the record bytes: staged ? LDS[x - shift] : global[x]
  auto vat = [&](int64_t x) { return vstaged ? (const uint8_t*)vst[wave] + (x - vshift) : vbytes + x; };
  auto kat = [&](int64_t x) { return kstaged ? (const uint8_t*)kst[wave] + (x - kshift) : kbytes + x; };
  bool ok = i < n;  // deserialized without error
  bool key_ok = false, row_ok = false;
  uint32_t fnull = 0;  // per output column: NULL
  if (i < n) {
    // ---- key (KAFKA format)
    if (q.key_format == KHIP_FMT_NONE) {
      key_ok = true;
      if (o.key_i64) o.key_i64[i] = 0;
    } else if (bit_get(kval, i)) {
      const int64_t k0 = koff[i], kn = koff[i + 1] - k0;
      if (q.key_type == KHIP_TYPE_INT64) {
        if (kn == 8) o.key_i64[i] = (int64_t)be_load(kat(k0), 8);
        else ok = false;
      } else if (q.key_type == KHIP_TYPE_INT32) {
        if (kn == 4) o.key_i64[i] = (int64_t)(int32_t)(uint32_t)be_load(kat(k0), 4);
        else ok = false;
      }
      key_ok = true;  // STRING keys: the bytes themselves
    }
    // ---- value
    row_ok = bit_get(vval, i);
    if (ok && row_ok) {
      const int64_t v0 = voff[i], vn = voff[i + 1] - v0;
      const uint8_t* p = vat(v0);
      for (int c = 0; c < q.n_out; c++) fnull |= 1u << c;
      if (q.value_format == KHIP_FMT_KAFKA) {
        const int f = 0;
        const int c = q.fout[f];
        const int t = q.ftype[f];
        if (t == KHIP_TYPE_INT32 && vn != 4) ok = false;
        else if ((t == KHIP_TYPE_INT64 || t == KHIP_TYPE_DOUBLE) && vn != 8) ok = false;
        else if (c >= 0) {
          fnull &= ~(1u << c);
          if (t == KHIP_TYPE_INT32) ((int32_t*)o.col[c])[i] = (int32_t)(uint32_t)be_load(p, 4);
          else if (t == KHIP_TYPE_STRING) ((int64_t*)o.col[c])[i] = 0;
          else ((uint64_t*)o.col[c])[i] = be_load(p, 8);
        }
      } else if (q.value_format == KHIP_FMT_DELIMITED) {
        // CSVFormat.DEFAULT: RFC 4180 fields, quote '"' (doubled inside), first record only
        int64_t j = 0;
        int f = 0;
        bool more = vn > 0;
        if (!more) ok = false;  // "No fields in record"
        while (ok && more) {
          int64_t s, e;
          bool quoted = false, inner_quote = false;
          if (j < vn && p[j] == '"') {
            quoted = true;
            int64_t k = j + 1;
            while (true) {
              if (k >= vn) { ok = false; break; }  // EOF inside an encapsulated token
              if (p[k] == '"') {
                if (k + 1 < vn && p[k + 1] == '"') { inner_quote = true; k += 2; continue; }
                break;
              }
              k++;
            }
            if (!ok) break;
            s = j + 1;
            e = k;
            j = k + 1;
            if (j < vn && p[j] != q.delimiter && p[j] != '\n' && p[j] != '\r') { ok = false; break; }
          } else {
            s = j;
            while (j < vn && p[j] != q.delimiter && p[j] != '\n' && p[j] != '\r') j++;
            e = j;
          }
          more = j < vn && p[j] == q.delimiter;
          j++;
          if (f >= q.n_fields) { ok = false; break; }  // column count mismatch
          const int c = q.fout[f];
          if (e > s && q.ftype[f] != KHIP_TYPE_STRING) {  // every field parses (an unread one too)
            const int st = inner_quote ? 1 : put_number(q, f, p + s, e - s, false, c >= 0 ? o.col[c] : nullptr, i);
            if (st == 1) { ok = false; break; }
            if (st == 2) {
              const unsigned long long slot = atomicAdd(o.n_fix, 1ULL);
              if ((int64_t)slot < o.fix_cap) {
                o.fix[4 * slot] = i;
                o.fix[4 * slot + 1] = c;
                o.fix[4 * slot + 2] = v0 + s;
                o.fix[4 * slot + 3] = e - s;
              }
            }
            if (c >= 0) fnull &= ~(1u << c);
          } else if (e > s && c >= 0) {  // a non-empty VARCHAR (empty field = NULL)
            ((int64_t*)o.col[c])[i] = 0;
            fnull &= ~(1u << c);
          }
          (void)quoted;
          f++;
        }
        if (ok && f != q.n_fields) ok = false;
      } else if (q.value_format == KHIP_FMT_AVRO) {
        // Confluent wire format: magic 0, 4-byte big-endian schema id, the writer record's fields in
        // order; each lands in its ksql column (by name, resolved at create) or is skipped
        if (vn < 5 || p[0] != 0 || q.avro_incompat) ok = false;
        else if (q.avro_id >= 0 && (int32_t)(uint32_t)be_load(p + 1, 4) != q.avro_id) ok = false;
        int64_t j = 5;
        for (int w = 0; ok && w < q.avro_nw; w++) {
          bool isnull = false;
          if (q.aw_union[w]) {  // readIndex() = readInt()
            uint64_t br;
            if (!avro_varint(p, vn, &j, 5, &br)) { ok = false; break; }
            const int32_t idx = zz32((uint32_t)br);
            if (idx != 0 && idx != 1) { ok = false; break; }  // no such union branch
            isnull = idx == q.aw_union[w] - 1;
          }
          const int f = q.aw_field[w];
          const int c = f >= 0 ? q.fout[f] : -1;
          if (isnull) {
            if (c >= 0) fnull |= 1u << c;  // a later field of the same column overwrites
            continue;
          }
          uint64_t bits = 0;  // the value as the column stores it
          switch (q.aw_type[w]) {
            case KHIP_AVRO_BOOLEAN:
              if (j >= vn) { ok = false; break; }
              bits = p[j++] == 1;
              break;
            case KHIP_AVRO_INT: {
              uint64_t v;
              if (!avro_varint(p, vn, &j, 5, &v)) { ok = false; break; }
              bits = (uint64_t)(int64_t)zz32((uint32_t)v);
              break;
            }
            case KHIP_AVRO_LONG: {
              uint64_t v;
              if (!avro_varint(p, vn, &j, 10, &v)) { ok = false; break; }
              bits = (uint64_t)zz64(v);
              break;
            }
            case KHIP_AVRO_FLOAT: {
              if (vn - j < 4) { ok = false; break; }
              const uint32_t u = (uint32_t)le_load(p + j, 4);
              j += 4;
              float fv;
              __builtin_memcpy(&fv, &u, 4);
              const double dv = (double)fv;  // Number.doubleValue() of a Float
              __builtin_memcpy(&bits, &dv, 8);
              break;
            }
            case KHIP_AVRO_DOUBLE:
              if (vn - j < 8) { ok = false; break; }
              bits = le_load(p + j, 8);
              j += 8;
              break;
            default: {  // STRING / BYTES: long length, then the bytes
              uint64_t v;
              if (!avro_varint(p, vn, &j, 10, &v)) { ok = false; break; }
              const int64_t len = zz64(v);
              if (len < 0 || len > vn - j) { ok = false; break; }  // negative length / EOF
              j += len;
              break;
            }
          }
          if (!ok || c < 0) continue;
          fnull &= ~(1u << c);
          const int t = q.ftype[f];
          if (t == KHIP_TYPE_INT32) ((int32_t*)o.col[c])[i] = (int32_t)bits;
          else if (t == KHIP_TYPE_STRING) ((int64_t*)o.col[c])[i] = 0;  // String.valueOf(any primitive)
          else ((uint64_t*)o.col[c])[i] = bits;  // BIGINT (int widened) / DOUBLE (float widened)
        }
      } else {  // JSON
        int64_t j = 0;
        while (j < vn && json_ws(p[j])) j++;
        if (j >= vn || p[j] != '{') ok = false;
        Tok ex[MAXF], ci[MAXF];
        for (int f = 0; f < q.n_fields; f++) {
          ex[f].kind = -1;
          ci[f].kind = -1;
        }
        j++;
        bool first = true;
        while (ok) {
          while (j < vn && json_ws(p[j])) j++;
          if (j >= vn) { ok = false; break; }
          if (p[j] == '}') { if (!first) ok = false; break; }  // "{}" only (trailing commas are errors)
          first = false;
          Tok kt;
          const int64_t kend = p[j] == '"' ? json_skip(p, j, vn, &kt) : -1;
          if (kend < 0) { ok = false; break; }
          j = kend;
          while (j < vn && json_ws(p[j])) j++;
          if (j >= vn || p[j] != ':') { ok = false; break; }
          j++;
          while (j < vn && json_ws(p[j])) j++;
          if (j >= vn) { ok = false; break; }
          Tok vt;
          vt.esc = 0;
          const int64_t vend = json_skip(p, j, vn, &vt);
          if (vend < 0) { ok = false; break; }
          j = vend;
          // field name: exact match wins, else the upper-cased name (last such field; Unicode
          // upper case as Java's toUpperCase, KsqlJsonDeserializer.java:301-306)
          uint8_t nb[SD_NAME_BYTES];
          int nl = 0;
          const uint8_t* kp = p + kt.off;
          if (kt.esc) {
            if (!json_unescape(p + kt.off, kt.len, nb, SD_NAME_BYTES, &nl)) nl = -1;
            kp = nb;
          } else {
            nl = kt.len <= SD_NAME_BYTES ? (int)kt.len : -1;
          }
          if (nl >= 0) {
            for (int f = 0; f < q.n_fields; f++) {
              bool same = q.name_len[f] == nl;
              for (int k = 0; same && k < nl; k++) same = kp[k] == q.name[f][k];
              if (same) ex[f] = vt;
              else if (upper_equals(kUpperDev, kp, nl, q.name[f], q.name_len[f])) ci[f] = vt;
            }
          }
          while (j < vn && json_ws(p[j])) j++;
          if (j < vn && p[j] == ',') { j++; continue; }
          if (j < vn && p[j] == '}') break;
          ok = false;
        }
        for (int f = 0; ok && f < q.n_fields; f++) {  // every schema field is coerced (:273-300)
          const int c = q.fout[f];
          const Tok t = ex[f].kind >= 0 ? ex[f] : ci[f];
          if (t.kind <= 0) continue;  // missing or JSON null: NULL
          if (q.ftype[f] == KHIP_TYPE_STRING) {  // asText(): any value is a non-null string
            if (c >= 0) {
              ((int64_t*)o.col[c])[i] = 0;
              fnull &= ~(1u << c);
            }
            continue;
          }
          if (t.kind != 1 && t.kind != 2) { ok = false; break; }  // boolean / object / array
          int st;
          if (t.kind == 2) {  // a string: Integer.parseInt / Long.parseLong / Double.parseDouble
            uint8_t sb[96];
            int sn;
            const uint8_t* sp = p + t.off;
            int64_t sl = t.len;
            if (t.esc) {
              if (!json_unescape(p + t.off, t.len, sb, 96, &sn)) { ok = false; break; }
              sp = sb;
              sl = sn;
            }
            st = put_number(q, f, sp, sl, false, c >= 0 ? o.col[c] : nullptr, i);
            if (st == 2 && t.esc) st = 1;  // escaped long decimals: not supported here
          } else {
            st = put_number(q, f, p + t.off, t.len, true, c >= 0 ? o.col[c] : nullptr, i);
          }
          if (st == 1) { ok = false; break; }
          if (c < 0) continue;
          if (st == 2) {
            const unsigned long long slot = atomicAdd(o.n_fix, 1ULL);
            if ((int64_t)slot < o.fix_cap) {
              o.fix[4 * slot] = i;
              o.fix[4 * slot + 1] = c;
              o.fix[4 * slot + 2] = v0 + t.off;
              o.fix[4 * slot + 3] = t.len | (t.kind == 1 ? (1LL << 32) : 0);
            }
          }
          fnull &= ~(1u << c);
        }
      }
    }
  }
  const bool err = i < n && !ok;
  const uint64_t bk = __ballot(i < n && ok && key_ok), br = __ballot(i < n && ok && row_ok);
  const int64_t wbase = i - lane;
  if (lane == 0 && wbase < n) {
    const int64_t nbytes = std::min<int64_t>(8, (n - wbase + 7) / 8);
    for (int b = 0; b < nbytes; b++) {
      o.key_valid[wbase / 8 + b] = (uint8_t)(bk >> (8 * b));
      o.row_valid[wbase / 8 + b] = (uint8_t)(br >> (8 * b));
    }
  }
  for (int c = 0; c < q.n_out; c++) {
    const uint64_t bv = __ballot(i < n && ok && row_ok && !((fnull >> c) & 1));
    if (lane == 0 && wbase < n) {
      const int64_t nbytes = std::min<int64_t>(8, (n - wbase + 7) / 8);
      for (int b = 0; b < nbytes; b++) o.col_valid[c][wbase / 8 + b] = (uint8_t)(bv >> (8 * b));
    }
  }
  const uint64_t be = __ballot(err);
  if (lane == 0 && be) atomicAdd(o.n_err, (unsigned long long)__popcll(be));
}

// The deferred doubles (more than 19 significant digits, rounding decided by big integers).
__global__ __launch_bounds__(64) void k_serde_fix(const int64_t* __restrict__ fix, int64_t nfix,
                                                  const uint8_t* __restrict__ vbytes, SerdeOut o,
                                                  const SerdeParams q) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nfix) return;
  const int64_t row = fix[4 * k], c = fix[4 * k + 1], off = fix[4 * k + 2];
  const int64_t len = fix[4 * k + 3] & 0xFFFFFFFFLL;
  const bool json_num = (fix[4 * k + 3] >> 32) & 1;
  int f = 0;
  while (f < q.n_fields && q.fout[f] != c) f++;
  double d;
  const int st = np::java_parse_double(vbytes + off, len, &d, !json_num, true);
  if (st != np::PD_OK) {  // the record fails after all
    atomicAnd((unsigned int*)(o.key_valid + (row >> 5) * 4), ~(1u << (row & 31)));
    atomicAnd((unsigned int*)(o.row_valid + (row >> 5) * 4), ~(1u << (row & 31)));
    atomicAdd(o.n_err, 1ULL);
    return;
  }
  const int t = q.ftype[f];
  if (t == KHIP_TYPE_INT32) ((int32_t*)o.col[c])[row] = java_d2i(d);
  else if (t == KHIP_TYPE_INT64) ((int64_t*)o.col[c])[row] = java_d2l(d);
  else ((double*)o.col[c])[row] = d;
}

}  // namespace khip

using namespace khip;

struct khip_serde {
  khip_serde_desc desc{};
  SerdeParams q{};
  std::vector<int32_t> out_type;  // per output column: element type
  int device = 0;
  hipStream_t stream = nullptr;
  DevBuf key_i64, key_valid, row_valid, cols[SD_MAX_FIELDS], cvalid[SD_MAX_FIELDS], ctr, fix;
  DevBuf st_ts, st_koff, st_kbytes, st_kval, st_voff, st_vbytes, st_vval;
  std::vector<const void*> col_ptrs;
  std::vector<const uint8_t*> val_ptrs;
  int64_t fix_cap = 0;
};

static khip_status sstage(khip_serde* s, DevBuf& b, const void* src, size_t bytes) {
  KHIP_TRY(b.ensure(std::max<size_t>(bytes, 8)));
  if (bytes) KHIP_TRY_HIP(hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, s->stream));
  return KHIP_OK;
}

extern "C" {

khip_status khip_serde_create(const khip_serde_desc* d, khip_serde** out) {
  clear_error();
  if (!d || !out) return fail(KHIP_E_INVALID, "null argument");
  if (d->key_format != KHIP_FMT_NONE && d->key_format != KHIP_FMT_KAFKA)
    return fail(KHIP_E_UNSUPPORTED, "key format (KAFKA or none)");
  if (d->key_format == KHIP_FMT_KAFKA && d->key_type != KHIP_TYPE_INT32 && d->key_type != KHIP_TYPE_INT64 &&
      d->key_type != KHIP_TYPE_STRING)
    return fail(KHIP_E_UNSUPPORTED, "key type");
  if (d->value_format != KHIP_FMT_KAFKA && d->value_format != KHIP_FMT_DELIMITED && d->value_format != KHIP_FMT_JSON &&
      d->value_format != KHIP_FMT_AVRO)
    return fail(KHIP_E_UNSUPPORTED, "value format (KAFKA, DELIMITED, JSON, AVRO)");
  if (d->value_format == KHIP_FMT_AVRO &&
      (d->avro_n_fields < 0 || d->avro_n_fields > SD_MAX_FIELDS || (d->avro_n_fields && (!d->avro_field_names ||
                                                                                     !d->avro_field_types))))
    return fail(KHIP_E_INVALID, "AVRO writer schema: 0..32 fields with names and types");
  if (d->n_fields < 1 || d->n_fields > SD_MAX_FIELDS) return fail(KHIP_E_UNSUPPORTED, "1..32 value fields");
  if (d->value_format == KHIP_FMT_KAFKA && d->n_fields != 1)
    return fail(KHIP_E_INVALID, "the KAFKA format carries one field");
  khip_serde* s = new khip_serde();
  s->desc = *d;
  SerdeParams& q = s->q;
  q.key_format = d->key_format;
  q.key_type = d->key_type;
  q.value_format = d->value_format;
  q.n_fields = d->n_fields;
  q.delimiter = d->delimiter ? d->delimiter : ',';
  int n_out = 0;
  for (int f = 0; f < d->n_fields; f++) {
    const int t = d->field_types[f];
    if (t < KHIP_TYPE_INT32 || t > KHIP_TYPE_STRING) {
      delete s;
      return fail(KHIP_E_UNSUPPORTED, "field type");
    }
    q.ftype[f] = t;
    q.fout[f] = d->field_out ? d->field_out[f] : f;
    if (q.fout[f] >= 0) n_out = std::max(n_out, q.fout[f] + 1);
    if (d->value_format == KHIP_FMT_JSON || d->value_format == KHIP_FMT_AVRO) {
      const char* nm = d->field_names ? d->field_names[f] : nullptr;
      const size_t L = nm ? strlen(nm) : 0;
      if (!nm || L > SD_NAME_BYTES) {
        delete s;
        return fail(KHIP_E_INVALID, "JSON / AVRO field names (<= 64 bytes) required");
      }
      q.name_len[f] = (int32_t)L;
      memcpy(q.name[f], nm, L);
    }
  }
  if (d->value_format == KHIP_FMT_AVRO) {
    // writer field → ksql field: the field of the same name, else of the upper-cased name
    // (ConnectDataTranslator.toKsqlStruct: Java's toUpperCase, Unicode as above); validateSchema
    // (:123-146) runs on every mapped field of every record, so one incompatible type fails them all
    q.avro_id = d->avro_schema_id;
    q.avro_nw = d->avro_n_fields;
    q.avro_incompat = 0;
    for (int w = 0; w < d->avro_n_fields; w++) {
      const int at = d->avro_field_types[w];
      const int un = d->avro_field_union ? d->avro_field_union[w] : 0;
      const char* wn = d->avro_field_names[w];
      if (at < KHIP_AVRO_BOOLEAN || at > KHIP_AVRO_BYTES || un < 0 || un > 2 || !wn) {
        delete s;
        return fail(KHIP_E_UNSUPPORTED, "AVRO writer field: primitive type, plain or a union with null");
      }
      const std::string up = upper_utf8_host(wn);  // (Avro names are ASCII; same rule as JSON)
      int fx = -1, fu = -1;
      for (int f = 0; f < d->n_fields; f++) {
        const std::string kn(d->field_names[f]);
        if (kn == wn && fx < 0) fx = f;
        if (kn == up && fu < 0) fu = f;
      }
      const int f = fx >= 0 ? fx : fu;
      q.aw_type[w] = (int8_t)at;
      q.aw_union[w] = (int8_t)un;
      q.aw_field[w] = (int8_t)f;
      if (f < 0) continue;
      const int kt = d->field_types[f];
      const bool okt = kt == KHIP_TYPE_STRING ? at != KHIP_AVRO_BYTES
                       : kt == KHIP_TYPE_INT64 ? (at == KHIP_AVRO_INT || at == KHIP_AVRO_LONG)
                       : kt == KHIP_TYPE_INT32 ? at == KHIP_AVRO_INT
                                               : (at == KHIP_AVRO_FLOAT || at == KHIP_AVRO_DOUBLE);
      if (!okt) q.avro_incompat = 1;
    }
  }
  q.n_out = n_out;
  s->out_type.assign(n_out, KHIP_TYPE_INT64);
  for (int f = 0; f < d->n_fields; f++)
    if (q.fout[f] >= 0) s->out_type[q.fout[f]] = q.ftype[f] == KHIP_TYPE_STRING ? KHIP_TYPE_INT64 : q.ftype[f];
  s->device = d->device;
  DeviceGuard g(s->device);
  if (hipStreamCreateWithFlags(&s->stream, hipStreamDefault) != hipSuccess) {
    delete s;
    return fail(KHIP_E_DEVICE, "hipStreamCreate failed (no device?)");
  }
  *out = s;
  return KHIP_OK;
}

khip_status khip_serde_decode(khip_serde* s, const khip_raw_batch* in, khip_batch* out, int64_t* n_errors) {
  clear_error();
  if (!s || !in || !out) return fail(KHIP_E_INVALID, "null argument");
  const int64_t n = in->n_rows;
  if (n < 0 || !in->value_offsets || (n && !in->ts)) return fail(KHIP_E_INVALID, "raw batch shape");
  if (s->q.key_format != KHIP_FMT_NONE && !in->key_offsets) return fail(KHIP_E_INVALID, "missing key offsets");
  DeviceGuard g(s->device);
  const SerdeParams& q = s->q;
  const int64_t* ts = in->ts;
  const int64_t *koff = in->key_offsets, *voff = in->value_offsets;
  const uint8_t *kb = in->key_bytes, *kv = in->key_valid, *vb = in->value_bytes, *vv = in->value_valid;
  const size_t bm = (size_t)(n + 7) / 8;
  if (in->mem == KHIP_MEM_HOST) {
    KHIP_TRY(sstage(s, s->st_ts, ts, n * 8));
    ts = s->st_ts.as<int64_t>();
    KHIP_TRY(sstage(s, s->st_voff, voff, (n + 1) * 8));
    const int64_t vbytes = voff[n];
    KHIP_TRY(sstage(s, s->st_vbytes, vb, (size_t)vbytes));
    voff = s->st_voff.as<int64_t>();
    vb = s->st_vbytes.as<uint8_t>();
    if (vv) { KHIP_TRY(sstage(s, s->st_vval, vv, bm)); vv = s->st_vval.as<uint8_t>(); }
    if (koff) {
      const int64_t kbytes = koff[n];
      KHIP_TRY(sstage(s, s->st_koff, koff, (n + 1) * 8));
      KHIP_TRY(sstage(s, s->st_kbytes, kb, (size_t)kbytes));
      koff = s->st_koff.as<int64_t>();
      kb = s->st_kbytes.as<uint8_t>();
    }
    if (kv) { KHIP_TRY(sstage(s, s->st_kval, kv, bm)); kv = s->st_kval.as<uint8_t>(); }
  } else if (in->mem != KHIP_MEM_DEVICE) {
    return fail(KHIP_E_INVALID, "batch mem");
  }
  const size_t bm4 = ((size_t)(n + 31) / 32) * 4 + 8;  // word-aligned: k_serde_fix clears bits atomically
  SerdeOut o{};
  if (q.key_format == KHIP_FMT_NONE || q.key_type != KHIP_TYPE_STRING) {
    KHIP_TRY(s->key_i64.ensure(std::max<int64_t>(n, 1) * 8));
    o.key_i64 = s->key_i64.as<int64_t>();
  }
  KHIP_TRY(s->key_valid.ensure(bm4));
  KHIP_TRY(s->row_valid.ensure(bm4));
  o.key_valid = s->key_valid.as<uint8_t>();
  o.row_valid = s->row_valid.as<uint8_t>();
  for (int c = 0; c < q.n_out; c++) {
    KHIP_TRY(s->cols[c].ensure(std::max<int64_t>(n, 1) * (s->out_type[c] == KHIP_TYPE_INT32 ? 4 : 8)));
    KHIP_TRY(s->cvalid[c].ensure(bm4));
    o.col[c] = s->cols[c].p;
    o.col_valid[c] = s->cvalid[c].as<uint8_t>();
  }
  KHIP_TRY(s->ctr.ensure(16));
  KHIP_TRY_HIP(hipMemsetAsync(s->ctr.p, 0, 16, s->stream));
  o.n_err = s->ctr.as<unsigned long long>();
  o.n_fix = o.n_err + 1;
  if (s->fix_cap == 0) {
    s->fix_cap = 1024;
    KHIP_TRY(s->fix.ensure((size_t)s->fix_cap * 32));
  }
  o.fix = s->fix.as<int64_t>();
  o.fix_cap = s->fix_cap;
  unsigned long long c2[2] = {0, 0};
  if (n > 0) {
    for (int attempt = 0; attempt < 2; attempt++) {
      if (q.n_fields <= 4)
        hipLaunchKernelGGL(k_serde_decode<4>, dim3(ceil_div(n, 256)), dim3(256), 0, s->stream, q, n, koff, kb, kv, voff, vb,
                           vv, o);
      else
        hipLaunchKernelGGL(k_serde_decode<SD_MAX_FIELDS>, dim3(ceil_div(n, 256)), dim3(256), 0, s->stream, q, n, koff, kb,
                           kv, voff, vb, vv, o);
      KHIP_TRY_HIP(hipGetLastError());
      KHIP_TRY_HIP(hipMemcpyAsync(c2, s->ctr.p, 16, hipMemcpyDeviceToHost, s->stream));
      KHIP_TRY_HIP(hipStreamSynchronize(s->stream));
      if ((int64_t)c2[1] <= s->fix_cap) break;
      s->fix_cap = (int64_t)next_pow2(c2[1]);  // room for every deferred double, decode again
      s->fix.release();
      KHIP_TRY(s->fix.ensure((size_t)s->fix_cap * 32));
      o.fix = s->fix.as<int64_t>();
      o.fix_cap = s->fix_cap;
      KHIP_TRY_HIP(hipMemsetAsync(s->ctr.p, 0, 16, s->stream));
    }
    if (c2[1]) {
      hipLaunchKernelGGL(k_serde_fix, dim3(ceil_div((int64_t)c2[1], 64)), dim3(64), 0, s->stream, o.fix,
                         (int64_t)c2[1], vb, o, q);
      KHIP_TRY_HIP(hipGetLastError());
      KHIP_TRY_HIP(hipMemcpyAsync(c2, s->ctr.p, 8, hipMemcpyDeviceToHost, s->stream));
      KHIP_TRY_HIP(hipStreamSynchronize(s->stream));
    }
  }
  if (n_errors) *n_errors = (int64_t)c2[0];
  s->col_ptrs.assign(q.n_out, nullptr);
  s->val_ptrs.assign(q.n_out, nullptr);
  for (int c = 0; c < q.n_out; c++) {
    s->col_ptrs[c] = s->cols[c].p;
    s->val_ptrs[c] = s->cvalid[c].as<uint8_t>();
  }
  memset(out, 0, sizeof(*out));
  out->n_rows = n;
  out->mem = KHIP_MEM_DEVICE;
  out->n_cols = q.n_out;
  out->ts = ts;
  out->key_valid = s->key_valid.as<uint8_t>();
  out->row_valid = s->row_valid.as<uint8_t>();
  if (q.key_format == KHIP_FMT_KAFKA && q.key_type == KHIP_TYPE_STRING) {
    out->key_offsets = koff;
    out->key_bytes = kb;
  } else {
    out->key_i64 = s->key_i64.as<int64_t>();
  }
  out->col_data = s->col_ptrs.data();
  out->col_valid = s->val_ptrs.data();
  return KHIP_OK;
}

khip_status khip_serde_destroy(khip_serde* s) {
  if (!s) return KHIP_OK;
  DeviceGuard g(s->device);
  if (s->stream) hipStreamSynchronize(s->stream);
  DevBuf* bufs[] = {&s->key_i64, &s->key_valid, &s->row_valid, &s->ctr, &s->fix, &s->st_ts, &s->st_koff,
                    &s->st_kbytes, &s->st_kval, &s->st_voff, &s->st_vbytes, &s->st_vval};
  for (DevBuf* b : bufs) b->release();
  for (int c = 0; c < SD_MAX_FIELDS; c++) {
    s->cols[c].release();
    s->cvalid[c].release();
  }
  if (s->stream) hipStreamDestroy(s->stream);
  delete s;
  return KHIP_OK;
}

}  // extern "C"
