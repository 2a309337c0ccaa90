// khip_sink.hip — serialization of columnar rows into Kafka record bytes (gfx950).
//
// The output side of GenericKeySerDe / GenericRowSerDe (include/ksqldb_hip.h "serialization"):
// an aggregate's changelog rows become sink records — the inner key in the key format, Kafka
// Streams' windowed key suffix, the value in the value format or a null value for a tombstone —
// and several GROUP BY columns become the serialized composite key the aggregate groups by.
//
// Two passes over tiles of 256 rows, one thread per row: k_sink_measure runs the very
// encoder the write pass runs, with a counting writer, so a row's length and its bytes can never
// disagree, and sums each tile's lengths; one block scans the tile sums; k_sink_write scans its
// tile's lengths in the block, adds the tile's carry and writes each record at its offset, and
// the offsets.  A KAFKA INT32 / BIGINT key has a fixed width (no key lengths; a BIGINT key and its
// window suffix leave as 8-byte words), and a JSON column's '{' / ',' + escaped name + ':' is built
// once on the host.  Doubles print
// through the Schubfach shortest-decimal algorithm (R. Giulietti 2020; java.lang.Double.toString
// since JDK 19) with the 126-bit powers of ten of tools/gen_dtoa.py, so every digit is computed
// exactly with 64-bit integer arithmetic.  Byte parity of DOUBLE text therefore assumes the
// reference runs on JDK 19 or later: JDK <= 18's FloatingDecimal prints longer digit strings for
// some values (tests/sink_ref.py lists them); on such a JVM the values still parse to the same
// double, but the bytes differ (DESIGN.md §(c), unpinned).
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "khip_util.hpp"

namespace khip {

constexpr int SK_MAX = KHIP_SINK_MAX_COLS;
constexpr int SK_NAME = 64;
constexpr int SK_PRE = 72;  // a JSON column's text before its value, escaped name included
// The write pass's outputs leave as nontemporal stores: k_sink_write 717 / 719 us per 22M rows
// against 750 / 751 (profiles/r05/ab/sink_two_pass.txt).
#ifndef KHIP_SINK_NT
#define KHIP_SINK_NT 1
#endif
template <class T>
__device__ __forceinline__ void sk_st(T* p, T v) {
  if (KHIP_SINK_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

constexpr int SK_SCAN_T = 1024;
constexpr int SK_SCAN_I = 8;  // items per thread per scan block

__device__ const uint64_t kDtoaG[617][2] = {
#include "khip_dtoa.inc"
};

struct SinkParams {
  int32_t key_format, n_key, window_kind, value_format, n_val, delim;
  int32_t ktype[SK_MAX], vtype[SK_MAX], vsrc[SK_MAX];
  int32_t kname_len[SK_MAX], vname_len[SK_MAX];
  uint8_t kname[SK_MAX][SK_NAME], vname[SK_MAX][SK_NAME];
  // JSON object columns: '{' (first) or ',', the escaped quoted name and ':' — built once on the
  // host by the device's own escaper (put_json_str); length -1 when longer than SK_PRE
  int32_t kpre_len[SK_MAX], vpre_len[SK_MAX];
  alignas(8) uint8_t kpre[SK_MAX][SK_PRE];
  alignas(8) uint8_t vpre[SK_MAX][SK_PRE];
};

// ------------------------------------------------------------------ writers

struct CountW {
  int64_t n = 0;
  __device__ __forceinline__ void put(uint8_t) { n++; }
};
struct MemW {
  uint8_t* p;
  __device__ __forceinline__ void put(uint8_t c) { *p++ = c; }
};
struct HostW {  // host: a JSON column prefix (SinkParams::kpre / vpre)
  uint8_t* p;
  int n, cap;
  void put(uint8_t c) {
    if (n < cap) p[n] = c;
    n++;
  }
};
struct BufW {  // a field's text, for the CSV quoting decision
  uint8_t b[40];
  int n = 0;
  __device__ __forceinline__ void put(uint8_t c) { b[n++] = c; }
};

// ------------------------------------------------------------------ numbers

// Long.toString.  The digits collect in a 24-byte shift register (d2:d1:d0, each new digit in at
// the bottom, so the most significant ends in byte 0): registers, where a digit array indexed by a
// variable would live in scratch memory.
template <class W>
__device__ __forceinline__ void put_i64(W& w, int64_t v) {
  uint64_t u = v < 0 ? 0ULL - (uint64_t)v : (uint64_t)v;
  uint64_t d0 = 0, d1 = 0, d2 = 0;
  int n = 0;
  auto push = [&](uint64_t dig) {
    d2 = (d2 << 8) | (d1 >> 56);
    d1 = (d1 << 8) | (d0 >> 56);
    d0 = (d0 << 8) | ('0' + dig);
    n++;
  };
  while (u >> 32) {
    push(u % 10);
    u /= 10;
  }
  uint32_t x = (uint32_t)u;
  do {
    push(x % 10);
    x /= 10;
  } while (x);
  if (v < 0) w.put('-');
  for (; n; n--) {
    w.put((uint8_t)d0);
    d0 = (d0 >> 8) | (d1 << 56);
    d1 = (d1 >> 8) | (d2 << 56);
    d2 >>= 8;
  }
}

__device__ __forceinline__ int flog10pow2(int q) { return (int)(((int64_t)q * 661971961083LL) >> 41); }
__device__ __forceinline__ int flog10tqpow2(int q) { return (int)(((int64_t)q * 661971961083LL - 274743187321LL) >> 41); }
__device__ __forceinline__ int flog2pow10(int e) { return (int)(((int64_t)e * 913124641741LL) >> 38); }

constexpr uint64_t MASK63 = 0x7FFFFFFFFFFFFFFFULL;

// round to odd of the product g * cp (Schubfach's rop)
__device__ __forceinline__ uint64_t sk_rop(uint64_t g1, uint64_t g0, uint64_t cp) {
  const uint64_t x1 = __umul64hi(g0, cp);
  const uint64_t y0 = g1 * cp;
  const uint64_t y1 = __umul64hi(g1, cp);
  const uint64_t z = (y0 >> 1) + x1;
  const uint64_t vbp = y1 + (z >> 63);
  return vbp | (((z & MASK63) + MASK63) >> 63);
}

// c 2^q → the shortest decimal f 10^e in its rounding interval (closest; even on ties)
__device__ void sk_to_decimal(int q, uint64_t c, int dk, uint64_t* fo, int* eo) {
  const uint64_t out = c & 1;
  const uint64_t cb = c << 2, cbr = cb + 2;
  uint64_t cbl;
  int k;
  if (c != (1ULL << 52) || q == -1074) {
    cbl = cb - 2;
    k = flog10pow2(q);
  } else {
    cbl = cb - 1;
    k = flog10tqpow2(q);
  }
  const int h = q + flog2pow10(-k) + 2;
  const uint64_t g1 = kDtoaG[k + 324][0], g0 = kDtoaG[k + 324][1];
  const uint64_t vb = sk_rop(g1, g0, cb << h);
  const uint64_t vbl = sk_rop(g1, g0, cbl << h);
  const uint64_t vbr = sk_rop(g1, g0, cbr << h);
  const uint64_t s = vb >> 2;
  if (s >= 100) {
    const uint64_t sp10 = 10 * __umul64hi(s, 115292150460684698ULL << 4);
    const uint64_t tp10 = sp10 + 10;
    const bool upin = vbl + out <= sp10 << 2;
    const bool wpin = (tp10 << 2) + out <= vbr;
    if (upin != wpin) {
      *fo = upin ? sp10 : tp10;
      *eo = k;
      return;
    }
  }
  const uint64_t t = s + 1;
  const bool uin = vbl + out <= s << 2;
  const bool win = (t << 2) + out <= vbr;
  if (uin != win) {
    *fo = uin ? s : t;
    *eo = k + dk;
    return;
  }
  const int64_t cmp = (int64_t)(vb - ((s + t) << 1));
  *fo = cmp < 0 || (cmp == 0 && (s & 1) == 0) ? s : t;
  *eo = k + dk;
}

// Double.toString of a finite double
template <class W>
__device__ void put_f64(W& w, double v) {
  const uint64_t bits = (uint64_t)__double_as_longlong(v);
  const uint64_t t = bits & ((1ULL << 52) - 1);
  const int bq = (int)((bits >> 52) & 0x7FF);
  if (bits >> 63) w.put('-');
  uint64_t f;
  int e;
  if (bq != 0) {
    const int mq = 1075 - bq;
    const uint64_t c = (1ULL << 52) | t;
    if (mq > 0 && mq < 53 && ((c >> mq) << mq) == c) {
      f = c >> mq;
      e = 0;
    } else {
      sk_to_decimal(-mq, c, 0, &f, &e);
    }
  } else if (t != 0) {
    if (t < 3) sk_to_decimal(-1074, 10 * t, -1, &f, &e);
    else sk_to_decimal(-1074, t, 0, &f, &e);
  } else {
    w.put('0');
    w.put('.');
    w.put('0');
    return;
  }
  // digits of f, then Java's layout (DoubleToDecimal.toChars): plain for 1e-3 <= |v| < 1e7,
  // computerized scientific notation otherwise; at least one digit after the point
  uint8_t d[20];
  int L = 0;
  {
    uint8_t r[20];
    uint64_t u = f;
    do {
      r[L++] = (uint8_t)('0' + u % 10);
      u /= 10;
    } while (u);
    for (int i = 0; i < L; i++) d[i] = r[L - 1 - i];
  }
  const int e10 = e + L;  // |v| = 0.d 10^e10
  int nd = L;
  while (nd > 1 && d[nd - 1] == '0') nd--;
  if (e10 > 0 && e10 <= 7) {
    for (int i = 0; i < e10; i++) w.put(i < nd ? d[i] : (uint8_t)'0');
    w.put('.');
    if (nd > e10) {
      for (int i = e10; i < nd; i++) w.put(d[i]);
    } else {
      w.put('0');
    }
  } else if (e10 > -3 && e10 <= 0) {
    w.put('0');
    w.put('.');
    for (int i = 0; i < -e10; i++) w.put('0');
    for (int i = 0; i < nd; i++) w.put(d[i]);
  } else {
    w.put(d[0]);
    w.put('.');
    if (nd > 1) {
      for (int i = 1; i < nd; i++) w.put(d[i]);
    } else {
      w.put('0');
    }
    w.put('E');
    put_i64(w, (int64_t)(e10 - 1));
  }
}

// Double.toString of any double (NaN, Infinity, -Infinity)
template <class W>
__device__ void put_f64_any(W& w, double v) {
  if (v != v) {
    w.put('N'); w.put('a'); w.put('N');
  } else if (v == __builtin_inf() || v == -__builtin_inf()) {
    if (v < 0) w.put('-');
    const char* s = "Infinity";
    for (int i = 0; i < 8; i++) w.put((uint8_t)s[i]);
  } else {
    put_f64(w, v);
  }
}

// ------------------------------------------------------------------ values

struct Val {
  int64_t i;  // INT32 / INT64 (sign-extended); DOUBLE: the bits
  const uint8_t* s;
  int64_t len;  // STRING
  bool null;
};

// f(byte) over s[0..len), the bytes loaded eight at a time: on gfx950 a load issued behind a store
// waits for the store (one vmcnt counts both), so a byte-by-byte copy would wait a memory round
// trip per byte.
template <class F>
__host__ __device__ __forceinline__ void for_bytes(const uint8_t* s, int64_t len, F&& f) {
  for (int64_t j = 0; j < len; j += 8) {
    uint64_t x = 0;
#pragma unroll
    for (int b = 0; b < 8; b++)
      if (j + b < len) x |= (uint64_t)s[j + b] << (8 * b);
    const int m = len - j < 8 ? (int)(len - j) : 8;
    for (int b = 0; b < m; b++) f((uint8_t)(x >> (8 * b)));
  }
}

template <class W>
__device__ void put_be(W& w, uint64_t v, int nbytes) {
  for (int b = nbytes - 1; b >= 0; b--) w.put((uint8_t)(v >> (8 * b)));
}

// Jackson's string escaping: quote, backslash, the short escapes, \u00XX for other control bytes
template <class W>
__host__ __device__ void put_json_str(W& w, const uint8_t* s, int64_t len) {
  w.put('"');
  for_bytes(s, len, [&](uint8_t c) {
    if (c == '"' || c == '\\') {
      w.put('\\');
      w.put(c);
    } else if (c < 0x20) {
      w.put('\\');
      switch (c) {
        case 0x08: w.put('b'); break;
        case 0x09: w.put('t'); break;
        case 0x0A: w.put('n'); break;
        case 0x0C: w.put('f'); break;
        case 0x0D: w.put('r'); break;
        default: {
          const char* hx = "0123456789ABCDEF";
          w.put('u'); w.put('0'); w.put('0');
          w.put((uint8_t)hx[c >> 4]);
          w.put((uint8_t)hx[c & 15]);
        }
      }
    } else {
      w.put(c);
    }
  });
  w.put('"');
}

template <class W>
__device__ void put_json_val(W& w, int type, const Val& v) {
  if (v.null) {
    w.put('n'); w.put('u'); w.put('l'); w.put('l');
    return;
  }
  if (type == KHIP_TYPE_DOUBLE) {
    const double d = __longlong_as_double(v.i);
    if (d != d || d == __builtin_inf() || d == -__builtin_inf()) {  // QUOTE_NON_NUMERIC_NUMBERS
      w.put('"');
      put_f64_any(w, d);
      w.put('"');
    } else {
      put_f64(w, d);
    }
  } else if (type == KHIP_TYPE_STRING) {
    put_json_str(w, v.s, v.len);
  } else {
    put_i64(w, v.i);
  }
}

// commons-csv 1.4 CSVFormat.printAndQuote, QuoteMode.MINIMAL (KsqlDelimitedSerializer's CSVPrinter)
template <class W>
__device__ void put_csv_text(W& w, const uint8_t* s, int64_t len, bool first, uint8_t delim) {
  bool quote = false;
  if (len <= 0) {
    quote = first;
  } else {
    const uint8_t c = s[0];
    if (first && (c < 0x20 || (c > 0x21 && c < 0x23) || (c > 0x2B && c < 0x2D) || c > 0x7E)) {
      quote = true;
    } else if (c <= '#') {
      quote = true;
    } else {
      for (int64_t i = 0; i < len && !quote; i++) {
        const uint8_t x = s[i];
        quote = x == '\n' || x == '\r' || x == '"' || x == delim;
      }
      if (!quote) quote = s[len - 1] <= ' ';
    }
  }
  if (quote) w.put('"');
  for_bytes(s, len, [&](uint8_t c) {
    if (quote && c == '"') w.put('"');
    w.put(c);
  });
  if (quote) w.put('"');
}

template <class W>
__device__ void put_csv_val(W& w, int type, const Val& v, bool first, uint8_t delim) {
  if (v.null) return;  // CSVPrinter.print(null) with no null string: nothing, unquoted
  if (type == KHIP_TYPE_STRING) {
    put_csv_text(w, v.s, v.len, first, delim);
    return;
  }
  BufW b;
  if (type == KHIP_TYPE_DOUBLE) put_f64_any(b, __longlong_as_double(v.i));
  else put_i64(b, v.i);
  put_csv_text(w, b.b, b.n, first, delim);
}

// KAFKA format primitive bytes (kafka/KafkaSerdeFactory.java:42-46)
template <class W>
__device__ void put_kafka_val(W& w, int type, const Val& v) {
  if (type == KHIP_TYPE_INT32) put_be(w, (uint64_t)(uint32_t)v.i, 4);
  else if (type == KHIP_TYPE_STRING)
    for_bytes(v.s, v.len, [&](uint8_t c) { w.put(c); });
  else put_be(w, (uint64_t)v.i, 8);
}

// the inner key (never null: a null GROUP BY value drops the row upstream)
// A column prefix: 8-byte words from the parameters, put byte by byte from registers.
template <class W>
__device__ __forceinline__ void put_pre(W& w, const uint8_t* pre, int len) {
  for (int j = 0; j < len; j += 8) {
    const uint64_t x = *(const uint64_t*)(pre + j);
#pragma unroll
    for (int b = 0; b < 8; b++)
      if (j + b < len) w.put((uint8_t)(x >> (8 * b)));
  }
}

template <class W, class F>
__device__ void put_key(W& w, const SinkParams& q, F&& kval) {
  if (q.key_format == KHIP_FMT_KAFKA) {
    put_kafka_val(w, q.ktype[0], kval(0));
  } else if (q.key_format == KHIP_FMT_JSON) {
    if (q.n_key == 1) {
      put_json_val(w, q.ktype[0], kval(0));
    } else {
      for (int i = 0; i < q.n_key; i++) {
        if (q.kpre_len[i] >= 0) {
          put_pre(w, q.kpre[i], q.kpre_len[i]);
        } else {
          w.put(i ? ',' : '{');
          put_json_str(w, q.kname[i], q.kname_len[i]);
          w.put(':');
        }
        put_json_val(w, q.ktype[i], kval(i));
      }
      w.put('}');
    }
  } else {
    for (int i = 0; i < q.n_key; i++) {
      if (i) w.put((uint8_t)q.delim);
      put_csv_val(w, q.ktype[i], kval(i), i == 0, (uint8_t)q.delim);
    }
  }
}

template <class W, class F>
__device__ __forceinline__ void put_value(W& w, const SinkParams& q, F&& vval) {
  if (q.value_format == KHIP_FMT_KAFKA) {
    put_kafka_val(w, q.vtype[0], vval(0));
  } else if (q.value_format == KHIP_FMT_JSON) {
    if (q.n_val == 0) w.put('{');
    for (int i = 0; i < q.n_val; i++) {
      if (q.vpre_len[i] >= 0) {
        put_pre(w, q.vpre[i], q.vpre_len[i]);
      } else {
        w.put(i ? ',' : '{');
        put_json_str(w, q.vname[i], q.vname_len[i]);
        w.put(':');
      }
      put_json_val(w, q.vtype[i], vval(i));
    }
    w.put('}');
  } else {
    for (int i = 0; i < q.n_val; i++) {
      if (i) w.put((uint8_t)q.delim);
      put_csv_val(w, q.vtype[i], vval(i), i == 0, (uint8_t)q.delim);
    }
  }
}

// ------------------------------------------------------------------ rows → records

struct RowsDev {
  int32_t key_serialized;
  const int64_t* key_i64;
  const int64_t* key_off;
  const uint8_t* key_bytes;
  const int64_t* ws;
  const int64_t* we;
  const uint8_t* tomb;
  const void* col[SK_MAX];
  const uint8_t* cnull[SK_MAX];
};

__device__ __forceinline__ Val row_key_val(const SinkParams& q, const RowsDev& r, int64_t i) {
  Val v{0, nullptr, 0, false};
  if (q.ktype[0] == KHIP_TYPE_STRING) {
    v.s = r.key_bytes + r.key_off[i];
    v.len = r.key_off[i + 1] - r.key_off[i];
  } else {
    v.i = q.ktype[0] == KHIP_TYPE_INT32 ? (int64_t)(int32_t)r.key_i64[i] : r.key_i64[i];
  }
  return v;
}

__device__ __forceinline__ Val row_value_val(const SinkParams& q, const RowsDev& r, int64_t i, int c) {
  Val v{0, nullptr, 0, false};
  const int src = q.vsrc[c];
  if (src == KHIP_SINK_SRC_WS) {
    v.i = r.ws[i];
  } else if (src == KHIP_SINK_SRC_WE) {
    v.i = r.we[i];
  } else {
    v.null = r.cnull[src] && r.cnull[src][i];
    if (q.vtype[c] == KHIP_TYPE_INT32) v.i = ((const int32_t*)r.col[src])[i];
    else v.i = ((const int64_t*)r.col[src])[i];  // INT64, DOUBLE bits
  }
  return v;
}

// The row's window bounds, loaded before any of its bytes are stored.
struct RowWin {
  int64_t ws, we;
};
__device__ __forceinline__ RowWin row_win(const SinkParams& q, const RowsDev& r, int64_t i) {
  RowWin x{0, 0};
  if (q.window_kind != KHIP_WINDOW_NONE) x.ws = r.ws[i];
  if (q.window_kind == KHIP_WINDOW_SESSION) x.we = r.we[i];
  return x;
}

template <class W>
__device__ __forceinline__ void encode_key_row(W& w, const SinkParams& q, const RowsDev& r, int64_t i) {
  const RowWin win = row_win(q, r, i);
  if (r.key_serialized) {
    const int64_t b0 = r.key_off[i], b1 = r.key_off[i + 1];
    for_bytes(r.key_bytes + b0, b1 - b0, [&](uint8_t c) { w.put(c); });
  } else {
    const Val kv = row_key_val(q, r, i);
    put_key(w, q, [&](int) { return kv; });
  }
  if (q.window_kind == KHIP_WINDOW_TUMBLING || q.window_kind == KHIP_WINDOW_HOPPING) {
    put_be(w, (uint64_t)win.ws, 8);
  } else if (q.window_kind == KHIP_WINDOW_SESSION) {
    put_be(w, (uint64_t)win.we, 8);
    put_be(w, (uint64_t)win.ws, 8);
  }
}

// a value that is a null record: a tombstone, or a KAFKA-format value whose one column is NULL
__device__ __forceinline__ bool value_is_null(const SinkParams& q, const RowsDev& r, int64_t i) {
  if (r.tomb && r.tomb[i]) return true;
  return q.value_format == KHIP_FMT_KAFKA && row_value_val(q, r, i, 0).null;
}

// Tiles of SK_TILE = 256 rows, one block of 256 threads, one row per thread (eight rows per
// thread in rounds, measured earlier, kept the write pass's row state live across rounds: 171
// VGPRs).
constexpr int SK_TR = 1;
// k_sink_write at 4 waves per SIMD (<= 128 VGPRs; the spills are in the DOUBLE printer): 782-802
// us per 22M rows against 840 at 5 and 890 uncapped (138 VGPRs), profiles/r05/ab/sink_two_pass.txt
#ifndef KHIP_SINK_MINB
#define KHIP_SINK_MINB 4
#endif
#define KHIP_SINK_WRITE_LB __launch_bounds__(256, KHIP_SINK_MINB)
constexpr int SK_TILE = 256 * SK_TR;

// Sums of (a, b) over the block; every thread gets them.
__device__ __forceinline__ void sk_block_sum2(int64_t& a, int64_t& b, int64_t (*ws)[4]) {
  for (int off = 32; off; off >>= 1) {
    a += __shfl_xor(a, off, 64);
    b += __shfl_xor(b, off, 64);
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    ws[0][wave] = a;
    ws[1][wave] = b;
  }
  __syncthreads();
  a = ws[0][0] + ws[0][1] + ws[0][2] + ws[0][3];
  b = ws[1][0] + ws[1][1] + ws[1][2] + ws[1][3];
  __syncthreads();
}

// Exclusive scans of (a, b) over the block; the block totals in ta, tb.
__device__ __forceinline__ void sk_block_scan2(int64_t& a, int64_t& b, int64_t& ta, int64_t& tb, int64_t (*ws)[4]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t ia = a, ib = b;
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t ya = __shfl_up(ia, off, 64), yb = __shfl_up(ib, off, 64);
    if (lane >= off) {
      ia += ya;
      ib += yb;
    }
  }
  if (lane == 63) {
    ws[0][wave] = ia;
    ws[1][wave] = ib;
  }
  __syncthreads();
  int64_t pa = 0, pb = 0;
  ta = tb = 0;
  for (int w = 0; w < 4; w++) {
    pa += w < wave ? ws[0][w] : 0;
    pb += w < wave ? ws[1][w] : 0;
    ta += ws[0][w];
    tb += ws[1][w];
  }
  __syncthreads();
  a = pa + ia - a;
  b = pb + ib - b;
}

// Pass 1: each row's key / value length at klen / vlen[i + 1] (keys skipped when every key is kfix
// bytes), each tile's sums at tsum[1 + tile] (keys) and tsum[nT + 2 + tile] (values).
__global__ __launch_bounds__(256) void k_sink_measure(const SinkParams* __restrict__ qp, RowsDev r, int64_t n, int kfix,
                                                      int64_t nT, int64_t* __restrict__ klen, int64_t* __restrict__ vlen,
                                                      int64_t* __restrict__ tsum) {
  __shared__ int64_t ws[2][4];
  const SinkParams& q = *qp;
  const int64_t base = (int64_t)blockIdx.x * SK_TILE;
  int64_t sk = 0, sv = 0;
#pragma unroll 1
  for (int u = 0; u < SK_TR; u++) {
    const int64_t i = base + u * 256 + threadIdx.x;
    if (i >= n) break;
    if (!kfix) {
      CountW kw;
      encode_key_row(kw, q, r, i);
      klen[i + 1] = kw.n;
      sk += kw.n;
    }
    CountW vw;
    if (!value_is_null(q, r, i)) put_value(vw, q, [&](int c) { return row_value_val(q, r, i, c); });
    vlen[i + 1] = vw.n;
    sv += vw.n;
  }
  sk_block_sum2(sk, sv, ws);
  if (threadIdx.x == 0) {
    tsum[1 + blockIdx.x] = sk;
    tsum[nT + 2 + blockIdx.x] = sv;
  }
}

// A fixed-width KAFKA BIGINT key and its window suffix as big-endian 8-byte words (kb + 8-aligned),
// every load before the first store.
__device__ __forceinline__ void put_key_words(const SinkParams& q, const RowsDev& r, int64_t i, uint64_t* o) {
  const RowWin win = row_win(q, r, i);
  const uint64_t k = __builtin_bswap64((uint64_t)r.key_i64[i]);
  if (q.window_kind == KHIP_WINDOW_TUMBLING || q.window_kind == KHIP_WINDOW_HOPPING) {
    if (((uintptr_t)o & 15) == 0) {
      if (KHIP_SINK_NT) {
        __builtin_nontemporal_store(k, o);
        __builtin_nontemporal_store(__builtin_bswap64((uint64_t)win.ws), o + 1);
      } else {
        *(ulonglong2*)o = make_ulonglong2(k, __builtin_bswap64((uint64_t)win.ws));
      }
    } else {
      o[0] = k;
      o[1] = __builtin_bswap64((uint64_t)win.ws);
    }
  } else if (q.window_kind == KHIP_WINDOW_SESSION) {
    o[0] = k;
    o[1] = __builtin_bswap64((uint64_t)win.we);
    o[2] = __builtin_bswap64((uint64_t)win.ws);
  } else {
    o[0] = k;
  }
}

// A wave's value bytes, staged contiguously in LDS (lds[0..L)), to dst[0..L): 16-byte aligned
// chunks, one per lane and round — whole 16-byte stores inside, bytes at the two edge chunks
// (shared with the neighbouring waves).  lds has 16 readable bytes past L.
__device__ __forceinline__ void sk_wave_copy(const uint8_t* lds, int L, uint8_t* __restrict__ dst) {
  const int lane = threadIdx.x & 63;
  const int A = (int)((uintptr_t)dst & 15);
  const int nch = (A + L + 15) >> 4;
  const uint32_t* l32 = (const uint32_t*)lds;
  for (int c = lane; c < nch; c += 64) {
    const int o = 16 * c - A;
    uint8_t* g = dst + o;
    if (o >= 0 && o + 16 <= L) {
      const int ao = o >> 2, sh = o & 3;
      const uint32_t w0 = l32[ao], w1 = l32[ao + 1], w2 = l32[ao + 2], w3 = l32[ao + 3], w4 = l32[ao + 4];
      uint4 v;
      v.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
      v.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
      v.z = __builtin_amdgcn_alignbyte(w3, w2, sh);
      v.w = __builtin_amdgcn_alignbyte(w4, w3, sh);
      if (KHIP_SINK_NT) {
        __builtin_nontemporal_store(v.x, (uint32_t*)g);
        __builtin_nontemporal_store(v.y, (uint32_t*)g + 1);
        __builtin_nontemporal_store(v.z, (uint32_t*)g + 2);
        __builtin_nontemporal_store(v.w, (uint32_t*)g + 3);
      } else {
        *(uint4*)g = v;
      }
    } else {
      for (int b = 0; b < 16; b++)
        if (o + b >= 0 && o + b < L) g[b] = lds[o + b];
    }
  }
}

constexpr int SK_WBUF = 2048;  // staged value bytes per wave: 64 rows of 32


// Pass 2 (after sk_scan made tsum the tiles' offsets): the tile scans its rows' lengths in the
// block and adds its carry.  A wave whose 64 values take at most SK_WBUF bytes (one contiguous
// range of the output) encodes them into LDS at their places in that range and copies the range
// out in 16-byte stores (sk_wave_copy); a longer wave writes each value at its offset byte by byte.
// Every load of a row comes before its first global store (on gfx950 a load behind a store waits
// for the store).  Each row's end offsets go over its own length slots (koff / voff[i + 1]: only
// this thread reads them, so no other tile's lengths are overwritten before they are read).
// kwords: the key as kfix / 8 words.
__global__ KHIP_SINK_WRITE_LB void k_sink_write(const SinkParams* __restrict__ qp, RowsDev r, int64_t n, int kfix,
                                                    int kwords, int64_t nT, const int64_t* __restrict__ tsum,
                                                    int64_t* __restrict__ koff, uint8_t* __restrict__ kb,
                                                    int64_t* __restrict__ voff, uint8_t* __restrict__ vb,
                                                    uint8_t* __restrict__ vnull) {
  __shared__ int64_t ws[2][4];
  __shared__ uint32_t vst[4][SK_WBUF / 4 + 4];
  const SinkParams& q = *qp;
  const int wave = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * SK_TILE + threadIdx.x;
  const bool in = i < n;
  const int64_t kl = !in ? 0 : kfix ? kfix : koff[i + 1];
  const int64_t vl = in ? voff[i + 1] : 0;
  int64_t ko = kl, vo = vl, tk, tv;
  sk_block_scan2(ko, vo, tk, tv, ws);
  ko += kfix ? (int64_t)blockIdx.x * SK_TILE * kfix : tsum[blockIdx.x];
  vo += tsum[nT + 1 + blockIdx.x];
  const int64_t wbase = __shfl(vo, 0, 64), wlen = __shfl(vo + vl, 63, 64) - wbase;  // past-n lanes: vl 0
  const bool staged = wlen <= SK_WBUF;
  uint8_t* vls = (uint8_t*)vst[wave];
  bool isnull = true;
  Val v0{0, nullptr, 0, true}, v1 = v0, v2 = v0, v3 = v0;  // the first four value columns
  if (in) {
    isnull = value_is_null(q, r, i);
    if (!isnull) {
      if (q.n_val > 0) v0 = row_value_val(q, r, i, 0);
      if (q.n_val > 1) v1 = row_value_val(q, r, i, 1);
      if (q.n_val > 2) v2 = row_value_val(q, r, i, 2);
      if (q.n_val > 3) v3 = row_value_val(q, r, i, 3);
    }
  }
  auto vget = [&](int c) {
    return c == 0 ? v0 : c == 1 ? v1 : c == 2 ? v2 : c == 3 ? v3 : row_value_val(q, r, i, c);
  };
  if (in && staged && !isnull) {
    MemW vw{vls + (vo - wbase)};
    put_value(vw, q, vget);
  }
  __syncthreads();
  if (staged && wlen > 0) sk_wave_copy(vls, (int)wlen, vb + wbase);
  if (in) {
    if (kwords) {
      put_key_words(q, r, i, (uint64_t*)(kb + ko));
    } else {
      MemW kw{kb + ko};
      encode_key_row(kw, q, r, i);
    }
    sk_st(vnull + i, (uint8_t)(isnull ? 1 : 0));
    if (!staged && !isnull) {
      MemW vw{vb + vo};
      put_value(vw, q, vget);
    }
    sk_st(koff + i + 1, ko + kl);
    sk_st(voff + i + 1, vo + vl);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    koff[0] = 0;
    voff[0] = 0;
  }
}

// ------------------------------------------------------------------ GROUP BY columns → key bytes

struct KeySrcDev {
  const void* data[SK_MAX];
  const int64_t* off[SK_MAX];
  const uint8_t* bytes[SK_MAX];
  const uint8_t* valid[SK_MAX];
};

__device__ __forceinline__ Val src_key_val(const SinkParams& q, const KeySrcDev& k, int64_t i, int c) {
  Val v{0, nullptr, 0, false};
  v.null = !bit_get(k.valid[c], i);
  if (q.ktype[c] == KHIP_TYPE_STRING) {
    v.s = k.bytes[c] + k.off[c][i];
    v.len = k.off[c][i + 1] - k.off[c][i];
  } else if (q.ktype[c] == KHIP_TYPE_INT32) {
    v.i = ((const int32_t*)k.data[c])[i];
  } else {
    v.i = ((const int64_t*)k.data[c])[i];
  }
  return v;
}

__device__ __forceinline__ bool src_key_null(const SinkParams& q, const KeySrcDev& k, int64_t i) {
  for (int c = 0; c < q.n_key; c++)
    if (src_key_val(q, k, i, c).null) return true;
  return false;
}

__global__ __launch_bounds__(256) void k_key_measure(const SinkParams* __restrict__ qp, KeySrcDev k, int64_t n,
                                                     int64_t* __restrict__ klen, uint8_t* __restrict__ kvalid) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const SinkParams& q = *qp;
  const bool ok = i < n && !src_key_null(q, k, i);
  const uint64_t b = __ballot(ok);
  if (i < n) {
    CountW w;
    if (ok) put_key(w, q, [&](int c) { return src_key_val(q, k, i, c); });
    klen[i + 1] = w.n;
  }
  // each wave writes its 64 rows' validity bits (8 bytes; the buffer is padded to whole waves)
  if ((threadIdx.x & 63) == 0 && i < n) *(uint64_t*)(kvalid + (i >> 3)) = b;
}

__global__ __launch_bounds__(256) void k_key_write(const SinkParams* __restrict__ qp, KeySrcDev k, int64_t n,
                                                   const int64_t* __restrict__ koff, uint8_t* __restrict__ kb) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const SinkParams& q = *qp;
  if (koff[i + 1] == koff[i]) return;
  MemW w{kb + koff[i]};
  put_key(w, q, [&](int c) { return src_key_val(q, k, i, c); });
}

// ------------------------------------------------------------------ scan (lengths → offsets)

// v[1..n] lengths → v[0..n] exclusive offsets from 0, in place.  Block b scans items
// [b*S, (b+1)*S) of v[1..]: pass 1 block sums, pass 2 one block over the sums, pass 3 in-block
// scan plus the block's carry.
__device__ __forceinline__ int64_t sk_block_scan(int64_t x, int64_t* wsum, int64_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t incl = x;
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  int64_t before = 0, tot = 0;
  for (int k = 0; k < SK_SCAN_T / 64; k++) {
    before += k < wave ? wsum[k] : 0;
    tot += wsum[k];
  }
  __syncthreads();
  *total = tot;
  return before + incl - x;  // exclusive
}

__global__ __launch_bounds__(SK_SCAN_T) void k_sk_scan1(const int64_t* __restrict__ v, int64_t n,
                                                        int64_t* __restrict__ bsum) {
  __shared__ int64_t wsum[SK_SCAN_T / 64];
  const int64_t base = (int64_t)blockIdx.x * SK_SCAN_T * SK_SCAN_I + (int64_t)threadIdx.x * SK_SCAN_I;
  int64_t s = 0;
  for (int u = 0; u < SK_SCAN_I; u++) s += base + u < n ? v[1 + base + u] : 0;
  int64_t tot;
  sk_block_scan(s, wsum, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SK_SCAN_T) void k_sk_scan2(int64_t* __restrict__ bsum, int64_t nb) {
  __shared__ int64_t wsum[SK_SCAN_T / 64];
  int64_t carry = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += SK_SCAN_T) {
    const int64_t b = b0 + threadIdx.x;
    const int64_t x = b < nb ? bsum[b] : 0;
    int64_t tot;
    const int64_t ex = sk_block_scan(x, wsum, &tot);
    if (b < nb) bsum[b] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) bsum[nb] = carry;
}

__global__ __launch_bounds__(SK_SCAN_T) void k_sk_scan3(int64_t* __restrict__ v, int64_t n,
                                                        const int64_t* __restrict__ bsum) {
  __shared__ int64_t wsum[SK_SCAN_T / 64];
  const int64_t base = (int64_t)blockIdx.x * SK_SCAN_T * SK_SCAN_I + (int64_t)threadIdx.x * SK_SCAN_I;
  int64_t x[SK_SCAN_I], s = 0;
  for (int u = 0; u < SK_SCAN_I; u++) {
    x[u] = base + u < n ? v[1 + base + u] : 0;
    s += x[u];
  }
  int64_t tot;
  int64_t run = bsum[blockIdx.x] + sk_block_scan(s, wsum, &tot);
  for (int u = 0; u < SK_SCAN_I; u++) {
    run += x[u];
    if (base + u < n) v[1 + base + u] = run;  // inclusive at i + 1 = exclusive at i + 1
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) v[0] = 0;
}

}  // namespace khip

using namespace khip;

struct khip_sink {
  khip_sink_desc desc{};
  SinkParams q{};
  int device = 0;
  hipStream_t stream = nullptr;
  DevBuf dq, bsum, bsum2, tsum, koff, kbytes, kvalid, voff, vbytes, vnull;
  DevBuf st_key, st_koff, st_kbytes, st_ws, st_we, st_tomb, st_col[SK_MAX], st_null[SK_MAX], st_cv[SK_MAX];
  std::vector<int64_t> h_koff;  // khip_sink_key of a host batch: the keys, in host memory
  std::vector<uint8_t> h_kbytes, h_kvalid;
};

namespace {

khip_status sk_stage(khip_sink* s, DevBuf& b, const void* src, size_t bytes, const void** dst) {
  if (!src) {
    *dst = nullptr;
    return KHIP_OK;
  }
  KHIP_TRY(b.ensure(std::max<size_t>(bytes, 8)));
  if (bytes) KHIP_TRY_HIP(hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, s->stream));
  *dst = b.p;
  return KHIP_OK;
}

// in place: off[1..n] lengths → off[0..n] offsets; returns the total (synchronises the stream)
// v[1..n] lengths → v[0..n] offsets, in place, on the stream (ws: the block sums); *total ← v[n]
// (a host copy: complete once the stream is synchronised, here when sync).
khip_status sk_scan(khip_sink* s, DevBuf& ws, int64_t* off, int64_t n, int64_t* total, bool sync = true) {
  const int64_t per = (int64_t)SK_SCAN_T * SK_SCAN_I;
  const int64_t nb = std::max<int64_t>(1, ceil_div(n, per));
  KHIP_TRY(ws.ensure((size_t)(nb + 1) * 8));
  int64_t* bs = ws.as<int64_t>();
  hipLaunchKernelGGL(k_sk_scan1, dim3(nb), dim3(SK_SCAN_T), 0, s->stream, off, n, bs);
  hipLaunchKernelGGL(k_sk_scan2, dim3(1), dim3(SK_SCAN_T), 0, s->stream, bs, nb);
  hipLaunchKernelGGL(k_sk_scan3, dim3(nb), dim3(SK_SCAN_T), 0, s->stream, off, n, bs);
  KHIP_TRY_HIP(hipGetLastError());
  KHIP_TRY_HIP(hipMemcpyAsync(total, bs + nb, 8, hipMemcpyDeviceToHost, s->stream));
  if (sync) KHIP_TRY_HIP(hipStreamSynchronize(s->stream));
  return KHIP_OK;
}

bool sk_type_ok(int t, bool str) {
  return t == KHIP_TYPE_INT32 || t == KHIP_TYPE_INT64 || t == KHIP_TYPE_DOUBLE || (str && t == KHIP_TYPE_STRING);
}

}  // namespace

extern "C" {

khip_status khip_sink_create(const khip_sink_desc* d, khip_sink** out) {
  clear_error();
  if (!d || !out) return fail(KHIP_E_INVALID, "null argument");
  const int kf = d->key_format, vf = d->value_format;
  if (kf != KHIP_FMT_KAFKA && kf != KHIP_FMT_JSON && kf != KHIP_FMT_DELIMITED)
    return fail(KHIP_E_UNSUPPORTED, "sink key format (KAFKA, JSON, DELIMITED)");
  if (vf != KHIP_FMT_KAFKA && vf != KHIP_FMT_JSON && vf != KHIP_FMT_DELIMITED)
    return fail(KHIP_E_UNSUPPORTED, "sink value format (KAFKA, JSON, DELIMITED)");
  if (d->n_key_cols < 1 || d->n_key_cols > SK_MAX || !d->key_types) return fail(KHIP_E_INVALID, "1..32 key columns");
  if (kf == KHIP_FMT_KAFKA && d->n_key_cols != 1)
    return fail(KHIP_E_UNSUPPORTED, "the KAFKA key format carries one column");
  if (d->n_value_cols < 0 || d->n_value_cols > SK_MAX || (d->n_value_cols && (!d->value_types || !d->value_src)))
    return fail(KHIP_E_INVALID, "0..32 value columns with types and sources");
  if (vf == KHIP_FMT_KAFKA && d->n_value_cols != 1) return fail(KHIP_E_UNSUPPORTED, "the KAFKA value format carries one column");
  if (d->window_kind < KHIP_WINDOW_NONE || d->window_kind > KHIP_WINDOW_SESSION) return fail(KHIP_E_INVALID, "window kind");
  khip_sink* s = new khip_sink();
  s->desc = *d;
  SinkParams& q = s->q;
  q.key_format = kf;
  q.value_format = vf;
  q.n_key = d->n_key_cols;
  q.n_val = d->n_value_cols;
  q.window_kind = d->window_kind;
  q.delim = d->delimiter ? d->delimiter : ',';
  auto name = [&](const char* const* names, int i, uint8_t* dst, int32_t* len) -> bool {
    const char* nm = names ? names[i] : nullptr;
    const size_t L = nm ? strlen(nm) : 0;
    if (!nm || L > SK_NAME) return false;
    memcpy(dst, nm, L);
    *len = (int32_t)L;
    return true;
  };
  for (int i = 0; i < q.n_key; i++) {
    q.ktype[i] = d->key_types[i];
    if (!sk_type_ok(q.ktype[i], true)) {
      delete s;
      return fail(KHIP_E_UNSUPPORTED, "key column type");
    }
    if (kf == KHIP_FMT_JSON && q.n_key > 1 && !name(d->key_names, i, q.kname[i], &q.kname_len[i])) {
      delete s;
      return fail(KHIP_E_INVALID, "JSON key column names (<= 64 bytes) required");
    }
  }
  for (int i = 0; i < q.n_val; i++) {
    q.vtype[i] = d->value_types[i];
    q.vsrc[i] = d->value_src[i];
    if (!sk_type_ok(q.vtype[i], false) || q.vsrc[i] < KHIP_SINK_SRC_WE || q.vsrc[i] >= SK_MAX ||
        q.vsrc[i] == -1) {
      delete s;
      return fail(KHIP_E_INVALID, "value column type (INT32/INT64/DOUBLE) and source");
    }
    if (q.vsrc[i] < 0 && q.vtype[i] != KHIP_TYPE_INT64) {
      delete s;
      return fail(KHIP_E_INVALID, "WINDOWSTART / WINDOWEND are BIGINT");
    }
    if (vf == KHIP_FMT_JSON && !name(d->value_names, i, q.vname[i], &q.vname_len[i])) {
      delete s;
      return fail(KHIP_E_INVALID, "JSON value column names (<= 64 bytes) required");
    }
  }
  auto prefix = [](int i, const uint8_t* nm, int len, uint8_t* dst, int32_t* dlen) {
    HostW w{dst, 0, SK_PRE};
    w.put(i ? ',' : '{');
    put_json_str(w, nm, len);
    w.put(':');
    *dlen = w.n <= SK_PRE ? w.n : -1;
  };
  for (int i = 0; i < SK_MAX; i++) q.kpre_len[i] = q.vpre_len[i] = -1;
  if (kf == KHIP_FMT_JSON && q.n_key > 1)
    for (int i = 0; i < q.n_key; i++) prefix(i, q.kname[i], q.kname_len[i], q.kpre[i], &q.kpre_len[i]);
  if (vf == KHIP_FMT_JSON)
    for (int i = 0; i < q.n_val; i++) prefix(i, q.vname[i], q.vname_len[i], q.vpre[i], &q.vpre_len[i]);
  s->device = d->device;
  DeviceGuard g(s->device);
  if (hipStreamCreateWithFlags(&s->stream, hipStreamDefault) != hipSuccess) {
    delete s;
    return fail(KHIP_E_DEVICE, "hipStreamCreate failed (no device?)");
  }
  khip_status st = s->dq.ensure(sizeof(SinkParams));
  if (st == KHIP_OK && hipMemcpy(s->dq.p, &s->q, sizeof(SinkParams), hipMemcpyHostToDevice) != hipSuccess)
    st = fail(KHIP_E_DEVICE, "copying the sink parameters");
  if (st != KHIP_OK) {
    khip_sink_destroy(s);
    return st;
  }
  *out = s;
  return KHIP_OK;
}

khip_status khip_sink_key(khip_sink* s, const khip_batch* in, const khip_key_col* cols, khip_batch* out) {
  clear_error();
  if (!s || !in || !cols || !out) return fail(KHIP_E_INVALID, "null argument");
  const SinkParams& q = s->q;
  const int64_t n = in->n_rows;
  if (n < 0) return fail(KHIP_E_INVALID, "batch rows");
  if (in->mem != KHIP_MEM_HOST && in->mem != KHIP_MEM_DEVICE) return fail(KHIP_E_INVALID, "batch mem");
  KeySrcDev k{};
  for (int c = 0; c < q.n_key; c++) {
    const bool str = q.ktype[c] == KHIP_TYPE_STRING;
    if (n && (str ? !(cols[c].offsets && cols[c].bytes) : !cols[c].data))
      return fail(KHIP_E_INVALID, "key column " + std::to_string(c) + " arrays");
    k.data[c] = cols[c].data;
    k.off[c] = cols[c].offsets;
    k.bytes[c] = cols[c].bytes;
    k.valid[c] = cols[c].valid;
  }
  DeviceGuard g(s->device);
  const size_t bm = (size_t)(n + 7) / 8;
  if (in->mem == KHIP_MEM_HOST && n) {
    const void* p;
    for (int c = 0; c < q.n_key; c++) {
      if (q.ktype[c] == KHIP_TYPE_STRING) {
        KHIP_TRY(sk_stage(s, s->st_col[c], cols[c].offsets, (size_t)(n + 1) * 8, &p));
        k.off[c] = (const int64_t*)p;
        KHIP_TRY(sk_stage(s, s->st_null[c], cols[c].bytes, (size_t)cols[c].offsets[n], &p));
        k.bytes[c] = (const uint8_t*)p;
      } else {
        KHIP_TRY(sk_stage(s, s->st_col[c], cols[c].data, (size_t)n * (q.ktype[c] == KHIP_TYPE_INT32 ? 4 : 8), &p));
        k.data[c] = p;
      }
      KHIP_TRY(sk_stage(s, s->st_cv[c], cols[c].valid, bm, &p));
      k.valid[c] = (const uint8_t*)p;
    }
  }
  KHIP_TRY(s->koff.ensure((size_t)(n + 1) * 8));
  KHIP_TRY(s->kvalid.ensure(((size_t)(n + 63) / 64) * 8 + 8));
  int64_t* koff = s->koff.as<int64_t>();
  int64_t total = 0;
  if (n) {
    hipLaunchKernelGGL(k_key_measure, dim3(ceil_div(n, 256)), dim3(256), 0, s->stream, s->dq.as<SinkParams>(), k, n, koff,
                       s->kvalid.as<uint8_t>());
    KHIP_TRY_HIP(hipGetLastError());
    KHIP_TRY(sk_scan(s, s->bsum, koff, n, &total));
    KHIP_TRY(s->kbytes.ensure((size_t)std::max<int64_t>(total, 8)));
    hipLaunchKernelGGL(k_key_write, dim3(ceil_div(n, 256)), dim3(256), 0, s->stream, s->dq.as<SinkParams>(), k, n, koff,
                       s->kbytes.as<uint8_t>());
    KHIP_TRY_HIP(hipGetLastError());
  } else {
    KHIP_TRY(s->kbytes.ensure(8));
    KHIP_TRY_HIP(hipMemsetAsync(koff, 0, 8, s->stream));
  }
  *out = *in;
  out->key_i64 = nullptr;
  if (in->mem == KHIP_MEM_HOST) {  // a host batch gets host keys (the rest stays the caller's)
    s->h_koff.resize((size_t)n + 1);
    s->h_kbytes.resize((size_t)std::max<int64_t>(total, 1));
    s->h_kvalid.resize(bm + 8);
    KHIP_TRY_HIP(hipMemcpyAsync(s->h_koff.data(), koff, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost, s->stream));
    if (total) KHIP_TRY_HIP(hipMemcpyAsync(s->h_kbytes.data(), s->kbytes.p, (size_t)total, hipMemcpyDeviceToHost, s->stream));
    if (n) KHIP_TRY_HIP(hipMemcpyAsync(s->h_kvalid.data(), s->kvalid.p, bm, hipMemcpyDeviceToHost, s->stream));
    KHIP_TRY_HIP(hipStreamSynchronize(s->stream));
    out->key_offsets = s->h_koff.data();
    out->key_bytes = s->h_kbytes.data();
    out->key_valid = s->h_kvalid.data();
    return KHIP_OK;
  }
  out->key_offsets = koff;
  out->key_bytes = s->kbytes.as<uint8_t>();
  out->key_valid = s->kvalid.as<uint8_t>();
  return KHIP_OK;
}

khip_status khip_sink_encode(khip_sink* s, const khip_sink_rows* rows, khip_sink_out* out) {
  clear_error();
  if (!s || !rows || !out) return fail(KHIP_E_INVALID, "null argument");
  const SinkParams& q = s->q;
  const int64_t n = rows->n_rows;
  if (n < 0 || !out->key_offsets || !out->value_offsets || !out->value_null) return fail(KHIP_E_INVALID, "rows / outputs");
  const bool windowed = q.window_kind != KHIP_WINDOW_NONE;
  if (n && windowed && !rows->window_start) return fail(KHIP_E_INVALID, "a windowed key needs window_start");
  if (n && q.window_kind == KHIP_WINDOW_SESSION && !rows->window_end) return fail(KHIP_E_INVALID, "a session key needs window_end");
  const bool str_key = rows->key_serialized || q.ktype[0] == KHIP_TYPE_STRING;
  if (!rows->key_serialized && (q.n_key != 1 || q.ktype[0] == KHIP_TYPE_DOUBLE))
    return fail(KHIP_E_INVALID, "row keys: one INT32/INT64/STRING key column, or serialized keys");
  if (n && (str_key ? !(rows->key_offsets && rows->key_bytes) : !rows->key_i64))
    return fail(KHIP_E_INVALID, "row key arrays");
  int ncol = 0;
  int ctype[SK_MAX];
  bool used[SK_MAX];  // columns some value column reads: only those are staged or passed on
  for (int c = 0; c < SK_MAX; c++) {
    ctype[c] = KHIP_TYPE_INT64;
    used[c] = false;
  }
  for (int c = 0; c < q.n_val; c++) {
    const int src = q.vsrc[c];
    if (src == KHIP_SINK_SRC_WS && n && !rows->window_start) return fail(KHIP_E_INVALID, "WINDOWSTART source");
    if (src == KHIP_SINK_SRC_WE && n && !rows->window_end) return fail(KHIP_E_INVALID, "WINDOWEND source");
    if (src >= 0) {
      if (n && (!rows->col_data || !rows->col_data[src])) return fail(KHIP_E_INVALID, "value source column");
      ncol = std::max(ncol, src + 1);
      ctype[src] = q.vtype[c];
      used[src] = true;
    }
  }
  DeviceGuard g(s->device);
  RowsDev r{};
  r.key_serialized = rows->key_serialized;
  r.key_i64 = rows->key_i64;
  r.key_off = rows->key_offsets;
  r.key_bytes = rows->key_bytes;
  r.ws = rows->window_start;
  r.we = rows->window_end;
  r.tomb = rows->tombstone;
  for (int c = 0; c < ncol; c++) {
    r.col[c] = used[c] && rows->col_data ? rows->col_data[c] : nullptr;
    r.cnull[c] = used[c] && rows->col_null ? rows->col_null[c] : nullptr;
  }
  if (rows->mem == KHIP_MEM_HOST && n) {
    const void* p;
    if (str_key) {
      KHIP_TRY(sk_stage(s, s->st_koff, rows->key_offsets, (size_t)(n + 1) * 8, &p));
      r.key_off = (const int64_t*)p;
      KHIP_TRY(sk_stage(s, s->st_kbytes, rows->key_bytes, (size_t)rows->key_offsets[n], &p));
      r.key_bytes = (const uint8_t*)p;
    } else {
      KHIP_TRY(sk_stage(s, s->st_key, rows->key_i64, (size_t)n * 8, &p));
      r.key_i64 = (const int64_t*)p;
    }
    KHIP_TRY(sk_stage(s, s->st_ws, rows->window_start, (size_t)n * 8, &p));
    r.ws = (const int64_t*)p;
    KHIP_TRY(sk_stage(s, s->st_we, rows->window_end, (size_t)n * 8, &p));
    r.we = (const int64_t*)p;
    KHIP_TRY(sk_stage(s, s->st_tomb, rows->tombstone, (size_t)n, &p));
    r.tomb = (const uint8_t*)p;
    for (int c = 0; c < ncol; c++) {
      if (!used[c] || !rows->col_data[c]) continue;
      KHIP_TRY(sk_stage(s, s->st_col[c], rows->col_data[c], (size_t)n * (ctype[c] == KHIP_TYPE_INT32 ? 4 : 8), &p));
      r.col[c] = p;
      KHIP_TRY(sk_stage(s, s->st_null[c], rows->col_null ? rows->col_null[c] : nullptr, (size_t)n, &p));
      r.cnull[c] = (const uint8_t*)p;
    }
  } else if (rows->mem != KHIP_MEM_HOST && rows->mem != KHIP_MEM_DEVICE) {
    return fail(KHIP_E_INVALID, "rows mem");
  }
  if (out->mem != KHIP_MEM_HOST && out->mem != KHIP_MEM_DEVICE) return fail(KHIP_E_INVALID, "output mem");
  const bool dev_out = out->mem == KHIP_MEM_DEVICE;
  // offsets: straight into device outputs, else into the handle's buffers
  int64_t *koff = dev_out ? out->key_offsets : nullptr, *voff = dev_out ? out->value_offsets : nullptr;
  if (!dev_out) {
    KHIP_TRY(s->koff.ensure((size_t)(n + 1) * 8));
    KHIP_TRY(s->voff.ensure((size_t)(n + 1) * 8));
    koff = s->koff.as<int64_t>();
    voff = s->voff.as<int64_t>();
  }
  int64_t ktot = 0, vtot = 0;
  const int64_t nT = ceil_div(n, SK_TILE);
  // every key the same width: a KAFKA INT32 / BIGINT key and its window suffix
  int kfix = 0;
  if (!rows->key_serialized && q.key_format == KHIP_FMT_KAFKA && q.ktype[0] != KHIP_TYPE_STRING)
    kfix = (q.ktype[0] == KHIP_TYPE_INT64 ? 8 : 4) +
           (q.window_kind == KHIP_WINDOW_SESSION ? 16 : q.window_kind != KHIP_WINDOW_NONE ? 8 : 0);
  if (n) {
    KHIP_TRY(s->tsum.ensure((size_t)(2 * (nT + 1)) * 8));
    int64_t* ts = s->tsum.as<int64_t>();
    hipLaunchKernelGGL(k_sink_measure, dim3((unsigned)nT), dim3(256), 0, s->stream, s->dq.as<SinkParams>(), r, n, kfix, nT,
                       koff, voff, ts);
    KHIP_TRY_HIP(hipGetLastError());
    int64_t tk = 0, tv = 0;
    if (!kfix) KHIP_TRY(sk_scan(s, s->bsum, ts, nT, &tk, false));
    KHIP_TRY(sk_scan(s, s->bsum2, ts + nT + 1, nT, &tv, true));
    ktot = kfix ? (int64_t)kfix * n : tk;
    vtot = tv;
  } else {
    const int64_t z = 0;
    if (dev_out) {
      KHIP_TRY_HIP(hipMemcpyAsync(koff, &z, 8, hipMemcpyHostToDevice, s->stream));
      KHIP_TRY_HIP(hipMemcpyAsync(voff, &z, 8, hipMemcpyHostToDevice, s->stream));
      KHIP_TRY_HIP(hipStreamSynchronize(s->stream));
    }
  }
  out->key_len = ktot;
  out->value_len = vtot;
  if (ktot > out->key_capacity || vtot > out->value_capacity) return fail(KHIP_E_BUFFER, "sink output capacity too small");
  if (n && (ktot && !out->key_bytes)) return fail(KHIP_E_INVALID, "key_bytes");
  if (n && (vtot && !out->value_bytes)) return fail(KHIP_E_INVALID, "value_bytes");
  uint8_t *kb = out->key_bytes, *vb = out->value_bytes, *vn = out->value_null;
  if (!dev_out) {
    KHIP_TRY(s->kbytes.ensure((size_t)std::max<int64_t>(ktot, 8)));
    KHIP_TRY(s->vbytes.ensure((size_t)std::max<int64_t>(vtot, 8)));
    KHIP_TRY(s->vnull.ensure((size_t)std::max<int64_t>(n, 8)));
    kb = s->kbytes.as<uint8_t>();
    vb = s->vbytes.as<uint8_t>();
    vn = s->vnull.as<uint8_t>();
  }
  if (n) {
    const int kwords = kfix && q.ktype[0] == KHIP_TYPE_INT64 && ((uintptr_t)kb & 7) == 0 ? kfix / 8 : 0;
    hipLaunchKernelGGL(k_sink_write, dim3((unsigned)nT), dim3(256), 0, s->stream, s->dq.as<SinkParams>(), r, n, kfix,
                       kwords, nT, s->tsum.as<int64_t>(), koff, kb, voff, vb, vn);
    KHIP_TRY_HIP(hipGetLastError());
  }
  if (!dev_out) {
    KHIP_TRY_HIP(hipMemcpyAsync(out->key_offsets, koff, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost, s->stream));
    KHIP_TRY_HIP(hipMemcpyAsync(out->value_offsets, voff, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost, s->stream));
    if (n) KHIP_TRY_HIP(hipMemcpyAsync(out->value_null, vn, (size_t)n, hipMemcpyDeviceToHost, s->stream));
    if (ktot) KHIP_TRY_HIP(hipMemcpyAsync(out->key_bytes, kb, (size_t)ktot, hipMemcpyDeviceToHost, s->stream));
    if (vtot) KHIP_TRY_HIP(hipMemcpyAsync(out->value_bytes, vb, (size_t)vtot, hipMemcpyDeviceToHost, s->stream));
  }
  KHIP_TRY_HIP(hipStreamSynchronize(s->stream));
  return KHIP_OK;
}

khip_status khip_sink_sync(khip_sink* s) {
  clear_error();
  if (!s) return fail(KHIP_E_INVALID, "null argument");
  DeviceGuard g(s->device);
  KHIP_TRY_HIP(hipStreamSynchronize(s->stream));
  return KHIP_OK;
}

khip_status khip_sink_destroy(khip_sink* s) {
  if (!s) return KHIP_OK;
  DeviceGuard g(s->device);
  if (s->stream) hipStreamSynchronize(s->stream);
  DevBuf* bufs[] = {&s->dq, &s->bsum, &s->bsum2, &s->tsum, &s->koff, &s->kbytes, &s->kvalid, &s->voff, &s->vbytes, &s->vnull, &s->st_key,
                    &s->st_koff, &s->st_kbytes, &s->st_ws, &s->st_we, &s->st_tomb};
  for (DevBuf* b : bufs) b->release();
  for (int c = 0; c < SK_MAX; c++) {
    s->st_col[c].release();
    s->st_null[c].release();
    s->st_cv[c].release();
  }
  if (s->stream) hipStreamDestroy(s->stream);
  delete s;
  return KHIP_OK;
}

}  // extern "C"
