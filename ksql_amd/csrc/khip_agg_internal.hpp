// khip_agg_internal.hpp — shared declarations of the aggregate engines.
#pragma once

#include <vector>

#include "khip_dict.hpp"
#include "khip_util.hpp"

namespace khip {

constexpr int BLOCK = 256;
constexpr int ITEMS = 8;
constexpr int RPB = BLOCK * ITEMS;  // records per block (k_blockmax and k_apply agree)
constexpr int MAX_COLS = 8;
constexpr int MAX_OPS = 40;
constexpr int MAX_PROBE = 2048;
constexpr int MAX_FANOUT = 4095;  // windows per record encodable in a claim reference
constexpr int64_t EMPTY_WS = INT64_MIN;
constexpr int NPART = 8;

enum { P_ACCEPTED, P_NULL_KEY, P_NULL_ROW, P_BAD_TS, P_APPLIED, P_LATE, P_FAILED, P_NEW };

enum OpKind : int8_t { OP_INC = 0, OP_INC_VALID, OP_ADD_I64, OP_ADD_F64, OP_MIN, OP_MAX };

struct UpdOp {
  int8_t kind;
  int8_t col;
  int16_t word;
};

struct ApplyParams {
  int32_t windowed;
  int32_t slot_words;
  int64_t size, adv, grace;
  int32_t n_cols;
  int32_t n_ops;
  int32_t col_type[MAX_COLS];
  UpdOp ops[MAX_OPS];
};

struct ColPtrs {
  const void* data[MAX_COLS];
  const uint8_t* valid[MAX_COLS];
};

// How one aggregate's result is decoded from the state words.
struct AggOut {
  int32_t kind;   // KHIP_AGG_*
  int32_t type;   // input column type (INT64 for COUNT*)
  int32_t w_val;  // value word
  int32_t w_cnt;  // non-null count word (-1 if none)
};

struct HavingDev {
  int32_t active;
  int32_t op;
  AggOut a;
  int64_t i64;
  double f64;
  // pull-query filter (khip_agg_get; KsMaterializedWindowTable.get): key in the sorted unique
  // `keys` (when n_keys > 0) and WINDOWSTART / WINDOWEND inside closed bounds (windowed tables)
  int32_t pull;
  int32_t pull_windowed;
  const int64_t* keys;
  int64_t n_keys;
  int64_t ws_lo, ws_hi, we_lo, we_hi, size_ms;
  int32_t log2P;  // partitioned engine: partitions = 2^log2P (partition-directed lookups)
  const int64_t* host_keys;  // host copy of `keys` (host side only)
  // partitioned engine, > 256 keys: keys grouped by partition (sorted within each), offsets P+1
  const int64_t* pkeys;
  const int64_t* pkoff;
  // window store retention (RETENTION, default size + grace; S/StreamAggregateBuilder.java:293,
  // 322,350): rows with ws < vis_from have expired from the store (windowed tables)
  int32_t vis;
  int64_t vis_from;
  // EMIT FINAL (S/StreamAggregateBuilder.java:282-285): the windows that closed during the last
  // push (ws + size in (fin_c0, fin_c1]) minus those that had already expired at the record
  // that closed them (n_lost sorted disjoint ws ranges [lost[2i], lost[2i+1]])
  int32_t fin;
  int32_t n_lost;
  int64_t fin_c0, fin_c1, fin_size;
  const int64_t* lost;
  int32_t session;  // SESSION rows: WINDOWEND is the row's own end (word 2), not ws + size
  // KHIP_TIME_PARTITION: retention and EMIT FINAL per task.  A row's task is its key's partition
  // (co-partitioned keys), found through the handle's key map (pm_key / pm_part, open addressing,
  // INT64_MIN = empty; the key INT64_MIN itself at pm_part[pm_mask + 1]); its bounds are that
  // partition's: p_vis[p] (vis_from), p_fin[2p], p_fin[2p + 1] (fin_c0, fin_c1) and the lost ws
  // ranges p_lost[2 * p_lost_off[p] .. 2 * p_lost_off[p + 1]).  pm_key == null: the fields above.
  const int64_t* pm_key;
  const int32_t* pm_part;
  uint64_t pm_mask;
  int32_t pm_pruned;  // keys whose windows had all expired left the map: a key not found is one of them
  const int64_t* p_vis;
  const int64_t* p_fin;
  const int64_t* p_lost_off;
  const int64_t* p_lost;
};

__device__ __forceinline__ uint64_t pmap_hash(int64_t k) {
  uint64_t z = (uint64_t)k * 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 31)) * 0xBF58476D1CE4E5B9ULL;
  return z ^ (z >> 29);
}

// The partition of key k in the key map, or -1 when the key never reached it.
__device__ __forceinline__ int pmap_find(const int64_t* __restrict__ keys, const int32_t* __restrict__ parts,
                                         uint64_t mask, int64_t k) {
  if (k == INT64_MIN) return parts[mask + 1];
  uint64_t s = pmap_hash(k) & mask;
  for (uint64_t probe = 0; probe <= mask; probe++) {
    const int64_t c = keys[s];
    if (c == k) return parts[s];
    if (c == INT64_MIN) return -1;
    s = (s + 1) & mask;
  }
  return -1;
}

// Retention and EMIT FINAL selection of a row [key, ws, ...] (no-ops unless h.vis / h.fin).
__device__ __forceinline__ bool store_ok(const uint64_t* s, const HavingDev& h) {
  const int64_t ws = (int64_t)s[1];
  int64_t vis_from = h.vis_from, c0 = h.fin_c0, c1 = h.fin_c1;
  const int64_t* lost = h.lost;
  int n_lost = h.n_lost;
  if (h.pm_key && (h.vis || h.fin)) {  // KHIP_TIME_PARTITION: the bounds of the row's own task
    const int p = pmap_find(h.pm_key, h.pm_part, h.pm_mask, (int64_t)s[0]);
    if (p >= 0) {
      vis_from = h.p_vis[p];
      c0 = h.p_fin[2 * p];
      c1 = h.p_fin[2 * p + 1];
      lost = h.p_lost + 2 * h.p_lost_off[p];
      n_lost = (int)(h.p_lost_off[p + 1] - h.p_lost_off[p]);
    } else if (h.pm_pruned) {
      return false;  // every window of the key had expired in its task when the key left the map
    }
  }
  if (h.vis && ws < vis_from) return false;
  if (h.fin) {
    const int64_t end = ws + h.fin_size;
    if (end <= c0 || end > c1) return false;
    int lo = 0, hi = n_lost;  // first range starting after ws
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (lost[2 * mid] <= ws) lo = mid + 1;
      else hi = mid;
    }
    if (lo > 0 && ws <= lost[2 * (lo - 1) + 1]) return false;
  }
  return true;
}

__device__ __forceinline__ bool pull_ok(const uint64_t* s, const HavingDev& h) {
  if (!store_ok(s, h)) return false;
  if (!h.pull) return true;
  if (h.n_keys > 0) {
    const int64_t k = (int64_t)s[0];
    int64_t lo = 0, hi = h.n_keys;  // lower_bound
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (h.keys[mid] < k) lo = mid + 1;
      else hi = mid;
    }
    if (lo >= h.n_keys || h.keys[lo] != k) return false;
  }
  if (h.pull_windowed) {
    const int64_t ws = (int64_t)s[1], we = h.session ? (int64_t)s[2] : ws + h.size_ms;
    if (ws < h.ws_lo || ws > h.ws_hi || we < h.we_lo || we > h.we_hi) return false;
  }
  return true;
}

// ------------------------------------------------------------------ device utils

__device__ __forceinline__ int64_t wave_incl_max(int64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    int64_t t = __shfl_up(v, off, 64);
    if (lane >= off) v = t > v ? t : v;
  }
  return v;
}

// Inclusive prefix max over the block (blockDim.x threads, multiple of 64).
__device__ __forceinline__ int64_t block_incl_max(int64_t v, int64_t* lds, int64_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_incl_max(v);
  if (lane == 63) lds[wave] = v;
  __syncthreads();
  int64_t pre = INT64_MIN, tot = INT64_MIN;
  for (int w = 0; w < nw; w++) {
    int64_t x = lds[w];
    if (w < wave) pre = x > pre ? x : pre;
    tot = x > tot ? x : tot;
  }
  __syncthreads();
  *total = tot;
  return v > pre ? v : pre;
}

__device__ __forceinline__ int64_t wave_sum(int64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ uint64_t ld_relaxed(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Bytes [8k, 8k + 8) of p (little-endian, as an unaligned load would give them) from the aligned
// words holding them: `cur` = aligned word k, `nxt` = aligned word k + 1 (sh = 8 * (p & 7)).
__device__ __forceinline__ uint64_t funnel_word(uint64_t cur, uint64_t nxt, int sh) {
  return sh ? (cur >> sh) | (nxt << (64 - sh)) : cur;
}

// Long keys: 8 key bytes per step read as aligned 8-byte words (a byte per load made the chain of
// a 40-byte URL 40 dependent loads; C1's dictionary probe), the same value as the bytewise rule:
// h over the full little-endian words, then the tail bytes zero-extended.
__device__ __forceinline__ uint64_t hash_bytes_dev(const uint8_t* p, int64_t n) {
  uint64_t h = 0x84222325cbf29ce4ULL ^ (uint64_t)n;
  const uint64_t a = (uint64_t)p;
  // (pointer arithmetic, not an integer cast: the loads stay global_load, not flat_load)
  const uint64_t* base = (const uint64_t*)(p - (a & 7));
  const int sh = (int)(a & 7) * 8;
  const int64_t na = n > 0 ? (int64_t)(((a & 7) + (uint64_t)n + 7) >> 3) : 0;  // aligned words holding key bytes
  uint64_t cur = na > 0 ? base[0] : 0ULL;
  int64_t k = 0;
  for (; 8 * k + 8 <= n; k++) {
    const uint64_t nxt = k + 1 < na ? base[k + 1] : 0ULL;
    h = mix64(h ^ funnel_word(cur, nxt, sh)) * 0x9E3779B97F4A7C15ULL;
    cur = nxt;
  }
  const int64_t left = n - 8 * k;  // 0..7 tail bytes
  uint64_t w = 0;
  if (left > 0) w = funnel_word(cur, k + 1 < na ? base[k + 1] : 0ULL, sh) & ((1ULL << (8 * left)) - 1);
  return mix64(h ^ w ^ ((uint64_t)(n & 7) << 59));
}

// Short keys (n <= 8 * KW_MAX bytes) as little-endian words read with aligned 8-byte loads (only
// the words holding key bytes; bytes past n are 0): w[k] is what an unaligned load of bytes
// [8k, 8k + 8) would give.  One to four loads instead of a load per byte.
constexpr int KW_MAX = 3;
__device__ __forceinline__ void key_words(const uint8_t* p, int64_t n, uint64_t (&w)[KW_MAX]) {
  const uint64_t a = (uint64_t)p;
  // (pointer arithmetic, not an integer cast: the loads stay global_load, not flat_load)
  const uint64_t* base = (const uint64_t*)(p - (a & 7));
  const int sh = (int)(a & 7) * 8;
  const int na = (int)(((a & 7) + (uint64_t)n + 7) >> 3);  // aligned words holding key bytes
  uint64_t A[KW_MAX + 1];
#pragma unroll
  for (int k = 0; k <= KW_MAX; k++) A[k] = k < na ? base[k] : 0ULL;
#pragma unroll
  for (int k = 0; k < KW_MAX; k++) {
    uint64_t x = sh ? (A[k] >> sh) | (A[k + 1] << (64 - sh)) : A[k];
    const int64_t left = n - 8 * k;  // key bytes in this word
    if (left <= 0) x = 0;
    else if (left < 8) x &= (1ULL << (8 * left)) - 1;
    w[k] = x;
  }
}

// hash_bytes_dev over key_words' words (the same value).
__device__ __forceinline__ uint64_t hash_key_words(const uint64_t (&w)[KW_MAX], int64_t n) {
  uint64_t h = 0x84222325cbf29ce4ULL ^ (uint64_t)n;
  const int full = (int)(n >> 3);
  uint64_t tail = 0;
#pragma unroll
  for (int k = 0; k < KW_MAX; k++) {
    if (k < full) h = mix64(h ^ w[k]) * 0x9E3779B97F4A7C15ULL;
    else if (k == full) tail = w[k];
  }
  return mix64(h ^ tail ^ ((uint64_t)(n & 7) << 59));
}

// key_words of a key against n bytes at an 8-aligned arena entry (padding bytes ignored).
__device__ __forceinline__ bool key_words_eq_aligned(const uint64_t (&w)[KW_MAX], const uint8_t* e, int64_t n) {
  const uint64_t* q = (const uint64_t*)e;
  bool eq = true;
#pragma unroll
  for (int k = 0; k < KW_MAX; k++) {
    const int64_t left = n - 8 * k;
    if (left <= 0) break;
    uint64_t x = q[k];
    if (left < 8) x &= (1ULL << (8 * left)) - 1;
    eq = eq && x == w[k];
  }
  return eq;
}

// n bytes at an 8-aligned arena entry e against the key bytes at p, 8 bytes per step (e's padding
// past n ignored).
__device__ __forceinline__ bool bytes_eq_aligned(const uint8_t* e, const uint8_t* p, int64_t n) {
  const uint64_t* q = (const uint64_t*)e;
  const uint64_t a = (uint64_t)p;
  const uint64_t* base = (const uint64_t*)(p - (a & 7));
  const int sh = (int)(a & 7) * 8;
  const int64_t na = n > 0 ? (int64_t)(((a & 7) + (uint64_t)n + 7) >> 3) : 0;
  uint64_t cur = na > 0 ? base[0] : 0ULL;
  for (int64_t k = 0; 8 * k < n; k++) {
    const uint64_t nxt = k + 1 < na ? base[k + 1] : 0ULL;
    uint64_t x = funnel_word(cur, nxt, sh) ^ q[k];
    const int64_t left = n - 8 * k;
    if (left < 8) x &= (1ULL << (8 * left)) - 1;
    if (x) return false;
    cur = nxt;
  }
  return true;
}

__device__ __forceinline__ int64_t load_col_raw(const ColPtrs& c, int32_t type, int col, int64_t i) {
  if (type == KHIP_TYPE_INT32) return (int64_t)((const int32_t*)c.data[col])[i];
  return ((const int64_t*)c.data[col])[i];  // INT64, or DOUBLE bits
}

// One aggregate's result from its value word and non-null count word.  Returns false for
// SQL NULL; sets *iv for integer results, *dv for DOUBLE results.
__device__ __forceinline__ bool decode_words(uint64_t val, uint64_t cntw, const AggOut& a, int64_t* iv, double* dv) {
  switch (a.kind) {
    case KHIP_AGG_COUNT_STAR:
    case KHIP_AGG_COUNT:
      *iv = (int64_t)val;
      return true;
    case KHIP_AGG_SUM:
      if (a.type == KHIP_TYPE_DOUBLE) __builtin_memcpy(dv, &val, 8);
      else if (a.type == KHIP_TYPE_INT32) *iv = (int64_t)(int32_t)val;
      else *iv = (int64_t)val;
      return true;
    case KHIP_AGG_MIN:
    case KHIP_AGG_MAX:
      if ((int64_t)cntw == 0) return false;
      if (a.type == KHIP_TYPE_DOUBLE) *dv = f64_from_order_key((int64_t)val);
      else *iv = (int64_t)val;
      return true;
    case KHIP_AGG_AVG: {
      const int64_t c = (int64_t)cntw;
      if (c == 0) { *dv = 0.0; return true; }
      if (a.type == KHIP_TYPE_DOUBLE) {
        double sum;
        __builtin_memcpy(&sum, &val, 8);
        *dv = sum / (double)c;
      } else if (a.type == KHIP_TYPE_INT32) {
        *dv = (double)(int32_t)val / (double)c;
      } else {
        *dv = (double)(int64_t)val / (double)c;
      }
      return true;
    }
  }
  return false;
}

__device__ __forceinline__ bool decode_result(const uint64_t* s, const AggOut& a, int64_t* iv, double* dv) {
  return decode_words(s[a.w_val], a.w_cnt >= 0 ? s[a.w_cnt] : 0, a, iv, dv);
}

__device__ __forceinline__ bool result_is_double(const AggOut& a) {
  if (a.kind == KHIP_AGG_AVG) return true;
  if (a.kind == KHIP_AGG_COUNT || a.kind == KHIP_AGG_COUNT_STAR) return false;
  return a.type == KHIP_TYPE_DOUBLE;
}

// HAVING on an aggregate's value / count words (no pull filter)
__device__ __forceinline__ bool having_ok_words(uint64_t val, uint64_t cntw, const HavingDev& h) {
  if (!h.active) return true;
  int64_t iv = 0;
  double dv = 0.0;
  if (!decode_words(val, cntw, h.a, &iv, &dv)) return false;
  int c;
  if (result_is_double(h.a)) {
    if (dv != dv) return h.op == KHIP_OP_NE;
    c = dv < h.f64 ? -1 : (dv > h.f64 ? 1 : 0);
  } else {
    c = iv < h.i64 ? -1 : (iv > h.i64 ? 1 : 0);
  }
  switch (h.op) {
    case KHIP_OP_GT: return c > 0;
    case KHIP_OP_GE: return c >= 0;
    case KHIP_OP_LT: return c < 0;
    case KHIP_OP_LE: return c <= 0;
    case KHIP_OP_EQ: return c == 0;
    case KHIP_OP_NE: return c != 0;
  }
  return false;
}

// The query's HAVING alone (no pull-query filter): the engines' own row checks.
__device__ __forceinline__ bool having_only(const uint64_t* s, const HavingDev& h) {
  if (!h.active) return true;
  int64_t iv = 0;
  double dv = 0.0;
  if (!decode_result(s, h.a, &iv, &dv)) return false;
  int c;
  if (result_is_double(h.a)) {
    if (dv != dv) return h.op == KHIP_OP_NE;
    c = dv < h.f64 ? -1 : (dv > h.f64 ? 1 : 0);
  } else {
    c = iv < h.i64 ? -1 : (iv > h.i64 ? 1 : 0);
  }
  switch (h.op) {
    case KHIP_OP_GT: return c > 0;
    case KHIP_OP_GE: return c >= 0;
    case KHIP_OP_LT: return c < 0;
    case KHIP_OP_LE: return c <= 0;
    case KHIP_OP_EQ: return c == 0;
    case KHIP_OP_NE: return c != 0;
  }
  return false;
}

__device__ __forceinline__ bool having_ok(const uint64_t* s, const HavingDev& h) {
  if (!pull_ok(s, h)) return false;
  if (!h.active) return true;
  int64_t iv = 0;
  double dv = 0.0;
  if (!decode_result(s, h.a, &iv, &dv)) return false;
  int c;
  if (result_is_double(h.a)) {
    if (dv != dv) return h.op == KHIP_OP_NE;
    c = dv < h.f64 ? -1 : (dv > h.f64 ? 1 : 0);
  } else {
    c = iv < h.i64 ? -1 : (iv > h.i64 ? 1 : 0);
  }
  switch (h.op) {
    case KHIP_OP_GT: return c > 0;
    case KHIP_OP_GE: return c >= 0;
    case KHIP_OP_LT: return c < 0;
    case KHIP_OP_LE: return c <= 0;
    case KHIP_OP_EQ: return c == 0;
    case KHIP_OP_NE: return c != 0;
  }
  return false;
}


// kernels shared by the engines (defined in khip_agg.hip)
__global__ void k_blockmax(const int64_t* __restrict__ ts, const uint8_t* __restrict__ kv,
                           const uint8_t* __restrict__ rv, int64_t n, int64_t* __restrict__ blockmax,
                           const int64_t* __restrict__ st_at);
__global__ void k_scan_blocks(const int64_t* __restrict__ blockmax, int64_t nb, int64_t* __restrict__ prefix,
                              int64_t* __restrict__ stream_time);
__global__ void k_scan_excl(int64_t* __restrict__ v, int64_t n, int64_t* __restrict__ total);
__global__ void k_compact(const uint64_t* __restrict__ table, int64_t cap, int sw, HavingDev h,
                          uint64_t* __restrict__ out, int64_t max_rows, unsigned long long* __restrict__ counter);

// partitioned-engine column prefix kernels (khip_agg_part.hip; also used by khip_shuffle.hip)
__global__ void k_part_colsum(const uint32_t* __restrict__ hist, int64_t nT, int P, int TC, int64_t* __restrict__ csum);
__global__ void k_part_colbase(int64_t* __restrict__ csum, int P, int TC, int64_t* __restrict__ R);
__global__ void k_part_colprefix(uint32_t* __restrict__ hist, int64_t nT, int P, int TC,
                                 const int64_t* __restrict__ csum, const int64_t* __restrict__ pbase, int pstride);

struct InitWords {
  int64_t w[32];
};

// Partitioned engine state (khip_agg_part.hip).
struct PartState {
  int64_t P = 0;          // partitions (power of two), partition = top bits of mix64(key)
  int log2P = 0;
  int64_t cmax = 0;       // region capacity (rows) per partition and buffer
  int H = 0;              // LDS hash entries per workgroup
  int H_eff = 0;          // max groups placed in LDS before the partition is retried
  int nwords = 3;         // u64 words per group actually used (key, ws, rowtime, state)
  int lds_bytes = 0;
  DevBuf pbase, R, ctr, counts;
  DevBuf buf[2];          // region storage: P x cmax rows x sw words, double buffered
  DevBuf sel, cnt, newcnt, fail;  // per partition: buffer select, rows, rows being written, flags
  DevBuf hist, tilemax, tilemin, tileprefix, tpart, scan_tmp;
  DevBuf tilekr;  // per tile: largest key, ~smallest key (R8 records)
  // scattered records, AoS, rw u64 words each: key, ts (-1 = no window applied),
  // [meta = jlo | validity << 16, if meta_word = 2], [the referenced value columns], pad to even
  DevBuf srec;
  int rw = 2, meta_word = -1;
  uint32_t vcols = 0;
  int8_t col_word[MAX_COLS] = {-1, -1, -1, -1, -1, -1, -1, -1};
  std::vector<uint8_t> psbits;  // learned sub-pass bits per partition (pass 0 starts there)
  DevBuf work;            // retry work items
  int64_t scat_cap = 0;
  // closed windows (ws + size <= streamTime - grace): never updated again, moved out of the
  // partition regions into an append-only store so the live table stays LDS-sized
  DevBuf closed, closed_ctr;
  DevBuf closed2, pctr;   // the retention purge's second closed store and its counters (kept: no
                          // allocation per push)
  int64_t closed_cap = 0, closed_n = 0;
  // identity-CAS mode: wr = [window-index base, enabled] of the current push; res = window-
  // index range of the resident rows (conservative); res_fresh = no resident rows yet
  DevBuf wr, res;
  bool res_fresh = true;
  // two-level scatter: pass-A records, per-tile bucket histogram / offsets, bucket scans
  DevBuf srecA, hcoarse, scan_tmpB, RB;
  // k_part_merge (delta-only LDS): entries, LDS bytes, plane layout (khip_agg_part.hip)
  int mH = 0, m_lds = 0, rt_off = 0, m_list_off = 0, n_cu = 256;
  int flag_off = 0;       // k_part_agg: LDS byte offset of the changelog flag plane
  int64_t purged_to = INT64_MIN;  // closed store: expired rows (ws < purged_to) already dropped
  int32_t plane_off[MAX_OPS] = {};
  int8_t plane_w64[MAX_OPS] = {};
  int8_t word_op[32] = {};
  // the query's HAVING maintained on the device: rows passing it per partition (hcnt; hnew =
  // being written this push), their sum (ctr[11]) and the closed store's (ctr[12]); having_total
  // = both, as of the last push.  hvalid = false once a push took a path that does not maintain
  // them (fallback kernel, split) until the next reset.
  DevBuf hcnt, hnew;
  int64_t having_total = 0;
  bool hvalid = true;
  HostBuf pinfo;  // pinned: push info (window range, event-time span) and end-of-push stats
  // COUNT(*) pipeline (khip_agg_c1.hip): bucket bases, the
  // refine's per-chunk partition offsets, records of each partition in the last push (prn), and
  // whether the last push took that pipeline (k_part_chg then reads prn instead of pbase)
  DevBuf c1bb, c1seg, c1info, prn;
  DevBuf c1rc, c1rp, c1ro, c1scan, c1ci;  // step-run layout: [bucket][step] counts, their scan, step
                                          // offsets; per refine chunk its first step and run count
  int64_t c1_kbase = 0;             // key base for the next push's records (valid when c1_kb_valid)
  bool c1_kb_valid = false, c1_kretry = false;
  int64_t c1_wide_n = 0;            // pushes with wide records (compact ones are tried every 64th)
  std::vector<uint8_t> c1psbits;    // the pipelines' sub-pass bits per partition (their own LDS tables)
  int64_t c1ps_hmax = 0, hint_groups = 1024;
  bool last_c1 = false;
  int c1_skip = 0;  // pushes left before the pipeline is tried again after a declined push
  DevBuf c1vq;  // the value pipeline's merge parameters (device copy)
  HostBuf c1vq_h;  // their pinned staging, one slot per identity width (a pageable source would
                   // make the copy wait for the stream: a ~20 us bubble before every merge)
  bool c1_wide = false;  // the pipeline's record format for the next push (key range past 32 bits)
};

// SESSION engine state (khip_agg_session.hip): the session store sorted by (key, start) and
// the per-push scratch.
// Table-aggregation state (khip_agg_table.hip, engine 3): the source table's current rows by
// PRIMARY KEY id, HBM open addressing, TS_WORDS + n_cols u64 per slot (see the file header).
struct TaggState {
  DevBuf src;           // source-table slots
  int64_t src_cap = 0, src_occ = 0;
  int src_sw = 8;
  int key_type = -1;    // source PRIMARY KEY type (fixed by the first push)
  bool dense = false;   // source slots by id − dbase (khip_agg_table.hip src_prepare), else hashed
  int64_t dbase = 0;
  KeyDict dict;         // UTF8 PRIMARY KEYs → ids
  DevBuf sid, skey, skey2, sidx, sidx2, rec, tmp, tmp2, ctr, claimed, gclaimed, blk, st_koff, st_kbytes, st_kv, st_key, shash;
};

struct SessState {
  DevBuf rows, rows2;  // store (n rows) and the next push's output
  int64_t n = 0;
  DevBuf skey, sidx, skey2, sidx2, st_after, ukeys, ucnt, nseg, useg, s0, cap, scap, fin, fin_pre;
  DevBuf srow, sfl, trow, crow, ctomb, keep, keep_pre, ctr, tmp, tmp2, gath, blockkr;
  int64_t nchg = 0;    // changelog rows of the last push (crow / ctomb)
};

}  // namespace khip

using namespace khip;

struct khip_agg {
  khip_agg_desc desc{};
  std::vector<int32_t> col_types;
  std::vector<khip_agg_spec> aggs;
  int device = 0;
  hipStream_t stream = nullptr;
  int64_t grace = 0;
  int windowed = 0;
  int max_fanout = 1;
  ApplyParams ap{};
  InitWords init{};
  std::vector<AggOut> outs;
  int sw = 4;
  // table
  DevBuf table;
  int64_t cap = 0;
  int64_t occ = 0;  // resident groups
  // per-batch scratch
  DevBuf blockmax, blockprefix, partials, resume, counters, stream_time;
  DevBuf st_keys, st_ts, st_kv, st_rv, st_koff, st_kbytes;  // host staging copies
  DevBuf st_cols[MAX_COLS], st_cval[MAX_COLS];
  DevBuf kid, khash;  // UTF8
  int64_t resume_n = 0;
  // UTF8 dictionary
  KeyDict dict;
  int64_t host_stream_time = -1;
  // profiling (KHIP_FLAG_PROFILE)
  bool profile = false;
  hipEvent_t ev[8] = {};  // 0-4 atomic engine phases, 5-7 partitioned engine
  khip_kernel_times times{};
  int engine = 0;  // 0 partitioned (LDS-owned groups), 1 global-atomic, 2 SESSION store, 3 table source
                   // (the global-atomic table, updated by khip_agg_push_table)
  khip::HavingDev having{};  // the query's HAVING (desc.has_having), maintained by the merge kernel
  khip::PartState part;
  khip::SessState sess;     // engine 2 (SESSION windows)
  khip::TaggState tagg;     // engine 3 (table source: KHIP_FLAG_TABLE_SOURCE)
  // ---- retention and emission (include/ksqldb_hip.h khip_agg_changes)
  int64_t retention = 0;     // windowed: RETENTION or size + grace
  bool changelog = false;    // KHIP_FLAG_CHANGELOG: keep the push's EMIT CHANGES rows
  int64_t st_before = -1;    // stream time before the last push
  DevBuf chg;                // partitioned engine: per row slot (P x cmax) emission flags, see CHG_*
  DevBuf lostbuf, lostctr;   // EMIT FINAL: expired-at-close ws ranges found by the last push
  int64_t lost_cap = 0;
  std::vector<int64_t> lost; // sorted [lo, hi] pairs of the last push
  // KHIP_TIME_SUPPLIED (khip_agg_supplied_close, ABI 8): the GLOBAL stream time around the next
  // push and the union of the ranks' lost ranges, consumed by that push
  bool sup_set = false;
  int64_t sup_before = -1, sup_after = -1;
  std::vector<int64_t> sup_lost;
  bool chg_ready = false;    // changes of the last push computed (rows / tombstones below)
  std::vector<uint64_t> chg_rows;
  std::vector<uint8_t> chg_tomb;
  int64_t chg_n = 0;
  // ---- stream-time domains (ABI 5, khip_stream_time.hip): per-partition stream times (pst,
  // pst2 = the next batch's), the push's per-row stream time, scan scratch, staged partition ids
  DevBuf pst, pst2, st_col, st_agg, st_seen, st_part;
  // KHIP_TIME_PARTITION, windowed: per-task retention and EMIT FINAL (khip_stream_time.hip).  The
  // key map (key → partition, pm_key / pm_part), its capacity (power of two) and keys; host copies
  // of the partitions' stream times after / before the last push; the last push's lost ws ranges
  // per partition (EMIT FINAL: plost pairs, plost_off[P + 1]); pdom: the per-partition bounds of
  // one compaction (device)
  // pm_ts: each key's latest record time (ts >= 0; 0 = none), by which keys whose windows have
  // all expired leave the map (pmap_prune); pm_pruned: some have, so a row whose key is not in the
  // map is an expired one
  DevBuf pm_key, pm_part, pm_ts, pm_ctr, pdom;
  int64_t pm_cap = 0, pm_occ = 0, pm_last = -1;
  bool pm_pruned = false;
  std::vector<int64_t> pst_host, pst_prev_host, plost, plost_off;
};

// Emission flags of a row written by the last push (khip_agg::chg): touched by one of its
// records, HAVING held before the push, HAVING holds now (no HAVING: both set).
constexpr uint8_t CHG_TOUCHED = 1, CHG_OLD = 2, CHG_NEW = 4;

inline void ev_record(khip_agg* a, int i) {
  if (a->profile) (void)hipEventRecord(a->ev[i], a->stream);
}
inline double ev_ms(khip_agg* a, int i, int j) {
  float ms = 0.f;
  if (a->profile) (void)hipEventElapsedTime(&ms, a->ev[i], a->ev[j]);
  return (double)ms;
}
inline void ev_record_part(khip_agg* a, int i) { ev_record(a, 3 + i); }

namespace khip {
khip_status part_init(khip_agg* a, int64_t hint);
void part_release(khip_agg* a);
khip_status part_reset(khip_agg* a);
// st_at: per-row stream time (ABI 5 domains other than TASK), or null (computed per handle)
khip_status part_push(khip_agg* a, int64_t n, const int64_t* keys, const int64_t* ts, const uint8_t* kv,
                      const uint8_t* rv, const ColPtrs& cols, int64_t* tot, const int64_t* st_at);
// Shuffled rows as the input (khip_agg_push_shuffled): khip_shuffle_pack's row layout, rw words
// per row — [key][ts][columns except the key column][validity bits] — the argument in word
// vword, its validity in bit vbit of the last word.  Every row has a key, a row and ts >= 0.
struct RowsIn {
  const uint64_t* rows;
  int32_t rw, vword, vbit;
};
void shuffle_layout(const khip_shuffle* s, int* key_col, int* n_cols, const int32_t** types);
khip_status part_push_rows(khip_agg* a, int64_t n, const RowsIn& ri, int key_col, int64_t* tot, bool* done,
                           bool supplied);
// KHIP_TIME_PARTITION, windowed (khip_stream_time.hip): record every accepted row's key → partition
// (KHIP_E_INVALID when a key arrives on two partitions); EMIT FINAL's lost ws ranges per partition
// from the push's per-row stream time (st) — collected into a->plost by partition_lost_finish;
// the per-partition bounds of a compaction (retention: h.vis; EMIT FINAL: h.fin) attached to h.
khip_status pmap_insert(khip_agg* a, const int64_t* keys, const uint8_t* kv, const uint8_t* rv, const int64_t* ts,
                        const int32_t* part, int64_t n);
khip_status partition_lost(khip_agg* a, const int64_t* ts, const uint8_t* kv, const uint8_t* rv, const int32_t* part,
                           const int64_t* st, int64_t n);
khip_status partition_lost_finish(khip_agg* a);
khip_status partition_bounds(khip_agg* a, HavingDev& h);
int64_t partition_vis_from(const khip_agg* a, int64_t pst);
khip_status pmap_clear(khip_agg* a);
void pmap_release(khip_agg* a);
khip_status part_compact(khip_agg* a, const HavingDev& h, std::vector<uint64_t>* rows, int64_t* count);
bool part_having_count(khip_agg* a, int64_t* n);
khip_status part_changes(khip_agg* a, std::vector<uint64_t>* rows, std::vector<uint8_t>* tomb, int64_t* count);
khip_status part_purge_closed(khip_agg* a, const HavingDev& vis);
khip_status sess_push(khip_agg* a, int64_t n, const int64_t* keys, const int64_t* ts, const uint8_t* kv,
                      const uint8_t* rv, const ColPtrs& cols, int64_t* tot, const int64_t* st_at);
khip_status sess_changes(khip_agg* a, std::vector<uint64_t>* rows, std::vector<uint8_t>* tomb, int64_t* count);
void sess_release(khip_agg* a);
// table source (khip_agg_table.hip): batch rows (group ids, group-key hashes, group validity kv,
// tombstones rv, ts, argument columns) + device source PRIMARY KEY ids / validity
khip_status tagg_push(khip_agg* a, int64_t n, const int64_t* gkeys, const int64_t* ghash, const uint8_t* kv,
                      const uint8_t* rv, const int64_t* ts, const ColPtrs& cols, const int64_t* src_id,
                      const uint8_t* src_kv, int64_t* tot);
void tagg_release(khip_agg* a);
khip_status tagg_reset(khip_agg* a);
// the global-atomic table (khip_agg.hip), shared with engine 3
khip_status agg_grow_table(khip_agg* a, int64_t new_cap);
__global__ void k_finalize(uint64_t* __restrict__ table, int64_t cap, int sw, const int64_t* __restrict__ keys,
                           const int64_t* __restrict__ ts, int windowed, int64_t size, int64_t adv);
// the first visible window start after the last push (INT64_MIN: nothing expired)
int64_t visible_from(const khip_agg* a);
khip_status emit_final_lost(khip_agg* a, const int64_t* ts, const uint8_t* kv, const uint8_t* rv, int64_t n,
                            int64_t tile, const int64_t* tile_prefix);
// khip_stream_time.hip: the per-row stream time column (one seeded segment, or the partition runs
// of `part` seeded with / updating a->pst), and the PARTITION domain's handle stream time
khip_status stream_time_column(khip_agg* a, const int64_t* ts, const uint8_t* kv, const uint8_t* rv,
                               const int32_t* part, int64_t n, int64_t seed, int64_t* st, int64_t* last);
khip_status stream_time_partition_min(khip_agg* a);
}  // namespace khip


