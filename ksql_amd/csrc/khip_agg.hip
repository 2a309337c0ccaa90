// khip_agg.hip — windowed / unwindowed GROUP BY aggregation on MI355X (gfx950).
//
// Replaces, for one query task, the Kafka Streams KStreamWindowAggregate /
// KStreamAggregate processor + RocksDB window store + KudafAggregator chain that
// KSPlanBuilder.visitStreamWindowedAggregate / visitStreamAggregate build
// (S/KSPlanBuilder.java:293-304, :144-155; S/StreamAggregateBuilder.java:156-222,
// :81-138).  Semantics: SURVEY.md §8.0, restated in oracle/oracle.c R1–R6.
//
// Data layout in HBM (one handle):
//   table   : cap slots (power of two) × slot_words u64, AoS, 32 or 64 B per slot so a
//             group is one cache line: [w0 key | claim ref][w1 windowStart | EMPTY]
//             [rowtime][state words ...].
//   state   : deduplicated per input column: non-null count, sum (i64 / f64 bits),
//             min / max as total-order int64 keys; one COUNT(*) word.
//   dict    : UTF8 keys only — open-addressing dictionary → stable key id
//             (= byte offset of the key's entry in an append-only arena).
//
// Per micro-batch (all on the handle's stream):
//   k_blockmax → k_scan_blocks : stream time before each 2048-record block
//                                (exclusive prefix max, carried across batches)
//   [UTF8] k_dict_probe → k_dict_commit → k_dict_resolve (khip_dict.hpp)
//   k_apply     : in-block prefix max → late test → window fan-out → find-or-claim the
//                 (key, ws) slot with one 64-bit CAS whose value references the batch
//                 row (no spin, no fence) → agent-scope atomics for the state
//   k_finalize  : turn this batch's claim references into resident (key, ws)
//   failures (probe budget exhausted) are resumed after a table doubling, exactly.
#include <algorithm>
#include <cstring>
#include <numeric>
#include <vector>

#include "khip_util.hpp"

#include "khip_agg_internal.hpp"

namespace khip {

// ------------------------------------------------------------------- kernels

__global__ __launch_bounds__(BLOCK) void k_blockmax(const int64_t* __restrict__ ts,
                                                    const uint8_t* __restrict__ kv,
                                                    const uint8_t* __restrict__ rv, int64_t n,
                                                    int64_t* __restrict__ blockmax,
                                                    const int64_t* __restrict__ st_at) {
  __shared__ int64_t lds[BLOCK / 64];
  const int64_t base = (int64_t)blockIdx.x * RPB;
  int64_t m = -1;
#pragma unroll
  for (int k = 0; k < ITEMS; k++) {
    const int64_t i = base + k * BLOCK + threadIdx.x;
    if (i < n && bit_get(kv, i) && bit_get(rv, i)) {
      // ABI 5 domains: the row's given stream time (an upper bound of its ts), else its ts
      const int64_t t = ts[i] < 0 ? -1 : (st_at ? st_at[i] : ts[i]);
      m = t > m ? t : m;
    }
  }
  int64_t tot;
  block_incl_max(m, lds, &tot);
  if (threadIdx.x == 0) blockmax[blockIdx.x] = tot;
}

// Exclusive prefix max over nb block maxima, seeded and updated with *stream_time.
__global__ __launch_bounds__(1024) void k_scan_blocks(const int64_t* __restrict__ blockmax,
                                                      int64_t nb, int64_t* __restrict__ prefix,
                                                      int64_t* __restrict__ stream_time) {
  __shared__ int64_t lds[1024 / 64];
  __shared__ int64_t incl_all[1024];
  int64_t carry = *stream_time;
  for (int64_t b0 = 0; b0 < nb; b0 += blockDim.x) {
    const int64_t b = b0 + threadIdx.x;
    const int64_t v = b < nb ? blockmax[b] : INT64_MIN;
    int64_t tot;
    const int64_t incl = block_incl_max(v, lds, &tot);
    incl_all[threadIdx.x] = incl;
    __syncthreads();
    const int64_t excl = threadIdx.x == 0 ? INT64_MIN : incl_all[threadIdx.x - 1];
    if (b < nb) prefix[b] = excl > carry ? excl : carry;
    carry = tot > carry ? tot : carry;
    __syncthreads();
  }
  if (threadIdx.x == 0) *stream_time = carry;
}

// EMIT FINAL (S/StreamAggregateBuilder.java:282-285, Kafka Streams EmitStrategy.onWindowClose):
// with the emission check after every record, a window is emitted by the record whose stream
// time first reaches ws + size + grace, unless the window store had already expired it there:
// the store's observed time is then floor(M / adv) * adv (M = that record's stream time), so
// the window is lost iff ws < floor(M / adv) * adv - retention.  That needs M to jump into a later
// advance bucket in one record.  Per record (arrival order, accepted rows only; prefix = stream
// time before each RPB block): a record that moves the stream time from Mp to M > Mp with
// floor(M / adv) > floor(Mp / adv) loses the window starts in
//   [Mp - size - grace + 1, min(M - size - grace, floor(M / adv) * adv - retention - 1)]
// (rounded to multiples of adv); non-empty ranges are appended to lost[] as (lo, hi) pairs.
__global__ __launch_bounds__(BLOCK) void k_emit_lost(const int64_t* __restrict__ ts, const uint8_t* __restrict__ kv,
                                                     const uint8_t* __restrict__ rv, int64_t n,
                                                     const int64_t* __restrict__ prefix, int64_t size, int64_t adv,
                                                     int64_t grace, int64_t retention, int64_t* __restrict__ lost,
                                                     int64_t cap, unsigned long long* __restrict__ ctr) {
  __shared__ int64_t lmax[BLOCK];
  const int64_t i0 = (int64_t)blockIdx.x * RPB + (int64_t)threadIdx.x * ITEMS;
  int64_t m = -1;
  for (int k = 0; k < ITEMS; k++) {
    const int64_t i = i0 + k;
    if (i < n && bit_get(kv, i) && bit_get(rv, i) && ts[i] > m) m = ts[i];
  }
  lmax[threadIdx.x] = m;
  __syncthreads();
  for (int off = 1; off < BLOCK; off <<= 1) {  // inclusive prefix max over the block's threads
    const int64_t y = threadIdx.x >= off ? lmax[threadIdx.x - off] : -1;
    __syncthreads();
    if (y > lmax[threadIdx.x]) lmax[threadIdx.x] = y;
    __syncthreads();
  }
  int64_t mp = prefix[blockIdx.x];
  if (threadIdx.x > 0 && lmax[threadIdx.x - 1] > mp) mp = lmax[threadIdx.x - 1];
  const int64_t sg = size + grace;
  for (int k = 0; k < ITEMS; k++) {
    const int64_t i = i0 + k;
    if (i >= n || !bit_get(kv, i) || !bit_get(rv, i)) continue;
    const int64_t t = ts[i];
    if (t <= mp) continue;
    const int64_t bp = mp < 0 ? -1 : mp / adv, b = t / adv;
    if (b > bp) {
      int64_t lo = mp - sg + 1;
      int64_t hi = t - sg;
      const int64_t exp_hi = b * adv - retention - 1;
      hi = hi < exp_hi ? hi : exp_hi;
      lo = lo < 0 ? 0 : lo;
      lo = (lo + adv - 1) / adv * adv;  // window starts are multiples of adv
      if (lo <= hi) {
        const unsigned long long slot = atomicAdd(ctr, 1ULL);
        if ((int64_t)slot < cap) {
          lost[2 * slot] = lo;
          lost[2 * slot + 1] = hi;
        }
      }
    }
    mp = t;
  }
}

// Find or claim the (key, ws) slot and apply the record's aggregate updates.
// Claim reference: bit63 | fp15 << 48 | window index j << 36 | batch row (36 bits).
__device__ __forceinline__ int upsert_apply(const ApplyParams& p, uint64_t* __restrict__ table,
                                             uint64_t mask, int64_t hkey, int64_t key, int64_t ws,
                                             int64_t j, int64_t row, int64_t t,
                                             const int64_t* __restrict__ keys,
                                             const int64_t* __restrict__ ts, const ColPtrs& cols) {
  const uint64_t h = group_hash(hkey, ws);
  const uint64_t fp = (h >> 49) & 0x7FFFULL;
  const uint64_t myref = (1ULL << 63) | (fp << 48) | ((uint64_t)j << 36) | (uint64_t)row;
  uint64_t slot = h & mask;
  const int sw = p.slot_words;
  for (int probe = 0; probe < MAX_PROBE; probe++) {
    uint64_t* s = table + slot * (uint64_t)sw;
    const int64_t w1 = (int64_t)s[1];
    bool hit = false;
    int isnew = 0;
    if (w1 != EMPTY_WS) {
      hit = (w1 == ws) && ((int64_t)s[0] == key);
    } else {
      uint64_t w0 = ld_relaxed(s);
      if (w0 == 0) {
        const uint64_t old = atomicCAS((unsigned long long*)s, 0ULL, (unsigned long long)myref);
        if (old == 0) {
          hit = true;
          isnew = 1;
        } else {
          w0 = old;
        }
      }
      if (!hit && ((w0 >> 48) & 0x7FFFULL) == fp) {
        const int64_t idx = (int64_t)(w0 & ((1ULL << 36) - 1));
        const int64_t jj = (int64_t)((w0 >> 36) & 0xFFFULL);
        if (keys[idx] == key) {
          const int64_t ws2 = p.windowed ? first_window_start(ts[idx], p.size, p.adv) + jj * p.adv : 0;
          hit = ws2 == ws;
        }
      }
    }
    if (hit) {
      __hip_atomic_fetch_max((int64_t*)&s[2], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int o = 0; o < p.n_ops; o++) {
        const UpdOp op = p.ops[o];
        int64_t* w = (int64_t*)&s[op.word];
        if (op.kind == OP_INC) {
          __hip_atomic_fetch_add(w, (int64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          continue;
        }
        if (!bit_get(cols.valid[op.col], row)) continue;
        const int32_t ty = p.col_type[op.col];
        switch (op.kind) {
          case OP_INC_VALID:
            __hip_atomic_fetch_add(w, (int64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          case OP_ADD_I64:
            __hip_atomic_fetch_add((uint64_t*)w, (uint64_t)load_col_raw(cols, ty, op.col, row),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          case OP_ADD_F64: {
            const double v = ((const double*)cols.data[op.col])[row];
            unsafeAtomicAdd((double*)w, v);
            break;
          }
          case OP_MIN:
          case OP_MAX: {
            int64_t k = load_col_raw(cols, ty, op.col, row);
            if (ty == KHIP_TYPE_DOUBLE) {
              double d;
              __builtin_memcpy(&d, &k, 8);
              k = f64_order_key(d);
            }
            if (op.kind == OP_MIN)
              __hip_atomic_fetch_min(w, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
              __hip_atomic_fetch_max(w, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          default:
            break;
        }
      }
      return 1 + isnew;
    }
    slot = (slot + 1) & mask;
  }
  return 0;
}

__global__ __launch_bounds__(BLOCK) void k_apply(ApplyParams p, const int64_t* __restrict__ hkeys,
                                                 const int64_t* __restrict__ keys,
                                                 const int64_t* __restrict__ ts,
                                                 const uint8_t* __restrict__ kv,
                                                 const uint8_t* __restrict__ rv, ColPtrs cols,
                                                 const int64_t* __restrict__ blockprefix, int64_t n,
                                                 uint64_t* __restrict__ table, uint64_t mask,
                                                 int32_t* __restrict__ resume,
                                                 int64_t* __restrict__ partials, int resume_mode,
                                                 const int64_t* __restrict__ st_at) {
  __shared__ int64_t lds_scan[BLOCK / 64];
  __shared__ unsigned long long lds_cnt[NPART];
  if (threadIdx.x < NPART) lds_cnt[threadIdx.x] = 0;
  int64_t cnt[NPART];
#pragma unroll
  for (int k = 0; k < NPART; k++) cnt[k] = 0;
  const int64_t base = (int64_t)blockIdx.x * RPB;
  int64_t carry = blockprefix[blockIdx.x];
  for (int k = 0; k < ITEMS; k++) {
    const int64_t i = base + k * BLOCK + threadIdx.x;
    const bool in = i < n;
    const int64_t t = in ? ts[i] : -1;
    const bool kval = in && bit_get(kv, i);
    const bool rval = in && bit_get(rv, i);
    const bool valid = kval && rval && t >= 0;
    int64_t tot;
    const int64_t incl = block_incl_max(valid ? t : -1, lds_scan, &tot);
    int64_t st = incl > carry ? incl : carry;  // stream time after this record
    carry = tot > carry ? tot : carry;
    if (!in) continue;
    if (st_at) st = st_at[i];  // ABI 5 domains: given per row
    int64_t j0 = 0;
    if (resume_mode) {
      j0 = resume[i];
      if (j0 < 0) continue;
      resume[i] = -1;
    } else {
      if (!kval) { cnt[P_NULL_KEY]++; continue; }
      if (!rval) { cnt[P_NULL_ROW]++; continue; }
      if (t < 0) { cnt[P_BAD_TS]++; continue; }
      cnt[P_ACCEPTED]++;
    }
    const int64_t key = keys[i];
    const int64_t hkey = hkeys[i];
    if (p.windowed) {
      const int64_t close = st - p.grace;
      const int64_t ws0 = first_window_start(t, p.size, p.adv);
      int64_t j = j0;
      for (int64_t ws = ws0 + j0 * p.adv; ws <= t; ws += p.adv, j++) {
        if (ws + p.size <= close) {  // window closed: late
          cnt[P_LATE]++;
          continue;
        }
        const int r = upsert_apply(p, table, mask, hkey, key, ws, j, i, t, keys, ts, cols);
        if (r == 0) {
          resume[i] = (int32_t)j;
          cnt[P_FAILED]++;
          break;
        }
        cnt[P_APPLIED]++;
        cnt[P_NEW] += r - 1;
      }
    } else {
      const int r = upsert_apply(p, table, mask, hkey, key, 0, 0, i, t, keys, ts, cols);
      if (r == 0) {
        resume[i] = 0;
        cnt[P_FAILED]++;
      } else {
        cnt[P_APPLIED]++;
        cnt[P_NEW] += r - 1;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NPART; k++) {
    const int64_t s = wave_sum(cnt[k]);
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(&lds_cnt[k], (unsigned long long)s);
  }
  __syncthreads();
  if (threadIdx.x < NPART) partials[(int64_t)blockIdx.x * NPART + threadIdx.x] = (int64_t)lds_cnt[threadIdx.x];
}

// Claim references of this batch → resident (key, ws).
__global__ __launch_bounds__(256) void k_finalize(uint64_t* __restrict__ table, int64_t cap, int sw,
                                                  const int64_t* __restrict__ keys,
                                                  const int64_t* __restrict__ ts, int windowed,
                                                  int64_t size, int64_t adv) {
  for (int64_t slot = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; slot < cap;
       slot += (int64_t)gridDim.x * blockDim.x) {
    uint64_t* s = table + slot * (uint64_t)sw;
    if ((int64_t)s[1] != EMPTY_WS) continue;
    const uint64_t w0 = s[0];
    if (w0 == 0) continue;
    const int64_t idx = (int64_t)(w0 & ((1ULL << 36) - 1));
    const int64_t jj = (int64_t)((w0 >> 36) & 0xFFFULL);
    s[0] = (uint64_t)keys[idx];
    s[1] = (uint64_t)(windowed ? first_window_start(ts[idx], size, adv) + jj * adv : 0);
  }
}

__global__ __launch_bounds__(256) void k_init_table(uint64_t* __restrict__ table, int64_t cap, int sw,
                                                    InitWords init) {
  const int64_t total = cap * sw;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x)
    table[e] = (uint64_t)init.w[e & (sw - 1)];
}

// Sum nb rows of K partial counters into out[K] (accumulating).
__global__ __launch_bounds__(256) void k_reduce_partials(const int64_t* __restrict__ partials, int64_t nb,
                                                         int K, int64_t* __restrict__ out) {
  __shared__ unsigned long long acc[NPART];
  if (threadIdx.x < NPART) acc[threadIdx.x] = 0;
  __syncthreads();
  for (int k = 0; k < K; k++) {
    int64_t s = 0;
    for (int64_t b = threadIdx.x; b < nb; b += blockDim.x) s += partials[b * K + k];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) atomicAdd(&acc[k], (unsigned long long)s);
  }
  __syncthreads();
  if (threadIdx.x < K) out[threadIdx.x] += (int64_t)acc[threadIdx.x];
}

// Re-insert resident slots into a larger table.
__global__ __launch_bounds__(256) void k_rehash(const uint64_t* __restrict__ old, int64_t oldcap,
                                                uint64_t* __restrict__ nt, uint64_t nmask, int sw,
                                                int utf8, const uint8_t* __restrict__ arena) {
  for (int64_t slot = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; slot < oldcap;
       slot += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t* s = old + slot * (uint64_t)sw;
    const int64_t ws = (int64_t)s[1];
    if (ws == EMPTY_WS) continue;
    const int64_t key = (int64_t)s[0];
    // (a UTF8 group's hash key: its key hash, or an inline id itself — as k_dict_probe's khash)
    const int64_t hkey = utf8 && !kid_inline(key) ? *(const int64_t*)(arena + key) : key;
    uint64_t d = group_hash(hkey, ws) & nmask;
    while (true) {
      uint64_t* q = nt + d * (uint64_t)sw;
      if (atomicCAS((unsigned long long*)&q[1], (unsigned long long)EMPTY_WS, (unsigned long long)ws) ==
          (unsigned long long)EMPTY_WS) {
        q[0] = (uint64_t)key;
        for (int w = 2; w < sw; w++) q[w] = s[w];
        break;
      }
      d = (d + 1) & nmask;
    }
  }
}

// Compact resident slots passing HAVING into `out` (sw words per row); out may be null
// (count only).  One atomic per block reserves the output range.
__global__ __launch_bounds__(256) void k_compact(const uint64_t* __restrict__ table, int64_t cap, int sw,
                                                 HavingDev h, uint64_t* __restrict__ out, int64_t max_rows,
                                                 unsigned long long* __restrict__ counter) {
  __shared__ int lds_n[256 / 64];
  __shared__ unsigned long long lds_base;
  for (int64_t s0 = (int64_t)blockIdx.x * blockDim.x; s0 < cap; s0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t slot = s0 + threadIdx.x;
    const uint64_t* s = table + slot * (uint64_t)sw;
    const bool take = slot < cap && (int64_t)s[1] != EMPTY_WS && having_ok(s, h);
    const uint64_t bal = __ballot(take);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int before = __popcll(bal & ((1ULL << lane) - 1));
    if (lane == 0) lds_n[wave] = __popcll(bal);
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); w++) {
      if (w < wave) off += lds_n[w];
      tot += lds_n[w];
    }
    if (threadIdx.x == 0) lds_base = tot ? atomicAdd(counter, (unsigned long long)tot) : 0;
    __syncthreads();
    if (take && out && (int64_t)(lds_base + off + before) < max_rows) {
      uint64_t* o = out + (lds_base + off + before) * (uint64_t)sw;
      for (int w = 0; w < sw; w++) o[w] = s[w];
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- UTF8 dictionary (khip_dict.hpp)
// Slot (32 B, one random access): w0 dict word: 0 empty | fresh: bit63 | fp22 << 40 | batch row
// (40 bits) | resident: bit62 | fp22 << 40 | o / 8 (40 bits); w1 = o | min(len, 0xFFFF) << 48 (the
// key's id = its arena offset o, and its length); w2, w3 = the key's first 16 bytes as words
// (keys of up to 16 bytes compare there; longer ones against the arena entry).  Arena entry at o
// (8-aligned): [u64 hash][i64 len][bytes, padded to 8].  A map is three passes, none over the
// whole table:
//   k_dict_probe    per row: hash, probe; a resident slot compares in place; an empty slot is
//                   claimed (fresh word naming the row; the slot and its arena entry's place go to
//                   one of DICT_NL claim lists, one block-aggregated append); a fresh slot of the same fingerprint, claimed by
//                   another row of this batch, leaves the row PENDING on it
//   k_dict_commit   per claim: the arena entry (its list's base + its place in the list), the slot
//                   made resident with the key's words, the claiming row's id (no atomics)
//   k_dict_resolve  per pending row: the (now resident) slot compares; a different key of the same
//                   fingerprint goes on a retry list (probed again: the slot no longer misleads it)
// A probe gives up after DICT_PROBE slots (the table is then too full: dict_map unclaims the
// batch's fresh words, grows the table and maps the batch again).
constexpr int DICT_PROBE = 256;
constexpr uint64_t DICT_LOW = (1ULL << 40) - 1;
constexpr int DICT_NL = 1024;  // claim lists (one per block residue: no hot append word)
constexpr int64_t KID_PEND = (int64_t)1 << 62;
constexpr uint64_t DICT_ID = (1ULL << 48) - 1;

__device__ __forceinline__ int64_t entry_bytes(int64_t len) { return 16 + ((len + 7) & ~7LL); }

#ifdef KHIP_TUNING
// Tuning build: KHIP_DICT_HASHMASK keeps only these bits of every key hash (different keys then
// share whole hashes, not just fingerprints: tests/test_gpu_dict.py); KHIP_KEY_INLINE=0 sends the
// digit keys through the dictionary too.
__constant__ uint64_t g_dict_hmask = ~0ULL;
__constant__ int g_key_inline = 1;
#endif

// The key of batch row i: words (short keys), hash.
struct DKey {
  uint64_t kw[KW_MAX];
  uint64_t h;
  int64_t len;
  const uint8_t* kb;
  bool sk;
};
__device__ __forceinline__ void dkey_words(DKey& k, const int64_t* __restrict__ koff, const uint8_t* __restrict__ kbytes,
                                           int64_t i) {
  const int64_t o0 = koff[i];
  k.len = koff[i + 1] - o0;
  k.kb = kbytes + o0;
  k.sk = k.len <= 8 * KW_MAX;
  if (k.sk) key_words(k.kb, k.len, k.kw);
}
__device__ __forceinline__ void dkey_hash(DKey& k) {
  k.h = k.sk ? hash_key_words(k.kw, k.len) : hash_bytes_dev(k.kb, k.len);
#ifdef KHIP_TUNING
  k.h &= g_dict_hmask;
#endif
}
__device__ __forceinline__ void dkey_load(DKey& k, const int64_t* __restrict__ koff, const uint8_t* __restrict__ kbytes,
                                          int64_t i) {
  dkey_words(k, koff, kbytes, i);
  dkey_hash(k);
}

// Key k's inline id (khip_dict.hpp), when it is 0..17 ASCII digits.
__device__ __forceinline__ bool key_inline(const DKey& k, int64_t* code) {
#ifdef KHIP_TUNING
  if (!g_key_inline) return false;
#endif
  static_assert(KW_MAX == 3, "inline keys are read from three key words");
  return k.sk && inline_id_words(k.kw, k.len, code);
}

// A resident slot (w0 fingerprint already matched) holds key k?
__device__ __forceinline__ bool dslot_eq(const ulonglong2& a, const ulonglong2& b, const DKey& k,
                                         const uint8_t* __restrict__ arena) {
  const int64_t slen = (int64_t)(a.y >> 48);
  if (k.len <= 16) return slen == k.len && b.x == k.kw[0] && b.y == (k.len > 8 ? k.kw[1] : 0ULL);
  if (slen != (k.len < 0xFFFF ? k.len : 0xFFFF)) return false;
  const int64_t o = (int64_t)(a.y & DICT_ID);
  if (*(const uint64_t*)(arena + o) != k.h || *(const int64_t*)(arena + o + 8) != k.len) return false;
  return k.sk ? key_words_eq_aligned(k.kw, arena + o + 16, k.len) : bytes_eq_aligned(arena + o + 16, k.kb, k.len);
}

// rows: null (row j = j) or a row list (the retry pass).  lists: DICT_NL regions of lcap entries
// [slot | the entry's byte offset in its list << 34]; lw[L]: entries << 40 | entry bytes of list L.
// nd[0] += the rows that probed (valid, not inline), nd[1] += the rows left pending (counted per
// wave by ballots, summed per block in LDS at the end: one global atomic per block).
__global__ __launch_bounds__(256) void k_dict_probe(ulonglong2* __restrict__ slots, uint64_t dmask,
                                                    const uint8_t* __restrict__ arena, const int64_t* __restrict__ koff,
                                                    const uint8_t* __restrict__ kbytes, const uint8_t* __restrict__ kv,
                                                    const uint8_t* __restrict__ rv, const int64_t* __restrict__ ts,
                                                    const int64_t* __restrict__ rows, int64_t n,
                                                    int64_t* __restrict__ kid, int64_t* __restrict__ khash,
                                                    uint64_t* __restrict__ lists, int64_t lcap,
                                                    unsigned long long* __restrict__ lw, int* __restrict__ fail,
                                                    uint64_t fpm, unsigned long long* __restrict__ nd) {
  __shared__ unsigned long long wsum[4];  // per wave: claims << 40 | entry bytes
  __shared__ unsigned long long bbase;
  __shared__ unsigned long long bsum[2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int L = blockIdx.x & (DICT_NL - 1);
  if (threadIdx.x < 2) bsum[threadIdx.x] = 0;
  unsigned long long bprobed = 0, bpend = 0;  // (the wave's counts over its tiles)
  for (int64_t j0 = blockIdx.x * (int64_t)blockDim.x; j0 < n; j0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = j0 + threadIdx.x;
    bool claimed = false, probed = false, pending = false;
    uint64_t cslot = 0, eb = 0;
    if (j < n) {
      const int64_t i = rows ? rows[j] : j;
      if (!(bit_get(kv, i) && bit_get(rv, i) && (ts == nullptr || ts[i] >= 0))) {
        kid[i] = 0;
        if (khash) khash[i] = 0;
      } else {
        DKey k;
        dkey_words(k, koff, kbytes, i);
        int64_t code;
        const bool inl = key_inline(k, &code);
        k.h = 0;
        if (!inl) dkey_hash(k);
        probed = !inl;
        if (khash) khash[i] = inl ? code : (int64_t)k.h;
        const uint64_t fp = (k.h >> 40) & fpm;
        const uint64_t fresh = (1ULL << 63) | (fp << 40) | (uint64_t)i;
        uint64_t slot = k.h & dmask;
        bool done = inl;
        if (inl) kid[i] = code;
        for (int probe = 0; probe < DICT_PROBE && !done; probe++) {
          ulonglong2 a = slots[2 * slot];  // a stale empty / fresh word is settled by the CAS below
          uint64_t w = a.x;
          if (w == 0) {
            const uint64_t old = atomicCAS((unsigned long long*)&slots[2 * slot].x, 0ULL, (unsigned long long)fresh);
            if (old == 0) {
              kid[i] = -(int64_t)(slot + 1);  // commit writes the id
              claimed = true;
              cslot = slot;
              eb = (uint64_t)entry_bytes(k.len);
              done = true;
              break;
            }
            w = old;
          }
          if (((w >> 40) & 0x3FFFFFULL) == fp) {
            if (w >> 63) {  // claimed by another row of this batch: resolved after the commit
              kid[i] = -(int64_t)(slot + 1) - KID_PEND;
              pending = true;
              done = true;
            } else {
              const ulonglong2 b = slots[2 * slot + 1];
              if (a.x != w) a = slots[2 * slot];  // (the word moved on since the first read)
              if (dslot_eq(a, b, k, arena)) {
                kid[i] = (int64_t)(a.y & DICT_ID);
                done = true;
              }
            }
          }
          if (!done) slot = (slot + 1) & dmask;
        }
        if (!done) {
          kid[i] = 0;
          *fail = 1;
        }
      }
    }
    bprobed += (unsigned long long)__popcll(__ballot(probed));
    bpend += (unsigned long long)__popcll(__ballot(pending));
    // the block's claims → list L: one atomic per block and tile for both the count and the bytes
    const uint64_t x = claimed ? ((1ULL << 40) | eb) : 0ULL;
    uint64_t incl = x;
    for (int off = 1; off < 64; off <<= 1) {
      const uint64_t y = __shfl_up(incl, off, 64);
      if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint64_t before = 0, tot = 0;
    for (int k = 0; k < 4; k++) {
      before += k < wave ? wsum[k] : 0;
      tot += wsum[k];
    }
    if (threadIdx.x == 0) bbase = tot ? atomicAdd(&lw[L], (unsigned long long)tot) : 0ULL;
    __syncthreads();
    if (claimed) {
      const uint64_t at = bbase + before + incl - x;  // this claim's entries << 40 | bytes before it
      const uint64_t idx = at >> 40, boff = at & ((1ULL << 40) - 1);
      if ((int64_t)idx < lcap && boff < (1ULL << 30)) lists[(uint64_t)L * lcap + idx] = cslot | (boff << 34);
      else *fail = 2;  // (lcap covers every row a list's blocks can claim)
    }
  }
  __syncthreads();
  if (lane == 0 && bprobed) atomicAdd(&bsum[0], bprobed);
  if (lane == 0 && bpend) atomicAdd(&bsum[1], bpend);
  __syncthreads();
  if (threadIdx.x < 2 && bsum[threadIdx.x]) atomicAdd(&nd[threadIdx.x], bsum[threadIdx.x]);
}

// The inline ids of a batch, before any dictionary work: rows without a key get 0, inline keys
// their id (khash: the id), other keys KID_DICT; nd[0] += the rows left for the dictionary, nd[1]
// += the inline rows (one atomic per block each; ts is not read: a late row's id is never used).
// Branch-free loads, R rows per thread: every row's offsets, then every row's first four aligned
// key words (clamped to the words that hold its bytes, so no load leaves the key column; an empty
// key reads the word of the column's first byte, or nothing when the column is empty), then the
// SWAR check per row.
constexpr int64_t KID_DICT = INT64_MIN;
template <int R>
__global__ __launch_bounds__(256) void k_key_inline(const int64_t* __restrict__ koff, const uint8_t* __restrict__ kbytes,
                                                    const uint8_t* __restrict__ kv, const uint8_t* __restrict__ rv,
                                                    const int64_t* __restrict__ ts, int64_t n, int64_t* __restrict__ kid,
                                                    int64_t* __restrict__ khash, unsigned long long* __restrict__ nd) {
  (void)ts;
  const int64_t kfirst = koff[0];
  const bool has_bytes = koff[n] > kfirst;
  const uint8_t* anchor = kbytes + kfirst;  // (a byte of the column when has_bytes)
  __shared__ unsigned int bsum[2];
  if (threadIdx.x < 2) bsum[threadIdx.x] = 0;
  unsigned int cnt = 0, ninl = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j0 < n; j0 += stride * R) {
    int64_t o0[R], len[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int64_t i = j0 + r * stride < n ? j0 + r * stride : n - 1;
      o0[r] = koff[i];
      len[r] = koff[i + 1] - o0[r];
    }
    uint64_t A[R][KW_MAX + 1];
#pragma unroll
    for (int r = 0; r < R; r++) {
      const uint8_t* p = kbytes + o0[r];
      const int64_t lb = len[r] < 8 * KW_MAX ? len[r] : 8 * KW_MAX;  // (longer keys are never inline)
      const uint64_t a = (uint64_t)p;
      const uint64_t* base = (const uint64_t*)(p - (a & 7));
      const int last = lb > 0 ? (int)(((a & 7) + (uint64_t)lb - 1) >> 3) : 0;
      const uint64_t* b0 = lb > 0 ? base : (const uint64_t*)(anchor - ((uint64_t)anchor & 7));
#pragma unroll
      for (int k = 0; k <= KW_MAX; k++) A[r][k] = has_bytes ? b0[k < last ? k : last] : 0ULL;
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int64_t i = j0 + r * stride;
      if (i >= n) break;
      int64_t code = 0;
      if (bit_get(kv, i) && bit_get(rv, i)) {
        // key_words from the loaded aligned words
        const uint64_t a = (uint64_t)(kbytes + o0[r]);
        const int sh = (int)(a & 7) * 8;
        DKey k;
        k.len = len[r];
        k.sk = k.len <= 8 * KW_MAX;
#pragma unroll
        for (int q = 0; q < KW_MAX; q++) {
          uint64_t x = sh ? (A[r][q] >> sh) | (A[r][q + 1] << (64 - sh)) : A[r][q];
          const int64_t left = k.len - 8 * q;
          if (left <= 0) x = 0;
          else if (left < 8) x &= (1ULL << (8 * left)) - 1;
          k.kw[q] = x;
        }
        if (key_inline(k, &code)) {
          ninl++;
        } else {
          code = KID_DICT;
          cnt++;
        }
      }
      kid[i] = code;
      if (khash) khash[i] = code;
    }
  }
  __syncthreads();
  if (cnt) atomicAdd(&bsum[0], cnt);
  if (ninl) atomicAdd(&bsum[1], ninl);
  __syncthreads();
  if (threadIdx.x < 2 && bsum[threadIdx.x]) atomicAdd(&nd[threadIdx.x], (unsigned long long)bsum[threadIdx.x]);
}

// The lists' arena bases after a probe round (one block, a thread per list): lbase[L] = the arena's
// used bytes + the entry bytes of the lists before L; the used bytes and the key count advance.
// Nothing when the round failed (c's first word: the probe's failure flag).
__global__ __launch_bounds__(1024) void k_dict_bases(unsigned long long* __restrict__ c,
                                                     const unsigned long long* __restrict__ lw,
                                                     int64_t* __restrict__ lbase) {
  static_assert(DICT_NL == 1024, "a thread per list");
  __shared__ unsigned long long ws[16], wk[16];
  if (*(const volatile int*)c != 0) return;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const unsigned long long x = lw[t];
  const unsigned long long by = x & ((1ULL << 40) - 1), ke = x >> 40;
  unsigned long long incl = by, kin = ke;
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned long long y = __shfl_up(incl, off, 64), z = __shfl_up(kin, off, 64);
    if (lane >= off) {
      incl += y;
      kin += z;
    }
  }
  if (lane == 63) {
    ws[wave] = incl;
    wk[wave] = kin;
  }
  __syncthreads();
  unsigned long long before = 0, tot = 0, ktot = 0;
  for (int k = 0; k < 16; k++) {
    before += k < wave ? ws[k] : 0ULL;
    tot += ws[k];
    ktot += wk[k];
  }
  lbase[t] = (int64_t)(c[1] + before + incl - by);
  __syncthreads();  // (every thread has read c[1])
  if (t == 0) {
    c[1] += tot;
    c[2] += ktot;
  }
}

// One thread per claim (list L, entries t, t + stride, ...): the arena entry at its list's base +
// its byte offset, the slot made resident with the key's words, the claiming row's id.  lbase[L]:
// the list's arena base.  Nothing when the round failed.
__global__ __launch_bounds__(256) void k_dict_commit(ulonglong2* __restrict__ slots, const uint64_t* __restrict__ lists,
                                                     int64_t lcap, const unsigned long long* __restrict__ lw,
                                                     const int64_t* __restrict__ lbase, uint8_t* __restrict__ arena,
                                                     const int64_t* __restrict__ koff, const uint8_t* __restrict__ kbytes,
                                                     int64_t* __restrict__ kid, const unsigned long long* __restrict__ c) {
  if (*(const volatile int*)c != 0) return;
  const int L = blockIdx.y;
  const int64_t cntL = (int64_t)(lw[L] >> 40);
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < cntL; t += (int64_t)gridDim.x * blockDim.x) {
  const uint64_t le = lists[(uint64_t)L * lcap + t];
  const uint64_t slot = le & ((1ULL << 34) - 1);
  const uint64_t w = slots[2 * slot].x;
  const int64_t r = (int64_t)(w & DICT_LOW);
  DKey k;
  dkey_load(k, koff, kbytes, r);
  const int64_t o = lbase[L] + (int64_t)(le >> 34);
  *(uint64_t*)(arena + o) = k.h;
  *(int64_t*)(arena + o + 8) = k.len;
  if (k.sk) {
    for (int q = 0; q < (int)((k.len + 7) >> 3); q++) ((uint64_t*)(arena + o + 16))[q] = k.kw[q];
  } else {
    for (int64_t b = 0; b < k.len; b++) arena[o + 16 + b] = k.kb[b];
  }
  const uint64_t fp = (w >> 40) & 0x3FFFFFULL;
  const uint64_t lenw = (uint64_t)(k.len < 0xFFFF ? k.len : 0xFFFF) << 48;
  slots[2 * slot + 1] = make_ulonglong2(k.len <= 16 ? k.kw[0] : 0ULL, k.len <= 16 && k.len > 8 ? k.kw[1] : 0ULL);
  slots[2 * slot] = make_ulonglong2((1ULL << 62) | (fp << 40) | ((uint64_t)o >> 3), (uint64_t)o | lenw);
  kid[r] = o;
  }
}

// Rows left pending on a slot another row claimed: the slot is resident now.  A different key of
// the same fingerprint goes on the retry list.
__global__ __launch_bounds__(256) void k_dict_resolve(const ulonglong2* __restrict__ slots,
                                                      const uint8_t* __restrict__ arena,
                                                      const int64_t* __restrict__ koff,
                                                      const uint8_t* __restrict__ kbytes, const int64_t* __restrict__ rows,
                                                      int64_t n, int64_t* __restrict__ kid,
                                                      int64_t* __restrict__ retry, unsigned long long* __restrict__ nretry,
                                                      const unsigned long long* __restrict__ c,
                                                      const unsigned long long* __restrict__ npend) {
  if (*(const volatile int*)c != 0 || *npend == 0) return;  // (a failed round, or no row pending)
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = rows ? rows[j] : j;
    const int64_t x = kid[i];
    if (x >= -KID_PEND) continue;  // an id, or the claimer's (written by the commit)
    const uint64_t slot = (uint64_t)(-(x + KID_PEND) - 1);
    DKey k;
    dkey_load(k, koff, kbytes, i);
    const ulonglong2 a = slots[2 * slot], b = slots[2 * slot + 1];
    if (dslot_eq(a, b, k, arena)) {
      kid[i] = (int64_t)(a.y & DICT_ID);
    } else {
      kid[i] = 0;
      retry[atomicAdd(nretry, 1ULL)] = i;
    }
  }
}

// Read-only dictionary probe (pull queries, join probes): key bytes → resident key id (arena
// offset), or -1 when the key was never seen.  Every slot is resident between maps.
__global__ __launch_bounds__(256) void k_dict_find(const ulonglong2* __restrict__ slots, uint64_t dmask,
                                                   const uint8_t* __restrict__ arena,
                                                   const int64_t* __restrict__ koff, const uint8_t* __restrict__ kbytes,
                                                   int64_t n, int64_t* __restrict__ kid, uint64_t fpm) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    DKey k;
    dkey_words(k, koff, kbytes, i);
    int64_t code;
    if (key_inline(k, &code)) {
      kid[i] = code;
      continue;
    }
    dkey_hash(k);
    const uint64_t fp = (k.h >> 40) & fpm;
    uint64_t slot = k.h & dmask;
    int64_t found = -1;
    for (int probe = 0; probe <= (int)dmask && probe < (1 << 20); probe++) {
      const ulonglong2 a = slots[2 * slot];
      if (a.x == 0) break;
      if (((a.x >> 40) & 0x3FFFFFULL) == fp && dslot_eq(a, slots[2 * slot + 1], k, arena)) {
        found = (int64_t)(a.y & DICT_ID);
        break;
      }
      slot = (slot + 1) & dmask;
    }
    kid[i] = found;
  }
}

// A failed map: the batch's fresh claims → empty (the table is as before the batch).
__global__ __launch_bounds__(256) void k_dict_unclaim(ulonglong2* __restrict__ slots, int64_t dcap) {
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < dcap; s += (int64_t)gridDim.x * blockDim.x)
    if (slots[2 * s].x >> 63) slots[2 * s] = make_ulonglong2(0ULL, 0ULL);
}

// Exclusive prefix sum of v[0..n) in place (single block); total added to *total.  Each thread
// owns 16 consecutive elements of a 16K-element chunk: one wave scan and one barrier per chunk.
__global__ __launch_bounds__(1024) void k_scan_excl(int64_t* __restrict__ v, int64_t n, int64_t* __restrict__ total) {
  __shared__ int64_t wsum[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t carry = 0;
  for (int64_t b0 = 0; b0 < n; b0 += 1024 * 16) {
    const int64_t base = b0 + (int64_t)threadIdx.x * 16;
    int64_t x[16], s = 0;
#pragma unroll
    for (int u = 0; u < 16; u++) {
      x[u] = base + u < n ? v[base + u] : 0;
      s += x[u];
    }
    int64_t incl = s;
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t y = __shfl_up(incl, off, 64);
      if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int64_t before = 0, tot = 0;
    for (int k = 0; k < 16; k++) {
      before += k < wave ? wsum[k] : 0;
      tot += wsum[k];
    }
    int64_t run = carry + before + incl - s;
#pragma unroll
    for (int u = 0; u < 16; u++) {
      if (base + u < n) v[base + u] = run;
      run += x[u];
    }
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total += carry;
}

__global__ __launch_bounds__(256) void k_dict_rehash(const ulonglong2* __restrict__ os, int64_t ocap,
                                                     ulonglong2* __restrict__ ns, uint64_t nmask,
                                                     const uint8_t* __restrict__ arena) {
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < ocap; s += (int64_t)gridDim.x * blockDim.x) {
    const ulonglong2 a = os[2 * s];
    if (a.x == 0) continue;
    const uint64_t h = *(const uint64_t*)(arena + (a.y & DICT_ID));
    uint64_t d = h & nmask;
    while (atomicCAS((unsigned long long*)&ns[2 * d].x, 0ULL, (unsigned long long)a.x) != 0ULL) d = (d + 1) & nmask;
    ns[2 * d + 1] = os[2 * s + 1];
    ns[2 * d].y = a.y;
  }
}

// ------------------------------------------------------------------- host side

static int grid_for(int64_t work, int per_block, int cap_blocks = 2048 * 8) {
  int64_t g = ceil_div(std::max<int64_t>(work, 1), per_block);
  return (int)std::min<int64_t>(g, cap_blocks);
}

// ---- KeyDict (khip_dict.hpp)

// The fingerprint bits a probe compares before the key (22; the tuning build's KHIP_DICT_FPMASK
// narrows them so that different keys meet on claimed slots: the pending / retry rounds).
static uint64_t dict_fp_mask() { return (uint64_t)knob("KHIP_DICT_FPMASK", 0x3FFFFF) & 0x3FFFFFULL; }

static khip_status dict_grow(KeyDict& d, hipStream_t s, int64_t new_cap) {
  DevBuf ns;
  KHIP_TRY(ns.ensure((size_t)new_cap * 32));
  KHIP_TRY_HIP(hipMemsetAsync(ns.p, 0, (size_t)new_cap * 32, s));
  if (d.dcap > 0 && d.docc > 0) {
    hipLaunchKernelGGL(k_dict_rehash, dim3(grid_for(d.dcap, 256)), dim3(256), 0, s, d.slots.as<ulonglong2>(), d.dcap,
                       ns.as<ulonglong2>(), (uint64_t)(new_cap - 1), d.arena.as<uint8_t>());
    KHIP_TRY_HIP(hipGetLastError());
  }
  KHIP_TRY_HIP(hipStreamSynchronize(s));
  d.slots.release();
  d.slots = std::move(ns);
  ns.p = nullptr;
  d.dcap = new_cap;
  return KHIP_OK;
}

khip_status dict_init(KeyDict& d, hipStream_t s) {
#ifdef KHIP_TUNING
  const uint64_t hm = (uint64_t)knob("KHIP_DICT_HASHMASK", -1);
  KHIP_TRY_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_dict_hmask), &hm, 8));
  const int inl = (int)knob("KHIP_KEY_INLINE", 1);
  KHIP_TRY_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_key_inline), &inl, 4));
#endif
  KHIP_TRY(d.ctr.ensure(64 + 16 * DICT_NL));  // (dict_round's counters)
  return dict_grow(d, s, 4096);
}

// One round over `rows` (null: every row): probe, commit the claims, resolve the pending rows.
// Returns the rows to retry (a different key behind a pending row's fingerprint) in d.retry,
// their count in *nretry; *failed when a probe ran out of budget (nothing committed then).
// Counters (d.ctr, u64): [0] probe failure | [1] arena bytes used | [2] keys added | [3] retries |
// [4 ..] DICT_NL list words | then DICT_NL list arena bases | rows probed | rows pending.
static khip_status dict_round(KeyDict& d, hipStream_t s, const int64_t* koff, const uint8_t* kbytes, const uint8_t* kv,
                              const uint8_t* rv, const int64_t* ts, const int64_t* rows, int64_t n, int64_t* kid,
                              int64_t* khash, int64_t* nretry, bool* failed) {
  unsigned long long* c = d.ctr.as<unsigned long long>();
  unsigned long long* lw = c + 4;
  int64_t* lbase = (int64_t*)(c + 4 + DICT_NL);
  unsigned long long* nd = c + 4 + 2 * DICT_NL;
  const int g = grid_for(n, 256);
  // a list takes the claims of blocks L, L + DICT_NL, ...: at most every row those blocks visit
  const int64_t lcap = ceil_div(g, DICT_NL) * 256 * ceil_div(n, 256LL * g);
  KHIP_TRY(d.lists.ensure((size_t)lcap * DICT_NL * 8));
  KHIP_TRY(d.retry.ensure((size_t)std::max<int64_t>(n, 1) * 8));
  KHIP_TRY_HIP(hipMemsetAsync(c, 0, 8, s));
  KHIP_TRY_HIP(hipMemsetAsync(c + 3, 0, 8 + 8 * DICT_NL, s));
  KHIP_TRY_HIP(hipMemsetAsync(nd, 0, 16, s));
  // probe → list bases → commit → resolve, with no host round trip in between: each later kernel
  // does nothing when the probe failed (the table is grown and the round mapped again)
  hipLaunchKernelGGL(k_dict_probe, dim3(g), dim3(256), 0, s, d.slots.as<ulonglong2>(), (uint64_t)(d.dcap - 1),
                     d.arena.as<uint8_t>(), koff, kbytes, kv, rv, ts, rows, n, kid, khash, d.lists.as<uint64_t>(), lcap,
                     lw, (int*)c, dict_fp_mask(), nd);
  hipLaunchKernelGGL(k_dict_bases, dim3(1), dim3(DICT_NL), 0, s, c, (const unsigned long long*)lw, lbase);
  hipLaunchKernelGGL(k_dict_commit, dim3((unsigned)std::min<int64_t>(4, ceil_div(lcap, 256LL)), DICT_NL), dim3(256), 0,
                     s, d.slots.as<ulonglong2>(), d.lists.as<uint64_t>(), lcap, lw, lbase, d.arena.as<uint8_t>(), koff,
                     kbytes, kid, (const unsigned long long*)c);
  hipLaunchKernelGGL(k_dict_resolve, dim3(g), dim3(256), 0, s, d.slots.as<ulonglong2>(), d.arena.as<uint8_t>(), koff,
                     kbytes, rows, n, kid, d.retry.as<int64_t>(), c + 3, (const unsigned long long*)c,
                     (const unsigned long long*)(nd + 1));
  KHIP_TRY_HIP(hipGetLastError());
  unsigned long long h[6];
  KHIP_TRY_HIP(hipMemcpyAsync(h, c, 32, hipMemcpyDeviceToHost, s));
  KHIP_TRY_HIP(hipMemcpyAsync(h + 4, nd, 16, hipMemcpyDeviceToHost, s));
  KHIP_TRY_HIP(hipStreamSynchronize(s));
  *failed = (h[0] & 0xFFFFFFFFULL) != 0;
  d.round_probed = (int64_t)h[4];
  if (!rows) d.last_probed = d.round_probed;  // (the first round sees every row)
  *nretry = *failed ? 0 : (int64_t)h[3];
  if (!*failed) {  // (cumulative over the map's rounds)
    d.round_used = (int64_t)h[1];
    d.round_keys = (int64_t)h[2];
  }
  return KHIP_OK;
}

khip_status dict_map(KeyDict& d, hipStream_t s, const int64_t* koff, const uint8_t* kbytes, int64_t key_bytes_total,
                     const uint8_t* kv, const uint8_t* rv, const int64_t* ts, int64_t n, int64_t* kid, int64_t* khash) {
  // inline ids first: a batch whose keys are all inline (or invalid) never touches the dictionary.
  // (Skipped while the maps find no inline key at all — the probe turns inline keys into their ids
  // too — and tried again every 16th map.)
  if (d.last_inline != 0 || (++d.maps & 15) == 0) {
    unsigned long long* nd = d.ctr.as<unsigned long long>() + 4 + 2 * DICT_NL + 2;
    KHIP_TRY_HIP(hipMemsetAsync(nd, 0, 16, s));
    // rows per thread (1 / 2 / 4 / 8: 751 / 740 / 807 / 982 us on C2 --utf8, profiles/r05/ab/inline_rows.txt)
    const int ir = (int)knob("KHIP_INLINE_R", 2);
    auto ik = ir >= 8 ? k_key_inline<8> : (ir >= 4 ? k_key_inline<4> : (ir >= 2 ? k_key_inline<2> : k_key_inline<1>));
    hipLaunchKernelGGL(ik, dim3(grid_for(ceil_div(n, (int64_t)std::max(ir, 1)), 256, 4096)), dim3(256), 0, s, koff, kbytes, kv,
                       rv, ts, n, kid, khash, nd);
    KHIP_TRY_HIP(hipGetLastError());
    unsigned long long h[2] = {0, 0};
    KHIP_TRY_HIP(hipMemcpyAsync(h, nd, 16, hipMemcpyDeviceToHost, s));
    KHIP_TRY_HIP(hipStreamSynchronize(s));
    d.last_inline = (int64_t)h[1];
    if (h[0] == 0) {
      d.last_probed = d.round_probed = 0;
      if (d.last_added < 0) d.last_added = 0;
      return KHIP_OK;
    }
  }
  // room for the keys this batch may add at load <= 1/2: an eighth of the rows on the first map,
  // then twice the last map's new keys (at least 1/16 of the rows that reached the dictionary:
  // inline keys never do) — a batch that brings more fails its probes and is mapped again into a
  // larger table, so the table tracks the key count, not the batch size
  const int64_t est =
      d.last_added < 0 ? std::max<int64_t>(n / 8, 4096)
                       : std::min<int64_t>(n, std::max<int64_t>({2 * d.last_added, std::min(n, d.last_probed) / 16, 4096}));
  if (2 * (d.docc + est) > d.dcap) KHIP_TRY(dict_grow(d, s, next_pow2(2 * (d.docc + est))));
  const int64_t need = d.arena_used + key_bytes_total + 16 * n + 16;
  if ((size_t)need > d.arena.bytes) {
    DevBuf na;
    KHIP_TRY(na.ensure((size_t)std::max<int64_t>(need * 2, 1 << 20)));
    if (d.arena_used) KHIP_TRY_HIP(hipMemcpyAsync(na.p, d.arena.p, d.arena_used, hipMemcpyDeviceToDevice, s));
    KHIP_TRY_HIP(hipStreamSynchronize(s));
    d.arena.release();
    d.arena = std::move(na);
    na.p = nullptr;
  }
  unsigned long long* c = d.ctr.as<unsigned long long>();
  const unsigned long long start[3] = {0ULL, (unsigned long long)d.arena_used, 0ULL};
  KHIP_TRY_HIP(hipMemcpyAsync(c, start, 24, hipMemcpyHostToDevice, s));
  d.round_used = d.arena_used;
  d.round_keys = 0;
  const int64_t* rows = nullptr;
  int64_t m = n;
  DevBuf rl;  // a retry round's rows (the previous round's retry list)
  for (int round = 0, grown = 0; m > 0; round++) {
    int64_t nretry = 0;
    bool failed = false;
    KHIP_TRY(dict_round(d, s, koff, kbytes, kv, rv, ts, rows, m, kid, khash, &nretry, &failed));
    if (failed) {  // undo this round's claims, grow, and map its rows again
      if (++grown > 6 || d.dcap >= ((int64_t)1 << 34)) return fail(KHIP_E_DEVICE, "key dictionary probe budget exhausted");
      hipLaunchKernelGGL(k_dict_unclaim, dim3(grid_for(d.dcap, 256)), dim3(256), 0, s, d.slots.as<ulonglong2>(), d.dcap);
      KHIP_TRY_HIP(hipGetLastError());
      // (room for every row that probed, as distinct keys, at load <= 1/2)
      KHIP_TRY(dict_grow(d, s, std::max<int64_t>(d.dcap * 4, next_pow2(2 * (d.docc + d.round_probed)))));
      continue;
    }
    if (round > 64) return fail(KHIP_E_DEVICE, "key dictionary: rows unresolved after 64 rounds");
    if (nretry == 0) break;
    KHIP_TRY(rl.ensure((size_t)nretry * 8));
    KHIP_TRY_HIP(hipMemcpyAsync(rl.p, d.retry.p, (size_t)nretry * 8, hipMemcpyDeviceToDevice, s));
    rows = rl.as<int64_t>();
    m = nretry;
  }
  d.arena_used = d.round_used;
  d.docc += d.round_keys;
  d.last_added = d.round_keys;
  return KHIP_OK;
}

khip_status dict_find(KeyDict& d, hipStream_t s, const int64_t* koff, const uint8_t* kbytes, int64_t n, int64_t* kid) {
  if (n <= 0) return KHIP_OK;
  hipLaunchKernelGGL(k_dict_find, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, d.slots.as<ulonglong2>(),
                     (uint64_t)(d.dcap - 1), d.arena.as<uint8_t>(), koff, kbytes, n, kid, dict_fp_mask());
  KHIP_TRY_HIP(hipGetLastError());
  return KHIP_OK;
}

khip_status dict_clear(KeyDict& d, hipStream_t s) {
  // the next batches likely bring as many keys as the dictionary held: a table far larger than
  // that (sized by a first map's every-row estimate) is given back
  const int64_t held = d.docc;
  const int64_t keep = std::max<int64_t>(4096, next_pow2(4 * std::max<int64_t>(held, 1)));
  d.docc = 0;
  if (d.dcap >= 4 * keep) KHIP_TRY(dict_grow(d, s, keep));
  if (d.dcap) KHIP_TRY_HIP(hipMemsetAsync(d.slots.p, 0, d.dcap * 32, s));
  if (held > 0) d.last_added = held;  // the next map re-inserts about as many
  d.arena_used = 0;
  return KHIP_OK;
}

void dict_release(KeyDict& d) {
  DevBuf* bufs[] = {&d.slots, &d.arena, &d.ctr, &d.lists, &d.retry};
  for (DevBuf* b : bufs) b->release();
  d.dcap = d.docc = d.arena_used = 0;
}

}  // namespace khip

using namespace khip;

static khip_status plan_state(khip_agg* a) {
  const khip_agg_desc& d = a->desc;
  int word = 3;  // w0, w1, rowtime
  int w_star = -1;
  std::vector<int> w_cnt(d.n_cols, -1), w_sum(d.n_cols, -1), w_min(d.n_cols, -1), w_max(d.n_cols, -1);
  for (int i = 0; i < d.n_aggs; i++) {
    const khip_agg_spec& s = a->aggs[i];
    if (s.kind == KHIP_AGG_COUNT_STAR) {
      if (w_star < 0) w_star = word++;
      continue;
    }
    const int c = s.arg_col;
    // the column's non-null count: COUNT(col), AVG's divisor, MIN/MAX's null test.  SUM alone needs
    // none (SUM over only NULLs is 0, SumKudaf's initial value): its rows stay 32 bytes
    if (s.kind != KHIP_AGG_SUM && w_cnt[c] < 0) w_cnt[c] = word++;
    if ((s.kind == KHIP_AGG_SUM || s.kind == KHIP_AGG_AVG) && w_sum[c] < 0) w_sum[c] = word++;
    if (s.kind == KHIP_AGG_MIN && w_min[c] < 0) w_min[c] = word++;
    if (s.kind == KHIP_AGG_MAX && w_max[c] < 0) w_max[c] = word++;
  }
  if (word > 32) return fail(KHIP_E_UNSUPPORTED, "too many aggregate state words (max 29)");
  a->sw = (int)next_pow2(std::max(word, 4));
  ApplyParams& p = a->ap;
  p.windowed = a->windowed;
  p.slot_words = a->sw;
  p.size = d.size_ms;
  p.adv = d.advance_ms;
  p.grace = a->grace;
  p.n_cols = d.n_cols;
  for (int c = 0; c < d.n_cols; c++) p.col_type[c] = a->col_types[c];
  int n = 0;
  auto add = [&](int8_t kind, int col, int w) {
    p.ops[n].kind = kind;
    p.ops[n].col = (int8_t)col;
    p.ops[n].word = (int16_t)w;
    n++;
  };
  if (w_star >= 0) add(OP_INC, 0, w_star);
  for (int c = 0; c < d.n_cols; c++) {
    if (w_cnt[c] >= 0) add(OP_INC_VALID, c, w_cnt[c]);
    if (w_sum[c] >= 0) add(a->col_types[c] == KHIP_TYPE_DOUBLE ? OP_ADD_F64 : OP_ADD_I64, c, w_sum[c]);
    if (w_min[c] >= 0) add(OP_MIN, c, w_min[c]);
    if (w_max[c] >= 0) add(OP_MAX, c, w_max[c]);
  }
  p.n_ops = n;
  for (int w = 0; w < 32; w++) a->init.w[w] = 0;
  a->init.w[1] = EMPTY_WS;
  a->init.w[2] = INT64_MIN;
  for (int c = 0; c < d.n_cols; c++) {
    if (w_min[c] >= 0) a->init.w[w_min[c]] = INT64_MAX;
    if (w_max[c] >= 0) a->init.w[w_max[c]] = INT64_MIN;
  }
  a->outs.clear();
  for (int i = 0; i < d.n_aggs; i++) {
    const khip_agg_spec& s = a->aggs[i];
    AggOut o{};
    o.kind = s.kind;
    o.type = s.kind == KHIP_AGG_COUNT_STAR ? KHIP_TYPE_INT64 : a->col_types[s.arg_col];
    o.w_cnt = s.kind == KHIP_AGG_COUNT_STAR ? -1 : w_cnt[s.arg_col];
    switch (s.kind) {
      case KHIP_AGG_COUNT_STAR: o.w_val = w_star; break;
      case KHIP_AGG_COUNT: o.w_val = w_cnt[s.arg_col]; break;
      case KHIP_AGG_SUM:
      case KHIP_AGG_AVG: o.w_val = w_sum[s.arg_col]; break;
      case KHIP_AGG_MIN: o.w_val = w_min[s.arg_col]; break;
      case KHIP_AGG_MAX: o.w_val = w_max[s.arg_col]; break;
    }
    a->outs.push_back(o);
  }
  return KHIP_OK;
}

static khip_status init_table(khip_agg* a, DevBuf& buf, int64_t cap) {
  KHIP_TRY(buf.ensure((size_t)cap * a->sw * 8));
  hipLaunchKernelGGL(k_init_table, dim3(grid_for(cap * a->sw, 256)), dim3(256), 0, a->stream,
                     buf.as<uint64_t>(), cap, a->sw, a->init);
  KHIP_TRY_HIP(hipGetLastError());
  return KHIP_OK;
}

khip_status khip::agg_grow_table(khip_agg* a, int64_t new_cap) {
  DevBuf nt;
  KHIP_TRY(init_table(a, nt, new_cap));
  if (a->cap > 0 && a->occ > 0) {
    hipLaunchKernelGGL(k_rehash, dim3(grid_for(a->cap, 256)), dim3(256), 0, a->stream, a->table.as<uint64_t>(),
                       a->cap, nt.as<uint64_t>(), (uint64_t)(new_cap - 1), a->sw,
                       a->desc.key_type == KHIP_KEY_UTF8 ? 1 : 0, a->dict.arena.as<uint8_t>());
    KHIP_TRY_HIP(hipGetLastError());
  }
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  a->table.release();
  a->table = std::move(nt);
  nt.p = nullptr;
  nt.bytes = 0;
  a->cap = new_cap;
  return KHIP_OK;
}

static khip_status grow_table(khip_agg* a, int64_t new_cap) { return agg_grow_table(a, new_cap); }

namespace khip {

int64_t visible_from(const khip_agg* a) {
  if (!a->windowed) return INT64_MIN;
  // PARTITION: every task's store expires by its own stream time (per row through the key map,
  // partition_bounds); the handle-wide bound is the smallest of the tasks' (what every task has
  // expired), INT64_MIN while some task has expired nothing
  if (a->desc.time_domain == KHIP_TIME_PARTITION) {
    if (a->pst_host.empty()) return INT64_MIN;
    int64_t m = INT64_MAX;
    for (int64_t t : a->pst_host) m = std::min(m, partition_vis_from(a, t));
    return m;
  }
  if (a->host_stream_time < 0) return INT64_MIN;
  const int64_t adv = a->desc.advance_ms;
  const int64_t vf = a->host_stream_time / adv * adv - a->retention;  // the store's observed time - retention
  return vf > 0 ? vf : INT64_MIN;  // window starts are >= 0: nothing has expired yet
}

// EMIT FINAL: the window starts this batch closes after they expired (k_emit_lost), computed from
// the batch alone before the engine runs; collected by finish_lost() after the push's sync.
khip_status emit_final_lost(khip_agg* a, const int64_t* ts, const uint8_t* kv, const uint8_t* rv, int64_t n,
                            int64_t seed_st, const int64_t*) {
  const int64_t nb = ceil_div(n, RPB);
  KHIP_TRY(a->blockmax.ensure(nb * 8));
  KHIP_TRY(a->blockprefix.ensure(nb * 8 + 8));
  KHIP_TRY(a->lostctr.ensure(16));
  if (a->lost_cap == 0) {
    a->lost_cap = 4096;
    KHIP_TRY(a->lostbuf.ensure((size_t)a->lost_cap * 16));
  }
  int64_t* seed = a->blockprefix.as<int64_t>() + nb;  // stream time before the batch
  KHIP_TRY(a->part.pinfo.ensure(512));
  int64_t* hs = a->part.pinfo.as<int64_t>() + 24;
  hs[0] = seed_st;  // the stream time before the batch
  KHIP_TRY_HIP(hipMemcpyAsync(seed, hs, 8, hipMemcpyHostToDevice, a->stream));
  KHIP_TRY_HIP(hipMemsetAsync(a->lostctr.p, 0, 8, a->stream));
  hipLaunchKernelGGL(k_blockmax, dim3(nb), dim3(BLOCK), 0, a->stream, ts, kv, rv, n, a->blockmax.as<int64_t>(),
                     (const int64_t*)nullptr);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, a->stream, a->blockmax.as<int64_t>(), nb,
                     a->blockprefix.as<int64_t>(), seed);
  hipLaunchKernelGGL(k_emit_lost, dim3(nb), dim3(BLOCK), 0, a->stream, ts, kv, rv, n, a->blockprefix.as<int64_t>(),
                     a->desc.size_ms, a->desc.advance_ms, a->grace, a->retention, a->lostbuf.as<int64_t>(), a->lost_cap,
                     a->lostctr.as<unsigned long long>());
  KHIP_TRY_HIP(hipGetLastError());
  return KHIP_OK;
}

// After the push's sync: the lost ranges → host (sorted, merged); re-run with room if the
// buffer overflowed (the batch is still valid: the caller owns it until the push returns).
static khip_status finish_lost_seed(khip_agg* a, const int64_t* ts, const uint8_t* kv, const uint8_t* rv, int64_t n,
                                   int64_t seed_st) {
  int64_t cnt = 0;
  KHIP_TRY_HIP(hipMemcpy(&cnt, a->lostctr.p, 8, hipMemcpyDeviceToHost));
  if (cnt > a->lost_cap) {
    a->lost_cap = next_pow2(cnt);
    a->lostbuf.release();
    KHIP_TRY(a->lostbuf.ensure((size_t)a->lost_cap * 16));
    KHIP_TRY(emit_final_lost(a, ts, kv, rv, n, seed_st, nullptr));
    KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
    KHIP_TRY_HIP(hipMemcpy(&cnt, a->lostctr.p, 8, hipMemcpyDeviceToHost));
  }
  std::vector<std::pair<int64_t, int64_t>> r((size_t)cnt);
  if (cnt) KHIP_TRY_HIP(hipMemcpy(r.data(), a->lostbuf.p, (size_t)cnt * 16, hipMemcpyDeviceToHost));
  std::sort(r.begin(), r.end());
  a->lost.clear();
  for (auto& x : r) {
    if (!a->lost.empty() && x.first <= a->lost.back() + 1) {
      a->lost.back() = std::max(a->lost.back(), x.second);
    } else {
      a->lost.push_back(x.first);
      a->lost.push_back(x.second);
    }
  }
  return KHIP_OK;
}

static khip_status finish_lost(khip_agg* a, const int64_t* ts, const uint8_t* kv, const uint8_t* rv, int64_t n) {
  return finish_lost_seed(a, ts, kv, rv, n, a->st_before);
}

// Sorted [lo, hi] pairs, overlapping or adjacent ones merged.
static std::vector<int64_t> merge_ranges(std::vector<std::pair<int64_t, int64_t>> r) {
  std::sort(r.begin(), r.end());
  std::vector<int64_t> out;
  for (auto& x : r) {
    if (!out.empty() && x.first <= out.back() + 1) {
      out.back() = std::max(out.back(), x.second);
    } else {
      out.push_back(x.first);
      out.push_back(x.second);
    }
  }
  return out;
}

}  // namespace khip

extern "C" {

khip_status khip_agg_result_type(const khip_agg_desc* d, int32_t i, int32_t* out) {
  if (!d || !out || i < 0 || i >= d->n_aggs) return fail(KHIP_E_INVALID, "bad aggregate index");
  const khip_agg_spec& s = d->aggs[i];
  if (s.kind == KHIP_AGG_COUNT_STAR || s.kind == KHIP_AGG_COUNT) *out = KHIP_TYPE_INT64;
  else if (s.kind == KHIP_AGG_AVG) *out = KHIP_TYPE_DOUBLE;
  else *out = d->col_types[s.arg_col];
  return KHIP_OK;
}

khip_status khip_agg_create(const khip_agg_desc* desc, khip_agg** out) {
  clear_error();
  if (!desc || !out) return fail(KHIP_E_INVALID, "null argument");
  const khip_agg_desc& d = *desc;
  if (d.window_kind < KHIP_WINDOW_NONE || d.window_kind > KHIP_WINDOW_SESSION)
    return fail(KHIP_E_INVALID, "unknown window kind");
  if (d.window_kind != KHIP_WINDOW_NONE) {
    if (d.size_ms <= 0) return fail(KHIP_E_INVALID, "window size must be > 0");
    if (d.window_kind == KHIP_WINDOW_HOPPING && (d.advance_ms <= 0 || d.advance_ms > d.size_ms))
      return fail(KHIP_E_INVALID, "hopping advance must be in (0, size]");
  }
  if (d.key_type != KHIP_KEY_INT64 && d.key_type != KHIP_KEY_UTF8) return fail(KHIP_E_INVALID, "key type");
  if (d.n_cols < 0 || d.n_cols > MAX_COLS) return fail(KHIP_E_UNSUPPORTED, "at most 8 value columns");
  if (d.n_aggs < 0 || d.n_aggs > 16) return fail(KHIP_E_UNSUPPORTED, "at most 16 aggregates");
  for (int c = 0; c < d.n_cols; c++)
    if (d.col_types[c] < KHIP_TYPE_INT32 || d.col_types[c] > KHIP_TYPE_DOUBLE)
      return fail(KHIP_E_INVALID, "column type");
  for (int i = 0; i < d.n_aggs; i++) {
    const khip_agg_spec& s = d.aggs[i];
    if (s.kind < KHIP_AGG_COUNT_STAR || s.kind > KHIP_AGG_AVG) return fail(KHIP_E_INVALID, "aggregate kind");
    if (s.kind != KHIP_AGG_COUNT_STAR && (s.arg_col < 0 || s.arg_col >= d.n_cols))
      return fail(KHIP_E_INVALID, "aggregate argument column");
  }
  if (d.emit != KHIP_EMIT_CHANGES && d.emit != KHIP_EMIT_FINAL) return fail(KHIP_E_INVALID, "emit strategy");
  if (d.flags & KHIP_FLAG_TABLE_SOURCE) {  // table aggregation: undoable aggregates, no windows
    if (d.window_kind != KHIP_WINDOW_NONE) return fail(KHIP_E_UNSUPPORTED, "windowed aggregation of a table source");
    for (int i = 0; i < d.n_aggs; i++)
      if (d.aggs[i].kind == KHIP_AGG_MIN || d.aggs[i].kind == KHIP_AGG_MAX)  // E/structured/SchemaKGroupedTable.java:82-95
        return fail(KHIP_E_UNSUPPORTED, "MIN/MAX cannot be applied to a table source, only to a stream source");
    if (d.flags & KHIP_FLAG_CHANGELOG) return fail(KHIP_E_UNSUPPORTED, "changelog of a table-source aggregation");
  }
  if (d.emit == KHIP_EMIT_FINAL && d.window_kind == KHIP_WINDOW_NONE)
    return fail(KHIP_E_INVALID, "EMIT FINAL needs a windowed aggregation");
  if (d.window_kind != KHIP_WINDOW_NONE && d.retention_ms != KHIP_RETENTION_DEFAULT) {
    // TimeWindowedKStreamImpl: retention < size + grace is an IllegalArgumentException
    const int64_t g = grace_of(d);
    if (d.retention_ms < 0 || d.retention_ms < d.size_ms + g)
      return fail(KHIP_E_INVALID, "retention must be at least window size + grace");
  }
  if (d.time_domain < KHIP_TIME_TASK || d.time_domain > KHIP_TIME_SUPPLIED) return fail(KHIP_E_INVALID, "time domain");
  if (d.time_domain != KHIP_TIME_TASK) {
    // SESSION windows take the SUPPLIED (GLOBAL) stream time with EMIT CHANGES: the replay reads
    // each row's given stream time.  EMIT FINAL needs the stream time BEFORE each row, which the
    // shuffle does not carry; PARTITION needs per-task session expiry.
    if (d.window_kind == KHIP_WINDOW_SESSION && (d.time_domain == KHIP_TIME_PARTITION || d.emit == KHIP_EMIT_FINAL))
      return fail(KHIP_E_UNSUPPORTED, "SESSION windows: PARTITION stream time, or EMIT FINAL under SUPPLIED");
    if (d.flags & KHIP_FLAG_TABLE_SOURCE) return fail(KHIP_E_UNSUPPORTED, "stream-time domains of a table source");
    if (d.time_domain == KHIP_TIME_PARTITION && (d.n_partitions < 1 || d.n_partitions > 65536))
      return fail(KHIP_E_INVALID, "n_partitions must be in [1, 65536]");
  }
  if (d.has_having) {
    if (d.having.agg_index < 0 || d.having.agg_index >= d.n_aggs) return fail(KHIP_E_INVALID, "having agg index");
    if (d.having.op < KHIP_OP_GT || d.having.op > KHIP_OP_NE) return fail(KHIP_E_INVALID, "having op");
  }
  khip_agg* a = new khip_agg();
  a->desc = d;
  a->col_types.assign(d.col_types, d.col_types + d.n_cols);
  a->aggs.assign(d.aggs, d.aggs + d.n_aggs);
  a->desc.col_types = a->col_types.data();
  a->desc.aggs = a->aggs.data();
  if (d.window_kind == KHIP_WINDOW_TUMBLING || d.window_kind == KHIP_WINDOW_SESSION) a->desc.advance_ms = d.size_ms;
  a->windowed = d.window_kind != KHIP_WINDOW_NONE;
  a->grace = grace_of(a->desc);
  a->max_fanout = a->windowed ? (int)ceil_div(a->desc.size_ms, a->desc.advance_ms) : 1;
  if (a->windowed && ceil_div(a->desc.size_ms, a->desc.advance_ms) > MAX_FANOUT) {
    delete a;
    return fail(KHIP_E_UNSUPPORTED, "hopping fan-out above 4095 windows per record");
  }
  a->device = d.device;
  khip_status st = plan_state(a);
  if (st != KHIP_OK) {
    delete a;
    return st;
  }
  if (d.has_having) {
    a->having.active = 1;
    a->having.op = d.having.op;
    a->having.a = a->outs[d.having.agg_index];
    a->having.i64 = d.having.i64;
    a->having.f64 = d.having.f64;
  }
  DeviceGuard g(a->device);
  if (hipStreamCreateWithFlags(&a->stream, hipStreamDefault) != hipSuccess) {
    delete a;
    return fail(KHIP_E_DEVICE, "hipStreamCreate failed (no device?)");
  }
  a->profile = (d.flags & KHIP_FLAG_PROFILE) != 0;
  a->engine = d.window_kind == KHIP_WINDOW_SESSION ? 2
              : (d.flags & KHIP_FLAG_TABLE_SOURCE) ? 3
              : ((d.flags & KHIP_FLAG_ENGINE_ATOMIC) ? 1 : 0);
  a->changelog = (d.flags & KHIP_FLAG_CHANGELOG) != 0 && d.emit == KHIP_EMIT_CHANGES;
  if (a->windowed)
    a->retention = d.retention_ms == KHIP_RETENTION_DEFAULT ? a->desc.size_ms + a->grace : d.retention_ms;
  if (a->changelog && a->engine == 1) {  // (SESSION windows keep their changelog themselves)
    khip_agg_destroy(a);
    return fail(KHIP_E_UNSUPPORTED, "EMIT CHANGES changelog needs the partitioned engine");
  }
  if (a->profile)
    // timing only (KHIP_FLAG_PROFILE): no system-scope fence at each event — with it every
    // event wrote back and invalidated the L2 (≈ 54 µs per C2 push over its 4-5 events)
    for (int e = 0; e < 8; e++) hipEventCreateWithFlags(&a->ev[e], hipEventDisableSystemFence);
  int64_t cap = (a->engine == 1 || a->engine == 3) ? next_pow2(std::max<int64_t>(1024, d.capacity_hint > 0 ? d.capacity_hint * 2 : 1 << 16))
                                : 1024;
  if ((st = init_table(a, a->table, cap)) != KHIP_OK || (st = a->stream_time.ensure(8)) != KHIP_OK ||
      (st = a->counters.ensure(8 * NPART)) != KHIP_OK ||
      (a->engine == 0 && (st = part_init(a, d.capacity_hint > 0 ? d.capacity_hint : (1 << 20))) != KHIP_OK)) {
    khip_agg_destroy(a);
    return st;
  }
  a->cap = cap;
  int64_t m1 = -1;
  hipMemcpyAsync(a->stream_time.p, &m1, 8, hipMemcpyHostToDevice, a->stream);
  if (d.time_domain == KHIP_TIME_PARTITION) {  // every partition's stream time: none yet
    if ((st = a->pst.ensure((size_t)d.n_partitions * 8)) != KHIP_OK ||
        (st = a->pst2.ensure((size_t)d.n_partitions * 8)) != KHIP_OK) {
      khip_agg_destroy(a);
      return st;
    }
    hipMemsetAsync(a->pst.p, 0xFF, (size_t)d.n_partitions * 8, a->stream);
  }
  if (d.key_type == KHIP_KEY_UTF8) {
    if ((st = dict_init(a->dict, a->stream)) != KHIP_OK) {
      khip_agg_destroy(a);
      return st;
    }
  }
  if (hipStreamSynchronize(a->stream) != hipSuccess) {
    khip_agg_destroy(a);
    return fail(KHIP_E_DEVICE, "device init failed");
  }
  *out = a;
  return KHIP_OK;
}

static khip_status stage(khip_agg* a, DevBuf& buf, const void* src, size_t bytes) {
  KHIP_TRY(buf.ensure(bytes));
  if (bytes) KHIP_TRY_HIP(hipMemcpyAsync(buf.p, src, bytes, hipMemcpyHostToDevice, a->stream));
  return KHIP_OK;
}

// The batch's device pointers: host batches are staged into the handle's buffers (asynchronously,
// on its stream); UTF8 key byte totals of device batches are fetched (synchronise before use).
static khip_status resolve_batch(khip_agg* a, const khip_batch* b, const int64_t** keys_o, const int64_t** ts_o,
                                 const uint8_t** kv_o, const uint8_t** rv_o, const int64_t** koff_o,
                                 const uint8_t** kbytes_o, ColPtrs* cols_o, int64_t* key_bytes_total_o) {
  const int64_t n = b->n_rows;
  const bool utf8 = a->desc.key_type == KHIP_KEY_UTF8;
  const int64_t* keys = b->key_i64;
  const int64_t* ts = b->ts;
  const uint8_t* kv = b->key_valid;
  const uint8_t* rv = b->row_valid;
  const int64_t* koff = b->key_offsets;
  const uint8_t* kbytes = b->key_bytes;
  ColPtrs cols{};
  const size_t bm = (size_t)(n + 7) / 8;
  int64_t key_bytes_total = 0;
  if (b->mem == KHIP_MEM_HOST) {
    KHIP_TRY(stage(a, a->st_ts, b->ts, n * 8));
    ts = a->st_ts.as<int64_t>();
    if (kv) { KHIP_TRY(stage(a, a->st_kv, kv, bm)); kv = a->st_kv.as<uint8_t>(); }
    if (rv) { KHIP_TRY(stage(a, a->st_rv, rv, bm)); rv = a->st_rv.as<uint8_t>(); }
    if (utf8) {
      key_bytes_total = b->key_offsets[n];
      KHIP_TRY(stage(a, a->st_koff, b->key_offsets, (n + 1) * 8));
      KHIP_TRY(stage(a, a->st_kbytes, b->key_bytes, (size_t)std::max<int64_t>(key_bytes_total, 1)));
      koff = a->st_koff.as<int64_t>();
      kbytes = a->st_kbytes.as<uint8_t>();
    } else {
      KHIP_TRY(stage(a, a->st_keys, b->key_i64, n * 8));
      keys = a->st_keys.as<int64_t>();
    }
    for (int c = 0; c < a->desc.n_cols; c++) {
      const size_t es = a->col_types[c] == KHIP_TYPE_INT32 ? 4 : 8;
      KHIP_TRY(stage(a, a->st_cols[c], b->col_data[c], n * es));
      cols.data[c] = a->st_cols[c].p;
      const uint8_t* cv = b->col_valid ? b->col_valid[c] : nullptr;
      if (cv) {
        KHIP_TRY(stage(a, a->st_cval[c], cv, bm));
        cols.valid[c] = a->st_cval[c].as<uint8_t>();
      }
    }
  } else if (b->mem == KHIP_MEM_DEVICE) {
    for (int c = 0; c < a->desc.n_cols; c++) {
      cols.data[c] = b->col_data[c];
      cols.valid[c] = b->col_valid ? b->col_valid[c] : nullptr;
    }
    if (utf8)
      KHIP_TRY_HIP(hipMemcpyAsync(&key_bytes_total, koff + n, 8, hipMemcpyDeviceToHost, a->stream));
  } else {
    return fail(KHIP_E_INVALID, "batch mem");
  }
  *keys_o = keys;
  *ts_o = ts;
  *kv_o = kv;
  *rv_o = rv;
  *koff_o = koff;
  *kbytes_o = kbytes;
  *cols_o = cols;
  *key_bytes_total_o = key_bytes_total;
  return KHIP_OK;
}

// KHIP_TIME_SUPPLIED with a close context: the handle's stream time becomes the GLOBAL one after the
// batch (closing windows and retention as one task over the whole stream).
static khip_status supplied_advance(khip_agg* a) {
  if (a->sup_after > a->host_stream_time) {
    a->host_stream_time = a->sup_after;
    KHIP_TRY(a->part.pinfo.ensure(512));
    int64_t* hs = a->part.pinfo.as<int64_t>() + 25;
    hs[0] = a->sup_after;
    KHIP_TRY_HIP(hipMemcpyAsync(a->stream_time.p, hs, 8, hipMemcpyHostToDevice, a->stream));
    KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  }
  return KHIP_OK;
}

// ABI 6.  Received shuffle rows into the aggregation: the value pipeline reads them where they lie
// (khip_agg_c1.hip, RowsIn); any other push unpacks them into the handle's staging columns and runs
// as a device batch.  Same results and statistics as khip_agg_push of the unpacked batch.
khip_status khip_agg_push_shuffled(khip_agg* a, const khip_shuffle* sh, const uint64_t* rows, int64_t n,
                                   khip_batch_stats* stats) {
  clear_error();
  if (!a || !sh || (n > 0 && !rows)) return fail(KHIP_E_INVALID, "null argument");
  if (n < 0) return fail(KHIP_E_INVALID, "row count");
  int kc = 0, nc = 0;
  const int32_t* types = nullptr;
  shuffle_layout(sh, &kc, &nc, &types);
  if (nc != a->desc.n_cols) return fail(KHIP_E_INVALID, "the shuffle's columns are not the aggregation's");
  for (int c = 0; c < nc; c++)
    if (types[c] != a->col_types[c]) return fail(KHIP_E_INVALID, "the shuffle's column types are not the aggregation's");
  if (a->desc.key_type == KHIP_KEY_UTF8) return fail(KHIP_E_UNSUPPORTED, "shuffled rows carry an integer GROUP BY key");
  if (a->engine == 3) return fail(KHIP_E_STATE, "table-source aggregation: use khip_agg_push_table");
  if (a->desc.time_domain == KHIP_TIME_PARTITION)
    return fail(KHIP_E_UNSUPPORTED, "KHIP_TIME_PARTITION: received rows carry no source partition");
  const bool sup = a->desc.time_domain == KHIP_TIME_SUPPLIED;
  const int rw = khip_shuffle_row_words(sh);
  if (sup && rw != 3 + nc)
    return fail(KHIP_E_INVALID, "KHIP_TIME_SUPPLIED: the shuffle carries no stream time (KHIP_SHUFFLE_STREAM_TIME)");
  DeviceGuard g(a->device);
  if (n > 0 && n < (1LL << 31) && a->engine == 0 && a->desc.emit != KHIP_EMIT_FINAL) {
    khip_batch_stats s{};
    s.rows_in = n;
    a->st_before = a->host_stream_time;
    a->chg_ready = false;
    a->lost.clear();
    int64_t tot[NPART] = {0};
    bool done = false;
    KHIP_TRY(part_push_rows(a, n, RowsIn{rows, rw, 0, 0}, kc, tot, &done, sup));
    if (done) {
      a->occ += tot[P_NEW];
      if (a->profile) {
        a->times.stream_time_ms += ev_ms(a, 3, 4);
        a->times.partition_ms += ev_ms(a, 4, 5);
        a->times.apply_ms += ev_ms(a, 5, 6);
        a->times.records += n;
        a->times.apply_launches++;
      }
      if (a->windowed) {  // retention: drop expired windows from the closed store
        HavingDev vis{};
        vis.vis = 1;
        vis.vis_from = visible_from(a);
        if (vis.vis_from != INT64_MIN) KHIP_TRY(part_purge_closed(a, vis));
      }
      s.rows_accepted = tot[P_ACCEPTED];
      s.dropped_null_key = tot[P_NULL_KEY];
      s.dropped_null_row = tot[P_NULL_ROW];
      s.dropped_bad_ts = tot[P_BAD_TS];
      s.windows_applied = tot[P_APPLIED];
      s.windows_late = tot[P_LATE];
      s.stream_time = a->host_stream_time;
      if (stats) *stats = s;
      return KHIP_OK;
    }
  }
  // the rows as columns (the staging buffers: a device batch never uses them)
  const size_t bm = (size_t)(n + 7) / 8;
  KHIP_TRY(a->st_keys.ensure((size_t)std::max<int64_t>(n, 1) * 8));
  KHIP_TRY(a->st_ts.ensure((size_t)std::max<int64_t>(n, 1) * 8));
  void* cd[MAX_COLS] = {};
  uint8_t* cv[MAX_COLS] = {};
  for (int c = 0; c < nc; c++) {
    KHIP_TRY(a->st_cols[c].ensure((size_t)std::max<int64_t>(n, 1) * 8));
    KHIP_TRY(a->st_cval[c].ensure(std::max<size_t>(bm, 1)));
    cd[c] = a->st_cols[c].p;
    cv[c] = a->st_cval[c].as<uint8_t>();
  }
  if (n > 0)
    KHIP_TRY(khip_shuffle_unpack(const_cast<khip_shuffle*>(sh), rows, n, a->st_keys.as<int64_t>(), a->st_ts.as<int64_t>(),
                                 cd, cv));
  khip_batch b{};
  if (sup) {  // the GLOBAL stream time each row was routed with
    KHIP_TRY(a->st_col.ensure((size_t)std::max<int64_t>(n, 1) * 8));
    if (n > 0) KHIP_TRY(khip_shuffle_unpack_stream_time(const_cast<khip_shuffle*>(sh), rows, n, a->st_col.as<int64_t>()));
    b.stream_time = a->st_col.as<int64_t>();
  }
  b.mem = KHIP_MEM_DEVICE;
  b.n_rows = n;
  b.n_cols = nc;
  b.key_i64 = a->st_keys.as<int64_t>();
  b.ts = a->st_ts.as<int64_t>();
  b.col_data = (const void* const*)cd;
  b.col_valid = (const uint8_t* const*)cv;
  return khip_agg_push(a, &b, stats);
}

khip_status khip_agg_push_table(khip_agg* a, const khip_batch* b, const khip_table_src* src,
                                khip_batch_stats* stats) {
  clear_error();
  if (!a || !b || !src) return fail(KHIP_E_INVALID, "null argument");
  if (a->engine != 3) return fail(KHIP_E_STATE, "handle not created with KHIP_FLAG_TABLE_SOURCE");
  if (b->n_rows < 0 || b->n_cols < a->desc.n_cols) return fail(KHIP_E_INVALID, "batch shape");
  if (src->key_type != KHIP_KEY_INT64 && src->key_type != KHIP_KEY_UTF8) return fail(KHIP_E_INVALID, "source key type");
  TaggState& T = a->tagg;
  if (T.key_type >= 0 && T.key_type != src->key_type) return fail(KHIP_E_INVALID, "source key type changed");
  const int64_t n = b->n_rows;
  const bool utf8 = a->desc.key_type == KHIP_KEY_UTF8, src_utf8 = src->key_type == KHIP_KEY_UTF8;
  if (n > 0) {
    if (!b->ts || (utf8 ? (!b->key_offsets || !b->key_bytes) : !b->key_i64))
      return fail(KHIP_E_INVALID, "missing GROUP BY key or timestamp column");
    if (src_utf8 ? (!src->key_offsets || !src->key_bytes) : !src->key_i64)
      return fail(KHIP_E_INVALID, "missing source PRIMARY KEY column");
    for (int c = 0; c < a->desc.n_cols; c++)
      if (!b->col_data || !b->col_data[c]) return fail(KHIP_E_INVALID, "missing value column");
  }
  DeviceGuard g(a->device);
  if (T.key_type < 0) {
    if (src_utf8) KHIP_TRY(dict_init(T.dict, a->stream));
    T.key_type = src->key_type;
  }
  khip_batch_stats s{};
  s.rows_in = n;
  a->chg_ready = false;
  if (n == 0) {
    s.stream_time = a->host_stream_time;
    if (stats) *stats = s;
    return KHIP_OK;
  }
  const int64_t* keys;
  const int64_t* ts;
  const uint8_t *kv, *rv;
  const int64_t* koff;
  const uint8_t* kbytes;
  ColPtrs cols{};
  int64_t key_bytes_total = 0;
  KHIP_TRY(resolve_batch(a, b, &keys, &ts, &kv, &rv, &koff, &kbytes, &cols, &key_bytes_total));
  // the source PRIMARY KEYs on the device
  const int64_t* sk = src->key_i64;
  const int64_t* skoff = src->key_offsets;
  const uint8_t* skb = src->key_bytes;
  const uint8_t* skv = src->key_valid;
  int64_t src_bytes = 0;
  if (b->mem == KHIP_MEM_HOST) {
    const size_t bm = (size_t)(n + 7) / 8;
    if (skv) { KHIP_TRY(stage(a, T.st_kv, skv, bm)); skv = T.st_kv.as<uint8_t>(); }
    if (src_utf8) {
      src_bytes = src->key_offsets[n];
      KHIP_TRY(stage(a, T.st_koff, src->key_offsets, (n + 1) * 8));
      KHIP_TRY(stage(a, T.st_kbytes, src->key_bytes, (size_t)std::max<int64_t>(src_bytes, 1)));
      skoff = T.st_koff.as<int64_t>();
      skb = T.st_kbytes.as<uint8_t>();
    } else {
      KHIP_TRY(stage(a, T.st_key, src->key_i64, n * 8));
      sk = T.st_key.as<int64_t>();
    }
  } else if (src_utf8) {
    KHIP_TRY_HIP(hipMemcpyAsync(&src_bytes, skoff + n, 8, hipMemcpyDeviceToHost, a->stream));
  }
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));  // key byte totals of device batches
  // GROUP BY keys → ids (UTF8: the group dictionary; rows that cannot add to a group are skipped)
  const int64_t* hkeys = keys;
  if (utf8) {
    KHIP_TRY(a->kid.ensure(n * 8));
    KHIP_TRY(a->khash.ensure(n * 8));
    KHIP_TRY(dict_map(a->dict, a->stream, koff, kbytes, key_bytes_total, kv, rv, ts, n, a->kid.as<int64_t>(),
                      a->khash.as<int64_t>()));
    keys = a->kid.as<int64_t>();
    hkeys = a->khash.as<int64_t>();
  }
  if (src_utf8) {
    KHIP_TRY(T.sid.ensure(n * 8));
    KHIP_TRY(T.shash.ensure(n * 8));
    KHIP_TRY(dict_map(T.dict, a->stream, skoff, skb, src_bytes, skv, nullptr, ts, n, T.sid.as<int64_t>(),
                      T.shash.as<int64_t>()));
    sk = T.sid.as<int64_t>();
  }
  int64_t tot[NPART] = {0};
  KHIP_TRY(tagg_push(a, n, keys, hkeys, kv, rv, ts, cols, sk, skv, tot));
  s.rows_accepted = tot[P_ACCEPTED];
  s.dropped_null_key = tot[P_NULL_KEY];
  s.dropped_bad_ts = tot[P_BAD_TS];
  s.windows_applied = tot[P_APPLIED];
  s.stream_time = a->host_stream_time;
  if (stats) *stats = s;
  return KHIP_OK;
}

khip_status khip_agg_push(khip_agg* a, const khip_batch* b, khip_batch_stats* stats) {
  clear_error();
  if (!a || !b) return fail(KHIP_E_INVALID, "null argument");
  if (b->n_rows < 0 || b->n_cols < a->desc.n_cols) return fail(KHIP_E_INVALID, "batch shape");
  if (b->n_rows >= (1LL << 36)) return fail(KHIP_E_UNSUPPORTED, "batch larger than 2^36 rows");
  if (a->engine == 3) return fail(KHIP_E_STATE, "table-source aggregation: use khip_agg_push_table");
  const int64_t n = b->n_rows;
  const bool utf8 = a->desc.key_type == KHIP_KEY_UTF8;
  if (!b->ts || (utf8 ? (!b->key_offsets || !b->key_bytes) : !b->key_i64))
    if (n > 0) return fail(KHIP_E_INVALID, "missing key or timestamp column");
  for (int c = 0; c < a->desc.n_cols; c++)
    if (n > 0 && (!b->col_data || !b->col_data[c])) return fail(KHIP_E_INVALID, "missing value column");
  DeviceGuard g(a->device);
  khip_batch_stats s{};
  s.rows_in = n;
  const bool supd = a->desc.time_domain == KHIP_TIME_SUPPLIED;
  if (supd && a->desc.emit == KHIP_EMIT_FINAL && !a->sup_set)
    return fail(KHIP_E_INVALID, "KHIP_TIME_SUPPLIED + EMIT FINAL: khip_agg_supplied_close before every push");
  const bool sctx = supd && a->sup_set;
  a->sup_set = false;
  a->st_before = sctx ? a->sup_before : a->host_stream_time;
  a->chg_ready = false;
  a->lost.clear();
  if (n == 0 && !sctx) {  // nothing changes, nothing closes
    a->chg_ready = true;
    a->chg_n = 0;
    s.stream_time = a->host_stream_time;
    if (stats) *stats = s;
    return KHIP_OK;
  }
  if (n == 0) {  // SUPPLIED: nothing arrived here, but the GLOBAL stream time may close windows
    KHIP_TRY(supplied_advance(a));
    if (a->desc.emit == KHIP_EMIT_FINAL) a->lost = a->sup_lost;
    else a->chg_ready = true, a->chg_n = 0;
    s.stream_time = a->host_stream_time;
    if (stats) *stats = s;
    return KHIP_OK;
  }
  if (a->changelog && n >= (1LL << 31)) return fail(KHIP_E_UNSUPPORTED, "changelog pushes above 2^31 rows");
  const bool final_emit = a->desc.emit == KHIP_EMIT_FINAL;
  // ---- device pointers (stage host batches)
  const int64_t* keys;
  const int64_t* ts;
  const uint8_t *kv, *rv;
  const int64_t* koff;
  const uint8_t* kbytes;
  ColPtrs cols{};
  int64_t key_bytes_total = 0;
  KHIP_TRY(resolve_batch(a, b, &keys, &ts, &kv, &rv, &koff, &kbytes, &cols, &key_bytes_total));
  const bool pdomain = a->desc.time_domain == KHIP_TIME_PARTITION;
  // (SESSION windows close sessions themselves: sess_push)
  if (final_emit && !pdomain && !sctx && a->engine != 2) KHIP_TRY(emit_final_lost(a, ts, kv, rv, n, a->st_before, nullptr));
  // ---- ABI 5 stream-time domains: the stream time observed at every row
  const int64_t* st_at = nullptr;
  const int32_t* part = nullptr;
  if (a->desc.time_domain == KHIP_TIME_SUPPLIED) {
    if (!b->stream_time) return fail(KHIP_E_INVALID, "KHIP_TIME_SUPPLIED: the batch has no stream_time column");
    if (b->mem == KHIP_MEM_HOST) {
      KHIP_TRY(stage(a, a->st_col, b->stream_time, n * 8));
      st_at = a->st_col.as<int64_t>();
    } else {
      st_at = b->stream_time;
    }
  } else if (a->desc.time_domain == KHIP_TIME_PARTITION) {
    if (!b->partition) return fail(KHIP_E_INVALID, "KHIP_TIME_PARTITION: the batch has no partition column");
    part = b->partition;
    if (b->mem == KHIP_MEM_HOST) {
      KHIP_TRY(stage(a, a->st_part, b->partition, n * 4));
      part = a->st_part.as<int32_t>();
    }
    KHIP_TRY(a->st_col.ensure((size_t)n * 8));
    KHIP_TRY(stream_time_column(a, ts, kv, rv, part, n, -1, a->st_col.as<int64_t>(), nullptr));
    st_at = a->st_col.as<int64_t>();
    if (final_emit) KHIP_TRY(partition_lost(a, ts, kv, rv, part, st_at, n));
  }
  // ---- UTF8 keys → stable key ids
  const int64_t* hkeys = keys;
  if (utf8) {
    KHIP_TRY_HIP(hipStreamSynchronize(a->stream));  // key_bytes_total for device batches
    ev_record(a, 1);
    KHIP_TRY(a->kid.ensure(n * 8));
    // the key hashes only feed the global-atomic engine's slot hashing (the others hash the ids)
    const bool want_hash = a->engine == 1;
    if (want_hash) KHIP_TRY(a->khash.ensure(n * 8));
    KHIP_TRY(dict_map(a->dict, a->stream, koff, kbytes, key_bytes_total, kv, rv, ts, n, a->kid.as<int64_t>(),
                      want_hash ? a->khash.as<int64_t>() : nullptr));
    keys = a->kid.as<int64_t>();
    hkeys = want_hash ? a->khash.as<int64_t>() : keys;
    ev_record(a, 2);
  }
  // per-task retention / EMIT FINAL: every accepted key's partition (the tasks share one table)
  // A batch that puts a key on a second partition is rejected before it changes the handle's
  // stream times: the partitions' stream times go back to their values before the batch (the
  // batch's new keys stay recorded with the partitions it named, as its dictionary entries stay).
  if (pdomain && a->windowed) {
    const khip_status ps = pmap_insert(a, keys, kv, rv, ts, part, n);
    if (ps != KHIP_OK) {
      std::swap(a->pst, a->pst2);
      return ps;
    }
  }
  int64_t tot[NPART] = {0};
  if (a->engine == 2) {
    if (n >= (1LL << 31)) return fail(KHIP_E_UNSUPPORTED, "SESSION pushes above 2^31 rows");
    // SUPPLIED with a close context: the GLOBAL stream time after the batch bounds the store's
    // expiry (sess_push expires against the handle's stream time after the push)
    if (sctx) KHIP_TRY(supplied_advance(a));
    KHIP_TRY(sess_push(a, n, keys, ts, kv, rv, cols, tot, st_at));
  } else if (a->engine == 0) {
    // ---- partitioned engine, in slices of < 2^31 records (multiple of 8: bitmaps stay byte aligned)
    const int64_t slice = 1LL << 31;
    for (int64_t off = 0; off < n; off += slice) {
      const int64_t m = std::min(slice, n - off);
      ColPtrs cs = cols;
      for (int c = 0; c < a->desc.n_cols; c++) {
        cs.data[c] = (const char*)cols.data[c] + off * (a->col_types[c] == KHIP_TYPE_INT32 ? 4 : 8);
        if (cs.valid[c]) cs.valid[c] += off / 8;
      }
      KHIP_TRY(part_push(a, m, keys + off, ts + off, kv ? kv + off / 8 : nullptr, rv ? rv + off / 8 : nullptr, cs,
                         tot, st_at ? st_at + off : nullptr));
    }
    a->occ += tot[P_NEW];
    if (a->profile) {  // events of the last slice
      a->times.stream_time_ms += ev_ms(a, 3, 4);
      a->times.partition_ms += ev_ms(a, 4, 5);
      a->times.apply_ms += ev_ms(a, 5, 6);
      if (utf8) a->times.dict_ms += ev_ms(a, 1, 2);
      a->times.records += n;
      a->times.apply_launches++;
    }
  } else {
  // ---- scratch
  const int64_t nb = ceil_div(n, RPB);
  KHIP_TRY(a->blockmax.ensure(nb * 8));
  KHIP_TRY(a->blockprefix.ensure(nb * 8));
  KHIP_TRY(a->partials.ensure(nb * 8 * NPART));
  if (a->resume_n < n) {
    KHIP_TRY(a->resume.ensure(n * 4));
    KHIP_TRY_HIP(hipMemsetAsync(a->resume.p, 0xFF, n * 4, a->stream));
    a->resume_n = n;
  }
  KHIP_TRY_HIP(hipMemsetAsync(a->counters.p, 0, 8 * NPART, a->stream));
  // ---- stream time before each block (atomic engine)
  ev_record(a, 0);
  hipLaunchKernelGGL(k_blockmax, dim3(nb), dim3(BLOCK), 0, a->stream, ts, kv, rv, n, a->blockmax.as<int64_t>(),
                     st_at);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, a->stream, a->blockmax.as<int64_t>(), nb,
                     a->blockprefix.as<int64_t>(), a->stream_time.as<int64_t>());
  KHIP_TRY_HIP(hipGetLastError());
  ev_record(a, 2);
  // ---- grow the group table ahead of time if the resident load is high
  if (2 * a->occ > a->cap) KHIP_TRY(grow_table(a, a->cap * 4));
  // ---- apply (+ resume passes after doubling on probe exhaustion)
  const int64_t occ0 = a->occ;
  double apply_ms = 0, fin_ms = 0;
  for (int pass = 0;; pass++) {
    ev_record(a, 3);
    hipLaunchKernelGGL(k_apply, dim3(nb), dim3(BLOCK), 0, a->stream, a->ap, hkeys, keys, ts, kv, rv, cols,
                       a->blockprefix.as<int64_t>(), n, a->table.as<uint64_t>(), (uint64_t)(a->cap - 1),
                       a->resume.as<int32_t>(), a->partials.as<int64_t>(), pass > 0 ? 1 : 0, st_at);
    ev_record(a, 4);
    hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(256), 0, a->stream, a->partials.as<int64_t>(), nb, NPART,
                       a->counters.as<int64_t>());
    hipLaunchKernelGGL(k_finalize, dim3(grid_for(a->cap, 256)), dim3(256), 0, a->stream, a->table.as<uint64_t>(),
                       a->cap, a->sw, keys, ts, a->windowed, a->desc.size_ms, a->desc.advance_ms);
    KHIP_TRY_HIP(hipGetLastError());
    ev_record(a, 5);
    int64_t c[NPART];
    KHIP_TRY_HIP(hipMemcpyAsync(c, a->counters.p, 8 * NPART, hipMemcpyDeviceToHost, a->stream));
    KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
    const int64_t failed = c[P_FAILED] - tot[P_FAILED];
    for (int k = 0; k < NPART; k++) tot[k] = c[k];
    a->occ = occ0 + tot[P_NEW];  // every claim is counted exactly once
    if (a->profile) {
      apply_ms += ev_ms(a, 3, 4);
      fin_ms += ev_ms(a, 4, 5);
      if (pass == 0) {
        a->times.stream_time_ms += ev_ms(a, 0, 3);
        if (utf8) a->times.dict_ms += ev_ms(a, 1, 2);
        a->times.records += n;
      }
      a->times.apply_launches++;
    }
    if (failed == 0) break;
    if (pass > 40) return fail(KHIP_E_DEVICE, "aggregate table could not absorb the batch");
    KHIP_TRY(grow_table(a, a->cap * 2));
  }
  a->times.apply_ms += apply_ms;
  a->times.finalize_ms += fin_ms;
  }
  if (a->engine == 1) {  // the other engines brought it back with their end-of-push counters
    KHIP_TRY_HIP(hipMemcpyAsync(&a->host_stream_time, a->stream_time.p, 8, hipMemcpyDeviceToHost, a->stream));
    KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  }
  // one task per partition: the handle's stream time (closing windows, retention) is the slowest's
  if (pdomain) KHIP_TRY(stream_time_partition_min(a));
  if (sctx) KHIP_TRY(supplied_advance(a));  // one task over the whole stream: the GLOBAL stream time
  if (final_emit && sctx) a->lost = a->sup_lost;
  else if (final_emit && a->engine != 2) KHIP_TRY(pdomain ? partition_lost_finish(a) : finish_lost(a, ts, kv, rv, n));
  if (a->engine == 0 && a->windowed) {  // retention: drop expired windows from the closed store
    HavingDev vis{};
    vis.vis = 1;
    vis.vis_from = visible_from(a);
    if (vis.vis_from != INT64_MIN) {
      KHIP_TRY(partition_bounds(a, vis));  // PARTITION: each row by its own task's bound
      KHIP_TRY(part_purge_closed(a, vis));
    }
  }
  s.rows_accepted = tot[P_ACCEPTED];
  s.dropped_null_key = tot[P_NULL_KEY];
  s.dropped_null_row = tot[P_NULL_ROW];
  s.dropped_bad_ts = tot[P_BAD_TS];
  s.windows_applied = tot[P_APPLIED];
  s.windows_late = tot[P_LATE];
  s.stream_time = a->host_stream_time;
  if (stats) *stats = s;
  return KHIP_OK;
}

khip_status khip_stream_time_scan(khip_agg* a, const khip_batch* b, int64_t seed, int64_t* out, int64_t* out_max) {
  clear_error();
  if (!a || !b || !out_max || (b->n_rows > 0 && (!out || !b->ts))) return fail(KHIP_E_INVALID, "null argument");
  if (b->n_rows < 0) return fail(KHIP_E_INVALID, "batch shape");
  DeviceGuard g(a->device);
  const int64_t n = b->n_rows;
  *out_max = seed < -1 ? -1 : seed;
  if (n == 0) return KHIP_OK;
  const int64_t* ts = b->ts;
  const uint8_t *kv = b->key_valid, *rv = b->row_valid;
  int64_t* dst = out;
  const size_t bm = (size_t)(n + 7) / 8;
  if (b->mem == KHIP_MEM_HOST) {
    KHIP_TRY(stage(a, a->st_ts, b->ts, n * 8));
    ts = a->st_ts.as<int64_t>();
    if (kv) { KHIP_TRY(stage(a, a->st_kv, kv, bm)); kv = a->st_kv.as<uint8_t>(); }
    if (rv) { KHIP_TRY(stage(a, a->st_rv, rv, bm)); rv = a->st_rv.as<uint8_t>(); }
    KHIP_TRY(a->st_col.ensure((size_t)n * 8));
    dst = a->st_col.as<int64_t>();
  } else if (b->mem != KHIP_MEM_DEVICE) {
    return fail(KHIP_E_INVALID, "batch mem");
  }
  KHIP_TRY(a->st_seen.ensure(8));
  int64_t* last = a->st_seen.as<int64_t>();
  KHIP_TRY(stream_time_column(a, ts, kv, rv, nullptr, n, seed < -1 ? -1 : seed, dst, last));
  if (b->mem == KHIP_MEM_HOST) KHIP_TRY_HIP(hipMemcpyAsync(out, dst, (size_t)n * 8, hipMemcpyDeviceToHost, a->stream));
  KHIP_TRY_HIP(hipMemcpyAsync(out_max, last, 8, hipMemcpyDeviceToHost, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  return KHIP_OK;
}

khip_status khip_agg_lost_windows(khip_agg* a, const khip_batch* b, int64_t seed, int64_t* ranges, int64_t capacity,
                                  int64_t* n_ranges) {
  clear_error();
  if (!a || !b || !n_ranges || (b->n_rows > 0 && !b->ts)) return fail(KHIP_E_INVALID, "null argument");
  if (b->n_rows < 0) return fail(KHIP_E_INVALID, "batch shape");
  if (!a->windowed || a->engine == 2 || a->desc.emit != KHIP_EMIT_FINAL)
    return fail(KHIP_E_INVALID, "lost windows: an EMIT FINAL TUMBLING / HOPPING aggregation");
  DeviceGuard g(a->device);
  const int64_t n = b->n_rows;
  *n_ranges = 0;
  if (n == 0) return KHIP_OK;
  const int64_t* ts = b->ts;
  const uint8_t *kv = b->key_valid, *rv = b->row_valid;
  const size_t bm = (size_t)(n + 7) / 8;
  if (b->mem == KHIP_MEM_HOST) {
    KHIP_TRY(stage(a, a->st_ts, b->ts, n * 8));
    ts = a->st_ts.as<int64_t>();
    if (kv) { KHIP_TRY(stage(a, a->st_kv, kv, bm)); kv = a->st_kv.as<uint8_t>(); }
    if (rv) { KHIP_TRY(stage(a, a->st_rv, rv, bm)); rv = a->st_rv.as<uint8_t>(); }
  } else if (b->mem != KHIP_MEM_DEVICE) {
    return fail(KHIP_E_INVALID, "batch mem");
  }
  const int64_t sd = seed < -1 ? -1 : seed;
  KHIP_TRY(emit_final_lost(a, ts, kv, rv, n, sd, nullptr));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  const std::vector<int64_t> keep = a->lost;  // (the handle's own last push)
  KHIP_TRY(finish_lost_seed(a, ts, kv, rv, n, sd));
  std::vector<int64_t> got;
  got.swap(a->lost);
  a->lost = keep;
  *n_ranges = (int64_t)got.size() / 2;
  if (*n_ranges > capacity || (*n_ranges > 0 && !ranges)) return fail(KHIP_E_BUFFER, "ranges capacity");
  std::copy(got.begin(), got.end(), ranges);
  return KHIP_OK;
}

khip_status khip_agg_supplied_close(khip_agg* a, int64_t st_before, int64_t st_after, const int64_t* ranges,
                                    int64_t n_ranges) {
  clear_error();
  if (!a || n_ranges < 0 || (n_ranges > 0 && !ranges)) return fail(KHIP_E_INVALID, "null argument");
  if (a->desc.time_domain != KHIP_TIME_SUPPLIED) return fail(KHIP_E_INVALID, "handle not KHIP_TIME_SUPPLIED");
  if (st_after < st_before) return fail(KHIP_E_INVALID, "stream time after the batch below the one before");
  std::vector<std::pair<int64_t, int64_t>> r((size_t)n_ranges);
  for (int64_t k = 0; k < n_ranges; k++) {
    if (ranges[2 * k] > ranges[2 * k + 1]) return fail(KHIP_E_INVALID, "lost range with lo > hi");
    r[k] = {ranges[2 * k], ranges[2 * k + 1]};
  }
  a->sup_lost = merge_ranges(std::move(r));
  a->sup_before = st_before < -1 ? -1 : st_before;
  a->sup_after = st_after < -1 ? -1 : st_after;
  a->sup_set = true;
  return KHIP_OK;
}

// No row of the table has expired (retention) yet: every group counted in occ is visible.  The
// partitioned engine purges its closed store after every push; its live rows satisfy
// ws + size > (stream time before the last push) - grace, so they are all visible while that
// bound is at or above the first visible window start.  The atomic engine keeps every row.
static bool no_expired_live(const khip_agg* a) {
  if (a->engine == 2) return true;  // the session store drops expired sessions at every push
  if (a->desc.time_domain == KHIP_TIME_PARTITION && a->windowed) {  // no task has expired a window
    for (int64_t t : a->pst_host)
      if (partition_vis_from(a, t) != INT64_MIN) return false;
    return true;
  }
  const int64_t vf = visible_from(a);
  if (vf == INT64_MIN) return true;
  if (a->engine != 0 || a->st_before < 0) return false;
  return vf <= a->st_before - a->grace - a->desc.size_ms + 1;
}

static khip_status compact_rows(khip_agg* a, const khip_having* h, std::vector<uint64_t>* rows, int64_t* count,
                                const HavingDev* pull = nullptr) {
  HavingDev hd{};
  if (pull) hd = *pull;
  if (a->windowed && !hd.fin && a->engine != 2) {  // the store: expired windows are gone (retention)
    hd.vis = 1;
    hd.vis_from = visible_from(a);
  }
  hd.session = a->engine == 2;
  KHIP_TRY(partition_bounds(a, hd));  // PARTITION: each row's retention / EMIT FINAL bounds are its task's
  if (h) {
    if (h->agg_index < 0 || h->agg_index >= a->desc.n_aggs) return fail(KHIP_E_INVALID, "having agg index");
    if (h->op < KHIP_OP_GT || h->op > KHIP_OP_NE) return fail(KHIP_E_INVALID, "having op");
    hd.active = 1;
    hd.op = h->op;
    hd.a = a->outs[h->agg_index];
    hd.i64 = h->i64;
    hd.f64 = h->f64;
  }
  if (a->engine == 0) {
    KHIP_TRY(part_compact(a, hd, rows, count));
    if (rows && *count > a->occ) return fail(KHIP_E_STATE, "group count bookkeeping mismatch");
    return KHIP_OK;
  }
  // global-atomic table, or the SESSION store (a flat row array)
  const uint64_t* src = a->engine == 2 ? a->sess.rows.as<uint64_t>() : a->table.as<uint64_t>();
  const int64_t nsrc = a->engine == 2 ? a->sess.n : a->cap;
  DevBuf ctr, out;
  KHIP_TRY(ctr.ensure(8));
  KHIP_TRY_HIP(hipMemsetAsync(ctr.p, 0, 8, a->stream));
  const int grid = grid_for(std::max<int64_t>(nsrc, 1), 256, 4096);
  if (rows) KHIP_TRY(out.ensure((size_t)std::max<int64_t>(a->occ, 1) * a->sw * 8));
  if (nsrc)
    hipLaunchKernelGGL(k_compact, dim3(grid), dim3(256), 0, a->stream, src, nsrc, a->sw, hd,
                       rows ? out.as<uint64_t>() : nullptr, std::max<int64_t>(a->occ, 1), ctr.as<unsigned long long>());
  KHIP_TRY_HIP(hipGetLastError());
  int64_t n = 0;
  KHIP_TRY_HIP(hipMemcpyAsync(&n, ctr.p, 8, hipMemcpyDeviceToHost, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  *count = n;
  if (rows && n > a->occ) return fail(KHIP_E_STATE, "group count bookkeeping mismatch");
  if (rows) {
    rows->resize((size_t)n * a->sw);
    if (n) KHIP_TRY_HIP(hipMemcpy(rows->data(), out.p, (size_t)n * a->sw * 8, hipMemcpyDeviceToHost));
  }
  ctr.release();
  out.release();
  return KHIP_OK;
}

khip_status khip_agg_count_rows(khip_agg* a, const khip_having* h, int64_t* n) {
  clear_error();
  if (!a || !n) return fail(KHIP_E_INVALID, "null argument");
  DeviceGuard g(a->device);
  // every row while none has expired: the group count every engine maintains, no table scan
  if (!h && no_expired_live(a)) {
    *n = a->occ;
    return KHIP_OK;
  }
  // the query's own HAVING: counts maintained by the aggregate kernel, no table scan
  if (h && a->engine == 0 && a->desc.has_having && h->agg_index == a->desc.having.agg_index &&
      h->op == a->desc.having.op && h->i64 == a->desc.having.i64 &&
      (h->f64 == a->desc.having.f64 || (h->f64 != h->f64 && a->desc.having.f64 != a->desc.having.f64)) &&
      no_expired_live(a) && part_having_count(a, n))
    return KHIP_OK;
  return compact_rows(a, h, nullptr, n);
}

// The host copy of a UTF8 handle's arena: an id's key length (an inline id's is in the id).
static khip_status arena_host(khip_agg* a, std::vector<uint8_t>* arena) {
  arena->resize(a->dict.arena_used);
  if (a->dict.arena_used)
    KHIP_TRY_HIP(hipMemcpy(arena->data(), a->dict.arena.p, a->dict.arena_used, hipMemcpyDeviceToHost));
  return KHIP_OK;
}
static int64_t kid_len(const std::vector<uint8_t>& arena, int64_t kid) {
  return kid_inline(kid) ? (kid >> 57) & 31 : *(const int64_t*)(arena.data() + kid + 8);
}

khip_status khip_agg_snapshot_size(khip_agg* a, int64_t* n_rows, int64_t* key_bytes) {
  clear_error();
  if (!a) return fail(KHIP_E_INVALID, "null argument");
  DeviceGuard g(a->device);
  if (n_rows) {
    *n_rows = a->occ;
    if (!no_expired_live(a)) KHIP_TRY(compact_rows(a, nullptr, nullptr, n_rows));
  }
  if (key_bytes) {
    if (a->desc.key_type == KHIP_KEY_UTF8) {
      std::vector<uint64_t> rows;
      int64_t n = 0;
      KHIP_TRY(compact_rows(a, nullptr, &rows, &n));
      std::vector<uint8_t> arena;
      KHIP_TRY(arena_host(a, &arena));
      int64_t kb = 0;
      for (int64_t r = 0; r < n; r++) kb += kid_len(arena, (int64_t)rows[r * a->sw]);
      *key_bytes = kb;
    } else {
      *key_bytes = 0;
    }
  }
  return KHIP_OK;
}

// Sort compacted rows by (key, window start) and write them to the caller's snapshot buffers
// (ResultTransformer map() + WindowBoundsPopulator).
static khip_status emit_snapshot(khip_agg* a, const std::vector<uint64_t>& rows, int64_t n, khip_snapshot* out,
                                 const std::vector<uint8_t>* tomb_in = nullptr, uint8_t* tomb_out = nullptr) {
  const int sw = a->sw;
  const bool utf8 = a->desc.key_type == KHIP_KEY_UTF8;
  // UTF8: each row's key bytes — its arena entry, or its inline id's digits (decoded once per row)
  std::vector<uint8_t> arena, inl;
  std::vector<const uint8_t*> kp;
  std::vector<int64_t> kl;
  if (utf8) {
    KHIP_TRY(arena_host(a, &arena));
    int64_t ni = 0;
    for (int64_t r = 0; r < n; r++) ni += kid_inline((int64_t)rows[r * sw]) ? 1 : 0;
    inl.resize((size_t)ni * KEY_INLINE_MAX);
    kp.resize(n);
    kl.resize(n);
    ni = 0;
    for (int64_t r = 0; r < n; r++) {
      const int64_t kid = (int64_t)rows[r * sw];
      if (kid_inline(kid)) {
        uint8_t* o = inl.data() + ni++ * KEY_INLINE_MAX;
        kl[r] = kid_inline_bytes(kid, o);
        kp[r] = o;
      } else {
        kl[r] = *(const int64_t*)(arena.data() + kid + 8);
        kp[r] = arena.data() + kid + 16;
      }
    }
  }
  std::vector<int64_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  const bool session = a->engine == 2;
  std::sort(order.begin(), order.end(), [&](int64_t x, int64_t y) {
    const int64_t kx = (int64_t)rows[x * sw], ky = (int64_t)rows[y * sw];
    if (kx != ky) {
      if (!utf8) return kx < ky;
      const int64_t lx = kl[x], ly = kl[y];
      const int c = memcmp(kp[x], kp[y], (size_t)std::min(lx, ly));
      if (c) return c < 0;
      if (lx != ly) return lx < ly;
    }
    if (session && tomb_in && (*tomb_in)[x] != (*tomb_in)[y]) return (*tomb_in)[x] > (*tomb_in)[y];  // deletes first
    if (rows[x * sw + 1] != rows[y * sw + 1]) return (int64_t)rows[x * sw + 1] < (int64_t)rows[y * sw + 1];
    return (int64_t)rows[x * sw + 2] < (int64_t)rows[y * sw + 2];
  });
  if (n > out->capacity) {
    out->n_rows = n;
    return fail(KHIP_E_BUFFER, "snapshot capacity too small");
  }
  int64_t kb = 0;
  if (utf8 && out->key_offsets) out->key_offsets[0] = 0;
  for (int64_t r = 0; r < n; r++) {
    const uint64_t* s = &rows[order[r] * sw];
    const int64_t key = (int64_t)s[0], ws = (int64_t)s[1];
    if (tomb_out) tomb_out[r] = tomb_in ? (*tomb_in)[order[r]] : 0;
    if (utf8) {
      const int64_t len = kl[order[r]];
      if (kb + len > out->key_bytes_capacity) return fail(KHIP_E_BUFFER, "snapshot key bytes capacity too small");
      if (out->key_bytes && len) memcpy(out->key_bytes + kb, kp[order[r]], (size_t)len);
      kb += len;
      if (out->key_offsets) out->key_offsets[r + 1] = kb;
    } else if (out->key_i64) {
      out->key_i64[r] = key;
    }
    if (out->window_start) out->window_start[r] = a->windowed ? ws : 0;
    if (out->window_end) out->window_end[r] = a->windowed ? (session ? (int64_t)s[2] : ws + a->desc.size_ms) : 0;
    if (out->rowtime) out->rowtime[r] = (int64_t)s[2];
    for (int i = 0; i < a->desc.n_aggs; i++) {
      const AggOut& o = a->outs[i];
      int64_t iv = 0;
      double dv = 0.0;
      bool isnull = false;
      switch (o.kind) {
        case KHIP_AGG_COUNT_STAR:
        case KHIP_AGG_COUNT: iv = (int64_t)s[o.w_val]; break;
        case KHIP_AGG_SUM:
          if (o.type == KHIP_TYPE_DOUBLE) memcpy(&dv, &s[o.w_val], 8);
          else iv = (int64_t)s[o.w_val];
          break;
        case KHIP_AGG_MIN:
        case KHIP_AGG_MAX:
          if ((int64_t)s[o.w_cnt] == 0) isnull = true;
          else if (o.type == KHIP_TYPE_DOUBLE) dv = f64_from_order_key((int64_t)s[o.w_val]);
          else iv = (int64_t)s[o.w_val];
          break;
        case KHIP_AGG_AVG: {
          const int64_t c = (int64_t)s[o.w_cnt];
          if (c == 0) dv = 0.0;
          else if (o.type == KHIP_TYPE_DOUBLE) { double sum; memcpy(&sum, &s[o.w_val], 8); dv = sum / (double)c; }
          else if (o.type == KHIP_TYPE_INT32) dv = (double)(int32_t)s[o.w_val] / (double)c;
          else dv = (double)(int64_t)s[o.w_val] / (double)c;
          break;
        }
      }
      int32_t rt;
      khip_agg_result_type(&a->desc, i, &rt);
      if (out->agg_values && out->agg_values[i]) {
        if (rt == KHIP_TYPE_INT32) ((int32_t*)out->agg_values[i])[r] = isnull ? 0 : (int32_t)iv;
        else if (rt == KHIP_TYPE_INT64) ((int64_t*)out->agg_values[i])[r] = isnull ? 0 : iv;
        else ((double*)out->agg_values[i])[r] = isnull ? 0.0 : dv;
      }
      if (out->agg_null && out->agg_null[i]) out->agg_null[i][r] = isnull ? 1 : 0;
    }
  }
  out->n_rows = n;
  out->key_bytes_len = kb;
  return KHIP_OK;
}

khip_status khip_agg_snapshot(khip_agg* a, const khip_having* h, khip_snapshot* out) {
  clear_error();
  if (!a || !out) return fail(KHIP_E_INVALID, "null argument");
  DeviceGuard g(a->device);
  std::vector<uint64_t> rows;
  int64_t n = 0;
  KHIP_TRY(compact_rows(a, h, &rows, &n));
  return emit_snapshot(a, rows, n, out);
}

khip_status khip_agg_get(khip_agg* a, const khip_pull* q, const khip_having* h, khip_snapshot* out) {
  clear_error();
  if (!a || !q || !out) return fail(KHIP_E_INVALID, "null argument");
  if (q->n_keys < 0 || (q->n_keys > 0 && a->desc.key_type == KHIP_KEY_INT64 && !q->keys))
    return fail(KHIP_E_INVALID, "pull keys");
  const bool utf8 = a->desc.key_type == KHIP_KEY_UTF8;
  if (q->n_keys > 0 && utf8 && (!q->key_offsets || !q->key_bytes || q->key_offsets[0] != 0))
    return fail(KHIP_E_INVALID, "pull UTF8 keys need key_offsets (from 0) and key_bytes");
  DeviceGuard g(a->device);
  HavingDev pd{};
  pd.pull = 1;
  pd.pull_windowed = a->windowed;
  pd.ws_lo = q->ws_lo;
  pd.ws_hi = q->ws_hi;
  pd.we_lo = q->we_lo;
  pd.we_hi = q->we_hi;
  pd.size_ms = a->desc.size_ms;
  DevBuf dkeys;
  std::vector<int64_t> k;  // outlives the copy: compact_rows synchronises the stream
  if (q->n_keys > 0 && utf8) {
    // key bytes → dictionary ids on the device (read-only probe; digit keys: their inline ids);
    // unseen keys match nothing
    const int64_t nk = q->n_keys, nb = q->key_offsets[nk];
    k.assign((size_t)nk, -1);
    {
      DevBuf doff, dbytes, dkid;
      KHIP_TRY(doff.ensure((size_t)(nk + 1) * 8));
      KHIP_TRY(dbytes.ensure((size_t)std::max<int64_t>(nb, 1)));
      KHIP_TRY(dkid.ensure((size_t)nk * 8));
      KHIP_TRY_HIP(hipMemcpyAsync(doff.p, q->key_offsets, (size_t)(nk + 1) * 8, hipMemcpyHostToDevice, a->stream));
      if (nb) KHIP_TRY_HIP(hipMemcpyAsync(dbytes.p, q->key_bytes, (size_t)nb, hipMemcpyHostToDevice, a->stream));
      KHIP_TRY(dict_find(a->dict, a->stream, doff.as<int64_t>(), dbytes.as<uint8_t>(), nk, dkid.as<int64_t>()));
      KHIP_TRY_HIP(hipMemcpyAsync(k.data(), dkid.p, (size_t)nk * 8, hipMemcpyDeviceToHost, a->stream));
      KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
    }
    std::sort(k.begin(), k.end());
    k.erase(std::unique(k.begin(), k.end()), k.end());
    if (k.size() > 1 && k[0] == -1) k.erase(k.begin());  // -1 (unseen) never matches a row
    KHIP_TRY(dkeys.ensure(k.size() * 8));
    KHIP_TRY_HIP(hipMemcpyAsync(dkeys.p, k.data(), k.size() * 8, hipMemcpyHostToDevice, a->stream));
    pd.keys = dkeys.as<int64_t>();
    pd.n_keys = (int64_t)k.size();
  } else if (q->n_keys > 0) {
    k.assign(q->keys, q->keys + q->n_keys);
    std::sort(k.begin(), k.end());
    k.erase(std::unique(k.begin(), k.end()), k.end());
    KHIP_TRY(dkeys.ensure(k.size() * 8));
    KHIP_TRY_HIP(hipMemcpyAsync(dkeys.p, k.data(), k.size() * 8, hipMemcpyHostToDevice, a->stream));
    pd.keys = dkeys.as<int64_t>();
    pd.n_keys = (int64_t)k.size();
  }
  if (pd.n_keys > 0) pd.host_keys = k.data();
  std::vector<uint64_t> rows;
  int64_t n = 0;
  KHIP_TRY(compact_rows(a, h, &rows, &n, &pd));
  return emit_snapshot(a, rows, n, out);
}

// The rows the last push emitted (khip_agg_changes), computed once per push on first request.
static khip_status compute_changes(khip_agg* a) {
  if (a->chg_ready) return KHIP_OK;
  a->chg_rows.clear();
  a->chg_tomb.clear();
  a->chg_n = 0;
  if (a->desc.emit == KHIP_EMIT_FINAL && a->engine == 2) {
    // the sessions the push closed (sess_push: k_sess_apply / k_sess_keep)
    KHIP_TRY(sess_changes(a, &a->chg_rows, &a->chg_tomb, &a->chg_n));
  } else if (a->desc.emit == KHIP_EMIT_FINAL) {
    // windows closed by the push and still visible when they closed, passing HAVING
    HavingDev fd{};
    fd.fin = 1;
    fd.fin_c0 = a->st_before - a->grace;
    fd.fin_c1 = a->host_stream_time - a->grace;
    fd.fin_size = a->desc.size_ms;
    if (a->desc.time_domain == KHIP_TIME_PARTITION) {
      // per task (partition_bounds): a row closes when ITS partition's stream time passes its end;
      // a row whose key is not in the map closes nowhere
      fd.fin_c0 = fd.fin_c1 = 0;
      bool moved = false;
      for (size_t p = 0; p < a->pst_host.size(); p++) moved = moved || a->pst_host[p] > a->pst_prev_host[p];
      if (moved) fd.fin_c1 = 1;  // (only gates the compaction below)
    }
    DevBuf dl;
    if (!a->lost.empty()) {
      KHIP_TRY(dl.ensure(a->lost.size() * 8));
      KHIP_TRY_HIP(hipMemcpyAsync(dl.p, a->lost.data(), a->lost.size() * 8, hipMemcpyHostToDevice, a->stream));
      fd.lost = dl.as<int64_t>();
      fd.n_lost = (int32_t)(a->lost.size() / 2);
    }
    if (fd.fin_c1 > fd.fin_c0) {
      if (a->desc.time_domain == KHIP_TIME_PARTITION) fd.fin_c1 = 0;
      KHIP_TRY(compact_rows(a, a->desc.has_having ? &a->desc.having : nullptr, &a->chg_rows, &a->chg_n, &fd));
    }
    a->chg_tomb.assign((size_t)a->chg_n, 0);
  } else if (a->changelog && a->engine == 2) {
    KHIP_TRY(sess_changes(a, &a->chg_rows, &a->chg_tomb, &a->chg_n));
  } else if (a->changelog) {
    KHIP_TRY(part_changes(a, &a->chg_rows, &a->chg_tomb, &a->chg_n));
  } else {
    return fail(KHIP_E_STATE, "handle created without KHIP_FLAG_CHANGELOG (EMIT CHANGES)");
  }
  a->chg_ready = true;
  return KHIP_OK;
}

khip_status khip_agg_changes_size(khip_agg* a, int64_t* n_rows, int64_t* key_bytes) {
  clear_error();
  if (!a) return fail(KHIP_E_INVALID, "null argument");
  DeviceGuard g(a->device);
  KHIP_TRY(compute_changes(a));
  if (n_rows) *n_rows = a->chg_n;
  if (key_bytes) {
    int64_t kb = 0;
    if (a->desc.key_type == KHIP_KEY_UTF8 && a->chg_n) {
      std::vector<uint8_t> arena;
      KHIP_TRY(arena_host(a, &arena));
      for (int64_t r = 0; r < a->chg_n; r++) kb += kid_len(arena, (int64_t)a->chg_rows[r * a->sw]);
    }
    *key_bytes = kb;
  }
  return KHIP_OK;
}

khip_status khip_agg_changes(khip_agg* a, khip_snapshot* out, uint8_t* tombstone) {
  clear_error();
  if (!a || !out) return fail(KHIP_E_INVALID, "null argument");
  DeviceGuard g(a->device);
  KHIP_TRY(compute_changes(a));
  return emit_snapshot(a, a->chg_rows, a->chg_n, out, &a->chg_tomb, tombstone);
}

khip_status khip_agg_reset(khip_agg* a) {
  clear_error();
  if (!a) return fail(KHIP_E_INVALID, "null argument");
  DeviceGuard g(a->device);
  a->chg_ready = true;
  a->chg_n = 0;
  a->st_before = -1;
  a->lost.clear();
  if (a->engine == 0) {
    KHIP_TRY(part_reset(a));  // also the stream time
  } else if (a->engine == 2) {
    a->sess.n = 0;
    a->sess.nchg = 0;
    int64_t m1 = -1;
    KHIP_TRY_HIP(hipMemcpyAsync(a->stream_time.p, &m1, 8, hipMemcpyHostToDevice, a->stream));
  } else {
    hipLaunchKernelGGL(k_init_table, dim3(grid_for(a->cap * a->sw, 256)), dim3(256), 0, a->stream,
                       a->table.as<uint64_t>(), a->cap, a->sw, a->init);
    int64_t m1 = -1;
    KHIP_TRY_HIP(hipMemcpyAsync(a->stream_time.p, &m1, 8, hipMemcpyHostToDevice, a->stream));
    if (a->engine == 3) KHIP_TRY(tagg_reset(a));
  }
  if (a->desc.key_type == KHIP_KEY_UTF8) {
    KHIP_TRY(dict_clear(a->dict, a->stream));
  }
  if (a->desc.time_domain == KHIP_TIME_PARTITION) {
    KHIP_TRY_HIP(hipMemsetAsync(a->pst.p, 0xFF, (size_t)a->desc.n_partitions * 8, a->stream));
    a->pst_host.assign((size_t)a->desc.n_partitions, -1);
    a->pst_prev_host.assign((size_t)a->desc.n_partitions, -1);
    a->plost.clear();
    a->plost_off.clear();
    KHIP_TRY(pmap_clear(a));  // forget the keys' partitions (keeps the allocation)
  }
  // asynchronous on the handle's stream (every later call on the handle is ordered behind it)
  KHIP_TRY_HIP(hipGetLastError());
  a->occ = 0;
  a->host_stream_time = -1;
  return KHIP_OK;
}

khip_status khip_agg_sync(khip_agg* a) {
  if (!a) return fail(KHIP_E_INVALID, "null argument");
  DeviceGuard g(a->device);
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  return KHIP_OK;
}

khip_status khip_agg_kernel_times(khip_agg* a, khip_kernel_times* out, int32_t reset) {
  if (!a || !out) return fail(KHIP_E_INVALID, "null argument");
  if (!a->profile) return fail(KHIP_E_STATE, "handle created without KHIP_FLAG_PROFILE");
  *out = a->times;
  if (reset) a->times = khip_kernel_times{};
  return KHIP_OK;
}

khip_status khip_agg_stream(khip_agg* a, void** s) {
  if (!a || !s) return fail(KHIP_E_INVALID, "null argument");
  *s = (void*)a->stream;
  return KHIP_OK;
}

khip_status khip_agg_destroy(khip_agg* a) {
  if (!a) return KHIP_OK;
  DeviceGuard g(a->device);
  if (a->stream) hipStreamSynchronize(a->stream);
  DevBuf* bufs[] = {&a->table, &a->blockmax, &a->blockprefix, &a->partials, &a->resume, &a->counters,
                    &a->stream_time, &a->st_keys, &a->st_ts, &a->st_kv, &a->st_rv, &a->st_koff,
                    &a->st_kbytes, &a->kid, &a->khash, &a->chg, &a->lostbuf, &a->lostctr,
                    &a->pst, &a->pst2, &a->st_col, &a->st_agg, &a->st_seen, &a->st_part};
  for (DevBuf* b : bufs) b->release();
  for (int c = 0; c < MAX_COLS; c++) {
    a->st_cols[c].release();
    a->st_cval[c].release();
  }
  dict_release(a->dict);
  pmap_release(a);
  tagg_release(a);
  part_release(a);
  sess_release(a);
  for (int e = 0; e < 8; e++)
    if (a->ev[e]) hipEventDestroy(a->ev[e]);
  if (a->stream) hipStreamDestroy(a->stream);
  delete a;
  return KHIP_OK;
}

}  // extern "C"
