// khip_join.hip — stream-table join on MI355X (gfx950).
//
// Replaces the table side built by SourceBuilder.buildKTable (S/SourceBuilder.java:87-137,
// a RocksDB KV store of the latest value per key) and the per-record Kafka Streams
// KStreamKTableJoin lookup + KsqlValueJoiner.apply that StreamTableJoinBuilder.build wires
// (S/StreamTableJoinBuilder.java:38-88, S/KsqlValueJoiner.java:41-63).
//
// HBM layout: cap slots (power of two), AoS, slot_words u64 per slot:
//   [0] key  [1] meta  [2] last-writer tag  [3..] right-side columns (one word each)
//   meta: bit63 = claimed by this upsert batch (bits 0..39 = batch row),
//         bit62 = resident (key valid), bit61 = live (has a value; 0 = deleted),
//         bits 0..31 = null mask of the right columns (when resident).
//   COMPACT (one INT payload column, e.g. C4's level): 16-byte slots [0] key [1] meta with the
//   value in bits 0..31 and its NULL flag in bit 32; the last-writer tags live in a separate
//   array (read only by the upserts), so a probe's home pair is one 32-byte read.
//
// Upsert (arrival order, last writer wins, tombstone deletes):
//   k_upsert_claim   find-or-claim each key's slot (CAS on meta, claim references the
//                    batch row, new slots appended to a claimed list); atomicMax of
//                    (row + 1) into the tag word elects the last writer of the batch
//   k_upsert_finalize claimed slots only → resident keys
//   k_upsert_apply   the elected row writes value + live bit (or clears live) and zeroes
//                    the tag, so tags never carry over between batches
// Probe: one thread per stream row, coalesced key/ts loads, one slot line per probe;
// output is row-aligned (selection bitmaps built with __ballot, 8 B per wave) so no
// compaction pass is needed on the device path.
//
// Dense probe index (one INT/BIGINT value column, keys in a range at most 4x the live key
// count, e.g. C4's users 1..1e8): cell[key - kmin] of W = 1/2/4/8 bytes, bit 0 live, bit 1
// NULL value, bits 2.. value - vmin — or 2-bit cells when every value is one of three and none
// is NULL (dense_store).  C4 is 1e8 2-bit cells (25 MB): it stays in the 256 MB MALL (and more
// of it in the XCDs' L2s than the 100 MB of byte cells), so the probes' random reads are cache
// hits instead of random 64 B HBM lines into the 8.6 GB slot table.  Built from the slot table on the first probe after it became
// eligible and kept in step by the upserts' winning rows (a key or value outside the index's
// ranges drops it; the next probe rebuilds it over the new ranges).
//
// STRING-keyed tables (KHIP_KEY_UTF8): key bytes are mapped to stable ids by the device key
// dictionary (khip_dict.hpp) — inserting on upsert, read-only on probe (an unseen key is -1,
// which no slot holds) — and the slot table works on the ids.  Identity is byte equality of the
// serialized KAFKA STRING key, as in the reference (S/JoinParamsFactory.java:65-84 requires the
// two sides' key types to match; the lookup is a byte-keyed store get).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "khip_dict.hpp"
#include "khip_util.hpp"

namespace khip {

constexpr int JMAX_COLS = 16;
constexpr int JMAX_PROBE = 4096;
constexpr uint64_t M_CLAIM = 1ULL << 63;
constexpr uint64_t M_RESIDENT = 1ULL << 62;
constexpr uint64_t M_LIVE = 1ULL << 61;

struct JCols {
  const void* data[JMAX_COLS];
  const uint8_t* valid[JMAX_COLS];
};

struct JWhere {
  int32_t active;
  int32_t col;
  int32_t op;
  int32_t type;
  int64_t i64;
  double f64;
};

__device__ __forceinline__ uint64_t jld(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t key_hash(int64_t k) { return mix64((uint64_t)k ^ 0x2545F4914F6CDD1DULL); }

// A key's home slot: always the first of an aligned PAIR of slots (64 bytes for one payload
// column), so one probe's first read brings two slots of its linear-probe sequence — at the
// tables' load factor (<= 1/2) nearly every lookup ends inside its home pair.
__device__ __forceinline__ uint64_t home_slot(int64_t k, uint64_t mask) { return key_hash(k) & mask & ~1ULL; }

// Payload column c of a slot and its NULL flag, in either layout (cmp: COMPACT).
__device__ __forceinline__ uint64_t slot_col(const uint64_t* s, uint64_t meta, int c, bool cmp) {
  return cmp ? (uint64_t)(int64_t)(int32_t)(uint32_t)meta : s[3 + c];
}
__device__ __forceinline__ bool slot_null(uint64_t meta, int c, bool cmp) {
  return cmp ? ((meta >> 32) & 1ULL) != 0 : ((meta >> c) & 1ULL) != 0;
}

__global__ __launch_bounds__(256) void k_upsert_claim(uint64_t* __restrict__ table, uint64_t mask, int sw,
                                                      const int64_t* __restrict__ keys,
                                                      const uint8_t* __restrict__ kv, int64_t n,
                                                      int64_t* __restrict__ slot_of, int* __restrict__ fail,
                                                      unsigned long long* __restrict__ new_keys,
                                                      int64_t* __restrict__ claimed, uint64_t* __restrict__ tags) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    slot_of[i] = -1;
    if (!bit_get(kv, i)) continue;
    const int64_t key = keys[i];
    uint64_t slot = home_slot(key, mask);
    const uint64_t claim = M_CLAIM | (uint64_t)i;
    bool done = false;
    for (int probe = 0; probe < JMAX_PROBE && !done; probe++) {
      uint64_t* s = table + slot * (uint64_t)sw;
      uint64_t m = jld(&s[1]);
      if (m == 0) {
        const uint64_t old = atomicCAS((unsigned long long*)&s[1], 0ULL, (unsigned long long)claim);
        if (old == 0) {
          claimed[atomicAdd(new_keys, 1ULL)] = (int64_t)slot;
          done = true;
        } else {
          m = old;
        }
      }
      if (!done) {
        if (m & M_CLAIM) {
          done = keys[(int64_t)(m & ((1ULL << 40) - 1))] == key;
        } else {
          done = (int64_t)s[0] == key;
        }
      }
      if (done) {
        slot_of[i] = (int64_t)slot;
        atomicMax((unsigned long long*)(tags ? &tags[slot] : &s[2]), (unsigned long long)(i + 1));
      } else {
        slot = (slot + 1) & mask;
      }
    }
    if (!done) *fail = 1;
  }
}

__global__ __launch_bounds__(256) void k_upsert_finalize(uint64_t* __restrict__ table, int sw,
                                                         const int64_t* __restrict__ keys,
                                                         const int64_t* __restrict__ claimed,
                                                         const unsigned long long* __restrict__ n_claimed) {
  const int64_t nc = (int64_t)*n_claimed;
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nc; k += (int64_t)gridDim.x * blockDim.x) {
    uint64_t* s = table + (uint64_t)claimed[k] * (uint64_t)sw;
    const uint64_t m = s[1];
    if (m & M_CLAIM) {
      s[0] = (uint64_t)keys[(int64_t)(m & ((1ULL << 40) - 1))];
      s[1] = M_RESIDENT;  // not live until a value is written
    }
  }
}

#ifndef KHIP_JOIN_QUARTER
#define KHIP_JOIN_QUARTER 1  // 2-bit dense cells when they fit (A/B builds set 0)
#endif

// Dense probe index parameters (active = 0: none).
struct JDense {
  int32_t active;
  int32_t w;         // cell bytes: 1, 2, 4, 8; 0 = 2-bit cells (see dense_load)
  int64_t kmin, nkeys;  // cells for keys kmin .. kmin + nkeys - 1
  int64_t vmin;
  uint64_t vspan;    // values vmin .. vmin + vspan - 1 encodable
  uint8_t* cells;
  int* invalid;      // set when an upsert falls outside the ranges
};

// 2-bit cells (w = 0): 0 absent, 1 + (value - vmin) for values vmin .. vmin + 2, no NULL — C4's
// three levels over 1e8 users are 25 MB instead of 100 MB, which random gathers read at 7.1e10/s
// instead of 5.7e10/s (more of the index hits each XCD's L2; profiles/r06/random_gather_c4_index.csv).
// Sixteen cells share a 32-bit word, so stores are word atomics (one writer per key, never per word).
__device__ __forceinline__ void dense_store(const JDense& d, int64_t idx, uint64_t cell) {
  switch (d.w) {
    case 0: {
      unsigned int* wd = (unsigned int*)d.cells + (idx >> 4);
      const int sh = 2 * (int)(idx & 15);
      const unsigned int c2 = (cell & 1) ? (unsigned int)(cell >> 2) + 1u : 0u;
      atomicAnd(wd, ~(3u << sh));
      if (c2) atomicOr(wd, c2 << sh);
      break;
    }
    case 1: d.cells[idx] = (uint8_t)cell; break;
    case 2: ((uint16_t*)d.cells)[idx] = (uint16_t)cell; break;
    case 4: ((uint32_t*)d.cells)[idx] = (uint32_t)cell; break;
    default: ((uint64_t*)d.cells)[idx] = cell; break;
  }
}

// The cell in the common format (bit 0 live, bit 1 NULL, bits 2.. value - vmin).
__device__ __forceinline__ uint64_t dense_load(const JDense& d, int64_t idx) {
  switch (d.w) {
    case 0: {
      const uint64_t c2 = (d.cells[idx >> 2] >> (2 * (int)(idx & 3))) & 3;
      return c2 ? (1 | ((c2 - 1) << 2)) : 0;
    }
    case 1: return d.cells[idx];
    case 2: return ((const uint16_t*)d.cells)[idx];
    case 4: return ((const uint32_t*)d.cells)[idx];
    default: return ((const uint64_t*)d.cells)[idx];
  }
}

// The cell of a live key (value word raw, NULL flag) — false if it does not fit the index.
__device__ __forceinline__ bool dense_cell(const JDense& d, uint64_t raw, bool isnull, uint64_t* cell) {
  if (isnull) {
    *cell = 3;
    return d.w != 0;  // 2-bit cells hold no NULL
  }
  const uint64_t off = (uint64_t)((int64_t)raw - d.vmin);
  if ((int64_t)raw < d.vmin || off >= d.vspan) return false;
  *cell = 1 | (off << 2);
  return true;
}

// Hashed probe index (one INT/BIGINT value column whose keys are too spread for the dense one,
// e.g. C4 --sparse-ids: user ids over 2^40): open addressing over 8-byte words
// [(key - kmin) << cb | cell] (cell as the dense index's, cb bits; EMPTY = all ones; a deleted key
// keeps its word with cell 0).  A key's home is the first word of an aligned pair, so a lookup is
// ONE 16-byte read — the slot table's compact pair is two (32 bytes) — and the index is a quarter
// of the slot table.  Built like the dense index, kept in step by the upserts' winning rows.
struct JHix {
  int32_t active;
  int32_t cb;            // cell bits
  int64_t kmin;
  uint64_t krel_max;     // keys kmin .. kmin + krel_max - 1 encodable
  uint64_t mask;         // words - 1 (a power of two >= 2)
  int64_t vmin;
  uint64_t vspan;        // values vmin .. vmin + vspan - 1 encodable
  uint64_t* words;
  int* invalid;          // set when a key / value falls outside the ranges or a probe runs long
};
constexpr uint64_t HIX_EMPTY = ~0ULL;
constexpr int HIX_PROBE = 512;

__device__ __forceinline__ uint64_t hix_home(int64_t k, uint64_t mask) { return key_hash(k) & mask & ~1ULL; }

// Insert or overwrite key k's cell (one writer per key at a time); false when the probe ran long.
__device__ __forceinline__ bool hix_put(const JHix& h, int64_t k, uint64_t cell) {
  const uint64_t krel = (uint64_t)(k - h.kmin);
  const uint64_t word = (krel << h.cb) | cell;
  uint64_t d = hix_home(k, h.mask);
  for (int probe = 0; probe < HIX_PROBE; probe++) {
    uint64_t w = __hip_atomic_load(&h.words[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (w == HIX_EMPTY) {
      w = atomicCAS((unsigned long long*)&h.words[d], (unsigned long long)HIX_EMPTY, (unsigned long long)word);
      if (w == HIX_EMPTY) return true;
    }
    if ((w >> h.cb) == krel) {
      __hip_atomic_store(&h.words[d], word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return true;
    }
    d = (d + 1) & h.mask;
  }
  return false;
}

// Key k of the upsert's winning row → its index cell (cell 0: deleted); any miss of the ranges
// invalidates the index (rebuilt over the new ranges by the next probe).
__device__ __forceinline__ void hix_update(const JHix& h, int64_t k, bool del, uint64_t raw, bool isnull) {
  if (!h.active) return;
  const uint64_t krel = (uint64_t)(k - h.kmin);
  uint64_t cell = 0;
  bool ok = k >= h.kmin && krel < h.krel_max;
  if (ok && !del) {
    if (isnull) {
      cell = 3;
    } else {
      const uint64_t off = (uint64_t)((int64_t)raw - h.vmin);
      ok = (int64_t)raw >= h.vmin && off < h.vspan;
      cell = 1 | (off << 2);
    }
  }
  if (!ok || !hix_put(h, k, cell)) *h.invalid = 1;
}

__global__ __launch_bounds__(256) void k_upsert_apply(uint64_t* __restrict__ table, int sw,
                                                      const int64_t* __restrict__ slot_of,
                                                      const uint8_t* __restrict__ rv, int64_t n, int ncols, const int32_t* __restrict__ types_dev, JCols cols,
                                                      JDense dn, uint64_t* __restrict__ tags, JHix hx) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t slot = slot_of[i];
    if (slot < 0) continue;
    uint64_t* s = table + slot * (uint64_t)sw;
    uint64_t* tg = tags ? &tags[slot] : &s[2];
    if (*tg != (uint64_t)(i + 1)) continue;  // not the last writer of this key
    *tg = 0;  // only the winner matches: clearing cannot change another row's decision
    const int64_t kidx = (int64_t)s[0] - dn.kmin;
    const bool kin = dn.active && (int64_t)s[0] >= dn.kmin && kidx < dn.nkeys;
    if (dn.active && !kin) *dn.invalid = 1;
    if (!bit_get(rv, i)) {
      s[1] = M_RESIDENT;  // tombstone: delete
      if (kin) dense_store(dn, kidx, 0);
      hix_update(hx, (int64_t)s[0], true, 0, false);
      continue;
    }
    if (tags) {  // COMPACT: the INT value in the meta word
      const bool v = bit_get(cols.valid[0], i);
      const int32_t x = v ? ((const int32_t*)cols.data[0])[i] : 0;
      s[1] = M_RESIDENT | M_LIVE | (v ? (uint64_t)(uint32_t)x : (1ULL << 32));
      if (kin) {
        uint64_t cell;
        if (dense_cell(dn, (uint64_t)(int64_t)x, !v, &cell)) dense_store(dn, kidx, cell);
        else *dn.invalid = 1;
      }
      hix_update(hx, (int64_t)s[0], false, (uint64_t)(int64_t)x, !v);
      continue;
    }
    uint64_t nullmask = 0;
    for (int c = 0; c < ncols; c++) {
      const bool v = bit_get(cols.valid[c], i);
      uint64_t w = 0;
      if (v) {
        if (types_dev[c] == KHIP_TYPE_INT32) w = (uint64_t)(int64_t)((const int32_t*)cols.data[c])[i];
        else w = ((const uint64_t*)cols.data[c])[i];
      } else {
        nullmask |= 1ULL << c;
      }
      s[3 + c] = w;
    }
    s[1] = M_RESIDENT | M_LIVE | nullmask;
    if (kin) {
      uint64_t cell;
      if (dense_cell(dn, s[3], nullmask & 1, &cell)) dense_store(dn, kidx, cell);
      else *dn.invalid = 1;
    }
    hix_update(hx, (int64_t)s[0], false, s[3], nullmask & 1);
  }
}

// Ranges of the live slots: [kmin, kmax, vmin, vmax, live] (value over non-null values).
__global__ __launch_bounds__(256) void k_table_ranges(const uint64_t* __restrict__ table, int64_t cap, int sw,
                                                      unsigned long long* __restrict__ out, int cmp) {
  int64_t kmn = INT64_MAX, kmx = INT64_MIN, vmn = INT64_MAX, vmx = INT64_MIN, live = 0, nulls = 0;
  for (int64_t slot = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; slot < cap;
       slot += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t* s = table + slot * (uint64_t)sw;
    const uint64_t m = s[1];
    if (!(m & M_LIVE)) continue;
    const int64_t k = (int64_t)s[0];
    kmn = k < kmn ? k : kmn;
    kmx = k > kmx ? k : kmx;
    live++;
    if (!slot_null(m, 0, cmp)) {
      const int64_t v = (int64_t)slot_col(s, m, 0, cmp);
      vmn = v < vmn ? v : vmn;
      vmx = v > vmx ? v : vmx;
    } else {
      nulls++;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const int64_t a = __shfl_xor(kmn, off, 64), b = __shfl_xor(kmx, off, 64), c = __shfl_xor(vmn, off, 64),
                  d = __shfl_xor(vmx, off, 64);
    kmn = a < kmn ? a : kmn;
    kmx = b > kmx ? b : kmx;
    vmn = c < vmn ? c : vmn;
    vmx = d > vmx ? d : vmx;
    live += __shfl_xor(live, off, 64);
    nulls += __shfl_xor(nulls, off, 64);
  }
  if ((threadIdx.x & 63) == 0 && live) {
    // order-preserving unsigned view of the signed ranges for the 64-bit atomics
    const uint64_t bias = 1ULL << 63;
    atomicMin(&out[0], (unsigned long long)((uint64_t)kmn ^ bias));
    atomicMax(&out[1], (unsigned long long)((uint64_t)kmx ^ bias));
    atomicMin(&out[2], (unsigned long long)((uint64_t)vmn ^ bias));
    atomicMax(&out[3], (unsigned long long)((uint64_t)vmx ^ bias));
    atomicAdd(&out[4], (unsigned long long)live);
    if (nulls) atomicAdd(&out[5], (unsigned long long)nulls);
  }
}

// Fill the dense index from the live slots (cells of absent keys were zeroed).
__global__ __launch_bounds__(256) void k_dense_build(const uint64_t* __restrict__ table, int64_t cap, int sw, JDense dn,
                                                     int cmp) {
  for (int64_t slot = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; slot < cap;
       slot += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t* s = table + slot * (uint64_t)sw;
    const uint64_t m = s[1];
    if (!(m & M_LIVE)) continue;
    uint64_t cell;
    if (dense_cell(dn, slot_col(s, m, 0, cmp), slot_null(m, 0, cmp), &cell)) dense_store(dn, (int64_t)s[0] - dn.kmin, cell);
    else *dn.invalid = 1;
  }
}

// Fill the hashed index from the live slots (words start EMPTY).
__global__ __launch_bounds__(256) void k_hix_build(const uint64_t* __restrict__ table, int64_t cap, int sw, JHix hx,
                                                   int cmp) {
  for (int64_t slot = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; slot < cap;
       slot += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t* s = table + slot * (uint64_t)sw;
    const uint64_t m = s[1];
    if (!(m & M_LIVE)) continue;
    hix_update(hx, (int64_t)s[0], false, slot_col(s, m, 0, cmp), slot_null(m, 0, cmp));
  }
}

__device__ __forceinline__ bool where_ok(const uint64_t* s, uint64_t meta, const JWhere& w) {
  if (!w.active) return true;
  if (meta & (1ULL << w.col)) return false;  // NULL never satisfies
  const uint64_t raw = s[3 + w.col];
  int c;
  if (w.type == KHIP_TYPE_DOUBLE) {
    double d;
    __builtin_memcpy(&d, &raw, 8);
    if (d != d) return w.op == KHIP_OP_NE;
    c = d < w.f64 ? -1 : (d > w.f64 ? 1 : 0);
  } else {
    const int64_t v = (int64_t)raw;
    c = v < w.i64 ? -1 : (v > w.i64 ? 1 : 0);
  }
  switch (w.op) {
    case KHIP_OP_GT: return c > 0;
    case KHIP_OP_GE: return c >= 0;
    case KHIP_OP_LT: return c < 0;
    case KHIP_OP_LE: return c <= 0;
    case KHIP_OP_EQ: return c == 0;
    case KHIP_OP_NE: return c != 0;
  }
  return false;
}

constexpr int JCTR = 64;  // emitted-row counters of a probe (khip_table_probe_device)

struct JOut {
  uint8_t* emit;
  uint8_t* matched;
  void* col_data[JMAX_COLS];
  uint8_t* col_null[JMAX_COLS];
  int64_t* slot_out;  // host path: -1 not emitted, 0 emitted miss, slot + 1 emitted hit
};

__device__ __forceinline__ bool where_ok_raw(uint64_t raw, uint64_t meta, const JWhere& w, bool cmp = false) {
  if (!w.active) return true;
  if (slot_null(meta, w.col, cmp)) return false;  // NULL never satisfies
  int c;
  if (w.type == KHIP_TYPE_DOUBLE) {
    double d;
    __builtin_memcpy(&d, &raw, 8);
    if (d != d) return w.op == KHIP_OP_NE;
    c = d < w.f64 ? -1 : (d > w.f64 ? 1 : 0);
  } else {
    const int64_t v = (int64_t)raw;
    c = v < w.i64 ? -1 : (v > w.i64 ? 1 : 0);
  }
  switch (w.op) {
    case KHIP_OP_GT: return c > 0;
    case KHIP_OP_GE: return c >= 0;
    case KHIP_OP_LT: return c < 0;
    case KHIP_OP_LE: return c <= 0;
    case KHIP_OP_EQ: return c == 0;
    case KHIP_OP_NE: return c != 0;
  }
  return false;
}

// PR stream rows per thread (row = block base + r * 256 + thread, so for every r a wave
// covers 64 consecutive rows and its bitmaps are one 8-byte store).  The home slot of all
// PR rows (32 bytes: key, meta, tag, first column — one line) is loaded before any is
// examined, so a wave keeps 4 x PR independent HBM reads in flight: the table is far larger
// than the caches and every probe is a random line, so the kernel is latency/MLP-bound.
template <int PR, bool CMP>
__global__ __launch_bounds__(256) void k_probe(const uint64_t* __restrict__ table, uint64_t mask, int sw,
                                               const int64_t* __restrict__ keys, const int64_t* __restrict__ ts,
                                               const uint8_t* __restrict__ kv, const uint8_t* __restrict__ rv,
                                               int64_t n, int inner, JWhere w, int ncols,
                                               const int32_t* __restrict__ types_dev, JOut out,
                                               unsigned long long* __restrict__ n_emitted) {
  const int64_t base = (int64_t)blockIdx.x * 256 * PR;
  const int lane = threadIdx.x & 63;
  int64_t key[PR];
  bool act[PR];
  longlong2 h0[PR], g0[PR];          // (key, meta) of the home pair's two slots
  uint64_t c0a[CMP ? 1 : PR], c0b[CMP ? 1 : PR];  // their first payload words (CMP: in the meta words)
#pragma unroll
  for (int r = 0; r < PR; r++) {
    const int64_t i = base + r * 256 + threadIdx.x;
    const int64_t ic = i < n ? i : n - 1;
    key[r] = keys[ic];
    act[r] = i < n && ts[ic] >= 0 && bit_get(kv, ic) && bit_get(rv, ic);
  }
#pragma unroll
  for (int r = 0; r < PR; r++) {  // the home slot is recomputed at use: fewer live registers, more waves
    const uint64_t* sp = table + home_slot(key[r], mask) * (uint64_t)sw;
    h0[r] = *(const longlong2*)sp;
    g0[r] = *(const longlong2*)(sp + sw);
    if constexpr (!CMP) {  // CMP: the value is in the meta word, the pair is one 32-byte read
      c0a[r] = sp[3];
      c0b[r] = sp[sw + 3];
    }
  }
  int cnt = 0;
#pragma unroll
  for (int r = 0; r < PR; r++) {
    const int64_t i = base + r * 256 + threadIdx.x;
    bool hit = false, emit = false;
    int64_t found = -1;
    uint64_t meta = 0, v0 = 0;
    if (act[r]) {
      uint64_t m = (uint64_t)h0[r].y;
      int64_t k0 = h0[r].x;
      uint64_t c0 = CMP ? (uint64_t)h0[r].y : c0a[CMP ? 0 : r], c1 = CMP ? (uint64_t)g0[r].y : c0b[CMP ? 0 : r];
      uint64_t sl = home_slot(key[r], mask);
      // c0 / c1 opaque (registers, not "loads of c0a / c0b"): otherwise the compiler sinks the
      // loads to the hit through a pointer phi (a home-pair word in a private array | a probed
      // slot), which keeps the array in scratch — each word stored right after its load, a wait
      // per probe
      asm volatile("" : "+v"(c0), "+v"(c1));
      // the home pair's second slot from registers; linear probing past the pair (rare)
      for (int probe = 0; probe < JMAX_PROBE; probe++) {
        if (m == 0) break;
        if (k0 == key[r]) {
          if (m & M_LIVE) {
            hit = true;
            found = (int64_t)sl;
            meta = m;
            v0 = CMP ? (uint64_t)(int64_t)(int32_t)(uint32_t)c0 : c0;
          }
          break;
        }
        sl = (sl + 1) & mask;
        if (probe == 0) {
          k0 = g0[r].x;
          m = (uint64_t)g0[r].y;
          c0 = c1;
        } else {
          const uint64_t* s = table + sl * (uint64_t)sw;
          k0 = (int64_t)s[0];
          m = s[1];
          c0 = CMP ? m : s[3];
        }
      }
      emit = inner ? hit : true;
      if (emit && w.active)
        emit = hit && where_ok_raw(w.col == 0 ? v0 : table[found * (uint64_t)sw + 3 + w.col], meta, w, CMP);
    }
    const uint64_t be = __ballot(emit), bh = __ballot(hit);
    const int64_t wbase = i - lane;
    if (lane == 0 && wbase < n) {
      // n may not be a multiple of 64: write whole bytes only up to the batch end
      const int64_t nbytes = std::min<int64_t>(8, (n - wbase + 7) / 8);
      if (nbytes == 8 && !(((uintptr_t)out.emit | (uintptr_t)out.matched) & 7)) {
        if (out.emit) *(uint64_t*)(out.emit + wbase / 8) = be;
        if (out.matched) *(uint64_t*)(out.matched + wbase / 8) = bh;
      } else {
        for (int b = 0; b < nbytes; b++) {
          if (out.emit) out.emit[wbase / 8 + b] = (uint8_t)(be >> (8 * b));
          if (out.matched) out.matched[wbase / 8 + b] = (uint8_t)(bh >> (8 * b));
        }
      }
    }
    for (int c = 0; c < ncols; c++) {
      // rows past the batch end keep a 0 bit (the bitmap's last byte is partial when n % 8 != 0)
      const bool isnull = i < n && (!hit || slot_null(meta, c, CMP));
      const uint64_t bn = __ballot(isnull);
      if (out.col_null[c] && lane == 0 && wbase < n) {
        const int64_t nbytes = std::min<int64_t>(8, (n - wbase + 7) / 8);
        if (nbytes == 8 && !((uintptr_t)out.col_null[c] & 7)) {
          *(uint64_t*)(out.col_null[c] + wbase / 8) = bn;
        } else {
          for (int b = 0; b < nbytes; b++) out.col_null[c][wbase / 8 + b] = (uint8_t)(bn >> (8 * b));
        }
      }
      if (i < n && out.col_data[c]) {
        const uint64_t raw = hit ? (c == 0 ? v0 : table[found * (uint64_t)sw + 3 + c]) : 0;
        if (types_dev[c] == KHIP_TYPE_INT32) ((int32_t*)out.col_data[c])[i] = (int32_t)raw;
        else ((uint64_t*)out.col_data[c])[i] = raw;
      }
    }
    if (out.slot_out && i < n) out.slot_out[i] = emit ? found + 1 : -1;  // 0 = emitted LEFT miss
    cnt += lane == 0 ? __popcll(be) : 0;
  }
  // one of JCTR counters per block (the host sums them): every wave adding to one word serialized
  // at the memory side (~2M adds per 1e9-row probe)
  if (n_emitted && lane == 0 && cnt) atomicAdd(&n_emitted[blockIdx.x & (JCTR - 1)], (unsigned long long)cnt);
}

// Probe through the dense index: one random cell read (MALL-resident for C4) per stream row,
// PR rows per thread issued before any is used; output identical to k_probe.
template <int PR>
__global__ __launch_bounds__(256) void k_probe_dense(JDense dn, const int64_t* __restrict__ keys,
                                                     const int64_t* __restrict__ ts, const uint8_t* __restrict__ kv,
                                                     const uint8_t* __restrict__ rv, int64_t n, int inner, JWhere w,
                                                     int32_t ctype, JOut out, unsigned long long* __restrict__ n_emitted) {
  const int64_t base = (int64_t)blockIdx.x * 256 * PR;
  const int lane = threadIdx.x & 63;
  bool act[PR];
  uint64_t cell[PR];
#pragma unroll
  for (int r = 0; r < PR; r++) {
    const int64_t i = base + r * 256 + threadIdx.x;
    const int64_t ic = i < n ? i : n - 1;
    const int64_t k = keys[ic] - dn.kmin;
    act[r] = i < n && ts[ic] >= 0 && bit_get(kv, ic) && bit_get(rv, ic);
    const bool kin = keys[ic] >= dn.kmin && k < dn.nkeys;
    cell[r] = kin ? dense_load(dn, k) : 0;
  }
  int cnt = 0;
#pragma unroll
  for (int r = 0; r < PR; r++) {
    const int64_t i = base + r * 256 + threadIdx.x;
    const bool hit = act[r] && (cell[r] & 1);
    const bool isnull = !hit || (cell[r] & 2);
    const uint64_t raw = isnull ? 0 : (uint64_t)(dn.vmin + (int64_t)(cell[r] >> 2));
    bool emit = act[r] && (inner ? hit : true);
    if (emit && w.active) emit = hit && where_ok_raw(raw, isnull ? 1ULL : 0ULL, w);
    const uint64_t be = __ballot(emit), bh = __ballot(hit), bn = __ballot(i < n && isnull);
    const int64_t wbase = i - lane;
    if (lane == 0 && wbase < n) {
      const int64_t nbytes = std::min<int64_t>(8, (n - wbase + 7) / 8);
      if (nbytes == 8 && !(((uintptr_t)out.emit | (uintptr_t)out.matched | (uintptr_t)out.col_null[0]) & 7)) {
        if (out.emit) *(uint64_t*)(out.emit + wbase / 8) = be;
        if (out.matched) *(uint64_t*)(out.matched + wbase / 8) = bh;
        if (out.col_null[0]) *(uint64_t*)(out.col_null[0] + wbase / 8) = bn;
      } else {
        for (int b = 0; b < nbytes; b++) {
          if (out.emit) out.emit[wbase / 8 + b] = (uint8_t)(be >> (8 * b));
          if (out.matched) out.matched[wbase / 8 + b] = (uint8_t)(bh >> (8 * b));
          if (out.col_null[0]) out.col_null[0][wbase / 8 + b] = (uint8_t)(bn >> (8 * b));
        }
      }
    }
    if (i < n && out.col_data[0]) {
      if (ctype == KHIP_TYPE_INT32) ((int32_t*)out.col_data[0])[i] = (int32_t)raw;
      else ((uint64_t*)out.col_data[0])[i] = raw;
    }
    if (out.slot_out && i < n) out.slot_out[i] = emit ? (hit ? 1 : 0) : -1;
    cnt += lane == 0 ? __popcll(be) : 0;
  }
  // one of JCTR counters per block (the host sums them): every wave adding to one word serialized
  // at the memory side (~2M adds per 1e9-row probe)
  if (n_emitted && lane == 0 && cnt) atomicAdd(&n_emitted[blockIdx.x & (JCTR - 1)], (unsigned long long)cnt);
}

// Probe through the hashed index: one 16-byte read (the home pair) per stream row, PR rows per
// thread issued before any is used.  A row whose key is neither in its home pair nor stopped by an
// empty word there (≈ α² of them) chases the following pairs — every such row of the thread in the
// same round, so their dependent reads overlap instead of running one row after another.
// Output identical to k_probe_dense.
template <int PR>
__global__ __launch_bounds__(256) void k_probe_hix(JHix hx, const int64_t* __restrict__ keys,
                                                   const int64_t* __restrict__ ts, const uint8_t* __restrict__ kv,
                                                   const uint8_t* __restrict__ rv, int64_t n, int inner, JWhere w,
                                                   int32_t ctype, JOut out, unsigned long long* __restrict__ n_emitted) {
  const int64_t base = (int64_t)blockIdx.x * 256 * PR;
  const int lane = threadIdx.x & 63;
  const uint64_t cmask = (1ULL << hx.cb) - 1;
  bool act[PR];
  uint32_t inr = 0;  // bit r: row r's key is inside the index's key range (else: no such key)
  uint64_t krel[PR];
  ulonglong2 pw[PR];
#pragma unroll
  for (int r = 0; r < PR; r++) {
    const int64_t i = base + r * 256 + threadIdx.x;
    const int64_t ic = i < n ? i : n - 1;
    const int64_t key = keys[ic];
    act[r] = i < n && ts[ic] >= 0 && bit_get(kv, ic) && bit_get(rv, ic);
    krel[r] = (uint64_t)(key - hx.kmin);
    if (key >= hx.kmin && krel[r] < hx.krel_max) inr |= 1u << r;
    pw[r] = *(const ulonglong2*)(hx.words + hix_home(key, hx.mask));
  }
  // the home pairs; pend bit r: row r chases on from pair dd[r]
  uint32_t cellv[PR];
  uint64_t dd[PR];
  uint32_t pend = 0;
#pragma unroll
  for (int r = 0; r < PR; r++) {
    cellv[r] = 0;
    dd[r] = hix_home((int64_t)krel[r] + hx.kmin, hx.mask);
    if (!act[r] || !((inr >> r) & 1u) || pw[r].x == HIX_EMPTY) continue;
    if ((pw[r].x >> hx.cb) == krel[r]) cellv[r] = (uint32_t)(pw[r].x & cmask);
    else if (pw[r].y == HIX_EMPTY) continue;
    else if ((pw[r].y >> hx.cb) == krel[r]) cellv[r] = (uint32_t)(pw[r].y & cmask);
    else pend |= 1u << r;
  }
  for (int round = 1; round < HIX_PROBE / 2 && __ballot(pend != 0); round++) {
    ulonglong2 q[PR];
#pragma unroll
    for (int r = 0; r < PR; r++) {
      if (!((pend >> r) & 1u)) continue;
      dd[r] = (dd[r] + 2) & hx.mask;
      q[r] = *(const ulonglong2*)(hx.words + dd[r]);
    }
#pragma unroll
    for (int r = 0; r < PR; r++) {
      if (!((pend >> r) & 1u)) continue;
      bool stop = true;
      if (q[r].x == HIX_EMPTY) {
      } else if ((q[r].x >> hx.cb) == krel[r]) {
        cellv[r] = (uint32_t)(q[r].x & cmask);
      } else if (q[r].y == HIX_EMPTY) {
      } else if ((q[r].y >> hx.cb) == krel[r]) {
        cellv[r] = (uint32_t)(q[r].y & cmask);
      } else {
        stop = false;
      }
      if (stop) pend &= ~(1u << r);
    }
  }
  int cnt = 0;
#pragma unroll
  for (int r = 0; r < PR; r++) {
    const int64_t i = base + r * 256 + threadIdx.x;
    const uint64_t cell = cellv[r];
    const bool hit = act[r] && (cell & 1);
    const bool isnull = !hit || (cell & 2);
    const uint64_t raw = isnull ? 0 : (uint64_t)(hx.vmin + (int64_t)(cell >> 2));
    bool emit = act[r] && (inner ? hit : true);
    if (emit && w.active) emit = hit && where_ok_raw(raw, isnull ? 1ULL : 0ULL, w);
    const uint64_t be = __ballot(emit), bh = __ballot(hit), bn = __ballot(i < n && isnull);
    const int64_t wbase = i - lane;
    if (lane == 0 && wbase < n) {
      const int64_t nbytes = std::min<int64_t>(8, (n - wbase + 7) / 8);
      if (nbytes == 8 && !(((uintptr_t)out.emit | (uintptr_t)out.matched | (uintptr_t)out.col_null[0]) & 7)) {
        if (out.emit) *(uint64_t*)(out.emit + wbase / 8) = be;
        if (out.matched) *(uint64_t*)(out.matched + wbase / 8) = bh;
        if (out.col_null[0]) *(uint64_t*)(out.col_null[0] + wbase / 8) = bn;
      } else {
        for (int b = 0; b < nbytes; b++) {
          if (out.emit) out.emit[wbase / 8 + b] = (uint8_t)(be >> (8 * b));
          if (out.matched) out.matched[wbase / 8 + b] = (uint8_t)(bh >> (8 * b));
          if (out.col_null[0]) out.col_null[0][wbase / 8 + b] = (uint8_t)(bn >> (8 * b));
        }
      }
    }
    if (i < n && out.col_data[0]) {
      if (ctype == KHIP_TYPE_INT32) ((int32_t*)out.col_data[0])[i] = (int32_t)raw;
      else ((uint64_t*)out.col_data[0])[i] = raw;
    }
    if (out.slot_out && i < n) out.slot_out[i] = emit ? (hit ? 1 : 0) : -1;
    cnt += lane == 0 ? __popcll(be) : 0;
  }
  if (n_emitted && lane == 0 && cnt) atomicAdd(&n_emitted[blockIdx.x & (JCTR - 1)], (unsigned long long)cnt);
}

__global__ __launch_bounds__(256) void k_table_rehash(const uint64_t* __restrict__ old, int64_t ocap,
                                                      uint64_t* __restrict__ nt, uint64_t nmask, int sw, int cmp) {
  for (int64_t slot = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; slot < ocap;
       slot += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t* s = old + slot * (uint64_t)sw;
    const uint64_t m = s[1];
    if (!(m & M_LIVE)) continue;  // deleted keys are dropped on rehash
    uint64_t d = home_slot((int64_t)s[0], nmask);
    while (atomicCAS((unsigned long long*)&nt[d * sw + 1], 0ULL, (unsigned long long)m) != 0ULL) d = (d + 1) & nmask;
    uint64_t* q = nt + d * (uint64_t)sw;
    q[0] = s[0];
    if (cmp) continue;  // COMPACT: key + meta (value inside); the tags array is zero
    q[2] = 0;
    for (int w = 3; w < sw; w++) q[w] = s[w];
  }
}

__global__ __launch_bounds__(256) void k_count_live(const uint64_t* __restrict__ table, int64_t cap, int sw,
                                                    unsigned long long* __restrict__ n_live) {
  int64_t c = 0;
  for (int64_t slot = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; slot < cap;
       slot += (int64_t)gridDim.x * blockDim.x)
    c += (table[slot * (uint64_t)sw + 1] & M_LIVE) ? 1 : 0;
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(n_live, (unsigned long long)c);
}

static int jgrid(int64_t work, int cap_blocks = 8192) {
  return (int)std::min<int64_t>(ceil_div(std::max<int64_t>(work, 1), 256), cap_blocks);
}

}  // namespace khip

using namespace khip;

struct khip_table {
  khip_table_desc desc{};
  std::vector<int32_t> col_types;
  int device = 0;
  hipStream_t stream = nullptr;
  int sw = 4;
  bool compact = false;  // 16-byte slots (one INT payload column), last-writer tags beside
  DevBuf tags;
  DevBuf table, types_dev, slot_of, scratch, st_keys, st_ts, st_kv, st_rv, st_cols[JMAX_COLS],
      st_cval[JMAX_COLS], out_emit, out_matched, out_cols[JMAX_COLS], out_nulls[JMAX_COLS], out_slot;
  int64_t cap = 0;
  int64_t occ = 0;  // resident keys (live or deleted)
  DevBuf claimed;    // slots claimed by the current upsert batch
  // dense probe index (JDense): in step with the slot table while dense_ok
  bool dense_ok = false;
  int64_t dense_eval_occ = -1;  // resident keys when eligibility was last evaluated (-1: never)
  JDense dn{};
  DevBuf dcells, dinvalid, drange;
  // hashed probe index (JHix): keys too spread for the dense one
  bool hix_ok = false;
  JHix hx{};
  DevBuf hwords, hinvalid;
  // STRING keys
  bool utf8 = false;
  KeyDict dict;
  DevBuf kid, khash, st_koff, st_kbytes;
};

static khip_status prepare_hix(khip_table* t, int64_t live, int64_t kmin, int64_t kmax, int64_t vmin,
                               unsigned __int128 vrange);

// Build a probe index if the table qualifies — one INT/BIGINT value column, values fitting a cell
// of at most 24 bits: the dense index when the live keys span at most 4x their count (or 2^20),
// else the hashed index when (key - kmin) and the cell fit 64 bits.  Evaluated again only after
// the table doubled since an unsuccessful try.
static khip_status prepare_dense(khip_table* t) {
  if (t->dense_ok || t->hix_ok || t->utf8 || t->desc.n_cols != 1 || t->col_types[0] == KHIP_TYPE_DOUBLE ||
      !knob("KHIP_PROBE_DENSE", 1))
    return KHIP_OK;
  if (t->dense_eval_occ >= 0 && t->occ < 2 * t->dense_eval_occ) return KHIP_OK;
  t->dense_eval_occ = std::max<int64_t>(t->occ, 1);
  KHIP_TRY(t->drange.ensure(64));
  unsigned long long init[6] = {~0ULL, 0ULL, ~0ULL, 0ULL, 0ULL, 0ULL}, r[6];
  unsigned long long* out = t->drange.as<unsigned long long>();
  KHIP_TRY_HIP(hipMemcpyAsync(out, init, sizeof(init), hipMemcpyHostToDevice, t->stream));
  hipLaunchKernelGGL(k_table_ranges, dim3(jgrid(t->cap, 4096)), dim3(256), 0, t->stream, t->table.as<uint64_t>(), t->cap,
                     t->sw, out, t->compact ? 1 : 0);
  KHIP_TRY_HIP(hipGetLastError());
  KHIP_TRY_HIP(hipMemcpyAsync(r, out, sizeof(r), hipMemcpyDeviceToHost, t->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(t->stream));
  const int64_t live = (int64_t)r[4];
  if (live == 0) return KHIP_OK;
  const uint64_t bias = 1ULL << 63;
  const int64_t kmin = (int64_t)(r[0] ^ bias), kmax = (int64_t)(r[1] ^ bias);
  int64_t vmin = (int64_t)(r[2] ^ bias), vmax = (int64_t)(r[3] ^ bias);
  if (r[2] == ~0ULL) vmin = vmax = 0;  // every value NULL
  const unsigned __int128 krange = (unsigned __int128)((__int128)kmax - (__int128)kmin) + 1;
  const unsigned __int128 vrange = (unsigned __int128)((__int128)vmax - (__int128)vmin) + 1;
  if (krange > (unsigned __int128)std::max<int64_t>(4 * live, 1 << 20) || krange > ((unsigned __int128)1 << 34))
    return prepare_hix(t, live, kmin, kmax, vmin, vrange);
  int bits = 2;
  while (bits < 64 && ((unsigned __int128)1 << (bits - 2)) < vrange) bits++;
  if (((unsigned __int128)1 << (bits - 2)) < vrange) return KHIP_OK;
  // 2-bit cells when every live value is one of three and none is NULL (C4's levels)
  const bool quarter = vrange <= 3 && r[5] == 0 && knob("KHIP_PROBE_QUARTER", KHIP_JOIN_QUARTER);
  const int w = quarter ? 0 : (bits <= 8 ? 1 : (bits <= 16 ? 2 : (bits <= 32 ? 4 : 8)));
  // room for keys appended past the current maximum before the index must be rebuilt
  const int64_t nkeys = (int64_t)krange + (int64_t)krange / 8 + 1024;
  const size_t cbytes = quarter ? (size_t)((nkeys + 15) / 16) * 4 : (size_t)nkeys * w;
  KHIP_TRY(t->dcells.ensure(cbytes));
  KHIP_TRY(t->dinvalid.ensure(8));
  KHIP_TRY_HIP(hipMemsetAsync(t->dcells.p, 0, cbytes, t->stream));
  KHIP_TRY_HIP(hipMemsetAsync(t->dinvalid.p, 0, 8, t->stream));
  JDense d{};
  d.active = 1;
  d.w = w;
  d.kmin = kmin;
  d.nkeys = nkeys;
  d.vmin = vmin;
  d.vspan = w == 0 ? 3 : (w == 8 ? (1ULL << 62) : (1ULL << (8 * w - 2)));
  d.cells = t->dcells.as<uint8_t>();
  d.invalid = t->dinvalid.as<int>();
  hipLaunchKernelGGL(k_dense_build, dim3(jgrid(t->cap, 8192)), dim3(256), 0, t->stream, t->table.as<uint64_t>(), t->cap,
                     t->sw, d, t->compact ? 1 : 0);
  KHIP_TRY_HIP(hipGetLastError());
  int bad = 0;
  KHIP_TRY_HIP(hipMemcpyAsync(&bad, t->dinvalid.p, 4, hipMemcpyDeviceToHost, t->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(t->stream));
  if (bad) return KHIP_OK;
  t->dn = d;
  t->dense_ok = true;
  return KHIP_OK;
}

static khip_status prepare_hix(khip_table* t, int64_t live, int64_t kmin, int64_t kmax, int64_t vmin,
                               unsigned __int128 vrange) {
  if (!knob("KHIP_PROBE_HIX", 1)) return KHIP_OK;
  int cb = 2;
  while (cb < 24 && ((unsigned __int128)1 << (cb - 2)) < vrange) cb++;
  if (((unsigned __int128)1 << (cb - 2)) < vrange) return KHIP_OK;
  // keys appended past the current maximum keep their words while they fit (key - kmin) < krel_max
  const unsigned __int128 krange = (unsigned __int128)((__int128)kmax - (__int128)kmin) + 1;
  const uint64_t krel_max = (1ULL << (64 - cb)) - 1;
  if (krange >= (unsigned __int128)krel_max) return KHIP_OK;
  const int64_t words = next_pow2(std::max<int64_t>(2 * live + live / 4, 1024));
  KHIP_TRY(t->hwords.ensure((size_t)words * 8));
  KHIP_TRY(t->hinvalid.ensure(8));
  KHIP_TRY_HIP(hipMemsetAsync(t->hwords.p, 0xFF, (size_t)words * 8, t->stream));
  KHIP_TRY_HIP(hipMemsetAsync(t->hinvalid.p, 0, 8, t->stream));
  JHix h{};
  h.active = 1;
  h.cb = cb;
  h.kmin = kmin;
  h.krel_max = krel_max;
  h.mask = (uint64_t)(words - 1);
  h.vmin = vmin;
  h.vspan = 1ULL << (cb - 2);
  h.words = t->hwords.as<uint64_t>();
  h.invalid = t->hinvalid.as<int>();
  hipLaunchKernelGGL(k_hix_build, dim3(jgrid(t->cap, 8192)), dim3(256), 0, t->stream, t->table.as<uint64_t>(), t->cap,
                     t->sw, h, t->compact ? 1 : 0);
  KHIP_TRY_HIP(hipGetLastError());
  int bad = 0;
  KHIP_TRY_HIP(hipMemcpyAsync(&bad, t->hinvalid.p, 4, hipMemcpyDeviceToHost, t->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(t->stream));
  if (bad) return KHIP_OK;
  t->hx = h;
  t->hix_ok = true;
  return KHIP_OK;
}

static khip_status table_alloc(khip_table* t, DevBuf& buf, int64_t cap) {
  KHIP_TRY(buf.ensure((size_t)cap * t->sw * 8));
  KHIP_TRY_HIP(hipMemsetAsync(buf.p, 0, (size_t)cap * t->sw * 8, t->stream));
  if (t->compact) {  // the last-writer tags, one per slot (zero between upserts)
    t->tags.release();
    KHIP_TRY(t->tags.ensure((size_t)cap * 8));
    KHIP_TRY_HIP(hipMemsetAsync(t->tags.p, 0, (size_t)cap * 8, t->stream));
  }
  return KHIP_OK;
}

static khip_status table_grow(khip_table* t, int64_t new_cap) {
  DevBuf nt;
  KHIP_TRY(table_alloc(t, nt, new_cap));
  hipLaunchKernelGGL(k_table_rehash, dim3(jgrid(t->cap)), dim3(256), 0, t->stream, t->table.as<uint64_t>(), t->cap,
                     nt.as<uint64_t>(), (uint64_t)(new_cap - 1), t->sw, t->compact ? 1 : 0);
  KHIP_TRY_HIP(hipGetLastError());
  unsigned long long* ctr;
  KHIP_TRY(t->scratch.ensure(64));
  ctr = t->scratch.as<unsigned long long>();
  KHIP_TRY_HIP(hipMemsetAsync(ctr, 0, 8, t->stream));
  hipLaunchKernelGGL(k_count_live, dim3(jgrid(new_cap, 2048)), dim3(256), 0, t->stream, nt.as<uint64_t>(), new_cap,
                     t->sw, ctr);
  unsigned long long live = 0;
  KHIP_TRY_HIP(hipMemcpyAsync(&live, ctr, 8, hipMemcpyDeviceToHost, t->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(t->stream));
  t->table.release();
  t->table = std::move(nt);
  nt.p = nullptr;
  t->cap = new_cap;
  t->occ = (int64_t)live;
  return KHIP_OK;
}

static khip_status jstage(khip_table* t, DevBuf& buf, const void* src, size_t bytes) {
  KHIP_TRY(buf.ensure(bytes));
  if (bytes) KHIP_TRY_HIP(hipMemcpyAsync(buf.p, src, bytes, hipMemcpyHostToDevice, t->stream));
  return KHIP_OK;
}

// Resolve batch pointers to device memory (staging host batches).
static khip_status jresolve(khip_table* t, const khip_batch* b, int ncols, const int64_t** keys,
                            const int64_t** ts, const uint8_t** kv, const uint8_t** rv, JCols* cols) {
  const int64_t n = b->n_rows;
  const size_t bm = (size_t)(n + 7) / 8;
  *keys = b->key_i64;
  *ts = b->ts;
  *kv = b->key_valid;
  *rv = b->row_valid;
  memset(cols, 0, sizeof(*cols));
  if (b->mem == KHIP_MEM_DEVICE) {
    for (int c = 0; c < ncols; c++) {
      cols->data[c] = b->col_data[c];
      cols->valid[c] = b->col_valid ? b->col_valid[c] : nullptr;
    }
    return KHIP_OK;
  }
  if (b->mem != KHIP_MEM_HOST) return fail(KHIP_E_INVALID, "batch mem");
  if (!t->utf8) {
    KHIP_TRY(jstage(t, t->st_keys, b->key_i64, n * 8));
    *keys = t->st_keys.as<int64_t>();
  }
  if (b->ts) {
    KHIP_TRY(jstage(t, t->st_ts, b->ts, n * 8));
    *ts = t->st_ts.as<int64_t>();
  }
  if (*kv) { KHIP_TRY(jstage(t, t->st_kv, b->key_valid, bm)); *kv = t->st_kv.as<uint8_t>(); }
  if (*rv) { KHIP_TRY(jstage(t, t->st_rv, b->row_valid, bm)); *rv = t->st_rv.as<uint8_t>(); }
  for (int c = 0; c < ncols; c++) {
    const size_t es = t->col_types[c] == KHIP_TYPE_INT32 ? 4 : 8;
    KHIP_TRY(jstage(t, t->st_cols[c], b->col_data[c], n * es));
    cols->data[c] = t->st_cols[c].p;
    const uint8_t* cv = b->col_valid ? b->col_valid[c] : nullptr;
    if (cv) {
      KHIP_TRY(jstage(t, t->st_cval[c], cv, bm));
      cols->valid[c] = t->st_cval[c].as<uint8_t>();
    }
  }
  return KHIP_OK;
}

// The batch's table keys on the device: the BIGINT/INT keys as given (jresolve), or the ids of
// its STRING keys — inserted into the dictionary for an upsert, looked up read-only for a probe
// (-1 = never upserted).
static khip_status resolve_keys(khip_table* t, const khip_batch* b, bool upsert, const uint8_t* kv,
                                const int64_t** keys) {
  if (!t->utf8) return KHIP_OK;
  const int64_t n = b->n_rows;
  const int64_t* koff = b->key_offsets;
  const uint8_t* kbytes = b->key_bytes;
  int64_t nbytes = 0;
  if (b->mem == KHIP_MEM_HOST) {
    nbytes = b->key_offsets[n];
    KHIP_TRY(jstage(t, t->st_koff, b->key_offsets, (size_t)(n + 1) * 8));
    KHIP_TRY(jstage(t, t->st_kbytes, b->key_bytes, (size_t)nbytes));
    KHIP_TRY(t->st_kbytes.ensure(8));
    koff = t->st_koff.as<int64_t>();
    kbytes = t->st_kbytes.as<uint8_t>();
  } else if (upsert) {
    KHIP_TRY_HIP(hipMemcpyAsync(&nbytes, koff + n, 8, hipMemcpyDeviceToHost, t->stream));
    KHIP_TRY_HIP(hipStreamSynchronize(t->stream));
  }
  KHIP_TRY(t->kid.ensure((size_t)n * 8));
  if (upsert) {
    KHIP_TRY(t->khash.ensure((size_t)n * 8));
    KHIP_TRY(dict_map(t->dict, t->stream, koff, kbytes, nbytes, kv, nullptr, nullptr, n, t->kid.as<int64_t>(),
                      t->khash.as<int64_t>()));
  } else {
    KHIP_TRY(dict_find(t->dict, t->stream, koff, kbytes, n, t->kid.as<int64_t>()));
  }
  *keys = t->kid.as<int64_t>();
  return KHIP_OK;
}

static khip_status make_where(khip_table* t, const khip_where* w, JWhere* jw) {
  memset(jw, 0, sizeof(*jw));
  if (!w) return KHIP_OK;
  if (w->right_col < 0 || w->right_col >= t->desc.n_cols) return fail(KHIP_E_INVALID, "where column");
  if (w->op < KHIP_OP_GT || w->op > KHIP_OP_NE) return fail(KHIP_E_INVALID, "where op");
  jw->active = 1;
  jw->col = w->right_col;
  jw->op = w->op;
  jw->type = t->col_types[w->right_col];
  jw->i64 = w->i64;
  jw->f64 = w->f64;
  return KHIP_OK;
}

extern "C" {

khip_status khip_table_create(const khip_table_desc* d, khip_table** out) {
  clear_error();
  if (!d || !out) return fail(KHIP_E_INVALID, "null argument");
  if (d->key_type != KHIP_KEY_INT64 && d->key_type != KHIP_KEY_UTF8)
    return fail(KHIP_E_UNSUPPORTED, "table keys must be INT/BIGINT or STRING");
  if (d->n_cols < 0 || d->n_cols > JMAX_COLS) return fail(KHIP_E_UNSUPPORTED, "at most 16 table columns");
  for (int c = 0; c < d->n_cols; c++)
    if (d->col_types[c] < KHIP_TYPE_INT32 || d->col_types[c] > KHIP_TYPE_DOUBLE)
      return fail(KHIP_E_INVALID, "column type");
  khip_table* t = new khip_table();
  t->desc = *d;
  t->col_types.assign(d->col_types, d->col_types + d->n_cols);
  t->desc.col_types = t->col_types.data();
  t->device = d->device;
  t->utf8 = d->key_type == KHIP_KEY_UTF8;
  // one INT payload column: 16-byte slots (the value inside the meta word); else
  // [key, meta, tag, columns...] rounded up to a power of two
  t->compact = d->n_cols == 1 && d->col_types[0] == KHIP_TYPE_INT32 && knob("KHIP_JOIN_COMPACT", 1) != 0;
  t->sw = t->compact ? 2 : (int)next_pow2(std::max(4, 3 + d->n_cols));
  DeviceGuard g(t->device);
  if (hipStreamCreateWithFlags(&t->stream, hipStreamDefault) != hipSuccess) {
    delete t;
    return fail(KHIP_E_DEVICE, "hipStreamCreate failed (no device?)");
  }
  // load factor <= 1/2: with linear probing a hit then costs ~1.5 slot reads and a miss ~2.5
  // (at 3/4 it was 2.5 and 8.5: dependent random HBM reads, the probe kernel's latency chain)
  t->cap = next_pow2(std::max<int64_t>(1024, d->capacity_hint > 0 ? d->capacity_hint * 2 : 1 << 16));
  khip_status st;
  if ((st = table_alloc(t, t->table, t->cap)) != KHIP_OK ||
      (st = t->types_dev.ensure(sizeof(int32_t) * JMAX_COLS)) != KHIP_OK ||
      (st = t->scratch.ensure(64 + 8 * JCTR)) != KHIP_OK || (t->utf8 && (st = dict_init(t->dict, t->stream)) != KHIP_OK)) {
    khip_table_destroy(t);
    return st;
  }
  if (d->n_cols)
    hipMemcpyAsync(t->types_dev.p, t->col_types.data(), sizeof(int32_t) * d->n_cols, hipMemcpyHostToDevice, t->stream);
  if (hipStreamSynchronize(t->stream) != hipSuccess) {
    khip_table_destroy(t);
    return fail(KHIP_E_DEVICE, "device init failed");
  }
  *out = t;
  return KHIP_OK;
}

khip_status khip_table_upsert(khip_table* t, const khip_batch* b) {
  clear_error();
  if (!t || !b) return fail(KHIP_E_INVALID, "null argument");
  const int64_t n = b->n_rows;
  if (n < 0 || b->n_cols < t->desc.n_cols) return fail(KHIP_E_INVALID, "batch shape");
  if (n == 0) return KHIP_OK;
  if (n >= (1LL << 40)) return fail(KHIP_E_UNSUPPORTED, "upsert batch too large");
  if (t->utf8 ? (!b->key_offsets || !b->key_bytes) : !b->key_i64) return fail(KHIP_E_INVALID, "missing key column");
  DeviceGuard g(t->device);
  const int64_t* keys;
  const int64_t* ts;
  const uint8_t *kv, *rv;
  JCols cols;
  KHIP_TRY(jresolve(t, b, t->desc.n_cols, &keys, &ts, &kv, &rv, &cols));
  KHIP_TRY(resolve_keys(t, b, true, kv, &keys));
  // keep the load factor <= 1/2 even if every row were a new key
  if (2 * (t->occ + n) > t->cap) KHIP_TRY(table_grow(t, next_pow2(2 * (t->occ + n))));
  KHIP_TRY(t->slot_of.ensure(n * 8));
  KHIP_TRY(t->claimed.ensure(n * 8));
  unsigned long long* ctr = t->scratch.as<unsigned long long>();
  int* failp = (int*)(t->scratch.as<uint8_t>() + 16);
  KHIP_TRY_HIP(hipMemsetAsync(t->scratch.p, 0, 64, t->stream));
  hipLaunchKernelGGL(k_upsert_claim, dim3(jgrid(n)), dim3(256), 0, t->stream, t->table.as<uint64_t>(),
                     (uint64_t)(t->cap - 1), t->sw, keys, kv, n, t->slot_of.as<int64_t>(), failp, ctr,
                     t->claimed.as<int64_t>(), t->compact ? t->tags.as<uint64_t>() : (uint64_t*)nullptr);
  hipLaunchKernelGGL(k_upsert_finalize, dim3(jgrid(n)), dim3(256), 0, t->stream, t->table.as<uint64_t>(), t->sw, keys,
                     t->claimed.as<int64_t>(), (const unsigned long long*)ctr);
  hipLaunchKernelGGL(k_upsert_apply, dim3(jgrid(n)), dim3(256), 0, t->stream, t->table.as<uint64_t>(), t->sw,
                     t->slot_of.as<int64_t>(), rv, n, t->desc.n_cols, t->types_dev.as<int32_t>(), cols,
                     t->dense_ok ? t->dn : JDense{}, t->compact ? t->tags.as<uint64_t>() : (uint64_t*)nullptr,
                     t->hix_ok ? t->hx : JHix{});
  KHIP_TRY_HIP(hipGetLastError());
  unsigned long long added = 0;
  int failed = 0, dense_bad = 0, hix_bad = 0;
  KHIP_TRY_HIP(hipMemcpyAsync(&added, ctr, 8, hipMemcpyDeviceToHost, t->stream));
  KHIP_TRY_HIP(hipMemcpyAsync(&failed, failp, 4, hipMemcpyDeviceToHost, t->stream));
  if (t->dense_ok) KHIP_TRY_HIP(hipMemcpyAsync(&dense_bad, t->dinvalid.p, 4, hipMemcpyDeviceToHost, t->stream));
  if (t->hix_ok) KHIP_TRY_HIP(hipMemcpyAsync(&hix_bad, t->hinvalid.p, 4, hipMemcpyDeviceToHost, t->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(t->stream));
  if (failed) return fail(KHIP_E_DEVICE, "table probe budget exhausted");
  t->occ += (int64_t)added;
  // a key or value outside an index, or a hashed index filling up (resident keys, deleted ones
  // included, against its words): rebuilt over the new ranges / size by the next probe
  if (dense_bad || hix_bad || (t->hix_ok && 5 * t->occ > 3 * (int64_t)(t->hx.mask + 1))) {
    t->dense_ok = t->hix_ok = false;
    t->dense_eval_occ = -1;
  }
  return KHIP_OK;
}

khip_status khip_table_size(khip_table* t, int64_t* n) {
  clear_error();
  if (!t || !n) return fail(KHIP_E_INVALID, "null argument");
  DeviceGuard g(t->device);
  unsigned long long* ctr = t->scratch.as<unsigned long long>();
  KHIP_TRY_HIP(hipMemsetAsync(ctr, 0, 8, t->stream));
  hipLaunchKernelGGL(k_count_live, dim3(jgrid(t->cap, 2048)), dim3(256), 0, t->stream, t->table.as<uint64_t>(), t->cap,
                     t->sw, ctr);
  unsigned long long live = 0;
  KHIP_TRY_HIP(hipMemcpyAsync(&live, ctr, 8, hipMemcpyDeviceToHost, t->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(t->stream));
  *n = (int64_t)live;
  return KHIP_OK;
}

static khip_status probe_launch(khip_table* t, const khip_batch* b, int32_t join_type, const khip_where* w,
                                const JOut& out, unsigned long long* n_emitted) {
  const int64_t n = b->n_rows;
  const int64_t* keys;
  const int64_t* ts;
  const uint8_t *kv, *rv;
  JCols cols;
  KHIP_TRY(jresolve(t, b, 0, &keys, &ts, &kv, &rv, &cols));
  if (!ts) return fail(KHIP_E_INVALID, "missing timestamp column");
  KHIP_TRY(resolve_keys(t, b, false, kv, &keys));
  JWhere jw;
  KHIP_TRY(make_where(t, w, &jw));
  KHIP_TRY(prepare_dense(t));
  if (t->dense_ok) {
    // rows per thread: every cell read of a thread is issued before any is used (MLP); measured on
    // C4 (1e9 probes, 100 MB of cells): 4 → 49 ms, 8 → 28 ms, 16 → 20.1 ms, 32 → 19.8 ms, 64 →
    // 73 ms (profiles/r04/ab/c4_dense_rows_per_thread.txt)
    const int dpr = (int)knob("KHIP_PROBE_DPR", 32);
    auto dk = dpr >= 64 ? k_probe_dense<64>
                        : (dpr >= 32 ? k_probe_dense<32> : (dpr >= 16 ? k_probe_dense<16> : k_probe_dense<8>));
    const int pr = dpr >= 64 ? 64 : (dpr >= 32 ? 32 : (dpr >= 16 ? 16 : 8));
    hipLaunchKernelGGL(dk, dim3(ceil_div(n, 256 * pr)), dim3(256), 0, t->stream, t->dn, keys, ts, kv, rv, n,
                       join_type == KHIP_JOIN_INNER ? 1 : 0, jw, t->col_types[0], out, n_emitted);
    KHIP_TRY_HIP(hipGetLastError());
    return KHIP_OK;
  }
  if (t->hix_ok) {
    // (8: 96 VGPRs, 5 waves per SIMD — 16 rows held 184 and ran at 2: 30.9 -> 25.0 ms per 1e9
    // probes, profiles/r05/ab/c4_sparse_hpr.txt)
    const int hpr = (int)knob("KHIP_PROBE_HPR", 8);
    auto hk = hpr >= 32 ? k_probe_hix<32> : (hpr >= 16 ? k_probe_hix<16> : (hpr >= 8 ? k_probe_hix<8> : k_probe_hix<4>));
    const int pr = hpr >= 32 ? 32 : (hpr >= 16 ? 16 : (hpr >= 8 ? 8 : 4));
    hipLaunchKernelGGL(hk, dim3(ceil_div(n, 256 * pr)), dim3(256), 0, t->stream, t->hx, keys, ts, kv, rv, n,
                       join_type == KHIP_JOIN_INNER ? 1 : 0, jw, t->col_types[0], out, n_emitted);
    KHIP_TRY_HIP(hipGetLastError());
    return KHIP_OK;
  }
  const int pr_env = (int)knob("KHIP_PROBE_PR", 8);  // measured with 16-byte slots: 8 > 6 > 4, 12, 16 (profiles/r04/)
  const int PR = pr_env >= 16 ? 16 : (pr_env >= 8 ? 8 : (pr_env >= 4 ? 4 : 1));  // 6 and 12 measured slower
  auto kern = t->compact ? (PR == 16 ? k_probe<16, true> : (PR == 8 ? k_probe<8, true> : (PR == 4 ? k_probe<4, true> : k_probe<1, true>)))
                         : (PR == 16 ? k_probe<16, false> : (PR == 8 ? k_probe<8, false> : (PR == 4 ? k_probe<4, false> : k_probe<1, false>)));
  hipLaunchKernelGGL(kern, dim3(ceil_div(n, 256 * PR)), dim3(256), 0, t->stream, t->table.as<uint64_t>(),
                     (uint64_t)(t->cap - 1), t->sw, keys, ts, kv, rv, n, join_type == KHIP_JOIN_INNER ? 1 : 0, jw,
                     t->desc.n_cols, t->types_dev.as<int32_t>(), out, n_emitted);
  KHIP_TRY_HIP(hipGetLastError());
  return KHIP_OK;
}

khip_status khip_table_probe(khip_table* t, const khip_batch* b, int32_t join_type, const khip_where* w,
                             khip_join_out* out) {
  clear_error();
  if (!t || !b || !out) return fail(KHIP_E_INVALID, "null argument");
  if (join_type != KHIP_JOIN_LEFT && join_type != KHIP_JOIN_INNER) return fail(KHIP_E_INVALID, "join type");
  const int64_t n = b->n_rows;
  if (n < 0) return fail(KHIP_E_INVALID, "batch shape");
  if (n == 0) {
    out->n_rows = 0;
    return KHIP_OK;
  }
  if ((t->utf8 ? (!b->key_offsets || !b->key_bytes) : !b->key_i64) || !b->ts)
    return fail(KHIP_E_INVALID, "missing key or timestamp column");
  DeviceGuard g(t->device);
  const int nc = t->desc.n_cols;
  JOut o{};
  KHIP_TRY(t->out_slot.ensure(n * 8));
  o.slot_out = t->out_slot.as<int64_t>();
  for (int c = 0; c < nc; c++) {
    KHIP_TRY(t->out_cols[c].ensure(n * 8));
    KHIP_TRY(t->out_nulls[c].ensure((n + 7) / 8 + 8));
    o.col_data[c] = t->out_cols[c].p;
    o.col_null[c] = t->out_nulls[c].as<uint8_t>();
  }
  KHIP_TRY(probe_launch(t, b, join_type, w, o, nullptr));
  // compact on the host in arrival order (the host path is for parity/small batches)
  std::vector<int64_t> slot(n);
  KHIP_TRY_HIP(hipMemcpyAsync(slot.data(), o.slot_out, n * 8, hipMemcpyDeviceToHost, t->stream));
  std::vector<std::vector<uint8_t>> cd(nc), cn(nc);
  for (int c = 0; c < nc; c++) {
    const size_t es = t->col_types[c] == KHIP_TYPE_INT32 ? 4 : 8;
    cd[c].resize(n * es);
    cn[c].resize((n + 7) / 8);
    KHIP_TRY_HIP(hipMemcpyAsync(cd[c].data(), o.col_data[c], n * es, hipMemcpyDeviceToHost, t->stream));
    KHIP_TRY_HIP(hipMemcpyAsync(cn[c].data(), o.col_null[c], (n + 7) / 8, hipMemcpyDeviceToHost, t->stream));
  }
  KHIP_TRY_HIP(hipStreamSynchronize(t->stream));
  int64_t m = 0;
  for (int64_t i = 0; i < n; i++) {
    if (slot[i] == -1) continue;
    if (m < out->capacity) {
      const bool hit = slot[i] > 0;
      if (out->stream_row) out->stream_row[m] = i;
      if (out->matched) out->matched[m] = hit ? 1 : 0;
      for (int c = 0; c < nc; c++) {
        const bool isnull = (cn[c][i >> 3] >> (i & 7)) & 1;
        if (out->col_null && out->col_null[c]) out->col_null[c][m] = isnull ? 1 : 0;
        if (out->col_data && out->col_data[c]) {
          if (t->col_types[c] == KHIP_TYPE_INT32) ((int32_t*)out->col_data[c])[m] = isnull ? 0 : ((int32_t*)cd[c].data())[i];
          else ((uint64_t*)out->col_data[c])[m] = isnull ? 0 : ((uint64_t*)cd[c].data())[i];
        }
      }
    }
    m++;
  }
  out->n_rows = m;
  if (m > out->capacity) return fail(KHIP_E_BUFFER, "join output capacity too small");
  return KHIP_OK;
}

khip_status khip_table_probe_device(khip_table* t, const khip_batch* b, int32_t join_type, const khip_where* w,
                                    const khip_join_dev_out* out, int64_t* n_emitted) {
  clear_error();
  if (!t || !b || !out) return fail(KHIP_E_INVALID, "null argument");
  if (b->mem != KHIP_MEM_DEVICE) return fail(KHIP_E_INVALID, "probe_device needs a device batch");
  if (join_type != KHIP_JOIN_LEFT && join_type != KHIP_JOIN_INNER) return fail(KHIP_E_INVALID, "join type");
  const int64_t n = b->n_rows;
  if (n < 0) return fail(KHIP_E_INVALID, "batch shape");
  if (n == 0) {
    if (n_emitted) *n_emitted = 0;
    return KHIP_OK;
  }
  if ((t->utf8 ? (!b->key_offsets || !b->key_bytes) : !b->key_i64) || !b->ts)
    return fail(KHIP_E_INVALID, "missing key or timestamp column");
  DeviceGuard g(t->device);
  JOut o{};
  o.emit = out->emit;
  o.matched = out->matched;
  for (int c = 0; c < t->desc.n_cols; c++) {
    o.col_data[c] = out->col_data ? out->col_data[c] : nullptr;
    o.col_null[c] = out->col_null ? out->col_null[c] : nullptr;
  }
  unsigned long long* ctr = nullptr;
  if (n_emitted) {
    ctr = t->scratch.as<unsigned long long>() + 8;  // JCTR words after the 64-byte scratch block
    KHIP_TRY_HIP(hipMemsetAsync(ctr, 0, 8 * JCTR, t->stream));
  }
  KHIP_TRY(probe_launch(t, b, join_type, w, o, ctr));
  if (n_emitted) {
    unsigned long long v[JCTR];
    KHIP_TRY_HIP(hipMemcpyAsync(v, ctr, sizeof(v), hipMemcpyDeviceToHost, t->stream));
    KHIP_TRY_HIP(hipStreamSynchronize(t->stream));
    int64_t tot = 0;
    for (int k = 0; k < JCTR; k++) tot += (int64_t)v[k];
    *n_emitted = tot;
  }
  return KHIP_OK;
}

khip_status khip_table_sync(khip_table* t) {
  if (!t) return fail(KHIP_E_INVALID, "null argument");
  DeviceGuard g(t->device);
  KHIP_TRY_HIP(hipStreamSynchronize(t->stream));
  return KHIP_OK;
}

khip_status khip_table_destroy(khip_table* t) {
  if (!t) return KHIP_OK;
  DeviceGuard g(t->device);
  if (t->stream) hipStreamSynchronize(t->stream);
  DevBuf* bufs[] = {&t->table, &t->types_dev, &t->slot_of, &t->claimed, &t->scratch, &t->st_keys, &t->st_ts, &t->st_kv,
                    &t->st_rv, &t->out_emit, &t->out_matched, &t->out_slot, &t->dcells, &t->dinvalid, &t->drange,
                    &t->kid, &t->khash, &t->st_koff, &t->st_kbytes, &t->tags, &t->hwords, &t->hinvalid};
  for (DevBuf* x : bufs) x->release();
  dict_release(t->dict);
  for (int c = 0; c < JMAX_COLS; c++) {
    t->st_cols[c].release();
    t->st_cval[c].release();
    t->out_cols[c].release();
    t->out_nulls[c].release();
  }
  if (t->stream) hipStreamDestroy(t->stream);
  delete t;
  return KHIP_OK;
}

}  // extern "C"
