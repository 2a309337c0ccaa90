// khip_agg_table.hip — table aggregation (CREATE TABLE .. AS SELECT .. FROM <TABLE> GROUP BY ..)
// on MI355X (gfx950): engine 3 of khip_agg.
//
// Replaces, for one query task, KSPlanBuilder.visitTableGroupBy + visitTableAggregate
// (S/TableGroupByBuilderBase.java:62-111, S/TableAggregateBuilder.java:54-108): Kafka Streams'
// KTable.groupBy(mapper).aggregate(initializer, KudafAggregator, KudafUndoAggregator) — per
// source-table change, the key's previous row is undone from its group (TableUdaf.undo,
// X/function/udaf/KudafUndoAggregator.java:29-55) and the new row applied to its group.  Semantics
// restated in oracle/oracle.c R12.
//
// Group state lives in the global-atomic engine's HBM table (khip_agg.hip: [key | claim ref,
// ws = 0 | EMPTY, rowtime, state words]), so snapshots, pull queries, HAVING counts and growth
// are that engine's.  The source table is a second open-addressing table keyed by PRIMARY KEY id:
//   [0] key  [1] meta: 0 empty | bit63 claimed by this push | bit62 resident; bits 40..55 the
//                      key's row flags (bit0 live, bit1 GROUP BY value non-null, bits 8.. argument
//                      validity)
//   [2] group id  [3] group-key hash (UTF8 GROUP BY keys only)  [..] argument words (raw 8 bytes)
// — 32-byte slots for an INT GROUP BY key and one argument column.
//
// Per push (all on the handle's stream):
//   k_tagg_range   the push's PRIMARY KEY range (per-block partials, one reducing workgroup)
//   k_tagg_keys    sort key = PRIMARY KEY id − kmin (dropped rows sort last), value = row; the row's
//                  packed change record (one 16-byte load per two words in k_tagg_apply); counts
//   radix sort over the range's bits only (khip_sort.hpp; stable: a key's rows keep their arrival order)
//   k_tagg_apply   one thread per distinct PRIMARY KEY (segment leader): find-or-claim its source
//                  slot (a CAS on the meta word: no spin), then replay its rows in
//                  order — undo the previous row (-1 / -x) from its group, apply the new row (+1 /
//                  +x; the group is found or claimed with the atomic engine's reference CAS) —
//                  and store the last row.  Group updates are agent-scope atomics; the row time
//                  is an atomic max.  Integer state is exact (wrapping adds commute); DOUBLE sums
//                  are order-dependent only by rounding.
//   k_tagg_grp_finalize  this push's group claims → resident groups (the claimed slots only)
//   k_tagg_src_finalize  source claims → resident keys
#include <algorithm>
#include <vector>

#include "khip_agg_internal.hpp"
#include "khip_sort.hpp"
#include "khip_util.hpp"

namespace khip {

constexpr uint64_t TS_CLAIM = 1ULL << 63;
constexpr uint64_t TS_RESIDENT = 1ULL << 62;
constexpr uint64_t TF_LIVE = 1, TF_GVALID = 2;
constexpr int TS_MAX_PROBE = 4096;

enum { TC_ACCEPTED, TC_NULL_KEY, TC_BAD_TS, TC_UPDATES, TC_NEW_GROUPS, TC_NEW_KEYS, TC_FAILED, TC_GLIST, TC_KMINN, TC_KMAX,
       TC_KACC, TC_TSMAX, TC_GMINN, TC_GMAX, TC_N };

__device__ __forceinline__ uint64_t src_hash(int64_t id) { return mix64((uint64_t)id ^ 0x3C6EF372FE94F82BULL); }

__device__ __forceinline__ uint64_t id_ord(int64_t k) { return (uint64_t)k ^ (1ULL << 63); }

// Per block: the accepted rows' PRIMARY KEY range (order-preserving words: min as max of ~u), the
// GROUP BY key range of the accepted rows that apply to a group (bounds the groups a push can
// create) and the largest timestamp of the accepted non-tombstone rows (the stream time the push
// reaches; stored +1, so 0 = none).  r[0..4) = kmin~, kmax, gmin~, gmax.
__global__ __launch_bounds__(256) void k_tagg_range(const int64_t* __restrict__ src_id, const uint8_t* __restrict__ src_kv,
                                                    const uint8_t* __restrict__ rv, const int64_t* __restrict__ ts,
                                                    const int64_t* __restrict__ gkeys, const uint8_t* __restrict__ gkv,
                                                    int64_t n, ulonglong4* __restrict__ blk,
                                                    unsigned long long* __restrict__ blkts) {
  __shared__ uint64_t l[5][4];
  uint64_t r[5] = {0, 0, 0, 0, 0};  // kmin~, kmax, gmin~, gmax, ts max + 1
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = ts[i];
    if (bit_get(src_kv, i) && t >= 0) {
      const uint64_t u = id_ord(src_id[i]);
      r[0] = ~u > r[0] ? ~u : r[0];
      r[1] = u > r[1] ? u : r[1];
      if (bit_get(rv, i)) {
        r[4] = (uint64_t)t + 1 > r[4] ? (uint64_t)t + 1 : r[4];
        if (bit_get(gkv, i)) {
          const uint64_t g = id_ord(gkeys[i]);
          r[2] = ~g > r[2] ? ~g : r[2];
          r[3] = g > r[3] ? g : r[3];
        }
      }
    }
  }
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 5; k++) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const uint64_t a = __shfl_xor(r[k], off, 64);
      r[k] = a > r[k] ? a : r[k];
    }
    if ((threadIdx.x & 63) == 0) l[k][wave] = r[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 0; k < 5; k++)
      for (int w = 1; w < 4; w++) r[k] = l[k][w] > r[k] ? l[k][w] : r[k];
    blk[blockIdx.x] = make_ulonglong4(r[0], r[1], r[2], r[3]);
    blkts[blockIdx.x] = r[4];
  }
}

// Per-block ranges → ctr[TC_KMINN] / ctr[TC_KMAX], ctr[TC_GMINN] / ctr[TC_GMAX] (one workgroup;
// 0 / 0 when none) and ctr[TC_TSMAX] (largest accepted row timestamp + 1, 0: none).
__global__ __launch_bounds__(256) void k_tagg_range_reduce(const ulonglong4* __restrict__ blk,
                                                           const unsigned long long* __restrict__ blkts, int nb,
                                                           unsigned long long* __restrict__ ctr) {
  __shared__ uint64_t l[5][4];
  uint64_t r[5] = {0, 0, 0, 0, 0};
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    const ulonglong4 v = blk[b];
    r[0] = v.x > r[0] ? v.x : r[0];
    r[1] = v.y > r[1] ? v.y : r[1];
    r[2] = v.z > r[2] ? v.z : r[2];
    r[3] = v.w > r[3] ? v.w : r[3];
    r[4] = blkts[b] > r[4] ? blkts[b] : r[4];
  }
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 5; k++) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const uint64_t a = __shfl_xor(r[k], off, 64);
      r[k] = a > r[k] ? a : r[k];
    }
    if ((threadIdx.x & 63) == 0) l[k][wave] = r[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 0; k < 5; k++)
      for (int w = 1; w < 4; w++) r[k] = l[k][w] > r[k] ? l[k][w] : r[k];
    ctr[TC_KMINN] = r[0];
    ctr[TC_KMAX] = r[1];
    ctr[TC_GMINN] = r[2];
    ctr[TC_GMAX] = r[3];
    ctr[TC_TSMAX] = r[4];
  }
}

// Packed change record, one per batch row, written by k_tagg_keys in arrival order and gathered by
// k_tagg_apply in sorted order (one 16-byte load per two words instead of a gather per column):
//   [0] ts  [1] group id  [2] flags: RF_ACC accepted | TF_LIVE not a tombstone | TF_GVALID GROUP BY
//   value non-null | argument validity << 8  [3] group-key hash (UTF8 GROUP BY only: an INT key's
//   hash input is the key itself)  [3 + U8 ..] argument words (raw 8 bytes; 0 when null)
// Rows dropped at intake (null PRIMARY KEY, negative ts) carry flags 0.
constexpr uint64_t RF_ACC = 4;

__host__ __device__ constexpr int tagg_rec_words(int nc, bool u8) { return (3 + (u8 ? 1 : 0) + nc + 1) & ~1; }

__device__ __forceinline__ int64_t load_word(const ColPtrs& c, int32_t type, int col, int64_t i) {
  return type == KHIP_TYPE_INT32 ? (int64_t)((const int32_t*)c.data[col])[i] : ((const int64_t*)c.data[col])[i];
}

struct TaggKeysArgs {
  const int64_t* src_id;
  const uint8_t* src_kv;
  const int64_t* ts;
  const int64_t* gkeys;
  const int64_t* ghash;
  const uint8_t* kv;
  const uint8_t* rv;
  ColPtrs cols;
  int32_t col_type[MAX_COLS];
  int64_t n, kmin;
  uint64_t drop;
};

// Sort key = PRIMARY KEY id − kmin (dropped rows: `drop`, which sorts last), value = row; the
// row's packed change record; counts.
template <int NC, bool U8>
__global__ __launch_bounds__(256) void k_tagg_keys(TaggKeysArgs K, uint64_t* __restrict__ skey, uint32_t* __restrict__ sidx,
                                                   uint64_t* __restrict__ rec, unsigned long long* __restrict__ ctr) {
  constexpr int RW = tagg_rec_words(NC, U8);
  int64_t acc = 0, nk = 0, bt = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < K.n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool kv = bit_get(K.src_kv, i);
    const int64_t t = K.ts[i];
    const bool ok = kv && t >= 0;
    skey[i] = ok ? (uint64_t)K.src_id[i] - (uint64_t)K.kmin : K.drop;
    sidx[i] = (uint32_t)i;
    acc += ok;
    nk += !kv;
    bt += kv && t < 0;
    uint64_t w[RW];
#pragma unroll
    for (int k = 0; k < RW; k++) w[k] = 0;
    w[0] = (uint64_t)t;
    if (ok) {
      uint64_t f = RF_ACC;
      if (bit_get(K.rv, i)) {
        f |= TF_LIVE;
        if (bit_get(K.kv, i)) {
          f |= TF_GVALID;
          w[1] = (uint64_t)K.gkeys[i];
          if (U8) w[3] = (uint64_t)K.ghash[i];
        }
#pragma unroll
        for (int c = 0; c < NC; c++) {
          const bool v = bit_get(K.cols.valid[c], i);
          w[3 + U8 + c] = v ? (uint64_t)load_word(K.cols, K.col_type[c], c, i) : 0;
          f |= (v ? 1ULL : 0ULL) << (8 + c);
        }
      }
      w[2] = f;
    }
    ulonglong2* o = (ulonglong2*)(rec + i * RW);
#pragma unroll
    for (int k = 0; k < RW / 2; k++) o[k] = make_ulonglong2(w[2 * k], w[2 * k + 1]);
  }
  // one add per block and counter (same-address adds from every wave would serialize)
  __shared__ int64_t lc[3][4];
  const int64_t c3[3] = {wave_sum(acc), wave_sum(nk), wave_sum(bt)};
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane < 3) lc[lane][wave] = c3[lane];
  __syncthreads();
  if (threadIdx.x < 3) {
    const int64_t v = lc[threadIdx.x][0] + lc[threadIdx.x][1] + lc[threadIdx.x][2] + lc[threadIdx.x][3];
    const int slot[3] = {TC_ACCEPTED, TC_NULL_KEY, TC_BAD_TS};
    if (v) atomicAdd(&ctr[slot[threadIdx.x]], (unsigned long long)v);
  }
}

// One row's aggregate contribution: group, argument words + flags (TF_* | validity mask << 8).
// NC (the handle's argument column count) is a template parameter: the words stay in registers
// (a run-time bound would index them dynamically and put every row in scratch memory).
template <int NC>
struct TRow {
  int64_t gid, ghash;
  uint32_t flags;
  int64_t w[NC > 0 ? NC : 1];
};

// r.w[col] for a run-time col without dynamic register indexing
template <int NC>
__device__ __forceinline__ int64_t wpick(const TRow<NC>& r, int col) {
  int64_t v = 0;
#pragma unroll
  for (int c = 0; c < NC; c++) v = c == col ? r.w[c] : v;
  return v;
}

// The group of one change, found — or claimed when claim_row >= 0 (the claim references that
// batch row, whose GROUP BY key is the group's) — with the atomic engine's reference CAS.
// Returns the slot, or -1 on probe exhaustion (an undo's group missing counts the same); *isnew
// when this call claimed it.  The slot's words are read with plain 16-byte loads: within a push a
// slot only moves empty → claimed (a stale empty read is settled by the CAS).
__device__ __forceinline__ int64_t group_find(uint64_t* __restrict__ table, uint64_t mask, int sw, int64_t gid,
                                              int64_t ghash, int64_t claim_row, const int64_t* __restrict__ gkeys,
                                              bool* isnew) {
  const uint64_t h = group_hash(ghash, 0);
  const uint64_t fp = (h >> 49) & 0x7FFFULL;
  const uint64_t myref = (1ULL << 63) | (fp << 48) | (uint64_t)(claim_row < 0 ? 0 : claim_row);
  uint64_t slot = h & mask;
  *isnew = false;
  for (int probe = 0; probe < MAX_PROBE; probe++) {
    uint64_t* s = table + slot * (uint64_t)sw;
    const ulonglong2 w01 = *(const ulonglong2*)s;
    if ((int64_t)w01.y != EMPTY_WS) {
      if ((int64_t)w01.x == gid) return (int64_t)slot;
    } else {
      uint64_t w0 = w01.x;
      if (w0 == 0) {
        if (claim_row < 0) return -1;  // an undo always finds its group
        const uint64_t old = atomicCAS((unsigned long long*)s, 0ULL, (unsigned long long)myref);
        if (old == 0) {
          *isnew = true;
          return (int64_t)slot;
        }
        w0 = old;
      }
      if (((w0 >> 48) & 0x7FFFULL) == fp && gkeys[(int64_t)(w0 & ((1ULL << 36) - 1))] == gid) return (int64_t)slot;
    }
    slot = (slot + 1) & mask;
  }
  return -1;
}

// One op's net change from `add`'s contribution minus `sub`'s (the raw word: int64 for the
// counts and integer sums, a double's bits for DOUBLE sums; 0 = unchanged).
template <int NC>
__device__ __forceinline__ uint64_t op_delta(const UpdOp op, bool has_add, const TRow<NC>& add, bool has_sub,
                                             const TRow<NC>& sub) {
  const bool va = has_add && (op.kind == OP_INC || ((add.flags >> (8 + op.col)) & 1u));
  const bool vs = has_sub && (op.kind == OP_INC || ((sub.flags >> (8 + op.col)) & 1u));
  if (!va && !vs) return 0;  // null arguments (undo too): unchanged
  switch (op.kind) {
    case OP_INC:  // COUNT(*) = COUNT(ROWTIME): never null
    case OP_INC_VALID:
      return (uint64_t)((int64_t)va - (int64_t)vs);
    case OP_ADD_I64:  // INT / BIGINT: wrapping (INT truncated to 32 bits when read)
      return (va ? (uint64_t)wpick(add, op.col) : 0) - (vs ? (uint64_t)wpick(sub, op.col) : 0);
    case OP_ADD_F64: {
      const double x = va ? __longlong_as_double(wpick(add, op.col)) : 0.0;
      const double y = vs ? __longlong_as_double(wpick(sub, op.col)) : 0.0;
      return (uint64_t)__double_as_longlong(va && vs ? x - y : (va ? x : -y));
    }
    default:  // MIN / MAX are rejected at create (not undoable)
      return 0;
  }
}

// Adds one op's raw delta to a state word (agent-scope atomic: the atomic path).
__device__ __forceinline__ void op_add_atomic(const UpdOp op, uint64_t* w, uint64_t d) {
  if (op.kind == OP_ADD_F64) {
    if (d) unsafeAtomicAdd((double*)w, __longlong_as_double((long long)d));
  } else if (d) {
    __hip_atomic_fetch_add(w, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

constexpr int TA_C = 2048;  // sorted positions per k_tagg_apply workgroup

struct TaggArgs {
  ApplyParams p;
  uint64_t* table;  // group table
  uint64_t gmask;
  uint64_t* src;    // source table
  uint64_t smask;
  int32_t ssw;
  int64_t n;
  int64_t* glist;   // group slots claimed by this push
  int64_t kmin;     // sort keys are PRIMARY KEY id − kmin
  uint64_t drop;    // the sort key of dropped rows (shared with the largest key when the range is 2^64)
  int64_t dbase;    // dense layout: the id of slot 0
};

template <int NC, bool U8>
__device__ __forceinline__ TRow<NC> rec_row(const uint64_t* __restrict__ rec, int64_t r, int64_t* t, uint32_t* f) {
  constexpr int RW = tagg_rec_words(NC, U8);
  uint64_t w[RW];
  const ulonglong2* p = (const ulonglong2*)(rec + r * RW);
#pragma unroll
  for (int k = 0; k < RW / 2; k++) {
    const ulonglong2 v = p[k];
    w[2 * k] = v.x;
    w[2 * k + 1] = v.y;
  }
  TRow<NC> x;
  *t = (int64_t)w[0];
  *f = (uint32_t)w[2];
  x.gid = (int64_t)w[1];
  x.ghash = U8 ? (int64_t)w[3] : (int64_t)w[1];
  x.flags = (uint32_t)w[2] & ~(uint32_t)RF_ACC;
#pragma unroll
  for (int c = 0; c < NC; c++) x.w[c] = (int64_t)w[3 + U8 + c];
  return x;
}

// Source slot, hash layout: [0] key  [1] meta: 0 empty | TS_CLAIM (claimed by this push) |
// TS_RESIDENT, with the key's row flags (TF_* | validity << 8) in bits 40..55  [2] group id  [3]
// group-key hash (UTF8 GROUP BY only)  [3 + U8 ..] argument words.  Dense layout (slot = id −
// dbase, no key word, no claim: only this push's thread for the key touches it): [0] meta (0 |
// TS_RESIDENT, flags)  [1] group id  [2] hash (UTF8)  [2 + U8 ..] argument words.  Slots are a
// power of two of words.
constexpr int TS_FSHIFT = 40;
constexpr uint64_t TS_FMASK = 0xFFFFULL << TS_FSHIFT;
__host__ __device__ constexpr int tagg_slot_words(int nc, bool u8, bool dense) {
  return (dense ? 2 : 3) + (u8 ? 1 : 0) + nc;
}

// Workgroup w takes sorted positions [w * TA_C, (w + 1) * TA_C); one thread per distinct PRIMARY
// KEY (segment leader).  Hash layout: claimed[j] = the source slot the leader at j claimed, else -1.
template <int NC, bool U8, bool DENSE>
__global__ __launch_bounds__(256) void k_tagg_apply(TaggArgs A, const uint64_t* __restrict__ skey,
                                                    const uint32_t* __restrict__ sidx, const uint64_t* __restrict__ rec,
                                                    const int64_t* __restrict__ gkeys, int64_t* __restrict__ claimed,
                                                    unsigned long long* __restrict__ ctr) {
  constexpr int MW = DENSE ? 0 : 1;  // meta word; the group id follows it
  constexpr int NP = (tagg_slot_words(NC, U8, DENSE) + 1) / 2;  // 16-byte pairs of the slot
  int64_t upd = 0, newg = 0, failed = 0, newk = 0;
  const int64_t lo = (int64_t)blockIdx.x * TA_C, hi = lo + TA_C < A.n ? lo + TA_C : A.n;
  for (int64_t j = lo + threadIdx.x; j < hi; j += blockDim.x) {
    int64_t fresh_slot = -1;
    const uint64_t k = skey[j];
    const bool leader = j == 0 || skey[j - 1] != k;
    int64_t end = j + 1;
    if (leader) {
      while (end < A.n && skey[end] == k) end++;
    }
    if (leader) do {  // `continue` below leaves this segment's body
    if (k == A.drop) {  // dropped rows (and, for a 2^64 range, the largest key's rows)
      bool any = false;
      for (int64_t q = j; q < end && !any; q++) any = (rec[(int64_t)sidx[q] * tagg_rec_words(NC, U8) + 2] & RF_ACC) != 0;
      if (!any) continue;
    }
    const int64_t id = (int64_t)(k + (uint64_t)A.kmin);
    uint64_t* s = nullptr;
    bool fresh = false;
    if constexpr (DENSE) {  // the host keeps every accepted id of the push inside [dbase, dbase + cap)
      s = A.src + (uint64_t)(id - A.dbase) * (uint64_t)A.ssw;
    } else {  // find or claim the key's source slot (only this thread holds this key)
      uint64_t slot = src_hash(id) & A.smask;
      for (int probe = 0; probe < TS_MAX_PROBE; probe++) {
        uint64_t* c = A.src + slot * (uint64_t)A.ssw;
        const ulonglong2 km = *(const ulonglong2*)c;  // a stale empty read is settled by the CAS
        uint64_t m = km.y;
        if (m == 0) {
          const uint64_t old = atomicCAS((unsigned long long*)&c[1], 0ULL, (unsigned long long)TS_CLAIM);
          if (old == 0) {
            s = c;
            fresh = true;
            fresh_slot = (int64_t)slot;
            break;
          }
          m = old;
        }
        // another key's claim of this push, or a resident key
        if (!(m & TS_CLAIM) && (int64_t)km.x == id) {
          s = c;
          break;
        }
        slot = (slot + 1) & A.smask;
      }
      if (!s) {
        failed++;
        continue;
      }
    }
    uint64_t sv[2 * NP];
#pragma unroll
    for (int k2 = 0; k2 < NP; k2++) {
      const ulonglong2 v = ((const ulonglong2*)s)[k2];
      sv[2 * k2] = v.x;
      sv[2 * k2 + 1] = v.y;
    }
    if (DENSE) fresh = sv[MW] == 0;
    newk += fresh;
    TRow<NC> prev{};
    if (!fresh) {
      prev.flags = (uint32_t)((sv[MW] & TS_FMASK) >> TS_FSHIFT);
      prev.gid = (int64_t)sv[MW + 1];
      prev.ghash = U8 ? (int64_t)sv[MW + 2] : prev.gid;
#pragma unroll
      for (int c = 0; c < NC; c++) prev.w[c] = (int64_t)sv[MW + 2 + U8 + c];
    }
    // One group change: + `add`'s contribution − `sub`'s (both null: a touch, the row time only).
    auto change = [&](const TRow<NC>& g, bool has_add, const TRow<NC>& add, bool has_sub, const TRow<NC>& sub,
                      int64_t t, int64_t claim_row) {
      bool isnew = false;
      const int64_t gs = group_find(A.table, A.gmask, A.p.slot_words, g.gid, g.ghash, claim_row, gkeys, &isnew);
      if (gs < 0) {
        failed++;
        return;
      }
      newg += isnew;
      if (isnew) A.glist[atomicAdd(&ctr[TC_GLIST], 1ULL)] = gs;  // finalized by k_tagg_grp_finalize
      uint64_t* gsl = A.table + (uint64_t)gs * (uint64_t)A.p.slot_words;
      // the row time only grows: no atomic when the slot already holds t or later (a stale read
      // is only ever lower, and then the atomic runs)
      if (isnew || (int64_t)gsl[2] < t)
        __hip_atomic_fetch_max((int64_t*)&gsl[2], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int q = 0; q < A.p.n_ops; q++) {
        const UpdOp op = A.p.ops[q];
        op_add_atomic(op, &gsl[op.word], op_delta<NC>(op, has_add, add, has_sub, sub));
      }
    };
    // Replay the key's changes in arrival order.  Every change undoes the previous row from its
    // group and applies the new one; over the push these telescope: the stored row A0 is undone
    // once (at the first change's time), the last row applied once (at its time), and every
    // intermediate row's +x / −x cancel — its group only takes the row time (and exists: a group
    // a row passed through stays, with its count back where it was).  Integer state is exact;
    // DOUBLE sums differ from the one-by-one order only by rounding.  `upd` counts the
    // undo/apply operations of the one-by-one replay (the push's statistics).
    const TRow<NC> a0 = prev;  // the stored row
    const bool a0_live = (a0.flags & (TF_LIVE | TF_GVALID)) == (TF_LIVE | TF_GVALID);
    bool first = true;
    int64_t t_first = 0, t_app = 0, r_app = -1;  // time / row of the current row's apply
    for (int64_t q = j; q < end; q++) {
      const int64_t r = sidx[q];
      int64_t t;
      uint32_t f;
      const TRow<NC> cur = rec_row<NC, U8>(rec, r, &t, &f);
      if (!(f & RF_ACC)) continue;
      if ((prev.flags & (TF_LIVE | TF_GVALID)) == (TF_LIVE | TF_GVALID)) {  // undo the previous row
        if (!first)  // an intermediate row: its group's row time is max(apply, undo)
          change(prev, false, prev, false, prev, t > t_app ? t : t_app, r_app);
        upd++;
      }
      if (first) t_first = t;
      first = false;
      r_app = -1;
      if (!(f & TF_LIVE)) {  // tombstone: the key leaves the table
        prev.flags = 0;
        continue;
      }
      if (f & TF_GVALID) {
        upd++;
        t_app = t;
        r_app = r;
      }
      prev = cur;
    }
    const bool last_live = r_app >= 0;  // the last row is live with a GROUP BY value (applied)
    if (!first) {
      if (a0_live && last_live && a0.gid == prev.gid) {  // one group: net (last − stored)
        change(prev, true, prev, true, a0, t_app > t_first ? t_app : t_first, r_app);
      } else {
        if (a0_live) change(a0, false, a0, true, a0, t_first, -1);
        if (last_live) change(prev, true, prev, false, prev, t_app, r_app);
      }
    }
    // the key's last row (or its deletion); a fresh hash slot keeps its claim until k_tagg_src_finalize
#pragma unroll
    for (int k2 = 0; k2 < 2 * NP; k2++) sv[k2] = 0;
    if (!DENSE) sv[0] = (uint64_t)id;
    sv[MW] = (!DENSE && fresh ? TS_CLAIM : TS_RESIDENT) | ((uint64_t)(prev.flags & 0xFFFFu) << TS_FSHIFT);
    sv[MW + 1] = (uint64_t)prev.gid;
    if (U8) sv[MW + 2] = (uint64_t)prev.ghash;
#pragma unroll
    for (int c = 0; c < NC; c++) sv[MW + 2 + U8 + c] = (uint64_t)prev.w[c];
#pragma unroll
    for (int k2 = 0; k2 < NP; k2++) ((ulonglong2*)s)[k2] = make_ulonglong2(sv[2 * k2], sv[2 * k2 + 1]);
    } while (0);
    if (!DENSE) claimed[j] = fresh_slot;
  }
  __shared__ int64_t lc[4][4];  // one add per block and counter
  const int64_t c4[4] = {wave_sum(upd), wave_sum(newg), wave_sum(failed), wave_sum(newk)};
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane < 4) lc[lane][wave] = c4[lane];
  __syncthreads();
  if (threadIdx.x < 4) {
    const int64_t v = lc[threadIdx.x][0] + lc[threadIdx.x][1] + lc[threadIdx.x][2] + lc[threadIdx.x][3];
    const int slot[4] = {TC_UPDATES, TC_NEW_GROUPS, TC_FAILED, TC_NEW_KEYS};
    if (v) atomicAdd(&ctr[slot[threadIdx.x]], (unsigned long long)v);
  }
}

// This push's group claims → resident groups (key word from the claiming row, ws = 0): only the
// claimed slots are visited, not the table.
__global__ __launch_bounds__(256) void k_tagg_grp_finalize(uint64_t* __restrict__ table, int sw,
                                                           const int64_t* __restrict__ list,
                                                           const unsigned long long* __restrict__ n_list,
                                                           const int64_t* __restrict__ gkeys) {
  const int64_t nc = (int64_t)*n_list;
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nc; k += (int64_t)gridDim.x * blockDim.x) {
    uint64_t* s = table + (uint64_t)list[k] * (uint64_t)sw;
    const uint64_t w0 = s[0];
    if ((int64_t)s[1] == EMPTY_WS && w0 != 0) {
      s[0] = (uint64_t)gkeys[(int64_t)(w0 & ((1ULL << 36) - 1))];
      s[1] = 0;
    }
  }
}

// This push's source claims → resident keys (k_tagg_apply wrote the key word and the flags;
// claimed[j] = the slot the leader at sorted position j claimed, else -1).
__global__ __launch_bounds__(256) void k_tagg_src_finalize(uint64_t* __restrict__ src, int ssw,
                                                           const int64_t* __restrict__ claimed, int64_t n) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = claimed[k];
    if (c < 0) continue;
    uint64_t* s = src + (uint64_t)c * (uint64_t)ssw;
    const uint64_t m = s[1];
    if (m & TS_CLAIM) s[1] = TS_RESIDENT | (m & TS_FMASK);
  }
}

__global__ __launch_bounds__(256) void k_tagg_src_rehash(const uint64_t* __restrict__ old, int64_t ocap,
                                                         uint64_t* __restrict__ nt, uint64_t nmask, int ssw) {
  for (int64_t slot = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; slot < ocap;
       slot += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t* s = old + slot * (uint64_t)ssw;
    const uint64_t m = s[1];
    if (!(m & TS_RESIDENT)) continue;
    if (!(((m & TS_FMASK) >> TS_FSHIFT) & TF_LIVE)) continue;  // deleted keys are dropped on rehash
    uint64_t d = src_hash((int64_t)s[0]) & nmask;
    while (atomicCAS((unsigned long long*)&nt[d * ssw + 1], 0ULL, (unsigned long long)m) != 0ULL) d = (d + 1) & nmask;
    uint64_t* q = nt + d * (uint64_t)ssw;
    q[0] = s[0];
    for (int w = 2; w < ssw; w++) q[w] = s[w];
  }
}

// Dense layout → hash layout (a push whose ids leave the dense window): every live key is
// inserted with its words (deleted keys are dropped, as on rehash).
__global__ __launch_bounds__(256) void k_tagg_dense_to_hash(const uint64_t* __restrict__ dense, int64_t dcap, int dsw,
                                                            int64_t dbase, uint64_t* __restrict__ nt, uint64_t nmask,
                                                            int ssw, int nwords) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < dcap; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t* d = dense + i * (uint64_t)dsw;
    const uint64_t m = d[0];
    if (!(m & TS_RESIDENT) || !(((m & TS_FMASK) >> TS_FSHIFT) & TF_LIVE)) continue;
    const int64_t id = (int64_t)((uint64_t)dbase + (uint64_t)i);
    uint64_t h = src_hash(id) & nmask;
    while (atomicCAS((unsigned long long*)&nt[h * ssw + 1], 0ULL, (unsigned long long)m) != 0ULL) h = (h + 1) & nmask;
    uint64_t* q = nt + h * (uint64_t)ssw;
    q[0] = (uint64_t)id;
    for (int w = 0; w < nwords; w++) q[2 + w] = d[1 + w];  // group id, hash, argument words
  }
}

__global__ __launch_bounds__(256) void k_tagg_src_count(const uint64_t* __restrict__ src, int64_t cap, int ssw,
                                                        unsigned long long* __restrict__ n) {
  int64_t c = 0;
  for (int64_t slot = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; slot < cap;
       slot += (int64_t)gridDim.x * blockDim.x)
    c += (src[slot * (uint64_t)ssw + 1] & TS_RESIDENT) ? 1 : 0;
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(n, (unsigned long long)c);
}

static int tgrid(int64_t work, int cap_blocks = 8192) {
  return (int)std::min<int64_t>(ceil_div(std::max<int64_t>(work, 1), 256), cap_blocks);
}

static khip_status src_alloc(khip_agg* a, DevBuf& buf, int64_t cap, int sw) {
  KHIP_TRY(buf.ensure((size_t)cap * sw * 8));
  KHIP_TRY_HIP(hipMemsetAsync(buf.p, 0, (size_t)cap * sw * 8, a->stream));
  return KHIP_OK;
}

// Live resident keys of a hash-layout table (deleted keys included), synchronously.
static khip_status src_count(khip_agg* a, const DevBuf& t, int64_t cap, int sw, int64_t* occ) {
  TaggState& T = a->tagg;
  KHIP_TRY(T.blk.ensure(8));
  KHIP_TRY_HIP(hipMemsetAsync(T.blk.p, 0, 8, a->stream));
  hipLaunchKernelGGL(k_tagg_src_count, dim3(tgrid(cap, 2048)), dim3(256), 0, a->stream, t.as<uint64_t>(), cap, sw,
                     T.blk.as<unsigned long long>());
  unsigned long long c = 0;
  KHIP_TRY_HIP(hipMemcpyAsync(&c, T.blk.p, 8, hipMemcpyDeviceToHost, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  *occ = (int64_t)c;
  return KHIP_OK;
}

// Grow the hash-layout source table, or move a dense one into a new hash table (deleted keys are
// dropped; the live ones re-inserted).
static khip_status src_grow(khip_agg* a, int64_t new_cap, int hsw, int nwords) {
  TaggState& T = a->tagg;
  DevBuf nt;
  KHIP_TRY(src_alloc(a, nt, new_cap, hsw));
  if (T.src_cap > 0 && T.src_occ > 0) {
    if (T.dense)
      hipLaunchKernelGGL(k_tagg_dense_to_hash, dim3(tgrid(T.src_cap)), dim3(256), 0, a->stream, T.src.as<uint64_t>(),
                         T.src_cap, T.src_sw, T.dbase, nt.as<uint64_t>(), (uint64_t)(new_cap - 1), hsw, nwords);
    else
      hipLaunchKernelGGL(k_tagg_src_rehash, dim3(tgrid(T.src_cap)), dim3(256), 0, a->stream, T.src.as<uint64_t>(),
                         T.src_cap, nt.as<uint64_t>(), (uint64_t)(new_cap - 1), hsw);
    KHIP_TRY_HIP(hipGetLastError());
  }
  int64_t occ = 0;
  KHIP_TRY(src_count(a, nt, new_cap, hsw, &occ));
  T.src.release();
  T.src = std::move(nt);
  nt.p = nullptr;
  T.src_cap = new_cap;
  T.src_occ = occ;
  T.src_sw = hsw;
  T.dense = false;
  return KHIP_OK;
}

// (Re)allocate the dense layout over [base, base + cap), keeping the slots of the current dense
// window (which it contains).
static khip_status src_dense(khip_agg* a, int64_t base, int64_t cap, int dsw) {
  TaggState& T = a->tagg;
  DevBuf nt;
  KHIP_TRY(src_alloc(a, nt, cap, dsw));
  if (T.dense && T.src_cap > 0)
    KHIP_TRY_HIP(hipMemcpyAsync(nt.as<uint64_t>() + (uint64_t)(T.dbase - base) * dsw, T.src.p,
                                (size_t)T.src_cap * dsw * 8, hipMemcpyDeviceToDevice, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  T.src.release();
  T.src = std::move(nt);
  nt.p = nullptr;
  T.src_cap = cap;
  T.src_sw = dsw;
  T.dbase = base;
  T.dense = true;
  return KHIP_OK;
}

// Source-table layout for a push whose accepted ids span [pmin, pmin + range] (none: range < 0).
// Dense while every id seen stays in a window of at most TAGG_DENSE_F slots per key the table may
// hold (and INT ids): slot = id − dbase, visited in sorted-id order by k_tagg_apply.  Otherwise —
// or once a push leaves that bound — the hash layout, at load <= 1/2 counting every row as a new
// key (a push cannot be resumed half-way: its undo/apply sequence is not idempotent).
constexpr int64_t TAGG_DENSE_F = 4;
static khip_status src_prepare(khip_agg* a, int64_t n, int64_t pmin, int64_t range, int nc, bool u8) {
  TaggState& T = a->tagg;
  const int hsw = (int)next_pow2(std::max(4, tagg_slot_words(nc, u8, false)));
  const int dsw = (int)next_pow2(std::max(2, tagg_slot_words(nc, u8, true)));
  const int nwords = 1 + (u8 ? 1 : 0) + nc;
  const bool can_dense = T.key_type != KHIP_KEY_UTF8 && knob("KHIP_TAGG_DENSE", 1) != 0;
  const int64_t keys = std::max<int64_t>(T.src_occ + n, 1 << 16);
  const int64_t dmax = std::min<int64_t>(TAGG_DENSE_F * keys, (int64_t)(32LL << 30) / (dsw * 8));
  if (range < 0) {  // nothing accepted: nothing to place
    if (T.src_cap == 0) KHIP_TRY(src_grow(a, 1024, hsw, nwords));
    return KHIP_OK;
  }
  if ((T.src_cap == 0 || T.dense) && can_dense) {
    int64_t lo = pmin, hi = (int64_t)((uint64_t)pmin + (uint64_t)range);  // inclusive
    if (T.dense && T.src_cap > 0) {
      lo = std::min(lo, T.dbase);
      hi = std::max(hi, T.dbase + T.src_cap - 1);
    }
    const uint64_t span = (uint64_t)hi - (uint64_t)lo;  // window - 1
    if ((uint64_t)range < (1ULL << 62) && span < (uint64_t)dmax) {
      if (!T.dense || lo != T.dbase || hi != T.dbase + T.src_cap - 1) {
        KHIP_TRY(src_dense(a, lo, next_pow2((int64_t)span + 1), dsw));
      }
      return KHIP_OK;
    }
  }
  if (T.src_cap == 0 || T.dense) KHIP_TRY(src_grow(a, next_pow2(std::max<int64_t>(1024, 2 * (T.src_occ + n))), hsw, nwords));
  else if (2 * (T.src_occ + n) > T.src_cap) KHIP_TRY(src_grow(a, next_pow2(2 * (T.src_occ + n)), hsw, nwords));
  return KHIP_OK;
}

khip_status tagg_push(khip_agg* a, int64_t n, const int64_t* gkeys, const int64_t* ghash, const uint8_t* kv,
                      const uint8_t* rv, const int64_t* ts, const ColPtrs& cols, const int64_t* src_id,
                      const uint8_t* src_kv, int64_t* tot) {
  TaggState& T = a->tagg;
  hipStream_t st = a->stream;
  if (n >= (1LL << 31)) return fail(KHIP_E_UNSUPPORTED, "table-source pushes above 2^31 rows");
  const bool u8 = a->desc.key_type == KHIP_KEY_UTF8;
  const int nc = a->desc.n_cols;
  KHIP_TRY(T.skey.ensure(n * 8));
  KHIP_TRY(T.skey2.ensure(n * 8));
  KHIP_TRY(T.sidx.ensure(n * 4));
  KHIP_TRY(T.sidx2.ensure(n * 4));
  KHIP_TRY(T.claimed.ensure(n * 8));
  KHIP_TRY(T.rec.ensure((size_t)n * tagg_rec_words(nc, u8) * 8));
  KHIP_TRY(T.gclaimed.ensure(n * 8));
  KHIP_TRY(T.ctr.ensure(TC_N * 8));
  unsigned long long* ctr = T.ctr.as<unsigned long long>();
  KHIP_TRY_HIP(hipMemsetAsync(ctr, 0, TC_N * 8, st));
  // the push's PRIMARY KEY range: the sort runs over (id − kmin) and only the bits that range needs
  const int rb = tgrid(n);
  KHIP_TRY(T.blk.ensure((size_t)rb * 40));
  unsigned long long* blkts = (unsigned long long*)(T.blk.as<ulonglong4>() + rb);
  hipLaunchKernelGGL(k_tagg_range, dim3(rb), dim3(256), 0, st, src_id, src_kv, rv, ts, gkeys, kv, n,
                     T.blk.as<ulonglong4>(), blkts);
  hipLaunchKernelGGL(k_tagg_range_reduce, dim3(1), dim3(256), 0, st, T.blk.as<ulonglong4>(), blkts, rb, ctr);
  unsigned long long kr[2] = {0, 0}, gr[2] = {0, 0};
  KHIP_TRY_HIP(hipMemcpyAsync(kr, ctr + TC_KMINN, sizeof(kr), hipMemcpyDeviceToHost, st));
  KHIP_TRY_HIP(hipMemcpyAsync(gr, ctr + TC_GMINN, sizeof(gr), hipMemcpyDeviceToHost, st));
  KHIP_TRY_HIP(hipStreamSynchronize(st));
  // group capacity ahead of time: the push creates at most min(n, distinct GROUP BY keys) groups,
  // and its GROUP BY keys (or dictionary ids) all lie in [gmin, gmax]
  int64_t new_groups = 0;
  if (gr[0] | gr[1]) {
    const uint64_t gspan = ((uint64_t)gr[1] ^ (1ULL << 63)) - (~(uint64_t)gr[0] ^ (1ULL << 63));
    new_groups = gspan >= (uint64_t)n ? n : (int64_t)gspan + 1;
  }
  // 8 slots per group: hot groups rarely share a cache line (2 / 4 / 8 / 32 measured within 2 %,
  // profiles/r03/ab/tagg_group_load.txt); the table stays O(groups), not O(rows) as before
  const int64_t glf = knob("KHIP_TAGG_GLF", 8);
  if (glf * (a->occ + new_groups) > a->cap) KHIP_TRY(agg_grow_table(a, next_pow2(glf * (a->occ + new_groups))));
  int64_t kmin = 0;
  uint64_t range = 0;
  if (kr[0] | kr[1]) {  // some row accepted (both words are 0 only when none was)
    kmin = (int64_t)(~(uint64_t)kr[0] ^ (1ULL << 63));
    range = (uint64_t)(int64_t)((uint64_t)kr[1] ^ (1ULL << 63)) - (uint64_t)kmin;
  }
  KHIP_TRY(src_prepare(a, n, kmin, (kr[0] | kr[1]) ? (int64_t)std::min<uint64_t>(range, (uint64_t)INT64_MAX) : -1, nc,
                       u8));
  const uint64_t drop = range != ~0ULL ? range + 1 : range;  // full 64-bit range: dropped rows share
  const int end_bit = drop ? 64 - __builtin_clzll(drop) : 1;  // the last key's segment (rows re-checked)
  TaggKeysArgs K{};
  K.src_id = src_id;
  K.src_kv = src_kv;
  K.ts = ts;
  K.gkeys = gkeys;
  K.ghash = ghash;
  K.kv = kv;
  K.rv = rv;
  K.cols = cols;
  for (int c = 0; c < MAX_COLS; c++) K.col_type[c] = a->ap.col_type[c];
  K.n = n;
  K.kmin = kmin;
  K.drop = drop;
  using KeysFn = void (*)(TaggKeysArgs, uint64_t*, uint32_t*, uint64_t*, unsigned long long*);
  static const KeysFn kkeys[2][MAX_COLS + 1] = {
      {k_tagg_keys<0, false>, k_tagg_keys<1, false>, k_tagg_keys<2, false>, k_tagg_keys<3, false>, k_tagg_keys<4, false>,
       k_tagg_keys<5, false>, k_tagg_keys<6, false>, k_tagg_keys<7, false>, k_tagg_keys<8, false>},
      {k_tagg_keys<0, true>, k_tagg_keys<1, true>, k_tagg_keys<2, true>, k_tagg_keys<3, true>, k_tagg_keys<4, true>,
       k_tagg_keys<5, true>, k_tagg_keys<6, true>, k_tagg_keys<7, true>, k_tagg_keys<8, true>}};
  hipLaunchKernelGGL(kkeys[u8][nc], dim3(tgrid(n)), dim3(256), 0, st, K, T.skey.as<uint64_t>(), T.sidx.as<uint32_t>(),
                     T.rec.as<uint64_t>(), ctr);
  KHIP_TRY_HIP(hipGetLastError());
  uint64_t* kin = T.skey.as<uint64_t>();
  uint64_t* kout = T.skey2.as<uint64_t>();
  uint32_t* vin = T.sidx.as<uint32_t>();
  uint32_t* vout = T.sidx2.as<uint32_t>();
  KHIP_TRY(ksort::sort_pairs<uint32_t>(st, T.tmp, T.tmp2, kin, kout, vin, vout, n, end_bit));
  TaggArgs A{};
  A.p = a->ap;
  A.table = a->table.as<uint64_t>();
  A.gmask = (uint64_t)(a->cap - 1);
  A.src = T.src.as<uint64_t>();
  A.smask = (uint64_t)(T.src_cap - 1);
  A.ssw = T.src_sw;
  A.n = n;
  A.glist = T.gclaimed.as<int64_t>();
  A.kmin = kmin;
  A.drop = drop;
  A.dbase = T.dbase;
  using ApplyFn = void (*)(TaggArgs, const uint64_t*, const uint32_t*, const uint64_t*, const int64_t*, int64_t*,
                           unsigned long long*);
#define KHIP_TAPPLY(U, D)                                                                                        \
  {k_tagg_apply<0, U, D>, k_tagg_apply<1, U, D>, k_tagg_apply<2, U, D>, k_tagg_apply<3, U, D>,                  \
   k_tagg_apply<4, U, D>, k_tagg_apply<5, U, D>, k_tagg_apply<6, U, D>, k_tagg_apply<7, U, D>,                  \
   k_tagg_apply<8, U, D>}
  static const ApplyFn kapply[2][2][MAX_COLS + 1] = {{KHIP_TAPPLY(false, false), KHIP_TAPPLY(true, false)},
                                                     {KHIP_TAPPLY(false, true), KHIP_TAPPLY(true, true)}};
#undef KHIP_TAPPLY
  hipLaunchKernelGGL(kapply[T.dense][u8][nc], dim3(ceil_div(n, TA_C)), dim3(256), 0, st, A, kout, vout,
                     T.rec.as<uint64_t>(), gkeys, T.claimed.as<int64_t>(), ctr);
  KHIP_TRY_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_tagg_grp_finalize, dim3(tgrid(n, 1024)), dim3(256), 0, st, a->table.as<uint64_t>(), a->sw,
                     T.gclaimed.as<int64_t>(), (const unsigned long long*)&ctr[TC_GLIST], gkeys);
  if (!T.dense)  // hash layout: this push's claims → resident keys
    hipLaunchKernelGGL(k_tagg_src_finalize, dim3(tgrid(n)), dim3(256), 0, st, T.src.as<uint64_t>(), T.src_sw,
                       T.claimed.as<int64_t>(), n);
  KHIP_TRY_HIP(hipGetLastError());
  unsigned long long c[TC_N];
  KHIP_TRY_HIP(hipMemcpyAsync(c, ctr, sizeof(c), hipMemcpyDeviceToHost, st));
  KHIP_TRY_HIP(hipStreamSynchronize(st));
  if (c[TC_FAILED]) return fail(KHIP_E_DEVICE, "table aggregation: hash table probe budget exhausted");
  T.src_occ += (int64_t)c[TC_NEW_KEYS];
  a->occ += (int64_t)c[TC_NEW_GROUPS];
  if (c[TC_TSMAX] && (int64_t)c[TC_TSMAX] - 1 > a->host_stream_time) {  // the oracle's stream time (oracle.c:862)
    a->host_stream_time = (int64_t)c[TC_TSMAX] - 1;
    KHIP_TRY_HIP(hipMemcpyAsync(a->stream_time.p, &a->host_stream_time, 8, hipMemcpyHostToDevice, st));
    KHIP_TRY_HIP(hipStreamSynchronize(st));
  }
  tot[P_ACCEPTED] += (int64_t)c[TC_ACCEPTED];
  tot[P_NULL_KEY] += (int64_t)c[TC_NULL_KEY];
  tot[P_BAD_TS] += (int64_t)c[TC_BAD_TS];
  tot[P_APPLIED] += (int64_t)c[TC_UPDATES];
  tot[P_NEW] += (int64_t)c[TC_NEW_GROUPS];
  return KHIP_OK;
}

khip_status tagg_reset(khip_agg* a) {
  TaggState& T = a->tagg;
  if (T.src_cap) KHIP_TRY_HIP(hipMemsetAsync(T.src.p, 0, (size_t)T.src_cap * T.src_sw * 8, a->stream));
  T.src_occ = 0;
  if (T.key_type == KHIP_KEY_UTF8) KHIP_TRY(dict_clear(T.dict, a->stream));
  return KHIP_OK;
}

void tagg_release(khip_agg* a) {
  TaggState& T = a->tagg;
  DevBuf* bufs[] = {&T.src,     &T.sid,    &T.skey,      &T.skey2, &T.sidx,   &T.sidx2, &T.rec,
                    &T.tmp,     &T.ctr,    &T.claimed,   &T.gclaimed, &T.blk,  &T.st_koff,
                    &T.st_kbytes, &T.st_kv, &T.st_key,   &T.shash};
  for (DevBuf* b : bufs) b->release();
  dict_release(T.dict);
  T.src_cap = T.src_occ = 0;
}

}  // namespace khip
