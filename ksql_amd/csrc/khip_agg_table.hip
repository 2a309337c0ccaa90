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
//   [0] key  [1] meta: 0 empty | bit63 claimed by this push (bits 0..39 = sorted position) |
//                      bit62 resident
//   [2] flags: bit0 live, bit1 GROUP BY value non-null, bits 8.. argument validity
//   [3] group id  [4] group-key hash  [5..] argument words (raw 8 bytes)
//
// Per push (all on the handle's stream):
//   k_tagg_range   the push's PRIMARY KEY range (per-block partials, one reducing workgroup)
//   k_tagg_keys    sort key = PRIMARY KEY id − kmin (dropped rows sort last), value = row; counts
//   radix sort over the range's bits only (khip_sort.hpp; stable: a key's rows keep their arrival order)
//   k_tagg_apply   one thread per distinct PRIMARY KEY (segment leader): find-or-claim its source
//                  slot (claim references the sorted position: no spin), then replay its rows in
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

constexpr int TS_WORDS = 5;
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

// Sort key = PRIMARY KEY id − kmin (dropped rows: `drop`, which sorts last), value = row; counts.
__global__ __launch_bounds__(256) void k_tagg_keys(const int64_t* __restrict__ src_id, const uint8_t* __restrict__ src_kv,
                                                   const int64_t* __restrict__ ts, int64_t n, int64_t kmin, uint64_t drop,
                                                   uint64_t* __restrict__ skey, uint32_t* __restrict__ sidx,
                                                   unsigned long long* __restrict__ ctr) {
  int64_t acc = 0, nk = 0, bt = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool kv = bit_get(src_kv, i);
    const bool ok = kv && ts[i] >= 0;
    skey[i] = ok ? (uint64_t)src_id[i] - (uint64_t)kmin : drop;
    sidx[i] = (uint32_t)i;
    acc += ok;
    nk += !kv;
    bt += kv && ts[i] < 0;
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

// One row's aggregate contribution: argument words + validity mask (bit c = column c non-null).
// NC (the handle's argument column count) is a template parameter: the words stay in registers
// (a run-time bound would index them dynamically and put every row in scratch memory).
template <int NC>
struct TRow {
  int64_t gid, ghash;
  uint32_t flags;  // TF_* | valid mask << 8
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

// One group's net change from one source key's changes in this push: + `add`'s contribution, −
// `sub`'s (either may be null; both null = a touch: the row time only — a group an intermediate
// row of the key passed through, whose +x / −x cancel).  The group is found, or claimed when
// claim_row >= 0 (the claim references that batch row, whose GROUP BY key is the group's).
// Returns 0 on probe exhaustion, 1 on update, 2 on update of a newly claimed group.
template <int NC>
__device__ __forceinline__ int group_net(const ApplyParams& p, uint64_t* __restrict__ table, uint64_t mask,
                                         int64_t gid, int64_t ghash, bool has_add, const TRow<NC>& add, bool has_sub,
                                         const TRow<NC>& sub, int64_t t,
                                         int64_t claim_row, const int64_t* __restrict__ gkeys,
                                         int64_t* __restrict__ glist, unsigned long long* __restrict__ ctr) {
  const uint64_t h = group_hash(ghash, 0);
  const uint64_t fp = (h >> 49) & 0x7FFFULL;
  const uint64_t myref = (1ULL << 63) | (fp << 48) | (uint64_t)(claim_row < 0 ? 0 : claim_row);
  uint64_t slot = h & mask;
  const int sw = p.slot_words;
  for (int probe = 0; probe < MAX_PROBE; probe++) {
    uint64_t* s = table + slot * (uint64_t)sw;
    const int64_t w1 = (int64_t)ld_relaxed(&s[1]);
    const int64_t w2 = (int64_t)ld_relaxed(&s[2]);  // row time, loaded beside the slot's state
    bool hit = false;
    int isnew = 0;
    if (w1 != EMPTY_WS) {
      hit = (int64_t)s[0] == gid;
    } else {
      uint64_t w0 = ld_relaxed(s);
      if (w0 == 0) {
        if (claim_row < 0) return 0;  // an undo always finds its group
        const uint64_t old = atomicCAS((unsigned long long*)s, 0ULL, (unsigned long long)myref);
        if (old == 0) {
          hit = true;
          isnew = 1;
          glist[atomicAdd(&ctr[TC_GLIST], 1ULL)] = (int64_t)slot;  // finalized by k_tagg_grp_finalize
        } else {
          w0 = old;
        }
      }
      if (!hit && ((w0 >> 48) & 0x7FFFULL) == fp) hit = gkeys[(int64_t)(w0 & ((1ULL << 36) - 1))] == gid;
    }
    if (hit) {
      // the row time only grows: no atomic when the slot already holds t or later (a stale or
      // pre-claim read is only ever lower, and then the atomic runs)
      if (isnew || w2 < t) __hip_atomic_fetch_max((int64_t*)&s[2], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int o = 0; o < p.n_ops; o++) {
        const UpdOp op = p.ops[o];
        int64_t* w = (int64_t*)&s[op.word];
        const bool va = has_add && (op.kind == OP_INC || ((add.flags >> (8 + op.col)) & 1u));
        const bool vs = has_sub && (op.kind == OP_INC || ((sub.flags >> (8 + op.col)) & 1u));
        if (!va && !vs) continue;  // null arguments (undo too): unchanged
        switch (op.kind) {
          case OP_INC:        // COUNT(*) = COUNT(ROWTIME): never null
          case OP_INC_VALID: {
            const int64_t d = (int64_t)va - (int64_t)vs;
            if (d) __hip_atomic_fetch_add(w, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          case OP_ADD_I64: {  // INT / BIGINT: wrapping (INT truncated to 32 bits when read)
            const uint64_t d = (va ? (uint64_t)wpick(add, op.col) : 0) - (vs ? (uint64_t)wpick(sub, op.col) : 0);
            if (d) __hip_atomic_fetch_add((uint64_t*)w, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          case OP_ADD_F64: {
            double x = 0, y = 0;
            if (va) x = __longlong_as_double(wpick(add, op.col));
            if (vs) y = __longlong_as_double(wpick(sub, op.col));
            unsafeAtomicAdd((double*)w, va && vs ? x - y : (va ? x : -y));
            break;
          }
          default:  // MIN / MAX are rejected at create (not undoable)
            break;
        }
      }
      return 1 + isnew;
    }
    slot = (slot + 1) & mask;
  }
  return 0;
}

struct TaggArgs {
  ApplyParams p;
  uint64_t* table;  // group table
  uint64_t gmask;
  uint64_t* src;    // source table
  uint64_t smask;
  int32_t ssw;
  int32_t n_cols;
  int32_t col_type[MAX_COLS];
  int64_t n;
  int64_t* glist;   // group slots claimed by this push
  int64_t kmin;     // sort keys are PRIMARY KEY id − kmin
};

__device__ __forceinline__ int64_t load_word(const ColPtrs& c, int32_t type, int col, int64_t i) {
  return type == KHIP_TYPE_INT32 ? (int64_t)((const int32_t*)c.data[col])[i] : ((const int64_t*)c.data[col])[i];
}

template <int NC>
__global__ __launch_bounds__(256) void k_tagg_apply(TaggArgs A, const uint64_t* __restrict__ skey,
                                                    const uint32_t* __restrict__ sidx, const int64_t* __restrict__ gkeys,
                                                    const int64_t* __restrict__ ghash, const uint8_t* __restrict__ kv,
                                                    const uint8_t* __restrict__ rv, const int64_t* __restrict__ ts,
                                                    ColPtrs cols, const uint8_t* __restrict__ src_kv,
                                                    int64_t* __restrict__ claimed, unsigned long long* __restrict__ ctr) {
  int64_t upd = 0, newg = 0, failed = 0;
  const int lane = threadIdx.x & 63;
  const uint64_t below = lane ? (~0ULL >> (64 - lane)) : 0ULL;
  // every lane of a wave runs the same iterations: new source slots are listed with one counter
  // add per wave (a returning same-address atomic per new key would serialize)
  for (int64_t j0 = blockIdx.x * (int64_t)blockDim.x; j0 < A.n; j0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = j0 + threadIdx.x;
    int64_t fresh_slot = -1;
    if (j < A.n) do {  // `continue` below leaves this record's body
    const uint64_t k = skey[j];
    if (j > 0 && skey[j - 1] == k) continue;  // not the segment leader
    int64_t end = j + 1;
    while (end < A.n && skey[end] == k) end++;
    // a segment of dropped rows only (UINT64_MAX that no accepted key shares)
    bool any = false;
    for (int64_t q = j; q < end && !any; q++) {
      const int64_t r = sidx[q];
      any = bit_get(src_kv, r) && ts[r] >= 0;
    }
    if (!any) continue;
    const int64_t id = (int64_t)(k + (uint64_t)A.kmin);
    // find or claim the key's source slot (only this thread holds this key)
    uint64_t slot = src_hash(id) & A.smask;
    uint64_t* s = nullptr;
    bool fresh = false;
    for (int probe = 0; probe < TS_MAX_PROBE; probe++) {
      uint64_t* c = A.src + slot * (uint64_t)A.ssw;
      uint64_t m = ld_relaxed(&c[1]);
      if (m == 0) {
        const uint64_t old = atomicCAS((unsigned long long*)&c[1], 0ULL, (unsigned long long)(TS_CLAIM | (uint64_t)j));
        if (old == 0) {
          s = c;
          fresh = true;
          break;
        }
        m = old;
      }
      // another key's claim of this push (compare by its sorted key) or a resident key
      if (!(m & TS_CLAIM) && (int64_t)c[0] == id) {
        s = c;
        break;
      }
      slot = (slot + 1) & A.smask;
    }
    if (!s) {
      failed++;
      continue;
    }
    TRow<NC> prev{};
    if (!fresh) {
      prev.flags = (uint32_t)s[2];
      prev.gid = (int64_t)s[3];
      prev.ghash = (int64_t)s[4];
      _Pragma("unroll") for (int c = 0; c < NC; c++) prev.w[c] = (int64_t)s[TS_WORDS + c];
    } else {
      fresh_slot = (int64_t)slot;
    }
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
      const int64_t t = ts[r];
      if (!bit_get(src_kv, r) || t < 0) continue;
      if ((prev.flags & (TF_LIVE | TF_GVALID)) == (TF_LIVE | TF_GVALID)) {  // undo the previous row
        if (!first) {  // an intermediate row: its group's row time is max(apply, undo)
          const int u = group_net<NC>(A.p, A.table, A.gmask, prev.gid, prev.ghash, false, prev, false, prev,
                                      t > t_app ? t : t_app, r_app, gkeys, A.glist, ctr);
          if (u == 0) failed++;
          newg += u == 2;
        }
        upd++;
      }
      if (first) t_first = t;
      first = false;
      r_app = -1;
      if (!bit_get(rv, r)) {  // tombstone: the key leaves the table
        prev.flags = 0;
        continue;
      }
      TRow<NC> cur{};
      cur.flags = TF_LIVE;
      if (bit_get(kv, r)) {
        cur.flags |= TF_GVALID;
        cur.gid = gkeys[r];
        cur.ghash = ghash[r];
      }
      _Pragma("unroll") for (int c = 0; c < NC; c++) {
        const bool v = bit_get(cols.valid[c], r);
        cur.w[c] = v ? load_word(cols, A.col_type[c], c, r) : 0;
        cur.flags |= (v ? 1u : 0u) << (8 + c);
      }
      if (cur.flags & TF_GVALID) {
        upd++;
        t_app = t;
        r_app = r;
      }
      prev = cur;
    }
    const bool last_live = r_app >= 0;  // the last row is live with a GROUP BY value (applied)
    if (!first) {
      if (a0_live && last_live && a0.gid == prev.gid) {  // one group: net (last − stored)
        const int u = group_net<NC>(A.p, A.table, A.gmask, prev.gid, prev.ghash, true, prev, true, a0,
                                    t_app > t_first ? t_app : t_first, r_app, gkeys, A.glist, ctr);
        if (u == 0) failed++;
        newg += u == 2;
      } else {
        if (a0_live) {
          const int u = group_net<NC>(A.p, A.table, A.gmask, a0.gid, a0.ghash, false, a0, true, a0, t_first, -1, gkeys, A.glist, ctr);
          if (u == 0) failed++;
        }
        if (last_live) {
          const int u = group_net<NC>(A.p, A.table, A.gmask, prev.gid, prev.ghash, true, prev, false, prev, t_app, r_app, gkeys,
                                      A.glist, ctr);
          if (u == 0) failed++;
          newg += u == 2;
        }
      }
    }
    // the key's last row (or its deletion)
    s[2] = prev.flags;
    s[3] = (uint64_t)prev.gid;
    s[4] = (uint64_t)prev.ghash;
    _Pragma("unroll") for (int c = 0; c < NC; c++) s[TS_WORDS + c] = (uint64_t)prev.w[c];
    } while (0);
    const uint64_t mk = __ballot(fresh_slot >= 0);
    if (mk) {
      const int first = __ffsll((unsigned long long)mk) - 1;
      unsigned long long x0 = 0;
      if (lane == first) x0 = atomicAdd(&ctr[TC_NEW_KEYS], (unsigned long long)__popcll(mk));
      x0 = __shfl(x0, first, 64);
      if (fresh_slot >= 0) claimed[(int64_t)x0 + __popcll(mk & below)] = fresh_slot;
    }
  }
  __shared__ int64_t lc[3][4];  // one add per block and counter
  const int64_t c3[3] = {wave_sum(upd), wave_sum(newg), wave_sum(failed)};
  const int wave = threadIdx.x >> 6;
  if (lane < 3) lc[lane][wave] = c3[lane];
  __syncthreads();
  if (threadIdx.x < 3) {
    const int64_t v = lc[threadIdx.x][0] + lc[threadIdx.x][1] + lc[threadIdx.x][2] + lc[threadIdx.x][3];
    const int slot[3] = {TC_UPDATES, TC_NEW_GROUPS, TC_FAILED};
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

// This push's source claims → resident keys (the claim holds the sorted position of the key).
__global__ __launch_bounds__(256) void k_tagg_src_finalize(uint64_t* __restrict__ src, int ssw,
                                                           const int64_t* __restrict__ claimed,
                                                           const unsigned long long* __restrict__ n_claimed,
                                                           const uint64_t* __restrict__ skey, int64_t kmin) {
  const int64_t nc = (int64_t)*n_claimed;
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nc; k += (int64_t)gridDim.x * blockDim.x) {
    uint64_t* s = src + (uint64_t)claimed[k] * (uint64_t)ssw;
    const uint64_t m = s[1];
    if (m & TS_CLAIM) {
      s[0] = skey[(int64_t)(m & ((1ULL << 40) - 1))] + (uint64_t)kmin;
      s[1] = TS_RESIDENT;
    }
  }
}

__global__ __launch_bounds__(256) void k_tagg_src_rehash(const uint64_t* __restrict__ old, int64_t ocap,
                                                         uint64_t* __restrict__ nt, uint64_t nmask, int ssw) {
  for (int64_t slot = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; slot < ocap;
       slot += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t* s = old + slot * (uint64_t)ssw;
    if (!(s[1] & TS_RESIDENT)) continue;
    if (!(s[2] & TF_LIVE)) continue;  // deleted keys are dropped on rehash
    uint64_t d = src_hash((int64_t)s[0]) & nmask;
    while (atomicCAS((unsigned long long*)&nt[d * ssw + 1], 0ULL, (unsigned long long)TS_RESIDENT) != 0ULL)
      d = (d + 1) & nmask;
    uint64_t* q = nt + d * (uint64_t)ssw;
    q[0] = s[0];
    for (int w = 2; w < ssw; w++) q[w] = s[w];
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

static khip_status src_alloc(khip_agg* a, DevBuf& buf, int64_t cap) {
  TaggState& T = a->tagg;
  KHIP_TRY(buf.ensure((size_t)cap * T.src_sw * 8));
  KHIP_TRY_HIP(hipMemsetAsync(buf.p, 0, (size_t)cap * T.src_sw * 8, a->stream));
  return KHIP_OK;
}

// Grow the source table (deleted keys are dropped; the live ones re-inserted).
static khip_status src_grow(khip_agg* a, int64_t new_cap) {
  TaggState& T = a->tagg;
  DevBuf nt;
  KHIP_TRY(src_alloc(a, nt, new_cap));
  if (T.src_cap > 0 && T.src_occ > 0) {
    hipLaunchKernelGGL(k_tagg_src_rehash, dim3(tgrid(T.src_cap)), dim3(256), 0, a->stream, T.src.as<uint64_t>(),
                       T.src_cap, nt.as<uint64_t>(), (uint64_t)(new_cap - 1), T.src_sw);
    KHIP_TRY_HIP(hipGetLastError());
  }
  KHIP_TRY(T.ctr.ensure(TC_N * 8));
  KHIP_TRY_HIP(hipMemsetAsync(T.ctr.p, 0, 8, a->stream));
  hipLaunchKernelGGL(k_tagg_src_count, dim3(tgrid(new_cap, 2048)), dim3(256), 0, a->stream, nt.as<uint64_t>(), new_cap,
                     T.src_sw, T.ctr.as<unsigned long long>());
  unsigned long long occ = 0;
  KHIP_TRY_HIP(hipMemcpyAsync(&occ, T.ctr.p, 8, hipMemcpyDeviceToHost, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  T.src.release();
  T.src = nt;
  nt.p = nullptr;
  T.src_cap = new_cap;
  T.src_occ = (int64_t)occ;
  return KHIP_OK;
}

khip_status tagg_push(khip_agg* a, int64_t n, const int64_t* gkeys, const int64_t* ghash, const uint8_t* kv,
                      const uint8_t* rv, const int64_t* ts, const ColPtrs& cols, const int64_t* src_id,
                      const uint8_t* src_kv, int64_t* tot) {
  TaggState& T = a->tagg;
  hipStream_t st = a->stream;
  if (n >= (1LL << 31)) return fail(KHIP_E_UNSUPPORTED, "table-source pushes above 2^31 rows");
  T.src_sw = (int)next_pow2(std::max(8, TS_WORDS + a->desc.n_cols));
  // capacity ahead of time: every row a new key / a new group at load <= 1/2 (a push cannot be
  // resumed half-way: its undo/apply sequence is not idempotent)
  if (T.src_cap == 0) KHIP_TRY(src_grow(a, next_pow2(std::max<int64_t>(1024, 2 * n))));
  else if (2 * (T.src_occ + n) > T.src_cap) KHIP_TRY(src_grow(a, next_pow2(2 * (T.src_occ + n))));
  KHIP_TRY(T.skey.ensure(n * 8));
  KHIP_TRY(T.skey2.ensure(n * 8));
  KHIP_TRY(T.sidx.ensure(n * 4));
  KHIP_TRY(T.sidx2.ensure(n * 4));
  KHIP_TRY(T.claimed.ensure(n * 8));
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
  const uint64_t drop = range != ~0ULL ? range + 1 : range;  // full 64-bit range: dropped rows share
  const int end_bit = drop ? 64 - __builtin_clzll(drop) : 1;  // the last key's segment (rows re-checked)
  hipLaunchKernelGGL(k_tagg_keys, dim3(tgrid(n)), dim3(256), 0, st, src_id, src_kv, ts, n, kmin, drop,
                     T.skey.as<uint64_t>(), T.sidx.as<uint32_t>(), ctr);
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
  A.n_cols = a->desc.n_cols;
  for (int c = 0; c < MAX_COLS; c++) A.col_type[c] = a->ap.col_type[c];
  A.n = n;
  A.glist = T.gclaimed.as<int64_t>();
  A.kmin = kmin;
  static void (*const kapply[MAX_COLS + 1])(TaggArgs, const uint64_t*, const uint32_t*, const int64_t*, const int64_t*,
                                            const uint8_t*, const uint8_t*, const int64_t*, ColPtrs, const uint8_t*,
                                            int64_t*, unsigned long long*) = {
      k_tagg_apply<0>, k_tagg_apply<1>, k_tagg_apply<2>, k_tagg_apply<3>, k_tagg_apply<4>,
      k_tagg_apply<5>, k_tagg_apply<6>, k_tagg_apply<7>, k_tagg_apply<8>};
  hipLaunchKernelGGL(kapply[A.n_cols], dim3(tgrid(n, 16384)), dim3(256), 0, st, A, kout, vout, gkeys, ghash, kv, rv,
                     ts, cols, src_kv, T.claimed.as<int64_t>(), ctr);
  hipLaunchKernelGGL(k_tagg_grp_finalize, dim3(tgrid(n, 1024)), dim3(256), 0, st, a->table.as<uint64_t>(), a->sw,
                     T.gclaimed.as<int64_t>(), (const unsigned long long*)&ctr[TC_GLIST], gkeys);
  hipLaunchKernelGGL(k_tagg_src_finalize, dim3(tgrid(n)), dim3(256), 0, st, T.src.as<uint64_t>(), T.src_sw,
                     T.claimed.as<int64_t>(), (const unsigned long long*)&ctr[TC_NEW_KEYS], kout, kmin);
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
  DevBuf* bufs[] = {&T.src, &T.sid, &T.skey, &T.skey2, &T.sidx, &T.sidx2, &T.tmp, &T.ctr, &T.claimed, &T.gclaimed,
                    &T.st_koff, &T.st_kbytes, &T.st_kv, &T.st_key, &T.shash};
  for (DevBuf* b : bufs) b->release();
  dict_release(T.dict);
  T.src_cap = T.src_occ = 0;
}

}  // namespace khip
