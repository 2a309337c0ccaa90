// khip_agg_session.hip — SESSION-windowed GROUP BY on MI355X (gfx950).
//
// Replaces KStreamSessionWindowAggregate + the RocksDB session store that
// StreamAggregateBuilder.visitSessionWindowExpression builds (S/StreamAggregateBuilder.java:
// 296-323; merger = KudafAggregator.getMerger, X/function/udaf/KudafAggregator.java:87-111).
// Semantics: oracle rule R11 (pinned by Q/session-windows.json).
//
// HBM layout: the session store is one array of rows sorted by (key, session start), the row
// layout of the other engines: [key, start, end (= row time), state words ...].  Sessions of a
// key are disjoint, so sorted by start they are also sorted by end.
//
// Per push (all on the handle's stream):
//   k_sess_range / k_scan_blocks stream time before each 2048-record block; the key range
//   k_sess_prep                  per record: accepted?, stream time after it, packed with ts into
//                                8 bytes relative to the push's time base (16 when the push spans
//                                2^32 ms); (key - kmin, record) pairs
//   radix sort (khip_sort.hpp)   records grouped by key, arrival order kept inside a key; only
//                                the bits of the push's key range are sorted
//   k_sess_gather                (argument columns or 16-byte records: the sort carries row
//                                indices) the records in sorted order
//   run-length encode            one segment per batch key
//   k_sess_bounds                the key's store range (binary search), scratch capacity
//   k_sess_apply                 ONE THREAD PER KEY replays the key's records in arrival order
//                                against its sessions (merging is inherently sequential per key,
//                                keys are independent): find the overlapping run, merge, late
//                                drop, expiry; emits the push's changelog rows (updates and
//                                tombstones of merged-away sessions)
//   k_sess_keep / k_sess_scatter the new store = untouched keys' sessions (minus expired) merged
//                                in key order with the rewritten keys' sessions

#include <algorithm>
#include <vector>

#include "khip_util.hpp"

#include "khip_agg_internal.hpp"
#include "khip_sort.hpp"

namespace khip {

constexpr uint8_t SF_TOUCHED = 1, SF_ORIG = 2, SF_OLDP = 4;

struct SessParams {
  ApplyParams ap;
  InitWords init;
  HavingDev having;
  int32_t sw;
  int64_t gap, grace, retention;
  // EMIT FINAL (Kafka 3.4 KStreamSessionWindowAggregate.maybeForwardFinalResult; oracle R11): the
  // push emits the sessions whose end passes into [fin_lo, close after the push), fin_lo =
  // max(0, close before the push), close = stream time - grace - gap
  int32_t fin;
  int64_t fin_lo;
};

// Accepted records (valid key and value, ts >= 0): per-block ts maximum (for the stream-time
// prefix), and the key range of the push (min / max as order-preserving unsigned words,
// atomic-max'd: ctr[C_KMINN] = max of ~u, ctr[C_KMAX] = max of u, ctr[C_KACC] = accepted).
// Coalesced: element k of thread t is base + k * BLOCK + t.
constexpr int C_KMINN = 20, C_KMAX = 21, C_KACC = 22, C_TBASE = 23;

__device__ __forceinline__ uint64_t key_ord(int64_t k) { return (uint64_t)k ^ (1ULL << 63); }

__device__ __forceinline__ bool sess_ok(const uint8_t* kv, const uint8_t* rv, const int64_t* ts, int64_t i,
                                        int64_t* t) {
  *t = ts[i];
  return bit_get(kv, i) && bit_get(rv, i) && *t >= 0;
}

__global__ __launch_bounds__(BLOCK) void k_sess_range(const int64_t* __restrict__ keys, const int64_t* __restrict__ ts,
                                                      const uint8_t* __restrict__ kv, const uint8_t* __restrict__ rv,
                                                      int64_t n, int64_t* __restrict__ blockmax,
                                                      ulonglong2* __restrict__ blockkr, int64_t* __restrict__ blockacc,
                                                      int64_t* __restrict__ blocktmin, const int64_t* __restrict__ st_at) {
  __shared__ int64_t lds[BLOCK / 64];
  __shared__ uint64_t lk[3][BLOCK / 64];
  __shared__ int64_t la[BLOCK / 64];
  const int64_t base = (int64_t)blockIdx.x * RPB;
  int64_t m = -1, tmn = INT64_MAX;
  uint64_t kmn = 0, kmx = 0;
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < ITEMS; k++) {
    const int64_t i = base + k * BLOCK + threadIdx.x;
    int64_t t;
    if (i < n && sess_ok(kv, rv, ts, i, &t)) {
      const int64_t sx = st_at ? st_at[i] : t;  // KHIP_TIME_SUPPLIED: the row's given stream time
      m = sx > m ? sx : m;
      tmn = t < tmn ? t : tmn;
      const uint64_t u = key_ord(keys[i]);
      kmn = ~u > kmn ? ~u : kmn;
      kmx = u > kmx ? u : kmx;
      acc++;
    }
  }
  int64_t tot;
  block_incl_max(m, lds, &tot);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t a = __shfl_xor(kmn, off, 64), b = __shfl_xor(kmx, off, 64);
    const int64_t c = __shfl_xor(tmn, off, 64);
    kmn = a > kmn ? a : kmn;
    kmx = b > kmx ? b : kmx;
    tmn = c < tmn ? c : tmn;
  }
  acc = wave_sum(acc);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    lk[0][wave] = kmn;
    lk[1][wave] = kmx;
    lk[2][wave] = (uint64_t)tmn;
    la[wave] = acc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < BLOCK / 64; w++) {
      kmn = lk[0][w] > kmn ? lk[0][w] : kmn;
      kmx = lk[1][w] > kmx ? lk[1][w] : kmx;
      tmn = (int64_t)lk[2][w] < tmn ? (int64_t)lk[2][w] : tmn;
      acc += la[w];
    }
    blockmax[blockIdx.x] = tot;
    blockkr[blockIdx.x] = make_ulonglong2(kmn, kmx);
    blockacc[blockIdx.x] = acc;
    blocktmin[blockIdx.x] = tmn;
  }
}

// The per-block key ranges → ctr[C_KMINN], ctr[C_KMAX], ctr[C_KACC]; ctr[C_TBASE] = the base of
// the push's packed replay records: the smallest accepted ts, or the stream time before the push
// when that is smaller and set (every stream time a record of the push sees is -1 or >= it).
// Runs before k_scan_blocks advances *stream_time (one workgroup).
__global__ __launch_bounds__(1024) void k_sess_range_reduce(const ulonglong2* __restrict__ blockkr,
                                                            const int64_t* __restrict__ blockacc,
                                                            const int64_t* __restrict__ blocktmin, int64_t nb,
                                                            const int64_t* __restrict__ stream_time,
                                                            unsigned long long* __restrict__ ctr) {
  __shared__ uint64_t l[4][1024 / 64];
  uint64_t kmn = 0, kmx = 0;
  int64_t acc = 0, tmn = INT64_MAX;
  for (int64_t b = threadIdx.x; b < nb; b += blockDim.x) {
    const ulonglong2 v = blockkr[b];
    kmn = v.x > kmn ? v.x : kmn;
    kmx = v.y > kmx ? v.y : kmx;
    acc += blockacc[b];
    tmn = blocktmin[b] < tmn ? blocktmin[b] : tmn;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t a = __shfl_xor(kmn, off, 64), b = __shfl_xor(kmx, off, 64);
    const int64_t c = __shfl_xor(tmn, off, 64);
    kmn = a > kmn ? a : kmn;
    kmx = b > kmx ? b : kmx;
    tmn = c < tmn ? c : tmn;
  }
  acc = wave_sum(acc);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    l[0][wave] = kmn;
    l[1][wave] = kmx;
    l[2][wave] = (uint64_t)acc;
    l[3][wave] = (uint64_t)tmn;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); w++) {
      kmn = l[0][w] > kmn ? l[0][w] : kmn;
      kmx = l[1][w] > kmx ? l[1][w] : kmx;
      acc += (int64_t)l[2][w];
      tmn = (int64_t)l[3][w] < tmn ? (int64_t)l[3][w] : tmn;
    }
    const int64_t p = *stream_time;
    if (p >= 0 && p < tmn) tmn = p;
    ctr[C_KMINN] = kmn;
    ctr[C_KMAX] = kmx;
    ctr[C_KACC] = (unsigned long long)acc;
    ctr[C_TBASE] = (unsigned long long)(tmn == INT64_MAX ? 0 : tmn);
  }
}

// Packed 8-byte replay record: (stream time before - tbase + 1) << 32 | (ts - tbase + 1), each half
// 0 for -1 (a dropped record / no stream time yet); used when the push's times span < 2^32 - 1.
// The replay takes the stream time after an accepted record as max(before, ts); the one before it
// is EMIT FINAL's (a session merged away by the record was emitted if the close time before the
// record had passed its end).
__device__ __forceinline__ uint64_t rec_pack(int64_t t, int64_t st, int64_t tbase) {
  const uint64_t lo = t >= 0 ? (uint64_t)(t - tbase + 1) : 0, hi = st >= 0 ? (uint64_t)(st - tbase + 1) : 0;
  return (hi << 32) | lo;
}
__device__ __forceinline__ void rec_unpack(uint64_t r, int64_t tbase, int64_t& t, int64_t& st) {
  const uint32_t lo = (uint32_t)r, hi = (uint32_t)(r >> 32);
  t = lo ? tbase + (int64_t)lo - 1 : -1;
  st = hi ? tbase + (int64_t)hi - 1 : -1;
}

// Per record (coalesced): the task's stream time before it (block prefix, then the block's running
// max), the packed replay record {ts or -1 when dropped, stream time before}, and the (key - kmin,
// row) pair to sort (dropped rows get the sentinel `drop`, which sorts last); drop counters.
__global__ __launch_bounds__(BLOCK) void k_sess_prep(const int64_t* __restrict__ keys, const int64_t* __restrict__ ts,
                                                     const uint8_t* __restrict__ kv, const uint8_t* __restrict__ rv,
                                                     int64_t n, const int64_t* __restrict__ prefix, int64_t kmin,
                                                     uint64_t drop, uint64_t* __restrict__ skey,
                                                     uint32_t* __restrict__ sidx, longlong2* __restrict__ rec,
                                                     uint64_t* __restrict__ rec8, int64_t tbase,
                                                     int64_t* __restrict__ blockcnt, const int64_t* __restrict__ st_at) {
  // wave w owns records [base + w * 64 * ITEMS, +64 * ITEMS), read 64 at a time (coalesced); the
  // running max is a wave scan per step, the earlier waves' maxima join after one block barrier
  __shared__ int64_t wmax[BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * RPB + (int64_t)wave * 64 * ITEMS + lane;
  int64_t stv[ITEMS], tv[ITEMS];
  int64_t carry = -1;  // the wave's running maximum before the step
  int nk = 0, nr = 0, nt = 0, na = 0;
#pragma unroll
  for (int k = 0; k < ITEMS; k++) {
    const int64_t i = base + k * 64;
    int64_t t = -1;
    bool ok = false;
    if (i < n) {
      t = ts[i];
      const bool a = bit_get(kv, i), b = bit_get(rv, i);
      ok = a && b && t >= 0;
      nk += !a;
      nr += a && !b;
      nt += a && b && t < 0;
      na += ok;
    }
    tv[k] = ok ? t : -1;
    int64_t incl = wave_incl_max(tv[k]);
    incl = incl > carry ? incl : carry;
    const int64_t ex = __shfl_up(incl, 1, 64);  // the lane before's inclusive maximum
    stv[k] = lane ? ex : carry;                 // exclusive: the stream time before the record
    carry = __shfl(incl, 63, 64);
  }
  if (lane == 0) wmax[wave] = carry;
  __syncthreads();
  int64_t pre = prefix[blockIdx.x];
  for (int w = 0; w < wave; w++) pre = wmax[w] > pre ? wmax[w] : pre;
#pragma unroll
  for (int k = 0; k < ITEMS; k++) {
    const int64_t i = base + k * 64;
    if (i < n) {
      const bool ok = tv[k] >= 0;
      skey[i] = ok ? (uint64_t)keys[i] - (uint64_t)kmin : drop;
      if (sidx) sidx[i] = (uint32_t)i;
      // KHIP_TIME_SUPPLIED: the row's given stream time (the GLOBAL one after it, >= its ts), which
      // the replay's max(before, ts) keeps as it is (EMIT CHANGES only: EMIT FINAL needs the one
      // before the row, which the shuffle does not carry)
      const int64_t sa = st_at ? (ok ? st_at[i] : -1) : (stv[k] > pre ? stv[k] : pre);
      if (rec8) rec8[i] = rec_pack(tv[k], sa, tbase);
      else rec[i] = make_longlong2(tv[k], sa);
    }
  }
  // drop counters: one row of 4 per block (summed by k_sess_cnt_reduce; same-address atomics
  // from every wave would serialize)
  __shared__ int64_t wc[BLOCK / 64][4];
  const int64_t c4[4] = {wave_sum(nk), wave_sum(nr), wave_sum(nt), wave_sum(na)};
  if (lane < 4) wc[wave][lane] = c4[lane];
  __syncthreads();
  if (threadIdx.x < 4) {
    int64_t v = 0;
    for (int w = 0; w < BLOCK / 64; w++) v += wc[w][threadIdx.x];
    blockcnt[blockIdx.x * 4 + threadIdx.x] = v;
  }
}

// Per-block drop counters → ctr[P_NULL_KEY, P_NULL_ROW, P_BAD_TS, P_ACCEPTED] (one workgroup).
__global__ __launch_bounds__(1024) void k_sess_cnt_reduce(const int64_t* __restrict__ blockcnt, int64_t nb,
                                                          unsigned long long* __restrict__ ctr) {
  __shared__ int64_t l[4][1024 / 64];
  int64_t v[4] = {0, 0, 0, 0};
  for (int64_t b = threadIdx.x; b < nb; b += blockDim.x)
    for (int k = 0; k < 4; k++) v[k] += blockcnt[b * 4 + k];
  const int wave = threadIdx.x >> 6;
  for (int k = 0; k < 4; k++) {
    const int64_t x = wave_sum(v[k]);
    if ((threadIdx.x & 63) == 0) l[k][wave] = x;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    int64_t x = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); w++) x += l[threadIdx.x][w];
    const int slot[4] = {P_NULL_KEY, P_NULL_ROW, P_BAD_TS, P_ACCEPTED};
    ctr[slot[threadIdx.x]] += (unsigned long long)x;
  }
}

// Replay records in sorted order: g[r] = rec[sidx[r]] (the random reads leave the per-key chain).
template <class R>
__global__ __launch_bounds__(256) void k_sess_gather(const uint32_t* __restrict__ sidx, const R* __restrict__ rec,
                                                     int64_t n, R* __restrict__ g) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
    g[r] = rec[sidx[r]];
}

__global__ void k_sess_setn(int* __restrict__ p, int v) { *p = v; }

// Run-length-encoded keys back to absolute keys.
__global__ __launch_bounds__(256) void k_sess_ukeys(int64_t* __restrict__ ukeys, const int* __restrict__ nseg, int64_t kmin) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < *nseg) ukeys[j] = (int64_t)((uint64_t)ukeys[j] + (uint64_t)kmin);
}

__device__ __forceinline__ int64_t lower_key(const uint64_t* __restrict__ rows, int sw, int64_t n, int64_t key) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)rows[mid * sw] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int64_t lower_val(const int64_t* __restrict__ v, int64_t n, int64_t key) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (v[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Per batch key: its store range [s0, s1) and its scratch capacity (store sessions + records).
__global__ __launch_bounds__(256) void k_sess_bounds(const uint64_t* __restrict__ store, int64_t ns, int sw,
                                                     const int64_t* __restrict__ ukeys, const int* __restrict__ ucnt,
                                                     const int* __restrict__ nseg, int64_t* __restrict__ s0,
                                                     int64_t* __restrict__ cap) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= *nseg) return;
  const int64_t k = ukeys[j];
  const int64_t a = lower_key(store, sw, ns, k);
  int64_t b = a;
  while (b < ns && (int64_t)store[b * sw] == k) b++;
  s0[j] = a;
  cap[j] = (b - a) + ucnt[j];
}

__device__ __forceinline__ void sess_apply_record(const SessParams& q, uint64_t* row, const ColPtrs& cols, int64_t i) {
  for (int o = 0; o < q.ap.n_ops; o++) {
    const UpdOp op = q.ap.ops[o];
    uint64_t& w = row[op.word];
    if (op.kind == OP_INC) {
      w += 1;
      continue;
    }
    if (!bit_get(cols.valid[op.col], i)) continue;
    if (op.kind == OP_INC_VALID) {
      w += 1;
      continue;
    }
    const int64_t raw = load_col_raw(cols, q.ap.col_type[op.col], op.col, i);
    switch (op.kind) {
      case OP_ADD_I64: w += (uint64_t)raw; break;
      case OP_ADD_F64: {
        double a, b;
        __builtin_memcpy(&a, &w, 8);
        __builtin_memcpy(&b, &raw, 8);
        a += b;
        __builtin_memcpy(&w, &a, 8);
        break;
      }
      case OP_MIN:
      case OP_MAX: {
        int64_t k = raw;
        if (q.ap.col_type[op.col] == KHIP_TYPE_DOUBLE) {
          double d;
          __builtin_memcpy(&d, &raw, 8);
          k = f64_order_key(d);
        }
        if (op.kind == OP_MIN ? k < (int64_t)w : k > (int64_t)w) w = (uint64_t)k;
        break;
      }
      default: break;
    }
  }
}

// dst = merge(dst, src) (KudafAggregator.getMerger): counts and sums add, MIN/MAX compare.
__device__ __forceinline__ void sess_merge(const SessParams& q, uint64_t* dst, const uint64_t* src) {
  for (int o = 0; o < q.ap.n_ops; o++) {
    const UpdOp op = q.ap.ops[o];
    uint64_t& w = dst[op.word];
    const uint64_t x = src[op.word];
    switch (op.kind) {
      case OP_INC:
      case OP_INC_VALID:
      case OP_ADD_I64: w += x; break;
      case OP_ADD_F64: {
        double a, b;
        __builtin_memcpy(&a, &w, 8);
        __builtin_memcpy(&b, &x, 8);
        a += b;
        __builtin_memcpy(&w, &a, 8);
        break;
      }
      case OP_MIN: if ((int64_t)x < (int64_t)w) w = x; break;
      case OP_MAX: if ((int64_t)x > (int64_t)w) w = x; break;
      default: break;
    }
  }
}

__device__ __forceinline__ void row_copy(uint64_t* d, const uint64_t* s, int sw) {
  for (int w = 0; w < sw; w++) d[w] = s[w];
}

// One batch key: replay its records (arrival order) against its sessions.  R / F: the key's
// scratch rows and flags (LDS or HBM), T: removed original sessions (HBM), orig: its store rows.
// Returns the sessions left after expiry (compacted at R); chg rows appended to the changelog.
// FIN (EMIT FINAL) is a template parameter: the EMIT CHANGES replay compiles without the close
// checks (with them as a run-time branch the replay took 157 VGPRs and 800 B of scratch per lane
// instead of 69 and 52: session leg 9.6 -> 11.1 ms/step).  Rows are checked with having_only (the
// query's HAVING; the pull-query filter of having_ok made the FINAL replay copy its parameters to
// scratch: 81 VGPRs and no scratch now).
template <bool FIN>
__device__ __forceinline__ int64_t sess_replay(const SessParams& q, int64_t key, const uint64_t* orig, int64_t norig,
                                               const longlong2* g, const uint64_t* g8, int64_t tbase,
                                               const uint32_t* sidx, int64_t nrec,
                                               uint64_t* R, uint8_t* F, uint64_t* T, const ColPtrs& cols,
                                               int64_t vis_end, int64_t close_end, uint64_t* __restrict__ crow,
                                               uint8_t* __restrict__ ctomb, unsigned long long* __restrict__ ctr,
                                               int keep_changes, int64_t& applied, int64_t& late) {
  const int sw = q.sw;
  int64_t m = 0, nt = 0;
  for (int64_t k = 0; k < norig; k++) {  // the key's sessions, sorted by start (and end)
    const uint64_t* src = orig + k * sw;
    row_copy(R + m * sw, src, sw);
    F[m] = SF_ORIG | (having_only(src, q.having) ? SF_OLDP : 0);
    m++;
  }
  for (int64_t r = 0; r < nrec; r++) {
    int64_t t, stb;
    if (g8) {
      rec_unpack(g8[r], tbase, t, stb);
    } else {
      const longlong2 gr = g[r];
      t = gr.x;
      stb = gr.y;
    }
    if (t < 0) continue;  // dropped (only where the sentinel shares the last key's segment)
    const int64_t st = stb > t ? stb : t;  // the stream time after the record
    const int64_t i = q.ap.n_cols ? (int64_t)sidx[r] : 0;
    const int64_t vis = st - q.retention, close = st - q.grace - q.gap;
    // overlapping run: visible sessions with end >= t - gap and start <= t + gap
    const int64_t from = t - q.gap > vis ? t - q.gap : vis;
    int64_t lo = 0, hi = m;
    while (lo < hi) {  // first session with end >= from
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)R[mid * sw + 2] < from) lo = mid + 1;
      else hi = mid;
    }
    hi = lo;
    while (hi < m && (int64_t)R[hi * sw + 1] <= t + q.gap) hi++;
    int64_t ms = t, me = t;
    if (hi > lo) {
      ms = (int64_t)R[lo * sw + 1] < t ? (int64_t)R[lo * sw + 1] : t;
      me = (int64_t)R[(hi - 1) * sw + 2] > t ? (int64_t)R[(hi - 1) * sw + 2] : t;
    }
    if (me < close) {  // the merged session is already closed: late
      late++;
      continue;
    }
    applied++;
    if (hi - lo == 1 && (int64_t)R[lo * sw + 1] == t && (int64_t)R[lo * sw + 2] == t) {  // [t, t] itself
      sess_apply_record(q, R + lo * sw, cols, i);
      F[lo] |= SF_TOUCHED;
      continue;
    }
    if constexpr (FIN) {
      // EMIT FINAL: a merged-away session the close time before this record had already passed
      // was emitted then (it is leaving the store only now); sessions of earlier pushes that
      // passed it were emitted by those pushes
      const int64_t cb = stb >= 0 ? stb - q.grace - q.gap : INT64_MIN;
      for (int64_t k = lo; k < hi; k++) {
        const int64_t e = (int64_t)R[k * sw + 2];
        if (e >= q.fin_lo && e < cb && having_only(R + k * sw, q.having)) {
          row_copy(T + nt * sw, R + k * sw, sw);
          nt++;
        }
      }
    } else {
      // the merged-away sessions that existed before the push: their deletions are emitted
      for (int64_t k = lo; k < hi; k++) {
        if (F[k] & SF_ORIG) {
          row_copy(T + nt * sw, R + k * sw, sw);
          T[nt * sw + 0] = (uint64_t)F[k];  // flags ride in the key word (the key is known)
          nt++;
        }
      }
    }
    // merged row, in place at lo: the first overlapped session, the later ones merged into it in
    // store order (by end) — or the initial row for a new session
    uint64_t* M = R + lo * sw;
    if (hi > lo) {
      for (int64_t k = lo + 1; k < hi; k++) sess_merge(q, M, R + k * sw);
    }
    const int64_t removed = hi - lo;
    if (removed == 0) {  // a new session: shift the later ones right, initial row at lo
      for (int64_t k = m; k > lo; k--) {
        row_copy(R + k * sw, R + (k - 1) * sw, sw);
        F[k] = F[k - 1];
      }
      m++;
      for (int w = 3; w < sw; w++) M[w] = (uint64_t)q.init.w[w];
    } else if (removed > 1) {  // close the gap left by the merged sessions
      for (int64_t k = hi; k < m; k++) {
        row_copy(R + (k - removed + 1) * sw, R + k * sw, sw);
        F[k - removed + 1] = F[k];
      }
      m -= removed - 1;
    }
    M[0] = (uint64_t)key;
    M[1] = (uint64_t)ms;
    M[2] = (uint64_t)me;
    F[lo] = SF_TOUCHED;
    sess_apply_record(q, R + lo * sw, cols, i);
  }
  if constexpr (FIN) {
    // EMIT FINAL: the sessions merged away after their close (above), and those of the store
    // after the push whose end the close time passed during it
    int64_t nc = nt;
    for (int64_t k = 0; k < m; k++) {
      const int64_t e = (int64_t)R[k * sw + 2];
      nc += (e >= q.fin_lo && e < close_end && having_only(R + k * sw, q.having)) ? 1 : 0;
    }
    int64_t c = nc ? (int64_t)atomicAdd(&ctr[16], (unsigned long long)nc) : 0;
    for (int64_t k = 0; k < nt; k++) {
      row_copy(crow + c * sw, T + k * sw, sw);
      ctomb[c++] = 0;
    }
    for (int64_t k = 0; k < m; k++) {
      const int64_t e = (int64_t)R[k * sw + 2];
      if (!(e >= q.fin_lo && e < close_end && having_only(R + k * sw, q.having))) continue;
      row_copy(crow + c * sw, R + k * sw, sw);
      ctomb[c++] = 0;
    }
  } else if (keep_changes) {
    // changelog: touched sessions (rows, or tombstones when HAVING stopped holding), deleted
    // sessions that existed before the push (tombstones when HAVING held)
    int64_t nc = 0;
    for (int64_t k = 0; k < m; k++)
      if (F[k] & SF_TOUCHED) nc += (having_only(R + k * sw, q.having) || ((F[k] & SF_ORIG) && (F[k] & SF_OLDP))) ? 1 : 0;
    for (int64_t k = 0; k < nt; k++) nc += (T[k * sw] & SF_OLDP) ? 1 : 0;
    int64_t c = nc ? (int64_t)atomicAdd(&ctr[16], (unsigned long long)nc) : 0;
    for (int64_t k = 0; k < m; k++) {
      if (!(F[k] & SF_TOUCHED)) continue;
      const bool now = having_only(R + k * sw, q.having);
      if (!now && !((F[k] & SF_ORIG) && (F[k] & SF_OLDP))) continue;
      row_copy(crow + c * sw, R + k * sw, sw);
      ctomb[c++] = now ? 0 : 1;
    }
    for (int64_t k = 0; k < nt; k++) {
      if (!(T[k * sw] & SF_OLDP)) continue;
      row_copy(crow + c * sw, T + k * sw, sw);
      crow[c * sw] = (uint64_t)key;
      ctomb[c++] = 1;
    }
  }
  // expired sessions leave the store (end < stream time after the push - retention)
  int64_t kept = 0;
  for (int64_t k = 0; k < m; k++) {
    if ((int64_t)R[k * sw + 2] < vis_end) continue;
    if (kept != k) row_copy(R + kept * sw, R + k * sw, sw);
    kept++;
  }
  return kept;
}

// The wave's keys' row runs copied with every lane busy: lane k's run is `words` words from
// src + soff to dst + doff; the runs are laid end to end and each word finds its run by a binary
// search over the lanes' inclusive prefix (consecutive words of a run: consecutive addresses).
__device__ __forceinline__ void wave_copy_runs(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst,
                                               int64_t soff, int64_t doff, int64_t words) {
  const int lane = threadIdx.x & 63;
  int64_t incl = words;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  const int64_t W = __shfl(incl, 63, 64);
  for (int64_t x0 = 0; x0 < W; x0 += 64) {  // uniform trip count: every lane takes part in the shuffles
    const int64_t x = x0 + lane;
    int lo = 0;
#pragma unroll
    for (int step = 32; step; step >>= 1)
      if (__shfl(incl, lo + step - 1, 64) <= x) lo += step;
    lo = lo > 63 ? 63 : lo;
    const int64_t e = __shfl(incl, lo, 64) - __shfl(words, lo, 64);
    const int64_t so = __shfl(soff, lo, 64), d = __shfl(doff, lo, 64);
    if (x < W) dst[d + (x - e)] = src[so + (x - e)];
  }
}

// Scratch budget of one wave's keys in LDS (rows of sw words + 1 flag byte each); waves whose
// keys need more replay in HBM scratch.  The records are read from HBM by each lane (a key's
// records are contiguous, and the wave's keys are neighbours: their lines are shared through L1),
// so the LDS holds only the rows and six waves fit a CU.
#ifndef KHIP_SESS_LDS
#define KHIP_SESS_LDS 24576
#endif
constexpr int SESS_LDS = KHIP_SESS_LDS;

// One wave per 64 batch keys, one lane per key.  The wave's records (one contiguous range of the
// sorted records) and its keys' scratch rows are staged in LDS when they fit, so the per-key
// sequential replay runs against LDS; the keys' final rows then leave with coalesced stores.
template <bool FIN>
__global__ __launch_bounds__(64) void k_sess_apply(SessParams q, const uint64_t* __restrict__ store,
                                                   const int64_t* __restrict__ ukeys, const int* __restrict__ ucnt,
                                                   const int64_t* __restrict__ useg, const int* __restrict__ nseg,
                                                   const int64_t* __restrict__ s0, const int64_t* __restrict__ cap,
                                                   const int64_t* __restrict__ scap, const uint32_t* __restrict__ sidx,
                                                   const longlong2* __restrict__ g, const uint64_t* __restrict__ g8,
                                                   int64_t tbase, ColPtrs cols,
                                                   const int64_t* __restrict__ st_end, uint64_t* __restrict__ srow,
                                                   uint8_t* __restrict__ sfl, uint64_t* __restrict__ trow,
                                                   int64_t* __restrict__ fin, uint64_t* __restrict__ crow,
                                                   uint8_t* __restrict__ ctomb, unsigned long long* __restrict__ ctr,
                                                   int keep_changes, int64_t nseg_eff) {
  __shared__ uint64_t lds[SESS_LDS / 8];
  const int lane = threadIdx.x;
  const int64_t j0 = (int64_t)blockIdx.x * 64, j = j0 + lane;
  const int64_t jl = (nseg_eff - 1 < j0 + 63) ? nseg_eff - 1 : j0 + 63;
  const int sw = q.sw;
  const int64_t R1 = useg[jl] + ucnt[jl];
  const int64_t C0 = scap[j0], C1 = scap[jl] + cap[jl];
  const int64_t need = (C1 - C0) * (sw * 8 + 1);
  const bool in_lds = need <= SESS_LDS;
  const int64_t vis_end = *st_end - q.retention;
  const int64_t close_end = FIN && *st_end >= 0 ? *st_end - q.grace - q.gap : INT64_MIN;
  int64_t applied = 0, late = 0, kept = 0;
  const bool mine = j < nseg_eff;
  (void)R1;
  if (in_lds) {
    uint64_t* lrow = lds;
    uint8_t* lfl = (uint8_t*)(lrow + (C1 - C0) * sw);
    if (mine) {
      const int64_t base = scap[j], r0 = useg[j];
      kept = sess_replay<FIN>(q, ukeys[j], store + s0[j] * sw, cap[j] - ucnt[j], g ? g + r0 : nullptr, g8 ? g8 + r0 : nullptr, tbase,
                         sidx ? sidx + r0 : nullptr,
                         ucnt[j], lrow + (base - C0) * sw, lfl + (base - C0), trow + base * sw, cols, vis_end, close_end, crow,
                         ctomb, ctr, keep_changes, applied, late);
      fin[j] = kept;
    }
    __syncthreads();
    // the keys' final rows → HBM scratch (at scap), the wave's runs flattened over its lanes
    const int64_t off = mine ? scap[j] - C0 : 0;
    wave_copy_runs(lrow, srow, off * sw, (C0 + off) * sw, mine ? kept * sw : 0);
  } else if (mine) {
    const int64_t base = scap[j], r0 = useg[j];
    kept = sess_replay<FIN>(q, ukeys[j], store + s0[j] * sw, cap[j] - ucnt[j], g ? g + r0 : nullptr, g8 ? g8 + r0 : nullptr, tbase,
                         sidx ? sidx + r0 : nullptr, ucnt[j],
                       srow + base * sw, sfl + base, trow + base * sw, cols, vis_end, close_end, crow, ctomb, ctr,
                       keep_changes,
                       applied, late);
    fin[j] = kept;
  }
  applied = wave_sum(applied);
  late = wave_sum(late);
  if (lane == 0) {
    if (applied) atomicAdd(&ctr[P_APPLIED], (unsigned long long)applied);
    if (late) atomicAdd(&ctr[P_LATE], (unsigned long long)late);
  }
}

// Store rows that survive untouched: key not in the batch and not expired.  EMIT FINAL (q.fin):
// the untouched keys' sessions whose end the push's close time passed are emitted (wave-aggregated
// appends to the changelog rows).
__global__ __launch_bounds__(256) void k_sess_keep(const uint64_t* __restrict__ store, int64_t ns, int sw,
                                                   const int64_t* __restrict__ ukeys, const int* __restrict__ nseg,
                                                   const int64_t* __restrict__ st_end, int64_t retention,
                                                   int* __restrict__ keep, SessParams q, uint64_t* __restrict__ crow,
                                                   uint8_t* __restrict__ ctomb, unsigned long long* __restrict__ ctr) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  bool emit = false;
  const uint64_t* s = store + (i < ns ? i : 0) * sw;
  if (i < ns) {
    const int64_t k = (int64_t)s[0];
    const int64_t nu = *nseg;
    const int64_t p = lower_val(ukeys, nu, k);
    const bool in_batch = p < nu && ukeys[p] == k;
    keep[i] = (!in_batch && (int64_t)s[2] >= *st_end - retention) ? 1 : 0;
    if (q.fin && !in_batch && *st_end >= 0) {
      const int64_t e = (int64_t)s[2];
      emit = e >= q.fin_lo && e < *st_end - q.grace - q.gap && having_only(s, q.having);
    }
  }
  if (!q.fin) return;
  const uint64_t bl = __ballot(emit);
  if (!bl) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((unsigned long long)bl) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(&ctr[16], (unsigned long long)__popcll(bl));
  base = __shfl(base, leader, 64);
  if (emit) {
    const unsigned long long c = base + __popcll(bl & ((1ULL << lane) - 1));
    row_copy(crow + c * sw, s, sw);
    ctomb[c] = 0;
  }
}

// New store: kept rows and the rewritten keys' sessions, in key order.
__global__ __launch_bounds__(256) void k_sess_scatter_store(const uint64_t* __restrict__ store, int64_t ns, int sw,
                                                            const int* __restrict__ keep,
                                                            const int* __restrict__ keep_pre,
                                                            const int64_t* __restrict__ ukeys,
                                                            const int* __restrict__ nseg,
                                                            const int64_t* __restrict__ fin_pre,
                                                            uint64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= ns || !keep[i]) return;
  const uint64_t* s = store + i * sw;
  const int64_t p = lower_val(ukeys, *nseg, (int64_t)s[0]);
  row_copy(out + ((int64_t)keep_pre[i] + fin_pre[p]) * sw, s, sw);
}

// The rewritten keys' sessions into the new store: one wave per 64 batch keys, their row runs
// copied with every lane of the wave busy (wave_copy_runs).
__global__ __launch_bounds__(256) void k_sess_scatter_seg(const uint64_t* __restrict__ store, int64_t ns, int sw,
                                                          const int* __restrict__ keep_pre,
                                                          const int* __restrict__ keep, const int64_t* __restrict__ ukeys,
                                                          int64_t nseg, const int64_t* __restrict__ fin,
                                                          const int64_t* __restrict__ fin_pre,
                                                          const int64_t* __restrict__ scap,
                                                          const uint64_t* __restrict__ srow, uint64_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t j0 = ((int64_t)blockIdx.x * 256 + (threadIdx.x & ~63));
  if (j0 >= nseg) return;
  int64_t dst = 0, src = 0, words = 0;
  const int64_t jl = j0 + lane;
  if (jl < nseg) {
    const int64_t a = ns ? lower_key(store, sw, ns, ukeys[jl]) : 0;
    const int64_t kept_before = a < ns ? (int64_t)keep_pre[a] : (ns ? (int64_t)keep_pre[ns - 1] + keep[ns - 1] : 0);
    dst = (kept_before + fin_pre[jl]) * sw;
    src = scap[jl] * sw;
    words = fin[jl] * sw;
  }
  wave_copy_runs(srow, out, src, dst, words);
}

// ------------------------------------------------------------------ host side

khip_status sess_push(khip_agg* a, int64_t n, const int64_t* keys, const int64_t* ts, const uint8_t* kv,
                      const uint8_t* rv, const ColPtrs& cols, int64_t* tot, const int64_t* st_at) {
  SessState& S = a->sess;
  hipStream_t st = a->stream;
  const int sw = a->sw;
  const int64_t nb = ceil_div(n, RPB);
  KHIP_TRY(a->blockmax.ensure(nb * 8));
  KHIP_TRY(a->blockprefix.ensure(nb * 8));
  KHIP_TRY(S.ctr.ensure(32 * 8));
  KHIP_TRY_HIP(hipMemsetAsync(S.ctr.p, 0, 32 * 8, st));
  KHIP_TRY(S.blockkr.ensure(nb * 32));
  int64_t* blockacc = (int64_t*)(S.blockkr.as<char>() + nb * 16);
  int64_t* blocktmin = (int64_t*)(S.blockkr.as<char>() + nb * 24);
  hipLaunchKernelGGL(k_sess_range, dim3(nb), dim3(BLOCK), 0, st, keys, ts, kv, rv, n, a->blockmax.as<int64_t>(),
                     S.blockkr.as<ulonglong2>(), blockacc, blocktmin, st_at);
  hipLaunchKernelGGL(k_sess_range_reduce, dim3(1), dim3(1024), 0, st, S.blockkr.as<ulonglong2>(), blockacc, blocktmin,
                     nb, a->stream_time.as<int64_t>(), S.ctr.as<unsigned long long>());
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, st, a->blockmax.as<int64_t>(), nb,
                     a->blockprefix.as<int64_t>(), a->stream_time.as<int64_t>());
  // the push's key range: the sort runs over (key - kmin) and only the bits that range needs;
  // its time base and the stream time after it: packed 8-byte replay records when the span fits
  unsigned long long kr[4] = {0, 0, 0, 0};
  int64_t st_after_push = -1;
  KHIP_TRY_HIP(hipMemcpyAsync(kr, S.ctr.as<unsigned long long>() + C_KMINN, sizeof(kr), hipMemcpyDeviceToHost, st));
  KHIP_TRY_HIP(hipMemcpyAsync(&st_after_push, a->stream_time.p, 8, hipMemcpyDeviceToHost, st));
  KHIP_TRY_HIP(hipStreamSynchronize(st));
  const int64_t tbase = (int64_t)kr[3];
  const bool packed = st_after_push < 0 || (uint64_t)(st_after_push - tbase) < 0xFFFFFFF0ULL;
  int64_t kmin = 0;
  uint64_t range = 0;
  if (kr[2]) {
    kmin = (int64_t)(~(uint64_t)kr[0] ^ (1ULL << 63));
    const int64_t kmax = (int64_t)((uint64_t)kr[1] ^ (1ULL << 63));
    range = (uint64_t)kmax - (uint64_t)kmin;
  }
  const bool sentinel = range != ~0ULL;  // dropped rows get a key of their own (range + 1)
  const uint64_t drop = sentinel ? range + 1 : range;
  const int end_bit = drop ? 64 - __builtin_clzll(drop) : 1;
  // Packed records without argument columns ride through the sort as its 8-byte value.  With
  // columns (or 16-byte records) the sort carries 4-byte row indices and one gather brings the
  // records into sorted order (a 16-byte value would cost the sort more than the gather).
  const bool by_idx = !packed || a->desc.n_cols > 0;
  KHIP_TRY(S.skey.ensure(n * 8));
  KHIP_TRY(S.skey2.ensure(n * 8));
  KHIP_TRY(S.st_after.ensure(n * 16));
  KHIP_TRY(S.gath.ensure(n * 16));
  if (by_idx) {
    KHIP_TRY(S.sidx.ensure(n * 4));
    KHIP_TRY(S.sidx2.ensure(n * 4));
  }
  hipLaunchKernelGGL(k_sess_prep, dim3(nb), dim3(BLOCK), 0, st, keys, ts, kv, rv, n, a->blockprefix.as<int64_t>(), kmin,
                     drop, S.skey.as<uint64_t>(), by_idx ? S.sidx.as<uint32_t>() : nullptr,
                     packed ? nullptr : S.st_after.as<longlong2>(), packed ? S.st_after.as<uint64_t>() : nullptr, tbase,
                     (int64_t*)S.blockkr.p, st_at);
  hipLaunchKernelGGL(k_sess_cnt_reduce, dim3(1), dim3(1024), 0, st, (const int64_t*)S.blockkr.p, nb,
                     S.ctr.as<unsigned long long>());
  KHIP_TRY_HIP(hipGetLastError());
  // group by key, arrival order kept within a key (LSD radix sort is stable)
  uint64_t* k_in = S.skey.as<uint64_t>();
  uint64_t* k_out = S.skey2.as<uint64_t>();
  uint32_t* v_out = by_idx ? S.sidx2.as<uint32_t>() : nullptr;
  const dim3 ggrid((int)std::min<int64_t>(ceil_div(n, 256), 16384));
  if (by_idx) {
    uint32_t* v_in = S.sidx.as<uint32_t>();
    KHIP_TRY(ksort::sort_pairs<uint32_t>(st, S.tmp, S.tmp2, k_in, k_out, v_in, v_out, n, end_bit));
    if (packed) {
      auto kg = k_sess_gather<uint64_t>;
      hipLaunchKernelGGL(kg, ggrid, dim3(256), 0, st, v_out, S.st_after.as<uint64_t>(), n, S.gath.as<uint64_t>());
    } else {
      auto kg = k_sess_gather<longlong2>;
      hipLaunchKernelGGL(kg, ggrid, dim3(256), 0, st, v_out, S.st_after.as<longlong2>(), n, S.gath.as<longlong2>());
    }
  } else {
    KHIP_TRY(ksort::sort_pairs<uint64_t>(st, S.tmp, S.tmp2, k_in, k_out, S.st_after.as<uint64_t>(),
                                         S.gath.as<uint64_t>(), n, end_bit));
  }
  KHIP_TRY(S.ukeys.ensure(n * 8));
  KHIP_TRY(S.ucnt.ensure(n * 4));
  KHIP_TRY(S.nseg.ensure(16));
  KHIP_TRY(S.useg.ensure((size_t)(n + 1) * 8));
  // key segments: unique keys, counts and starts (useg = the counts' exclusive prefix)
  int64_t nseg64 = 0;
  KHIP_TRY(ksort::rle_sorted(st, S.tmp, k_out, n, S.ukeys.as<uint64_t>(), S.ucnt.as<int>(), S.useg.as<int64_t>(),
                             S.nseg.as<int>(), &nseg64));
  int nseg = (int)nseg64;
  uint64_t last = 0;
  if (nseg > 0) {
    KHIP_TRY_HIP(hipMemcpyAsync(&last, S.ukeys.as<uint64_t>() + nseg - 1, 8, hipMemcpyDeviceToHost, st));
    KHIP_TRY_HIP(hipStreamSynchronize(st));
    if (sentinel && last == drop) nseg--;  // the dropped rows' segment is not a key
  }
  if (nseg > 0)
    hipLaunchKernelGGL(k_sess_ukeys, dim3(ceil_div(nseg, 256)), dim3(256), 0, st, S.ukeys.as<int64_t>(),
                       S.nseg.as<int>(), kmin);
  KHIP_TRY(S.s0.ensure((size_t)(nseg + 1) * 8));
  KHIP_TRY(S.cap.ensure((size_t)(nseg + 1) * 8));
  KHIP_TRY(S.scap.ensure((size_t)(nseg + 1) * 8));
  KHIP_TRY(S.fin.ensure((size_t)(nseg + 1) * 8));
  KHIP_TRY(S.fin_pre.ensure((size_t)(nseg + 1) * 8));
  hipLaunchKernelGGL(k_sess_setn, dim3(1), dim3(1), 0, st, S.nseg.as<int>(), nseg);
  const uint64_t* store = S.rows.as<uint64_t>();
  const int64_t ns = S.n;
  if (nseg > 0)
    hipLaunchKernelGGL(k_sess_bounds, dim3(ceil_div(nseg, 256)), dim3(256), 0, st, store, ns, sw, S.ukeys.as<int64_t>(),
                     S.ucnt.as<int>(), S.nseg.as<int>(), S.s0.as<int64_t>(), S.cap.as<int64_t>());
  KHIP_TRY((ksort::scan_excl<int64_t, int64_t>(st, S.tmp, S.cap.as<int64_t>(), S.scap.as<int64_t>(), nseg, false,
                                                 nullptr)));
  const int64_t scr = ns + n;  // total scratch rows >= sum of capacities
  KHIP_TRY(S.srow.ensure((size_t)scr * sw * 8));
  KHIP_TRY(S.sfl.ensure((size_t)scr));
  KHIP_TRY(S.trow.ensure((size_t)scr * sw * 8));
  const bool fin = a->desc.emit == KHIP_EMIT_FINAL;
  const bool keep_changes = a->changelog || fin;
  if (keep_changes) {
    KHIP_TRY(S.crow.ensure((size_t)scr * sw * 8));
    KHIP_TRY(S.ctomb.ensure((size_t)scr));
  }
  SessParams q{};
  q.ap = a->ap;
  q.init = a->init;
  q.having = a->having;
  q.sw = sw;
  q.gap = a->desc.size_ms;
  q.grace = a->grace;
  q.retention = a->retention;
  q.fin = fin ? 1 : 0;
  {
    const int64_t cp = a->st_before >= 0 ? a->st_before - a->grace - a->desc.size_ms : 0;
    q.fin_lo = cp > 0 ? cp : 0;
  }
  if (nseg > 0)
    hipLaunchKernelGGL(fin ? k_sess_apply<true> : k_sess_apply<false>, dim3(ceil_div(nseg, 64)), dim3(64), 0, st, q, store, S.ukeys.as<int64_t>(),
                     S.ucnt.as<int>(), S.useg.as<int64_t>(), S.nseg.as<int>(), S.s0.as<int64_t>(), S.cap.as<int64_t>(),
                     S.scap.as<int64_t>(), v_out, packed ? nullptr : S.gath.as<longlong2>(),
                     packed ? S.gath.as<uint64_t>() : nullptr, tbase, cols,
                     a->stream_time.as<int64_t>(), S.srow.as<uint64_t>(), S.sfl.as<uint8_t>(), S.trow.as<uint64_t>(),
                     S.fin.as<int64_t>(), keep_changes ? S.crow.as<uint64_t>() : nullptr,
                     keep_changes ? S.ctomb.as<uint8_t>() : nullptr, S.ctr.as<unsigned long long>(), keep_changes ? 1 : 0,
                     (int64_t)nseg);
  KHIP_TRY_HIP(hipGetLastError());
  // the new store
  KHIP_TRY(S.keep.ensure((size_t)(ns + 1) * 4));
  KHIP_TRY(S.keep_pre.ensure((size_t)(ns + 1) * 4));
  if (ns) {
    hipLaunchKernelGGL(k_sess_keep, dim3(ceil_div(ns, 256)), dim3(256), 0, st, store, ns, sw, S.ukeys.as<int64_t>(),
                       S.nseg.as<int>(), a->stream_time.as<int64_t>(), a->retention, S.keep.as<int>(), q,
                       fin ? S.crow.as<uint64_t>() : nullptr, fin ? S.ctomb.as<uint8_t>() : nullptr,
                       S.ctr.as<unsigned long long>());
    KHIP_TRY((ksort::scan_excl<int, int>(st, S.tmp, S.keep.as<int>(), S.keep_pre.as<int>(), ns, false, nullptr)));
  }
  // fin_pre[nseg] = total rewritten rows (inclusive end) via a scan over nseg + 1 entries
  KHIP_TRY_HIP(hipMemsetAsync(S.fin.as<int64_t>() + nseg, 0, 8, st));
  KHIP_TRY((ksort::scan_excl<int64_t, int64_t>(st, S.tmp, S.fin.as<int64_t>(), S.fin_pre.as<int64_t>(), nseg + 1, false,
                                                 nullptr)));
  int64_t tail[2] = {0, 0};
  int kept_tail[2] = {0, 0};
  KHIP_TRY_HIP(hipMemcpyAsync(&tail[0], S.fin_pre.as<int64_t>() + nseg, 8, hipMemcpyDeviceToHost, st));
  if (ns) {
    KHIP_TRY_HIP(hipMemcpyAsync(&kept_tail[0], S.keep_pre.as<int>() + ns - 1, 4, hipMemcpyDeviceToHost, st));
    KHIP_TRY_HIP(hipMemcpyAsync(&kept_tail[1], S.keep.as<int>() + ns - 1, 4, hipMemcpyDeviceToHost, st));
  }
  KHIP_TRY_HIP(hipStreamSynchronize(st));
  const int64_t nkept = ns ? (int64_t)kept_tail[0] + kept_tail[1] : 0;
  const int64_t nnew = nkept + tail[0];
  KHIP_TRY(S.rows2.ensure((size_t)std::max<int64_t>(nnew, 1) * sw * 8));
  if (ns)
    hipLaunchKernelGGL(k_sess_scatter_store, dim3(ceil_div(ns, 256)), dim3(256), 0, st, store, ns, sw, S.keep.as<int>(),
                       S.keep_pre.as<int>(), S.ukeys.as<int64_t>(), S.nseg.as<int>(), S.fin_pre.as<int64_t>(),
                       S.rows2.as<uint64_t>());
  if (nseg > 0)
    hipLaunchKernelGGL(k_sess_scatter_seg, dim3(ceil_div(nseg, 256)), dim3(256), 0, st, store, ns, sw, S.keep_pre.as<int>(),
                     S.keep.as<int>(), S.ukeys.as<int64_t>(), (int64_t)nseg, S.fin.as<int64_t>(),
                     S.fin_pre.as<int64_t>(), S.scap.as<int64_t>(), S.srow.as<uint64_t>(), S.rows2.as<uint64_t>());
  KHIP_TRY_HIP(hipGetLastError());
  unsigned long long c[32];
  int64_t sth = -1;
  KHIP_TRY_HIP(hipMemcpyAsync(c, S.ctr.p, sizeof(c), hipMemcpyDeviceToHost, st));
  KHIP_TRY_HIP(hipMemcpyAsync(&sth, a->stream_time.p, 8, hipMemcpyDeviceToHost, st));
  KHIP_TRY_HIP(hipStreamSynchronize(st));
  std::swap(S.rows, S.rows2);
  S.n = nnew;
  S.nchg = keep_changes ? (int64_t)c[16] : 0;
  a->host_stream_time = sth;
  a->occ = nnew;
  tot[P_ACCEPTED] += (int64_t)c[P_ACCEPTED];
  tot[P_NULL_KEY] += (int64_t)c[P_NULL_KEY];
  tot[P_NULL_ROW] += (int64_t)c[P_NULL_ROW];
  tot[P_BAD_TS] += (int64_t)c[P_BAD_TS];
  tot[P_APPLIED] += (int64_t)c[P_APPLIED];
  tot[P_LATE] += (int64_t)c[P_LATE];
  return KHIP_OK;
}

khip_status sess_changes(khip_agg* a, std::vector<uint64_t>* rows, std::vector<uint8_t>* tomb, int64_t* count) {
  SessState& S = a->sess;
  const int64_t n = S.nchg;
  *count = n;
  rows->resize((size_t)n * a->sw);
  tomb->resize((size_t)n);
  if (n) {
    KHIP_TRY_HIP(hipMemcpy(rows->data(), S.crow.p, (size_t)n * a->sw * 8, hipMemcpyDeviceToHost));
    KHIP_TRY_HIP(hipMemcpy(tomb->data(), S.ctomb.p, (size_t)n, hipMemcpyDeviceToHost));
  }
  return KHIP_OK;
}

void sess_release(khip_agg* a) {
  SessState& S = a->sess;
  DevBuf* bufs[] = {&S.rows, &S.rows2, &S.skey, &S.sidx, &S.skey2, &S.sidx2, &S.st_after, &S.gath, &S.blockkr, &S.ukeys, &S.ucnt, &S.nseg,
                    &S.useg, &S.s0, &S.cap, &S.scap, &S.fin, &S.fin_pre, &S.srow, &S.sfl, &S.trow, &S.crow, &S.ctomb,
                    &S.keep, &S.keep_pre, &S.ctr, &S.tmp};
  for (DevBuf* b : bufs) b->release();
  S.n = 0;
  S.nchg = 0;
}

}  // namespace khip
