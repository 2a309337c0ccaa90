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
//   k_blockmax / k_scan_blocks   stream time before each 2048-record block
//   k_sess_prep                  per record: accepted?, stream time after it; (key, row) pairs
//   radix sort (hipcub, stable)  records grouped by key, arrival order kept inside a key
//   run-length encode            one segment per batch key
//   k_sess_bounds                the key's store range (binary search), scratch capacity
//   k_sess_apply                 ONE THREAD PER KEY replays the key's records in arrival order
//                                against its sessions (merging is inherently sequential per key,
//                                keys are independent): find the overlapping run, merge, late
//                                drop, expiry; emits the push's changelog rows (updates and
//                                tombstones of merged-away sessions)
//   k_sess_keep / k_sess_scatter the new store = untouched keys' sessions (minus expired) merged
//                                in key order with the rewritten keys' sessions
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include "khip_util.hpp"

#include "khip_agg_internal.hpp"

namespace khip {

constexpr uint8_t SF_TOUCHED = 1, SF_ORIG = 2, SF_OLDP = 4;

struct SessParams {
  ApplyParams ap;
  InitWords init;
  HavingDev having;
  int32_t sw;
  int64_t gap, grace, retention;
};

// Per record: accepted (valid key and value, ts >= 0), the task's stream time after it (in-block
// running max seeded with the block prefix), and the (key, row) pair to sort; drop counters.
__global__ __launch_bounds__(BLOCK) void k_sess_prep(const int64_t* __restrict__ keys, const int64_t* __restrict__ ts,
                                                     const uint8_t* __restrict__ kv, const uint8_t* __restrict__ rv,
                                                     int64_t n, const int64_t* __restrict__ prefix,
                                                     int64_t* __restrict__ skey, int64_t* __restrict__ sidx,
                                                     int64_t* __restrict__ st_after,
                                                     unsigned long long* __restrict__ ctr) {
  __shared__ int64_t lmax[BLOCK];
  const int64_t i0 = (int64_t)blockIdx.x * RPB + (int64_t)threadIdx.x * ITEMS;
  int64_t m = -1;
  int nk = 0, nr = 0, nt = 0, na = 0;
  for (int k = 0; k < ITEMS; k++) {
    const int64_t i = i0 + k;
    if (i >= n) break;
    if (!bit_get(kv, i)) { nk++; continue; }
    if (!bit_get(rv, i)) { nr++; continue; }
    if (ts[i] < 0) { nt++; continue; }
    na++;
    m = ts[i] > m ? ts[i] : m;
  }
  lmax[threadIdx.x] = m;
  __syncthreads();
  for (int off = 1; off < BLOCK; off <<= 1) {
    const int64_t y = threadIdx.x >= off ? lmax[threadIdx.x - off] : -1;
    __syncthreads();
    if (y > lmax[threadIdx.x]) lmax[threadIdx.x] = y;
    __syncthreads();
  }
  int64_t st = prefix[blockIdx.x];
  if (threadIdx.x > 0 && lmax[threadIdx.x - 1] > st) st = lmax[threadIdx.x - 1];
  for (int k = 0; k < ITEMS; k++) {
    const int64_t i = i0 + k;
    if (i >= n) break;
    const bool ok = bit_get(kv, i) && bit_get(rv, i) && ts[i] >= 0;
    if (ok && ts[i] > st) st = ts[i];
    st_after[i] = st;
    skey[i] = ok ? keys[i] : INT64_MAX;  // dropped rows sort last (skipped by the replay)
    sidx[i] = i;
  }
  const int64_t s0 = wave_sum(nk), s1 = wave_sum(nr), s2 = wave_sum(nt), s3 = wave_sum(na);
  if ((threadIdx.x & 63) == 0) {
    if (s0) atomicAdd(&ctr[P_NULL_KEY], (unsigned long long)s0);
    if (s1) atomicAdd(&ctr[P_NULL_ROW], (unsigned long long)s1);
    if (s2) atomicAdd(&ctr[P_BAD_TS], (unsigned long long)s2);
    if (s3) atomicAdd(&ctr[P_ACCEPTED], (unsigned long long)s3);
  }
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

// One thread per batch key: replay its records (arrival order) against its sessions.
// scratch rows / flags at base = scap[j]; removed original sessions go to trow at the same base.
// Outputs: fin[j] = sessions left after expiry (compacted at base), chg rows appended to the
// changelog buffer, applied / late counters.
__global__ __launch_bounds__(64) void k_sess_apply(SessParams q, const uint64_t* __restrict__ store,
                                                   const int64_t* __restrict__ ukeys, const int* __restrict__ ucnt,
                                                   const int64_t* __restrict__ useg, const int* __restrict__ nseg,
                                                   const int64_t* __restrict__ s0, const int64_t* __restrict__ cap,
                                                   const int64_t* __restrict__ scap, const int64_t* __restrict__ sidx,
                                                   const int64_t* __restrict__ ts, const uint8_t* __restrict__ kv,
                                                   const uint8_t* __restrict__ rv, ColPtrs cols,
                                                   const int64_t* __restrict__ st_after,
                                                   const int64_t* __restrict__ st_end, uint64_t* __restrict__ srow,
                                                   uint8_t* __restrict__ sfl, uint64_t* __restrict__ trow,
                                                   int64_t* __restrict__ fin, uint64_t* __restrict__ crow,
                                                   uint8_t* __restrict__ ctomb, unsigned long long* __restrict__ ctr,
                                                   int keep_changes) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= *nseg) return;
  const int sw = q.sw;
  const int64_t key = ukeys[j];
  const int64_t base = scap[j];
  uint64_t* R = srow + base * sw;
  uint8_t* F = sfl + base;
  uint64_t* T = trow + base * sw;
  const int64_t norig = cap[j] - ucnt[j];
  int64_t m = 0, nt = 0;
  for (int64_t k = 0; k < norig; k++) {  // the key's sessions, sorted by start (and end)
    const uint64_t* src = store + (s0[j] + k) * sw;
    row_copy(R + m * sw, src, sw);
    F[m] = SF_ORIG | (having_ok(src, q.having) ? SF_OLDP : 0);
    m++;
  }
  int64_t applied = 0, late = 0;
  const int64_t r0 = useg[j], r1 = r0 + ucnt[j];
  for (int64_t r = r0; r < r1; r++) {
    const int64_t i = sidx[r];
    if (!bit_get(kv, i) || !bit_get(rv, i) || ts[i] < 0) continue;
    const int64_t t = ts[i], st = st_after[i];
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
    uint64_t acc[32];
    acc[0] = (uint64_t)key;
    acc[1] = (uint64_t)ms;
    acc[2] = (uint64_t)me;
    for (int w = 3; w < sw; w++) acc[w] = (uint64_t)q.init.w[w];
    for (int64_t k = lo; k < hi; k++) {  // store order (by end), merged into the initial row
      sess_merge(q, acc, R + k * sw);
      if (F[k] & SF_ORIG) {  // existed before the push: its deletion is emitted
        row_copy(T + nt * sw, R + k * sw, sw);
        T[nt * sw + 0] = (uint64_t)F[k];  // flags ride in the key word (the key is known)
        nt++;
      }
    }
    const int64_t removed = hi - lo;
    if (removed == 0) {  // a new session: shift the later ones right
      for (int64_t k = m; k > lo; k--) {
        row_copy(R + k * sw, R + (k - 1) * sw, sw);
        F[k] = F[k - 1];
      }
      m++;
    } else if (removed > 1) {  // close the gap left by the merged sessions
      for (int64_t k = hi; k < m; k++) {
        row_copy(R + (k - removed + 1) * sw, R + k * sw, sw);
        F[k - removed + 1] = F[k];
      }
      m -= removed - 1;
    }
    row_copy(R + lo * sw, acc, sw);
    F[lo] = SF_TOUCHED;
    sess_apply_record(q, R + lo * sw, cols, i);
  }
  // changelog: touched sessions (rows, or tombstones when HAVING stopped holding), deleted
  // sessions that existed before the push (tombstones when HAVING held)
  if (keep_changes) {
    int64_t nc = 0;
    for (int64_t k = 0; k < m; k++)
      if (F[k] & SF_TOUCHED) nc += (having_ok(R + k * sw, q.having) || ((F[k] & SF_ORIG) && (F[k] & SF_OLDP))) ? 1 : 0;
    for (int64_t k = 0; k < nt; k++) nc += (T[k * sw] & SF_OLDP) ? 1 : 0;
    int64_t c = nc ? (int64_t)atomicAdd(&ctr[16], (unsigned long long)nc) : 0;
    for (int64_t k = 0; k < m; k++) {
      if (!(F[k] & SF_TOUCHED)) continue;
      const bool now = having_ok(R + k * sw, q.having);
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
  const int64_t vis_end = *st_end - q.retention;
  int64_t kept = 0;
  for (int64_t k = 0; k < m; k++) {
    if ((int64_t)R[k * sw + 2] < vis_end) continue;
    if (kept != k) row_copy(R + kept * sw, R + k * sw, sw);
    kept++;
  }
  fin[j] = kept;
  if (applied) atomicAdd(&ctr[P_APPLIED], (unsigned long long)applied);
  if (late) atomicAdd(&ctr[P_LATE], (unsigned long long)late);
}

// Store rows that survive untouched: key not in the batch and not expired.
__global__ __launch_bounds__(256) void k_sess_keep(const uint64_t* __restrict__ store, int64_t ns, int sw,
                                                   const int64_t* __restrict__ ukeys, const int* __restrict__ nseg,
                                                   const int64_t* __restrict__ st_end, int64_t retention,
                                                   int* __restrict__ keep) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= ns) return;
  const uint64_t* s = store + i * sw;
  const int64_t k = (int64_t)s[0];
  const int64_t nu = *nseg;
  const int64_t p = lower_val(ukeys, nu, k);
  const bool in_batch = p < nu && ukeys[p] == k;
  keep[i] = (!in_batch && (int64_t)s[2] >= *st_end - retention) ? 1 : 0;
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

__global__ __launch_bounds__(64) void k_sess_scatter_seg(const uint64_t* __restrict__ store, int64_t ns, int sw,
                                                         const int* __restrict__ keep_pre,
                                                         const int* __restrict__ keep, const int64_t* __restrict__ ukeys,
                                                         const int* __restrict__ nseg, const int64_t* __restrict__ fin,
                                                         const int64_t* __restrict__ fin_pre,
                                                         const int64_t* __restrict__ scap,
                                                         const uint64_t* __restrict__ srow, uint64_t* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= *nseg) return;
  const int64_t a = lower_key(store, sw, ns, ukeys[j]);
  const int64_t kept_before = a < ns ? (int64_t)keep_pre[a] : (ns ? (int64_t)keep_pre[ns - 1] + keep[ns - 1] : 0);
  uint64_t* d = out + (kept_before + fin_pre[j]) * sw;
  const uint64_t* s = srow + scap[j] * sw;
  for (int64_t k = 0; k < fin[j] * sw; k++) d[k] = s[k];
}

// ------------------------------------------------------------------ host side

template <class F>
static khip_status cub_call(DevBuf& tmp, hipStream_t st, F&& f) {
  size_t bytes = 0;
  if (f(nullptr, bytes) != hipSuccess) return fail(KHIP_E_DEVICE, "hipcub size query failed");
  KHIP_TRY(tmp.ensure(std::max<size_t>(bytes, 16)));
  if (f(tmp.p, bytes) != hipSuccess) return fail(KHIP_E_DEVICE, "hipcub call failed");
  (void)st;
  return KHIP_OK;
}

khip_status sess_push(khip_agg* a, int64_t n, const int64_t* keys, const int64_t* ts, const uint8_t* kv,
                      const uint8_t* rv, const ColPtrs& cols, int64_t* tot) {
  SessState& S = a->sess;
  hipStream_t st = a->stream;
  const int sw = a->sw;
  const int64_t nb = ceil_div(n, RPB);
  KHIP_TRY(a->blockmax.ensure(nb * 8));
  KHIP_TRY(a->blockprefix.ensure(nb * 8));
  KHIP_TRY(S.ctr.ensure(32 * 8));
  KHIP_TRY_HIP(hipMemsetAsync(S.ctr.p, 0, 32 * 8, st));
  hipLaunchKernelGGL(k_blockmax, dim3(nb), dim3(BLOCK), 0, st, ts, kv, rv, n, a->blockmax.as<int64_t>());
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, st, a->blockmax.as<int64_t>(), nb,
                     a->blockprefix.as<int64_t>(), a->stream_time.as<int64_t>());
  KHIP_TRY(S.skey.ensure(n * 8));
  KHIP_TRY(S.sidx.ensure(n * 8));
  KHIP_TRY(S.skey2.ensure(n * 8));
  KHIP_TRY(S.sidx2.ensure(n * 8));
  KHIP_TRY(S.st_after.ensure(n * 8));
  hipLaunchKernelGGL(k_sess_prep, dim3(nb), dim3(BLOCK), 0, st, keys, ts, kv, rv, n, a->blockprefix.as<int64_t>(),
                     S.skey.as<int64_t>(), S.sidx.as<int64_t>(), S.st_after.as<int64_t>(),
                     S.ctr.as<unsigned long long>());
  KHIP_TRY_HIP(hipGetLastError());
  // group by key, arrival order kept within a key (LSD radix sort is stable)
  const int ni = (int)n;
  int64_t* k_in = S.skey.as<int64_t>();
  int64_t* k_out = S.skey2.as<int64_t>();
  int64_t* v_in = S.sidx.as<int64_t>();
  int64_t* v_out = S.sidx2.as<int64_t>();
  KHIP_TRY(cub_call(S.tmp, st, [&](void* p, size_t& b) {
    return hipcub::DeviceRadixSort::SortPairs(p, b, k_in, k_out, v_in, v_out, ni, 0, 64, st);
  }));
  KHIP_TRY(S.ukeys.ensure(n * 8));
  KHIP_TRY(S.ucnt.ensure(n * 4));
  KHIP_TRY(S.nseg.ensure(16));
  KHIP_TRY(cub_call(S.tmp, st, [&](void* p, size_t& b) {
    return hipcub::DeviceRunLengthEncode::Encode(p, b, k_out, S.ukeys.as<int64_t>(), S.ucnt.as<int>(), S.nseg.as<int>(),
                                                 ni, st);
  }));
  int nseg = 0;
  KHIP_TRY_HIP(hipMemcpyAsync(&nseg, S.nseg.p, 4, hipMemcpyDeviceToHost, st));
  KHIP_TRY_HIP(hipStreamSynchronize(st));
  KHIP_TRY(S.useg.ensure((size_t)(nseg + 1) * 8));
  KHIP_TRY(S.s0.ensure((size_t)(nseg + 1) * 8));
  KHIP_TRY(S.cap.ensure((size_t)(nseg + 1) * 8));
  KHIP_TRY(S.scap.ensure((size_t)(nseg + 1) * 8));
  KHIP_TRY(S.fin.ensure((size_t)(nseg + 1) * 8));
  KHIP_TRY(S.fin_pre.ensure((size_t)(nseg + 1) * 8));
  KHIP_TRY(cub_call(S.tmp, st, [&](void* p, size_t& b) {
    return hipcub::DeviceScan::ExclusiveSum(p, b, S.ucnt.as<int>(), S.useg.as<int64_t>(), nseg, st);
  }));
  const uint64_t* store = S.rows.as<uint64_t>();
  const int64_t ns = S.n;
  hipLaunchKernelGGL(k_sess_bounds, dim3(ceil_div(nseg, 256)), dim3(256), 0, st, store, ns, sw, S.ukeys.as<int64_t>(),
                     S.ucnt.as<int>(), S.nseg.as<int>(), S.s0.as<int64_t>(), S.cap.as<int64_t>());
  KHIP_TRY(cub_call(S.tmp, st, [&](void* p, size_t& b) {
    return hipcub::DeviceScan::ExclusiveSum(p, b, S.cap.as<int64_t>(), S.scap.as<int64_t>(), nseg, st);
  }));
  const int64_t scr = ns + n;  // total scratch rows >= sum of capacities
  KHIP_TRY(S.srow.ensure((size_t)scr * sw * 8));
  KHIP_TRY(S.sfl.ensure((size_t)scr));
  KHIP_TRY(S.trow.ensure((size_t)scr * sw * 8));
  const bool keep_changes = a->changelog;
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
  hipLaunchKernelGGL(k_sess_apply, dim3(ceil_div(nseg, 64)), dim3(64), 0, st, q, store, S.ukeys.as<int64_t>(),
                     S.ucnt.as<int>(), S.useg.as<int64_t>(), S.nseg.as<int>(), S.s0.as<int64_t>(), S.cap.as<int64_t>(),
                     S.scap.as<int64_t>(), v_out, ts, kv, rv, cols, S.st_after.as<int64_t>(),
                     a->stream_time.as<int64_t>(), S.srow.as<uint64_t>(), S.sfl.as<uint8_t>(), S.trow.as<uint64_t>(),
                     S.fin.as<int64_t>(), keep_changes ? S.crow.as<uint64_t>() : nullptr,
                     keep_changes ? S.ctomb.as<uint8_t>() : nullptr, S.ctr.as<unsigned long long>(), keep_changes ? 1 : 0);
  KHIP_TRY_HIP(hipGetLastError());
  // the new store
  KHIP_TRY(S.keep.ensure((size_t)(ns + 1) * 4));
  KHIP_TRY(S.keep_pre.ensure((size_t)(ns + 1) * 4));
  if (ns) {
    hipLaunchKernelGGL(k_sess_keep, dim3(ceil_div(ns, 256)), dim3(256), 0, st, store, ns, sw, S.ukeys.as<int64_t>(),
                       S.nseg.as<int>(), a->stream_time.as<int64_t>(), a->retention, S.keep.as<int>());
    KHIP_TRY(cub_call(S.tmp, st, [&](void* p, size_t& b) {
      return hipcub::DeviceScan::ExclusiveSum(p, b, S.keep.as<int>(), S.keep_pre.as<int>(), (int)ns, st);
    }));
  }
  // fin_pre[nseg] = total rewritten rows (inclusive end) via a scan over nseg + 1 entries
  KHIP_TRY_HIP(hipMemsetAsync(S.fin.as<int64_t>() + nseg, 0, 8, st));
  KHIP_TRY(cub_call(S.tmp, st, [&](void* p, size_t& b) {
    return hipcub::DeviceScan::ExclusiveSum(p, b, S.fin.as<int64_t>(), S.fin_pre.as<int64_t>(), nseg + 1, st);
  }));
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
  hipLaunchKernelGGL(k_sess_scatter_seg, dim3(ceil_div(nseg, 64)), dim3(64), 0, st, store, ns, sw, S.keep_pre.as<int>(),
                     S.keep.as<int>(), S.ukeys.as<int64_t>(), S.nseg.as<int>(), S.fin.as<int64_t>(),
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
  DevBuf* bufs[] = {&S.rows, &S.rows2, &S.skey, &S.sidx, &S.skey2, &S.sidx2, &S.st_after, &S.ukeys, &S.ucnt, &S.nseg,
                    &S.useg, &S.s0, &S.cap, &S.scap, &S.fin, &S.fin_pre, &S.srow, &S.sfl, &S.trow, &S.crow, &S.ctomb,
                    &S.keep, &S.keep_pre, &S.ctr, &S.tmp};
  for (DevBuf* b : bufs) b->release();
  S.n = 0;
  S.nchg = 0;
}

}  // namespace khip
