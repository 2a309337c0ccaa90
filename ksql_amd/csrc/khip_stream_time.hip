// khip_stream_time.hip — per-row stream time for the ABI 5 stream-time domains
// (include/ksqldb_hip.h KHIP_TIME_*).
//
// KStreamWindowAggregate keeps one observedStreamTime per task and raises it with every record
// that reaches the processor, before the record's late test (S/StreamAggregateBuilder.java:
// 287-294; SURVEY §8.0 "Stream time and late drop").  The engines compute it themselves for one
// task per handle (KHIP_TIME_TASK).  Here it is computed as a column, st[i] = the stream time
// observed at row i, for
//   - KHIP_TIME_PARTITION: one task per Kafka partition (the batch's `partition` column; each
//     partition's rows one contiguous run): a segmented inclusive prefix max, a segment per run,
//     seeded with that partition's stream time before the batch (kept on the device per handle);
//   - khip_stream_time_scan: one segment seeded by the caller (the upstream half of
//     KHIP_TIME_SUPPLIED: a rank's contiguous arrival chunk of the global stream).
// Rows with a null key, a null value or ts < 0 never reach the aggregate: they do not raise it.
//
//   k_st_tiles   per 4096-row tile: its segmented aggregate (a segment starts in it?, max since the
//                last segment start); run starts validated (partition in range, one run each)
//   k_st_carry   one workgroup: exclusive segmented scan of the tile aggregates → tile carry-in
//   k_st_apply   per tile: block-wide segmented scan with the carry-in → st[i]; every run's last
//                row writes its partition's new stream time
//   k_st_min     the smallest partition stream time → the handle's stream time (eviction of closed
//                windows must wait for the slowest task)
#include <algorithm>
#include <array>

#include "khip_agg_internal.hpp"

namespace khip {

constexpr int ST_NT = 1024;
constexpr int ST_PER = 4;  // rows per thread
constexpr int ST_TILE = ST_NT * ST_PER;

struct SegV {
  int f;      // a segment starts in the span
  int64_t v;  // max since the last segment start (or over the span)
};

__device__ __forceinline__ SegV seg_combine(SegV a, SegV b) { return SegV{a.f | b.f, b.f ? b.v : (a.v > b.v ? a.v : b.v)}; }

struct StIn {
  const int64_t* ts;
  const uint8_t* kv;
  const uint8_t* rv;
  const int32_t* part;  // null: one segment starting at row 0
  int64_t n;
  const int64_t* pst;  // per-partition stream time before the batch (part != null)
  int64_t seed;        // the single segment's seed (part == null)
  int32_t npart;
};

// Row i's (segment start?, value with the segment's seed folded into its first row).
__device__ __forceinline__ SegV st_elem(const StIn& in, int64_t i, int32_t* p_out, bool check, int* err,
                                        unsigned int* seen) {
  const int64_t t = in.ts[i];
  const bool valid = bit_get(in.kv, i) && bit_get(in.rv, i) && t >= 0;
  int64_t v = valid ? t : -1;
  int f;
  int32_t p = 0;
  if (in.part) {
    p = in.part[i];
    f = i == 0 || in.part[i - 1] != p;
    if (f) {
      if (p < 0 || p >= in.npart) {
        if (check) atomicOr(err, 1);
        p = 0;
      } else if (check && atomicAdd(&seen[p], 1u) != 0u) {
        atomicOr(err, 2);  // a partition with two runs
      }
      const int64_t s = in.pst[p];
      v = s > v ? s : v;
    }
  } else {
    f = i == 0;
    if (f) v = in.seed > v ? in.seed : v;
  }
  *p_out = p;
  return SegV{f, v};
}

// Block-wide exclusive segmented scan of one SegV per thread (ST_NT threads); returns the thread's
// exclusive prefix combined after `carry`, and the block total in *tot.
__device__ __forceinline__ SegV st_block_excl(SegV x, SegV carry, SegV* tot) {
  __shared__ int wf[ST_NT / 64];
  __shared__ int64_t wv[ST_NT / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  SegV inc = x;
  for (int off = 1; off < 64; off <<= 1) {
    const int of = __shfl_up(inc.f, off, 64);
    const int64_t ov = __shfl_up(inc.v, off, 64);
    if (lane >= off) inc = seg_combine(SegV{of, ov}, inc);
  }
  if (lane == 63) {
    wf[wave] = inc.f;
    wv[wave] = inc.v;
  }
  __syncthreads();
  SegV pre = carry;
  SegV all = SegV{0, -1};
  for (int w = 0; w < ST_NT / 64; w++) {
    const SegV ww{wf[w], wv[w]};
    if (w < wave) pre = seg_combine(pre, ww);
    all = seg_combine(all, ww);
  }
  __syncthreads();
  const int ef = __shfl_up(inc.f, 1, 64);
  const int64_t ev = __shfl_up(inc.v, 1, 64);
  *tot = all;
  return lane == 0 ? pre : seg_combine(pre, SegV{ef, ev});
}

__global__ __launch_bounds__(ST_NT) void k_st_tiles(StIn in, SegV* __restrict__ agg, int* __restrict__ err,
                                                    unsigned int* __restrict__ seen) {
  const int64_t base = (int64_t)blockIdx.x * ST_TILE + (int64_t)threadIdx.x * ST_PER;
  SegV x{0, -1};
  for (int k = 0; k < ST_PER; k++) {
    const int64_t i = base + k;
    if (i >= in.n) break;
    int32_t p;
    x = seg_combine(x, st_elem(in, i, &p, true, err, seen));
  }
  SegV tot;
  st_block_excl(x, SegV{0, -1}, &tot);
  if (threadIdx.x == 0) agg[blockIdx.x] = tot;
}

// carry[t] = combine(agg[0..t)) (thread j owns a contiguous range of tiles)
__global__ __launch_bounds__(ST_NT) void k_st_carry(const SegV* __restrict__ agg, int64_t nT, SegV* __restrict__ carry) {
  const int64_t K = (nT + ST_NT - 1) / ST_NT;
  const int64_t t0 = threadIdx.x * K, t1 = t0 + K < nT ? t0 + K : nT;
  SegV x{0, -1};
  for (int64_t t = t0; t < t1; t++) x = seg_combine(x, agg[t]);
  SegV tot;
  SegV run = st_block_excl(x, SegV{0, -1}, &tot);
  for (int64_t t = t0; t < t1; t++) {
    carry[t] = run;
    run = seg_combine(run, agg[t]);
  }
}

__global__ __launch_bounds__(ST_NT) void k_st_apply(StIn in, const SegV* __restrict__ carry, int64_t* __restrict__ st,
                                                    int64_t* __restrict__ pst_next, int64_t* __restrict__ last) {
  const int64_t base = (int64_t)blockIdx.x * ST_TILE + (int64_t)threadIdx.x * ST_PER;
  SegV e[ST_PER];
  int32_t p[ST_PER];
  SegV x{0, -1};
  for (int k = 0; k < ST_PER; k++) {
    const int64_t i = base + k;
    e[k] = SegV{0, -1};
    p[k] = 0;
    if (i < in.n) e[k] = st_elem(in, i, &p[k], false, nullptr, nullptr);
    x = seg_combine(x, e[k]);
  }
  SegV tot;
  SegV run = st_block_excl(x, carry[blockIdx.x], &tot);
  for (int k = 0; k < ST_PER; k++) {
    const int64_t i = base + k;
    if (i >= in.n) break;
    run = seg_combine(run, e[k]);
    st[i] = run.v;
    const bool seg_end = i + 1 == in.n || (in.part ? in.part[i + 1] != p[k] : false);
    if (seg_end && in.part) pst_next[p[k]] = run.v;
    if (i + 1 == in.n && last) *last = run.v;
  }
}

__global__ __launch_bounds__(256) void k_st_min(const int64_t* __restrict__ pst, int32_t npart,
                                                int64_t* __restrict__ stream_time) {
  __shared__ int64_t w[4];
  int64_t m = INT64_MAX;
  for (int p = threadIdx.x; p < npart; p += 256) m = pst[p] < m ? pst[p] : m;
  for (int off = 32; off > 0; off >>= 1) {
    const int64_t o = __shfl_xor(m, off, 64);
    m = o < m ? o : m;
  }
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 4; k++) m = w[k] < m ? w[k] : m;
    *stream_time = m == INT64_MAX ? -1 : m;
  }
}

// st[0..n) for one segment (part == null, seeded with `seed`) or the partition runs of `part`
// (seeded with and updating a->pst).  Device pointers; on a->stream.  *last: the final value of
// the single segment (device; may be null).
khip_status stream_time_column(khip_agg* a, const int64_t* ts, const uint8_t* kv, const uint8_t* rv,
                               const int32_t* part, int64_t n, int64_t seed, int64_t* st, int64_t* last) {
  const int64_t nT = ceil_div(n, ST_TILE);
  KHIP_TRY(a->st_agg.ensure((size_t)nT * sizeof(SegV) * 2 + 64));
  SegV* agg = a->st_agg.as<SegV>();
  SegV* carry = agg + nT;
  int* err = (int*)(carry + nT);
  StIn in{ts, kv, rv, part, n, part ? a->pst.as<int64_t>() : nullptr, seed, a->desc.n_partitions};
  unsigned int* seen = nullptr;
  if (part) {
    KHIP_TRY(a->st_seen.ensure((size_t)a->desc.n_partitions * 4));
    seen = a->st_seen.as<unsigned int>();
    KHIP_TRY_HIP(hipMemsetAsync(seen, 0, (size_t)a->desc.n_partitions * 4, a->stream));
    KHIP_TRY_HIP(hipMemcpyAsync(a->pst2.p, a->pst.p, (size_t)a->desc.n_partitions * 8, hipMemcpyDeviceToDevice,
                                a->stream));
  }
  KHIP_TRY_HIP(hipMemsetAsync(err, 0, 4, a->stream));
  if (n > 0) {
    hipLaunchKernelGGL(k_st_tiles, dim3(nT), dim3(ST_NT), 0, a->stream, in, agg, err, seen);
    hipLaunchKernelGGL(k_st_carry, dim3(1), dim3(ST_NT), 0, a->stream, agg, nT, carry);
    hipLaunchKernelGGL(k_st_apply, dim3(nT), dim3(ST_NT), 0, a->stream, in, carry, st,
                       part ? a->pst2.as<int64_t>() : nullptr, last);
    KHIP_TRY_HIP(hipGetLastError());
  }
  if (part) {
    int herr = 0;
    KHIP_TRY_HIP(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, a->stream));
    KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
    if (herr & 1) return fail(KHIP_E_INVALID, "batch partition outside [0, n_partitions)");
    if (herr & 2) return fail(KHIP_E_INVALID, "a partition's rows must form one contiguous run per batch");
    std::swap(a->pst, a->pst2);  // the partitions' stream times after the batch
  }
  return KHIP_OK;
}

// The handle's stream time in the PARTITION domain: the smallest partition stream time.  Every
// declared partition counts, one that has not received a record yet included (its stream time is
// -1): closed windows leave the live table by this bound, and a partition that starts late must
// still find its windows there.  An idle partition therefore holds eviction back (memory, not
// results: visibility, retention and EMIT FINAL are per partition, partition_bounds).  The host
// keeps copies of the partitions' stream times after and before the push.
khip_status stream_time_partition_min(khip_agg* a) {
  hipLaunchKernelGGL(k_st_min, dim3(1), dim3(256), 0, a->stream, a->pst.as<int64_t>(), a->desc.n_partitions,
                     a->stream_time.as<int64_t>());
  KHIP_TRY_HIP(hipGetLastError());
  int64_t h = -1;
  const size_t P = (size_t)a->desc.n_partitions;
  a->pst_host.resize(P);
  a->pst_prev_host.resize(P);
  KHIP_TRY_HIP(hipMemcpyAsync(&h, a->stream_time.p, 8, hipMemcpyDeviceToHost, a->stream));
  KHIP_TRY_HIP(hipMemcpyAsync(a->pst_host.data(), a->pst.p, P * 8, hipMemcpyDeviceToHost, a->stream));
  KHIP_TRY_HIP(hipMemcpyAsync(a->pst_prev_host.data(), a->pst2.p, P * 8, hipMemcpyDeviceToHost, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  a->host_stream_time = h;
  return KHIP_OK;
}

// ------------------------------------------------------------------ per-task retention / EMIT FINAL
// KHIP_TIME_PARTITION runs n_partitions tasks in one table; each task's window store expires and
// closes windows by ITS stream time (StreamAggregateBuilder.java:282-285 emitStrategy, :293
// window.getRetention(), applied per task by Kafka Streams).  Rows carry no partition, but keys
// are co-partitioned, so a key map (key → partition) recorded at every push gives each row its
// task at compaction time (store_ok).

constexpr int PM_PROBE = 256;

// ctr[0]: keys added (wave sums), ctr[1]: probe budget exhausted, ctr[2]: a key on two partitions
__global__ __launch_bounds__(256) void k_pmap_insert(const int64_t* __restrict__ keys, const uint8_t* __restrict__ kv,
                                                     const uint8_t* __restrict__ rv, const int64_t* __restrict__ ts,
                                                     const int32_t* __restrict__ part, int64_t n,
                                                     int64_t* __restrict__ pk, int32_t* __restrict__ pp,
                                                     unsigned long long* __restrict__ pts, uint64_t mask,
                                                     unsigned long long* __restrict__ ctr) {
  int64_t added = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (!(bit_get(kv, i) && bit_get(rv, i) && ts[i] >= 0)) continue;
    const int64_t k = keys[i];
    const int32_t p = part[i];
    const unsigned long long t = (unsigned long long)ts[i];
    if (k == INT64_MIN) {  // (its own slot, never pruned)
      const int old = atomicCAS(&pp[mask + 1], -1, p);
      if (old != -1 && old != p) atomicOr(&ctr[2], 1ULL);
      continue;
    }
    uint64_t sl = pmap_hash(k) & mask;
    bool done = false;
    for (int probe = 0; probe < PM_PROBE && !done; probe++) {
      int64_t c = (int64_t)__hip_atomic_load((uint64_t*)&pk[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (c == INT64_MIN) {
        const unsigned long long old = atomicCAS((unsigned long long*)&pk[sl], (unsigned long long)INT64_MIN,
                                                 (unsigned long long)k);
        if ((int64_t)old == INT64_MIN) {
          __hip_atomic_store(&pp[sl], p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          atomicMax(&pts[sl], t);
          added++;
          done = true;
          break;
        }
        c = (int64_t)old;
      }
      if (c == k) {
        // the claimer (another row of this batch, already past its CAS) stores its partition right
        // after it: wait for it, so that the same new key on two partitions in one batch is seen
        int32_t q = __hip_atomic_load(&pp[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int spin = 0; q == -1 && spin < (1 << 20); spin++) {
          __builtin_amdgcn_s_sleep(1);
          q = __hip_atomic_load(&pp[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (q == -1) atomicOr(&ctr[1], 1ULL);  // (never seen: counted as a failed insert, retried)
        if (q != -1 && q != p) atomicOr(&ctr[2], 1ULL);
        if (__hip_atomic_load(&pts[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < t) atomicMax(&pts[sl], t);
        done = true;
        break;
      }
      sl = (sl + 1) & mask;
    }
    if (!done) atomicOr(&ctr[1], 1ULL);
  }
  added = wave_sum(added);
  if ((threadIdx.x & 63) == 0 && added) atomicAdd(&ctr[0], (unsigned long long)added);
}

// The map's entries into a new map; with `cut` (per partition), only the keys whose latest record
// time reaches their partition's cut (pmap_prune).  kept: the entries moved (wave sums).
__global__ __launch_bounds__(256) void k_pmap_rehash(const int64_t* __restrict__ ok, const int32_t* __restrict__ op,
                                                     const uint64_t* __restrict__ ots, int64_t ocap,
                                                     const int64_t* __restrict__ cut, int n_parts,
                                                     int64_t* __restrict__ nk, int32_t* __restrict__ np,
                                                     uint64_t* __restrict__ nts, uint64_t nmask,
                                                     unsigned long long* __restrict__ kept) {
  int64_t moved = 0;
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < ocap; s += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = ok[s];
    if (k == INT64_MIN) continue;
    const int p = op[s];
    if (cut && p >= 0 && p < n_parts && (int64_t)ots[s] < cut[p]) continue;
    uint64_t d = pmap_hash(k) & nmask;
    while (atomicCAS((unsigned long long*)&nk[d], (unsigned long long)INT64_MIN, (unsigned long long)k) !=
           (unsigned long long)INT64_MIN)
      d = (d + 1) & nmask;
    np[d] = p;
    nts[d] = ots[s];
    moved++;
  }
  moved = wave_sum(moved);
  if ((threadIdx.x & 63) == 0 && moved) atomicAdd(kept, (unsigned long long)moved);
}

__global__ __launch_bounds__(256) void k_fill_i64(int64_t* __restrict__ p, int64_t n, int64_t v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

static int pm_grid(int64_t n) { return (int)std::min<int64_t>(std::max<int64_t>(ceil_div(n, 256), 1), 8192); }

// A new map of `cap` slots holding the current one's entries — all of them, or (cut != null) those
// of keys whose latest record time reaches their partition's cut.
static khip_status pmap_rebuild(khip_agg* a, int64_t cap, const int64_t* cut_host) {
  DevBuf nk, np, nt, cut;
  KHIP_TRY(nk.ensure((size_t)cap * 8));
  KHIP_TRY(np.ensure((size_t)(cap + 1) * 4));
  KHIP_TRY(nt.ensure((size_t)cap * 8));
  KHIP_TRY(a->pm_ctr.ensure(24));
  hipLaunchKernelGGL(k_fill_i64, dim3(pm_grid(cap)), dim3(256), 0, a->stream, nk.as<int64_t>(), cap, INT64_MIN);
  KHIP_TRY_HIP(hipMemsetAsync(np.p, 0xFF, (size_t)(cap + 1) * 4, a->stream));
  KHIP_TRY_HIP(hipMemsetAsync(nt.p, 0, (size_t)cap * 8, a->stream));
  unsigned long long kept = 0;
  if (a->pm_cap > 0) {
    const int P = a->desc.n_partitions;
    if (cut_host) {
      KHIP_TRY(cut.ensure((size_t)P * 8));
      KHIP_TRY_HIP(hipMemcpyAsync(cut.p, cut_host, (size_t)P * 8, hipMemcpyHostToDevice, a->stream));
    }
    KHIP_TRY_HIP(hipMemsetAsync(a->pm_ctr.p, 0, 8, a->stream));
    hipLaunchKernelGGL(k_pmap_rehash, dim3(pm_grid(a->pm_cap)), dim3(256), 0, a->stream, a->pm_key.as<int64_t>(),
                       a->pm_part.as<int32_t>(), a->pm_ts.as<uint64_t>(), a->pm_cap,
                       cut_host ? cut.as<int64_t>() : nullptr, P, nk.as<int64_t>(), np.as<int32_t>(), nt.as<uint64_t>(),
                       (uint64_t)(cap - 1), a->pm_ctr.as<unsigned long long>());
    KHIP_TRY_HIP(hipMemcpyAsync(np.as<int32_t>() + cap, a->pm_part.as<int32_t>() + a->pm_cap, 4,
                                hipMemcpyDeviceToDevice, a->stream));
    KHIP_TRY_HIP(hipMemcpyAsync(&kept, a->pm_ctr.p, 8, hipMemcpyDeviceToHost, a->stream));
  }
  KHIP_TRY_HIP(hipGetLastError());
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));  // (cut_host is the caller's)
  a->pm_key = std::move(nk);
  a->pm_part = std::move(np);
  a->pm_ts = std::move(nt);
  a->pm_cap = cap;
#ifdef KHIP_TUNING
  if (cut_host && getenv("KHIP_TRACE_PMAP"))
    fprintf(stderr, "pmap_prune: kept %llu of %lld keys\n", kept, (long long)a->pm_occ);
#endif
  if (cut_host && (int64_t)kept < a->pm_occ) a->pm_pruned = true;
  a->pm_occ = (int64_t)kept;
  return KHIP_OK;
}

static khip_status pmap_grow(khip_agg* a, int64_t cap) { return pmap_rebuild(a, cap, nullptr); }

// Before the map grows: the keys whose every window has expired in their task leave it (ADVICE r05:
// the map otherwise grows with every key ever seen).  A key's windows all start at or before its
// latest record time, so a key whose latest time is below its partition's retention cut (the
// visible_from rule at the partition's stream time before this push) has only expired windows,
// which with retention >= size + grace also closed before this push (EMIT FINAL emits none of them
// again); its rows stay invisible (store_ok: a key missing from a pruned map is expired).  A key
// that comes back is inserted afresh.  SESSION stores keep the whole map.
static khip_status pmap_prune(khip_agg* a) {
  const int P = a->desc.n_partitions;
  if (a->engine == 2 || a->pst_host.size() != (size_t)P || a->retention < a->desc.size_ms + a->grace) return KHIP_OK;
  std::vector<int64_t> cut((size_t)P);
  bool any = false;
  for (int p = 0; p < P; p++) {
    cut[p] = partition_vis_from(a, a->pst_host[p]);
    any = any || cut[p] != INT64_MIN;
  }
  if (!any) return KHIP_OK;
  return pmap_rebuild(a, a->pm_cap, cut.data());
}

khip_status pmap_insert(khip_agg* a, const int64_t* keys, const uint8_t* kv, const uint8_t* rv, const int64_t* ts,
                        const int32_t* part, int64_t n) {
  if (n <= 0) return KHIP_OK;
  // room for the keys this batch may add (as the key dictionary sizes itself: every row on the
  // first push, then twice the last push's new keys, at least n / 16); a batch that brings more
  // exhausts a probe budget and is inserted again into a larger map (inserts are idempotent)
  const int64_t est = a->pm_last < 0 ? n : std::min<int64_t>(n, std::max<int64_t>({2 * a->pm_last, n / 16, 4096}));
  if (a->pm_cap > 0 && 2 * (a->pm_occ + est) > a->pm_cap) KHIP_TRY(pmap_prune(a));
  if (a->pm_cap == 0 || 2 * (a->pm_occ + est) > a->pm_cap)
    KHIP_TRY(pmap_grow(a, next_pow2(std::max<int64_t>(4 * (a->pm_occ + est), 4096))));
  KHIP_TRY(a->pm_ctr.ensure(24));
  for (int attempt = 0;; attempt++) {
    KHIP_TRY_HIP(hipMemsetAsync(a->pm_ctr.p, 0, 24, a->stream));
    hipLaunchKernelGGL(k_pmap_insert, dim3(pm_grid(n)), dim3(256), 0, a->stream, keys, kv, rv, ts, part, n,
                       a->pm_key.as<int64_t>(), a->pm_part.as<int32_t>(), a->pm_ts.as<unsigned long long>(),
                       (uint64_t)(a->pm_cap - 1),
                       a->pm_ctr.as<unsigned long long>());
    KHIP_TRY_HIP(hipGetLastError());
    unsigned long long c[3];
    KHIP_TRY_HIP(hipMemcpyAsync(c, a->pm_ctr.p, 24, hipMemcpyDeviceToHost, a->stream));
    KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
    a->pm_occ += (int64_t)c[0];
    if (c[2]) return fail(KHIP_E_INVALID, "KHIP_TIME_PARTITION: a GROUP BY key arrived on two partitions "
                                          "(keys must be co-partitioned)");
    if (!c[1]) {
      a->pm_last = (int64_t)c[0];
      return KHIP_OK;
    }
    if (attempt >= 6) return fail(KHIP_E_DEVICE, "partition key map probe budget exhausted");
    KHIP_TRY(pmap_grow(a, a->pm_cap * 4));
  }
}

khip_status pmap_clear(khip_agg* a) {
  if (a->pm_cap == 0) return KHIP_OK;
  hipLaunchKernelGGL(k_fill_i64, dim3(pm_grid(a->pm_cap)), dim3(256), 0, a->stream, a->pm_key.as<int64_t>(), a->pm_cap,
                     INT64_MIN);
  KHIP_TRY_HIP(hipMemsetAsync(a->pm_part.p, 0xFF, (size_t)(a->pm_cap + 1) * 4, a->stream));
  KHIP_TRY_HIP(hipMemsetAsync(a->pm_ts.p, 0, (size_t)a->pm_cap * 8, a->stream));
  KHIP_TRY_HIP(hipGetLastError());
  a->pm_occ = 0;
  a->pm_pruned = false;
  return KHIP_OK;
}

void pmap_release(khip_agg* a) {
  a->pm_key.release();
  a->pm_part.release();
  a->pm_ts.release();
  a->pm_ctr.release();
  a->pdom.release();
  a->pm_cap = a->pm_occ = 0;
  a->pm_pruned = false;
  a->pm_last = -1;
}

// EMIT FINAL, per task: the k_emit_lost rule with each record's own partition stream time before it
// (the previous row of its run, or the partition's stream time before the batch).  lost: (p, lo, hi).
__global__ __launch_bounds__(256) void k_emit_lost_part(const int64_t* __restrict__ ts, const uint8_t* __restrict__ kv,
                                                        const uint8_t* __restrict__ rv, const int32_t* __restrict__ part,
                                                        const int64_t* __restrict__ st,
                                                        const int64_t* __restrict__ pst_before, int64_t n, int64_t size,
                                                        int64_t adv, int64_t grace, int64_t retention,
                                                        int64_t* __restrict__ lost, int64_t cap,
                                                        unsigned long long* __restrict__ ctr) {
  const int64_t sg = size + grace;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (!bit_get(kv, i) || !bit_get(rv, i)) continue;
    const int32_t p = part[i];
    const int64_t mp = (i > 0 && part[i - 1] == p) ? st[i - 1] : pst_before[p];
    const int64_t t = ts[i];
    if (t <= mp) continue;
    const int64_t bp = mp < 0 ? -1 : mp / adv, b = t / adv;
    if (b <= bp) continue;
    int64_t lo = mp - sg + 1;
    int64_t hi = t - sg;
    const int64_t exp_hi = b * adv - retention - 1;
    hi = hi < exp_hi ? hi : exp_hi;
    lo = lo < 0 ? 0 : lo;
    lo = (lo + adv - 1) / adv * adv;
    if (lo <= hi) {
      const unsigned long long slot = atomicAdd(ctr, 1ULL);
      if ((int64_t)slot < cap) {
        lost[3 * slot] = p;
        lost[3 * slot + 1] = lo;
        lost[3 * slot + 2] = hi;
      }
    }
  }
}

// Call after stream_time_column (a->pst2 = the partitions' stream times before the batch).
khip_status partition_lost(khip_agg* a, const int64_t* ts, const uint8_t* kv, const uint8_t* rv, const int32_t* part,
                           const int64_t* st, int64_t n) {
  KHIP_TRY(a->lostctr.ensure(16));
  if (a->lost_cap == 0) a->lost_cap = 4096;
  for (int attempt = 0; attempt < 2; attempt++) {
    KHIP_TRY(a->lostbuf.ensure((size_t)a->lost_cap * 24));
    KHIP_TRY_HIP(hipMemsetAsync(a->lostctr.p, 0, 8, a->stream));
    hipLaunchKernelGGL(k_emit_lost_part, dim3(pm_grid(n)), dim3(256), 0, a->stream, ts, kv, rv, part, st,
                       a->pst2.as<int64_t>(), n, a->desc.size_ms, a->desc.advance_ms, a->grace, a->retention,
                       a->lostbuf.as<int64_t>(), a->lost_cap, a->lostctr.as<unsigned long long>());
    KHIP_TRY_HIP(hipGetLastError());
    int64_t cnt = 0;
    KHIP_TRY_HIP(hipMemcpyAsync(&cnt, a->lostctr.p, 8, hipMemcpyDeviceToHost, a->stream));
    KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
    if (cnt <= a->lost_cap) break;
    a->lost_cap = next_pow2(cnt);
    a->lostbuf.release();
  }
  return KHIP_OK;
}

// The lost (p, lo, hi) triples of the last push → per partition sorted, merged ws ranges.
khip_status partition_lost_finish(khip_agg* a) {
  int64_t cnt = 0;
  KHIP_TRY_HIP(hipMemcpyAsync(&cnt, a->lostctr.p, 8, hipMemcpyDeviceToHost, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  std::vector<int64_t> t((size_t)cnt * 3);
  if (cnt) KHIP_TRY_HIP(hipMemcpyAsync(t.data(), a->lostbuf.p, (size_t)cnt * 24, hipMemcpyDeviceToHost, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  std::vector<std::array<int64_t, 3>> r((size_t)cnt);
  for (int64_t k = 0; k < cnt; k++) r[k] = {t[3 * k], t[3 * k + 1], t[3 * k + 2]};
  std::sort(r.begin(), r.end());
  const int P = a->desc.n_partitions;
  a->plost.clear();
  a->plost_off.assign((size_t)P + 1, 0);
  int64_t cur_p = -1;
  for (auto& x : r) {
    if (x[0] == cur_p && !a->plost.empty() && x[1] <= a->plost.back() + 1) {
      a->plost.back() = std::max(a->plost.back(), x[2]);
    } else {
      a->plost.push_back(x[1]);
      a->plost.push_back(x[2]);
      a->plost_off[(size_t)x[0] + 1]++;
      cur_p = x[0];
    }
  }
  for (int p = 0; p < P; p++) a->plost_off[p + 1] += a->plost_off[p];
  return KHIP_OK;
}

// A partition's first visible window start (the visible_from rule with its own stream time).
int64_t partition_vis_from(const khip_agg* a, int64_t pst) {
  if (pst < 0) return INT64_MIN;
  const int64_t adv = a->desc.advance_ms;
  const int64_t vf = pst / adv * adv - a->retention;
  return vf > 0 ? vf : INT64_MIN;
}

khip_status partition_bounds(khip_agg* a, HavingDev& h) {
  if (a->desc.time_domain != KHIP_TIME_PARTITION || !a->windowed || a->pm_cap == 0 || !(h.vis || h.fin))
    return KHIP_OK;
  const int P = a->desc.n_partitions;
  std::vector<int64_t> host;
  host.reserve((size_t)P * 4 + 2 + a->plost.size());
  const bool have = a->pst_host.size() == (size_t)P;
  for (int p = 0; p < P; p++) host.push_back(partition_vis_from(a, have ? a->pst_host[p] : -1));
  for (int p = 0; p < P; p++) {
    host.push_back((have ? a->pst_prev_host[p] : -1) - a->grace);
    host.push_back((have ? a->pst_host[p] : -1) - a->grace);
  }
  const bool lost_ok = a->plost_off.size() == (size_t)P + 1;
  for (int p = 0; p <= P; p++) host.push_back(lost_ok ? a->plost_off[p] : 0);
  host.insert(host.end(), a->plost.begin(), a->plost.end());
  KHIP_TRY(a->pdom.ensure(host.size() * 8));
  KHIP_TRY_HIP(hipMemcpyAsync(a->pdom.p, host.data(), host.size() * 8, hipMemcpyHostToDevice, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));  // `host` goes out of scope
  const int64_t* d = a->pdom.as<int64_t>();
  h.pm_key = a->pm_key.as<int64_t>();
  h.pm_part = a->pm_part.as<int32_t>();
  h.pm_mask = (uint64_t)(a->pm_cap - 1);
  h.pm_pruned = a->pm_pruned ? 1 : 0;
  h.p_vis = d;
  h.p_fin = d + P;
  h.p_lost_off = d + 3 * P;
  h.p_lost = d + 4 * P + 1;
  return KHIP_OK;
}

}  // namespace khip
