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

// The handle's stream time in the PARTITION domain: the smallest partition stream time.
khip_status stream_time_partition_min(khip_agg* a) {
  hipLaunchKernelGGL(k_st_min, dim3(1), dim3(256), 0, a->stream, a->pst.as<int64_t>(), a->desc.n_partitions,
                     a->stream_time.as<int64_t>());
  KHIP_TRY_HIP(hipGetLastError());
  int64_t h = -1;
  KHIP_TRY_HIP(hipMemcpyAsync(&h, a->stream_time.p, 8, hipMemcpyDeviceToHost, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  a->host_stream_time = h;
  return KHIP_OK;
}

}  // namespace khip
