// khip_shuffle.hip — repartition for non-key GROUP BY / PARTITION BY, and the RCCL exchange.
//
// Replaces the repartition topic round-trip of StreamGroupByBuilderBase.build
// (S/StreamGroupByBuilderBase.java:101-103: filter(v != null).groupBy(mapper) → sink
// "<ctx>-repartition" → source) and StreamSelectKeyBuilder (S/StreamSelectKeyBuilder.java:73-74):
//   k_shuf_hist      per 4096-record tile: drop null value / null new key / negative ts
//                    (S/GroupByParamsFactory.java:92-100), count rows per destination
//   (column prefix)  reuses the partitioned engine's k_part_colsum/colbase/colprefix
//   k_shuf_pack      STABLE scatter of packed rows to their destination's contiguous run
//                    (wave ballots per destination + cross-wave LDS prefix keep arrival order)
//   khip_comm_alltoall  grouped ncclSend/ncclRecv, one pair per peer over xGMI (every MI355X
//                    pair has a direct link, so this is per-link bound, not a ring)
//   k_shuf_pack1     one destination: the same rows in one pass (decoupled look-back, no histogram)
//   k_shuf_packv     several destinations in one pass (ABI 7): each wave counts its contiguous run
//                    of the tile per destination, the tile looks back over the earlier tiles'
//                    per-destination counts, rows go to per-destination regions of the send buffer
//   khip_comm_alltoall_v  the all-to-all over those regions
//   k_shuf_unpack    packed rows → columnar batch (bitmaps built with __ballot)
// KHIP_SHUFFLE_STREAM_TIME rows carry the batch's stream_time word before the validity word.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "khip_agg_internal.hpp"
#include "khip_sort.hpp"

namespace khip {


constexpr int SH_THREADS = 256;
constexpr int SH_ITEMS = 16;
constexpr int64_t SH_TILE = (int64_t)SH_THREADS * SH_ITEMS;
constexpr int SH_MAX_PARTS = 256;
constexpr int SH_MAX_COLS = 8;

struct ShCols {
  int32_t key_bytes;
  const void* data[SH_MAX_COLS];
  const uint8_t* valid[SH_MAX_COLS];
  int32_t type[SH_MAX_COLS];
  const int64_t* st;  // KHIP_SHUFFLE_STREAM_TIME: the batch's stream_time column (else null)
  int64_t st_seed;    // the word written is max(st_seed, st[i]) (khip_shuffle_stream_time_seed)
};

__device__ __forceinline__ uint64_t sh_st(const ShCols& c, int64_t i) {
  const int64_t v = c.st[i];
  return (uint64_t)(v > c.st_seed ? v : c.st_seed);
}

// Kafka's default partitioner over the KAFKA-format key (big-endian 4 / 8 bytes,
// ksqldb-serde/.../kafka/KafkaSerdeFactory.java:42-43): toPositive(murmur2(bytes)) % n_parts,
// so a record lands on the same partition the reference's repartition topic would give it.
__device__ __forceinline__ uint32_t murmur2_word(uint32_t h, uint32_t k) {
  const uint32_t m = 0x5bd1e995u;
  k *= m;
  k ^= k >> 24;
  k *= m;
  return (h * m) ^ k;
}

__device__ __forceinline__ uint32_t shuffle_dest(int64_t key, int key_bytes, int n_parts) {
  const uint32_t m = 0x5bd1e995u;
  const uint64_t v = (uint64_t)key;
  uint32_t h = 0x9747b28cu ^ (uint32_t)key_bytes;
  // the little-endian load of big-endian bytes is a byte swap of each 32-bit half
  if (key_bytes == 8) {
    h = murmur2_word(h, __builtin_bswap32((uint32_t)(v >> 32)));
    h = murmur2_word(h, __builtin_bswap32((uint32_t)v));
  } else {
    h = murmur2_word(h, __builtin_bswap32((uint32_t)v));
  }
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (h & 0x7fffffffu) % (uint32_t)n_parts;
}

__device__ __forceinline__ int64_t sh_raw(const ShCols& c, int col, int64_t i) {
  if (c.type[col] == KHIP_TYPE_INT32) return (int64_t)((const int32_t*)c.data[col])[i];
  return ((const int64_t*)c.data[col])[i];
}

__device__ __forceinline__ bool sh_valid(const ShCols& c, int key_col, const uint8_t* rv, const int64_t* ts,
                                         int64_t i) {
  return bit_get(rv, i) && bit_get(c.valid[key_col], i) && ts[i] >= 0;
}

__global__ __launch_bounds__(SH_THREADS) void k_shuf_hist(ShCols c, int key_col, const uint8_t* __restrict__ rv,
                                                          const int64_t* __restrict__ ts, int64_t n, int n_parts,
                                                          uint32_t* __restrict__ hist) {
  __shared__ uint32_t lh[SH_MAX_PARTS];
  for (int d = threadIdx.x; d < n_parts; d += SH_THREADS) lh[d] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * SH_TILE;
  for (int r = 0; r < SH_ITEMS; r++) {
    const int64_t i = base + (int64_t)r * SH_THREADS + threadIdx.x;
    if (i < n && sh_valid(c, key_col, rv, ts, i)) atomicAdd(&lh[shuffle_dest(sh_raw(c, key_col, i), c.key_bytes, n_parts)], 1u);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < n_parts; d += SH_THREADS) hist[(int64_t)blockIdx.x * n_parts + d] = lh[d];
}

__global__ __launch_bounds__(SH_THREADS) void k_shuf_pack(ShCols c, int n_cols, int key_col,
                                                          const uint8_t* __restrict__ rv, const int64_t* __restrict__ ts,
                                                          int64_t n, int n_parts, const uint32_t* __restrict__ offs,
                                                          uint64_t* __restrict__ out, int row_words) {
  __shared__ uint32_t cur[SH_MAX_PARTS];
  __shared__ uint32_t wcnt[SH_THREADS / 64][SH_MAX_PARTS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int d = threadIdx.x; d < n_parts; d += SH_THREADS) cur[d] = offs[(int64_t)blockIdx.x * n_parts + d];
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * SH_TILE;
  const uint64_t lt = (1ULL << lane) - 1;
  for (int r = 0; r < SH_ITEMS; r++) {
    const int64_t i = base + (int64_t)r * SH_THREADS + threadIdx.x;
    const bool v = i < n && sh_valid(c, key_col, rv, ts, i);
    const int64_t key = v ? sh_raw(c, key_col, i) : 0;
    const int d = v ? (int)shuffle_dest(key, c.key_bytes, n_parts) : -1;
    // rank among earlier lanes of this wave with the same destination; wave totals → LDS.
    // One ballot per destination PRESENT in the wave (peeled by leader lane), not per n_parts.
    for (int dd = lane; dd < n_parts; dd += 64) wcnt[wave][dd] = 0;
    int rank = 0;
    uint64_t pending = __ballot(v);
    while (pending) {
      const int dl = __shfl(d, __ffsll((unsigned long long)pending) - 1);
      const uint64_t m = __ballot(d == dl);
      if (d == dl) rank = __popcll(m & lt);
      if (lane == 0) wcnt[wave][dl] = (uint32_t)__popcll(m);
      pending &= ~m;
    }
    __syncthreads();
    if (v) {
      uint32_t pos = cur[d] + rank;
      for (int w = 0; w < wave; w++) pos += wcnt[w][d];
      uint64_t* o = out + (uint64_t)pos * row_words;
      o[0] = (uint64_t)key;
      o[1] = (uint64_t)ts[i];
      // the key column travels as word 0 only (its validity is implied)
      uint64_t vm = 1ULL << key_col;
      int w = 2;
      for (int cc = 0; cc < n_cols; cc++) {
        if (cc == key_col) continue;
        const bool cv = bit_get(c.valid[cc], i);
        o[w++] = cv ? (uint64_t)sh_raw(c, cc, i) : 0ULL;
        vm |= (cv ? 1ULL : 0ULL) << cc;
      }
      if (c.st) o[w++] = sh_st(c, i);
      o[w] = vm;
    }
    __syncthreads();
    for (int dd = threadIdx.x; dd < n_parts; dd += SH_THREADS) {
      uint32_t s = 0;
      for (int w = 0; w < SH_THREADS / 64; w++) s += wcnt[w][dd];
      cur[dd] += s;
    }
    __syncthreads();
  }
}

// One destination (a single task: the repartition keeps every row here): the pack is a stable
// compaction, and needs no histogram pass.  Tiles are taken in ticket order; a tile counts its
// valid rows (ballots per wave and round), publishes the count and looks back over the earlier
// tiles' published counts / inclusive prefixes for its first output row (decoupled look-back, as
// khip_sort.hpp's k_rs_pass), then writes its rows in arrival order.  A tile waits only on
// tiles with earlier tickets, which are already running.  status[nT] and *ticket start at 0; the
// last tile leaves the total in *total.
constexpr uint64_t SH_AGG = 1ULL << 62, SH_INC = 2ULL << 62, SH_VAL = (1ULL << 62) - 1;

// Decoupled look-back by one whole wave: the exclusive prefix of tile `tile` over the status words
// status[j * stride] of the tiles j < tile (AGG | the tile's count, or INC | its inclusive prefix).
// The 64 lanes read 64 predecessors at once and stop at the nearest INC: a walk by one thread paid
// a memory round trip per predecessor, and the pack waited on that chain (C5's one-destination
// pack ran 1.93 ms with it, 1.45 ms with no look-back at all).  A predecessor that has not
// published yet is running (tickets are taken in dispatch order) and publishes its count before it
// looks back itself, so the wait ends.  (Measured: pack1 1.92 -> 1.84 ms; most of the 0.48 ms the
// look-back costs is the wait for predecessors' counts, not the walk.)
__device__ __forceinline__ uint64_t sh_wave_lookback(const uint64_t* status, int64_t tile, uint64_t stride) {
  const int lane = threadIdx.x & 63;
  uint64_t excl = 0;
  for (int64_t j0 = tile - 1; j0 >= 0; j0 -= 64) {
    const int64_t j = j0 - lane;
    uint64_t st = j >= 0 ? __hip_atomic_load(status + (uint64_t)j * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                         : SH_INC;  // before tile 0: an inclusive prefix of 0
    while (__ballot(!(st & ~SH_VAL))) {
      __builtin_amdgcn_s_sleep(1);
      if (!(st & ~SH_VAL))
        st = __hip_atomic_load(status + (uint64_t)j * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const uint64_t inc = __ballot((st & SH_INC) != 0);
    const int first = inc ? __ffsll((unsigned long long)inc) - 1 : 64;
    uint64_t v = lane <= first ? (st & SH_VAL) : 0;  // the nearest INC and the aggregates after it
#pragma unroll
    for (int off = 32; off; off >>= 1) v += __shfl_xor(v, off, 64);
    excl += v;
    if (inc) break;
  }
  return excl;
}

// Batch row i as its packed row, in registers: 2 + NC + ST words, padded to an even count so that
// a row of an even word count leaves as 16-byte pairs.
template <int NC, int ST>
struct ShRow {
  static constexpr int W = 2 + NC + ST;
  static constexpr int RW = W + (W & 1);
  uint64_t w[RW];
};

template <int NC, int ST>
__device__ __forceinline__ void sh_build_t(const ShCols& c, int key_col, int64_t tsv, int64_t i, ShRow<NC, ST>& r) {
#pragma unroll
  for (int k = 0; k < ShRow<NC, ST>::RW; k++) r.w[k] = 0;
  r.w[0] = (uint64_t)sh_raw(c, key_col, i);
  r.w[1] = (uint64_t)tsv;
  uint64_t vm = 1ULL << key_col;  // the key column travels as word 0 only (its validity is implied)
  int w = 2;
#pragma unroll
  for (int cc = 0; cc < NC; cc++) {
    if (cc == key_col) continue;
    const bool cv = bit_get(c.valid[cc], i);
    const uint64_t x = cv ? (uint64_t)sh_raw(c, cc, i) : 0ULL;
#pragma unroll
    for (int k = 2; k < 2 + NC - 1; k++) r.w[k] = k == w ? x : r.w[k];  // no dynamic register index
    w++;
    vm |= (cv ? 1ULL : 0ULL) << cc;
  }
  if (ST) r.w[1 + NC] = sh_st(c, i);
  r.w[1 + NC + ST] = vm;
}
template <int NC, int ST>
__device__ __forceinline__ void sh_build(const ShCols& c, int key_col, const int64_t* __restrict__ ts, int64_t i,
                                         ShRow<NC, ST>& r) {
  sh_build_t<NC, ST>(c, key_col, ts[i], i, r);
}

template <int NC, int ST>
__device__ __forceinline__ void sh_store(uint64_t* o, const ShRow<NC, ST>& r) {
  constexpr int W = ShRow<NC, ST>::W;
  if (W % 2 == 0) {
#pragma unroll
    for (int k = 0; k < W / 2; k++) ((ulonglong2*)o)[k] = make_ulonglong2(r.w[2 * k], r.w[2 * k + 1]);
  } else {
#pragma unroll
    for (int k = 0; k < W; k++) o[k] = r.w[k];
  }
}

template <int NC, int ST>  // the column count and the stream-time word: the row is built in registers
__global__ __launch_bounds__(SH_THREADS) void k_shuf_pack1(ShCols c, int key_col,
                                                           const uint8_t* __restrict__ rv, const int64_t* __restrict__ ts,
                                                           int64_t n, int64_t nT, uint64_t* __restrict__ status,
                                                           unsigned int* __restrict__ ticket, uint64_t* __restrict__ out,
                                                           unsigned long long* __restrict__ total) {
  constexpr int W = SH_THREADS / 64;
  __shared__ uint32_t wcnt[SH_ITEMS][W];
  __shared__ int64_t lbase;
  __shared__ uint32_t ltile;
  __shared__ int64_t lts[SH_ITEMS][SH_THREADS];  // the tile's ts, read once (the second pass missed L2)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t lt = lane ? (~0ULL >> (64 - lane)) : 0ULL;
  if (threadIdx.x == 0) ltile = atomicAdd(ticket, 1u);
  __syncthreads();
  const int64_t tile = ltile;
  const int64_t base = tile * SH_TILE;
  uint32_t vmask = 0;  // bit r: this thread's row of round r is kept (ts and the rows re-read below: L2)
#pragma unroll
  for (int r = 0; r < SH_ITEMS; r++) {
    const int64_t i = base + (int64_t)r * SH_THREADS + threadIdx.x;
    const int64_t tv = i < n ? ts[i] : -1;
    lts[r][threadIdx.x] = tv;
    const bool v = i < n && tv >= 0 && bit_get(rv, i) && bit_get(c.valid[key_col], i);
    const uint64_t m = __ballot(v);
    if (lane == 0) wcnt[r][wave] = (uint32_t)__popcll(m);
    vmask |= (v ? 1u : 0u) << r;
  }
  __syncthreads();
  if (wave == 0) {
    uint32_t acc = 0;
    if (lane == 0) {  // exclusive prefix in (round, wave) order = arrival order
      for (int r = 0; r < SH_ITEMS; r++)
        for (int w = 0; w < W; w++) {
          const uint32_t e = wcnt[r][w];
          wcnt[r][w] = acc;
          acc += e;
        }
      __hip_atomic_store(status + tile, (tile == 0 ? SH_INC : SH_AGG) | acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    acc = __shfl(acc, 0, 64);
    const uint64_t excl = sh_wave_lookback(status, tile, 1);
    if (lane == 0) {
      if (tile > 0)
        __hip_atomic_store(status + tile, SH_INC | (excl + acc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      lbase = (int64_t)excl;
      if (tile == nT - 1) *total = excl + acc;
    }
  }
  __syncthreads();
  for (int r = 0; r < SH_ITEMS; r++) {
    const bool v = (vmask >> r) & 1u;
    const uint32_t rank = (uint32_t)__popcll(__ballot(v) & lt);
    if (!v) continue;
    const int64_t i = base + (int64_t)r * SH_THREADS + threadIdx.x;
    ShRow<NC, ST> row;
    sh_build_t<NC, ST>(c, key_col, lts[r][threadIdx.x], i, row);
    sh_store<NC, ST>(out + (uint64_t)(lbase + wcnt[r][wave] + rank) * ShRow<NC, ST>::W, row);
  }
}

// One destination without the look-back (KHIP_PACK1_SPLIT): a count pass (ts and the two
// validity bitmaps: 8.25 B/row) gives every tile its row count, a scan its first output row, and
// the write pass is k_shuf_pack1 with that base — no tile waits on another's count (the look-back
// wait cost the one-pass pack ~0.4 ms of its 1.84 at C5, more than reading ts twice).
#ifndef KHIP_PACK1_SPLIT
#define KHIP_PACK1_SPLIT 1
#endif
__global__ __launch_bounds__(SH_THREADS) void k_shuf_count1(const uint8_t* __restrict__ kvalid,
                                                            const uint8_t* __restrict__ rv, const int64_t* __restrict__ ts,
                                                            int64_t n, int64_t* __restrict__ tcnt) {
  __shared__ int wsum[SH_THREADS / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * SH_TILE;
  int cnt = 0;
#pragma unroll
  for (int r = 0; r < SH_ITEMS; r++) {
    const int64_t i = base + (int64_t)r * SH_THREADS + threadIdx.x;
    const bool v = i < n && ts[i] >= 0 && bit_get(rv, i) && bit_get(kvalid, i);
    cnt += (int)__popcll(__ballot(v));
  }
  if (lane == 0) wsum[wave] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < SH_THREADS / 64; w++) t += wsum[w];
    tcnt[blockIdx.x] = t;
  }
}

template <int NC, int ST>
__global__ __launch_bounds__(SH_THREADS) void k_shuf_write1(ShCols c, int key_col,
                                                            const uint8_t* __restrict__ rv, const int64_t* __restrict__ ts,
                                                            int64_t n, const int64_t* __restrict__ tbase,
                                                            uint64_t* __restrict__ out) {
  constexpr int W = SH_THREADS / 64;
  __shared__ uint32_t wcnt[SH_ITEMS][W];
  __shared__ int64_t lts[SH_ITEMS][SH_THREADS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t lt = lane ? (~0ULL >> (64 - lane)) : 0ULL;
  const int64_t tile = blockIdx.x;
  const int64_t base = tile * SH_TILE;
  uint32_t vmask = 0;
#pragma unroll
  for (int r = 0; r < SH_ITEMS; r++) {
    const int64_t i = base + (int64_t)r * SH_THREADS + threadIdx.x;
    const int64_t tv = i < n ? ts[i] : -1;
    lts[r][threadIdx.x] = tv;
    const bool v = i < n && tv >= 0 && bit_get(rv, i) && bit_get(c.valid[key_col], i);
    const uint64_t m = __ballot(v);
    if (lane == 0) wcnt[r][wave] = (uint32_t)__popcll(m);
    vmask |= (v ? 1u : 0u) << r;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // exclusive prefix in (round, wave) order = arrival order
    uint32_t acc = 0;
    for (int r = 0; r < SH_ITEMS; r++)
      for (int w = 0; w < W; w++) {
        const uint32_t e = wcnt[r][w];
        wcnt[r][w] = acc;
        acc += e;
      }
  }
  __syncthreads();
  const int64_t lbase = tbase[tile];
  for (int r = 0; r < SH_ITEMS; r++) {
    const bool v = (vmask >> r) & 1u;
    const uint32_t rank = (uint32_t)__popcll(__ballot(v) & lt);
    if (!v) continue;
    const int64_t i = base + (int64_t)r * SH_THREADS + threadIdx.x;
    ShRow<NC, ST> row;
    sh_build_t<NC, ST>(c, key_col, lts[r][threadIdx.x], i, row);
    sh_store<NC, ST>(out + (uint64_t)(lbase + wcnt[r][wave] + rank) * ShRow<NC, ST>::W, row);
  }
}

// Several destinations in one pass (khip_shuffle_pack_v).  Tiles of SH_TILE rows in ticket order;
// wave w of a tile owns the contiguous run [w * SH_TILE / W, (w + 1) * SH_TILE / W) of it, so a
// wave's rounds are in arrival order and it ranks its rows per destination against wave-private
// running counts in LDS (a ballot per destination present in the round, no block barrier).  One
// barrier, then thread d (< n_parts) prefixes the waves' counts of destination d, publishes the
// tile's count and looks back over the earlier tiles' counts / inclusive prefixes of d (decoupled
// look-back, status[tile * n_parts + d]).  The rows (re-read: L2) are written at
// d * stride + (the tile's place in d) + (the wave's place) + rank; a row past its region's stride
// is not written and raises *overflow (the host packs again with the exact stride, from the totals
// the last tile leaves in totals[d]).
template <int NC, int ST>
__global__ __launch_bounds__(SH_THREADS) void k_shuf_packv(ShCols c, int key_col, const uint8_t* __restrict__ rv,
                                                           const int64_t* __restrict__ ts, int64_t n, int64_t nT,
                                                           int n_parts, uint64_t* __restrict__ status,
                                                           unsigned int* __restrict__ ticket, uint64_t* __restrict__ out,
                                                           int64_t stride, unsigned long long* __restrict__ totals,
                                                           unsigned int* __restrict__ overflow) {
  constexpr int W = SH_THREADS / 64;
  constexpr int PER_WAVE = SH_TILE / W;  // 1024 rows: SH_ITEMS rounds of 64
  __shared__ uint32_t wc[W][SH_MAX_PARTS];
  __shared__ int64_t dbase[SH_MAX_PARTS];
  __shared__ uint32_t ltile;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t lt = lane ? (~0ULL >> (64 - lane)) : 0ULL;
  if (threadIdx.x == 0) ltile = atomicAdd(ticket, 1u);
  for (int d = lane; d < n_parts; d += 64) wc[wave][d] = 0;  // the wave's own counts: no barrier needed
  __syncthreads();
  const int64_t tile = ltile;
  const int64_t wbase = tile * SH_TILE + (int64_t)wave * PER_WAVE;
  uint32_t rec[SH_ITEMS];  // destination << 16 | rank within the wave's rows of that destination
#pragma unroll
  for (int r = 0; r < SH_ITEMS; r++) {
    const int64_t i = wbase + (int64_t)r * 64 + lane;
    const bool v = i < n && ts[i] >= 0 && bit_get(rv, i) && bit_get(c.valid[key_col], i);
    const int d = v ? (int)shuffle_dest(sh_raw(c, key_col, i), c.key_bytes, n_parts) : -1;
    uint32_t x = 0xFFFFFFFFu;
    uint64_t pending = __ballot(v);
    while (pending) {  // one ballot per destination present in the round
      const int dl = __shfl(d, __ffsll((unsigned long long)pending) - 1);
      const uint64_t m = __ballot(d == dl);
      const uint32_t b = wc[wave][dl];
      if (d == dl) x = ((uint32_t)dl << 16) | (b + (uint32_t)__popcll(m & lt));
      if (lane == 0) wc[wave][dl] = b + (uint32_t)__popcll(m);
      pending &= ~m;
    }
    rec[r] = x;
  }
  __syncthreads();
  for (int d = threadIdx.x; d < n_parts; d += SH_THREADS) {
    uint32_t acc = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
      const uint32_t e = wc[w][d];
      wc[w][d] = acc;
      acc += e;
    }
    // (one thread per destination walks back: the destinations' walks run side by side in a wave;
    // a wave-wide look-back per destination, its 64 predecessors' words strided by n_parts, ran
    // 2.3-2.9 ms against 1.8-2.1 at 2-8 destinations)
    uint64_t* sd = status + (uint64_t)tile * n_parts + d;
    __hip_atomic_store(sd, (tile == 0 ? SH_INC : SH_AGG) | acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t excl = 0;
    for (int64_t j = tile - 1; j >= 0;) {
      const uint64_t st = __hip_atomic_load(status + (uint64_t)j * n_parts + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!(st & ~SH_VAL)) {
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      excl += st & SH_VAL;
      if (st & SH_INC) break;
      j--;
    }
    if (tile > 0) __hip_atomic_store(sd, SH_INC | (excl + acc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    dbase[d] = (int64_t)excl;
    if (tile == nT - 1) totals[d] = excl + acc;
  }
  __syncthreads();
  bool over = false;
#pragma unroll
  for (int r = 0; r < SH_ITEMS; r++) {
    const uint32_t x = rec[r];
    if (x == 0xFFFFFFFFu) continue;
    const int d = (int)(x >> 16);
    const int64_t pos = dbase[d] + wc[wave][d] + (x & 0xFFFFu);
    if (pos >= stride) {
      over = true;
      continue;
    }
    const int64_t i = wbase + (int64_t)r * 64 + lane;
    ShRow<NC, ST> row;
    sh_build<NC, ST>(c, key_col, ts, i, row);
    sh_store<NC, ST>(out + ((uint64_t)d * (uint64_t)stride + (uint64_t)pos) * ShRow<NC, ST>::W, row);
  }
  if (__ballot(over) && lane == 0) atomicOr(overflow, 1u);
}

__global__ __launch_bounds__(256) void k_shuf_unpack(const uint64_t* __restrict__ rows, int64_t n, int n_cols,
                                                     int key_col, int row_words, ShCols types, int64_t* __restrict__ key,
                                                     int64_t* __restrict__ ts, void* const* __restrict__ col_data,
                                                     uint8_t* const* __restrict__ col_valid) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const bool in = i < n;
  const uint64_t* r = rows + (in ? i : 0) * (uint64_t)row_words;
  const uint64_t vm = in ? r[row_words - 1] : 0;
  if (in) {
    key[i] = (int64_t)r[0];
    ts[i] = (int64_t)r[1];
  }
  const int lane = threadIdx.x & 63;
  const int64_t wbase = i - lane;
  for (int c = 0, w = 2; c < n_cols; c++) {
    const uint64_t word = c == key_col ? (in ? r[0] : 0) : (in ? r[w++] : 0);
    if (in && col_data[c]) {
      if (types.type[c] == KHIP_TYPE_INT32) ((int32_t*)col_data[c])[i] = (int32_t)word;
      else ((uint64_t*)col_data[c])[i] = word;
    }
    const uint64_t b = __ballot(in && ((vm >> c) & 1));
    if (col_valid && col_valid[c] && lane == 0 && wbase < n) {
      const int64_t nbytes = std::min<int64_t>(8, (n - wbase + 7) / 8);
      for (int k = 0; k < nbytes; k++) col_valid[c][wbase / 8 + k] = (uint8_t)(b >> (8 * k));
    }
  }
}

__global__ __launch_bounds__(256) void k_shuf_unpack_st(const uint64_t* __restrict__ rows, int64_t n, int row_words,
                                                        int64_t* __restrict__ st) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) st[i] = (int64_t)rows[i * row_words + row_words - 2];
}

}  // namespace khip

using namespace khip;

struct khip_shuffle {
  khip_shuffle_desc desc{};
  std::vector<int32_t> types;
  hipStream_t stream = nullptr;
  DevBuf hist, csum, pbase, R, ptrs;
  DevBuf tcnt, tbase, scan_tmp;  // the one-destination pack's tile counts and their prefix
  int64_t st_seed = -1;  // khip_shuffle_stream_time_seed
};

struct khip_comm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0, device = 0;
  hipStream_t stream = nullptr;
  DevBuf cnt;
};

namespace khip {
// The packed-row layout of a shuffle (khip_agg_push_shuffled reads received rows with it).
void shuffle_layout(const khip_shuffle* s, int* key_col, int* n_cols, const int32_t** types) {
  *key_col = s->desc.key_col;
  *n_cols = s->desc.n_cols;
  *types = s->types.data();
}
}  // namespace khip

extern "C" {

khip_status khip_shuffle_create(const khip_shuffle_desc* d, khip_shuffle** out) {
  clear_error();
  if (!d || !out) return fail(KHIP_E_INVALID, "null argument");
  if (d->n_parts < 1 || d->n_parts > SH_MAX_PARTS) return fail(KHIP_E_UNSUPPORTED, "1..256 destinations");
  if (d->n_cols < 1 || d->n_cols > SH_MAX_COLS) return fail(KHIP_E_UNSUPPORTED, "1..8 value columns");
  if (d->key_col < 0 || d->key_col >= d->n_cols) return fail(KHIP_E_INVALID, "key column");
  for (int c = 0; c < d->n_cols; c++)
    if (d->col_types[c] < KHIP_TYPE_INT32 || d->col_types[c] > KHIP_TYPE_DOUBLE) return fail(KHIP_E_INVALID, "column type");
  if (d->col_types[d->key_col] == KHIP_TYPE_DOUBLE) return fail(KHIP_E_UNSUPPORTED, "DOUBLE group key");
  khip_shuffle* s = new khip_shuffle();
  s->desc = *d;
  s->types.assign(d->col_types, d->col_types + d->n_cols);
  s->desc.col_types = s->types.data();
  DeviceGuard g(d->device);
  if (hipStreamCreateWithFlags(&s->stream, hipStreamDefault) != hipSuccess) {
    delete s;
    return fail(KHIP_E_DEVICE, "hipStreamCreate failed (no device?)");
  }
  *out = s;
  return KHIP_OK;
}

static int shuffle_st(const khip_shuffle* s) { return (s->desc.flags & KHIP_SHUFFLE_STREAM_TIME) ? 1 : 0; }

int32_t khip_shuffle_row_words(const khip_shuffle* s) { return s ? 2 + s->desc.n_cols + shuffle_st(s) : 0; }

// The rows of each destination's region in khip_shuffle_pack_v: the even share plus 1/16 and a
// tile (a uniform hash over n_parts destinations stays within a few standard deviations, ~sqrt(n/N)).
static int64_t packv_stride(int64_t n, int N) { return ceil_div(n, N) + ceil_div(n, 16LL * N) + SH_TILE; }

int64_t khip_shuffle_pack_capacity(const khip_shuffle* s, int64_t n) {
  if (!s || n < 0) return 0;
  const int N = s->desc.n_parts;
  return N == 1 ? n : std::max<int64_t>(n, (int64_t)N * packv_stride(n, N));
}

static khip_status shuffle_cols(khip_shuffle* s, const khip_batch* b, ShCols* c) {
  if (b->n_cols < s->desc.n_cols || !b->ts || !b->col_data) return fail(KHIP_E_INVALID, "batch shape");
  if (shuffle_st(s) && !b->stream_time)
    return fail(KHIP_E_INVALID, "KHIP_SHUFFLE_STREAM_TIME: the batch has no stream_time column");
  *c = ShCols{};
  for (int k = 0; k < s->desc.n_cols; k++) {
    c->data[k] = b->col_data[k];
    c->valid[k] = b->col_valid ? b->col_valid[k] : nullptr;
    c->type[k] = s->types[k];
  }
  c->key_bytes = s->types[s->desc.key_col] == KHIP_TYPE_INT32 ? 4 : 8;
  c->st = shuffle_st(s) ? b->stream_time : nullptr;
  c->st_seed = s->st_seed;
  return KHIP_OK;
}

using Write1Fn = void (*)(ShCols, int, const uint8_t*, const int64_t*, int64_t, const int64_t*, uint64_t*);
using Pack1Fn = void (*)(ShCols, int, const uint8_t*, const int64_t*, int64_t, int64_t, uint64_t*, unsigned int*,
                         uint64_t*, unsigned long long*);
using PackvFn = void (*)(ShCols, int, const uint8_t*, const int64_t*, int64_t, int64_t, int, uint64_t*,
                         unsigned int*, uint64_t*, int64_t, unsigned long long*, unsigned int*);
#define KHIP_SH_FNS(K, ST) {K<1, ST>, K<2, ST>, K<3, ST>, K<4, ST>, K<5, ST>, K<6, ST>, K<7, ST>, K<8, ST>}

// The contiguous multi-destination pack: per-tile histograms, their column prefix, the stable
// scatter (two reads of the source's key column).  Destination d's rows at the sum of counts[0..d).
static khip_status pack_contiguous(khip_shuffle* s, const khip_batch* b, const ShCols& c, uint64_t* send,
                                   int64_t capacity, int64_t* counts) {
  const int64_t n = b->n_rows;
  const int N = s->desc.n_parts;
  const int64_t nT = ceil_div(n, SH_TILE);
  const int TC = (int)std::min<int64_t>(nT, 64);
  KHIP_TRY(s->hist.ensure((size_t)nT * N * 4));
  KHIP_TRY(s->csum.ensure((size_t)TC * N * 8));
  KHIP_TRY(s->pbase.ensure((N + 1) * 8));
  KHIP_TRY(s->R.ensure((N + 1) * 8));
  hipLaunchKernelGGL(k_shuf_hist, dim3(nT), dim3(SH_THREADS), 0, s->stream, c, s->desc.key_col, b->row_valid, b->ts, n,
                     N, s->hist.as<uint32_t>());
  hipLaunchKernelGGL(k_part_colsum, dim3(ceil_div(N, 256), TC), dim3(256), 0, s->stream, s->hist.as<uint32_t>(), nT, N,
                     TC, s->csum.as<int64_t>());
  hipLaunchKernelGGL(k_part_colbase, dim3(ceil_div(N, 256)), dim3(256), 0, s->stream, s->csum.as<int64_t>(), N, TC,
                     s->R.as<int64_t>());
  KHIP_TRY_HIP(hipMemcpyAsync(s->pbase.p, s->R.p, N * 8, hipMemcpyDeviceToDevice, s->stream));
  KHIP_TRY_HIP(hipMemsetAsync(s->pbase.as<int64_t>() + N, 0, 8, s->stream));
  hipLaunchKernelGGL(k_scan_excl, dim3(1), dim3(1024), 0, s->stream, s->pbase.as<int64_t>(), (int64_t)N,
                     s->pbase.as<int64_t>() + N);
  hipLaunchKernelGGL(k_part_colprefix, dim3(ceil_div(N, 256), TC), dim3(256), 0, s->stream, s->hist.as<uint32_t>(), nT,
                     N, TC, s->csum.as<int64_t>(), s->pbase.as<int64_t>(), 1);
  KHIP_TRY_HIP(hipGetLastError());
  std::vector<int64_t> R(N);
  KHIP_TRY_HIP(hipMemcpyAsync(R.data(), s->R.p, N * 8, hipMemcpyDeviceToHost, s->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(s->stream));
  int64_t tot = 0;
  for (int d = 0; d < N; d++) tot += R[d];
  for (int d = 0; d < N; d++) counts[d] = R[d];
  if (tot > capacity || !send) return fail(KHIP_E_BUFFER, "send buffer too small");
  hipLaunchKernelGGL(k_shuf_pack, dim3(nT), dim3(SH_THREADS), 0, s->stream, c, s->desc.n_cols, s->desc.key_col,
                     b->row_valid, b->ts, n, N, s->hist.as<uint32_t>(), send, khip_shuffle_row_words(s));
  KHIP_TRY_HIP(hipGetLastError());
  KHIP_TRY_HIP(hipStreamSynchronize(s->stream));
  return KHIP_OK;
}

khip_status khip_shuffle_pack(khip_shuffle* s, const khip_batch* b, uint64_t* send, int64_t capacity, int64_t* counts) {
  clear_error();
  if (!s || !b || !counts) return fail(KHIP_E_INVALID, "null argument");
  if (b->mem != KHIP_MEM_DEVICE) return fail(KHIP_E_INVALID, "pack needs a device batch");
  const int64_t n = b->n_rows;
  const int N = s->desc.n_parts;
  if (n == 0) {
    for (int d = 0; d < N; d++) counts[d] = 0;
    return KHIP_OK;
  }
  if (n >= (1LL << 31)) return fail(KHIP_E_UNSUPPORTED, "pack batch larger than 2^31 rows");
  DeviceGuard g(s->desc.device);
  ShCols c;
  KHIP_TRY(shuffle_cols(s, b, &c));
  const int64_t nT = ceil_div(n, SH_TILE);
  if (N == 1 && send && capacity >= n && KHIP_PACK1_SPLIT) {  // one destination: count, scan, write
    KHIP_TRY(s->tcnt.ensure((size_t)nT * 8));
    KHIP_TRY(s->tbase.ensure((size_t)(nT + 1) * 8));
    hipLaunchKernelGGL(k_shuf_count1, dim3(nT), dim3(SH_THREADS), 0, s->stream, c.valid[s->desc.key_col], b->row_valid,
                       b->ts, n, s->tcnt.as<int64_t>());
    KHIP_TRY_HIP(hipGetLastError());
    KHIP_TRY((ksort::scan_excl<int64_t, int64_t>(s->stream, s->scan_tmp, s->tcnt.as<int64_t>(), s->tbase.as<int64_t>(), nT,
                                                 true, nullptr)));
    static const Write1Fn w1[2][SH_MAX_COLS] = {KHIP_SH_FNS(k_shuf_write1, 0), KHIP_SH_FNS(k_shuf_write1, 1)};
    hipLaunchKernelGGL(w1[shuffle_st(s)][s->desc.n_cols - 1], dim3(nT), dim3(SH_THREADS), 0, s->stream, c,
                       s->desc.key_col, b->row_valid, b->ts, n, s->tbase.as<int64_t>(), send);
    KHIP_TRY_HIP(hipGetLastError());
    int64_t tot = 0;
    KHIP_TRY_HIP(hipMemcpyAsync(&tot, s->tbase.as<int64_t>() + nT, 8, hipMemcpyDeviceToHost, s->stream));
    KHIP_TRY_HIP(hipStreamSynchronize(s->stream));
    counts[0] = tot;
    return KHIP_OK;
  }
  if (N == 1 && send && capacity >= n) {  // one destination: a one-pass stable compaction
    KHIP_TRY(s->R.ensure((size_t)(nT + 2) * 8));
    uint64_t* status = s->R.as<uint64_t>();
    unsigned int* ticket = (unsigned int*)(status + nT);
    unsigned long long* total = (unsigned long long*)(status + nT + 1);
    KHIP_TRY_HIP(hipMemsetAsync(status, 0, (size_t)(nT + 2) * 8, s->stream));
    static const Pack1Fn k1[2][SH_MAX_COLS] = {KHIP_SH_FNS(k_shuf_pack1, 0), KHIP_SH_FNS(k_shuf_pack1, 1)};
    hipLaunchKernelGGL(k1[shuffle_st(s)][s->desc.n_cols - 1], dim3(nT), dim3(SH_THREADS), 0, s->stream, c,
                       s->desc.key_col, b->row_valid, b->ts, n, nT, status, ticket, send, total);
    KHIP_TRY_HIP(hipGetLastError());
    unsigned long long tot = 0;
    KHIP_TRY_HIP(hipMemcpyAsync(&tot, total, 8, hipMemcpyDeviceToHost, s->stream));
    KHIP_TRY_HIP(hipStreamSynchronize(s->stream));
    counts[0] = (int64_t)tot;
    return KHIP_OK;
  }
  return pack_contiguous(s, b, c, send, capacity, counts);
}

khip_status khip_shuffle_pack_v(khip_shuffle* s, const khip_batch* b, uint64_t* send, int64_t capacity, int64_t* counts,
                                int64_t* offsets) {
  clear_error();
  if (!s || !b || !counts || !offsets) return fail(KHIP_E_INVALID, "null argument");
  if (b->mem != KHIP_MEM_DEVICE) return fail(KHIP_E_INVALID, "pack needs a device batch");
  const int64_t n = b->n_rows;
  const int N = s->desc.n_parts;
  if (n == 0) {
    for (int d = 0; d < N; d++) counts[d] = offsets[d] = 0;
    return KHIP_OK;
  }
  if (n >= (1LL << 31)) return fail(KHIP_E_UNSUPPORTED, "pack batch larger than 2^31 rows");
  if (!send || capacity < khip_shuffle_pack_capacity(s, n))
    return fail(KHIP_E_BUFFER, "send buffer smaller than khip_shuffle_pack_capacity");
  if (N == 1) {
    offsets[0] = 0;
    return khip_shuffle_pack(s, b, send, capacity, counts);
  }
  DeviceGuard g(s->desc.device);
  ShCols c;
  KHIP_TRY(shuffle_cols(s, b, &c));
  const int64_t nT = ceil_div(n, SH_TILE);
  // status[nT * N] | ticket, overflow (one word) | totals[N]
  KHIP_TRY(s->R.ensure((size_t)(nT * N + 1 + N) * 8));
  uint64_t* status = s->R.as<uint64_t>();
  unsigned int* ticket = (unsigned int*)(status + nT * N);
  unsigned int* overflow = ticket + 1;
  unsigned long long* totals = (unsigned long long*)(status + nT * N + 1);
  static const PackvFn kv[2][SH_MAX_COLS] = {KHIP_SH_FNS(k_shuf_packv, 0), KHIP_SH_FNS(k_shuf_packv, 1)};
  int64_t stride = packv_stride(n, N);
  for (int attempt = 0; attempt < 2; attempt++) {
    KHIP_TRY_HIP(hipMemsetAsync(status, 0, (size_t)(nT * N + 1 + N) * 8, s->stream));
    hipLaunchKernelGGL(kv[shuffle_st(s)][s->desc.n_cols - 1], dim3(nT), dim3(SH_THREADS), 0, s->stream, c,
                       s->desc.key_col, b->row_valid, b->ts, n, nT, N, status, ticket, send, stride, totals, overflow);
    KHIP_TRY_HIP(hipGetLastError());
    std::vector<uint64_t> tail((size_t)N + 1);
    KHIP_TRY_HIP(hipMemcpyAsync(tail.data(), status + nT * N, (size_t)(N + 1) * 8, hipMemcpyDeviceToHost, s->stream));
    KHIP_TRY_HIP(hipStreamSynchronize(s->stream));
    const bool over = (tail[0] >> 32) != 0;
    int64_t mx = 0;
    for (int d = 0; d < N; d++) {
      counts[d] = (int64_t)tail[1 + d];
      offsets[d] = (int64_t)d * stride;
      mx = std::max(mx, counts[d]);
    }
    if (!over) return KHIP_OK;
    if ((int64_t)N * mx > capacity) break;  // a skewed batch: the exact regions do not fit
    stride = mx;                            // the exact stride always fits the largest destination
  }
  KHIP_TRY(pack_contiguous(s, b, c, send, capacity, counts));
  for (int64_t d = 0, o = 0; d < N; d++) {
    offsets[d] = o;
    o += counts[d];
  }
  return KHIP_OK;
}

khip_status khip_shuffle_unpack(khip_shuffle* s, const uint64_t* rows, int64_t n, int64_t* key, int64_t* ts,
                                void* const* col_data, uint8_t* const* col_valid) {
  clear_error();
  if (!s || (n > 0 && (!rows || !key || !ts))) return fail(KHIP_E_INVALID, "null argument");
  if (n == 0) return KHIP_OK;
  DeviceGuard g(s->desc.device);
  const int nc = s->desc.n_cols;
  ShCols t{};
  for (int k = 0; k < nc; k++) t.type[k] = s->types[k];
  // column pointer arrays must be readable by the kernel: stage them in device memory
  std::vector<uint64_t> host(2 * SH_MAX_COLS, 0);
  for (int k = 0; k < nc; k++) {
    host[k] = (uint64_t)(col_data ? col_data[k] : nullptr);
    host[SH_MAX_COLS + k] = (uint64_t)(col_valid ? col_valid[k] : nullptr);
  }
  KHIP_TRY(s->ptrs.ensure(host.size() * 8));
  KHIP_TRY_HIP(hipMemcpyAsync(s->ptrs.p, host.data(), host.size() * 8, hipMemcpyHostToDevice, s->stream));
  hipLaunchKernelGGL(k_shuf_unpack, dim3(ceil_div(n, 256)), dim3(256), 0, s->stream, rows, n, nc, s->desc.key_col,
                     khip_shuffle_row_words(s), t, key, ts, (void* const*)s->ptrs.p,
                     (uint8_t* const*)(s->ptrs.as<uint64_t>() + SH_MAX_COLS));
  KHIP_TRY_HIP(hipGetLastError());
  KHIP_TRY_HIP(hipStreamSynchronize(s->stream));
  return KHIP_OK;
}

khip_status khip_shuffle_unpack_stream_time(khip_shuffle* s, const uint64_t* rows, int64_t n, int64_t* stream_time) {
  clear_error();
  if (!s || (n > 0 && (!rows || !stream_time))) return fail(KHIP_E_INVALID, "null argument");
  if (!shuffle_st(s)) return fail(KHIP_E_INVALID, "the shuffle carries no stream time (KHIP_SHUFFLE_STREAM_TIME)");
  if (n == 0) return KHIP_OK;
  DeviceGuard g(s->desc.device);
  hipLaunchKernelGGL(k_shuf_unpack_st, dim3(ceil_div(n, 256)), dim3(256), 0, s->stream, rows, n,
                     khip_shuffle_row_words(s), stream_time);
  KHIP_TRY_HIP(hipGetLastError());
  KHIP_TRY_HIP(hipStreamSynchronize(s->stream));
  return KHIP_OK;
}

khip_status khip_shuffle_stream_time_seed(khip_shuffle* s, int64_t seed) {
  clear_error();
  if (!s) return fail(KHIP_E_INVALID, "null argument");
  if (!shuffle_st(s)) return fail(KHIP_E_INVALID, "the shuffle carries no stream time (KHIP_SHUFFLE_STREAM_TIME)");
  s->st_seed = seed < -1 ? -1 : seed;
  return KHIP_OK;
}

khip_status khip_shuffle_sync(khip_shuffle* s) {
  if (!s) return fail(KHIP_E_INVALID, "null argument");
  DeviceGuard g(s->desc.device);
  KHIP_TRY_HIP(hipStreamSynchronize(s->stream));
  return KHIP_OK;
}

khip_status khip_shuffle_destroy(khip_shuffle* s) {
  if (!s) return KHIP_OK;
  DeviceGuard g(s->desc.device);
  hipStreamSynchronize(s->stream);
  s->hist.release();
  s->csum.release();
  s->pbase.release();
  s->R.release();
  s->ptrs.release();
  hipStreamDestroy(s->stream);
  delete s;
  return KHIP_OK;
}

// ------------------------------------------------------------------------ RCCL

#define KHIP_TRY_NCCL(expr)                                                       \
  do {                                                                            \
    ncclResult_t _r = (expr);                                                     \
    if (_r != ncclSuccess) {                                                      \
      ::khip::set_error(std::string(#expr) + ": " + ncclGetErrorString(_r));      \
      return KHIP_E_COMM;                                                         \
    }                                                                             \
  } while (0)

khip_status khip_comm_unique_id(uint8_t id[KHIP_COMM_ID_BYTES]) {
  clear_error();
  if (!id) return fail(KHIP_E_INVALID, "null argument");
  ncclUniqueId u;
  KHIP_TRY_NCCL(ncclGetUniqueId(&u));
  memcpy(id, u.internal, KHIP_COMM_ID_BYTES);
  return KHIP_OK;
}

khip_status khip_comm_init(int32_t nranks, int32_t rank, const uint8_t id[KHIP_COMM_ID_BYTES], int32_t device,
                           khip_comm** out) {
  clear_error();
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return fail(KHIP_E_INVALID, "bad communicator arguments");
  DeviceGuard g(device);
  khip_comm* c = new khip_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamDefault) != hipSuccess) {
    delete c;
    return fail(KHIP_E_DEVICE, "hipStreamCreate failed");
  }
  ncclUniqueId u;
  memcpy(u.internal, id, KHIP_COMM_ID_BYTES);
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) {
    hipStreamDestroy(c->stream);
    delete c;
    return fail(KHIP_E_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  *out = c;
  return KHIP_OK;
}

// Inside ncclGroupStart/End: remember the first failure but keep going, so the group is always
// closed (an open group on one rank leaves its peers blocked in their own ncclGroupEnd).
struct GroupErr {
  ncclResult_t r = ncclSuccess;
  const char* what = nullptr;
  void note(ncclResult_t x, const char* w) {
    if (x != ncclSuccess && r == ncclSuccess) {
      r = x;
      what = w;
    }
  }
  khip_status finish(ncclResult_t end) {
    note(end, "ncclGroupEnd");
    if (r == ncclSuccess) return KHIP_OK;
    ::khip::set_error(std::string(what) + ": " + ncclGetErrorString(r));
    return KHIP_E_COMM;
  }
};

khip_status khip_comm_exchange_counts(khip_comm* c, const int64_t* send_counts, int64_t* recv_counts) {
  clear_error();
  if (!c || !send_counts || !recv_counts) return fail(KHIP_E_INVALID, "null argument");
  DeviceGuard g(c->device);
  const int N = c->nranks;
  KHIP_TRY(c->cnt.ensure(2 * N * 8));
  int64_t* dsend = c->cnt.as<int64_t>();
  int64_t* drecv = dsend + N;
  KHIP_TRY_HIP(hipMemcpyAsync(dsend, send_counts, N * 8, hipMemcpyHostToDevice, c->stream));
  KHIP_TRY_NCCL(ncclGroupStart());
  GroupErr ge;
  for (int p = 0; p < N; p++) {
    ge.note(ncclSend(dsend + p, 1, ncclInt64, p, c->comm, c->stream), "ncclSend");
    ge.note(ncclRecv(drecv + p, 1, ncclInt64, p, c->comm, c->stream), "ncclRecv");
  }
  KHIP_TRY(ge.finish(ncclGroupEnd()));
  KHIP_TRY_HIP(hipMemcpyAsync(recv_counts, drecv, N * 8, hipMemcpyDeviceToHost, c->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(c->stream));
  return KHIP_OK;
}

khip_status khip_comm_alltoall(khip_comm* c, const uint64_t* send, const int64_t* send_counts, uint64_t* recv,
                               int64_t recv_capacity, const int64_t* recv_counts, int32_t row_words) {
  clear_error();
  if (!c || !send_counts || !recv_counts || row_words < 1) return fail(KHIP_E_INVALID, "null argument");
  DeviceGuard g(c->device);
  const int N = c->nranks;
  int64_t tot = 0;
  for (int p = 0; p < N; p++) tot += recv_counts[p];
  if (tot > recv_capacity) return fail(KHIP_E_BUFFER, "receive buffer smaller than the exchanged counts");
  int64_t so = 0, ro = 0;
  KHIP_TRY_NCCL(ncclGroupStart());
  GroupErr ge;
  for (int p = 0; p < N; p++) {
    if (send_counts[p])
      ge.note(ncclSend(send + so * row_words, (size_t)send_counts[p] * row_words, ncclUint64, p, c->comm, c->stream),
              "ncclSend");
    if (recv_counts[p])
      ge.note(ncclRecv(recv + ro * row_words, (size_t)recv_counts[p] * row_words, ncclUint64, p, c->comm, c->stream),
              "ncclRecv");
    so += send_counts[p];
    ro += recv_counts[p];
  }
  KHIP_TRY(ge.finish(ncclGroupEnd()));
  KHIP_TRY_HIP(hipStreamSynchronize(c->stream));
  return KHIP_OK;
}

khip_status khip_comm_alltoall_v(khip_comm* c, const uint64_t* send, const int64_t* send_counts,
                                 const int64_t* send_offsets, uint64_t* recv, int64_t recv_capacity,
                                 const int64_t* recv_counts, int32_t row_words) {
  clear_error();
  if (!c || !send_counts || !send_offsets || !recv_counts || row_words < 1) return fail(KHIP_E_INVALID, "null argument");
  DeviceGuard g(c->device);
  const int N = c->nranks;
  int64_t tot = 0;
  for (int p = 0; p < N; p++) tot += recv_counts[p];
  if (tot > recv_capacity) return fail(KHIP_E_BUFFER, "receive buffer smaller than the exchanged counts");
  int64_t ro = 0;
  KHIP_TRY_NCCL(ncclGroupStart());
  GroupErr ge;
  for (int p = 0; p < N; p++) {
    if (send_counts[p])
      ge.note(ncclSend(send + send_offsets[p] * row_words, (size_t)send_counts[p] * row_words, ncclUint64, p, c->comm,
                       c->stream),
              "ncclSend");
    if (recv_counts[p])
      ge.note(ncclRecv(recv + ro * row_words, (size_t)recv_counts[p] * row_words, ncclUint64, p, c->comm, c->stream),
              "ncclRecv");
    ro += recv_counts[p];
  }
  KHIP_TRY(ge.finish(ncclGroupEnd()));
  KHIP_TRY_HIP(hipStreamSynchronize(c->stream));
  return KHIP_OK;
}

khip_status khip_comm_destroy(khip_comm* c) {
  if (!c) return KHIP_OK;
  DeviceGuard g(c->device);
  hipStreamSynchronize(c->stream);
  if (c->comm) ncclCommDestroy(c->comm);
  c->cnt.release();
  hipStreamDestroy(c->stream);
  delete c;
  return KHIP_OK;
}

}  // extern "C"
