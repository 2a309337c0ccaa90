// khip_agg_c1.hip — the windowed COUNT(*) pipeline of the partitioned engine (C2's query:
// `SELECT k, COUNT(*) ... WINDOW TUMBLING ... GROUP BY k [HAVING ...]`).
//
// Same contract as part_push's general path (khip_agg_part.hip) — per record (SURVEY §8.0,
// Kafka Streams' KStreamWindowAggregate as called from S/StreamAggregateBuilder.java:287-294):
// stream time, TimeWindows.windowsFor, late drop, store update, row time = max ts — but the input
// is read once, and every record moves as 8 bytes:
//
//   k_c1_scatter  keys, ts, validity: every record → (key - kb, ts - T0), two int32s; invalid
//                 records (null key / row, ts < 0) as sentinels; each 4096-record step leaves as
//                 one run in bucket order (B coarse buckets: top bits of the key hash) with its
//                 per-bucket counts (the step-run layout: no histogram pass ahead of it); per step
//                 the largest and smallest accepted ts, per tile the counters and the key range.
//                 Optimistic: no record is assumed late.
//   (scan_excl over the [bucket][step] counts: each run's place in its bucket; k_c1_bases)
//   k_c1_check    one workgroup: stream time before each 4096-record step (exclusive prefix
//                 max), and the push is ACCEPTED only if no step can hold a late record (the
//                 general path's `fast` test per step), every ts fits ts - T0 in 31 bits and the
//                 keys fit 32 bits above the base kb; otherwise nothing was written and the host
//                 runs the general path (or the same push with kb = the key minimum).
//                 Also the window range, the group-identity width and the refine's chunk list.
//   k_c1_refine   per 8K-record chunk of a bucket, read from its step runs: sentinels dropped,
//                 keys rebased to the key minimum, records counting-sorted by their partition
//                 inside the bucket (LDS), written bucket-contiguously; the chunk's per-partition
//                 offsets (u16) go to a segment table
//   k_c1_merge    persistent workgroups, one partition per item: the partition's records are its
//                 segments of the bucket's chunks; (key - kmin, window) → a 32-bit identity when
//                 it fits (no key hash on the record path), LDS identity CAS + u32 row-time max +
//                 u32 count, claimed entries listed (the write-out walks the list, not the table);
//                 resident rows merged, closed rows evicted, HAVING counts and changelog flags
//                 maintained exactly as k_part_merge_c1 does (k_part_commit publishes)
//
// Algorithmic bytes per record: 16 + 8 (scatter) + 8 + 8 (refine) + 8 (merge read)
// + the table rows written (32 B per group) — against 16 + 24 + 16 + 8 + rows for the general
// path (DESIGN.md §(d)).
#include <algorithm>
#include <cstdio>
#include <type_traits>
#include <vector>

#include "khip_part.hpp"
#include "khip_sort.hpp"

namespace khip {

constexpr int C1_TILE = 65536;   // records per hist / scatter tile (the general path's tile)
constexpr int C1_NT = 512;       // workgroup size of every kernel here
constexpr int C1_CH = 8192;      // refine chunk (records), 16 per thread
// Record loads of the refines and merges: plain loads.  Nontemporal ones (rounds 3-5) re-fetched
// the lines two neighbouring runs or segments share and cost C2 1.94 -> 1.88 ms / step, C5's
// value refine 921 -> 839 us (profiles/r05/ab/record_loads_temporal.txt).
template <class T>
__device__ __forceinline__ T c1_ld(const T* p) {
  return *p;
}
constexpr int C1_SEGMAX = 512;   // chunks of one bucket the merge can hold (4M records)
constexpr int C1_SEGB = 7;       // the merge's segment lookup: one entry per 32, 64 or 128 records of an
constexpr int C1_SEGOF = 512;    // item (the finest that fits 512 entries; past 64K records: binary search)
constexpr uint32_t C1_SENT = 0x80000000u;  // low word of a sentinel record (ts - T0 never is)

// c1info (int64) slots
enum {
  CI_KMIN = 0,   // atomics (the scatters), reset by k_c1_check for the next push
  CI_KMAX = 1,
  CI_TFAIL = 2,  // some accepted ts - T0 outside int32 (k_c1_scatter)
  CI_T0 = 3,     // time base (the scatters' block 0)
  CI_GATE = 4,   // accepted (k_part_commit reads gate[4])
  CI_WBASE = 5,  // smallest window index (records and live resident rows)
  CI_WBITS = 6,
  CI_ID32 = 7,   // identity mode: 1 = u32 (krel << wbits | wrel), 0 = u64 (krel << 32 | wrel)
  CI_TMIN = 8,   // smallest accepted ts (row-time deltas are relative to it)
  CI_TMAX = 9,
  CI_KBITS = 10,
  CI_NCHUNK = 11,  // refine work items
  CI_KMINC = 12,   // kmin copied for the refine / merge
  CI_WHI = 13,     // largest relative window index
  CI_KRANGE = 14,
  CI_WIDE = 15,    // records of this push: 1 = key hash + u32 ts words (the key range is too wide)
  CI_REASON = 16,  // declined: 1 = the key range needs the wide records (the host retries with them)
  CI_FITS = 17,    // the key range fits the compact records (a wide push tells the host)
  CI_KBASE = 18,   // the key base of this push's records (the scatters)
  CI_KSHIFT = 19,  // kmin - kbase: the refines rebase the records to the key minimum
  CI_KFAIL = 20,   // some key fell outside the records' key field above kbase (the scatters)
  CI_N = 24
};

__device__ __forceinline__ int bits_of(uint64_t v) { return v ? 64 - __clzll((long long)v) : 0; }

// A c1info word another kernel produced (atomics / stores of the scatters, stores of
// k_c1_check): read with a device-coherent vector load, never through the scalar cache.
__device__ __forceinline__ int64_t ci_ld(const int64_t* ci, int k) {
  const uint64_t v = (uint64_t)__hip_atomic_load(&ci[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // uniform: back into scalar registers
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// ------------------------------------------------------------------ step-run layout
// The scatters write no bucket-contiguous output (that needs every tile's bucket counts first: a
// histogram pass over the keys): each step of S records leaves as ONE contiguous run of S records
// in bucket order at out[gs * S], and its per-bucket count / offset go to rcnt[b][gs] / roff[b][gs]
// (bucket-major; held in LDS for the tile's steps and written per bucket at its end).  The exclusive scan of rcnt gives each (bucket, step) run's place in the bucket's
// order (rpos); the refine reads a bucket's chunk from its step runs.  The key range, the time base
// and the bucket counts are all learned in the one read of the input.
template <int U, int NT, class R, bool W>
__device__ __forceinline__ uint32_t stage_step_runs(const R (&rec)[U], const uint32_t (&t32)[U], const uint32_t (&bin)[U],
                                                const bool (&ok)[U], int nb, uint32_t* cnt, uint32_t* sbase, int* wsum,
                                                R* sp, uint32_t* lt32, R* __restrict__ out, uint32_t* __restrict__ outT,
                                                int64_t gs, uint32_t* lrc, uint16_t* lro) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  uint32_t rank[U];
#pragma unroll
  for (int u = 0; u < U; u++) rank[u] = ok[u] ? atomicAdd(&cnt[bin[u]], 1u) : 0u;
  lds_barrier();
  const uint32_t c = t < nb ? cnt[t] : 0u;
  uint32_t incl = c;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) wsum[wave] = (int)incl;
  lds_barrier();
  uint32_t before = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < NT / 64; k++) {
    before += k < wave ? (uint32_t)wsum[k] : 0u;
    tot += (uint32_t)wsum[k];
  }
  if (t < nb) {
    sbase[t] = before + incl - c;
    lrc[t] = c;  // the step's row of the tile's run counts / offsets (flush_run_counts)
    lro[t] = (uint16_t)(before + incl - c);
    cnt[t] = 0u;
  }
  lds_barrier();
#pragma unroll
  for (int u = 0; u < U; u++)
    if (ok[u]) {
      const uint32_t i = sbase[bin[u]] + rank[u];
      sp[i] = rec[u];
      if (W) lt32[i] = t32[u];
    }
  lds_barrier();
  R* o = out + gs * (int64_t)(U * NT);
  for (uint32_t j = t; j < tot; j += NT) o[j] = sp[j];
  if (W) {
    uint32_t* oT = outT + gs * (int64_t)(U * NT);
    for (uint32_t j = t; j < tot; j += NT) oT[j] = lt32[j];
  }
  // the next step's first barrier (after its rank atomics) orders these LDS reads before any
  // rewrite of sbase / the stage
  return tot;
}

// The step's staged key offsets (key - kb, kbits wide, above bit 32 of the record's first word)
// → the workgroup's LDS minimum / maximum (one atomic pair per wave); registers only for the step.
template <int NT, class R>
__device__ __forceinline__ void step_krange(const R* sp, uint32_t tot, uint32_t kmask, uint32_t* lkr) {
  uint32_t mn = 0xFFFFFFFFu, mx = 0u;
  for (uint32_t j = threadIdx.x; j < tot; j += NT) {
    uint64_t w;
    if constexpr (sizeof(R) == 16) w = ((const ulonglong2*)sp)[j].x;
    else w = (uint64_t)((const int64_t*)sp)[j];
    const uint32_t kr = (uint32_t)(w >> 32) & kmask;
    mn = kr < mn ? kr : mn;
    mx = kr > mx ? kr : mx;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t a = __shfl_xor(mn, off, 64), b = __shfl_xor(mx, off, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  if ((threadIdx.x & 63) == 0 && mx >= mn) {
    atomicMin(&lkr[0], mn);
    atomicMax(&lkr[1], mx);
  }
}

// LDS of a step-run scatter: per bucket its step count and staged base, the staged records (and
// their ts words when W).
__host__ __device__ constexpr size_t run_stage_lds(int nb, int S, int rec_bytes, bool w) {
  return (size_t)nb * 8 + (size_t)S * rec_bytes + (w ? (size_t)S * 4 : 0);
}
// ... then the tile's run counts u32[spt][nb] and offsets u16[spt][nb], written out per bucket at
// the end of the tile
__host__ __device__ constexpr size_t run_cnt_lds(int nb, int spt) { return (size_t)nb * spt * 6; }

// The tile's SPT run counts / offsets of bucket b leave as whole 16-byte stores (rcnt[b][t * SPT ..],
// roff[b][t * SPT ..]: 64 + 32 B for SPT = 16) instead of a 4-byte and a 2-byte store per step and
// bucket, which the memory side turned into 32-byte partial writes (C2: ~250 MB a push).  Steps
// past the input (the last tile's) are empty runs.  Thread b wrote row entries lrc[st][b] itself.
template <int SPT, int NT>
__device__ __forceinline__ void flush_run_counts(const uint32_t* lrc, const uint16_t* lro, int B, int st_last, int64_t t,
                                                 int64_t nSt, uint32_t* __restrict__ rcnt, uint16_t* __restrict__ roff) {
  static_assert(SPT % 8 == 0, "whole 16-byte stores");
  for (int b = threadIdx.x; b < B; b += NT) {
    uint32_t* rc = rcnt + (int64_t)b * nSt + t * SPT;
    uint16_t* ro = roff + (int64_t)b * nSt + t * SPT;
#pragma unroll
    for (int q = 0; q < SPT / 4; q++) {
      uint32_t v[4];
#pragma unroll
      for (int k = 0; k < 4; k++) v[k] = 4 * q + k <= st_last ? lrc[(4 * q + k) * B + b] : 0u;
      *(uint4*)(rc + 4 * q) = make_uint4(v[0], v[1], v[2], v[3]);
    }
#pragma unroll
    for (int q = 0; q < SPT / 8; q++) {
      uint32_t w[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int s0 = 8 * q + 2 * k;
        const uint32_t lo = s0 <= st_last ? lro[s0 * B + b] : 0u, hi = s0 + 1 <= st_last ? lro[(s0 + 1) * B + b] : 0u;
        w[k] = lo | hi << 16;
      }
      *(uint4*)(ro + 8 * q) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

// The time base, the key base and the tile's key range — shared by both scatters.  T0: the stream
// time before the push, else the first ts (k_c1_check's 31-bit ts test is relative to it).  kb:
// the host's base (the last push's key minimum less a margin), else keys[0] − half the key field;
// the records hold (key − kb), and k_c1_check rebases them to the push's key minimum (CI_KSHIFT)
// or declines when some key falls outside the field.
__device__ __forceinline__ void run_bases(const int64_t* __restrict__ keys, const int64_t* __restrict__ ts, int64_t n,
                                          const int64_t* __restrict__ stream_time, int64_t kb_in, int has_kb,
                                          int kfield, int64_t* ci, int64_t* T0, int64_t* kb) {
  const int64_t st0 = *stream_time;
  const int64_t t0 = n > 0 ? ts[0] : 0;
  *T0 = st0 >= 0 ? st0 : (t0 > 0 ? t0 : 0);
  *kb = has_kb ? kb_in : (int64_t)((uint64_t)keys[0] - (1ULL << (kfield - 1)));
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ci[CI_T0] = *T0;
    ci[CI_KBASE] = *kb;
  }
}

// The workgroup's key range → CI_KMIN / CI_KMAX atomics (kb + the staged offsets' extremes), and
// CI_KFAIL when some key fell outside the record's key field above kb (thread 0, after the loop).
__device__ __forceinline__ void run_krange(const uint32_t* lkr, int kfail, int64_t kb, int64_t* ci) {
  if (lkr[1] >= lkr[0]) {
    atomicMin((long long*)&ci[CI_KMIN], (long long)((uint64_t)kb + lkr[0]));
    atomicMax((long long*)&ci[CI_KMAX], (long long)((uint64_t)kb + lkr[1]));
  }
  if (kfail) atomicOr((unsigned long long*)&ci[CI_KFAIL], 1ULL);
}

// ------------------------------------------------------------------ k_c1_scatter
// Records of tile t → step runs.  8-byte record: (key - kb) << 32 | (uint32)(ts - T0); invalid
// records keep their key word (their bucket is the key's) with the sentinel low word.
// WIDE (the key range does not fit 32 bits): the record is the 64-bit key hash (key = its inverse)
// and ts - T0 goes to a parallel u32 array (srecT), staged beside it.
template <int U, int NT, bool WIDE, bool ST>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void k_c1_scatter(
    const int64_t* __restrict__ keys, const int64_t* __restrict__ ts, const uint8_t* __restrict__ kv,
    const uint8_t* __restrict__ rv, int64_t n, int64_t nT, int log2B, uint32_t* __restrict__ rcnt,
    uint16_t* __restrict__ roff, int64_t nSt, uint64_t* __restrict__ srec, int64_t* __restrict__ tilestat,
    int64_t* __restrict__ tpart, int64_t* __restrict__ ci, const int64_t* __restrict__ st_at,
    uint32_t* __restrict__ srecT, int64_t size, int64_t adv, FastDiv fd, int64_t grace,
    const int64_t* __restrict__ stream_time, int64_t kb_in, int has_kb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int wsum[NT / 64];
  __shared__ unsigned long long lc[4];
  __shared__ int lt[2][2];  // [step parity][max | min] of the step's accepted ts - T0 (LDS atomics)
  __shared__ int lfail, lkfail;
  __shared__ uint32_t lkr[2];  // min / max of the staged key offsets (not WIDE)
  constexpr int S = U * NT;
  constexpr int SPT = C1_TILE / S;
  const int B = 1 << log2B;
  const int64_t t = tile_of(blockIdx.x, nT);
  uint32_t* cnt = (uint32_t*)smem;
  uint32_t* sbase = cnt + B;
  int64_t* sp = (int64_t*)(smem + (size_t)B * 8);
  uint32_t* lt32 = (uint32_t*)(sp + S);  // WIDE: the staged ts - T0
  uint32_t* lrc = (uint32_t*)(smem + run_stage_lds(B, S, 8, WIDE));
  uint16_t* lro = (uint16_t*)(lrc + SPT * B);
  for (int b = threadIdx.x; b < B; b += NT) cnt[b] = 0u;
  if (threadIdx.x < 4) lc[threadIdx.x] = 0;
  if (threadIdx.x < 2) {
    lt[threadIdx.x][0] = INT32_MIN;
    lt[threadIdx.x][1] = INT32_MAX;
  }
  if (threadIdx.x == 0) {
    lfail = lkfail = 0;
    lkr[0] = 0xFFFFFFFFu;
    lkr[1] = 0u;
  }
  int64_t T0, kb;
  run_bases(keys, ts, n, stream_time, kb_in, has_kb, 32, ci, &T0, &kb);
  const int shift = log2B == 0 ? 64 : 64 - log2B;
  const uint32_t bmask = (uint32_t)(B - 1);
  const int64_t base = t * C1_TILE;
  const int64_t end = base + C1_TILE < n ? base + C1_TILE : n;
  int c_acc = 0, c_nk = 0, c_nr = 0, c_bt = 0;  // < 2^16 per tile
  uint32_t kor = 0u;
  int64_t x[U], k[U];
  auto load_step = [&](int64_t i0, int64_t (&dx)[U], int64_t (&dk)[U]) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      int64_t i = i0 + (int64_t)u * NT;
      i = i < end ? i : end - 1;
      dx[u] = ts[i];
      dk[u] = keys[i];
    }
  };
  // Thread 0 folds each step's accepted-ts range (LDS slots lt[st & 1], reset for step st + 2)
  // into the tile's late-record summary for k_c1_check: the stream-time maximum, the smallest ts,
  // the largest stream time every step stays below (bound: the step's earliest window still
  // open, S/StreamAggregateBuilder.java:272-277) and whether the tile's own running maximum
  // already passes a step's bound.  The check then needs only the stream time carried INTO the
  // tile: carry <= bound (and ok) <=> no record of the tile is late.
  int64_t t_rmax = -1, t_min = INT64_MAX, t_bound = INT64_MAX;
  bool t_ok = true;
  auto publish = [&](int64_t, int st) {
    const int mx = lt[st & 1][0], mn = lt[st & 1][1];
    if (mx != INT32_MIN) {
      const int64_t smx = T0 + mx, smn = T0 + mn;
      t_rmax = smx > t_rmax ? smx : t_rmax;
      t_min = smn < t_min ? smn : t_min;
      const int64_t fw = first_window_start_fd(smn, size, adv, fd) + size;
      const int64_t b = grace > ((int64_t)1 << 61) ? INT64_MAX : fw + grace - 1;
      t_bound = b < t_bound ? b : t_bound;
      t_ok = t_ok && t_rmax <= b;
    }
    lt[st & 1][0] = INT32_MIN;
    lt[st & 1][1] = INT32_MAX;
  };
  lds_barrier();
  int64_t s0 = base;
  int st_last = -1;
  if (s0 < end) load_step(s0 + threadIdx.x, x, k);
  for (int st = 0; s0 < end; s0 += S, st++) {  // uniform across the block: barriers inside
    st_last = st;
    const int64_t i0 = s0 + threadIdx.x;
    bool ok[U];
    uint32_t bin[U], t32[U];
    int64_t rec[U];
    // this step's accepted ts range, relative to T0 (k_c1_check's late test): 32-bit, every
    // accepted ts - T0 and stream time - T0 fits (else tfail declines the push)
    int tmx = INT32_MIN, tmn = INT32_MAX;
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t i = i0 + (int64_t)u * NT;
      ok[u] = i < end;
      const bool kok = bit_get(kv, ok[u] ? i : base), rok = bit_get(rv, ok[u] ? i : base);
      const bool valid = ok[u] && kok && rok && x[u] >= 0;
      c_nk += ok[u] && !kok;
      c_nr += ok[u] && kok && !rok;
      c_bt += ok[u] && kok && rok && x[u] < 0;
      c_acc += valid;
      const int64_t sx = ST ? st_at[ok[u] ? i : base] : x[u];  // ABI 5 domains: the given stream time
      const int64_t d = x[u] - T0;
      if (valid && (d <= (int64_t)INT32_MIN || d > (int64_t)INT32_MAX)) {  // rare: an LDS flag, not a loop-carried mask
        lfail = 1;
#ifdef KHIP_TUNING
        if (ci[CI_N - 1] == 1 && (threadIdx.x & 63) == 0) printf("[c1 scatter] t %ld i %ld x %ld T0 %ld\n", (long)t, (long)i, (long)x[u], (long)T0);
#endif
      }
      if constexpr (ST) {
        const int64_t ds = sx - T0;
        if (valid && (ds <= (int64_t)INT32_MIN || ds > (int64_t)INT32_MAX)) lfail = 1;
        tmx = valid && (int)ds > tmx ? (int)ds : tmx;
      } else {
        tmx = valid && (int)d > tmx ? (int)d : tmx;
      }
      tmn = valid && (int)d < tmn ? (int)d : tmn;
      const uint64_t hk = key_hash(k[u]);
      bin[u] = stage_bin(hk, shift, bmask);
      t32[u] = valid ? (uint32_t)d : C1_SENT;
      const uint64_t kd = (uint64_t)k[u] - (uint64_t)kb;
      if (!WIDE) kor |= ok[u] ? (uint32_t)(kd >> 32) : 0u;  // nonzero: a key outside the field above kb
      rec[u] = WIDE ? (int64_t)hk : (int64_t)((kd << 32) | (uint64_t)t32[u]);
    }
    // the next step's loads go into x / k (dead now) and stay in flight through this step's stage
    if (s0 + S < end) load_step(i0 + S, x, k);
    const uint32_t tot = stage_step_runs<U, NT, int64_t, WIDE>(rec, t32, bin, ok, B, cnt, sbase, wsum, sp, lt32,
                                                               (int64_t*)srec, srecT, t * SPT + st, lrc + st * B,
                                                               lro + st * B);
    if (!WIDE) step_krange<NT, int64_t>(sp, tot, 0xFFFFFFFFu, lkr);
    // the step's ts range: the wave's first (one LDS atomic per wave, not 64 to one address),
    // after the stage so that its registers are free; published by thread 0 one step later
    // (after the next stage's barriers), the last step's after the loop
    for (int off = 32; off > 0; off >>= 1) {
      const int a = __shfl_xor(tmx, off, 64), b = __shfl_xor(tmn, off, 64);
      tmx = a > tmx ? a : tmx;
      tmn = b < tmn ? b : tmn;
    }
    if ((threadIdx.x & 63) == 0 && tmx != INT32_MIN) {
      atomicMax(&lt[st & 1][0], tmx);
      atomicMin(&lt[st & 1][1], tmn);
    }
    if (threadIdx.x == 0 && st > 0) publish(s0 - S, st - 1);
  }
  flush_run_counts<SPT, NT>(lrc, lro, B, st_last, t, nSt, rcnt, roff);
  if (!WIDE && kor) lkfail = 1;
  __syncthreads();
  if (threadIdx.x == 0 && s0 > base) publish(s0 - S, st_last);
  if (!WIDE && threadIdx.x == 0) run_krange(lkr, lkfail, kb, ci);
  c_acc = wave_sum(c_acc);
  c_nk = wave_sum(c_nk);
  c_nr = wave_sum(c_nr);
  c_bt = wave_sum(c_bt);
  if ((threadIdx.x & 63) == 0) {
    if (c_acc) atomicAdd(&lc[0], (unsigned long long)c_acc);
    if (c_nk) atomicAdd(&lc[1], (unsigned long long)c_nk);
    if (c_nr) atomicAdd(&lc[2], (unsigned long long)c_nr);
    if (c_bt) atomicAdd(&lc[3], (unsigned long long)c_bt);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t* tp = tpart + t * T_NPART;
    tp[T_ACCEPTED] = (int64_t)lc[0];
    tp[T_NULL_KEY] = (int64_t)lc[1];
    tp[T_NULL_ROW] = (int64_t)lc[2];
    tp[T_BAD_TS] = (int64_t)lc[3];
    tp[T_APPLIED] = (int64_t)lc[0];  // TUMBLING: one window per accepted record, none late (checked)
    tp[T_LATE] = 0;
    if (lfail) atomicOr((unsigned long long*)&ci[CI_TFAIL], 1ULL);
    int64_t* ts4 = tilestat + t * 4;
    ts4[0] = t_rmax;
    ts4[1] = t_min;
    ts4[2] = t_bound;
    ts4[3] = t_ok ? 1 : 0;
  }
}

// The exact key range of a push (the host's fallback when a key fell outside the key field; keys
// every `stride` words):
// out[0] = max of ~key (= ~min), out[1] = max of key (both start at INT64_MIN).
__global__ __launch_bounds__(256) void k_c1_krange(const int64_t* __restrict__ keys, int64_t stride, int64_t n,
                                                   long long* __restrict__ out) {
  int64_t mx = INT64_MIN, mxn = INT64_MIN;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = keys[i * stride];
    mx = k > mx ? k : mx;
    mxn = ~k > mxn ? ~k : mxn;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const int64_t a = __shfl_xor(mx, off, 64), b = __shfl_xor(mxn, off, 64);
    mx = a > mx ? a : mx;
    mxn = b > mxn ? b : mxn;
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&out[0], (long long)mxn);
    atomicMax(&out[1], (long long)mx);
  }
}

// Bucket bases from the scanned run counts: bb[b] = rpos[b][0], bb[B] = the total.
__global__ __launch_bounds__(256) void k_c1_bases(const uint32_t* __restrict__ rpos, int64_t nSt, int B,
                                                  int64_t* __restrict__ bb) {
  for (int b = threadIdx.x; b <= B; b += blockDim.x) bb[b] = (int64_t)rpos[(int64_t)b * nSt];
}

// Refine work item w → its bucket (cstart), its first step s0 and run count R (cinfo[2w],
// [2w + 1]): one thread per item, binary searches over cstart and the bucket's scanned run
// positions — so a refine workgroup starts with one round of table loads, not the searches.
__global__ __launch_bounds__(256) void k_c1_chunks(const int* __restrict__ cstart, int B, const int64_t* __restrict__ bb,
                                                   const uint32_t* __restrict__ rpos, int64_t nSt, int ch,
                                                   const int64_t* __restrict__ ci, uint32_t* __restrict__ cinfo) {
  if (ci_ld(ci, CI_GATE) == 0) return;
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= (int)ci_ld(ci, CI_NCHUNK)) return;
  int a = 0, e = B;  // the last bucket with cstart[b] <= w, in [a, e)
  while (e - a > 1) {
    const int m = (a + e) >> 1;
    if (cstart[m] <= w) a = m;
    else e = m;
  }
  const int b = a;
  const int64_t lo = bb[b] + (int64_t)(w - cstart[b]) * ch;
  const int64_t len = bb[b + 1] - lo < ch ? bb[b + 1] - lo : ch;
  const uint32_t* rp = rpos + (int64_t)b * nSt;
  int64_t sa = 0, se = nSt;  // s0: the last step whose run starts at or before lo
  while (se - sa > 1) {
    const int64_t m = (sa + se) >> 1;
    if ((int64_t)rp[m] <= lo) sa = m;
    else se = m;
  }
  int64_t ta = sa, te = nSt;  // the first step after s0 whose run starts at or past lo + len (or nSt)
  while (te - ta > 1) {
    const int64_t m = (ta + te) >> 1;
    if ((int64_t)rp[m] < lo + len) ta = m;
    else te = m;
  }
  cinfo[2 * w] = (uint32_t)sa;
  cinfo[2 * w + 1] = (uint32_t)(te - sa);
}

// The chunk's source positions: map[j] = where the chunk's record j lies in the step runs (u32 per
// record, in the refine's not yet used stage).  One thread per run of the chunk (cinfo): one round
// of loads of its position / end / step offset, then the run's slice of the map.
__device__ __forceinline__ void chunk_map(const uint32_t* __restrict__ rp, const uint16_t* __restrict__ ro,
                                          const uint32_t* __restrict__ cinfo, int w, int64_t S, int64_t lo, int len,
                                          uint32_t* map) {
  const int64_t s0 = cinfo[2 * w];
  const int R = (int)cinfo[2 * w + 1];
  for (int k = threadIdx.x; k < R; k += blockDim.x) {
    const int64_t s = s0 + k, p = (int64_t)rp[s], pe = (int64_t)rp[s + 1];  // rp[nSt] = the next bucket's start
    const int64_t a = p > lo ? p : lo, e = pe < lo + len ? pe : lo + len;
    const uint32_t src = (uint32_t)(s * S + (int64_t)ro[s] + (a - p));
    for (int64_t x = a; x < e; x++) map[x - lo] = src + (uint32_t)(x - a);
  }
  __syncthreads();
}

// ------------------------------------------------------------------ k_c1_check
// One workgroup.  Accept the push when no scatter step (4096 consecutive records) can hold a late
// record: the step's earliest window outlives the largest stream time the step reaches,
// max(stream time before the step, the step's max ts) - grace (the general path's per-tile `fast`
// test at step granularity; S/StreamAggregateBuilder.java:272-277 for the grace).
// Accepted: publish the stream time, the window range (k_part_wrange's rules, resident rows
// included), the identity width and the refine's chunk list (cstart); reset the counters the
// merge and commit use.  Declined: nothing persistent is touched.
__global__ __launch_bounds__(1024) void k_c1_check(
    const int64_t* __restrict__ tilestat, int64_t nT, int64_t size, int64_t adv, FastDiv fd, int64_t grace,
    int64_t close0, int fresh, int log2B, int log2P, int wide, int ch, int kbmax, int pbits,
    const int64_t* __restrict__ bb, int* __restrict__ cstart,
    int64_t* __restrict__ ci, int64_t* __restrict__ stream_time, int64_t* __restrict__ res,
    unsigned long long* __restrict__ ctr, unsigned long long* __restrict__ closed_ctr, unsigned long long closed_n) {
  __shared__ int64_t wmx[16];
  __shared__ int64_t red[4][16];
  __shared__ int lslow;
  __shared__ int lnch[512 + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) lslow = 0;
  const int64_t st0 = *stream_time;
  // thread j owns tiles [j K, (j + 1) K): their stream-time maximum, the block's exclusive prefix
  // of those (the stream time carried into each tile), then each tile's summary (k_c1_scatter)
  const int64_t K = (nT + 1023) / 1024;
  const int64_t g0 = threadIdx.x * K, g1 = g0 + K < nT ? g0 + K : nT;
  int64_t m = -1;
  for (int64_t g = g0; g < g1; g++) m = tilestat[4 * g] > m ? tilestat[4 * g] : m;
  const int64_t incl = wave_incl_max(m);
  if (lane == 63) wmx[wave] = incl;
  __syncthreads();
  int64_t pre = st0;
  for (int w = 0; w < wave; w++) pre = wmx[w] > pre ? wmx[w] : pre;
  const int64_t excl = __shfl_up(incl, 1, 64);
  int64_t run = lane == 0 ? pre : (excl > pre ? excl : pre);  // stream time before tile g0
  int64_t gmn = INT64_MAX, gmx = -1;
  bool slow = false;
  for (int64_t g = g0; g < g1; g++) {
    const int64_t* t4 = tilestat + 4 * g;
    const int64_t mx = t4[0], mn = t4[1];
    if (mn != INT64_MAX) {
      slow |= t4[3] == 0 || run > t4[2];  // a record of the tile may be late
      gmn = mn < gmn ? mn : gmn;
    }
    run = mx > run ? mx : run;
    gmx = mx > gmx ? mx : gmx;
  }
  if (slow) lslow = 1;
  for (int off = 32; off > 0; off >>= 1) {
    const int64_t a = __shfl_xor(gmn, off, 64), b = __shfl_xor(gmx, off, 64);
    gmn = a < gmn ? a : gmn;
    gmx = b > gmx ? b : gmx;
  }
  if (lane == 0) {
    red[0][wave] = gmn;
    red[1][wave] = gmx;
  }
  // chunks per bucket → cstart (exclusive prefix), largest bucket's chunk count
  const int B = 1 << log2B;
  for (int b = threadIdx.x; b < B; b += 1024) lnch[b] = (int)((bb[b + 1] - bb[b] + ch - 1) / ch);
  __syncthreads();
  if (threadIdx.x) return;
  for (int w = 0; w < 16; w++) {
    gmn = red[0][w] < gmn ? red[0][w] : gmn;
    gmx = red[1][w] > gmx ? red[1][w] : gmx;
  }
  int acc = 0, mxc = 0;
  for (int b = 0; b < B; b++) {
    cstart[b] = acc;
    acc += lnch[b];
    mxc = lnch[b] > mxc ? lnch[b] : mxc;
  }
  cstart[B] = acc;
  const int64_t kmin = ci_ld(ci, CI_KMIN), kmax = ci_ld(ci, CI_KMAX);
  const bool tfail = ci_ld(ci, CI_TFAIL) != 0, kfail = ci_ld(ci, CI_KFAIL) != 0;
  ci[CI_KMIN] = INT64_MAX;  // ready for the next push's atomics
  ci[CI_KMAX] = INT64_MIN;
  ci[CI_TFAIL] = 0;
  ci[CI_KFAIL] = 0;
  // (wide records: the scatter tracks no key range)
  bool ok = !lslow && !tfail && mxc <= C1_SEGMAX && (wide || kmax >= kmin);
#ifdef KHIP_TUNING
  if (ci[CI_N - 1] == 1)  // debug (tuning build, KHIP_C1_DEBUG=1): the decision's inputs
    printf("[c1 check] tfail %d slow %d mxc %d kmin %ld kmax %ld gmn %ld gmx %ld T0 %ld st0 %ld nT %ld\n", (int)tfail,
           (int)lslow, mxc, (long)kmin, (long)kmax, (long)gmn, (long)gmx, (long)ci[CI_T0], (long)st0, (long)nT);
#endif
  // compact records: every key within the key field above the push's base kb (the scatters wrote
  // key - kb; kfail: some key was not — the host then learns the true range and re-runs the push
  // with kb = kmin, or with wide records), and the range within 32 key bits (value records 31)
  const uint64_t krange = kmax >= kmin ? (uint64_t)kmax - (uint64_t)kmin : 0;
  const bool fits = !wide && !kfail && krange < ((1ULL << kbmax) - 1);
  const int64_t kb = ci_ld(ci, CI_KBASE);
  ci[CI_FITS] = fits ? 1 : 0;
  ci[CI_REASON] = ok && !wide && kfail ? 2 : (ok && !wide && !fits ? 1 : 0);
  ci[CI_KMINC] = kmin;
  ci[CI_KSHIFT] = (int64_t)((uint64_t)kmin - (uint64_t)kb);
  ok = ok && (wide || fits);
  // window range of this push's records and of the live resident rows (k_part_wrange)
  int64_t lo = INT64_MAX, hi = INT64_MIN;
  if (gmx >= 0) {
    const int64_t l = gmn - size + adv;
    lo = (int64_t)fast_udiv((uint64_t)(l > 0 ? l : 0), fd);
    hi = (int64_t)fast_udiv((uint64_t)gmx, fd);
  }
  if (!fresh) {
    int64_t rlo = res[0];
    const int64_t rhi = res[1];
    if (close0 != INT64_MIN && rlo != INT64_MAX) {  // live: ws > close0 - size
      const int64_t c = close0 - size;
      const int64_t lb = c >= 0 ? (int64_t)fast_udiv((uint64_t)c, fd) + 1 : 0;
      rlo = rlo > lb ? rlo : lb;
    }
    lo = rlo < lo ? rlo : lo;
    hi = rhi > hi ? rhi : hi;
  }
  const bool none = lo > hi;  // nothing live, nothing new
  if (none) lo = hi = 0;
  ok = ok && (uint64_t)(hi - lo) < (wide ? ((uint64_t)1 << log2P) - 1 : (pbits ? 0x7FFFFFFEull : 0xFFFFFFFEull));
  const int wbits = bits_of((uint64_t)(hi - lo)), kbits = bits_of(krange);
  ci[CI_GATE] = ok ? 1 : 0;
  if (!ok) return;
  ci[CI_WBASE] = lo;
  ci[CI_WHI] = hi - lo;
  ci[CI_WBITS] = wbits;
  ci[CI_KBITS] = kbits;
  ci[CI_KRANGE] = (int64_t)krange;
  ci[CI_ID32] = !wide && kbits + wbits + pbits <= 31 ? 1 : 0;  // pbits: the pane flag
  ci[CI_WIDE] = wide;
  ci[CI_TMIN] = gmx >= 0 ? gmn : 0;
  ci[CI_TMAX] = gmx;
  ci[CI_NCHUNK] = acc;
  *stream_time = gmx > st0 ? gmx : st0;
  res[0] = none ? INT64_MAX : lo;
  res[1] = none ? INT64_MIN : hi;
  ctr[0] = ctr[1] = ctr[2] = 0ULL;
  if (closed_ctr) *closed_ctr = closed_n;
}

// ------------------------------------------------------------------ k_c1_refine
// Work item w = chunk c of bucket b (cstart): its records are counting-sorted by partition
// inside the bucket (F = 2^fbits bins) in LDS and written back to the same positions of the
// output; seg[w][f] (u16) = partition f's first record in the chunk, seg[w][F] = valid records.
// WIDE: records are key hashes (srcA / srec) with ts - T0 in parallel u32 arrays (srcAT / srecT);
// the two are staged one after the other through the same LDS.
template <int U, int NT, bool WIDE>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void k_c1_refine(
    const uint64_t* __restrict__ srcA, const int64_t* __restrict__ bb, const int* __restrict__ cstart, int log2B,
    int log2P, int fbits, uint64_t* __restrict__ srec, uint16_t* __restrict__ seg, const int64_t* __restrict__ ci,
    const uint32_t* __restrict__ srcAT, uint32_t* __restrict__ srecT, const uint32_t* __restrict__ rpos,
    const uint16_t* __restrict__ roff, int64_t nSt, int64_t S, const uint32_t* __restrict__ cinfo) {
  if (ci_ld(ci, CI_GATE) == 0) return;
  const int w = blockIdx.x;
  if (w >= (int)ci_ld(ci, CI_NCHUNK)) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int lb, lnv;
  __shared__ int wsum[NT / 64];
  static_assert(U * NT == C1_CH, "refine chunk");
  const int F = 1 << fbits, B = 1 << log2B;
  uint32_t* cnt = (uint32_t*)smem;
  uint32_t* sbase = cnt + F;
  uint64_t* stage = (uint64_t*)(smem + (size_t)F * 8);
  for (int f = threadIdx.x; f < F; f += NT) cnt[f] = 0u;
  if (threadIdx.x == 0) lb = -1;
  __syncthreads();
  for (int b = threadIdx.x; b < B; b += NT)
    if (cstart[b] <= w && w < cstart[b + 1]) lb = b;
  __syncthreads();
  const int b = lb;
  if (b < 0) return;  // (cannot happen: w < cstart[B])
  const int64_t lo = bb[b] + (int64_t)(w - cstart[b]) * C1_CH;
  const int64_t bend = bb[b + 1];
  const int len = (int)(bend - lo < C1_CH ? bend - lo : C1_CH);
  const int64_t kmin = ci_ld(ci, CI_KMINC);
  const uint64_t kshift = WIDE ? 0 : (uint64_t)ci_ld(ci, CI_KSHIFT) << 32;  // records hold key - kb
  const int shift = 64 - log2P;
  // where the chunk's records lie in the step runs (a map in the not yet used stage)
  const uint32_t* rp = rpos + (int64_t)b * nSt;
  const uint16_t* ro = roff + (int64_t)b * nSt;
  chunk_map(rp, ro, cinfo, w, S, lo, len, (uint32_t*)stage);
  uint64_t r[U];
  uint32_t f[U], rank[U], t32[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int j = threadIdx.x + u * NT;
    const uint32_t src = ((const uint32_t*)stage)[j < len ? j : len - 1];
    r[u] = c1_ld(srcA + src) - kshift;
    if constexpr (WIDE) t32[u] = c1_ld(srcAT + src);
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int j = threadIdx.x + u * NT;
    const bool v = j < len && (WIDE ? t32[u] : (uint32_t)r[u]) != C1_SENT;
    f[u] = WIDE ? (uint32_t)(r[u] >> shift) & (uint32_t)(F - 1)
                : (uint32_t)(key_hash(kmin + (int64_t)(r[u] >> 32)) >> shift) & (uint32_t)(F - 1);
    rank[u] = v ? atomicAdd(&cnt[f[u]], 1u) : 0xFFFFFFFFu;
  }
  __syncthreads();
  // exclusive scan of the F counts (F <= NT)
  {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t c = t < F ? cnt[t] : 0u;
    uint32_t incl = c;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(incl, off, 64);
      if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wave] = (int)incl;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; k++) {
      before += k < wave ? (uint32_t)wsum[k] : 0u;
      tot += (uint32_t)wsum[k];
    }
    if (t < F) {
      sbase[t] = before + incl - c;
      seg[(int64_t)w * (F + 1) + t] = (uint16_t)(before + incl - c);
    }
    if (t == 0) {
      seg[(int64_t)w * (F + 1) + F] = (uint16_t)tot;
      lnv = (int)tot;
    }
  }
  __syncthreads();
  const int nv = lnv;
#pragma unroll
  for (int u = 0; u < U; u++)
    if (rank[u] != 0xFFFFFFFFu) stage[sbase[f[u]] + rank[u]] = r[u];
  __syncthreads();
  for (int j = threadIdx.x; j < nv; j += NT) srec[lo + j] = stage[j];
  if constexpr (WIDE) {  // the ts words through the same LDS
    __syncthreads();
    uint32_t* stage32 = (uint32_t*)stage;
#pragma unroll
    for (int u = 0; u < U; u++)
      if (rank[u] != 0xFFFFFFFFu) stage32[sbase[f[u]] + rank[u]] = t32[u];
    __syncthreads();
    for (int j = threadIdx.x; j < nv; j += NT) srecT[lo + j] = stage32[j];
  }
}

// KHIP_AGG_PROBE (tuning build): wall-clock time per merge phase summed over the persistent
// workgroups (thread 0's view): 0 item start + eviction, 1 records, 2 pane fold, 3 mark + count
// + reserve, 4 write-out.  dbg == nullptr in every other run.
#ifdef KHIP_TUNING
#define C1M_T(k)                                                                        \
  do {                                                                                  \
    if (dbg && threadIdx.x == 0) {                                                      \
      const unsigned long long now_ = wall_clock64();                                   \
      atomicAdd(&dbg[(k)], now_ - t_last);                                              \
      t_last = now_;                                                                    \
    }                                                                                   \
  } while (0)
#define C1M_T0 unsigned long long t_last = dbg ? wall_clock64() : 0ULL
#else  // the release build carries no probe (its registers would cost the merge)
#define C1M_T(k) \
  do {           \
  } while (0)
#define C1M_T0 (void)dbg
#endif

// ------------------------------------------------------------------ k_c1_merge
struct C1Q {
  int32_t log2P, fbits, log2H, sw, hv_active, hv_op, hmax;
  int64_t size, adv, cmax, hv_i64;
  FastDiv fd;
  FastDiv32 fd32;
  uint8_t* chg;  // changelog: per-row-slot emission flags (CHG_*), or null
};

__device__ __forceinline__ bool c1q_having(const C1Q& q, uint64_t c) {
  const int64_t v = (int64_t)c;
  switch (q.hv_op) {
    case KHIP_OP_GT: return v > q.hv_i64;
    case KHIP_OP_GE: return v >= q.hv_i64;
    case KHIP_OP_LT: return v < q.hv_i64;
    case KHIP_OP_LE: return v <= q.hv_i64;
    case KHIP_OP_EQ: return v == q.hv_i64;
    case KHIP_OP_NE: return v != q.hv_i64;
  }
  return true;
}

// identity → 32-bit hash (slot = its top log2H bits; sub-pass = bits of a remix)
template <class ID>
__device__ __forceinline__ uint32_t c1_hash(ID id) {
  if constexpr (sizeof(ID) == 4) return (uint32_t)id * 0x9E3779B1u;
  else return ((uint32_t)id * 0x9E3779B1u) ^ ((uint32_t)(id >> 32) * 0x85EBCA77u);
}
__device__ __forceinline__ uint32_t c1_sub(uint32_t h, int sbits) {
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  return (h >> 12) & ((1u << sbits) - 1u);
}

template <class ID>
__device__ __forceinline__ int c1_find_id(const KLDS ID* ids, ID id, uint32_t e, int H) {
  for (int probe = 0; probe < H; probe++) {
    const ID v = ids[e];
    if (v == id) return (int)e;
    if (v == (ID)~(ID)0) return -1;
    e = (e + 1) & (uint32_t)(H - 1);
  }
  return -1;
}

// Work item: p (work == nullptr: item w is partition w) or work[w] = p | sbits << 16 | sub << 20
// (a retry with 2^sbits sub-passes).  LDS: ids ID[H + 64] | rt u32[H + 64] | ct u32[H + 64] |
// list u16[H] | segment prefix u32[SEGMAX + 1] | segment bases i32[SEGMAX] (n < 2^31).
template <int NT, int AU, class ID, bool WIDE>
__global__ __launch_bounds__(NT, 4) void k_c1_merge(
    C1Q q, const uint32_t* __restrict__ work, int64_t nwork, const int64_t* __restrict__ bb,
    const int* __restrict__ cstart, const uint16_t* __restrict__ seg, const uint64_t* __restrict__ srec, int first,
    uint64_t* __restrict__ buf0, uint64_t* __restrict__ buf1, const uint8_t* __restrict__ sel,
    const int64_t* __restrict__ cnt, unsigned long long* __restrict__ newcnt, uint8_t* __restrict__ fail,
    unsigned long long* __restrict__ need, int64_t close0, uint64_t* __restrict__ closed,
    unsigned long long* __restrict__ closed_n, const int64_t* __restrict__ ci, unsigned long long* __restrict__ hnew,
    unsigned long long* __restrict__ hclosed, uint32_t* __restrict__ prn, const uint32_t* __restrict__ srecT,
    unsigned long long* __restrict__ dbg) {
  if (ci_ld(ci, CI_GATE) == 0) return;
  if ((ci_ld(ci, CI_WIDE) != 0) != WIDE) return;                            // the other record format's
  if (!WIDE && (ci_ld(ci, CI_ID32) != 0) != (sizeof(ID) == 4)) return;     // the other identity width's
  static_assert(!WIDE || sizeof(ID) == 8, "wide records use 64-bit identities");
  constexpr int NW = NT / 64;
  constexpr ID EMPTY = (ID)~(ID)0;
  const int log2H = q.log2H;
  const int H = 1 << log2H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  KLDS ID* ids = (KLDS ID*)(KLDS char*)smem;
  KLDS uint32_t* rt = (KLDS uint32_t*)((KLDS char*)smem + (size_t)(H + 64) * sizeof(ID));
  KLDS uint32_t* ct = rt + (H + 64);
  KLDS uint16_t* list = (KLDS uint16_t*)(ct + (H + 64));
  // segment k: prefix of the lengths | (base - prefix) << 32, so a lookup reads k and k + 1 at once
  KLDS uint64_t* sg2 = (KLDS uint64_t*)((KLDS char*)list + (((size_t)H * 2 + 15) & ~(size_t)15));
  KLDS int64_t* lbb = (KLDS int64_t*)(sg2 + C1_SEGMAX + 4);  // [B + 1] bucket bases
  KLDS int32_t* lcs = (KLDS int32_t*)(lbb + (1 << (q.log2P - q.fbits)) + 1);  // [B + 1] chunk starts
  KLDS uint16_t* segof = (KLDS uint16_t*)(lcs + (1 << (q.log2P - q.fbits)) + 2);  // [C1_SEGOF] block → segment
  __shared__ int lovf, nnew;
  __shared__ int wsum[NW], csum[NW];
  __shared__ unsigned long long lbase, cbase;
  const int F = 1 << q.fbits;
  const int64_t wbase = ci_ld(ci, CI_WBASE), whi = ci_ld(ci, CI_WHI), T0 = ci_ld(ci, CI_T0), tmin = ci_ld(ci, CI_TMIN);
  const int wbits = (int)ci_ld(ci, CI_WBITS);
  const int64_t kmin = ci_ld(ci, CI_KMINC);
  const uint64_t krange = (uint64_t)ci_ld(ci, CI_KRANGE);
  const int32_t tmin32 = (int32_t)(tmin - T0);
  const int64_t wstart = wbase * q.adv;  // the first window's start: every record ts >= it
  const bool r32 = ci_ld(ci, CI_TMAX) - wstart < ((int64_t)1 << 32);
  const uint32_t tsh32 = (uint32_t)(T0 - wstart);  // ts - wstart = (uint32) t32 + tsh32
  const bool evict = close0 != INT64_MIN;
  C1M_T0;
  const uint32_t dummy = (uint32_t)H + (uint32_t)lane;
  for (int i = threadIdx.x; i < H + 64; i += NT) {
    ids[i] = EMPTY;
    rt[i] = 0u;
    ct[i] = 0u;
  }
  if (threadIdx.x == 0) {
    lovf = 0;
    nnew = 0;
  }
  // identity of a resident row (false: no record of this push can match it) and its sub-pass hash
  auto row_id = [&](const uint64_t* row, ID* id, uint32_t* h) -> bool {
    const int64_t wi = (int64_t)fast_udiv((uint64_t)row[1], q.fd) - wbase;
    if constexpr (WIDE) {  // (key hash without its partition bits) << log2P | window
      if (wi < 0 || wi > whi) {
        *h = (uint32_t)(key_hash((int64_t)row[0]) >> 32) ^ (uint32_t)row[1];
        return false;
      }
      *id = (ID)((key_hash((int64_t)row[0]) << q.log2P) | (uint64_t)wi);
      *h = c1_hash<ID>(*id);
      return true;
    }
    const uint64_t krel = (uint64_t)((int64_t)row[0] - kmin);
    if (krel > krange || wi < 0 || wi > whi) {
      *h = (uint32_t)(key_hash((int64_t)row[0]) >> 32) ^ (uint32_t)row[1];
      return false;
    }
    if constexpr (sizeof(ID) == 4) *id = (ID)(((uint32_t)krel << wbits) | (uint32_t)wi);
    else *id = (ID)((krel << 32) | (uint64_t)wi);
    *h = c1_hash<ID>(*id);
    return true;
  };
  // item w's descriptor, and its segments in LDS (prefix of their lengths, each one's base:
  // record li = srec[sbs[s] + li]).  fetch issues the global loads only (the raw words stay in
  // registers, nothing waits on them): it runs for item w + grid at the start of item w, so the
  // loads are in flight through w's records.  prep (the whole workgroup, barriers inside) turns
  // them into the LDS segment table once w's records are in the table.
  struct Pre {
    uint32_t p;
    int sbits, sub, nseg;
    int64_t nrow, bb0;
    uint32_t selw;
    uint16_t s00, s01, s10, s11;  // seg[k0][f], seg[k0][f + 1], seg[k0 + 1][f], seg[k0 + 1][f + 1]
  };
  struct It {
    uint32_t p;
    int sbits, sub, nseg, segb;  // segb: log2 of the records per segment-lookup block
    int64_t rn, nrow;
    bool isel;
  };
  auto fetch = [&](int64_t w, Pre& r) {
    uint32_t p;
    int sbits = 0, sub = 0;
    if (work) {
      const uint32_t x = work[w];
      p = x & 0xFFFFu;
      sbits = (x >> 16) & 0xF;
      sub = (int)(x >> 20);
    } else {
      p = (uint32_t)w;
    }
    p = __builtin_amdgcn_readfirstlane(p);
    const int b = (int)(p >> q.fbits), f = (int)(p & (uint32_t)(F - 1));
    const int cs = lcs[b];
    int nseg = lcs[b + 1] - cs;
    if (nseg < 0 || nseg > C1_SEGMAX) nseg = 0;  // (k_c1_check guarantees 0 <= nseg <= SEGMAX)
    r.p = p;
    r.sbits = sbits;
    r.sub = sub;
    r.nseg = nseg;
    r.nrow = cnt[p];
    r.selw = ((const uint32_t*)sel)[p >> 2];
    r.bb0 = lbb[b];
    const int k0 = threadIdx.x * 2;
    r.s00 = r.s01 = r.s10 = r.s11 = 0;
    if (k0 < nseg) {
      const uint16_t* sg = seg + (int64_t)(cs + k0) * (F + 1) + f;
      r.s00 = sg[0];
      r.s01 = sg[1];
    }
    if (k0 + 1 < nseg) {
      const uint16_t* sg = seg + (int64_t)(cs + k0 + 1) * (F + 1) + f;
      r.s10 = sg[0];
      r.s11 = sg[1];
    }
  };
  auto prep = [&](const Pre& r, It& it) {
    const int nseg = r.nseg;
    it.p = r.p;
    it.sbits = r.sbits;
    it.sub = r.sub;
    it.nseg = nseg;
    it.nrow = r.nrow;
    it.isel = ((r.selw >> (8 * (r.p & 3))) & 0xFFu) != 0;
    const int k0 = threadIdx.x * 2;
    const int len0 = k0 < nseg ? (int)r.s01 - (int)r.s00 : 0;
    const int len1 = k0 + 1 < nseg ? (int)r.s11 - (int)r.s10 : 0;
    const int64_t base0 = r.bb0 + (int64_t)k0 * C1_CH + r.s00;
    const int64_t base1 = r.bb0 + (int64_t)(k0 + 1) * C1_CH + r.s10;
    const int s = len0 + len1;
    int incl = s;
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(incl, off, 64);
      if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    lds_barrier();
    int before = 0;
    int tot = 0;
    for (int k = 0; k < NW; k++) {
      before += k < wave ? wsum[k] : 0;
      tot += wsum[k];
    }
    const int ex = before + incl - s;
    // the finest lookup block that covers the item in C1_SEGOF entries (segments hold C1_CH / F
    // records on average: 32-record blocks make the lookup a read and at most a step or two)
    const int segb = tot <= (C1_SEGOF << 5) ? 5 : (tot <= (C1_SEGOF << 6) ? 6 : C1_SEGB);
    const int bm = (1 << segb) - 1;
    if (k0 < nseg) sg2[k0] = (uint32_t)ex | (uint64_t)(uint32_t)(int32_t)(base0 - ex) << 32;
    if (k0 + 1 < nseg) sg2[k0 + 1] = (uint32_t)(ex + len0) | (uint64_t)(uint32_t)(int32_t)(base1 - (ex + len0)) << 32;
    // segment lookup: block j (records [j << segb, (j + 1) << segb)) starts in segment segof[j]
    for (int bj = (ex + bm) >> segb, be = (ex + len0 + bm) >> segb; bj < be && bj < C1_SEGOF; bj++)
      segof[bj] = (uint16_t)k0;
    for (int bj = (ex + len0 + bm) >> segb, be = (ex + s + bm) >> segb; bj < be && bj < C1_SEGOF; bj++)
      segof[bj] = (uint16_t)(k0 + 1);
    if (k0 < nseg && k0 + 2 >= nseg) sg2[nseg] = (uint32_t)(ex + s);  // the total
    if (nseg == 0 && threadIdx.x == 0) sg2[0] = 0u;
    lds_barrier();
    it.rn = (uint32_t)sg2[nseg];
    it.segb = segb;
  };
  uint64_t ra[AU], rb[AU];
  uint32_t ta[AU], tb[AU];  // WIDE: the records' ts words
  // records li = l0 + thread + u NT of the item whose segments are in LDS (indices clamped to the
  // last record: every load is unconditional, so the waits stay counted)
  auto load = [&](uint64_t (&x)[AU], uint32_t (&tx)[AU], int64_t l0, int64_t rn, int nseg, int segb) {
#pragma unroll
    for (int u = 0; u < AU; u++) {
      int64_t li = l0 + threadIdx.x + (int64_t)u * NT;
      li = li < rn ? li : rn - 1;
      int lo = 0;  // the last segment starting at or before li
      int64_t at;
      if (rn <= ((int64_t)C1_SEGOF << segb)) {  // from the block's segment, a step or two on
        lo = segof[li >> segb];
        uint64_t sa = sg2[lo], sb = sg2[lo + 1];  // one ds_read2_b64
        while (lo + 1 < nseg && (int64_t)(uint32_t)sb <= li) {
          lo++;
          sa = sb;
          sb = sg2[lo + 1];
        }
        at = (int64_t)(int32_t)(sa >> 32) + li;
      } else {
        int hi = nseg;
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if ((int64_t)(uint32_t)sg2[mid] <= li) lo = mid;
          else hi = mid;
        }
        at = (int64_t)(int32_t)(sg2[lo] >> 32) + li;
      }
      x[u] = c1_ld(srec + at);
      if constexpr (WIDE) tx[u] = c1_ld(srecT + at);
    }
  };
  // the item's first two chunks (register sets A and B): a chunk is always two chunks ahead of
  // the one being applied
  auto load01 = [&](const It& x) {
    if (x.rn > 0) load(ra, ta, 0, x.rn, x.nseg, x.segb);
    if (x.rn > (int64_t)AU * NT) load(rb, tb, (int64_t)AU * NT, x.rn, x.nseg, x.segb);
  };
  // the bucket table (chunk starts, bucket bases) in LDS for every descriptor
  for (int k = threadIdx.x; k <= (1 << (q.log2P - q.fbits)); k += NT) {
    lcs[k] = cstart[k];
    lbb[k] = bb[k];
  }
  lds_barrier();
  // the first item, and its first chunks in flight; each item prepares the next one (segments and
  // first chunks) as soon as its own records are in the table, so those loads overlap its
  // resident-row, count and write-out phases
  Pre pr{};
  It nx{};
  if (blockIdx.x < nwork) {
    fetch(blockIdx.x, pr);
    prep(pr, nx);
    load01(nx);
  }
  for (int64_t w = blockIdx.x; w < nwork; w += gridDim.x) {
    const It it = nx;
    const uint32_t p = it.p;
    const int sbits = it.sbits, sub = it.sub, nseg = it.nseg, segb = it.segb;
    const int64_t rn = it.rn, nrow = it.nrow;
    const bool isel = it.isel;
    const int64_t wn = w + gridDim.x;
    if (wn < nwork) fetch(wn, pr);
    if (first && threadIdx.x == 0) prn[p] = (uint32_t)rn;
    if (rn == 0 && first) {  // untouched partition: nothing to rewrite
      if (wn < nwork) {
        prep(pr, nx);
        load01(nx);
      }
      continue;
    }
    const uint64_t* src = (isel ? buf1 : buf0) + (uint64_t)p * q.cmax * q.sw;
    // (closed resident rows leave for the closed store in the write-out, phase 4: one pass over the
    // resident rows there, the closed store's slots reserved with the region's)
    C1M_T(0);
    // 1. records → delta entries, two register sets (chunk c + 1 in flight while c is applied;
    //    chunk 0 was loaded with the item's segments)
    // R32: the push's record times relative to the first window's start fit 32 bits (a 32-bit
    // window division instead of the 64-bit one)
    // The record set's next chunk is loaded into the same registers right after its identities'
    // CASes are issued (prefetch): the chunk's segment lookups and the table-full flag then return
    // with the CASes (LDS returns in order), not behind this chunk's plane atomics, and the loads
    // have a whole chunk to land.  Returns false when the table is (about to be) full.
    auto apply = [&](const uint64_t (&xr)[AU], const uint32_t (&txr)[AU], int64_t l0, auto R32, auto&& prefetch) -> bool {
      ID id[AU];
      uint32_t e[AU], tr[AU];
      bool pend[AU], claimed[AU];
#pragma unroll
      for (int u = 0; u < AU; u++) {
        const int64_t li = l0 + threadIdx.x + (int64_t)u * NT;
        const uint64_t v = xr[u];
        const int32_t t32 = WIDE ? (int32_t)txr[u] : (int32_t)(uint32_t)v;
        const uint64_t krel = v >> 32;
        uint64_t wi;
        if constexpr (decltype(R32)::value) wi = fast_udiv32((uint32_t)t32 + tsh32, q.fd32);
        else wi = fast_udiv((uint64_t)(T0 + (int64_t)t32), q.fd) - (uint64_t)wbase;
        ID x;
        if constexpr (WIDE) x = (ID)((v << q.log2P) | wi);  // v = the key hash
        else if constexpr (sizeof(ID) == 4) x = (ID)(((uint32_t)krel << wbits) | (uint32_t)wi);
        else x = (ID)((krel << 32) | wi);
        const uint32_t h = c1_hash<ID>(x);
        bool act = li < rn;
        if (sbits) act = act && (int)c1_sub(h, sbits) == sub;
        id[u] = act ? x : EMPTY;
        e[u] = act ? h >> (32 - log2H) : dummy;
        tr[u] = (uint32_t)(t32 - tmin32) + 1u;
      }
      ID old[AU];
#pragma unroll
      for (int u = 0; u < AU; u++) {
        old[u] = EMPTY;
        __hip_atomic_compare_exchange_strong(&ids[e[u]], &old[u], id[u], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      const int full = *(volatile KLDS int*)&lovf;
      prefetch();
#pragma unroll
      for (int u = 0; u < AU; u++) {
        claimed[u] = id[u] != EMPTY && old[u] == EMPTY;
        pend[u] = old[u] != EMPTY && old[u] != id[u];
      }
      for (int probes = 1;; probes++) {  // collisions: every pending record probes on together
        bool anyp = false;
#pragma unroll
        for (int u = 0; u < AU; u++) anyp |= pend[u];
        if (!__ballot(anyp)) break;
        if (probes >= H) {
          lovf = 1;
#pragma unroll
          for (int u = 0; u < AU; u++)
            if (pend[u]) id[u] = EMPTY;
          break;
        }
#pragma unroll
        for (int u = 0; u < AU; u++) {
          if (!pend[u]) continue;
          e[u] = (e[u] + 1) & (uint32_t)(H - 1);
          ID o2 = EMPTY;
          __hip_atomic_compare_exchange_strong(&ids[e[u]], &o2, id[u], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
          claimed[u] = o2 == EMPTY;
          pend[u] = o2 != EMPTY && o2 != id[u];
        }
      }
      int nnow;
      {
        bool cl[AU];
#pragma unroll
        for (int u = 0; u < AU; u++) cl[u] = claimed[u] && id[u] != EMPTY;
        nnow = mg_list_append_n<AU>(cl, e, list, &nnew);
      }
#pragma unroll
      for (int u = 0; u < AU; u++) {
        if (id[u] == EMPTY) continue;
        __hip_atomic_fetch_max(&rt[e[u]], tr[u], WG_RLX);
        __hip_atomic_fetch_add(&ct[e[u]], 1u, WG_RLX);
      }
      return !full && nnow <= q.hmax;
    };
    const int64_t nch = (rn + (int64_t)AU * NT - 1) / ((int64_t)AU * NT);
    if (rn > 0) {  // chunks 0 and 1 are in flight (load01); each set is reloaded as it is applied
      for (int64_t c = 0; c < nch; c += 2) {
        auto pa = [&] { if (c + 2 < nch) load(ra, ta, (c + 2) * AU * NT, rn, nseg, segb); };
        const bool ga = r32 ? apply(ra, ta, c * AU * NT, std::true_type{}, pa) : apply(ra, ta, c * AU * NT, std::false_type{}, pa);
        if (!ga || c + 1 >= nch) break;
        auto pb = [&] { if (c + 3 < nch) load(rb, tb, (c + 3) * AU * NT, rn, nseg, segb); };
        const bool gb = r32 ? apply(rb, tb, (c + 1) * AU * NT, std::true_type{}, pb)
                            : apply(rb, tb, (c + 1) * AU * NT, std::false_type{}, pb);
        if (!gb) break;
      }
    }
    lds_barrier();
    // the item's records are in the table (its segments are no longer read): the next item's
    // segments and first chunks now
    if (wn < nwork) {
      prep(pr, nx);
      load01(nx);
    }
    C1M_T(1);
    const int nl = nnew < H ? nnew : H;
    if (lovf || nnew > q.hmax) {  // more groups than the table takes: retried with 2x sub-passes
      if (threadIdx.x == 0) fail[p] |= 1;
      for (int i = threadIdx.x; i < nl; i += NT) {
        const uint32_t e = list[i];
        ids[e] = EMPTY;
        rt[e] = 0u;
        ct[e] = 0u;
      }
      lds_barrier();
      if (threadIdx.x == 0) {
        lovf = 0;
        nnew = 0;
      }
      lds_barrier();
      continue;
    }
    // 2. resident rows: mark the delta entries they absorb; count live and closed rows
    int n_mine = 0, n_cl = 0;
    for (int64_t r = threadIdx.x; r < nrow; r += NT) {
      const uint64_t* row = src + r * q.sw;
      ID id;
      uint32_t h;
      const bool has = row_id(row, &id, &h);
      if (sbits && (int)c1_sub(h, sbits) != sub) continue;
      if (evict && (int64_t)row[1] + q.size <= close0) {
        n_cl++;
        continue;
      }
      if (has) {
        const int e = c1_find_id<ID>(ids, id, h >> (32 - log2H), H);
        if (e >= 0) rt[e] |= RT_MATCHED;  // one resident row per identity: a plain store
      }
      n_mine++;
    }
    if (nrow > 0) lds_barrier();  // the marks before the list walk reads them (uniform: nrow is the item's)
    // the wave's share of the list: new (unmatched) entries
    const int per = ((nl + NW - 1) / NW + 63) & ~63;
    const int lb0 = wave * per, lb1 = lb0 + per < nl ? lb0 + per : nl;
    int nnw = 0;
    for (int k = lb0; k < lb1; k += 64) {
      const int i = k + lane;
      const uint32_t e = i < lb1 ? list[i] : dummy;
      const bool isnew = i < lb1 && !(rt[e] & RT_MATCHED);
      nnw += (int)__popcll(__ballot(isnew));
    }
    // 3. per-wave row counts → the partition's region range (one atomic per work item), and the
    //    closed store's slots for its closed rows
    const int wave_rows = (int)wave_sum(n_mine) + nnw;
    const int wave_cl = (int)wave_sum(n_cl);
    if (lane == 0) {
      wsum[wave] = wave_rows;
      csum[wave] = wave_cl;
    }
    lds_barrier();
    int wave_before = 0, total = 0, cl_before = 0, cl_total = 0;
    for (int k = 0; k < NW; k++) {
      if (k < wave) wave_before += wsum[k], cl_before += csum[k];
      total += wsum[k];
      cl_total += csum[k];
    }
    if (threadIdx.x == 0) {
      if (work) lbase = total ? atomicAdd(&newcnt[p], (unsigned long long)total) : 0ULL;
      else {
        lbase = 0;
        newcnt[p] = (unsigned long long)total;
      }
      // (an item that does not fit its region is retried and reserves nothing here)
      cbase = cl_total && (int64_t)(lbase + total) <= q.cmax ? atomicAdd(closed_n, (unsigned long long)cl_total) : 0ULL;
    }
    lds_barrier();
    if ((int64_t)(lbase + total) > q.cmax) {
      if (threadIdx.x == 0) {
        fail[p] |= 2;
        atomicMax(need, (unsigned long long)(lbase + total));
      }
      for (int i = threadIdx.x; i < nl; i += NT) {
        const uint32_t e = list[i];
        ids[e] = EMPTY;
        rt[e] = 0u;
        ct[e] = 0u;
      }
      lds_barrier();
      if (threadIdx.x == 0) nnew = 0;
      lds_barrier();
      continue;
    }
    C1M_T(3);
    // 4. write: resident rows (merged), then the wave's new entries (ballot ranks: consecutive rows)
    uint64_t* dst0 = (isel ? buf0 : buf1) + (uint64_t)p * q.cmax * q.sw;
    uint64_t cur = lbase + (uint64_t)wave_before;
    uint64_t ccur = cbase + (uint64_t)cl_before;
    const uint64_t lt = (1ULL << lane) - 1;
    int nh = 0, nhc = 0;
    for (int64_t r0 = wave * 64; r0 < nrow; r0 += NT) {
      const int64_t r = r0 + lane;
      const uint64_t* row = src + (r < nrow ? r : 0) * q.sw;
      bool live = r < nrow, cl = false;
      int e = -1;
      if (live) {
        ID id;
        uint32_t h;
        const bool has = row_id(row, &id, &h);
        if (sbits) live = (int)c1_sub(h, sbits) == sub;
        cl = live && evict && (int64_t)row[1] + q.size <= close0;
        live = live && !cl;
        if (live && has) e = c1_find_id<ID>(ids, id, h >> (32 - log2H), H);
      }
      const uint64_t bc = __ballot(cl);
      if (cl) {
        uint64_t* cd = closed + (ccur + __popcll(bc & lt)) * q.sw;
        for (int k = 0; k < q.sw; k++) cd[k] = row[k];
        nhc += q.hv_active && c1q_having(q, row[3]) ? 1 : 0;
      }
      ccur += __popcll(bc);
      const uint64_t bl = __ballot(live);
      if (live) {
        const uint64_t ri = cur + __popcll(bl & lt);
        uint64_t* dst = dst0 + ri * q.sw;
        uint64_t w2 = row[2], c = row[3];
        if (e >= 0) {
          const int64_t t = tmin + (int64_t)(rt[e] & ~RT_MATCHED) - 1;
          w2 = t > (int64_t)w2 ? (uint64_t)t : w2;
          c += ct[e];
        }
        *(longlong2*)dst = make_longlong2((int64_t)row[0], (int64_t)row[1]);
        *(longlong2*)(dst + 2) = make_longlong2((int64_t)w2, (int64_t)c);
        const bool now = !q.hv_active || c1q_having(q, c);
        nh += q.hv_active && now ? 1 : 0;
        if (q.chg)
          q.chg[(uint64_t)p * q.cmax + ri] =
              e >= 0 ? (uint8_t)(CHG_TOUCHED | (!q.hv_active || c1q_having(q, row[3]) ? CHG_OLD : 0) | (now ? CHG_NEW : 0))
                     : (uint8_t)0;
      }
      cur += __popcll(bl);
    }
    if (nrow > 0) lds_barrier();  // every wave's resident rows have read their entries: the list walk clears them
    const uint32_t wmask = wbits ? (1u << wbits) - 1u : 0u;
    for (int k = lb0; k < lb1; k += 64) {
      const int i = k + lane;
      const uint32_t e = i < lb1 ? list[i] : dummy;
      const uint32_t rv = rt[e];
      const bool used = i < lb1;
      const bool isnew = used && !(rv & RT_MATCHED);
      const uint64_t bl = __ballot(isnew);
      if (isnew) {
        const uint64_t ri = cur + __popcll(bl & lt);
        uint64_t* dst = dst0 + ri * q.sw;
        const ID id = ids[e];
        int64_t key, wi;
        if constexpr (WIDE) {  // the partition's bits above the identity's key-hash bits
          wi = (int64_t)((uint64_t)id & (((uint64_t)1 << q.log2P) - 1));
          key = key_of_hash(((uint64_t)p << (64 - q.log2P)) | ((uint64_t)id >> q.log2P));
        } else if constexpr (sizeof(ID) == 4) {
          key = kmin + (int64_t)((uint32_t)id >> wbits);
          wi = (int64_t)((uint32_t)id & wmask);
        } else {
          key = kmin + (int64_t)((uint64_t)id >> 32);
          wi = (int64_t)((uint64_t)id & 0xFFFFFFFFull);
        }
        const uint32_t c = ct[e];
        *(longlong2*)dst = make_longlong2(key, (wbase + wi) * q.adv);
        *(longlong2*)(dst + 2) = make_longlong2(tmin + (int64_t)rv - 1, (int64_t)c);
        const bool now = !q.hv_active || c1q_having(q, c);
        nh += q.hv_active && now ? 1 : 0;
        if (q.chg) q.chg[(uint64_t)p * q.cmax + ri] = (uint8_t)(CHG_TOUCHED | (now ? CHG_NEW : 0));
      }
      if (used) {  // every listed (used) entry leaves cleared for the next item
        ids[e] = EMPTY;
        rt[e] = 0u;
        ct[e] = 0u;
      }
      cur += __popcll(bl);
    }
    if (q.hv_active) {
      nh = (int)wave_sum(nh);
      nhc = (int)wave_sum(nhc);
      if (lane == 0 && nh) atomicAdd(&hnew[p], (unsigned long long)nh);
      if (lane == 0 && nhc) atomicAdd(hclosed, (unsigned long long)nhc);
    }
    lds_barrier();  // the table is clear for the next item
    C1M_T(4);
    if (threadIdx.x == 0) nnew = 0;
    lds_barrier();
  }
}

// ------------------------------------------------------------------ value records (c1v)
// The same pipeline for a query whose aggregates all read ONE argument column (COUNT(col), SUM,
// AVG, MIN, MAX, with or without COUNT(*)): records are 16 bytes, {(key - kmin) << 32 |
// (uint32)(ts - T0), bit 63 = the argument is not NULL; the argument's bits (INT sign-extended,
// BIGINT, DOUBLE raw)}, so the key range must fit 31 bits.  HOPPING windows whose size is a
// multiple of the advance go through panes: a record updates ONE entry, its pane (key, ts /
// advance), and after the records every pane is folded into its F windows — F updates per pane,
// not per record.  TUMBLING is the F = 1 case (the pane is the window).
constexpr int C1V_CH = 4096;  // refine chunk of 16-byte records (64 KB of LDS stage)
constexpr int C1V_MAXW = 8;   // row words (key, ws, rowtime + at most 5 state words)

typedef uint64_t c1v_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ ulonglong2 ld_nt2(const ulonglong2* p) {  // 16-byte load (c1_ld)
  const c1v_u2 v = c1_ld((const c1v_u2*)p);
  return make_ulonglong2(v.x, v.y);
}

struct C1VCol {
  const void* data;
  const uint8_t* valid;
  int32_t type;
};


// Records of tile t → step runs, as k_c1_scatter, 16 bytes each (key - kb in 31 bits, the
// argument's non-null flag in bit 63).  HOP: the windows
// applied per accepted record (windowsFor's count) for the batch statistics.
template <int U, int NT, bool ST, bool ROWS>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void k_c1v_scatter(
    const int64_t* __restrict__ keys, const int64_t* __restrict__ ts, const uint8_t* __restrict__ kv,
    const uint8_t* __restrict__ rv, C1VCol vc, RowsIn ri, int64_t n, int64_t nT, int log2B, uint32_t* __restrict__ rcnt,
    uint16_t* __restrict__ roff, int64_t nSt, ulonglong2* __restrict__ srec, int64_t* __restrict__ tilestat,
    int64_t* __restrict__ tpart, int64_t* __restrict__ ci, const int64_t* __restrict__ st_at, int64_t size, int64_t adv,
    FastDiv fd, int hop, int64_t grace, const int64_t* __restrict__ stream_time, int64_t kb_in, int has_kb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int wsum[NT / 64];
  __shared__ unsigned long long lc[5];
  __shared__ int lt[2][2];
  __shared__ int lfail, lkfail;
  __shared__ uint32_t lkr[2];  // min / max of the staged key offsets
  constexpr int S = U * NT;
  constexpr int SPT = C1_TILE / S;
  const int B = 1 << log2B;
  const int64_t t = tile_of(blockIdx.x, nT);
  uint32_t* cnt = (uint32_t*)smem;
  uint32_t* sbase = cnt + B;
  ulonglong2* sp = (ulonglong2*)(smem + (size_t)B * 8);  // B >= 32: 16-byte aligned
  uint32_t* lrc = (uint32_t*)(smem + run_stage_lds(B, S, 16, false));
  uint16_t* lro = (uint16_t*)(lrc + SPT * B);
  for (int b = threadIdx.x; b < B; b += NT) cnt[b] = 0u;
  if (threadIdx.x < 5) lc[threadIdx.x] = 0;
  if (threadIdx.x < 2) {
    lt[threadIdx.x][0] = INT32_MIN;
    lt[threadIdx.x][1] = INT32_MAX;
  }
  if (threadIdx.x == 0) {
    lfail = lkfail = 0;
    lkr[0] = 0xFFFFFFFFu;
    lkr[1] = 0u;
  }
  int64_t T0, kb;
  if constexpr (ROWS) run_bases((const int64_t*)ri.rows, (const int64_t*)ri.rows + 1, n, stream_time, kb_in, has_kb, 31, ci, &T0, &kb);
  else run_bases(keys, ts, n, stream_time, kb_in, has_kb, 31, ci, &T0, &kb);
  const int shift = log2B == 0 ? 64 : 64 - log2B;
  const uint32_t bmask = (uint32_t)(B - 1);
  const int64_t base = t * C1_TILE;
  const int64_t end = base + C1_TILE < n ? base + C1_TILE : n;
  int c_acc = 0, c_nk = 0, c_nr = 0, c_bt = 0, c_app = 0;
  uint32_t kor = 0u;
  int64_t x[U], k[U], v[U];
  uint32_t vm[ROWS ? U : 1];  // ROWS: the rows' validity words (low half)
  int64_t rst[ROWS && ST ? U : 1];  // ROWS && ST: the rows' stream-time words (KHIP_SHUFFLE_STREAM_TIME)
  auto load_step = [&](int64_t i0) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      int64_t i = i0 + (int64_t)u * NT;
      i = i < end ? i : end - 1;
      if constexpr (ROWS) {
        const uint64_t* r = ri.rows + i * (int64_t)ri.rw;
        if (ri.rw == 4 && ri.vword == 2) {  // [key, ts, argument, validity]: two 16-byte loads
          const ulonglong2 a = ((const ulonglong2*)r)[0], b = ((const ulonglong2*)r)[1];
          k[u] = (int64_t)a.x;
          x[u] = (int64_t)a.y;
          v[u] = (int64_t)b.x;
          vm[u] = (uint32_t)b.y;
        } else {
          k[u] = (int64_t)r[0];
          x[u] = (int64_t)r[1];
          v[u] = (int64_t)r[ri.vword];
          vm[u] = (uint32_t)r[ri.rw - 1];
        }
        if constexpr (ST) rst[u] = (int64_t)r[ri.rw - 2];
      } else {
        x[u] = ts[i];
        k[u] = keys[i];
        v[u] = vc.type == KHIP_TYPE_INT32 ? (int64_t)((const int32_t*)vc.data)[i] : ((const int64_t*)vc.data)[i];
      }
    }
  };
  int64_t t_rmax = -1, t_min = INT64_MAX, t_bound = INT64_MAX;  // the tile's summary (k_c1_scatter)
  bool t_ok = true;
  auto publish = [&](int64_t, int st) {
    const int mx = lt[st & 1][0], mn = lt[st & 1][1];
    if (mx != INT32_MIN) {
      const int64_t smx = T0 + mx, smn = T0 + mn;
      t_rmax = smx > t_rmax ? smx : t_rmax;
      t_min = smn < t_min ? smn : t_min;
      const int64_t fw = first_window_start_fd(smn, size, adv, fd) + size;
      const int64_t b = grace > ((int64_t)1 << 61) ? INT64_MAX : fw + grace - 1;
      t_bound = b < t_bound ? b : t_bound;
      t_ok = t_ok && t_rmax <= b;
    }
    lt[st & 1][0] = INT32_MIN;
    lt[st & 1][1] = INT32_MAX;
  };
  lds_barrier();
  int64_t s0 = base;
  int st_last = -1;
  if (s0 < end) load_step(s0 + threadIdx.x);
  for (int st = 0; s0 < end; s0 += S, st++) {
    st_last = st;
    const int64_t i0 = s0 + threadIdx.x;
    bool ok[U];
    uint32_t bin[U];
    ulonglong2 rec[U];
    int tmx = INT32_MIN, tmn = INT32_MAX;
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t i = i0 + (int64_t)u * NT;
      ok[u] = i < end;
      const int64_t ii = ok[u] ? i : base;
      const bool kok = ROWS || bit_get(kv, ii), rok = ROWS || bit_get(rv, ii);
      const bool vok = ROWS ? ((vm[ROWS ? u : 0] >> ri.vbit) & 1u) != 0 : bit_get(vc.valid, ii);
      const bool valid = ok[u] && kok && rok && x[u] >= 0;
      c_nk += ok[u] && !kok;
      c_nr += ok[u] && kok && !rok;
      c_bt += ok[u] && kok && rok && x[u] < 0;
      c_acc += valid;
      const int64_t d = x[u] - T0;
      if (valid && (d <= (int64_t)INT32_MIN || d > (int64_t)INT32_MAX)) {  // rare: an LDS flag, not a loop-carried mask
        lfail = 1;
#ifdef KHIP_TUNING
        if (ci[CI_N - 1] == 1 && (threadIdx.x & 63) == 0) printf("[c1 scatter] t %ld i %ld x %ld T0 %ld\n", (long)t, (long)i, (long)x[u], (long)T0);
#endif
      }
      if constexpr (ST) {
        const int64_t ds = (ROWS ? rst[ROWS ? u : 0] : st_at[ii]) - T0;
        if (valid && (ds <= (int64_t)INT32_MIN || ds > (int64_t)INT32_MAX)) lfail = 1;
        tmx = valid && (int)ds > tmx ? (int)ds : tmx;
      } else {
        tmx = valid && (int)d > tmx ? (int)d : tmx;
      }
      tmn = valid && (int)d < tmn ? (int)d : tmn;
      if (hop && valid) {  // windowsFor: starts in (ts - size, ts], multiples of adv, >= 0
        const int64_t lo = x[u] - size + adv;
        c_app += (int)((int64_t)fast_udiv((uint64_t)x[u], fd) - (int64_t)fast_udiv((uint64_t)(lo > 0 ? lo : 0), fd) + 1);
      }
      bin[u] = stage_bin(key_hash(k[u]), shift, bmask);
      const uint64_t kd = (uint64_t)k[u] - (uint64_t)kb;
      kor |= ok[u] ? (uint32_t)(kd >> 31) : 0u;  // nonzero: a key outside the 31-bit field above kb
      const uint64_t w0 = ((kd & 0x7FFFFFFFull) << 32) | (uint64_t)(valid ? (uint32_t)d : C1_SENT);
      rec[u] = make_ulonglong2(w0 | (vok ? (1ULL << 63) : 0ULL), (uint64_t)v[u]);
    }
    if (s0 + S < end) load_step(i0 + S);
    uint32_t t32u[U];  // (no ts words: 16-byte records carry the ts)
    const uint32_t tot = stage_step_runs<U, NT, ulonglong2, false>(rec, t32u, bin, ok, B, cnt, sbase, wsum, sp, nullptr,
                                                                   srec, nullptr, t * SPT + st, lrc + st * B,
                                                                   lro + st * B);
    step_krange<NT, ulonglong2>(sp, tot, 0x7FFFFFFFu, lkr);
    for (int off = 32; off > 0; off >>= 1) {
      const int a = __shfl_xor(tmx, off, 64), b = __shfl_xor(tmn, off, 64);
      tmx = a > tmx ? a : tmx;
      tmn = b < tmn ? b : tmn;
    }
    if ((threadIdx.x & 63) == 0 && tmx != INT32_MIN) {
      atomicMax(&lt[st & 1][0], tmx);
      atomicMin(&lt[st & 1][1], tmn);
    }
    if (threadIdx.x == 0 && st > 0) publish(s0 - S, st - 1);
  }
  flush_run_counts<SPT, NT>(lrc, lro, B, st_last, t, nSt, rcnt, roff);
  if (kor) lkfail = 1;
  __syncthreads();
  if (threadIdx.x == 0 && s0 > base) publish(s0 - S, st_last);
  if (threadIdx.x == 0) run_krange(lkr, lkfail, kb, ci);
  c_acc = wave_sum(c_acc);
  c_nk = wave_sum(c_nk);
  c_nr = wave_sum(c_nr);
  c_bt = wave_sum(c_bt);
  c_app = wave_sum(c_app);
  if ((threadIdx.x & 63) == 0) {
    if (c_acc) atomicAdd(&lc[0], (unsigned long long)c_acc);
    if (c_nk) atomicAdd(&lc[1], (unsigned long long)c_nk);
    if (c_nr) atomicAdd(&lc[2], (unsigned long long)c_nr);
    if (c_bt) atomicAdd(&lc[3], (unsigned long long)c_bt);
    if (c_app) atomicAdd(&lc[4], (unsigned long long)c_app);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t* tp = tpart + t * T_NPART;
    tp[T_ACCEPTED] = (int64_t)lc[0];
    tp[T_NULL_KEY] = (int64_t)lc[1];
    tp[T_NULL_ROW] = (int64_t)lc[2];
    tp[T_BAD_TS] = (int64_t)lc[3];
    tp[T_APPLIED] = hop ? (int64_t)lc[4] : (int64_t)lc[0];  // none late (checked)
    tp[T_LATE] = 0;
    if (lfail) atomicOr((unsigned long long*)&ci[CI_TFAIL], 1ULL);
    int64_t* ts4 = tilestat + t * 4;
    ts4[0] = t_rmax;
    ts4[1] = t_min;
    ts4[2] = t_bound;
    ts4[3] = t_ok ? 1 : 0;
  }
}

// Chunk w of its bucket (C1V_CH records): sentinels dropped, counting-sorted by partition,
// written back in place; the segment table as k_c1_refine's.
template <int U, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void k_c1v_refine(
    const ulonglong2* __restrict__ srcA, const int64_t* __restrict__ bb, const int* __restrict__ cstart, int log2B,
    int log2P, int fbits, ulonglong2* __restrict__ srec, uint16_t* __restrict__ seg, const int64_t* __restrict__ ci,
    const uint32_t* __restrict__ rpos, const uint16_t* __restrict__ roff, int64_t nSt, int64_t S,
    const uint32_t* __restrict__ cinfo) {
  if (ci_ld(ci, CI_GATE) == 0) return;
  const int w = blockIdx.x;
  if (w >= (int)ci_ld(ci, CI_NCHUNK)) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int lb, lnv;
  __shared__ int wsum[NT / 64];
  constexpr int CH = U * NT;
  static_assert(CH == C1V_CH, "refine chunk");
  const int F = 1 << fbits, B = 1 << log2B;
  uint32_t* cnt = (uint32_t*)smem;
  uint32_t* sbase = cnt + F;
  ulonglong2* stage = (ulonglong2*)(smem + (((size_t)F * 8 + 15) & ~(size_t)15));
  for (int f = threadIdx.x; f < F; f += NT) cnt[f] = 0u;
  if (threadIdx.x == 0) lb = -1;
  __syncthreads();
  for (int b = threadIdx.x; b < B; b += NT)
    if (cstart[b] <= w && w < cstart[b + 1]) lb = b;
  __syncthreads();
  const int b = lb;
  if (b < 0) return;
  const int64_t lo = bb[b] + (int64_t)(w - cstart[b]) * CH;
  const int64_t bend = bb[b + 1];
  const int len = (int)(bend - lo < CH ? bend - lo : CH);
  const int64_t kmin = ci_ld(ci, CI_KMINC);
  const uint64_t kshift = (uint64_t)ci_ld(ci, CI_KSHIFT) << 32;  // records hold key - kb
  const int shift = 64 - log2P;
  // where the chunk's records lie in the step runs (a map in the not yet used stage)
  const uint32_t* rp = rpos + (int64_t)b * nSt;
  const uint16_t* ro = roff + (int64_t)b * nSt;
  chunk_map(rp, ro, cinfo, w, S, lo, len, (uint32_t*)stage);
  ulonglong2 r[U];
  uint32_t f[U], rank[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int j = threadIdx.x + u * NT;
    const uint32_t src = ((const uint32_t*)stage)[j < len ? j : len - 1];
    r[u] = ld_nt2(srcA + src);
    r[u].x -= kshift;
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int j = threadIdx.x + u * NT;
    const bool v = j < len && (uint32_t)r[u].x != C1_SENT;
    f[u] = (uint32_t)(key_hash(kmin + (int64_t)((r[u].x >> 32) & 0x7FFFFFFFull)) >> shift) & (uint32_t)(F - 1);
    rank[u] = v ? atomicAdd(&cnt[f[u]], 1u) : 0xFFFFFFFFu;
  }
  __syncthreads();
  {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t c = t < F ? cnt[t] : 0u;
    uint32_t incl = c;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(incl, off, 64);
      if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wave] = (int)incl;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; k++) {
      before += k < wave ? (uint32_t)wsum[k] : 0u;
      tot += (uint32_t)wsum[k];
    }
    if (t < F) {
      sbase[t] = before + incl - c;
      seg[(int64_t)w * (F + 1) + t] = (uint16_t)(before + incl - c);
    }
    if (t == 0) {
      seg[(int64_t)w * (F + 1) + F] = (uint16_t)tot;
      lnv = (int)tot;
    }
  }
  __syncthreads();
  const int nv = lnv;
#pragma unroll
  for (int u = 0; u < U; u++)
    if (rank[u] != 0xFFFFFFFFu) stage[sbase[f[u]] + rank[u]] = r[u];
  __syncthreads();
  for (int j = threadIdx.x; j < nv; j += NT) srec[lo + j] = stage[j];
}

// Merge parameters of the value pipeline.  LDS: ids ID[H + 64] | 8-byte planes (sum, min, max,
// present ones) | u32 planes (row time, COUNT(*), non-null count) | list u16[H] | segment prefix
// | segment bases | bucket bases | chunk starts (byte offsets below, from c1v_layout).
struct C1VQ {
  int32_t log2P, fbits, log2H, sw, hmax, f64, fan;
  int32_t off_sum, off_min, off_max, off_rt, off_star, off_cnt, off_list, off_spre;
  int32_t word_op[C1V_MAXW];  // kind of the update op writing row word k (-1: none)
  int64_t size, adv, cmax;
  FastDiv fd;
  FastDiv32 fd32;
  uint64_t init[C1V_MAXW];
  HavingDev having;
  uint8_t* chg;
};

template <class T>
__device__ __forceinline__ KLDS T* c1v_plane(char* smem, int off) {
  return (KLDS T*)((KLDS char*)smem + off);
}

// Plane masks: a merge instantiation specialised for the planes a query has (PM != 0, the
// benchmarks' shapes), or PM = 0 reading them from the parameters (every other shape).
constexpr int PM_STAR = 1, PM_CNT = 2, PM_SUM = 4, PM_MIN = 8, PM_MAX = 16, PM_F64 = 32, PM_SPEC = 64;
constexpr int PM_C5 = PM_SPEC | PM_SUM;                                   // SUM(BIGINT)
constexpr int PM_C3 = PM_SPEC | PM_CNT | PM_SUM | PM_MIN | PM_MAX | PM_F64;  // SUM/AVG/MIN/MAX(DOUBLE)
template <int PM>
struct C1VP {
  const C1VQ& q;
  __device__ __forceinline__ bool star() const { return PM ? (PM & PM_STAR) != 0 : q.off_star >= 0; }
  __device__ __forceinline__ bool cnt() const { return PM ? (PM & PM_CNT) != 0 : q.off_cnt >= 0; }
  __device__ __forceinline__ bool sum() const { return PM ? (PM & PM_SUM) != 0 : q.off_sum >= 0; }
  __device__ __forceinline__ bool mn() const { return PM ? (PM & PM_MIN) != 0 : q.off_min >= 0; }
  __device__ __forceinline__ bool mx() const { return PM ? (PM & PM_MAX) != 0 : q.off_max >= 0; }
  __device__ __forceinline__ bool f64() const { return PM ? (PM & PM_F64) != 0 : q.f64 != 0; }
};

// Row word k (k >= 3) of a (key, window) combined with delta entry e: the word's update op
// applied to the entry's plane.
template <int PM>
__device__ __forceinline__ uint64_t c1v_word(const C1VQ& q, char* smem, int e, int k, uint64_t w) {
  const C1VP<PM> v{q};
  switch (q.word_op[k]) {
    case OP_INC: return v.star() ? w + c1v_plane<uint32_t>(smem, q.off_star)[e] : w;
    case OP_INC_VALID: return v.cnt() ? w + c1v_plane<uint32_t>(smem, q.off_cnt)[e] : w;
    case OP_ADD_I64: return v.sum() && !v.f64() ? w + c1v_plane<uint64_t>(smem, q.off_sum)[e] : w;
    case OP_ADD_F64:
      if (v.sum() && v.f64()) {
        double a, b = c1v_plane<double>(smem, q.off_sum)[e];
        __builtin_memcpy(&a, &w, 8);
        a += b;
        __builtin_memcpy(&w, &a, 8);
      }
      return w;
    case OP_MIN:
      if (v.mn()) {
        const int64_t m = c1v_plane<int64_t>(smem, q.off_min)[e];
        if (m < (int64_t)w) w = (uint64_t)m;
      }
      return w;
    case OP_MAX:
      if (v.mx()) {
        const int64_t m = c1v_plane<int64_t>(smem, q.off_max)[e];
        if (m > (int64_t)w) w = (uint64_t)m;
      }
      return w;
    default: return w;
  }
}

// Write one row word by word (no row array in registers: the write-out runs while the next
// item's record chunks are in flight), from the resident row (src) or, src == nullptr, from the
// initial words + key / window start / row time; e >= 0: combined with delta entry e (rtabs =
// its row time).  *was / *now: the HAVING before and after.
template <int PM>
__device__ __forceinline__ void c1v_emit(const C1VQ& q, char* smem, uint64_t* __restrict__ dst,
                                         const uint64_t* __restrict__ src, int e, int64_t key, int64_t ws, int64_t rtabs,
                                         bool* was, bool* now) {
  const int hv = q.having.a.w_val, hc = q.having.a.w_cnt;
  uint64_t ov = 0, oc = 0, nv = 0, nc = 0;
#pragma unroll
  for (int k = 0; k < C1V_MAXW; k++) {
    if (k >= q.sw) break;
    uint64_t w = src ? src[k] : (k == 0 ? (uint64_t)key : k == 1 ? (uint64_t)ws : k == 2 ? (uint64_t)rtabs : q.init[k]);
    if (k == hv) ov = w;
    if (k == hc) oc = w;
    if (e >= 0) {
      if (k == 2 && src) w = rtabs > (int64_t)w ? (uint64_t)rtabs : w;
      if (k >= 3) w = c1v_word<PM>(q, smem, e, k, w);
    }
    if (k == hv) nv = w;
    if (k == hc) nc = w;
    dst[k] = w;
  }
  *was = q.having.active ? having_ok_words(ov, oc, q.having) : true;
  *now = q.having.active ? having_ok_words(nv, nc, q.having) : true;
}

// Clear delta entry e for the next item.
template <int PM>
__device__ __forceinline__ void c1v_clear(const C1VQ& q, char* smem, int e) {
  const C1VP<PM> v{q};
  c1v_plane<uint32_t>(smem, q.off_rt)[e] = 0u;
  if (v.star()) c1v_plane<uint32_t>(smem, q.off_star)[e] = 0u;
  if (v.cnt()) c1v_plane<uint32_t>(smem, q.off_cnt)[e] = 0u;
  if (v.sum()) c1v_plane<uint64_t>(smem, q.off_sum)[e] = 0ULL;
  if (v.mn()) c1v_plane<int64_t>(smem, q.off_min)[e] = INT64_MAX;
  if (v.mx()) c1v_plane<int64_t>(smem, q.off_max)[e] = INT64_MIN;
}

// One (record or pane) contribution into delta entry e: row time, then the update planes.
// cv: the argument's non-null count (a record: 0 / 1), sum its bits (sum), mn / mx its order keys.
template <int PM>
__device__ __forceinline__ void c1v_add(const C1VQ& q, char* smem, uint32_t e, uint32_t tr, uint32_t cs, uint32_t cv,
                                        uint64_t sum, int64_t mn, int64_t mx) {
  const C1VP<PM> v{q};
  KLDS uint32_t* prt = &c1v_plane<uint32_t>(smem, q.off_rt)[e];
  __hip_atomic_fetch_max(prt, tr, WG_RLX);
  if (v.star() && cs) __hip_atomic_fetch_add(&c1v_plane<uint32_t>(smem, q.off_star)[e], cs, WG_RLX);
  if (cv) {
    if (v.cnt()) __hip_atomic_fetch_add(&c1v_plane<uint32_t>(smem, q.off_cnt)[e], cv, WG_RLX);
    if (v.sum()) {
      if (v.f64()) {
        double d;
        __builtin_memcpy(&d, &sum, 8);
        __hip_atomic_fetch_add(&c1v_plane<double>(smem, q.off_sum)[e], d, WG_RLX);
      } else {
        __hip_atomic_fetch_add(&c1v_plane<uint64_t>(smem, q.off_sum)[e], sum, WG_RLX);
      }
    }
    if (v.mn()) {
      KLDS int64_t* pm = &c1v_plane<int64_t>(smem, q.off_min)[e];
      __hip_atomic_fetch_min(pm, mn, WG_RLX);
    }
    if (v.mx()) {
      KLDS int64_t* pm = &c1v_plane<int64_t>(smem, q.off_max)[e];
      __hip_atomic_fetch_max(pm, mx, WG_RLX);
    }
  }
}

// identity of (krel, relative window or pane index): u32 krel << (wbits + PB) | pane << wbits | wi,
// u64 krel << 32 | pane << 31 | wi
template <class ID, bool PANES>
__device__ __forceinline__ ID c1v_id(uint64_t krel, uint64_t wi, bool pane, int wbits) {
  if constexpr (sizeof(ID) == 4)
    return (ID)(((uint32_t)krel << (wbits + (PANES ? 1 : 0))) | ((PANES && pane) ? (1u << wbits) : 0u) | (uint32_t)wi);
  else
    return (ID)((krel << 32) | ((PANES && pane) ? (1ULL << 31) : 0ULL) | wi);
}
template <class ID, bool PANES>
__device__ __forceinline__ bool c1v_is_pane(ID id, int wbits) {
  if constexpr (!PANES) return false;
  if constexpr (sizeof(ID) == 4) return ((uint32_t)id >> wbits) & 1u;
  else return ((uint64_t)id >> 31) & 1ULL;
}

// WPE: waves per SIMD the register budget allows (4: <= 128 VGPRs, two workgroups per CU; 2:
// <= 256, one)
template <int NT, int AU, class ID, bool PANES, int WPE, int PM>
__global__ __launch_bounds__(NT, WPE) void k_c1v_merge(
    const C1VQ* __restrict__ qp, const uint32_t* __restrict__ work, int64_t nwork, const int64_t* __restrict__ bb,
    const int* __restrict__ cstart, const uint16_t* __restrict__ seg, const ulonglong2* __restrict__ srec, int first,
    uint64_t* __restrict__ buf0, uint64_t* __restrict__ buf1, const uint8_t* __restrict__ sel,
    const int64_t* __restrict__ cnt, unsigned long long* __restrict__ newcnt, uint8_t* __restrict__ fail,
    unsigned long long* __restrict__ need, int64_t close0, uint64_t* __restrict__ closed,
    unsigned long long* __restrict__ closed_n, const int64_t* __restrict__ ci, unsigned long long* __restrict__ hnew,
    unsigned long long* __restrict__ hclosed, uint32_t* __restrict__ prn, unsigned long long* __restrict__ dbg) {
  if (ci_ld(ci, CI_GATE) == 0) return;
  if ((ci_ld(ci, CI_ID32) != 0) != (sizeof(ID) == 4)) return;  // the other identity width's
  const C1VQ& q = *qp;  // in device memory: its fields are loaded where used (SGPR pressure)
  constexpr int NW = NT / 64;
  constexpr ID EMPTY = (ID)~(ID)0;
  const int log2H = q.log2H;
  const int H = 1 << log2H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  KLDS ID* ids = (KLDS ID*)(KLDS char*)smem;
  KLDS uint32_t* rt = c1v_plane<uint32_t>(smem, q.off_rt);
  KLDS uint16_t* list = c1v_plane<uint16_t>(smem, q.off_list);
  KLDS uint64_t* sg2 = c1v_plane<uint64_t>(smem, q.off_spre);  // as k_c1_merge's
  KLDS uint16_t* segof = (KLDS uint16_t*)(sg2 + C1_SEGMAX + 4);
  // the bucket tables (chunk starts, bucket bases) are read from memory per item (their 3 KB of
  // LDS let a 2^12-entry table of 32-bit identities fit two workgroups per CU)
  __shared__ int lovf, nnew;
  __shared__ int wsum[NW], csum[NW];
  __shared__ unsigned long long lbase, cbase;
  const int F = 1 << q.fbits;
  const int64_t wbase = ci_ld(ci, CI_WBASE), whi = ci_ld(ci, CI_WHI), T0 = ci_ld(ci, CI_T0), tmin = ci_ld(ci, CI_TMIN);
  const int wbits = (int)ci_ld(ci, CI_WBITS);
  const int64_t kmin = ci_ld(ci, CI_KMINC);
  const uint64_t krange = (uint64_t)ci_ld(ci, CI_KRANGE);
  const int32_t tmin32 = (int32_t)(tmin - T0);
  const int64_t wstart = wbase * q.adv;
  const bool r32 = ci_ld(ci, CI_TMAX) - wstart < ((int64_t)1 << 32);
  const uint32_t tsh32 = (uint32_t)(T0 - wstart);
  const bool evict = close0 != INT64_MIN;
  C1M_T0;
  const uint32_t dummy = (uint32_t)H + (uint32_t)lane;
  for (int i = threadIdx.x; i < H + 64; i += NT) {
    ids[i] = EMPTY;
    c1v_clear<PM>(q, smem, i);
  }
  if (threadIdx.x == 0) {
    lovf = 0;
    nnew = 0;
  }
  // identity and slot hash of a resident row (false: no record of this push can match it).
  // Sub-passes split a partition by KEY (subh): a pane and its windows stay in one sub-pass.
  auto row_id = [&](const uint64_t* row, ID* id, uint32_t* h) -> bool {
    const int64_t wi = (int64_t)fast_udiv((uint64_t)row[1], q.fd) - wbase;
    const uint64_t krel = (uint64_t)((int64_t)row[0] - kmin);
    if (krel > krange || wi < 0 || wi > whi) return false;
    *id = c1v_id<ID, PANES>(krel, (uint64_t)wi, false, wbits);
    *h = c1_hash<ID>(*id);
    return true;
  };
  auto subh = [&](int64_t key) -> uint32_t { return (uint32_t)(uint64_t)(key - kmin) * 0x9E3779B1u; };
  // probe for id from its home slot; claims it if absent (listed); -1 when the table is full
  auto claim = [&](ID id, bool act) -> int {
    uint32_t e = act ? c1_hash<ID>(id) >> (32 - log2H) : dummy;
    ID old = EMPTY;
    __hip_atomic_compare_exchange_strong(&ids[e], &old, act ? id : EMPTY, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_WORKGROUP);
    bool got = act && old == EMPTY;
    bool pend = act && old != EMPTY && old != id;
    for (int probes = 1;; probes++) {
      if (!__ballot(pend)) break;
      if (probes >= H) {  // the table is full: the item is retried (claimed entries stay listed)
        if (pend) {
          lovf = 1;
          act = false;
        }
        pend = false;
        break;
      }
      if (pend) {
        e = (e + 1) & (uint32_t)(H - 1);
        ID o2 = EMPTY;
        __hip_atomic_compare_exchange_strong(&ids[e], &o2, id, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP);
        got = o2 == EMPTY;
        pend = o2 != EMPTY && o2 != id;
      }
    }
    mg_list_append(act && got, e, list, &nnew);
    return act ? (int)e : -1;
  };
  struct Pre {
    uint32_t p;
    int sbits, sub, nseg;
    int64_t nrow, bb0;
    uint32_t selw;
    uint16_t s00, s01, s10, s11;
  };
  struct It {
    uint32_t p;
    int sbits, sub, nseg, segb;  // segb: log2 of the records per segment-lookup block
    int64_t rn, nrow;
    bool isel;
  };
  auto fetch = [&](int64_t w, Pre& r) {
    uint32_t p;
    int sbits = 0, sub = 0;
    if (work) {
      const uint32_t x = work[w];
      p = x & 0xFFFFu;
      sbits = (x >> 16) & 0xF;
      sub = (int)(x >> 20);
    } else {
      p = (uint32_t)w;
    }
    p = __builtin_amdgcn_readfirstlane(p);
    const int b = (int)(p >> q.fbits), f = (int)(p & (uint32_t)(F - 1));
    const int cs = cstart[b];
    int nseg = cstart[b + 1] - cs;
    if (nseg < 0 || nseg > C1_SEGMAX) nseg = 0;
    r.p = p;
    r.sbits = sbits;
    r.sub = sub;
    r.nseg = nseg;
    r.nrow = cnt[p];
    r.selw = ((const uint32_t*)sel)[p >> 2];
    r.bb0 = bb[b];
    const int k0 = threadIdx.x * 2;
    r.s00 = r.s01 = r.s10 = r.s11 = 0;
    if (k0 < nseg) {
      const uint16_t* sg = seg + (int64_t)(cs + k0) * (F + 1) + f;
      r.s00 = sg[0];
      r.s01 = sg[1];
    }
    if (k0 + 1 < nseg) {
      const uint16_t* sg = seg + (int64_t)(cs + k0 + 1) * (F + 1) + f;
      r.s10 = sg[0];
      r.s11 = sg[1];
    }
  };
  auto prep = [&](const Pre& r, It& it) {
    const int nseg = r.nseg;
    it.p = r.p;
    it.sbits = r.sbits;
    it.sub = r.sub;
    it.nseg = nseg;
    it.nrow = r.nrow;
    it.isel = ((r.selw >> (8 * (r.p & 3))) & 0xFFu) != 0;
    const int k0 = threadIdx.x * 2;
    const int len0 = k0 < nseg ? (int)r.s01 - (int)r.s00 : 0;
    const int len1 = k0 + 1 < nseg ? (int)r.s11 - (int)r.s10 : 0;
    const int64_t base0 = r.bb0 + (int64_t)k0 * C1V_CH + r.s00;
    const int64_t base1 = r.bb0 + (int64_t)(k0 + 1) * C1V_CH + r.s10;
    const int s = len0 + len1;
    int incl = s;
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(incl, off, 64);
      if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    lds_barrier();
    int before = 0;
    int tot = 0;
    for (int k = 0; k < NW; k++) {
      before += k < wave ? wsum[k] : 0;
      tot += wsum[k];
    }
    const int ex = before + incl - s;
    // the finest lookup block that covers the item in C1_SEGOF entries (segments hold C1_CH / F
    // records on average: 32-record blocks make the lookup a read and at most a step or two)
    const int segb = tot <= (C1_SEGOF << 5) ? 5 : (tot <= (C1_SEGOF << 6) ? 6 : C1_SEGB);
    const int bm = (1 << segb) - 1;
    if (k0 < nseg) {
      sg2[k0] = (uint32_t)ex | (uint64_t)(uint32_t)(int32_t)(base0 - ex) << 32;
    }
    if (k0 + 1 < nseg) {
      sg2[k0 + 1] = (uint32_t)(ex + len0) | (uint64_t)(uint32_t)(int32_t)(base1 - (ex + len0)) << 32;
    }
    // segment lookup: block j (records [j << segb, (j + 1) << segb)) starts in segment segof[j]
    for (int bj = (ex + bm) >> segb, be = (ex + len0 + bm) >> segb; bj < be && bj < C1_SEGOF; bj++)
      segof[bj] = (uint16_t)k0;
    for (int bj = (ex + len0 + bm) >> segb, be = (ex + s + bm) >> segb; bj < be && bj < C1_SEGOF; bj++)
      segof[bj] = (uint16_t)(k0 + 1);
    if (k0 < nseg && k0 + 2 >= nseg) sg2[nseg] = (uint32_t)(ex + s);
    if (nseg == 0 && threadIdx.x == 0) sg2[0] = 0u;
    lds_barrier();
    it.rn = (uint32_t)sg2[nseg];
    it.segb = segb;
  };
  ulonglong2 ra[AU], rb[AU];
  auto load = [&](ulonglong2 (&x)[AU], int64_t l0, int64_t rn, int nseg, int segb) {
#pragma unroll
    for (int u = 0; u < AU; u++) {
      int64_t li = l0 + threadIdx.x + (int64_t)u * NT;
      li = li < rn ? li : rn - 1;
      int lo = 0;  // the last segment starting at or before li
      int64_t at;
      if (rn <= ((int64_t)C1_SEGOF << segb)) {  // from the block's segment, a step or two on
        lo = segof[li >> segb];
        uint64_t sa = sg2[lo], sb = sg2[lo + 1];
        while (lo + 1 < nseg && (int64_t)(uint32_t)sb <= li) {
          lo++;
          sa = sb;
          sb = sg2[lo + 1];
        }
        at = (int64_t)(int32_t)(sa >> 32) + li;
      } else {
        int hi = nseg;
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if ((int64_t)(uint32_t)sg2[mid] <= li) lo = mid;
          else hi = mid;
        }
        at = (int64_t)(int32_t)(sg2[lo] >> 32) + li;
      }
      x[u] = ld_nt2(srec + at);
    }
  };
  auto load01 = [&](const It& x) {
    if (x.rn > 0) load(ra, 0, x.rn, x.nseg, x.segb);
    if (x.rn > (int64_t)AU * NT) load(rb, (int64_t)AU * NT, x.rn, x.nseg, x.segb);
  };
  lds_barrier();  // the table and flags initialised above
  Pre pr{};
  It nx{};
  if (blockIdx.x < nwork) {
    fetch(blockIdx.x, pr);
    prep(pr, nx);
    load01(nx);
  }
  for (int64_t w = blockIdx.x; w < nwork; w += gridDim.x) {
    const It it = nx;
    const uint32_t p = it.p;
    const int sbits = it.sbits, sub = it.sub, nseg = it.nseg, segb = it.segb;
    const int64_t rn = it.rn, nrow = it.nrow;
    const bool isel = it.isel;
    const int64_t wn = w + gridDim.x;
    if (wn < nwork) fetch(wn, pr);
    if (first && threadIdx.x == 0) prn[p] = (uint32_t)rn;
    if (rn == 0 && first) {
      if (wn < nwork) {
        prep(pr, nx);
        load01(nx);
      }
      continue;
    }
    const uint64_t* src = (isel ? buf1 : buf0) + (uint64_t)p * q.cmax * q.sw;
    // (closed resident rows leave for the closed store in the write-out, phase 4: one pass over the
    // resident rows there, the closed store's slots reserved with the region's)
    C1M_T(0);
    // 1. records → their pane (window) entries: the AU identities' CASes back to back, then the
    //    collisions probe on together (as k_c1_merge)
    //    The set's next chunk is loaded into the same registers right after the CASes are issued
    //    (prefetch; what the planes need is kept aside first), as k_c1_merge.
    auto apply = [&](const ulonglong2 (&xr)[AU], int64_t l0, auto R32, auto&& prefetch) -> bool {
      ID id[AU];
      uint32_t e[AU], trv[AU];
      uint64_t arg[AU];
      bool pend[AU], claimed[AU], nn[AU];
#pragma unroll
      for (int u = 0; u < AU; u++) {
        const int64_t li = l0 + threadIdx.x + (int64_t)u * NT;
        const uint64_t w0 = xr[u].x;
        trv[u] = (uint32_t)((int32_t)(uint32_t)w0 - tmin32) + 1u;
        nn[u] = (w0 >> 63) != 0;
        arg[u] = xr[u].y;
        const uint64_t krel = (w0 >> 32) & 0x7FFFFFFFull;
        uint64_t wi;
        if constexpr (decltype(R32)::value) wi = fast_udiv32((uint32_t)w0 + tsh32, q.fd32);
        else wi = fast_udiv((uint64_t)(T0 + (int64_t)(int32_t)(uint32_t)w0), q.fd) - (uint64_t)wbase;
        const ID x = c1v_id<ID, PANES>(krel, wi, PANES, wbits);
        bool act = li < rn;
        if (sbits) act = act && (int)c1_sub((uint32_t)krel * 0x9E3779B1u, sbits) == sub;
        id[u] = act ? x : EMPTY;
        e[u] = act ? c1_hash<ID>(x) >> (32 - log2H) : dummy;
      }
      ID old[AU];
#pragma unroll
      for (int u = 0; u < AU; u++) {
        old[u] = EMPTY;
        __hip_atomic_compare_exchange_strong(&ids[e[u]], &old[u], id[u], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      const int full = *(volatile KLDS int*)&lovf;
      prefetch();
#pragma unroll
      for (int u = 0; u < AU; u++) {
        claimed[u] = id[u] != EMPTY && old[u] == EMPTY;
        pend[u] = old[u] != EMPTY && old[u] != id[u];
      }
      for (int probes = 1;; probes++) {
        bool anyp = false;
#pragma unroll
        for (int u = 0; u < AU; u++) anyp |= pend[u];
        if (!__ballot(anyp)) break;
        if (probes >= H) {
          lovf = 1;
#pragma unroll
          for (int u = 0; u < AU; u++)
            if (pend[u]) id[u] = EMPTY;
          break;
        }
#pragma unroll
        for (int u = 0; u < AU; u++) {
          if (!pend[u]) continue;
          e[u] = (e[u] + 1) & (uint32_t)(H - 1);
          ID o2 = EMPTY;
          __hip_atomic_compare_exchange_strong(&ids[e[u]], &o2, id[u], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
          claimed[u] = o2 == EMPTY;
          pend[u] = o2 != EMPTY && o2 != id[u];
        }
      }
      int nnow;
      {
        bool cl[AU];
#pragma unroll
        for (int u = 0; u < AU; u++) cl[u] = claimed[u] && id[u] != EMPTY;
        nnow = mg_list_append_n<AU>(cl, e, list, &nnew);
      }
#pragma unroll
      for (int u = 0; u < AU; u++) {
        if (id[u] == EMPTY) continue;
        int64_t ok_ = (int64_t)arg[u];
        if (C1VP<PM>{q}.f64() && (C1VP<PM>{q}.mn() || C1VP<PM>{q}.mx())) {
          double d;
          __builtin_memcpy(&d, &arg[u], 8);
          ok_ = f64_order_key(d);
        }
        c1v_add<PM>(q, smem, e[u], trv[u], 1u, nn[u] ? 1u : 0u, arg[u], ok_, ok_);
      }
      return !full && nnow <= q.hmax;
    };
    const int64_t nch = (rn + (int64_t)AU * NT - 1) / ((int64_t)AU * NT);
    if (rn > 0 && PANES) {
      // HOPPING items run many chunks (C3: ~8): a straight-line body (a chunk past the end applies
      // nothing; its loads, clamped to the last record, read one line) whose wait for one register
      // set counts the other set's loads as in flight; the table-full check once per two chunks
      auto records = [&](auto R32) {
        for (int64_t c = 0; c < nch; c += 2) {
          const bool ga = apply(ra, c * AU * NT, R32, [&] { load(ra, (c + 2) * AU * NT, rn, nseg, segb); });
          const bool gb = apply(rb, (c + 1) * AU * NT, R32, [&] { load(rb, (c + 3) * AU * NT, rn, nseg, segb); });
          if (!ga || !gb) break;
        }
      };
      if (r32) records(std::true_type{});
      else records(std::false_type{});
    } else if (rn > 0) {
      for (int64_t c = 0; c < nch; c += 2) {
        auto pa = [&] { if (c + 2 < nch) load(ra, (c + 2) * AU * NT, rn, nseg, segb); };
        const bool ga = r32 ? apply(ra, c * AU * NT, std::true_type{}, pa) : apply(ra, c * AU * NT, std::false_type{}, pa);
        if (!ga || c + 1 >= nch) break;
        auto pb = [&] { if (c + 3 < nch) load(rb, (c + 3) * AU * NT, rn, nseg, segb); };
        const bool gb = r32 ? apply(rb, (c + 1) * AU * NT, std::true_type{}, pb)
                            : apply(rb, (c + 1) * AU * NT, std::false_type{}, pb);
        if (!gb) break;
      }
    }
    lds_barrier();
    if (wn < nwork) {
      prep(pr, nx);
      load01(nx);
    }
    C1M_T(1);
    // 1b. panes → their windows (the window entries are claimed as a record's would be)
    if (PANES && q.fan > 1 && !lovf && nnew <= q.hmax) {
      const int nn0 = nnew;
      lds_barrier();  // every thread has read nn0 before the fold lists windows
      for (int i0 = 0; i0 < nn0; i0 += NT) {  // uniform trip count: claim's ballots converge
        const int li = i0 + threadIdx.x;
        const int pe = li < nn0 ? (int)list[li] : 0;
        const ID pid = li < nn0 ? ids[pe] : EMPTY;
        const bool isp = li < nn0 && pid != EMPTY && c1v_is_pane<ID, PANES>(pid, wbits);
        uint64_t krel, pw;
        if constexpr (sizeof(ID) == 4) {
          krel = (uint64_t)((uint32_t)pid >> (wbits + 1));
          pw = (uint64_t)((uint32_t)pid & ((1u << wbits) - 1u));
          if (wbits == 0) pw = 0;
        } else {
          krel = (uint64_t)pid >> 32;
          pw = (uint64_t)pid & 0x7FFFFFFFull;
        }
        const uint32_t prt = isp ? rt[pe] : 0u;
        const C1VP<PM> pv{q};
        const uint32_t pcs = isp && pv.star() ? c1v_plane<uint32_t>(smem, q.off_star)[pe] : 0u;
        const uint32_t pcv = isp && pv.cnt() ? c1v_plane<uint32_t>(smem, q.off_cnt)[pe] : (isp ? 1u : 0u);
        const uint64_t psum = isp && pv.sum() ? c1v_plane<uint64_t>(smem, q.off_sum)[pe] : 0ULL;
        const int64_t pmn = isp && pv.mn() ? c1v_plane<int64_t>(smem, q.off_min)[pe] : INT64_MAX;
        const int64_t pmx = isp && pv.mx() ? c1v_plane<int64_t>(smem, q.off_max)[pe] : INT64_MIN;
        for (int j = 0; j < q.fan; j++) {
          // window pw - j (its start is >= 0: windowsFor never returns a negative start)
          const bool act = isp && (int64_t)pw - j + wbase >= 0 && (int64_t)pw - j >= 0;
          const int e = claim(c1v_id<ID, PANES>(krel, pw - (uint64_t)j, false, wbits), act);
          if (e >= 0) c1v_add<PM>(q, smem, (uint32_t)e, prt, pcs, pcv, psum, pmn, pmx);
        }
      }
      lds_barrier();
    }
    C1M_T(2);
    const int nl = nnew < H ? nnew : H;
    if (lovf || nnew > q.hmax) {
      if (threadIdx.x == 0) fail[p] |= 1;
      for (int i = threadIdx.x; i < nl; i += NT) {
        const uint32_t e = list[i];
        ids[e] = EMPTY;
        c1v_clear<PM>(q, smem, (int)e);
      }
      lds_barrier();
      if (threadIdx.x == 0) {
        lovf = 0;
        nnew = 0;
      }
      lds_barrier();
      continue;
    }
    // 2. resident rows: mark the delta entries they absorb; count live and closed rows
    int n_mine = 0, n_cl = 0;
    for (int64_t r = threadIdx.x; r < nrow; r += NT) {
      const uint64_t* row = src + r * q.sw;
      if (sbits && (int)c1_sub(subh((int64_t)row[0]), sbits) != sub) continue;
      if (evict && (int64_t)row[1] + q.size <= close0) {
        n_cl++;
        continue;
      }
      ID id;
      uint32_t h;
      const bool has = row_id(row, &id, &h);
      if (has) {
        const int e = c1_find_id<ID>(ids, id, h >> (32 - log2H), H);
        if (e >= 0) rt[e] |= RT_MATCHED;
      }
      n_mine++;
    }
    if (nrow > 0) lds_barrier();  // the marks before the list walk reads them (uniform: nrow is the item's)
    const int per = ((nl + NW - 1) / NW + 63) & ~63;
    const int lb0 = wave * per, lb1 = lb0 + per < nl ? lb0 + per : nl;
    int nnw = 0;
    for (int k = lb0; k < lb1; k += 64) {
      const int i = k + lane;
      const uint32_t e = i < lb1 ? list[i] : dummy;
      const bool isnew = i < lb1 && !(rt[e] & RT_MATCHED) && !c1v_is_pane<ID, PANES>(ids[e], wbits);
      nnw += (int)__popcll(__ballot(isnew));
    }
    // 3. the partition's region range, and the closed store's slots for its closed rows
    const int wave_rows = (int)wave_sum(n_mine) + nnw;
    const int wave_cl = (int)wave_sum(n_cl);
    if (lane == 0) {
      wsum[wave] = wave_rows;
      csum[wave] = wave_cl;
    }
    lds_barrier();
    int wave_before = 0, total = 0, cl_before = 0, cl_total = 0;
    for (int k = 0; k < NW; k++) {
      if (k < wave) wave_before += wsum[k], cl_before += csum[k];
      total += wsum[k];
      cl_total += csum[k];
    }
    if (threadIdx.x == 0) {
      if (work) lbase = total ? atomicAdd(&newcnt[p], (unsigned long long)total) : 0ULL;
      else {
        lbase = 0;
        newcnt[p] = (unsigned long long)total;
      }
      // (an item that does not fit its region is retried and reserves nothing here)
      cbase = cl_total && (int64_t)(lbase + total) <= q.cmax ? atomicAdd(closed_n, (unsigned long long)cl_total) : 0ULL;
    }
    lds_barrier();
    if ((int64_t)(lbase + total) > q.cmax) {
      if (threadIdx.x == 0) {
        fail[p] |= 2;
        atomicMax(need, (unsigned long long)(lbase + total));
      }
      for (int i = threadIdx.x; i < nl; i += NT) {
        const uint32_t e = list[i];
        ids[e] = EMPTY;
        c1v_clear<PM>(q, smem, (int)e);
      }
      lds_barrier();
      if (threadIdx.x == 0) nnew = 0;
      lds_barrier();
      continue;
    }
    C1M_T(3);
    // 4. write: resident rows (merged; closed ones to the closed store), then the wave's new window
    //    entries
    uint64_t* dst0 = (isel ? buf0 : buf1) + (uint64_t)p * q.cmax * q.sw;
    uint64_t cur = lbase + (uint64_t)wave_before;
    uint64_t ccur = cbase + (uint64_t)cl_before;
    const uint64_t lt = (1ULL << lane) - 1;
    int nh = 0, nhc = 0;
    for (int64_t r0 = wave * 64; r0 < nrow; r0 += NT) {
      const int64_t r = r0 + lane;
      const uint64_t* row = src + (r < nrow ? r : 0) * q.sw;
      const bool mine = r < nrow && (!sbits || (int)c1_sub(subh((int64_t)row[0]), sbits) == sub);
      const bool cl = mine && evict && (int64_t)row[1] + q.size <= close0;
      const bool live = mine && !cl;
      int e = -1;
      if (live) {
        ID id;
        uint32_t h;
        if (row_id(row, &id, &h)) e = c1_find_id<ID>(ids, id, h >> (32 - log2H), H);
      }
      const uint64_t bc = __ballot(cl);
      if (cl) {  // (the query's HAVING alone: the merge's copy never carries pull / retention / FINAL bounds)
        uint64_t* cd = closed + (ccur + __popcll(bc & lt)) * q.sw;
        for (int k = 0; k < q.sw; k++) cd[k] = row[k];
        nhc += having_ok_words(q.having.a.w_val >= 0 ? row[q.having.a.w_val] : 0,
                               q.having.a.w_cnt >= 0 ? row[q.having.a.w_cnt] : 0, q.having) ? 1 : 0;
      }
      ccur += __popcll(bc);
      const uint64_t bl = __ballot(live);
      if (live) {
        const uint64_t ri = cur + __popcll(bl & lt);
        uint64_t* dst = dst0 + ri * q.sw;
        bool was, now;
        const int64_t t = e >= 0 ? tmin + (int64_t)(rt[e] & ~RT_MATCHED) - 1 : 0;
        c1v_emit<PM>(q, smem, dst, row, e, 0, 0, t, &was, &now);
        nh += q.having.active && now ? 1 : 0;
        if (q.chg)
          q.chg[(uint64_t)p * q.cmax + ri] =
              e >= 0 ? (uint8_t)(CHG_TOUCHED | (was ? CHG_OLD : 0) | (now ? CHG_NEW : 0)) : (uint8_t)0;
      }
      cur += __popcll(bl);
    }
    if (nrow > 0) lds_barrier();  // the resident rows have read their entries before the walk clears them
    const uint32_t wmask = wbits ? (1u << wbits) - 1u : 0u;
    for (int k = lb0; k < lb1; k += 64) {
      const int i = k + lane;
      const uint32_t e = i < lb1 ? list[i] : dummy;
      const uint32_t rv = rt[e];
      const ID id = ids[e];
      const bool isnew = i < lb1 && !(rv & RT_MATCHED) && !c1v_is_pane<ID, PANES>(id, wbits);
      const uint64_t bl = __ballot(isnew);
      if (isnew) {
        const uint64_t ri = cur + __popcll(bl & lt);
        uint64_t* dst = dst0 + ri * q.sw;
        int64_t key, wi;
        if constexpr (sizeof(ID) == 4) {
          key = kmin + (int64_t)((uint32_t)id >> (wbits + (PANES ? 1 : 0)));
          wi = (int64_t)((uint32_t)id & wmask);
        } else {
          key = kmin + (int64_t)((uint64_t)id >> 32);
          wi = (int64_t)((uint64_t)id & 0x7FFFFFFFull);
        }
        bool was, now;
        c1v_emit<PM>(q, smem, dst, nullptr, (int)e, key, (wbase + wi) * q.adv, tmin + (int64_t)rv - 1, &was, &now);
        nh += q.having.active && now ? 1 : 0;
        if (q.chg) q.chg[(uint64_t)p * q.cmax + ri] = (uint8_t)(CHG_TOUCHED | (now ? CHG_NEW : 0));
      }
      if (i < lb1) {
        ids[e] = EMPTY;
        c1v_clear<PM>(q, smem, (int)e);
      }
      cur += __popcll(bl);
    }
    if (q.having.active) {
      nh = (int)wave_sum(nh);
      nhc = (int)wave_sum(nhc);
      if (lane == 0 && nh) atomicAdd(&hnew[p], (unsigned long long)nh);
      if (lane == 0 && nhc) atomicAdd(hclosed, (unsigned long long)nhc);
    }
    lds_barrier();
    C1M_T(4);
    if (threadIdx.x == 0) nnew = 0;
    lds_barrier();
  }
}

// ------------------------------------------------------------------ host side

size_t c1_merge_lds(int log2H, int idw, int log2B) {
  const size_t H = (size_t)1 << log2H, B = (size_t)1 << log2B;
  return (H + 64) * (idw + 8) + ((H * 2 + 15) & ~(size_t)15) + (C1_SEGMAX + 4) * 8 + (B + 1) * 12 + 8 +
         C1_SEGOF * 2;  // (segment table: 8 B per entry, both layouts fit)
}

// Whether the COUNT(*) pipeline may take this push (the general path's c1 plan, TUMBLING, the
// two-level partition layout).  The push may still be declined on the device (k_c1_check).
bool c1_eligible(khip_agg* a, int64_t n) {
  PartState& s = a->part;
  const bool cnt1 = a->ap.n_ops == 1 && a->ap.ops[0].kind == OP_INC && a->ap.ops[0].word == 3 && a->sw == 4 &&
                    s.rw == 2;
  return cnt1 && a->windowed && a->desc.window_kind == KHIP_WINDOW_TUMBLING && s.log2P >= 11 && s.log2P <= 16 &&
         s.mH >= 256 && a->desc.advance_ms <= ((int64_t)1 << 31) && !(a->desc.flags & KHIP_FLAG_PART_CLAIM) &&
         n > 0 && n < ((int64_t)1 << 31) && knob("KHIP_C1P", 1) != 0 && knob("KHIP_PAD", 0) == 0 &&
         knob("KHIP_MERGE", 1) != 0 && knob("KHIP_SCATTER2", 1) != 0;
}

// The value pipeline: every update op reads one argument column (or is COUNT(*)), at most one op
// per kind, TUMBLING or HOPPING with size a multiple of the advance (panes), rows of <= 8 words.
// *col = the argument column.
bool c1v_eligible(khip_agg* a, int64_t n, int* col) {
  PartState& s = a->part;
  if (!a->windowed || a->sw > C1V_MAXW || a->ap.n_ops < 1 || s.rw < 2) return false;
  const int64_t size = a->desc.size_ms, adv = a->desc.advance_ms;
  if (a->desc.window_kind == KHIP_WINDOW_HOPPING) {
    if (size % adv != 0 || size / adv > 16) return false;
  } else if (a->desc.window_kind != KHIP_WINDOW_TUMBLING) {
    return false;
  }
  int c = -1, seen = 0;
  for (int o = 0; o < a->ap.n_ops; o++) {
    const UpdOp op = a->ap.ops[o];
    if (op.kind < OP_INC || op.kind > OP_MAX || op.word < 3 || op.word >= a->sw) return false;
    const int bit = op.kind == OP_ADD_F64 ? (1 << OP_ADD_I64) : (1 << op.kind);
    if (seen & bit) return false;
    seen |= bit;
    if (op.kind == OP_INC) continue;
    if (c >= 0 && op.col != c) return false;
    c = op.col;
  }
  if (c < 0) return false;  // COUNT(*) alone: the COUNT(*) pipeline's
  const int t = a->ap.col_type[c];
  if (t != KHIP_TYPE_INT32 && t != KHIP_TYPE_INT64 && t != KHIP_TYPE_DOUBLE) return false;
  *col = c;
  return s.log2P >= 11 && s.log2P <= 16 && s.mH >= 256 && adv <= ((int64_t)1 << 31) &&
         !(a->desc.flags & KHIP_FLAG_PART_CLAIM) && n > 0 && n < ((int64_t)1 << 31) && knob("KHIP_C1V", 1) != 0 &&
         knob("KHIP_PAD", 0) == 0 && knob("KHIP_MERGE", 1) != 0 && knob("KHIP_SCATTER2", 1) != 0;
}

// Dynamic LDS of a value merge that still fits two workgroups per CU (160 KB, less the kernel's
// static LDS).
constexpr size_t C1V_LDS2 = 80 * 1024 - 256;

// LDS layout of k_c1v_merge (byte offsets into q); returns the bytes.
static size_t c1v_layout(khip_agg* a, int log2H, int idw, int log2B, C1VQ* q) {
  const size_t E = ((size_t)1 << log2H) + 64, H = (size_t)1 << log2H, B = (size_t)1 << log2B;
  size_t off = E * idw;
  off = (off + 7) & ~(size_t)7;
  q->off_sum = q->off_min = q->off_max = q->off_star = q->off_cnt = -1;
  for (int o = 0; o < a->ap.n_ops; o++) {
    const int k = a->ap.ops[o].kind;
    if (k == OP_ADD_I64 || k == OP_ADD_F64) q->off_sum = 1;
    if (k == OP_MIN) q->off_min = 1;
    if (k == OP_MAX) q->off_max = 1;
    if (k == OP_INC) q->off_star = 1;
    if (k == OP_INC_VALID) q->off_cnt = 1;
  }
  auto place = [&](int32_t* f, size_t bytes) {
    if (*f < 0) return;
    *f = (int32_t)off;
    off += E * bytes;
  };
  place(&q->off_sum, 8);
  place(&q->off_min, 8);
  place(&q->off_max, 8);
  q->off_rt = (int32_t)off;
  off += E * 4;
  place(&q->off_star, 4);
  place(&q->off_cnt, 4);
  off = (off + 15) & ~(size_t)15;
  q->off_list = (int32_t)off;
  off += (H * 2 + 15) & ~(size_t)15;
  q->off_spre = (int32_t)off;
  off += (C1_SEGMAX + 4) * 8 + C1_SEGOF * 2;
  (void)B;
  return off;
}

// Returns KHIP_OK with *declined = true when k_c1_check declined the push (nothing persistent was
// touched: the caller runs the general path on the same batch).
// cols != nullptr: the value pipeline over argument column vcol (c1v_eligible).
khip_status c1_push(khip_agg* a, int64_t n, const int64_t* keys, const int64_t* ts, const uint8_t* kv,
                    const uint8_t* rv, int64_t* tot, bool* declined, const int64_t* st_at, bool* retry_wide,
                    const ColPtrs* cols, int vcol, const RowsIn* rows) {
  PartState& s = a->part;
  *declined = false;
  *retry_wide = false;
  const bool val = cols != nullptr || rows != nullptr;
  const bool panes = val && a->desc.window_kind == KHIP_WINDOW_HOPPING;
  const int pbits = panes ? 1 : 0;
  const int CH = val ? C1V_CH : C1_CH;
  constexpr int UV = 4;  // value scatter: records per thread per step
  const int P = (int)s.P;
  const int fbits = s.log2P - s.log2P / 2;
  const int log2B = s.log2P - fbits;
  const int B = 1 << log2B, F = 1 << fbits;
  const int64_t nT = ceil_div(n, C1_TILE);
  const int64_t S = val ? (int64_t)UV * C1_NT : (int64_t)8 * C1_NT;  // scatter step (records)
  const int64_t nSt = nT * (C1_TILE / S);                             // steps (runs per bucket)
  const int64_t nchunk_max = ceil_div(n, CH) + B;
  KHIP_TRY(s.c1rc.ensure((size_t)B * nSt * 4));
  KHIP_TRY(s.c1rp.ensure(((size_t)B * nSt + 1) * 4));
  KHIP_TRY(s.c1ro.ensure((size_t)B * nSt * 2));
  KHIP_TRY(s.c1bb.ensure((size_t)(B + 1) * 8));
  const size_t seg_bytes = ((size_t)nchunk_max * (F + 1) * 2 + 255) & ~(size_t)255;  // cstart 256-B aligned
  KHIP_TRY(s.c1seg.ensure(seg_bytes + (size_t)(B + 1) * 4));
  KHIP_TRY(s.tilemax.ensure(nT * 32));  // per tile: stream-time max, smallest ts, late bound, ok
  KHIP_TRY(s.tpart.ensure(nT * 8 * T_NPART));
  KHIP_TRY(s.prn.ensure((size_t)P * 4));
  KHIP_TRY(s.res.ensure(16));
  KHIP_TRY(s.closed_ctr.ensure(8));
  if (s.scat_cap < n) {
    KHIP_TRY(s.srec.ensure((size_t)(n + 1) * s.rw * 8));
    s.scat_cap = n;
  }
  KHIP_TRY(s.srec.ensure((size_t)(n + 1) * 16));  // (s.rw >= 2: no-ops)
  KHIP_TRY(s.srecA.ensure((size_t)(n + 1) * std::max(s.rw, 2) * 8));
  if (!s.c1info.p) {
    KHIP_TRY(s.c1info.ensure(CI_N * 8));
    int64_t init[CI_N] = {};
    init[CI_KMIN] = INT64_MAX;
    init[CI_KMAX] = INT64_MIN;
    KHIP_TRY_HIP(hipMemcpy(s.c1info.p, init, sizeof(init), hipMemcpyHostToDevice));
  }
  int64_t* ci = s.c1info.as<int64_t>();
#ifdef KHIP_TUNING
  {
    const int64_t dbg = knob("KHIP_C1_DEBUG", 0);
    KHIP_TRY_HIP(hipMemcpyAsync(ci + CI_N - 1, &dbg, 8, hipMemcpyHostToDevice, a->stream));
    KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  }
#endif
  int* cstart = (int*)(s.c1seg.as<char>() + seg_bytes);
  uint16_t* seg = s.c1seg.as<uint16_t>();
  const int64_t adv = a->desc.advance_ms;
  const FastDiv fd = make_fastdiv(adv);
  const int64_t close0 = a->host_stream_time >= 0 ? a->host_stream_time - a->grace : INT64_MIN;
  if (s.closed_cap < s.closed_n + (a->occ - s.closed_n)) {  // worst case every live row closes in this push
    const int64_t live = a->occ - s.closed_n;
    const int64_t ncap = next_pow2(std::max<int64_t>(1024, s.closed_n + live));
    DevBuf nc;
    KHIP_TRY(nc.ensure((size_t)ncap * a->sw * 8));
    if (s.closed_n)
      KHIP_TRY_HIP(hipMemcpyAsync(nc.p, s.closed.p, (size_t)s.closed_n * a->sw * 8, hipMemcpyDeviceToDevice, a->stream));
    KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
    s.closed.release();
    s.closed = std::move(nc);
    nc.p = nullptr;
    s.closed_cap = ncap;
  }
  // wide records (key hash + u32 ts words) when the key range did not fit 32 bits last time: the
  // host predicts the format, k_c1_check declines a compact push whose keys do not fit
  const bool wide = !val && s.c1_wide;
  uint32_t* srecAT = (uint32_t*)(s.srecA.as<uint64_t>() + n + 1);  // WIDE ts words (12 B/record in all)
  uint32_t* srecT = (uint32_t*)(s.srec.as<uint64_t>() + n + 1);
  uint32_t* rc = s.c1rc.as<uint32_t>();
  uint32_t* rp = s.c1rp.as<uint32_t>();
  uint16_t* ro = s.c1ro.as<uint16_t>();
  const int has_kb = s.c1_kb_valid ? 1 : 0;
  // 1. records → step runs (the key range, time base and bucket counts in the same read)
  ev_record_part(a, 0);
  if (val) {
    const C1VCol vc{rows ? nullptr : cols->data[vcol], rows ? nullptr : cols->valid[vcol], a->ap.col_type[vcol]};
    const RowsIn ri = rows ? *rows : RowsIn{};
    auto sk = rows ? (st_at ? k_c1v_scatter<UV, C1_NT, true, true> : k_c1v_scatter<UV, C1_NT, false, true>)
                   : (st_at ? k_c1v_scatter<UV, C1_NT, true, false> : k_c1v_scatter<UV, C1_NT, false, false>);
    const size_t lds = run_stage_lds(B, UV * C1_NT, 16, false) + run_cnt_lds(B, C1_TILE / (UV * C1_NT));
    if (lds > 64 * 1024) hipFuncSetAttribute((const void*)sk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(sk, dim3(nT), dim3(C1_NT), lds, a->stream, keys, ts, kv, rv, vc, ri, n, nT, log2B, rc, ro, nSt,
                       (ulonglong2*)s.srecA.p, s.tilemax.as<int64_t>(), s.tpart.as<int64_t>(), ci, st_at,
                       a->desc.size_ms, adv, fd, a->desc.size_ms != adv ? 1 : 0, a->grace,
                       (const int64_t*)a->stream_time.as<int64_t>(), s.c1_kbase, has_kb);
    KHIP_TRY_HIP(hipGetLastError());
  } else {
    constexpr int U = 8;
    auto sk = wide ? (st_at ? k_c1_scatter<U, C1_NT, true, true> : k_c1_scatter<U, C1_NT, true, false>)
                   : (st_at ? k_c1_scatter<U, C1_NT, false, true> : k_c1_scatter<U, C1_NT, false, false>);
    const size_t lds = run_stage_lds(B, U * C1_NT, 8, wide) + run_cnt_lds(B, C1_TILE / (U * C1_NT));
    if (lds > 64 * 1024) hipFuncSetAttribute((const void*)sk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(sk, dim3(nT), dim3(C1_NT), lds, a->stream, keys, ts, kv, rv, n, nT, log2B, rc, ro, nSt,
                       s.srecA.as<uint64_t>(), s.tilemax.as<int64_t>(), s.tpart.as<int64_t>(), ci, st_at, srecAT,
                       a->desc.size_ms, adv, fd, a->grace, (const int64_t*)a->stream_time.as<int64_t>(), s.c1_kbase,
                       has_kb);
    KHIP_TRY_HIP(hipGetLastError());
  }
  // 2. each (bucket, step) run's place in its bucket's order; the bucket bases
  KHIP_TRY((ksort::scan_excl<uint32_t, uint32_t>(a->stream, s.c1scan, rc, rp, (int64_t)B * nSt, true, nullptr)));
  hipLaunchKernelGGL(k_c1_bases, dim3(1), dim3(256), 0, a->stream, (const uint32_t*)rp, nSt, B, s.c1bb.as<int64_t>());
  ev_record_part(a, 1);
  // 4. accept or decline
  hipLaunchKernelGGL(k_c1_check, dim3(1), dim3(1024), 0, a->stream, s.tilemax.as<int64_t>(), nT,
                     a->desc.size_ms, adv, fd, a->grace, close0, s.res_fresh ? 1 : 0, log2B, s.log2P, wide ? 1 : 0,
                     val ? C1V_CH : C1_CH, val ? 31 : 32, pbits, s.c1bb.as<int64_t>(), cstart, ci,
                     a->stream_time.as<int64_t>(), s.res.as<int64_t>(),
                     s.ctr.as<unsigned long long>(), s.closed_ctr.as<unsigned long long>(),
                     (unsigned long long)s.closed_n);
  // 5. refine: each chunk's step runs (k_c1_chunks), chunks → partition-sorted, segment table
  KHIP_TRY(s.c1ci.ensure((size_t)nchunk_max * 8));
  hipLaunchKernelGGL(k_c1_chunks, dim3((unsigned)ceil_div(nchunk_max, 256)), dim3(256), 0, a->stream, (const int*)cstart, B,
                     (const int64_t*)s.c1bb.as<int64_t>(), (const uint32_t*)rp, nSt, CH, (const int64_t*)ci,
                     s.c1ci.as<uint32_t>());
  if (val) {
    auto rk = k_c1v_refine<C1V_CH / C1_NT, C1_NT>;
    const size_t lds = (((size_t)F * 8 + 15) & ~(size_t)15) + (size_t)C1V_CH * 16;
    hipFuncSetAttribute((const void*)rk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(rk, dim3((unsigned)nchunk_max), dim3(C1_NT), lds, a->stream, (const ulonglong2*)s.srecA.p,
                       s.c1bb.as<int64_t>(), cstart, log2B, s.log2P, fbits, (ulonglong2*)s.srec.p, seg, ci,
                       (const uint32_t*)rp, (const uint16_t*)ro, nSt, S, (const uint32_t*)s.c1ci.as<uint32_t>());
    KHIP_TRY_HIP(hipGetLastError());
  } else {
    constexpr int U = C1_CH / C1_NT;
    auto rk = wide ? k_c1_refine<U, C1_NT, true> : k_c1_refine<U, C1_NT, false>;
    const size_t lds = (size_t)F * 8 + (size_t)C1_CH * 8;
    if (lds > 64 * 1024) hipFuncSetAttribute((const void*)rk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(rk, dim3((unsigned)nchunk_max), dim3(C1_NT), lds, a->stream,
                       s.srecA.as<uint64_t>(), s.c1bb.as<int64_t>(), cstart, log2B, s.log2P, fbits,
                       s.srec.as<uint64_t>(), seg, ci, (const uint32_t*)srecAT, srecT, (const uint32_t*)rp,
                       (const uint16_t*)ro, nSt, S, (const uint32_t*)s.c1ci.as<uint32_t>());
    KHIP_TRY_HIP(hipGetLastError());
  }
  ev_record_part(a, 2);
  // 6. merge partitions (+ retries), as part_push's pass loop
  const int log2H = (int)knob("KHIP_C1_LOG2H", 12);
  C1Q cq{};
  cq.log2P = s.log2P;
  cq.fbits = fbits;
  cq.log2H = log2H;
  cq.sw = a->sw;
  cq.hv_active = a->having.active;
  cq.hv_op = a->having.op;
  cq.hv_i64 = a->having.i64;
  cq.hmax = (int)((int64_t)(1 << log2H) * 3 / 4);
  cq.size = a->desc.size_ms;
  cq.adv = adv;
  cq.fd = fd;
  cq.fd32 = make_fastdiv32((uint32_t)adv);
  // the value pipeline's merge: the largest table (up to 2^12 entries) whose LDS lets two
  // workgroups share a CU
  C1VQ vq0{};
  int v_log2H = 12;
  int v_pm = 0;  // the plane mask when a specialised merge exists for it
  const int v_wpc = (int)knob("KHIP_C1V_WG_PER_CU", 2);  // merge workgroups per CU
  if (val) {
    // sized for 32-bit identities (the common case); 64-bit ones (a key range past 31 - window
    // bits) run at one workgroup per CU when their table does not fit two
    while (v_log2H > 9 && c1v_layout(a, v_log2H, 4, log2B, &vq0) > C1V_LDS2) v_log2H--;
    v_log2H = (int)knob("KHIP_C1V_LOG2H", v_log2H);

    vq0.log2P = s.log2P;
    vq0.fbits = fbits;
    vq0.log2H = v_log2H;
    vq0.sw = a->sw;
    vq0.hmax = (int)((int64_t)(1 << v_log2H) * 3 / 4);
    vq0.fan = (int)(a->desc.size_ms / adv);
    vq0.f64 = 0;
    for (int k = 0; k < C1V_MAXW; k++) {
      vq0.word_op[k] = -1;
      vq0.init[k] = (uint64_t)a->init.w[k];
    }
    for (int o = 0; o < a->ap.n_ops; o++) {
      vq0.word_op[a->ap.ops[o].word] = a->ap.ops[o].kind;
      if (a->ap.ops[o].kind == OP_ADD_F64) vq0.f64 = 1;
    }
    if (a->ap.col_type[vcol] == KHIP_TYPE_DOUBLE) vq0.f64 = 1;
    for (int o = 0; o < a->ap.n_ops; o++) {
      const int k = a->ap.ops[o].kind;
      v_pm |= k == OP_INC ? PM_STAR : k == OP_INC_VALID ? PM_CNT : k == OP_MIN ? PM_MIN : k == OP_MAX ? PM_MAX : PM_SUM;
    }
    v_pm |= PM_SPEC | (vq0.f64 ? PM_F64 : 0);
    if ((v_pm != PM_C5 && v_pm != PM_C3) || knob("KHIP_C1V_SPEC", 1) == 0) v_pm = 0;
    vq0.size = a->desc.size_ms;
    vq0.adv = adv;
    vq0.fd = fd;
    vq0.fd32 = make_fastdiv32((uint32_t)adv);
    vq0.having = a->having;
  }
  int64_t added_total = 0;
  // sub-passes per partition: the pipeline's own LDS table (hmax), not the general merge's — a
  // partition starts with enough of them for the hinted groups, and keeps those a push needed
  {
    const int64_t hm = val ? vq0.hmax : cq.hmax;
    if ((int64_t)s.c1psbits.size() != P || s.c1ps_hmax != hm) {
      int s0 = 0;
      while (s0 < 12 && s.hint_groups / P > (hm * 7 / 10) << s0) s0++;
      s.c1psbits.assign(P, (uint8_t)s0);
      s.c1ps_hmax = hm;
    }
  }
  std::vector<int> sbits(s.c1psbits.begin(), s.c1psbits.end());
  std::vector<uint32_t> plist, work;
  bool subs0 = false;
  for (int p = 0; p < P && !subs0; p++) subs0 = sbits[p] > 0;
  if (subs0) {
    for (int p = 0; p < P; p++)
      for (int k = 0; k < (1 << sbits[p]); k++) work.push_back((uint32_t)p | ((uint32_t)sbits[p] << 16) | ((uint32_t)k << 20));
    KHIP_TRY(s.work.ensure(work.size() * 4));
    KHIP_TRY_HIP(hipMemcpyAsync(s.work.p, work.data(), work.size() * 4, hipMemcpyHostToDevice, a->stream));
  }
  std::vector<uint8_t> host_fail;
  const bool probe = knob("KHIP_AGG_PROBE", 0) != 0;
  DevBuf dbgbuf;
  if (probe) {
    KHIP_TRY(dbgbuf.ensure(64));
    KHIP_TRY_HIP(hipMemsetAsync(dbgbuf.p, 0, 64, a->stream));
  }
  for (int pass = 0;; pass++) {
    unsigned long long* dbg = probe && pass == 0 ? dbgbuf.as<unsigned long long>() : nullptr;
    cq.cmax = s.cmax;
    cq.chg = a->changelog ? a->chg.as<uint8_t>() : nullptr;
    if (pass > 0) KHIP_TRY_HIP(hipMemsetAsync(s.ctr.p, 0, 24, a->stream));
    const uint32_t* wk = (pass == 0 && !subs0) ? nullptr : s.work.as<uint32_t>();
    const int64_t nwork = (pass == 0 && !subs0) ? P : (int64_t)work.size();
    const int64_t grid = std::min<int64_t>(nwork, (int64_t)s.n_cu * knob("KHIP_MERGE_WG_PER_CU", 2));
    // compact records: both identity widths are launched, the one k_c1_check did not choose exits
    // at once; wide records: 64-bit identities
    for (int idw = wide ? 1 : 0; idw < 2 && val; idw++) {
      C1VQ vq = vq0;
      const size_t lds = c1v_layout(a, v_log2H, idw == 0 ? 4 : 8, log2B, &vq);
      vq.cmax = s.cmax;
      vq.chg = a->changelog ? a->chg.as<uint8_t>() : nullptr;
      // the benchmarks' plane shapes have instantiations of their own (PM_C5, PM_C3), every other
      // one reads the planes from the parameters; AU 2 at <= 128 VGPRs (two workgroups per CU)
      auto pick = [&](auto pmc) {
        constexpr int PMv = decltype(pmc)::value;
        return panes ? (idw == 0 ? k_c1v_merge<512, 2, uint32_t, true, 4, PMv> : k_c1v_merge<512, 2, uint64_t, true, 4, PMv>)
                     : (idw == 0 ? k_c1v_merge<512, 2, uint32_t, false, 4, PMv> : k_c1v_merge<512, 2, uint64_t, false, 4, PMv>);
      };
      auto mk = v_pm == PM_C5 ? pick(std::integral_constant<int, PM_C5>{})
                              : (v_pm == PM_C3 ? pick(std::integral_constant<int, PM_C3>{}) : pick(std::integral_constant<int, 0>{}));
      hipFuncSetAttribute((const void*)mk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      KHIP_TRY(s.c1vq.ensure(sizeof(C1VQ)));
      KHIP_TRY(s.c1vq_h.ensure(2 * sizeof(C1VQ)));
      C1VQ* hq = (C1VQ*)s.c1vq_h.p + idw;
      *hq = vq;
      KHIP_TRY_HIP(hipMemcpyAsync(s.c1vq.p, hq, sizeof(C1VQ), hipMemcpyHostToDevice, a->stream));
      const int64_t vgrid = std::min<int64_t>(nwork, (int64_t)s.n_cu * (lds <= C1V_LDS2 ? v_wpc : 1));
      hipLaunchKernelGGL(mk, dim3(vgrid), dim3(512), lds, a->stream, s.c1vq.as<C1VQ>(), wk, nwork, s.c1bb.as<int64_t>(), cstart, seg,
                         (const ulonglong2*)s.srec.p, pass == 0 ? 1 : 0, s.buf[0].as<uint64_t>(), s.buf[1].as<uint64_t>(),
                         s.sel.as<uint8_t>(), s.cnt.as<int64_t>(), s.newcnt.as<unsigned long long>(),
                         s.fail.as<uint8_t>(), s.ctr.as<unsigned long long>() + 2, close0, s.closed.as<uint64_t>(),
                         s.closed_ctr.as<unsigned long long>(), ci,
                         s.hnew.as<unsigned long long>(), s.ctr.as<unsigned long long>() + 12, s.prn.as<uint32_t>(), dbg);
    }
    for (int idw = wide ? 1 : 0; idw < 2 && !val; idw++) {
      auto mk = wide ? k_c1_merge<512, 3, uint64_t, true>
                     : (idw == 0 ? k_c1_merge<512, 4, uint32_t, false> : k_c1_merge<512, 4, uint64_t, false>);
      const size_t lds = c1_merge_lds(log2H, idw == 0 ? 4 : 8, log2B);
      hipFuncSetAttribute((const void*)mk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(mk, dim3(grid), dim3(512), lds, a->stream, cq, wk, nwork, s.c1bb.as<int64_t>(), cstart, seg,
                         s.srec.as<uint64_t>(), pass == 0 ? 1 : 0, s.buf[0].as<uint64_t>(), s.buf[1].as<uint64_t>(),
                         s.sel.as<uint8_t>(), s.cnt.as<int64_t>(), s.newcnt.as<unsigned long long>(),
                         s.fail.as<uint8_t>(), s.ctr.as<unsigned long long>() + 2, close0, s.closed.as<uint64_t>(),
                         s.closed_ctr.as<unsigned long long>(), ci,
                         s.hnew.as<unsigned long long>(), s.ctr.as<unsigned long long>() + 12, s.prn.as<uint32_t>(),
                         (const uint32_t*)srecT, dbg);
    }
    KHIP_TRY_HIP(hipGetLastError());
    const int nl = pass == 0 ? P : (int)plist.size();
    hipLaunchKernelGGL(k_part_commit, dim3(ceil_div(std::max(nl, 1), 256)), dim3(256), 0, a->stream,
                       pass == 0 ? (const int64_t*)ci : (const int64_t*)nullptr, P, s.pbase.as<int64_t>(),
                       s.prn.as<uint32_t>(), pass == 0 ? nullptr : s.work.as<uint32_t>() + work.size(), nl,
                       s.sel.as<uint8_t>(), s.cnt.as<int64_t>(), s.newcnt.as<unsigned long long>(),
                       s.fail.as<uint8_t>(), s.ctr.as<unsigned long long>(), s.hcnt.as<unsigned long long>(),
                       s.hnew.as<unsigned long long>());
    KHIP_TRY_HIP(hipGetLastError());
    if (pass == 0) {
      ev_record_part(a, 3);
      hipLaunchKernelGGL(k_part_stats, dim3(1), dim3(256), 0, a->stream, s.tpart.as<int64_t>(), nT,
                         s.closed_ctr.as<unsigned long long>(), a->stream_time.as<int64_t>(),
                         s.ctr.as<unsigned long long>());
      KHIP_TRY_HIP(hipMemcpyAsync(s.pinfo.as<int64_t>() + 32, ci, CI_N * 8, hipMemcpyDeviceToHost, a->stream));
    }
    unsigned long long* c2 = s.pinfo.as<unsigned long long>() + 8;
    KHIP_TRY_HIP(hipMemcpyAsync(c2, s.ctr.p, 13 * 8, hipMemcpyDeviceToHost, a->stream));
    // the closed store's rows after this pass (closed rows leave in the pass that writes their
    // item): read with the counters, no second round trip
    KHIP_TRY_HIP(hipMemcpyAsync(s.pinfo.as<unsigned long long>() + 58, s.closed_ctr.p, 8, hipMemcpyDeviceToHost,
                                a->stream));
    KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
    const int64_t* hci = s.pinfo.as<int64_t>() + 32;
    if (pass == 0 && hci[CI_GATE] == 0) {  // declined: nothing was written
      if (hci[CI_REASON] == 2 && !s.c1_kretry) {  // a key outside the field above kb: the true range
        long long kr[2] = {INT64_MIN, INT64_MIN};
        KHIP_TRY(s.c1scan.ensure(16));
        KHIP_TRY_HIP(hipMemcpyAsync(s.c1scan.p, kr, 16, hipMemcpyHostToDevice, a->stream));
        hipLaunchKernelGGL(k_c1_krange, dim3((unsigned)std::min<int64_t>(ceil_div(n, 256), 2048)), dim3(256), 0,
                           a->stream, rows ? (const int64_t*)rows->rows : keys, rows ? (int64_t)rows->rw : 1, n,
                           s.c1scan.as<long long>());
        KHIP_TRY_HIP(hipMemcpyAsync(kr, s.c1scan.p, 16, hipMemcpyDeviceToHost, a->stream));
        KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
        const int64_t kmin = (int64_t)~(uint64_t)kr[0], kmax = (int64_t)kr[1];
        if ((uint64_t)kmax - (uint64_t)kmin < (1ULL << (val ? 31 : 32)) - 1) {  // again with kb = kmin
          s.c1_kbase = kmin;
          s.c1_kb_valid = true;
          s.c1_kretry = true;
          const khip_status r = c1_push(a, n, keys, ts, kv, rv, tot, declined, st_at, retry_wide, cols, vcol, rows);
          s.c1_kretry = false;
          return r;
        }
        *declined = true;
        *retry_wide = !val;  // the range itself is past the compact records
        if (*retry_wide) s.c1_wide = true;
        return KHIP_OK;
      }
      *declined = true;
      *retry_wide = !val && hci[CI_REASON] == 1;  // only the record format was wrong
      if (*retry_wide) s.c1_wide = true;
      return KHIP_OK;
    }
    if (pass == 0 && wide && ++s.c1_wide_n % 64 == 0) s.c1_wide = false;  // now and then: compact records again?
    if (pass == 0 && !wide) {  // the next push's key base: this one's minimum, less a margin for keys below it
      const int64_t km = hci[CI_KMINC], slack = (int64_t)1 << (val ? 26 : 28);
      s.c1_kbase = km >= INT64_MIN + slack ? km - slack : km;
      s.c1_kb_valid = true;
    }
    if (dbg) {
      unsigned long long ph[8] = {};
      if (hipMemcpy(ph, dbgbuf.p, sizeof(ph), hipMemcpyDeviceToHost) == hipSuccess) {
        const double g = (double)std::min<int64_t>(P, 2 * s.n_cu) * 100.0;  // 100 MHz ticks → us per workgroup
        fprintf(stderr, "[%s merge probe] per workgroup (us): start+evict %.1f records %.1f fold %.1f "
                "mark+count+reserve %.1f write %.1f\n", val ? "c1v" : "c1", ph[0] / g, ph[1] / g, ph[2] / g, ph[3] / g,
                ph[4] / g);
      }
    }
    added_total += (int64_t)c2[0];
    if (c2[1] == 0) break;
    if (pass > 24) return fail(KHIP_E_DEVICE, "partitioned aggregation could not place the batch");
    host_fail.resize(P);
    KHIP_TRY_HIP(hipMemcpy(host_fail.data(), s.fail.p, P, hipMemcpyDeviceToHost));
    KHIP_TRY_HIP(hipMemsetAsync(s.fail.p, 0, P, a->stream));
    bool grow = false;
    plist.clear();
    work.clear();
    for (int p = 0; p < P; p++) {
      if (!host_fail[p]) continue;
      if (host_fail[p] & 1) sbits[p] = sbits[p] + 1;
      if (host_fail[p] & 2) grow = true;
      plist.push_back((uint32_t)p);
      if (sbits[p] > 12) return fail(KHIP_E_DEVICE, "partition needs more than 4096 sub-passes (extreme key skew)");
      for (int k = 0; k < (1 << sbits[p]); k++) work.push_back((uint32_t)p | ((uint32_t)sbits[p] << 16) | ((uint32_t)k << 20));
    }
    if (grow) KHIP_TRY(part_regrow(a, next_pow2(std::max<int64_t>(s.cmax * 2, (int64_t)c2[2] * 5 / 4 + 64))));
    std::vector<uint32_t> both(work);
    both.insert(both.end(), plist.begin(), plist.end());
    KHIP_TRY(s.work.ensure(both.size() * 4));
    KHIP_TRY_HIP(hipMemcpyAsync(s.work.p, both.data(), both.size() * 4, hipMemcpyHostToDevice, a->stream));
  }
  for (int p = 0; p < P; p++) s.c1psbits[p] = (uint8_t)std::max<int>(s.c1psbits[p], sbits[p]);
  s.res_fresh = false;
  s.last_c1 = true;
  {
    const unsigned long long* hc = s.pinfo.as<unsigned long long>() + 8;
    s.having_total = (int64_t)(hc[11] + hc[12]);
  }
  const unsigned long long* st = s.pinfo.as<unsigned long long>() + 8;
  // the closed store's rows after every pass (read with the last pass's counters)
  const int64_t cn = (int64_t)s.pinfo.as<unsigned long long>()[58];
  added_total += cn - s.closed_n;  // evicted rows left the live regions but are still groups
  s.closed_n = cn;
  a->host_stream_time = (int64_t)st[4 + T_NPART];
  int64_t c[T_NPART];
  for (int k = 0; k < T_NPART; k++) c[k] = (int64_t)st[3 + k];
  tot[P_ACCEPTED] += c[T_ACCEPTED];
  tot[P_NULL_KEY] += c[T_NULL_KEY];
  tot[P_NULL_ROW] += c[T_NULL_ROW];
  tot[P_BAD_TS] += c[T_BAD_TS];
  tot[P_APPLIED] += c[T_APPLIED];
  tot[P_LATE] += c[T_LATE];
  tot[P_NEW] += added_total;
  return KHIP_OK;
}

}  // namespace khip
