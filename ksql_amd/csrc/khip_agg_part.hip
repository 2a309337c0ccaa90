// khip_agg_part.hip — partitioned (LDS-owned) windowed aggregation engine, the default.
//
// Why: the global-atomic engine (k_apply) pays one random HBM line plus 2+ memory-side
// 64-bit atomics per (record, window); scattered atomics run ~17x below the HBM rate
// (MI355X_MICROARCH.md, Global float atomics).  Here every (key, window) group is owned
// by exactly one workgroup, so all updates are LDS atomics and HBM only sees coalesced
// streams:
//
//   k_part_hist      tile of 64K records (XCD-swizzled tile index): validity, stream-time
//                    tile max, LDS histogram over P key partitions → hist[t][p] (u32)
//   k_scan_blocks    exclusive prefix max of tile maxima (stream time before each tile)
//   k_part_colsum / k_part_colbase / k_scan_excl / k_part_colprefix
//                    column prefix sums → each (tile, partition) chunk's output offset
//   k_part_scatter   in-tile stream time (block scan), late test, first applied window,
//                    record → its partition's contiguous range (LDS cursors), SoA
//   k_part_agg       one workgroup per partition: load the partition's resident groups
//                    (compact rows) into an LDS hash table, apply its records (window
//                    fan-out, LDS atomics), write the compacted rows to the other buffer
//   k_part_commit    flip the partition's buffer, publish its row count
// A partition whose groups overflow the LDS table (or its region) writes nothing and is
// retried with 2x sub-passes (groups split by hash bits) / a grown region — exact, since
// its previous rows are untouched in the other buffer.
#include <algorithm>
#include <cstring>
#include <vector>

#include <cstdlib>

#include "khip_agg_internal.hpp"
#include "khip_part.hpp"

namespace khip {

constexpr int PT_THREADS = 1024;
constexpr int R8_NT = 512;  // k_part_scatter_r8 / k_part_refine_r8 workgroup size (two per CU)
constexpr int W_NT = 512;   // k_part_scatter_w workgroup size (two per CU)
constexpr int PT_ITEMS = 64;  // default records per thread per tile (KHIP_TILE_ITEMS overrides)
constexpr int AG_THREADS = 1024;
constexpr uint32_t L_CLAIM = 1u;
constexpr uint32_t L_READY = 2u;
constexpr int MAX_P_LOG2 = 15;    // LDS histogram: 32768 x u32 = 128 KB (of 160 KB)
constexpr int SPLIT_P_LOG2 = 14;  // growth by splitting stops here (more partitions cost the
                                  // scatter more than they save the LDS aggregate)
constexpr int TC_MAX = 64;      // tile chunks for the column prefix


struct ColTypes {
  int32_t t[MAX_COLS];
};

struct RecLayout {
  int32_t rw, meta_word;
  uint32_t vcols;  // columns whose validity bit goes into meta
  int8_t col_word[MAX_COLS];
  int8_t word_col[2 + 1 + MAX_COLS + 1];  // word → column (-1: key/ts/meta/pad)
};

struct PartAggParams {
  int32_t windowed;
  int32_t nwords;  // 3 + state words actually used
  int32_t sw;      // row stride (u64 words) in regions
  int32_t H;
  int32_t H_eff;
  int32_t rw;         // scattered record stride (u64 words)
  int32_t meta_word;  // 2 or -1
  int8_t col_word[MAX_COLS];
  int64_t size, adv;
  FastDiv fd;  // division by adv
  int32_t dbg_mode;  // KHIP_AGG_MODE (timing experiments only; results wrong when != 0)
  int32_t log2P;
  int64_t cmax;
  int32_t n_cols;
  int32_t n_ops;
  int32_t col_type[MAX_COLS];
  UpdOp ops[MAX_OPS];
  InitWords init;
  // changelog (khip_agg::changelog): byte offset of the LDS flag plane (H bytes: bit 0 touched,
  // bit 1 HAVING held before the push) and the per-row-slot emission flags (CHG_*)
  int32_t flag_off;
  uint8_t* chg;
  HavingDev having;
};


// Packed group identity (identity-CAS mode): inside partition p the top log2P bits of the
// key hash are p, so (hk << log2P) keeps the key exactly; the low log2P bits hold the
// window index relative to wbase (< 2^log2P - 1, so an identity is never EMPTY_ID).
__device__ __forceinline__ uint64_t ident_of(uint64_t hk, int64_t widx_rel, int log2P) {
  return (hk << log2P) | (uint64_t)widx_rel;
}


__device__ __forceinline__ uint32_t slot_of(uint64_t hk, int64_t ws, int H) {
  return ((uint32_t)hk + (uint32_t)ws * 0x9E3779B1u) & (uint32_t)(H - 1);
}

// 30-bit fingerprint kept with the slot state (low 2 bits): most probes of another group end
// on the state word alone
__device__ __forceinline__ uint32_t fp_of(uint64_t hk, int64_t ws) {
  return ((uint32_t)(hk >> 32) ^ ((uint32_t)ws * 0xC2B2AE35u)) & ~3u;
}

// sub-pass of a group: 12 bits from hash bits 16..47 (below every partition bit, above the slot bits)
__device__ __forceinline__ bool sub_ok(uint64_t hk, int64_t ws, int sbits, int sub) {
  return sbits == 0 || (int)((((uint32_t)(hk >> 16) + (uint32_t)ws * 0x85EBCA77u) >> 20) & ((1u << sbits) - 1)) == sub;
}


__global__ __launch_bounds__(PT_THREADS) void k_part_hist(const int64_t* __restrict__ keys,
                                                          const int64_t* __restrict__ ts,
                                                          const uint8_t* __restrict__ kv,
                                                          const uint8_t* __restrict__ rv, int64_t n, int64_t tile,
                                                          int log2P, int pad, int64_t nT, uint32_t* __restrict__ hist,
                                                          int64_t* __restrict__ tilemax, int64_t* __restrict__ tilemin,
                                                          int64_t* __restrict__ tpart, int fbits,
                                                          uint32_t* __restrict__ hcoarse,
                                                          int64_t* __restrict__ tilekr,
                                                          const int64_t* __restrict__ st_at) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* lh = (uint32_t*)smem;
  __shared__ int64_t lmax[PT_THREADS / 64];
  __shared__ int64_t lmin[PT_THREADS / 64];
  __shared__ int64_t lkr[2][PT_THREADS / 64];
  __shared__ unsigned long long lc[4];
  const int P = 1 << log2P;
  const int64_t t = tile_of(blockIdx.x, nT);
  for (int p = threadIdx.x; p < P; p += PT_THREADS) lh[p] = 0;
  if (threadIdx.x < 4) lc[threadIdx.x] = 0;
  __syncthreads();
  int64_t m = -1, mn = INT64_MAX, c_acc = 0, c_nk = 0, c_nr = 0, c_bt = 0;
  int64_t kmx = INT64_MIN, kmxn = INT64_MIN;  // accepted keys: max of key and of ~key (= ~min)
  const int64_t base = t * tile;
  const int64_t end = base + tile < n ? base + tile : n;
  for (int64_t i0 = base + threadIdx.x; i0 < end; i0 += 4 * PT_THREADS) {
    int64_t x[4], k[4];
    bool ok[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {  // issue the loads of 4 records before using any
      const int64_t i = i0 + u * PT_THREADS;
      ok[u] = i < end;
      x[u] = ok[u] ? ts[i] : 0;
      k[u] = ok[u] ? keys[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int64_t i = i0 + u * PT_THREADS;
      if (!ok[u]) continue;
      if (!bit_get(kv, i)) { c_nk++; continue; }
      if (!bit_get(rv, i)) { c_nr++; continue; }
      if (x[u] < 0) { c_bt++; continue; }
      c_acc++;
      const int64_t sx = st_at ? st_at[i] : x[u];  // ABI 5 domains: the row's given stream time
      m = sx > m ? sx : m;
      mn = x[u] < mn ? x[u] : mn;
      kmx = k[u] > kmx ? k[u] : kmx;
      kmxn = ~k[u] > kmxn ? ~k[u] : kmxn;
      atomicAdd(&lh[part_of(k[u], log2P)], 1u);
    }
  }
  int64_t tot;
  block_incl_max(m, lmax, &tot);
  int64_t totmin;
  block_incl_max(-mn, lmin, &totmin);  // min via max of negation (mn >= 0 or INT64_MAX)
  if (tilekr) {  // the tile's key range (R8 records: keys relative to the push's smallest)
    for (int off = 32; off > 0; off >>= 1) {
      const int64_t a = __shfl_xor(kmx, off, 64), b = __shfl_xor(kmxn, off, 64);
      kmx = a > kmx ? a : kmx;
      kmxn = b > kmxn ? b : kmxn;
    }
    if ((threadIdx.x & 63) == 0) {
      lkr[0][threadIdx.x >> 6] = kmx;
      lkr[1][threadIdx.x >> 6] = kmxn;
    }
  }
  c_acc = wave_sum(c_acc); c_nk = wave_sum(c_nk); c_nr = wave_sum(c_nr); c_bt = wave_sum(c_bt);
  if ((threadIdx.x & 63) == 0) {
    if (c_acc) atomicAdd(&lc[0], (unsigned long long)c_acc);
    if (c_nk) atomicAdd(&lc[1], (unsigned long long)c_nk);
    if (c_nr) atomicAdd(&lc[2], (unsigned long long)c_nr);
    if (c_bt) atomicAdd(&lc[3], (unsigned long long)c_bt);
  }
  __syncthreads();
  uint32_t* hrow = hist + t * (int64_t)P;
  // pad: each (tile, partition) run rounded up to whole 64-byte segments (4 records)
  for (int p = threadIdx.x; p < P; p += PT_THREADS) hrow[p] = pad ? (lh[p] + 3u) & ~3u : lh[p];
  if (hcoarse) {  // two-level scatter: bucket b = partitions [b << fbits, (b + 1) << fbits)
    const int B = P >> fbits;
    for (int b = threadIdx.x; b < B; b += PT_THREADS) {
      uint32_t c = 0;
      for (int f = 0; f < (1 << fbits); f++) c += lh[(b << fbits) + ((f + b) & ((1 << fbits) - 1))];
      hcoarse[t * (int64_t)B + b] = c;
    }
  }
  if (threadIdx.x == 0) {
    tilemax[t] = tot;
    tilemin[t] = -totmin;
    if (tilekr) {
      int64_t a = INT64_MIN, b = INT64_MIN;
      for (int w = 0; w < PT_THREADS / 64; w++) {
        a = lkr[0][w] > a ? lkr[0][w] : a;
        b = lkr[1][w] > b ? lkr[1][w] : b;
      }
      tilekr[2 * t] = a;      // INT64_MIN: no accepted record
      tilekr[2 * t + 1] = b;  // ~(smallest key)
    }
    int64_t* tp = tpart + t * T_NPART;
    tp[T_ACCEPTED] = (int64_t)lc[0];
    tp[T_NULL_KEY] = (int64_t)lc[1];
    tp[T_NULL_ROW] = (int64_t)lc[2];
    tp[T_BAD_TS] = (int64_t)lc[3];
  }
}

// csum[c][p] = sum over the tiles of chunk c of hist[t][p]
__global__ __launch_bounds__(256) void k_part_colsum(const uint32_t* __restrict__ hist, int64_t nT, int P, int TC,
                                                     int64_t* __restrict__ csum) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  const int c = blockIdx.y;
  if (p >= P) return;
  const int64_t t0 = nT * c / TC, t1 = nT * (c + 1) / TC;
  int64_t s = 0;
  for (int64_t t = t0; t < t1; t++) s += hist[t * P + p];
  csum[(int64_t)c * P + p] = s;
}

// in place: csum[c][p] → exclusive prefix over c; R[p] = column total.  The chunk sums are
// loaded 16 at a time before any store (the in-place stores would otherwise order every load
// behind the previous store: TC dependent round trips per thread).
__global__ __launch_bounds__(256) void k_part_colbase(int64_t* __restrict__ csum, int P, int TC,
                                                      int64_t* __restrict__ R) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  int64_t acc = 0;
  for (int c0 = 0; c0 < TC; c0 += 16) {
    int64_t v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) v[u] = c0 + u < TC ? csum[(int64_t)(c0 + u) * P + p] : 0;
#pragma unroll
    for (int u = 0; u < 16; u++) {
      if (c0 + u < TC) csum[(int64_t)(c0 + u) * P + p] = acc;
      acc += v[u];
    }
  }
  R[p] = acc;
}

// v[0..n) → its exclusive prefix sum in place, v[n] = the total (one workgroup; each thread
// owns 16 consecutive elements per 16K-element chunk: one wave scan + one barrier per chunk).
__global__ __launch_bounds__(1024) void k_part_pscan(int64_t* __restrict__ v, int64_t n) {
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
  if (threadIdx.x == 0) v[n] = carry;
}

// hist[t][p] → absolute output offset of (tile t, partition p)
__global__ __launch_bounds__(256) void k_part_colprefix(uint32_t* __restrict__ hist, int64_t nT, int P, int TC,
                                                        const int64_t* __restrict__ csum,
                                                        const int64_t* __restrict__ pbase, int pstride) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  const int c = blockIdx.y;
  if (p >= P) return;
  const int64_t t0 = nT * c / TC, t1 = nT * (c + 1) / TC;
  int64_t acc = pbase[(int64_t)p * pstride] + csum[(int64_t)c * P + p];
  for (int64_t t = t0; t < t1; t++) {
    const uint32_t v = hist[t * P + p];
    hist[t * P + p] = (uint32_t)acc;
    acc += v;
  }
}

// 12-byte (key hash, ts) record of the narrow layout (rw = 2) when k_part_merge runs: the key
// hash, and ts relative to the push's earliest accepted ts (trel = ts - tbase + 1; 0 = no window
// applied).  A quarter less traffic through the scatter, the refine and the merge's reads.
struct R12 {
  uint32_t lo, hi, trel;
};

__device__ __forceinline__ void r12_store(uint64_t* __restrict__ srec, uint64_t i, uint64_t hk, uint32_t trel) {
  *(R12*)((char*)srec + i * 12) = R12{(uint32_t)hk, (uint32_t)(hk >> 32), trel};
}


// LDS-staged scatter step (k_part_scatter's narrow fast path, k_part_refine of narrow records).
// U records per thread (hk, pay, ok) go to bin (hk >> shift) & mask, whose next output position
// is cur[bin].  Instead of every lane storing its record to its own bin's run (64 lines touched
// per store instruction), the step's records are ranked per bin (LDS atomics), placed in LDS in
// bin order, and written back out by consecutive threads: each bin's records of the step leave
// as one contiguous run (~S / nb records) in whole-line, coalesced stores.
//   out: 0 = (hk, pay) 16 bytes; 1 = R12 (pay = trel); 2 = R12 in, (hk, ts) 16 bytes out;
//        3 = R8 (pay = the 8-byte record)
struct StageLds {
  uint32_t* cur;    // [nb] next output record of each bin (global index)
  uint32_t* cnt;    // [nb] records of the step per bin
  uint32_t* sbase;  // [nb] the bin's first staged slot
  uint32_t* gpos;   // [nb] output position of the bin's first record of the step
  uint64_t* sk;     // [S] staged key hashes
  int64_t* sp;      // [S] staged payloads
  int* wsum;        // [16]
};


template <int U>
__device__ __forceinline__ void stage_step(const int64_t (&hk)[U], const int64_t (&pay)[U], const bool (&ok)[U],
                                           int shift, uint32_t mask, int nb, const StageLds& L,
                                           uint64_t* __restrict__ srec, int out, int64_t tbase) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  uint32_t rank[U];
#pragma unroll
  for (int u = 0; u < U; u++) rank[u] = ok[u] ? atomicAdd(&L.cnt[stage_bin((uint64_t)hk[u], shift, mask)], 1u) : 0u;
  lds_barrier();
  // exclusive scan of the bin counts (nb <= PT_THREADS)
  const uint32_t c = t < nb ? L.cnt[t] : 0u;
  uint32_t incl = c;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) L.wsum[wave] = (int)incl;
  lds_barrier();
  uint32_t before = 0, tot = 0;
  for (int k = 0; k < PT_THREADS / 64; k++) {
    before += k < wave ? (uint32_t)L.wsum[k] : 0u;
    tot += (uint32_t)L.wsum[k];
  }
  if (t < nb) {
    L.sbase[t] = before + incl - c;
    L.gpos[t] = L.cur[t];
    L.cur[t] += c;
    L.cnt[t] = 0u;
  }
  lds_barrier();
#pragma unroll
  for (int u = 0; u < U; u++) {
    if (!ok[u]) continue;
    const uint32_t i = L.sbase[stage_bin((uint64_t)hk[u], shift, mask)] + rank[u];
    L.sk[i] = (uint64_t)hk[u];
    L.sp[i] = pay[u];
  }
  lds_barrier();
  for (uint32_t j = t; j < tot; j += PT_THREADS) {
    const uint64_t h = L.sk[j];
    const int64_t p = L.sp[j];
    const uint32_t b = stage_bin(h, shift, mask);
    const uint64_t dst = (uint64_t)L.gpos[b] + (j - L.sbase[b]);
    if (out == 3) {  // R8: the payload is the record
      srec[dst] = (uint64_t)p;
    } else if (out == 0) {
      *(longlong2*)(srec + dst * 2) = make_longlong2((int64_t)h, p);
    } else if (out == 1) {
      r12_store(srec, dst, h, (uint32_t)p);
    } else {
      *(longlong2*)(srec + dst * 2) = make_longlong2((int64_t)h, p ? tbase + p - 1 : -1);
    }
  }
  // the next step's first barrier (after its rank atomics) orders these LDS reads before any
  // rewrite of sbase / gpos / the stage
}

// stage_step for self-contained 8-byte records (R8): only the record is staged (8 bytes per record
// instead of 16: a step of U = 8 records per thread fits twice in a CU's LDS, so two workgroups
// overlap one's barriers with the other's loads); the write-out recomputes each staged record's
// bin with binof.  L.sp holds U * PT_THREADS records.
template <int U, class BinOf>
__device__ __forceinline__ void stage_step8(const int64_t (&rec)[U], const uint32_t (&bin)[U], const bool (&ok)[U],
                                            int nb, const StageLds& L, uint64_t* __restrict__ srec, BinOf binof) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  uint32_t rank[U];
#pragma unroll
  for (int u = 0; u < U; u++) rank[u] = ok[u] ? atomicAdd(&L.cnt[bin[u]], 1u) : 0u;
  lds_barrier();
  const uint32_t c = t < nb ? L.cnt[t] : 0u;
  uint32_t incl = c;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) L.wsum[wave] = (int)incl;
  lds_barrier();
  uint32_t before = 0, tot = 0;
  for (int k = 0; k < PT_THREADS / 64; k++) {
    before += k < wave ? (uint32_t)L.wsum[k] : 0u;
    tot += (uint32_t)L.wsum[k];
  }
  if (t < nb) {
    L.sbase[t] = before + incl - c;
    L.gpos[t] = L.cur[t];
    L.cur[t] += c;
    L.cnt[t] = 0u;
  }
  lds_barrier();
#pragma unroll
  for (int u = 0; u < U; u++)
    if (ok[u]) L.sp[L.sbase[bin[u]] + rank[u]] = rec[u];
  lds_barrier();
  for (uint32_t j = t; j < tot; j += PT_THREADS) {
    const int64_t p = L.sp[j];
    const uint32_t b = binof(p);
    srec[(uint64_t)L.gpos[b] + (j - L.sbase[b])] = (uint64_t)p;
  }
}

// LDS carve-up for stage_step: nb bins, S staged records
__host__ __device__ constexpr size_t stage_lds_bytes(int nb, int S) {
  return ((size_t)nb * 16 + 15) / 16 * 16 + (size_t)S * 16;
}

// stage_step for 32-byte records (rw = 4: key hash, ts, and two more words — meta and one value
// column, or two values): staged as two 16-byte halves (L.sk/L.sp hold words 0/1, L.sk + S /
// L.sp + S words 2/3: the carve-up of stage_lds_bytes(nb, 2 * S)), written out per bin as whole
// 32-byte records in consecutive, coalesced stores.
template <int U, int NT = PT_THREADS>
__device__ __forceinline__ void stage_step_w(const int64_t (&hk)[U], const int64_t (&ts)[U], const int64_t (&w2)[U],
                                             const int64_t (&w3)[U], const bool (&ok)[U], int shift, uint32_t mask,
                                             int nb, const StageLds& L, uint64_t* __restrict__ srec) {
  constexpr int S = U * NT;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  uint32_t rank[U];
#pragma unroll
  for (int u = 0; u < U; u++) rank[u] = ok[u] ? atomicAdd(&L.cnt[stage_bin((uint64_t)hk[u], shift, mask)], 1u) : 0u;
  lds_barrier();
  const uint32_t c = t < nb ? L.cnt[t] : 0u;
  uint32_t incl = c;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) L.wsum[wave] = (int)incl;
  lds_barrier();
  uint32_t before = 0, tot = 0;
  for (int k = 0; k < NT / 64; k++) {
    before += k < wave ? (uint32_t)L.wsum[k] : 0u;
    tot += (uint32_t)L.wsum[k];
  }
  if (t < nb) {
    L.sbase[t] = before + incl - c;
    L.gpos[t] = L.cur[t];
    L.cur[t] += c;
    L.cnt[t] = 0u;
  }
  lds_barrier();
  longlong2* lo = (longlong2*)L.sk;  // [S] words 0, 1
  longlong2* hi = lo + S;             // [S] words 2, 3
#pragma unroll
  for (int u = 0; u < U; u++) {
    if (!ok[u]) continue;
    const uint32_t i = L.sbase[stage_bin((uint64_t)hk[u], shift, mask)] + rank[u];
    lo[i] = make_longlong2(hk[u], ts[u]);
    hi[i] = make_longlong2(w2[u], w3[u]);
  }
  lds_barrier();
  for (uint32_t j = t; j < tot; j += NT) {
    const longlong2 a = lo[j], b = hi[j];
    const uint32_t bn = stage_bin((uint64_t)a.x, shift, mask);
    uint64_t* r = srec + ((uint64_t)L.gpos[bn] + (j - L.sbase[bn])) * 4;
    *(longlong2*)r = a;
    *(longlong2*)(r + 2) = b;
  }
}

__device__ __forceinline__ StageLds stage_carve(char* smem, int nb, int S, int* wsum) {
  StageLds L;
  L.cur = (uint32_t*)smem;
  L.cnt = L.cur + nb;
  L.sbase = L.cnt + nb;
  L.gpos = L.sbase + nb;
  L.sk = (uint64_t*)(smem + ((size_t)nb * 16 + 15) / 16 * 16);
  L.sp = (int64_t*)(L.sk + S);
  L.wsum = wsum;
  return L;
}

__device__ __forceinline__ void scatter_one(int64_t key, int64_t x, int64_t jlo, int64_t i, int log2P, uint32_t* cur,
                                            uint64_t* __restrict__ srec, const RecLayout& L, const ColPtrs& cols,
                                            int n_cols, const ColTypes& ctypes, bool applied, bool r12,
                                            int64_t tbase, int r8tb, int64_t kbase) {
  const uint64_t hk = key_hash(key);
  const uint32_t pos = atomicAdd(&cur[part_of_hk(hk, log2P)], 1u);
  if (r12 && r8tb) {  // R8: (key - kbase) << tb | trel
    srec[pos] = ((uint64_t)(key - kbase) << r8tb) | (applied ? (uint64_t)(x - tbase + 1) : 0ULL);
    return;
  }
  if (r12) {  // narrow layout only
    r12_store(srec, pos, hk, applied ? (uint32_t)(x - tbase + 1) : 0u);
    return;
  }
  uint64_t* r = srec + (uint64_t)pos * L.rw;
  *(longlong2*)r = make_longlong2((int64_t)hk, applied ? x : -1);  // one 16-byte store: key hash, ts
  if (L.rw > 2) {  // then the rest of the record, 16 bytes at a time, contiguous
    uint32_t vm = 0;
    for (int c = 0; c < n_cols; c++)
      if ((L.vcols >> c) & 1u) vm |= (bit_get(cols.valid[c], i) ? 1u : 0u) << c;
    for (int w = 2; w < L.rw; w += 2) {
      int64_t v[2];
      for (int k = 0; k < 2; k++) {
        const int col = L.word_col[w + k];
        v[k] = (w + k) == L.meta_word ? (int64_t)((uint32_t)jlo | (vm << 16))
                                      : (col >= 0 ? load_col_raw(cols, ctypes.t[col], col, i) : 0);
      }
      *(longlong2*)(r + w) = make_longlong2(v[0], v[1]);
    }
  }
}

template <int U, bool NARROW>
__global__ __launch_bounds__(PT_THREADS) void k_part_scatter(
    const int64_t* __restrict__ keys, const int64_t* __restrict__ ts, const uint8_t* __restrict__ kv,
    const uint8_t* __restrict__ rv, ColPtrs cols, int n_cols, ColTypes ctypes, int64_t n, int64_t tile, int log2P,
    int pad, int64_t nT, const uint32_t* __restrict__ offs, const int64_t* __restrict__ pbase,
    const int64_t* __restrict__ tileprefix, const int64_t* __restrict__ tilemax,
    const int64_t* __restrict__ tilemin, int windowed, int64_t size, int64_t adv, FastDiv fd, int64_t grace,
    RecLayout L, uint64_t* __restrict__ srec, int64_t dummy, int64_t* __restrict__ tpart,
    const int64_t* __restrict__ wr, int r12_ok, int stage, int skip_r8, const int64_t* __restrict__ st_at) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* cur = (uint32_t*)smem;
  __shared__ int wsum[PT_THREADS / 64];
  const bool r12 = r12_ok && wr[4] != 0;  // k_part_merge runs: 12-byte records
  const int64_t tbase = wr[5];
  const int r8tb = r12 ? (int)wr[7] : 0;    // ... or 8-byte ones (k_part_wrange)
  const int64_t kbase = wr[6];
  __shared__ int64_t lmax[PT_THREADS / 64];
  __shared__ unsigned long long lc[2];
  const int P = 1 << log2P;
  const int64_t t = tile_of(blockIdx.x, nT);
  for (int p = threadIdx.x; p < P; p += PT_THREADS) cur[p] = offs[t * P + p];
  if (threadIdx.x < 2) lc[threadIdx.x] = 0;
  __syncthreads();
  int64_t carry = tileprefix[t];
  int64_t c_app = 0, c_late = 0;
  const int64_t base = t * tile;
  const int64_t end = base + tile < n ? base + tile : n;
  // Fast path: no record of this tile can be late when even its earliest first window
  // outlives the largest stream time the tile can reach (max(prefix, tile max)).
  const int64_t smax = carry > tilemax[t] ? carry : tilemax[t];
  const int64_t tmin = tilemin[t];
  const bool fast = !windowed || tmin == INT64_MAX || first_window_start(tmin, size, adv) + size > smax - grace;
  if (skip_r8 && fast && stage && (NARROW ? r8tb != 0 : L.rw == 4)) return;  // k_part_scatter_r8 / _w's tile
  if (fast && NARROW && stage) {
    // (key hash, ts) records through the LDS stage (stage_step), next step's loads in flight
    constexpr int S = U * PT_THREADS;
    // the host sized the stage for S 8-byte records: R8 steps use it whole (stage_step8), the
    // 12/16-byte records go through it in two half steps of 16-byte (hash, payload) pairs
    const StageLds SL = stage_carve(smem, P, S / 2, wsum);
    StageLds SL8 = SL;
    SL8.sp = (int64_t*)SL.sk;
    for (int p = threadIdx.x; p < P; p += PT_THREADS) SL.cnt[p] = 0u;
    lds_barrier();
    const int shift = log2P == 0 ? 64 : 64 - log2P;
    const uint32_t bmask = (uint32_t)(P - 1);
    int64_t x[U], k[U], nxx[U], nxk[U];
    auto load_step = [&](int64_t i0, int64_t (&dx)[U], int64_t (&dk)[U]) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        int64_t i = i0 + (int64_t)u * PT_THREADS;
        i = i < end ? i : end - 1;
        dx[u] = ts[i];
        dk[u] = keys[i];
      }
    };
    // steps are uniform across the block (every thread runs every step: barriers inside).  The
    // R8 and the 12/16-byte step loops are separate loops (R8C: compile-time), so the registers
    // of one are not allocated around the other (one shared loop spilled the next step's
    // prefetched records to scratch every step)
    auto run = [&](auto r8c) {
      constexpr bool R8C = decltype(r8c)::value;
    int64_t s0 = base;
    if (s0 < end) load_step(s0 + threadIdx.x, x, k);
    for (; s0 < end; s0 += S) {
      const int64_t i0 = s0 + threadIdx.x;
      if (s0 + S < end) load_step(i0 + S, nxx, nxk);
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; u++) {  // in place: k → key hash, x → payload
        const int64_t i = i0 + (int64_t)u * PT_THREADS;
        ok[u] = i < end && x[u] >= 0 && bit_get(kv, i) && bit_get(rv, i);
        if (windowed) {
          const int64_t lo = x[u] - size + adv;
          c_app += ok[u] ? (int64_t)fast_udiv((uint64_t)x[u], fd) - (int64_t)fast_udiv((uint64_t)(lo > 0 ? lo : 0), fd) + 1
                         : 0;
        } else {
          c_app += ok[u] ? 1 : 0;
        }
        x[u] = R8C ? (int64_t)(((uint64_t)(k[u] - kbase) << r8tb) | (uint64_t)(x[u] - tbase + 1))
                   : (r12 ? x[u] - tbase + 1 : x[u]);
        k[u] = (int64_t)key_hash(k[u]);  // records carry the key hash (key = its inverse)
      }
      if constexpr (R8C) {
        uint32_t bin[U];
#pragma unroll
        for (int u = 0; u < U; u++) bin[u] = stage_bin((uint64_t)k[u], shift, bmask);
        stage_step8<U>(x, bin, ok, P, SL8, srec, [&](int64_t p) {
          return stage_bin(key_hash(kbase + (int64_t)((uint64_t)p >> r8tb)), shift, bmask);
        });
      } else {
        constexpr int H = U / 2;
        int64_t kh[H], xh[H];
        bool okh[H];
#pragma unroll
        for (int half = 0; half < 2; half++) {
#pragma unroll
          for (int u = 0; u < H; u++) {
            kh[u] = k[half * H + u];
            xh[u] = x[half * H + u];
            okh[u] = ok[half * H + u];
          }
          stage_step<H>(kh, xh, okh, shift, bmask, P, SL, srec, r12 ? 1 : 0, tbase);
        }
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        x[u] = nxx[u];
        k[u] = nxk[u];
      }
    }
    };
    if (r8tb)
      run(std::true_type{});
    else
      run(std::false_type{});
  } else if (fast && NARROW) {
    // 16-byte (key, ts) records: straight-line steps (no branch around a load or store, so
    // every wait is counted), next step's loads issued before this step's cursors/stores;
    // rejected or out-of-range lanes store to the dummy record
    int64_t x[U], k[U], nxx[U], nxk[U];
    auto load_step = [&](int64_t i0, int64_t (&dx)[U], int64_t (&dk)[U]) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        int64_t i = i0 + (int64_t)u * PT_THREADS;
        i = i < end ? i : end - 1;
        dx[u] = ts[i];
        dk[u] = keys[i];
      }
    };
    int64_t i0 = base + threadIdx.x;
    if (i0 < end) load_step(i0, x, k);
    for (; i0 < end; i0 += U * PT_THREADS) {
      const int64_t in = i0 + U * PT_THREADS;
      if (in < end) load_step(in, nxx, nxk);
      uint32_t pos[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int64_t i = i0 + (int64_t)u * PT_THREADS;
        const bool ok = i < end && x[u] >= 0 && bit_get(kv, i) && bit_get(rv, i);
        if (windowed) {
          const int64_t lo = x[u] - size + adv;
          c_app += ok ? (int64_t)fast_udiv((uint64_t)x[u], fd) - (int64_t)fast_udiv((uint64_t)(lo > 0 ? lo : 0), fd) + 1
                      : 0;
        } else {
          c_app += ok ? 1 : 0;
        }
        if (r8tb) x[u] = (int64_t)(((uint64_t)(k[u] - kbase) << r8tb) | (uint64_t)(x[u] - tbase + 1));
        k[u] = (int64_t)key_hash(k[u]);  // records carry the key hash (key = its inverse)
        pos[u] = atomicAdd(&cur[part_of_hk((uint64_t)k[u], log2P)], ok ? 1u : 0u);
        if (!ok) pos[u] = 0xFFFFFFFFu;
      }
      if (r8tb) {
#pragma unroll
        for (int u = 0; u < U; u++) srec[pos[u] == 0xFFFFFFFFu ? (uint64_t)dummy : (uint64_t)pos[u]] = (uint64_t)x[u];
      } else if (r12) {
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint64_t dst = pos[u] == 0xFFFFFFFFu ? (uint64_t)dummy : (uint64_t)pos[u];
          r12_store(srec, dst, (uint64_t)k[u], (uint32_t)(x[u] - tbase + 1));
        }
      } else {
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint64_t dst = pos[u] == 0xFFFFFFFFu ? (uint64_t)dummy : (uint64_t)pos[u];
          *(longlong2*)(srec + dst * 2) = make_longlong2(k[u], x[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        x[u] = nxx[u];
        k[u] = nxk[u];
      }
    }
  } else if (fast && !NARROW && stage && L.rw == 4) {
    // 32-byte records through the LDS stage (stage_step_w): each bin's records of a step leave
    // as one contiguous run of whole records instead of one scattered record per lane; the next
    // step's key / ts / value loads are in flight during this step's barriers
    constexpr int WU = U >= 16 ? 4 : 2;
    constexpr int S = WU * PT_THREADS;
    const StageLds SL = stage_carve(smem, P, 2 * S, wsum);
    for (int p = threadIdx.x; p < P; p += PT_THREADS) SL.cnt[p] = 0u;
    lds_barrier();
    const int shift = log2P == 0 ? 64 : 64 - log2P;
    const uint32_t bmask = (uint32_t)(P - 1);
    const int c2 = L.word_col[2], c3 = L.word_col[3];
    int64_t x[WU], k[WU], v2[WU], v3[WU], nx[WU], nk[WU], nv2[WU], nv3[WU];
    auto load_step = [&](int64_t i0, int64_t (&dx)[WU], int64_t (&dk)[WU], int64_t (&d2)[WU], int64_t (&d3)[WU]) {
#pragma unroll
      for (int u = 0; u < WU; u++) {
        int64_t i = i0 + (int64_t)u * PT_THREADS;
        i = i < end ? i : end - 1;
        dx[u] = ts[i];
        dk[u] = keys[i];
        d2[u] = c2 >= 0 ? load_col_raw(cols, ctypes.t[c2], c2, i) : 0;
        d3[u] = c3 >= 0 ? load_col_raw(cols, ctypes.t[c3], c3, i) : 0;
      }
    };
    if (base < end) load_step(base + threadIdx.x, x, k, v2, v3);
    for (int64_t s0 = base; s0 < end; s0 += S) {  // uniform across the block: barriers inside
      const int64_t i0 = s0 + threadIdx.x;
      if (s0 + S < end) load_step(i0 + S, nx, nk, nv2, nv3);
      int64_t hk[WU], w2[WU], w3[WU];
      bool ok[WU];
#pragma unroll
      for (int u = 0; u < WU; u++) {
        const int64_t i = i0 + (int64_t)u * PT_THREADS;
        const int64_t ic = i < end ? i : end - 1;
        ok[u] = i < end && x[u] >= 0 && bit_get(kv, ic) && bit_get(rv, ic);
        uint32_t vm = 0;
        for (int c = 0; c < n_cols; c++)
          if ((L.vcols >> c) & 1u) vm |= (bit_get(cols.valid[c], ic) ? 1u : 0u) << c;
        w2[u] = L.meta_word == 2 ? (int64_t)(vm << 16) : v2[u];
        w3[u] = L.meta_word == 3 ? (int64_t)(vm << 16) : v3[u];
        if (windowed) {
          const int64_t lo = x[u] - size + adv;
          c_app += ok[u] ? (int64_t)fast_udiv((uint64_t)x[u], fd) - (int64_t)fast_udiv((uint64_t)(lo > 0 ? lo : 0), fd) + 1
                         : 0;
        } else {
          c_app += ok[u] ? 1 : 0;
        }
        hk[u] = (int64_t)key_hash(k[u]);
      }
      stage_step_w<WU>(hk, x, w2, w3, ok, shift, bmask, P, SL, srec);
#pragma unroll
      for (int u = 0; u < WU; u++) {
        x[u] = nx[u];
        k[u] = nk[u];
        v2[u] = nv2[u];
        v3[u] = nv3[u];
      }
    }
  } else if (fast) {
    // U records per thread per step: the loads of a step are issued together, and since
    // vmcnt retires loads and stores in issue order, fewer steps = fewer waits behind the
    // previous step's scattered stores
    for (int64_t i0 = base + threadIdx.x; i0 < end; i0 += U * PT_THREADS) {
      int64_t x[U], k[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int64_t i = i0 + u * PT_THREADS;
        ok[u] = i < end;
        x[u] = ok[u] ? ts[i] : -1;
        k[u] = ok[u] ? keys[i] : 0;
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int64_t i = i0 + u * PT_THREADS;
        if (!ok[u] || x[u] < 0 || !bit_get(kv, i) || !bit_get(rv, i)) continue;
        // windows [ws0, floor(x/adv)*adv] step adv, ws0 = floor(max(0, x-size+adv)/adv)*adv
        const int64_t lo = x[u] - size + adv;
        const int64_t nwin =
            windowed ? (int64_t)fast_udiv((uint64_t)x[u], fd) - (int64_t)fast_udiv((uint64_t)(lo > 0 ? lo : 0), fd) + 1
                     : 1;
        c_app += nwin;
        scatter_one(k[u], x[u], 0, i, log2P, cur, srec, L, cols, n_cols, ctypes, true, r12, tbase, r8tb, kbase);
      }
    }
  } else {
    for (int64_t r = 0; base + r * PT_THREADS < end; r++) {  // uniform across the block
      const int64_t i = base + (int64_t)r * PT_THREADS + threadIdx.x;
      const bool in = i < end;
      const int64_t x = in ? ts[i] : -1;
      const bool valid = in && bit_get(kv, i) && bit_get(rv, i) && x >= 0;
      int64_t tot;
      const int64_t incl = block_incl_max(valid ? x : -1, lmax, &tot);
      int64_t st = incl > carry ? incl : carry;
      carry = tot > carry ? tot : carry;
      if (!valid) continue;
      if (st_at) st = st_at[i];  // ABI 5 domains: given per row
      int64_t jlo = 0, nwin = 1;
      if (windowed) {
        const int64_t ws0 = first_window_start_fd(x, size, adv, fd);
        nwin = (int64_t)fast_udiv((uint64_t)(x - ws0), fd) + 1;
        // applied iff ws + size > st - grace  ⇔  ws >= st - grace - size + 1
        const int64_t wmin = st - grace - size + 1;
        if (wmin > ws0) jlo = (wmin - ws0 + adv - 1) / adv;
        if (jlo > nwin) jlo = nwin;
      }
      c_late += jlo;
      c_app += nwin - jlo;
      scatter_one(keys[i], x, jlo, i, log2P, cur, srec, L, cols, n_cols, ctypes, nwin > jlo, r12, tbase, r8tb, kbase);
    }
  }
  c_app = wave_sum(c_app);
  c_late = wave_sum(c_late);
  if ((threadIdx.x & 63) == 0) {
    if (c_app) atomicAdd(&lc[0], (unsigned long long)c_app);
    if (c_late) atomicAdd(&lc[1], (unsigned long long)c_late);
  }
  __syncthreads();
  if (pad) {  // fill each run's tail up to the next run's start with skipped records (ts = -1)
    for (int p = threadIdx.x; p < P; p += PT_THREADS) {
      const int64_t stop = t + 1 < nT ? (int64_t)offs[(t + 1) * P + p] : pbase[p + 1];
      for (int64_t q = cur[p]; q < stop; q++) *(longlong2*)(srec + (uint64_t)q * L.rw) = make_longlong2(0, -1);
    }
  }
  if (threadIdx.x == 0) {
    tpart[t * T_NPART + T_APPLIED] = (int64_t)lc[0];
    tpart[t * T_NPART + T_LATE] = (int64_t)lc[1];
  }
}

// One block's range [lo, hi) of bucket b → its partitions' runs (cursors in LDS).  N12: the
// 12-byte narrow records (RW = 2 layout) k_part_scatter wrote for k_part_merge; out16: widen
// them back to 16-byte (key hash, ts) records for the merge (tbase = the push's rowtime base).
template <int RW, bool N12>
__device__ __forceinline__ void refine_range(const uint64_t* __restrict__ srcA, uint32_t* cur, int64_t lo, int64_t hi,
                                             int log2P, int F, int64_t dummy, uint64_t* __restrict__ srec, int mode,
                                             bool out16, int64_t tbase) {
  // Straight-line steps (no branch around a load, so the waits stay counted): U records
  // per thread; the next step's loads are issued before this step's LDS cursors and
  // stores; out-of-range lanes load a clamped index and store to the dummy record.
  constexpr int U = RW <= 2 ? 8 : (RW <= 4 ? 4 : (RW <= 8 ? 2 : 1));  // ~64 VGPRs of records in flight
  constexpr int H2 = N12 ? 1 : RW / 2;
  longlong2 r[U][H2], nx[U][H2];
  R12 r3[U], nx3[U];
  auto load_step = [&](int64_t i0, longlong2 (&d)[U][H2], R12 (&d3)[U]) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      int64_t i = i0 + (int64_t)u * PT_THREADS;
      i = i < hi ? i : hi - 1;
      if constexpr (N12) {
        d3[u] = *(const R12*)((const char*)srcA + (uint64_t)i * 12);
      } else {
#pragma unroll
        for (int k = 0; k < H2; k++) d[u][k] = ((const longlong2*)(srcA + (uint64_t)i * RW))[k];
      }
    }
  };
  int64_t i0 = lo + threadIdx.x;
  load_step(i0, r, r3);
  for (; i0 < hi; i0 += U * PT_THREADS) {
    const int64_t in = i0 + U * PT_THREADS;
    if (in < hi) load_step(in, nx, nx3);
    uint32_t pos[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const bool ok = i0 + (int64_t)u * PT_THREADS < hi;
      const uint64_t hk = N12 ? ((uint64_t)r3[u].hi << 32 | r3[u].lo) : (uint64_t)r[u][0].x;
      const uint32_t f = part_of_hk(hk, log2P) & (uint32_t)(F - 1);
      pos[u] = atomicAdd(&cur[f], ok ? 1u : 0u);
      if (!ok) pos[u] = 0xFFFFFFFFu;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint64_t dst = pos[u] == 0xFFFFFFFFu ? (uint64_t)dummy : (uint64_t)pos[u];
      if (mode == 1) dst = pos[u] == 0xFFFFFFFFu ? (uint64_t)dummy : (uint64_t)(i0 + (int64_t)u * PT_THREADS);
      if constexpr (N12) {
        if (out16)
          *(longlong2*)(srec + dst * 2) = make_longlong2((int64_t)((uint64_t)r3[u].hi << 32 | r3[u].lo),
                                                         r3[u].trel ? tbase + (int64_t)r3[u].trel - 1 : -1);
        else
          *(R12*)((char*)srec + dst * 12) = r3[u];
      } else {
#pragma unroll
        for (int k = 0; k < H2; k++) ((longlong2*)(srec + dst * RW))[k] = r[u][k];
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      if constexpr (N12) {
        r3[u] = nx3[u];
      } else {
#pragma unroll
        for (int k = 0; k < H2; k++) r[u][k] = nx[u][k];
      }
    }
  }
}

// refine_range through the LDS stage (narrow records): out as in stage_step
template <bool N12, int U>
__device__ __forceinline__ void refine_staged(const uint64_t* __restrict__ srcA, const StageLds& SL, int64_t lo,
                                              int64_t hi, int log2P, int F, uint64_t* __restrict__ srec, int out,
                                              int64_t tbase) {
  constexpr int S = U * PT_THREADS;
  int64_t hk[U], nhk[U];
  int64_t pay[U], npay[U];
  auto load_step = [&](int64_t i0, int64_t (&dh)[U], int64_t (&dp)[U]) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      int64_t i = i0 + (int64_t)u * PT_THREADS;
      i = i < hi ? i : hi - 1;
      if constexpr (N12) {
        const R12 v = *(const R12*)((const char*)srcA + (uint64_t)i * 12);
        dh[u] = (int64_t)((uint64_t)v.hi << 32 | v.lo);
        dp[u] = (int64_t)v.trel;
      } else {
        const longlong2 v = *(const longlong2*)(srcA + (uint64_t)i * 2);
        dh[u] = v.x;
        dp[u] = v.y;
      }
    }
  };
  int64_t s0 = lo;
  load_step(s0 + threadIdx.x, hk, pay);
  for (; s0 < hi; s0 += S) {
    const int64_t i0 = s0 + threadIdx.x;
    if (s0 + S < hi) load_step(i0 + S, nhk, npay);
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; u++) ok[u] = i0 + (int64_t)u * PT_THREADS < hi;
    stage_step<U>(hk, pay, ok, 64 - log2P, (uint32_t)(F - 1), F, SL, srec, out, tbase);
#pragma unroll
    for (int u = 0; u < U; u++) {
      hk[u] = nhk[u];
      pay[u] = npay[u];
    }
  }
}

// refine_range for 32-byte records (RW = 4) through the LDS stage (stage_step_w), next step's
// loads in flight
template <int U, int NT = PT_THREADS>
__device__ __forceinline__ void refine_staged_w(const uint64_t* __restrict__ srcA, const StageLds& SL, int64_t lo,
                                                int64_t hi, int log2P, int F, uint64_t* __restrict__ srec) {
  constexpr int S = U * NT;
  longlong2 a[U], b[U], na[U], nb[U];
  auto load_step = [&](int64_t i0, longlong2 (&da)[U], longlong2 (&db)[U]) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      int64_t i = i0 + (int64_t)u * NT;
      i = i < hi ? i : hi - 1;
      da[u] = ((const longlong2*)(srcA + (uint64_t)i * 4))[0];
      db[u] = ((const longlong2*)(srcA + (uint64_t)i * 4))[1];
    }
  };
  int64_t s0 = lo;
  load_step(s0 + threadIdx.x, a, b);
  for (; s0 < hi; s0 += S) {
    const int64_t i0 = s0 + threadIdx.x;
    if (s0 + S < hi) load_step(i0 + S, na, nb);
    int64_t hk[U], ts[U], w2[U], w3[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      ok[u] = i0 + (int64_t)u * NT < hi;
      hk[u] = a[u].x;
      ts[u] = a[u].y;
      w2[u] = b[u].x;
      w3[u] = b[u].y;
    }
    stage_step_w<U, NT>(hk, ts, w2, w3, ok, 64 - log2P, (uint32_t)(F - 1), F, SL, srec);
#pragma unroll
    for (int u = 0; u < U; u++) {
      a[u] = na[u];
      b[u] = nb[u];
    }
  }
}

// R8 records (8 bytes: (key - kbase) << tb | trel) of one block's range → their partitions,
// through the LDS stage (staged) or straight to each partition's cursor
template <int U>
__device__ __forceinline__ void refine_r8(const uint64_t* __restrict__ srcA, const StageLds* SL, uint32_t* cur,
                                          int64_t lo, int64_t hi, int log2P, int F, uint64_t* __restrict__ srec,
                                          int tb, int64_t kbase, int64_t dummy) {
  constexpr int S = U * PT_THREADS;
  int64_t hk[U], pay[U], npay[U];
  auto load_step = [&](int64_t i0, int64_t (&dp)[U]) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      int64_t i = i0 + (int64_t)u * PT_THREADS;
      i = i < hi ? i : hi - 1;
      dp[u] = (int64_t)__builtin_nontemporal_load(srcA + i);
    }
  };
  int64_t s0 = lo;
  load_step(s0 + threadIdx.x, pay);
  for (; s0 < hi; s0 += S) {
    const int64_t i0 = s0 + threadIdx.x;
    if (s0 + S < hi) load_step(i0 + S, npay);
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      ok[u] = i0 + (int64_t)u * PT_THREADS < hi;
      hk[u] = (int64_t)key_hash(kbase + (int64_t)((uint64_t)pay[u] >> tb));
    }
    if (SL) {
      uint32_t bin[U];
#pragma unroll
      for (int u = 0; u < U; u++) bin[u] = stage_bin((uint64_t)hk[u], 64 - log2P, (uint32_t)(F - 1));
      StageLds SL8 = *SL;
      SL8.sp = (int64_t*)SL->sk;
      stage_step8<U>(pay, bin, ok, F, SL8, srec, [&](int64_t p) {
        return stage_bin(key_hash(kbase + (int64_t)((uint64_t)p >> tb)), 64 - log2P, (uint32_t)(F - 1));
      });
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t pos = atomicAdd(&cur[part_of_hk((uint64_t)hk[u], log2P) & (uint32_t)(F - 1)], ok[u] ? 1u : 0u);
        srec[ok[u] ? (uint64_t)pos : (uint64_t)dummy] = (uint64_t)pay[u];
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) pay[u] = npay[u];
  }
}

// Two-level scatter, pass B: block (bucket b, tile group g) moves the records that pass A
// (k_part_scatter over the B = P >> fbits buckets) put in bucket b for tiles [t0, t1) — one
// contiguous range, since pass A lays each bucket out tile-major — to their partitions' final
// runs (cursors = the fine offsets of tile t0).  Every partition's run per group is G tiles
// long, so the stores combine into whole lines where pass A alone would leave ~64-byte runs.
template <int RW>
__device__ __forceinline__ void refine_block(int64_t vb, const uint64_t* __restrict__ srcA,
                                             const uint32_t* __restrict__ offA, const uint32_t* __restrict__ offs,
                                             const int64_t* __restrict__ pbase, int64_t nT, int G, int log2P,
                                             int fbits, int64_t dummy, uint64_t* __restrict__ srec, int mode,
                                             const int64_t* __restrict__ wr, int r12_ok, int stage) {
  __shared__ uint32_t cur[1 << 12];
  const int F = 1 << fbits, P = 1 << log2P, B = P >> fbits;
  const int64_t ng = (nT + G - 1) / G;
  const int b = (int)(vb / ng);
  const int64_t g = vb % ng;
  const int64_t t0 = g * G, t1 = t0 + G < nT ? t0 + G : nT;
  if (RW == 2 && stage) {  // narrow records through the LDS stage
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int wsum[PT_THREADS / 64];
    // the stage holds stage * PT_THREADS 8-byte records (stage = records per thread): R8 steps use
    // it whole, the 12/16-byte records half as many 16-byte pairs per step
    const StageLds SL = stage_carve(smem, F, stage * PT_THREADS / 2, wsum);
    for (int f = threadIdx.x; f < F; f += PT_THREADS) {
      SL.cur[f] = offs[t0 * P + ((int64_t)b << fbits) + f];
      SL.cnt[f] = 0u;
    }
    const int64_t lo = offA[t0 * B + b];
    const int64_t hi = t1 < nT ? (int64_t)offA[t1 * B + b] : pbase[(int64_t)(b + 1) << fbits];
    lds_barrier();
    if (hi <= lo) return;
    const bool n12 = r12_ok && wr[4] != 0;
    if (n12 && wr[7]) {
      if (stage >= 8) refine_r8<8>(srcA, &SL, nullptr, lo, hi, log2P, F, srec, (int)wr[7], wr[6], dummy);
      else refine_r8<4>(srcA, &SL, nullptr, lo, hi, log2P, F, srec, (int)wr[7], wr[6], dummy);
      return;
    }
    if (stage >= 8) {
      if (n12) refine_staged<true, 4>(srcA, SL, lo, hi, log2P, F, srec, r12_ok == 2 ? 2 : 1, wr[5]);
      else refine_staged<false, 4>(srcA, SL, lo, hi, log2P, F, srec, 0, 0);
    } else {
      if (n12) refine_staged<true, 2>(srcA, SL, lo, hi, log2P, F, srec, r12_ok == 2 ? 2 : 1, wr[5]);
      else refine_staged<false, 2>(srcA, SL, lo, hi, log2P, F, srec, 0, 0);
    }
    return;
  }
  if (RW == 4 && stage) {  // 32-byte records through the LDS stage (stage = records per thread per step)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int wsum[PT_THREADS / 64];
    const StageLds SL = stage_carve(smem, F, 2 * stage * PT_THREADS, wsum);
    for (int f = threadIdx.x; f < F; f += PT_THREADS) {
      SL.cur[f] = offs[t0 * P + ((int64_t)b << fbits) + f];
      SL.cnt[f] = 0u;
    }
    const int64_t lo = offA[t0 * B + b];
    const int64_t hi = t1 < nT ? (int64_t)offA[t1 * B + b] : pbase[(int64_t)(b + 1) << fbits];
    lds_barrier();
    if (hi <= lo) return;
    if (stage >= 4) refine_staged_w<4>(srcA, SL, lo, hi, log2P, F, srec);
    else refine_staged_w<2>(srcA, SL, lo, hi, log2P, F, srec);
    return;
  }
  for (int f = threadIdx.x; f < F; f += PT_THREADS) cur[f] = offs[t0 * P + ((int64_t)b << fbits) + f];
  __syncthreads();
  const int64_t lo = offA[t0 * B + b];
  const int64_t hi = t1 < nT ? (int64_t)offA[t1 * B + b] : pbase[(int64_t)(b + 1) << fbits];
  if (hi <= lo) return;
  if (RW == 2 && r12_ok && wr[4] != 0 && wr[7])
    refine_r8<8>(srcA, nullptr, cur, lo, hi, log2P, F, srec, (int)wr[7], wr[6], dummy);
  else if (RW == 2 && r12_ok && wr[4] != 0)
    refine_range<RW, true>(srcA, cur, lo, hi, log2P, F, dummy, srec, mode, r12_ok == 2, wr[5]);
  else
    refine_range<RW, false>(srcA, cur, lo, hi, log2P, F, dummy, srec, mode, false, 0);
}

// Blocks (bucket, tile group) = vb in [0, B * ng).  Narrow records: grid-strided, and the host
// launches a grid of two workgroups per CU when k_part_refine_r8 may take the push instead
// (skip_r8), so that when it does, this launch costs ~500 exiting workgroups instead of ~12K.
template <int RW>
__global__ __launch_bounds__(PT_THREADS) void k_part_refine(const uint64_t* __restrict__ srcA,
                                                            const uint32_t* __restrict__ offA,
                                                            const uint32_t* __restrict__ offs,
                                                            const int64_t* __restrict__ pbase, int64_t nT, int G,
                                                            int log2P, int fbits, int64_t dummy,
                                                            uint64_t* __restrict__ srec, int mode,
                                                            const int64_t* __restrict__ wr, int r12_ok, int stage,
                                                            int skip_r8) {
  if (RW == 2 && stage && skip_r8 && r12_ok && wr[4] != 0 && wr[7]) return;  // k_part_refine_r8's
  if constexpr (RW == 2) {
    const int64_t nblk = (int64_t)((1 << log2P) >> fbits) * ((nT + G - 1) / G);
    for (int64_t vb = blockIdx.x; vb < nblk; vb += gridDim.x) {
      refine_block<RW>(vb, srcA, offA, offs, pbase, nT, G, log2P, fbits, dummy, srec, mode, wr, r12_ok, stage);
      __syncthreads();  // the block's LDS (cursors, stage) is reused by the next one
    }
  } else {  // wide records (no R8 alternative): one block per workgroup (the loop cost registers)
    refine_block<RW>(blockIdx.x, srcA, offA, offs, pbase, nT, G, log2P, fbits, dummy, srec, mode, wr, r12_ok, stage);
  }
}

// ------------------------------------------------------------------ R8 scatter / refine
// The R8 (8-byte record) steps of k_part_scatter and k_part_refine as kernels of their own, of NT
// threads: register allocation sees only this path (inside the general kernels the other record
// layouts' loops put it at the 128-VGPR cap with the next step's prefetched records spilled to
// scratch, one 1024-thread workgroup per CU), and two NT = 512 workgroups share a CU, so one's
// four stage barriers per step overlap the other's loads and stores.  Each staged record keeps
// its bin beside it in LDS (u16), so the write-out does not hash the key again.

// Pass A for a push whose records are R8 (wr[4] && wr[7], decided on the device by
// k_part_wrange): the tiles with no late record (k_part_scatter's `fast` test); k_part_scatter
// (skip_r8) takes the others.  Same output as k_part_scatter's staged R8 path.
template <int U, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void k_part_scatter_r8(
    const int64_t* __restrict__ keys, const int64_t* __restrict__ ts, const uint8_t* __restrict__ kv,
    const uint8_t* __restrict__ rv, int64_t n, int64_t tile, int log2P, int64_t nT, const uint32_t* __restrict__ offs,
    const int64_t* __restrict__ tileprefix, const int64_t* __restrict__ tilemax, const int64_t* __restrict__ tilemin,
    int windowed, int64_t size, int64_t adv, FastDiv fd, int64_t grace, uint64_t* __restrict__ srec,
    int64_t* __restrict__ tpart, const int64_t* __restrict__ wr) {
  if (wr[4] == 0 || wr[7] == 0) return;
  const int64_t t = tile_of(blockIdx.x, nT);
  const int64_t carry = tileprefix[t];
  const int64_t smax = carry > tilemax[t] ? carry : tilemax[t];
  const int64_t tmin = tilemin[t];
  const bool fast = !windowed || tmin == INT64_MAX || first_window_start(tmin, size, adv) + size > smax - grace;
  if (!fast) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int wsum[NT / 64];
  __shared__ unsigned long long lc;
  constexpr int S = U * NT;
  const int P = 1 << log2P;
  const StageR8 L = stage_r8_carve(smem, P, S, wsum);
  for (int p = threadIdx.x; p < P; p += NT) {
    L.cur[p] = offs[t * P + p];
    L.cnt[p] = 0u;
  }
  if (threadIdx.x == 0) lc = 0;
  const int tb = (int)wr[7];
  const int64_t tbase = wr[5], kbase = wr[6];
  const int shift = log2P == 0 ? 64 : 64 - log2P;
  const uint32_t bmask = (uint32_t)(P - 1);
  const int64_t base = t * tile;
  const int64_t end = base + tile < n ? base + tile : n;
  int64_t c_app = 0;
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
  lds_barrier();
  int64_t s0 = base;
  if (s0 < end) load_step(s0 + threadIdx.x, x, k);
  for (; s0 < end; s0 += S) {  // uniform across the block: barriers inside
    const int64_t i0 = s0 + threadIdx.x;
    bool ok[U];
    uint32_t bin[U];
    int64_t rec[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t i = i0 + (int64_t)u * NT;
      ok[u] = i < end && x[u] >= 0 && bit_get(kv, i) && bit_get(rv, i);
      if (windowed) {
        const int64_t lo = x[u] - size + adv;
        c_app += ok[u] ? (int64_t)fast_udiv((uint64_t)x[u], fd) - (int64_t)fast_udiv((uint64_t)(lo > 0 ? lo : 0), fd) + 1
                       : 0;
      } else {
        c_app += ok[u] ? 1 : 0;
      }
      bin[u] = stage_bin(key_hash(k[u]), shift, bmask);
      rec[u] = (int64_t)(((uint64_t)(k[u] - kbase) << tb) | (uint64_t)(x[u] - tbase + 1));
    }
    // the next step's loads go into x / k (dead now) and stay in flight through this step's stage
    if (s0 + S < end) load_step(i0 + S, x, k);
    stage_step_r8<U, NT>(rec, bin, ok, P, L, srec);
  }
  c_app = wave_sum(c_app);
  if ((threadIdx.x & 63) == 0 && c_app) atomicAdd(&lc, (unsigned long long)c_app);
  __syncthreads();
  if (threadIdx.x == 0) {
    tpart[t * T_NPART + T_APPLIED] = (int64_t)lc;
    tpart[t * T_NPART + T_LATE] = 0;
  }
}

// Pass B of R8 records (k_part_refine's staged R8 path): block (bucket b, tile group g).
template <int U, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void k_part_refine_r8(const uint64_t* __restrict__ srcA,
                                                          const uint32_t* __restrict__ offA,
                                                          const uint32_t* __restrict__ offs,
                                                          const int64_t* __restrict__ pbase, int64_t nT, int G,
                                                          int log2P, int fbits, uint64_t* __restrict__ srec,
                                                          const int64_t* __restrict__ wr) {
  if (wr[4] == 0 || wr[7] == 0) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int wsum[NT / 64];
  constexpr int S = U * NT;
  const int F = 1 << fbits, P = 1 << log2P, B = P >> fbits;
  const int64_t ng = (nT + G - 1) / G;
  const int b = (int)(blockIdx.x / ng);
  const int64_t g = blockIdx.x % ng;
  const int64_t t0 = g * G, t1 = t0 + G < nT ? t0 + G : nT;
  const StageR8 L = stage_r8_carve(smem, F, S, wsum);
  for (int f = threadIdx.x; f < F; f += NT) {
    L.cur[f] = offs[t0 * P + ((int64_t)b << fbits) + f];
    L.cnt[f] = 0u;
  }
  const int64_t lo = offA[t0 * B + b];
  const int64_t hi = t1 < nT ? (int64_t)offA[t1 * B + b] : pbase[(int64_t)(b + 1) << fbits];
  lds_barrier();
  if (hi <= lo) return;
  const int tb = (int)wr[7];
  const int64_t kbase = wr[6];
  const int shift = 64 - log2P;
  const uint32_t fmask = (uint32_t)(F - 1);
  int64_t pay[U], npay[U];
  auto load_step = [&](int64_t i0, int64_t (&dp)[U]) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      int64_t i = i0 + (int64_t)u * NT;
      i = i < hi ? i : hi - 1;
      dp[u] = (int64_t)__builtin_nontemporal_load(srcA + i);
    }
  };
  int64_t s0 = lo;
  load_step(s0 + threadIdx.x, pay);
  for (; s0 < hi; s0 += S) {  // uniform across the block: barriers inside
    const int64_t i0 = s0 + threadIdx.x;
    if (s0 + S < hi) load_step(i0 + S, npay);
    bool ok[U];
    uint32_t bin[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      ok[u] = i0 + (int64_t)u * NT < hi;
      bin[u] = stage_bin(key_hash(kbase + (int64_t)((uint64_t)pay[u] >> tb)), shift, fmask);
    }
    stage_step_r8<U, NT>(pay, bin, ok, F, L, srec);
#pragma unroll
    for (int u = 0; u < U; u++) pay[u] = npay[u];
  }
}

// ------------------------------------------------------------------ wide scatter / refine
// The 32-byte-record (rw = 4: key hash, ts, meta / value words; C3) staged steps of k_part_scatter
// as a kernel of its own, of NT = 512 threads, two workgroups per CU — the same change as the R8
// kernels above — for the tiles with no late record (the host launches k_part_scatter with skip
// set for the rest).  C3: 1956 → 1815 µs per push.  The same split of the wide refine pass was
// slower (1784 → 1989 µs; profiles/r03/ab/wide_kernels.txt) and is not kept.
template <int WU, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void k_part_scatter_w(
    const int64_t* __restrict__ keys, const int64_t* __restrict__ ts, const uint8_t* __restrict__ kv,
    const uint8_t* __restrict__ rv, ColPtrs cols, int n_cols, ColTypes ctypes, int64_t n, int64_t tile, int log2P,
    int64_t nT, const uint32_t* __restrict__ offs, const int64_t* __restrict__ tileprefix,
    const int64_t* __restrict__ tilemax, const int64_t* __restrict__ tilemin, int windowed, int64_t size, int64_t adv,
    FastDiv fd, int64_t grace, RecLayout L, uint64_t* __restrict__ srec, int64_t* __restrict__ tpart) {
  const int64_t t = tile_of(blockIdx.x, nT);
  const int64_t carry = tileprefix[t];
  const int64_t smax = carry > tilemax[t] ? carry : tilemax[t];
  const int64_t tmin = tilemin[t];
  const bool fast = !windowed || tmin == INT64_MAX || first_window_start(tmin, size, adv) + size > smax - grace;
  if (!fast) return;  // k_part_scatter's tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int wsum[NT / 64];
  __shared__ unsigned long long lc;
  constexpr int S = WU * NT;
  const int P = 1 << log2P;
  const StageLds SL = stage_carve(smem, P, 2 * S, wsum);
  for (int p = threadIdx.x; p < P; p += NT) {
    SL.cur[p] = offs[t * P + p];
    SL.cnt[p] = 0u;
  }
  if (threadIdx.x == 0) lc = 0;
  lds_barrier();
  const int shift = log2P == 0 ? 64 : 64 - log2P;
  const uint32_t bmask = (uint32_t)(P - 1);
  const int c2 = L.word_col[2], c3 = L.word_col[3];
  const int64_t base = t * tile;
  const int64_t end = base + tile < n ? base + tile : n;
  int64_t c_app = 0;
  int64_t x[WU], k[WU], v2[WU], v3[WU], nx[WU], nk[WU], nv2[WU], nv3[WU];
  auto load_step = [&](int64_t i0, int64_t (&dx)[WU], int64_t (&dk)[WU], int64_t (&d2)[WU], int64_t (&d3)[WU]) {
#pragma unroll
    for (int u = 0; u < WU; u++) {
      int64_t i = i0 + (int64_t)u * NT;
      i = i < end ? i : end - 1;
      dx[u] = ts[i];
      dk[u] = keys[i];
      d2[u] = c2 >= 0 ? load_col_raw(cols, ctypes.t[c2], c2, i) : 0;
      d3[u] = c3 >= 0 ? load_col_raw(cols, ctypes.t[c3], c3, i) : 0;
    }
  };
  if (base < end) load_step(base + threadIdx.x, x, k, v2, v3);
  for (int64_t s0 = base; s0 < end; s0 += S) {  // uniform across the block: barriers inside
    const int64_t i0 = s0 + threadIdx.x;
    if (s0 + S < end) load_step(i0 + S, nx, nk, nv2, nv3);
    int64_t hk[WU], w2[WU], w3[WU];
    bool ok[WU];
#pragma unroll
    for (int u = 0; u < WU; u++) {
      const int64_t i = i0 + (int64_t)u * NT;
      const int64_t ic = i < end ? i : end - 1;
      ok[u] = i < end && x[u] >= 0 && bit_get(kv, ic) && bit_get(rv, ic);
      uint32_t vm = 0;
      for (int c = 0; c < n_cols; c++)
        if ((L.vcols >> c) & 1u) vm |= (bit_get(cols.valid[c], ic) ? 1u : 0u) << c;
      w2[u] = L.meta_word == 2 ? (int64_t)(vm << 16) : v2[u];
      w3[u] = L.meta_word == 3 ? (int64_t)(vm << 16) : v3[u];
      if (windowed) {
        const int64_t lo = x[u] - size + adv;
        c_app += ok[u] ? (int64_t)fast_udiv((uint64_t)x[u], fd) - (int64_t)fast_udiv((uint64_t)(lo > 0 ? lo : 0), fd) + 1
                       : 0;
      } else {
        c_app += ok[u] ? 1 : 0;
      }
      hk[u] = (int64_t)key_hash(k[u]);
    }
    stage_step_w<WU, NT>(hk, x, w2, w3, ok, shift, bmask, P, SL, srec);
#pragma unroll
    for (int u = 0; u < WU; u++) {
      x[u] = nx[u];
      k[u] = nk[u];
      v2[u] = nv2[u];
      v3[u] = nv3[u];
    }
  }
  c_app = wave_sum(c_app);
  if ((threadIdx.x & 63) == 0 && c_app) atomicAdd(&lc, (unsigned long long)c_app);
  __syncthreads();
  if (threadIdx.x == 0) {
    tpart[t * T_NPART + T_APPLIED] = (int64_t)lc;
    tpart[t * T_NPART + T_LATE] = 0;
  }
}

// ------------------------------------------------------------------ k_part_agg
// Work item: blockIdx.x = partition (work == nullptr), or work[blockIdx.x] =
// p | sub_bits << 16 | sub << 20  (retry with 2^sub_bits sub-passes, sub_bits <= 12).
// LDS: lref u32[H] | words i64[nwords][H]  (word 0 key, 1 ws, 2 rowtime, 3.. state)


__device__ __forceinline__ void lds_apply(const PartAggParams& q, lds_i64* lw, int H, int e, int64_t t,
                                          uint32_t vmask, const uint64_t* __restrict__ srec, int64_t gi, int64_t w3) {
  __hip_atomic_fetch_max(&lw[2 * H + e], t, WG_RLX);
  for (int o = 0; o < q.n_ops; o++) {
    const UpdOp op = q.ops[o];
    lds_i64* w = &lw[op.word * H + e];
    if (op.kind == OP_INC) {
      __hip_atomic_fetch_add(w, (int64_t)1, WG_RLX);
      continue;
    }
    if (!((vmask >> op.col) & 1u)) continue;
    const int cw = q.col_word[op.col];  // word 3 came with the record's second 16 bytes
    const int64_t raw = cw == 3 ? w3 : (int64_t)srec[(uint64_t)gi * q.rw + cw];
    switch (op.kind) {
      case OP_INC_VALID: __hip_atomic_fetch_add(w, (int64_t)1, WG_RLX); break;
      case OP_ADD_I64: __hip_atomic_fetch_add((KLDS uint64_t*)w, (uint64_t)raw, WG_RLX); break;
      case OP_ADD_F64: {
        double d;
        __builtin_memcpy(&d, &raw, 8);
        __hip_atomic_fetch_add((lds_f64*)w, d, WG_RLX);
        break;
      }
      case OP_MIN:
      case OP_MAX: {
        int64_t k = raw;
        if (q.col_type[op.col] == KHIP_TYPE_DOUBLE) {
          double d;
          __builtin_memcpy(&d, &raw, 8);
          k = f64_order_key(d);
        }
        if (op.kind == OP_MIN) __hip_atomic_fetch_min(w, k, WG_RLX);
        else __hip_atomic_fetch_max(w, k, WG_RLX);
        break;
      }
      default: break;
    }
  }
}

__global__ __launch_bounds__(AG_THREADS) void k_part_agg(PartAggParams q, const uint32_t* __restrict__ work,
                                                         const int64_t* __restrict__ pbase,
                                                         const uint64_t* __restrict__ srec, int first,
                                                         uint64_t* __restrict__ buf0, uint64_t* __restrict__ buf1,
                                                         const uint8_t* __restrict__ sel,
                                                         const int64_t* __restrict__ cnt,
                                                         unsigned long long* __restrict__ newcnt,
                                                         uint8_t* __restrict__ fail,
                                                         unsigned long long* __restrict__ need, int64_t close0,
                                                         uint64_t* __restrict__ closed,
                                                         unsigned long long* __restrict__ closed_n,
                                                         const int64_t* __restrict__ wr,
                                                         unsigned long long* __restrict__ dbg) {
#define AGG_T(k) do { if (dbg && threadIdx.x == 0) dbg[blockIdx.x * 6 + (k)] = wall_clock64(); } while (0)
  AGG_T(0);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = q.H;
  lds_u32* lref = (lds_u32*)smem;
  lds_i64* lw = (lds_i64*)(smem + (((size_t)H * 4 + 15) & ~(size_t)15));
  volatile lds_u32* vlref = lref;
  volatile lds_i64* vlw = lw;
  __shared__ int lovf;
  __shared__ int lcnt[AG_THREADS / 64];
  __shared__ unsigned long long lbase;
  uint32_t p;
  int sbits = 0, sub = 0;
  if (work) {
    const uint32_t w = work[blockIdx.x];
    p = w & 0xFFFFu;
    sbits = (w >> 16) & 0xF;
    sub = (int)(w >> 20);
  } else {
    p = blockIdx.x;
  }
  const int64_t rbase = pbase[p], rn = pbase[p + 1] - rbase;
  if (rn == 0 && first) return;  // untouched partition: nothing to rewrite
  // the first AU records of every thread are loaded before the LDS table is initialised,
  // so the HBM latency overlaps the init instead of following it
  constexpr int AU = 8;
  const bool wide = q.rw > 2;
  longlong2 rec[AU], ext[AU];
#pragma unroll
  for (int u = 0; u < AU; u++) {
    const int64_t li = threadIdx.x + (int64_t)u * AG_THREADS;
    const longlong2* r = (const longlong2*)(srec + (uint64_t)(rbase + li) * q.rw);
    rec[u] = li < rn ? r[0] : make_longlong2(0, -1);
    ext[u] = (wide && li < rn) ? r[1] : make_longlong2(0, 0);
  }
  // identity-CAS mode (the window range of this push fits the packed identity, wr[1]):
  // plane 0 holds the 64-bit identities, every state word starts initialised, and a group
  // is found or created by ONE 64-bit CAS — no claim/ready protocol, no spinning.
  // Otherwise only the slot states are initialised and a claimer writes its entry's words.
  const bool idm = wr[1] != 0;
  const int64_t wbase = wr[0];
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
  if (idm) {
    for (int i = threadIdx.x; i < H / 2; i += AG_THREADS) ((KLDS i64x2*)lw)[i] = i64x2{-1LL, -1LL};
    for (int w = 2; w < q.nwords; w++) {
      const int64_t v = q.init.w[w];
      for (int i = threadIdx.x; i < H / 2; i += AG_THREADS) ((KLDS i64x2*)(lw + w * H))[i] = i64x2{v, v};
    }
  } else {
    for (int i = threadIdx.x; i < H / 4; i += AG_THREADS) ((KLDS u32x4*)lref)[i] = u32x4{0u, 0u, 0u, 0u};
  }
  lds_u32* lflag = q.flag_off ? (lds_u32*)(smem + q.flag_off) : nullptr;  // 4 entries per word
  if (lflag)
    for (int i = threadIdx.x; i < H / 4; i += AG_THREADS) lflag[i] = 0u;
  if (threadIdx.x == 0) lovf = 0;
  __syncthreads();
  AGG_T(1);
  // 1. resident rows of this partition (distinct groups: insert without comparing).  Rows of
  //    windows already closed before this push (ws + size <= close0) go to the closed store.
  const uint64_t* src = (sel[p] ? buf1 : buf0) + (uint64_t)p * q.cmax * q.sw;
  const int64_t nrow = cnt[p];
  const bool evict = q.windowed && close0 != INT64_MIN;
  // the first pass moves the closed rows; a retried partition already moved them (its region
  // still holds them until it succeeds), so retries only skip them
  if (evict && first) {
    int ne = 0;
    for (int64_t r = threadIdx.x; r < nrow; r += AG_THREADS) {
      const uint64_t* row = src + r * q.sw;
      ne += ((int64_t)row[1] + q.size <= close0) && sub_ok(key_hash((int64_t)row[0]), (int64_t)row[1], sbits, sub);
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int incl = ne;
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(incl, off, 64);
      if (lane >= off) incl += y;
    }
    if (lane == 63) lcnt[wave] = incl;
    __syncthreads();
    int before = 0, total = 0;
    for (int w = 0; w < AG_THREADS / 64; w++) {
      if (w < wave) before += lcnt[w];
      total += lcnt[w];
    }
    if (threadIdx.x == 0) lbase = total ? atomicAdd(closed_n, (unsigned long long)total) : 0ULL;
    __syncthreads();
    uint64_t* dst = closed + (lbase + (uint64_t)(before + incl - ne)) * q.sw;
    for (int64_t r = threadIdx.x; r < nrow; r += AG_THREADS) {
      const uint64_t* row = src + r * q.sw;
      if (!((int64_t)row[1] + q.size <= close0) || !sub_ok(key_hash((int64_t)row[0]), (int64_t)row[1], sbits, sub))
        continue;
      for (int w = 0; w < q.sw; w++) dst[w] = row[w];
      dst += q.sw;
    }
    __syncthreads();
  }
  for (int64_t r = threadIdx.x; r < nrow; r += AG_THREADS) {
    const uint64_t* row = src + r * q.sw;
    const int64_t key = (int64_t)row[0], ws = (int64_t)row[1];
    if (evict && ws + q.size <= close0) continue;
    const uint64_t hk = key_hash(key);
    if (!sub_ok(hk, ws, sbits, sub)) continue;
    uint32_t e = slot_of(hk, ws, H);
    int probe = 0;
    if (idm) {
      const uint64_t id = ident_of(hk, (int64_t)fast_udiv((uint64_t)ws, q.fd) - wbase, q.log2P);
      for (; probe < H; probe++) {
        uint64_t expect = EMPTY_ID;
        if (__hip_atomic_compare_exchange_strong((KLDS uint64_t*)&lw[e], &expect, id, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
          break;
        e = (e + 1) & (uint32_t)(H - 1);
      }
      if (probe == H) {
        lovf = 1;
        break;
      }
      for (int w = 2; w < q.nwords; w++) lw[w * H + e] = (int64_t)row[w];
      if (lflag && having_ok(row, q.having)) __hip_atomic_fetch_or(&lflag[e >> 2], 2u << ((e & 3) * 8), WG_RLX);
      continue;
    }
    for (; probe < H; probe++) {
      uint32_t expect = 0u;
      if (__hip_atomic_compare_exchange_strong(&lref[e], &expect, fp_of(hk, ws) | L_READY, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP))
        break;
      e = (e + 1) & (uint32_t)(H - 1);
    }
    if (probe == H) {  // more resident groups than LDS slots: retry with sub-passes
      lovf = 1;
      break;
    }
    for (int w = 0; w < q.nwords; w++) lw[w * H + e] = (int64_t)row[w];
    if (lflag && having_ok(row, q.having)) __hip_atomic_fetch_or(&lflag[e >> 2], 2u << ((e & 3) * 8), WG_RLX);
  }
  if (dbg) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  __syncthreads();
  AGG_T(2);
  // 2. this batch's records.  Slot states: 0 empty → L_CLAIM (the CAS winner writes key, ws
  //    and the initial words) → L_READY; a loser waits for READY (the winner is another wave,
  //    or an earlier instruction of its own wave), then compares key/ws in LDS.  A probe
  //    sequence that wraps the whole table marks the partition for a retry with sub-passes.
  for (int64_t l0 = threadIdx.x; l0 < rn; l0 += AU * AG_THREADS) {
    if (*(volatile KLDS int*)&lovf) break;
    if (l0 != threadIdx.x) {
#pragma unroll
      for (int u = 0; u < AU; u++) {  // AU records in flight per thread
        const int64_t li = l0 + u * AG_THREADS;
        const longlong2* r = (const longlong2*)(srec + (uint64_t)(rbase + li) * q.rw);
        rec[u] = li < rn ? r[0] : make_longlong2(0, -1);
        ext[u] = (wide && li < rn) ? r[1] : make_longlong2(0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < AU; u++) {  // unrolled: rec[]/ext[] stay in registers (no scratch)
      const int64_t t = rec[u].y;
      if (t < 0) continue;  // every window late (or past the end)
      const uint64_t hk = (uint64_t)rec[u].x;  // the scatter stores the key hash
      const int64_t key = key_of_hash(hk);
      const int64_t gi = rbase + l0 + u * AG_THREADS;
      const uint32_t meta = q.meta_word == 2 ? (uint32_t)ext[u].x : 0u;
      const int64_t jlo = meta & 0xFFFFu;
      const uint32_t vmask = meta >> 16;
      const int64_t w3 = ext[u].y;
      int64_t ws = 0, wlast = 0, widx = 0;
      if (q.windowed) {
        int64_t lo = t - q.size + q.adv;
        widx = (int64_t)fast_udiv((uint64_t)(lo > 0 ? lo : 0), q.fd) + jlo;
        ws = widx * q.adv;
        wlast = t;
      }
      for (; ws <= wlast; ws += q.adv, widx++) {
        if (!sub_ok(hk, ws, sbits, sub)) continue;
        uint32_t e = slot_of(hk, ws, H);
        if (idm) {
          const uint64_t id = ident_of(hk, widx - wbase, q.log2P);
          bool got = false;
          for (int probe = 0; probe < H; probe++) {
            uint64_t old = EMPTY_ID;
            __hip_atomic_compare_exchange_strong((KLDS uint64_t*)&lw[e], &old, id, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
            if (old == EMPTY_ID || old == id) {
              got = true;
              break;
            }
            e = (e + 1) & (uint32_t)(H - 1);
          }
          if (!got) {
            lovf = 1;
            break;
          }
          if (!(q.dbg_mode & 1)) lds_apply(q, lw, H, (int)e, t, vmask, srec, gi, w3);
          if (lflag) __hip_atomic_fetch_or(&lflag[e >> 2], 1u << ((e & 3) * 8), WG_RLX);
          continue;
        }
        const uint32_t fp = fp_of(hk, ws);
        bool found = q.dbg_mode & 2;
        for (int probe = 0; probe < H && !(q.dbg_mode & 2); probe++) {
          // state, key and ws in one round trip (issue order = LDS service order: a READY
          // state read before the key/ws reads guarantees they see the claimer's words)
          uint32_t v = vlref[e];
          int64_t k0 = vlw[e], w0 = vlw[H + e];
          if (v == 0u) {
            uint32_t old = 0u;
            __hip_atomic_compare_exchange_strong(&lref[e], &old, fp | L_CLAIM, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
            if (old == 0u) {
              vlw[e] = key;
              vlw[H + e] = ws;
              for (int w = 2; w < q.nwords; w++) vlw[w * H + e] = q.init.w[w];
              // LDS serves one wave's requests in issue order: once READY is visible, so are
              // the entry's words.  Only the compiler must not reorder.
              __atomic_signal_fence(__ATOMIC_SEQ_CST);
              vlref[e] = fp | L_READY;
              found = true;
              break;
            }
            v = old;
            k0 = vlw[e];
            w0 = vlw[H + e];
          }
          if ((v & ~3u) == fp) {  // same fingerprint: maybe this group
            if ((v & 3u) == L_CLAIM) {  // the claimer is a few stores away
              for (int spin = 0; (v & 3u) == L_CLAIM && spin <= (1 << 20); spin++) {
                __builtin_amdgcn_s_sleep(1);
                v = vlref[e];
              }
              if ((v & 3u) == L_CLAIM) break;  // never expected: fail the partition rather than hang
              __atomic_signal_fence(__ATOMIC_SEQ_CST);
              k0 = vlw[e];  // read after READY was seen
              w0 = vlw[H + e];
            }
            if (k0 == key && w0 == ws) {
              found = true;
              break;
            }
          }
          e = (e + 1) & (uint32_t)(H - 1);
        }
        if (!found) {
          lovf = 1;
          break;
        }
        if (!(q.dbg_mode & 1)) lds_apply(q, lw, H, (int)e, t, vmask, srec, gi, w3);
        if (lflag) __hip_atomic_fetch_or(&lflag[e >> 2], 1u << ((e & 3) * 8), WG_RLX);
      }
    }
  }
  __syncthreads();
  AGG_T(3);
  if (lovf) {
    if (threadIdx.x == 0) fail[p] |= 1;
    return;
  }
  // 3. compacted rows → the other buffer (contiguous entry range per thread keeps order)
  const int per = (H + AG_THREADS - 1) / AG_THREADS;
  const int e0 = threadIdx.x * per, e1 = e0 + per < H ? e0 + per : H;
  int mine = 0;
  if (idm) {
    for (int e = e0; e < e1; e++) mine += (uint64_t)lw[e] != EMPTY_ID;
  } else {
    for (int e = e0; e < e1; e++) mine += lref[e] != 0u;
  }
  // block exclusive scan of `mine`
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int incl = mine;
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) lcnt[wave] = incl;
  __syncthreads();
  int before = 0, total = 0;
  for (int w = 0; w < AG_THREADS / 64; w++) {
    if (w < wave) before += lcnt[w];
    total += lcnt[w];
  }
  if (threadIdx.x == 0) lbase = total ? atomicAdd(&newcnt[p], (unsigned long long)total) : 0ULL;
  __syncthreads();
  if ((int64_t)(lbase + total) > q.cmax) {
    if (threadIdx.x == 0) {
      fail[p] |= 2;
      atomicMax(need, (unsigned long long)(lbase + total));  // rows this partition needs (lower bound)
    }
    return;
  }
  const uint64_t row0 = lbase + (uint64_t)(before + incl - mine);  // this thread's first row
  uint64_t* dst = (sel[p] ? buf0 : buf1) + (uint64_t)p * q.cmax * q.sw + row0 * q.sw;
  uint8_t* cdst = lflag ? q.chg + (uint64_t)p * q.cmax + row0 : nullptr;
  const int hv = q.having.a.w_val, hc = q.having.a.w_cnt;
  for (int e = e0; e < e1; e++) {
    if (idm ? (uint64_t)lw[e] == EMPTY_ID : lref[e] == 0u) continue;
    if (cdst) {  // emission flags of the row (CHG_*): HAVING on the entry's new words
      const uint32_t f = (lflag[e >> 2] >> ((e & 3) * 8)) & 0xFFu;
      uint8_t c = 0;
      if (f & 1u) {
        const bool now = !q.having.active ||
                         having_ok_words((uint64_t)lw[hv * H + e], hc < 0 ? 0ULL : (uint64_t)lw[hc * H + e], q.having);
        c = (uint8_t)(CHG_TOUCHED | ((f & 2u) || !q.having.active ? CHG_OLD : 0) | (now ? CHG_NEW : 0));
      }
      *cdst++ = c;
    }
    if (idm) {
      const uint64_t id = (uint64_t)lw[e];
      if (id == EMPTY_ID) continue;
      const uint64_t hk = ((uint64_t)p << (64 - q.log2P)) | (id >> q.log2P);
      dst[0] = (uint64_t)key_of_hash(hk);
      dst[1] = (uint64_t)(((int64_t)(id & ((1ULL << q.log2P) - 1)) + wbase) * (q.windowed ? q.adv : 0));
      for (int w = 2; w < q.sw; w++) dst[w] = w < q.nwords ? (uint64_t)lw[w * H + e] : 0ULL;
    } else {
      if (lref[e] == 0u) continue;
      for (int w = 0; w < q.sw; w++) dst[w] = w < q.nwords ? (uint64_t)lw[w * H + e] : 0ULL;
    }
    dst += q.sw;
  }
  AGG_T(4);
  if (dbg) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    AGG_T(5);
  }
#undef AGG_T
}

// ------------------------------------------------------------------ k_part_merge
// The default aggregate kernel when the push's windows fit the packed identity (wr[1]) and
// its event-time span fits 31 bits.  One work item = one partition (or one of its sub-passes).
// Unlike k_part_agg, LDS holds only the groups THIS PUSH touches, as deltas in compact planes:
//   id u64[H] | rowtime u32[H] (ts - tbase + 1, 0 = none; bit 31 = matched by a resident row)
//   | one plane per update op: u64 (SUM, MIN, MAX) then u32 (COUNT, non-null count)
// and the partition's resident rows are merged on the way out (old row ⊕ delta → new buffer),
// so the LDS footprint does not grow with the resident state (C2 COUNT(*): 16 B per group →
// 4096 groups in 64 KB, two workgroups per CU).  Phases:
//   0. pass 0 only: resident rows of windows closed before this push → closed store
//   1. records (prefetched before the LDS init): window fan-out, find-or-claim the packed
//      identity with one 64-bit LDS CAS, LDS atomics on the delta planes
//   2. resident rows: probe their identity, mark the matched delta entries
//   3. count (resident live rows + unmatched deltas) per wave, block scan, reserve the
//      partition's region range with one atomic, check capacity
//   4. write merged resident rows, then new rows, wave-compacted (ballot ranks) so each store
//      instruction covers consecutive rows; count the rows passing the query's HAVING
// A partition whose deltas overflow H writes nothing and is retried with 2x sub-passes (it
// has already moved its closed rows in pass 0; retries skip them).
// k_part_merge workgroup size: 512 threads, two persistent workgroups per CU (one's global
// round trips hidden by the other's LDS work; measured on C2: 256 x 4 needs 2^15 partitions
// to fit its tables and loses more in the hist/refine than it gains)
#ifndef KHIP_MG_AU_CNT1
#define KHIP_MG_AU_CNT1 4  // k_part_merge COUNT(*) records per thread per chunk
#endif
#ifndef KHIP_MG_AU_GEN
#define KHIP_MG_AU_GEN 2   // k_part_merge (other update sets) records per thread per chunk
#endif
#ifndef KHIP_MG_AU_GEN_WIDE
#define KHIP_MG_AU_GEN_WIDE 2  // the same with 16-byte (+ argument word) records
#endif

struct MergeParams {
  int32_t windowed;
  int32_t sw;      // row words in the regions
  int32_t nwords;  // words used (3 + state words)
  int32_t H;       // LDS delta entries (multiple of 64)
  int32_t rw;      // scattered record words
  int32_t meta_word;
  int32_t log2P;
  int32_t n_ops;
  int64_t size, adv;
  FastDiv fd;
  int64_t cmax;
  int8_t col_word[MAX_COLS];
  int32_t col_type[MAX_COLS];
  UpdOp ops[MAX_OPS];
  int32_t plane_off[MAX_OPS];  // byte offset of op o's delta plane
  int8_t plane_w64[MAX_OPS];   // 1: u64 plane, 0: u32 plane
  int32_t rt_off;              // byte offset of the rowtime plane
  int32_t lds_bytes;
  InitWords init;
  HavingDev having;  // the query's HAVING (active = 0: none): rows passing it are counted
  int32_t dbg;       // tuning build: KHIP_MERGE_DEBUG prints the delta table of touched partitions
  int32_t r12;       // records are R12 (narrow layout; k_part_scatter / k_part_refine wrote them so)
  uint8_t* chg;      // changelog: per-row-slot emission flags (CHG_*), or null
  int32_t div32;     // windowed with adv <= 2^31: R12 window indices in 32-bit arithmetic (fd32)
  FastDiv32 fd32;
  int32_t list_off;  // byte offset of the LDS list of the entries the item's records claimed (u16 x H)
  int32_t fan;       // most windows a record can fall in (ceil(size / advance); 1 without windows)
  int32_t pane;      // HOPPING with size % advance == 0 and fan <= MG_FB: pane aggregation allowed
};


__device__ __forceinline__ uint32_t mg_slot(uint64_t id, int H) {
  const uint32_t h = ((uint32_t)id * 0x9E3779B1u) ^ (uint32_t)(id >> 32) * 0x85EBCA77u;
  return (uint32_t)(((uint64_t)h * (uint32_t)H) >> 32);
}


template <class T>
__device__ __forceinline__ KLDS T* mg_plane(char* smem, int32_t off) {
  return (KLDS T*)((KLDS char*)smem + off);
}

// Per row word, copied to LDS at kernel start (row words are indexed at run time; the kernel
// argument struct is only read at compile-time offsets): the word's update op kind (-1: none),
// its delta plane's byte offset and width, and the initial value of a new group.
struct MgOp {  // one update op, as the record phase needs it
  int32_t kind;
  int32_t col;
  int32_t off;  // delta plane byte offset
  int32_t cw;   // record word of the op's column
  int32_t dbl;  // DOUBLE column (MIN/MAX on the total-order key)
};

constexpr int MG_FB = 6;  // k_part_merge: fan-outs up to this issue a record's window CASes together

struct MgWord {
  int32_t kind;
  int32_t off;
  int32_t w64;
  int32_t pad;
  int64_t init;
};

// Word w (>= 3) of the merged row: resident row `old` (nullptr: a new group) ⊕ delta entry e.
__device__ __forceinline__ uint64_t mg_word(const MgWord* tab, char* smem, int w, const uint64_t* old, int e) {
  const MgWord t = tab[w];
  if (t.kind < 0) return old ? old[w] : (uint64_t)t.init;
  uint64_t d;
  if (t.w64) d = (uint64_t)mg_plane<int64_t>(smem, t.off)[e];
  else d = (uint64_t)mg_plane<uint32_t>(smem, t.off)[e];
  if (!old) return d;
  const uint64_t o = old[w];
  switch (t.kind) {
    case OP_INC:
    case OP_INC_VALID:
    case OP_ADD_I64: return o + d;
    case OP_ADD_F64: {
      double a, b;
      __builtin_memcpy(&a, &o, 8);
      __builtin_memcpy(&b, &d, 8);
      a += b;
      uint64_t r;
      __builtin_memcpy(&r, &a, 8);
      return r;
    }
    case OP_MIN: return (int64_t)d < (int64_t)o ? d : o;
    case OP_MAX: return (int64_t)d > (int64_t)o ? d : o;
  }
  return o;
}

// Resident row → its delta entry: -2 = not in this work item (closed, or another sub-pass),
// -1 = live but untouched by this push, else the entry index.
__device__ __forceinline__ int mg_find(const MergeParams& q, const KLDS uint64_t* ids, const uint64_t* row, bool evict,
                                       int64_t close0, int sbits, int sub, int64_t wbase, int H) {
  const int64_t key = (int64_t)row[0], ws = (int64_t)row[1];
  if (evict && ws + q.size <= close0) return -2;
  const uint64_t hk = key_hash(key);
  if (!sub_ok(hk, ws, sbits, sub)) return -2;
  const int64_t widx = q.windowed ? (int64_t)fast_udiv((uint64_t)ws, q.fd) : 0;
  const uint64_t id = ident_of(hk, widx - wbase, q.log2P);
  uint32_t e = mg_slot(id, H);
  for (int probe = 0; probe < H; probe++) {
    const uint64_t v = ids[e];
    if (v == id) return (int)e;
    if (v == EMPTY_ID) return -1;
    e = e + 1 == (uint32_t)H ? 0u : e + 1;
  }
  return -1;
}

// One chunk of a partition's scattered records, AU per thread (rows l0 + tid + u * NT), kept as
// the raw words the load returns: converting them right after the load would make the wave wait for
// it there — and, since vmcnt retires loads and stores in issue order, for every row store issued
// before it.  Every lane loads (the index is clamped to the item's last record, so lanes past the
// end re-read one line); mg_decode marks them invalid.
struct MgRaw {
  uint32_t w[4];  // R12: key hash lo, hi, trel; 16-byte record: key hash lo, hi, ts lo, hi
};

// Record of chunk l0 taken by this thread's unit u.  STRIDE: a wave's 64 lanes take records
// AU * NT / 64 apart (the whole chunk) instead of 64 consecutive ones: a partition's records are in
// arrival order, and with few keys per partition consecutive records update the same (key, window)
// entries — same-address LDS atomics that serialize (C3: 6 keys per partition, ~14 bank-conflict
// cycles per LDS instruction with consecutive records).  Only items of at least one full chunk
// stride (stride = rn >= AU * NT, uniform): in a smaller item every record is in one wave and the
// lanes' same-address atomics apply in arrival order, as the reference's sequential DOUBLE sums do
// (the QTT comparator's 1e-6 absolute tolerance on large sums needs that order).
template <int AU, int NT, bool STRIDE>
__device__ __forceinline__ int64_t mg_li(int64_t l0, int u, bool stride) {
  if (STRIDE && stride) return l0 + (int64_t)(threadIdx.x & 63) * (AU * NT / 64) + (int64_t)(threadIdx.x >> 6) * AU + u;
  return l0 + threadIdx.x + (int64_t)u * NT;
}

template <int AU, int NT, bool R12M, bool STRIDE>
__device__ __forceinline__ void mg_load(MgRaw (&raw)[AU], longlong2 (&ext)[AU], const uint64_t* __restrict__ srec,
                                        int64_t rbase, int64_t rn, int64_t l0, int rw, bool wide) {
#pragma unroll
  for (int u = 0; u < AU; u++) {
    const int64_t li = mg_li<AU, NT, STRIDE>(l0, u, rn >= AU * NT);
    const uint64_t idx = (uint64_t)(rbase + (li < rn ? li : (rn > 0 ? rn - 1 : 0)));
    if constexpr (R12M) {  // a compile-time choice: a run-time one merges both paths' registers,
                           // which consumes the loaded words at the load
      const R12 v = *(const R12*)((const char*)srec + idx * 12);
      raw[u].w[0] = v.lo;
      raw[u].w[1] = v.hi;
      raw[u].w[2] = v.trel;
      raw[u].w[3] = 0u;
    } else {
      const uint4 v = *(const uint4*)(srec + idx * rw);
      raw[u].w[0] = v.x;
      raw[u].w[1] = v.y;
      raw[u].w[2] = v.z;
      raw[u].w[3] = v.w;
      if (wide) ext[u] = ((const longlong2*)(srec + idx * rw))[1];
    }
  }
}

// (key hash, ts) of a raw record; ts = -1 for no window (R12 trel 0) or a lane past the item's end.
template <bool R12M>
__device__ __forceinline__ longlong2 mg_decode(const MgRaw& r, int64_t tbase, bool valid) {
  const int64_t hk = (int64_t)((uint64_t)r.w[1] << 32 | r.w[0]);
  const int64_t t = R12M ? (r.w[2] ? tbase + (int64_t)r.w[2] - 1 : -1) : (int64_t)((uint64_t)r.w[3] << 32 | r.w[2]);
  return make_longlong2(hk, valid ? t : -1);
}

struct MgItem {
  uint32_t p;
  int sbits, sub;
  int64_t rbase, rn;
  int64_t nrow;  // the partition's resident rows
  bool sel;      // which ping-pong buffer holds them
};

// The work item's descriptor, read one item ahead with wave-uniform (scalar) loads: a vector
// load here would, at its first use, wait for every store the previous item's write-out issued.
__device__ __forceinline__ MgItem mg_item(const uint32_t* __restrict__ work, int64_t w,
                                          const int64_t* __restrict__ pbase, const uint8_t* __restrict__ sel,
                                          const int64_t* __restrict__ cnt) {
  MgItem it;
  if (work) {
    const uint32_t x = work[w];
    it.p = x & 0xFFFFu;
    it.sbits = (x >> 16) & 0xF;
    it.sub = (int)(x >> 20);
  } else {
    it.p = (uint32_t)w;
    it.sbits = 0;
    it.sub = 0;
  }
  it.p = __builtin_amdgcn_readfirstlane(it.p);
  it.rbase = pbase[it.p];
  it.rn = pbase[it.p + 1] - it.rbase;
  it.nrow = cnt[it.p];
  it.sel = ((((const uint32_t*)sel)[it.p >> 2] >> (8 * (it.p & 3))) & 0xFFu) != 0;  // sel: P >= 64 bytes
  return it;
}

// Reset delta entry e to its initial state (empty identity, no rowtime, op identities).
__device__ __forceinline__ void mg_clear(char* smem, KLDS uint64_t* ids, KLDS uint32_t* rt, const MgOp* otab,
                                         int n_ops, int e) {
  ids[e] = EMPTY_ID;
  rt[e] = 0u;
  for (int o = 0; o < n_ops; o++) {
    const MgOp op = otab[o];
    if (op.kind == OP_INC || op.kind == OP_INC_VALID) mg_plane<uint32_t>(smem, op.off)[e] = 0u;
    else mg_plane<int64_t>(smem, op.off)[e] = op.kind == OP_MIN ? INT64_MAX : (op.kind == OP_MAX ? INT64_MIN : 0);
  }
}

// CNT1: the query's only update is COUNT(*) (one u32 delta plane at word 3) and its records are
// (key hash, ts) pairs with one window each — the record phase and the write-out skip the
// generic op machinery (C1, C2).
//
// Persistent: gridDim.x workgroups (two per CU) walk the work items w = blockIdx.x + k * gridDim.x.
// Barriers inside the item loop wait for LDS only (lds_barrier): the write-out's row stores and
// the next item's record prefetch stay in flight across them.
// The next item's first record chunk is loaded into registers before the current item's
// resident-merge and write-out, and inside an item chunk c + 1 is loaded before chunk c is
// applied, so HBM latency overlaps the LDS work; the write-out leaves every delta entry cleared
// for the next item (no separate table init).
#ifndef KHIP_MG_WPE
#define KHIP_MG_WPE 4  // k_part_merge: minimum waves per SIMD (4: <= 128 VGPRs, two 512-thread workgroups per CU)
#endif
template <bool CNT1, int NT, bool R12M>
__global__ __launch_bounds__(NT, KHIP_MG_WPE) void k_part_merge(
    MergeParams q, const uint32_t* __restrict__ work, int64_t nwork, const int64_t* __restrict__ pbase,
    const uint64_t* __restrict__ srec, int first, uint64_t* __restrict__ buf0, uint64_t* __restrict__ buf1,
    const uint8_t* __restrict__ sel, const int64_t* __restrict__ cnt, unsigned long long* __restrict__ newcnt,
    uint8_t* __restrict__ fail, unsigned long long* __restrict__ need, int64_t close0, uint64_t* __restrict__ closed,
    unsigned long long* __restrict__ closed_n, const int64_t* __restrict__ wr,
    unsigned long long* __restrict__ hnew, unsigned long long* __restrict__ hclosed,
    unsigned long long* __restrict__ dbg) {
#define MG_T(k) do { if (dbg && threadIdx.x == 0) atomicAdd(&dbg[(k)], (unsigned long long)(wall_clock64() - t_last)); t_last = wall_clock64(); } while (0)
  if (wr[4] == 0) return;  // k_part_wrange declined the merge path for this push
  unsigned long long t_last = wall_clock64();
  const int64_t tbase = wr[5];
  // R12 records: window index relative to wbase = qw0 + (r0 + trel - 1) / adv in 32-bit arithmetic
  // (trel < 2^31, r0 < adv <= 2^31), with tbase = q0 * adv + r0 and qw0 = q0 - wbase
  const int64_t q0 = q.windowed ? (int64_t)fast_udiv((uint64_t)tbase, q.fd) : 0;
  const uint32_t r0 = (uint32_t)(tbase - q0 * q.adv);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int lovf;
  __shared__ int nnew;  // entries claimed by the item's records (listed in nl)
  __shared__ int wsum[NT / 64];
  __shared__ unsigned long long lbase;
  __shared__ MgWord wtab[32];
  __shared__ MgOp otab[MAX_OPS];
  constexpr int AU = CNT1 ? KHIP_MG_AU_CNT1 : (R12M ? KHIP_MG_AU_GEN : KHIP_MG_AU_GEN_WIDE);  // records per thread per chunk (two chunks in registers)
  constexpr int NW = NT / 64;
  const int H = q.H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t dummy = (uint32_t)H + (uint32_t)lane;
  const bool wide = !CNT1 && q.rw > 2;
  // R12M: narrow records arrive in the 12-byte form (q.r12)
  const int64_t wbase = wr[0];
  const int64_t qw0 = q0 - wbase;
  const bool evict = q.windowed && close0 != INT64_MIN;
  KLDS uint64_t* ids = mg_plane<uint64_t>(smem, 0);
  KLDS uint32_t* rt = mg_plane<uint32_t>(smem, q.rt_off);
  KLDS uint32_t* cnt1 = mg_plane<uint32_t>(smem, q.plane_off[0]);  // CNT1: the COUNT(*) deltas
  KLDS uint16_t* nl = mg_plane<uint16_t>(smem, q.list_off);
  if (threadIdx.x < q.n_ops) {
    const int o = threadIdx.x;
    MgOp t;
    t.kind = q.ops[o].kind;
    t.col = q.ops[o].col;
    t.off = q.plane_off[o];
    t.cw = q.col_word[q.ops[o].col];
    t.dbl = q.col_type[q.ops[o].col] == KHIP_TYPE_DOUBLE;
    otab[o] = t;
  }
  if (threadIdx.x < 32) {
    const int w = threadIdx.x;
    int o = -1;
    for (int k = 0; k < q.n_ops; k++)
      if (q.ops[k].word == w) o = k;
    MgWord t;
    t.kind = o < 0 ? -1 : q.ops[o].kind;
    t.off = o < 0 ? 0 : q.plane_off[o];
    t.w64 = o < 0 ? 0 : q.plane_w64[o];
    t.pad = 0;
    t.init = q.init.w[w];
    wtab[w] = t;
  }
  int64_t w = blockIdx.x;
  MgItem it{};
  // two register sets: the records of chunk c + 1 are in flight while chunk c is applied
  MgRaw rawA[AU], rawB[AU];
  longlong2 extA[AU], extB[AU];
  if (w < nwork) {
    it = mg_item(work, w, pbase, sel, cnt);
    mg_load<AU, NT, R12M, !CNT1>(rawA, extA, srec, it.rbase, it.rn, 0, q.rw, wide);
  }
  if (threadIdx.x == 0) {
    lovf = 0;
    nnew = 0;
  }
  lds_barrier();  // otab / wtab / lovf / nnew
  // One argument column (every op on it, plus COUNT(*)): the ops' plane offsets in wave-uniform
  // registers, so a (record, window) update is straight-line code with no op-table reads (C3:
  // COUNT / SUM / MIN / MAX of one DOUBLE).  -1 = op absent.  Other shapes walk otab.
  int oc_star = -1, oc_cnt = -1, oc_sum = -1, oc_min = -1, oc_max = -1, oc_col = -1, oc_cw = 3, oc_f64 = 0;
  bool onecol = true;
  for (int o = 0; o < q.n_ops; o++) {
    const MgOp t = otab[o];
    if (t.kind == OP_INC) {
      oc_star = t.off;
      continue;
    }
    if (oc_col >= 0 && t.col != oc_col) onecol = false;
    oc_col = t.col;
    oc_cw = t.cw;
    oc_f64 = t.dbl;
    if (t.kind == OP_INC_VALID) oc_cnt = t.off;
    else if (t.kind == OP_ADD_I64 || t.kind == OP_ADD_F64) oc_sum = t.off, oc_f64 = t.kind == OP_ADD_F64;
    else if (t.kind == OP_MIN) oc_min = t.off;
    else if (t.kind == OP_MAX) oc_max = t.off;
  }
  const bool dbl_col = oc_col >= 0 && q.col_type[oc_col < 0 ? 0 : oc_col] == KHIP_TYPE_DOUBLE;
  // Panes (HOPPING, size a multiple of the advance): a record whose windows are all open updates
  // ONE entry — its pane, the advance-long slice it falls in, identity (key, slice index + PB) —
  // instead of its F windows; after the records, each pane is folded into its F windows (F updates
  // per pane instead of per record).  Items of at least one full chunk stride without sub-passes.
  const bool panes_ok = !CNT1 && q.pane && wr[8] != 0;
  const int64_t PB = panes_ok ? ((int64_t)1 << (q.log2P - 1)) : 0;
  for (int i = threadIdx.x; i < H + 64; i += NT) mg_clear(smem, ids, rt, otab, q.n_ops, i);
  lds_barrier();
  MG_T(0);
  for (; w < nwork; w += gridDim.x) {
    const uint32_t p = it.p;
    const int sbits = it.sbits, sub = it.sub;
    const int64_t rbase = it.rbase, rn = it.rn;
    const bool pmode = panes_ok && sbits == 0 && rn >= (int64_t)AU * NT;
    const int64_t wnext = w + gridDim.x;
    MgItem nit{};
    if (wnext < nwork) nit = mg_item(work, wnext, pbase, sel, cnt);  // its loads are issued now, used later
    if (rn == 0 && first) {  // untouched partition: nothing to rewrite
      if (wnext < nwork) mg_load<AU, NT, R12M, !CNT1>(rawA, extA, srec, nit.rbase, nit.rn, 0, q.rw, wide);
      it = nit;
      continue;
    }
    const uint64_t* src = (it.sel ? buf1 : buf0) + (uint64_t)p * q.cmax * q.sw;
    const int64_t nrow = it.nrow;
    // 0. closed resident rows → closed store (pass 0 only; retries skip them)
    if (evict && first) {
      int ne = 0, nh = 0;
      for (int64_t r = threadIdx.x; r < nrow; r += NT) {
        const uint64_t* row = src + r * q.sw;
        ne += ((int64_t)row[1] + q.size <= close0) && sub_ok(key_hash((int64_t)row[0]), (int64_t)row[1], sbits, sub);
      }
      int incl = ne;
      for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
      }
      if (lane == 63) wsum[wave] = incl;
      lds_barrier();
      int before = 0, total = 0;
      for (int k = 0; k < NW; k++) {
        if (k < wave) before += wsum[k];
        total += wsum[k];
      }
      if (threadIdx.x == 0) lbase = total ? atomicAdd(closed_n, (unsigned long long)total) : 0ULL;
      lds_barrier();
      uint64_t* dst = closed + (lbase + (uint64_t)(before + incl - ne)) * q.sw;
      for (int64_t r = threadIdx.x; r < nrow; r += NT) {
        const uint64_t* row = src + r * q.sw;
        if (!((int64_t)row[1] + q.size <= close0) ||
            !sub_ok(key_hash((int64_t)row[0]), (int64_t)row[1], sbits, sub))
          continue;
        for (int k = 0; k < q.sw; k++) dst[k] = row[k];
        dst += q.sw;
        nh += having_ok(row, q.having) ? 1 : 0;
      }
      if (q.having.active) {
        nh = (int)wave_sum(nh);
        if (lane == 0 && nh) atomicAdd(hclosed, (unsigned long long)nh);
      }
      lds_barrier();
    }
    MG_T(1);
    // 1. this item's records, two chunks per round: chunk c + 1 (set B) is loaded before chunk c
    //    (set A, loaded before the previous item's write-out or in the last round) is applied, and
    //    chunk c + 2 before chunk c + 1.  Loads are unconditional, so every wait is counted exactly.
    auto apply_chunk = [&](const MgRaw (&raw)[AU], const longlong2 (&ext)[AU], int64_t l0) {
      longlong2 rec[AU];
#pragma unroll
      for (int u = 0; u < AU; u++) rec[u] = mg_decode<R12M>(raw[u], tbase, mg_li<AU, NT, !CNT1>(l0, u, rn >= AU * NT) < rn);
      if constexpr (CNT1) {
        // one window per record: w = ts / adv (TUMBLING) or 0 (no window); ts < 0: skip.  The AU
        // identities' CASes are issued back to back; collisions probe on afterwards.
        uint64_t id[AU], old[AU];
        uint32_t e[AU];
        bool pend[AU];
#pragma unroll
        for (int u = 0; u < AU; u++) {
          const int64_t t = rec[u].y;
          const uint64_t hk = (uint64_t)rec[u].x;
          int64_t wrel;  // window index - wbase
          if (R12M && q.div32) {
            const uint32_t trel = raw[u].w[2];
            wrel = qw0 + (int64_t)fast_udiv32(r0 + trel - 1u, q.fd32);
          } else {
            wrel = (q.windowed ? (int64_t)fast_udiv((uint64_t)(t < 0 ? 0 : t), q.fd) : 0) - wbase;
          }
          const bool act = t >= 0 && (sbits == 0 || sub_ok(hk, (wrel + wbase) * q.adv, sbits, sub));
          id[u] = act ? ident_of(hk, wrel, q.log2P) : EMPTY_ID;
          e[u] = act ? mg_slot(id[u], H) : dummy;
        }
#pragma unroll
        for (int u = 0; u < AU; u++) {
          old[u] = EMPTY_ID;
          __hip_atomic_compare_exchange_strong(&ids[e[u]], &old[u], id[u], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
        }
#pragma unroll
        for (int u = 0; u < AU; u++) {
          pend[u] = old[u] != EMPTY_ID && old[u] != id[u];
          mg_list_append(id[u] != EMPTY_ID && old[u] == EMPTY_ID, e[u], nl, &nnew);
        }
        for (int probes = 1;; probes++) {
          bool anyp = false;
#pragma unroll
          for (int u = 0; u < AU; u++) anyp |= pend[u];
          if (!__ballot(anyp)) break;
          if (probes >= H) {
            lovf = 1;
            break;
          }
          bool got[AU];
#pragma unroll
          for (int u = 0; u < AU; u++) {
            got[u] = false;
            if (!pend[u]) continue;
            e[u] = e[u] + 1 == (uint32_t)H ? 0u : e[u] + 1;
            uint64_t o2 = EMPTY_ID;
            __hip_atomic_compare_exchange_strong(&ids[e[u]], &o2, id[u], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
            pend[u] = o2 != EMPTY_ID && o2 != id[u];
            got[u] = o2 == EMPTY_ID;
          }
#pragma unroll
          for (int u = 0; u < AU; u++) mg_list_append(got[u], e[u], nl, &nnew);
        }
#pragma unroll
        for (int u = 0; u < AU; u++) {
          if (id[u] == EMPTY_ID || pend[u]) continue;
          __hip_atomic_fetch_max(&rt[e[u]], R12M ? raw[u].w[2] : (uint32_t)(rec[u].y - tbase + 1), WG_RLX);
          __hip_atomic_fetch_add(&cnt1[e[u]], 1u, WG_RLX);
        }
      } else {
        int64_t w0[AU], wn[AU];  // first applied window index, last window index
        uint32_t trel[AU];
#pragma unroll
        for (int u = 0; u < AU; u++) {
          const int64_t t = rec[u].y;
          const uint32_t meta = q.meta_word == 2 ? (uint32_t)ext[u].x : 0u;
          trel[u] = (uint32_t)(t - tbase + 1);
          if (t < 0) {  // every window late (or past the end)
            w0[u] = 1;
            wn[u] = 0;
          } else if (q.windowed) {
            wn[u] = (int64_t)fast_udiv((uint64_t)t, q.fd);
            if (q.size == q.adv) {
              w0[u] = wn[u] + (int64_t)(meta & 0xFFFFu);  // TUMBLING: one window
            } else {
              const int64_t lo = t - q.size + q.adv;
              w0[u] = (int64_t)fast_udiv((uint64_t)(lo > 0 ? lo : 0), q.fd) + (int64_t)(meta & 0xFFFFu);
            }
          } else {
            w0[u] = 0;
            wn[u] = 0;
          }
        }
        // one (record u, window) update into delta entry ent: row time, then the update ops
        auto upd = [&](int u, uint32_t ent) {
          __hip_atomic_fetch_max(&rt[ent], trel[u], WG_RLX);
          const uint32_t vmask = q.meta_word == 2 ? ((uint32_t)ext[u].x >> 16) : 0u;
          const int64_t gi = rbase + mg_li<AU, NT, !CNT1>(l0, u, rn >= AU * NT);
          auto apply_op = [&](const MgOp op) {
            if (op.kind == OP_INC) {
              __hip_atomic_fetch_add(&mg_plane<uint32_t>(smem, op.off)[ent], 1u, WG_RLX);
              return;
            }
            if (!((vmask >> op.col) & 1u)) return;
            if (op.kind == OP_INC_VALID) {
              __hip_atomic_fetch_add(&mg_plane<uint32_t>(smem, op.off)[ent], 1u, WG_RLX);
              return;
            }
            const int64_t raw = op.cw == 3 ? ext[u].y : (int64_t)srec[(uint64_t)gi * q.rw + op.cw];
            KLDS int64_t* pl = mg_plane<int64_t>(smem, op.off);
            switch (op.kind) {
              case OP_ADD_I64: __hip_atomic_fetch_add((KLDS uint64_t*)&pl[ent], (uint64_t)raw, WG_RLX); break;
              case OP_ADD_F64: {
                double d;
                __builtin_memcpy(&d, &raw, 8);
                __hip_atomic_fetch_add((KLDS double*)&pl[ent], d, WG_RLX);
                break;
              }
              case OP_MIN:
              case OP_MAX: {
                int64_t k = raw;
                if (op.dbl) {
                  double d;
                  __builtin_memcpy(&d, &raw, 8);
                  k = f64_order_key(d);
                }
                if (op.kind == OP_MIN) __hip_atomic_fetch_min(&pl[ent], k, WG_RLX);
                else __hip_atomic_fetch_max(&pl[ent], k, WG_RLX);
                break;
              }
              default: break;
            }
          };
          if (onecol) {
            if (oc_star >= 0) __hip_atomic_fetch_add(&mg_plane<uint32_t>(smem, oc_star)[ent], 1u, WG_RLX);
            if (oc_col >= 0 && ((vmask >> oc_col) & 1u)) {
              if (oc_cnt >= 0) __hip_atomic_fetch_add(&mg_plane<uint32_t>(smem, oc_cnt)[ent], 1u, WG_RLX);
              const int64_t raw = oc_cw == 3 ? ext[u].y : (int64_t)srec[(uint64_t)gi * q.rw + oc_cw];
              double d;
              __builtin_memcpy(&d, &raw, 8);
              if (oc_sum >= 0) {
                if (oc_f64) __hip_atomic_fetch_add(&mg_plane<double>(smem, oc_sum)[ent], d, WG_RLX);
                else __hip_atomic_fetch_add(&mg_plane<uint64_t>(smem, oc_sum)[ent], (uint64_t)raw, WG_RLX);
              }
              const int64_t k = dbl_col ? f64_order_key(d) : raw;
              if (oc_min >= 0) __hip_atomic_fetch_min(&mg_plane<int64_t>(smem, oc_min)[ent], k, WG_RLX);
              if (oc_max >= 0) __hip_atomic_fetch_max(&mg_plane<int64_t>(smem, oc_max)[ent], k, WG_RLX);
            }
          } else {
            for (int o = 0; o < q.n_ops; o++) apply_op(otab[o]);
          }
        };
        if (q.fan <= MG_FB) {
          // every window of a record at once: its identity CASes are in flight together, so a
          // thread waits for LDS results once per record instead of once per window (LDS results
          // return in order: a CAS's wait also covers every atomic issued before it)
#pragma unroll
          for (int u = 0; u < AU; u++) {
            uint64_t id[MG_FB], old[MG_FB];
            uint32_t e[MG_FB];
            bool act[MG_FB], pend[MG_FB];
            const uint64_t hk = (uint64_t)rec[u].x;
            // every window open (no late offset): the record's pane instead of its windows
            const bool pr = pmode && (q.meta_word != 2 || ((uint32_t)ext[u].x & 0xFFFFu) == 0u);
#pragma unroll
            for (int j = 0; j < MG_FB; j++) {
              const int64_t widx = w0[u] + j;
              if (pr) {
                act[j] = j == 0 && w0[u] <= wn[u];
                id[j] = act[j] ? ident_of(hk, wn[u] - wbase + PB, q.log2P) : EMPTY_ID;
              } else {
                act[j] = j < q.fan && widx <= wn[u] && (sbits == 0 || sub_ok(hk, widx * q.adv, sbits, sub));
                id[j] = act[j] ? ident_of(hk, widx - wbase, q.log2P) : EMPTY_ID;
              }
              e[j] = act[j] ? mg_slot(id[j], H) : dummy;
            }
#pragma unroll
            for (int j = 0; j < MG_FB; j++) {
              if (j >= q.fan) break;
              old[j] = EMPTY_ID;
              __hip_atomic_compare_exchange_strong(&ids[e[j]], &old[j], id[j], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
            }
#pragma unroll
            for (int j = 0; j < MG_FB; j++) {
              if (j >= q.fan) break;
              pend[j] = act[j] && old[j] != EMPTY_ID && old[j] != id[j];
              mg_list_append(act[j] && old[j] == EMPTY_ID, e[j], nl, &nnew);
            }
            for (int probes = 1;; probes++) {  // collisions: every pending window probes on together
              bool anyp = false;
#pragma unroll
              for (int j = 0; j < MG_FB; j++) anyp |= j < q.fan && pend[j];
              if (!__ballot(anyp)) break;
              if (probes >= H) {
                lovf = 1;
#pragma unroll
                for (int j = 0; j < MG_FB; j++) act[j] = false;
                break;
              }
              bool got[MG_FB];
#pragma unroll
              for (int j = 0; j < MG_FB; j++) {
                got[j] = false;
                if (j >= q.fan || !pend[j]) continue;
                e[j] = e[j] + 1 == (uint32_t)H ? 0u : e[j] + 1;
                uint64_t o2 = EMPTY_ID;
                __hip_atomic_compare_exchange_strong(&ids[e[j]], &o2, id[j], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP);
                pend[j] = o2 != EMPTY_ID && o2 != id[j];
                got[j] = o2 == EMPTY_ID;
              }
#pragma unroll
              for (int j = 0; j < MG_FB; j++) {
                if (j >= q.fan) break;
                mg_list_append(got[j], e[j], nl, &nnew);
              }
            }
#pragma unroll
            for (int j = 0; j < MG_FB; j++) {
              if (j >= q.fan) break;
              if (act[j]) upd(u, e[j]);
            }
          }
        } else {
          for (int64_t j = 0;; j++) {
            bool any = false;
            bool act[AU];
            uint64_t id[AU];
            uint32_t e[AU];
  #pragma unroll
            for (int u = 0; u < AU; u++) {
              const int64_t widx = w0[u] + j;
              const uint64_t hk = (uint64_t)rec[u].x;  // the scatter stores the key hash
              const bool has = widx <= wn[u];
              any |= has;
              act[u] = has && (sbits == 0 || sub_ok(hk, widx * q.adv, sbits, sub));
              id[u] = act[u] ? ident_of(hk, widx - wbase, q.log2P) : EMPTY_ID;
              e[u] = act[u] ? mg_slot(id[u], H) : dummy;
            }
            if (!__ballot(any)) break;
            uint64_t old[AU];
  #pragma unroll
            for (int u = 0; u < AU; u++) {
              old[u] = EMPTY_ID;
              __hip_atomic_compare_exchange_strong(&ids[e[u]], &old[u], id[u], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            bool pend[AU];
  #pragma unroll
            for (int u = 0; u < AU; u++) {
              pend[u] = act[u] && old[u] != EMPTY_ID && old[u] != id[u];
              mg_list_append(act[u] && old[u] == EMPTY_ID, e[u], nl, &nnew);
            }
            for (int probes = 1;; probes++) {
              bool anyp = false;
  #pragma unroll
              for (int u = 0; u < AU; u++) anyp |= pend[u];
              if (!__ballot(anyp)) break;
              if (probes >= H) {
                lovf = 1;
  #pragma unroll
                for (int u = 0; u < AU; u++) act[u] = false;
                break;
              }
              bool got[AU];
  #pragma unroll
              for (int u = 0; u < AU; u++) {
                got[u] = false;
                if (!pend[u]) continue;
                e[u] = e[u] + 1 == (uint32_t)H ? 0u : e[u] + 1;
                uint64_t o2 = EMPTY_ID;
                __hip_atomic_compare_exchange_strong(&ids[e[u]], &o2, id[u], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP);
                pend[u] = o2 != EMPTY_ID && o2 != id[u];
                got[u] = o2 == EMPTY_ID;
              }
  #pragma unroll
              for (int u = 0; u < AU; u++) mg_list_append(got[u], e[u], nl, &nnew);
            }
  #pragma unroll
            for (int u = 0; u < AU; u++)
              if (act[u]) upd(u, e[u]);
            if (*(volatile KLDS int*)&lovf) break;
          }
        }
      }
    };
    const int64_t nch = (rn + (int64_t)AU * NT - 1) / ((int64_t)AU * NT);
    for (int64_t c = 0; c < nch; c += 2) {
      mg_load<AU, NT, R12M, !CNT1>(rawB, extB, srec, rbase, rn, (c + 1) * AU * NT, q.rw, wide);
      apply_chunk(rawA, extA, c * AU * NT);
      if (*(volatile KLDS int*)&lovf || c + 1 >= nch) break;
      mg_load<AU, NT, R12M, !CNT1>(rawA, extA, srec, rbase, rn, (c + 2) * AU * NT, q.rw, wide);
      apply_chunk(rawB, extB, (c + 1) * AU * NT);
      if (*(volatile KLDS int*)&lovf) break;
    }
    lds_barrier();
    MG_T(2);
    // the next item's first chunk is in flight from here on
    if (wnext < nwork) mg_load<AU, NT, R12M, !CNT1>(rawA, extA, srec, nit.rbase, nit.rn, 0, q.rw, wide);
    if constexpr (!CNT1) {
      if (pmode && !lovf) {
        // 1b. fold: each pane into its F windows, whose entries are found or claimed as a record's
        const int nn0 = nnew;
        lds_barrier();  // every thread has read nn0 before the fold lists its windows
        for (int i0 = 0; i0 < nn0; i0 += NT) {  // uniform trip count: the probe loop is convergent
          const int li = i0 + threadIdx.x;
          const int pe = li < nn0 ? (int)nl[li] : -1;
          const uint64_t pid = pe >= 0 ? ids[pe] : EMPTY_ID;
          const int64_t rel = (int64_t)(pid & ((1ULL << q.log2P) - 1));
          const bool isp = pid != EMPTY_ID && rel >= PB;
          const int64_t pw = rel - PB + wbase;  // the pane's slice index = the index of its last window
          const uint64_t hk = ((uint64_t)p << (64 - q.log2P)) | (pid >> q.log2P);
          uint64_t id[MG_FB], old[MG_FB];
          uint32_t e[MG_FB];
          bool act[MG_FB], pend[MG_FB];
#pragma unroll
          for (int j = 0; j < MG_FB; j++) {
            act[j] = isp && j < q.fan && pw - j >= 0;
            id[j] = act[j] ? ident_of(hk, pw - j - wbase, q.log2P) : EMPTY_ID;
            e[j] = act[j] ? mg_slot(id[j], H) : dummy;
          }
#pragma unroll
          for (int j = 0; j < MG_FB; j++) {
            old[j] = EMPTY_ID;
            __hip_atomic_compare_exchange_strong(&ids[e[j]], &old[j], id[j], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
          }
#pragma unroll
          for (int j = 0; j < MG_FB; j++) {
            pend[j] = act[j] && old[j] != EMPTY_ID && old[j] != id[j];
            mg_list_append(act[j] && old[j] == EMPTY_ID, e[j], nl, &nnew);
          }
          for (int probes = 1;; probes++) {
            bool anyp = false;
#pragma unroll
            for (int j = 0; j < MG_FB; j++) anyp |= pend[j];
            if (!__ballot(anyp)) break;
            if (probes >= H) {
              lovf = 1;
#pragma unroll
              for (int j = 0; j < MG_FB; j++) act[j] = false;
              break;
            }
            bool got[MG_FB];
#pragma unroll
            for (int j = 0; j < MG_FB; j++) {
              got[j] = false;
              if (!pend[j]) continue;
              e[j] = e[j] + 1 == (uint32_t)H ? 0u : e[j] + 1;
              uint64_t o2 = EMPTY_ID;
              __hip_atomic_compare_exchange_strong(&ids[e[j]], &o2, id[j], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
              pend[j] = o2 != EMPTY_ID && o2 != id[j];
              got[j] = o2 == EMPTY_ID;
            }
#pragma unroll
            for (int j = 0; j < MG_FB; j++) mg_list_append(got[j], e[j], nl, &nnew);
          }
          if (!isp) continue;
          const uint32_t prt = rt[pe];
#pragma unroll
          for (int j = 0; j < MG_FB; j++) {
            if (!act[j]) continue;
            const uint32_t we = e[j];
            __hip_atomic_fetch_max(&rt[we], prt, WG_RLX);
            for (int o = 0; o < q.n_ops; o++) {
              const MgOp op = otab[o];
              if (op.kind == OP_INC || op.kind == OP_INC_VALID) {
                __hip_atomic_fetch_add(&mg_plane<uint32_t>(smem, op.off)[we], mg_plane<uint32_t>(smem, op.off)[pe], WG_RLX);
                continue;
              }
              KLDS int64_t* pl = mg_plane<int64_t>(smem, op.off);
              const int64_t v = pl[pe];
              switch (op.kind) {
                case OP_ADD_I64: __hip_atomic_fetch_add((KLDS uint64_t*)&pl[we], (uint64_t)v, WG_RLX); break;
                case OP_ADD_F64: {
                  double d;
                  __builtin_memcpy(&d, &v, 8);
                  __hip_atomic_fetch_add((KLDS double*)&pl[we], d, WG_RLX);
                  break;
                }
                case OP_MIN: __hip_atomic_fetch_min(&pl[we], v, WG_RLX); break;
                case OP_MAX: __hip_atomic_fetch_max(&pl[we], v, WG_RLX); break;
                default: break;
              }
            }
          }
        }
        lds_barrier();
      }
    }
    if (lovf) {  // more groups than the table: retried with 2x sub-passes
      if (threadIdx.x == 0) fail[p] |= 1;
      for (int i = threadIdx.x; i < H; i += NT) mg_clear(smem, ids, rt, otab, q.n_ops, i);
      lds_barrier();
      if (threadIdx.x == 0) {
        lovf = 0;
        nnew = 0;
      }
      lds_barrier();
      it = nit;
      continue;
    }
    // 2. resident rows: mark the delta entries they absorb; count live rows
    int n_mine = 0;
    for (int64_t r0 = 0; r0 < nrow; r0 += NT) {
      const int64_t r = r0 + threadIdx.x;
      if (r >= nrow) break;
      const int e = mg_find(q, ids, src + r * q.sw, evict, close0, sbits, sub, wbase, H);
      if (e >= 0) rt[e] |= RT_MATCHED;  // one resident row per identity: a plain store
      n_mine += e != -2 ? 1 : 0;
    }
    lds_barrier();
    const int nn = nnew;  // read by every thread here; reset after the next barrier
    // (pane entries are not rows)
    for (int i = threadIdx.x; i < nn; i += NT)
      n_mine += !(rt[nl[i]] & RT_MATCHED) && !(PB && (int64_t)(ids[nl[i]] & ((1ULL << q.log2P) - 1)) >= PB) ? 1 : 0;
    // 3. per-wave row counts → the partition's region range (one atomic per work item)
    const int wave_rows = (int)wave_sum(n_mine);
    if (lane == 0) wsum[wave] = wave_rows;
    lds_barrier();
    int wave_before = 0, total = 0;
    for (int k = 0; k < NW; k++) {
      if (k < wave) wave_before += wsum[k];
      total += wsum[k];
    }
    if (threadIdx.x == 0) {
      if (work) {  // sub-passes of one partition append to its region
        lbase = total ? atomicAdd(&newcnt[p], (unsigned long long)total) : 0ULL;
      } else {  // the partition's only work item: no atomic round trip
        lbase = 0;
        newcnt[p] = (unsigned long long)total;
      }
    }
    lds_barrier();
    MG_T(3);
    if ((int64_t)(lbase + total) > q.cmax) {
      if (threadIdx.x == 0) {
        fail[p] |= 2;
        atomicMax(need, (unsigned long long)(lbase + total));
        nnew = 0;
      }
      for (int i = threadIdx.x; i < H; i += NT) mg_clear(smem, ids, rt, otab, q.n_ops, i);
      lds_barrier();
      it = nit;
      continue;
    }
    // 4. write: lanes take ranks from ballots so consecutive lanes store consecutive rows; each
    //    wave owns a contiguous output range.  Delta entries are cleared once consumed.
    uint64_t* dst0 = (it.sel ? buf0 : buf1) + (uint64_t)p * q.cmax * q.sw;
    uint64_t cur = lbase + (uint64_t)wave_before;
    const uint64_t lt = (1ULL << lane) - 1;
    const int hv = q.having.a.w_val, hc = q.having.a.w_cnt;
    int nh = 0;
    for (int64_t r0 = 0; r0 < nrow; r0 += NT) {
      const int64_t r = r0 + threadIdx.x;
      const uint64_t* row = src + (r < nrow ? r : 0) * q.sw;
      const int e = r < nrow ? mg_find(q, ids, row, evict, close0, sbits, sub, wbase, H) : -2;
      const bool live = e != -2;
      const uint64_t b = __ballot(live);
      if (live) {
        const uint64_t ri = cur + __popcll(b & lt);
        uint64_t* dst = dst0 + ri * q.sw;
        uint64_t w2 = row[2];
        if (e >= 0) {
          const uint32_t rr = rt[e] & ~RT_MATCHED;
          const int64_t t = rr ? tbase + (int64_t)rr - 1 : INT64_MIN;
          w2 = t > (int64_t)w2 ? (uint64_t)t : w2;
        }
        *(longlong2*)dst = make_longlong2((int64_t)row[0], (int64_t)row[1]);
        bool now;
        if constexpr (CNT1) {
          const uint64_t c = row[3] + (e >= 0 ? (uint64_t)cnt1[e] : 0ULL);
          *(longlong2*)(dst + 2) = make_longlong2((int64_t)w2, (int64_t)c);
          now = having_ok_words(c, 0, q.having);
        } else {
          for (int k = 2; k < q.sw; k += 2) {
            const uint64_t a = k == 2 ? w2 : (e >= 0 ? mg_word(wtab, smem, k, row, e) : row[k]);
            const uint64_t c = e >= 0 ? mg_word(wtab, smem, k + 1, row, e) : row[k + 1];
            *(longlong2*)(dst + k) = make_longlong2((int64_t)a, (int64_t)c);
          }
          now = !q.having.active ||
                having_ok_words(e >= 0 ? mg_word(wtab, smem, hv, row, e) : row[hv],
                                hc < 0 ? 0 : (e >= 0 ? mg_word(wtab, smem, hc, row, e) : row[hc]), q.having);
        }
        if (q.having.active) nh += now ? 1 : 0;
        if (q.chg) {  // emission flags: touched rows, HAVING before (the old row) and after
          uint8_t f = 0;
          if (e >= 0)
            f = (uint8_t)(CHG_TOUCHED | (having_ok_words(row[hv], hc < 0 ? 0ULL : row[hc], q.having) ? CHG_OLD : 0) |
                          (now ? CHG_NEW : 0));
          q.chg[(uint64_t)p * q.cmax + ri] = f;
        }
      }
      cur += __popcll(b);
    }
    lds_barrier();  // resident rows have read their entries: the loop below clears them all
    if (threadIdx.x == 0) nnew = 0;  // every thread read it (nn) before the barrier above
    for (int i0 = wave * 64; i0 < nn; i0 += NT) {  // the claimed entries, 64 per wave step
      const int li = i0 + lane;
      const int e = li < nn ? (int)nl[li] : H + lane;  // past the list: the lane's dummy entry
      const uint64_t id = li < nn ? ids[e] : EMPTY_ID;
      const bool isnew = id != EMPTY_ID && !(rt[e] & RT_MATCHED) &&
                         !(PB && (int64_t)(id & ((1ULL << q.log2P) - 1)) >= PB);  // panes are not rows
      const uint64_t b = __ballot(isnew);
      if (isnew) {
        const uint64_t ri = cur + __popcll(b & lt);
        uint64_t* dst = dst0 + ri * q.sw;
        const uint64_t hk = ((uint64_t)p << (64 - q.log2P)) | (id >> q.log2P);
        const int64_t ws = (((int64_t)(id & ((1ULL << q.log2P) - 1))) + wbase) * (q.windowed ? q.adv : 0);
        *(longlong2*)dst = make_longlong2(key_of_hash(hk), ws);
        bool now;
        if constexpr (CNT1) {
          const uint32_t c = cnt1[e];
          *(longlong2*)(dst + 2) = make_longlong2(tbase + (int64_t)rt[e] - 1, (int64_t)c);
          now = having_ok_words(c, 0, q.having);
        } else {
          for (int k = 2; k < q.sw; k += 2) {
            const uint64_t a = k == 2 ? (uint64_t)(tbase + (int64_t)rt[e] - 1) : mg_word(wtab, smem, k, nullptr, e);
            *(longlong2*)(dst + k) = make_longlong2((int64_t)a, (int64_t)mg_word(wtab, smem, k + 1, nullptr, e));
          }
          now = !q.having.active || having_ok_words(mg_word(wtab, smem, hv, nullptr, e),
                                                    hc < 0 ? 0 : mg_word(wtab, smem, hc, nullptr, e), q.having);
        }
        if (q.having.active) nh += now ? 1 : 0;
        if (q.chg) q.chg[(uint64_t)p * q.cmax + ri] = (uint8_t)(CHG_TOUCHED | (now ? CHG_NEW : 0));
      }
      if (id != EMPTY_ID) {
        if constexpr (CNT1) {
          ids[e] = EMPTY_ID;
          rt[e] = 0u;
          cnt1[e] = 0u;
        } else {
          mg_clear(smem, ids, rt, otab, q.n_ops, e);
        }
      }
      cur += __popcll(b);
    }
    if (q.having.active) {
      nh = (int)wave_sum(nh);
      if (lane == 0 && nh) atomicAdd(&hnew[p], (unsigned long long)nh);
    }
    lds_barrier();  // the table is clear for the next item
    MG_T(4);
    it = nit;
  }
#undef MG_T
}

// ------------------------------------------------------------------ k_part_merge_c1
// The COUNT(*) merge over 12-byte records (C1, C2: TUMBLING or no window, one u32 count), written
// for its instruction count.  k_part_merge<true, 512, true> issued ~200 VALU instructions per
// record (64-bit identities and slots, a claimed-entry list with a ballot and an LDS atomic per
// record, the generic sub-pass / op machinery): on C2 its VALU issue alone was ~60 % of its time
// (SQ_INSTS_VALU 3.2e8 per push, profiles/r03/).  Here every per-record step is 32-bit:
//   identity  lo = key hash bits 0..31, hi = (key hash bits 32..63 << log2P) | window index - wbase
//             (the partition's top log2P hash bits are implied): one 64-bit LDS CAS
//   slot      (hash lo + window * 0x9E3779B1) >> (32 - log2H), H a power of two, linear probing
//   state     u32 rowtime delta (ts - tbase + 1; bit 31: matched by a resident row), u32 count
// The write-out scans the table (each wave a contiguous 1/NW of it, ballots kept in scalar
// registers between the count and the write) instead of keeping a list of claimed entries.
// LDS = (H + 64) x 16 B: ids | rowtime | count, the 64 per-lane dummy entries absorb the inactive
// lanes' CASes.  Phases, the persistent item loop, retries and HAVING / changelog bookkeeping are
// k_part_merge's (the contract is the same; k_part_commit publishes the result).

// k_part_merge_c1's parameters: only what it reads (a large by-value argument struct keeps its
// fields live in scalar registers across the item loop; the spills cost VALU moves)
struct C1Params {
  int32_t log2P, log2H, sw, hv_active, hv_op;
  int64_t size, adv, cmax, hv_i64;
  FastDiv fd;
  FastDiv32 fd32;
  uint8_t* chg;  // changelog: per-row-slot emission flags (CHG_*), or null
};

// HAVING on the COUNT(*) word (the query's only aggregate)
__device__ __forceinline__ bool c1_having(const C1Params& q, uint64_t c) {
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

__device__ __forceinline__ int c1_find(const KLDS uint64_t* ids, uint64_t id, uint32_t e, int H) {
  for (int probe = 0; probe < H; probe++) {
    const uint64_t v = ids[e];
    if (v == id) return (int)e;
    if (v == EMPTY_ID) return -1;
    e = (e + 1) & (uint32_t)(H - 1);
  }
  return -1;
}

// RM: the record layout this instantiation reads (0: R12, 1: R8); the host launches both and the
// one that does not match k_part_wrange's choice (wr[7]) exits at once.  One instantiation with
// both layouts spilled the prefetched records to scratch (a spill waits for its load).
template <int NT, int AU, int RM>
__global__ __launch_bounds__(NT, 4) void k_part_merge_c1(
    C1Params q, const uint32_t* __restrict__ work, int64_t nwork, const int64_t* __restrict__ pbase,
    const uint64_t* __restrict__ srec, int first, uint64_t* __restrict__ buf0, uint64_t* __restrict__ buf1,
    const uint8_t* __restrict__ sel, const int64_t* __restrict__ cnt, unsigned long long* __restrict__ newcnt,
    uint8_t* __restrict__ fail, unsigned long long* __restrict__ need, int64_t close0, uint64_t* __restrict__ closed,
    unsigned long long* __restrict__ closed_n, const int64_t* __restrict__ wr, unsigned long long* __restrict__ hnew,
    unsigned long long* __restrict__ hclosed, unsigned long long* __restrict__ dbg) {
  if (wr[4] == 0) return;  // k_part_wrange declined the merge path for this push
  if ((wr[7] != 0) != (RM == 1)) return;  // the other record layout's instantiation
  // dbg (KHIP_AGG_PROBE): wall-clock time per phase summed over the workgroups (thread 0's view)
  unsigned long long t_last = dbg ? wall_clock64() : 0ULL;
#define C1_T(k)                                                                        \
  do {                                                                                 \
    if (dbg && threadIdx.x == 0) {                                                     \
      const unsigned long long now = wall_clock64();                                   \
      atomicAdd(&dbg[(k)], now - t_last);                                              \
      t_last = now;                                                                    \
    }                                                                                  \
  } while (0)
  constexpr int NW = NT / 64;
  const int log2H = q.log2H;
  const int H = 1 << log2H;
  const int EPW = H / NW;  // entries per wave in the write-out scan (a multiple of 64)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  KLDS uint64_t* ids = mg_plane<uint64_t>(smem, 0);
  KLDS uint32_t* rt = mg_plane<uint32_t>(smem, (H + 64) * 8);
  KLDS uint32_t* ct = mg_plane<uint32_t>(smem, (H + 64) * 12);
  __shared__ int lovf;
  __shared__ int wsum[NW];
  __shared__ unsigned long long lbase;
  const int64_t tbase = wr[5], wbase = wr[0];
  const int64_t q0 = (int64_t)fast_udiv((uint64_t)tbase, q.fd);
  const uint32_t r0 = (uint32_t)(tbase - q0 * q.adv);
  const uint32_t qw0 = (uint32_t)(q0 - wbase);
  const int log2P = q.log2P;
  const uint32_t wmask = (1u << log2P) - 1u;
  const bool evict = close0 != INT64_MIN;
  const uint32_t dummy = (uint32_t)H + (uint32_t)lane;
  for (int i = threadIdx.x; i < H + 64; i += NT) {
    ids[i] = EMPTY_ID;
    rt[i] = 0u;
    ct[i] = 0u;
  }
  if (threadIdx.x == 0) lovf = 0;
  // window index of a record relative to wbase (the packed identity's low log2P bits); the host
  // launches this kernel only for windowed queries with adv <= 2^31 (q.div32)
  const FastDiv32 fd32 = q.fd32;
  auto wrel_of = [&](uint32_t trel) -> uint32_t { return qw0 + fast_udiv32(r0 + trel - 1u, fd32); };
  // the identity and home slot of a resident row
  auto row_id = [&](const uint64_t* row, uint64_t* id, uint32_t* e) {
    const uint64_t hk = key_hash((int64_t)row[0]);
    const uint32_t w = (uint32_t)((int64_t)fast_udiv((uint64_t)row[1], q.fd) - wbase);
    const uint32_t lo = (uint32_t)hk;
    *id = ((uint64_t)(((uint32_t)(hk >> 32) << log2P) | w) << 32) | lo;
    *e = (lo + w * C1_GOLD) >> (32 - log2H);
  };
  // two register sets of records: chunk c + 1 in flight while chunk c is applied.  Every load is
  // unconditional (indices clamped to the item's last record; an empty item reads record rbase,
  // which exists: srec has a spare record), so the compiler counts the loads in flight exactly on
  // every path and each wait covers only the set about to be applied.  A record stays
  // the (lo, hi, trel) triple the load returns (a uint3: the load writes the registers the apply
  // reads; splitting it into per-field arrays made the compiler copy — and so wait for — each load
  // right after issuing it)
  // R8 records (k_part_wrange chose them for this push): one 8-byte word, (key - kbase) << r8tb |
  // trel; the key hash is recomputed here
  const int r8tb = RM == 1 ? (int)wr[7] : 0;
  const int64_t kbase = wr[6];
  const uint64_t r8mask = r8tb ? (~0ULL >> (64 - r8tb)) : 0ULL;
  uint3 ra[AU], rb[AU];
  auto load = [&](uint3 (&x)[AU], int64_t rbase, int64_t rn, int64_t l0) {
    if constexpr (RM == 1) {
      const uint32_t* base = (const uint32_t*)srec + (uint64_t)rbase * 2;
#pragma unroll
      for (int u = 0; u < AU; u++) {
        const int64_t li = l0 + threadIdx.x + (int64_t)u * NT;
        const uint32_t* r = base + (uint64_t)(li < rn ? li : (rn > 0 ? rn - 1 : 0)) * 2;
        x[u].x = __builtin_nontemporal_load(r);
        x[u].y = __builtin_nontemporal_load(r + 1);
      }
      return;
    }
    const uint32_t* base = (const uint32_t*)srec + (uint64_t)rbase * 3;
#pragma unroll
    for (int u = 0; u < AU; u++) {
      const int64_t li = l0 + threadIdx.x + (int64_t)u * NT;
      const uint32_t* r = base + (uint64_t)(li < rn ? li : (rn > 0 ? rn - 1 : 0)) * 3;
      // three dword loads, not one dwordx3: a 3-register tuple must start at an even register, and
      // the re-aligning copy would wait for the load right after issuing it
      x[u].x = __builtin_nontemporal_load(r);
      x[u].y = __builtin_nontemporal_load(r + 1);
      x[u].z = __builtin_nontemporal_load(r + 2);
    }
  };
  int64_t w = blockIdx.x;
  MgItem it{};
  if (w < nwork) it = mg_item(work, w, pbase, sel, cnt);
  load(ra, it.rbase, it.rn, 0);
  lds_barrier();
  for (; w < nwork; w += gridDim.x) {
    const uint32_t p = it.p;
    const int sbits = it.sbits, sub = it.sub;
    const int64_t rbase = it.rbase, rn = it.rn;
    const int64_t wnext = w + gridDim.x;
    MgItem nit = it;  // past the last item: harmless reloads of this one
    if (wnext < nwork) nit = mg_item(work, wnext, pbase, sel, cnt);
    if (rn == 0 && first) {  // untouched partition: nothing to rewrite
      load(ra, nit.rbase, nit.rn, 0);
      it = nit;
      continue;
    }
    const uint64_t* src = (it.sel ? buf1 : buf0) + (uint64_t)p * q.cmax * q.sw;
    const int64_t nrow = it.nrow;
    // 0. closed resident rows → closed store (pass 0 only; retries skip them)
    if (evict && first) {
      int ne = 0, nh = 0;
      for (int64_t r = threadIdx.x; r < nrow; r += NT) {
        const uint64_t* row = src + r * q.sw;
        ne += ((int64_t)row[1] + q.size <= close0) && sub_ok(key_hash((int64_t)row[0]), (int64_t)row[1], sbits, sub);
      }
      int incl = ne;
      for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
      }
      if (lane == 63) wsum[wave] = incl;
      lds_barrier();
      int before = 0, total = 0;
      for (int k = 0; k < NW; k++) {
        if (k < wave) before += wsum[k];
        total += wsum[k];
      }
      if (threadIdx.x == 0) lbase = total ? atomicAdd(closed_n, (unsigned long long)total) : 0ULL;
      lds_barrier();
      uint64_t* dst = closed + (lbase + (uint64_t)(before + incl - ne)) * q.sw;
      for (int64_t r = threadIdx.x; r < nrow; r += NT) {
        const uint64_t* row = src + r * q.sw;
        if (!((int64_t)row[1] + q.size <= close0) || !sub_ok(key_hash((int64_t)row[0]), (int64_t)row[1], sbits, sub))
          continue;
        for (int k = 0; k < q.sw; k++) dst[k] = row[k];
        dst += q.sw;
        nh += q.hv_active && c1_having(q, row[3]) ? 1 : 0;
      }
      if (q.hv_active) {
        nh = (int)wave_sum(nh);
        if (lane == 0 && nh) atomicAdd(hclosed, (unsigned long long)nh);
      }
      lds_barrier();
    }
    C1_T(0);
    // 1. records → delta entries
    auto apply = [&](const uint3 (&xr)[AU], int64_t l0) {
      uint64_t id[AU], old[AU];
      uint32_t e[AU];
      bool pend[AU];
      uint3 x[AU];
#pragma unroll
      for (int u = 0; u < AU; u++) {
        if constexpr (RM == 1) {  // (lo, hi) of the key hash, trel
          const uint64_t v = ((uint64_t)xr[u].y << 32) | xr[u].x;
          const uint64_t hk = key_hash(kbase + (int64_t)(v >> r8tb));
          x[u] = make_uint3((uint32_t)hk, (uint32_t)(hk >> 32), (uint32_t)(v & r8mask));
        } else {
          x[u] = xr[u];
        }
      }
#pragma unroll
      for (int u = 0; u < AU; u++) {
        const int64_t li = l0 + threadIdx.x + (int64_t)u * NT;
        const uint32_t trel = x[u].z;
        const uint32_t wi = wrel_of(trel);
        bool act = li < rn && trel != 0u;
        if (sbits) act = act && sub_ok(((uint64_t)x[u].y << 32) | x[u].x, ((int64_t)wi + wbase) * q.adv, sbits, sub);
        id[u] = act ? ((uint64_t)((x[u].y << log2P) | wi) << 32) | x[u].x : EMPTY_ID;
        e[u] = act ? (x[u].x + wi * C1_GOLD) >> (32 - log2H) : dummy;
      }
#pragma unroll
      for (int u = 0; u < AU; u++) {
        old[u] = EMPTY_ID;
        __hip_atomic_compare_exchange_strong(&ids[e[u]], &old[u], id[u], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP);
      }
#pragma unroll
      for (int u = 0; u < AU; u++) pend[u] = old[u] != EMPTY_ID && old[u] != id[u];
      for (int probes = 1;; probes++) {  // collisions: every pending record probes on together
        bool anyp = false;
#pragma unroll
        for (int u = 0; u < AU; u++) anyp |= pend[u];
        if (!__ballot(anyp)) break;
        if (probes >= H) {
          lovf = 1;
#pragma unroll
          for (int u = 0; u < AU; u++)
            if (pend[u]) id[u] = EMPTY_ID;
          break;
        }
#pragma unroll
        for (int u = 0; u < AU; u++) {
          if (!pend[u]) continue;
          e[u] = (e[u] + 1) & (uint32_t)(H - 1);
          uint64_t o2 = EMPTY_ID;
          __hip_atomic_compare_exchange_strong(&ids[e[u]], &o2, id[u], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
          pend[u] = o2 != EMPTY_ID && o2 != id[u];
        }
      }
#pragma unroll
      for (int u = 0; u < AU; u++) {
        if (id[u] == EMPTY_ID) continue;
        __hip_atomic_fetch_max(&rt[e[u]], x[u].z, WG_RLX);
        __hip_atomic_fetch_add(&ct[e[u]], 1u, WG_RLX);
      }
    };
    const int64_t nch = (rn + (int64_t)AU * NT - 1) / ((int64_t)AU * NT);
    for (int64_t c = 0; c < nch; c += 2) {
      load(rb, rbase, rn, (c + 1) * AU * NT);
      apply(ra, c * AU * NT);
      if (c + 1 >= nch || *(volatile KLDS int*)&lovf) break;
      load(ra, rbase, rn, (c + 2) * AU * NT);
      apply(rb, (c + 1) * AU * NT);
      if (*(volatile KLDS int*)&lovf) break;
    }
    lds_barrier();
    C1_T(1);
    // the next item's first chunk is in flight from here on (its second one too was measured
    // slower: the count phase then waits behind those loads)
    load(ra, nit.rbase, nit.rn, 0);
    if (lovf) {  // more groups than the table: retried with 2x sub-passes
      if (threadIdx.x == 0) fail[p] |= 1;
      for (int i = threadIdx.x; i < H; i += NT) {
        ids[i] = EMPTY_ID;
        rt[i] = 0u;
        ct[i] = 0u;
      }
      lds_barrier();
      if (threadIdx.x == 0) lovf = 0;
      lds_barrier();
      it = nit;
      continue;
    }
    // 2. resident rows: mark the delta entries they absorb; count live rows
    int n_mine = 0;
    for (int64_t r = threadIdx.x; r < nrow; r += NT) {
      const uint64_t* row = src + r * q.sw;
      if (evict && (int64_t)row[1] + q.size <= close0) continue;
      if (sbits && !sub_ok(key_hash((int64_t)row[0]), (int64_t)row[1], sbits, sub)) continue;
      uint64_t id;
      uint32_t e0;
      row_id(row, &id, &e0);
      const int e = c1_find(ids, id, e0, H);
      if (e >= 0) rt[e] |= RT_MATCHED;  // one resident row per identity: a plain store
      n_mine++;
    }
    lds_barrier();
    // the wave's share of the table: new (unmatched) entries, one ballot per 64 entries
    const int ebase = wave * EPW;
    int nnew = 0;
    for (int k = 0; k < EPW; k += 64) {
      const int e = ebase + k + lane;
      const bool isnew = ids[e] != EMPTY_ID && !(rt[e] & RT_MATCHED);
      nnew += (int)__popcll(__ballot(isnew));
    }
    // 3. per-wave row counts → the partition's region range (one atomic per work item)
    const int wave_rows = (int)wave_sum(n_mine) + nnew;
    if (lane == 0) wsum[wave] = wave_rows;
    lds_barrier();
    int wave_before = 0, total = 0;
    for (int k = 0; k < NW; k++) {
      if (k < wave) wave_before += wsum[k];
      total += wsum[k];
    }
    if (threadIdx.x == 0) {
      if (work) {  // sub-passes of one partition append to its region
        lbase = total ? atomicAdd(&newcnt[p], (unsigned long long)total) : 0ULL;
      } else {  // the partition's only work item: no atomic round trip
        lbase = 0;
        newcnt[p] = (unsigned long long)total;
      }
    }
    lds_barrier();
    if ((int64_t)(lbase + total) > q.cmax) {
      if (threadIdx.x == 0) {
        fail[p] |= 2;
        atomicMax(need, (unsigned long long)(lbase + total));
      }
      for (int i = threadIdx.x; i < H; i += NT) {
        ids[i] = EMPTY_ID;
        rt[i] = 0u;
        ct[i] = 0u;
      }
      lds_barrier();
      it = nit;
      continue;
    }
    C1_T(2);
    // 4. write: resident rows (merged), then the wave's new entries; lanes take ranks from ballots
    //    so each store instruction covers consecutive rows
    uint64_t* dst0 = (it.sel ? buf0 : buf1) + (uint64_t)p * q.cmax * q.sw;
    uint64_t cur = lbase + (uint64_t)wave_before;
    const uint64_t lt = (1ULL << lane) - 1;
    int nh = 0;
    for (int64_t r0 = wave * 64; r0 < nrow; r0 += NT) {
      const int64_t r = r0 + lane;
      const uint64_t* row = src + (r < nrow ? r : 0) * q.sw;
      bool live = r < nrow && !(evict && (int64_t)row[1] + q.size <= close0);
      if (live && sbits) live = sub_ok(key_hash((int64_t)row[0]), (int64_t)row[1], sbits, sub);
      int e = -1;
      if (live) {
        uint64_t id;
        uint32_t e0;
        row_id(row, &id, &e0);
        e = c1_find(ids, id, e0, H);
      }
      const uint64_t b = __ballot(live);
      if (live) {
        const uint64_t ri = cur + __popcll(b & lt);
        uint64_t* dst = dst0 + ri * q.sw;
        uint64_t w2 = row[2], c = row[3];
        if (e >= 0) {
          const int64_t t = tbase + (int64_t)(rt[e] & ~RT_MATCHED) - 1;
          w2 = t > (int64_t)w2 ? (uint64_t)t : w2;
          c += ct[e];
        }
        *(longlong2*)dst = make_longlong2((int64_t)row[0], (int64_t)row[1]);
        *(longlong2*)(dst + 2) = make_longlong2((int64_t)w2, (int64_t)c);
        const bool now = !q.hv_active || c1_having(q, c);
        nh += q.hv_active && now ? 1 : 0;
        if (q.chg)
          q.chg[(uint64_t)p * q.cmax + ri] =
              e >= 0 ? (uint8_t)(CHG_TOUCHED | (!q.hv_active || c1_having(q, row[3]) ? CHG_OLD : 0) | (now ? CHG_NEW : 0))
                     : (uint8_t)0;
      }
      cur += __popcll(b);
    }
    lds_barrier();  // every wave's resident rows have read their entries: the scan below clears them
    const uint64_t hkp = (uint64_t)p << (32 - log2P);
    for (int k = 0; k < EPW; k += 64) {
      const int e = ebase + k + lane;
      const uint64_t id = ids[e];
      const uint32_t rv = rt[e];
      const bool isnew = id != EMPTY_ID && !(rv & RT_MATCHED);
      const uint64_t b = __ballot(isnew);
      if (isnew) {
        const uint64_t ri = cur + __popcll(b & lt);
        uint64_t* dst = dst0 + ri * q.sw;
        const uint32_t ih = (uint32_t)(id >> 32);
        const uint64_t hk = ((hkp | (ih >> log2P)) << 32) | (uint32_t)id;
        const int64_t ws = ((int64_t)(ih & wmask) + wbase) * q.adv;
        const uint32_t c = ct[e];
        *(longlong2*)dst = make_longlong2(key_of_hash(hk), ws);
        *(longlong2*)(dst + 2) = make_longlong2(tbase + (int64_t)rv - 1, (int64_t)c);
        const bool now = !q.hv_active || c1_having(q, c);
        nh += q.hv_active && now ? 1 : 0;
        if (q.chg) q.chg[(uint64_t)p * q.cmax + ri] = (uint8_t)(CHG_TOUCHED | (now ? CHG_NEW : 0));
      }
      if (id != EMPTY_ID) {  // every entry of the wave's share leaves cleared for the next item
        ids[e] = EMPTY_ID;
        rt[e] = 0u;
        ct[e] = 0u;
      }
      cur += __popcll(b);
    }
    if (q.hv_active) {
      nh = (int)wave_sum(nh);
      if (lane == 0 && nh) atomicAdd(&hnew[p], (unsigned long long)nh);
    }
    lds_barrier();  // the table is clear for the next item
    C1_T(3);
    it = nit;
  }
#undef C1_T
}

// Window-index range of this push for the packed identity: the batch's windows plus the
// live resident ones (res = conservative [min, max] window index of resident rows; rows of
// windows closed before this push are evicted before they are encoded).
// wr = [wbase, identity ok, tmin, tmax, k_part_merge runs, rowtime base].  The aggregate kernel
// is chosen here, on the device, so the host never waits between the scatter and the aggregate:
// k_part_merge needs the packed identity and an event-time span below 2^31 - 2 ms (u32 rowtime
// deltas); when it declines, the host re-runs pass 0 with k_part_agg after the push's one sync.
// Also zeroes the pass counters and publishes the closed-store row count (no host copies).
__global__ __launch_bounds__(1024) void k_part_wrange(const int64_t* __restrict__ tilemin,
                                                      const int64_t* __restrict__ tilemax, int64_t nT, int windowed,
                                                      int64_t size, int64_t adv, FastDiv fd, int64_t close0,
                                                      int log2P, int fresh, int allow, int merge_allow,
                                                      int64_t* __restrict__ res, int64_t* __restrict__ wr,
                                                      unsigned long long* __restrict__ ctr,
                                                      unsigned long long* __restrict__ closed_ctr,
                                                      unsigned long long closed_n,
                                                      const int64_t* __restrict__ tilekr, int r8_allow) {
  __shared__ int64_t smin[16], smax[16], skx[16], skn[16];
  int64_t mn = INT64_MAX, mx = -1, kx = INT64_MIN, kn = INT64_MIN;
  for (int64_t t = threadIdx.x; t < nT; t += 1024) {
    mn = tilemin[t] < mn ? tilemin[t] : mn;
    mx = tilemax[t] > mx ? tilemax[t] : mx;
    if (tilekr) {
      kx = tilekr[2 * t] > kx ? tilekr[2 * t] : kx;
      kn = tilekr[2 * t + 1] > kn ? tilekr[2 * t + 1] : kn;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const int64_t a = __shfl_xor(mn, off, 64), b = __shfl_xor(mx, off, 64);
    const int64_t c = __shfl_xor(kx, off, 64), d = __shfl_xor(kn, off, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
    kx = c > kx ? c : kx;
    kn = d > kn ? d : kn;
  }
  if ((threadIdx.x & 63) == 0) {
    smin[threadIdx.x >> 6] = mn;
    smax[threadIdx.x >> 6] = mx;
    skx[threadIdx.x >> 6] = kx;
    skn[threadIdx.x >> 6] = kn;
  }
  __syncthreads();
  if (threadIdx.x) return;
  for (int w = 0; w < 16; w++) {
    mn = smin[w] < mn ? smin[w] : mn;
    mx = smax[w] > mx ? smax[w] : mx;
    kx = skx[w] > kx ? skx[w] : kx;
    kn = skn[w] > kn ? skn[w] : kn;
  }
  wr[2] = mn;  // event-time span of the accepted records (INT64_MAX / -1: none)
  wr[3] = mx;
  wr[5] = mx < 0 ? 0 : mn;
  const bool span_ok = mx < 0 || mx - mn < ((int64_t)1 << 31) - 2;
  // R8 records (8 bytes: key - kbase above the rowtime delta) when the push's key range and
  // event-time span fit one word together: wr[6] = kbase, wr[7] = rowtime-delta bits (0: R12)
  wr[6] = 0;
  wr[7] = 0;
  if (r8_allow && tilekr && mx >= 0 && span_ok) {
    const int64_t kmin = ~kn;
    const uint64_t krange = (uint64_t)kx - (uint64_t)kmin;
    const uint64_t trange = (uint64_t)(mx - mn + 1);  // trel in [0, mx - mn + 1]
    const int kb = krange ? 64 - __clzll((long long)krange) : 0;
    const int tb = 64 - __clzll((long long)trange);
    if (kb + tb <= 64) {
      wr[6] = kmin;
      wr[7] = tb;
    }
  }
  ctr[0] = ctr[1] = ctr[2] = 0ULL;
  if (closed_ctr) *closed_ctr = closed_n;
  int64_t lo = INT64_MAX, hi = INT64_MIN;
  if (mx >= 0) {  // some accepted record
    if (windowed) {
      const int64_t l = mn - size + adv;
      lo = (int64_t)fast_udiv((uint64_t)(l > 0 ? l : 0), fd);
      hi = (int64_t)fast_udiv((uint64_t)mx, fd);
    } else {
      lo = hi = 0;
    }
  }
  if (!fresh) {
    int64_t rlo = res[0];
    const int64_t rhi = res[1];
    if (windowed && close0 != INT64_MIN && rlo != INT64_MAX) {  // live: ws > close0 - size
      const int64_t c = close0 - size;
      const int64_t lb = c >= 0 ? (int64_t)fast_udiv((uint64_t)c, fd) + 1 : 0;
      rlo = rlo > lb ? rlo : lb;
    }
    lo = rlo < lo ? rlo : lo;
    hi = rhi > hi ? rhi : hi;
  }
  const bool fits = allow && log2P >= 1 && log2P < 63;
  if (lo > hi) {  // nothing live, nothing new
    wr[0] = 0;
    wr[1] = fits;
    wr[4] = merge_allow && fits && span_ok;
    wr[8] = 0;
    res[0] = INT64_MAX;
    res[1] = INT64_MIN;
    return;
  }
  wr[0] = lo;
  wr[1] = fits && hi - lo < ((int64_t)1 << log2P) - 1;
  // panes (k_part_merge): pane identities use window indices offset by 2^(log2P - 1)
  wr[8] = fits && log2P >= 2 && hi - lo < ((int64_t)1 << (log2P - 1)) - 1;
  wr[4] = merge_allow && wr[1] && span_ok;
  res[0] = lo;
  res[1] = hi;
}

// Publish the partitions processed in this pass (all touched ones, or the retry list).
// gate (k_part_merge's pass 0): nothing to publish when k_part_wrange declined the merge.
// out[11] = rows passing the query's HAVING over all live partitions (maintained: += new - old).
__global__ __launch_bounds__(256) void k_part_commit(const int64_t* __restrict__ gate, int P,
                                                     const int64_t* __restrict__ pbase,
                                                     const uint32_t* __restrict__ prn,
                                                     const uint32_t* __restrict__ plist, int nlist,
                                                     uint8_t* __restrict__ sel, int64_t* __restrict__ cnt,
                                                     unsigned long long* __restrict__ newcnt,
                                                     const uint8_t* __restrict__ fail,
                                                     unsigned long long* __restrict__ out /* [new groups, failed] */,
                                                     unsigned long long* __restrict__ hcnt,
                                                     unsigned long long* __restrict__ hnew) {
  if (gate && gate[4] == 0) return;
  const int k = blockIdx.x * 256 + threadIdx.x;
  int64_t added = 0, failed = 0, hdelta = 0;
  if (plist ? k < nlist : k < P) {
    const uint32_t p = plist ? plist[k] : (uint32_t)k;
    if (plist || (prn ? prn[p] != 0 : pbase[p + 1] > pbase[p])) {
      if (fail[p] == 0) {
        added = (int64_t)newcnt[p] - cnt[p];
        cnt[p] = (int64_t)newcnt[p];
        sel[p] ^= 1;
        if (hcnt) {
          hdelta = (int64_t)hnew[p] - (int64_t)hcnt[p];
          hcnt[p] = hnew[p];
        }
      } else {
        failed = 1;
      }
      newcnt[p] = 0;
      if (hnew) hnew[p] = 0;
    }
  }
  added = wave_sum(added);
  failed = wave_sum(failed);
  hdelta = wave_sum(hdelta);
  if ((threadIdx.x & 63) == 0) {
    if (added) atomicAdd(&out[0], (unsigned long long)added);
    if (failed) atomicAdd(&out[1], (unsigned long long)failed);
    if (hdelta) atomicAdd(&out[11], (unsigned long long)hdelta);
  }
}

// End-of-push counters in one place (one device-to-host copy per push): out[3 + k] = sum over
// tiles of the per-tile counters k, out[3 + T_NPART] = closed rows, out[4 + T_NPART] = stream time.
__global__ __launch_bounds__(256) void k_part_stats(const int64_t* __restrict__ tpart, int64_t nT,
                                                    const unsigned long long* __restrict__ closed_n,
                                                    const int64_t* __restrict__ stream_time,
                                                    unsigned long long* __restrict__ out) {
  __shared__ unsigned long long acc[T_NPART];
  if (threadIdx.x < T_NPART) acc[threadIdx.x] = 0;
  __syncthreads();
  for (int k = 0; k < T_NPART; k++) {
    int64_t v = 0;
    for (int64_t t = threadIdx.x; t < nT; t += 256) v += tpart[t * T_NPART + k];
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&acc[k], (unsigned long long)v);
  }
  __syncthreads();
  if (threadIdx.x < T_NPART) out[3 + threadIdx.x] = acc[threadIdx.x];
  if (threadIdx.x == 0) {
    out[3 + T_NPART] = closed_n ? *closed_n : 0ULL;
    out[4 + T_NPART] = (unsigned long long)*stream_time;
  }
}

// Copy every partition's rows into new region buffers with a larger capacity.
__global__ __launch_bounds__(256) void k_part_regrow(const uint64_t* __restrict__ b0, const uint64_t* __restrict__ b1,
                                                     const uint8_t* __restrict__ sel, const int64_t* __restrict__ cnt,
                                                     int64_t ocmax, uint64_t* __restrict__ nb0, int64_t ncmax, int sw) {
  const int64_t p = blockIdx.x;
  const uint64_t* src = (sel[p] ? b1 : b0) + (uint64_t)p * ocmax * sw;
  uint64_t* dst = nb0 + (uint64_t)p * ncmax * sw;
  const int64_t words = cnt[p] * sw;
  for (int64_t w = threadIdx.x; w < words; w += 256) dst[w] = src[w];
}

__global__ __launch_bounds__(256) void k_part_regrow_flags(const uint8_t* __restrict__ f, const int64_t* __restrict__ cnt,
                                                           int64_t ocmax, uint8_t* __restrict__ nf, int64_t ncmax) {
  const int64_t p = blockIdx.x;
  for (int64_t r = threadIdx.x; r < cnt[p]; r += 256) nf[p * ncmax + r] = f[p * ocmax + r];
}

// Double the partition count: rows of partition p move to 2p / 2p+1 (next hash bit).
// nb == nullptr: count only (ncnt = child row counts, used to size the new regions).
__global__ __launch_bounds__(256) void k_part_split(const uint64_t* __restrict__ b0, const uint64_t* __restrict__ b1,
                                                    const uint8_t* __restrict__ sel, const int64_t* __restrict__ cnt,
                                                    int64_t cmax, int sw, int new_log2P, uint64_t* __restrict__ nb,
                                                    int64_t ncmax, int64_t* __restrict__ ncnt) {
  __shared__ unsigned int lc[2];
  const int64_t p = blockIdx.x;
  if (threadIdx.x < 2) lc[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t* src = (sel[p] ? b1 : b0) + (uint64_t)p * cmax * sw;
  for (int64_t r = threadIdx.x; r < cnt[p]; r += 256) {
    const uint64_t* row = src + r * sw;
    const uint32_t child = part_of((int64_t)row[0], new_log2P);  // == 2p or 2p+1
    const unsigned k = atomicAdd(&lc[child & 1], 1u);
    if (!nb) continue;
    uint64_t* dst = nb + ((uint64_t)child * ncmax + k) * sw;
    for (int w = 0; w < sw; w++) dst[w] = row[w];
  }
  __syncthreads();
  if (threadIdx.x < 2) ncnt[2 * p + threadIdx.x] = lc[threadIdx.x];
}

// Per partition: rows passing HAVING (count) — or write them at offs[p].
__global__ __launch_bounds__(256) void k_part_rows(const uint64_t* __restrict__ b0, const uint64_t* __restrict__ b1,
                                                   const uint8_t* __restrict__ sel, const int64_t* __restrict__ cnt,
                                                   int64_t cmax, int sw, HavingDev h, int64_t* __restrict__ counts,
                                                   const int64_t* __restrict__ offs, uint64_t* __restrict__ out) {
  __shared__ int lcnt[4];
  __shared__ int64_t lbase;
  __shared__ int lhit;
  const int64_t p = blockIdx.x;
  HavingDev hp = h;  // this partition's view of the query keys
  if (h.pkoff) {
    // point lookup, many keys: the keys of this partition only (grouped on the host)
    const int64_t k0 = h.pkoff[p], k1 = h.pkoff[p + 1];
    if (k0 == k1) {
      if (threadIdx.x == 0 && counts) counts[p] = 0;
      return;
    }
    hp.keys = h.pkeys + k0;
    hp.n_keys = k1 - k0;
  } else if (h.pull && h.n_keys > 0 && h.n_keys <= (int64_t)blockDim.x) {
    // point lookup: only the partitions owning one of the query keys are read
    if (threadIdx.x == 0) lhit = 0;
    __syncthreads();
    if (threadIdx.x < h.n_keys && part_of(h.keys[threadIdx.x], h.log2P) == (uint32_t)p) lhit = 1;
    __syncthreads();
    if (!lhit) {
      if (threadIdx.x == 0 && counts) counts[p] = 0;
      return;
    }
  }
  const uint64_t* src = (sel[p] ? b1 : b0) + (uint64_t)p * cmax * sw;
  const int64_t n = cnt[p];
  if (threadIdx.x == 0) lbase = out ? offs[p] : 0;
  int64_t total = 0;
  for (int64_t r0 = 0; r0 < n; r0 += 256) {
    const int64_t r = r0 + threadIdx.x;
    const bool take = r < n && having_ok(src + r * sw, hp);
    const uint64_t bal = __ballot(take);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) lcnt[wave] = __popcll(bal);
    __syncthreads();
    int before = __popcll(bal & ((1ULL << lane) - 1)), tot = 0;
    for (int w = 0; w < 4; w++) {
      if (w < wave) before += lcnt[w];
      tot += lcnt[w];
    }
    if (take && out) {
      uint64_t* o = out + (lbase + total + before) * (uint64_t)sw;
      for (int w = 0; w < sw; w++) o[w] = src[r * sw + w];
    }
    total += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0 && counts) counts[p] = total;
}

// EMIT CHANGES (the record cache flushed at the push's commit, C/util/KsqlConstants.java:40-41):
// per partition the last push's records reached, the rows it touched whose HAVING holds now
// (emitted as rows) or held before the push (emitted as tombstones, S/TableFilterBuilder.java:
// 63-75).  counts[p] (count pass) or rows at offs[p] + tombstone flags (write pass).
__global__ __launch_bounds__(256) void k_part_chg(const uint64_t* __restrict__ b0, const uint64_t* __restrict__ b1,
                                                  const uint8_t* __restrict__ sel, const int64_t* __restrict__ cnt,
                                                  int64_t cmax, int sw, const int64_t* __restrict__ pbase,
                                                  const uint32_t* __restrict__ prn,
                                                  const uint8_t* __restrict__ chg, int64_t* __restrict__ counts,
                                                  const int64_t* __restrict__ offs, uint64_t* __restrict__ out,
                                                  uint8_t* __restrict__ otomb) {
  __shared__ int lcnt[4];
  const int64_t p = blockIdx.x;
  if (prn ? prn[p] == 0 : pbase[p + 1] == pbase[p]) {  // no record of the push: its flags are stale
    if (threadIdx.x == 0 && counts) counts[p] = 0;
    return;
  }
  const uint64_t* src = (sel[p] ? b1 : b0) + (uint64_t)p * cmax * sw;
  const uint8_t* fl = chg + (uint64_t)p * cmax;
  const int64_t n = cnt[p];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t total = 0;
  const int64_t base = out ? offs[p] : 0;
  for (int64_t r0 = 0; r0 < n; r0 += 256) {
    const int64_t r = r0 + threadIdx.x;
    const uint8_t f = r < n ? fl[r] : 0;
    const bool take = (f & CHG_TOUCHED) && (f & (CHG_OLD | CHG_NEW));
    const uint64_t bal = __ballot(take);
    if (lane == 0) lcnt[wave] = __popcll(bal);
    __syncthreads();
    int before = __popcll(bal & ((1ULL << lane) - 1)), tot = 0;
    for (int w = 0; w < 4; w++) {
      if (w < wave) before += lcnt[w];
      tot += lcnt[w];
    }
    if (take && out) {
      const int64_t o = base + total + before;
      for (int w = 0; w < sw; w++) out[o * sw + w] = src[r * sw + w];
      otomb[o] = (f & CHG_NEW) ? 0 : 1;
    }
    total += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0 && counts) counts[p] = total;
}

// ------------------------------------------------------------------ host side

static int part_ceil_log2(int64_t v) {
  int l = 0;
  while ((1LL << l) < v) l++;
  return l;
}

khip_status part_init(khip_agg* a, int64_t hint) {
  PartState& s = a->part;
  const int nwords = 3 + (int)(a->ap.n_ops > 0 ? 0 : 0);
  (void)nwords;
  // words used = highest word index + 1 (rows are padded to a->sw)
  int used = 3;
  for (int o = 0; o < a->ap.n_ops; o++) used = std::max(used, a->ap.ops[o].word + 1);
  s.nwords = used;
  const int entry = 4 + 8 * used;
  // LDS table: the largest power of two within the budget (default 80 KB: two workgroups
  // per CU overlap one's load/write-back phases with the other's LDS work)
  const int64_t budget = knob("KHIP_LDS_KB", 150) * 1024;
  int H = 256;
  while ((int64_t)(H * 2) * entry + 16 <= budget && H < 16384) H *= 2;
  s.H = H;
  s.H_eff = H * 3 / 4;
  s.lds_bytes = (int)((((size_t)H * 4 + 15) & ~(size_t)15) + (size_t)H * 8 * used);
  if (a->changelog) {  // k_part_agg's emission flag plane: one byte per entry
    s.flag_off = s.lds_bytes;
    s.lds_bytes += H;
  }
  // k_part_merge layout: id u64 | u64 delta planes | rowtime u32 | u32 delta planes, sized so
  // two workgroups share a CU; partitions are sized for whichever kernel holds fewer groups
  {
    int n64 = 0, n32 = 0;
    for (int o = 0; o < a->ap.n_ops; o++) (a->ap.ops[o].kind == OP_INC || a->ap.ops[o].kind == OP_INC_VALID ? n32 : n64)++;
    const int mentry = 8 + 8 * n64 + 4 + 4 * n32 + 2;  // + the u16 claimed-entry list
    const int64_t mbudget = knob("KHIP_MERGE_LDS_KB", 76) * 1024;  // two persistent workgroups per CU
    int mH = (int)std::min<int64_t>(16384, mbudget / mentry - 64) & ~63;
    s.mH = mH;
    const int ms = mH + 64;  // plane stride: H entries + one dummy entry per lane
    int off = ms * 8;
    for (int o = 0; o < a->ap.n_ops; o++)
      if (!(a->ap.ops[o].kind == OP_INC || a->ap.ops[o].kind == OP_INC_VALID)) {
        s.plane_off[o] = off;
        s.plane_w64[o] = 1;
        off += ms * 8;
      }
    s.rt_off = off;
    off += ms * 4;
    for (int o = 0; o < a->ap.n_ops; o++)
      if (a->ap.ops[o].kind == OP_INC || a->ap.ops[o].kind == OP_INC_VALID) {
        s.plane_off[o] = off;
        s.plane_w64[o] = 0;
        off += ms * 4;
      }
    s.m_list_off = off;
    off += (mH * 2 + 15) & ~15;
    s.m_lds = off;
    for (int w = 0; w < 32; w++) s.word_op[w] = -1;
    for (int o = 0; o < a->ap.n_ops; o++) s.word_op[a->ap.ops[o].word] = (int8_t)o;
    if (mH >= 256) s.H_eff = std::min(s.H_eff, mH * 3 / 4);
  }
  // partitions: at most ~H_eff/2 groups each at the hinted size
  const int64_t groups = std::max<int64_t>(hint, 1024);
  s.hint_groups = groups;
  // at least 256 partitions: one merge workgroup per CU for small tables (C1's 40K groups in 64
  // partitions left three quarters of the CUs idle: k_part_merge_c1 28 -> 16 us at 256,
  // profiles/r06/ab/c1_partitions.txt); (the packed identity needs >= 64: window ranges up to 63)
  s.log2P = std::min(SPLIT_P_LOG2, std::max(8, part_ceil_log2(groups * 2 / s.H_eff)));
  // hinted groups would need sub-passes at 2^14 partitions (each re-reads the partition's
  // records): one more partition bit instead (measured: C5 push 12.1 → 9.8 ms)
  if (s.log2P == SPLIT_P_LOG2 && groups >> SPLIT_P_LOG2 > (int64_t)s.H_eff * 7 / 10) s.log2P = MAX_P_LOG2;
  s.log2P = (int)std::min<int64_t>(MAX_P_LOG2, knob("KHIP_PART_LOG2", s.log2P));
  s.P = 1LL << s.log2P;
  s.cmax = next_pow2(std::max<int64_t>(64, 2 * groups / s.P + 64));
  // more hinted groups per partition than one LDS table holds (P is capped by the LDS
  // histogram): start every partition with enough sub-passes instead of failing pass 0
  int s0 = 0;
  while (s0 < 12 && groups / s.P > ((int64_t)s.H_eff * 7 / 10) << s0) s0++;
  s.psbits.assign(s.P, (uint8_t)s0);
  // scattered record layout: key, ts, [meta], the value columns the update ops read
  bool colref[MAX_COLS] = {false};  // value read (SUM/MIN/MAX); COUNT(col) needs only validity
  s.vcols = 0;
  for (int o = 0; o < a->ap.n_ops; o++) {
    if (a->ap.ops[o].kind == OP_INC) continue;
    s.vcols |= 1u << a->ap.ops[o].col;
    if (a->ap.ops[o].kind != OP_INC_VALID) colref[a->ap.ops[o].col] = true;
  }
  const bool meta = a->desc.window_kind == KHIP_WINDOW_HOPPING || s.vcols != 0;
  s.meta_word = meta ? 2 : -1;
  int w = meta ? 3 : 2;
  for (int c = 0; c < MAX_COLS; c++) s.col_word[c] = (c < a->desc.n_cols && colref[c]) ? (int8_t)w++ : (int8_t)-1;
  s.rw = (w + 1) & ~1;
  KHIP_TRY(s.sel.ensure(s.P));
  KHIP_TRY(s.fail.ensure(s.P));
  KHIP_TRY(s.cnt.ensure(s.P * 8));
  KHIP_TRY(s.newcnt.ensure(s.P * 8));
  KHIP_TRY(s.pbase.ensure((s.P + 1) * 8));
  KHIP_TRY(s.R.ensure((s.P + 1) * 8));
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, a->device) == hipSuccess && ncu > 0)
      s.n_cu = ncu;
  }
  KHIP_TRY(s.ctr.ensure(128));
  KHIP_TRY(s.hcnt.ensure(s.P * 8));
  KHIP_TRY(s.hnew.ensure(s.P * 8));
  KHIP_TRY(s.pinfo.ensure(512));
  KHIP_TRY_HIP(hipMemsetAsync(s.hcnt.p, 0, s.P * 8, a->stream));
  KHIP_TRY_HIP(hipMemsetAsync(s.hnew.p, 0, s.P * 8, a->stream));
  KHIP_TRY_HIP(hipMemsetAsync(s.ctr.p, 0, 128, a->stream));
  s.having_total = 0;
  s.hvalid = true;
  for (int b = 0; b < 2; b++) KHIP_TRY(s.buf[b].ensure((size_t)s.P * s.cmax * a->sw * 8));
  if (a->changelog) KHIP_TRY(a->chg.ensure((size_t)s.P * s.cmax));
  KHIP_TRY_HIP(hipMemsetAsync(s.sel.p, 0, s.P, a->stream));
  KHIP_TRY_HIP(hipMemsetAsync(s.fail.p, 0, s.P, a->stream));
  KHIP_TRY_HIP(hipMemsetAsync(s.cnt.p, 0, s.P * 8, a->stream));
  KHIP_TRY_HIP(hipMemsetAsync(s.newcnt.p, 0, s.P * 8, a->stream));
  return KHIP_OK;
}

void part_release(khip_agg* a) {
  PartState& s = a->part;
  s.pinfo.release();
  s.c1vq_h.release();
  DevBuf* bufs[] = {&s.hcnt, &s.hnew, &s.srecA, &s.hcoarse, &s.scan_tmpB, &s.RB, &s.wr, &s.res, &s.closed, &s.closed_ctr, &s.closed2, &s.pctr, &s.buf[0], &s.buf[1], &s.sel, &s.cnt, &s.newcnt, &s.fail, &s.hist,
                    &s.tilemax, &s.tilemin, &s.tilekr,
                    &s.tileprefix, &s.tpart, &s.scan_tmp, &s.srec, &s.work,
                    &s.c1rc, &s.c1rp, &s.c1ro, &s.c1scan, &s.c1ci, &s.c1bb, &s.c1seg, &s.c1info, &s.prn, &s.c1vq,
                    &s.pbase, &s.R, &s.ctr, &s.counts};
  for (DevBuf* b : bufs) b->release();
}

// Empty every partition (one launch for all per-partition state, the counters and the stream time).
__global__ __launch_bounds__(256) void k_part_reset(int64_t P, unsigned long long* __restrict__ hcnt,
                                                    unsigned long long* __restrict__ hnew, int64_t* __restrict__ cnt,
                                                    unsigned long long* __restrict__ newcnt, uint8_t* __restrict__ fail,
                                                    unsigned long long* __restrict__ ctr,
                                                    int64_t* __restrict__ stream_time) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p < P) {
    hcnt[p] = 0;
    hnew[p] = 0;
    cnt[p] = 0;
    newcnt[p] = 0;
    fail[p] = 0;
  }
  if (p < 16) ctr[p] = 0;
  if (p == 0) *stream_time = -1;
}

khip_status part_reset(khip_agg* a) {
  PartState& s = a->part;
  s.closed_n = 0;
  s.purged_to = INT64_MIN;
  s.res_fresh = true;
  s.hvalid = true;
  s.having_total = 0;
  s.last_c1 = false;
  s.c1_skip = 0;  // (c1_wide, a prediction about the keys, stays)
  hipLaunchKernelGGL(k_part_reset, dim3(ceil_div(std::max<int64_t>(s.P, 16), 256)), dim3(256), 0, a->stream, s.P,
                     s.hcnt.as<unsigned long long>(), s.hnew.as<unsigned long long>(), s.cnt.as<int64_t>(),
                     s.newcnt.as<unsigned long long>(), s.fail.as<uint8_t>(), s.ctr.as<unsigned long long>(),
                     a->stream_time.as<int64_t>());
  KHIP_TRY_HIP(hipGetLastError());
  return KHIP_OK;
}

static PartAggParams part_params(khip_agg* a) {
  PartState& s = a->part;
  PartAggParams q{};
  q.windowed = a->windowed;
  q.nwords = s.nwords;
  q.sw = a->sw;
  q.H = s.H;
  q.H_eff = s.H_eff;
  q.rw = s.rw;
  q.meta_word = s.meta_word;
  for (int c = 0; c < MAX_COLS; c++) q.col_word[c] = s.col_word[c];
  q.size = a->desc.size_ms;
  q.adv = a->windowed ? a->desc.advance_ms : 1;
  q.fd = make_fastdiv((uint64_t)q.adv);
  q.dbg_mode = (int32_t)knob("KHIP_AGG_MODE", 0);
  q.log2P = s.log2P;
  q.cmax = s.cmax;
  q.n_cols = a->desc.n_cols;
  q.n_ops = a->ap.n_ops;
  for (int c = 0; c < MAX_COLS; c++) q.col_type[c] = a->ap.col_type[c];
  for (int o = 0; o < a->ap.n_ops; o++) q.ops[o] = a->ap.ops[o];
  q.init = a->init;
  q.having = a->having;
  q.flag_off = a->changelog ? s.flag_off : 0;
  q.chg = a->changelog ? a->chg.as<uint8_t>() : nullptr;
  return q;
}

khip_status part_regrow(khip_agg* a, int64_t ncmax) {
  PartState& s = a->part;
  DevBuf nb[2], nchg;
  for (int b = 0; b < 2; b++) KHIP_TRY(nb[b].ensure((size_t)s.P * ncmax * a->sw * 8));
  hipLaunchKernelGGL(k_part_regrow, dim3(s.P), dim3(256), 0, a->stream, s.buf[0].as<uint64_t>(),
                     s.buf[1].as<uint64_t>(), s.sel.as<uint8_t>(), s.cnt.as<int64_t>(), s.cmax, nb[0].as<uint64_t>(),
                     ncmax, a->sw);
  KHIP_TRY_HIP(hipGetLastError());
  if (a->changelog) {  // committed partitions keep this push's emission flags
    KHIP_TRY(nchg.ensure((size_t)s.P * ncmax));
    hipLaunchKernelGGL(k_part_regrow_flags, dim3(s.P), dim3(256), 0, a->stream, a->chg.as<uint8_t>(), s.cnt.as<int64_t>(),
                       s.cmax, nchg.as<uint8_t>(), ncmax);
    KHIP_TRY_HIP(hipGetLastError());
  }
  KHIP_TRY_HIP(hipMemsetAsync(s.sel.p, 0, s.P, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  for (int b = 0; b < 2; b++) {
    s.buf[b].release();
    s.buf[b] = std::move(nb[b]);
    nb[b].p = nullptr;
  }
  if (a->changelog) {
    a->chg.release();
    a->chg = std::move(nchg);
    nchg.p = nullptr;
  }
  s.cmax = ncmax;
  return KHIP_OK;
}

static khip_status part_split(khip_agg* a) {
  PartState& s = a->part;
  const int64_t P2 = s.P * 2;
  DevBuf nb[2], ncnt, nsel, nnew, nfail;
  KHIP_TRY(ncnt.ensure(P2 * 8));
  // 1. child row counts → region capacity for the new layout
  hipLaunchKernelGGL(k_part_split, dim3(s.P), dim3(256), 0, a->stream, s.buf[0].as<uint64_t>(), s.buf[1].as<uint64_t>(),
                     s.sel.as<uint8_t>(), s.cnt.as<int64_t>(), s.cmax, a->sw, s.log2P + 1, nullptr, (int64_t)0,
                     ncnt.as<int64_t>());
  std::vector<int64_t> hc(P2);
  KHIP_TRY_HIP(hipMemcpyAsync(hc.data(), ncnt.p, P2 * 8, hipMemcpyDeviceToHost, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  const int64_t mx = *std::max_element(hc.begin(), hc.end());
  const int64_t ncmax = next_pow2(std::max<int64_t>(64, mx * 3 / 2 + 64));
  // 2. move the rows
  for (int b = 0; b < 2; b++) KHIP_TRY(nb[b].ensure((size_t)P2 * ncmax * a->sw * 8));
  KHIP_TRY(nsel.ensure(P2));
  KHIP_TRY(nnew.ensure(P2 * 8));
  KHIP_TRY(nfail.ensure(P2));
  hipLaunchKernelGGL(k_part_split, dim3(s.P), dim3(256), 0, a->stream, s.buf[0].as<uint64_t>(), s.buf[1].as<uint64_t>(),
                     s.sel.as<uint8_t>(), s.cnt.as<int64_t>(), s.cmax, a->sw, s.log2P + 1, nb[0].as<uint64_t>(), ncmax,
                     ncnt.as<int64_t>());
  KHIP_TRY_HIP(hipGetLastError());
  KHIP_TRY_HIP(hipMemsetAsync(nsel.p, 0, P2, a->stream));
  KHIP_TRY_HIP(hipMemsetAsync(nnew.p, 0, P2 * 8, a->stream));
  KHIP_TRY_HIP(hipMemsetAsync(nfail.p, 0, P2, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  DevBuf* olds[] = {&s.buf[0], &s.buf[1], &s.cnt, &s.sel, &s.newcnt, &s.fail};
  DevBuf* news[] = {&nb[0], &nb[1], &ncnt, &nsel, &nnew, &nfail};
  for (int k = 0; k < 6; k++) {
    olds[k]->release();
    *olds[k] = std::move(*news[k]);
    news[k]->p = nullptr;
  }
  // a child holds about half of its parent's groups: one sub-pass bit fewer
  std::vector<uint8_t> nps(P2);
  for (int64_t c = 0; c < P2; c++) nps[c] = s.psbits[c >> 1] ? (uint8_t)(s.psbits[c >> 1] - 1) : 0;
  s.psbits.swap(nps);
  s.P = P2;
  s.log2P += 1;
  s.cmax = ncmax;
  if (a->changelog) {  // rewritten by the push that follows (untouched partitions are not read)
    a->chg.release();
    KHIP_TRY(a->chg.ensure((size_t)P2 * ncmax));
  }
  // per-partition HAVING counts do not survive the re-layout: the full scan serves HAVING
  // counts until the next reset
  KHIP_TRY(s.hcnt.ensure(P2 * 8));
  KHIP_TRY(s.hnew.ensure(P2 * 8));
  KHIP_TRY_HIP(hipMemsetAsync(s.hnew.p, 0, P2 * 8, a->stream));
  s.hvalid = false;
  KHIP_TRY(s.pbase.ensure((s.P + 1) * 8));
  KHIP_TRY(s.R.ensure((s.P + 1) * 8));
  return KHIP_OK;
}

static void agg_probe_report(DevBuf& b, int nb) {
  std::vector<unsigned long long> t((size_t)nb * 6 + 8);
  if (hipMemcpy(t.data(), b.p, t.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
  unsigned long long lo = ~0ULL, hi = 0;
  double ph[5] = {0, 0, 0, 0, 0};
  int m = 0;
  for (int i = 0; i < nb; i++) {
    const unsigned long long* r = &t[(size_t)i * 6];
    if (!r[0] || !r[5]) continue;
    m++;
    lo = std::min(lo, r[0]);
    hi = std::max(hi, r[5]);
    for (int k = 0; k < 5; k++) ph[k] += (double)(r[k + 1] - r[k]);
  }
  if (!m) return;
  fprintf(stderr, "[agg probe] %d/%d wgs, span %.1f us, avg per wg (us): phases %.2f %.2f %.2f %.2f %.2f "
          "(k_part_agg: init resident records write drain; k_part_merge: init records mark+reserve write drain)\n",
          m, nb, (hi - lo) / 100.0, ph[0] / m / 100, ph[1] / m / 100, ph[2] / m / 100, ph[3] / m / 100, ph[4] / m / 100);
}

// One push slice (n < 2^31).  tot[] receives the P_* counters.
// Shuffled rows (khip_agg_push_shuffled) through the value pipeline, read where they lie; *done =
// false when the pipeline does not apply or declined the push (the caller unpacks the rows and
// runs the general path, which then skips the pipeline as after any decline).
// supplied: KHIP_TIME_SUPPLIED, the rows carry their stream-time word (the scatter reads it there).
khip_status part_push_rows(khip_agg* a, int64_t n, const RowsIn& ri, int key_col, int64_t* tot, bool* done,
                           bool supplied) {
  PartState& s = a->part;
  *done = false;
  while (s.log2P < SPLIT_P_LOG2 && a->occ - s.closed_n > s.P * (int64_t)s.H_eff / 2) KHIP_TRY(part_split(a));
  s.last_c1 = false;
  int vcol = -1;
  if (s.c1_skip > 0 || !c1v_eligible(a, n, &vcol)) return KHIP_OK;
  RowsIn r = ri;
  r.vword = vcol == key_col ? 0 : 2 + vcol - (vcol > key_col ? 1 : 0);
  r.vbit = vcol;
  bool declined = false, retry_wide = false;
  // st_at only selects the stream-time scatter here (never read as a column: ROWS reads the word)
  const int64_t* st_flag = supplied ? (const int64_t*)ri.rows : nullptr;
  KHIP_TRY(c1_push(a, n, nullptr, nullptr, nullptr, nullptr, tot, &declined, st_flag, &retry_wide, nullptr, vcol, &r));
  if (a->profile) (declined ? a->times.c1_declined : a->times.c1_pushes)++;
  if (declined) s.c1_skip = 8;
  *done = !declined;
  return KHIP_OK;
}

khip_status part_push(khip_agg* a, int64_t n, const int64_t* keys, const int64_t* ts, const uint8_t* kv,
                      const uint8_t* rv, const ColPtrs& cols, int64_t* tot, const int64_t* st_at) {
  PartState& s = a->part;
  // keep the resident groups per partition well inside the LDS table (split = exact re-layout)
  // live groups only: closed (evicted) windows live in the flat store, not in the LDS tables
  while (s.log2P < SPLIT_P_LOG2 && a->occ - s.closed_n > s.P * (int64_t)s.H_eff / 2) KHIP_TRY(part_split(a));
  // the windowed COUNT(*) pipeline (khip_agg_c1.hip) when it applies; a push it declines (a tile
  // that may hold late records, a ts span or key range too wide) runs the general path below, and
  // the next few pushes go straight there
  s.last_c1 = false;
  int vcol = -1;
  if (s.c1_skip > 0) {
    s.c1_skip--;
  } else if (c1_eligible(a, n) || c1v_eligible(a, n, &vcol)) {
    // COUNT(*) alone: 8-byte records; one argument column: 16-byte value records
    const ColPtrs* vc = vcol >= 0 ? &cols : nullptr;
    bool declined = false, retry_wide = false;
    KHIP_TRY(c1_push(a, n, keys, ts, kv, rv, tot, &declined, st_at, &retry_wide, vc, vcol));
    if (declined && retry_wide)  // the keys needed the wide records: this push again with them
      KHIP_TRY(c1_push(a, n, keys, ts, kv, rv, tot, &declined, st_at, &retry_wide, vc, vcol));
    if (a->profile) (declined ? a->times.c1_declined : a->times.c1_pushes)++;
    if (!declined) return KHIP_OK;
    s.c1_skip = 8;
  }
  const int P = (int)s.P;
  // records per thread per tile: PT_ITEMS, fewer when that leaves fewer tiles than CUs (one
  // workgroup per tile: C1's 1M records were 16 tiles on 256 CUs — k_part_scatter_r8 87 -> 11 us and
  // k_part_hist 39 -> 14 us at 4 items, profiles/r06/ab/c1_tile_items.txt) and the per-tile
  // partition counts stay small (nT x P words, which the offset scans read)
  int64_t items = PT_ITEMS;
  while (items > 4 && ceil_div(n, (int64_t)PT_THREADS * items) < s.n_cu &&
         ceil_div(n, (int64_t)PT_THREADS * (items >> 1)) * s.P <= (1LL << 21))
    items >>= 1;
  const int64_t tile = (int64_t)PT_THREADS * knob("KHIP_TILE_ITEMS", items);
  const int pad = (int)knob("KHIP_PAD", 0);
  const int64_t nT = ceil_div(n, tile);
  const int TC = (int)std::min<int64_t>(nT, TC_MAX);
  KHIP_TRY(s.hist.ensure((size_t)nT * P * 4));
  KHIP_TRY(s.tilemax.ensure(nT * 8));
  KHIP_TRY(s.tilemin.ensure(nT * 8));
  KHIP_TRY(s.tilekr.ensure(nT * 16));
  KHIP_TRY(s.tileprefix.ensure(nT * 8));
  KHIP_TRY(s.tpart.ensure(nT * 8 * T_NPART));
  KHIP_TRY(s.scan_tmp.ensure((size_t)TC * P * 8));
  const int64_t ncap = pad ? n + 3 * (int64_t)P * nT : n;  // padded runs
  // two-level scatter (pass A: B = P >> fbits buckets; pass B: partitions inside a bucket)
  // once single-level runs get short (P large against the tile)
  const bool lvl2 = !pad && s.log2P >= 11 && knob("KHIP_SCATTER2", 1) != 0;
  const int fbits = lvl2 ? s.log2P - s.log2P / 2 : 0;
  const int B = P >> fbits;
  if (s.scat_cap < ncap) {
    const int64_t n = ncap;
    KHIP_TRY(s.srec.ensure((size_t)(n + 1) * s.rw * 8));  // AoS records (+1: dummy store target)
    s.scat_cap = ncap;
  }
  if (lvl2) {
    KHIP_TRY(s.srecA.ensure((size_t)(n + 1) * s.rw * 8));
    KHIP_TRY(s.hcoarse.ensure((size_t)nT * B * 4));
    KHIP_TRY(s.scan_tmpB.ensure((size_t)TC * B * 8));
    KHIP_TRY(s.RB.ensure((size_t)(B + 1) * 8));
  }
  ColTypes ct{};
  for (int c = 0; c < MAX_COLS; c++) ct.t[c] = a->ap.col_type[c];
  RecLayout L{};
  L.rw = s.rw;
  L.meta_word = s.meta_word;
  L.vcols = s.vcols;
  for (int w = 0; w < (int)sizeof(L.word_col); w++) L.word_col[w] = -1;
  for (int c = 0; c < MAX_COLS; c++) {
    L.col_word[c] = s.col_word[c];
    if (s.col_word[c] >= 0) L.word_col[s.col_word[c]] = (int8_t)c;
  }
  const size_t hist_lds = (size_t)P * 4;
  if (hist_lds > 64 * 1024)
    hipFuncSetAttribute((const void*)k_part_hist, hipFuncAttributeMaxDynamicSharedMemorySize, (int)hist_lds);
  // 1. histogram + tile stream-time maxima
  ev_record_part(a, 0);
  hipLaunchKernelGGL(k_part_hist, dim3(nT), dim3(PT_THREADS), hist_lds, a->stream, keys, ts, kv, rv, n, tile, s.log2P,
                     pad, nT,
                     s.hist.as<uint32_t>(), s.tilemax.as<int64_t>(), s.tilemin.as<int64_t>(), s.tpart.as<int64_t>(),
                     fbits, lvl2 ? s.hcoarse.as<uint32_t>() : (uint32_t*)nullptr, s.tilekr.as<int64_t>(), st_at);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, a->stream, s.tilemax.as<int64_t>(), nT,
                     s.tileprefix.as<int64_t>(), a->stream_time.as<int64_t>());
  // window range of the push (packed identity) and its event-time span → host: they pick the
  // aggregate kernel (k_part_merge needs the identity and a span below 2^31 ms)
  const PartAggParams q0 = part_params(a);
  const int64_t close0 = (a->windowed && a->host_stream_time >= 0) ? a->host_stream_time - a->grace : INT64_MIN;
  KHIP_TRY(s.wr.ensure(128));
  KHIP_TRY(s.res.ensure(16));
  KHIP_TRY(s.closed_ctr.ensure(8));
  const bool merge_allow = s.mH >= 256 && knob("KHIP_MERGE", 1) != 0;
  // which merge kernel pass 0 runs (host-known): the lean COUNT(*) merge reads R8 records too
  const bool narrow = s.rw == 2;
  const int64_t r12_mode = knob("KHIP_R12", 1);  // 1: 12-byte records end to end; 2: pass A only
  const bool r12_ok = narrow && !pad && merge_allow && r12_mode != 0;
  const bool r12_merge = r12_ok && (r12_mode == 1 || !lvl2);  // what k_part_merge reads
  // COUNT(*) alone: row = [key, ws, rowtime, count] (sw 4), one u32 delta plane
  // and (key hash, ts) records with one window each (TUMBLING or no window: no meta word)
  const bool cnt1 = a->ap.n_ops == 1 && a->ap.ops[0].kind == OP_INC && a->ap.ops[0].word == 3 && a->sw == 4 &&
                    s.rw == 2 && a->desc.window_kind != KHIP_WINDOW_HOPPING;
  const int mt = (int)knob("KHIP_MERGE_THREADS", 512);
  const bool c1_plan = cnt1 && r12_merge && a->windowed && q0.adv <= (int64_t)1 << 31 && mt >= 512 &&
                       knob("KHIP_MERGE_C1", 1) != 0;
  const bool r8_allow = c1_plan && knob("KHIP_R8", 1) != 0;
  hipLaunchKernelGGL(k_part_wrange, dim3(1), dim3(1024), 0, a->stream, s.tilemin.as<int64_t>(), s.tilemax.as<int64_t>(),
                     nT, a->windowed, a->desc.size_ms, q0.adv, q0.fd, close0, s.log2P, s.res_fresh ? 1 : 0,
                     (a->desc.flags & KHIP_FLAG_PART_CLAIM) ? 0 : 1, merge_allow ? 1 : 0, s.res.as<int64_t>(),
                     s.wr.as<int64_t>(), s.ctr.as<unsigned long long>(),
                     a->windowed ? s.closed_ctr.as<unsigned long long>() : (unsigned long long*)nullptr,
                     (unsigned long long)s.closed_n, s.tilekr.as<int64_t>(), r8_allow ? 1 : 0);
  s.res_fresh = false;
  int64_t* pin = s.pinfo.as<int64_t>();  // wr[0..6), read after the pass-0 sync
  KHIP_TRY_HIP(hipMemcpyAsync(pin, s.wr.p, 48, hipMemcpyDeviceToHost, a->stream));
  // 2. offsets
  hipLaunchKernelGGL(k_part_colsum, dim3(ceil_div(P, 256), TC), dim3(256), 0, a->stream, s.hist.as<uint32_t>(), nT, P,
                     TC, s.scan_tmp.as<int64_t>());
  hipLaunchKernelGGL(k_part_colbase, dim3(ceil_div(P, 256)), dim3(256), 0, a->stream, s.scan_tmp.as<int64_t>(), P, TC,
                     s.pbase.as<int64_t>());
  hipLaunchKernelGGL(k_part_pscan, dim3(1), dim3(1024), 0, a->stream, s.pbase.as<int64_t>(), (int64_t)P);
  hipLaunchKernelGGL(k_part_colprefix, dim3(ceil_div(P, 256), TC), dim3(256), 0, a->stream, s.hist.as<uint32_t>(), nT,
                     P, TC, s.scan_tmp.as<int64_t>(), s.pbase.as<int64_t>(), 1);
  if (lvl2) {  // bucket b's region = its partitions' regions [pbase[b << fbits], pbase[(b + 1) << fbits])
    hipLaunchKernelGGL(k_part_colsum, dim3(ceil_div(B, 256), TC), dim3(256), 0, a->stream, s.hcoarse.as<uint32_t>(), nT,
                       B, TC, s.scan_tmpB.as<int64_t>());
    hipLaunchKernelGGL(k_part_colbase, dim3(ceil_div(B, 256)), dim3(256), 0, a->stream, s.scan_tmpB.as<int64_t>(), B, TC,
                       s.RB.as<int64_t>());
    hipLaunchKernelGGL(k_part_colprefix, dim3(ceil_div(B, 256), TC), dim3(256), 0, a->stream, s.hcoarse.as<uint32_t>(),
                       nT, B, TC, s.scan_tmpB.as<int64_t>(), s.pbase.as<int64_t>(), 1 << fbits);
  }
  ev_record_part(a, 1);
  // 3. scatter (12-byte records for k_part_merge when the layout is narrow: r12_ok, decided
  //    on the device by wr[4])
  const int U = (int)knob("KHIP_SCATTER_U", narrow ? 8 : 16);
  auto scat = narrow ? (U >= 16 ? k_part_scatter<16, true> : (U >= 8 ? k_part_scatter<8, true> : (U >= 6 ? k_part_scatter<6, true> : k_part_scatter<4, true>)))
                     : (U >= 16 ? k_part_scatter<16, false> : (U >= 8 ? k_part_scatter<8, false> : k_part_scatter<4, false>));
  // narrow records leave through the LDS stage (stage_step): bins = B buckets (two-level) or P
  const int nbins = lvl2 ? B : P;
  const int Ut = U >= 16 ? 16 : (U >= 8 ? 8 : (narrow && U >= 6 ? 6 : 4));  // the instantiated records per thread per step
  const bool stage = narrow && !pad && nbins <= PT_THREADS && Ut <= 8 && knob("KHIP_STAGE", 1) != 0;
  // 32-byte records (key hash, ts, meta / value words) through the LDS stage too (2 x 1024 per step)
  const bool wstage = !narrow && s.rw == 4 && !pad && nbins <= PT_THREADS && knob("KHIP_WSTAGE", 1) != 0;
  const int wu = Ut >= 16 ? 4 : 2;  // k_part_scatter's WU: staged 32-byte records per thread per step
  // R8 records (decided on the device) through k_part_scatter_r8 / k_part_refine_r8
  const bool r8k = r8_allow && stage && Ut == 8 && nbins <= R8_NT && (!lvl2 || (1 << fbits) <= R8_NT) &&
                   knob("KHIP_R8K", 1) != 0;
  // 32-byte records through k_part_scatter_w (host-known)
  const bool wk = wstage && nbins <= W_NT && knob("KHIP_WK", 1) != 0;
  const size_t scat_lds = stage ? stage_lds_bytes(nbins, Ut * PT_THREADS / 2)
                                : (wstage ? stage_lds_bytes(nbins, 2 * wu * PT_THREADS)
                                          : (lvl2 ? (size_t)B * 4 : hist_lds));
  if (scat_lds > 64 * 1024)
    hipFuncSetAttribute((const void*)scat, hipFuncAttributeMaxDynamicSharedMemorySize, (int)scat_lds);
  hipLaunchKernelGGL(scat, dim3(nT), dim3(PT_THREADS), scat_lds, a->stream, keys, ts, kv, rv,
                     cols, a->desc.n_cols, ct, n, tile, s.log2P - fbits, pad, nT,
                     lvl2 ? s.hcoarse.as<uint32_t>() : s.hist.as<uint32_t>(), s.pbase.as<int64_t>(),
                     s.tileprefix.as<int64_t>(),
                     s.tilemax.as<int64_t>(), s.tilemin.as<int64_t>(), a->windowed, a->desc.size_ms,
                     a->windowed ? a->desc.advance_ms : 1, make_fastdiv(a->windowed ? a->desc.advance_ms : 1),
                     a->grace, L, lvl2 ? s.srecA.as<uint64_t>() : s.srec.as<uint64_t>(), ncap,
                     s.tpart.as<int64_t>(), s.wr.as<int64_t>(), r12_ok ? 1 : 0, (stage || wstage) ? 1 : 0,
                     (r8k || wk) ? 1 : 0, st_at);
  KHIP_TRY_HIP(hipGetLastError());
  if (wk) {  // the wide staged tiles
    auto sw_ = wu >= 4 ? k_part_scatter_w<4, W_NT> : k_part_scatter_w<2, W_NT>;
    const size_t sw_lds = stage_lds_bytes(nbins, 2 * wu * W_NT);
    if (sw_lds > 64 * 1024) hipFuncSetAttribute((const void*)sw_, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sw_lds);
    hipLaunchKernelGGL(sw_, dim3(nT), dim3(W_NT), sw_lds, a->stream, keys, ts, kv, rv, cols, a->desc.n_cols, ct, n, tile,
                       s.log2P - fbits, nT, lvl2 ? s.hcoarse.as<uint32_t>() : s.hist.as<uint32_t>(),
                       s.tileprefix.as<int64_t>(), s.tilemax.as<int64_t>(), s.tilemin.as<int64_t>(), a->windowed,
                       a->desc.size_ms, a->windowed ? a->desc.advance_ms : 1,
                       make_fastdiv(a->windowed ? a->desc.advance_ms : 1), a->grace, L,
                       lvl2 ? s.srecA.as<uint64_t>() : s.srec.as<uint64_t>(), s.tpart.as<int64_t>());
    KHIP_TRY_HIP(hipGetLastError());
  }
  const int r8u = knob("KHIP_R8_U", 8) >= 8 ? 8 : 4;  // R8 records per thread per staged step
  if (r8k) {  // the R8 tiles (exits at once unless k_part_wrange chose R8)
    auto s8 = r8u == 8 ? k_part_scatter_r8<8, R8_NT> : k_part_scatter_r8<4, R8_NT>;
    const size_t s8_lds = stage_r8_lds_bytes(nbins, r8u * R8_NT);
    if (s8_lds > 64 * 1024) hipFuncSetAttribute((const void*)s8, hipFuncAttributeMaxDynamicSharedMemorySize, (int)s8_lds);
    hipLaunchKernelGGL(s8, dim3(nT), dim3(R8_NT), s8_lds, a->stream, keys, ts, kv, rv, n, tile, s.log2P - fbits, nT,
                       lvl2 ? s.hcoarse.as<uint32_t>() : s.hist.as<uint32_t>(), s.tileprefix.as<int64_t>(),
                       s.tilemax.as<int64_t>(), s.tilemin.as<int64_t>(), a->windowed, a->desc.size_ms,
                       a->windowed ? a->desc.advance_ms : 1, make_fastdiv(a->windowed ? a->desc.advance_ms : 1),
                       a->grace, lvl2 ? s.srecA.as<uint64_t>() : s.srec.as<uint64_t>(), s.tpart.as<int64_t>(),
                       s.wr.as<int64_t>());
    KHIP_TRY_HIP(hipGetLastError());
  }
  if (lvl2) {
    const int64_t per_blk = knob("KHIP_REFINE_RECS", 8192);  // measured: 8K records per block (1 KB runs) beat 32K
    const int G = (int)std::max<int64_t>(1, std::min<int64_t>(nT, per_blk * B / tile));
    const int64_t ng = ceil_div(nT, G);
    void (*ref)(const uint64_t*, const uint32_t*, const uint32_t*, const int64_t*, int64_t, int, int, int, int64_t,
                uint64_t*, int, const int64_t*, int, int, int);
    switch (s.rw) {
      case 2: ref = k_part_refine<2>; break;
      case 4: ref = k_part_refine<4>; break;
      case 6: ref = k_part_refine<6>; break;
      case 8: ref = k_part_refine<8>; break;
      case 10: ref = k_part_refine<10>; break;
      default: ref = k_part_refine<12>; break;
    }
    const bool rstage = s.rw == 2 && (1 << fbits) <= PT_THREADS && knob("KHIP_STAGE", 1) != 0;
    const bool rwstage = s.rw == 4 && (1 << fbits) <= PT_THREADS && knob("KHIP_WSTAGE", 1) != 0;
    const int ru = rwstage ? (knob("KHIP_REFINE_WU", 4) >= 4 ? 4 : 2)  // 32-byte records per thread per step
                           : (knob("KHIP_REFINE_U", 8) >= 8 ? 8 : 4);   // records per thread per staged step
    const size_t ref_lds = rstage ? stage_lds_bytes(1 << fbits, ru * PT_THREADS / 2)
                                  : (rwstage ? stage_lds_bytes(1 << fbits, 2 * ru * PT_THREADS) : 0);
    if (ref_lds) hipFuncSetAttribute((const void*)ref, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ref_lds);
    const int64_t ref_grid = (r8k && rstage) ? std::min<int64_t>(B * ng, 2 * s.n_cu) : B * ng;
    hipLaunchKernelGGL(ref, dim3((unsigned)ref_grid), dim3(PT_THREADS), ref_lds, a->stream, s.srecA.as<uint64_t>(),
                       s.hcoarse.as<uint32_t>(), s.hist.as<uint32_t>(), s.pbase.as<int64_t>(), nT, G, s.log2P, fbits,
                       ncap, s.srec.as<uint64_t>(), (int)knob("KHIP_REFINE_MODE", 0), s.wr.as<int64_t>(),
                       r12_ok ? (r12_merge ? 1 : 2) : 0, (rstage || rwstage) ? ru : 0, (r8k && rstage) ? 1 : 0);
    KHIP_TRY_HIP(hipGetLastError());
    if (r8k && rstage) {
      auto r8 = r8u == 8 ? k_part_refine_r8<8, R8_NT> : k_part_refine_r8<4, R8_NT>;
      const size_t r8_lds = stage_r8_lds_bytes(1 << fbits, r8u * R8_NT);
      if (r8_lds > 64 * 1024) hipFuncSetAttribute((const void*)r8, hipFuncAttributeMaxDynamicSharedMemorySize, (int)r8_lds);
      hipLaunchKernelGGL(r8, dim3((unsigned)(B * ng)), dim3(R8_NT), r8_lds, a->stream, s.srecA.as<uint64_t>(),
                         s.hcoarse.as<uint32_t>(), s.hist.as<uint32_t>(), s.pbase.as<int64_t>(), nT, G, s.log2P, fbits,
                         s.srec.as<uint64_t>(), s.wr.as<int64_t>());
      KHIP_TRY_HIP(hipGetLastError());
    }
  }
  ev_record_part(a, 2);
  // 4. aggregate partitions (+ retries).  k_part_merge is launched speculatively (it and its
  //    commit exit when k_part_wrange declined it); pass 0 is then redone with k_part_agg.
  bool merge = merge_allow;
  MergeParams mq{};
  if (merge) {
    mq.windowed = a->windowed;
    mq.sw = a->sw;
    mq.nwords = s.nwords;
    mq.H = s.mH;
    mq.rw = s.rw;
    mq.meta_word = s.meta_word;
    mq.log2P = s.log2P;
    mq.n_ops = a->ap.n_ops;
    mq.size = q0.size;
    mq.adv = q0.adv;
    mq.fd = q0.fd;
    mq.div32 = a->windowed && q0.adv <= (int64_t)1 << 31 ? 1 : 0;
    mq.fd32 = make_fastdiv32((uint32_t)(mq.div32 ? q0.adv : 1));
    for (int c = 0; c < MAX_COLS; c++) {
      mq.col_word[c] = s.col_word[c];
      mq.col_type[c] = a->ap.col_type[c];
    }
    for (int o = 0; o < a->ap.n_ops; o++) {
      mq.ops[o] = a->ap.ops[o];
      mq.plane_off[o] = s.plane_off[o];
      mq.plane_w64[o] = s.plane_w64[o];
    }
    mq.rt_off = s.rt_off;
    mq.list_off = s.m_list_off;
    mq.fan = a->windowed ? (int32_t)std::min<int64_t>((q0.size + q0.adv - 1) / q0.adv, 1 << 20) : 1;
    mq.pane = a->windowed && mq.fan > 1 && mq.fan <= MG_FB && q0.size % q0.adv == 0 && knob("KHIP_PANES", 1) ? 1 : 0;
    mq.lds_bytes = s.m_lds;
    mq.init = a->init;
    mq.having = a->having;
    mq.dbg = (int32_t)knob("KHIP_MERGE_DEBUG", 0);
    mq.r12 = r12_merge ? 1 : 0;
    mq.chg = a->changelog ? a->chg.as<uint8_t>() : nullptr;
  }
  if (a->windowed) {  // worst case every live row closes in this push
    const int64_t live = a->occ - s.closed_n;
    if (s.closed_cap < s.closed_n + live) {
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
  }
  int64_t added_total = 0;
  std::vector<uint8_t> host_fail;
  std::vector<int> sbits(s.psbits.begin(), s.psbits.end());
  std::vector<uint32_t> plist, work;
  // pass 0: one work item per partition, or its learned 2^sbits sub-passes
  bool subs0 = false;
  for (int p = 0; p < P && !subs0; p++) subs0 = sbits[p] > 0;
  if (subs0) {
    for (int p = 0; p < P; p++)
      for (int k = 0; k < (1 << sbits[p]); k++) work.push_back((uint32_t)p | ((uint32_t)sbits[p] << 16) | ((uint32_t)k << 20));
    KHIP_TRY(s.work.ensure(work.size() * 4));
    KHIP_TRY_HIP(hipMemcpyAsync(s.work.p, work.data(), work.size() * 4, hipMemcpyHostToDevice, a->stream));
  }
  // KHIP_AGG_PROBE=1: per-workgroup phase timestamps of pass 0 (wall clock, 100 MHz) → stderr
  const bool probe = knob("KHIP_AGG_PROBE", 0) != 0;
  DevBuf dbgbuf;
  unsigned long long* dbg = nullptr;
  bool c1_ran = false;
  for (int pass = 0;; pass++) {
    PartAggParams q = q0;
    dbg = nullptr;
    if (probe && pass == 0) {
      KHIP_TRY(dbgbuf.ensure((size_t)std::max<int64_t>(P, (int64_t)work.size()) * 6 * 8 + 64));
      KHIP_TRY_HIP(hipMemsetAsync(dbgbuf.p, 0, dbgbuf.bytes, a->stream));
      dbg = dbgbuf.as<unsigned long long>();
    }
    q.cmax = s.cmax;
    mq.cmax = s.cmax;
    q.chg = mq.chg = a->changelog ? a->chg.as<uint8_t>() : nullptr;  // a retry's regrow moves them
    if (pass > 0) KHIP_TRY_HIP(hipMemsetAsync(s.ctr.p, 0, 24, a->stream));  // pass 0: k_part_wrange
    const uint32_t* wk = (pass == 0 && !subs0) ? nullptr : s.work.as<uint32_t>();
    const int64_t nwork = (pass == 0 && !subs0) ? P : (int64_t)work.size();
    if (merge) {
      const int c1h = (int)knob("KHIP_C1_LOG2H", 12);
      c1_ran = c1_plan;
      if (c1_ran) {  // the lean COUNT(*) merge
        const int au = (int)knob("KHIP_C1_AU", 6);
        const int lds = ((1 << c1h) + 64) * 16;
        // both record layouts' instantiations (R8 only when k_part_wrange may choose it)
        for (int rm = r8_allow ? 1 : 0; rm >= 0; rm--) {
        auto mk = rm ? (au >= 8 ? k_part_merge_c1<512, 8, 1> : (au >= 6 ? k_part_merge_c1<512, 6, 1> : k_part_merge_c1<512, 4, 1>))
                     : (au >= 8 ? k_part_merge_c1<512, 8, 0> : (au >= 6 ? k_part_merge_c1<512, 6, 0> : k_part_merge_c1<512, 4, 0>));
        hipFuncSetAttribute((const void*)mk, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        const int64_t grid = std::min<int64_t>(nwork, (int64_t)s.n_cu * knob("KHIP_MERGE_WG_PER_CU", 2));
        C1Params cq{};
        cq.log2P = mq.log2P;
        cq.log2H = c1h;
        cq.sw = mq.sw;
        cq.size = mq.size;
        cq.adv = mq.adv;
        cq.cmax = mq.cmax;
        cq.fd = mq.fd;
        cq.fd32 = mq.fd32;
        cq.chg = mq.chg;
        cq.hv_active = a->having.active;
        cq.hv_op = a->having.op;
        cq.hv_i64 = a->having.i64;
        hipLaunchKernelGGL(mk, dim3(grid), dim3(512), lds, a->stream, cq, wk, nwork, s.pbase.as<int64_t>(),
                           s.srec.as<uint64_t>(), pass == 0 ? 1 : 0, s.buf[0].as<uint64_t>(), s.buf[1].as<uint64_t>(),
                           s.sel.as<uint8_t>(), s.cnt.as<int64_t>(), s.newcnt.as<unsigned long long>(),
                           s.fail.as<uint8_t>(), s.ctr.as<unsigned long long>() + 2, close0, s.closed.as<uint64_t>(),
                           s.closed_ctr.as<unsigned long long>(), s.wr.as<int64_t>(),
                           s.hnew.as<unsigned long long>(), s.ctr.as<unsigned long long>() + 12, dbg);
        }
      } else {
      auto mk = mq.r12 ? (mt >= 512 ? (cnt1 ? k_part_merge<true, 512, true> : k_part_merge<false, 512, true>)
                                    : (cnt1 ? k_part_merge<true, 256, true> : k_part_merge<false, 256, true>))
                       : (mt >= 512 ? (cnt1 ? k_part_merge<true, 512, false> : k_part_merge<false, 512, false>)
                                    : (cnt1 ? k_part_merge<true, 256, false> : k_part_merge<false, 256, false>));
      hipFuncSetAttribute((const void*)mk, hipFuncAttributeMaxDynamicSharedMemorySize, s.m_lds);
      const int64_t grid = std::min<int64_t>(nwork, (int64_t)s.n_cu * knob("KHIP_MERGE_WG_PER_CU", mt >= 512 ? KHIP_MG_WPE / 2 : KHIP_MG_WPE));
      hipLaunchKernelGGL(mk, dim3(grid), dim3(mt >= 512 ? 512 : 256), s.m_lds, a->stream, mq, wk, nwork, s.pbase.as<int64_t>(),
                         s.srec.as<uint64_t>(), pass == 0 ? 1 : 0, s.buf[0].as<uint64_t>(), s.buf[1].as<uint64_t>(),
                         s.sel.as<uint8_t>(), s.cnt.as<int64_t>(), s.newcnt.as<unsigned long long>(),
                         s.fail.as<uint8_t>(), s.ctr.as<unsigned long long>() + 2, close0, s.closed.as<uint64_t>(),
                         s.closed_ctr.as<unsigned long long>(), s.wr.as<int64_t>(),
                         s.hnew.as<unsigned long long>(), s.ctr.as<unsigned long long>() + 12, dbg);
      }
    } else {
      hipFuncSetAttribute((const void*)k_part_agg, hipFuncAttributeMaxDynamicSharedMemorySize, s.lds_bytes);
      hipLaunchKernelGGL(k_part_agg, dim3(nwork), dim3(AG_THREADS), s.lds_bytes, a->stream, q, wk,
                         s.pbase.as<int64_t>(), s.srec.as<uint64_t>(), pass == 0 ? 1 : 0, s.buf[0].as<uint64_t>(),
                         s.buf[1].as<uint64_t>(), s.sel.as<uint8_t>(), s.cnt.as<int64_t>(),
                         s.newcnt.as<unsigned long long>(), s.fail.as<uint8_t>(),
                         s.ctr.as<unsigned long long>() + 2, close0, s.closed.as<uint64_t>(),
                         s.closed_ctr.as<unsigned long long>(), s.wr.as<int64_t>(), dbg);
    }
    const int nl = pass == 0 ? P : (int)plist.size();
    hipLaunchKernelGGL(k_part_commit, dim3(ceil_div(std::max(nl, 1), 256)), dim3(256), 0, a->stream,
                       (merge && pass == 0) ? s.wr.as<int64_t>() : (const int64_t*)nullptr, P,
                       s.pbase.as<int64_t>(), (const uint32_t*)nullptr,
                       pass == 0 ? nullptr : s.work.as<uint32_t>() + work.size(), nl,
                       s.sel.as<uint8_t>(), s.cnt.as<int64_t>(), s.newcnt.as<unsigned long long>(),
                       s.fail.as<uint8_t>(), s.ctr.as<unsigned long long>(), s.hcnt.as<unsigned long long>(),
                       s.hnew.as<unsigned long long>());
    KHIP_TRY_HIP(hipGetLastError());
    if (pass == 0) {
      ev_record_part(a, 3);
      hipLaunchKernelGGL(k_part_stats, dim3(1), dim3(256), 0, a->stream, s.tpart.as<int64_t>(), nT,
                         a->windowed ? s.closed_ctr.as<unsigned long long>() : (unsigned long long*)nullptr,
                         a->stream_time.as<int64_t>(), s.ctr.as<unsigned long long>());
    }
    unsigned long long* c2 = s.pinfo.as<unsigned long long>() + 8;
    KHIP_TRY_HIP(hipMemcpyAsync(c2, s.ctr.p, 13 * 8, hipMemcpyDeviceToHost, a->stream));
    KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
    if (pass == 0 && merge && pin[4] == 0) {  // declined on the device: nothing was written
      merge = false;
      s.hvalid = false;  // k_part_agg does not maintain the HAVING counts
      pass = -1;
      continue;
    }
    added_total += (int64_t)c2[0];
    if (dbg && merge) {  // k_part_merge: per-phase time summed over its persistent workgroups
      unsigned long long ph[8] = {};
      if (hipMemcpy(ph, dbgbuf.p, sizeof(ph), hipMemcpyDeviceToHost) == hipSuccess) {
        const double g = (double)std::min<int64_t>(P, 2 * s.n_cu) * 100.0;  // 100 MHz ticks → us per workgroup
        if (c1_ran)
          fprintf(stderr, "[merge c1 probe] per workgroup (us): item start+evict %.1f records %.1f mark+count+reserve %.1f "
                  "write %.1f\n", ph[0] / g, ph[1] / g, ph[2] / g, ph[3] / g);
        else
          fprintf(stderr, "[merge probe] per workgroup (us): setup %.1f evict %.1f records %.1f mark+reserve %.1f write %.1f\n",
                  ph[0] / g, ph[1] / g, ph[2] / g, ph[3] / g, ph[4] / g);
      }
    } else if (dbg) {
      agg_probe_report(dbgbuf, (int)((pass == 0 && !subs0) ? P : (int64_t)work.size()));
    }
    if (c2[1] == 0) break;
    if (pass > 24) return fail(KHIP_E_DEVICE, "partitioned aggregation could not place the batch");
    // retry the failed partitions: LDS overflow → twice the sub-passes; region overflow → grow
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
    // grow straight to what the largest overflowing partition needed (sub-passes of one
    // partition append to the same region, so its full row count is at least `need`)
    if (grow) KHIP_TRY(part_regrow(a, next_pow2(std::max<int64_t>(s.cmax * 2, (int64_t)c2[2] * 5 / 4 + 64))));
    std::vector<uint32_t> both(work);
    both.insert(both.end(), plist.begin(), plist.end());
    KHIP_TRY(s.work.ensure(both.size() * 4));
    KHIP_TRY_HIP(hipMemcpyAsync(s.work.p, both.data(), both.size() * 4, hipMemcpyHostToDevice, a->stream));
  }
  for (int p = 0; p < P; p++) s.psbits[p] = (uint8_t)std::max<int>(s.psbits[p], sbits[p]);
  if (!merge) s.hvalid = false;
  {
    const unsigned long long* hc = s.pinfo.as<unsigned long long>() + 8;
    s.having_total = (int64_t)(hc[11] + hc[12]);  // live rows + closed rows passing HAVING
  }
  // 5. counters (k_part_stats after pass 0: evictions only happen there)
  const unsigned long long* st = s.pinfo.as<unsigned long long>() + 8;
  if (a->windowed) {
    const int64_t cn = (int64_t)st[3 + T_NPART];
    added_total += cn - s.closed_n;  // evicted rows left the live regions but are still groups
    s.closed_n = cn;
  }
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

// The query's HAVING row count from the counts k_part_merge / k_part_commit maintain on the
// device (copied back with every push's counters): no kernel, no table scan.  Returns false
// when they are not valid (a push took a path that does not keep them): the caller then scans.
bool part_having_count(khip_agg* a, int64_t* n) {
  PartState& s = a->part;
  if (!s.hvalid || !a->having.active) return false;
  *n = s.having_total;
  return true;
}

// Rows passing `h` (all partitions) → rows (sw words each), or just the count.
khip_status part_compact(khip_agg* a, const HavingDev& h_in, std::vector<uint64_t>* rows, int64_t* count) {
  PartState& s = a->part;
  HavingDev h = h_in;
  h.log2P = s.log2P;
  // more query keys than one block checks at once: group them by partition on the host so
  // every k_part_rows block reads only its own keys (and partitions without keys exit)
  DevBuf pk, pko;
  std::vector<int64_t> hpk, hpko;
  if (h.pull && h.n_keys > 256 && h.host_keys) {
    const int64_t nk = h.n_keys;
    const int P = (int)s.P;
    std::vector<std::pair<uint32_t, int64_t>> kp((size_t)nk);
    for (int64_t i = 0; i < nk; i++) {
      const int64_t key = h.host_keys[i];
      const uint64_t hk = mix64((uint64_t)key ^ 0x6A09E667F3BCC908ULL);  // key_hash
      kp[(size_t)i] = {s.log2P == 0 ? 0u : (uint32_t)(hk >> (64 - s.log2P)), key};
    }
    std::sort(kp.begin(), kp.end());
    hpk.resize((size_t)nk);
    hpko.assign((size_t)P + 1, 0);
    for (int64_t i = 0; i < nk; i++) {
      hpk[(size_t)i] = kp[(size_t)i].second;
      hpko[kp[(size_t)i].first + 1]++;
    }
    for (int q = 0; q < P; q++) hpko[q + 1] += hpko[q];
    KHIP_TRY(pk.ensure((size_t)nk * 8));
    KHIP_TRY(pko.ensure((size_t)(P + 1) * 8));
    KHIP_TRY_HIP(hipMemcpyAsync(pk.p, hpk.data(), (size_t)nk * 8, hipMemcpyHostToDevice, a->stream));
    KHIP_TRY_HIP(hipMemcpyAsync(pko.p, hpko.data(), (size_t)(P + 1) * 8, hipMemcpyHostToDevice, a->stream));
    h.pkeys = pk.as<int64_t>();
    h.pkoff = pko.as<int64_t>();
  }
  const int P = (int)s.P;
  KHIP_TRY(s.counts.ensure((P + 1) * 8));
  hipLaunchKernelGGL(k_part_rows, dim3(P), dim3(256), 0, a->stream, s.buf[0].as<uint64_t>(), s.buf[1].as<uint64_t>(),
                     s.sel.as<uint8_t>(), s.cnt.as<int64_t>(), s.cmax, a->sw, h, s.counts.as<int64_t>(), nullptr,
                     nullptr);
  KHIP_TRY_HIP(hipMemsetAsync(s.counts.as<int64_t>() + P, 0, 8, a->stream));
  hipLaunchKernelGGL(k_scan_excl, dim3(1), dim3(1024), 0, a->stream, s.counts.as<int64_t>(), (int64_t)P,
                     s.counts.as<int64_t>() + P);
  KHIP_TRY_HIP(hipGetLastError());
  int64_t nl = 0;
  KHIP_TRY_HIP(hipMemcpyAsync(&nl, s.counts.as<int64_t>() + P, 8, hipMemcpyDeviceToHost, a->stream));
  // closed rows (flat store) passing h
  DevBuf& cctr = s.pctr;
  KHIP_TRY(cctr.ensure(16));
  KHIP_TRY_HIP(hipMemsetAsync(cctr.p, 0, 8, a->stream));
  if (s.closed_n) {
    hipLaunchKernelGGL(k_compact, dim3((int)std::min<int64_t>(ceil_div(s.closed_n, 256), 4096)), dim3(256), 0, a->stream,
                       s.closed.as<uint64_t>(), s.closed_n, a->sw, h, (uint64_t*)nullptr, (int64_t)0,
                       cctr.as<unsigned long long>());
  }
  int64_t nc = 0;
  KHIP_TRY_HIP(hipMemcpyAsync(&nc, cctr.p, 8, hipMemcpyDeviceToHost, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  const int64_t n = nl + nc;
  *count = n;
  if (!rows) return KHIP_OK;
  DevBuf out;
  KHIP_TRY(out.ensure((size_t)std::max<int64_t>(n, 1) * a->sw * 8));
  if (nc) {
    KHIP_TRY_HIP(hipMemsetAsync(cctr.p, 0, 8, a->stream));
    hipLaunchKernelGGL(k_compact, dim3((int)std::min<int64_t>(ceil_div(s.closed_n, 256), 4096)), dim3(256), 0, a->stream,
                       s.closed.as<uint64_t>(), s.closed_n, a->sw, h, out.as<uint64_t>() + (size_t)nl * a->sw, nc,
                       cctr.as<unsigned long long>());
  }
  hipLaunchKernelGGL(k_part_rows, dim3(P), dim3(256), 0, a->stream, s.buf[0].as<uint64_t>(), s.buf[1].as<uint64_t>(),
                     s.sel.as<uint8_t>(), s.cnt.as<int64_t>(), s.cmax, a->sw, h, nullptr, s.counts.as<int64_t>(),
                     out.as<uint64_t>());
  KHIP_TRY_HIP(hipGetLastError());
  rows->resize((size_t)n * a->sw);
  if (n) KHIP_TRY_HIP(hipMemcpyAsync(rows->data(), out.p, (size_t)n * a->sw * 8, hipMemcpyDeviceToHost, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  out.release();
  return KHIP_OK;
}

khip_status part_changes(khip_agg* a, std::vector<uint64_t>* rows, std::vector<uint8_t>* tomb, int64_t* count) {
  PartState& s = a->part;
  const int P = (int)s.P;
  KHIP_TRY(s.counts.ensure((P + 1) * 8));
  hipLaunchKernelGGL(k_part_chg, dim3(P), dim3(256), 0, a->stream, s.buf[0].as<uint64_t>(), s.buf[1].as<uint64_t>(),
                     s.sel.as<uint8_t>(), s.cnt.as<int64_t>(), s.cmax, a->sw, s.pbase.as<int64_t>(),
                     s.last_c1 ? s.prn.as<uint32_t>() : (const uint32_t*)nullptr, a->chg.as<uint8_t>(), s.counts.as<int64_t>(), nullptr, nullptr, nullptr);
  KHIP_TRY_HIP(hipMemsetAsync(s.counts.as<int64_t>() + P, 0, 8, a->stream));
  hipLaunchKernelGGL(k_scan_excl, dim3(1), dim3(1024), 0, a->stream, s.counts.as<int64_t>(), (int64_t)P,
                     s.counts.as<int64_t>() + P);
  KHIP_TRY_HIP(hipGetLastError());
  int64_t n = 0;
  KHIP_TRY_HIP(hipMemcpyAsync(&n, s.counts.as<int64_t>() + P, 8, hipMemcpyDeviceToHost, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  *count = n;
  DevBuf out, ot;
  KHIP_TRY(out.ensure((size_t)std::max<int64_t>(n, 1) * a->sw * 8));
  KHIP_TRY(ot.ensure((size_t)std::max<int64_t>(n, 1)));
  hipLaunchKernelGGL(k_part_chg, dim3(P), dim3(256), 0, a->stream, s.buf[0].as<uint64_t>(), s.buf[1].as<uint64_t>(),
                     s.sel.as<uint8_t>(), s.cnt.as<int64_t>(), s.cmax, a->sw, s.pbase.as<int64_t>(),
                     s.last_c1 ? s.prn.as<uint32_t>() : (const uint32_t*)nullptr, a->chg.as<uint8_t>(), nullptr, s.counts.as<int64_t>(), out.as<uint64_t>(), ot.as<uint8_t>());
  KHIP_TRY_HIP(hipGetLastError());
  rows->resize((size_t)n * a->sw);
  tomb->resize((size_t)n);
  if (n) {
    KHIP_TRY_HIP(hipMemcpyAsync(rows->data(), out.p, (size_t)n * a->sw * 8, hipMemcpyDeviceToHost, a->stream));
    KHIP_TRY_HIP(hipMemcpyAsync(tomb->data(), ot.p, (size_t)n, hipMemcpyDeviceToHost, a->stream));
  }
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  return KHIP_OK;
}

// Retention: drop the closed store's rows that expired from the window store (vis: h.vis_from),
// keeping the maintained HAVING count of the closed rows (ctr[12]) and the group count in step.
khip_status part_purge_closed(khip_agg* a, const HavingDev& vis) {
  PartState& s = a->part;
  if (s.closed_n == 0 || vis.vis_from <= s.purged_to) return KHIP_OK;
  const int grid = (int)std::min<int64_t>(ceil_div(s.closed_n, 256), 4096);
  // one pass: the kept rows go to the second store (which then becomes the store) and are counted;
  // one host round trip for both counts (the buffers are the handle's: no allocation per push)
  DevBuf& ctr = s.pctr;
  KHIP_TRY(ctr.ensure(16));
  DevBuf& nc = s.closed2;
  KHIP_TRY(nc.ensure((size_t)s.closed_cap * a->sw * 8));
  KHIP_TRY_HIP(hipMemsetAsync(ctr.p, 0, 16, a->stream));
  hipLaunchKernelGGL(k_compact, dim3(grid), dim3(256), 0, a->stream, s.closed.as<uint64_t>(), s.closed_n, a->sw, vis,
                     nc.as<uint64_t>(), s.closed_cap, ctr.as<unsigned long long>());
  HavingDev vh = vis;  // kept rows passing the query's HAVING
  vh.active = a->having.active;
  vh.op = a->having.op;
  vh.a = a->having.a;
  vh.i64 = a->having.i64;
  vh.f64 = a->having.f64;
  if (vh.active)
    hipLaunchKernelGGL(k_compact, dim3(grid), dim3(256), 0, a->stream, s.closed.as<uint64_t>(), s.closed_n, a->sw, vh,
                       (uint64_t*)nullptr, (int64_t)0, ctr.as<unsigned long long>() + 1);
  KHIP_TRY_HIP(hipGetLastError());
  int64_t kc[2] = {0, 0};
  KHIP_TRY_HIP(hipMemcpyAsync(kc, ctr.p, 16, hipMemcpyDeviceToHost, a->stream));
  KHIP_TRY_HIP(hipStreamSynchronize(a->stream));
  s.purged_to = vis.vis_from;
  const int64_t keep = kc[0];
  if (keep == s.closed_n) return KHIP_OK;  // nothing expired: the store stays (its copy is unused)
  if (vh.active) {  // ctr[12]: closed rows passing HAVING
    unsigned long long* hc = s.pinfo.as<unsigned long long>() + 40;
    *hc = (unsigned long long)kc[1];
    KHIP_TRY_HIP(hipMemcpyAsync(s.ctr.as<unsigned long long>() + 12, hc, 8, hipMemcpyHostToDevice, a->stream));
    s.having_total += kc[1] - (int64_t)s.pinfo.as<unsigned long long>()[8 + 12];
    KHIP_TRY_HIP(hipStreamSynchronize(a->stream));  // (hc is pinned host memory the next push reuses)
  }
  std::swap(s.closed, s.closed2);
  a->occ -= s.closed_n - keep;
  s.closed_n = keep;
  return KHIP_OK;
}

}  // namespace khip
