// khip_part.hpp — device helpers shared by the partitioned aggregation kernels
// (khip_agg_part.hip: the general engine; khip_agg_c1.hip: the COUNT(*) pipeline).
#pragma once

#include "khip_agg_internal.hpp"

namespace khip {

enum { T_ACCEPTED, T_NULL_KEY, T_NULL_ROW, T_BAD_TS, T_APPLIED, T_LATE, T_NPART };

// Key hash: its top log2P bits pick the partition; inside a partition the LDS slot and the
// sub-pass of a (key, windowStart) group mix its low bits with ws (cheap 32-bit math).
__device__ __forceinline__ uint64_t key_hash(int64_t key) { return mix64((uint64_t)key ^ 0x6A09E667F3BCC908ULL); }

// inverse of key_hash (mix64 is a bijection): key = unmix64(hk) ^ C
__device__ __forceinline__ int64_t key_of_hash(uint64_t h) {
  h ^= h >> 33;
  h *= 0x9cb4b2f8129337dbULL;  // inverse of 0xc4ceb9fe1a85ec53 mod 2^64
  h ^= h >> 33;
  h *= 0x4f74430c22a54005ULL;  // inverse of 0xff51afd7ed558ccd mod 2^64
  h ^= h >> 33;
  return (int64_t)(h ^ 0x6A09E667F3BCC908ULL);
}

constexpr uint64_t EMPTY_ID = ~0ULL;

__device__ __forceinline__ uint32_t part_of_hk(uint64_t hk, int log2P) {
  return log2P == 0 ? 0u : (uint32_t)(hk >> (64 - log2P));
}

__device__ __forceinline__ uint32_t part_of(int64_t key, int log2P) { return part_of_hk(key_hash(key), log2P); }

__device__ __forceinline__ int64_t tile_of(int64_t b, int64_t nT) {
  // blocks b, b+8, b+16 ... share an XCD (round-robin dispatch): give each XCD a contiguous
  // run of tiles so consecutive tiles' writes to one partition combine in that XCD's L2
  const int64_t per = nT / 8, rem = nT % 8, x = b % 8, k = b / 8;
  return x * per + (x < rem ? x : rem) + k;
}

// barrier without the vmcnt(0) that __syncthreads() implies: LDS writes are waited for, the
// wave's outstanding global loads (prefetches) and stores stay in flight
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

#define KLDS __attribute__((address_space(3)))
typedef KLDS uint32_t lds_u32;
typedef KLDS int64_t lds_i64;
typedef KLDS double lds_f64;
#define WG_RLX __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP

constexpr uint32_t RT_MATCHED = 0x80000000u;

// Append the claimed entries of the wave's lanes to the item's list (one LDS atomic per wave);
// called by every lane of the wave (convergent).
__device__ __forceinline__ void mg_list_append(bool claimed, uint32_t e, KLDS uint16_t* nl, int* nnew) {
  const uint64_t b = __ballot(claimed);
  if (!b) return;
  const int lane = threadIdx.x & 63, leader = __ffsll((long long)b) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(nnew, __popcll(b));
  base = __shfl(base, leader, 64);
  if (claimed) nl[base + __popcll(b & ((1ULL << lane) - 1))] = (uint16_t)e;
}

// mg_list_append for AU entries per lane at once: one LDS atomic per wave for all of them.
// Returns the list's length after this wave's entries (0 when the wave appended none).
template <int AU>
__device__ __forceinline__ int mg_list_append_n(const bool (&claimed)[AU], const uint32_t (&e)[AU], KLDS uint16_t* nl,
                                                int* nnew) {
  uint64_t b[AU];
  int tot = 0;
#pragma unroll
  for (int u = 0; u < AU; u++) {
    b[u] = __ballot(claimed[u]);
    tot += __popcll(b[u]);
  }
  if (!tot) return 0;
  const int lane = threadIdx.x & 63;
  int base = 0;
  if (lane == 0) base = atomicAdd(nnew, tot);
  base = __builtin_amdgcn_readfirstlane(base);  // (convergent call: lane 0 is the first active lane)
  const uint64_t lt = (1ULL << lane) - 1;
#pragma unroll
  for (int u = 0; u < AU; u++) {
    if (claimed[u]) nl[base + __popcll(b[u] & lt)] = (uint16_t)e[u];
    base += __popcll(b[u]);
  }
  return base;
}

constexpr uint32_t C1_GOLD = 0x9E3779B1u;

__device__ __forceinline__ uint32_t stage_bin(uint64_t hk, int shift, uint32_t mask) {
  return shift >= 64 ? 0u : (uint32_t)(hk >> shift) & mask;
}

// LDS-staged scatter of 8-byte records (k_part_scatter_r8 / k_part_refine_r8 / k_c1_scatter):
struct StageR8 {
  uint32_t* cur;    // [nb] next output record of each bin
  uint32_t* cnt;    // [nb] records of the step per bin
  uint32_t* sbase;  // [nb] the bin's first staged slot
  uint32_t* gpos;   // [nb] output position of the bin's first record of the step
  int64_t* sp;      // [S] staged records
  uint16_t* sbin;   // [S] their bins
  int* wsum;        // [NT / 64]
};

__host__ __device__ constexpr size_t stage_r8_lds_bytes(int nb, int S) {
  return (size_t)nb * 16 + (size_t)S * 8 + ((size_t)S * 2 + 15) / 16 * 16;
}

__device__ __forceinline__ StageR8 stage_r8_carve(char* smem, int nb, int S, int* wsum) {
  StageR8 L;
  L.cur = (uint32_t*)smem;
  L.cnt = L.cur + nb;
  L.sbase = L.cnt + nb;
  L.gpos = L.sbase + nb;
  L.sp = (int64_t*)(smem + (size_t)nb * 16);
  L.sbin = (uint16_t*)(L.sp + S);
  L.wsum = wsum;
  return L;
}

// One step: U records per thread (ok = present) → rank per bin, bin-ordered in LDS, written out
// per bin as one contiguous run by consecutive threads.  nb <= NT.
template <int U, int NT>
__device__ __forceinline__ void stage_step_r8(const int64_t (&rec)[U], const uint32_t (&bin)[U], const bool (&ok)[U],
                                              int nb, const StageR8& L, uint64_t* __restrict__ srec) {
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
#pragma unroll
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
#pragma unroll
  for (int u = 0; u < U; u++)
    if (ok[u]) {
      const uint32_t i = L.sbase[bin[u]] + rank[u];
      L.sp[i] = rec[u];
      L.sbin[i] = (uint16_t)bin[u];
    }
  lds_barrier();
  for (uint32_t j = t; j < tot; j += NT) {
    const uint32_t b = L.sbin[j];
    srec[(uint64_t)L.gpos[b] + (j - L.sbase[b])] = (uint64_t)L.sp[j];
  }
  // the next step's first barrier (after its rank atomics) orders these LDS reads before any
  // rewrite of sbase / gpos / the stage
}

// kernels and host helpers of khip_agg_part.hip used by khip_agg_c1.hip
__global__ void k_part_pscan(int64_t* __restrict__ v, int64_t n);
__global__ void k_part_stats(const int64_t* __restrict__ tpart, int64_t nT, const unsigned long long* __restrict__ closed_n,
                             const int64_t* __restrict__ stream_time, unsigned long long* __restrict__ out);
khip_status part_regrow(khip_agg* a, int64_t ncmax);
// khip_agg_c1.hip: the windowed COUNT(*) pipeline (declined = the general path must run)
bool c1_eligible(khip_agg* a, int64_t n);
bool c1v_eligible(khip_agg* a, int64_t n, int* col);
khip_status c1_push(khip_agg* a, int64_t n, const int64_t* keys, const int64_t* ts, const uint8_t* kv,
                    const uint8_t* rv, int64_t* tot, bool* declined, const int64_t* st_at, bool* retry_wide,
                    const ColPtrs* cols = nullptr, int vcol = -1, const RowsIn* rows = nullptr);
__global__ void k_part_commit(const int64_t* __restrict__ gate, int P, const int64_t* __restrict__ pbase,
                              const uint32_t* __restrict__ prn, const uint32_t* __restrict__ plist, int nlist,
                              uint8_t* __restrict__ sel, int64_t* __restrict__ cnt,
                              unsigned long long* __restrict__ newcnt, const uint8_t* __restrict__ fail,
                              unsigned long long* __restrict__ out, unsigned long long* __restrict__ hcnt,
                              unsigned long long* __restrict__ hnew);

}  // namespace khip
