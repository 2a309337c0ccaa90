// khip_sort.hpp — device sort / scan / run-length primitives for the SESSION and table-aggregation
// engines (gfx950), in place of a library's.
//
//   sort_pairs<V>   stable LSD radix sort of (u64 key, V value) pairs over key bits [0, end_bit),
//                   8-bit digits.  k_rs_ghist counts every pass's digits in one read of the keys;
//                   then one kernel per pass (k_rs_pass) reads and writes each pair once: tiles of
//                   8192 pairs taken in ticket order rank their items stably per digit (wave ballots
//                   + per-wave running counts), publish their digit counts, stage the items in LDS
//                   in digit order and find their output offsets by decoupled look-back over the
//                   earlier tiles' published counts, so no per-pass histogram or scan pass remains.
//   scan_excl<I,O>  exclusive prefix sum (block sums → one block over the sums → per block, rounds
//                   of 1024 coalesced items scanned with the running carry).
//   rle_sorted      run-length segments of sorted keys: unique keys, counts, segment starts, count
//                   (head counts per block → their prefix → heads written by ballot rank).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "khip_util.hpp"

namespace khip {
namespace ksort {
namespace {  // each including translation unit gets its own copy of the kernels

constexpr int RS_T = 1024;  // threads per tile
constexpr int RS_W = RS_T / 64;
constexpr int SC_T = 1024, SC_I = 8;  // scan / run-length: threads, items per thread

// ------------------------------------------------------------------ block helpers

// Exclusive prefix of x over the block in thread order (every thread calls; two barriers).
// wsum: LDS scratch of blockDim / 64 words.  *total: the block's sum.
template <class T>
__device__ __forceinline__ T blk_scan_excl(T x, T* wsum, T* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  T incl = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const T y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  T before = 0, tot = 0;
  const int nw = (int)(blockDim.x >> 6);
  for (int k = 0; k < nw; k++) {
    before += k < wave ? wsum[k] : 0;
    tot += wsum[k];
  }
  __syncthreads();
  *total = tot;
  return before + incl - x;
}

// ------------------------------------------------------------------ scan

// Per block of SC_T * SC_I items: its sum (coalesced reads; order does not matter for a sum).
template <class I>
__global__ __launch_bounds__(SC_T) void k_sc_sums(const I* __restrict__ in, int64_t n, int64_t* __restrict__ bsum) {
  __shared__ int64_t wsum[SC_T / 64];
  const int64_t base = (int64_t)blockIdx.x * SC_T * SC_I + threadIdx.x;
  int64_t s = 0;
#pragma unroll
  for (int u = 0; u < SC_I; u++) s += base + u * SC_T < n ? (int64_t)in[base + u * SC_T] : 0;
  int64_t tot;
  blk_scan_excl(s, wsum, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SC_T) void k_sc_top(int64_t* __restrict__ bsum, int64_t nb) {
  __shared__ int64_t wsum[SC_T / 64];
  int64_t carry = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += SC_T) {
    const int64_t b = b0 + threadIdx.x;
    const int64_t x = b < nb ? bsum[b] : 0;
    int64_t tot;
    const int64_t ex = blk_scan_excl(x, wsum, &tot);
    if (b < nb) bsum[b] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) bsum[nb] = carry;
}

// The block's items in rounds of SC_T consecutive items (coalesced), one block scan per round.
template <class I, class O>
__global__ __launch_bounds__(SC_T) void k_sc_apply(const I* __restrict__ in, int64_t n, const int64_t* __restrict__ bsum,
                                                   O* __restrict__ out) {
  __shared__ int64_t wsum[SC_T / 64];
  const int64_t base = (int64_t)blockIdx.x * SC_T * SC_I + threadIdx.x;
  I x[SC_I];
#pragma unroll
  for (int u = 0; u < SC_I; u++) x[u] = base + u * SC_T < n ? in[base + u * SC_T] : (I)0;
  int64_t carry = bsum[blockIdx.x];
#pragma unroll
  for (int u = 0; u < SC_I; u++) {
    int64_t tot;
    const int64_t ex = blk_scan_excl((int64_t)x[u], wsum, &tot);
    if (base + u * SC_T < n) out[base + u * SC_T] = (O)(carry + ex);
    carry += tot;
  }
}

template <class O>
__global__ void k_sc_total(const int64_t* __restrict__ s, O* __restrict__ d) {
  *d = (O)*s;
}

// out[i] = sum of in[0..i); also out[n] = the total when with_total (out must hold n + 1).
// in and out may alias.  tmp: scratch; total_host (may be null): the total, synchronously.
template <class I, class O>
khip_status scan_excl(hipStream_t st, DevBuf& tmp, const I* in, O* out, int64_t n, bool with_total,
                      int64_t* total_host) {
  const int64_t per = (int64_t)SC_T * SC_I;
  const int64_t nb = std::max<int64_t>(1, ceil_div(n, per));
  KHIP_TRY(tmp.ensure((size_t)(nb + 1) * 8));
  int64_t* bs = tmp.as<int64_t>();
  auto sums = k_sc_sums<I>;
  auto apply = k_sc_apply<I, O>;
  auto total = k_sc_total<O>;
  hipLaunchKernelGGL(sums, dim3(nb), dim3(SC_T), 0, st, in, n, bs);
  hipLaunchKernelGGL(k_sc_top, dim3(1), dim3(SC_T), 0, st, bs, nb);
  hipLaunchKernelGGL(apply, dim3(nb), dim3(SC_T), 0, st, in, n, bs, out);
  KHIP_TRY_HIP(hipGetLastError());
  if (with_total) {  // out[n] = the total
    hipLaunchKernelGGL(total, dim3(1), dim3(1), 0, st, bs + nb, out + n);
    KHIP_TRY_HIP(hipGetLastError());
  }
  if (total_host) {
    KHIP_TRY_HIP(hipMemcpyAsync(total_host, bs + nb, 8, hipMemcpyDeviceToHost, st));
    KHIP_TRY_HIP(hipStreamSynchronize(st));
  }
  return KHIP_OK;
}

// ------------------------------------------------------------------ run-length segments

// Segment heads of sorted keys (i == 0 or key[i] != key[i - 1]) per block of SC_T * SC_I.
__global__ __launch_bounds__(SC_T) void k_rle_count(const uint64_t* __restrict__ key, int64_t n,
                                                    int64_t* __restrict__ bcnt) {
  __shared__ int64_t wsum[SC_T / 64];
  const int64_t base = (int64_t)blockIdx.x * SC_T * SC_I + threadIdx.x;
  int64_t h = 0;
#pragma unroll
  for (int u = 0; u < SC_I; u++) {
    const int64_t i = base + u * SC_T;
    h += i < n && (i == 0 || key[i] != key[i - 1]);
  }
  int64_t tot;
  blk_scan_excl(h, wsum, &tot);
  if (threadIdx.x == 0) bcnt[blockIdx.x] = tot;
}

// The heads in element order (rounds of SC_T items, a ballot rank per wave): ukeys[s], start[s];
// the last block also writes start[nseg] = n and *nseg.
__global__ __launch_bounds__(SC_T) void k_rle_write(const uint64_t* __restrict__ key, int64_t n,
                                                    const int64_t* __restrict__ bpre, int64_t nb,
                                                    uint64_t* __restrict__ ukeys, int64_t* __restrict__ start,
                                                    int* __restrict__ nseg) {
  __shared__ uint32_t wcnt[SC_T / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t lt = lane ? (~0ULL >> (64 - lane)) : 0ULL;
  const int64_t base = (int64_t)blockIdx.x * SC_T * SC_I + threadIdx.x;
  int64_t seg = bpre[blockIdx.x];
  for (int u = 0; u < SC_I; u++) {
    const int64_t i = base + u * SC_T;
    uint64_t k = 0;
    bool h = false;
    if (i < n) {
      k = key[i];
      h = i == 0 || k != key[i - 1];
    }
    const uint64_t b = __ballot(h);
    if (lane == 0) wcnt[wave] = (uint32_t)__popcll(b);
    __syncthreads();
    uint32_t before = 0, tot = 0;
    for (int w = 0; w < SC_T / 64; w++) {
      before += w < wave ? wcnt[w] : 0u;
      tot += wcnt[w];
    }
    if (h) {
      const int64_t s = seg + before + (uint32_t)__popcll(b & lt);
      ukeys[s] = k;
      start[s] = i;
    }
    seg += tot;
    __syncthreads();
  }
  if (blockIdx.x == nb - 1 && threadIdx.x == 0) {
    start[seg] = n;
    *nseg = (int)seg;
  }
}

__global__ __launch_bounds__(256) void k_rle_counts(const int64_t* __restrict__ start, const int* __restrict__ nseg,
                                                    int* __restrict__ cnt) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < *nseg) cnt[j] = (int)(start[j + 1] - start[j]);
}

// Segments of equal keys in sorted `key[0..n)`: ukeys[s], cnt[s], start[s] (start[nseg] = n),
// *nseg_dev; returns the count on the host.  ukeys / cnt / start hold n (+ 1) entries.
inline khip_status rle_sorted(hipStream_t st, DevBuf& tmp, const uint64_t* key, int64_t n, uint64_t* ukeys, int* cnt,
                              int64_t* start, int* nseg_dev, int64_t* nseg_host) {
  const int64_t per = (int64_t)SC_T * SC_I;
  const int64_t nb = std::max<int64_t>(1, ceil_div(n, per));
  KHIP_TRY(tmp.ensure((size_t)(nb + 1) * 8));
  int64_t* bc = tmp.as<int64_t>();
  hipLaunchKernelGGL(k_rle_count, dim3(nb), dim3(SC_T), 0, st, key, n, bc);
  hipLaunchKernelGGL(k_sc_top, dim3(1), dim3(SC_T), 0, st, bc, nb);
  hipLaunchKernelGGL(k_rle_write, dim3(nb), dim3(SC_T), 0, st, key, n, bc, nb, ukeys, start, nseg_dev);
  hipLaunchKernelGGL(k_rle_counts, dim3(std::max<int64_t>(1, ceil_div(n, 256))), dim3(256), 0, st, start, nseg_dev, cnt);
  KHIP_TRY_HIP(hipGetLastError());
  if (nseg_host) {
    KHIP_TRY_HIP(hipMemcpyAsync(nseg_host, bc + nb, 8, hipMemcpyDeviceToHost, st));
    KHIP_TRY_HIP(hipStreamSynchronize(st));
  }
  return KHIP_OK;
}

// ------------------------------------------------------------------ radix sort


// Every pass's digit counts in one read of the keys: ghist[p * 256 + digit].
__global__ __launch_bounds__(RS_T) void k_rs_ghist(const uint64_t* __restrict__ key, int64_t n, int passes,
                                                   uint32_t* __restrict__ ghist) {
  __shared__ uint32_t c[8][256];
  for (int i = threadIdx.x; i < 8 * 256; i += RS_T) (&c[0][0])[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * RS_T + threadIdx.x; i < n; i += (int64_t)gridDim.x * RS_T) {
    const uint64_t k = key[i];
    for (int p = 0; p < passes; p++) atomicAdd(&c[p][(uint32_t)(k >> (8 * p)) & 255u], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < passes * 256; i += RS_T) {
    const uint32_t v = (&c[0][0])[i];
    if (v) atomicAdd(&ghist[i], v);
  }
}

// Tile status words of the decoupled look-back: flag in the top two bits, a digit count below.
constexpr uint64_t RS_AGG = 1ULL << 62, RS_INC = 2ULL << 62, RS_VAL = (1ULL << 62) - 1;

__device__ __forceinline__ uint64_t rs_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void rs_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// LDS of k_rs_pass: per digit the global output base, the tile's digit starts, a scan scratch,
// then the per-(wave, digit) counts — reused, once the ranks are known, as the staging area.
template <int T, int IPT, class V>
__host__ __device__ constexpr size_t rs_lds_bytes() {
  return 256 * 8 + 256 * 4 + 64 + ((size_t)T * IPT * (8 + sizeof(V)) > (size_t)(T / 64) * 256 * 4
                                        ? (size_t)T * IPT * (8 + sizeof(V))
                                        : (size_t)(T / 64) * 256 * 4);
}

// One LSD pass, one read and one write of the pairs.  Tiles are taken in ticket order; a tile
// ranks its items stably per digit (per wave: 8 ballots find the lanes with the same digit, the
// wave's running per-digit counts give the order across its rounds; the waves' counts are then
// prefixed per digit), publishes its digit counts, stages the items in LDS in digit order, and
// looks back over the earlier tiles' published counts / inclusive prefixes for its output offset
// per digit; the items then leave so each (digit, tile) run is a run of consecutive stores.
// A tile waits only on tiles with earlier tickets, which are already running.
template <int T, int IPT, class V>
__global__ __launch_bounds__(T) void k_rs_pass(const uint64_t* __restrict__ kin, const V* __restrict__ vin,
                                                  int64_t n, int shift, const uint32_t* __restrict__ ghist,
                                                  uint64_t* __restrict__ status, unsigned int* __restrict__ ticket,
                                                  uint64_t* __restrict__ kout, V* __restrict__ vout) {
  constexpr int TILE = T * IPT, W = T / 64;  // wave w owns [w * 64 * IPT, +64 * IPT) of the tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int64_t* gpos = (int64_t*)smem;                 // [256] output index of the digit's first tile item
  uint32_t* dstart = (uint32_t*)(gpos + 256);     // [256] tile-local digit starts
  uint32_t* scr = dstart + 256;                   // [16] scan scratch; scr[15]: the ticket
  uint32_t* wc = scr + 16;                        // [T / 64][256] per-wave digit counts
  uint64_t* sk = (uint64_t*)wc;                   // [TILE] staged keys (after the ranks)
  V* sv = (V*)(sk + TILE);                        // [TILE] staged values
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t lt = lane ? (~0ULL >> (64 - lane)) : 0ULL;
  for (int i = threadIdx.x; i < W * 256; i += T) wc[i] = 0;
  if (threadIdx.x == 0) scr[15] = atomicAdd(ticket, 1u);
  __syncthreads();
  const int64_t tile = scr[15];
  const int64_t tbase = tile * TILE;
  const int64_t base = tbase + (int64_t)wave * 64 * IPT + lane;
  uint64_t k[IPT];
  V v[IPT];
  uint32_t rank[IPT];
#pragma unroll
  for (int u = 0; u < IPT; u++) {
    const int64_t i = base + u * 64;
    const int64_t ic = i < n ? i : n - 1;
    k[u] = kin[ic];
    v[u] = vin[ic];
  }
  uint32_t* mine = wc + wave * 256;
#pragma unroll
  for (int u = 0; u < IPT; u++) {  // the wave's rounds in element order: stable
    const bool valid = base + u * 64 < n;
    const uint32_t d = (uint32_t)(k[u] >> shift) & 255u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const uint64_t m = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? m : ~m;
    }
    const uint32_t rw = (uint32_t)__popcll(peers & lt);
    const uint32_t before = valid ? mine[d] : 0u;
    rank[u] = before + rw;
    __builtin_amdgcn_wave_barrier();
    if (valid && rw == 0) mine[d] = before + (uint32_t)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // per digit: the waves' offsets (prefix over the waves), the tile's count, published at once
  uint32_t cnt = 0;
  if (threadIdx.x < 256) {
    for (int w = 0; w < W; w++) {
      const uint32_t e = wc[w * 256 + threadIdx.x];
      wc[w * 256 + threadIdx.x] = cnt;
      cnt += e;
    }
    rs_store(status + tile * 256 + threadIdx.x, (tile == 0 ? RS_INC : RS_AGG) | cnt);
  }
  // tile digit starts and the pass's global digit bases (both exclusive scans over the digits)
  uint32_t tot32;
  const uint32_t ds = blk_scan_excl<uint32_t>(threadIdx.x < 256 ? cnt : 0u, scr, &tot32);
  if (threadIdx.x < 256) dstart[threadIdx.x] = ds;
  const uint32_t gh = threadIdx.x < 256 ? ghist[threadIdx.x] : 0u;
  uint64_t tot64;
  const uint64_t gb = blk_scan_excl<uint64_t>(gh, (uint64_t*)gpos, &tot64);  // gpos as scratch
  __syncthreads();
#pragma unroll
  for (int u = 0; u < IPT; u++) {
    const uint32_t d = (uint32_t)(k[u] >> shift) & 255u;
    rank[u] += wc[wave * 256 + d] + dstart[d];
  }
  __syncthreads();  // every rank read before the staging overwrites wc
#pragma unroll
  for (int u = 0; u < IPT; u++) {
    if (base + u * 64 < n) {
      sk[rank[u]] = k[u];
      sv[rank[u]] = v[u];
    }
  }
  // look-back: the digit's count over the earlier tiles
  if (threadIdx.x < 256) {
    uint64_t excl = 0;
    for (int64_t j = tile - 1; j >= 0;) {
      const uint64_t s = rs_load(status + j * 256 + threadIdx.x);
      if (!(s & ~RS_VAL)) {
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      excl += s & RS_VAL;
      if (s & RS_INC) break;
      j--;
    }
    if (tile > 0) rs_store(status + tile * 256 + threadIdx.x, RS_INC | (excl + cnt));
    gpos[threadIdx.x] = (int64_t)(gb + excl) - (int64_t)ds;
  }
  __syncthreads();
  const int64_t m = n - tbase < (int64_t)TILE ? n - tbase : (int64_t)TILE;
  for (int64_t j = threadIdx.x; j < m; j += T) {
    const uint64_t kk = sk[j];
    const int64_t dst = gpos[(uint32_t)(kk >> shift) & 255u] + j;
    kout[dst] = kk;
    vout[dst] = sv[j];
  }
}

// Stable sort of (key, value) pairs by key bits [0, end_bit) (n < 2^32).  The sorted pairs end
// in (k_out, v_out); k_in / v_in are clobbered.  tmp: histograms and tile status; alt: a third
// key / value buffer, used when the pass count is even.
template <int T, int IPT, class V>
khip_status sort_run(hipStream_t st, DevBuf& tmp, DevBuf& alt, uint64_t* k_in, uint64_t* k_out, V* v_in, V* v_out,
                     int64_t n, int passes) {
  constexpr int64_t TILE = (int64_t)T * IPT;
  const int64_t nT = ceil_div(n, TILE);
  const size_t st_bytes = (size_t)nT * 256 * 8;
  // [ghist passes x 256 u32 | tickets 8 u32 | status passes x nT x 256 u64]
  const size_t head = 8 * 256 * 4 + 64;
  KHIP_TRY(tmp.ensure(head + st_bytes * passes));
  uint32_t* ghist = tmp.as<uint32_t>();
  unsigned int* tick = ghist + 8 * 256;
  uint64_t* status = (uint64_t*)(tmp.as<char>() + head);
  KHIP_TRY_HIP(hipMemsetAsync(tmp.p, 0, head + st_bytes * passes, st));
  hipLaunchKernelGGL(k_rs_ghist, dim3((int)std::min<int64_t>(ceil_div(n, RS_T * 16), 2048)), dim3(RS_T), 0, st, k_in,
                     n, passes, ghist);
  constexpr size_t lds = rs_lds_bytes<T, IPT, V>();
  auto pk = k_rs_pass<T, IPT, V>;
  hipFuncSetAttribute((const void*)pk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  // the destinations alternate so the last pass writes (k_out, v_out): with an even pass count
  // the first pass goes to the third buffer
  uint64_t* ka = k_in;
  V* va = v_in;
  uint64_t* kb;
  V* vb;
  if (passes & 1) {
    kb = k_out;
    vb = v_out;
  } else {
    KHIP_TRY(alt.ensure((size_t)n * (8 + sizeof(V))));
    kb = alt.as<uint64_t>();
    vb = (V*)(kb + n);
  }
  for (int p = 0; p < passes; p++) {
    hipLaunchKernelGGL(pk, dim3(nT), dim3(T), lds, st, ka, va, n, 8 * p, ghist + p * 256,
                       (uint64_t*)(status + (size_t)p * nT * 256), tick + p, kb, vb);
    KHIP_TRY_HIP(hipGetLastError());
    if (p == passes - 1) break;
    // next: read what this pass wrote; write to k_out on the last pass, else the other buffer
    uint64_t* nk = (kb == k_out) ? k_in : k_out;
    V* nv = (vb == v_out) ? v_in : v_out;
    if (p + 1 == passes - 1) {
      nk = k_out;
      nv = v_out;
    }
    ka = kb;
    va = vb;
    kb = nk;
    vb = nv;
  }
  return KHIP_OK;
}

// Stable sort of (key, value) pairs by key bits [0, end_bit) (n < 2^32).  The sorted pairs end
// in (k_out, v_out); k_in / v_in are clobbered.  tmp: histograms and tile status; alt: a third
// key / value buffer, used when the pass count is even.
template <class V>
khip_status sort_pairs(hipStream_t st, DevBuf& tmp, DevBuf& alt, uint64_t* k_in, uint64_t* k_out, V* v_in, V* v_out,
                       int64_t n, int end_bit) {
  if (n <= 0) return KHIP_OK;
  if (n >= (1LL << 32)) return fail(KHIP_E_INVALID, "sort: too many items");
  const int passes = std::min(8, std::max(1, (end_bit + 7) / 8));
  // tiles of 1024 x 8 pairs (SESSION, 100M pairs of 8 + 8 B, per pass: 873 us; 1024 x 4: 1286,
  // 512 x 8: 986, 512 x 16: 931, 256 x 16: 1009 — profiles/r03/ab/sort_tiles.txt)
  if (knob("KHIP_RS_CFG", 0) == 1) return sort_run<512, 16, V>(st, tmp, alt, k_in, k_out, v_in, v_out, n, passes);
  return sort_run<1024, 8, V>(st, tmp, alt, k_in, k_out, v_in, v_out, n, passes);
}

}  // namespace
}  // namespace ksort
}  // namespace khip
