// random_atomic.hip — the update rate a group table of few hot groups runs against (table
// aggregation's k_tagg_apply: every source-key change undoes / applies its rows with agent-scope
// atomics on a group slot).
//
// `groups` slots of 64 bytes spread over a table of `bytes` (slot = mix(g) & mask, as the group
// table's hash places them); each thread updates R random groups.  Modes: 8-byte loads, relaxed
// agent-scope atomic add (no return), atomic max (no return), and the k_tagg_apply pattern per
// update (16-byte slot load + atomic max + two atomic adds).  Reports operations (updates) per
// second.  Build: hipcc -O3 --offload-arch=gfx950 -o random_atomic random_atomic.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  x ^= x >> 31;
  return x;
}

template <int MODE, int R>
__global__ __launch_bounds__(256) void k_upd(uint64_t* __restrict__ table, uint64_t mask, uint64_t groups, int64_t n,
                                             uint64_t seed, unsigned long long* __restrict__ sink) {
  const int64_t base = (int64_t)blockIdx.x * 256 * R;
  uint64_t acc = 0;
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int64_t i = base + r * 256 + threadIdx.x;
    if (i >= n) break;
    const uint64_t g = mix(seed + (uint64_t)i) % groups;
    uint64_t* s = table + (mix(g ^ 0x9E3779B97F4A7C15ULL) & mask) * 8;
    if (MODE == 0) {
      acc ^= s[3];
    } else if (MODE == 1) {
      __hip_atomic_fetch_add(&s[3], 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (MODE == 2) {
      __hip_atomic_fetch_max((int64_t*)&s[2], (int64_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const ulonglong2 w = *(const ulonglong2*)&s[2];
      if ((int64_t)w.x < (int64_t)i)
        __hip_atomic_fetch_max((int64_t*)&s[2], (int64_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&s[3], 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&s[4], (uint64_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      acc ^= w.y;
    }
  }
  if (acc == 0x123456789ULL) atomicAdd(sink, 1ULL);
}

template <int MODE, int R>
static double run(uint64_t* table, uint64_t slots, uint64_t groups, int64_t n, unsigned long long* sink) {
  const int64_t blocks = (n + 256 * R - 1) / (256 * R);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k_upd<MODE, R>), dim3(blocks), dim3(256), 0, 0, table, slots - 1, groups, n, 1ULL, sink);
  hipEventRecord(e0, 0);
  const int reps = 3;
  for (int k = 0; k < reps; k++)
    hipLaunchKernelGGL((k_upd<MODE, R>), dim3(blocks), dim3(256), 0, 0, table, slots - 1, groups, n, 7ULL + k, sink);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return (double)n * reps / (ms / 1000.0);
}

int main() {
  const int64_t n = 50000000;
  unsigned long long* sink;
  hipMalloc(&sink, 8);
  const uint64_t bytes = 64ULL << 20;  // 2^20 slots of 64 B (table aggregation's group table, 1e5 groups x 8)
  uint64_t* table = nullptr;
  hipMalloc(&table, bytes);
  hipMemset(table, 0, bytes);
  const uint64_t slots = bytes / 64;
  printf("groups,mode,updates_per_s\n");
  const uint64_t gs[] = {1000, 100000, 1000000};
  for (uint64_t g : gs) {
    printf("%llu,load8,%.4g\n", (unsigned long long)g, run<0, 4>(table, slots, g, n, sink));
    printf("%llu,atomic_add,%.4g\n", (unsigned long long)g, run<1, 4>(table, slots, g, n, sink));
    printf("%llu,atomic_max,%.4g\n", (unsigned long long)g, run<2, 4>(table, slots, g, n, sink));
    printf("%llu,tagg_update,%.4g\n", (unsigned long long)g, run<3, 4>(table, slots, g, n, sink));
    fflush(stdout);
  }
  hipFree(table);
  hipFree(sink);
  return 0;
}
