// LDS operation throughput on gfx950: random-address u32 add (no return), u32 max (no return),
// u64 CAS (with return), u64 read, per CU.  Tuning aid for k_part_merge (which does one CAS,
// one max and one add per record); not part of the library.
//   hipcc -O3 --offload-arch=gfx950 tools/lds_atomic_bench.hip -o tools/lds_atomic_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ENTRIES = 4096;  // 32 KB of u64
constexpr int ITERS = 256;

template <int MODE>
__global__ __launch_bounds__(512) void k_lds(unsigned long long* out, int spread) {
  __shared__ unsigned long long t64[ENTRIES];
  __shared__ uint32_t t32[ENTRIES];
  for (int i = threadIdx.x; i < ENTRIES; i += 512) {
    t64[i] = 0;
    t32[i] = 0;
  }
  __syncthreads();
  uint32_t x = threadIdx.x * 2654435761u + blockIdx.x * 40503u;
  unsigned long long acc = 0;
  for (int it = 0; it < ITERS; it++) {
    uint32_t e[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      x = x * 1664525u + 1013904223u;
      e[u] = (x >> 8) & (uint32_t)(spread - 1);
    }
    if (MODE == 0) {
#pragma unroll
      for (int u = 0; u < 4; u++) __hip_atomic_fetch_add(&t32[e[u]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (MODE == 1) {
#pragma unroll
      for (int u = 0; u < 4; u++) __hip_atomic_fetch_max(&t32[e[u]], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (MODE == 2) {
#pragma unroll
      for (int u = 0; u < 4; u++) {
        unsigned long long o = 0;
        __hip_atomic_compare_exchange_strong(&t64[e[u]], &o, (unsigned long long)x, __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        acc += o;
      }
    } else if (MODE == 3) {
#pragma unroll
      for (int u = 0; u < 4; u++) acc += __hip_atomic_load(&t64[e[u]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (MODE == 4) {
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const unsigned long long o = __hip_atomic_fetch_add(&t64[e[u]], 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        acc += o;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 0; i < ENTRIES; i++) acc += t64[i] + t32[i];
  }
  if (acc == 42) out[0] = acc;
}

template <int MODE>
static double run(int blocks, int spread) {
  unsigned long long* d;
  hipMalloc(&d, 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k_lds<MODE><<<blocks, 512>>>(d, spread);
  hipEventRecord(a);
  for (int r = 0; r < 5; r++) k_lds<MODE><<<blocks, 512>>>(d, spread);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  hipFree(d);
  const double ops = 5.0 * blocks * 512.0 * ITERS * 4;
  return ops / (ms * 1e-3);
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  const double hz = clk * 1e3;
  const char* names[] = {"u32 add (no ret)", "u32 max (no ret)", "u64 CAS (ret)", "u64 read", "u64 add (ret)"};
  for (int spread : {4096, 1024, 64}) {
    for (int m = 0; m < 5; m++) {
      double r = 0;
      const int blocks = ncu * 4;
      switch (m) {
        case 0: r = run<0>(blocks, spread); break;
        case 1: r = run<1>(blocks, spread); break;
        case 2: r = run<2>(blocks, spread); break;
        case 3: r = run<3>(blocks, spread); break;
        case 4: r = run<4>(blocks, spread); break;
      }
      printf("spread %5d  %-18s %8.2f Gop/s  %6.2f lane-ops/clk/CU\n", spread, names[m], r / 1e9, r / ncu / hz);
    }
  }
  return 0;
}
