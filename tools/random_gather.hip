// random_gather.hip — the random-access ceiling a hash probe runs against (C4's general path).
//
// Reads `n` uniformly random `W`-byte words (W = 8 .. 128, W-aligned) from a table of `bytes`, each thread
// issuing R independent loads before using any (memory-level parallelism), and reports loads/s.
// Table sizes span the MALL (256 MB) to C4's 8.6 GB slot table; the keys are a splitmix64 stream
// hashed to slots, as k_probe does.  Build: hipcc -O3 --offload-arch=gfx950 -o random_gather
// random_gather.hip; run on the GPU: ./random_gather > out.txt
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  x ^= x >> 31;
  return x;
}

template <int W, int R>
__global__ __launch_bounds__(256) void k_gather(const uint64_t* __restrict__ table, uint64_t slots, int64_t n,
                                                uint64_t seed, unsigned long long* __restrict__ sink) {
  constexpr int WW = W / 8;
  const int64_t base = (int64_t)blockIdx.x * 256 * R;
  uint64_t acc = 0;
  uint64_t v[R][WW];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int64_t i = base + r * 256 + threadIdx.x;
    const uint64_t slot = __umul64hi(mix(seed + (uint64_t)(i < n ? i : 0)), slots);  // uniform over any size
    const uint64_t* p = table + slot * WW;
#pragma unroll
    for (int w = 0; w < WW; w++) v[r][w] = p[w];
  }
#pragma unroll
  for (int r = 0; r < R; r++)
#pragma unroll
    for (int w = 0; w < WW; w++) acc ^= v[r][w];
  if (acc == 0x123456789ULL) atomicAdd(sink, 1ULL);  // keeps the loads live; never true in practice
}

template <int W, int R>
static double run(const uint64_t* table, uint64_t slots, int64_t n, unsigned long long* sink) {
  const int64_t blocks = (n + 256 * R - 1) / (256 * R);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k_gather<W, R>), dim3(blocks), dim3(256), 0, 0, table, slots, n, 1ULL, sink);
  hipEventRecord(e0, 0);
  const int reps = 3;
  for (int k = 0; k < reps; k++)
    hipLaunchKernelGGL((k_gather<W, R>), dim3(blocks), dim3(256), 0, 0, table, slots, n, 7ULL + k, sink);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return (double)n * reps / (ms / 1000.0);
}

int main(int argc, char** argv) {
  const int64_t n = 200000000;
  unsigned long long* sink;
  hipMalloc(&sink, 8);
  // table sizes (MB) from the command line, default the MALL (256 MB) to C4's slot table
  std::vector<uint64_t> sizes = {256ULL << 20, 1ULL << 30, 4ULL << 30, 8ULL << 30};
  if (argc > 1) {
    sizes.clear();
    for (int a = 1; a < argc; a++) sizes.push_back((uint64_t)atoll(argv[a]) << 20);
  }
  printf("table_bytes,word_bytes,loads_per_thread,loads_per_s\n");
  for (uint64_t bytes : sizes) {
    uint64_t* table = nullptr;
    if (hipMalloc(&table, bytes) != hipSuccess) {
      printf("%llu,alloc failed\n", (unsigned long long)bytes);
      continue;
    }
    hipMemset(table, 1, bytes);
    printf("%llu,8,4,%.4g\n", (unsigned long long)bytes, run<8, 4>(table, bytes / 8, n, sink));
    printf("%llu,8,16,%.4g\n", (unsigned long long)bytes, run<8, 16>(table, bytes / 8, n, sink));
    printf("%llu,16,4,%.4g\n", (unsigned long long)bytes, run<16, 4>(table, bytes / 16, n, sink));
    printf("%llu,16,16,%.4g\n", (unsigned long long)bytes, run<16, 16>(table, bytes / 16, n, sink));
    printf("%llu,32,4,%.4g\n", (unsigned long long)bytes, run<32, 4>(table, bytes / 32, n, sink));
    printf("%llu,32,8,%.4g\n", (unsigned long long)bytes, run<32, 8>(table, bytes / 32, n, sink));
    printf("%llu,64,2,%.4g\n", (unsigned long long)bytes, run<64, 2>(table, bytes / 64, n, sink));
    printf("%llu,64,4,%.4g\n", (unsigned long long)bytes, run<64, 4>(table, bytes / 64, n, sink));
    printf("%llu,128,2,%.4g\n", (unsigned long long)bytes, run<128, 2>(table, bytes / 128, n, sink));
    fflush(stdout);
    hipFree(table);
  }
  hipFree(sink);
  return 0;
}
