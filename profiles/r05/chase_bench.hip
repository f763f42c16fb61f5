// Dependent-load latency and random-access throughput against table size on one MI355X:
// how much of a gossip round's dependent chain is address translation (TLB reach) rather than
// DRAM. Each lane walks its own chain of 8-B loads; hop k's address depends on hop k-1's value.
//   mode "any":  every hop lands anywhere in the table (a new 2 MiB page almost every hop)
//   mode "page": every hop stays inside the lane's own 2 MiB region (after the first)
// Latency: 1 wave (64 chains). Throughput: `waves` waves. Prints one JSON line per case.
//   hipcc --offload-arch=gfx950 -O3 -o chase_bench chase_bench.hip && ./chase_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__device__ __host__ inline uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void fill(uint64_t *t, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    t[i] = mix(i);
}

// page: region of 2 MiB (262144 words) per chain
__global__ void chase(const uint64_t *t, uint64_t n, int hops, int page, unsigned long long *sink) {
  const uint64_t gid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t x = mix(gid * 0x51ED27ull + 1);
  const uint64_t region = 262144ull;
  const uint64_t nreg = n / region;
  const uint64_t base = page ? (mix(gid) % nreg) * region : 0;
  uint64_t acc = 0;
  for (int k = 0; k < hops; k++) {
    const uint64_t idx = page ? base + (x % region) : (x % n);
    const uint64_t v = __builtin_nontemporal_load(&t[idx]);
    acc += v;
    x = mix(v ^ x);
  }
  if (acc == 0x12345) sink[0] = acc;
}

int main(int argc, char **argv) {
  const double sizes_gb[] = {0.25, 4.0, 32.0, 137.0};
  const int waves_tp = argc > 1 ? atoi(argv[1]) : 16384;
  uint64_t max_n = (uint64_t)(137.0 * (1ull << 30)) / 8;
  uint64_t *t;
  CK(hipMalloc(&t, max_n * 8));
  unsigned long long *sink;
  CK(hipMalloc(&sink, 8));
  fill<<<4096, 256>>>(t, max_n);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (double gb : sizes_gb) {
    const uint64_t n = (uint64_t)(gb * (1ull << 30)) / 8;
    for (int page = 0; page < 2; page++) {
      if (page && n < 262144ull * 4) continue;
      for (int tp = 0; tp < 2; tp++) {
        const int blocks = tp ? waves_tp : 1;
        const int hops = tp ? 64 : 256;
        chase<<<blocks, 64>>>(t, n, 8, page, sink);  // warm the code path
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        chase<<<blocks, 64>>>(t, n, hops, page, sink);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        const double loads = (double)blocks * 64 * hops;
        printf("{\"table_GB\": %.2f, \"mode\": \"%s\", \"waves\": %d, \"hops\": %d, \"ms\": %.3f, "
               "\"ns_per_hop\": %.1f, \"loads_per_s\": %.4g}\n",
               gb, page ? "page" : "any", blocks, hops, ms, 1e6 * ms / hops, loads / (ms * 1e-3));
        fflush(stdout);
      }
    }
  }
  CK(hipFree(t));
  return 0;
}
