// gather_bench.hip — the ceiling of the gossip merge's memory pattern on MI355X: uniformly random
// 8-B gathers (and scatters) over a table the size of cfg 5's views (137 GB), the access every
// gossip record-merge makes to its receiver's view slot. Reports gathers/s and the bytes the
// HBM must move for them, to calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE for this pattern
// (MI355X_MICROARCH.md: "FETCH/WRITE are uncalibrated for scattered 8-B accesses").
//
//   hipcc --offload-arch=gfx950 -O3 -o gather_bench gather_bench.hip
//   ./gather_bench [table_GB=137] [accesses_M=256]
//
// Kernels (one 64-bit access per lane per step; ILP independent accesses in flight per lane):
//   gather<ILP>   : v = table[h(i)], xor-accumulated (one 8-B load per access)
//   scatter<ILP>  : table[h(i)] = i (one 8-B store per access)
//   rmw<ILP>      : table[h(i)] = max(table[h(i)], i) (load then dependent store: a merge)
//   gather_run16  : 16 adjacent words per random start (a packet's records of one owner)
// The printed JSON line per kernel has: accesses, ms, accesses/s, GB/s of useful 8-B words, and
// GB/s if every access moved a 64-B or 128-B line.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHK(x)                                                                       \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t pick(uint64_t i, uint64_t n) { return __umul64hi(mix(i), n); }

template <int ILP>
__global__ __launch_bounds__(256) void k_gather(const uint64_t *t, uint64_t n, uint64_t steps, uint64_t *out) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
  uint64_t acc = 0;
  for (uint64_t s = 0; s < steps; s++) {
    uint64_t v[ILP];
#pragma unroll
    for (int k = 0; k < ILP; k++) v[k] = t[pick((s * ILP + k) * nt + tid, n)];
#pragma unroll
    for (int k = 0; k < ILP; k++) acc ^= v[k];
  }
  if (acc == 0x12345) out[tid] = acc;  // keeps the loads alive
}
template <int ILP>
__global__ __launch_bounds__(256) void k_scatter(uint64_t *t, uint64_t n, uint64_t steps) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t s = 0; s < steps; s++)
#pragma unroll
    for (int k = 0; k < ILP; k++) {
      const uint64_t i = (s * ILP + k) * nt + tid;
      t[pick(i ^ 0x5555, n)] = i;
    }
}
template <int ILP>
__global__ __launch_bounds__(256) void k_rmw(uint64_t *t, uint64_t n, uint64_t steps) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t s = 0; s < steps; s++) {
    uint64_t idx[ILP], v[ILP];
#pragma unroll
    for (int k = 0; k < ILP; k++) {
      idx[k] = pick(((s * ILP + k) * nt + tid) ^ 0xAAAA, n);
      v[k] = t[idx[k]];
    }
#pragma unroll
    for (int k = 0; k < ILP; k++) {
      const uint64_t i = (s * ILP + k) * nt + tid;
      if (i > v[k]) t[idx[k]] = i;
    }
  }
}
// 16 adjacent words per start: 4 lanes x 4 words... here one lane reads a 16-word run as 8 16-B loads
__global__ __launch_bounds__(256) void k_gather_run16(const uint64_t *t, uint64_t n, uint64_t steps, uint64_t *out) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
  // a group of 16 lanes reads one 16-word run (128 B), one word per lane: coalesced into one line
  const uint64_t grp = tid / 16, lane = tid % 16;
  uint64_t acc = 0;
  for (uint64_t s = 0; s < steps; s++) {
    const uint64_t base = pick(s * (nt / 16) + grp, n / 16) * 16;
    acc ^= t[base + lane];
  }
  if (acc == 0x12345) out[tid] = acc;
}

int main(int argc, char **argv) {
  const double gb = argc > 1 ? atof(argv[1]) : 137.0;
  const double acc_m = argc > 2 ? atof(argv[2]) : 256.0;
  const uint64_t n = (uint64_t)(gb * 1e9 / 8.0);
  uint64_t *t = nullptr, *out = nullptr;
  CHK(hipMalloc(&t, n * 8));
  CHK(hipMemset(t, 0, n * 8));
  const int blocks = 256 * 64, threads = 256;  // 64 blocks per CU
  const uint64_t nt = (uint64_t)blocks * threads;
  CHK(hipMalloc(&out, nt * 8));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  auto run = [&](const char *name, int ilp, auto launch) {
    uint64_t steps = (uint64_t)(acc_m * 1e6 / (double)(nt * ilp));
    if (!steps) steps = 1;
    launch(steps);  // warm-up
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a));
    launch(steps);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    const double acc = (double)steps * nt * ilp * (strcmp(name, "gather_run16") == 0 ? 1.0 : 1.0);
    const double per_s = acc / (ms * 1e-3);
    printf("{\"kernel\": \"%s\", \"ilp\": %d, \"table_GB\": %.1f, \"accesses\": %.0f, \"ms\": %.3f, "
           "\"accesses_per_s\": %.4e, \"useful_GBps\": %.1f, \"GBps_if_64B\": %.1f, \"GBps_if_128B\": %.1f}\n",
           name, ilp, gb, acc, ms, per_s, per_s * 8 / 1e9, per_s * 64 / 1e9, per_s * 128 / 1e9);
    fflush(stdout);
  };
  run("gather", 1, [&](uint64_t s) { k_gather<1><<<blocks, threads>>>(t, n, s, out); });
  run("gather", 4, [&](uint64_t s) { k_gather<4><<<blocks, threads>>>(t, n, s, out); });
  run("gather", 8, [&](uint64_t s) { k_gather<8><<<blocks, threads>>>(t, n, s, out); });
  run("gather", 16, [&](uint64_t s) { k_gather<16><<<blocks, threads>>>(t, n, s, out); });
  run("scatter", 1, [&](uint64_t s) { k_scatter<1><<<blocks, threads>>>(t, n, s); });
  run("scatter", 8, [&](uint64_t s) { k_scatter<8><<<blocks, threads>>>(t, n, s); });
  run("rmw", 1, [&](uint64_t s) { k_rmw<1><<<blocks, threads>>>(t, n, s); });
  run("rmw", 8, [&](uint64_t s) { k_rmw<8><<<blocks, threads>>>(t, n, s); });
  run("gather_run16", 1, [&](uint64_t s) { k_gather_run16<<<blocks, threads>>>(t, n, s, out); });
  CHK(hipFree(t));
  CHK(hipFree(out));
  return 0;
}
