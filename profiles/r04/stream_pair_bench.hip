// stream_pair_bench.hip — what a push-pull round can reach on MI355X: one 256-thread block per
// host pair streams both 4 MB rows of a 137 GB view table (cfg 5: 32768 rows x 524288 words, 16384
// pairs) and folds them (max of the words, the merge's data flow without its bookkeeping). Variants:
//   reg_pf1   : 16-B nontemporal loads into registers, the next 1024-word tile in flight (k_ae's shape)
//   reg_pf2   : two tiles in flight
//   glds_ring : LDS-DMA (global_load_lds_dwordx4, nontemporal) into a ring of NBUF tiles per block,
//               counted vmcnt + raw barriers, the block reads its words back from LDS
// Prints one JSON line per variant: ms, GB/s of the 137 GB read.
//
//   hipcc --offload-arch=gfx950 -O3 -o stream_pair_bench stream_pair_bench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                              \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2u64 ldnt(const uint64_t *p) { return __builtin_nontemporal_load(reinterpret_cast<const v2u64 *>(p)); }

// BAR: one __syncthreads_or per tile (k_ae's retransmit check); ALU: the merge rule's compares
// PERM: the pair's rows are scattered over the table like k_ae's seeded pairing (odd-multiplier
// permutation of the row numbers, H a power of two) instead of adjacent
template <int PF, bool BAR = false, bool ALU = false, bool PERM = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_reg(const uint64_t *t, uint32_t R,
                                                                                      uint64_t *out) {
  const uint32_t H = 2 * gridDim.x, ra = PERM ? (2 * blockIdx.x * 0x9E3779B1u + 12345u) & (H - 1) : 2 * blockIdx.x;
  const uint32_t rb = PERM ? ((2 * blockIdx.x + 1) * 0x9E3779B1u + 12345u) & (H - 1) : ra + 1;
  const uint64_t *A = t + (size_t)ra * R, *B = t + (size_t)rb * R;
  const uint32_t tid = threadIdx.x;
  v2u64 qa[PF][2], qb[PF][2];
  auto load = [&](uint32_t base, v2u64 *xa, v2u64 *xb) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t r0 = base + 512 * h + 2 * tid;
      xa[h] = ldnt(&A[r0]);
      xb[h] = ldnt(&B[r0]);
    }
  };
#pragma unroll
  for (int s = 0; s < PF; s++) load(1024u * s, qa[s], qb[s]);
  uint64_t acc = 0;
  for (uint32_t base = 0; base < R; base += 1024u * PF) {
#pragma unroll
    for (int s = 0; s < PF; s++) {
      v2u64 wa[2] = {qa[s][0], qa[s][1]}, wb[2] = {qb[s][0], qb[s][1]};
      if (base + 1024u * (PF + s) < R) load(base + 1024u * (PF + s), qa[s], qb[s]);
      uint32_t fl = 0;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        if (ALU) {  // merge_word both ways: stale gate, absent, strictly newer, DRAINING stickiness
          const uint64_t x[2] = {wa[h].x, wa[h].y}, y[2] = {wb[h].x, wb[h].y};
#pragma unroll
          for (int k = 0; k < 2; k++) {
            const int64_t tx = (int64_t)(x[k] >> 3), ty = (int64_t)(y[k] >> 3);
            const bool sx = tx < (int64_t)R, sy = ty < (int64_t)R;
            const bool ax = (y[k] & 7) == 7 || (!sx && tx > ty), ay = (x[k] & 7) == 7 || (!sy && ty > tx);
            const uint64_t nx = ax ? (((y[k] & 7) == 4 && (x[k] & 7) == 0) ? (x[k] & ~7ull) | 4 : x[k]) : y[k];
            const uint64_t ny = ay ? x[k] : y[k];
            acc += (nx != y[k]) + (ny != x[k]) + sx + sy;
            fl |= (uint32_t)(ax | ay) << (2 * h + k);
          }
        } else {
          acc += (wa[h].x > wb[h].x) + (wa[h].y > wb[h].y);
        }
        acc ^= wa[h].x ^ wb[h].y;
      }
      if (BAR && __syncthreads_or(fl != 0 && acc == 0x1234567)) out[blockIdx.x] = 1;
    }
  }
  if (acc == 0x1234567) out[blockIdx.x] = acc;
}

// LDS-DMA ring: tile = 1024 words of A + 1024 of B = 16 KB; each thread's two 16-B pieces per row
// half: 4 global_load_lds_dwordx4 per thread per tile (each wave-instruction writes 1 KB linearly).
template <int NBUF>
__global__ __launch_bounds__(256) void k_glds(const uint64_t *t, uint32_t R, uint64_t *out) {
  __shared__ __attribute__((aligned(16))) uint64_t ring[NBUF][2][1024];
  const uint64_t *A = t + (size_t)(2 * blockIdx.x) * R, *B = A + R;
  const uint32_t tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const uint32_t ntile = R / 1024;
  auto issue = [&](uint32_t tile) {
    const uint32_t b = tile % NBUF;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      // wave wv, half h: words [512h + 128wv, +128) of the tile, 16 B per lane, lane-linear in LDS
      const uint32_t off = 512 * h + 128 * wv;
      __builtin_amdgcn_global_load_lds((const void *)(A + (size_t)tile * 1024 + off + 2 * lane),
                                       (__attribute__((address_space(3))) void *)&ring[b][0][off], 16, 0, 2);
      __builtin_amdgcn_global_load_lds((const void *)(B + (size_t)tile * 1024 + off + 2 * lane),
                                       (__attribute__((address_space(3))) void *)&ring[b][1][off], 16, 0, 2);
    }
  };
#pragma unroll
  for (int s = 0; s < NBUF - 1; s++) issue(s);
  uint64_t acc = 0;
  for (uint32_t tile = 0; tile < ntile; tile++) {
    // the tile's 4 DMAs landed when at most (NBUF - 2) tiles' (4 each) remain in flight
    if (NBUF == 2 || tile + NBUF - 2 >= ntile) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail
    else if (NBUF == 3) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's DMA of this tile landed; the slot read next is free
    if (tile + NBUF - 1 < ntile) issue(tile + NBUF - 1);
    const uint32_t b = tile % NBUF;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t r = 512 * h + 2 * tid;
      const v2u64 wa = *reinterpret_cast<const v2u64 *>(&ring[b][0][r]);
      const v2u64 wb = *reinterpret_cast<const v2u64 *>(&ring[b][1][r]);
      acc += (wa.x > wb.x) + (wa.y > wb.y);
      acc ^= wa.x ^ wb.y;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (acc == 0x1234567) out[blockIdx.x] = acc;
}

int main(int argc, char **argv) {
  const uint32_t H = argc > 1 ? atoi(argv[1]) : 32768, R = argc > 2 ? atoi(argv[2]) : 524288;
  const size_t words = (size_t)H * R;
  uint64_t *t = nullptr, *out = nullptr;
  CHK(hipMalloc(&t, words * 8));
  CHK(hipMemset(t, 1, words * 8));
  CHK(hipMalloc(&out, (H / 2) * 8));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  auto run = [&](const char *name, auto launch) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; rep++) {
      CHK(hipEventRecord(a));
      launch();
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms = 0;
      CHK(hipEventElapsedTime(&ms, a, b));
      if (rep && ms < best) best = ms;
    }
    printf("{\"variant\": \"%s\", \"GB\": %.1f, \"ms\": %.3f, \"GBps\": %.1f}\n", name, words * 8 / 1e9, best,
           words * 8 / 1e9 / (best * 1e-3));
    fflush(stdout);
  };
  run("reg_pf1", [&] { k_reg<1><<<H / 2, 256>>>(t, R, out); });
  run("reg_pf2", [&] { k_reg<2><<<H / 2, 256>>>(t, R, out); });
  run("reg_pf1_bar", [&] { k_reg<1, true><<<H / 2, 256>>>(t, R, out); });
  run("reg_pf1_alu", [&] { k_reg<1, false, true><<<H / 2, 256>>>(t, R, out); });
  run("reg_pf1_alu_bar", [&] { k_reg<1, true, true><<<H / 2, 256>>>(t, R, out); });
  run("reg_pf2_alu_bar", [&] { k_reg<2, true, true><<<H / 2, 256>>>(t, R, out); });
  // k_ae holds 123 VGPRs -> 4 waves/SIMD (4 blocks per CU); the reg kernels above fit 6-8. 36 KB of
  // dynamic LDS per block pins them to 4 blocks per CU, k_ae's residency
  const size_t occ4 = 36 * 1024;
  run("reg_pf1_alu_bar_occ4", [&] { k_reg<1, true, true><<<H / 2, 256, occ4>>>(t, R, out); });
  run("reg_pf2_alu_bar_occ4", [&] { k_reg<2, true, true><<<H / 2, 256, occ4>>>(t, R, out); });
  run("reg_pf1_alu_bar_perm", [&] { k_reg<1, true, true, true><<<H / 2, 256>>>(t, R, out); });
  run("reg_pf1_alu_bar_perm_occ4", [&] { k_reg<1, true, true, true><<<H / 2, 256, occ4>>>(t, R, out); });
  run("reg_pf1_occ4", [&] { k_reg<1><<<H / 2, 256, occ4>>>(t, R, out); });
  run("glds_ring2", [&] { k_glds<2><<<H / 2, 256>>>(t, R, out); });
  run("glds_ring3", [&] { k_glds<3><<<H / 2, 256>>>(t, R, out); });
  run("glds_ring4", [&] { k_glds<4><<<H / 2, 256>>>(t, R, out); });
  CHK(hipFree(t));
  CHK(hipFree(out));
  return 0;
}
