// gx_sort.hip — device radix sorts for the catalog readers (EachServiceSorted, ByService).
// rocPRIM's LSD radix sort is stable, which the readers rely on: records enter in key order, so
// equal sort keys leave in key order. A separate translation unit keeps rocPRIM's headers out of
// the engine's build.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocprim/device/device_radix_sort.hpp>

#define GX_HIDDEN __attribute__((visibility("hidden")))

// keys_in/vals_in are consumed; results in keys_out/vals_out. tmp = nullptr queries *tmp_bytes.
extern "C" GX_HIDDEN int gx_sort_u64_pairs(void *tmp, size_t *tmp_bytes, uint64_t *keys_in, uint64_t *keys_out,
                                           uint32_t *vals_in, uint32_t *vals_out, uint32_t n, int end_bit,
                                           hipStream_t s) {
  return (int)rocprim::radix_sort_pairs(tmp, *tmp_bytes, keys_in, keys_out, vals_in, vals_out, n, 0, end_bit, s);
}
extern "C" GX_HIDDEN int gx_sort_u32_pairs(void *tmp, size_t *tmp_bytes, uint32_t *keys_in, uint32_t *keys_out,
                                           uint32_t *vals_in, uint32_t *vals_out, uint32_t n, int end_bit,
                                           hipStream_t s) {
  return (int)rocprim::radix_sort_pairs(tmp, *tmp_bytes, keys_in, keys_out, vals_in, vals_out, n, 0, end_bit, s);
}
