// gp_sort.hip — the one library sort of libgp_reduce.so: hipCUB's (rocPRIM)
// radix sort of (u32 key, u32 value) pairs, used to build the destination-
// sorted residual of an unplanned scatter's index once (gp_reduce.hip, the
// unplanned calls' plan cache).  Its own translation unit: the template-heavy
// header takes most of the library's compile time.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <string>

#include "gp_reduce.h"

int gp_internal_radix_sort_pairs_u32(const uint32_t *keys_in, uint32_t *keys_out, const uint32_t *vals_in,
                                     uint32_t *vals_out, size_t n, int end_bit, hipStream_t s,
                                     std::string *error) {
  if (n == 0) return GP_OK;
  if (n > (size_t)INT32_MAX) {
    *error = "radix sort: more than 2^31 rows";
    return GP_ERR_UNSUPPORTED;
  }
  size_t temp_bytes = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, keys_in, keys_out, vals_in, vals_out,
                                                    (int)n, 0, end_bit, s);
  void *temp = nullptr;
  if (e == hipSuccess) e = hipMallocAsync(&temp, temp_bytes, s);
  if (e == hipSuccess)
    e = hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, vals_in, vals_out, (int)n, 0,
                                           end_bit, s);
  if (temp) {
    const hipError_t f = hipFreeAsync(temp, s);
    if (e == hipSuccess) e = f;
  }
  if (e != hipSuccess) {
    *error = std::string("radix sort: ") + hipGetErrorString(e);
    return GP_ERR_HIP;
  }
  return GP_OK;
}
