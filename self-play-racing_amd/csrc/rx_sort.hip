// rx_sort.hip -- radix sort of (spatial key, env id) pairs that re-groups the
// envs into spatially coherent wavefronts between k_dyn and k_rays
// (scheduling only; no result depends on the order).  rocPRIM via hipCUB.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "rx_internal.h"

extern "C" int rx_sort_pairs(void* tmp, size_t* tmp_bytes, const uint32_t* kin, uint32_t* kout, const int32_t* vin,
                             int32_t* vout, int n, int end_bit, hipStream_t s) {
  return (int)hipcub::DeviceRadixSort::SortPairs(tmp, *tmp_bytes, kin, kout, vin, vout, n, 0, end_bit, s);
}
