// kma_distance.h — launchers of the ProteinKmers.distance kernels (kma_distance.hip), used by
// kma_abi.cpp. Not part of the public ABI (see include/kmeranno.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kma {
hipError_t launch_window_keys(const uint8_t* res, const uint64_t* off, uint32_t n, int k,
                              int end_exclusive, uint64_t* keys, uint32_t* alpha, hipStream_t s);
hipError_t launch_segmented_sort(void* temp, size_t* temp_bytes, const uint64_t* in,
                                 uint64_t* out, uint64_t n_items, uint32_t n_seg,
                                 const uint64_t* seg_begin, const uint64_t* seg_end, int bits,
                                 hipStream_t s);
hipError_t launch_distinct(const uint64_t* sorted, const uint64_t* off, uint32_t n, uint32_t* size,
                           hipStream_t s);
hipError_t launch_pairs(const uint64_t* sa, const uint64_t* offa, const uint32_t* size_a,
                        const uint64_t* sb, const uint64_t* offb, const uint32_t* size_b,
                        const uint32_t* pa, const uint32_t* pb, uint64_t n_pairs, uint32_t* sim,
                        hipStream_t s);
}  // namespace kma
