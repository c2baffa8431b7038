// kma_distance.hip — ProteinKmers.distance on the GPU.
//
// GeneCopyProcessor.runCommand (genome/compare/GeneCopyProcessor.java:129-162) compares every
// target peg's ProteinKmers with those of the source pegs of the same function and keeps the
// closest one within maxDist. ProteinKmers (external org.theseed.sequence, restated): the SET
// of distinct length-K substrings at i = 0 .. L-K; distance = 1 - |A n B| / |A u B| (Jaccard),
// 1.0 when the sets share nothing.
//
// GPU form, for batches of proteins and any protein length:
//   window_keys_kernel  every window of every protein packed to a 5K-bit key (K <= 12) at its
//                       residue position; positions that start no window hold the sentinel
//   (rocPRIM) segmented radix sort of each protein's positions
//   distinct_kernel     |S| per protein: first occurrences of non-sentinel keys (wave per protein)
//   pair_kernel         per (a, b) pair: the distinct keys of the smaller set, each looked up by
//                       binary search in the other's sorted keys (wave per pair, lanes stride)
// Integer work only; outputs are (|A|, |B|, |A n B|) per pair, the host forms the distance in
// double exactly as the restated Java expression.
#include <cstring>  // (rocprim.hpp uses memset without including it)
#include <rocprim/rocprim.hpp>

#include "kma_distance.h"

namespace kma {
namespace {

constexpr uint64_t kSentinel = ~0ull;

__device__ __forceinline__ uint32_t dwave_sum(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
  return v;
}

// Wave per protein: keys[p] for every residue position p of protein s (relative to off[0]);
// a window starts at i < n_win(s) = L - K + 1 (or L - K with end_exclusive). A byte outside
// A-Z / '*' in a window raises *alpha (the caller refuses the batch).
__global__ __launch_bounds__(256) void window_keys_kernel(const uint8_t* __restrict__ res,
                                                          const uint64_t* __restrict__ off,
                                                          uint32_t n, int k, int end_exclusive,
                                                          uint64_t* __restrict__ keys,
                                                          uint32_t* __restrict__ alpha) {
  __shared__ uint8_t lut[256];
  const int t = threadIdx.x;
  lut[t] = (t >= 'A' && t <= 'Z') ? (uint8_t)(t - 'A' + 1) : (t == '*' ? 27 : 0);
  __syncthreads();
  const uint32_t lane = t & 63;
  const uint64_t o0 = off[0];
  for (uint64_t s = (uint64_t)blockIdx.x * 4 + (t >> 6); s < n; s += (uint64_t)gridDim.x * 4) {
    const uint64_t lo = off[s], hi = off[s + 1];
    const int64_t n_win = (int64_t)(hi - lo) - k + (end_exclusive ? 0 : 1);
    bool bad = false;
    for (uint64_t p = lo + lane; p < hi; p += 64) {
      const int64_t i = (int64_t)(p - lo);
      uint64_t key = kSentinel;
      if (i < n_win) {
        uint64_t v = 0;
        bool ok = true;
        for (int j = 0; j < k; ++j) {
          const uint32_t c = lut[res[p + j]];
          ok = ok && c != 0u;
          v = (v << 5) | c;
        }
        bad = bad || !ok;
        key = v;
      }
      keys[p - o0] = key;
    }
    if (__ballot(bad) && lane == 0) atomicOr(alpha, 1u);
  }
}

// Wave per protein: distinct non-sentinel keys of its sorted segment.
__global__ __launch_bounds__(256) void distinct_kernel(const uint64_t* __restrict__ sorted,
                                                       const uint64_t* __restrict__ off,
                                                       uint32_t n, uint32_t* __restrict__ size) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t o0 = off[0];
  for (uint64_t s = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); s < n;
       s += (uint64_t)gridDim.x * 4) {
    const uint64_t lo = off[s] - o0, hi = off[s + 1] - o0;
    uint32_t c = 0;
    for (uint64_t p = lo + lane; p < hi; p += 64) {
      const uint64_t v = sorted[p];
      c += (v != kSentinel && (p == lo || sorted[p - 1] != v)) ? 1u : 0u;
    }
    c = dwave_sum(c);
    if (lane == 0) size[s] = c;
  }
}

// First index in [lo, hi) with key >= v.
__device__ __forceinline__ uint64_t lower_bound(const uint64_t* __restrict__ a, uint64_t lo,
                                                uint64_t hi, uint64_t v) {
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Wave per pair: |A n B| by looking up the distinct keys of the smaller set in the larger.
__global__ __launch_bounds__(256) void pair_kernel(const uint64_t* __restrict__ sa,
                                                   const uint64_t* __restrict__ offa,
                                                   const uint32_t* __restrict__ size_a,
                                                   const uint64_t* __restrict__ sb,
                                                   const uint64_t* __restrict__ offb,
                                                   const uint32_t* __restrict__ size_b,
                                                   const uint32_t* __restrict__ pa,
                                                   const uint32_t* __restrict__ pb,
                                                   uint64_t n_pairs, uint32_t* __restrict__ sim) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t a0 = offa[0], b0 = offb[0];
  for (uint64_t q = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); q < n_pairs;
       q += (uint64_t)gridDim.x * 4) {
    const uint32_t ia = pa[q], ib = pb[q];
    // segments; distinct keys come first in sort order, sentinels last
    const uint64_t* s1 = sa;
    uint64_t lo1 = offa[ia] - a0, hi1 = offa[ia + 1] - a0;
    const uint64_t* s2 = sb;
    uint64_t lo2 = offb[ib] - b0, hi2 = offb[ib + 1] - b0;
    if (size_a[ia] > size_b[ib]) {  // scan the smaller set
      const uint64_t* ts = s1; s1 = s2; s2 = ts;
      uint64_t t0 = lo1; lo1 = lo2; lo2 = t0;
      t0 = hi1; hi1 = hi2; hi2 = t0;
    }
    uint32_t c = 0;
    for (uint64_t p = lo1 + lane; p < hi1; p += 64) {
      const uint64_t v = s1[p];
      if (v == kSentinel || (p > lo1 && s1[p - 1] == v)) continue;
      const uint64_t j = lower_bound(s2, lo2, hi2, v);
      c += (j < hi2 && s2[j] == v) ? 1u : 0u;
    }
    c = dwave_sum(c);
    if (lane == 0) sim[q] = c;
  }
}

unsigned grid_waves(uint64_t n) {
  const uint64_t g = (n + 3) / 4;
  return (unsigned)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

}  // namespace

hipError_t launch_window_keys(const uint8_t* res, const uint64_t* off, uint32_t n, int k,
                              int end_exclusive, uint64_t* keys, uint32_t* alpha,
                              hipStream_t s) {
  hipLaunchKernelGGL(window_keys_kernel, dim3(grid_waves(n)), dim3(256), 0, s, res, off, n, k,
                     end_exclusive, keys, alpha);
  return hipGetLastError();
}

hipError_t launch_segmented_sort(void* temp, size_t* temp_bytes, const uint64_t* in,
                                 uint64_t* out, uint64_t n_items, uint32_t n_seg,
                                 const uint64_t* seg_begin, const uint64_t* seg_end, int bits,
                                 hipStream_t s) {
  return rocprim::segmented_radix_sort_keys(temp, *temp_bytes, in, out, (unsigned)n_items, n_seg,
                                            seg_begin, seg_end, 0u, (unsigned)bits, s);
}

hipError_t launch_distinct(const uint64_t* sorted, const uint64_t* off, uint32_t n, uint32_t* size,
                           hipStream_t s) {
  hipLaunchKernelGGL(distinct_kernel, dim3(grid_waves(n)), dim3(256), 0, s, sorted, off, n, size);
  return hipGetLastError();
}

hipError_t launch_pairs(const uint64_t* sa, const uint64_t* offa, const uint32_t* size_a,
                        const uint64_t* sb, const uint64_t* offb, const uint32_t* size_b,
                        const uint32_t* pa, const uint32_t* pb, uint64_t n_pairs, uint32_t* sim,
                        hipStream_t s) {
  hipLaunchKernelGGL(pair_kernel, dim3(grid_waves(n_pairs)), dim3(256), 0, s, sa, offa, size_a,
                     sb, offb, size_b, pa, pb, n_pairs, sim);
  return hipGetLastError();
}

}  // namespace kma
