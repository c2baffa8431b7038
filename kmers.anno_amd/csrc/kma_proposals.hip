// kma_proposals.hip — the projector's proposal sweep on the device (§8(f)2).
//
// KmerProcessor.annotateGenome (KmerProcessor.java:209-264): the peg join's connections
// (kma_connect_pegs) are grouped into framed location lists (FramedLocationLists.connect,
// FramedLocationLists.java:156-171: one list per frame and peg, sorted by contig and left), and
// every start i of every list long enough to reach minKmers is swept: evidence = 1 + the
// locations after i on i's contig whose right edge is below left_i + maxLen, best edge = the
// largest such right edge. The Java loop is O(size^2) per list; here each start is one thread
// and, as all kmer locations have the same length (3K), the qualifying locations are a prefix of
// i's contig run, found by two binary searches: O(log size) per start.
//
//   prop_keys    list key (frame * n_peg + peg) per connection
//   radix sort   stable: connections arrive in canonical (contig, left) order, so each list
//                comes out sorted as SortedLocationList keeps it
//   prop_heads / scan / prop_starts   list boundaries
//   prop_sweep   one thread per start: evidence, best edge, the too-short test
//   scan / prop_emit                  proposals in list order
//
// Restated external semantics (Location, Frame, SortedLocationList are not in the reference)
// are those of oracle/kma_oracle.c orc_propose.
#include <cstring>  // (rocprim.hpp uses memset without including it)
#include <rocprim/rocprim.hpp>

#include "../../include/kmeranno.h"
#include "kma_internal.h"
#include "kma_device.h"

namespace kma {
namespace {

__device__ __forceinline__ uint32_t frame_index(uint8_t strand, int32_t left, int k) {
  const int32_t end = strand == '+' ? left + 3 * k - 1 : left;  // Location.getFrame (restated)
  return (strand == '+' ? 3u : 0u) + (uint32_t)(end % 3);
}

__global__ __launch_bounds__(256) void prop_keys_kernel(PropArgs a) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < a.n; i += gridDim.x * 256u) {
    const kma_hit h = a.hits[i];
    a.keys[i] = frame_index(h.strand, h.left, a.k) * a.n_peg + h.fid;
    a.idx[i] = i;
  }
}

// Sorted connections: list heads (flag), contig / left gathered for the sweep's searches.
__global__ __launch_bounds__(256) void prop_heads_kernel(PropArgs a) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < a.n; i += gridDim.x * 256u) {
    a.head[i] = (i == 0 || a.skeys[i] != a.skeys[i - 1]) ? 1u : 0u;
    const kma_hit h = a.hits[a.sidx[i]];
    a.scontig[i] = h.contig;
    a.sleft[i] = h.left;
  }
}

// list_no[i] = inclusive count of heads; starts[list] = its first position, starts[lists] = n.
__global__ __launch_bounds__(256) void prop_starts_kernel(PropArgs a) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < a.n; i += gridDim.x * 256u) {
    if (a.head[i]) a.starts[a.list_no[i] - 1] = i;
    if (i + 1 == a.n) a.starts[a.list_no[i]] = a.n;
  }
}

// Largest j in [lo, hi) with v[j] <= x (v non-decreasing on [lo, hi), v[lo] <= x).
template <typename T>
__device__ __forceinline__ uint32_t last_le(const T* v, uint32_t lo, uint32_t hi, T x) {
  while (hi - lo > 1) {
    const uint32_t mid = lo + ((hi - lo) >> 1);
    if (v[mid] <= x) lo = mid; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ void count_wave(uint64_t* stat, bool pred) {
  const uint64_t m = __ballot(pred);
  if (m && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(m)) atomicAdd((unsigned long long*)stat, (unsigned long long)__popcll(m));
}

__global__ __launch_bounds__(256) void prop_sweep_kernel(PropArgs a) {
  const int32_t span = 3 * a.k - 1;
  const double real_strength = a.min_strength / 3;
  const uint32_t n_iter = (a.n + 255u) / 256u * 256u;  // every lane reaches the ballots
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n_iter; i += gridDim.x * 256u) {
    const bool live = i < a.n;
    bool head = false, too_few = false, too_short = false, keep = false;
    uint32_t evidence = 0;
    int32_t best = 0;
    if (live) {
      const uint32_t l = a.list_no[i] - 1, s = a.starts[l], e = a.starts[l + 1];
      const int64_t size = (int64_t)(e - s), pos = (int64_t)(i - s);
      const uint32_t peg = a.skeys[i] % a.n_peg;
      const int32_t peg_bp = (int32_t)a.peg_len[peg] * 3;
      const int32_t max_len = (int32_t)(peg_bp * a.max_fuzz + 1);
      const int32_t min_len = (int32_t)(peg_bp * a.min_fuzz);
      const int32_t min_kmers = (int32_t)(peg_bp * real_strength);
      head = pos == 0;
      too_few = head && min_kmers > size;
      if (min_kmers <= size && pos <= size - min_kmers && pos < size) {
        const uint32_t c = a.scontig[i];
        const int32_t left = a.sleft[i];
        const uint32_t ce = last_le(a.scontig, i, e, c) + 1;  // i's contig run is [i, ce)
        // contigRange(i) locations with right < left + maxLen: left_j <= left + maxLen - span - 1
        const int64_t lim = (int64_t)left + max_len - span - 1;
        uint32_t jm = i;
        if (ce > i + 1 && (int64_t)a.sleft[i + 1] <= lim)
          jm = last_le(a.sleft, i + 1, ce, (int32_t)(lim > INT32_MAX ? INT32_MAX : lim));
        evidence = 1u + (jm - i);
        best = a.sleft[jm] + span;
        too_short = best < left + min_len;
        keep = !too_short;
      }
    }
    count_wave(a.stats + 0, head);
    count_wave(a.stats + 1, too_few);
    count_wave(a.stats + 2, too_short);
    count_wave(a.stats + 3, keep);
    if (live) {
      a.keep[i] = keep ? 1u : 0u;
      a.evidence[i] = evidence;
      a.best[i] = best;
    }
  }
}

__global__ __launch_bounds__(256) void prop_emit_kernel(PropArgs a) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < a.n; i += gridDim.x * 256u) {
    if (!a.keep[i]) continue;
    const uint64_t o = a.out_pos[i];
    if (o >= a.cap) continue;
    const kma_hit h = a.hits[a.sidx[i]];
    kma_proposal p;
    p.peg = h.fid;
    p.contig = h.contig;
    p.left = h.left;
    p.right = a.best[i];
    p.evidence = a.evidence[i];
    p.strand = h.strand;
    p.frame = (uint8_t)(a.skeys[i] / a.n_peg);
    p.pad = 0;
    a.out[o] = p;
  }
}

unsigned grid_of(uint64_t n) {
  const uint64_t g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

}  // namespace

// The whole sweep on `stream`; a.stats (4 u64) must be zeroed before. Scratch sizes: see
// kma_abi.cpp (kma_propose_pegs). temp == nullptr: *temp_bytes = the sort / scan scratch.
hipError_t launch_propose(PropArgs a, void* temp, size_t* temp_bytes, hipStream_t stream) {
  const size_t n = a.n;
  const rocprim::plus<uint32_t> add;
  if (!temp) {
    size_t s1 = 0, s2 = 0, s3 = 0;
    hipError_t e = rocprim::radix_sort_pairs(nullptr, s1, a.keys, a.skeys, a.idx, a.sidx, n, 0u,
                                             32u, stream);
    if (e != hipSuccess) return e;
    e = rocprim::inclusive_scan(nullptr, s2, a.head, a.list_no, n, add, stream);
    if (e != hipSuccess) return e;
    e = rocprim::exclusive_scan(nullptr, s3, a.keep, a.out_pos, 0u, n, add, stream);
    if (e != hipSuccess) return e;
    *temp_bytes = std::max(s1, std::max(s2, s3));
    return hipSuccess;
  }
  const unsigned g = grid_of(a.n);
  hipLaunchKernelGGL(prop_keys_kernel, dim3(g), dim3(256), 0, stream, a);
  size_t tb = *temp_bytes;
  hipError_t e = rocprim::radix_sort_pairs(temp, tb, a.keys, a.skeys, a.idx, a.sidx, n, 0u, 32u,
                                           stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(prop_heads_kernel, dim3(g), dim3(256), 0, stream, a);
  tb = *temp_bytes;
  e = rocprim::inclusive_scan(temp, tb, a.head, a.list_no, n, add, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(prop_starts_kernel, dim3(g), dim3(256), 0, stream, a);
  hipLaunchKernelGGL(prop_sweep_kernel, dim3(g), dim3(256), 0, stream, a);
  tb = *temp_bytes;
  e = rocprim::exclusive_scan(temp, tb, a.keep, a.out_pos, 0u, n, add, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(prop_emit_kernel, dim3(g), dim3(256), 0, stream, a);
  return hipGetLastError();
}

}  // namespace kma
