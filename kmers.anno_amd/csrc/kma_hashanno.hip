// kma_hashanno.hip — the hash annotator's scoring loop on the device (§8(f)3).
//
// HashAnnotationProcessor.processGenome (HashAnnotationProcessor.java:221-328): a genome's
// proteins go into a GenomeProteinKmers index (:233-248), every prototype of the role
// annotation file is scored against it in file order (processProposal, :259-271), and each
// protein keeps its best proposal (getProposal, :278-306). GenomeProteinKmers is external
// (org.theseed.proteins.kmers, not in the reference); restated as in oracle/kma_oracle.c
// orc_hash_annotate: distinct K-mer sets (ProteinKmers, windows i = 0 .. L-K), similarity =
// shared / (|A| + |B| - shared), a prototype becomes a protein's proposal when its similarity
// is >= minSim and above the current one (earlier prototypes win ties).
//
// GPU form (sorts and scans; no per-pair loop):
//   genome:     window keys, per-protein segmented sort, distinct sizes, (key, protein) pairs
//               of distinct keys sorted by key, unique keys U with their protein ranges
//   prototypes: window keys, segmented sort, distinct sizes; every distinct key looked up in U
//               (binary search) and one candidate (prototype, protein) emitted per protein of
//               its range; candidates sorted and run-length encoded: the run length IS the
//               number of shared distinct kmers
//   score:      similarity per (prototype, protein) in double (the Java expression), match
//               counts per prototype, best similarity per protein (u64 atomicMax on the
//               non-negative double's bits), then the smallest prototype index at that value
#include <cstring>  // (rocprim.hpp uses memset without including it)
#include <rocprim/rocprim.hpp>

#include "kma_hashanno.h"

namespace kma {
namespace {

constexpr uint64_t kSent = ~0ull;

unsigned grid1(uint64_t n) {
  const uint64_t g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}
unsigned grid_w(uint64_t n) {  // wave per item
  const uint64_t g = (n + 3) / 4;
  return (unsigned)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

// Wave per protein: owner[p] = protein of position p; first[p] = 1 at the first occurrence of a
// non-sentinel key in the protein's sorted segment.
__global__ __launch_bounds__(256) void owner_first_kernel(const uint64_t* __restrict__ sorted,
                                                          const uint64_t* __restrict__ off,
                                                          uint32_t n, uint32_t* __restrict__ owner,
                                                          uint8_t* __restrict__ first) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t o0 = off[0];
  for (uint64_t s = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); s < n;
       s += (uint64_t)gridDim.x * 4) {
    const uint64_t lo = off[s] - o0, hi = off[s + 1] - o0;
    for (uint64_t p = lo + lane; p < hi; p += 64) {
      const uint64_t v = sorted[p];
      owner[p] = (uint32_t)s;
      first[p] = (v != kSent && (p == lo || sorted[p - 1] != v)) ? 1 : 0;
    }
  }
}

__global__ __launch_bounds__(256) void run_heads_kernel(const uint64_t* __restrict__ k,
                                                        uint64_t n, uint8_t* __restrict__ head,
                                                        uint32_t* __restrict__ idx) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    head[i] = (i == 0 || k[i] != k[i - 1]) ? 1 : 0;
    idx[i] = (uint32_t)i;
  }
}

__global__ void set_end_kernel(uint32_t* ustart, const uint64_t* n_u, uint64_t n_pairs) {
  ustart[*n_u] = (uint32_t)n_pairs;
}

// Largest u with U[u] <= v, or n if none / not equal.
__device__ __forceinline__ uint64_t find_key(const uint64_t* __restrict__ U, uint64_t n,
                                             uint64_t v) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (U[mid] < v) lo = mid + 1; else hi = mid;
  }
  return (lo < n && U[lo] == v) ? lo : n;
}

// Per prototype position: the genome proteins sharing its key (first occurrences only).
__global__ __launch_bounds__(256) void cand_count_kernel(HashArgs a) {
  const uint64_t n_u = *a.n_u;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < a.n_ppos; i += gridDim.x * 256ull) {
    uint32_t c = 0, u = 0;
    if (a.pfirst[i]) {
      const uint64_t f = find_key(a.ukeys, n_u, a.psorted[i]);
      if (f < n_u) {
        u = (uint32_t)f;
        c = a.ustart[f + 1] - a.ustart[f];
      }
    }
    a.ccount[i] = c;
    a.cu[i] = u;
  }
}

// The slice's candidates: positions [pos_lo, pos_hi), written from cand_base.
__global__ __launch_bounds__(256) void cand_emit_kernel(HashArgs a) {
  for (uint64_t i = a.pos_lo + blockIdx.x * 256ull + threadIdx.x; i < a.pos_hi;
       i += gridDim.x * 256ull) {
    const uint32_t c = a.ccount[i];
    if (!c) continue;
    const uint64_t o = a.coff[i] - a.cand_base, proto = a.powner[i];
    const uint32_t s = a.ustart[a.cu[i]];
    for (uint32_t j = 0; j < c; ++j) a.cand[o + j] = proto << 32 | a.gprot[s + j];
  }
}

__device__ __forceinline__ double sim_of(const HashArgs& a, uint64_t pair, uint32_t c,
                                         uint32_t& proto, uint32_t& gp) {
  proto = (uint32_t)(pair >> 32);
  gp = (uint32_t)pair;
  const double uni = (double)a.psize[proto] + (double)a.gsize[gp] - (double)c;
  return (double)c / uni;
}

__global__ __launch_bounds__(256) void score_kernel(HashArgs a) {
  const uint64_t n = *a.n_runs;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    uint32_t proto, gp;
    const double s = sim_of(a, a.runs[i], a.run_len[i], proto, gp);
    if (s >= a.min_sim) {
      atomicAdd(a.out_count + proto, 1u);
      atomicMax((unsigned long long*)(a.best_bits + gp),
                (unsigned long long)__double_as_longlong(s));
    }
  }
}

__global__ __launch_bounds__(256) void choose_kernel(HashArgs a) {
  const uint64_t n = *a.n_runs;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    uint32_t proto, gp;
    const double s = sim_of(a, a.runs[i], a.run_len[i], proto, gp);
    if (s >= a.min_sim && (uint64_t)__double_as_longlong(s) == a.best_bits[gp])
      atomicMin(a.best_proto + gp, proto);
  }
}

__global__ __launch_bounds__(256) void proto_cum_kernel(const uint64_t* __restrict__ coff,
                                                        const uint32_t* __restrict__ ccount,
                                                        const uint64_t* __restrict__ off,
                                                        uint32_t n_proto, uint64_t n_pos,
                                                        uint64_t* __restrict__ cum) {
  const uint64_t total = n_pos ? coff[n_pos - 1] + ccount[n_pos - 1] : 0;
  const uint64_t o0 = off[0];
  for (uint64_t p = blockIdx.x * 256ull + threadIdx.x; p <= n_proto; p += gridDim.x * 256ull) {
    const uint64_t pos = off[p] - o0;
    cum[p] = pos < n_pos ? coff[pos] : total;
  }
}

__global__ __launch_bounds__(256) void merge_best_kernel(uint64_t* __restrict__ best_bits,
                                                         uint32_t* __restrict__ best_proto,
                                                         uint64_t* __restrict__ slice_bits,
                                                         uint32_t* __restrict__ slice_proto,
                                                         uint32_t n) {
  for (uint64_t g = blockIdx.x * 256ull + threadIdx.x; g < n; g += gridDim.x * 256ull) {
    const uint32_t sp = slice_proto[g];
    if (sp != 0xFFFFFFFFu && (best_proto[g] == 0xFFFFFFFFu || slice_bits[g] > best_bits[g])) {
      best_bits[g] = slice_bits[g];
      best_proto[g] = sp;
    }
    slice_bits[g] = 0;
    slice_proto[g] = 0xFFFFFFFFu;
  }
}

}  // namespace

hipError_t launch_proto_cum(const uint64_t* coff, const uint32_t* ccount, const uint64_t* off,
                            uint32_t n_proto, uint64_t n_pos, uint64_t* cum, hipStream_t s) {
  hipLaunchKernelGGL(proto_cum_kernel, dim3(grid1((uint64_t)n_proto + 1)), dim3(256), 0, s, coff,
                     ccount, off, n_proto, n_pos, cum);
  return hipGetLastError();
}
hipError_t launch_merge_best(uint64_t* best_bits, uint32_t* best_proto, uint64_t* slice_bits,
                             uint32_t* slice_proto, uint32_t n, hipStream_t s) {
  hipLaunchKernelGGL(merge_best_kernel, dim3(grid1(n)), dim3(256), 0, s, best_bits, best_proto,
                     slice_bits, slice_proto, n);
  return hipGetLastError();
}

hipError_t launch_owner_first(const uint64_t* sorted, const uint64_t* off, uint32_t n,
                              uint32_t* owner, uint8_t* first, hipStream_t s) {
  hipLaunchKernelGGL(owner_first_kernel, dim3(grid_w(n)), dim3(256), 0, s, sorted, off, n, owner,
                     first);
  return hipGetLastError();
}
hipError_t launch_run_heads(const uint64_t* k, uint64_t n, uint8_t* head, uint32_t* idx,
                            hipStream_t s) {
  hipLaunchKernelGGL(run_heads_kernel, dim3(grid1(n)), dim3(256), 0, s, k, n, head, idx);
  return hipGetLastError();
}
hipError_t launch_set_end(uint32_t* ustart, const uint64_t* n_u, uint64_t n_pairs, hipStream_t s) {
  hipLaunchKernelGGL(set_end_kernel, dim3(1), dim3(1), 0, s, ustart, n_u, n_pairs);
  return hipGetLastError();
}
hipError_t launch_cand_count(const HashArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(cand_count_kernel, dim3(grid1(a.n_ppos)), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_cand_emit(const HashArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(cand_emit_kernel, dim3(grid1(a.pos_hi - a.pos_lo)), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_score(const HashArgs& a, uint64_t n_max, hipStream_t s) {
  hipLaunchKernelGGL(score_kernel, dim3(grid1(n_max)), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_choose(const HashArgs& a, uint64_t n_max, hipStream_t s) {
  hipLaunchKernelGGL(choose_kernel, dim3(grid1(n_max)), dim3(256), 0, s, a);
  return hipGetLastError();
}

// rocPRIM wrappers (temp == nullptr: size query).
hipError_t prim_select_flagged_u64(void* temp, size_t* tb, const uint64_t* in, const uint8_t* f,
                                  uint64_t* out, uint64_t* n_out, uint64_t n, hipStream_t s) {
  return rocprim::select(temp, *tb, in, f, out, n_out, (size_t)n, s);
}
hipError_t prim_select_flagged_u32(void* temp, size_t* tb, const uint32_t* in, const uint8_t* f,
                                  uint32_t* out, uint64_t* n_out, uint64_t n, hipStream_t s) {
  return rocprim::select(temp, *tb, in, f, out, n_out, (size_t)n, s);
}
hipError_t prim_sort_pairs_u64_u32(void* temp, size_t* tb, const uint64_t* ki, uint64_t* ko,
                                  const uint32_t* vi, uint32_t* vo, uint64_t n, int bits,
                                  hipStream_t s) {
  return rocprim::radix_sort_pairs(temp, *tb, ki, ko, vi, vo, (size_t)n, 0u, (unsigned)bits, s);
}
hipError_t prim_sort_keys_u64(void* temp, size_t* tb, const uint64_t* ki, uint64_t* ko, uint64_t n,
                             int bits, hipStream_t s) {
  return rocprim::radix_sort_keys(temp, *tb, ki, ko, (size_t)n, 0u, (unsigned)bits, s);
}
hipError_t prim_excl_sum_u32_u64(void* temp, size_t* tb, const uint32_t* in, uint64_t* out,
                                uint64_t n, hipStream_t s) {
  return rocprim::exclusive_scan(temp, *tb, in, out, (uint64_t)0, (size_t)n,
                                 rocprim::plus<uint64_t>(), s);
}
hipError_t prim_rle_u64(void* temp, size_t* tb, const uint64_t* in, uint64_t* uniq, uint32_t* len,
                       uint64_t* n_runs, uint64_t n, hipStream_t s) {
  return rocprim::run_length_encode(temp, *tb, in, (unsigned)n, uniq, len, n_runs, s);
}

}  // namespace kma
