// kma_partition.hip — the region-partitioned protein path (large batches: c4, c5).
//
// Same results as annotate_kernel (ApplyKmerProcessor.java:122-148 over ProteinKmers at :123:
// per protein the set of distinct table kmers hit, NONE / AMBIGUOUS / the role and its count),
// reorganised so that the table is read from L2 instead of by random requests (kma_internal.h,
// "region-partitioned protein path", for the phases and the record / result formats):
//
//   chunk_flags / scan / chunk_index   proteins -> chunks (and the direct-path list)
//   partition_kernel (P1)              windows -> records, region-sorted per chunk
//   probe_regions_kernel (P2)          region sweep per XCD: L2 probes, dedupe, results
//   vote_chunks_kernel (P3)            results -> per-protein vote
//
// Integer / byte work; the bound is HBM streaming (records and results) plus L2 gathers.
#include <hipcub/hipcub.hpp>

#include "../../include/kmeranno.h"
#include "kma_internal.h"
#include "kma_device.h"

namespace kma {
namespace {

constexpr uint64_t kKeyBits40 = (1ull << 40) - 1;

__device__ __forceinline__ uint64_t windows_of(uint64_t len, int k, int adj) {
  const int64_t n = (int64_t)len - k + adj;
  return n > 0 ? (uint64_t)n : 0ull;
}

// Inclusive prefix sum over a wave (all 64 lanes).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(v, d, 64);
    v += lane >= d ? u : 0u;
  }
  return v;
}

// Exclusive prefix sum over the block (NT threads); ws: NT / 64 words of LDS. Returns the
// exclusive prefix of this thread, and the block total in *total (every thread).
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* ws, uint32_t* total) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint32_t inc = wave_incl_scan(v);
  if (lane == 63) ws[wave] = inc;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const uint32_t x = ws[w];
    before += w < wave ? x : 0u;
    all += x;
  }
  __syncthreads();  // ws may be reused
  *total = all;
  return before + inc - v;
}

// ---------------------------------------------------------------------------------------------
// Chunking. Protein p is GIANT if it has more than kGiantWindows windows (direct path). A
// non-giant protein starts a chunk if it is the first, follows a giant, sits at a multiple of
// kChunkProteins, or starts in a different 2^kChunkSpanBits-residue interval than its
// predecessor. So a chunk holds <= kChunkProteins whole proteins that all start in one interval
// and spans <= kChunkMaxSpan residues.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void chunk_flags_kernel(PartArgs a) {
  const uint64_t o0 = a.offsets[0];
  const int adj = (a.flags & KMA_F_END_EXCLUSIVE) ? 0 : 1;
  for (uint32_t p = blockIdx.x * 256u + threadIdx.x; p < a.n_seq; p += gridDim.x * 256u) {
    const uint64_t s = a.offsets[p] - o0, e = a.offsets[p + 1] - o0;
    const bool giant = windows_of(e - s, a.k, adj) > kGiantWindows;
    bool start = false;
    if (!giant) {
      if (p == 0 || p % kChunkProteins == 0) {
        start = true;
      } else {
        const uint64_t ps = a.offsets[p - 1] - o0;
        start = windows_of(s - ps, a.k, adj) > kGiantWindows ||
                (ps >> kChunkSpanBits) != (s >> kChunkSpanBits);
      }
    }
    a.chunk_flags[p] = (uint64_t)giant << 32 | (uint64_t)start;
  }
}

__global__ __launch_bounds__(256) void chunk_index_kernel(PartArgs a) {
  for (uint32_t p = blockIdx.x * 256u + threadIdx.x; p < a.n_seq; p += gridDim.x * 256u) {
    const uint64_t f = a.chunk_flags[p], e = a.chunk_excl[p];
    const uint32_t giant = (uint32_t)(f >> 32), start = (uint32_t)f & 1u;
    const uint32_t ci = (uint32_t)e, gi = (uint32_t)(e >> 32);
    if (start) a.chunk_first[ci] = p;
    if (giant) a.list[gi] = p;
    // the last protein of its chunk: the next one starts a chunk or is giant (flags != 0)
    if (!giant && (p + 1 == a.n_seq || a.chunk_flags[p + 1] != 0)) a.chunk_end[ci + start - 1] = p + 1;
    if (p + 1 == a.n_seq) {
      a.counts[0] = ci + start;
      a.counts[1] = gi + giant;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// P1: one chunk per block step (persistent blocks of 512 threads). The chunk's residues are
// staged in LDS as 5-bit codes (0 = not encodable); each thread then walks a contiguous range of
// window starts with a rolling key and rolling m-mer hashes (one new code, one hash and one
// home-bucket hash per window, the same values as home_bucket()). Pass A counts the windows per
// table region, a block scan makes the chunk's region offsets (written to run_off), pass B
// recomputes each window and writes its record at its region's LDS cursor. A chunk with more
// than kRunCap windows in one region (low-complexity input) is handed to the direct path.
// ---------------------------------------------------------------------------------------------
constexpr int kP1Threads = 512;

template <int K, int M, typename F>
__device__ __forceinline__ void for_windows(const uint32_t* __restrict__ codes_w, uint32_t a_mis,
                                            uint32_t i0, uint32_t i1, const uint32_t* pst,
                                            const uint32_t* pwn, uint32_t np, uint32_t nb, F&& f) {
  // LDS index i holds the code of chunk position i - a_mis. Window starts i in [i0, i1).
  if (i0 >= i1) return;
  constexpr uint64_t kMask = (K >= 13) ? ~0ull : ((1ull << (5 * K)) - 1);
  constexpr int NH = M > 0 ? K - M + 1 : 1;
  constexpr uint32_t mmask = M > 0 ? (uint32_t)((1ull << (5 * M)) - 1) : 0u;
  uint64_t key = 0;
  uint32_t lastbad = 0;  // LDS index + 1 of the last code 0 seen
  uint32_t ring[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h) ring[h] = 0xFFFFFFFFu;
  // protein of the first window start (binary search over pst[0..np])
  const int32_t x_first = (int32_t)i0 - (int32_t)a_mis;
  uint32_t p = 0;
  {
    const uint32_t xq = x_first < 0 ? 0u : (uint32_t)x_first;
    uint32_t lo = 0, hi = np;  // largest p with pst[p] <= xq
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (pst[mid] <= xq) lo = mid; else hi = mid;
    }
    p = lo;
  }
  uint32_t pbeg = pst[p], pnext = pst[p + 1], pw = pwn[p];
  const uint32_t iend = i1 + K - 1;  // codes consumed: [i0, iend)
  for (uint32_t ib = i0 & ~3u; ib < iend; ib += 4) {
    const uint32_t w4 = codes_w[ib >> 2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = ib + j;
      if (i < i0 || i >= iend) continue;
      const uint32_t c = (w4 >> (8 * j)) & 0xFFu;
      key = ((key << 5) | c) & kMask;
      lastbad = c == 0u ? i + 1u : lastbad;
      if constexpr (M > 0) {
#pragma unroll
        for (int h = 0; h + 1 < NH; ++h) ring[h] = ring[h + 1];
        ring[NH - 1] = mix32(((uint32_t)key & mmask) * 0x9E3779B1u + 0x7F4A7C15u);
      }
      if (i + 1 < i0 + K) continue;  // the first window is not complete yet
      const uint32_t ws = i + 1 - K;  // window start (LDS index)
      if (ws < a_mis) continue;
      const uint32_t x = ws - a_mis;  // chunk position
      while (x >= pnext && p + 1 < np) {
        ++p;
        pbeg = pnext;
        pnext = pst[p + 1];
        pw = pwn[p];
      }
      if (lastbad > ws || x - pbeg >= pw || x < pbeg) continue;
      uint32_t h;
      if constexpr (M > 0) {
        uint32_t mh = ring[0];
#pragma unroll
        for (int q = 1; q < NH; ++q) mh = mh < ring[q] ? mh : ring[q];
        h = mix32(mh ^ 0x85EBCA77u);
      } else {
        h = mix32((uint32_t)key ^ mix32((uint32_t)(key >> 32) + 0x9E3779B9u));
      }
      f(x, p, key, home_from_hash(h, key, M, nb));
    }
  }
}

template <int K, int M>
__global__ __launch_bounds__(kP1Threads) void partition_kernel(PartArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t codes_w[(kChunkMaxSpan + 64) / 4];
  __shared__ uint32_t hist[kMaxRegions + 1];
  __shared__ uint32_t cur[kMaxRegions];
  __shared__ uint32_t pst[kChunkProteins + 1];
  __shared__ uint32_t pwn[kChunkProteins];
  __shared__ uint8_t lut[256];
  __shared__ uint32_t wsum[kP1Threads / 64];
  __shared__ uint32_t s_max, s_base;
  const int t = threadIdx.x;
  if (t < 256) lut[t] = a.lut[t];
  const uint32_t nc = a.counts[0];
  const uint64_t o0 = a.offsets[0];
  const uint32_t R = a.n_regions, R1 = R + 1;
  const int rb = a.region_bits;
  const uint32_t rmask = (1u << rb) - 1u;
  const uint32_t nb = a.n_buckets;
  const int adj = (a.flags & KMA_F_END_EXCLUSIVE) ? 0 : 1;
  for (uint32_t c = blockIdx.x; c < nc; c += gridDim.x) {
    const uint32_t first = a.chunk_first[c], np = a.chunk_end[c] - first;
    const uint32_t lo = (uint32_t)(a.offsets[first] - o0);
    const uint32_t span = (uint32_t)(a.offsets[first + np] - o0) - lo;
    __syncthreads();  // the previous chunk's LDS is no longer read (lut written on entry)
    // Codes: aligned u32 words of residues; LDS byte j holds position j - mis.
    const uint8_t* src = a.residues + o0 + lo;
    const uint32_t mis = (uint32_t)((uintptr_t)src & 3u);
    const uint32_t* srcw = reinterpret_cast<const uint32_t*>(src - mis);
    const uint32_t n_words = (span + mis + K + 3) / 4;
    for (uint32_t i = t; i < n_words; i += kP1Threads) {
      const uint32_t w = srcw[i];
      uint32_t o = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t q = 4 * i + j;  // LDS byte; position q - mis
        const uint32_t code = (q >= mis && q - mis < span) ? lut[(w >> (8 * j)) & 0xFFu] : 0u;
        o |= code << (8 * j);
      }
      codes_w[i] = o;
    }
    if (t <= (int)np) {
      const uint32_t b = (uint32_t)(a.offsets[first + t] - o0) - lo;
      pst[t] = b;
      if (t < (int)np)
        pwn[t] = (uint32_t)windows_of(a.offsets[first + t + 1] - a.offsets[first + t], K, adj);
    }
    for (uint32_t r = t; r <= R; r += kP1Threads) hist[r] = 0u;
    __syncthreads();
    // Thread ranges of window starts in LDS-index space, an odd number of words long (LDS banks).
    uint32_t lw = (span + mis + 4 * kP1Threads - 1) / (4 * kP1Threads);
    lw += (lw & 1u) ? 0u : 1u;
    const uint32_t i0 = min(span + mis, (uint32_t)t * 4u * lw);
    const uint32_t i1 = min(span + mis, i0 + 4u * lw);
    for_windows<K, M>(codes_w, mis, i0, i1, pst, pwn, np, nb,
                      [&](uint32_t, uint32_t, uint64_t, uint32_t b) {
                        atomicAdd(&hist[b >> rb], 1u);
                      });
    __syncthreads();
    // Block scan of the region counts (4 consecutive regions per thread).
    uint32_t v[4], sum = 0, mx = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t r = 4u * t + q;
      v[q] = r < R ? hist[r] : 0u;
      sum += v[q];
      mx = max(mx, v[q]);
    }
    if (t == 0) s_max = 0u;
    uint32_t total;
    uint32_t run = block_excl_scan<kP1Threads>(sum, wsum, &total);
    atomicMax(&s_max, mx);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t r = 4u * t + q;
      if (r < R) {
        hist[r] = run;
        cur[r] = run;
      }
      run += v[q];
    }
    if (t == 0) hist[R] = total;
    __syncthreads();
    const bool fallback = s_max > (uint32_t)kRunCap;
    uint16_t* row = a.run_off + (uint64_t)c * R1;  // chunk records < 2^16
    for (uint32_t r = t; r <= R; r += kP1Threads) row[r] = fallback ? 0 : (uint16_t)hist[r];
    if (t == 0) a.chunk_fb[c] = fallback ? 1 : 0;
    if (fallback) {  // block-uniform: the chunk's proteins take the direct path
      if (t == 0) s_base = atomicAdd(a.counts + 1, np);
      __syncthreads();
      if (t < (int)np) a.list[s_base + t] = first + t;
      continue;
    }
    uint64_t* rec = a.rec + lo;
    for_windows<K, M>(codes_w, mis, i0, i1, pst, pwn, np, nb,
                      [&](uint32_t, uint32_t p, uint64_t key, uint32_t b) {
                        const uint32_t slot = atomicAdd(&cur[b >> rb], 1u);
                        rec[slot] = key | (uint64_t)p << 40 | (uint64_t)(b & rmask) << 48;
                      });
  }
}

// ---------------------------------------------------------------------------------------------
// P2: region sweep. Block b belongs to XCD group g = b % 8 (the blocks dealt to one XCD) and
// takes chunks [j nc / NB, (j + 1) nc / NB) of every region r = g, g + 8, ... (j = b / 8,
// NB = grid / 8): the group's blocks work on the same region at the same time, so its 2 MiB of
// buckets are fetched into the XCD's L2 once and every further probe of the region hits there.
// A step takes the records of whole runs (<= kProbeBatch, 4 per lane), probes them with the
// quad-cooperative bucket loads of annotate_kernel, walks overflow chains in place, drops the
// second and later hits of a key in one protein (LDS set keyed by run, protein and key: equal
// keys of a protein share a run) and writes each record's result.
// ---------------------------------------------------------------------------------------------
constexpr int kP2Threads = 256;
constexpr int kP2Win = kProbeBatch / kP2Threads;  // records per lane per step

__device__ __forceinline__ bool set64_insert(unsigned long long* set, uint32_t cap,
                                             unsigned long long v) {
  uint32_t i = (uint32_t)(((uint64_t)mix32((uint32_t)v ^ mix32((uint32_t)(v >> 32))) * cap) >> 32);
  for (;;) {
    const unsigned long long o = atomicCAS(set + i, 0ull, v);
    if (o == 0ull) return true;
    if (o == v) return false;
    i = i + 1 == cap ? 0u : i + 1;
  }
}

template <int K, int M>
__global__ __launch_bounds__(kP2Threads) void probe_regions_kernel(PartArgs a) {
  __shared__ unsigned long long set[kPartSet];
  __shared__ uint32_t r_start[kMaxRunsPerBlock];
  __shared__ uint32_t r_pref[kMaxRunsPerBlock + 1];
  __shared__ uint32_t c_base[kMaxRunsPerBlock];
  __shared__ uint8_t c_fb[kMaxRunsPerBlock];
  __shared__ uint32_t wsum[kP2Threads / 64];
  const int t = threadIdx.x, part = t & 3;
  const uint32_t g = blockIdx.x & 7u, j = blockIdx.x >> 3, NB = gridDim.x >> 3;
  const uint32_t nc = a.counts[0];
  const uint32_t c0 = (uint32_t)((uint64_t)j * nc / NB), c1 = (uint32_t)((uint64_t)(j + 1) * nc / NB);
  const uint32_t ncb = c1 - c0;  // <= kMaxRunsPerBlock (the host sizes the grid)
  const uint64_t o0 = a.offsets[0];
  for (uint32_t i = t; i < ncb; i += kP2Threads) {
    c_base[i] = (uint32_t)(a.offsets[a.chunk_first[c0 + i]] - o0);
    c_fb[i] = a.chunk_fb[c0 + i];
  }
  const bool multiset = (a.flags & KMA_F_MULTISET) != 0;
  const uint32_t R = a.n_regions, R1 = R + 1;
  const int rb = a.region_bits;
  const uint64_t* __restrict__ slots = a.slots;
  const uint32_t nb = a.n_buckets;
  for (uint32_t r = g; r < R; r += 8) {
    __syncthreads();  // c_base ready / the previous region's tables no longer read
    // This region's run of each of the block's chunks: thread t owns runs 2t, 2t + 1.
    uint32_t len[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const uint32_t i = 2u * t + q;
      len[q] = 0;
      if (i < ncb && !c_fb[i]) {
        const uint16_t* row = a.run_off + (uint64_t)(c0 + i) * R1 + r;
        const uint32_t s = row[0];
        len[q] = (uint32_t)row[1] - s;
        r_start[i] = c_base[i] + s;
      }
    }
    uint32_t total;
    const uint32_t pre = block_excl_scan<kP2Threads>(len[0] + len[1], wsum, &total);
    if (2u * t < ncb) r_pref[2u * t] = pre;
    if (2u * t + 1 < ncb) r_pref[2u * t + 1] = pre + len[0];
    if (t == 0) r_pref[ncb] = total;
    __syncthreads();
    if (total == 0) continue;  // block-uniform
    uint32_t i0 = 0;
    while (i0 < ncb) {
      // Runs [i0, i1): as many whole runs as fit kProbeBatch records (a run is <= kRunCap).
      const uint32_t e0 = r_pref[i0];
      uint32_t lo = i0 + 1, hi = ncb;  // largest i1 in [i0 + 1, ncb] with r_pref[i1] - e0 <= batch
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (r_pref[mid] - e0 <= (uint32_t)kProbeBatch) lo = mid; else hi = mid - 1;
      }
      const uint32_t i1 = lo, n = r_pref[i1] - e0;
      if (n == 0) {
        i0 = i1;
        continue;
      }
      if (!multiset) {
        for (int q = t; q < kPartSet; q += kP2Threads) set[q] = 0ull;
        __syncthreads();
      }
      // Records of this step: lane t takes e = t + 256 u, u < kP2Win.
      uint64_t rec[kP2Win];
      uint32_t ri[kP2Win], run[kP2Win], bk[kP2Win];
#pragma unroll
      for (int u = 0; u < kP2Win; ++u) {
        const uint32_t e = (uint32_t)u * kP2Threads + t;
        ri[u] = 0;
        run[u] = 0;
        rec[u] = 0;
        if (e < n) {
          uint32_t l2 = i0, h2 = i1 - 1;  // largest run with r_pref[run] <= e0 + e
          while (l2 < h2) {
            const uint32_t mid = (l2 + h2 + 1) >> 1;
            if (r_pref[mid] <= e0 + e) l2 = mid; else h2 = mid - 1;
          }
          run[u] = l2;
          ri[u] = r_start[l2] + (e0 + e - r_pref[l2]);
        }
      }
#pragma unroll
      for (int u = 0; u < kP2Win; ++u)
        if ((uint32_t)u * kP2Threads + t < n) rec[u] = __builtin_nontemporal_load(a.rec + ri[u]);
#pragma unroll
      for (int u = 0; u < kP2Win; ++u)
        bk[u] = (uint32_t)u * kP2Threads + t < n ? (r << rb) | (uint32_t)(rec[u] >> 48) : kNone;
      // Quad-cooperative bucket loads (L2): lane `part` reads bytes [16 part, 16 part + 16).
      uint4 q[kP2Win][4][kBucketHalves];
#pragma unroll
      for (int u = 0; u < kP2Win; ++u) {
        const uint32_t bb[4] = {quad_bcast<0>(bk[u]), quad_bcast<1>(bk[u]), quad_bcast<2>(bk[u]),
                                quad_bcast<3>(bk[u])};
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          const uint4* bp = reinterpret_cast<const uint4*>(slots) + part +
                            (uint64_t)(bb[x] == kNone ? 0u : bb[x]) * kBucketQuads;
#pragma unroll
          for (int h = 0; h < kBucketHalves; ++h) q[u][x][h] = bp[4 * h];
        }
      }
#pragma unroll
      for (int u = 0; u < kP2Win; ++u) {
        const uint32_t klo = (uint32_t)rec[u], khi = (uint32_t)((rec[u] >> 32) & 0xFFu) << 24;
        uint32_t word = 0;
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          const uint32_t kl = x == 0 ? quad_bcast<0>(klo) : x == 1 ? quad_bcast<1>(klo)
                            : x == 2 ? quad_bcast<2>(klo) : quad_bcast<3>(klo);
          const uint32_t kh = x == 0 ? quad_bcast<0>(khi) : x == 1 ? quad_bcast<1>(khi)
                            : x == 2 ? quad_bcast<2>(khi) : quad_bcast<3>(khi);
          const uint32_t w = match_part(q[u][x], kl, kh, part);
          word = part == x ? w : word;
        }
        if (bk[u] == kNone) continue;
        const uint64_t key = rec[u] & kKeyBits40;
        const uint32_t lp = (uint32_t)(rec[u] >> 40) & 0xFFu;
        uint32_t fid = (word & kWordFid) - 1u, sid = 0;
        bool hit = (word & kWordFid) != 0u;
        if (!hit && word == 0x80000000u) hit = walk_chain(slots, nb, bk[u], key, fid, sid);
        bool fresh = hit;
        if (hit && !multiset)
          fresh = set64_insert(set, kPartSet, key | (uint64_t)lp << 40 | (uint64_t)(run[u] - i0) << 48);
        __builtin_nontemporal_store(fresh ? (lp << 24 | (fid + 1u)) : 0u, a.res + ri[u]);
      }
      if (!multiset) __syncthreads();  // the set is cleared again for the next step
      i0 = i1;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// P3: one chunk per block step. The chunk's results are contiguous (its records' places); the
// vote is annotate_kernel's: no hit -> NONE, smallest != largest fid -> AMBIGUOUS, else the
// role with count = distinct keys hit, CALLED iff count >= minHits (ApplyKmerProcessor:146).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void vote_chunks_kernel(PartArgs a) {
  __shared__ uint32_t pmin[kChunkProteins], pmax[kChunkProteins], pcnt[kChunkProteins];
  const int t = threadIdx.x;
  const uint32_t nc = a.counts[0];
  const uint64_t o0 = a.offsets[0];
  const uint32_t R1 = a.n_regions + 1;
  for (uint32_t c = blockIdx.x; c < nc; c += gridDim.x) {
    if (a.chunk_fb[c]) continue;  // block-uniform: the direct path writes these proteins
    const uint32_t first = a.chunk_first[c], np = a.chunk_end[c] - first;
    const uint32_t lo = (uint32_t)(a.offsets[first] - o0);
    const uint32_t nrec = a.run_off[(uint64_t)c * R1 + a.n_regions];
    __syncthreads();  // the previous chunk's outputs are read
    if (t < (int)np) {
      pmin[t] = 0xFFFFFFFFu;
      pmax[t] = 0u;
      pcnt[t] = 0u;
    }
    __syncthreads();
    const uint32_t* __restrict__ rp = a.res + lo;
    for (uint32_t i = t; i < nrec; i += 256) {
      const uint32_t v = __builtin_nontemporal_load(rp + i);
      if (v) {
        const uint32_t p = v >> 24, f = (v & 0xFFFFFFu) - 1u;
        atomicMin(&pmin[p], f);
        atomicMax(&pmax[p], f);
        atomicAdd(&pcnt[p], 1u);
      }
    }
    __syncthreads();
    if (t < (int)np) {
      const uint32_t mn = pmin[t], mx = pmax[t], cnt = pcnt[t];
      int32_t fid_out = -1, cnt_out = 0;
      uint8_t st;
      if (mn == 0xFFFFFFFFu) {
        st = KMA_STATUS_NONE;
      } else if (mn != mx) {
        st = KMA_STATUS_AMBIGUOUS;
      } else {
        fid_out = (int32_t)mn;
        cnt_out = (int32_t)cnt;
        st = cnt >= (uint32_t)a.min_hits ? KMA_STATUS_CALLED : KMA_STATUS_BELOW_MIN;
        if (st == KMA_STATUS_CALLED && a.tally && mn < a.n_fid) atomicAdd(a.tally + mn, 1u);
      }
      a.out_fid[first + t] = fid_out;
      a.out_count[first + t] = cnt_out;
      a.out_status[first + t] = st;
    }
  }
}

}  // namespace

// ---- launchers ----------------------------------------------------------------------------------
hipError_t launch_chunking(const PartArgs& a, void* temp, size_t* temp_bytes, hipStream_t stream) {
  if (!temp)
    return hipcub::DeviceScan::ExclusiveSum(nullptr, *temp_bytes, a.chunk_flags, a.chunk_excl,
                                            (int)a.n_seq, stream);
  const unsigned g = (unsigned)std::min<uint64_t>(4096, ((uint64_t)a.n_seq + 255) / 256);
  hipLaunchKernelGGL(chunk_flags_kernel, dim3(g ? g : 1), dim3(256), 0, stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, a.chunk_flags, a.chunk_excl,
                                       (int)a.n_seq, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(chunk_index_kernel, dim3(g ? g : 1), dim3(256), 0, stream, a);
  return hipGetLastError();
}

template <int K, int M>
struct PartitionLaunch {
  static hipError_t run(const PartArgs& a, unsigned blocks, hipStream_t stream) {
    hipLaunchKernelGGL((partition_kernel<K, M>), dim3(blocks), dim3(kP1Threads), 0, stream, a);
    return hipGetLastError();
  }
};
template <int K, int M>
struct ProbeRegionsLaunch {
  static hipError_t run(const PartArgs& a, unsigned blocks, hipStream_t stream) {
    hipLaunchKernelGGL((probe_regions_kernel<K, M>), dim3(blocks), dim3(kP2Threads), 0, stream, a);
    return hipGetLastError();
  }
};
template <int K, int M>
struct OccupancyQuery {
  static hipError_t run(int which, int* out) {
    if (which == 0)
      return hipOccupancyMaxActiveBlocksPerMultiprocessor(out, partition_kernel<K, M>, kP1Threads, 0);
    if (which == 1)
      return hipOccupancyMaxActiveBlocksPerMultiprocessor(out, probe_regions_kernel<K, M>,
                                                          kP2Threads, 0);
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(out, vote_chunks_kernel, 256, 0);
  }
};

hipError_t launch_partition(const PartArgs& a, unsigned blocks, hipStream_t stream) {
  return dispatch_km<PartitionLaunch>(a.k, a.mlen, a, blocks ? blocks : 1u, stream);
}
hipError_t launch_probe_regions(const PartArgs& a, unsigned blocks, hipStream_t stream) {
  return dispatch_km<ProbeRegionsLaunch>(a.k, a.mlen, a, blocks, stream);
}
hipError_t launch_vote_chunks(const PartArgs& a, unsigned blocks, hipStream_t stream) {
  hipLaunchKernelGGL(vote_chunks_kernel, dim3(blocks ? blocks : 1u), dim3(256), 0, stream, a);
  return hipGetLastError();
}
int partition_occupancy(int k, int m, int which) {
  int n = 0;
  if (dispatch_km<OccupancyQuery>(k, m, which, &n) != hipSuccess || n < 1) n = 1;
  return n;
}

}  // namespace kma
