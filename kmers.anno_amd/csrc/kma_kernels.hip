// kma_kernels.hip — CDNA4 (gfx950) kernels of the signature-kmer annotation hot path.
//
//   build_insert / build_finalize  signature-table construction (ApplyKmerProcessor.java:100-110)
//   proteins_kernel                ProteinKmers extraction + table probe + vote, one wave per
//                                  protein (ApplyKmerProcessor.java:122-147)
//   proteins_fallback_kernel       the same vote with a global-memory dedupe set for proteins
//                                  whose distinct hits overflow the per-wave LDS set
//   contigs_probe_kernel           6-frame translation + window + probe
//                                  (KmerReference.java:157-203, KmerPosition.java:50-93)
//   contigs_emit_kernel            canonical-order hit emission after a block-count scan
//
// Integer / byte work only: the bound is HBM (or Infinity-Cache) random access to 64-byte
// buckets, not MFMA. Every wave keeps one bucket load per lane in flight per chunk of 64
// windows; all per-protein state lives in registers and a wave-private LDS set.
#include <hipcub/hipcub.hpp>

#include "../../include/kmeranno.h"
#include "kma_internal.h"

namespace kma {
namespace {

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
  return v;
}
// Number of set bits of m in lanes below this lane (v_mbcnt).
__device__ __forceinline__ uint32_t popc_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// The K residues of the window starting at absolute byte `pos`, as one little-endian u64
// (byte j = residue j). Two aligned 8-byte loads + a funnel shift: consecutive lanes read
// consecutive words, so a wave's 64 windows coalesce into two or three 64-byte lines.
__device__ __forceinline__ uint64_t window_bytes(const uint8_t* __restrict__ res, uint64_t pos) {
  const uint64_t* src = reinterpret_cast<const uint64_t*>(res + (pos & ~7ull));
  const uint64_t lo = src[0], hi = src[1];
  const uint32_t sh = (uint32_t)(pos & 7) * 8u;
  return sh ? ((lo >> sh) | (hi << (64u - sh))) : lo;
}

// 5-bit packing through the table's residue LUT (LDS); false if a byte is not encodable.
__device__ __forceinline__ bool pack_window(const uint8_t* lut, uint64_t bytes, int k,
                                           uint64_t& key) {
  bool ok = true;
  uint64_t v = 0;
  for (int j = 0; j < k; ++j) {
    const uint32_t c = lut[(bytes >> (8 * j)) & 0xFFu];
    ok = ok && (c != 0u);
    v = (v << 5) | c;
  }
  key = v;
  return ok;
}

// Probe the bucketized table. Returns true on a hit with the fid and the global slot id.
__device__ __forceinline__ bool probe(const uint64_t* __restrict__ slots, uint64_t n_buckets,
                                      uint64_t key, uint32_t& fid, uint32_t& sid) {
  uint64_t b = home_bucket(key, n_buckets);
  for (uint64_t step = 0; step < n_buckets; ++step) {  // bounded even for a full foreign table
    const uint4* bp = reinterpret_cast<const uint4*>(slots + b * kSlotsPerBucket);
    const uint4 q0 = bp[0], q1 = bp[1], q2 = bp[2], q3 = bp[3];
    const uint64_t s[8] = {
        ((uint64_t)q0.y << 32) | q0.x, ((uint64_t)q0.w << 32) | q0.z,
        ((uint64_t)q1.y << 32) | q1.x, ((uint64_t)q1.w << 32) | q1.z,
        ((uint64_t)q2.y << 32) | q2.x, ((uint64_t)q2.w << 32) | q2.z,
        ((uint64_t)q3.y << 32) | q3.x, ((uint64_t)q3.w << 32) | q3.z};
    bool hit = false, empty = false;
#pragma unroll
    for (int j = 0; j < kSlotsPerBucket; ++j) {
      if ((s[j] >> kFidBits) == key) {
        hit = true;
        fid = (uint32_t)(s[j] & kFidMask);
        sid = (uint32_t)(b * kSlotsPerBucket + j);
      }
      empty |= (s[j] == 0);
    }
    if (hit) return true;
    if (empty) return false;
    b = (b + 1 == n_buckets) ? 0 : b + 1;
  }
  return false;
}

// ---------------------------------------------------------------------------------------------
// Table construction. Insert: claim the first empty slot of the probe chain with a 64-bit CAS
// (slot = key << 24, fid still 0) or find the key already there; either way record the row
// index with atomicMax so the LAST row of a duplicate key wins (HashMap.put semantics).
// Finalize: write the winning row's fid into the slot; collect entry count and max probe.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void build_insert_kernel(uint64_t* slots, uint32_t* winner,
                                                           uint64_t n_buckets,
                                                           const uint64_t* __restrict__ keys,
                                                           uint64_t n, uint32_t* status) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t key = keys[i];
    if (key == 0) continue;
    const uint64_t want = key << kFidBits;
    uint64_t b = home_bucket(key, n_buckets);
    bool done = false;
    for (uint64_t p = 0; p < n_buckets && !done; ++p) {
      for (int j = 0; j < kSlotsPerBucket; ++j) {
        uint64_t* sp = slots + b * kSlotsPerBucket + j;
        uint64_t v = __hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v == 0) {
          const uint64_t old = atomicCAS((unsigned long long*)sp, 0ull, want);
          v = old == 0 ? want : old;
        }
        if ((v >> kFidBits) == key) {
          atomicMax(winner + b * kSlotsPerBucket + j, (uint32_t)(i + 1));
          done = true;
          break;
        }
      }
      b = (b + 1 == n_buckets) ? 0 : b + 1;
    }
    if (!done) atomicOr(status, 1u);  // table full: cannot happen at load factor < 1
  }
}

__global__ __launch_bounds__(256) void build_finalize_kernel(uint64_t* slots,
                                                             const uint32_t* __restrict__ winner,
                                                             const uint32_t* __restrict__ fids,
                                                             uint64_t n_buckets, uint32_t* stats) {
  const uint64_t n_slots = n_buckets * kSlotsPerBucket;
  uint32_t entries = 0, max_probe = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_slots;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t w = winner[i];
    if (w == 0) continue;
    const uint64_t v = slots[i];
    slots[i] = v | ((uint64_t)fids[w - 1] & kFidMask);
    const uint64_t b = i / kSlotsPerBucket, h = home_bucket(v >> kFidBits, n_buckets);
    const uint32_t d = (uint32_t)((b + n_buckets - h) % n_buckets) + 1u;
    entries++;
    max_probe = max(max_probe, d);
  }
  entries = wave_sum(entries);
  max_probe = wave_max(max_probe);
  if ((threadIdx.x & 63) == 0) {
    if (entries) atomicAdd(stats + 0, entries);
    atomicMax(stats + 1, max_probe);
  }
}

// ---------------------------------------------------------------------------------------------
// Protein annotation: one wave per protein, 64 windows per step (lane = window).
// Vote state per lane: min fid, max fid, distinct-hit count; the protein is CALLED iff the
// wave-wide min == max (one role only) and the distinct count >= min_hits. Distinct counting
// (ProteinKmers is a set) inserts each hit's slot id into a wave-private LDS open-addressing
// set; a protein whose distinct hits would exceed kSetLimit is marked pending and finished by
// proteins_fallback_kernel with a global-memory set.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void proteins_kernel(ProteinArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t set_mem[kWavesPerBlock * kSetCap];
  __shared__ uint8_t lut[256];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  lut[tid] = a.lut[tid];
  uint32_t* set = set_mem + wave * kSetCap;
  uint4* set4 = reinterpret_cast<uint4*>(set);
#pragma unroll
  for (int i = lane; i < kSetCap / 4; i += 64) set4[i] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();

  const uint32_t s = blockIdx.x * kWavesPerBlock + wave;
  if (s >= a.n_seq) return;
  const uint64_t beg = a.offsets[s];
  const int64_t len = (int64_t)(a.offsets[s + 1] - beg);
  const int k = a.k;
  const int64_t n_win = len - k + ((a.flags & KMA_F_END_EXCLUSIVE) ? 0 : 1);
  const bool multiset = (a.flags & KMA_F_MULTISET) != 0;

  uint32_t fmin = 0xFFFFFFFFu, fmax = 0u, cnt = 0u;
  uint32_t total = 0u;  // wave-uniform: distinct entries in the LDS set
  bool ambiguous = false, overflow = false;
  for (int64_t w0 = 0; w0 < n_win; w0 += 64) {
    if (!multiset && !ambiguous && total + 64u > (uint32_t)kSetLimit) {
      overflow = true;
      break;
    }
    const int64_t w = w0 + lane;
    uint64_t key = 0;
    bool ok = w < n_win;
    if (ok) ok = pack_window(lut, window_bytes(a.residues, beg + (uint64_t)w), k, key);
    uint32_t fid = 0u, sid = 0u;
    const bool hit = ok && probe(a.slots, a.n_buckets, key, fid, sid);
    if (hit) {
      fmin = min(fmin, fid);
      fmax = max(fmax, fid);
    }
    if (multiset) {
      cnt += hit ? 1u : 0u;
    } else if (!ambiguous) {
      bool fresh = false;
      if (hit) {
        const uint32_t id = sid + 1u;
        uint32_t h = (id * 0x9E3779B1u) >> (32 - 11);  // kSetCap = 2^11
        for (;;) {
          const uint32_t old = atomicCAS(set + h, 0u, id);
          if (old == 0u) {
            fresh = true;
            break;
          }
          if (old == id) break;
          h = (h + 1u) & (kSetCap - 1);
        }
      }
      cnt += fresh ? 1u : 0u;
      total += (uint32_t)__popcll(__ballot(fresh));
      const uint32_t wmin = wave_min(fmin), wmax = wave_max(fmax);
      ambiguous = wmin != 0xFFFFFFFFu && wmin != wmax;
    }
  }
  const uint32_t wmin = wave_min(fmin), wmax = wave_max(fmax), wcnt = wave_sum(cnt);
  if (lane == 0) {
    int32_t fid_out = -1, cnt_out = 0;
    uint8_t st;
    if (wmin == 0xFFFFFFFFu) {
      st = KMA_STATUS_NONE;
    } else if (wmin != wmax) {
      st = KMA_STATUS_AMBIGUOUS;
    } else if (overflow) {
      st = kStatusPending;
      atomicOr(a.overflow_flag, 1u);
    } else {
      fid_out = (int32_t)wmin;
      cnt_out = (int32_t)wcnt;
      st = wcnt >= (uint32_t)a.min_hits ? KMA_STATUS_CALLED : KMA_STATUS_BELOW_MIN;
      if (st == KMA_STATUS_CALLED && a.tally && wmin < a.n_fid) atomicAdd(a.tally + wmin, 1u);
    }
    a.out_fid[s] = fid_out;
    a.out_count[s] = cnt_out;
    a.out_status[s] = st;
  }
}

__device__ __forceinline__ uint32_t block_reduce(uint32_t v, uint32_t* red, int op) {
  // op: 0 min, 1 max, 2 sum — 256 threads
  v = op == 0 ? wave_min(v) : op == 1 ? wave_max(v) : wave_sum(v);
  const int wave = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wave] = v;
  __syncthreads();
  uint32_t r = red[0];
  for (int w = 1; w < kWavesPerBlock; ++w)
    r = op == 0 ? min(r, red[w]) : op == 1 ? max(r, red[w]) : r + red[w];
  return r;
}

__global__ __launch_bounds__(256) void proteins_fallback_kernel(ProteinArgs a) {
  if (__hip_atomic_load(a.overflow_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
    return;
  __shared__ uint8_t lut[256];
  __shared__ uint32_t red[kWavesPerBlock];
  const int tid = threadIdx.x;
  lut[tid] = a.lut[tid];
  __syncthreads();
  uint32_t* set = a.scratch + (uint64_t)blockIdx.x * kFallbackCap;
  const int k = a.k;
  for (uint32_t s = blockIdx.x; s < a.n_seq; s += gridDim.x) {
    if (a.out_status[s] != kStatusPending) continue;  // block-uniform
    const uint64_t beg = a.offsets[s];
    const int64_t len = (int64_t)(a.offsets[s + 1] - beg);
    const int64_t n_win = len - k + ((a.flags & KMA_F_END_EXCLUSIVE) ? 0 : 1);
    if (n_win > (int64_t)(kFallbackCap / 2)) {
      if (tid == 0) {
        a.out_fid[s] = -1;
        a.out_count[s] = 0;
        a.out_status[s] = KMA_STATUS_TOO_LONG;
      }
      continue;
    }
    uint32_t cap = 64;
    while (cap < 2 * (uint32_t)n_win) cap <<= 1;
    for (uint32_t i = tid; i < cap; i += blockDim.x) set[i] = 0u;
    __syncthreads();
    uint32_t fmin = 0xFFFFFFFFu, fmax = 0u, cnt = 0u;
    for (int64_t w = tid; w < n_win; w += blockDim.x) {
      uint64_t key;
      if (!pack_window(lut, window_bytes(a.residues, beg + (uint64_t)w), k, key)) continue;
      uint32_t fid, sid;
      if (!probe(a.slots, a.n_buckets, key, fid, sid)) continue;
      fmin = min(fmin, fid);
      fmax = max(fmax, fid);
      const uint32_t id = sid + 1u;
      uint32_t h = (id * 0x9E3779B1u) & (cap - 1u);
      for (;;) {
        const uint32_t old = atomicCAS(set + h, 0u, id);
        if (old == 0u) {
          cnt++;
          break;
        }
        if (old == id) break;
        h = (h + 1u) & (cap - 1u);
      }
    }
    fmin = block_reduce(fmin, red, 0);
    fmax = block_reduce(fmax, red, 1);
    cnt = block_reduce(cnt, red, 2);
    if (tid == 0) {
      if (fmin != fmax) {  // cannot be NONE: the main kernel only defers proteins with hits
        a.out_fid[s] = -1;
        a.out_count[s] = 0;
        a.out_status[s] = KMA_STATUS_AMBIGUOUS;
      } else {
        a.out_fid[s] = (int32_t)fmin;
        a.out_count[s] = (int32_t)cnt;
        const bool called = cnt >= (uint32_t)a.min_hits;
        a.out_status[s] = called ? KMA_STATUS_CALLED : KMA_STATUS_BELOW_MIN;
        if (called && a.tally && fmin < a.n_fid) atomicAdd(a.tally + fmin, 1u);
      }
    }
    __syncthreads();  // the set is reused by the next protein
  }
}

// ---------------------------------------------------------------------------------------------
// 6-frame contig annotation. A block owns kContigTile consecutive forward positions x of the
// concatenated contigs. Position x anchors two windows whose DNA span is [x, x + 3K):
//   '+' : codons read forward at x, x+3, ..               (processKmers on getSequence)
//   '-' : reverse-complement codons, last codon first      (processKmers on getRSequence)
// Both have 1-based forward left edge x + 1 = KmerPosition.calcLeft. processKmers' end
// exclusion i < P_f - K works out to x + 3K + 3 <= len for '+' and 3 <= x <= len - 3K for '-'.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t contig_of(const uint64_t* __restrict__ off, uint32_t n,
                                              uint64_t g) {
  uint32_t lo = 0, hi = n;  // largest c with off[c] <= g
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (off[mid] <= g) lo = mid; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ uint32_t base2(uint8_t c) {  // T,C,A,G -> 0..3; other -> 4
  switch (c | 0x20) {
    case 't': case 'u': return 0u;
    case 'c': return 1u;
    case 'a': return 2u;
    case 'g': return 3u;
    default: return 4u;
  }
}

__global__ __launch_bounds__(256) void contigs_probe_kernel(ContigArgs a) {
  constexpr int kSpan = kContigTile + 3 * KMA_MAX_K;
  __shared__ uint8_t bases[kSpan];
  __shared__ uint8_t aa_p[kSpan], aa_m[kSpan];
  __shared__ uint8_t codes[64];
  __shared__ uint32_t wave_tot[kWavesPerBlock];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int k = a.k;
  const uint64_t g0 = (uint64_t)blockIdx.x * kContigTile;
  if (t < 64) codes[t] = a.codon_codes[t];
  for (int i = t; i < kSpan; i += blockDim.x) {
    const uint64_t g = g0 + i;
    bases[i] = (uint8_t)(g < a.total_bases ? base2(a.dna[g]) : 4u);
  }
  __syncthreads();
  for (int i = t; i < kSpan - 2; i += blockDim.x) {
    const uint32_t b0 = bases[i], b1 = bases[i + 1], b2 = bases[i + 2];
    if ((b0 | b1 | b2) & 4u) {
      aa_p[i] = aa_m[i] = 0;  // 'X'
    } else {
      aa_p[i] = codes[b0 * 16 + b1 * 4 + b2];
      aa_m[i] = codes[(b2 ^ 2u) * 16 + (b1 ^ 2u) * 4 + (b0 ^ 2u)];  // complement: x ^ 2
    }
  }
  __syncthreads();

  const uint64_t g = g0 + t;
  bool hp = false, hm = false;
  uint32_t fp = 0, fm = 0, contig = 0;
  if (g < a.total_bases) {
    contig = contig_of(a.offsets, a.n_contig, g);
    const int64_t x = (int64_t)(g - a.offsets[contig]);
    const int64_t len = (int64_t)(a.offsets[contig + 1] - a.offsets[contig]);
    bool pv = x + 3 * k + 3 <= len, mv = x >= 3 && x + 3 * k <= len;
    uint64_t kp = 0, km = 0;
    for (int j = 0; j < k; ++j) {
      const uint32_t cp = aa_p[t + 3 * j], cm = aa_m[t + 3 * j];
      pv = pv && cp != 0u;
      mv = mv && cm != 0u;
      kp = (kp << 5) | cp;
      km |= (uint64_t)cm << (5 * j);
    }
    uint32_t sid;
    hp = pv && probe(a.slots, a.n_buckets, kp, fp, sid);
    hm = mv && probe(a.slots, a.n_buckets, km, fm, sid);
    if (a.tally) {
      if (hp && fp < a.n_fid) atomicAdd(a.tally + (uint64_t)contig * a.n_fid + fp, 1u);
      if (hm && fm < a.n_fid) atomicAdd(a.tally + (uint64_t)contig * a.n_fid + fm, 1u);
    }
  }
  // Block-local compaction in canonical order (position, '+' before '-').
  const uint64_t bp = __ballot(hp), bm = __ballot(hm);
  if (lane == 0) wave_tot[wave] = (uint32_t)(__popcll(bp) + __popcll(bm));
  __syncthreads();
  uint32_t o = popc_below(bp) + popc_below(bm), total = 0;
  for (int w = 0; w < kWavesPerBlock; ++w) {
    if (w < wave) o += wave_tot[w];
    total += wave_tot[w];
  }
  uint64_t* st = a.staging + (uint64_t)blockIdx.x * (2 * kContigTile);
  if (hp) st[o++] = (g << 25) | fp;                // strand bit 24 = 0: '+'
  if (hm) st[o] = (g << 25) | (1ull << 24) | fm;   // '-'
  if (t == 0) a.block_counts[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void contigs_emit_kernel(ContigArgs a,
                                                           const uint64_t* __restrict__ prefix,
                                                           kma_hit* __restrict__ out) {
  const uint32_t n = a.block_counts[blockIdx.x];
  if ((uint32_t)threadIdx.x >= n) return;
  const uint64_t* st = a.staging + (uint64_t)blockIdx.x * (2 * kContigTile);
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint64_t v = st[i];
    const uint64_t g = v >> 25;
    const bool minus = (v >> 24) & 1u;
    const uint32_t c = contig_of(a.offsets, a.n_contig, g);
    const int64_t x = (int64_t)(g - a.offsets[c]);
    const int64_t len = (int64_t)(a.offsets[c + 1] - a.offsets[c]);
    kma_hit h;
    h.contig = c;
    h.left = (int32_t)(x + 1);
    h.fid = (uint32_t)(v & kFidMask);
    h.strand = minus ? '-' : '+';
    h.frame = (uint8_t)((minus ? (len - 3 * a.k - x) : x) % 3 + 1);
    h.pad = 0;
    out[prefix[blockIdx.x] + i] = h;
  }
}

}  // namespace

// ---- launchers ----------------------------------------------------------------------------------
static unsigned grid_for(uint64_t n, unsigned cap = 8192) {
  uint64_t g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > cap ? cap : g));
}

hipError_t launch_build_insert(uint64_t* slots, uint32_t* winner, uint64_t n_buckets,
                               const uint64_t* keys, uint64_t n, uint32_t* status,
                               hipStream_t stream) {
  hipLaunchKernelGGL(build_insert_kernel, dim3(grid_for(n)), dim3(256), 0, stream, slots, winner,
                     n_buckets, keys, n, status);
  return hipGetLastError();
}

hipError_t launch_build_finalize(uint64_t* slots, const uint32_t* winner, const uint32_t* fids,
                                 uint64_t n_buckets, uint32_t* stats, hipStream_t stream) {
  hipLaunchKernelGGL(build_finalize_kernel, dim3(grid_for(n_buckets * kSlotsPerBucket)),
                     dim3(256), 0, stream, slots, winner, fids, n_buckets, stats);
  return hipGetLastError();
}

hipError_t launch_proteins(const ProteinArgs& a, hipStream_t stream) {
  if (a.n_seq == 0) return hipSuccess;
  const unsigned blocks = (a.n_seq + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL(proteins_kernel, dim3(blocks), dim3(256), 0, stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(proteins_fallback_kernel, dim3(kFallbackBlocks), dim3(256), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_contigs_probe(const ContigArgs& a, uint64_t n_blocks, hipStream_t stream) {
  hipLaunchKernelGGL(contigs_probe_kernel, dim3((unsigned)n_blocks), dim3(256), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_contig_scan(const uint32_t* counts, uint64_t* prefix, uint64_t n, void* temp,
                              size_t* temp_bytes, hipStream_t stream) {
  return hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, counts, prefix, (int)n, stream);
}

hipError_t launch_contigs(const ContigArgs& a, uint64_t n_blocks, const uint64_t* d_prefix,
                          uint8_t* out_hits, hipStream_t stream) {
  hipLaunchKernelGGL(contigs_emit_kernel, dim3((unsigned)n_blocks), dim3(256), 0, stream, a,
                     d_prefix, reinterpret_cast<kma_hit*>(out_hits));
  return hipGetLastError();
}

}  // namespace kma
