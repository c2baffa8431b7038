// kma_kernels.hip — CDNA4 (gfx950) kernels of the signature-kmer annotation hot path.
//
//   build_insert / build_finalize  signature-table construction (ApplyKmerProcessor.java:100-110)
//   probe_kernel       K1: every residue position's K-window packed and probed in the table
//                      (the HashMap.get of ApplyKmerProcessor.java:130 for every kmer of every
//                      protein); writes fid + 1 (0 = miss) per position. HBM random access.
//   vote_kernel        K2: one wave per protein: ProteinKmers set semantics (distinct kmers,
//                      org.theseed.sequence.ProteinKmers at :123) + the first/confirm/conflict
//                      vote and min-hits threshold (:129-147) over K1's words.
//   vote_long_kernel   K2 for long proteins: one block per protein.
//   contigs_probe_kernel  6-frame translation + window + probe
//                      (KmerReference.java:157-203, KmerPosition.java:50-93)
//   contigs_emit_kernel   canonical-order hit emission after a block-count scan
//
// Integer / byte work only: the bound is HBM (or Infinity-Cache) random access to 64-byte
// buckets, not MFMA.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "../../include/kmeranno.h"
#include "kma_internal.h"

// K1 / K12 SGPRs are capped so that the hardware admits as many 256-thread blocks per CU as the
// occupancy API reports and the K1 grid assumes: it admits ⌊800 / (⌈sgpr/16⌉·16 + 16)⌋, so 98
// SGPRs (uncapped K1) gave 6 blocks where the API said 7 and the "exactly resident" grid had a
// 1/7 tail. Capped: 86 SGPRs (8 spilled to VGPR lanes, no scratch), 7 blocks; measured c2 K1
// 47.5 -> 45.1 us, c5 unchanged (KMA_SGPR_UNCAPPED builds restore the old allocation for A/B).
#ifndef KMA_SGPR_UNCAPPED
#define KMA_SGPR_ATTR __attribute__((amdgpu_num_sgpr(88)))
#else
#define KMA_SGPR_ATTR
#endif

namespace kma {
namespace {

// Wave-wide reductions (all 64 lanes active; result wave-uniform): DPP inside each row of 16
// lanes (quad swaps, half-row and row mirrors: ALU-speed, no LDS round trip as ds_bpermute
// takes), then the four row results by readlane.
template <typename Op>
__device__ __forceinline__ uint32_t wave_reduce(uint32_t v, Op op) {
  v = op(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false));   // [1,0,3,2]
  v = op(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false));   // [2,3,0,1]
  v = op(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false));  // half mirror
  v = op(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false));  // row mirror
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
  const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
  const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
  const uint32_t r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
  return op(op(r0, r1), op(r2, r3));
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
  return wave_reduce(v, [](uint32_t x, uint32_t y) { return x < y ? x : y; });
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
  return wave_reduce(v, [](uint32_t x, uint32_t y) { return x > y ? x : y; });
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  return wave_reduce(v, [](uint32_t x, uint32_t y) { return x + y; });
}
// Number of set bits of m in lanes below this lane (v_mbcnt).
__device__ __forceinline__ uint32_t popc_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// The residues of the window starting at byte `pos` as one little-endian u64 (byte j = residue
// j). Two aligned 8-byte loads + a funnel shift: consecutive lanes read consecutive words.
__device__ __forceinline__ uint64_t funnel(uint64_t lo, uint64_t hi, uint32_t sh) {
  return sh ? ((lo >> sh) | (hi << (64u - sh))) : lo;
}
__device__ __forceinline__ uint64_t window_bytes(const uint8_t* __restrict__ res, uint64_t pos) {
  const uint64_t* src = reinterpret_cast<const uint64_t*>(res + (pos & ~7ull));
  return funnel(src[0], src[1], (uint32_t)(pos & 7) * 8u);
}
// The two aligned words of a window, combined later (funnel) so that the load is not consumed
// in the step that issues it.
struct WinWords {
  uint64_t lo, hi;
  uint32_t sh;
};
__device__ __forceinline__ WinWords window_words(const uint8_t* __restrict__ res, uint64_t pos) {
  const uint64_t* src = reinterpret_cast<const uint64_t*>(res + (pos & ~7ull));
  return WinWords{src[0], src[1], (uint32_t)(pos & 7) * 8u};
}

// 5-bit packing through the table's residue LUT (LDS); false if a byte is not encodable.
template <int K>
__device__ __forceinline__ bool pack_window(const uint8_t* lut, uint64_t bytes, uint64_t& key) {
  uint32_t c[K];
#pragma unroll
  for (int j = 0; j < K; ++j) c[j] = lut[(uint32_t)(bytes >> (8 * j)) & 0xFFu];
  uint64_t v = 0;
  bool ok = true;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    ok = ok && c[j] != 0u;
    v = (v << 5) | c[j];
  }
  key = v;
  return ok;
}

// Scan one 64-byte bucket held in registers for `key`: hit (+ fid, slot index) / empty slot seen.
__device__ __forceinline__ void scan_bucket(const uint4 (&q)[4], uint64_t key, bool& hit,
                                            bool& empty, uint32_t& fid, uint32_t& slot) {
  const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32) << 24;
  const uint32_t lo[8] = {q[0].x, q[0].z, q[1].x, q[1].z, q[2].x, q[2].z, q[3].x, q[3].z};
  const uint32_t hi[8] = {q[0].y, q[0].w, q[1].y, q[1].w, q[2].y, q[2].w, q[3].y, q[3].w};
  hit = false;
  empty = false;
#pragma unroll
  for (int j = 0; j < kSlotsPerBucket; ++j) {
    const bool m = lo[j] == klo && (hi[j] & kKeyHiMask) == khi;
    fid = m ? (hi[j] & kFidMask) : fid;
    slot = m ? (uint32_t)j : slot;
    hit = hit || m;
    empty = empty || lo[j] == 0u;
  }
}

__device__ __forceinline__ void load_bucket(const uint64_t* __restrict__ slots, uint32_t b,
                                            uint4 (&q)[4]) {
  const uint4* bp = reinterpret_cast<const uint4*>(slots + (uint64_t)b * kSlotsPerBucket);
  q[0] = bp[0];
  q[1] = bp[1];
  q[2] = bp[2];
  q[3] = bp[3];
}

// The key's overflow bit in its home bucket (held in registers).
__device__ __forceinline__ bool ovf_bit(const uint4 (&q)[4], uint64_t key) {
  const uint32_t s = ovf_index((uint32_t)key);
  const uint4 v = q[s >> 1];
  return (((s & 1) ? v.w : v.y) & kOvfBit) != 0u;
}

// Walk the overflow chain after home bucket `b` (the key missed there and its overflow bit is
// set): stop at the key or at the first bucket with an empty slot. Returns true on a hit, with
// the key's fid and slot id (bucket * 8 + slot: the key's identity in this table).
__device__ __forceinline__ bool walk_chain(const uint64_t* __restrict__ slots, uint32_t n_buckets,
                                           uint32_t b, uint64_t key, uint32_t& fid,
                                           uint32_t& sid) {
  bool hit = false, empty = false;
  uint32_t slot = 0;
  for (uint32_t step = 1; step < n_buckets && !hit && !empty; ++step) {  // bounded
    b = (b + 1 == n_buckets) ? 0 : b + 1;
    uint4 q[4];
    load_bucket(slots, b, q);
    scan_bucket(q, key, hit, empty, fid, slot);
  }
  sid = b * kSlotsPerBucket + slot;
  return hit;
}

// Full probe from the home bucket (chains included). Returns true on a hit.
__device__ __forceinline__ bool probe(const uint64_t* __restrict__ slots, uint32_t n_buckets,
                                      int k, int m, uint64_t key, uint32_t& fid) {
  const uint32_t b = home_bucket(key, k, m, n_buckets);
  uint32_t slot = 0;
  uint4 q[4];
  load_bucket(slots, b, q);
  bool hit, empty;
  scan_bucket(q, key, hit, empty, fid, slot);
  if (hit) return true;
  if (!ovf_bit(q, key)) return false;
  uint32_t sid;
  return walk_chain(slots, n_buckets, b, key, fid, sid);
}

// ---------------------------------------------------------------------------------------------
// Table construction. Insert: claim the first empty slot of the probe chain with a 64-bit CAS
// (slot key bits, fid still 0; the slot's overflow bit may already be set) or find the key
// already there; either way record the row index with atomicMax so the LAST row of a duplicate
// key wins (HashMap.put semantics). A key placed past its home bucket sets its overflow bit
// there. Finalize: write the winning row's fid into the slot; collect entry count and max
// probe.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void build_insert_kernel(uint64_t* slots, uint32_t* winner,
                                                           uint32_t n_buckets, int k, int m,
                                                           const uint64_t* __restrict__ keys,
                                                           uint64_t n, uint32_t* status) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t key = keys[i];
    if (key == 0) continue;
    const uint64_t want = slot_make(key, 0);
    const uint32_t home = home_bucket(key, k, m, n_buckets);
    uint32_t b = home;
    bool done = false;
    for (uint32_t p = 0; p < n_buckets && !done; ++p) {
      for (int j = 0; j < kSlotsPerBucket; ++j) {
        uint64_t* sp = slots + (uint64_t)b * kSlotsPerBucket + j;
        uint64_t v = __hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while ((uint32_t)v == 0u) {  // empty (possibly with its overflow bit set): claim it
          const uint64_t old = atomicCAS((unsigned long long*)sp, (unsigned long long)v, v | want);
          v = old == v ? (v | want) : old;
        }
        if (slot_key(v) == key) {
          atomicMax(winner + (uint64_t)b * kSlotsPerBucket + j, (uint32_t)(i + 1));
          done = true;
          break;
        }
      }
      if (!done) b = (b + 1 == n_buckets) ? 0 : b + 1;
    }
    if (!done) {
      atomicOr(status, 1u);  // table full: cannot happen at load factor < 1
    } else if (b != home) {
      uint32_t* hi = reinterpret_cast<uint32_t*>(
                         slots + (uint64_t)home * kSlotsPerBucket + ovf_index((uint32_t)key)) + 1;
      atomicOr(hi, kOvfBit);
    }
  }
}

__global__ __launch_bounds__(256) void build_finalize_kernel(uint64_t* slots,
                                                             const uint32_t* __restrict__ winner,
                                                             const uint32_t* __restrict__ fids,
                                                             uint32_t n_buckets, int k, int m,
                                                             uint32_t* stats) {
  const uint64_t n_slots = (uint64_t)n_buckets * kSlotsPerBucket;
  uint32_t entries = 0, max_probe = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_slots;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t w = winner[i];
    if (w == 0) continue;
    const uint64_t v = slots[i];
    slots[i] = v | ((uint64_t)(fids[w - 1] & kFidMask) << 32);
    const uint32_t b = (uint32_t)(i / kSlotsPerBucket), h = home_bucket(slot_key(v), k, m, n_buckets);
    const uint32_t d = (b >= h ? b - h : b + n_buckets - h) + 1u;
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
// K1 — probe. Residue positions g of [offsets[0], offsets[n_seq]) in grid-stride steps of
// 256 x U; each thread issues its U windows' residue loads, then packs and issues all U
// first-bucket loads (U x 64 B in flight per lane) before consuming any; overflow chains (a full
// home bucket) are walked afterwards. Windows that straddle two proteins are probed too (their
// words are never read): K1 needs no protein boundaries, no LDS set and no barrier.
// Residue loads are unconditional (a lane past the end re-reads position 0) so that no loaded
// register is merged on a branch join, which would force a vmcnt(0) per load.
// ---------------------------------------------------------------------------------------------
template <int K, int M, int U>
__global__ __launch_bounds__(256) void probe_kernel(ProteinArgs a) {
  __shared__ uint8_t lut[256];
  const int t = threadIdx.x;
  if (a.reset_flag && blockIdx.x == 0 && t < 2) a.overflow_flag[t] = 0u;  // K2 runs after K1
  lut[t] = a.lut[t];
  __syncthreads();
  const uint64_t o0 = a.offsets[0];
  const uint64_t n_all = a.n_residues >= (uint64_t)K ? a.n_residues - K + 1 : 0;
  const uint64_t seg_hi = a.offsets[a.seq_hi] - o0;
  const uint64_t n_pos = seg_hi < n_all ? seg_hi : n_all;
  const uint8_t* __restrict__ res = a.residues + o0;
  const uint64_t* __restrict__ slots = a.slots;
  const uint32_t nb = a.n_buckets;
  for (uint64_t g0 = (a.offsets[a.seq_lo] - o0) + (uint64_t)blockIdx.x * (256 * U); g0 < n_pos;
       g0 += (uint64_t)gridDim.x * (256 * U)) {
    uint64_t bytes[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint64_t g = g0 + j * 256 + t;
      bytes[j] = window_bytes(res, g < n_pos ? g : 0);
    }
    uint64_t key[U];
    uint32_t bk[U];
    bool ok[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      ok[j] = pack_window<K>(lut, bytes[j], key[j]) && g0 + j * 256 + t < n_pos;
      bk[j] = home_bucket(key[j], K, M, nb);
    }
    uint4 q[U][4];  // undefined on lanes that do not probe: consumed unconditionally below
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (ok[j]) load_bucket(slots, bk[j], q[j]);
#pragma unroll
    for (int j = 0; j < U; ++j) {
      bool hit, empty;
      uint32_t fid = 0, slot = 0;
      scan_bucket(q[j], key[j], hit, empty, fid, slot);
      hit = ok[j] && hit;
      uint32_t sid = bk[j] * kSlotsPerBucket + slot;
      if (ok[j] && !hit && ovf_bit(q[j], key[j]))  // rare: walk the overflow chain
        hit = walk_chain(slots, nb, bk[j], key[j], fid, sid);
      const uint64_t g = g0 + j * 256 + t;
      if (g < n_pos) {
        a.hits[g] = hit ? fid + 1u : 0u;
        a.sids[g] = sid;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// K1, quad-cooperative form (default). Each lane packs the key of its own windows, then the
// four lanes of a quad probe their four windows' buckets together: for the window of quad lane
// r, lane p loads bytes [16p, 16p + 16) of the bucket (one dwordx4), so one wave instruction
// reads 16 whole 64-byte lines (the access shape with the higher measured random-gather rate,
// and 4x fewer VGPRs per probe than a lane reading a whole bucket). Matches are combined with
// DPP quad reductions and kept by the window's owner lane. Adjacent lanes hold consecutive
// windows, which share their minimizer home bucket half of the time: the repeated line is
// served by the CU's L1/L2 instead of HBM. Overflow chains (~1% of probes) are deferred to the
// wave's chain queue.
// ---------------------------------------------------------------------------------------------
template <int R>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, R * 0x55, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t quad_or(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
  return v | (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
}

// One quad's verdict on a bucket it loaded cooperatively (lane `part` holds slots 2part and
// 2part + 1 in v) for key (kl, kh): fid + 1 of the matching slot in bits 0..23 (0 = not in this
// bucket), the slot's index in the bucket in bits 24..26, and bit 31 = the key's overflow bit
// (chain walk needed if there is no match). Keys are unique in
// a table, so at most one lane matches and OR is the reduction. Every lane of the quad must
// call it (DPP). Branch-free on purpose: a short-circuit here lets the compiler split the
// 16-byte load into a lazily loaded tail behind a branch and a vmcnt(0).
__device__ __forceinline__ uint32_t match_part(const uint4 v, uint32_t kl, uint32_t kh,
                                               uint32_t part) {
  const uint32_t m0 = (uint32_t)(v.x == kl) & (uint32_t)((v.y & kKeyHiMask) == kh);
  const uint32_t m1 = (uint32_t)(v.z == kl) & (uint32_t)((v.w & kKeyHiMask) == kh);
  uint32_t w = (m0 * ((v.y & kFidMask) + 1u)) | (m1 * ((v.w & kFidMask) + 1u));
  w |= (m0 | m1) * ((2u * part + m1) << kSlotShift);  // slot within the bucket
  const uint32_t ob = ovf_index(kl);
  const uint32_t hi = (ob & 1u) ? v.w : v.y;
  w |= (uint32_t)((ob >> 1) == part) & (hi >> 23) & 1u ? 0x80000000u : 0u;
  return quad_or(w);
}

// Deferred overflow-chain walks (K1). A window whose home bucket misses with the key's overflow
// bit set is written as a miss and its position queued in the wave's LDS slice; the wave
// resolves its queue 64 walks at a time (one lane each: re-pack the key, walk the chain with
// whole-bucket loads, overwrite the word), so the walk's dependent latency is paid once per
// ~64 walks rather than once per probe step.
__device__ __forceinline__ void chain_push(uint64_t* q, uint32_t& n, bool pend, uint64_t g) {
  const uint64_t m = __ballot(pend);
  if (pend) q[n + popc_below(m)] = g;
  n += (uint32_t)__popcll(m);
}
template <int K, int M>
__device__ __forceinline__ void chain_flush(const ProteinArgs& a, const uint8_t* lut,
                                         const uint8_t* __restrict__ res, const uint64_t* q,
                                         uint32_t n) {
  __builtin_amdgcn_wave_barrier();  // queue writes of other lanes are visible (LDS in order)
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t e = lane; e < n; e += 64) {
    const uint64_t g = q[e];
    uint64_t key;
    pack_window<K>(lut, window_bytes(res, g), key);
    uint32_t fid = 0, sid = 0;
    const bool hit = walk_chain(a.slots, a.n_buckets, home_bucket(key, K, M, a.n_buckets), key,
                                fid, sid);
    a.hits[g] = hit ? fid + 1u : 0u;
    a.sids[g] = sid;
  }
  __builtin_amdgcn_wave_barrier();
}

// The K1 quad loop over positions g0 + j * 256 + t (j < U) in steps of `stride`, up to n_pos
// (positions relative to offsets[0]); `cq` is the calling wave's chain queue.
template <int K, int M, int U>
__device__ __forceinline__ void probe_span(const ProteinArgs& a, const uint8_t* lut, uint64_t* cq,
                                           const uint8_t* __restrict__ res, uint64_t g0,
                                           uint64_t n_pos, uint64_t stride) {
  const int t = threadIdx.x, part = t & 3;
  uint32_t cn = 0;  // wave-uniform queue length
  const uint64_t* __restrict__ slots = a.slots;
  const uint32_t nb = a.n_buckets;
  constexpr uint32_t kNone = 0xFFFFFFFFu;
  // Software pipeline: the residues of step i + 1 are loaded while step i's buckets are in
  // flight, so a wave's only exposed latency per step is the bucket gather.
  WinWords ww[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t g = g0 + j * 256 + t;
    ww[j] = window_words(res, g < n_pos ? g : 0);
  }
  for (; g0 < n_pos; g0 += stride) {
    uint32_t klo[U], khi[U], bk[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      uint64_t key;
      const bool ok = pack_window<K>(lut, funnel(ww[j].lo, ww[j].hi, ww[j].sh), key) &&
                      g0 + j * 256 + t < n_pos;
      klo[j] = (uint32_t)key;
      khi[j] = (uint32_t)(key >> 32) << 24;
      bk[j] = ok ? home_bucket(key, K, M, nb) : kNone;
    }
    // Cooperative loads: all 4U dwordx4 of the lane in flight before any compare. A window
    // that does not probe reads bucket 0 (its result is discarded): no branch-merged loads.
    uint4 q[U][4];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint32_t b0 = quad_bcast<0>(bk[j]), b1 = quad_bcast<1>(bk[j]);
      const uint32_t b2 = quad_bcast<2>(bk[j]), b3 = quad_bcast<3>(bk[j]);
      const uint4* base = reinterpret_cast<const uint4*>(slots) + part;
      q[j][0] = base[(uint64_t)(b0 == kNone ? 0u : b0) * 4];
      q[j][1] = base[(uint64_t)(b1 == kNone ? 0u : b1) * 4];
      q[j][2] = base[(uint64_t)(b2 == kNone ? 0u : b2) * 4];
      q[j][3] = base[(uint64_t)(b3 == kNone ? 0u : b3) * 4];
    }
    // Next step's residues (issued after the bucket loads: waiting for those leaves these in
    // flight, vmcnt counts in order).
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint64_t g = g0 + stride + j * 256 + t;
      ww[j] = window_words(res, g < n_pos ? g : 0);
    }
    uint32_t word[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      word[j] = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t kl = r == 0 ? quad_bcast<0>(klo[j]) : r == 1 ? quad_bcast<1>(klo[j])
                          : r == 2 ? quad_bcast<2>(klo[j]) : quad_bcast<3>(klo[j]);
        const uint32_t kh = r == 0 ? quad_bcast<0>(khi[j]) : r == 1 ? quad_bcast<1>(khi[j])
                          : r == 2 ? quad_bcast<2>(khi[j]) : quad_bcast<3>(khi[j]);
        // Branch-free on purpose: a short-circuit here lets the compiler split the 16-byte
        // load into a lazily loaded tail behind a branch and a vmcnt(0).
        const uint32_t x = match_part(q[j][r], kl, kh, part);
        word[j] = part == r ? x : word[j];
      }
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint64_t g = g0 + j * 256 + t;
      if (g < n_pos) {
        const uint32_t w = bk[j] != kNone ? word[j] & kWordFid : 0u;
        a.hits[g] = w;
        // Slot ids only under hits (K2 reads them nowhere else): misses store nothing.
        if (w) a.sids[g] = bk[j] * kSlotsPerBucket + ((word[j] >> kSlotShift) & 7u);
      }
      chain_push(cq, cn, bk[j] != kNone && word[j] == 0x80000000u, g);  // rare: chain walk
    }
    if (cn > kChainQ - 64 * U) {
      chain_flush<K, M>(a, lut, res, cq, cn);
      cn = 0;
    }
  }
  if (cn) chain_flush<K, M>(a, lut, res, cq, cn);
}

// K1 kernel (two-kernel form, KMA_FUSED=0): the same loop as probe_span written out in the
// kernel (the register allocation of the inlined function costs it one wave per SIMD).
template <int K, int M, int U>
__global__ __launch_bounds__(256) KMA_SGPR_ATTR void probe_quad_kernel(ProteinArgs a) {
  __shared__ uint8_t lut[256];
  __shared__ uint64_t chain_q[4][kChainQ];
  const int t = threadIdx.x, part = t & 3;
  uint64_t* cq = chain_q[t >> 6];
  uint32_t cn = 0;  // wave-uniform queue length
  if (a.reset_flag && blockIdx.x == 0 && t < 2) a.overflow_flag[t] = 0u;  // K2 runs after K1
  lut[t] = a.lut[t];
  __syncthreads();
  // This segment's positions: [offsets[seq_lo], offsets[seq_hi]) relative to offsets[0],
  // clipped to the last full window of the batch.
  const uint64_t o0 = a.offsets[0];
  const uint64_t n_all = a.n_residues >= (uint64_t)K ? a.n_residues - K + 1 : 0;
  const uint64_t seg_hi = a.offsets[a.seq_hi] - o0;
  const uint64_t n_pos = seg_hi < n_all ? seg_hi : n_all;
  const uint8_t* __restrict__ res = a.residues + o0;
  const uint64_t* __restrict__ slots = a.slots;
  const uint32_t nb = a.n_buckets;
  constexpr uint32_t kNone = 0xFFFFFFFFu;
  const uint64_t stride = (uint64_t)gridDim.x * (256 * U);
  // Software pipeline: the residues of step i + 1 are loaded while step i's buckets are in
  // flight, so a wave's only exposed latency per step is the bucket gather.
  uint64_t g0 = (a.offsets[a.seq_lo] - o0) + (uint64_t)blockIdx.x * (256 * U);
  WinWords ww[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t g = g0 + j * 256 + t;
    ww[j] = window_words(res, g < n_pos ? g : 0);
  }
  for (; g0 < n_pos; g0 += stride) {
    uint32_t klo[U], khi[U], bk[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      uint64_t key;
      const bool ok = pack_window<K>(lut, funnel(ww[j].lo, ww[j].hi, ww[j].sh), key) &&
                      g0 + j * 256 + t < n_pos;
      klo[j] = (uint32_t)key;
      khi[j] = (uint32_t)(key >> 32) << 24;
      bk[j] = ok ? home_bucket(key, K, M, nb) : kNone;
    }
    // Cooperative loads: all 4U dwordx4 of the lane in flight before any compare. A window
    // that does not probe reads bucket 0 (its result is discarded): no branch-merged loads.
    uint4 q[U][4];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint32_t b0 = quad_bcast<0>(bk[j]), b1 = quad_bcast<1>(bk[j]);
      const uint32_t b2 = quad_bcast<2>(bk[j]), b3 = quad_bcast<3>(bk[j]);
      const uint4* base = reinterpret_cast<const uint4*>(slots) + part;
      q[j][0] = base[(uint64_t)(b0 == kNone ? 0u : b0) * 4];
      q[j][1] = base[(uint64_t)(b1 == kNone ? 0u : b1) * 4];
      q[j][2] = base[(uint64_t)(b2 == kNone ? 0u : b2) * 4];
      q[j][3] = base[(uint64_t)(b3 == kNone ? 0u : b3) * 4];
    }
    // Next step's residues (issued after the bucket loads: waiting for those leaves these in
    // flight, vmcnt counts in order).
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint64_t g = g0 + stride + j * 256 + t;
      ww[j] = window_words(res, g < n_pos ? g : 0);
    }
    uint32_t word[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      word[j] = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t kl = r == 0 ? quad_bcast<0>(klo[j]) : r == 1 ? quad_bcast<1>(klo[j])
                          : r == 2 ? quad_bcast<2>(klo[j]) : quad_bcast<3>(klo[j]);
        const uint32_t kh = r == 0 ? quad_bcast<0>(khi[j]) : r == 1 ? quad_bcast<1>(khi[j])
                          : r == 2 ? quad_bcast<2>(khi[j]) : quad_bcast<3>(khi[j]);
        // Branch-free on purpose: a short-circuit here lets the compiler split the 16-byte
        // load into a lazily loaded tail behind a branch and a vmcnt(0).
        const uint32_t x = match_part(q[j][r], kl, kh, part);
        word[j] = part == r ? x : word[j];
      }
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint64_t g = g0 + j * 256 + t;
      if (g < n_pos) {
        const uint32_t w = bk[j] != kNone ? word[j] & kWordFid : 0u;
        a.hits[g] = w;
        // Slot ids only under hits (K2 reads them nowhere else): misses store nothing.
        if (w) a.sids[g] = bk[j] * kSlotsPerBucket + ((word[j] >> kSlotShift) & 7u);
      }
      chain_push(cq, cn, bk[j] != kNone && word[j] == 0x80000000u, g);  // rare: chain walk
    }
    if (cn > kChainQ - 64 * U) {
      chain_flush<K, M>(a, lut, res, cq, cn);
      cn = 0;
    }
  }
  if (cn) chain_flush<K, M>(a, lut, res, cq, cn);
}

// ---------------------------------------------------------------------------------------------
// K1, run form (KMA_PROBE=run). Each lane takes R consecutive windows (a run); with minimizer home
// buckets consecutive windows often share their bucket, so a bucket is requested only where
// the run's bucket changes — a repeated one reads the (cache-hot) bucket 0 line instead and
// reuses the registers of the previous window. Loads are quad-cooperative as in
// probe_quad_kernel (the four lanes of a quad read one bucket, a dwordx4 each), all distinct
// loads of the step in flight before any compare, and the next step's residues are loaded
// under them. One 24-byte residue read per lane covers its R + K - 1 residues; the run's R
// result words leave in one 16-byte store.
// ---------------------------------------------------------------------------------------------
template <int K, int M, int R>
__global__ __launch_bounds__(256) void probe_run_kernel(ProteinArgs a) {
  static_assert(R + K - 1 + 7 <= 24, "a run's residues must fit three aligned words");
  __shared__ uint8_t lut[256];
  __shared__ uint64_t chain_q[4][kChainQ];
  const int t = threadIdx.x, part = t & 3;
  uint64_t* cq = chain_q[t >> 6];
  uint32_t cn = 0;  // wave-uniform queue length
  if (a.reset_flag && blockIdx.x == 0 && t < 2) a.overflow_flag[t] = 0u;  // K2 runs after K1
  lut[t] = a.lut[t];
  __syncthreads();
  const uint64_t o0 = a.offsets[0];
  const uint64_t n_all = a.n_residues >= (uint64_t)K ? a.n_residues - K + 1 : 0;
  const uint64_t seg_hi = a.offsets[a.seq_hi] - o0;
  const uint64_t n_pos = seg_hi < n_all ? seg_hi : n_all;
  const uint8_t* __restrict__ res = a.residues + o0;
  const uint64_t* __restrict__ slots = a.slots;
  const uint4* __restrict__ part_base = reinterpret_cast<const uint4*>(slots) + part;
  const uint32_t nb = a.n_buckets;
  constexpr uint32_t kNone = 0xFFFFFFFFu;
  const uint64_t stride = (uint64_t)gridDim.x * (256 * R);
  uint64_t g0 = (a.offsets[a.seq_lo] - o0) + (uint64_t)blockIdx.x * (256 * R);
  // Residue words of this lane's run, loaded one step ahead.
  uint64_t rw[3];
  uint32_t rsh;
  {
    const uint64_t gl = g0 + (uint64_t)t * R, gc = gl < n_pos ? gl : 0;
    const uint64_t* src = reinterpret_cast<const uint64_t*>(res + (gc & ~7ull));
    rw[0] = src[0];
    rw[1] = src[1];
    rw[2] = src[2];
    rsh = (uint32_t)(gc & 7);
  }
  for (; g0 < n_pos; g0 += stride) {
    const uint64_t gl = g0 + (uint64_t)t * R;
    uint32_t klo[R], khi[R], bk[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t o = rsh + j;  // byte offset of window j in the 24-byte stream
      const uint64_t bytes = o < 8 ? funnel(rw[0], rw[1], o * 8) : funnel(rw[1], rw[2], (o - 8) * 8);
      uint64_t key;
      const bool ok = pack_window<K>(lut, bytes, key) && gl + j < n_pos;
      klo[j] = (uint32_t)key;
      khi[j] = (uint32_t)(key >> 32) << 24;
      bk[j] = ok ? home_bucket(key, K, M, nb) : kNone;
    }
    // Distinct buckets along the run: window j requests only if its bucket differs from j-1's.
    uint32_t fresh[R];
#pragma unroll
    for (int j = 0; j < R; ++j)
      fresh[j] = bk[j] != kNone && (j == 0 || bk[j] != bk[j - 1]) ? 1u : 0u;
    uint4 q[R][4];
#pragma unroll
    for (int j = 0; j < R; ++j) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t b = r == 0 ? quad_bcast<0>(bk[j]) : r == 1 ? quad_bcast<1>(bk[j])
                         : r == 2 ? quad_bcast<2>(bk[j]) : quad_bcast<3>(bk[j]);
        const uint32_t f = r == 0 ? quad_bcast<0>(fresh[j]) : r == 1 ? quad_bcast<1>(fresh[j])
                         : r == 2 ? quad_bcast<2>(fresh[j]) : quad_bcast<3>(fresh[j]);
        q[j][r] = part_base[(uint64_t)(f ? b : 0u) * 4];  // repeated bucket: hot line 0
      }
    }
    // Next step's residues under the bucket loads (raw words: consumed next step).
    {
      const uint64_t gn = gl + stride, gc = gn < n_pos ? gn : 0;
      const uint64_t* src = reinterpret_cast<const uint64_t*>(res + (gc & ~7ull));
      rw[0] = src[0];
      rw[1] = src[1];
      rw[2] = src[2];
      rsh = (uint32_t)(gc & 7);
    }
    uint32_t word[R], sid[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      word[j] = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t f = r == 0 ? quad_bcast<0>(fresh[j]) : r == 1 ? quad_bcast<1>(fresh[j])
                         : r == 2 ? quad_bcast<2>(fresh[j]) : quad_bcast<3>(fresh[j]);
        if (j > 0) {  // a repeated bucket takes the previous window's data (selects, no branch)
          q[j][r].x = f ? q[j][r].x : q[j - 1][r].x;
          q[j][r].y = f ? q[j][r].y : q[j - 1][r].y;
          q[j][r].z = f ? q[j][r].z : q[j - 1][r].z;
          q[j][r].w = f ? q[j][r].w : q[j - 1][r].w;
        }
        const uint32_t kl = r == 0 ? quad_bcast<0>(klo[j]) : r == 1 ? quad_bcast<1>(klo[j])
                          : r == 2 ? quad_bcast<2>(klo[j]) : quad_bcast<3>(klo[j]);
        const uint32_t kh = r == 0 ? quad_bcast<0>(khi[j]) : r == 1 ? quad_bcast<1>(khi[j])
                          : r == 2 ? quad_bcast<2>(khi[j]) : quad_bcast<3>(khi[j]);
        // Branch-free on purpose (a short-circuit lets the compiler split the 16-byte load).
        const uint32_t x = match_part(q[j][r], kl, kh, part);
        word[j] = part == r ? x : word[j];
      }
    }
    bool pend[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      pend[j] = bk[j] != kNone && word[j] == 0x80000000u;  // rare: chain walk, deferred
      sid[j] = bk[j] * kSlotsPerBucket + ((word[j] >> kSlotShift) & 7u);
      word[j] = bk[j] != kNone ? word[j] & kWordFid : 0u;
    }
    if (R == 4 && gl + R <= n_pos && (gl & 3) == 0) {
      *reinterpret_cast<uint4*>(a.hits + gl) = make_uint4(word[0], word[1], word[2], word[3]);
      *reinterpret_cast<uint4*>(a.sids + gl) = make_uint4(sid[0], sid[1], sid[2], sid[3]);
    } else {
#pragma unroll
      for (int j = 0; j < R; ++j)
        if (gl + j < n_pos) a.hits[gl + j] = word[j], a.sids[gl + j] = sid[j];
    }
#pragma unroll
    for (int j = 0; j < R; ++j) chain_push(cq, cn, pend[j], gl + j);
    if (cn > kChainQ - 64 * R) {
      chain_flush<K, M>(a, lut, res, cq, cn);
      cn = 0;
    }
  }
  if (cn) chain_flush<K, M>(a, lut, res, cq, cn);
}

// Open-addressing set of distinct hit keys (u64, 0 = empty) in LDS or global memory, capacity a
// power of two at least twice the keys it can receive. Returns true if newly inserted.
__device__ __forceinline__ uint32_t set_hash(uint64_t key) {
  return (uint32_t)key * 0x9E3779B1u ^ (uint32_t)(key >> 32) * 0x85EBCA77u;
}
__device__ __forceinline__ bool set_insert(unsigned long long* set, uint32_t mask, uint64_t key) {
  uint32_t h = set_hash(key) & mask;
  for (;;) {
    const unsigned long long old = atomicCAS(set + h, 0ull, (unsigned long long)key);
    if (old == 0ull) return true;
    if (old == key) return false;
    h = (h + 1u) & mask;
  }
}
// Set capacity for h keys: a power of two >= 2h (linear probing stays short at load <= 1/2;
// tighter sets measured slower: LDS CAS retries are dependent round trips).
__device__ __forceinline__ uint32_t set_cap(uint32_t h) {
  uint32_t cap = 8;
  while (cap < 2 * h) cap <<= 1;
  return cap;
}

// A protein with one role whose distinct-key set does not fit K2's LDS: appended to the
// workspace's pending list (its length is the word K1 zeroes) with what K2 learned of it, and
// counted by vote_long_kernel.
// Two lists: sets of up to kLongWaveSet ids (a wave each in vote_long_kernel; length in
// overflow_flag[0], records from pending[0]) and larger ones (a block each; length in
// overflow_flag[1], records from pending[pending_half]).
__device__ __forceinline__ void push_pending(const ProteinArgs& a, uint32_t s, uint32_t fid,
                                             uint32_t hits, uint64_t base, uint32_t n_win) {
  const bool big = set_cap(hits) > (uint32_t)kLongWaveSet;
  PendingRec* r = big ? a.pending + a.pending_half + atomicAdd(a.overflow_flag + 1, 1u)
                      : a.pending + atomicAdd(a.overflow_flag, 1u);
  *r = PendingRec{s, fid, hits, n_win, base};
}

__device__ __forceinline__ void write_vote(const ProteinArgs& a, uint32_t s, uint32_t mn,
                                           uint32_t mx, uint32_t cnt) {
  int32_t fid_out = -1, cnt_out = 0;
  uint8_t st;
  if (mn == 0xFFFFFFFFu) {
    st = KMA_STATUS_NONE;  // roleId == null
  } else if (mn != mx) {
    st = KMA_STATUS_AMBIGUOUS;  // badPeg
  } else {
    fid_out = (int32_t)mn;
    cnt_out = (int32_t)cnt;
    st = cnt >= (uint32_t)a.min_hits ? KMA_STATUS_CALLED : KMA_STATUS_BELOW_MIN;
    if (st == KMA_STATUS_CALLED && a.tally && mn < a.n_fid) atomicAdd(a.tally + mn, 1u);
  }
  a.out_fid[s] = fid_out;
  a.out_count[s] = cnt_out;
  a.out_status[s] = st;
}

__device__ __forceinline__ int64_t n_windows(const ProteinArgs& a, uint32_t s, int k) {
  return (int64_t)(a.offsets[s + 1] - a.offsets[s]) - k +
         ((a.flags & KMA_F_END_EXCLUSIVE) ? 0 : 1);
}

// The vote over a window range held by one thread group: V words and V residue windows per
// lane per step, all loaded before any is consumed (clamped addresses, no branch-merged loads).
// Hit keys are re-packed from the residues and inserted in `set` unless multiset.
template <int K, int V, int STRIDE>
__device__ __forceinline__ void vote_range(const ProteinArgs& a, const uint8_t* lut,
                                           const uint32_t* __restrict__ words,
                                           const uint8_t* __restrict__ res, int64_t n_win,
                                           int64_t first, unsigned long long* set, uint32_t mask,
                                           bool multiset, uint32_t& fmin, uint32_t& fmax,
                                           uint32_t& cnt) {
  for (int64_t w0 = first; w0 < n_win; w0 += (int64_t)STRIDE * V) {
    uint32_t h[V];
    uint64_t bytes[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int64_t w = w0 + v * STRIDE;
      const int64_t wc = w < n_win ? w : n_win - 1;
      const uint32_t x = words[wc];
      bytes[v] = window_bytes(res, (uint64_t)wc);
      h[v] = w < n_win ? x : 0u;
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {
      if (h[v]) {
        fmin = min(fmin, h[v] - 1u);
        fmax = max(fmax, h[v] - 1u);
        if (multiset) {
          cnt++;
        } else {
          uint64_t key;
          pack_window<K>(lut, bytes[v], key);
          cnt += set_insert(set, mask, key) ? 1u : 0u;
        }
      }
    }
  }
}

// ---- K2 chunks ---------------------------------------------------------------------------------
// A protein's windows are word indices [base, base + n_win) of the K1 words (base = its first
// residue relative to offsets[0]; word x belongs to residue offsets[0] + x). K2 cuts them into
// chunks of kChunk windows on a 4-aligned grid starting at base & ~3: lane l of a wave holds
// the four consecutive windows X..X+3, X = (base & ~3) + kChunk * q + 4l, so its words are one
// aligned 16-byte load and its residues (4 + K - 1 bytes) three aligned 8-byte words.
struct Chunk {
  uint32_t h[4];    // K1 word of each window (0: miss, outside the protein, or dead chunk)
  uint32_t sid[4];  // K1 slot id of each hit window: the key's identity in the table
};
static_assert(kVoteWin == 4, "a lane holds four consecutive windows of a chunk");

__device__ __forceinline__ uint32_t chunks_of(uint64_t base, uint32_t n_win) {
  return n_win ? (uint32_t)(((base & 3u) + n_win + kChunk - 1) / kChunk) : 0u;
}

// Load chunk q of the protein at word index `base` with n_win >= 1 windows (live) — or, for a
// dead chunk (!live), harmless reads of word 0 whose results are dropped. Unconditional,
// clamped loads: no branch-merged registers.
__device__ __forceinline__ void load_chunk(const ProteinArgs& a, uint64_t base, uint32_t n_win,
                                           uint32_t q, bool live, int lane, Chunk& c) {
  const uint64_t last = live ? base + n_win - 1 : 0;
  const uint64_t X = live ? (base & ~3ull) + (uint64_t)q * kChunk + 4u * lane : 0;
  const uint64_t Xc = X <= last ? X : (last & ~3ull);
  const uint4 w = *reinterpret_cast<const uint4*>(a.hits + Xc);
  const uint4 d = *reinterpret_cast<const uint4*>(a.sids + Xc);
  c.sid[0] = d.x;
  c.sid[1] = d.y;
  c.sid[2] = d.z;
  c.sid[3] = d.w;
  const uint32_t x[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) c.h[j] = (live && X + j >= base && X + j <= last) ? x[j] : 0u;
}

// Insert the chunk's hit keys in `set` (u32 entries: slot id + 1, 0 = empty; capacity cap, a
// power of two); returns the wave's number of new keys. A key's slot id is unique in the table,
// so equal ids are equal kmers. The first attempts of the lane's four inserts are independent
// CASes issued together (one LDS round trip); only a taken slot holding another id continues.
__device__ __forceinline__ uint32_t dedupe_insert(uint32_t* set, uint32_t cap, const Chunk& c) {
  uint32_t key[4], slot[4], old[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    key[j] = c.sid[j] + 1u;
    slot[j] = mix32(key[j]) & (cap - 1u);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) old[j] = c.h[j] ? atomicCAS(set + slot[j], 0u, key[j]) : key[j];
  uint32_t fresh = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (old[j] == 0u) {
      fresh++;
    } else if (old[j] != key[j]) {
      uint32_t i = slot[j];
      for (;;) {
        i = (i + 1u) & (cap - 1u);
        const uint32_t o = atomicCAS(set + i, 0u, key[j]);
        if (o == 0u) { fresh++; break; }
        if (o == key[j]) break;
      }
    }
  }
  return wave_sum(fresh);
}

// ---------------------------------------------------------------------------------------------
// K2 — vote. A block of kVoteWaves waves owns kVoteProteins consecutive proteins; their chunks
// are dealt to the waves round-robin (chunk c to wave c % kVoteWaves), so a long protein is
// spread over the block instead of one wave (no serial tail).
//   pass 1: a wave loads its first kVoteHold chunks (words + slot ids) at once and keeps them
//           in registers; per chunk, min fid, max fid and hits H go to LDS. No hit -> NONE; two
//           roles -> AMBIGUOUS (badPeg); multiset -> count H; H < 2 -> count H: no set.
//   pass 2: a protein with one role and H >= 2 gets a set of set_cap(H) u32 entries from the
//           block's LDS pool; each hit window's slot id (K1: the key's unique slot in the
//           table) is inserted, so a kmer occurring twice in one protein counts once
//           (ProteinKmers is a set). Chunks past the held ones (long proteins) are reloaded.
//   phase 3: proteins whose set did not fit beside the others take the whole pool in turn.
// A protein whose set exceeds the pool is marked pending for vote_long_kernel.
// The kernel is bound by dependent latency (offsets -> words -> LDS atomics; measured per phase
// with KMA_VOTE_TRACE builds), so every wave has all its loads in flight at once and blocks are
// small enough (LDS, registers) for many to be resident.
// ---------------------------------------------------------------------------------------------
// K2's LDS (a struct so that the fused kernel can overlay it on K1's chain queues).
template <int P>
struct VoteSmem {
  __attribute__((aligned(16))) uint32_t pool[kVotePool];
  uint64_t pbase_w[P];  // word index of window 0
  uint32_t pwin[P], chunk0[P + 1], pmin[P], pmax[P], phits[P], pcnt[P], pbase[P], pcap[P];
  uint32_t pool_top;
};

// The vote of proteins [p0, p0 + np) by the block (np <= P).
template <int K, int P>
__device__ __forceinline__ void vote_group(const ProteinArgs& a, VoteSmem<P>& sm, uint32_t p0,
                                           int np) {
  constexpr int W = kVoteWaves;
  constexpr int U = kVoteHold;
  static_assert(P <= 64 && (P & (P - 1)) == 0, "header is one wave; binary search needs 2^n");
  uint32_t* pool = sm.pool;
  uint64_t* pbase_w = sm.pbase_w;
  uint32_t *pwin = sm.pwin, *chunk0 = sm.chunk0, *pmin = sm.pmin, *pmax = sm.pmax,
           *phits = sm.phits, *pcnt = sm.pcnt, *pbase = sm.pbase, *pcap = sm.pcap;
  uint32_t& pool_top = sm.pool_top;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const bool multiset = (a.flags & KMA_F_MULTISET) != 0;
#ifdef KMA_VOTE_TRACE
  if (tid > 0 && tid < 7) a.scratch[blockIdx.x * 8 + tid] = 0;
  if (tid == 0) a.scratch[blockIdx.x * 8 + 0] = wall_clock64();
#define KMA_TRACE_AT(n) \
  if (tid == 0) a.scratch[blockIdx.x * 8 + (n)] = wall_clock64();
#else
#define KMA_TRACE_AT(n)
#endif
  if (wave == 0) {  // header: windows, chunk prefix (wave scan)
    uint32_t w = 0, nc = 0;
    uint64_t base = 0;
    if (lane < np) {
      const int64_t n = n_windows(a, p0 + lane, K);
      w = n > 0 ? (uint32_t)n : 0u;
      base = a.offsets[p0 + lane] - a.offsets[0];
      nc = chunks_of(base, w);
    }
    uint32_t incl = nc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = (uint32_t)__shfl_up((int)incl, o, 64);
      incl += lane >= o ? x : 0u;
    }
    if (lane < P) {
      pbase_w[lane] = base;
      pwin[lane] = w;
      chunk0[lane] = incl - nc;
      pmin[lane] = 0xFFFFFFFFu;
      pmax[lane] = 0u;
      phits[lane] = 0u;
      pcnt[lane] = 0u;
      pcap[lane] = 0u;
      if (lane == P - 1) chunk0[P] = incl;
    }
    if (lane == 0) pool_top = 0;
  }
  __syncthreads();
  KMA_TRACE_AT(1)
  const uint32_t n_chunks = chunk0[P];
#ifdef KMA_VOTE_TRACE
  if (tid == 0) a.scratch[blockIdx.x * 8 + 7] = n_chunks;
#endif
  // The protein of chunk c: the last p with chunk0[p] <= c (proteins without chunks skipped).
  auto owner = [&](uint32_t c) {
    uint32_t p = 0;
#pragma unroll
    for (uint32_t step = P / 2; step > 0; step >>= 1) p += chunk0[p + step] <= c ? step : 0u;
    return p;
  };
  auto reduce_chunk = [&](const Chunk& ch, uint32_t p) {
    uint32_t fmin = 0xFFFFFFFFu, fmax = 0u, hits = 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (ch.h[j]) {
        fmin = min(fmin, ch.h[j] - 1u);
        fmax = max(fmax, ch.h[j] - 1u);
        hits++;
      }
    fmin = wave_min(fmin);
    fmax = wave_max(fmax);
    hits = wave_sum(hits);
    if (lane == 0 && hits) {
      atomicMin(pmin + p, fmin);
      atomicMax(pmax + p, fmax);
      atomicAdd(phits + p, hits);
    }
  };
  // ---- pass 1 ----------------------------------------------------------------------------------
  Chunk held[U];
  uint32_t hp[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t c = wave + u * W;
    const bool live = c < n_chunks;  // wave-uniform
    const uint32_t p = owner(live ? c : 0u);
    hp[u] = p;
    load_chunk(a, pbase_w[p], pwin[p], live ? c - chunk0[p] : 0u, live, lane, held[u]);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) reduce_chunk(held[u], hp[u]);
  for (uint32_t c = wave + U * W; c < n_chunks; c += W) {  // long proteins
    const uint32_t p = owner(c);
    Chunk ch;
    load_chunk(a, pbase_w[p], pwin[p], c - chunk0[p], true, lane, ch);
    reduce_chunk(ch, p);
  }
  __syncthreads();
  KMA_TRACE_AT(2)
  // ---- decide; take sets from the pool -------------------------------------------------------
  // Outputs are written after the block's last barrier: a barrier waits for the block's
  // outstanding global stores (one vmcnt for loads and stores on this architecture).
  if (tid < np) {
    const uint32_t mn = pmin[tid], mx = pmax[tid], h = phits[tid];
    if (mn == 0xFFFFFFFFu || mn != mx || multiset || h < 2) {
      pcnt[tid] = h;  // final now: count = H
    } else {
      const uint32_t cap = set_cap(h);
      const uint32_t base = atomicAdd(&pool_top, cap);
      if (base + cap <= (uint32_t)kVotePool) {
        pbase[tid] = base;
        pcap[tid] = cap;
      } else if (cap <= (uint32_t)kVotePool) {
        pcap[tid] = cap | kDeferred;  // phase 3: the whole pool, after pass 2
      } else {
        pcap[tid] = kLongCap;  // vote_long_kernel, global-memory set
      }
    }
  }
  __syncthreads();
  KMA_TRACE_AT(3)
  // Every protein's output, after the last barrier.
  auto finish = [&]() {
    if (tid < np) {
      if (pcap[tid] == kLongCap) {
        push_pending(a, p0 + tid, pmin[tid], phits[tid], pbase_w[tid], pwin[tid]);
      } else {
        write_vote(a, p0 + tid, pmin[tid], pmax[tid], pcnt[tid]);
      }
    }
  };
  const uint32_t used = min(pool_top, (uint32_t)kVotePool);
  bool deferred = false;
  for (int p = 0; p < np; ++p) deferred |= (pcap[p] & kDeferred) && pcap[p] != kLongCap;
  if (used == 0 && !deferred) {  // block-uniform: no protein needs the pool
    finish();
    return;
  }
  uint4* pool4 = reinterpret_cast<uint4*>(pool);
  for (uint32_t i = tid; i < used / 4; i += 64 * W) pool4[i] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
  KMA_TRACE_AT(4)
  // ---- pass 2: distinct hit keys ----------------------------------------------------------------
#ifndef KMA_ABL_NOPASS2  // timing ablation only
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t c = wave + u * W, p = hp[u];
    const uint32_t cap = pcap[p];
    if (c >= n_chunks || cap == 0 || (cap & kDeferred)) continue;  // wave-uniform (kLongCap too)
    const uint32_t fresh = dedupe_insert(pool + pbase[p], cap, held[u]);
    if (lane == 0 && fresh) atomicAdd(pcnt + p, fresh);
  }
  for (uint32_t c = wave + U * W; c < n_chunks; c += W) {
    const uint32_t p = owner(c);
    const uint32_t cap = pcap[p];
    if (cap == 0 || (cap & kDeferred)) continue;  // wave-uniform
    Chunk ch;
    load_chunk(a, pbase_w[p], pwin[p], c - chunk0[p], true, lane, ch);
    const uint32_t fresh = dedupe_insert(pool + pbase[p], cap, ch);
    if (lane == 0 && fresh) atomicAdd(pcnt + p, fresh);
  }
#endif
  __syncthreads();
  KMA_TRACE_AT(5)
  // ---- phase 3: proteins that did not fit beside the others take the whole pool in turn ------
  for (int p = 0; p < np; ++p) {
    const uint32_t cap = pcap[p];
    if (!(cap & kDeferred) || cap == kLongCap) continue;  // block-uniform
    const uint32_t c2 = cap & ~kDeferred;
    __syncthreads();  // the pool's previous contents are no longer read
    for (uint32_t i = tid; i < c2 / 4; i += 64 * W) pool4[i] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    for (uint32_t c = chunk0[p] + wave; c < chunk0[p + 1]; c += W) {
      Chunk ch;
      load_chunk(a, pbase_w[p], pwin[p], c - chunk0[p], true, lane, ch);
      const uint32_t fresh = dedupe_insert(pool, c2, ch);
      if (lane == 0 && fresh) atomicAdd(pcnt + p, fresh);
    }
  }
  __syncthreads();
  finish();
  KMA_TRACE_AT(6)
#undef KMA_TRACE_AT
}

template <int K>
__global__ __launch_bounds__(64 * kVoteWaves) void vote_kernel(ProteinArgs a) {
  __shared__ VoteSmem<kVoteProteins> sm;
  const uint32_t p0 = a.seq_lo + blockIdx.x * kVoteProteins;
  vote_group<K, kVoteProteins>(a, sm, p0, (int)min<uint32_t>(kVoteProteins, a.seq_hi - p0));
}

// ---------------------------------------------------------------------------------------------
// K12 — fused probe + vote (default). A block owns kVoteProteins consecutive proteins: it probes
// every residue position of their span with K1's quad loop (words and slot ids to the
// workspace, where they stay L2-resident), then votes them with K2's block logic. No second
// kernel, no kernel boundary between the phases, and one block's vote (latency-bound LDS and
// L2 work) overlaps the bucket gathers of the blocks around it. K1's chain queues and K2's
// set pool share the block's LDS.
// ---------------------------------------------------------------------------------------------
template <int K, int M, int P>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7, 8))) KMA_SGPR_ATTR void annotate_kernel(ProteinArgs a) {
  constexpr int U = kProbeWin;
  __shared__ uint8_t lut[256];
  __shared__ union Smem {
    uint64_t chain_q[4][kChainQ];
    VoteSmem<P> vote;
  } sm;
  const int t = threadIdx.x;
  lut[t] = a.lut[t];
  const uint32_t p0 = a.seq_lo + blockIdx.x * P;
  const int np = (int)min<uint32_t>(P, a.seq_hi - p0);
  __syncthreads();
  const uint64_t o0 = a.offsets[0];
  const uint64_t n_all = a.n_residues >= (uint64_t)K ? a.n_residues - K + 1 : 0;
  const uint64_t lo = a.offsets[p0] - o0, hi = a.offsets[p0 + np] - o0;
  probe_span<K, M, U>(a, lut, sm.chain_q[t >> 6], a.residues + o0, lo, hi < n_all ? hi : n_all,
                      256 * U);
  __syncthreads();  // this block's words and slot ids are written (and visible to its waves)
  vote_group<K, P>(a, sm.vote, p0, np);
}

// ---------------------------------------------------------------------------------------------
// K2, wave form (KMA_VOTE=wave). One wave per protein, one pass, no barrier: the wave streams its
// protein's chunks (kWaveHold at a time, all in flight; 4 consecutive windows per lane as in
// vote_kernel), reducing min fid / max fid / hits H (DPP wave reductions) and inserting every
// hit's slot id into the wave's LDS set slice as it goes — speculatively, before the role is
// known, so no chunk is read twice and no wave waits for another:
//   NONE / AMBIGUOUS / multiset / H < 2 -> from the reductions;
//   one role, H >= 2 -> count = distinct slot ids (ProteinKmers is a set);
//   the set is capped at 3/4 of its kWaveSet slots: a protein that would pass the cap stops
//   inserting and, if it has one role and H >= 2, goes to vote_long_kernel (pending list).
// ---------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(256) void vote_wave_kernel(ProteinArgs a) {
  constexpr int U = kWaveHold;
  constexpr uint32_t S = kWaveSet;
  static_assert((S & (S - 1)) == 0 && S >= 512, "set slice: a power of two");
  __shared__ __attribute__((aligned(16))) uint32_t sets[4][S];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const uint32_t s = a.seq_lo + blockIdx.x * 4u + wave;
  if (s >= a.seq_hi) return;  // wave-uniform; no barrier anywhere in this kernel
  uint32_t* set = sets[wave];
  uint4* set4 = reinterpret_cast<uint4*>(set);
  for (uint32_t e = lane; e < S / 4; e += 64) set4[e] = make_uint4(0u, 0u, 0u, 0u);
  const uint64_t o0 = a.offsets[0], beg = a.offsets[s], end = a.offsets[s + 1];
  const int64_t n = (int64_t)(end - beg) - K + ((a.flags & KMA_F_END_EXCLUSIVE) ? 0 : 1);
  const uint32_t n_win = n > 0 ? (uint32_t)n : 0u;
  const uint64_t base = beg - o0;
  const uint32_t nc = chunks_of(base, n_win);
  uint32_t mn = 0xFFFFFFFFu, mx = 0u, hits = 0u, distinct = 0u;
  bool full = false;  // wave-uniform
  for (uint32_t c0 = 0; c0 < nc; c0 += U) {
    Chunk ch[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      load_chunk(a, base, n_win, c0 + u < nc ? c0 + u : 0u, c0 + u < nc, lane, ch[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (c0 + u >= nc) break;  // wave-uniform
      uint32_t fmin = 0xFFFFFFFFu, fmax = 0u, h = 0u;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (ch[u].h[j]) {
          fmin = min(fmin, ch[u].h[j] - 1u);
          fmax = max(fmax, ch[u].h[j] - 1u);
          h++;
        }
      h = wave_sum(h);
      if (h == 0u) continue;  // wave-uniform
      mn = min(mn, wave_min(fmin));
      mx = max(mx, wave_max(fmax));
      hits += h;
      full = full || distinct + h > S * 3 / 4;
      if (!full) distinct += dedupe_insert(set, S, ch[u]);
    }
  }
  if (lane == 0) {
    if (mn == 0xFFFFFFFFu || mn != mx || (a.flags & KMA_F_MULTISET) || hits < 2)
      write_vote(a, s, mn, mx, hits);
    else if (full)
      push_pending(a, s, mn, hits, base, n_win);  // vote_long_kernel
    else
      write_vote(a, s, mn, mx, distinct);
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

// K2 for the pending proteins (sets too large for K2's LDS): one block per protein,
// grid-striding over the workspace's pending list.
// Proteins of up to kLongSet / 2 windows keep their distinct-key set in LDS; longer ones are
// taken by the first kFallbackBlocks blocks with a set in their slice of workspace scratch
// (kFallbackCap u64); longer still are TOO_LONG.
template <int K>
__device__ void vote_long_one(const ProteinArgs& a, const uint8_t* lut, uint32_t s, int64_t n_win,
                              unsigned long long* set, uint32_t cap, uint32_t* red) {
  const int tid = threadIdx.x;
  const bool multiset = (a.flags & KMA_F_MULTISET) != 0;
  if (!multiset)
    for (uint32_t i = tid; i < cap; i += blockDim.x) set[i] = 0ull;
  __syncthreads();
  const uint64_t beg = a.offsets[s];
  uint32_t fmin = 0xFFFFFFFFu, fmax = 0u, cnt = 0u;
  vote_range<K, kVoteWin, 256>(a, lut, a.hits + (beg - a.offsets[0]), a.residues + beg, n_win,
                               tid, set, cap - 1, multiset, fmin, fmax, cnt);
  fmin = block_reduce(fmin, red, 0);
  fmax = block_reduce(fmax, red, 1);
  cnt = block_reduce(cnt, red, 2);
  if (tid == 0) write_vote(a, s, fmin, fmax, cnt);
  __syncthreads();  // the set is reused by the next protein
}

template <int K>
__global__ __launch_bounds__(256) void vote_long_kernel(ProteinArgs a) {
  const uint32_t nw = __hip_atomic_load(a.overflow_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t nb = __hip_atomic_load(a.overflow_flag + 1, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
  if (blockIdx.x * 4u >= nw && blockIdx.x >= nb) return;
  __shared__ __attribute__((aligned(16))) unsigned long long lds_set[kLongSet];
  __shared__ uint8_t lut[256];
  __shared__ uint32_t red[kWavesPerBlock];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  lut[tid] = a.lut[tid];
  __syncthreads();
  // Sets of up to kLongWaveSet slot ids: one wave per protein, a quarter of the LDS set each.
  // The role is known (K2 found one), so only the distinct keys are counted; all of the
  // protein's chunks (up to kLongHold at a time) are in flight together.
  uint32_t* wset = reinterpret_cast<uint32_t*>(lds_set) + wave * kLongWaveSet;
  for (uint32_t i = blockIdx.x * 4u + wave; i < nw; i += gridDim.x * 4u) {
    const PendingRec r = a.pending[i];
    const uint32_t cap = set_cap(r.hits);
    uint4* set4 = reinterpret_cast<uint4*>(wset);
    for (uint32_t e = lane; e < cap / 4; e += 64) set4[e] = make_uint4(0u, 0u, 0u, 0u);
    const uint32_t nc = chunks_of(r.base, r.n_win);
    uint32_t cnt = 0;
    for (uint32_t c = 0; c < nc; c += kLongHold) {
      Chunk ch[kLongHold];
#pragma unroll
      for (int u = 0; u < kLongHold; ++u)
        load_chunk(a, r.base, r.n_win, c + u < nc ? c + u : 0u, c + u < nc, lane, ch[u]);
#pragma unroll
      for (int u = 0; u < kLongHold; ++u)
        if (c + u < nc) cnt += dedupe_insert(wset, cap, ch[u]);
    }
    if (lane == 0) write_vote(a, r.s, r.fid, r.fid, cnt);
  }
  if (blockIdx.x >= nb) return;  // block-uniform
  __syncthreads();  // the wave slices are done: the whole set is the block's
  // Larger sets: one block per protein, the whole LDS set (up to kLongSet / 2 windows), else
  // the first kFallbackBlocks blocks with a set in workspace scratch.
  const PendingRec* big = a.pending + a.pending_half;
  unsigned long long* gset =
      reinterpret_cast<unsigned long long*>(a.scratch) + (uint64_t)blockIdx.x * kFallbackCap;
  for (uint32_t i = blockIdx.x; i < nb; i += gridDim.x) {
    const PendingRec r = big[i];
    if (r.n_win > kLongSet / 2) continue;
    uint32_t cap = 64;
    while (cap < 2 * r.n_win) cap <<= 1;
    vote_long_one<K>(a, lut, r.s, r.n_win, lds_set, cap, red);
  }
  if (blockIdx.x >= kFallbackBlocks) return;
  for (uint32_t i = blockIdx.x; i < nb; i += kFallbackBlocks) {
    const PendingRec r = big[i];
    if (r.n_win <= kLongSet / 2) continue;
    if (r.n_win > kFallbackCap / 2) {
      if (tid == 0) {
        a.out_fid[r.s] = -1;
        a.out_count[r.s] = 0;
        a.out_status[r.s] = KMA_STATUS_TOO_LONG;
      }
      continue;
    }
    uint32_t cap = 64;
    while (cap < 2 * r.n_win) cap <<= 1;
    vote_long_one<K>(a, lut, r.s, r.n_win, gset, cap, red);
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
  __shared__ uint32_t wave_tot[kWavesPerBlock];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int k = a.k;
  const uint64_t base = a.offsets[0], end = base + a.total_bases;
  const uint64_t r0 = (uint64_t)blockIdx.x * kContigTile;  // relative to base
  for (int i = t; i < kSpan; i += blockDim.x) {
    const uint64_t g = base + r0 + i;
    bases[i] = (uint8_t)(g < end ? base2(a.dna[g]) : 4u);
  }
  __syncthreads();
  for (int i = t; i < kSpan - 2; i += blockDim.x) {
    const uint32_t b0 = bases[i], b1 = bases[i + 1], b2 = bases[i + 2];
    if ((b0 | b1 | b2) & 4u) {
      aa_p[i] = aa_m[i] = 0;  // 'X'
    } else {
      aa_p[i] = a.codon_codes[b0 * 16 + b1 * 4 + b2];  // kernarg (scalar) loads
      aa_m[i] = a.codon_codes[(b2 ^ 2u) * 16 + (b1 ^ 2u) * 4 + (b0 ^ 2u)];  // complement: x ^ 2
    }
  }
  __syncthreads();

  const uint64_t r = r0 + t, g = base + r;
  bool hp = false, hm = false;
  uint32_t fp = 0, fm = 0, contig = 0;
  if (g < end) {
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
    hp = pv && probe(a.slots, a.n_buckets, k, a.mlen, kp, fp);
    hm = mv && probe(a.slots, a.n_buckets, k, a.mlen, km, fm);
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
  if (hp) st[o++] = (r << 25) | fp;                // strand bit 24 = 0: '+'
  if (hm) st[o] = (r << 25) | (1ull << 24) | fm;   // '-'
  if (t == 0) a.block_counts[blockIdx.x] = total;
}

// Quad form of the 6-frame probe (default; KMA_CPROBE=lane selects the kernel above). Same
// tile, translation and compaction; the two windows a position anchors ('+' and '-') are
// probed with the K1 quad-cooperative bucket loads (both probes' 8 dwordx4 of a lane in flight
// before any compare, DPP quad match), the block's contigs are found once (two searches by
// thread 0) and their offsets cached in LDS, so a position's contig costs no global loads.
constexpr int kOffCache = 64;

// contig_of by a whole wave, 64 candidates per dependent load: the largest c < n with
// off[c] <= g (off[0] <= g), in ceil(log64 n) rounds (one for up to 64 contigs) instead of
// log2 n dependent loads by one lane. Offsets are non-decreasing, so the lanes whose candidate
// is <= g form a prefix.
__device__ __forceinline__ uint32_t contig_of_wave(const uint64_t* __restrict__ off, uint32_t n,
                                                   uint64_t g) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t lo = 0, span = n;  // the answer lies in [lo, lo + span)
  while (span > 1) {          // wave-uniform
    const uint32_t step = (span + 63) / 64;
    const uint32_t c = lo + lane * step;
    const bool le = lane * step < span && off[c] <= g;
    const uint32_t k = (uint32_t)__popcll(__ballot(le)) - 1u;  // lane 0's candidate is lo
    const uint32_t nlo = lo + k * step;
    span = min(step, lo + span - nlo);
    lo = nlo;
  }
  return lo;
}

template <int K, int M>
__global__ __launch_bounds__(256) void contigs_probe_quad_kernel(ContigArgs a) {
  constexpr int kSpan = kContigTile + 3 * K;
  constexpr uint32_t kNone = 0xFFFFFFFFu;
  __shared__ uint8_t bases[kSpan];
  __shared__ uint8_t aa_p[kSpan], aa_m[kSpan];
  __shared__ uint64_t offc[kOffCache + 1];
  __shared__ uint32_t crange[2];
  __shared__ uint32_t wave_tot[kWavesPerBlock];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, part = t & 3;
  const uint64_t base = a.offsets[0], end = base + a.total_bases;
  const uint64_t r0 = (uint64_t)blockIdx.x * kContigTile;
  const uint32_t nb = a.n_buckets;
  if (wave < 2) {  // wave 0: the tile's first contig (and its offsets), wave 1: its last
    const uint64_t last = r0 + kContigTile < a.total_bases ? r0 + kContigTile : a.total_bases;
    const uint32_t c = contig_of_wave(a.offsets, a.n_contig, base + (wave ? last - 1 : r0));
    if (lane == 0) crange[wave] = c;
    if (wave == 0) {  // offsets c .. c + 64 (clamped): the tile's contigs if they are <= 64
      offc[lane] = a.offsets[min(c + lane, a.n_contig)];
      if (lane == 0) offc[kOffCache] = a.offsets[min(c + kOffCache, a.n_contig)];
    }
  }
  for (int i = t; i < kSpan; i += blockDim.x) {
    const uint64_t g = base + r0 + i;
    bases[i] = (uint8_t)(g < end ? base2(a.dna[g]) : 4u);
  }
  __syncthreads();
  const uint32_t c_lo = crange[0], nc = crange[1] - c_lo + 1;  // contigs meeting the tile
  for (int i = t; i < kSpan - 2; i += blockDim.x) {
    const uint32_t b0 = bases[i], b1 = bases[i + 1], b2 = bases[i + 2];
    if ((b0 | b1 | b2) & 4u) {
      aa_p[i] = aa_m[i] = 0;  // 'X'
    } else {
      aa_p[i] = a.codon_codes[b0 * 16 + b1 * 4 + b2];
      aa_m[i] = a.codon_codes[(b2 ^ 2u) * 16 + (b1 ^ 2u) * 4 + (b0 ^ 2u)];  // complement: x ^ 2
    }
  }
  __syncthreads();

  const uint64_t r = r0 + t, g = base + r;
  uint32_t contig = c_lo;
  int64_t x = 0, len = 0;
  if (g < end) {
    if (nc <= (uint32_t)kOffCache) {
      uint32_t lo = 0, hi = nc;  // largest i < nc with offc[i] <= g
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (offc[mid] <= g) lo = mid; else hi = mid;
      }
      contig = c_lo + lo;
      x = (int64_t)(g - offc[lo]);
      len = (int64_t)(offc[lo + 1] - offc[lo]);
    } else {
      contig = contig_of(a.offsets, a.n_contig, g);
      x = (int64_t)(g - a.offsets[contig]);
      len = (int64_t)(a.offsets[contig + 1] - a.offsets[contig]);
    }
  }
  bool pv = g < end && x + 3 * K + 3 <= len, mv = g < end && x >= 3 && x + 3 * K <= len;
  uint64_t key[2] = {0, 0};
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint32_t cp = aa_p[t + 3 * j], cm = aa_m[t + 3 * j];
    pv = pv && cp != 0u;
    mv = mv && cm != 0u;
    key[0] = (key[0] << 5) | cp;
    key[1] |= (uint64_t)cm << (5 * j);
  }
  uint32_t bk[2], klo[2], khi[2];
  bk[0] = pv ? home_bucket(key[0], K, M, nb) : kNone;
  bk[1] = mv ? home_bucket(key[1], K, M, nb) : kNone;
  uint4 q[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    klo[j] = (uint32_t)key[j];
    khi[j] = (uint32_t)(key[j] >> 32) << 24;
    const uint32_t b0 = quad_bcast<0>(bk[j]), b1 = quad_bcast<1>(bk[j]);
    const uint32_t b2 = quad_bcast<2>(bk[j]), b3 = quad_bcast<3>(bk[j]);
    const uint4* sp = reinterpret_cast<const uint4*>(a.slots) + part;
    q[j][0] = sp[(uint64_t)(b0 == kNone ? 0u : b0) * 4];
    q[j][1] = sp[(uint64_t)(b1 == kNone ? 0u : b1) * 4];
    q[j][2] = sp[(uint64_t)(b2 == kNone ? 0u : b2) * 4];
    q[j][3] = sp[(uint64_t)(b3 == kNone ? 0u : b3) * 4];
  }
  uint32_t word[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    word[j] = 0;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const uint32_t kl = rr == 0 ? quad_bcast<0>(klo[j]) : rr == 1 ? quad_bcast<1>(klo[j])
                        : rr == 2 ? quad_bcast<2>(klo[j]) : quad_bcast<3>(klo[j]);
      const uint32_t kh = rr == 0 ? quad_bcast<0>(khi[j]) : rr == 1 ? quad_bcast<1>(khi[j])
                        : rr == 2 ? quad_bcast<2>(khi[j]) : quad_bcast<3>(khi[j]);
      const uint32_t v = match_part(q[j][rr], kl, kh, part);
      word[j] = part == rr ? v : word[j];
    }
  }
  bool hit[2];
  uint32_t fid[2], sid[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const uint32_t w = bk[j] != kNone ? word[j] : 0u;
    hit[j] = (w & kWordFid) != 0u;
    fid[j] = (w & kWordFid) - 1u;
    sid[j] = bk[j] * kSlotsPerBucket + ((w >> kSlotShift) & 7u);
    if (w == 0x80000000u)  // rare: the home bucket missed with the key's overflow bit set
      hit[j] = walk_chain(a.slots, nb, bk[j], key[j], fid[j], sid[j]);
  }
  if (a.strict_pass) {  // KmerFactory.Strict: a key's locations counted by its slot id
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (!hit[j]) continue;
      if (a.strict_pass == 1) atomicAdd(a.slot_count + sid[j], 1u);
      else hit[j] = a.slot_count[sid[j]] == 1u;
    }
  }
  if (a.tally) {
    if (hit[0] && fid[0] < a.n_fid) atomicAdd(a.tally + (uint64_t)contig * a.n_fid + fid[0], 1u);
    if (hit[1] && fid[1] < a.n_fid) atomicAdd(a.tally + (uint64_t)contig * a.n_fid + fid[1], 1u);
  }
  // Block-local compaction in canonical order (position, '+' before '-').
  const uint64_t bp = __ballot(hit[0]), bm = __ballot(hit[1]);
  if (lane == 0) wave_tot[wave] = (uint32_t)(__popcll(bp) + __popcll(bm));
  __syncthreads();
  uint32_t o = popc_below(bp) + popc_below(bm), total = 0;
  for (int w = 0; w < kWavesPerBlock; ++w) {
    if (w < wave) o += wave_tot[w];
    total += wave_tot[w];
  }
  uint64_t* st = a.staging + (uint64_t)blockIdx.x * (2 * kContigTile);
  if (hit[0]) st[o++] = (r << 25) | fid[0];               // strand bit 24 = 0: '+'
  if (hit[1]) st[o] = (r << 25) | (1ull << 24) | fid[1];  // '-'
  if (t == 0) a.block_counts[blockIdx.x] = total;
}

// Peg windows (KmerReference.countPegKmers, KmerReference.java:124-147): one wave per peg;
// position i of peg s gets the packed key of window [i, i + K) if i < L - K (end exclusive)
// and the window has no 'X' and only standard symbols (others can never equal a translated
// contig kmer), else 0; every position of the batch is written.
__global__ __launch_bounds__(256) void peg_windows_kernel(const uint8_t* __restrict__ residues,
                                                          const uint64_t* __restrict__ offsets,
                                                          uint32_t n_peg, int k,
                                                          const uint8_t* __restrict__ lut_g,
                                                          uint64_t* __restrict__ keys,
                                                          uint32_t* __restrict__ pegs) {
  __shared__ uint8_t lut[256];
  lut[threadIdx.x] = threadIdx.x == 'X' ? 0 : lut_g[threadIdx.x];  // 'X' windows are skipped
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t o0 = offsets[0];
  for (uint64_t s = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); s < n_peg;
       s += (uint64_t)gridDim.x * 4) {
    const uint64_t lo = offsets[s], hi = offsets[s + 1];
    const int64_t end = (int64_t)(hi - lo) - k;  // windows i < end
    for (uint64_t p = lo + lane; p < hi; p += 64) {
      const int64_t i = (int64_t)(p - lo);
      uint64_t key = 0;
      if (i < end) {
        bool ok = true;
        for (int j = 0; j < k; ++j) {
          const uint32_t c = lut[residues[p + j]];
          ok = ok && c != 0u;
          key = (key << 5) | c;
        }
        key = ok ? key : 0;
      }
      keys[p - o0] = key;
      pegs[p - o0] = (uint32_t)s;
    }
  }
}

__global__ __launch_bounds__(256) void singleton_flags_kernel(const uint64_t* __restrict__ k,
                                                              uint64_t n,
                                                              uint8_t* __restrict__ flags) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * 256) {
    const uint64_t v = k[i];
    flags[i] = v != 0 && (i == 0 || k[i - 1] != v) && (i + 1 == n || k[i + 1] != v);
  }
}

// Signature build (BuildKmerProcessor.java:137-223). One wave per protein: the windows of
// ProteinKmers (i = 0..L-K, or i < L-K with end_exclusive) of interesting pegs (role >= 0) and
// buffered proteins (role -1) become key << 24 | role (kBuildNeg for buffered); every other
// position gets 0. A window with a byte the standard alphabet cannot encode raises alpha_flag
// (the host refuses the batch rather than drop a kmer the reference would keep).
__global__ __launch_bounds__(256) void build_windows_kernel(const uint8_t* __restrict__ residues,
                                                            const uint64_t* __restrict__ offsets,
                                                            uint32_t n_seq,
                                                            const int32_t* __restrict__ roles,
                                                            int k, int end_exclusive,
                                                            const uint8_t* __restrict__ lut_g,
                                                            uint64_t* __restrict__ out,
                                                            uint32_t* __restrict__ alpha_flag) {
  __shared__ uint8_t lut[256];
  lut[threadIdx.x] = lut_g[threadIdx.x];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t o0 = offsets[0];
  for (uint64_t s = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); s < n_seq;
       s += (uint64_t)gridDim.x * 4) {
    const uint64_t lo = offsets[s], hi = offsets[s + 1];
    const int32_t role = roles[s];
    const int64_t n_win = (int64_t)(hi - lo) - k + (end_exclusive ? 0 : 1);
    const bool counted = role >= -1;
    const uint64_t tag = role >= 0 ? (uint64_t)role : (uint64_t)kBuildNeg;
    bool bad = false;
    for (uint64_t p = lo + lane; p < hi; p += 64) {
      const int64_t i = (int64_t)(p - lo);
      uint64_t v = 0;
      if (counted && i < n_win) {
        uint64_t key = 0;
        bool ok = true;
        for (int j = 0; j < k; ++j) {
          const uint32_t c = lut[residues[p + j]];
          ok = ok && c != 0u;
          key = (key << 5) | c;
        }
        bad = bad || !ok;
        v = ok ? (key << 24) | tag : 0;
      }
      out[p - o0] = v;
    }
    if (__ballot(bad) && lane == 0) atomicOr(alpha_flag, 1u);
  }
}

__global__ __launch_bounds__(256) void signature_flags_kernel(const uint64_t* __restrict__ u,
                                                              const uint64_t* __restrict__ n_u,
                                                              uint8_t* __restrict__ flags) {
  const uint64_t n = *n_u;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * 256) {
    const uint64_t v = u[i], key = v >> 24;
    flags[i] = key != 0 && (v & kBuildNeg) != kBuildNeg && (i == 0 || (u[i - 1] >> 24) != key) &&
               (i + 1 == n || (u[i + 1] >> 24) != key);
  }
}

// Emit pass: block b's staged hits go to out[prefix[b] ..], those past `cap` are dropped; the
// last block publishes the total (the caller compares it with cap).
__global__ __launch_bounds__(256) void contigs_emit_kernel(ContigArgs a) {
  const uint32_t n = a.block_counts[blockIdx.x];
  const uint64_t p0 = a.prefix[blockIdx.x];
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *a.n_hits = p0 + n;
  const uint64_t* st = a.staging + (uint64_t)blockIdx.x * (2 * kContigTile);
  const uint64_t base = a.offsets[0];
  for (uint32_t i = threadIdx.x; i < n && p0 + i < a.cap; i += blockDim.x) {
    const uint64_t v = st[i];
    const uint64_t g = base + (v >> 25);
    const bool minus = (v >> 24) & 1u;
    const uint32_t c = contig_of(a.offsets, a.n_contig, g);
    const int64_t x = (int64_t)(g - a.offsets[c]);
    const int64_t len = (int64_t)(a.offsets[c + 1] - a.offsets[c]);
    kma_hit h;
    h.contig = c;
    h.left = (int32_t)(x + 1);
    h.fid = (uint32_t)v & 0xFFFFFFu;
    h.strand = minus ? '-' : '+';
    h.frame = (uint8_t)((minus ? (len - 3 * a.k - x) : x) % 3 + 1);
    h.pad = 0;
    a.out[p0 + i] = h;
  }
}

}  // namespace

// ---- launchers ----------------------------------------------------------------------------------
static unsigned grid_for(uint64_t n, unsigned cap = 8192) {
  uint64_t g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > cap ? cap : g));
}

hipError_t launch_build_insert(uint64_t* slots, uint32_t* winner, uint32_t n_buckets, int k,
                               int m, const uint64_t* keys, uint64_t n, uint32_t* status,
                               hipStream_t stream) {
  hipLaunchKernelGGL(build_insert_kernel, dim3(grid_for(n)), dim3(256), 0, stream, slots, winner,
                     n_buckets, k, m, keys, n, status);
  return hipGetLastError();
}

hipError_t launch_build_finalize(uint64_t* slots, const uint32_t* winner, const uint32_t* fids,
                                 uint32_t n_buckets, int k, int m, uint32_t* stats,
                                 hipStream_t stream) {
  hipLaunchKernelGGL(build_finalize_kernel,
                     dim3(grid_for((uint64_t)n_buckets * kSlotsPerBucket)), dim3(256), 0, stream,
                     slots, winner, fids, n_buckets, k, m, stats);
  return hipGetLastError();
}

// K1 form: quad-cooperative loads, one window per lane per step (default; measured fastest),
// or KMA_PROBE=run (runs of consecutive windows, repeated buckets not re-requested) /
// KMA_PROBE=lane (a lane reads a whole bucket).
static int probe_form() {
  static const int form = [] {
    const char* e = getenv("KMA_PROBE");
    return !e ? 1 : e[0] == 'l' ? 2 : e[0] == 'r' ? 0 : 1;
  }();
  return form;
}

// Resident blocks per CU of a K1 kernel (queried once): the grid is exactly the resident
// population, so no block waits for a second round (a grid-stride tail measured 9% at c5).
template <typename Kern>
static unsigned resident_blocks(Kern kern) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, 256, 0) != hipSuccess || n < 1)
    n = kProbeBlocksPerCU;
  if (getenv("KMA_DEBUG")) fprintf(stderr, "kma: K1 resident blocks per CU = %d\n", n);
  return (unsigned)n;
}

template <int K, int M, typename Kern>
static hipError_t launch_probe_grid(Kern kern, unsigned bpc, const ProteinArgs& a, int n_cu,
                                    hipStream_t stream) {
  // Grid from the batch average (the host does not see the segment's residue count).
  const uint64_t seg = a.seq_hi - a.seq_lo;
  const uint64_t n_pos = a.n_seq ? a.n_residues / a.n_seq * seg + 1 : 0;
  const uint64_t per_block = 256ull * kProbeWin;
  const uint64_t want = (n_pos + per_block - 1) / per_block;
  const uint64_t cap = (uint64_t)n_cu * bpc;
  if (!want || a.n_residues < (uint64_t)K) return hipSuccess;
  const dim3 grid((unsigned)(want < cap ? want : cap));
  hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, a);
  return hipGetLastError();
}

template <int K, int M>
static hipError_t launch_probe_km(const ProteinArgs& a, int n_cu, hipStream_t stream) {
  switch (probe_form()) {
    case 2: {
      static const unsigned bpc = resident_blocks(probe_kernel<K, M, kProbeWin>);
      return launch_probe_grid<K, M>(probe_kernel<K, M, kProbeWin>, bpc, a, n_cu, stream);
    }
    case 1: {
      static const unsigned bpc = resident_blocks(probe_quad_kernel<K, M, kProbeWin>);
      return launch_probe_grid<K, M>(probe_quad_kernel<K, M, kProbeWin>, bpc, a, n_cu, stream);
    }
    default: {
      static const unsigned bpc = resident_blocks(probe_run_kernel<K, M, kProbeWin>);
      return launch_probe_grid<K, M>(probe_run_kernel<K, M, kProbeWin>, bpc, a, n_cu, stream);
    }
  }
}

// Minimizer length is a template parameter of K1: m = min(K, 6), or 7 for large tables.
template <int K>
static hipError_t launch_probe_k(const ProteinArgs& a, int n_cu, hipStream_t stream) {
  constexpr int M6 = K < 6 ? K : 6;
  constexpr int M7 = K < 7 ? M6 : 7;
  if (a.mlen == M7 && M7 != M6) return launch_probe_km<K, M7>(a, n_cu, stream);
  if (a.mlen != M6) return hipErrorInvalidValue;
  return launch_probe_km<K, M6>(a, n_cu, stream);
}

template <int K>
static hipError_t launch_vote_k(const ProteinArgs& a, int n_cu, hipStream_t stream) {
  // Block-shared form by default: it spreads a long protein over the block's waves (measured
  // 18.8 vs 25 us at c2); KMA_VOTE=wave selects the barrier-free wave form (A/B).
  static const bool block_form = [] {
    const char* e = getenv("KMA_VOTE");
    return !(e && e[0] == 'w');
  }();
  if (block_form) {
    const unsigned blocks = (a.seq_hi - a.seq_lo + kVoteProteins - 1) / kVoteProteins;
    if (!blocks) return hipSuccess;
    hipLaunchKernelGGL(vote_kernel<K>, dim3(blocks), dim3(64 * kVoteWaves), 0, stream, a);
  } else {
    const uint64_t waves = a.seq_hi - a.seq_lo;  // one per protein
    const unsigned blocks = (unsigned)((waves + 3) / 4);
    if (!blocks) return hipSuccess;
    hipLaunchKernelGGL(vote_wave_kernel<K>, dim3(blocks), dim3(256), 0, stream, a);
  }
  return hipGetLastError();
}

template <int K>
static hipError_t launch_long_k(const ProteinArgs& a, int n_cu, hipStream_t stream) {
  // Usually nothing is pending and every block exits at once; the launch then costs the
  // same ~4.5 us at 1, 64 or 1024 blocks (measured): the dispatch and one flag read.
  const unsigned blocks = (unsigned)max(kFallbackBlocks, n_cu * kLongBlocksPerCU);
  hipLaunchKernelGGL(vote_long_kernel<K>, dim3(blocks), dim3(256), 0, stream, a);
  return hipGetLastError();
}

#define KMA_DISPATCH_K(FN)                              \
  switch (a.k) {                                         \
    case 1: return FN<1>(a, n_cu, stream);               \
    case 2: return FN<2>(a, n_cu, stream);               \
    case 3: return FN<3>(a, n_cu, stream);               \
    case 4: return FN<4>(a, n_cu, stream);               \
    case 5: return FN<5>(a, n_cu, stream);               \
    case 6: return FN<6>(a, n_cu, stream);               \
    case 7: return FN<7>(a, n_cu, stream);               \
    case 8: return FN<8>(a, n_cu, stream);               \
    default: return hipErrorInvalidValue;                \
  }

// Proteins per K12 block (KMA_FUSED_P=4|8 for A/B).
static int fused_proteins() {
  static const int p = [] {
    const char* e = getenv("KMA_FUSED_P");
    return e && atoi(e) == 8 ? 8 : 4;
  }();
  return p;
}

template <int K, int P>
static hipError_t launch_fused_kp(const ProteinArgs& a, hipStream_t stream) {
  constexpr int M6 = K < 6 ? K : 6;
  constexpr int M7 = K < 7 ? M6 : 7;
  const unsigned blocks = (a.seq_hi - a.seq_lo + P - 1) / P;
  if (!blocks) return hipSuccess;
  if (a.mlen == M7 && M7 != M6)
    hipLaunchKernelGGL((annotate_kernel<K, M7, P>), dim3(blocks), dim3(256), 0, stream, a);
  else if (a.mlen == M6)
    hipLaunchKernelGGL((annotate_kernel<K, M6, P>), dim3(blocks), dim3(256), 0, stream, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

template <int K>
static hipError_t launch_fused_k(const ProteinArgs& a, int n_cu, hipStream_t stream) {
  return fused_proteins() == 8 ? launch_fused_kp<K, 8>(a, stream)
                               : launch_fused_kp<K, 4>(a, stream);
}

// Batch size (proteins) from which K12 beats K1 + K2 (measured on MI355X, 10M-entry table:
// equal at 20k proteins, +11% at 40k, +18% at 300k, -2% at 10k): K12's vote is latency-bound
// and only hides behind other blocks' gathers when the grid is several resident
// populations deep; 2.5 populations.
uint32_t fused_min_proteins(int n_cu) {
  static const unsigned bpc = resident_blocks(annotate_kernel<8, 6, 4>);
  return (uint32_t)(2.5 * n_cu * bpc * fused_proteins());
}

hipError_t launch_fused(const ProteinArgs& a, int n_cu, hipStream_t stream) {
  if (a.n_seq == 0) return hipSuccess;
  KMA_DISPATCH_K(launch_fused_k)
}

hipError_t launch_probe(const ProteinArgs& a, int n_cu, hipStream_t stream) {
  if (a.n_seq == 0) return hipSuccess;
  KMA_DISPATCH_K(launch_probe_k)
}

hipError_t launch_vote(const ProteinArgs& a, int n_cu, hipStream_t stream) {
  if (a.n_seq == 0) return hipSuccess;
  KMA_DISPATCH_K(launch_vote_k)
}

hipError_t launch_long(const ProteinArgs& a, int n_cu, hipStream_t stream) {
  if (a.n_seq == 0) return hipSuccess;
  KMA_DISPATCH_K(launch_long_k)
}

template <int K>
static hipError_t launch_contigs_probe_k(const ContigArgs& a, uint64_t n_blocks,
                                         hipStream_t stream) {
  constexpr int M6 = K < 6 ? K : 6;
  constexpr int M7 = K < 7 ? M6 : 7;
  if (a.mlen == M7 && M7 != M6)
    hipLaunchKernelGGL((contigs_probe_quad_kernel<K, M7>), dim3((unsigned)n_blocks), dim3(256),
                       0, stream, a);
  else if (a.mlen == M6)
    hipLaunchKernelGGL((contigs_probe_quad_kernel<K, M6>), dim3((unsigned)n_blocks), dim3(256),
                       0, stream, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_contigs_probe(const ContigArgs& a, uint64_t n_blocks, hipStream_t stream) {
  // Quad form by default; KMA_CPROBE=lane selects the lane-per-bucket form (A/B).
  static const bool lane_form = [] {
    const char* e = getenv("KMA_CPROBE");
    return e && e[0] == 'l';
  }();
  if (lane_form && !a.strict_pass) {
    hipLaunchKernelGGL(contigs_probe_kernel, dim3((unsigned)n_blocks), dim3(256), 0, stream, a);
    return hipGetLastError();
  }
  switch (a.k) {
    case 1: return launch_contigs_probe_k<1>(a, n_blocks, stream);
    case 2: return launch_contigs_probe_k<2>(a, n_blocks, stream);
    case 3: return launch_contigs_probe_k<3>(a, n_blocks, stream);
    case 4: return launch_contigs_probe_k<4>(a, n_blocks, stream);
    case 5: return launch_contigs_probe_k<5>(a, n_blocks, stream);
    case 6: return launch_contigs_probe_k<6>(a, n_blocks, stream);
    case 7: return launch_contigs_probe_k<7>(a, n_blocks, stream);
    case 8: return launch_contigs_probe_k<8>(a, n_blocks, stream);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_contig_scan(const uint32_t* counts, uint64_t* prefix, uint64_t n, void* temp,
                              size_t* temp_bytes, hipStream_t stream) {
  return hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, counts, prefix, (int)n, stream);
}

hipError_t launch_peg_windows(const uint8_t* residues, const uint64_t* offsets, uint32_t n_peg,
                              int k, const uint8_t* lut, uint64_t* keys, uint32_t* pegs,
                              hipStream_t stream) {
  const unsigned g = (unsigned)std::min<uint64_t>(8192, ((uint64_t)n_peg + 3) / 4);
  hipLaunchKernelGGL(peg_windows_kernel, dim3(g ? g : 1), dim3(256), 0, stream, residues,
                     offsets, n_peg, k, lut, keys, pegs);
  return hipGetLastError();
}

hipError_t launch_sort_pairs(void* temp, size_t* temp_bytes, const uint64_t* keys_in,
                             uint64_t* keys_out, const uint32_t* vals_in, uint32_t* vals_out,
                             uint64_t n, int key_bits, hipStream_t stream) {
  return hipcub::DeviceRadixSort::SortPairs(temp, *temp_bytes, keys_in, keys_out, vals_in,
                                            vals_out, (int)n, 0, key_bits, stream);
}

hipError_t launch_singleton_flags(const uint64_t* sorted_keys, uint64_t n, uint8_t* flags,
                                  hipStream_t stream) {
  hipLaunchKernelGGL(singleton_flags_kernel, dim3(grid_for(n)), dim3(256), 0, stream,
                     sorted_keys, n, flags);
  return hipGetLastError();
}

hipError_t launch_select_flagged(void* temp, size_t* temp_bytes, const uint64_t* keys_in,
                                 const uint32_t* vals_in, const uint8_t* flags, uint64_t* keys_out,
                                 uint32_t* vals_out, uint64_t* n_out, uint64_t n,
                                 hipStream_t stream) {
  // Keys and values in one pass: select over an index-free zip is not needed, two passes over
  // the same flags keep the order identical.
  size_t need = 0;
  hipError_t e = hipcub::DeviceSelect::Flagged(nullptr, need, keys_in, flags, keys_out, n_out,
                                               (int)n, stream);
  if (e != hipSuccess) return e;
  size_t need2 = 0;
  e = hipcub::DeviceSelect::Flagged(nullptr, need2, vals_in, flags, vals_out, n_out, (int)n,
                                    stream);
  if (e != hipSuccess) return e;
  need = std::max(need, need2);
  if (!temp) {
    *temp_bytes = need;
    return hipSuccess;
  }
  e = hipcub::DeviceSelect::Flagged(temp, need, keys_in, flags, keys_out, n_out, (int)n, stream);
  if (e != hipSuccess) return e;
  return hipcub::DeviceSelect::Flagged(temp, need, vals_in, flags, vals_out, n_out, (int)n,
                                       stream);
}

hipError_t launch_build_windows(const uint8_t* residues, const uint64_t* offsets, uint32_t n_seq,
                                const int32_t* roles, int k, int end_exclusive, const uint8_t* lut,
                                uint64_t* out, uint32_t* alpha_flag, hipStream_t stream) {
  const unsigned g = (unsigned)std::min<uint64_t>(8192, ((uint64_t)n_seq + 3) / 4);
  hipLaunchKernelGGL(build_windows_kernel, dim3(g ? g : 1), dim3(256), 0, stream, residues,
                     offsets, n_seq, roles, k, end_exclusive, lut, out, alpha_flag);
  return hipGetLastError();
}

hipError_t launch_sort_keys(void* temp, size_t* temp_bytes, const uint64_t* in, uint64_t* out,
                            uint64_t n, int bits, hipStream_t stream) {
  return hipcub::DeviceRadixSort::SortKeys(temp, *temp_bytes, in, out, (int)n, 0, bits, stream);
}

hipError_t launch_unique(void* temp, size_t* temp_bytes, const uint64_t* in, uint64_t* out,
                         uint64_t* n_out, uint64_t n, hipStream_t stream) {
  return hipcub::DeviceSelect::Unique(temp, *temp_bytes, in, out, n_out, (int)n, stream);
}

hipError_t launch_signature_flags(const uint64_t* uniq, const uint64_t* n_uniq, uint64_t n_max,
                                  uint8_t* flags, hipStream_t stream) {
  hipLaunchKernelGGL(signature_flags_kernel, dim3(grid_for(n_max)), dim3(256), 0, stream, uniq,
                     n_uniq, flags);
  return hipGetLastError();
}

hipError_t launch_select_flagged_keys(void* temp, size_t* temp_bytes, const uint64_t* in,
                                      const uint8_t* flags, uint64_t* out, uint64_t* n_out,
                                      uint64_t n, hipStream_t stream) {
  return hipcub::DeviceSelect::Flagged(temp, *temp_bytes, in, flags, out, n_out, (int)n, stream);
}

hipError_t launch_contigs_emit(const ContigArgs& a, uint64_t n_blocks, hipStream_t stream) {
  hipLaunchKernelGGL(contigs_emit_kernel, dim3((unsigned)n_blocks), dim3(256), 0, stream, a);
  return hipGetLastError();
}

}  // namespace kma
