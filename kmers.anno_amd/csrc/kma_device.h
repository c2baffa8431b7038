// kma_device.h — device helpers shared by the probe kernels (kma_kernels.hip): wave reductions, window packing, bucket scans and the quad-cooperative
// bucket match. Internal; not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kma_internal.h"

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
// The two aligned words of a window, combined later (win_bytes: a funnel shift) so that the
// load is not consumed in the step that issues it. (One unaligned 8-byte load per window saves
// 3 VGPRs and measured 1% slower at c5, profiles/r03t/.)
struct WinWords {
  uint64_t lo, hi;
  uint32_t sh;
};
__device__ __forceinline__ WinWords window_words(const uint8_t* __restrict__ res, uint64_t pos) {
  const uint64_t* src = reinterpret_cast<const uint64_t*>(res + (pos & ~7ull));
  return WinWords{src[0], src[1], (uint32_t)(pos & 7) * 8u};
}
__device__ __forceinline__ uint64_t win_bytes(const WinWords& w) { return funnel(w.lo, w.hi, w.sh); }

// Packed residue streams (kma_pack_residues, pack_residues_kernel): residue j of a call is the
// 5-bit code at bits [5j, 5j + 5) of a big-endian bit stream (stream byte b holds bits
// [8b, 8b + 8), most significant first), so the window at residue j is the stream's 5K bits
// from bit 5j: exactly its key (first residue most significant). A window's words are the two
// aligned u64 around its first byte; `sh` packs the byte shift (bits 3..5) and the bit shift
// within the byte (bits 0..2).
__device__ __forceinline__ WinWords window_words_packed(const uint8_t* __restrict__ stream,
                                                        uint64_t j) {
  const uint64_t bit = 5 * j, byte = bit >> 3;
  const uint64_t* src = reinterpret_cast<const uint64_t*>(stream + (byte & ~7ull));
  return WinWords{src[0], src[1], (uint32_t)(((byte & 7) << 3) | (bit & 7))};
}
__device__ __forceinline__ uint64_t bswap64(uint64_t v) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  const uint32_t slo = __builtin_amdgcn_perm(0u, lo, 0x00010203u);  // byte-reverse each dword
  const uint32_t shi = __builtin_amdgcn_perm(0u, hi, 0x00010203u);
  return (uint64_t)slo << 32 | shi;
}
// The packed window's key. Residues that had no code (0) leave a zero 5-bit group, which no
// table key has (codes are 1..31): such a window is probed and misses, as its String would.
template <int K>
__device__ __forceinline__ uint64_t packed_key(const WinWords& w) {
  const uint64_t be = bswap64(funnel(w.lo, w.hi, w.sh & 56u));  // stream bytes, MSB first
  return (be << (w.sh & 7u)) >> (64 - 5 * K);
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

// One lane's scan of a whole bucket (the rare chain walk): the bucket's slots are loaded 64
// bytes at a time (4 dwordx4) and compared; hit (+ fid, slot index) / empty slot seen.
constexpr int kBucketQuads = kBucketBytes / 16;  // dwordx4 pieces per bucket
__device__ __forceinline__ void scan_half(const uint4 (&q)[4], int half, uint64_t key, bool& hit,
                                          bool& empty, uint32_t& fid, uint32_t& slot) {
  const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32) << 24;
  const uint32_t lo[8] = {q[0].x, q[0].z, q[1].x, q[1].z, q[2].x, q[2].z, q[3].x, q[3].z};
  const uint32_t hi[8] = {q[0].y, q[0].w, q[1].y, q[1].w, q[2].y, q[2].w, q[3].y, q[3].w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool m = lo[j] == klo && (hi[j] & kKeyHiMask) == khi;
    fid = m ? (hi[j] & kFidMask) : fid;
    slot = m ? (uint32_t)(8 * half + j) : slot;
    hit = hit || m;
    empty = empty || lo[j] == 0u;
  }
}

// Walk the overflow chain after home bucket `b` (the key missed there and its filter positions
// are set): stop at the key or at the first bucket with an empty slot. Returns true on a hit, with
// the key's fid and slot id (bucket * slots + slot: the key's identity in this table). The
// buckets can be loaded kWalkGroup at a time (all their dwordx4 in flight, then scanned in chain
// order): ceil(n / kWalkGroup) dependent round trips for n buckets. Measured at c5 LF 0.9 (linear
// chains then, up to 355 buckets): 1, 2, 4 take 20.6, 20.9, 20.6 ms (profiles/r02k_walk_group.log) — high-LF
// cost is the walks' request volume, not their latency — so 1 (fewest bytes) is the default.
#ifndef KMA_WALK_GROUP
#define KMA_WALK_GROUP 1
#endif
constexpr int kWalkGroup = KMA_WALK_GROUP;
// Two-choice tables (two_choice, kma_internal.h alt_bucket): the key's only other bucket is read
// instead, once; a miss there is definitive.
__device__ __forceinline__ bool walk_chain(const uint64_t* __restrict__ slots, uint32_t n_buckets,
                                           uint32_t b, uint64_t key, uint32_t& fid,
                                           uint32_t& sid, bool two_choice = false,
                                           uint32_t* walked = nullptr) {
  if (two_choice) {
    const uint32_t ab = alt_bucket(key, b, n_buckets);
    const uint4* bp = reinterpret_cast<const uint4*>(slots + (uint64_t)ab * kSlotsPerBucket);
    uint4 q[kBucketQuads];
#pragma unroll
    for (int i = 0; i < kBucketQuads; ++i) q[i] = bp[i];
    bool h = false, e = false;
    uint32_t slot = 0;
#pragma unroll
    for (int half = 0; half < kBucketHalves; ++half) {
      const uint4 part[4] = {q[4 * half], q[4 * half + 1], q[4 * half + 2], q[4 * half + 3]};
      scan_half(part, half, key, h, e, fid, slot);
    }
    sid = ab * kSlotsPerBucket + slot;
    if (walked) *walked = 1;
    return h;
  }
  bool hit = false, empty = false;
  const uint32_t home = b;
  uint32_t slot = 0, steps = 1;
  while (!hit && !empty && steps < n_buckets) {  // bounded
    uint32_t bb[kWalkGroup];
    uint4 q[kWalkGroup][kBucketQuads];
#pragma unroll
    for (int g = 0; g < kWalkGroup; ++g) {
      const uint32_t i = steps + g;
      b = chain_bucket(home, i < n_buckets ? i : 0u, n_buckets);
      bb[g] = b;
      const uint4* bp = reinterpret_cast<const uint4*>(slots + (uint64_t)b * kSlotsPerBucket);
#pragma unroll
      for (int i = 0; i < kBucketQuads; ++i) q[g][i] = bp[i];
    }
#pragma unroll
    for (int g = 0; g < kWalkGroup; ++g) {
      if (hit || empty || steps >= n_buckets) break;  // the chain ended in an earlier bucket
      bool h = false, e = false;
#pragma unroll
      for (int half = 0; half < kBucketHalves; ++half) {
        const uint4 part[4] = {q[g][4 * half], q[g][4 * half + 1], q[g][4 * half + 2],
                               q[g][4 * half + 3]};
        scan_half(part, half, key, h, e, fid, slot);
      }
      hit = h;
      empty = e;
      sid = bb[g] * kSlotsPerBucket + slot;
      ++steps;
    }
  }
  if (walked) *walked = steps - 1;  // chain buckets scanned (tuning counters)
  return hit;
}

template <int R>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, R * 0x55, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t quad_or(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
  return v | (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
}

// One quad's verdict on a bucket it loaded cooperatively: lane `part` holds slots 2part and
// 2part + 1 of each 64-byte half h of the bucket in v[h] (slots 8h + 2part, 8h + 2part + 1)
// for key (kl, kh) with filter mask `need` (filter_need of the key, the same in every lane of
// the quad): the verdict word of kma_internal.h (fid, hit flag, slot, absent bits). Lane `part` holds
// the filter positions of its two slots (position i in slot i / kFilterBits). Keys are unique
// in a table, so at most one lane matches and OR is the reduction. Every lane of the quad must
// call it (DPP). Branch-free on purpose: a short-circuit here lets the compiler split the
// 16-byte loads into a lazily loaded tail behind a branch and a vmcnt(0).
__device__ __forceinline__ uint32_t match_part_raw(const uint4 (&v)[kBucketHalves], uint32_t kl,
                                                   uint32_t kh, uint32_t need, uint32_t part) {
  constexpr uint32_t FB = kFilterBits, PM = (1u << (2 * FB)) - 1;  // positions per lane, half
  uint32_t w = 0, missing = 0;
#pragma unroll
  for (int h = 0; h < kBucketHalves; ++h) {
    // key match: (x ^ kl) | ((y ^ kh) & kKeyHiMask) == 0, two bitop3 (truth tables over
    // (src0, src1, src2) bits, index 4 src0 + 2 src1 + src2: 0x28 = (a ^ b) & c, 0xBE = (a ^ b)
    // | c) and a compare per slot, where the compiler's xor / xor / and_or took three, and the
    // verdict one select per slot: with the gather's sentinel-free bucket index (annotate_block)
    // SQ VALU per wave c5 2,458 -> 2,267, c3 1,927 -> 1,827, and (ABAB) c5 2.853-2.857 ->
    // 2.832-2.836 ms, c2 47.0 -> 45.0-45.2 us, c3's probe 73.1-73.6 -> 72.2-72.6 us, c4 2.689 ->
    // 2.711-2.715 ms (profiles/r06/match_gather_r06g/, r06h: the match alone costs c4 0.6%)
    const bool m0 = __builtin_amdgcn_bitop3_b32(
                        v[h].x, kl, __builtin_amdgcn_bitop3_b32(v[h].y, kh, kKeyHiMask, 0x28),
                        0xBE) == 0u;
    const bool m1 = __builtin_amdgcn_bitop3_b32(
                        v[h].z, kl, __builtin_amdgcn_bitop3_b32(v[h].w, kh, kKeyHiMask, 0x28),
                        0xBE) == 0u;
    // the slot's verdict: fid | slot within the bucket | hit flag (lane constants c0, c1), one
    // select each (keys are unique: at most one of m0, m1)
    const uint32_t c0 = ((8u * h + 2u * part) << kSlotShift) | kWordHit;
    const uint32_t s0 = (v[h].y & kFidMask) | c0;
    const uint32_t s1 = (v[h].w & kFidMask) | (c0 + (1u << kSlotShift));
    w |= m0 ? s0 : (m1 ? s1 : 0u);
    // the lane's positions: slot 8h + 2part (bits of .y), slot 8h + 2part + 1 (bits of .w)
    const uint32_t held = ((v[h].y >> kFidBits) & ((1u << FB) - 1u)) |
                          (((v[h].w >> kFidBits) & ((1u << FB) - 1u)) << FB);
    const uint32_t want = (need >> (2u * FB * (4u * h + part))) & PM;
    missing |= want & ~held;
  }
  if constexpr (2 * FB > 4) missing = (missing | missing >> FB) & ((1u << FB) - 1u);  // <= 4 bits
  return w | missing << kAbsentShift;  // nonzero: a filter position of the key is clear
}
__device__ __forceinline__ uint32_t match_part(const uint4 (&v)[kBucketHalves], uint32_t kl,
                                               uint32_t kh, uint32_t need, uint32_t part) {
  return quad_or(match_part_raw(v, kl, kh, need, part));
}

// Reduce-scatter over a quad of the four buckets' lane verdicts a[r] (match_part_raw): lane
// `part` returns the OR over the quad of a[part], i.e. its own window's verdict, by a two-round
// butterfly (3 DPP + 3 OR + 6 lane-constant selects) in place of four quad_or and a select per
// bucket (8 DPP + 8 OR + 4 selects).
#ifndef KMA_QUAD_XPOSE
#define KMA_QUAD_XPOSE 1
#endif
__device__ __forceinline__ uint32_t quad_reduce_scatter(const uint32_t (&a)[4], uint32_t part) {
  const bool hi2 = (part & 2u) != 0u, hi1 = (part & 1u) != 0u;
  const uint32_t s0 = hi2 ? a[0] : a[2], s1 = hi2 ? a[1] : a[3];  // the partner's half
  const uint32_t k0 = hi2 ? a[2] : a[0], k1 = hi2 ? a[3] : a[1];  // mine: r = (part & 2) | 0, 1
  const uint32_t b0 = k0 | (uint32_t)__builtin_amdgcn_mov_dpp((int)s0, 0x4E, 0xF, 0xF, false);
  const uint32_t b1 = k1 | (uint32_t)__builtin_amdgcn_mov_dpp((int)s1, 0x4E, 0xF, 0xF, false);
  const uint32_t sn = hi1 ? b0 : b1, kp = hi1 ? b1 : b0;
  return kp | (uint32_t)__builtin_amdgcn_mov_dpp((int)sn, 0xB1, 0xF, 0xF, false);
}

// Wide tables (K > 8, kma_internal.h): lane `part` of the quad holds slot `part` of the bucket
// in v (and its filter positions 2part .. in .z); same verdict word as match_part.
__device__ __forceinline__ uint32_t match_wide_raw(const uint4& v, uint32_t kl, uint32_t kh,
                                                   uint32_t need, uint32_t part) {
  const uint32_t m = (uint32_t)(v.x == kl) & (uint32_t)(v.y == kh);
  uint32_t w = m ? (v.z & kFidMask) | kWordHit | part << kSlotShift : 0u;
  const uint32_t held = (v.z >> kFidBits) & ((1u << kFilterBits) - 1u);
  const uint32_t want = (need >> (kFilterBits * part)) & ((1u << kFilterBits) - 1u);
  w |= (want & ~held) << kAbsentShift;
  return w;
}

// walk_chain for wide tables: whole 64-byte buckets of four 16-byte slots, one at a time.
__device__ __forceinline__ bool walk_chain_wide(const uint64_t* __restrict__ slots,
                                                uint32_t n_buckets, uint32_t b, uint64_t key,
                                                uint32_t& fid, uint32_t& sid) {
  const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);
  const uint32_t home = b;
  for (uint32_t steps = 1; steps < n_buckets; ++steps) {  // bounded
    b = chain_bucket(home, steps, n_buckets);
    const uint4* bp = reinterpret_cast<const uint4*>(slots) + (uint64_t)b * kWideSlots;
    uint4 q[kWideSlots];
#pragma unroll
    for (int i = 0; i < kWideSlots; ++i) q[i] = bp[i];
    // selects, not an early return per slot: that one is compiled into a dynamically indexed
    // copy of q in scratch memory
    bool empty = false, found = false;
    uint32_t z = 0, at = 0;
#pragma unroll
    for (int i = 0; i < kWideSlots; ++i) {
      const bool m = q[i].x == klo && q[i].y == khi;
      z = m ? q[i].z : z;
      at = m ? (uint32_t)i : at;
      found = found || m;
      empty = empty || q[i].x == 0u;
    }
    if (found) {
      fid = z & kFidMask;
      sid = b * kWideSlots + at;
      return true;
    }
    if (empty) return false;
  }
  return false;
}

// The protein kernel packs the block's protein index above the bucket index (buckets <
// kMaxBuckets); a window that does not probe carries bucket 0 (its load is discarded).
constexpr int kBucketBits = 32 - kSlotBits;  // buckets < kMaxBuckets
constexpr uint32_t kBucketIdx = (1u << kBucketBits) - 1u;

// Set-entry index of `key` in a set of `cap` entries (fast range, any capacity).
__device__ __forceinline__ uint32_t set_slot(uint32_t key, uint32_t cap) {
#if KMA_HASH_LITE
  uint32_t h = key * 0x9E3779B1u;
  h ^= h >> 16;
  return (uint32_t)(((uint64_t)h * cap) >> 32);
#else
  return (uint32_t)(((uint64_t)mix32(key * 0x9E3779B1u) * cap) >> 32);
#endif
}

}  // namespace

// Kernels are instantiated per (K, layout): the minimizer length is a template parameter so
// that the m-mer loop unrolls; layouts are m = min(K, 6), min(K, 7) and 0 (flat), and for K = 8
// m = 6 in the mod-sampling order (6 | kOrderMod). K = 9..12
// are wide tables (16-byte slots); kernels that take only narrow tables reject them.
template <int K, template <int, int> class Launch, typename... Args>
inline hipError_t dispatch_m(int m, Args&&... args) {
  constexpr int M6 = K < 6 ? K : 6;
  constexpr int M7 = K < 7 ? M6 : 7;
  if (m == 0) return Launch<K, 0>::run(args...);
  if (m == M6) return Launch<K, M6>::run(args...);
  if (m == M7) return Launch<K, M7>::run(args...);
  if constexpr (order_mod_valid(K, 6))  // the mod-sampling order (kma_internal.h): K = 8, m = 6
    if (m == (6 | kOrderMod)) return Launch<K, 6 | kOrderMod>::run(args...);
  return hipErrorInvalidValue;
}
template <template <int, int> class Launch, typename... Args>
inline hipError_t dispatch_km(int k, int m, Args&&... args) {
  switch (k) {
    case 1: return dispatch_m<1, Launch>(m, args...);
    case 2: return dispatch_m<2, Launch>(m, args...);
    case 3: return dispatch_m<3, Launch>(m, args...);
    case 4: return dispatch_m<4, Launch>(m, args...);
    case 5: return dispatch_m<5, Launch>(m, args...);
    case 6: return dispatch_m<6, Launch>(m, args...);
    case 7: return dispatch_m<7, Launch>(m, args...);
    case 8: return dispatch_m<8, Launch>(m, args...);
    case 9: return dispatch_m<9, Launch>(m, args...);  // wide tables (kma_internal.h)
    case 10: return dispatch_m<10, Launch>(m, args...);
    case 11: return dispatch_m<11, Launch>(m, args...);
    case 12: return dispatch_m<12, Launch>(m, args...);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace kma
