// kma_internal.h — shared between the HIP kernels (kma_kernels.hip) and the C-ABI layer
// (kma_abi.cpp). Not part of the public ABI (see include/kmeranno.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kmeranno.h"

namespace kma {

// ---- signature-table layout in HBM ------------------------------------------------------------
// n_buckets buckets of kSlotsPerBucket slots of one u64 (8 slots = 64 bytes, the default; 16 =
// 128 bytes, the KMA_BUCKET_SLOTS=16 build):
//   low dword  = key bits 0..31            (never 0 for a valid key: codes are 1..31)
//   high dword = key bits 32..39 << 24 | filter bits << 22 | fid (22 bits)
// A slot whose low dword is 0 is empty. A key lives in its home bucket or, if that was full,
// in the next buckets of its probe chain (chain_bucket below: hashed steps by default). The
// filter bits of a bucket (kFilterBits per slot, independent of the slot's key) form a Bloom
// filter of the keys homed there that live further down the chain: each such key sets the
// kFilterBits positions filter_pos(key, 0 ..) of its home bucket. A lookup that misses its home
// bucket walks the chain only if all its positions are set (then it stops at the key or at a
// bucket with an empty slot). Every compare is a 32-bit operation.
// Bucket width: the chip serves random 128-byte lines at the same request rate as 64-byte ones
// (kma_gather_bench quad2 vs quad: 5.43e10 lines/s both, profiles/r02_gather_shapes_b.jsonl),
// but a 128-byte probe doubles the load instructions and the registers per window in flight:
// measured slower at load factor 0.5 (c5 4.89 vs 4.48-4.63 ms, c2 70 vs 64 us), so 64-byte
// buckets are the default and 128-byte ones a build variant for crowded tables.
#ifndef KMA_BUCKET_SLOTS
#define KMA_BUCKET_SLOTS 8
#endif
constexpr int kSlotsPerBucket = KMA_BUCKET_SLOTS;
static_assert(kSlotsPerBucket == 8 || kSlotsPerBucket == 16, "64- or 128-byte buckets");
constexpr int kBucketBytes = kSlotsPerBucket * 8;
constexpr int kBucketHalves = kBucketBytes / 64;  // 64-byte pieces a quad loads per bucket
constexpr int kSlotBits = kSlotsPerBucket == 16 ? 4 : 3;
// Filter bits per slot, each displaced key setting that many positions of its home bucket (two
// of 16 at 8 slots): a miss walks a chain only when both its positions are set. Round 2 kept one
// bit per slot (fid in 23 bits); at c5's m = 6 layout (7.7% of keys displaced) a miss found its
// bit set in ~4% of home buckets, each a dependent round trip.
#ifndef KMA_FILTER_BITS
#define KMA_FILTER_BITS 2
#endif
constexpr int kFilterBits = KMA_FILTER_BITS;
static_assert(kFilterBits >= 1 && kFilterBits <= 3, "one to three filter bits per slot");
constexpr uint32_t kFidBits = 24 - kFilterBits;  // fid width (KMA_MAX_FID: 22 bits)
constexpr uint32_t kFidMask = (1u << kFidBits) - 1;
constexpr uint32_t kKeyHiMask = 0xFF000000u;   // key bits 32..39 in the high dword
// The probe's verdict word (match_part / match_wide): on a match the fid in bits 0..kFidBits-1
// and kWordHit (bit kFidBits), the slot in the bucket from bit 24 (kSlotShift), and from bit 28
// (kAbsentShift) the key's filter positions that are clear in its home bucket (nonzero: the key
// is not further down the chain). A probed window whose word is 0 missed its home bucket with
// every filter position set: it walks the chain. (fid + 1 for a hit and one absent bit cost an
// add and a compare-select per slot more: c5 settle 291 -> 259 VALU instructions per step.)
constexpr uint32_t kWordHit = 1u << kFidBits;
constexpr uint32_t kAbsentShift = 28;  // <= 4 filter positions per lane and bucket
constexpr uint32_t kSlotShift = 24;
constexpr uint32_t kSlotMask = kSlotsPerBucket - 1;
// Buckets per table: slot ids (bucket * slots + slot) stay 32-bit.
constexpr uint64_t kMaxBuckets = 1ull << (32 - kSlotBits);

__host__ __device__ inline uint64_t slot_make(uint64_t key, uint32_t fid) {
  return ((uint64_t)((uint32_t)(key >> 32) << 24 | (fid & kFidMask)) << 32) | (uint32_t)key;
}
// Filter position h (0 .. kFilterBits - 1) of a key in a bucket of S slots (from the key's low
// dword): position i lives in slot i / kFilterBits, at bit kFidBits + i % kFilterBits of the
// slot's high dword (narrow) or .z (wide).
// KMA_HASH_LITE (default 1): the probe's per-window hashes use one 32-bit multiply each where
// round 3's first build used two to four (the protein and 6-frame probes issue a VALU
// instruction every ~4 cycles per SIMD: c5 3,107 VALU instructions per wave, profiles/r03q_sq/).
// Both filter positions come from one product; the minimizer order is a multiplicative hash of
// the m-mer (a bijection: no ties); the home bucket a one-multiply mix of the minimizer; the
// paired-home bit the key's parity. c5: 3.84 vs 4.04 ms and 3.99 vs 4.11 ms against the
// murmur hashes on two boxes, displaced keys 7.58% vs 7.70% (profiles/r03r/, r03s/).
#ifndef KMA_HASH_LITE
#define KMA_HASH_LITE 1
#endif
template <int S>
__host__ __device__ inline uint32_t filter_pos(uint32_t klo, int h) {
  constexpr int n = S * kFilterBits;  // positions per bucket
  constexpr int bits = (n == 32) ? 5 : (n == 16) ? 4 : (n == 8) ? 3 : 2;
#if KMA_HASH_LITE
  const uint32_t x = klo * 0x9E3779B1u;
  if constexpr ((n & (n - 1)) != 0) {  // 3 bits per slot: 24 (12 wide) positions, fast range
    const uint32_t r = h == 0 ? x : h == 1 ? (x << 11 | x >> 21) : (x << 22 | x >> 10);
    return (uint32_t)(((uint64_t)r * n) >> 32);
  }
  return h ? (x >> (32 - 2 * bits)) & ((1u << bits) - 1u) : x >> (32 - bits);
#else
  return ((klo * (h ? 0x85EBCA77u : 0x9E3779B1u)) + (h ? 0x165667B1u : 0u)) >> (32 - bits);
#endif
}
// The key's filter positions as a mask over the bucket's S * kFilterBits positions (computed
// once per window by its lane and broadcast to the quad that probes it).
template <int S>
__host__ __device__ inline uint32_t filter_need(uint32_t klo) {
  uint32_t m = 0;
  for (int h = 0; h < kFilterBits; ++h) m |= 1u << filter_pos<S>(klo, h);
  return m;
}
__host__ __device__ inline uint64_t slot_key(uint64_t slot) {
  return ((uint64_t)(uint32_t)(slot >> 56) << 32) | (uint32_t)slot;
}

// ---- wide tables (K = 9..12: 5K-bit keys up to 60 bits) ------------------------------------------
// The projector's -K (KmerProcessor.java:86-88, KmerReference.setKmerSize) reaches 12; a 60-bit
// key does not fit the 8-byte slot. Wide tables use 16-byte slots, four per 64-byte bucket, so a
// probe is still one 64-byte line and each lane of a quad loads exactly one slot (one dwordx4):
//   .x = key bits 0..31 (never 0: the last six residues' codes), .y = key bits 32..63,
//   .z = filter bits << 22 | fid (22 bits), .w = 0.
// The filter has kFilterBits per slot; chains, layouts and the stop rule are those of the
// narrow table. Wide buckets are 64 bytes in every build.
constexpr int kWideSlots = 4;
constexpr int kWideSlotBits = 2;
constexpr int kMaxNarrowK = 8;
__host__ __device__ constexpr bool wide_k(int k) { return k > kMaxNarrowK; }
__host__ __device__ constexpr int slots_for_k(int k) { return wide_k(k) ? kWideSlots : kSlotsPerBucket; }

__host__ __device__ inline uint32_t mix32(uint32_t h) {  // murmur3 fmix32
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
__host__ __device__ inline uint32_t mix32_lite(uint32_t h) {  // one multiply
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  return h;
}
__host__ __device__ inline uint32_t parity32(uint32_t x) {
#ifdef __HIP_DEVICE_COMPILE__
  return (uint32_t)__popc(x) & 1u;
#else
  return (uint32_t)__builtin_popcount(x) & 1u;
#endif
}

// Minimizer of a packed K-mer: the smallest hash over its K - m + 1 m-mers (5-bit residue
// codes, first residue most significant). m is a table property (minimizer_len below).
__host__ __device__ inline uint32_t mmer_hash(uint32_t sub) {
#if KMA_HASH_LITE
  return sub * 0x9E3779B1u;
#else
  return mix32(sub * 0x9E3779B1u + 0x7F4A7C15u);
#endif
}
// Minimizer ORDER (round 6; a table property, a bit of the layout code and of the kernels' M):
// how a key picks the m-mer its home is a hash of. Consecutive windows of a protein share their
// home line when they pick the same m-mer, so the order's density (the fraction of windows whose
// pick differs from the previous window's) is the probe's home-line requests per window.
//   random (default): the m-mer of smallest multiplicative hash; density 2/(w + 1) = 0.50 for
//          K = 8, m = 6 (w = K - m + 1 = 3 m-mers per key).
//   mod-sampling (kOrderMod; Groot Koerkamp & Pibiri, "The mod-minimizer", WABI 2024) over
//          single residues (t = 1): x = the position of the smallest rank among the key's K
//          residues (rank 31 - code; ties: the first), and the m-mer at x mod w is picked.
//          Simulated on c5's 10^8-key table (scripts/order_sim.py, profiles/order_sim_r06.log):
//          density 0.420 vs 0.502, keys beyond a bucket's 8 slots 7.4% vs 6.1% (more keys in
//          their alternate); with UniProt's residue frequencies 0.421 (identity ranks 0.422,
//          rarest-first 0.419). The first build sampled 3-mers (t = 3, the positions of the
//          smallest multiplicative 3-mer hash: density 0.431, 7.8% beyond 8 slots): c5 kernel
//          2.88 ms against 3.08 ms for the random order (profiles/r06/order_ab_r06b/); t = 1 then
//          2.855-2.873 against 2.881-2.897 ms and at load factor 0.9 3.557 vs 3.672 ms (ABAB,
//          profiles/r06/mod_t1_r06f/): a lower density for 8 cheap ranks (shift + one bitop3
//          each) in place of 6 hashed 3-mers, and x mod 3's shift read from a nibble table.
//          On the 10^7 table (Infinity-Cache resident) the t = 3 order measured c4 2.637 vs
//          2.688 ms, c2 even (47.1 vs 46.7 us), but the 6-frame probe, two windows per position
//          and VALU-heavier, 77.2 vs 73.7 us (profiles/r06/order_small_tables_r06c/), so it
//          began as a size rule (tables beyond the Infinity Cache); with t = 1 and the cheaper
//          bucket match the 10^7 table measures c4 2.284 vs 2.763 ms, c2 -2%, c3 even
//          (profiles/r06/order_small_tables_r06j/), and every K = 8, m = 6 table takes it
//          (kma_abi.cpp minimizer_len). Not kept: the open-closed t = 3 variant (3-mers whose middle residue code is
//          below both neighbours' rank first; simulated density 0.410) at 3.03 ms against
//          2.88, its VALU per window costing more than the fewer home lines save; t = 2 and 4
//          simulate at 0.467 / 0.468.
// The order bit rides in the minimizer length m of layout codes and kernel templates; the
// minimizer length proper is m & kMinimizerMask.
constexpr int kOrderMod = KMA_LAYOUT_MOD_SAMPLING;
constexpr int kMinimizerMask = 0x3F;
__host__ __device__ constexpr bool order_mod_valid(int k, int m) {
  return k == 8 && (m & kMinimizerMask) == 6;  // the instantiated kernels (kma_device.h)
}
// The picked m-mer's multiplicative hash is the minimizer value (home_from_min mixes it once
// more; the raw m-mer code there loaded the buckets less evenly: 3.00% vs 2.72% of 3e7 keys past
// a bucket's slots, scripts/order_sim.py). K = 8, m = 6 only (order_mod_valid): the ranks carry
// 4 x in their low 5 bits, so the winner's low bits index the nibble table of the m-mer's shift
// 5 (2 - x mod 3) (x = 0..7: 10, 5, 0, 10, 5, 0, 10, 5).
__host__ __device__ inline uint32_t mod_sample(uint64_t key) {
  uint32_t best = 0xFFFFFFFFu;
  for (int i = 0; i < 8; ++i) {
    const uint32_t c = (uint32_t)(key >> (5 * (7 - i))) & 31u;
    const uint32_t g = (31u - c) << 5 | (uint32_t)(4 * i);
    best = best < g ? best : g;
  }
  const uint32_t lo = (uint32_t)key, hi = (uint32_t)(key >> 32);
#ifdef __HIP_DEVICE_COMPILE__
  const uint32_t sh = __builtin_amdgcn_ubfe(0x5A05A05Au, best, 4u);  // offset: best's low 5 bits
  const uint32_t sub = __builtin_amdgcn_alignbit(hi, lo, sh) & 0x3FFFFFFFu;
#else
  const uint32_t sh = (0x5A05A05Au >> (best & 31u)) & 15u;
  const uint32_t sub = (uint32_t)(((uint64_t)hi << 32 | lo) >> sh) & 0x3FFFFFFFu;
#endif
  return mmer_hash(sub);
}
__host__ __device__ inline uint32_t minimizer_hash(uint64_t key, int k, int m) {
  if (m & kOrderMod) return mod_sample(key);  // (k == 8, m & kMinimizerMask == 6)
  const uint32_t mask = (uint32_t)((1ull << (5 * m)) - 1);
  uint32_t best = 0xFFFFFFFFu;
  for (int p = 0; p <= k - m; ++p) {
    const uint32_t h = mmer_hash((uint32_t)(key >> (5 * (k - m - p))) & mask);
    best = best < h ? best : h;
  }
  return best;
}

// Home bucket = the key's MINIMIZER hashed onto [0, n_buckets) (Lemire fast range). Two
// consecutive windows of a protein share their minimizer with probability 2/(K - m + 2)
// (1/2 for K = 8, m = 6; 1/3 for m = 7), so they share their home bucket and the second
// request is served by a line the CU just fetched. Exactness is kept by the full-key compare.
// m = 0 is the flat layout (a hash of the whole key): the fallback for tables whose keys pile
// onto few minimizers (low-complexity or adversarial kmer sets).
//
// Paired homes (minimizer layouts): the minimizer hash picks a PAIR of adjacent 64-byte buckets
// — one 128-byte L2 line — and one bit of a hash of the key picks the bucket in it. A probe
// still reads 64 bytes, windows sharing a minimizer still share a line, and a minimizer's keys
// spread over two buckets instead of piling into one: displaced keys at c5 (m = 7) 3.55% ->
// 2.45%, c2 3.60% -> 2.18%; c5 4.54 -> 4.50 ms and 4.56 -> 4.52 ms on two boxes, c3 / c2 even
// (profiles/r02q_pair/). Round 2's first layout (one bucket per minimizer) was kept as a tuning
// variant until round 4 and is gone: it measured slower at every load but one
// (profiles/r03_layout/) and its adversarial sweep never produced a record.
__host__ __device__ inline uint32_t home_from_hash(uint32_t h, uint64_t key, int m,
                                                   uint32_t n_buckets) {
  if (m != 0 && n_buckets >= 2) {
    const uint32_t pair = (uint32_t)(((uint64_t)h * (n_buckets >> 1)) >> 32);
#if KMA_HASH_LITE
    return 2u * pair + parity32((uint32_t)key);
#else
    return 2u * pair + (((uint32_t)key * 0x2C1B3C6Du) >> 31);
#endif
  }
  return (uint32_t)(((uint64_t)h * n_buckets) >> 32);
}
// The home of a key (minimizer layouts) from its minimizer hash.
__host__ __device__ inline uint32_t home_from_min(uint32_t mn, uint64_t key, int m,
                                                  uint32_t n_buckets) {
#if KMA_HASH_LITE
  return home_from_hash(mix32_lite(mn ^ 0x85EBCA77u), key, m, n_buckets);
#else
  return home_from_hash(mix32(mn ^ 0x85EBCA77u), key, m, n_buckets);
#endif
}
__host__ __device__ inline uint32_t home_bucket(uint64_t key, int k, int m, uint32_t n_buckets) {
  if (m == 0)
    return home_from_hash(mix32((uint32_t)key ^ mix32((uint32_t)(key >> 32) + 0x9E3779B9u)),
                          key, m, n_buckets);
  return home_from_min(minimizer_hash(key, k, m), key, m, n_buckets);
}

// Step i of the probe chain of a key homed at `home` (step 0 = home).
//
// Hashed chains (KMA_CHAIN_HASH, tables of >= kHashChainMin buckets): step i >= 1 is a
// pseudo-random bucket other than the home (a hash of (home, i)), so a full bucket's overflow
// does not pile onto its neighbours (linear probing's primary clustering, which makes chains of
// hundreds of buckets at load factor 0.9). The sequence may revisit a bucket; a key sits at the
// first step that had a free slot, and a lookup still stops at the first bucket with an empty
// slot (slots never empty again), so the walk and its stop rule are unchanged. Default since
// round 2 (profiles/r02s_chain/): c5 at load factor 0.9 19.9 -> 7.7 ms (longest chain 356 ->
// 39), 0.75 5.75 -> 4.94 ms, 0.5 even (4.50 / 4.49 ms both ways, two runs); 0 = linear chains
// (every bucket once in the first n_buckets steps; also tables below kHashChainMin buckets).
// Measured and not kept: one linear step, then hashed (7.86 / 5.17 ms at 0.9 / 0.75), and with
// linear chains, the home's partner in its 128-byte line first (no faster).
#ifndef KMA_CHAIN_HASH
#define KMA_CHAIN_HASH 1
#endif
constexpr uint32_t kHashChainMin = 1024;
constexpr uint32_t kChainStepSearch = 4096;  // chain_step gives up (stats only) past this
__host__ __device__ inline bool chain_hashed(uint32_t n_buckets) {
  return KMA_CHAIN_HASH && n_buckets >= kHashChainMin;
}
__host__ __device__ inline uint32_t chain_bucket(uint32_t home, uint32_t i, uint32_t n_buckets) {
  if (chain_hashed(n_buckets)) {
    if (i == 0u) return home;
    const uint32_t r = (uint32_t)(((uint64_t)mix32(home * 0x9E3779B1u ^ i * 0x85EBCA77u) *
                                   (n_buckets - 1u)) >> 32);
    const uint32_t b = home + 1u + r;  // any bucket but the home
    return b >= n_buckets ? b - n_buckets : b;
  }
  const uint64_t b = (uint64_t)home + i;
  return (uint32_t)(b >= n_buckets ? b - n_buckets : b);
}
// Inverse (table statistics): the step at which the chain of `home` first reaches bucket b.
__host__ __device__ inline uint32_t chain_step(uint32_t home, uint32_t b, uint32_t n_buckets) {
  if (chain_hashed(n_buckets)) {
    for (uint32_t i = 0; i < kChainStepSearch; ++i)
      if (chain_bucket(home, i, n_buckets) == b) return i;
    return kChainStepSearch;
  }
  return b >= home ? b - home : b + n_buckets - home;
}

// ---- two-choice placement (round 5; narrow tables) ------------------------------------------------
// Chains make a displaced key cost a walk of hashed buckets: at load factor 0.9 (c5, m = 7) a
// walk loaded 4.05 buckets on average (a miss walks until a bucket with an empty slot, and few
// buckets have one), 0.40 bucket requests per probed window on top of the 0.67 home lines, and
// the kernel ran at the request ceiling (1.05 requests per window; profiles/r05/). Two-choice
// placement (bucketized cuckoo hashing) gives every key exactly two buckets: its home (the
// minimizer layout's, shared by consecutive windows) and alt_bucket (a hash of the whole key,
// never the home). The build (build_two_choice_*: keys deduplicated last-wins by a radix sort,
// then inserted with evictions between the two buckets, then the filters) puts each key in one
// of them; the filter bits of a home bucket are those of its keys that live in their alt. A
// lookup that misses its home with every filter position set reads the alt bucket: one request,
// and a miss there is definitive. A table that cannot be built this way (an insertion exceeds
// kMaxKicks evictions: load factors near 1 with crowded minimizers) is built with chains.
__host__ __device__ inline uint32_t alt_bucket(uint64_t key, uint32_t home, uint32_t n_buckets) {
  const uint32_t h = mix32((uint32_t)key * 0x2C1B3C6Du ^ mix32_lite((uint32_t)(key >> 32) + 0x68E31DA5u));
  const uint32_t b = (uint32_t)(((uint64_t)h * (n_buckets - 1u)) >> 32);  // any bucket but home
  return b >= home ? b + 1u : b;
}
constexpr uint32_t kMaxKicks = 2000;
// Layout codes of kma_table_build_device / kma_table_wrap_device / kma_table_layout_for: the
// minimizer length (0 = flat) | kLayoutTwoChoice for two-choice placement.
constexpr int kLayoutTwoChoice = KMA_LAYOUT_TWO_CHOICE;
constexpr int kLayoutMask = 0xFF;
// A two-choice minimizer table whose displaced share exceeds this is also built flat (keys piling
// onto few minimizers: their homes' filters fill and most misses read the alt bucket) and the
// flat one kept if it halves the displaced keys.
constexpr double kMaxDisplacedTwoChoice = 0.40;

// Layout (minimizer length m, 0 = flat) of a table of n_buckets buckets for K-mers. Keys
// sharing a minimizer share a bucket, so the m-mer space must stay large against the table,
// while consecutive windows share their minimizer (and a request) with probability
// 1 - 2/(K - m + 2): 1/2 for m = 6, 1/3 for m = 7. The size rule: m = 6 up to
// kMinimizer6Buckets buckets (134M keys at load factor 0.5), else 7 (m <= K); KMA_MINIMIZER=
// 0|6|7 in the environment forces a layout (read per call: tests run every layout in one
// process). Defined in kma_abi.cpp.
constexpr uint64_t kMinimizer6Buckets = kSlotsPerBucket == 16 ? (1ull << 24) : (1ull << 25);
// Wide tables (4 slots per bucket): the same key count, i.e. twice the buckets.
constexpr uint64_t kMinimizer6BucketsWide = 1ull << 26;
int minimizer_len(int k, uint64_t n_buckets);
// The creators then measure the table they built (kma_abi.cpp create_from_device_keys): every
// displaced key costs a dependent round trip when it is looked up, and false filter hits cost
// the misses the same. Measured at c5 (10^8 keys, paired homes, hashed chains; round 3 sweep,
// profiles/r03_layout/): m = 6 / m = 7 / flat take 4.12 / 4.11 / 5.57 ms at load factor 0.5
// (7.7 / 2.4 / 0.9% displaced), 5.82 / 5.00 / 5.95 ms at 0.75 (17.1 / 9.4 / 6.1%) and
// 10.0 / 7.74 / 7.72 ms at 0.9 (24.5 / 16.8 / 13.1%): m = 6's 12% fewer line requests pay off
// only while few keys are displaced. So:
//   1. an m = 6 table with more than kRetryDisplaced of its keys displaced is also built with
//      m = 7, and the one with fewer displaced keys kept;
//   2. a minimizer table still crowded (more than kMaxDisplaced displaced, or a chain longer
//      than kMaxChain buckets: keys piling onto few minimizers) is also built flat, and the flat
//      one kept if it halves the displaced keys or the longest chain.
constexpr double kRetryDisplaced = 0.10;
constexpr double kMaxDisplaced = 0.15;
constexpr uint32_t kMaxChain = 32;

// ---- protein path (annotate_kernel) ------------------------------------------------------------
// One kernel: a block owns kBlockProteins consecutive proteins, probes every window of them
// (quad-cooperative bucket gathers, kProbeWin windows per lane per step) and keeps, per
// protein, the smallest and largest fid hit and the SET of distinct keys hit (a key's slot id
// is its unique identity in the table) in LDS; the vote is read off those at the end. A
// protein's set takes ceil(1.5 x windows) u32 entries of the block's kSetPool-entry LDS pool;
// a protein that does not fit keeps its set in workspace memory instead (2 u32 per residue,
// at its own residues' offset: disjoint per protein). No words or slot ids go to HBM.
#ifndef KMA_BLOCK_PROTEINS
#define KMA_BLOCK_PROTEINS 8
#endif
#ifndef KMA_SET_POOL
#define KMA_SET_POOL 4096
#endif
#ifndef KMA_PROBE_WIN
#define KMA_PROBE_WIN (KMA_BUCKET_SLOTS == 16 ? 1 : 2)
#endif
// Windows per lane per step: each costs 4 dwordx4 per bucket half (16 VGPRs per 64 bytes) in
// flight. With the single protein kernel, 2 measured best on MI355X (profiles/r02i_variants.log:
// c5 4.39 vs 4.52 ms for 3, c2 65.4 vs 66.3 us; 4 is 23% slower at c2).
constexpr int kProbeWin = KMA_PROBE_WIN;
constexpr int kBlockProteins = KMA_BLOCK_PROTEINS;
constexpr int kSetPool = KMA_SET_POOL;
// Lane permutation of the probe loops (kma_kernels.hip): one load instruction covers 16
// consecutive windows, so windows sharing a minimizer share a line inside the instruction.
// c5 3.96 vs 4.03 ms (profiles/r03_ab/).
#ifndef KMA_LANE_PERM
#define KMA_LANE_PERM 1
#endif
#ifndef KMA_CHAIN_Q
#define KMA_CHAIN_Q 192
#endif
constexpr int kChainQ = KMA_CHAIN_Q;  // deferred chain walks per wave (8 bytes: key, protein)
// a step adds at most 64 kProbeWin entries to a wave's queue after a flush check
static_assert(kChainQ >= 64 * (kProbeWin + 1), "chain queue below two steps of windows");
constexpr uint32_t kGlobalSet = 0xFFFFFFFFu;  // pset[] marker: the set lives in workspace memory
constexpr int kWavesPerBlock = 4;
// annotate_kernel blocks resident per CU (= waves per SIMD): its LDS and VGPR budget.
#ifndef KMA_PROTEIN_OCC
#define KMA_PROTEIN_OCC 7
#endif
constexpr int kProteinOcc = KMA_PROTEIN_OCC;

struct ProteinArgs {
  const uint64_t* slots;
  uint32_t n_buckets;
  const uint8_t* lut;  // 256-byte residue -> 5-bit code table (device)
  const uint8_t* residues;
  const uint64_t* offsets;
  uint32_t n_seq;
  uint32_t n_residues;  // offsets[n_seq] - offsets[0] (< 2^32: positions are u32)
  int32_t k;
  int32_t mlen;  // table layout (minimizer length, 0 = flat)
  int32_t min_hits;
  uint32_t flags;
  int32_t* out_fid;
  int32_t* out_count;
  uint8_t* out_status;
  uint32_t* tally;  // may be null
  uint32_t n_fid;
  uint32_t* gset;   // workspace: 2 u32 per residue, sets of proteins that do not fit in LDS
  uint32_t block_proteins;  // proteins per block (1 .. kBlockProteins; the host sizes it)
  // Two-pass grid (defer_below > 0): 2 n_groups blocks; block b < n_groups annotates group b
  // (block_proteins proteins) if it has >= defer_below probe steps, block n_groups + b if it
  // has fewer, so that short groups start after every long one.
  uint32_t defer_below;
  uint32_t n_groups;
  // Input format: 0 = ASCII residues (a.residues + offsets[s]); 1 = the packed stream of
  // kma_device.h (5 bits per residue, stream residue 0 = residue offsets[0]).
  uint32_t packed;
  uint64_t stream_first;  // packed: stream residue index of residue offsets[0]
  uint32_t two_choice;    // table placement: 1 = a missed key's only other bucket is alt_bucket
};

struct ContigArgs {
  const uint64_t* slots;
  uint32_t n_buckets;
  const uint8_t* dna;          // contig s is dna[offsets[s] .. offsets[s+1])
  const uint64_t* offsets;     // n_contig + 1 (device); offsets[0] need not be 0
  uint32_t n_contig;
  uint64_t total_bases;        // offsets[n_contig] - offsets[0] (< 2^39)
  int32_t k;
  int32_t mlen;
  kma_hit* staging;            // n_blocks x kContigTile*2 final hit records (block order)
  uint32_t* block_counts;      // n_blocks (allocated in whole groups of kScanGroup)
  uint64_t* group_sum;         // ceil(n_blocks / kScanGroup) group sums, zero before the probe
                               // (which adds its block counts; null: no emit follows); the
                               // emit pass leaves them zero again
  uint32_t* emit_done;         // emit blocks done (zero before the emit; left zero)
  uint32_t n_groups;           // emit pass (set by launch_contigs_emit)
  uint32_t groups_scanned;     // emit pass: group_sum holds exclusive prefixes
  uint32_t* tally;             // may be null: n_contig x n_fid
  uint32_t n_fid;
  kma_hit* out;                // emit pass: hits [0, cap) in canonical order
  uint64_t cap;
  uint64_t* n_hits;            // emit pass: total hits (also when > cap)
  // KmerFactory.Strict (peg join): pass 1 counts the locations of every table key
  // (strict_pass = 1: atomicAdd per hit into slot_count[slot id], nothing else is meaningful),
  // pass 2 keeps only hits whose key has exactly one location (strict_pass = 2).
  uint32_t* slot_count;        // n_buckets * kSlotsPerBucket, zeroed before pass 1
  int32_t strict_pass;         // 0 = off
  uint32_t two_choice;         // table placement (ProteinArgs::two_choice)
  uint8_t codon_codes[64];     // by value (TCAG order): 5-bit aa code, 0 = stop
};
#ifndef KMA_CONTIG_POS
#define KMA_CONTIG_POS 1
#endif
// Forward positions per lane of the 6-frame probe (2 windows each). 2 raises the kernel to 97
// VGPRs (4 waves/SIMD) and measured slower at c3 (0.139 vs 0.124 ms, profiles/r02i_variants.log).
constexpr int kContigPos = KMA_CONTIG_POS;
// 256-position slices a 6-frame probe block works through one after the other (round 3: 1).
// The block's fixed work — contig search, DNA tile load, translation, compaction, its group-sum
// atomic — is paid once for all of them, and the slices' gathers follow each other while the
// other blocks of the CU overlap them; a lane keeps one slice's loads in flight, so VGPRs stay
// those of one slice (kContigPos = 2 holds two slices' loads at once: 97 VGPRs, 4 waves/SIMD,
// measured slower).
// Round 4: 2 slices (c3 0.124 -> 0.099 ms, profiles/r04/c3_seq_r04c.log), then 4 (0.0916 ->
// 0.087 ms against 3 slices' 0.088, ABAB, profiles/r04/c3_seq_ab_r04final.log). Round 5: 5 / 6 /
// 8 slices 0.0824 / 0.0829 / 0.0868 vs 0.0813 ms (probe 74.4 us at 4; ABAB,
// profiles/r05/c3_seq_ab_r05z/; parity green at 6 and 8).
#ifndef KMA_CONTIG_SEQ
#define KMA_CONTIG_SEQ 4
#endif
constexpr int kContigSeq = KMA_CONTIG_SEQ;
static_assert(kContigSeq == 1 || kContigPos == 1, "sequential slices take one position per lane");
constexpr int kContigTile = 256 * kContigPos * kContigSeq;  // forward positions per block
// Round 5 also built the probe's keys from per-frame 5-bit codon streams in LDS (one funnel
// shift and a borrow test per strand instead of K byte loads, compares and shifts per strand:
// 64 fewer VALU and 12 fewer LDS instructions per position and slice) and measured it slower
// both ways it was built (ABAB on one box each): streams built by a second pass over the codes,
// probe 0.0789 vs 0.0745 ms (profiles/r05/c3_stream_ab_r05e.log); codes ORed into the streams
// by the translation pass (LDS atomics), 0.0766 vs 0.0748 ms (c3_stream_ab_r05f.log). The VALU
// saved was not on the probe's critical path, the per-block phases were (the variant is in the
// history of kma_kernels.hip).
// A persistent 6-frame grid (one resident wave of blocks striding over the tiles, each block
// loading its next tile's DNA under the current tile's probes) was also built in round 5 and
// measured slower: probe 0.0796-0.0803 vs 0.0772-0.0773 ms for a block per tile, ABAB on one
// box (profiles/r05/c3_persistent_ab_r05m.log). The round-4 block clocks had put the tile load
// at 7.2 of a 20.6 us block, but that time is queueing behind the other blocks' bucket
// gathers: a tile costs the same with its DNA prefetched, and the static assignment (2 or 3
// tiles per block) lost the dispatcher's balancing of the last tiles.
constexpr uint32_t kScanGroup = 256;  // probe blocks per emit-offset group sum
// Up to this many groups (16 loads per lane, one round trip) an emit block sums the group sums
// before its own; beyond, a one-block scan turns them into prefixes first.
constexpr uint32_t kDirectGroups = 1024;

// ---- the projector's proposal sweep (kma_proposals.hip) ----------------------------------------
struct PropArgs {
  const kma_hit* hits;  // n connections in canonical (contig, left) order
  uint32_t n;
  const uint32_t* peg_len;  // n_peg protein lengths
  uint32_t n_peg;
  int32_t k;
  double min_strength, max_fuzz, min_fuzz;
  uint32_t *keys, *skeys, *idx, *sidx;      // list keys / sort permutation
  uint32_t *head, *list_no, *starts;        // list boundaries (starts: lists + 1)
  uint32_t* scontig;
  int32_t* sleft;
  uint32_t *keep, *evidence, *out_pos;
  int32_t* best;
  uint64_t* stats;      // 4: lists, too few kmers, too short, proposals
  kma_proposal* out;
  uint64_t cap;
};
hipError_t launch_propose(PropArgs a, void* temp, size_t* temp_bytes, hipStream_t stream);

// ---- launchers (kma_kernels.hip) --------------------------------------------------------------
// status[0] = table full; stats (finalize) = {entries, max chain, displaced keys}.
hipError_t launch_build_insert(uint64_t* slots, uint32_t* winner, uint32_t n_buckets, int k,
                               int m, const uint64_t* keys, uint64_t n, uint32_t* status,
                               hipStream_t stream);
hipError_t launch_build_finalize(uint64_t* slots, const uint32_t* winner, const uint32_t* fids,
                                 uint32_t n_buckets, int k, int m, uint32_t* stats,
                                 hipStream_t stream);
// Two-choice build of a narrow table (slots zeroed by the caller): keys (row order) sorted with
// their row indices into sorted_keys / sorted_rows (rocPRIM radix sort on the 5K key bits; temp
// == nullptr: size query into *temp_bytes), the last row of each key inserted with evictions,
// then the filters; status[0] = an insertion failed, status[1..3] = {entries, longest probe (1
// or 2), displaced keys}.
// Home-first placement's buffers (n entries each; all null: insertion order decides which keys
// of a crowded home live in their alt).
struct TwoChoiceScratch {
  uint32_t* home = nullptr;
  uint32_t* sorted_home = nullptr;
  uint32_t* sorted_idx = nullptr;
  uint8_t* away = nullptr;
  uint8_t* load = nullptr;  // n_buckets: keys homed per bucket (null: alt loads not considered)
};
hipError_t launch_build_two_choice(uint64_t* slots, uint32_t n_buckets, int k, int m,
                                   const uint64_t* keys, const uint32_t* fids, uint64_t n,
                                   uint64_t* sorted_keys, uint32_t* rows, uint32_t* sorted_rows,
                                   const TwoChoiceScratch& x, void* temp, size_t* temp_bytes,
                                   uint32_t* status, hipStream_t stream);
hipError_t launch_annotate(const ProteinArgs& a, hipStream_t stream);  // the protein path
// ASCII residues [offsets[0], offsets[0] + n) -> the packed stream (packed_bytes(n) bytes; the
// LUT of the table's replica): pack_residues_kernel.
hipError_t launch_pack_residues(const uint8_t* residues, const uint64_t* offsets, uint64_t n,
                                const uint8_t* lut, uint8_t* out, hipStream_t stream);
// Bytes of the packed stream of n residues: 40 per 64 residues and 16 of read padding.
__host__ __device__ constexpr uint64_t packed_bytes(uint64_t n) { return 40 * ((n + 63) / 64) + 16; }
hipError_t launch_contigs_emit(const ContigArgs& a, uint64_t n_blocks, hipStream_t stream);
hipError_t launch_contigs_probe(const ContigArgs& a, uint64_t n_blocks, hipStream_t stream);
// Peg-kmer singleton table (KmerReference.countPegKmers + CountMap.getSingletons): every
// window i < L-K without 'X' of every peg -> (key or 0, peg index) per residue position; sort;
// keep keys that occur exactly once.
hipError_t launch_peg_windows(const uint8_t* residues, const uint64_t* offsets, uint32_t n_peg,
                              int k, const uint8_t* lut, uint64_t* keys, uint32_t* pegs,
                              hipStream_t stream);
hipError_t launch_sort_pairs(void* temp, size_t* temp_bytes, const uint64_t* keys_in,
                             uint64_t* keys_out, const uint32_t* vals_in, uint32_t* vals_out,
                             uint64_t n, int key_bits, hipStream_t stream);
hipError_t launch_singleton_flags(const uint64_t* sorted_keys, uint64_t n, uint8_t* flags,
                                  hipStream_t stream);
// Signature build (BuildKmerProcessor): (key, role or kBuildNeg for a buffered protein) per
// window of ProteinKmers (key 0: no window); radix sort of the pairs by key; per key run, good
// iff one role and no buffered occurrence (RoleCounter); select.
constexpr uint32_t kBuildNeg = 0xFFFFFFu;
hipError_t launch_build_windows(const uint8_t* residues, const uint64_t* offsets, uint32_t n_seq,
                                const int32_t* roles, int k, int end_exclusive, const uint8_t* lut,
                                uint64_t* keys, uint32_t* tags, uint32_t* alpha_flag,
                                hipStream_t stream);
// flags[i] = 1 for the first pair of every good key's run (temp == nullptr: size query).
hipError_t launch_signature_flags(const uint64_t* keys, const uint32_t* tags, uint64_t n,
                                  uint8_t* flags, uint32_t* head_idx, uint32_t* run, void* temp,
                                  size_t* temp_bytes, hipStream_t stream);
hipError_t launch_select_flagged(void* temp, size_t* temp_bytes, const uint64_t* keys_in,
                                 const uint32_t* vals_in, const uint8_t* flags, uint64_t* keys_out,
                                 uint32_t* vals_out, uint64_t* n_out, uint64_t n,
                                 hipStream_t stream);

}  // namespace kma
