// kma_kernels.hip — CDNA4 (gfx950) kernels of the signature-kmer annotation hot path.
//
//   build_insert / build_finalize  signature-table construction (ApplyKmerProcessor.java:100-110)
//   annotate_kernel    the protein path in one kernel: every window of every protein packed and
//                      probed in the table (the HashMap.get of ApplyKmerProcessor.java:130 for
//                      every kmer of ProteinKmers at :123), per-protein distinct-key sets and
//                      fid range in LDS, then the vote and min-hits threshold (:129-147).
//   contigs_probe_quad_kernel  6-frame translation + window + probe + block compaction
//                      (KmerReference.java:157-203, KmerPosition.java:50-93)
//   contigs_emit_kernel   canonical-order hit emission after a block-count scan
//   peg_windows / singleton_flags / build_windows / signature_flags  table builders (A9, (f)1)
//
// Integer / byte work only: the bound is HBM (or Infinity-Cache) random access to 64-byte
// buckets, not MFMA.
#include <cstring>  // (rocprim.hpp uses memset without including it)
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "../../include/kmeranno.h"
#include "kma_internal.h"
#include "kma_device.h"


namespace kma {
namespace {


// ---------------------------------------------------------------------------------------------
// Table construction. Insert: claim the first empty slot of the probe chain with a 64-bit CAS
// (slot key bits, fid still 0; the slot's overflow bit may already be set) or find the key
// already there; either way record the row index with atomicMax so the LAST row of a duplicate
// key wins (HashMap.put semantics). A key placed past its home bucket sets its overflow bit
// there. Finalize: write the winning row's fid into the slot; collect entry count, longest
// chain and the number of keys displaced past their home bucket.
// ---------------------------------------------------------------------------------------------
// Wide tables (K > 8): the same with 16-byte slots (kma_internal.h): the claim is a 64-bit CAS
// of the slot's key words (x | y << 32, 0 = empty), the overflow bit and fid live in .z.
template <bool Wide>
__global__ __launch_bounds__(256) void build_insert_kernel(uint64_t* slots, uint32_t* winner,
                                                           uint32_t n_buckets, int k, int m,
                                                           const uint64_t* __restrict__ keys,
                                                           uint64_t n, uint32_t* status) {
  constexpr int S = Wide ? kWideSlots : kSlotsPerBucket;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t key = keys[i];
    if (key == 0 || (key >> (5 * k)) != 0) continue;  // no key / not a K-mer key: never stored
    const uint64_t want = Wide ? key : slot_make(key, 0);
    const uint32_t home = home_bucket(key, k, m, n_buckets);
    uint32_t b = home;
    bool done = false;
    for (uint32_t p = 0; p < n_buckets && !done; ++p) {
      b = chain_bucket(home, p, n_buckets);
      for (int j = 0; j < S; ++j) {
        const uint64_t si = (uint64_t)b * S + j;
        uint64_t* sp = slots + (Wide ? 2 * si : si);
        uint64_t v = __hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (Wide) {
          while (v == 0) {  // empty: claim it
            const uint64_t old = atomicCAS((unsigned long long*)sp, 0ull, (unsigned long long)want);
            v = old == 0 ? want : old;
          }
        } else {
          while ((uint32_t)v == 0u) {  // empty (possibly with its overflow bit set): claim it
            const uint64_t old = atomicCAS((unsigned long long*)sp, (unsigned long long)v, v | want);
            v = old == v ? (v | want) : old;
          }
        }
        if ((Wide ? v : slot_key(v)) == key) {
          atomicMax(winner + si, (uint32_t)(i + 1));
          done = true;
          break;
        }
      }
    }
    if (!done) {
      atomicOr(status, 1u);  // table full: cannot happen at load factor < 1
    } else if (b != home) {  // displaced: set the key's filter positions in its home bucket
      for (int f = 0; f < kFilterBits; ++f) {
        const uint32_t pos = filter_pos<S>((uint32_t)key, f);
        const uint64_t si = (uint64_t)home * S + pos / kFilterBits;
        uint32_t* meta = Wide ? reinterpret_cast<uint32_t*>(slots + 2 * si + 1)   // .z
                              : reinterpret_cast<uint32_t*>(slots + si) + 1;      // high dword
        const uint32_t bit = 1u << (kFidBits + pos % kFilterBits);
        if (!(__hip_atomic_load(meta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit))
          atomicOr(meta, bit);
      }
    }
  }
}

template <bool Wide>
__global__ __launch_bounds__(256) void build_finalize_kernel(uint64_t* slots,
                                                             const uint32_t* __restrict__ winner,
                                                             const uint32_t* __restrict__ fids,
                                                             uint32_t n_buckets, int k, int m,
                                                             uint32_t* stats) {
  constexpr int S = Wide ? kWideSlots : kSlotsPerBucket;
  const uint64_t n_slots = (uint64_t)n_buckets * S;
  uint32_t entries = 0, max_probe = 0, displaced = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_slots;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t w = winner[i];
    if (w == 0) continue;
    uint64_t key;
    if (Wide) {
      key = slots[2 * i];
      uint32_t* meta = reinterpret_cast<uint32_t*>(slots + 2 * i + 1);
      *meta = *meta | (fids[w - 1] & kFidMask);  // keep the filter bits
    } else {
      const uint64_t v = slots[i];
      slots[i] = v | ((uint64_t)(fids[w - 1] & kFidMask) << 32);
      key = slot_key(v);
    }
    const uint32_t b = (uint32_t)(i / S), h = home_bucket(key, k, m, n_buckets);
    const uint32_t d = chain_step(h, b, n_buckets) + 1u;
    entries++;
    displaced += d > 1u ? 1u : 0u;
    max_probe = max(max_probe, d);
  }
  entries = wave_sum(entries);
  max_probe = wave_max(max_probe);
  displaced = wave_sum(displaced);
  if ((threadIdx.x & 63) == 0) {
    if (entries) atomicAdd(stats + 0, entries);
    atomicMax(stats + 1, max_probe);
    if (displaced) atomicAdd(stats + 2, displaced);
  }
}

// ---------------------------------------------------------------------------------------------
// Two-choice build (narrow tables; kma_internal.h alt_bucket). The rows are radix-sorted by key
// with their row index (stable: a key's rows stay in file order), so the last row of every run
// is the row HashMap.put keeps; each such key is inserted into an empty slot of its home or alt
// bucket, or evicts a pseudo-random slot of a full one and carries the victim to the victim's
// other bucket (a random-walk cuckoo insertion; every slot exchange is one 64-bit atomic, so no
// key is lost or doubled). A key still in hand after kMaxKicks evictions marks the build failed
// (the caller builds the table with chains instead). The filter pass then sets, for every key
// stored in its alt bucket, its filter positions in its home bucket, and counts.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void iota_kernel(uint32_t* rows, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    rows[i] = (uint32_t)i;
}

__device__ __forceinline__ bool claim_empty(uint64_t* slots, uint32_t b, uint64_t v) {
  uint64_t* sp = slots + (uint64_t)b * kSlotsPerBucket;
#pragma unroll
  for (int j = 0; j < kSlotsPerBucket; ++j)
    if (__hip_atomic_load(sp + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0ull &&
        atomicCAS((unsigned long long*)(sp + j), 0ull, (unsigned long long)v) == 0ull)
      return true;
  return false;
}

__global__ __launch_bounds__(256) void build_two_choice_insert_kernel(
    uint64_t* slots, uint32_t n_buckets, int k, int m, const uint64_t* __restrict__ skeys,
    const uint32_t* __restrict__ srows, const uint32_t* __restrict__ fids, uint64_t n,
    const uint8_t* __restrict__ away, uint8_t phase, uint32_t* status) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    if (away && away[i] != phase) continue;  // phase 0: the keys kept home; 1: the others
    const uint64_t key = skeys[i];
    if (key == 0 || (key >> (5 * k)) != 0) continue;  // no key / not a K-mer key: never stored
    if (i + 1 < n && skeys[i + 1] == key) continue;   // a later row of this key wins
    uint64_t v = slot_make(key, fids[srows[i]]);
    uint32_t b1 = home_bucket(key, k, m, n_buckets);
    uint32_t b2 = alt_bucket(key, b1, n_buckets);
    uint32_t at = b1;  // the bucket to evict from when both are full
    uint32_t rng = (uint32_t)i * 0x9E3779B1u + 0x7F4A7C15u;
    bool done = false;
    for (uint32_t kick = 0; kick <= kMaxKicks; ++kick) {
      if (claim_empty(slots, b1, v) || claim_empty(slots, b2, v)) {
        done = true;
        break;
      }
      if (kick == kMaxKicks) break;
      rng = rng * 1664525u + 1013904223u;
      const uint32_t j = rng >> (32 - kSlotBits);
      const uint64_t old = atomicExch((unsigned long long*)(slots + (uint64_t)at * kSlotsPerBucket + j),
                                      (unsigned long long)v);
      if (old == 0ull) {  // (slots never empty again once claimed; kept for safety)
        done = true;
        break;
      }
      // the victim lived in `at`: its other bucket first (then `at`, for a slot freed meanwhile)
      v = old;
      const uint64_t vk = slot_key(old);
      const uint32_t h = home_bucket(vk, k, m, n_buckets);
      const uint32_t other = at == h ? alt_bucket(vk, h, n_buckets) : h;
      b1 = other;
      b2 = at;
      at = other;
    }
    if (!done) atomicOr(status, 1u);
  }
}

// Home-first placement (KMA_TC_SELECT): the keys of a home bucket that cannot all live there are
// chosen before any insertion. home_kernel: the home of every key the insert kernel stores (the
// last row of its run, a K-mer key), else kNoHome, with its sorted-key index; the pairs are then
// radix-sorted by home, and select_kernel takes each home's run: up to kSlotsPerBucket keys stay
// (away = 0: inserted first, into the home, where they all fit), the others go away (away = 1:
// inserted after every home is filled, so into their alt buckets, evicting only where an alt
// is full). The keys sent away are chosen greedily to set few filter positions in the home: each
// next one adds the fewest positions not yet set (first 64 keys of a run; the rest go away as
// they come). Against insertion order: c5 (10^8 keys, m = 6) simulated 2.8% -> 1.35% false
// filter hits per missed window; measured displaced keys 7.50 -> 7.18% (a key sent to a full
// alt still evicts), c5 kernel 3.124 -> 3.085 ms, LF 0.75 3.42 -> 3.37 ms (ABAB,
// profiles/r05/tc_select_ab/; KMA_TC_SELECT=0 restores insertion order). Keys whose alt is
// already filled by that bucket's own home keys go away last (each would evict one of them, a
// second displaced key): displaced 7.18 -> 6.99% at LF 0.5 and 17.55 -> 15.49% at 0.75, c5
// kernel 3.095 -> 3.084 and 3.374 -> 3.283 ms (profiles/r05/tc_alt_load_ab/; KMA_TC_ALT_LOAD=0).
constexpr uint32_t kNoHome = 0xFFFFFFFFu;
__global__ __launch_bounds__(256) void build_two_choice_home_kernel(
    const uint64_t* __restrict__ skeys, uint64_t n, int k, int m, uint32_t n_buckets,
    uint32_t* __restrict__ home, uint32_t* __restrict__ idx) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t key = skeys[i];
    const bool stored = key != 0 && (key >> (5 * k)) == 0 && !(i + 1 < n && skeys[i + 1] == key);
    home[i] = stored ? home_bucket(key, k, m, n_buckets) : kNoHome;
    idx[i] = (uint32_t)i;
  }
}
// Keys homed per bucket (capped at 255), from the runs of the sorted homes (zeroed before).
__global__ __launch_bounds__(256) void build_two_choice_load_kernel(
    const uint32_t* __restrict__ hs, uint64_t n, uint8_t* __restrict__ load) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t h = hs[i];
    if (h == kNoHome || (i > 0 && hs[i - 1] == h)) continue;
    uint64_t e = i + 1;
    while (e < n && hs[e] == h && e - i < 255) ++e;
    load[h] = (uint8_t)(e - i);
  }
}
__global__ __launch_bounds__(256) void build_two_choice_select_kernel(
    const uint32_t* __restrict__ hs, const uint32_t* __restrict__ ids,
    const uint64_t* __restrict__ skeys, uint64_t n, const uint8_t* __restrict__ load,
    uint32_t n_buckets, uint8_t* __restrict__ away) {
  constexpr uint32_t S = kSlotsPerBucket;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t h = hs[i];
    if (h == kNoHome) {
      away[ids[i]] = 2;  // not stored: neither phase
      continue;
    }
    // Past a run's first 64 keys (the run is contiguous: hs[i - 64] == h) a key goes away as it
    // comes, written by its own thread; a run's first thread decides its first W <= 64 keys. (One
    // thread per run walking the whole run was O(run) work: keys piling onto one home made the
    // build a single-thread job)
    if (i >= 64 && hs[i - 64] == h) {
      away[ids[i]] = 1;
      continue;
    }
    if (i > 0 && hs[i - 1] == h) continue;  // within the first 64: the run's first thread
    uint64_t e = i + 1;
    while (e < n && hs[e] == h && e - i < 64) ++e;
    const uint32_t W = (uint32_t)(e - i);
    for (uint64_t j = i; j < e; ++j) away[ids[j]] = 0;
    if (W <= S) continue;
    uint64_t chosen = 0;
    uint32_t set = 0;
    for (uint32_t it = 0; it < W - S; ++it) {
      uint32_t best = 0, best_new = 64, best_mask = 0;
      for (uint32_t j = 0; j < W; ++j) {
        if (chosen >> j & 1ull) continue;
        const uint64_t key = skeys[ids[i + j]];
        const uint32_t mask = filter_need<S>((uint32_t)key);
        // a key whose alt is filled by its own home keys would evict one of them (a second key
        // displaced): such keys go last
        const bool alt_full = load && load[alt_bucket(key, h, n_buckets)] >= S;
        const uint32_t fresh = (uint32_t)__popc(mask & ~set) + (alt_full ? 32u : 0u);
        if (fresh < best_new) {
          best = j;
          best_new = fresh;
          best_mask = mask;
          if (fresh == 0) break;
        }
      }
      chosen |= 1ull << best;
      set |= best_mask;
      away[ids[i + best]] = 1;
    }
  }
}

__global__ __launch_bounds__(256) void build_two_choice_filter_kernel(uint64_t* slots,
                                                                      uint32_t n_buckets, int k,
                                                                      int m, uint32_t* stats) {
  constexpr int S = kSlotsPerBucket;
  const uint64_t n_slots = (uint64_t)n_buckets * S;
  uint32_t entries = 0, displaced = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_slots;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t v = __hip_atomic_load(slots + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)v == 0u) continue;
    const uint64_t key = slot_key(v);
    const uint32_t b = (uint32_t)(i / S), h = home_bucket(key, k, m, n_buckets);
    entries++;
    if (b != h) {  // in its alt bucket: its filter positions in the home bucket
      displaced++;
      for (int f = 0; f < kFilterBits; ++f) {
        const uint32_t pos = filter_pos<S>((uint32_t)key, f);
        uint32_t* meta = reinterpret_cast<uint32_t*>(slots + (uint64_t)h * S + pos / kFilterBits) + 1;
        const uint32_t bit = 1u << (kFidBits + pos % kFilterBits);
        // read first: keys displaced from one crowded home would otherwise serialize on the
        // same words (one atomic each)
        if (!(__hip_atomic_load(meta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit))
          atomicOr(meta, bit);
      }
    }
  }
  entries = wave_sum(entries);
  displaced = wave_sum(displaced);
  if ((threadIdx.x & 63) == 0) {
    if (entries) atomicAdd(stats + 0, entries);
    atomicMax(stats + 1, displaced ? 2u : entries ? 1u : 0u);
    if (displaced) atomicAdd(stats + 2, displaced);
  }
}

// ---------------------------------------------------------------------------------------------
// The protein path (ApplyKmerProcessor.java:122-148 with ProteinKmers at :123): one kernel.
//
// A block owns kBlockProteins consecutive proteins. Every window of theirs is probed with
// quad-cooperative bucket loads: each lane packs its own windows' keys, then the four lanes of
// a quad read their four windows' buckets together (lane p loads bytes [16p, 16p + 16) of each:
// one wave instruction reads 16 whole 64-byte lines, the access shape with the higher measured
// random-gather rate) and combine matches with DPP quad ops. Adjacent lanes hold consecutive
// windows, which share their minimizer home bucket 1/3-1/2 of the time, so a repeated line is
// served by the CU's L1/L2 instead of HBM. Overflow chains (~1% of probes) are deferred to a
// per-wave LDS queue and walked 64 at a time.
//
// A hit updates its protein's record in LDS: smallest / largest fid (non-returning atomics)
// and the set of distinct keys hit (ProteinKmers is a set: a kmer occurring twice counts
// once; a key's slot id is its identity in the table). After one barrier the vote is read off
// the record, order-free: no hit -> NONE (roleId == null); smallest != largest -> AMBIGUOUS
// (badPeg); else the role with count = |set|, CALLED iff count >= minHits (:146). The Java
// loop's early break at the second role changes nothing it reports.
//
// Sets: ceil(1.5 x windows) u32 entries (load <= 2/3 however many windows hit) from the
// block's LDS pool, greedily in protein order; a protein that does not fit uses its own region
// of workspace memory (2 u32 per residue at its residues' offset), so any protein length is
// voted exactly. Windows that straddle two proteins are not probed.
// ---------------------------------------------------------------------------------------------

#ifdef KMA_BLOCK_CLOCK
// Tuning builds only (make variant VNAME=clk VFLAGS=-DKMA_BLOCK_CLOCK, scripts/block_clock.py):
// per block of the last protein launch, wall clock at 0 start, 1 records ready, 2 first step
// matched, 3 steps done, 4 chain walks done, 5 end; 6 hardware ids; 7 steps.
__device__ uint64_t g_block_clk[8 * 65536];
#define KMA_CLK_SET(i, v)                                          \
  do {                                                             \
    if (threadIdx.x == 0 && blockIdx.x < 65535)                    \
      g_block_clk[8 * blockIdx.x + (i)] = (v);                     \
  } while (0)
#define KMA_CLK(i) KMA_CLK_SET(i, wall_clock64())
#define KMA_CLK_HW()                                                \
  KMA_CLK_SET(6, (uint64_t)__builtin_amdgcn_s_getreg(20 | (15 << 11)) << 32 | \
                     (uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11)))
#else
#define KMA_CLK_SET(i, v) ((void)0)
#define KMA_CLK(i) ((void)0)
#define KMA_CLK_HW() ((void)0)
#endif

#ifdef KMA_TUNE_COUNT
// Tuning builds only (make variant VNAME=count VFLAGS=-DKMA_TUNE_COUNT): wave-level event
// counts of the protein launches since the last reset (kma_debug_walk_stats): 0 chain flushes,
// 1 queued walks, 2 probed windows, 3 home-bucket hits, 4 walk hits, 5 walk hits in the
// chain's first bucket, 6 chain buckets loaded by walks, 7 the sum over flush passes of the
// longest walk (buckets) in the pass.
__device__ unsigned long long g_walk_stats[8];
#define KMA_COUNT(i, v)                                                                    \
  do {                                                                                     \
    const unsigned long long kma_v_ = (unsigned long long)(v); /* wave-wide, all lanes */  \
    if ((threadIdx.x & 63) == 0)                                                           \
      __hip_atomic_fetch_add(&g_walk_stats[i], kma_v_, __ATOMIC_RELAXED,                   \
                             __HIP_MEMORY_SCOPE_AGENT);                                    \
  } while (0)
#else
#define KMA_COUNT(i, v) ((void)0)
#endif

// Per-block protein records (LDS). The layout keeps kProteinOcc blocks per CU resident.
template <int P>
struct ProteinSmem {
  __attribute__((aligned(16))) uint32_t pool[kSetPool];  // LDS sets: slot id + 1, 0 = empty
  uint32_t chain_q[kWavesPerBlock][2 * kChainQ];  // deferred chain walks: packed key, protein
  uint32_t pbeg[P + 1];  // protein starts relative to the span start; [np..P] = span end
  uint32_t pwin[P];      // windows of the protein (ProteinKmers: L - K + 1, or L - K)
  uint32_t pset[P];      // set base in `pool`, or kGlobalSet
  uint32_t pcap[P];      // set capacity (0: no set)
  uint32_t pmin[P], pmax[P], pcnt[P];  // smallest / largest fid hit; distinct keys (or hits)
  uint32_t plist[P];                   // kGlobalSet proteins: hits appended to their list
  uint32_t skip;                       // two-pass grid: the group belongs to the other pass
  uint8_t lut[256];
};
static_assert(sizeof(ProteinSmem<kBlockProteins>) <= 163840 / kProteinOcc,
              "protein-path LDS must leave kProteinOcc blocks per CU");

// Insert slot id + 1 in a set of `cap` u32 entries; true if it was not there.
__device__ __forceinline__ bool lds_set_insert(uint32_t* set, uint32_t cap, uint32_t key) {
  uint32_t i = set_slot(key, cap);
  for (;;) {
    const uint32_t o = atomicCAS(set + i, 0u, key);
    if (o == 0u) return true;
    if (o == key) return false;
    i = i + 1 == cap ? 0u : i + 1;
  }
}
__device__ __forceinline__ bool global_set_insert(uint32_t* set, uint32_t cap, uint32_t key) {
  uint32_t i = set_slot(key, cap);
  for (;;) {
    uint32_t o = 0u;
    __hip_atomic_compare_exchange_strong(set + i, &o, key, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    if (o == 0u) return true;
    if (o == key) return false;
    i = i + 1 == cap ? 0u : i + 1;
  }
}

// A hit of protein p (of the block) on the key with slot id `sid` and function `fid`. A protein
// whose set is in LDS inserts the slot id there (a fresh key counts); a protein whose set did not
// fit (kGlobalSet) appends it to its list in workspace memory (its own residues' region: 2 u32
// per residue), deduplicated after the probe steps (dedupe_lists). Round 3 kept a hash set
// there, zeroed by the block and filled by agent-scope CAS: at c5 0.23 GB of writes per launch
// for 9 MB of outputs, the set lines being evicted from L2 between hits under the gather load.
template <int P>
__device__ __forceinline__ void record_hit(ProteinSmem<P>& sm, const ProteinArgs& a,
                                           uint64_t span_lo, bool multiset, uint32_t p,
                                           uint32_t fid, uint32_t sid) {
  atomicMin(&sm.pmin[p], fid);
  atomicMax(&sm.pmax[p], fid);
  bool fresh = true;  // multiset: every hit counts
#ifdef KMA_TUNE_NO_SET  // tuning builds only (cost bound of the distinct-key sets; wrong counts)
  fresh = false;
  if (false) {
#else
  if (!multiset) {
#endif
    const uint32_t base = sm.pset[p];
    if (base != kGlobalSet) {
      fresh = lds_set_insert(sm.pool + base, sm.pcap[p], sid + 1u);
    } else {
      a.gset[2 * (span_lo + sm.pbeg[p]) + atomicAdd(&sm.plist[p], 1u)] = sid + 1u;
      fresh = false;
    }
  }
  if (fresh) atomicAdd(&sm.pcnt[p], 1u);
}

// After the probe steps (the LDS sets are final, the pool is free): the distinct slot ids of
// every kGlobalSet protein's list, counted into pcnt. A list of fewer than kSetPool hits is
// deduplicated in the pool (the usual case: it needs 2,730+ windows to have that many); a
// longer one (giant proteins) in a hash set of L entries in the second half of its region,
// zeroed here (agent-scope stores, the CAS inserts are agent-scope). Block-uniform loop.
// (Protein bounds from LDS: indexing the kernel's register copy pb[] by the loop counter makes
// the compiler spill it to scratch.)
template <int P>
__device__ __forceinline__ void dedupe_lists(ProteinSmem<P>& sm, const ProteinArgs& a,
                                             uint64_t span_lo) {
  const int t = threadIdx.x;
  for (int p = 0; p < P; ++p) {
    if (sm.pset[p] != kGlobalSet) continue;
    const uint32_t h = sm.plist[p], b0 = sm.pbeg[p];
    if (h == 0) continue;
    const uint32_t* list = a.gset + 2 * (span_lo + b0);
    uint32_t fresh = 0;
    if (h < (uint32_t)kSetPool) {
      uint4* pool4 = reinterpret_cast<uint4*>(sm.pool);
      for (uint32_t i = t; i < (uint32_t)kSetPool / 4; i += 256) pool4[i] = make_uint4(0u, 0u, 0u, 0u);
      __syncthreads();
      for (uint32_t i = t; i < h; i += 256) fresh += lds_set_insert(sm.pool, kSetPool, list[i]);
    } else {
      const uint32_t L = sm.pbeg[p + 1] - b0;  // > windows >= h: the set never fills
      uint32_t* set = a.gset + 2 * (span_lo + b0) + L;
      for (uint32_t i = t; i < L; i += 256)
        __hip_atomic_store(set + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence();  // (giant proteins only: an L2 writeback per such protein)
      __syncthreads();
      for (uint32_t i = t; i < h; i += 256) fresh += global_set_insert(set, L, list[i]);
    }
    fresh = wave_sum(fresh);
    if ((t & 63) == 0 && fresh) atomicAdd(&sm.pcnt[p], fresh);
    __syncthreads();  // the pool (or the set) is free for the next list
  }
}

// Which of the block's proteins holds span position x (pb: the block-uniform starts, in
// scalar registers).
template <int P>
__device__ __forceinline__ uint32_t protein_at(const uint32_t (&pb)[P + 1], uint32_t x) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 1; i < P; ++i) p += x >= pb[i] ? 1u : 0u;
  return p;
}
// Whether x (in protein p = protein_at(pb, x)) starts one of p's windows: pe[i] = pb[i] +
// windows of i <= pb[i + 1], so the proteins whose windows end at or below x are exactly those
// before p, plus p itself when x is past its last window. A compare count, like protein_at: a
// select of pe[p] is folded by the compiler into a dynamically indexed private array (scratch
// memory: 32 bytes per lane stored per block, ~2 GB of writes per c5 launch).
template <int P>
__device__ __forceinline__ bool window_at(const uint32_t (&pe)[P], uint32_t x, uint32_t p) {
  uint32_t ended = 0;
#pragma unroll
  for (int i = 0; i < P; ++i) ended += x >= pe[i] ? 1u : 0u;
  return ended == p;
}

// The lane's window within each 256-window slice. KMA_LANE_PERM: quad q's member p takes
// window 16 p + q of its wave, so that load instruction r (member r of every quad) reads the
// buckets of 16 consecutive windows — windows that share a minimizer then share a line inside
// one instruction.
__device__ __forceinline__ uint32_t lane_window(int t) {
#if KMA_LANE_PERM
  return (uint32_t)((t >> 6) * 64 + 16 * (t & 3) + ((t & 63) >> 2));
#else
  return (uint32_t)t;
#endif
}

// A group's inputs that precede its first probe step: its proteins, the offsets wave 0 reads
// (lane <= np: offsets[p0 + lane]) and the span start: two dependent round trips with the
// first residues (offsets, then residues: 4.5 and ~4 us of a ~37 us c5 block at 6 proteins,
// profiles/r03_ab/r03o block clocks). A persistent grid loading the next group's head under
// the current group's steps was tried: the group loop cost 48-112 bytes per lane of register
// spills (scratch memory) at 7 waves per SIMD.
// KMA_XCD_GROUPS: block b -> group so that the blocks dispatched to one XCD (b mod 8, the
// round-robin dispatch) take consecutive groups: their offsets and span-edge residue lines
// then meet in that XCD's L2. A bijection on [0, n): the last n mod 8 blocks keep their index.
// Measured (profiles/r03_session2/r03z_steps.log, arms interleaved): c5 3.618-3.631 vs
// 3.634-3.637 ms, c4 2.811 vs 2.824; c2 (two-pass grid) 2-7% slower, so not used there.
#ifndef KMA_XCD_GROUPS
#define KMA_XCD_GROUPS 1
#endif
__device__ __forceinline__ uint32_t xcd_group(uint32_t b, uint32_t n) {
#if KMA_XCD_GROUPS
  const uint32_t per = n >> 3;
  return b < 8u * per ? (b & 7u) * per + (b >> 3) : b;
#else
  (void)n;
  return b;
#endif
}

struct GroupHead {
  uint32_t p0, np;
  uint64_t beg_raw;
  uint64_t span_lo;
};
__device__ __forceinline__ void head_offsets(const ProteinArgs& a, uint32_t g, GroupHead& h) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  h.p0 = g * a.block_proteins;  // g < n_groups: p0 < n_seq
  h.np = min(a.block_proteins, a.n_seq - h.p0);
  h.beg_raw = wave == 0 && lane <= (int)h.np ? a.offsets[h.p0 + lane] : 0u;
  h.span_lo = a.offsets[h.p0] - a.offsets[0];
}
// Window x of the span is at position x + pos0 of `res`. ASCII residues: `res` is the aligned
// word at or below the span's first byte (d_residues is 8-byte aligned) and pos0 < 8 the byte
// offset; packed streams (Packed): `res` is the stream and pos0 the span's first residue in it
// (the stream starts at the call's first residue).
template <bool Packed>
__device__ __forceinline__ const uint8_t* head_res(const ProteinArgs& a, const GroupHead& h,
                                                   uint64_t& pos0) {
  if (Packed) {
    pos0 = a.stream_first + h.span_lo;
    return a.residues;
  }
  const uint8_t* res0 = a.residues + a.offsets[0] + h.span_lo;
  pos0 = (uintptr_t)res0 & 7u;
  return res0 - pos0;
}
template <bool Packed>
__device__ __forceinline__ WinWords load_win(const uint8_t* __restrict__ res, uint64_t pos) {
  return Packed ? window_words_packed(res, pos) : window_words(res, pos);
}
// The group's first probe step's residue words (clamped to the batch, which is readable past
// its end; windows past the span are masked in the loop).
template <int U, bool Packed>
__device__ __forceinline__ void head_residues(const ProteinArgs& a, const GroupHead& h,
                                              uint32_t tw, WinWords (&ww)[U]) {
  uint64_t pos0;
  const uint8_t* res = head_res<Packed>(a, h, pos0);
  const uint64_t lim = a.n_residues - h.span_lo;
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint32_t x = j * 256u + tw;
    ww[j] = load_win<Packed>(res, (x < lim ? x : 0u) + pos0);
  }
}

// The group h: proteins [p0, p0 + np) (np <= P), contiguous in the batch, whose first step's
// residue words are in ww. pass 0 / 1: a block of the two-pass grid, which annotates its group
// only if the group is long (pass 0) / short (pass 1: fewer than defer_below probe steps);
// pass -1: always. sm.lut is being loaded (read after the first barrier).
template <int K, int M, int P, bool Packed>
__device__ __forceinline__ void annotate_block(const ProteinArgs& a, ProteinSmem<P>& sm,
                                               const GroupHead& h, WinWords (&ww)[kProbeWin],
                                               const int pass = -1) {
  constexpr int U = kProbeWin;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, part = t & 3;
  const bool multiset = (a.flags & KMA_F_MULTISET) != 0;
  const uint32_t tw = lane_window(t);
  const uint32_t p0 = h.p0, np = h.np;
  const uint64_t beg_raw = h.beg_raw, span_lo = h.span_lo;
  const uint64_t o0 = a.offsets[0];
  uint64_t pos0;
  const uint8_t* __restrict__ res = head_res<Packed>(a, h, pos0);
  if (wave == 0) {  // the block's protein records
    const uint64_t beg = lane <= (int)np ? beg_raw - o0 : 0u;
    const uint64_t end = __shfl_down(beg, 1, 64);
    const uint64_t lo = __shfl(beg, 0, 64), span_end = __shfl(beg, (int)np, 64);
    if (pass >= 0 && lane == 0) {  // two-pass grid: is the group this pass's?
      const bool short_group = span_end - lo < (uint64_t)a.defer_below * 256u * kProbeWin;
      sm.skip = short_group != (pass == 1) ? 1u : 0u;
    }
    if (lane <= P) sm.pbeg[lane] = (uint32_t)((lane <= (int)np ? beg : span_end) - lo);
    if (lane < P) {
      uint32_t nw = 0;
      if (lane < (int)np) {
        const int64_t n = (int64_t)(end - beg) - K + ((a.flags & KMA_F_END_EXCLUSIVE) ? 0 : 1);
        nw = n > 0 ? (uint32_t)n : 0u;
      }
      sm.pwin[lane] = nw;
      sm.pcap[lane] = (nw == 0 || multiset) ? 0u : ((nw + (nw >> 1) + 4u) & ~3u);
      sm.pmin[lane] = 0xFFFFFFFFu;
      sm.pmax[lane] = 0u;
      sm.pcnt[lane] = 0u;
      sm.plist[lane] = 0u;
    }
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {  // LDS pool for the sets; workspace memory for those that do not fit
      uint32_t sum = 0;
      for (int p = 0; p < P; ++p) sum += sm.pcap[p];
      uint32_t top = 0;
      if (sum <= (uint32_t)kSetPool) {  // the usual case: every set in LDS, in protein order
        for (int p = 0; p < P; ++p) {
          sm.pset[p] = top;
          top += sm.pcap[p];
        }
      } else {
        // First fit by decreasing size (fewer windows left to workspace sets than protein
        // order: 1.9% vs 2.4% of c5's windows in a simulation of its length distribution).
        uint32_t done = 0;
        for (int it = 0; it < P; ++it) {
          int best = -1;
          for (int p = 0; p < P; ++p)
            if (!(done >> p & 1u) && (best < 0 || sm.pcap[p] > sm.pcap[best])) best = p;
          done |= 1u << best;
          const uint32_t cap = sm.pcap[best];
          const bool fits = top + cap <= (uint32_t)kSetPool;
          sm.pset[best] = fits ? top : kGlobalSet;  // (a list: appended, never zeroed)
          top += fits ? cap : 0u;
        }
      }
      sm.chain_q[0][0] = top;  // pool entries in use (read before the queues are)
    }
  }
  __syncthreads();
  if (pass >= 0 && sm.skip) return;  // block-uniform
  const uint32_t used = sm.chain_q[0][0];
  uint32_t pb[P + 1], pe[P];
#pragma unroll
  for (int i = 0; i <= P; ++i) pb[i] = __builtin_amdgcn_readfirstlane(sm.pbeg[i]);
#pragma unroll
  for (int i = 0; i < P; ++i) pe[i] = __builtin_amdgcn_readfirstlane(sm.pbeg[i] + sm.pwin[i]);
  const uint32_t span = pb[P];
  __syncthreads();  // `used` has been read by every wave
  uint4* pool4 = reinterpret_cast<uint4*>(sm.pool);
  KMA_CLK(1);
  for (uint32_t i = t; i < used / 4; i += 256) pool4[i] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();

  const uint64_t* __restrict__ slots = a.slots;
  const uint32_t nb = a.n_buckets;
  const bool two_choice = a.two_choice != 0;
  const uint8_t* lut = sm.lut;
  uint32_t* cq = sm.chain_q[wave];
  uint32_t cn = 0;  // wave-uniform queue length
  constexpr uint32_t stride = 256u * U;
  // Deferred chain walks, 64 queued windows at a time: lane (quad g, member p) takes entry
  // 16 p + g of the chunk; the chain's first bucket of every entry is loaded and matched by a
  // quad (the probe loop's cooperative loads: 2 line requests per bucket instead of 8 dwordx4
  // of one lane), and only an entry whose first chain bucket is full and misses walks on alone.
  // Deferred chain walks: one lane per queued window (its packed key and protein from the
  // queue), whole-bucket loads. Measured against alternatives at c5 (profiles/r03_ab): queueing
  // positions and re-packing the residues 3.955 vs 3.86 ms; the chain's first bucket matched by
  // quads with cooperative loads 4.01 vs 3.94 ms (6.31 vs 6.35 at load factor 0.9).
  auto chain_flush = [&]() {
    __builtin_amdgcn_wave_barrier();  // queue writes of other lanes are visible (LDS in order)
    KMA_COUNT(0, 1);
    KMA_COUNT(1, cn);
#ifdef KMA_TUNE_COUNT
    uint32_t wsum = 0, wmax = 0;
#endif
    for (uint32_t e = lane; e < cn; e += 64) {
      const uint32_t w2 = cq[2 * e + 1];
      const uint64_t key = (uint64_t)(w2 & 0xFFu) << 32 | cq[2 * e];
      const uint32_t p = w2 >> 8;
      uint32_t fid = 0, sid = 0;
#ifdef KMA_TUNE_COUNT
      uint32_t walked = 0;
      const bool hit = walk_chain(slots, nb, home_bucket(key, K, M, nb), key, fid, sid, two_choice,
                                  &walked);
#else
      const bool hit = walk_chain(slots, nb, home_bucket(key, K, M, nb), key, fid, sid, two_choice);
#endif
      if (hit) record_hit<P>(sm, a, span_lo, multiset, p, fid, sid);
#ifdef KMA_TUNE_COUNT
      {
        const uint32_t s1 = chain_bucket(home_bucket(key, K, M, nb), 1u, nb);
        const bool first = hit && sid / kSlotsPerBucket == s1;  // resolved in chain step 1
        KMA_COUNT(4, __popcll(__ballot(hit)));
        KMA_COUNT(5, __popcll(__ballot(first)));
        wsum += walked;
        wmax = walked > wmax ? walked : wmax;
      }
#endif
    }
#ifdef KMA_TUNE_COUNT
    KMA_COUNT(6, wave_sum(wsum));  // chain buckets loaded by walks (converged here)
    KMA_COUNT(7, wave_max(wmax));  // the flush waits for its longest walk
#endif
    __builtin_amdgcn_wave_barrier();
    cn = 0;
  };
  // A step's windows: packed keys (khi: key bits 32..39 << 24, bit 0 set for a window that
  // does not probe; the match reads khi's top byte only), filter masks and home buckets (bk:
  // protein << kBucketBits | home bucket, bucket 0 for a window that does not probe), from the
  // residues in ww. (A kNone sentinel in bk cost the gather a compare and a select per bucket;
  // a separate flag array, SGPR spills in the ASCII kernels.)
  struct Prep {
    uint32_t klo[U], khi[U], need[U], bk[U];
  };
  auto prep = [&](uint32_t xs, Prep& o) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint32_t x = xs + j * 256u + tw;
      const uint32_t p = protein_at<P>(pb, x);
      uint64_t key;
      bool ok;
      if (Packed) {  // (key 0: every residue without a code; it would match an empty slot)
        key = packed_key<K>(ww[j]);
        ok = key != 0 && x < span && window_at<P>(pe, x, p);
      } else {
        ok = pack_window<K>(lut, win_bytes(ww[j]), key) && x < span && window_at<P>(pe, x, p);
      }
      o.klo[j] = (uint32_t)key;
      o.khi[j] = (uint32_t)(key >> 32) << 24 | (ok ? 0u : 1u);  // bit 0: does not probe
      o.need[j] = filter_need<kSlotsPerBucket>(o.klo[j]);
      o.bk[j] = p << kBucketBits | (ok ? home_bucket(key, K, M, nb) : 0u);
    }
  };
  // Cooperative loads: the quad's four buckets, 64 bytes at a time (lane `part` reads bytes
  // [16 part, 16 part + 16) of each 64-byte half), all dwordx4 of the lane in flight before any
  // compare. A window that does not probe reads bucket 0 (result discarded).
  auto gather = [&](const Prep& c, uint4 (&q)[U][4][kBucketHalves]) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint32_t b0 = quad_bcast<0>(c.bk[j]), b1 = quad_bcast<1>(c.bk[j]);
      const uint32_t b2 = quad_bcast<2>(c.bk[j]), b3 = quad_bcast<3>(c.bk[j]);
      const uint32_t bb[4] = {b0, b1, b2, b3};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint4* bp = reinterpret_cast<const uint4*>(slots) + part +
                          (uint64_t)(bb[r] & kBucketIdx) * kBucketQuads;
#pragma unroll
        for (int h = 0; h < kBucketHalves; ++h) q[j][r][h] = bp[4 * h];
      }
    }
  };
  auto load_residues = [&](uint32_t xs) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint32_t x = xs + j * 256u + tw;
      ww[j] = load_win<Packed>(res, (x < span ? x : 0u) + pos0);
    }
  };
  // Compare the quad's buckets, record hits, queue chain walks.
  auto settle = [&](uint32_t x0, const Prep& c, const uint4 (&q)[U][4][kBucketHalves]) {
    uint32_t word[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      word[j] = 0;
      uint32_t raw[4];
      (void)raw;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t kl = r == 0 ? quad_bcast<0>(c.klo[j]) : r == 1 ? quad_bcast<1>(c.klo[j])
                          : r == 2 ? quad_bcast<2>(c.klo[j]) : quad_bcast<3>(c.klo[j]);
        const uint32_t kh = r == 0 ? quad_bcast<0>(c.khi[j]) : r == 1 ? quad_bcast<1>(c.khi[j])
                          : r == 2 ? quad_bcast<2>(c.khi[j]) : quad_bcast<3>(c.khi[j]);
        const uint32_t nd = r == 0 ? quad_bcast<0>(c.need[j]) : r == 1 ? quad_bcast<1>(c.need[j])
                          : r == 2 ? quad_bcast<2>(c.need[j]) : quad_bcast<3>(c.need[j]);
#if KMA_QUAD_XPOSE
        raw[r] = match_part_raw(q[j][r], kl, kh, nd, part);
#else
        const uint32_t v = match_part(q[j][r], kl, kh, nd, part);
        word[j] = part == r ? v : word[j];
#endif
      }
#if KMA_QUAD_XPOSE
      word[j] = quad_reduce_scatter(raw, part);
#endif
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const bool probed = (c.khi[j] & 1u) == 0u;
      const uint32_t w = probed ? word[j] : 0u;
#ifdef KMA_TUNE_COUNT
      KMA_COUNT(2, __popcll(__ballot(probed)));
      KMA_COUNT(3, __popcll(__ballot((w & kWordHit) != 0u)));
#endif
      if (w & kWordHit)
        record_hit<P>(sm, a, span_lo, multiset, c.bk[j] >> kBucketBits, w & kFidMask,
                      (c.bk[j] & kBucketIdx) * kSlotsPerBucket + ((w >> kSlotShift) & kSlotMask));
      // rare: the home bucket missed and the key's filter positions are set -> deferred walk
#ifdef KMA_TUNE_NO_WALK  // tuning builds only (cost bound of the chain walks; misses keys)
      const bool pend = false;
#else
      const bool pend = probed && w == 0u;
#endif
      const uint64_t m = __ballot(pend);
      if (pend) {  // queue entry: key bits 0..31; key bits 32..39 | protein << 8
        const uint32_t e = cn + popc_below(m);
        cq[2 * e] = c.klo[j];
        cq[2 * e + 1] = (c.khi[j] >> 24) | (c.bk[j] >> kBucketBits) << 8;
      }
      cn += (uint32_t)__popcll(m);
    }
    if (cn > (uint32_t)(kChainQ - 64 * U)) chain_flush();
  };
  // Software pipeline: the residues of step i + 1 are loaded while step i's buckets are in
  // flight, so a wave's only exposed latency per step is the bucket gather. (A two-stage
  // pipeline packing step i + 1 under step i's gather measured 6.51 vs 4.48 ms at c5,
  // profiles/r03_ab/r03h_steps.log.)
  for (uint32_t x0 = 0; x0 < span; x0 += stride) {
    Prep cur;
    prep(x0, cur);
    uint4 q[U][4][kBucketHalves];
    gather(cur, q);
    // next step's residues (issued after the bucket loads: waiting for those leaves these in
    // flight, vmcnt counts in order)
    load_residues(x0 + stride);  // (past the span: clamped to its first word)
    settle(x0, cur, q);
    if (x0 == 0) KMA_CLK(2);
  }
  KMA_CLK(3);
  KMA_CLK_SET(7, (span + stride - 1) / stride);
  if (cn) chain_flush();
  KMA_CLK(4);
  __syncthreads();  // every LDS set is final; the lists are complete
  if (!multiset) dedupe_lists<P>(sm, a, span_lo);
  if (t < (int)np) {
    const uint32_t mn = sm.pmin[t], mx = sm.pmax[t], cnt = sm.pcnt[t];
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
    a.out_fid[p0 + t] = fid_out;
    a.out_count[p0 + t] = cnt_out;
    a.out_status[p0 + t] = st;
  }
}

// Occupancy: kProteinOcc waves per SIMD (its LDS and VGPR budget); the flat layout's variants
// (a fallback for crowded tables: two full-key mixes per window) and the mod-sampling order's
// ASCII variant (the LUT pack of a window beside the order's ranks; small device calls only,
// larger ones pack first) need 6 to stay clear of scratch.
template <int K, int M, bool Packed>
constexpr int protein_occ() {
  return (M == 0 && (Packed || K < 8)) || (!Packed && (M & kOrderMod)) ? 6 : kProteinOcc;
}
template <int K, int M, int P, bool Packed>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(protein_occ<K, M, Packed>(), 8))) void annotate_kernel(
    ProteinArgs a) {
  __shared__ ProteinSmem<P> sm;
  KMA_CLK(0);
  const int t = threadIdx.x;
  // The ASCII kernel's LUT: loaded now, stored to LDS once the first residue loads are issued
  // (its store right here made the block wait for it before loading the offsets: one more
  // dependent round trip per block). Read after annotate_block's first barrier.
  const uint8_t lut_b = Packed ? 0 : a.lut[t];
  // Two-pass grid (defer_below > 0): blocks [0, n_groups) annotate the long groups, blocks
  // [n_groups, 2 n_groups) the short ones, so that every long group starts before any short
  // one (blocks are dispatched in index order); a block whose group is the other pass's exits
  // after reading its offsets.
  const bool second = a.defer_below && blockIdx.x >= a.n_groups;
  GroupHead h;
  WinWords ww[kProbeWin];
  // (the two-pass grid keeps block order: its long-first order is what it is for)
  const uint32_t b = blockIdx.x - (second ? a.n_groups : 0u);
  head_offsets(a, a.defer_below ? b : xcd_group(b, a.n_groups), h);
  head_residues<kProbeWin, Packed>(a, h, lane_window(t), ww);
  if (!Packed) sm.lut[t] = lut_b;
  annotate_block<K, M, P, Packed>(a, sm, h, ww, a.defer_below ? (second ? 1 : 0) : -1);
  KMA_CLK(5);
  KMA_CLK_HW();
}

#ifdef KMA_TUNE_COUNT
}  // namespace
}  // namespace kma
extern "C" int kma_debug_walk_stats(uint64_t* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(kma::g_walk_stats), 64, 0,
                                     hipMemcpyDeviceToHost);
  if (e == hipSuccess && reset) {
    const uint64_t z[8] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(kma::g_walk_stats), z, 64, 0, hipMemcpyHostToDevice);
  }
  return (int)e;
}
namespace kma {
namespace {
#endif

#ifdef KMA_BLOCK_CLOCK
}  // namespace
}  // namespace kma
extern "C" int kma_debug_block_clock(uint64_t* out, uint64_t n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(kma::g_block_clk), 8 * n, 0,
                                  hipMemcpyDeviceToHost);
}
namespace kma {
namespace {
#endif

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


// The two windows a position anchors ('+' and '-') are probed with the quad-cooperative bucket
// loads of the protein path (both probes' 8 dwordx4 of a lane in flight before any compare,
// DPP quad match); the tile's contigs are found once (two wave-parallel searches) and their
// offsets cached in LDS, so a position's contig costs no global loads. Hits are compacted per
// block in canonical order (position, '+' before '-'); group sums of the block counts and an emit
// pass (each block computes its offset from them) write every block's hits in order.
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

// Waves per SIMD of the 6-frame probe: 8 with one slice per block (64 VGPRs); the sequential
// slices' loop carries a few more scalar and vector values (SGPR spills land in VGPR lanes) and
// takes 7 to stay clear of scratch.
#ifndef KMA_CONTIG_OCC
#define KMA_CONTIG_OCC (KMA_CONTIG_SEQ > 1 ? 7 : 8)
#endif
template <int K, int M>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KMA_CONTIG_OCC, 8))) void contigs_probe_quad_kernel(
    ContigArgs a) {
  // K > 8: a wide table (16-byte slots, kma_internal.h): one slot per lane of the quad.
  constexpr bool kWide = wide_k(K);
  constexpr int kS = kWide ? kWideSlots : kSlotsPerBucket;   // slots per bucket
  constexpr int kQ = kWide ? 4 : kBucketQuads;                // dwordx4 per bucket
  constexpr int kH = kWide ? 1 : kBucketHalves;               // 64-byte pieces per bucket
  constexpr int kSpan = kContigTile + 3 * K;
  __shared__ uint8_t bases[kSpan];
  __shared__ uint8_t aa_p[kSpan], aa_m[kSpan];
  __shared__ uint64_t offc[kOffCache + 1];
  __shared__ uint32_t crange[2];
  constexpr int CP = kContigPos * kContigSeq;  // slices of 256 positions per block
  __shared__ uint32_t wave_tot[kWavesPerBlock * CP];
  __shared__ uint8_t codon[64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, part = t & 3;
  // offsets[0] through the constant address space: a scalar load (every block reads it, so the
  // scalar cache serves it) in place of a vector round trip before the tile's DNA load
  const uint64_t base = ((const __attribute__((address_space(4))) uint64_t*)a.offsets)[0];
  const uint64_t end = base + a.total_bases;
  const uint64_t r0 = (uint64_t)blockIdx.x * kContigTile;
  const uint32_t nb = a.n_buckets;
  KMA_CLK(0);
  // The tile's DNA bytes: every load issued before the contig search below, so that their
  // round trip overlaps the offsets' (as a strided loop of load, wait, store they took three
  // dependent trips: ~3.8 us of a ~12 us block, profiles/r04/clock_c3_r04g.json).
  constexpr int kTileIters = (kSpan + 255) / 256;
  uint8_t tb[kTileIters];
#pragma unroll
  for (int j = 0; j < kTileIters; ++j) {
    const int i = t + 256 * j;
    const uint64_t g = base + r0 + i;
    tb[j] = i < kSpan && g < end ? a.dna[g] : (uint8_t)'N';
  }
  if (wave == 3) codon[lane] = a.codon_codes[lane];  // LDS copy of the kernel-argument table
  if (a.n_contig < (uint32_t)kOffCache) {
    // Every offset fits the cache: wave 0 loads them once and finds the tile's first / last
    // contig by ballot (the largest c with offsets[c] <= g is a prefix count; offsets[0] = base).
    if (wave == 0) {
      const uint32_t n = a.n_contig;
      const uint64_t last = r0 + kContigTile < a.total_bases ? r0 + kContigTile : a.total_bases;
      const uint64_t v = a.offsets[min((uint32_t)lane, n)];
      const uint32_t lo = (uint32_t)__popcll(__ballot((uint32_t)lane < n && v <= base + r0)) - 1u;
      const uint32_t hi =
          (uint32_t)__popcll(__ballot((uint32_t)lane < n && v <= base + last - 1)) - 1u;
      offc[lane] = __shfl(v, (int)min(lo + (uint32_t)lane, n), 64);  // offsets[min(lo + i, n)]
      const uint64_t vn = __shfl(v, (int)n, 64);
      if (lane == 0) {
        offc[kOffCache] = vn;
        crange[0] = lo;
        crange[1] = hi;
      }
    }
  } else if (wave < 2) {  // wave 0: the tile's first contig (and its offsets), wave 1: its last
    const uint64_t last = r0 + kContigTile < a.total_bases ? r0 + kContigTile : a.total_bases;
    const uint32_t c = contig_of_wave(a.offsets, a.n_contig, base + (wave ? last - 1 : r0));
    if (lane == 0) crange[wave] = c;
    if (wave == 0) {  // offsets c .. c + 64 (clamped): the tile's contigs if they are <= 64
      offc[lane] = a.offsets[min(c + lane, a.n_contig)];
      if (lane == 0) offc[kOffCache] = a.offsets[min(c + kOffCache, a.n_contig)];
    }
  }
#pragma unroll
  for (int j = 0; j < kTileIters; ++j) {
    const int i = t + 256 * j;
    if (i < kSpan) bases[i] = (uint8_t)(base + r0 + i < end ? base2(tb[j]) : 4u);
  }
  __syncthreads();
  KMA_CLK(1);  // tile loaded, contigs found
  const uint32_t c_lo = crange[0], nc = crange[1] - c_lo + 1;  // contigs meeting the tile
  for (int i = t; i < kSpan - 2; i += blockDim.x) {
    const uint32_t b0 = bases[i], b1 = bases[i + 1], b2 = bases[i + 2];
    if ((b0 | b1 | b2) & 4u) {
      aa_p[i] = aa_m[i] = 0;  // 'X'
    } else {
      aa_p[i] = codon[b0 * 16 + b1 * 4 + b2];
      aa_m[i] = codon[(b2 ^ 2u) * 16 + (b1 ^ 2u) * 4 + (b0 ^ 2u)];  // complement: x ^ 2
    }
  }
  __syncthreads();
  KMA_CLK(2);  // translated

  // Each lane owns positions tp + 256 h (h < kContigPos): both windows of every one of them are
  // probed with all their dwordx4 in flight before any compare. KMA_LANE_PERM: quad q's member
  // p takes position 16 p + q of its wave, so that one load instruction covers 16 consecutive
  // positions (same-frame windows 3 apart share minimizers, hence lines); the results go back
  // to position order through LDS before the compaction.
  constexpr int CL = kContigPos;  // positions per lane held at once (per sequential slice)
#if KMA_LANE_PERM
  const uint32_t tp = (uint32_t)(wave * 64 + 16 * (lane & 3) + (lane >> 2));
#else
  const uint32_t tp = (uint32_t)t;
#endif
  // Contig, offset in it and its length of the tile's forward position tt (g < end).
  auto locate = [&](uint32_t tt, uint32_t& c, int64_t& x, int64_t& len) {
    const uint64_t g = base + r0 + tt;
    if (nc <= (uint32_t)kOffCache) {
      uint32_t lo = 0, hi = nc;  // largest i < nc with offc[i] <= g
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (offc[mid] <= g) lo = mid; else hi = mid;
      }
      c = c_lo + lo;
      x = (int64_t)(g - offc[lo]);
      len = (int64_t)(offc[lo + 1] - offc[lo]);
    } else {
      c = contig_of(a.offsets, a.n_contig, g);
      x = (int64_t)(g - a.offsets[c]);
      len = (int64_t)(a.offsets[c + 1] - a.offsets[c]);
    }
  };
  // Verdicts of every position go through LDS (fid + 1, 0 = no hit), lane t then takes position
  // t's (back to position order after KMA_LANE_PERM) for the compaction.
  __shared__ uint32_t xv[CP][2][256];
#pragma unroll 1
  for (int sq = 0; sq < kContigSeq; ++sq) {
  uint32_t contig[CL];
  uint64_t key[CL][2];
  uint32_t bk[CL][2];
  bool ok[CL][2];
#pragma unroll
  for (int h = 0; h < CL; ++h) {
    const uint32_t tt = tp + 256u * (sq * CL + h);
    const uint64_t g = base + r0 + tt;
    contig[h] = c_lo;
    int64_t x = 0, len = 0;
    if (g < end) locate(tt, contig[h], x, len);
    bool pv = g < end && x + 3 * K + 3 <= len, mv = g < end && x >= 3 && x + 3 * K <= len;
    key[h][0] = key[h][1] = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t cp = aa_p[tt + 3 * j], cm = aa_m[tt + 3 * j];
      pv = pv && cp != 0u;
      mv = mv && cm != 0u;
      key[h][0] = (key[h][0] << 5) | cp;
      key[h][1] |= (uint64_t)cm << (5 * j);
    }
    // invalid windows gather bucket 0 (one shared line; their verdicts are dropped)
    ok[h][0] = pv;
    ok[h][1] = mv;
    bk[h][0] = pv ? home_bucket(key[h][0], K, M, nb) : 0u;
    bk[h][1] = mv ? home_bucket(key[h][1], K, M, nb) : 0u;
  }
  uint4 q[CL][2][4][kH];  // every window's quad buckets: all dwordx4 in flight
  const uint4* lane_slots = reinterpret_cast<const uint4*>(a.slots) + part;
#pragma unroll
  for (int h = 0; h < CL; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint32_t b0 = quad_bcast<0>(bk[h][j]), b1 = quad_bcast<1>(bk[h][j]);
      const uint32_t b2 = quad_bcast<2>(bk[h][j]), b3 = quad_bcast<3>(bk[h][j]);
      const uint32_t bb[4] = {b0, b1, b2, b3};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint4* bp = lane_slots + (uint64_t)bb[r] * kQ;
#pragma unroll
        for (int hh = 0; hh < kH; ++hh) q[h][j][r][hh] = bp[4 * hh];
      }
    }
  KMA_CLK(3);  // bucket loads issued
#pragma unroll
  for (int h = 0; h < CL; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint32_t klo = (uint32_t)key[h][j];
      const uint32_t khi = kWide ? (uint32_t)(key[h][j] >> 32) : (uint32_t)(key[h][j] >> 32) << 24;
      const uint32_t need = filter_need<kS>(klo);
      uint32_t raw[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const uint32_t kl = rr == 0 ? quad_bcast<0>(klo) : rr == 1 ? quad_bcast<1>(klo)
                          : rr == 2 ? quad_bcast<2>(klo) : quad_bcast<3>(klo);
        const uint32_t kh = rr == 0 ? quad_bcast<0>(khi) : rr == 1 ? quad_bcast<1>(khi)
                          : rr == 2 ? quad_bcast<2>(khi) : quad_bcast<3>(khi);
        const uint32_t nd = rr == 0 ? quad_bcast<0>(need) : rr == 1 ? quad_bcast<1>(need)
                          : rr == 2 ? quad_bcast<2>(need) : quad_bcast<3>(need);
        if constexpr (kWide) raw[rr] = match_wide_raw(q[h][j][rr][0], kl, kh, nd, part);
        else raw[rr] = match_part_raw(q[h][j][rr], kl, kh, nd, part);
      }
      const uint32_t word = quad_reduce_scatter(raw, part);
      const uint32_t w = ok[h][j] ? word : 0u;
      bool hit = (w & kWordHit) != 0u;
      uint32_t fid = w & kFidMask;
      uint32_t sid = bk[h][j] * kS + ((w >> kSlotShift) & (kS - 1));
      if (ok[h][j] && w == 0u) {  // rare: home missed, every filter position set
        if constexpr (kWide)
          hit = walk_chain_wide(a.slots, nb, bk[h][j], key[h][j], fid, sid);
        else
          hit = walk_chain(a.slots, nb, bk[h][j], key[h][j], fid, sid, a.two_choice != 0);
      }
      if (a.strict_pass && hit) {  // KmerFactory.Strict: locations counted by slot id
        if (a.strict_pass == 1) atomicAdd(a.slot_count + sid, 1u);
        else hit = a.slot_count[sid] == 1u;
      }
      if (a.tally && hit && fid < a.n_fid)
        atomicAdd(a.tally + (uint64_t)contig[h] * a.n_fid + fid, 1u);
      xv[sq * CL + h][j][tp] = hit ? fid + 1u : 0u;
    }
  }  // sequential slices
  KMA_CLK(4);  // matched (chain walks done)
  __syncthreads();
  // Block-local compaction in canonical order (position, '+' before '-'): slice by slice, each
  // slice's verdicts read back from LDS twice (counts, then records) rather than kept live.
#pragma unroll 1
  for (int h = 0; h < CP; ++h) {
    const uint64_t bp = __ballot(xv[h][0][t] != 0u), bm = __ballot(xv[h][1][t] != 0u);
    if (lane == 0) wave_tot[h * kWavesPerBlock + wave] = (uint32_t)(__popcll(bp) + __popcll(bm));
  }
  __syncthreads();
  // Staged records are the final kma_hit (the emit pass only copies them): contig, left =
  // KmerPosition.calcLeft, fid, strand and frame (KmerPosition.java:50-93).
  uint32_t total = 0;
  uint4* st = reinterpret_cast<uint4*>(a.staging) + (uint64_t)blockIdx.x * (2 * kContigTile);
#pragma unroll 1
  for (int h = 0; h < CP; ++h) {
    const uint32_t v0 = xv[h][0][t], v1 = xv[h][1][t];
    const uint64_t bp = __ballot(v0 != 0u), bm = __ballot(v1 != 0u);
    uint32_t o = total + popc_below(bp) + popc_below(bm);
    for (int w = 0; w < kWavesPerBlock; ++w) {
      if (w < wave) o += wave_tot[h * kWavesPerBlock + w];
      total += wave_tot[h * kWavesPerBlock + w];
    }
    if (v0 | v1) {  // hits only at positions inside a contig (g < end)
      uint32_t c;
      int64_t x, len;
      locate(t + 256u * h, c, x, len);
      const uint32_t left = (uint32_t)(x + 1);
      if (v0) st[o++] = make_uint4(c, left, v0 - 1u, '+' | (uint32_t)(x % 3 + 1) << 8);
      if (v1) st[o] = make_uint4(c, left, v1 - 1u, '-' | (uint32_t)((len - 3 * K - x) % 3 + 1) << 8);
    }
  }
  if (t == 0) {
    a.block_counts[blockIdx.x] = total;
    // the emit pass's group sums (zeroed by the previous emit pass on this workspace)
    if (a.group_sum && total)
      __hip_atomic_fetch_add(a.group_sum + blockIdx.x / kScanGroup, (uint64_t)total,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  KMA_CLK(5);
  KMA_CLK_HW();
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

// Signature build (BuildKmerProcessor.java:137-223). One wave per protein: every window of
// ProteinKmers (i = 0..L-K, or i < L-K with end_exclusive) of an interesting peg (role >= 0) or
// a buffered protein (role -1) becomes (key, role or kBuildNeg); every other position gets key 0.
// A window with a byte the standard alphabet cannot encode raises alpha_flag (the host refuses
// the batch rather than drop a kmer the reference would keep). Keys are up to 60 bits (K <= 12).
__global__ __launch_bounds__(256) void build_windows_kernel(const uint8_t* __restrict__ residues,
                                                            const uint64_t* __restrict__ offsets,
                                                            uint32_t n_seq,
                                                            const int32_t* __restrict__ roles,
                                                            int k, int end_exclusive,
                                                            const uint8_t* __restrict__ lut_g,
                                                            uint64_t* __restrict__ keys,
                                                            uint32_t* __restrict__ tags,
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
    const uint32_t tag = role >= 0 ? (uint32_t)role : kBuildNeg;
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
        v = ok ? key : 0;
      }
      keys[p - o0] = v;
      tags[p - o0] = tag;
    }
    if (__ballot(bad) && lane == 0) atomicOr(alpha_flag, 1u);
  }
}

// RoleCounter over the (key, role) pairs sorted by key (RoleCounter.java:42-56: a kmer is good
// iff every count hit its first role; BuildKmerProcessor.java:191-208 removes kmers of buffered
// proteins). Pass 1: a run's first pair is flagged, and its index is the run id of every pair
// of the run (max-scan of head indices). Pass 2: a pair whose role differs from its run's
// first, or that comes from a buffered protein, clears the run's flag.
__global__ __launch_bounds__(256) void sig_heads_kernel(const uint64_t* __restrict__ k, uint64_t n,
                                                        uint8_t* __restrict__ flags,
                                                        uint32_t* __restrict__ head_idx) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * 256) {
    const uint64_t v = k[i];
    const bool head = v != 0 && (i == 0 || k[i - 1] != v);
    flags[i] = head ? 1 : 0;
    head_idx[i] = head ? (uint32_t)i : 0u;
  }
}

__global__ __launch_bounds__(256) void sig_clear_kernel(const uint64_t* __restrict__ k,
                                                        const uint32_t* __restrict__ tags,
                                                        const uint32_t* __restrict__ run,
                                                        uint64_t n, uint8_t* __restrict__ flags) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * 256) {
    if (k[i] == 0) continue;
    const uint32_t h = run[i], t = tags[i];
    if (t == kBuildNeg || t != tags[h]) flags[h] = 0;  // every writer stores 0
  }
}

// Exclusive prefix of block b's hit count (wave 0 of the emit block; wave-uniform result): the
// group sums of the groups before b's (kScanGroup probe blocks each, summed by the probe's
// atomics; every load issued at once: one round trip for up to 64 groups) — or, for calls of
// more than kDirectGroups groups, the exclusive group prefix contigs_group_scan_kernel left in
// place of the sums (one load) — plus the counts before b in its group.
__device__ __forceinline__ uint64_t emit_offset(const ContigArgs& a, uint32_t b) {
  const uint32_t lane = threadIdx.x & 63, g = b / kScanGroup;
  uint64_t s = 0;
  if (a.groups_scanned) {
    if (lane == 0) s = a.group_sum[g];
  } else {
    for (uint32_t i = lane; i < g; i += 64) s += a.group_sum[i];
  }
  const uint32_t c0 = g * kScanGroup + 4u * lane;  // counts are allocated in whole groups
  if (c0 < b) {
    const uint4 v = *reinterpret_cast<const uint4*>(a.block_counts + c0);
    s += (uint64_t)v.x + (c0 + 1 < b ? v.y : 0u) + (c0 + 2 < b ? v.z : 0u) +
         (c0 + 3 < b ? v.w : 0u);
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
  return s;
}

// Calls of more than kDirectGroups groups (> kDirectGroups x kScanGroup x kContigTile = 268M
// bases): one block turns the group sums into
// exclusive prefixes in place, so an emit block reads one value instead of summing every group
// before its own (which grows as blocks x groups: ~2e9 loads at 1 Gbp).
__global__ __launch_bounds__(1024) void contigs_group_scan_kernel(uint64_t* sums, uint32_t n) {
  __shared__ uint64_t part[1024];
  const uint32_t t = threadIdx.x, per = (n + 1023) / 1024;
  const uint64_t lo = (uint64_t)t * per, hi = lo + per < n ? lo + per : n;
  uint64_t s = 0;
  for (uint64_t i = lo; i < hi; ++i) s += sums[i];
  part[t] = s;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {  // inclusive Hillis-Steele scan of the parts
    const uint64_t v = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint64_t run = t ? part[t - 1] : 0u;
  for (uint64_t i = lo; i < hi; ++i) {
    const uint64_t x = sums[i];
    sums[i] = run;
    run += x;
  }
}

// Emit pass: an emit block takes kEmitSpan consecutive probe blocks; probe block b's staged
// records go to out[prefix[b] ..], those past `cap` are dropped; the last emit block publishes
// the total (the caller compares it with cap). The call leaves no state behind: every emit
// block counts itself done (one agent-scope atomic, issued once its offsets are read) and the
// block that finishes last zeroes the group sums and the counter for the next call (so calls
// on one workspace may be graph-captured and replayed). Measured alternatives for the offsets
// (c3, profiles/r03_ab/): a library two-kernel scan ~10 us; a ticket letting the probe's last
// block scan, 0.6 ms (20k atomics on one address serialize); a one-block scan kernel, ~18 us (a
// single CU's dependent round trips); a group-sum kernel between probe and emit, and one emit
// block per probe block (12.5 us for c3's 19.5k blocks of ~9 hits).
constexpr uint32_t kEmitSpan = 16;
__global__ __launch_bounds__(256) void contigs_emit_kernel(ContigArgs a, uint32_t n_blocks) {
  __shared__ uint64_t pre[kEmitSpan];
  __shared__ uint32_t cnt[kEmitSpan];
  __shared__ uint32_t last;
  const uint32_t b0 = blockIdx.x * kEmitSpan, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (wave == 0) {
    const uint32_t c = lane < kEmitSpan && b0 + lane < n_blocks ? a.block_counts[b0 + lane] : 0u;
    const uint64_t base = emit_offset(a, b0);
    uint64_t inc = c;  // inclusive scan over the span's counts (lanes < kEmitSpan)
#pragma unroll
    for (int d = 1; d < (int)kEmitSpan; d <<= 1) {
      const uint64_t v = __shfl_up(inc, d, 64);
      inc += lane >= (uint32_t)d ? v : 0u;
    }
    if (lane < kEmitSpan) {
      pre[lane] = base + inc - c;
      cnt[lane] = c;
    }
    if (blockIdx.x == gridDim.x - 1 && lane == kEmitSpan - 1) *a.n_hits = base + inc;
  }
  __syncthreads();
  // This block's reads of the group sums have returned (their values are in pre[], behind the
  // barrier), so a relaxed count suffices: the last block's zeroing cannot reach a read that
  // has already completed. (An acq_rel atomic here compiles to a whole-L2 writeback and
  // invalidate around it, buffer_wbl2 / buffer_inv, in every emit block: 18 vs ~5 us per c3
  // emit pass, profiles/r04_end/stats_c3_kernel_stats.csv.)
  if (t == 0)
    last = __hip_atomic_fetch_add(a.emit_done, 1u, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  // The span's records, flattened: thread t copies records t, t + 256, ... (kEmitU loads in
  // flight before their stores: no branch around a load, so the compiler keeps them in
  // registers and issues them back to back). Record r belongs to the last span block whose
  // first record is <= r. (A wave per probe block, a load-then-store loop per 64 records, took
  // a dependent round trip per iteration: 11.6 us per c3 emit pass, profiles/r04_final.)
  constexpr int kEmitU = 4;
  uint32_t first[kEmitSpan];  // span-local first record of each probe block
  const uint64_t p0 = pre[0];
#pragma unroll
  for (uint32_t k = 0; k < kEmitSpan; ++k) first[k] = (uint32_t)(pre[k] - p0);
  const uint32_t total = first[kEmitSpan - 1] + cnt[kEmitSpan - 1];
  const uint4* st = reinterpret_cast<const uint4*>(a.staging) + (uint64_t)b0 * (2 * kContigTile);
  uint4* out = reinterpret_cast<uint4*>(a.out);
  for (uint32_t r0 = 0; r0 < total; r0 += 256u * kEmitU) {
    uint4 v0, v1, v2, v3;
    uint32_t rr[kEmitU];
    uint64_t src[kEmitU];
#pragma unroll
    for (int u = 0; u < kEmitU; ++u) {
      const uint32_t r = r0 + 256u * u + t;
      rr[u] = r < total ? r : 0u;  // out of range: record 0 of the span (read, not stored)
      uint32_t i = 0, fi = 0;
#pragma unroll
      for (uint32_t k = 1; k < kEmitSpan; ++k)
        if (first[k] <= rr[u]) {
          i = k;
          fi = first[k];
        }
      src[u] = (uint64_t)i * (2 * kContigTile) + (rr[u] - fi);
    }
    v0 = st[src[0]];
    v1 = st[src[1]];
    v2 = st[src[2]];
    v3 = st[src[3]];
    const uint32_t r = r0 + t;
    if (r < total && p0 + r < a.cap) out[p0 + r] = v0;
    if (r + 256u < total && p0 + r + 256u < a.cap) out[p0 + r + 256u] = v1;
    if (r + 512u < total && p0 + r + 512u < a.cap) out[p0 + r + 512u] = v2;
    if (r + 768u < total && p0 + r + 768u < a.cap) out[p0 + r + 768u] = v3;
  }
  __syncthreads();
  if (last) {  // every other emit block has read its offsets: clean up for the next call
    for (uint32_t i = t; i < a.n_groups; i += 256) a.group_sum[i] = 0;
    if (t == 0) *a.emit_done = 0;
  }
}

// ---------------------------------------------------------------------------------------------
// Residue packing (ASCII -> the packed stream of kma_device.h): a thread turns 64 residues of
// the call (from d_residues + offsets[0]) into 5 stream words (320 bits), codes through the
// table's LUT (0 for a byte without a code). Aligned 8-byte loads around the residues, one
// funnel shift per word; the last, partial group by bytes. Reads 1 B and writes 0.625 B per
// residue: ~0.1 ms for c5's 310M residues.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void pack64(const uint8_t (&lut)[256], const uint8_t (&b)[64],
                                       uint64_t* __restrict__ out) {
  uint64_t w[5] = {0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const uint64_t c = lut[b[i]];
    const int k = (5 * i) >> 6, o = (5 * i) & 63;  // MSB-first bit o of stream word k
    if (o <= 59) {
      w[k] |= c << (59 - o);
    } else {
      w[k] |= c >> (o - 59);
      w[k + 1] |= c << (123 - o);
    }
  }
#pragma unroll
  for (int k = 0; k < 5; ++k) out[k] = bswap64(w[k]);  // stream bytes in memory order
}

__global__ __launch_bounds__(256) void pack_residues_kernel(const uint8_t* __restrict__ residues,
                                                            const uint64_t* __restrict__ offsets,
                                                            uint64_t n, const uint8_t* lut_g,
                                                            uint64_t* __restrict__ out) {
  __shared__ uint8_t lut[256];
  lut[threadIdx.x] = lut_g[threadIdx.x];
  __syncthreads();
  const uint8_t* base = residues + offsets[0];
  const uint32_t mis = (uint32_t)((uintptr_t)base & 7u);
  const uint64_t* aligned = reinterpret_cast<const uint64_t*>(base - mis);
  const uint64_t groups = (n + 63) / 64;
  for (uint64_t g = blockIdx.x * 256ull + threadIdx.x; g < groups; g += gridDim.x * 256ull) {
    uint8_t b[64];
    if (64 * g + 64 <= n) {  // whole group: 9 aligned words (the batch is readable past its end)
      uint64_t v[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) v[k] = aligned[8 * g + k];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint64_t x = funnel(v[k], v[k + 1], mis * 8u);
#pragma unroll
        for (int j = 0; j < 8; ++j) b[8 * k + j] = (uint8_t)(x >> (8 * j));
      }
    } else {
#pragma unroll
      for (int i = 0; i < 64; ++i) b[i] = 64 * g + i < n ? base[64 * g + i] : 0u;
    }
    pack64(lut, b, out + 5 * g);
  }
  if (blockIdx.x == 0 && threadIdx.x < 2) out[5 * groups + threadIdx.x] = 0;  // read padding
}

}  // namespace

// ---- launchers ----------------------------------------------------------------------------------
hipError_t launch_pack_residues(const uint8_t* residues, const uint64_t* offsets, uint64_t n,
                                const uint8_t* lut, uint8_t* out, hipStream_t stream) {
  const uint64_t groups = (n + 63) / 64;
  const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(4096, (groups + 255) / 256));
  hipLaunchKernelGGL(pack_residues_kernel, dim3(g), dim3(256), 0, stream, residues, offsets, n,
                     lut, reinterpret_cast<uint64_t*>(out));
  return hipGetLastError();
}

static unsigned grid_for(uint64_t n, unsigned cap = 8192) {
  uint64_t g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > cap ? cap : g));
}

hipError_t launch_build_insert(uint64_t* slots, uint32_t* winner, uint32_t n_buckets, int k,
                               int m, const uint64_t* keys, uint64_t n, uint32_t* status,
                               hipStream_t stream) {
  if (wide_k(k))
    hipLaunchKernelGGL(build_insert_kernel<true>, dim3(grid_for(n)), dim3(256), 0, stream, slots,
                       winner, n_buckets, k, m, keys, n, status);
  else
    hipLaunchKernelGGL(build_insert_kernel<false>, dim3(grid_for(n)), dim3(256), 0, stream, slots,
                       winner, n_buckets, k, m, keys, n, status);
  return hipGetLastError();
}

hipError_t launch_build_finalize(uint64_t* slots, const uint32_t* winner, const uint32_t* fids,
                                 uint32_t n_buckets, int k, int m, uint32_t* stats,
                                 hipStream_t stream) {
  const dim3 g(grid_for((uint64_t)n_buckets * slots_for_k(k)));
  if (wide_k(k))
    hipLaunchKernelGGL(build_finalize_kernel<true>, g, dim3(256), 0, stream, slots, winner, fids,
                       n_buckets, k, m, stats);
  else
    hipLaunchKernelGGL(build_finalize_kernel<false>, g, dim3(256), 0, stream, slots, winner, fids,
                       n_buckets, k, m, stats);
  return hipGetLastError();
}

#ifndef KMA_TC_SELECT
#define KMA_TC_SELECT 1
#endif
hipError_t launch_build_two_choice(uint64_t* slots, uint32_t n_buckets, int k, int m,
                                   const uint64_t* keys, const uint32_t* fids, uint64_t n,
                                   uint64_t* sorted_keys, uint32_t* rows, uint32_t* sorted_rows,
                                   const TwoChoiceScratch& x, void* temp, size_t* temp_bytes,
                                   uint32_t* status, hipStream_t stream) {
  if (wide_k(k) || n_buckets < 2) return hipErrorInvalidValue;
  // all 64 bits: a row whose key is not a K-mer key (bits above 5K) must not split a run
  if (!temp) {
    size_t t1 = 0, t2 = 0;
    hipError_t e = rocprim::radix_sort_pairs(nullptr, t1, keys, sorted_keys, rows, sorted_rows,
                                             (size_t)n, 0u, 64u, stream);
    if (e != hipSuccess) return e;
    e = rocprim::radix_sort_pairs(nullptr, t2, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)n, 0u, 32u,
                                  stream);
    *temp_bytes = KMA_TC_SELECT ? std::max(t1, t2) : t1;
    return e;
  }
  hipLaunchKernelGGL(iota_kernel, dim3(grid_for(n)), dim3(256), 0, stream, rows, n);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = rocprim::radix_sort_pairs(temp, *temp_bytes, keys, sorted_keys, rows, sorted_rows, (size_t)n,
                                0u, 64u, stream);
  if (e != hipSuccess) return e;
  if (KMA_TC_SELECT && x.home) {
    hipLaunchKernelGGL(build_two_choice_home_kernel, dim3(grid_for(n)), dim3(256), 0, stream,
                       sorted_keys, n, k, m, n_buckets, x.home, rows);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    e = rocprim::radix_sort_pairs(temp, *temp_bytes, x.home, x.sorted_home, rows, x.sorted_idx,
                                  (size_t)n, 0u, 32u, stream);
    if (e != hipSuccess) return e;
    if (x.load) {
      if ((e = hipMemsetAsync(x.load, 0, n_buckets, stream)) != hipSuccess) return e;
      hipLaunchKernelGGL(build_two_choice_load_kernel, dim3(grid_for(n)), dim3(256), 0, stream,
                         x.sorted_home, n, x.load);
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(build_two_choice_select_kernel, dim3(grid_for(n)), dim3(256), 0, stream,
                       x.sorted_home, x.sorted_idx, sorted_keys, n, x.load, n_buckets, x.away);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  const uint8_t* away = KMA_TC_SELECT ? x.away : nullptr;
  for (uint8_t phase = 0; phase < (away ? 2 : 1); ++phase) {
    hipLaunchKernelGGL(build_two_choice_insert_kernel, dim3(grid_for(n)), dim3(256), 0, stream,
                       slots, n_buckets, k, m, sorted_keys, sorted_rows, fids, n, away, phase,
                       status);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(build_two_choice_filter_kernel, dim3(grid_for((uint64_t)n_buckets * kSlotsPerBucket)),
                     dim3(256), 0, stream, slots, n_buckets, k, m, status + 1);
  return hipGetLastError();
}

// The kernel's protein capacity P (its compare chains, protein records and SGPRs scale with
// it): K = 8 kernels come in P = 4 / 6 / 8 and take the smallest that holds the call's block
// proteins (the defaults: 6 at c5, 4 at c2 / c4); other K use P = kBlockProteins.
template <int K, int M, int P>
hipError_t launch_annotate_p(const ProteinArgs& a, dim3 grid, hipStream_t stream) {
  if (a.packed)
    hipLaunchKernelGGL((annotate_kernel<K, M, P, true>), grid, dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL((annotate_kernel<K, M, P, false>), grid, dim3(256), 0, stream, a);
  return hipGetLastError();
}
template <int K, int M>
struct AnnotateLaunch {
  static hipError_t run(const ProteinArgs& a, hipStream_t stream) {
    if constexpr (wide_k(K)) {  // the protein path packs windows of <= 8 residues (one u64)
      return hipErrorInvalidValue;
    } else {
    constexpr int P = kBlockProteins;
    const unsigned bp = a.block_proteins >= 1 && a.block_proteins <= (uint32_t)P ? a.block_proteins : 4u;
    if (bp != a.block_proteins) return hipErrorInvalidValue;
    const unsigned blocks = (a.n_seq + bp - 1) / bp;
    if (a.n_groups != blocks) return hipErrorInvalidValue;
    const dim3 grid(a.defer_below ? 2 * blocks : blocks);
    if constexpr (K == 8 && P > 6) {
      if (bp <= 4) return launch_annotate_p<K, M, 4>(a, grid, stream);
      if (bp <= 6) return launch_annotate_p<K, M, 6>(a, grid, stream);
    }
    return launch_annotate_p<K, M, P>(a, grid, stream);
    }
  }
};

hipError_t launch_annotate(const ProteinArgs& a, hipStream_t stream) {
  if (a.n_seq == 0) return hipSuccess;
  return dispatch_km<AnnotateLaunch>(a.k, a.mlen, a, stream);
}

template <int K, int M>
struct ContigLaunch {
  static hipError_t run(const ContigArgs& a, uint64_t n_blocks, hipStream_t stream) {
    hipLaunchKernelGGL((contigs_probe_quad_kernel<K, M>), dim3((unsigned)n_blocks), dim3(256), 0,
                       stream, a);
    return hipGetLastError();
  }
};

hipError_t launch_contigs_probe(const ContigArgs& a, uint64_t n_blocks, hipStream_t stream) {
  return dispatch_km<ContigLaunch>(a.k, a.mlen, a, n_blocks, stream);
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
  return rocprim::radix_sort_pairs(temp, *temp_bytes, keys_in, keys_out, vals_in, vals_out,
                                   (size_t)n, 0u, (unsigned)key_bits, stream);
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
  // Keys and values: two passes over the same flags keep the order identical.
  size_t need = 0;
  hipError_t e = rocprim::select(nullptr, need, keys_in, flags, keys_out, n_out, (size_t)n,
                                 stream);
  if (e != hipSuccess) return e;
  size_t need2 = 0;
  e = rocprim::select(nullptr, need2, vals_in, flags, vals_out, n_out, (size_t)n, stream);
  if (e != hipSuccess) return e;
  need = std::max(need, need2);
  if (!temp) {
    *temp_bytes = need;
    return hipSuccess;
  }
  e = rocprim::select(temp, need, keys_in, flags, keys_out, n_out, (size_t)n, stream);
  if (e != hipSuccess) return e;
  return rocprim::select(temp, need, vals_in, flags, vals_out, n_out, (size_t)n, stream);
}

hipError_t launch_build_windows(const uint8_t* residues, const uint64_t* offsets, uint32_t n_seq,
                                const int32_t* roles, int k, int end_exclusive, const uint8_t* lut,
                                uint64_t* keys, uint32_t* tags, uint32_t* alpha_flag,
                                hipStream_t stream) {
  const unsigned g = (unsigned)std::min<uint64_t>(8192, ((uint64_t)n_seq + 3) / 4);
  hipLaunchKernelGGL(build_windows_kernel, dim3(g ? g : 1), dim3(256), 0, stream, residues,
                     offsets, n_seq, roles, k, end_exclusive, lut, keys, tags, alpha_flag);
  return hipGetLastError();
}

hipError_t launch_signature_flags(const uint64_t* keys, const uint32_t* tags, uint64_t n,
                                  uint8_t* flags, uint32_t* head_idx, uint32_t* run, void* temp,
                                  size_t* temp_bytes, hipStream_t stream) {
  if (!temp)
    return rocprim::inclusive_scan(nullptr, *temp_bytes, head_idx, run, (size_t)n,
                                   rocprim::maximum<uint32_t>(), stream);
  hipLaunchKernelGGL(sig_heads_kernel, dim3(grid_for(n)), dim3(256), 0, stream, keys, n, flags,
                     head_idx);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = rocprim::inclusive_scan(temp, *temp_bytes, head_idx, run, (size_t)n,
                              rocprim::maximum<uint32_t>(), stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(sig_clear_kernel, dim3(grid_for(n)), dim3(256), 0, stream, keys, tags, run,
                     n, flags);
  return hipGetLastError();
}

hipError_t launch_contigs_emit(const ContigArgs& a, uint64_t n_blocks, hipStream_t stream) {
  ContigArgs e = a;
  e.n_groups = (uint32_t)((n_blocks + kScanGroup - 1) / kScanGroup);
  e.groups_scanned = e.n_groups > kDirectGroups;
  if (e.groups_scanned) {
    hipLaunchKernelGGL(contigs_group_scan_kernel, dim3(1), dim3(1024), 0, stream, e.group_sum,
                       e.n_groups);
    if (hipError_t err = hipGetLastError()) return err;
  }
  const unsigned g = (unsigned)((n_blocks + kEmitSpan - 1) / kEmitSpan);
  hipLaunchKernelGGL(contigs_emit_kernel, dim3(g), dim3(256), 0, stream, e, (uint32_t)n_blocks);
  return hipGetLastError();
}

}  // namespace kma
