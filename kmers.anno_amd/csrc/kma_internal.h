// kma_internal.h — shared between the HIP kernels (kma_kernels.hip) and the C-ABI layer
// (kma_abi.cpp). Not part of the public ABI (see include/kmeranno.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kmeranno.h"

namespace kma {

// ---- signature-table layout in HBM ------------------------------------------------------------
// n_buckets x 64-byte buckets (n_buckets < 2^29); each bucket = 8 slots of one u64:
//   low dword  = key bits 0..31            (never 0 for a valid key: codes are 1..31)
//   high dword = key bits 32..39 << 24 | overflow bit << 23 | fid (23 bits)
// A slot whose low dword is 0 is empty. A key lives in its home bucket or, if that was full,
// in the next buckets (linear bucket probing, wrapping). The 8 overflow bits of a bucket (one
// per slot, independent of the slot's key) form a filter of the keys homed there that live
// further down the chain: overflow bit ovf_index(key) of the home bucket is set for each. A
// lookup that misses its home bucket walks the chain only if its bit is set (then it stops at
// the key or at a bucket with an empty slot), so a miss costs one 64-byte request except for
// ~1% of keys. Every compare is a 32-bit operation.
constexpr int kSlotsPerBucket = 8;
constexpr uint32_t kFidMask = (1u << 23) - 1;
constexpr uint32_t kOvfBit = 1u << 23;         // in the high dword
constexpr uint32_t kKeyHiMask = 0xFF000000u;   // key bits 32..39 in the high dword
// K1's per-window verdict while probing: fid + 1 in bits 0..23, slot in bucket at kSlotShift.
constexpr uint32_t kWordFid = (1u << 24) - 1;
constexpr uint32_t kSlotShift = 24;

__host__ __device__ inline uint64_t slot_make(uint64_t key, uint32_t fid) {
  return ((uint64_t)((uint32_t)(key >> 32) << 24 | (fid & kFidMask)) << 32) | (uint32_t)key;
}
// Which slot of the home bucket carries the key's overflow bit (from the key's low dword).
__host__ __device__ inline uint32_t ovf_index(uint32_t klo) { return (klo * 0x9E3779B1u) >> 29; }
__host__ __device__ inline uint64_t slot_key(uint64_t slot) {
  return ((uint64_t)(uint32_t)(slot >> 56) << 32) | (uint32_t)slot;
}

__host__ __device__ inline uint32_t mix32(uint32_t h) {  // murmur3 fmix32
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// Minimizer of a packed K-mer: the smallest hash over its K - m + 1 m-mers (5-bit residue
// codes, first residue most significant). m is a table property (minimizer_len below).
__host__ __device__ inline uint32_t minimizer_hash(uint64_t key, int k, int m) {
  const uint32_t mask = (uint32_t)((1ull << (5 * m)) - 1);
  uint32_t best = 0xFFFFFFFFu;
  for (int p = 0; p <= k - m; ++p) {
    const uint32_t sub = (uint32_t)(key >> (5 * (k - m - p))) & mask;
    const uint32_t h = mix32(sub * 0x9E3779B1u + 0x7F4A7C15u);
    best = best < h ? best : h;
  }
  return best;
}

// Home bucket = the key's MINIMIZER hashed onto [0, n_buckets) (Lemire fast range). Two
// consecutive windows of a protein share their minimizer with probability 2/(K - m + 2)
// (1/2 for K = 8, m = 6; 1/3 for m = 7), so they share their home bucket and one 64-byte
// request serves both: the probe kernel walks runs of consecutive windows and requests a bucket
// only when it changes. Exactness is kept by the full-key compare.
__host__ __device__ inline uint32_t home_bucket(uint64_t key, int k, int m, uint32_t n_buckets) {
#ifdef KMA_HOME_FLAT  // A/B build only: hash of the whole key
  const uint32_t h = mix32((uint32_t)key ^ mix32((uint32_t)(key >> 32) + 0x9E3779B9u));
  (void)k, (void)m;
#else
  const uint32_t h = mix32(minimizer_hash(key, k, m) ^ 0x85EBCA77u);
#endif
  return (uint32_t)(((uint64_t)h * n_buckets) >> 32);
}

// Minimizer length of a table of n_buckets buckets for K-mers. Keys sharing a minimizer share
// a bucket, so the m-mer space must stay large against the table: with 20 amino acids, m = 6
// gives 6.4e7 m-mers and overflows ~12% of keys past their home bucket at 1e8 keys, m = 7
// keeps that at ~2.6% (and still shares a bucket between consecutive windows 1/3 of the time).
// So m = 6 up to 2^22 buckets (16.8M keys at load factor 0.5), else 7 (m <= K). The table
// layout depends on it; build and lookup both derive it from (K, n_buckets). Defined in
// kma_abi.cpp (KMA_MINIMIZER=6|7 overrides it, for layout experiments only).
int minimizer_len(int k, uint64_t n_buckets);

// ---- kernel parameter blocks ------------------------------------------------------------------
// A protein K2 leaves to vote_long_kernel: one role (fid), hits H >= 2, its window range.
struct PendingRec {
  uint32_t s, fid, hits, n_win;
  uint64_t base;  // word index of window 0 (residue offsets[0] + base)
};

struct ProteinArgs {
  const uint64_t* slots;
  uint32_t n_buckets;
  const uint8_t* lut;  // 256-byte residue -> 5-bit code table (device)
  const uint8_t* residues;
  const uint64_t* offsets;
  uint32_t n_seq;
  uint64_t n_residues;  // offsets[n_seq] - offsets[0]
  int32_t k;
  int32_t mlen;  // minimizer length of the table
  int32_t min_hits;
  uint32_t flags;
  int32_t* out_fid;
  int32_t* out_count;
  uint8_t* out_status;
  uint32_t* tally;  // may be null
  uint32_t n_fid;
  uint32_t* hits;           // workspace: fid + 1 (0 = miss) per residue position
  uint32_t* sids;           // workspace: slot id of the hit (the key's identity in the table)
  uint32_t* overflow_flag;  // workspace: lengths of the two `pending` lists (K1 zeroes them)
  struct PendingRec* pending;  // workspace: proteins left to vote_long_kernel (two lists)
  uint32_t pending_half;       // start of the second list
  uint64_t* scratch;        // workspace: kFallbackBlocks x kFallbackCap u64
  uint32_t seq_lo, seq_hi;  // the segment [seq_lo, seq_hi) of proteins this launch covers
  uint32_t reset_flag;      // K1 of the first segment clears overflow_flag
};

// K1 probe kernel: kProbeWin windows per lane per step, all first-bucket loads in flight
// (3: 70 VGPRs, 7 waves/SIMD; 4 needs 125 VGPRs and measured 9% slower at c5). The grid is
// the resident population (hipOccupancy...); kProbeBlocksPerCU is only the fallback.
#ifndef KMA_PROBE_WIN
#define KMA_PROBE_WIN 3
#endif
#ifndef KMA_PROBE_BPC
#define KMA_PROBE_BPC 8
#endif
constexpr int kProbeWin = KMA_PROBE_WIN;
constexpr int kProbeBlocksPerCU = KMA_PROBE_BPC;
// K1 defers overflow-chain walks to a per-wave LDS queue of kChainQ positions, resolved a
// wave's 64 lanes at a time.
constexpr int kChainQ = 384;
// K2 vote kernel: kVoteWaves waves per block share the kChunk-window chunks of kVoteProteins
// proteins (kVoteWin consecutive windows per lane per chunk; a wave's first kVoteHold chunks
// stay in registers between the passes) and an LDS pool of kVotePool u32 set entries.
// Proteins whose set does not fit are finished by vote_long_kernel: one block each, an LDS set
// of kLongSet keys, else kFallbackCap keys of workspace scratch per block.
// (The KMA_VOTE_* macros exist for tuning builds: `make variant`.)
#ifndef KMA_VOTE_WAVES
#define KMA_VOTE_WAVES 4
#endif
#ifndef KMA_VOTE_PROTEINS
#define KMA_VOTE_PROTEINS 8
#endif
#ifndef KMA_VOTE_POOL
#define KMA_VOTE_POOL 4096
#endif
#ifndef KMA_VOTE_HOLD
#define KMA_VOTE_HOLD 2
#endif
constexpr int kWavesPerBlock = 4;
constexpr int kVoteWin = 4;
constexpr int kChunk = 64 * kVoteWin;
constexpr int kVoteWaves = KMA_VOTE_WAVES;
constexpr int kVoteProteins = KMA_VOTE_PROTEINS;
constexpr int kVotePool = KMA_VOTE_POOL;
constexpr int kVoteHold = KMA_VOTE_HOLD;
constexpr int kLongSet = 8192;
constexpr int kLongHold = 4;  // vote_long_kernel: chunks of a protein in flight per wave
constexpr int kLongWaveSet = kLongSet * 2 / 4;  // u32 slot ids per wave in vote_long_kernel
// K2 wave form: one protein per wave, kWaveHold chunks in flight, an LDS set slice of kWaveSet
// u32 slot ids per wave (4 waves per block), filled to at most 3/4.
#ifndef KMA_WAVE_HOLD
#define KMA_WAVE_HOLD 4
#endif
#ifndef KMA_WAVE_SET
#define KMA_WAVE_SET 1024
#endif
constexpr int kWaveHold = KMA_WAVE_HOLD;
constexpr int kWaveSet = KMA_WAVE_SET;
constexpr uint32_t kDeferred = 1u << 31;  // K2: set taken from the whole pool in phase 3
constexpr uint32_t kLongCap = 0xFFFFFFFFu;  // K2: set too large for the pool (vote_long_kernel)
constexpr int kLongBlocksPerCU = 4;
constexpr int kFallbackBlocks = 64;
constexpr uint32_t kFallbackCap = 1u << 17;  // u64 entries per block (1 MiB)

struct ContigArgs {
  const uint64_t* slots;
  uint32_t n_buckets;
  const uint8_t* dna;          // contig s is dna[offsets[s] .. offsets[s+1])
  const uint64_t* offsets;     // n_contig + 1 (device); offsets[0] need not be 0
  uint32_t n_contig;
  uint64_t total_bases;        // offsets[n_contig] - offsets[0] (< 2^39)
  int32_t k;
  int32_t mlen;
  uint64_t* staging;           // n_blocks x kContigTile*2 packed hits (relative position)
  uint32_t* block_counts;      // n_blocks
  const uint64_t* prefix;      // n_blocks: exclusive scan of block_counts (emit pass)
  uint32_t* tally;             // may be null: n_contig x n_fid
  uint32_t n_fid;
  kma_hit* out;                // emit pass: hits [0, cap) in canonical order
  uint64_t cap;
  uint64_t* n_hits;            // emit pass: total hits (also when > cap)
  // KmerFactory.Strict (peg join): pass 1 counts the locations of every table key
  // (strict_pass = 1: atomicAdd per hit into slot_count[slot id], nothing else is meaningful),
  // pass 2 keeps only hits whose key has exactly one location (strict_pass = 2).
  uint32_t* slot_count;        // n_buckets * 8, zeroed before pass 1
  int32_t strict_pass;         // 0 = off
  uint8_t codon_codes[64];     // by value (TCAG order): 5-bit aa code, 0 = stop
};
constexpr int kContigTile = 256;  // forward positions per block

// ---- launchers (kma_kernels.hip) --------------------------------------------------------------
hipError_t launch_build_insert(uint64_t* slots, uint32_t* winner, uint32_t n_buckets, int k,
                               int m, const uint64_t* keys, uint64_t n, uint32_t* status,
                               hipStream_t stream);
hipError_t launch_build_finalize(uint64_t* slots, const uint32_t* winner, const uint32_t* fids,
                                 uint32_t n_buckets, int k, int m, uint32_t* stats,
                                 hipStream_t stream);
hipError_t launch_probe(const ProteinArgs& a, int n_cu, hipStream_t stream);  // K1
hipError_t launch_vote(const ProteinArgs& a, int n_cu, hipStream_t stream);   // K2 (segment)
hipError_t launch_long(const ProteinArgs& a, int n_cu, hipStream_t stream);   // long proteins
hipError_t launch_fused(const ProteinArgs& a, int n_cu, hipStream_t stream);  // K12 = K1 + K2
uint32_t fused_min_proteins(int n_cu);  // K12 is used for batches of at least this many proteins
hipError_t launch_contigs_emit(const ContigArgs& a, uint64_t n_blocks, hipStream_t stream);
hipError_t launch_contig_scan(const uint32_t* counts, uint64_t* prefix, uint64_t n,
                              void* temp, size_t* temp_bytes, hipStream_t stream);
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
// Signature build (BuildKmerProcessor): composite = key << 24 | role (0xFFFFFF = buffered
// protein) per window of ProteinKmers; sort; unique; keep keys with one role and no buffered
// occurrence.
constexpr uint32_t kBuildNeg = 0xFFFFFFu;
hipError_t launch_build_windows(const uint8_t* residues, const uint64_t* offsets, uint32_t n_seq,
                                const int32_t* roles, int k, int end_exclusive, const uint8_t* lut,
                                uint64_t* out, uint32_t* alpha_flag, hipStream_t stream);
hipError_t launch_sort_keys(void* temp, size_t* temp_bytes, const uint64_t* in, uint64_t* out,
                            uint64_t n, int bits, hipStream_t stream);
hipError_t launch_unique(void* temp, size_t* temp_bytes, const uint64_t* in, uint64_t* out,
                         uint64_t* n_out, uint64_t n, hipStream_t stream);
hipError_t launch_signature_flags(const uint64_t* uniq, const uint64_t* n_uniq, uint64_t n_max,
                                  uint8_t* flags, hipStream_t stream);
hipError_t launch_select_flagged_keys(void* temp, size_t* temp_bytes, const uint64_t* in,
                                      const uint8_t* flags, uint64_t* out, uint64_t* n_out,
                                      uint64_t n, hipStream_t stream);
hipError_t launch_select_flagged(void* temp, size_t* temp_bytes, const uint64_t* keys_in,
                                 const uint32_t* vals_in, const uint8_t* flags, uint64_t* keys_out,
                                 uint32_t* vals_out, uint64_t* n_out, uint64_t n,
                                 hipStream_t stream);

}  // namespace kma
