// kma_internal.h — shared between the HIP kernels (kma_kernels.hip) and the C-ABI layer
// (kma_abi.cpp). Not part of the public ABI (see include/kmeranno.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kma {

// ---- signature-table layout in HBM ------------------------------------------------------------
// n_buckets x 64-byte buckets; each bucket = 8 slots of u64 (key << 24 | fid); slot 0 = empty.
// A key lives in its home bucket or, if that is full, in the next buckets (linear bucket probing,
// wrapping). Lookups stop at the first bucket holding the key or an empty slot.
constexpr int kSlotsPerBucket = 8;
constexpr int kFidBits = 24;
constexpr uint64_t kFidMask = (1ull << kFidBits) - 1;

__host__ __device__ inline uint64_t mix64(uint64_t k) {  // murmur3 fmix64 finaliser
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

__host__ __device__ inline uint64_t home_bucket(uint64_t key, uint64_t n_buckets) {
  // Lemire fast range: high 64 bits of mix(key) * n_buckets, any n_buckets (no power of two).
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(mix64(key), n_buckets);
#else
  return (uint64_t)(((unsigned __int128)mix64(key) * n_buckets) >> 64);
#endif
}

// ---- kernel parameter blocks ------------------------------------------------------------------
struct ProteinArgs {
  const uint64_t* slots;
  uint64_t n_buckets;
  const uint8_t* lut;  // 256-byte residue -> 5-bit code table (device)
  const uint8_t* residues;
  const uint64_t* offsets;
  uint32_t n_seq;
  int32_t k;
  int32_t min_hits;
  uint32_t flags;
  int32_t* out_fid;
  int32_t* out_count;
  uint8_t* out_status;
  uint32_t* tally;  // may be null
  uint32_t n_fid;
  uint32_t* overflow_flag;  // workspace: set when a protein needs the global dedupe pass
  uint32_t* scratch;        // workspace: kFallbackBlocks x kFallbackCap u32
};

// Per-wave LDS dedupe set of hit slot ids (u32, 0 = empty): capacity and the distinct-hit
// count at which a protein is deferred to the global-memory pass.
constexpr int kWavesPerBlock = 4;
constexpr int kSetCap = 2048;
constexpr int kSetLimit = 1536;
constexpr uint8_t kStatusPending = 0xFF;
// Global-memory dedupe pass for proteins with more than kSetLimit distinct hits.
constexpr int kFallbackBlocks = 64;
constexpr uint32_t kFallbackCap = 1u << 18;  // u32 entries per block (1 MiB)

struct ContigArgs {
  const uint64_t* slots;
  uint64_t n_buckets;
  const uint8_t* dna;
  const uint64_t* offsets;
  uint32_t n_contig;
  uint64_t total_bases;
  int32_t k;
  const uint8_t* codon_codes;  // 64 entries (TCAG order): 5-bit aa code, 0 = stop
  uint64_t* staging;           // n_blocks x kContigTile*2 packed hits
  uint32_t* block_counts;      // n_blocks
  uint32_t* tally;             // may be null: n_contig x n_fid
  uint32_t n_fid;
};
constexpr int kContigTile = 256;  // forward positions per block

// ---- launchers (kma_kernels.hip) --------------------------------------------------------------
hipError_t launch_build_insert(uint64_t* slots, uint32_t* winner, uint64_t n_buckets,
                               const uint64_t* keys, uint64_t n, uint32_t* status,
                               hipStream_t stream);
hipError_t launch_build_finalize(uint64_t* slots, const uint32_t* winner, const uint32_t* fids,
                                 uint64_t n_buckets, uint32_t* stats, hipStream_t stream);
hipError_t launch_proteins(const ProteinArgs& a, hipStream_t stream);
hipError_t launch_contigs(const ContigArgs& a, uint64_t n_blocks, const uint64_t* d_prefix,
                          uint8_t* out_hits, hipStream_t stream);
hipError_t launch_contig_scan(const uint32_t* counts, uint64_t* prefix, uint64_t n,
                              void* temp, size_t* temp_bytes, hipStream_t stream);
hipError_t launch_contigs_probe(const ContigArgs& a, uint64_t n_blocks, hipStream_t stream);

}  // namespace kma
