// kma_hashanno.h — launchers of the hash annotator's scoring kernels (kma_hashanno.hip), used by
// kma_abi.cpp. Not part of the public ABI (see include/kmeranno.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kma {

struct HashArgs {
  // prototypes: positions of the segment-sorted window keys
  uint64_t n_ppos;
  const uint8_t* pfirst;      // first occurrence of a distinct key
  const uint64_t* psorted;
  const uint32_t* powner;     // prototype of the position
  const uint32_t* psize;      // distinct kmers per prototype
  // genome: unique distinct keys with the proteins holding them
  const uint64_t* ukeys;
  const uint64_t* n_u;        // device count of ukeys
  const uint32_t* ustart;     // n_u + 1 range starts into gprot
  const uint32_t* gprot;      // proteins, sorted by key
  const uint32_t* gsize;      // distinct kmers per genome protein
  // candidates
  uint32_t* ccount;
  uint32_t* cu;
  const uint64_t* coff;
  uint64_t* cand;             // prototype << 32 | protein (the slice's, from cand_base)
  uint64_t pos_lo, pos_hi;    // the slice: prototype positions [pos_lo, pos_hi)
  uint64_t cand_base;         // coff[pos_lo]
  const uint64_t* runs;       // run-length encoded candidates
  const uint32_t* run_len;
  const uint64_t* n_runs;     // device
  // scoring
  double min_sim;
  uint32_t* out_count;        // per prototype: proteins with sim >= min_sim
  uint64_t* best_bits;        // per protein: best similarity of the slice (double bits), 0 = none
  uint32_t* best_proto;       // per protein: smallest prototype of the slice at that similarity
};

hipError_t launch_owner_first(const uint64_t* sorted, const uint64_t* off, uint32_t n,
                              uint32_t* owner, uint8_t* first, hipStream_t s);
hipError_t launch_run_heads(const uint64_t* k, uint64_t n, uint8_t* head, uint32_t* idx,
                            hipStream_t s);
hipError_t launch_set_end(uint32_t* ustart, const uint64_t* n_u, uint64_t n_pairs, hipStream_t s);
hipError_t launch_cand_count(const HashArgs& a, hipStream_t s);
hipError_t launch_cand_emit(const HashArgs& a, hipStream_t s);
hipError_t launch_score(const HashArgs& a, uint64_t n_max, hipStream_t s);
// cum[p] = candidates of prototypes before p (p <= n_proto; off: prototype position offsets).
hipError_t launch_proto_cum(const uint64_t* coff, const uint32_t* ccount, const uint64_t* off,
                            uint32_t n_proto, uint64_t n_pos, uint64_t* cum, hipStream_t s);
// Slices of prototypes in file order: a slice's best replaces the running one only when strictly
// higher (earlier prototypes win ties); the slice buffers are reset for the next slice.
hipError_t launch_merge_best(uint64_t* best_bits, uint32_t* best_proto, uint64_t* slice_bits,
                             uint32_t* slice_proto, uint32_t n, hipStream_t s);
hipError_t launch_choose(const HashArgs& a, uint64_t n_max, hipStream_t s);
hipError_t prim_select_flagged_u64(void* temp, size_t* tb, const uint64_t* in, const uint8_t* f,
                                  uint64_t* out, uint64_t* n_out, uint64_t n, hipStream_t s);
hipError_t prim_select_flagged_u32(void* temp, size_t* tb, const uint32_t* in, const uint8_t* f,
                                  uint32_t* out, uint64_t* n_out, uint64_t n, hipStream_t s);
hipError_t prim_sort_pairs_u64_u32(void* temp, size_t* tb, const uint64_t* ki, uint64_t* ko,
                                  const uint32_t* vi, uint32_t* vo, uint64_t n, int bits,
                                  hipStream_t s);
hipError_t prim_sort_keys_u64(void* temp, size_t* tb, const uint64_t* ki, uint64_t* ko, uint64_t n,
                             int bits, hipStream_t s);
hipError_t prim_excl_sum_u32_u64(void* temp, size_t* tb, const uint32_t* in, uint64_t* out,
                                uint64_t n, hipStream_t s);
hipError_t prim_rle_u64(void* temp, size_t* tb, const uint64_t* in, uint64_t* uniq, uint32_t* len,
                       uint64_t* n_runs, uint64_t n, hipStream_t s);

}  // namespace kma
