// kma_pack.h — host packing of ASCII residues into the protein kernel's packed stream
// (kma_pack.cpp; layout in kma_device.h). Internal; not part of the ABI.
#pragma once

#include <stdint.h>

namespace kma {
// Residues in[0, n) through the table's LUT into `out` (stream bytes 0 .. ceil(5n / 8)); the rest
// of out[0, out_cap) is zeroed. A byte without a code packs as 0 (its windows never match).
// `in` is read only in [0, n).
void pack_residues_host(const uint8_t lut[256], const uint8_t* in, uint64_t n, uint8_t* out,
                        uint64_t out_cap);
}  // namespace kma
