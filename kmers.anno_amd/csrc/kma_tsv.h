// kma_tsv.h — the library's native reader of apply's signature table file (kma_tsv.cpp), behind
// kma_table_create_from_tsv. Internal; not part of the ABI.
#pragma once

#include <stdint.h>

#include <functional>
#include <string>
#include <vector>

namespace kma {

// kmerdb.tbl as ApplyKmerProcessor.java:100-108 reads it (TabbedLineReader(file, 2): headerless,
// tab-separated, kmer in column 0 and role id in column 1, rows in file order; a line's CR is
// dropped; a row without a tab has the role ""): every row's key (0 for a kmer that is not of
// length k or holds a byte without a code) and its role as a dense fid in first-seen row order.
struct KmerTsv {
  std::vector<uint64_t> keys;   // one per row
  std::vector<uint32_t> fids;   // one per row
  std::vector<std::string> roles;  // fid -> role id
  uint64_t n_skipped = 0;       // rows whose kmer is not of length k
  uint8_t lut[256] = {};        // the residue codes the keys were packed with (make_lut's)
  int last_kmer_len = 0;        // the last row's kmer length (KmerReference.setKmerSize, :108)
};
// make_lut(seen, lut): the table's residue codes given the bytes seen in the file's k-length
// kmers (KMA_OK or a KMA_E_* code). Parsed on `threads` threads over a read-only mapping: pass 1
// counts rows, marks bytes and interns each chunk's roles in first-seen order (a local id per
// row); the chunks' roles are merged in file order into global fids; pass 2 packs the keys. Returns KMA_OK or a
// KMA_E_* code with a message in *err.
int read_kmer_tsv(const char* path, int k, unsigned threads,
                  const std::function<int(const bool* seen, uint8_t* lut)>& make_lut,
                  KmerTsv* out, std::string* err);

}  // namespace kma
