// gto.h — minimal reader for SEEDtk GTO (genome typed object) JSON files and the small text
// formats of the apply command. Restates only what the hot path consumes from the external
// org.theseed.genome.Genome / GenomeDirectory / io.TabbedLineReader / io.LineReader classes.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace kma_host {

// ---- JSON DOM (RFC 8259 subset sufficient for GTOs) ---------------------------------------------
struct Json {
  enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
  bool b = false;
  double num = 0;
  std::string str;
  std::vector<Json> arr;
  std::vector<std::pair<std::string, Json>> obj;
  const Json* get(const std::string& key) const;  // object member or nullptr
  std::string as_string(const std::string& dflt = "") const;
  long long as_int(long long dflt = 0) const;  // numbers and numeric strings
};
Json parse_json(const std::string& text);  // throws std::runtime_error with the byte offset

// ---- Genome ---------------------------------------------------------------------------------------
struct Feature {
  std::string id, type, function;
  std::string protein;  // protein_translation ("" when absent)
  bool is_peg() const { return type == "CDS" || type == "peg"; }
};
struct Contig {
  std::string id, dna;
};
struct Genome {
  std::string id, name;
  int genetic_code = 11;
  std::vector<Contig> contigs;
  std::vector<Feature> features;
  std::vector<const Feature*> pegs() const;  // Genome.getPegs(): CDS features in file order
};
Genome load_genome(const std::string& path);
// What `apply` reads (ApplyKmerProcessor.java:116-147): id, name, genetic code and the features'
// id / type / function / protein_translation. Every other member (contig DNA above all) is
// skipped without being built; contigs stays empty.
Genome load_genome_pegs(const std::string& path);

// GenomeDirectory: the *.gto files of a directory, sorted by file name.
std::vector<std::string> genome_files(const std::string& dir);
// The files of a directory whose names end in `suffix` (and are longer than it), sorted.
std::vector<std::string> files_with_suffix(const std::string& dir, const std::string& suffix);

// ---- text inputs of `apply` -------------------------------------------------------------------
// TabbedLineReader(file, 2) over the headerless kmerdb.tbl: rows (col0, col1) in file order.
struct KmerRows {
  std::string text;               // kmer bytes concatenated
  std::vector<uint64_t> offsets;  // rows + 1
  std::vector<uint32_t> fids;     // role of each row as a dense id (first-seen order)
  std::vector<std::string> roles; // fid -> role id
  std::string last_kmer;          // for KmerReference.setKmerSize(last.length())
};
KmerRows read_kmer_db(const std::string& path);
// LineReader over roles.in.use: first tab field of each line -> 1-based column (last wins).
std::map<std::string, int> read_roles(const std::string& path, int* n_lines);

bool is_directory(const std::string& path);
bool can_read(const std::string& path);

// A file mapped read-only (the apply loader reads ~6 MB per GTO, most of it contig DNA it skips;
// the FASTA reader cuts a mapped file into segments parsed in parallel): mapping the page cache
// saves a zero-filled buffer and a copy. Falls back to a read for what cannot be mapped.
struct MappedFile {
  const char* data = nullptr;
  size_t size = 0;
  explicit MappedFile(const std::string& path);  // throws std::runtime_error
  ~MappedFile();
  MappedFile(const MappedFile&) = delete;
  MappedFile& operator=(const MappedFile&) = delete;

 private:
  std::string fallback_;
  void* map_ = nullptr;  // the mapping (nullptr: fallback_ holds the bytes)
};

}  // namespace kma_host
