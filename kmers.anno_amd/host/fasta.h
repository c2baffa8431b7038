// fasta.h — protein FASTA input for the FASTA form of the apply command (`kma apply-fasta`).
//
// Restates what the reference reads through the external org.theseed.sequence.FastaInputStream
// (used for protein FASTA at anno/BuildKmerProcessor.java:196-198; the class is in the
// un-vendored org.theseed:sequence 1.0.0 artifact, pom.xml:48-72, so these rules are ASSUMED,
// not pinned by any reference fixture):
//   - lines end at "\n", "\r\n" or a lone "\r" (java.io.BufferedReader.readLine);
//   - a line starting with '>' opens a record: its label (the sequence id) runs to the first
//     space or tab, and the comment is everything after that one separator (the function, in
//     SEEDtk protein FASTA files: ">fig|83333.1.peg.4 Threonine synthase");
//   - every other line up to the next header is appended to the record's sequence as it is
//     (no case change, no filtering; blank lines add nothing);
//   - lines before the first header are ignored; a record with no sequence lines is empty.
//
// The file is mapped and cut into segments that start at record headers, so segments are parsed
// (and annotated) in parallel; the records of all segments, in segment order, are the records of
// the file in file order.
#pragma once

#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

namespace kma_host {

// The records of one segment: sequences concatenated (offsets: records + 1), and the label and
// comment of each record as views into the mapped file (valid while the MappedFile lives).
struct FastaSegment {
  std::string residues;
  std::vector<uint64_t> offsets{0};
  std::vector<std::string_view> ids, comments;
  uint32_t size() const { return (uint32_t)ids.size(); }
  void clear() {
    residues.clear();
    offsets.assign(1, 0);
    ids.clear();
    comments.clear();
  }
};

// Segment boundaries of data[0, size): about `target` bytes each, every boundary after the first
// at a header (a '>' that starts a line). The result starts with 0 and ends with size.
std::vector<size_t> fasta_segment_bounds(const char* data, size_t size, size_t target);

// Parse the records whose headers lie in [begin, end) into `out` (appended). `begin` is the
// start of the file or a boundary from fasta_segment_bounds.
void parse_fasta_segment(const char* begin, const char* end, FastaSegment& out);

}  // namespace kma_host
