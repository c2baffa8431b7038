// fasta.cpp — see fasta.h.
#include "fasta.h"

#include <cstring>

namespace kma_host {
namespace {

// The line at p: returns its end (terminator excluded) and sets *next to the next line's start.
// Terminators as java.io.BufferedReader.readLine: "\n", "\r\n" or a lone "\r".
inline const char* line_end(const char* p, const char* end, const char** next) {
  const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(end - p)));
  const char* lim = nl ? nl : end;
  if (const char* cr = static_cast<const char*>(std::memchr(p, '\r', (size_t)(lim - p)))) {
    *next = cr + 1 < end && cr[1] == '\n' ? cr + 2 : cr + 1;
    return cr;
  }
  *next = nl ? nl + 1 : end;
  return lim;
}

}  // namespace

std::vector<size_t> fasta_segment_bounds(const char* data, size_t size, size_t target) {
  std::vector<size_t> b{0};
  if (target == 0) target = 1;
  size_t at = target;
  while (at < size) {
    // the first header at or after `at`: a '>' at the start of a line
    size_t q = at;
    for (;;) {
      const void* hit = std::memchr(data + q, '>', size - q);
      if (!hit) {
        q = size;
        break;
      }
      q = (size_t)(static_cast<const char*>(hit) - data);
      if (data[q - 1] == '\n' || data[q - 1] == '\r') break;
      ++q;
    }
    if (q >= size) break;
    b.push_back(q);
    at = q + target;
  }
  b.push_back(size);
  return b;
}

void parse_fasta_segment(const char* begin, const char* end, FastaSegment& out) {
  const char* p = begin;
  const char* next = nullptr;
  while (p < end && *p != '>') {  // lines before the first header
    line_end(p, end, &next);
    p = next;
  }
  out.residues.reserve(out.residues.size() + (size_t)(end - p));
  while (p < end) {  // *p == '>'
    const char* he = line_end(p, end, &next);
    const char* label = p + 1;
    const char* sep = label;
    while (sep < he && *sep != ' ' && *sep != '\t') ++sep;
    out.ids.emplace_back(label, (size_t)(sep - label));
    out.comments.emplace_back(sep < he ? sep + 1 : he, sep < he ? (size_t)(he - sep - 1) : 0);
    p = next;
    while (p < end && *p != '>') {
      const char* le = line_end(p, end, &next);
      out.residues.append(p, (size_t)(le - p));
      p = next;
    }
    out.offsets.push_back(out.residues.size());
  }
}

}  // namespace kma_host
