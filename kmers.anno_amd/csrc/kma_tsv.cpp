// kma_tsv.cpp — the native kmerdb.tbl reader (kma_tsv.h). The reference loads the table row by
// row into a HashMap<String,String> (ApplyKmerProcessor.java:100-108: ~100-150 bytes of heap per
// row, 10-15 GB and minutes at 10^8 rows); here the file is mapped and parsed on the host's
// cores straight into packed keys and dense role ids, the form kma_table_create_packed builds
// from, so a JNI caller hands the library a path instead of 10^8 strings.
#include "kma_tsv.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <string_view>
#include <thread>

#include "../../include/kmeranno.h"

namespace kma {
namespace {

struct Mapping {
  const char* data = nullptr;
  size_t size = 0;
  ~Mapping() {
    if (data && size) munmap(const_cast<char*>(data), size);
  }
};

// One line [p, e) (no '\n') -> kmer and role views (TabbedLineReader(file, 2): column 0 and 1).
inline void split_row(const char* p, const char* e, std::string_view* kmer, std::string_view* role) {
  if (e > p && e[-1] == '\r') --e;
  const char* tab = static_cast<const char*>(memchr(p, '\t', (size_t)(e - p)));
  if (!tab) {
    *kmer = std::string_view(p, (size_t)(e - p));
    *role = std::string_view();
    return;
  }
  *kmer = std::string_view(p, (size_t)(tab - p));
  const char* r = tab + 1;
  const char* tab2 = static_cast<const char*>(memchr(r, '\t', (size_t)(e - r)));
  *role = std::string_view(r, (size_t)((tab2 ? tab2 : e) - r));
}

// Calls f(kmer, role) for every line starting in [lo, hi) of the mapping (lo is a line start).
template <class F>
void for_rows(const Mapping& m, size_t lo, size_t hi, F&& f) {
  const char* base = m.data;
  size_t pos = lo;
  while (pos < hi) {
    const char* p = base + pos;
    const char* nl = static_cast<const char*>(memchr(p, '\n', m.size - pos));
    const char* e = nl ? nl : base + m.size;
    std::string_view kmer, role;
    split_row(p, e, &kmer, &role);
    f(kmer, role);
    pos = nl ? (size_t)(nl - base) + 1 : m.size;
  }
}

// Role ids interned per chunk in an open-addressing table (std::unordered_map<string_view> cost
// ~100 ns per row: 2.6 s for 10^7 rows on one thread). A role id is a short string (SEED role
// ids, ROLE0000123): hashed 8 bytes at a time.
inline uint64_t role_hash(std::string_view r) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ r.size();
  size_t i = 0;
  for (; i + 8 <= r.size(); i += 8) {
    uint64_t w;
    memcpy(&w, r.data() + i, 8);
    h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
    h ^= h >> 31;
  }
  if (i < r.size()) {
    uint64_t w = 0;
    memcpy(&w, r.data() + i, r.size() - i);
    h = (h ^ w) * 0x94D049BB133111EBull;
    h ^= h >> 29;
  }
  return h * 0xBF58476D1CE4E5B9ull;
}
class RoleTable {
 public:
  RoleTable() : slots_(1024) {}
  // The id of role r (ids in first-seen order; `added` set for a new one).
  uint32_t intern(std::string_view r, bool* added) {
    const uint64_t h = role_hash(r);
    for (size_t i = h & (slots_.size() - 1);; i = (i + 1) & (slots_.size() - 1)) {
      Slot& s = slots_[i];
      if (s.id == kEmpty) {
        if (2 * (offs_.size() + 1) > slots_.size()) {  // keep the load <= 1/2
          grow();
          return intern(r, added);
        }
        s = Slot{h, (uint32_t)offs_.size()};
        offs_.push_back(arena_.size());
        arena_.append(r.data(), r.size());
        *added = true;
        return s.id;
      }
      if (s.h == h && role(s.id) == r) {
        *added = false;
        return s.id;
      }
    }
  }
  size_t size() const { return offs_.size(); }
  // The role of an id: its bytes live in the table's own arena (compact and cache-resident: a
  // view into the mapped file made every compare a miss to a random page, ~70 ns per row).
  std::string_view role(uint32_t id) const {
    const size_t e = id + 1 < offs_.size() ? offs_[id + 1] : arena_.size();
    return std::string_view(arena_.data() + offs_[id], e - offs_[id]);
  }

 private:
  static constexpr uint32_t kEmpty = 0xFFFFFFFFu;
  struct Slot {
    uint64_t h = 0;
    uint32_t id = kEmpty;
  };
  void grow() {
    std::vector<Slot> old(2 * slots_.size());
    old.swap(slots_);
    for (const Slot& s : old)
      if (s.id != kEmpty)
        for (size_t i = s.h & (slots_.size() - 1);; i = (i + 1) & (slots_.size() - 1))
          if (slots_[i].id == kEmpty) {
            slots_[i] = s;
            break;
          }
  }
  std::vector<Slot> slots_;
  std::vector<size_t> offs_;  // id -> start in arena_
  std::string arena_;
};

struct Chunk {
  size_t lo = 0, hi = 0;
  uint64_t rows = 0;
  bool seen[256] = {};
  RoleTable table;               // the chunk's roles -> local ids (first-seen order)
  std::vector<uint32_t> local;   // row -> local id (pass 2 maps it instead of a second lookup)
  std::vector<uint32_t> global;  // local id -> fid
  int last_len = -1;
};

template <class F>
void parallel(unsigned n, F f) {
  std::vector<std::thread> th;
  for (unsigned i = 1; i < n; ++i) th.emplace_back(f, i);
  f(0u);
  for (auto& t : th) t.join();
}

}  // namespace

int read_kmer_tsv(const char* path, int k, unsigned threads,
                  const std::function<int(const bool* seen, uint8_t* lut)>& make_lut,
                  KmerTsv* out, std::string* err) {
  Mapping m;
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    *err = std::string("cannot open ") + path + ": " + strerror(errno);
    return KMA_E_IO;
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode)) {
    close(fd);
    *err = std::string(path) + " is not a regular file";
    return KMA_E_IO;
  }
  m.size = (size_t)st.st_size;
  if (m.size) {
    void* p = mmap(nullptr, m.size, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
    if (p == MAP_FAILED) {
      close(fd);
      m.size = 0;
      *err = std::string("cannot map ") + path + ": " + strerror(errno);
      return KMA_E_IO;
    }
    m.data = static_cast<const char*>(p);
    (void)madvise(p, m.size, MADV_SEQUENTIAL);
  }
  close(fd);
  // Chunks of >= 1 MiB cut after a line end, one per thread.
  const unsigned nt = (unsigned)std::max<size_t>(1, std::min<size_t>(std::max(1u, threads), m.size >> 20));
  std::vector<Chunk> ch(nt);
  for (unsigned i = 0; i < nt; ++i) {
    size_t b = m.size * i / nt;
    if (i) {
      const char* nl = static_cast<const char*>(memchr(m.data + b, '\n', m.size - b));
      b = nl ? (size_t)(nl - m.data) + 1 : m.size;
    }
    ch[i].lo = b;
  }
  for (unsigned i = 0; i < nt; ++i) ch[i].hi = i + 1 < nt ? std::max(ch[i].lo, ch[i + 1].lo) : m.size;
  // pass 1: rows, bytes of k-length kmers, roles in first-seen order
  parallel(nt, [&](unsigned i) {
    Chunk& c = ch[i];
    for_rows(m, c.lo, c.hi, [&](std::string_view kmer, std::string_view role) {
      ++c.rows;
      c.last_len = (int)kmer.size();
      if (kmer.size() == (size_t)k)
        for (char x : kmer) c.seen[(uint8_t)x] = true;
      bool added;
      c.local.push_back(c.table.intern(role, &added));
    });
  });
  bool seen[256] = {};
  uint64_t rows = 0;
  for (const Chunk& c : ch) {
    for (int b = 0; b < 256; ++b) seen[b] = seen[b] || c.seen[b];
    rows += c.rows;
    if (c.last_len >= 0) out->last_kmer_len = c.last_len;
  }
  uint8_t* lut = out->lut;
  if (int rc = make_lut(seen, lut)) {
    *err = "more than 4 kmer symbols outside [A-Z*]";
    return rc;
  }
  RoleTable gid;  // chunks' roles in file order -> fids in first-seen order
  out->roles.clear();
  for (Chunk& c : ch) {
    c.global.resize(c.table.size());
    for (uint32_t j = 0; j < c.table.size(); ++j) {
      bool added;
      c.global[j] = gid.intern(c.table.role(j), &added);
      if (added) out->roles.emplace_back(c.table.role(j));
    }
  }
  if (out->roles.size() > (size_t)KMA_MAX_FID + 1) {
    *err = std::to_string(out->roles.size()) + " distinct roles (limit 2^22)";
    return KMA_E_INVALID;
  }
  out->keys.assign(rows, 0);
  out->fids.assign(rows, 0);
  std::vector<uint64_t> first(nt + 1, 0), skipped(nt, 0);
  for (unsigned i = 0; i < nt; ++i) first[i + 1] = first[i] + ch[i].rows;
  // pass 2: packed keys (0: not a k-mer or a byte without a code) and global fids
  parallel(nt, [&](unsigned i) {
    uint64_t r = first[i], sk = 0;
    const uint32_t* local = ch[i].local.data();
    const uint32_t* global = ch[i].global.data();
    for_rows(m, ch[i].lo, ch[i].hi, [&](std::string_view kmer, std::string_view) {
      uint64_t key = 0;
      if (kmer.size() == (size_t)k) {
        for (char x : kmer) {
          const uint8_t c = lut[(uint8_t)x];
          if (!c) {
            key = 0;
            break;
          }
          key = (key << 5) | c;
        }
      } else {
        ++sk;
      }
      out->keys[r] = key;
      out->fids[r] = global[local[r - first[i]]];
      ++r;
    });
    skipped[i] = sk;
  });
  out->n_skipped = 0;
  for (uint64_t s : skipped) out->n_skipped += s;
  return KMA_OK;
}

}  // namespace kma
