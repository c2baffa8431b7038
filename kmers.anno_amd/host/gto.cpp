// gto.cpp — see gto.h.
#include "gto.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string_view>
#include <unordered_map>

namespace kma_host {

const Json* Json::get(const std::string& key) const {
  if (kind != Object) return nullptr;
  for (const auto& kv : obj)
    if (kv.first == key) return &kv.second;
  return nullptr;
}

std::string Json::as_string(const std::string& dflt) const {
  if (kind == String) return str;
  if (kind == Number) {
    std::ostringstream o;
    o << (long long)num;
    return o.str();
  }
  return dflt;
}

long long Json::as_int(long long dflt) const {
  if (kind == Number) return (long long)num;
  if (kind == String && !str.empty()) return std::strtoll(str.c_str(), nullptr, 10);
  return dflt;
}

namespace {

struct Parser {
  const char* p;
  const char* begin;
  const char* end;
  [[noreturn]] void error(const char* what) {
    throw std::runtime_error(std::string("JSON parse error at byte ") +
                             std::to_string(p - begin) + ": " + what);
  }
  void ws() {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  static void put_utf8(std::string& s, uint32_t cp) {
    if (cp < 0x80) {
      s += (char)cp;
    } else if (cp < 0x800) {
      s += (char)(0xC0 | (cp >> 6));
      s += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      s += (char)(0xE0 | (cp >> 12));
      s += (char)(0x80 | ((cp >> 6) & 0x3F));
      s += (char)(0x80 | (cp & 0x3F));
    } else {
      s += (char)(0xF0 | (cp >> 18));
      s += (char)(0x80 | ((cp >> 12) & 0x3F));
      s += (char)(0x80 | ((cp >> 6) & 0x3F));
      s += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (end - p < 4) error("short \\u escape");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else error("bad \\u escape");
    }
    return v;
  }
  std::string string() {
    if (*p != '"') error("expected string");
    ++p;
    {  // the common case, no escape: one memchr to the closing quote, one for a backslash
      const char* q = static_cast<const char*>(std::memchr(p, '"', end - p));
      if (q && !std::memchr(p, '\\', q - p)) {
        std::string s(p, q);
        p = q + 1;
        return s;
      }
    }
    std::string s;
    for (;;) {
      const char* q = p;
      while (q < end && *q != '"' && *q != '\\') ++q;
      s.append(p, q);
      p = q;
      if (p >= end) error("unterminated string");
      if (*p == '"') {
        ++p;
        return s;
      }
      ++p;  // backslash
      if (p >= end) error("bad escape");
      char c = *p++;
      switch (c) {
        case '"': s += '"'; break;
        case '\\': s += '\\'; break;
        case '/': s += '/'; break;
        case 'b': s += '\b'; break;
        case 'f': s += '\f'; break;
        case 'n': s += '\n'; break;
        case 'r': s += '\r'; break;
        case 't': s += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            p += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(s, cp);
          break;
        }
        default: error("bad escape");
      }
    }
  }
  // Skip one value without building it (the apply loader's unwanted members: contig DNA,
  // feature locations, ...): strings by a memchr to each quote, containers by depth.
  void skip_string() {
    ++p;  // opening quote
    for (;;) {
      const char* q = static_cast<const char*>(std::memchr(p, '"', end - p));
      if (!q) error("unterminated string");
      const char* b = q;
      while (b > p && b[-1] == '\\') --b;
      p = q + 1;
      if (((q - b) & 1) == 0) return;  // an even run of backslashes: the quote closes
    }
  }
  void skip() {
    ws();
    if (p >= end) error("unexpected end");
    if (*p == '"') return skip_string();
    if (*p != '{' && *p != '[') {  // number / true / false / null: up to the next delimiter
      const char* q = p;
      while (q < end && *q != ',' && *q != '}' && *q != ']' && *q != ' ' && *q != '\n' &&
             *q != '\t' && *q != '\r')
        ++q;
      if (q == p) error("bad value");
      p = q;
      return;
    }
    int depth = 0;
    while (p < end) {
      const char c = *p;
      if (c == '"') {
        skip_string();
        continue;
      }
      ++p;
      if (c == '{' || c == '[') ++depth;
      else if ((c == '}' || c == ']') && --depth == 0) return;
    }
    error("unterminated container");
  }
  // An object key as a view into the text when it holds no escape (GTO keys never do), else
  // decoded into `buf`.
  std::string_view key(std::string& buf) {
    if (p >= end || *p != '"') error("expected string");
    const char* q = static_cast<const char*>(std::memchr(p + 1, '"', end - p - 1));
    if (q && !std::memchr(p + 1, '\\', q - p - 1)) {
      const std::string_view v(p + 1, (size_t)(q - p - 1));
      p = q + 1;
      return v;
    }
    buf = string();
    return buf;
  }
  // Members of an object, calling f(key) with p at the value; f consumes the value.
  // members() that stops after the member for which f returns true (p is then just past that
  // member's value; the rest of the object is not read). Returns whether it stopped early.
  template <class F>
  bool members_until(F f) {
    bool stopped = false;
    members_impl([&](std::string_view k) { return stopped = f(k); });
    return stopped;
  }
  template <class F>
  void members(F f) {
    members_impl([&](std::string_view k) {
      f(k);
      return false;
    });
  }
  template <class F>
  void members_impl(F f) {
    ws();
    if (p >= end || *p != '{') error("expected object");
    ++p;
    ws();
    if (p < end && *p == '}') {
      ++p;
      return;
    }
    std::string buf;
    for (;;) {
      ws();
      const std::string_view k = key(buf);
      ws();
      if (p >= end || *p != ':') error("expected ':'");
      ++p;
      ws();
      if (f(k)) return;
      ws();
      if (p < end && *p == ',') {
        ++p;
        continue;
      }
      if (p < end && *p == '}') {
        ++p;
        return;
      }
      error("expected ',' or '}'");
    }
  }
  template <class F>
  void elements(F f) {
    ws();
    if (p >= end || *p != '[') error("expected array");
    ++p;
    ws();
    if (p < end && *p == ']') {
      ++p;
      return;
    }
    for (;;) {
      ws();
      f();
      ws();
      if (p < end && *p == ',') {
        ++p;
        continue;
      }
      if (p < end && *p == ']') {
        ++p;
        return;
      }
      error("expected ',' or ']'");
    }
  }
  Json value() {
    ws();
    if (p >= end) error("unexpected end");
    Json v;
    switch (*p) {
      case '{': {
        ++p;
        v.kind = Json::Object;
        ws();
        if (p < end && *p == '}') {
          ++p;
          return v;
        }
        for (;;) {
          ws();
          std::string k = string();
          ws();
          if (p >= end || *p != ':') error("expected ':'");
          ++p;
          v.obj.emplace_back(std::move(k), value());
          ws();
          if (p < end && *p == ',') {
            ++p;
            continue;
          }
          if (p < end && *p == '}') {
            ++p;
            return v;
          }
          error("expected ',' or '}'");
        }
      }
      case '[': {
        ++p;
        v.kind = Json::Array;
        ws();
        if (p < end && *p == ']') {
          ++p;
          return v;
        }
        for (;;) {
          v.arr.push_back(value());
          ws();
          if (p < end && *p == ',') {
            ++p;
            continue;
          }
          if (p < end && *p == ']') {
            ++p;
            return v;
          }
          error("expected ',' or ']'");
        }
      }
      case '"':
        v.kind = Json::String;
        v.str = string();
        return v;
      case 't':
        if (end - p >= 4 && !std::strncmp(p, "true", 4)) {
          p += 4;
          v.kind = Json::Bool;
          v.b = true;
          return v;
        }
        error("bad literal");
      case 'f':
        if (end - p >= 5 && !std::strncmp(p, "false", 5)) {
          p += 5;
          v.kind = Json::Bool;
          return v;
        }
        error("bad literal");
      case 'n':
        if (end - p >= 4 && !std::strncmp(p, "null", 4)) {
          p += 4;
          return v;
        }
        error("bad literal");
      default: {
        char* q = nullptr;
        v.num = std::strtod(p, &q);
        if (q == p) error("bad value");
        p = q;
        v.kind = Json::Number;
        return v;
      }
    }
  }
};

std::string slurp(const std::string& path) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  std::string s;
  struct stat st;
  if (fstat(fileno(f), &st) == 0 && st.st_size > 0) s.resize((size_t)st.st_size);
  size_t n = s.empty() ? 0 : std::fread(&s[0], 1, s.size(), f);
  s.resize(n);
  char buf[1 << 16];  // whatever fstat did not announce (pipes, growing files)
  while (size_t m = std::fread(buf, 1, sizeof buf, f)) s.append(buf, m);
  std::fclose(f);
  return s;
}

std::string scalar_string(Parser& ps) {  // a string or number member as text
  ps.ws();
  if (ps.p < ps.end && *ps.p == '"') return ps.string();
  return ps.value().as_string();
}


}  // namespace

MappedFile::MappedFile(const std::string& path) {
  const int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("cannot open " + path);
  struct stat st;
  void* m = MAP_FAILED;
  if (fstat(fd, &st) == 0 && st.st_size > 0)
    m = ::mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
  ::close(fd);
  if (m != MAP_FAILED) {
    map_ = m;
    data = static_cast<const char*>(m);
    size = (size_t)st.st_size;
  } else {
    fallback_ = slurp(path);
    data = fallback_.data();
    size = fallback_.size();
  }
}

MappedFile::~MappedFile() {
  if (map_) ::munmap(map_, size);
}

Genome load_genome_pegs(const std::string& path) {
  const MappedFile text(path);
  Parser ps{text.data, text.data, text.data + text.size};
  Genome g;
  // Reading stops once id, scientific_name, genetic_code and features have been read: SEEDtk
  // GTOs put the contigs (the DNA: most of the file) after them (small.gto's member order), so
  // their pages are never touched. A file is then not checked past that point.
  // A member that appears twice keeps its first value, as Json::get (load_genome) does.
  unsigned seen = 0;
  const bool stopped = ps.members_until([&](std::string_view k) {
    if (k == "id" && !(seen & 1)) {
      g.id = scalar_string(ps);
      seen |= 1;
    } else if (k == "scientific_name" && !(seen & 2)) {
      g.name = scalar_string(ps);
      seen |= 2;
    } else if (k == "genetic_code" && !(seen & 4)) {
      g.genetic_code = (int)ps.value().as_int(11);
      seen |= 4;
    } else if (k == "features" && !(seen & 8)) {
      seen |= 8;
      ps.elements([&]() {
        Feature ft;
        unsigned fseen = 0;
        ps.members([&](std::string_view fk) {
          if (fk == "id" && !(fseen & 1)) ft.id = scalar_string(ps), fseen |= 1;
          else if (fk == "type" && !(fseen & 2)) ft.type = scalar_string(ps), fseen |= 2;
          else if (fk == "function" && !(fseen & 4)) ft.function = scalar_string(ps), fseen |= 4;
          else if (fk == "protein_translation" && !(fseen & 8)) ft.protein = scalar_string(ps), fseen |= 8;
          else ps.skip();
        });
        g.features.push_back(std::move(ft));
      });
    } else {
      ps.skip();  // contigs (their DNA), close genomes, subsystems, repeated members, ...
    }
    return seen == 15;
  });
  if (!stopped) {
    ps.ws();
    if (ps.p != ps.end) ps.error("trailing characters");
  }
  return g;
}

Json parse_json(const std::string& text) {
  Parser ps{text.data(), text.data(), text.data() + text.size()};
  Json v = ps.value();
  ps.ws();
  if (ps.p != ps.end) ps.error("trailing characters");
  return v;
}

std::vector<const Feature*> Genome::pegs() const {
  std::vector<const Feature*> out;
  for (const auto& f : features)
    if (f.is_peg()) out.push_back(&f);
  return out;
}

Genome load_genome(const std::string& path) {
  Json j = parse_json(slurp(path));
  Genome g;
  if (const Json* v = j.get("id")) g.id = v->as_string();
  if (const Json* v = j.get("scientific_name")) g.name = v->as_string();
  if (const Json* v = j.get("genetic_code")) g.genetic_code = (int)v->as_int(11);
  if (const Json* cs = j.get("contigs"))
    for (const Json& c : cs->arr) {
      Contig ct;
      if (const Json* v = c.get("id")) ct.id = v->as_string();
      if (const Json* v = c.get("dna")) ct.dna = v->as_string();
      g.contigs.push_back(std::move(ct));
    }
  if (const Json* fs = j.get("features"))
    for (const Json& f : fs->arr) {
      Feature ft;
      if (const Json* v = f.get("id")) ft.id = v->as_string();
      if (const Json* v = f.get("type")) ft.type = v->as_string();
      if (const Json* v = f.get("function")) ft.function = v->as_string();
      if (const Json* v = f.get("protein_translation")) ft.protein = v->as_string();
      g.features.push_back(std::move(ft));
    }
  return g;
}

std::vector<std::string> files_with_suffix(const std::string& dir, const std::string& suffix) {
  std::vector<std::string> out;
  DIR* d = opendir(dir.c_str());
  if (!d) throw std::runtime_error("cannot list " + dir);
  while (dirent* e = readdir(d)) {
    const std::string n = e->d_name;
    if (n.size() > suffix.size() && n.compare(n.size() - suffix.size(), suffix.size(), suffix) == 0)
      out.push_back(dir + "/" + n);
  }
  closedir(d);
  std::sort(out.begin(), out.end());
  return out;
}

std::vector<std::string> genome_files(const std::string& dir) { return files_with_suffix(dir, ".gto"); }

KmerRows read_kmer_db(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  KmerRows r;
  r.offsets.push_back(0);
  std::unordered_map<std::string, uint32_t> role_ids;
  std::string line;
  while (std::getline(f, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    const size_t tab = line.find('\t');
    const std::string kmer = line.substr(0, tab);
    std::string role;
    if (tab != std::string::npos) {
      const size_t tab2 = line.find('\t', tab + 1);
      role = line.substr(tab + 1, tab2 == std::string::npos ? std::string::npos : tab2 - tab - 1);
    }
    auto it = role_ids.find(role);
    if (it == role_ids.end()) {
      it = role_ids.emplace(role, (uint32_t)r.roles.size()).first;
      r.roles.push_back(role);
    }
    r.text += kmer;
    r.offsets.push_back(r.text.size());
    r.fids.push_back(it->second);
    r.last_kmer = kmer;
  }
  return r;
}

std::map<std::string, int> read_roles(const std::string& path, int* n_lines) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::map<std::string, int> idx;
  std::string line;
  int i = 1;
  while (std::getline(f, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    idx[line.substr(0, line.find('\t'))] = i++;  // StringUtils.substringBefore(line, "\t")
  }
  if (n_lines) *n_lines = i - 1;
  return idx;
}

bool is_directory(const std::string& path) {
  struct stat st;
  return stat(path.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

bool can_read(const std::string& path) {
  struct stat st;
  return stat(path.c_str(), &st) == 0 && S_ISREG(st.st_mode) && access(path.c_str(), R_OK) == 0;
}

}  // namespace kma_host
