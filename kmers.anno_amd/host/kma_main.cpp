// kma_main.cpp — the host side above the C ABI: a C++ mirror of the reference's command layer
// for the hot path (org.theseed.proteins.kmers.anno.App + ApplyKmerProcessor + the apply
// reporters), so `kma apply ...` is a drop-in for `kmers.anno apply ...`.
//
//   kma apply [-h] [-v] [-m N|--min N] [--format APPLY|VERIFY] [--device D]
//             kmerdb.tbl roles.in.use gtoDir
//       ApplyKmerProcessor.java:45-155 with rep/{Default,Verify}ApplyKmerReporter.java.
//   kma contigs [-v] [--device D] kmerdb.tbl gtoDir
//       the 6-frame form (KmerReference.getContigKmers, KmerReference.java:157-203) probed
//       against the same table: one line per hit, genome_id contig strand left right frame role.
//
// Every kmer probe and vote runs on the GPU through libkmeranno.so; this file only parses
// arguments, reads files, and formats reports exactly as the Java reporters do.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gto.h"
#include "kmeranno.h"

using namespace kma_host;

namespace {

bool g_verbose = false;

void log_info(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void log_info(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::fprintf(stderr, "[main] INFO  ");
  std::vfprintf(stderr, fmt, ap);
  std::fprintf(stderr, "\n");
  va_end(ap);
}

struct UsageError : std::runtime_error {  // args4j CmdLineException / ParseFailureException
  using std::runtime_error::runtime_error;
};
struct NotFound : std::runtime_error {  // FileNotFoundException
  using std::runtime_error::runtime_error;
};
struct NativeError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

void check(int rc, const char* what) {
  if (rc != KMA_OK) throw NativeError(std::string(what) + ": " + kma_last_error());
}

// ---- reporters (rep/ApplyKmerReporter.java and subclasses) -------------------------------------
class ApplyKmerReporter {
 public:
  virtual ~ApplyKmerReporter() = default;
  // ApplyKmerReporter.initReport (:43-54): role -> 1-based column from the roles file.
  void initReport(const std::string& rolesToUse) {
    roleIdxMap_ = read_roles(rolesToUse, nullptr);
    openReport();
  }
  virtual void openReport() = 0;
  virtual void openGenome(const Genome& g) = 0;
  virtual void recordFeature(const Feature& f, const std::string& role, int count) = 0;
  virtual void closeGenome() = 0;
  virtual void closeReport() {}
  int getRoleIdx(const std::string& role) const {  // :92-95, 0 when not interesting
    auto it = roleIdxMap_.find(role);
    return it == roleIdxMap_.end() ? 0 : it->second;
  }
  int getNumRoles() const { return (int)roleIdxMap_.size(); }

 private:
  std::map<std::string, int> roleIdxMap_;
};

class DefaultApplyKmerReporter : public ApplyKmerReporter {  // DefaultApplyKmerReporter.java
 public:
  void openReport() override { roleCounts_.assign(getNumRoles(), 0); }
  void openGenome(const Genome& g) override {
    genomeId_ = g.id;
    std::fill(roleCounts_.begin(), roleCounts_.end(), 0);
  }
  void recordFeature(const Feature&, const std::string& role, int) override {
    const int idx = getRoleIdx(role);
    if (idx > 0) {
      if (idx - 1 >= (int)roleCounts_.size())  // Java: ArrayIndexOutOfBoundsException
        throw std::runtime_error("role column " + std::to_string(idx) + " out of range");
      roleCounts_[idx - 1]++;
    }
  }
  void closeGenome() override {
    std::string line = genomeId_ + "\t";
    for (size_t i = 0; i < roleCounts_.size(); ++i) {
      if (i) line += '\t';
      line += std::to_string(roleCounts_[i]);
    }
    std::printf("%s\n", line.c_str());
  }

 private:
  std::vector<int> roleCounts_;
  std::string genomeId_;
};

class VerifyApplyKmerReporter : public ApplyKmerReporter {  // VerifyApplyKmerReporter.java
 public:
  void openReport() override { std::printf("genome_id\tpeg_id\trole\thits\tfunction\n"); }
  void openGenome(const Genome& g) override { genomeId_ = g.id; }
  void recordFeature(const Feature& f, const std::string& role, int count) override {
    std::printf("%s\t%s\t%s\t%d\t%s\n", genomeId_.c_str(), f.id.c_str(), role.c_str(), count,
                f.function.c_str());
  }
  void closeGenome() override {}

 private:
  std::string genomeId_;
};

using Clock = std::chrono::steady_clock;
double seconds(Clock::time_point t0) {
  return std::chrono::duration<double>(Clock::now() - t0).count();
}

// GenomeDirectory iteration with the GTOs parsed ahead by a thread pool (load_genome_pegs),
// at most `lookahead` genomes past the consumer; genomes are taken in file order.
class GenomeFeed {
 public:
  GenomeFeed(const std::vector<std::string>& files, int threads, size_t lookahead)
      : files_(files), slots_(files.size()), errors_(files.size()), ready_(files.size(), 0),
        lookahead_(std::max<size_t>(lookahead, 1)) {
    const int n = (int)std::max<size_t>(1, std::min<size_t>(threads, files.size()));
    for (int i = 0; i < n; ++i) pool_.emplace_back([this] { work(); });
  }
  ~GenomeFeed() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : pool_) t.join();
  }
  std::unique_ptr<Genome> take(size_t i) {
    std::unique_ptr<Genome> out;
    std::string err;
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [&] { return ready_[i] != 0; });
      out = std::move(slots_[i]);
      err = std::move(errors_[i]);
      taken_ = i + 1;
    }
    cv_.notify_all();
    if (!err.empty()) throw std::runtime_error(files_[i] + ": " + err);
    return out;
  }
  int threads() const { return (int)pool_.size(); }

 private:
  void work() {
    for (;;) {
      size_t i;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || next_ >= files_.size() || next_ < taken_ + lookahead_; });
        if (stop_ || next_ >= files_.size()) return;
        i = next_++;
      }
      std::unique_ptr<Genome> gen;
      std::string err;
      try {
        gen.reset(new Genome(load_genome_pegs(files_[i])));
      } catch (const std::exception& e) {
        err = e.what();
        if (err.empty()) err = "parse failure";
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        slots_[i] = std::move(gen);
        errors_[i] = std::move(err);
        ready_[i] = 1;
      }
      cv_.notify_all();
    }
  }
  const std::vector<std::string>& files_;
  std::vector<std::unique_ptr<Genome>> slots_;
  std::vector<std::string> errors_;
  std::vector<char> ready_;
  size_t lookahead_, next_ = 0, taken_ = 0;
  bool stop_ = false;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<std::thread> pool_;
};

// Consecutive genomes concatenated for one native call; pegs[first[g] .. first[g + 1]) are
// genome g's (Genome.getPegs order).
struct Batch {
  std::vector<std::unique_ptr<Genome>> genomes;
  std::vector<const Feature*> pegs;
  std::vector<uint32_t> first{0};
  std::string residues;
  std::vector<uint64_t> offsets{0};
  std::vector<int32_t> fid, count;
  std::vector<uint8_t> status;
  void clear() {
    genomes.clear();
    pegs.clear();
    first.assign(1, 0);
    residues.clear();
    offsets.assign(1, 0);
  }
  void add(std::unique_ptr<Genome> g) {
    for (const Feature* f : g->pegs()) {
      residues += f->protein;
      offsets.push_back(residues.size());
      pegs.push_back(f);
    }
    first.push_back((uint32_t)pegs.size());
    genomes.push_back(std::move(g));
  }
};

// ---- ApplyKmerProcessor -----------------------------------------------------------------------
class ApplyKmerProcessor {
 public:
  void setDefaults() {  // :77-80
    outputType_ = "APPLY";
    minHits_ = 5;
  }

  void parseCommand(const std::vector<std::string>& args) {
    setDefaults();
    std::vector<std::string> pos;
    for (size_t i = 0; i < args.size(); ++i) {
      const std::string& a = args[i];
      auto need = [&](const char* opt) -> std::string {
        if (i + 1 >= args.size()) throw UsageError(std::string("Option \"") + opt + "\" takes an operand");
        return args[++i];
      };
      if (a == "-h" || a == "--help") {
        help_ = true;
      } else if (a == "-v" || a == "--verbose") {
        g_verbose = true;
      } else if (a == "-m" || a == "--min") {
        const std::string v = need("-m");
        char* e = nullptr;
        const long n = std::strtol(v.c_str(), &e, 10);
        if (!*v.c_str() || *e) throw UsageError("\"" + v + "\" is not a valid value for \"-m\"");
        minHits_ = (int)n;
      } else if (a == "--format") {
        outputType_ = need("--format");
        if (outputType_ != "APPLY" && outputType_ != "VERIFY")
          throw UsageError("\"" + outputType_ + "\" is not a valid value for \"--format\"");
      } else if (a == "--device") {
        device_ = std::atoi(need("--device").c_str());
      } else if (a == "--threads") {
        parseThreads_ = std::max(1, std::atoi(need("--threads").c_str()));
      } else if (a == "--batch") {
        batchResidues_ = std::strtoull(need("--batch").c_str(), nullptr, 10);
      } else if (!a.empty() && a[0] == '-' && a.size() > 1) {
        throw UsageError("\"" + a + "\" is not a valid option");
      } else {
        pos.push_back(a);
      }
    }
    if (help_) return;
    if (pos.size() != 3) throw UsageError("Argument \"kmerdb.tbl roles.in.use gtoDir\" is required");
    kmerDbFile_ = pos[0];
    goodRoleFile_ = pos[1];
    inDir_ = pos[2];
    validateParms();
  }

  void validateParms() {  // :83-111
    if (!is_directory(inDir_))
      throw NotFound("Input directory " + inDir_ + " not found or invalid.");
    if (!can_read(kmerDbFile_))
      throw NotFound("Kmer database file " + kmerDbFile_ + " not found or unreadable.");
    if (minHits_ < 1) throw UsageError("Min-hits must be positive.");
    if (outputType_ == "VERIFY") reporter_.reset(new VerifyApplyKmerReporter());
    else reporter_.reset(new DefaultApplyKmerReporter());
    if (!can_read(goodRoleFile_))
      throw NotFound("Roles-to-use file " + goodRoleFile_ + " not found or unreadable.");
    log_info("Reading roles to use from %s.", goodRoleFile_.c_str());
    reporter_->initReport(goodRoleFile_);
    log_info("Loading kmer database from %s.", kmerDbFile_.c_str());
    const auto t0 = Clock::now();
    db_ = read_kmer_db(kmerDbFile_);
    // KmerReference.setKmerSize(lastKmer.length()) (:108) only affects the 6-frame code; the
    // protein extractor (ProteinKmers) keeps its own K = 8, so the table is built for K = 8.
    log_info("Kmer size is %zu.", db_.last_kmer.size());
    check(kma_table_create(db_.text.data(), db_.offsets.data(), db_.fids.data(), db_.fids.size(),
                           kProteinK, device_, 0.0, &table_),
          "kma_table_create");
    tableLoadS_ = seconds(t0);
    kma_table_info info;
    kma_table_info_get(table_, &info);
    if (g_verbose)
      log_info("%llu kmers loaded (%llu distinct, %llu not of length %d), %llu MiB on GPU %d.",
               (unsigned long long)info.n_rows, (unsigned long long)info.n_entries,
               (unsigned long long)info.n_skipped, kProteinK,
               (unsigned long long)(info.bytes >> 20), device_);
  }

  // :114-155. The reference loops genome by genome: parse a GTO, run every peg's ProteinKmers
  // through the map, report. Here the same reports come out in the same order, but
  //   - GTOs are parsed ahead by a pool of threads (GenomeFeed: the loader skips contig DNA),
  //   - consecutive genomes are batched into one native call of >= batch_residues residues
  //     (a 4k-peg genome is ~1.2M residues: a launch that small leaves most of the GPU idle),
  //   - the call runs while the pool parses the next genomes.
  void runCommand() {
    const std::vector<std::string> files = genome_files(inDir_);
    log_info("%zu genomes found in input directory.", files.size());
    const auto t0 = Clock::now();
    GenomeFeed feed(files, parseThreads_, 4 * batchGenomesHint());
    Batch b;
    uint64_t n_prot = 0, n_res = 0, n_calls = 0;
    double gpu_s = 0;
    for (size_t i = 0; i < files.size();) {
      b.clear();
      while (i < files.size() && (b.residues.size() < batchResidues_ || b.genomes.empty())) {
        b.add(feed.take(i++));
        if (!b.genomes.empty() && b.residues.size() >= batchResidues_) break;
      }
      const uint32_t n = (uint32_t)b.pegs.size();
      b.fid.resize(n);
      b.count.resize(n);
      b.status.resize(n);
      const auto c0 = Clock::now();
      if (n)  // one batched native call replaces the per-feature ProteinKmers + probe loop
        check(kma_annotate_proteins(table_, reinterpret_cast<const uint8_t*>(b.residues.data()),
                                    b.offsets.data(), n, minHits_, 0, b.fid.data(),
                                    b.count.data(), b.status.data(), nullptr, 0),
              "kma_annotate_proteins");
      gpu_s += seconds(c0);
      n_calls += n > 0;
      n_prot += n;
      n_res += b.residues.size();
      for (size_t g = 0; g < b.genomes.size(); ++g) {
        const Genome& genome = *b.genomes[g];
        log_info("Processing genome %s (%s).", genome.id.c_str(), genome.name.c_str());
        reporter_->openGenome(genome);
        for (uint32_t j = b.first[g]; j < b.first[g + 1]; ++j)
          if (b.status[j] == KMA_STATUS_CALLED)  // role != null && !badPeg && count >= minHits
            reporter_->recordFeature(*b.pegs[j], db_.roles[b.fid[j]], b.count[j]);
        reporter_->closeGenome();
      }
    }
    reporter_->closeReport();
    std::fflush(stdout);
    const double wall = seconds(t0);
    // one machine-readable line on stderr (bench.py's genome-directory workload reads it)
    std::fprintf(stderr,
                 "[kma] apply-stats {\"genomes\": %zu, \"proteins\": %llu, \"residues\": %llu, "
                 "\"calls\": %llu, \"loop_s\": %.6f, \"native_call_s\": %.6f, "
                 "\"parse_threads\": %d, \"batch_residues\": %llu, \"table_load_s\": %.6f}\n",
                 files.size(), (unsigned long long)n_prot, (unsigned long long)n_res,
                 (unsigned long long)n_calls, wall, gpu_s, feed.threads(),
                 (unsigned long long)batchResidues_, tableLoadS_);
  }

  bool help() const { return help_; }
  size_t batchGenomesHint() const {  // genomes of ~1.2M residues per batch
    return std::max<size_t>(2, batchResidues_ / 1200000 + 1);
  }
  ~ApplyKmerProcessor() {
    if (table_) kma_table_destroy(table_);
  }

  static constexpr int kProteinK = 8;  // org.theseed.sequence.ProteinKmers default size

 private:
  std::string outputType_;
  int minHits_ = 5;
  int device_ = 0;
  bool help_ = false;
  int parseThreads_ = (int)std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  uint64_t batchResidues_ = 16ull << 20;  // residues per native call (several genomes)
  double tableLoadS_ = 0;
  std::string kmerDbFile_, goodRoleFile_, inDir_;
  std::unique_ptr<ApplyKmerReporter> reporter_;
  KmerRows db_;
  kma_table* table_ = nullptr;
};

const char* kApplyUsage =
    "kma apply [options] kmerdb.tbl roles.in.use gtoDir\n"
    "  apply a discriminating-kmer database to genomes to create a role-count file\n"
    " -h, --help        display command-line usage\n"
    " -v, --verbose     display more frequent progress messages on the log\n"
    " -m, --min N       minimum number of hits required to call a role (default 5)\n"
    " --format FMT      reporting format: APPLY (default) or VERIFY\n"
    " --device D        HIP device ordinal (default 0)\n"
    " --threads N       GTO parser threads (default min(8, cores))\n"
    " --batch R         residues per native call, whole genomes (default 16777216)\n";

int run_apply(const std::vector<std::string>& args) {
  ApplyKmerProcessor p;
  p.parseCommand(args);
  if (p.help()) {
    std::fputs(kApplyUsage, stderr);
    return 0;
  }
  p.runCommand();
  return 0;
}

int run_contigs(const std::vector<std::string>& args) {
  int device = 0;
  std::vector<std::string> pos;
  for (size_t i = 0; i < args.size(); ++i) {
    if (args[i] == "--device" && i + 1 < args.size()) device = std::atoi(args[++i].c_str());
    else if (args[i] == "-v") g_verbose = true;
    else pos.push_back(args[i]);
  }
  if (pos.size() != 2) throw UsageError("usage: kma contigs [--device D] kmerdb.tbl gtoDir");
  if (!can_read(pos[0])) throw NotFound("Kmer database file " + pos[0] + " not found or unreadable.");
  if (!is_directory(pos[1])) throw NotFound("Input directory " + pos[1] + " not found or invalid.");
  KmerRows db = read_kmer_db(pos[0]);
  const int k = (int)db.last_kmer.size();  // KmerReference.setKmerSize(last kmer length)
  kma_table* t = nullptr;
  check(kma_table_create(db.text.data(), db.offsets.data(), db.fids.data(), db.fids.size(), k,
                         device, 0.0, &t),
        "kma_table_create");
  std::printf("genome_id\tcontig_id\tstrand\tleft\tright\tframe\trole\n");
  for (const std::string& path : genome_files(pos[1])) {
    Genome g = load_genome(path);
    std::string dna;
    std::vector<uint64_t> off{0};
    for (const Contig& c : g.contigs) {
      dna += c.dna;
      off.push_back(dna.size());
    }
    std::vector<kma_hit> hits(1024);
    uint64_t nh = 0;
    int rc;
    while ((rc = kma_annotate_contigs(t, reinterpret_cast<const uint8_t*>(dna.data()), off.data(),
                                      (uint32_t)g.contigs.size(), g.genetic_code, hits.data(),
                                      hits.size(), &nh, nullptr, 0)) == KMA_E_CAPACITY)
      hits.resize(nh);
    check(rc, "kma_annotate_contigs");
    for (uint64_t i = 0; i < nh; ++i) {
      const kma_hit& h = hits[i];
      std::printf("%s\t%s\t%c\t%d\t%d\t%d\t%s\n", g.id.c_str(), g.contigs[h.contig].id.c_str(),
                  h.strand, h.left, h.left + 3 * k - 1, h.frame, db.roles[h.fid].c_str());
    }
  }
  kma_table_destroy(t);
  return 0;
}

const char* kCommands =
    "Valid commands are\n"
    "  apply     apply a discriminating-kmer database to genomes to create a role-count file\n"
    "  contigs   6-frame contig kmers probed against a discriminating-kmer database\n";

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fputs(kCommands, stderr);
    return 1;
  }
  const std::string command = argv[1];
  std::vector<std::string> rest(argv + 2, argv + argc);
  try {
    if (command == "apply") return run_apply(rest);
    if (command == "contigs") return run_contigs(rest);
    if (command == "-h" || command == "--help") {
      std::fputs(kCommands, stdout);
      return 0;
    }
    std::fprintf(stderr, "Invalid command %s.\n", command.c_str());  // App.java:301
    return 1;
  } catch (const UsageError& e) {
    std::fprintf(stderr, "%s\n%s", e.what(), command == "apply" ? kApplyUsage : "");
    return 2;
  } catch (const NotFound& e) {
    std::fprintf(stderr, "java.io.FileNotFoundException: %s\n", e.what());
    return 1;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
}
