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
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fasta.h"
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
  // The same call with the role's dense id in the kmer database (the caller's map key): lets
  // a reporter cache per-role work (the default reporter's role -> column lookup).
  virtual void recordFeature(const Feature& f, uint32_t fid, const std::string& role, int count) {
    recordFeature(f, role, count);
  }
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
  void recordFeature(const Feature&, const std::string& role, int) override { count(getRoleIdx(role)); }
  void recordFeature(const Feature&, uint32_t fid, const std::string& role, int) override {
    if (fid >= colOfFid_.size()) colOfFid_.resize(fid + 1, -1);
    if (colOfFid_[fid] < 0) colOfFid_[fid] = getRoleIdx(role);
    count(colOfFid_[fid]);
  }
  void count(int idx) {
    if (idx > 0) {
      if (idx - 1 >= (int)roleCounts_.size())  // Java: ArrayIndexOutOfBoundsException
        throw std::runtime_error("role column " + std::to_string(idx) + " out of range");
      roleCounts_[idx - 1]++;
    }
  }
  void closeGenome() override {
    std::string line = genomeId_ + "\t";
    char num[16];
    for (size_t i = 0; i < roleCounts_.size(); ++i) {
      if (i) line += '\t';
      line.append(num, (size_t)std::snprintf(num, sizeof num, "%d", roleCounts_[i]));
    }
    line += '\n';
    std::fwrite(line.data(), 1, line.size(), stdout);
  }

 private:
  std::vector<int> roleCounts_;
  std::vector<int> colOfFid_;  // role column of a kmer-database role id (-1: not looked up)
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

// One genome of the directory as the apply loop consumes it: the parsed GTO, its pegs
// (Genome.getPegs order) and, when a parse worker annotated it, the native call's outputs.
struct ParsedGenome {
  std::unique_ptr<Genome> genome;
  std::vector<const Feature*> pegs;
  std::vector<int32_t> fid, count;
  std::vector<uint8_t> status;
  bool annotated = false;
  double call_s = 0;  // the worker's native call
};

// GenomeDirectory iteration with the GTOs parsed ahead by a thread pool (load_genome_pegs),
// at most `lookahead` genomes past the consumer; genomes are taken in file order. `after`
// (optional) runs on the worker once a genome is parsed (the per-genome native call).
class GenomeFeed {
 public:
  using After = std::function<void(ParsedGenome&)>;
  GenomeFeed(const std::vector<std::string>& files, int threads, size_t lookahead,
             After after = nullptr)
      : files_(files), slots_(files.size()), errors_(files.size()), ready_(files.size(), 0),
        lookahead_(std::max<size_t>(lookahead, 1)), after_(std::move(after)) {
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
  ParsedGenome take(size_t i) {
    ParsedGenome out;
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
  // Genomes the consumer is done with: freed by the workers (a parsed GTO is ~16k small
  // allocations; freeing them on the report thread cost ~0.5-0.9 ms per genome).
  void recycle(std::vector<ParsedGenome>& done) {
    {
      std::lock_guard<std::mutex> g(mu_);
      for (ParsedGenome& pg : done) trash_.push_back(std::move(pg));
    }
    done.clear();
    cv_.notify_all();  // (the consumer waits on the same condition)
  }

 private:
  void work() {
    for (;;) {
      std::vector<ParsedGenome> trash;
      size_t i = 0;
      bool parse = false;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] {
          return stop_ || !trash_.empty() || (next_ < files_.size() && next_ < taken_ + lookahead_);
        });
        if (!trash_.empty()) {
          trash.swap(trash_);
        } else if (stop_) {
          return;
        } else {
          i = next_++;
          parse = true;
        }
      }
      if (!parse) continue;  // (trash freed here, outside the lock)
      ParsedGenome pg;
      std::string err;
      try {
        pg.genome.reset(new Genome(load_genome_pegs(files_[i])));
        pg.pegs = pg.genome->pegs();
        if (after_) after_(pg);
      } catch (const std::exception& e) {
        err = e.what();
        if (err.empty()) err = "failure";
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        slots_[i] = std::move(pg);
        errors_[i] = std::move(err);
        ready_[i] = 1;
      }
      cv_.notify_all();
    }
  }
  const std::vector<std::string>& files_;
  std::vector<ParsedGenome> slots_;
  std::vector<std::string> errors_;
  std::vector<char> ready_;
  std::vector<ParsedGenome> trash_;
  size_t lookahead_, next_ = 0, taken_ = 0;
  bool stop_ = false;
  After after_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<std::thread> pool_;
};

// Concatenated proteins of one or more genomes for one native call.
struct ProteinBatch {
  std::string residues;
  std::vector<uint64_t> offsets{0};
  void clear() {
    residues.clear();
    offsets.assign(1, 0);
  }
  void add(const std::vector<const Feature*>& pegs) {
    for (const Feature* f : pegs) {
      residues += f->protein;
      offsets.push_back(residues.size());
    }
  }
  uint32_t size() const { return (uint32_t)(offsets.size() - 1); }
};

// A counting semaphore (C++17) and its scoped slot.
class Semaphore {
 public:
  explicit Semaphore(int n) : n_(std::max(1, n)) {}
  void acquire() {
    std::unique_lock<std::mutex> g(mu_);
    cv_.wait(g, [&] { return n_ > 0; });
    --n_;
  }
  void release() {
    {
      std::lock_guard<std::mutex> g(mu_);
      ++n_;
    }
    cv_.notify_one();
  }

 private:
  int n_;
  std::mutex mu_;
  std::condition_variable cv_;
};
struct CallSlot {
  Semaphore& s;
  explicit CallSlot(Semaphore& sem) : s(sem) { s.acquire(); }
  ~CallSlot() { s.release(); }
};

// ---- ApplyKmerProcessor -----------------------------------------------------------------------
class ApplyKmerProcessor {
 public:
  // fasta: the FASTA form (`kma apply-fasta`): protein FASTA files in place of the GTO directory.
  explicit ApplyKmerProcessor(bool fasta = false) : fasta_(fasta) {}

  void setDefaults() {  // :77-80
    // The FASTA form reports per sequence by default (VERIFY rows); APPLY gives a tally row per
    // file.
    outputType_ = fasta_ ? "VERIFY" : "APPLY";
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
      } else if (a == "--staging-threads") {
        stagingThreads_ = std::max(0, std::atoi(need("--staging-threads").c_str()));
      } else if (a == "--batch") {
        batchResidues_ = std::strtoull(need("--batch").c_str(), nullptr, 10);
        if (fasta_) fastaSegment_ = std::max<size_t>(1, (size_t)batchResidues_);
      } else if (a == "--callers" && fasta_) {
        callers_ = std::max(1, std::atoi(need("--callers").c_str()));
      } else if (!a.empty() && a[0] == '-' && a.size() > 1) {
        throw UsageError("\"" + a + "\" is not a valid option");
      } else {
        pos.push_back(a);
      }
    }
    if (help_) return;
    if (fasta_) {
      if (pos.size() < 3)
        throw UsageError("Argument \"kmerdb.tbl roles.in.use proteins.faa...\" is required");
      fastaInputs_.assign(pos.begin() + 2, pos.end());
    } else {
      if (pos.size() != 3) throw UsageError("Argument \"kmerdb.tbl roles.in.use gtoDir\" is required");
      inDir_ = pos[2];
    }
    kmerDbFile_ = pos[0];
    goodRoleFile_ = pos[1];
    validateParms();
  }

  void validateParms() {  // :83-111
    if (fasta_) {
      fastaFiles_.clear();
      for (const std::string& in : fastaInputs_) {
        if (is_directory(in)) {
          for (const std::string& f : fasta_files(in)) fastaFiles_.push_back(f);
        } else if (can_read(in)) {
          fastaFiles_.push_back(in);
        } else {
          throw NotFound("Input FASTA file " + in + " not found or unreadable.");
        }
      }
    } else if (!is_directory(inDir_)) {
      throw NotFound("Input directory " + inDir_ + " not found or invalid.");
    }
    if (!can_read(kmerDbFile_))
      throw NotFound("Kmer database file " + kmerDbFile_ + " not found or unreadable.");
    if (minHits_ < 1) throw UsageError("Min-hits must be positive.");
    if (stagingThreads_ >= 0) check(kma_option_set(KMA_OPT_HOST_THREADS, stagingThreads_), "kma_option_set");
    if (outputType_ == "VERIFY") reporter_.reset(new VerifyApplyKmerReporter());
    else reporter_.reset(new DefaultApplyKmerReporter());
    if (!can_read(goodRoleFile_))
      throw NotFound("Roles-to-use file " + goodRoleFile_ + " not found or unreadable.");
    log_info("Reading roles to use from %s.", goodRoleFile_.c_str());
    reporter_->initReport(goodRoleFile_);
    log_info("Loading kmer database from %s.", kmerDbFile_.c_str());
    const auto t0 = Clock::now();
    // The library reads kmerdb.tbl itself (kma_table_create_from_tsv: the file mapped and parsed
    // on the host's cores into packed keys and first-seen role ids), as a JNI caller would.
    // KmerReference.setKmerSize(lastKmer.length()) (:108) only affects the 6-frame code; the
    // protein extractor (ProteinKmers) keeps its own K = 8, so the table is built for K = 8.
    char* names = nullptr;
    uint64_t names_bytes = 0;
    uint32_t n_roles = 0;
    int last_len = 0;
    check(kma_table_create_from_tsv(kmerDbFile_.c_str(), kProteinK, 1, &device_, 0.0, &table_,
                                    &names, &names_bytes, &n_roles, &last_len),
          "kma_table_create_from_tsv");
    roles_.clear();
    roles_.reserve(n_roles);
    for (uint64_t o = 0; o < names_bytes; o += roles_.back().size() + 1) roles_.emplace_back(names + o);
    kma_free(names);
    log_info("Kmer size is %d.", last_len);
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
  // through the map, report. Here the same reports come out in the same order, while
  //   - GTOs are parsed ahead by a pool of threads (GenomeFeed: the loader skips contig DNA),
  //   - consecutive genomes are concatenated into one native call of >= R residues
  //     (--batch R, default 16M: c4-sized launches instead of ~4k-protein ones; 1,498 vs 1,244
  //     genomes/s over 500 GTOs, profiles/r04_end/bench_genomes.json), made on a caller thread
  //     while the pool parses ahead; --batch 0 instead has each parse worker make its
  //     own genome's call (concurrent host calls on one table: a pooled context and stream
  //     each, include/kmeranno.h),
  //   - the report thread only waits for genome i, then writes its report; batches are called
  //     on a caller thread, so a batch's call overlaps the previous batch's reports.
  void runCommand() {
    if (fasta_) return runFasta();
    const std::vector<std::string> files = genome_files(inDir_);
    log_info("%zu genomes found in input directory.", files.size());
    const auto t0 = Clock::now();
    std::atomic<uint64_t> calls{0}, call_us{0};
    const bool on_workers = batchResidues_ == 0;
    GenomeFeed::After annotate = [&](ParsedGenome& pg) {
      thread_local ProteinBatch b;
      b.clear();
      b.add(pg.pegs);
      call(b, pg, calls, call_us);
    };
    GenomeFeed feed(files, parseThreads_, on_workers ? 4 * (size_t)parseThreads_ : 4 * batchGenomesHint(),
                    on_workers ? annotate : nullptr);
    // Batched mode: a caller thread takes the parsed genomes in order, makes one native call per
    // batch and queues the annotated genomes for the report thread, so batch i + 1's call runs
    // while batch i is reported.
    std::mutex qmu;
    std::condition_variable qcv;
    std::deque<ParsedGenome> ready;
    bool caller_done = false, reports_failed = false;
    std::exception_ptr caller_error;
    double caller_wait_s = 0;
    std::thread caller;
    if (!on_workers) {
      caller = std::thread([&] {
        try {
          const size_t max_ready = 2 * batchGenomesHint();
          ProteinBatch b;
          std::vector<ParsedGenome> batch;
          std::exception_ptr take_error;  // a GTO that failed to parse ends the loop after
          for (size_t i = 0; i < files.size() && !take_error;) {  // the genomes before it
            batch.clear();
            b.clear();
            const auto w0 = Clock::now();
            while (i < files.size() && (batch.empty() || b.residues.size() < batchResidues_)) {
              try {
                batch.push_back(feed.take(i++));
              } catch (...) {
                take_error = std::current_exception();
                break;
              }
              b.add(batch.back().pegs);
            }
            caller_wait_s += seconds(w0);
            if (batch.empty()) break;
            ParsedGenome all;  // the batch's outputs, split back per genome below
            call(b, all, calls, call_us);
            size_t at = 0;
            for (ParsedGenome& pg : batch) {
              const size_t n = pg.pegs.size();
              pg.fid.assign(all.fid.begin() + at, all.fid.begin() + at + n);
              pg.count.assign(all.count.begin() + at, all.count.begin() + at + n);
              pg.status.assign(all.status.begin() + at, all.status.begin() + at + n);
              at += n;
            }
            std::unique_lock<std::mutex> g(qmu);
            qcv.wait(g, [&] { return ready.size() < max_ready || reports_failed; });
            if (reports_failed) break;
            for (ParsedGenome& pg : batch) ready.push_back(std::move(pg));
            g.unlock();
            qcv.notify_all();
          }
          if (take_error) std::rethrow_exception(take_error);
        } catch (...) {
          caller_error = std::current_exception();
        }
        {
          std::lock_guard<std::mutex> g(qmu);
          caller_done = true;
        }
        qcv.notify_all();
      });
    }
    std::vector<ParsedGenome> done;  // reported genomes: freed by the parse workers
    uint64_t n_prot = 0, n_res = 0;
    double wait_s = 0, report_s = 0, free_s = 0;
    struct JoinCaller {  // a failing report stops and joins the caller before unwinding
      std::thread& t;
      std::mutex& mu;
      std::condition_variable& cv;
      bool& failed;
      ~JoinCaller() {
        if (!t.joinable()) return;
        {
          std::lock_guard<std::mutex> g(mu);
          failed = true;
        }
        cv.notify_all();
        t.join();
      }
    } join_caller{caller, qmu, qcv, reports_failed};
    for (size_t i = 0; i < files.size(); ++i) {
      const auto f0 = Clock::now();
      if (done.size() >= 8) feed.recycle(done);
      free_s += seconds(f0);
      const auto w0 = Clock::now();
      if (on_workers) {
        done.push_back(feed.take(i));
      } else {
        std::unique_lock<std::mutex> g(qmu);
        qcv.wait(g, [&] { return !ready.empty() || caller_done; });
        if (ready.empty()) break;  // the caller failed (rethrown below)
        done.push_back(std::move(ready.front()));
        ready.pop_front();
        g.unlock();
        qcv.notify_all();
      }
      wait_s += seconds(w0);
      const auto r0 = Clock::now();
      const ParsedGenome& pg = done.back();
      const Genome& genome = *pg.genome;
      log_info("Processing genome %s (%s).", genome.id.c_str(), genome.name.c_str());
      reporter_->openGenome(genome);
      for (size_t j = 0; j < pg.pegs.size(); ++j)
        if (pg.status[j] == KMA_STATUS_CALLED)  // role != null && !badPeg && count >= minHits
          reporter_->recordFeature(*pg.pegs[j], (uint32_t)pg.fid[j], roles_[pg.fid[j]],
                                   pg.count[j]);
      reporter_->closeGenome();
      n_prot += pg.pegs.size();
      for (const Feature* f : pg.pegs) n_res += f->protein.size();
      report_s += seconds(r0);
    }
    if (caller.joinable()) caller.join();  // (it has queued every genome, or failed)
    if (caller_error) std::rethrow_exception(caller_error);
    feed.recycle(done);
    reporter_->closeReport();
    std::fflush(stdout);
    const double wall = seconds(t0);
    // one machine-readable line on stderr (bench.py's genome-directory workload reads it)
    std::fprintf(stderr,
                 "[kma] apply-stats {\"genomes\": %zu, \"proteins\": %llu, \"residues\": %llu, "
                 "\"calls\": %llu, \"loop_s\": %.6f, \"native_call_s\": %.6f, "
                 "\"report_wait_s\": %.6f, \"report_s\": %.6f, \"free_s\": %.6f, "
                 "\"caller_wait_s\": %.6f, \"calls_on\": \"%s\", "
                 "\"parse_threads\": %d, \"batch_residues\": %llu, \"table_load_s\": %.6f}\n",
                 files.size(), (unsigned long long)n_prot, (unsigned long long)n_res,
                 (unsigned long long)calls.load(), wall, call_us.load() * 1e-6, wait_s, report_s,
                 free_s, caller_wait_s, on_workers ? "parse workers" : "caller thread",
                 feed.threads(), (unsigned long long)batchResidues_, tableLoadS_);
  }

  // One native call on the proteins of `b`; outputs into pg (fid, count, status).
  void call(const ProteinBatch& b, ParsedGenome& pg, std::atomic<uint64_t>& calls,
            std::atomic<uint64_t>& call_us) const {
    call(b.residues, b.offsets, pg, calls, call_us);
  }
  void call(const std::string& residues, const std::vector<uint64_t>& offsets, ParsedGenome& pg,
            std::atomic<uint64_t>& calls, std::atomic<uint64_t>& call_us) const {
    const uint32_t n = (uint32_t)(offsets.size() - 1);
    pg.fid.resize(n);
    pg.count.resize(n);
    pg.status.resize(n);
    if (n == 0) return;
    const auto c0 = Clock::now();
    check(kma_annotate_proteins(table_, reinterpret_cast<const uint8_t*>(residues.data()),
                                offsets.data(), n, minHits_, 0, pg.fid.data(), pg.count.data(),
                                pg.status.data(), nullptr, 0),
          "kma_annotate_proteins");
    pg.annotated = true;
    pg.call_s = seconds(c0);
    calls += 1;
    call_us += (uint64_t)(pg.call_s * 1e6);
  }

  // The FASTA form (protein FASTA as read through FastaInputStream,
  // anno/BuildKmerProcessor.java:196-198; reader rules in host/fasta.h). Each file is one
  // "genome" (id: the file name without its last extension): VERIFY writes one row per called
  // sequence (genome_id, sequence id, role, hits, the header's comment as the function), APPLY
  // one tally row per file. A file is mapped and cut at record headers into segments of about
  // --batch bytes; a pool of threads parses segments and makes one native call per segment
  // (concurrent host calls on one table, each on a pooled context and stream), at most
  // 2 x threads segments ahead of this thread, which writes the segments' rows in file order.
  void runFasta() {
    log_info("%zu FASTA files to process.", fastaFiles_.size());
    const auto t0 = Clock::now();
    const bool verify = outputType_ == "VERIFY";
    // default segments: 4 MiB (--batch), two native calls in flight (--callers): measured on the
    // c4 FASTA file (1M proteins, 355 MB) 0.060-0.064 s per file, 16 MiB x 1 caller 0.064-0.071,
    // 16 MiB x 16 callers 0.24 (concurrent host calls contend for the staging pool and each
    // allocates its own pinned and device buffers; profiles/r05/fasta_sweep.log)
    const size_t seg_bytes = fastaSegment_;
    std::atomic<uint64_t> calls{0}, call_us{0}, parse_us{0}, format_us{0};
    uint64_t n_seq = 0, n_res = 0, n_called = 0, n_bytes = 0, n_segs_all = 0;
    double wait_s = 0, write_s = 0;
    int n_threads = 1;
    struct Segment {
      FastaSegment recs;
      ParsedGenome out;
      std::string text;  // VERIFY rows
      std::string err;
    };
    for (const std::string& path : fastaFiles_) {
      const MappedFile file(path);
      Genome g;
      g.id = g.name = fasta_genome_id(path);
      log_info("Processing FASTA file %s (%s).", path.c_str(), g.id.c_str());
      reporter_->openGenome(g);
      const std::vector<size_t> bounds = fasta_segment_bounds(file.data, file.size, seg_bytes);
      const size_t n_segs = bounds.size() - 1;
      std::vector<Segment> segs(n_segs);
      std::vector<char> ready(n_segs, 0);
      Semaphore callers(callers_);
      std::mutex mu;
      std::condition_variable cv;
      size_t next = 0, taken = 0;
      bool stop = false;
      const size_t lookahead = 2 * (size_t)parseThreads_;
      auto work = [&] {
        for (;;) {
          size_t i;
          {
            std::unique_lock<std::mutex> g(mu);
            cv.wait(g, [&] { return stop || (next < n_segs && next < taken + lookahead); });
            if (stop || next >= n_segs) return;
            i = next++;
          }
          Segment& s = segs[i];
          try {
            const auto p0 = Clock::now();
            parse_fasta_segment(file.data + bounds[i], file.data + bounds[i + 1], s.recs);
            parse_us += (uint64_t)(seconds(p0) * 1e6);
            {
              CallSlot slot(callers);  // at most --callers native calls at once
              call(s.recs.residues, s.recs.offsets, s.out, calls, call_us);
            }
            if (verify) {
              const auto f0 = Clock::now();
              format_verify(g.id, s);
              format_us += (uint64_t)(seconds(f0) * 1e6);
            }
          } catch (const std::exception& e) {
            s.err = *e.what() ? e.what() : "failure";
          }
          {
            std::lock_guard<std::mutex> g(mu);
            ready[i] = 1;
          }
          cv.notify_all();
        }
      };
      std::vector<std::thread> pool;
      n_threads = (int)std::max<size_t>(1, std::min<size_t>((size_t)parseThreads_, n_segs));
      for (int t = 0; t < n_threads; ++t) pool.emplace_back(work);
      struct Join {  // a failing segment stops the pool before unwinding
        std::vector<std::thread>& pool;
        std::mutex& mu;
        std::condition_variable& cv;
        bool& stop;
        ~Join() {
          {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
          }
          cv.notify_all();
          for (auto& t : pool) t.join();
        }
      } join{pool, mu, cv, stop};
      Feature dummy;
      for (size_t i = 0; i < n_segs; ++i) {
        const auto w0 = Clock::now();
        {
          std::unique_lock<std::mutex> g(mu);
          cv.wait(g, [&] { return ready[i] != 0; });
        }
        wait_s += seconds(w0);
        Segment& s = segs[i];
        if (!s.err.empty()) throw std::runtime_error(path + ": " + s.err);
        const auto r0 = Clock::now();
        const uint32_t n = s.recs.size();
        if (verify) {
          std::fwrite(s.text.data(), 1, s.text.size(), stdout);
        } else {
          for (uint32_t j = 0; j < n; ++j)
            if (s.out.status[j] == KMA_STATUS_CALLED)
              reporter_->recordFeature(dummy, (uint32_t)s.out.fid[j], roles_[s.out.fid[j]],
                                       s.out.count[j]);
        }
        for (uint32_t j = 0; j < n; ++j) n_called += s.out.status[j] == KMA_STATUS_CALLED;
        n_seq += n;
        n_res += s.recs.residues.size();
        write_s += seconds(r0);
        {
          std::lock_guard<std::mutex> g(mu);
          taken = i + 1;
        }
        cv.notify_all();
        s = Segment();  // free as we go
      }
      reporter_->closeGenome();
      n_bytes += file.size;
      n_segs_all += n_segs;
    }
    reporter_->closeReport();
    std::fflush(stdout);
    const double wall = seconds(t0);
    std::fprintf(stderr,
                 "[kma] apply-fasta-stats {\"files\": %zu, \"sequences\": %llu, \"residues\": "
                 "%llu, \"called\": %llu, \"bytes\": %llu, \"segments\": %llu, \"calls\": %llu, "
                 "\"loop_s\": %.6f, \"native_call_s\": %.6f, \"parse_s\": %.6f, \"format_s\": "
                 "%.6f, \"report_wait_s\": %.6f, \"write_s\": %.6f, \"threads\": %d, "
                 "\"segment_bytes\": %zu, \"callers\": %d, \"format\": \"%s\", "
                 "\"table_load_s\": %.6f}\n",
                 fastaFiles_.size(), (unsigned long long)n_seq, (unsigned long long)n_res,
                 (unsigned long long)n_called, (unsigned long long)n_bytes,
                 (unsigned long long)n_segs_all, (unsigned long long)calls.load(), wall,
                 call_us.load() * 1e-6, parse_us.load() * 1e-6, format_us.load() * 1e-6, wait_s,
                 write_s, n_threads, seg_bytes, callers_, outputType_.c_str(), tableLoadS_);
  }

  // VerifyApplyKmerReporter's rows (rep/VerifyApplyKmerReporter.java:42-45) of one segment's
  // called sequences: genome_id, peg_id (the FASTA label), role, hits, function (the comment).
  template <class Segment>
  void format_verify(const std::string& gid, Segment& s) const {
    std::string& t = s.text;
    char num[16];
    for (uint32_t j = 0; j < s.recs.size(); ++j) {
      if (s.out.status[j] != KMA_STATUS_CALLED) continue;
      t += gid;
      t += '\t';
      t += s.recs.ids[j];
      t += '\t';
      t += roles_[s.out.fid[j]];
      t += '\t';
      t.append(num, (size_t)std::snprintf(num, sizeof num, "%d", s.out.count[j]));
      t += '\t';
      t += s.recs.comments[j];
      t += '\n';
    }
  }

  // A FASTA file's "genome id": its name without directories and without its last extension.
  static std::string fasta_genome_id(const std::string& path) {
    std::string n = path.substr(path.find_last_of('/') == std::string::npos ? 0 : path.find_last_of('/') + 1);
    const size_t dot = n.find_last_of('.');
    return dot == std::string::npos || dot == 0 ? n : n.substr(0, dot);
  }

  // The FASTA files of a directory (*.faa, *.fa, *.fasta), sorted by name.
  static std::vector<std::string> fasta_files(const std::string& dir) {
    std::vector<std::string> out;
    for (const char* ext : {".faa", ".fa", ".fasta"})
      for (const std::string& f : files_with_suffix(dir, ext)) out.push_back(f);
    std::sort(out.begin(), out.end());
    return out;
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
  int parseThreads_ = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  int stagingThreads_ = -1;  // KMA_OPT_HOST_THREADS for this run (-1: the library's default)
  int callers_ = 2;          // FASTA form: native calls in flight at once
  size_t fastaSegment_ = (size_t)4 << 20;  // FASTA form: bytes per segment (--batch)
  uint64_t batchResidues_ = 16u << 20;  // 0: a native call per genome on its parse worker
  double tableLoadS_ = 0;
  std::string kmerDbFile_, goodRoleFile_, inDir_;
  const bool fasta_;
  std::vector<std::string> fastaInputs_, fastaFiles_;
  std::unique_ptr<ApplyKmerReporter> reporter_;
  std::vector<std::string> roles_;  // fid -> role id (kmerdb.tbl's first-seen order)
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
    " --threads N       GTO parser threads (default min(16, cores))\n"
    " --staging-threads N  library threads packing a call's residues (default: min(16, cores))\n"
    " --batch R         consecutive genomes batched into native calls of >= R residues\n"
    "                   (default 16777216); 0: each parser thread makes its genome's call\n";

const char* kApplyFastaUsage =
    "kma apply-fasta [options] kmerdb.tbl roles.in.use proteins.faa|dir ...\n"
    "  apply a discriminating-kmer database to protein FASTA files (each file: one genome)\n"
    " -h, --help        display command-line usage\n"
    " -v, --verbose     display more frequent progress messages on the log\n"
    " -m, --min N       minimum number of hits required to call a role (default 5)\n"
    " --format FMT      VERIFY (default): a row per called sequence; APPLY: a row per file\n"
    " --device D        HIP device ordinal (default 0)\n"
    " --threads N       parser / caller threads (default min(16, cores))\n"
    " --staging-threads N  library threads packing a call's residues (default: min(16, cores))\n"
    " --batch B         bytes of FASTA per segment (one native call each; default 4194304)\n"
    " --callers C       segments' native calls in flight at once (default 2)\n";

int run_apply(const std::vector<std::string>& args, bool fasta = false) {
  ApplyKmerProcessor p(fasta);
  p.parseCommand(args);
  if (p.help()) {
    std::fputs(fasta ? kApplyFastaUsage : kApplyUsage, stderr);
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

// `kma gto-dump file.gto`: what apply's loader reads from a GTO, one feature per line (id, type,
// function, protein), after the genome's id, name and genetic code; no device needed (tests
// compare it with a JSON library's reading).
int run_gto_dump(const std::vector<std::string>& args) {
  if (args.size() != 1) throw UsageError("usage: kma gto-dump file.gto");
  const Genome g = load_genome_pegs(args[0]);
  std::printf("%s\t%s\t%d\n", g.id.c_str(), g.name.c_str(), g.genetic_code);
  for (const Feature& f : g.features)
    std::printf("%s\t%s\t%s\t%s\n", f.id.c_str(), f.type.c_str(), f.function.c_str(),
                f.protein.c_str());
  return 0;
}

// `kma fasta-dump [--batch B] file.faa`: the records the FASTA form reads (host/fasta.h), one
// per line (label, comment, sequence), parsed in segments of about B bytes (default 16 MiB) as
// apply-fasta cuts them; no device needed (tests compare it with a restatement of the reader).
int run_fasta_dump(const std::vector<std::string>& args) {
  size_t seg = (size_t)16 << 20;
  std::vector<std::string> pos;
  for (size_t i = 0; i < args.size(); ++i) {
    if (args[i] == "--batch" && i + 1 < args.size()) seg = std::strtoull(args[++i].c_str(), nullptr, 10);
    else pos.push_back(args[i]);
  }
  if (pos.size() != 1) throw UsageError("usage: kma fasta-dump [--batch B] file.faa");
  if (!can_read(pos[0])) throw NotFound("Input FASTA file " + pos[0] + " not found or unreadable.");
  const MappedFile file(pos[0]);
  const std::vector<size_t> b = fasta_segment_bounds(file.data, file.size, seg);
  std::string out;
  for (size_t i = 0; i + 1 < b.size(); ++i) {
    FastaSegment s;
    parse_fasta_segment(file.data + b[i], file.data + b[i + 1], s);
    for (uint32_t j = 0; j < s.size(); ++j) {
      out.append(s.ids[j]);
      out += '\t';
      out.append(s.comments[j]);
      out += '\t';
      out.append(s.residues, s.offsets[j], s.offsets[j + 1] - s.offsets[j]);
      out += '\n';
    }
  }
  std::fwrite(out.data(), 1, out.size(), stdout);
  std::fprintf(stderr, "[kma] fasta-dump segments %zu\n", b.size() - 1);
  return 0;
}

const char* kCommands =
    "Valid commands are\n"
    "  apply     apply a discriminating-kmer database to genomes to create a role-count file\n"
    "  apply-fasta  the same on protein FASTA files (a row per called sequence)\n"
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
    if (command == "apply-fasta") return run_apply(rest, true);
    if (command == "contigs") return run_contigs(rest);
    if (command == "gto-dump") return run_gto_dump(rest);
    if (command == "fasta-dump") return run_fasta_dump(rest);
    if (command == "-h" || command == "--help") {
      std::fputs(kCommands, stdout);
      return 0;
    }
    std::fprintf(stderr, "Invalid command %s.\n", command.c_str());  // App.java:301
    return 1;
  } catch (const UsageError& e) {
    std::fprintf(stderr, "%s\n%s", e.what(),
                 command == "apply" ? kApplyUsage : command == "apply-fasta" ? kApplyFastaUsage : "");
    return 2;
  } catch (const NotFound& e) {
    std::fprintf(stderr, "java.io.FileNotFoundException: %s\n", e.what());
    return 1;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
}
