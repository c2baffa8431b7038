// kma_abi.cpp — the C ABI of libkmeranno.so (declared in include/kmeranno.h).
//
// Host-side orchestration only: argument checks, key packing, device allocation and copies,
// replica management and kernel launches (kma_kernels.hip). No compute falls back to the CPU:
// without a usable HIP device every entry point that needs one returns KMA_E_DEVICE.
//
// Host entry points (kma_annotate_proteins / kma_annotate_contigs) reuse per-table host
// contexts — a stream, a workspace, device buffers and pinned staging buffers per device —
// taken from the table's pool for the duration of one call, so a per-genome caller pays no
// allocation and concurrent callers never synchronise each other (each waits on its own
// stream only). A table may be replicated on several devices; a host call then cuts its batch
// into residue-balanced contiguous shards, one host thread per replica.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kmeranno.h"
#include "kma_distance.h"
#include "kma_hashanno.h"
#include "kma_internal.h"
#include "kma_pack.h"
#include "kma_tsv.h"

namespace {
// ---- options (kma_option_set; include/kmeranno.h) ----------------------------------------------
// Library-wide defaults, read per call; workspaces may override the protein-kernel ones. The
// environment is read only by tuning builds (-DKMA_TUNING_ENV=1, the A/B scripts' variants):
// a library a JVM loads must not change its kernel geometry because of a stray variable.
constexpr int kNumOpts = 11;
std::atomic<int64_t> g_opt[kNumOpts] = {{0}, {-1}, {0}, {-1}, {0}, {0}, {1}, {0}, {0}, {-1}, {0}};
constexpr int64_t kOptUnset = INT64_MIN;  // workspace override not set: the library default

bool option_valid(int opt, int64_t v) {
  switch (opt) {
    case KMA_OPT_LAYOUT: return v == -1 || v == 0 || v == 6 || v == 7 || v == (6 | kma::kOrderMod);
    case KMA_OPT_BLOCK_PROTEINS: return v >= 0 && v <= kma::kBlockProteins;
    case KMA_OPT_DEFER: return v >= -1 && v <= 64;
    case KMA_OPT_HOST_PIECES: return v >= 0 && v <= 16;
    case KMA_OPT_HASH_SLICE: return v >= 0;
    case KMA_OPT_PACKED_INPUT: return v >= 0 && v <= 2;
    case KMA_OPT_HOST_THREADS: return v >= 0 && v <= 64;
    case KMA_OPT_HOST_SLICE: return v >= 0 && v <= (int64_t)((1ull << 32) - 128);  // a call's limit
    case KMA_OPT_HOST_PIECE_MIN: return v >= 0 && v <= (int64_t)(1ull << 32);
    case KMA_OPT_PLACEMENT: return v >= -1 && v <= 1;
    default: return false;
  }
}

#if KMA_TUNING_ENV
struct EnvOptions {  // tuning builds: the A/B scripts' variables seed the defaults once
  EnvOptions() {
    const std::pair<const char*, int> vars[] = {
        {"KMA_MINIMIZER", KMA_OPT_LAYOUT}, {"KMA_BLOCK_PROTEINS", KMA_OPT_BLOCK_PROTEINS},
        {"KMA_DEFER", KMA_OPT_DEFER}, {"KMA_HOST_PIECES", KMA_OPT_HOST_PIECES},
        {"KMA_HASH_SLICE", KMA_OPT_HASH_SLICE}, {"KMA_PACKED_INPUT", KMA_OPT_PACKED_INPUT},
        {"KMA_HOST_THREADS", KMA_OPT_HOST_THREADS}, {"KMA_PLACEMENT", KMA_OPT_PLACEMENT}};
    for (const auto& [name, opt] : vars)
      if (const char* e = getenv(name); e && *e) {
        const int64_t v = strtoll(e, nullptr, 10);
        if (option_valid(opt, v)) g_opt[opt] = v;
      }
  }
} g_env_options;
#endif

int64_t opt(int o) { return g_opt[o].load(std::memory_order_relaxed); }

// MI355X's Infinity Cache (MALL): tables larger than this are probed from HBM.
constexpr uint64_t kInfinityCacheBytes = 256ull << 20;

// The forced table layout (KMA_OPT_LAYOUT): -1 = not forced.
int forced_layout() { return (int)opt(KMA_OPT_LAYOUT); }
// Table creators try two-choice placement first for narrow tables (KMA_OPT_PLACEMENT -1 / 1);
// 0 builds chains only.
bool two_choice_first(int k) { return !kma::wide_k(k) && opt(KMA_OPT_PLACEMENT) != 0; }

// CPUs this process may use: its affinity mask, bounded by a cgroup CPU quota (a container or a
// GPU box granted a share of a machine lists every CPU of the machine in the mask).
long cgroup_quota_cpus() {
  auto ceil_div = [](long long q, long long p) { return (long)((q + p - 1) / p); };
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {  // v2: "<quota|max> <period>"
    char q[32] = {};
    long long period = 0;
    const bool ok = fscanf(f, "%31s %lld", q, &period) == 2;
    fclose(f);
    if (ok && strcmp(q, "max") != 0 && period > 0 && atoll(q) > 0) return ceil_div(atoll(q), period);
    return 0;
  }
  long long quota = -1, period = 0;
  if (FILE* f = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {  // v1
    if (fscanf(f, "%lld", &quota) != 1) quota = -1;
    fclose(f);
  }
  if (FILE* f = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
    if (fscanf(f, "%lld", &period) != 1) period = 0;
    fclose(f);
  }
  return quota > 0 && period > 0 ? ceil_div(quota, period) : 0;
}
size_t host_cores() {
  static const size_t n = [] {
    size_t c = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) == 0 && CPU_COUNT(&set) > 0) c = (size_t)CPU_COUNT(&set);
    const long q = cgroup_quota_cpus();
    return q > 0 ? std::min(c, (size_t)q) : c;
  }();
  return n;
}

// Host threads one staging job (a replica's share of a host call) stages (copies or packs) its
// input with. KMA_OPT_HOST_THREADS is the whole call's budget, split over the replicas the call
// fans out to; by default each of n replicas takes host_cores() / n, at most 16 (packing 5 bits
// per residue keeps up with one PCIe link on ~16 threads). Round 5 gave every replica min(16,
// cores): an 8-replica call ran 8 jobs of 16 on one pool of at most 63 threads.
size_t staging_width(int n_replicas) {
  const size_t n = (size_t)std::max(1, n_replicas);
  const int64_t o = opt(KMA_OPT_HOST_THREADS);
  if (o > 0) return std::max<size_t>(1, (size_t)o / n);
  return std::clamp<size_t>(host_cores() / n, 1, 16);
}
// The width of the staging jobs of the calling thread: set for a replica's shard thread by the
// host call that fans out (ShardWidth), else a one-replica call's.
thread_local size_t t_shard_width = 0;
size_t staging_threads() { return t_shard_width ? t_shard_width : staging_width(1); }
struct ShardWidth {
  explicit ShardWidth(size_t w) { t_shard_width = w; }
  ~ShardWidth() { t_shard_width = 0; }
};

// Library-wide pool of staging threads (grown on demand, never shrunk; threads sleep when idle).
// run(n, width, fn) calls fn(0..n-1) on the calling thread plus up to width - 1 pool threads and
// returns when every call has returned. Several host calls may run jobs at once (kma apply's
// workers each stage their own batch; a replicated table's host call stages every replica's
// share at once): pool threads take the oldest job with free width, and a caller always works on
// its own job, so every job finishes even when the pool is busy. The pool grows to the summed
// width of the jobs running at once (round 5 grew it to one job's width: 8 replicas' jobs of 16
// shared at most 63 threads). Round 3 and early round 4 spawned threads per staging piece: a c5
// host call spent milliseconds creating ~120 threads, and pieces of 5 chunks kept 5 of 16
// threads busy.
class StagingPool {
 public:
  template <class F>
  void run(uint64_t n, size_t width, F&& fn) {
    run_with(n, width, std::forward<F>(fn), [](auto& help) { while (help()) {} });
  }
  // run() whose calling thread runs caller(help) instead of draining the job: help() makes one
  // of the job's calls (in index order with the pool threads) on the calling thread and returns
  // false once every call has been taken. The calling thread can so act on the job's progress
  // (the host call issues each segment's copy as soon as its chunks are packed) and help
  // whenever it would otherwise wait. Returns after every call has returned.
  template <class F, class C>
  void run_with(uint64_t n, size_t width, F&& fn, C&& caller) {
    width = std::max<size_t>(1, std::min<size_t>(width, n));
    Job j;
    j.n = n;
    j.width = width;
    j.call = [](void* f, uint64_t i) { (*static_cast<std::remove_reference_t<F>*>(f))(i); };
    j.fn = (void*)&fn;
    if (width > 1) {
      std::lock_guard<std::mutex> g(mu_);
      demand_ += width - 1;
      while (threads_.size() < demand_ && threads_.size() < kMaxThreads)
        threads_.emplace_back([this] { worker(); });
      jobs_.push_back(&j);
      cv_.notify_all();
    }
    auto help = [&j]() {
      const uint64_t i = j.next.fetch_add(1);
      if (i >= j.n) return false;
      j.call(j.fn, i);
      return true;
    };
    caller(help);
    drain(j);
    if (width > 1) {
      std::unique_lock<std::mutex> lk(mu_);
      jobs_.erase(std::remove(jobs_.begin(), jobs_.end(), &j), jobs_.end());
      demand_ -= width - 1;
      done_cv_.wait(lk, [&] { return j.active == 0; });
    }
  }
  ~StagingPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
      cv_.notify_all();
    }
    for (auto& t : threads_) t.join();
  }

 private:
  static constexpr size_t kMaxThreads = 255;
  struct Job {
    uint64_t n = 0;
    size_t width = 1;
    size_t active = 0;  // pool threads inside drain() (guarded by mu_)
    std::atomic<uint64_t> next{0};
    void (*call)(void*, uint64_t) = nullptr;
    void* fn = nullptr;
  };
  static void drain(Job& j) {
    for (uint64_t i; (i = j.next.fetch_add(1)) < j.n;) j.call(j.fn, i);
  }
  void worker() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      Job* j = nullptr;
      cv_.wait(lk, [&] {
        if (stop_) return true;
        for (Job* c : jobs_)
          if (c->active + 1 < c->width && c->next.load() < c->n) return (j = c) != nullptr;
        return false;
      });
      if (stop_) return;
      ++j->active;
      lk.unlock();
      drain(*j);
      lk.lock();
      if (--j->active == 0) done_cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<Job*> jobs_;
  std::vector<std::thread> threads_;
  size_t demand_ = 0;  // summed width - 1 of the jobs running (guarded by mu_)
  bool stop_ = false;
};

StagingPool& staging_pool() {
  static StagingPool* pool = new StagingPool();  // never destroyed: no join at process exit
  return *pool;
}

// dst[i] = src[i] - base for i < n, on the staging pool for large n (a host call's rebased
// offsets: 8 MB for c5's 1M proteins).
void rebase_offsets(uint64_t* dst, const uint64_t* src, uint64_t n, uint64_t base) {
  constexpr uint64_t kChunk = 1u << 17;
  staging_pool().run((n + kChunk - 1) / kChunk, n >= 4 * kChunk ? staging_threads() : 1,
                     [&](uint64_t c) {
                       const uint64_t e = std::min(n, (c + 1) * kChunk);
                       for (uint64_t i = c * kChunk; i < e; ++i) dst[i] = src[i] - base;
                     });
}

// The first s < n with offsets[s + 1] < offsets[s], or n: chunks on the staging pool, each a
// branch-free (vectorized) pass (c5's 1M offsets: a serial scan with an early exit per element
// ran ~0.5 ms before the call's first copy).
uint32_t offsets_decrease_at(const uint64_t* offsets, uint32_t n) {
  constexpr uint64_t kChunk = 1u << 16;
  const uint64_t n_chunks = (n + kChunk - 1) / kChunk;
  std::vector<uint8_t> bad(n_chunks);
  staging_pool().run(n_chunks, n >= 4 * kChunk ? staging_threads() : 1, [&](uint64_t c) {
    const uint64_t e = std::min<uint64_t>(n, (c + 1) * kChunk);
    uint64_t b = 0;
    for (uint64_t i = c * kChunk; i < e; ++i) b |= offsets[i + 1] < offsets[i];
    bad[c] = b != 0;
  });
  for (uint64_t c = 0; c < n_chunks; ++c)
    if (bad[c])
      for (uint64_t i = c * kChunk; i < n; ++i)
        if (offsets[i + 1] < offsets[i]) return (uint32_t)i;
  return n;
}

// memcpy on the staging pool in 1 MiB chunks (the outputs of a large host call).
void pool_memcpy(void* dst, const void* src, size_t n) {
  constexpr size_t kChunk = 1u << 20;
  staging_pool().run((n + kChunk - 1) / kChunk, n >= 4 * kChunk ? staging_threads() : 1,
                     [&](uint64_t c) {
                       const size_t o = c * kChunk;
                       std::memcpy(static_cast<uint8_t*>(dst) + o,
                                   static_cast<const uint8_t*>(src) + o, std::min(kChunk, n - o));
                     });
}
}  // namespace

// The size rule's minimizer code (m | order): m = min(K, 6) up to kMinimizer6Buckets buckets,
// else min(K, 7); K = 8, m = 6 tables take the mod-sampling order (kma_internal.h kOrderMod:
// fewer home-line requests per window). Until the order's single-residue form and the cheaper
// bucket match it was kept to tables beyond the Infinity Cache (its VALU slowed the 6-frame
// probe on the cache-resident 10^7 table); since then the 10^7 table measures c4 2.284 vs
// 2.763 ms, c2 42.4-42.8 vs 43.4-43.6 us, c3's probe 72.7-72.8 vs 72.9-73.2 us in it
// (profiles/r06/order_small_tables_r06j/). KMA_OPT_LAYOUT forces a code (6: the random order).
int kma::minimizer_len(int k, uint64_t n_buckets) {
  const int m6 = k < 6 ? k : 6, m7 = k < 7 ? k : 7;
  const int f = forced_layout();
  if (f == 0) return 0;
  if (f == 6) return m6;
  if (f == 7) return m7;
  if (f == (6 | kma::kOrderMod)) return kma::order_mod_valid(k, 6) ? 6 | kma::kOrderMod : m6;
  const uint64_t lim = kma::wide_k(k) ? kma::kMinimizer6BucketsWide : kma::kMinimizer6Buckets;
  const int m = n_buckets <= lim ? m6 : m7;
  return kma::order_mod_valid(k, m) ? m | kma::kOrderMod : m;
}

namespace {

constexpr uint64_t kResPad = 64;            // workspace positions past the last residue
constexpr uint64_t kMaxResidues = (1ull << 32) - 2 * kResPad;  // positions are u32 in kernels
using kma::kMaxBuckets;
constexpr uint32_t kTimingRing = 256;
constexpr int kMaxEv = 8;  // events per timed call

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define KMA_HIP(call)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (call);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(e_ == hipErrorOutOfMemory ? KMA_E_NOMEM : KMA_E_DEVICE, "%s: %s (%s:%d)", \
                  #call, hipGetErrorString(e_), __FILE__, __LINE__);                    \
  } while (0)

// Make `device` current for the scope; restore the caller's device after (torch keeps its own).
struct DeviceScope {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceScope(int device) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    err = hipSetDevice(device);
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// Device buffers freed on scope exit (one-shot builders only).
struct DevBufs {
  std::vector<void*> p;
  ~DevBufs() {
    for (void* q : p) (void)hipFree(q);
  }
  template <class T>
  hipError_t alloc(T** out, size_t bytes) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, bytes ? bytes : 1);
    if (e == hipSuccess) p.push_back(q);
    *out = static_cast<T*>(q);
    return e;
  }
};

// A device buffer that only grows (host contexts).
template <class T>
struct Grow {
  T* p = nullptr;
  size_t cap = 0;  // elements
  hipError_t reserve(size_t n) {
    if (p && n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n + n / 4, 256);
    hipError_t e = hipMalloc(&p, want * sizeof(T));
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};
// Pinned host staging that only grows.
struct Pinned {
  uint8_t* p = nullptr;
  size_t cap = 0;
  hipError_t reserve(size_t n) {
    if (p && n <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n + n / 4, 4096);
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), want, hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

void standard_lut(uint8_t lut[256]) {
  std::memset(lut, 0, 256);
  for (int c = 'A'; c <= 'Z'; ++c) lut[c] = (uint8_t)(c - 'A' + 1);
  lut[(uint8_t)'*'] = 27;
}

int check_k(int k) {
  if (k < 1 || k > KMA_MAX_K) return fail(KMA_E_INVALID, "kmer size %d outside 1..%d", k, KMA_MAX_K);
  return KMA_OK;
}

// Slot array geometry of a table of K-mers: narrow (K <= 8, kSlotsPerBucket u64 slots per
// bucket) or wide (K 9..12, four 16-byte slots per 64-byte bucket; kma_internal.h).
uint64_t bucket_bytes(int k) { return kma::wide_k(k) ? 64u : (uint64_t)kma::kBucketBytes; }
uint64_t buckets_for_k(uint64_t n_keys, double load_factor, int k) {
  if (load_factor <= 0) load_factor = 0.5;
  const int spb = kma::slots_for_k(k);
  const double slots = (double)(n_keys ? n_keys : 1) / load_factor;
  const uint64_t nb = (uint64_t)((slots + spb - 1) / spb);
  return nb < 1 ? 1 : nb;
}

// Pack rows [lo, hi) with the LUT; 0 for rows of the wrong length or with unencodable bytes.
void pack_rows(const uint8_t* lut, const char* text, const uint64_t* off, uint64_t lo, uint64_t hi,
               int k, uint64_t* keys) {
  for (uint64_t r = lo; r < hi; ++r) {
    const uint64_t b = off[r], e = off[r + 1];
    uint64_t key = 0;
    if (e - b == (uint64_t)k) {
      for (int j = 0; j < k; ++j) {
        const uint8_t c = lut[(uint8_t)text[b + j]];
        if (!c) {
          key = 0;
          break;
        }
        key = (key << 5) | c;
      }
    }
    keys[r] = key;
  }
}

template <class F>
void parallel_rows(uint64_t n, F f) {
  unsigned nt = (unsigned)std::min<size_t>(16, host_cores());
  if (n < (1u << 16)) nt = 1;
  std::vector<std::thread> th;
  const uint64_t chunk = (n + nt - 1) / nt;
  for (unsigned t = 0; t < nt; ++t) {
    const uint64_t lo = t * chunk, hi = std::min(n, lo + chunk);
    if (lo < hi) th.emplace_back(f, lo, hi);
  }
  for (auto& x : th) x.join();
}

// NCBI translation tables, codons in T, C, A, G order.
const char* ncbi_code(int gc) {
  switch (gc) {
    case 1: case 11: return "FFLLSSSSYY**CC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG";
    case 2: return "FFLLSSSSYY**CCWWLLLLPPPPHHQQRRRRIIMMTTTTNNKKSS**VVVVAAAADDEEGGGG";
    case 3: return "FFLLSSSSYY**CCWWTTTTPPPPHHQQRRRRIIMMTTTTNNKKSSRRVVVVAAAADDEEGGGG";
    case 4: return "FFLLSSSSYY**CCWWLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG";
    case 5: return "FFLLSSSSYY**CCWWLLLLPPPPHHQQRRRRIIMMTTTTNNKKSSSSVVVVAAAADDEEGGGG";
    case 6: return "FFLLSSSSYYQQCC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG";
    case 9: return "FFLLSSSSYY**CCWWLLLLPPPPHHQQRRRRIIIMTTTTNNNKSSSSVVVVAAAADDEEGGGG";
    case 10: return "FFLLSSSSYY**CCCWLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG";
    case 12: return "FFLLSSSSYY**CC*WLLLSPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG";
    case 13: return "FFLLSSSSYY**CCWWLLLLPPPPHHQQRRRRIIMMTTTTNNKKSSGGVVVVAAAADDEEGGGG";
    case 14: return "FFLLSSSSYYY*CCWWLLLLPPPPHHQQRRRRIIIMTTTTNNNKSSSSVVVVAAAADDEEGGGG";
    case 16: return "FFLLSSSSYY*LCC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG";
    case 21: return "FFLLSSSSYY**CCWWLLLLPPPPHHQQRRRRIIMMTTTTNNNKSSSSVVVVAAAADDEEGGGG";
    case 22: return "FFLLSS*SYY*LCC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG";
    case 23: return "FF*LSSSSYY**CC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG";
    case 24: return "FFLLSSSSYY**CCWWLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSSKVVVVAAAADDEEGGGG";
    case 25: return "FFLLSSSSYY**CCGWLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG";
    default: return nullptr;
  }
}

// Contiguous shards [b[i], b[i+1]) of n units (proteins, contigs) with near-equal payload
// (residues, bases): cut where the payload prefix crosses i/parts of the total.
std::vector<uint32_t> shard_bounds(const uint64_t* off, uint32_t n, int parts) {
  std::vector<uint32_t> b(parts + 1, 0);
  b[parts] = n;
  const uint64_t base = off[0], total = off[n] - base;
  for (int i = 1; i < parts; ++i) {
    const uint64_t target = base + (uint64_t)((double)total * i / parts);
    const uint64_t* it = std::lower_bound(off + 1, off + n + 1, target);
    b[i] = std::max(b[i - 1], std::min(n, (uint32_t)(it - off)));
  }
  return b;
}

}  // namespace

// ---- objects ---------------------------------------------------------------------------------
struct kma_workspace {
  int device = 0;
  int n_cu = 256;
  uint32_t* d_gset = nullptr;  // protein sets that do not fit in LDS: 2 u32 per residue
  uint8_t* d_packed = nullptr; // the call's residues packed (kma_internal.h packed_bytes)
  bool host_ctx = false;       // a host context's workspace: no d_packed (kma_annotate_proteins)
  uint64_t res_cap = 0;        // residues per call
  // 6-frame path (kma_workspace_reserve_contigs): staged hits, block counts, scan.
  kma_hit* d_cstage = nullptr;
  uint32_t* d_ccounts = nullptr;
  // Emit-offset group sums (cgroups u64) and the emit pass's done counter (one u64 after
  // them): zero between calls — the probe adds into the sums, the emit pass's last block
  // zeroes both — so a call keeps no host state and may be graph-captured.
  uint64_t* d_cprefix = nullptr;
  uint64_t cgroups = 0;
  bool cpending = false;  // a probe was set up whose emit pass has not been enqueued
  uint64_t contig_cap = 0;  // bases
  // Per-workspace overrides of KMA_OPT_BLOCK_PROTEINS / KMA_OPT_DEFER (kOptUnset: the default).
  int64_t opt_block_proteins = kOptUnset;
  int64_t opt_defer = kOptUnset;
  // Per-phase timing (kma_workspace_timing): a ring of calls, each kMaxEv events (phase i runs
  // from event i to event i + 1) and its phase names.
  bool timing = false;
  std::vector<hipEvent_t> events;
  std::vector<const char* const*> names;  // per ring slot
  std::vector<int> n_phases;              // per ring slot
  uint32_t n_timed = 0;
};

namespace {
// One replica of a table's slot array on one device.
struct Replica {
  int device = 0;
  uint64_t* d_slots = nullptr;
  bool owned = false;
  uint8_t* d_lut = nullptr;
};

// Per-call resources of the host entry points on one device (kept in the table's pool).
constexpr int kMaxPieces = 16;  // host protein calls: H2D / kernel pipeline depth (events)
struct HostCtx {
  int device = 0;
  hipStream_t stream = nullptr;
  // H2D of piece i + 1 under the kernel of piece i, pieces alternating over two copy streams
  // (two DMA engines: 57 vs 50 GB/s for c5's packed stream, profiles/r04/link_r04g.json)
  hipStream_t copy[2] = {};
  hipStream_t d2h = nullptr;  // pieces' outputs back while later pieces copy and run
  hipEvent_t piece_ready[kMaxPieces] = {};
  hipEvent_t piece_ready2[kMaxPieces] = {};  // streamed copies: piece i's data on copy[1]
  hipEvent_t piece_done[kMaxPieces] = {};  // piece i's kernel (on `stream`)
  hipEvent_t out_ready[kMaxPieces] = {};   // piece i's outputs in pinned memory (on d2h)
  kma_workspace* ws = nullptr;
  Grow<uint8_t> d_in;     // residues / DNA (+ padding)
  Grow<uint64_t> d_off;   // offsets
  Grow<uint8_t> d_out;    // outputs (fid, count, tally, status / hit count, tally)
  Grow<uint32_t> d_aux;   // 6-frame STRICT: locations per table slot
  Grow<kma_hit> d_hits;   // 6-frame hits
  Pinned h_in, h_out;     // pinned staging for both directions
};
}  // namespace

struct kma_table {
  int k = 8;
  int mlen = 6;  // layout: minimizer length, 0 = flat
  bool two_choice = false;  // placement (kma_internal.h alt_bucket): else overflow chains
  uint64_t n_buckets = 0;
  uint8_t lut[256] = {};
  kma_table_info info = {};
  // Replicas: appended by kma_table_replicate while host or device calls may run on the table,
  // so they are read and appended under reps_mu; calls work on a copy (replicas() below).
  std::vector<Replica> reps;
  mutable std::mutex reps_mu;
  std::mutex pool_mu;
  std::vector<HostCtx*> idle;  // host contexts not in use
};

extern "C" int kma_workspace_destroy(kma_workspace* ws);
extern "C" int kma_workspace_create(int device, kma_workspace** out);

namespace {

void destroy_ctx(HostCtx* c) {
  DeviceScope ds(c->device);
  if (c->ws) kma_workspace_destroy(c->ws);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  for (hipStream_t cs : c->copy)
    if (cs) (void)hipStreamDestroy(cs);
  if (c->d2h) (void)hipStreamDestroy(c->d2h);
  for (hipEvent_t* ev : {c->piece_ready, c->piece_ready2, c->piece_done, c->out_ready})
    for (int i = 0; i < kMaxPieces; ++i)
      if (ev[i]) (void)hipEventDestroy(ev[i]);
  c->d_in.release();
  c->d_off.release();
  c->d_out.release();
  c->d_aux.release();
  c->d_hits.release();
  c->h_in.release();
  c->h_out.release();
  delete c;
}

// Take a host context for `device` from the table's pool (or make one).
int acquire_ctx(kma_table* t, int device, HostCtx** out) {
  {
    std::lock_guard<std::mutex> g(t->pool_mu);
    for (size_t i = 0; i < t->idle.size(); ++i)
      if (t->idle[i]->device == device) {
        *out = t->idle[i];
        t->idle.erase(t->idle.begin() + i);
        return KMA_OK;
      }
  }
  DeviceScope ds(device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", device);
  HostCtx* c = new HostCtx();
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  for (hipStream_t& cs : c->copy)
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&cs, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->d2h, hipStreamNonBlocking);
  for (hipEvent_t* ev : {c->piece_ready, c->piece_ready2, c->piece_done, c->out_ready})
    for (int i = 0; i < kMaxPieces && e == hipSuccess; ++i)
      e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
  if (e != hipSuccess) {
    destroy_ctx(c);
    return fail(KMA_E_DEVICE, "stream / event create: %s", hipGetErrorString(e));
  }
  if (int rc = kma_workspace_create(device, &c->ws)) {
    destroy_ctx(c);
    return rc;
  }
  c->ws->host_ctx = true;
  *out = c;
  return KMA_OK;
}
void release_ctx(kma_table* t, HostCtx* c) {
  std::lock_guard<std::mutex> g(t->pool_mu);
  t->idle.push_back(c);
}
struct CtxGuard {
  kma_table* t;
  HostCtx* c;
  ~CtxGuard() {
    if (!c) return;
    // A call that failed after queueing work returns early: let the context's copies and
    // kernels drain before the next call reuses its pinned and device buffers.
    for (hipStream_t cs : c->copy) (void)hipStreamSynchronize(cs);
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->d2h);
    release_ctx(t, c);
  }
};

// A copy of the table's replicas (safe against a concurrent kma_table_replicate).
std::vector<Replica> replicas(const kma_table* t) {
  std::lock_guard<std::mutex> g(t->reps_mu);
  return t->reps;
}
bool replica_on(const kma_table* t, int device, Replica* out) {
  std::lock_guard<std::mutex> g(t->reps_mu);
  for (const Replica& r : t->reps)
    if (r.device == device) {
      *out = r;
      return true;
    }
  return false;
}

int add_replica(kma_table* t, int device, uint64_t* d_slots, bool owned) {
  Replica r;
  r.device = device;
  r.d_slots = d_slots;
  r.owned = owned;
  DeviceScope ds(device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", device);
  hipError_t e = hipMalloc(&r.d_lut, 256);
  if (e == hipSuccess) e = hipMemcpy(r.d_lut, t->lut, 256, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (r.d_lut) (void)hipFree(r.d_lut);
    return fail(KMA_E_DEVICE, "table LUT upload: %s", hipGetErrorString(e));
  }
  std::lock_guard<std::mutex> g(t->reps_mu);
  t->reps.push_back(r);
  t->info.n_replicas = (int32_t)t->reps.size();
  return KMA_OK;
}

kma_table* new_table(int device, int k, int m, uint64_t n_buckets, const uint8_t lut[256],
                     bool two_choice = false) {
  kma_table* t = new kma_table();
  t->k = k;
  t->mlen = m;
  t->two_choice = two_choice;
  t->info.two_choice = two_choice ? 1 : 0;
  t->n_buckets = n_buckets;
  std::memcpy(t->lut, lut, 256);
  t->info.n_buckets = n_buckets;
  t->info.bytes = n_buckets * bucket_bytes(k);
  t->info.slots_per_bucket = kma::slots_for_k(k);
  t->info.k = k;
  t->info.device = device;
  t->info.minimizer_len = m & kma::kMinimizerMask;
  t->info.minimizer_order = (m & kma::kOrderMod) ? 1 : 0;
  int ne = 0;
  for (int c = 0; c < 256; ++c)
    if (lut[c] >= 28) t->info.extra_syms[lut[c] - 28] = (uint8_t)c, ++ne;
  t->info.n_extra_syms = ne;
  return t;
}

void free_table(kma_table* t) {
  for (HostCtx* c : t->idle) destroy_ctx(c);
  for (Replica& r : t->reps) {
    DeviceScope ds(r.device);
    if (r.owned && r.d_slots) (void)hipFree(r.d_slots);
    if (r.d_lut) (void)hipFree(r.d_lut);
  }
  delete t;
}

int build_on_device(uint64_t* d_slots, uint64_t n_buckets, int k, int m, uint32_t* d_winner,
                    const uint64_t* d_keys, const uint32_t* d_fids, uint64_t n, uint32_t* d_status,
                    hipStream_t s) {
  if (n_buckets >= kMaxBuckets) return fail(KMA_E_INVALID, "%llu buckets or more",
                                           (unsigned long long)kMaxBuckets);
  KMA_HIP(hipMemsetAsync(d_slots, 0, n_buckets * bucket_bytes(k), s));
  KMA_HIP(hipMemsetAsync(d_winner, 0, n_buckets * kma::slots_for_k(k) * sizeof(uint32_t), s));
  KMA_HIP(hipMemsetAsync(d_status, 0, 4 * sizeof(uint32_t), s));
  KMA_HIP(kma::launch_build_insert(d_slots, d_winner, (uint32_t)n_buckets, k, m, d_keys, n,
                                   d_status, s));
  KMA_HIP(kma::launch_build_finalize(d_slots, d_winner, d_fids, (uint32_t)n_buckets, k, m,
                                     d_status + 1, s));
  return KMA_OK;
}

// Two-choice build (kma_kernels.hip launch_build_two_choice) into zeroed slots on stream s; its
// sort buffers are allocated here and freed after the stream has drained them.
int build_two_choice_on_device(uint64_t* d_slots, uint64_t n_buckets, int k, int m,
                               const uint64_t* d_keys, const uint32_t* d_fids, uint64_t n,
                               uint32_t* d_status, hipStream_t s) {
  if (n_buckets >= kMaxBuckets) return fail(KMA_E_INVALID, "%llu buckets or more",
                                           (unsigned long long)kMaxBuckets);
  if (n_buckets < 2) return fail(KMA_E_INVALID, "two-choice placement needs 2 buckets or more");
  if (n >= (1ull << 32)) return fail(KMA_E_INVALID, "2^32 rows or more");
  KMA_HIP(hipMemsetAsync(d_slots, 0, n_buckets * bucket_bytes(k), s));
  KMA_HIP(hipMemsetAsync(d_status, 0, 4 * sizeof(uint32_t), s));
  if (n == 0) return KMA_OK;
  size_t temp_bytes = 0;
  kma::TwoChoiceScratch x;
  KMA_HIP(kma::launch_build_two_choice(d_slots, (uint32_t)n_buckets, k, m, d_keys, d_fids, n,
                                       nullptr, nullptr, nullptr, x, nullptr, &temp_bytes,
                                       d_status, s));
  DevBufs tmp;
  uint64_t* skeys;
  uint32_t *rows, *srows;
  void* temp;
  KMA_HIP(tmp.alloc(&skeys, n * 8));
  KMA_HIP(tmp.alloc(&rows, n * 4));
  KMA_HIP(tmp.alloc(&srows, n * 4));
  KMA_HIP(tmp.alloc(&temp, temp_bytes));
  KMA_HIP(tmp.alloc(&x.home, n * 4));  // home-first placement (kma_kernels.hip)
  KMA_HIP(tmp.alloc(&x.sorted_home, n * 4));
  KMA_HIP(tmp.alloc(&x.sorted_idx, n * 4));
  KMA_HIP(tmp.alloc(&x.away, n));
#ifndef KMA_TC_ALT_LOAD
#define KMA_TC_ALT_LOAD 1
#endif
  if (KMA_TC_ALT_LOAD) KMA_HIP(tmp.alloc(&x.load, n_buckets));
  KMA_HIP(kma::launch_build_two_choice(d_slots, (uint32_t)n_buckets, k, m, d_keys, d_fids, n,
                                       skeys, rows, srows, x, temp, &temp_bytes, d_status, s));
  KMA_HIP(hipStreamSynchronize(s));  // before DevBufs frees the sort buffers
  return KMA_OK;
}

// Table from device-resident keys/fids on `device` (n rows; fids already checked). Narrow tables
// are built with two-choice placement first (round 5; KMA_OPT_PLACEMENT 0 skips it), at the size
// rule's layout (a crowded minimizer table also flat, kept if it halves the displaced keys).
// Chained tables (wide K, or a two-choice build that failed) are laid out by the size rule and
// then by measurement (kma_internal.h, kRetryDisplaced / kMaxDisplaced): an m = 6 table with
// many displaced keys is rebuilt with m = 7 (kept if it displaces fewer), a still crowded
// minimizer table is rebuilt flat (kept if that halves the displaced keys or the longest
// chain). KMA_OPT_LAYOUT forces a layout.
int create_from_device_keys(const uint64_t* d_keys, const uint32_t* d_fids, uint64_t n, int k,
                            int device, double lf, const uint8_t lut[256], kma_table** out) {
  const uint64_t nb = buckets_for_k(n, lf, k);
  if (nb >= kMaxBuckets)
    return fail(KMA_E_INVALID, "table too large: %llu buckets", (unsigned long long)nb);
  DevBufs tmp;
  uint32_t *d_winner, *d_status;
  KMA_HIP(tmp.alloc(&d_winner, nb * kma::slots_for_k(k) * 4));
  KMA_HIP(tmp.alloc(&d_status, 16));
  auto build = [&](int m, uint64_t** slots, uint32_t st[4]) -> int {
    KMA_HIP(hipMalloc(slots, nb * bucket_bytes(k)));
    int rc = build_on_device(*slots, nb, k, m, d_winner, d_keys, d_fids, n, d_status, nullptr);
    if (rc == KMA_OK) {
      hipError_t e = hipMemcpy(st, d_status, 16, hipMemcpyDeviceToHost);
      if (e != hipSuccess) rc = fail(KMA_E_DEVICE, "build: %s", hipGetErrorString(e));
      else if (st[0]) rc = fail(KMA_E_TABLE_FULL, "signature table full");
    }
    if (rc != KMA_OK) {
      (void)hipFree(*slots);
      *slots = nullptr;
    }
    return rc;
  };
  int m = kma::minimizer_len(k, nb);
  uint64_t* d_slots = nullptr;
  uint32_t st[4] = {};
  auto displaced = [](const uint32_t s[4]) { return (double)s[3] / std::max<uint32_t>(s[1], 1); };
  if (two_choice_first(k) && nb >= 2) {
    // Two-choice placement at the size rule's (or the forced) layout; a crowded minimizer table
    // is also built flat and the flat one kept if it halves the displaced keys; a minimizer build
    // that fails (an insertion exceeded kMaxKicks) is retried flat; a build that still fails
    // falls through to the chained rule below.
    uint32_t s2[4] = {};
    auto build2 = [&](int m2, uint64_t** slots, uint32_t out[4]) -> int {
      KMA_HIP(hipMalloc(slots, nb * bucket_bytes(k)));
      int rc = build_two_choice_on_device(*slots, nb, k, m2, d_keys, d_fids, n, d_status, nullptr);
      if (rc == KMA_OK) {
        hipError_t e = hipMemcpy(out, d_status, 16, hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = fail(KMA_E_DEVICE, "build: %s", hipGetErrorString(e));
      }
      if (rc != KMA_OK || out[0]) {
        (void)hipFree(*slots);
        *slots = nullptr;
      }
      return rc;
    };
    uint64_t* d2 = nullptr;
    if (int rc = build2(m, &d2, s2)) return rc;
    if (s2[0] && m != 0 && forced_layout() < 0) {
      // A minimizer table whose insertions ran out of evictions (keys piling onto few
      // minimizers: their homes full, so they all compete for alternates) is built flat with
      // two-choice placement before falling back to chains: adversarial keys sharing 2,000
      // minimizers at LF 0.9 got a flat chained table with chains of 30 buckets
      // (profiles/r05/robustness_r05k.jsonl).
      if (int rc = build2(0, &d2, s2)) return rc;
      if (!s2[0]) m = 0;  // (else the chained rule below starts from the size rule's m)
    }
    if (!s2[0]) {  // built
      d_slots = d2;
      std::memcpy(st, s2, sizeof st);
      if (forced_layout() < 0 && m != 0 && displaced(st) > kma::kMaxDisplacedTwoChoice) {
        uint64_t* d3 = nullptr;
        uint32_t s3[4] = {};
        if (int rc = build2(0, &d3, s3)) {
          (void)hipFree(d_slots);
          return rc;
        }
        if (d3 && 2ull * s3[3] < st[3]) {
          (void)hipFree(d_slots);
          d_slots = d3;
          std::memcpy(st, s3, sizeof st);
          m = 0;
        } else if (d3) {
          (void)hipFree(d3);
        }
      }
      kma_table* t = new_table(device, k, m, nb, lut, true);
      if (int rc = add_replica(t, device, d_slots, true)) {
        (void)hipFree(d_slots);
        delete t;
        return rc;
      }
      t->info.n_rows = n;
      t->info.n_entries = st[1];
      t->info.max_probe = st[2];
      t->info.n_displaced = st[3];
      *out = t;
      return KMA_OK;
    }
  }
  if (int rc = build(m, &d_slots, st)) return rc;
  // Replace the current table (slots, stats, m) by a build with layout m2 when keep() says so.
  auto try_layout = [&](int m2, bool (*keep)(const uint32_t*, const uint32_t*)) -> int {
    uint64_t* d2 = nullptr;
    uint32_t s2[4] = {};
    if (int rc = build(m2, &d2, s2)) {
      (void)hipFree(d_slots);
      return rc;
    }
    const bool better = keep(st, s2);
    (void)hipFree(better ? d_slots : d2);
    if (better) {
      d_slots = d2;
      std::memcpy(st, s2, sizeof st);
      m = m2;
    }
    return KMA_OK;
  };
  const int m6 = std::min(k, 6), m7 = std::min(k, 7);
  if (forced_layout() < 0) {
    if ((m & kma::kMinimizerMask) == m6 && m6 != m7 && displaced(st) > kma::kRetryDisplaced)
      if (int rc = try_layout(m7, [](const uint32_t* a, const uint32_t* b) { return b[3] < a[3]; }))
        return rc;
    const bool crowded = displaced(st) > kma::kMaxDisplaced || st[2] > kma::kMaxChain;
    if (m != 0 && crowded)
      if (int rc = try_layout(0, [](const uint32_t* a, const uint32_t* b) {
            return 2ull * b[3] < a[3] || (a[2] > kma::kMaxChain && 2 * b[2] < a[2]);
          }))
        return rc;
  }
  kma_table* t = new_table(device, k, m, nb, lut);
  if (int rc = add_replica(t, device, d_slots, true)) {
    (void)hipFree(d_slots);
    delete t;
    return rc;
  }
  t->info.n_rows = n;
  t->info.n_entries = st[1];
  t->info.max_probe = st[2];
  t->info.n_displaced = st[3];
  *out = t;
  return KMA_OK;
}

// Shared by both create forms: keys packed on the host with `lut`.
int create_from_keys(const std::vector<uint64_t>& keys, const uint32_t* fids, uint64_t n, int k,
                     int device, double lf, const uint8_t lut[256], uint64_t n_skipped,
                     kma_table** out) {
  if (lf <= 0) lf = 0.5;
  if (lf > 0.95) return fail(KMA_E_INVALID, "load factor %.3f > 0.95", lf);
  for (uint64_t r = 0; r < n; ++r)
    if (fids[r] > KMA_MAX_FID) return fail(KMA_E_INVALID, "fid %u of row %llu exceeds 2^22-1",
                                            fids[r], (unsigned long long)r);
  DeviceScope ds(device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d): %s", device,
                                        hipGetErrorString(ds.err));
  DevBufs tmp;
  uint64_t* d_keys;
  uint32_t* d_fids;
  KMA_HIP(tmp.alloc(&d_keys, n * 8));
  KMA_HIP(tmp.alloc(&d_fids, n * 4));
  KMA_HIP(hipMemcpy(d_keys, keys.data(), n * 8, hipMemcpyHostToDevice));
  KMA_HIP(hipMemcpy(d_fids, fids, n * 4, hipMemcpyHostToDevice));
  const int rc = create_from_device_keys(d_keys, d_fids, n, k, device, lf, lut, out);
  if (rc != KMA_OK) return rc;
  (*out)->info.n_skipped = n_skipped;
  return KMA_OK;
}

// Run f(i) for i in [0, n) on n threads (inline for one) and return the first failure, with
// its message moved to the calling thread (kma_last_error is thread-local).
template <class F>
int fan_out(int n, F f) {
  if (n == 1) return f(0);
  std::vector<int> rc(n, KMA_OK);
  std::vector<std::string> msg(n);
  std::vector<std::thread> th;
  for (int i = 0; i < n; ++i)
    th.emplace_back([&, i] {
      rc[i] = f(i);
      if (rc[i] != KMA_OK) msg[i] = g_err;
    });
  for (auto& x : th) x.join();
  for (int i = 0; i < n; ++i)
    if (rc[i] != KMA_OK) {
      g_err = msg[i];
      return rc[i];
    }
  return KMA_OK;
}

// A layout code (kma_table_build_device / kma_table_wrap_device) -> minimizer code (m | order)
// and placement. -1 is kma_table_layout_for's code for (k, n_buckets) in both entry points, so a
// table built with -1 and wrapped with -1 agree (a caller whose -1 build reports a failed
// two-choice insertion rebuilds with an explicit chained code and wraps with that code).
int resolve_layout(int k, uint64_t n_buckets, int layout, int* m, bool* two) {
  const int code = layout < 0 ? kma::minimizer_len(k, n_buckets) |
                                    (two_choice_first(k) && n_buckets >= 2 ? kma::kLayoutTwoChoice : 0)
                              : layout;
  if (code & ~(kma::kLayoutMask | kma::kLayoutTwoChoice))
    return fail(KMA_E_INVALID, "layout code %d has unknown bits", layout);
  *m = code & kma::kLayoutMask;
  *two = (code & kma::kLayoutTwoChoice) != 0;
  const int mm = *m & kma::kMinimizerMask;
  if ((*m & ~kma::kMinimizerMask) & ~kma::kOrderMod)
    return fail(KMA_E_INVALID, "layout code %d has unknown bits", layout);
  if ((*m & kma::kOrderMod) ? !kma::order_mod_valid(k, *m)
                            : (mm != 0 && mm != std::min(k, 6) && mm != std::min(k, 7)))
    return fail(KMA_E_INVALID,
                "layout %d is not 0, min(K, 6) or min(K, 7) (| mod-sampling: K = 8, m = 6)", layout);
  if (*two && kma::wide_k(k)) return fail(KMA_E_INVALID, "two-choice placement takes K <= 8");
  return KMA_OK;
}

}  // namespace

extern "C" {

int kma_abi_version(void) { return KMA_ABI_VERSION; }

int kma_option_set(int option, int64_t value) {
  if (option < 1 || option >= kNumOpts || !option_valid(option, value))
    return fail(KMA_E_INVALID, "option %d: value %lld out of range", option, (long long)value);
  g_opt[option] = value;
  return KMA_OK;
}

int kma_option_get(int option, int64_t* value) {
  if (!value || option < 1 || option >= kNumOpts)
    return fail(KMA_E_INVALID, "option %d unknown (or null value)", option);
  *value = opt(option);
  return KMA_OK;
}

const char* kma_last_error(void) { return g_err.c_str(); }

int kma_device_count(int* out_n) {
  if (!out_n) return fail(KMA_E_INVALID, "null out_n");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *out_n = 0;
    return fail(KMA_E_DEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e));
  }
  *out_n = n;
  return KMA_OK;
}

uint64_t kma_table_buckets_for(uint64_t n_keys, double load_factor) {
  return buckets_for_k(n_keys, load_factor, kma::kMaxNarrowK);
}

uint64_t kma_table_buckets_for_k(uint64_t n_keys, double load_factor, int k) {
  return buckets_for_k(n_keys, load_factor, k);
}

int kma_bucket_slots_for(int k) { return check_k(k) ? 0 : kma::slots_for_k(k); }

int kma_table_layout_for(int k, uint64_t n_buckets) {
  return kma::minimizer_len(k, n_buckets) |
         (two_choice_first(k) && n_buckets >= 2 ? kma::kLayoutTwoChoice : 0);
}

int kma_bucket_slots(void) { return kma::kSlotsPerBucket; }

int kma_pack_kmers(const kma_table* table, const char* text, const uint64_t* offsets, uint64_t n,
                   uint64_t* out_keys) {
  if (!table || (!text && n) || !offsets || (!out_keys && n))
    return fail(KMA_E_INVALID, "null argument");
  pack_rows(table->lut, text, offsets, 0, n, table->k, out_keys);
  return KMA_OK;
}

int kma_table_create(const char* text, const uint64_t* offsets, const uint32_t* fids, uint64_t n,
                     int k, int device, double load_factor, kma_table** out) {
  if (!out || (n && (!text || !offsets || !fids))) return fail(KMA_E_INVALID, "null argument");
  if (int rc = check_k(k)) return rc;
  // Alphabet: standard A-Z and '*', plus up to four other bytes found in K-length rows.
  bool seen[256] = {};
  for (uint64_t r = 0; r < n; ++r)
    if (offsets[r + 1] - offsets[r] == (uint64_t)k)
      for (uint64_t i = offsets[r]; i < offsets[r + 1]; ++i) seen[(uint8_t)text[i]] = true;
  uint8_t lut[256];
  standard_lut(lut);
  int extra = 0;
  for (int c = 0; c < 256; ++c)
    if (seen[c] && !lut[c]) {
      if (extra == 4) return fail(KMA_E_ALPHABET, "more than 4 kmer symbols outside [A-Z*]");
      lut[c] = (uint8_t)(28 + extra++);
    }
  std::vector<uint64_t> keys(n);
  parallel_rows(n, [&](uint64_t lo, uint64_t hi) {
    pack_rows(lut, text, offsets, lo, hi, k, keys.data());
  });
  uint64_t skipped = 0;
  for (uint64_t r = 0; r < n; ++r) skipped += offsets[r + 1] - offsets[r] != (uint64_t)k;
  return create_from_keys(keys, fids, n, k, device, load_factor, lut, skipped, out);
}

int kma_table_create_from_tsv(const char* path, int k, int n_devices, const int* device_ids,
                              double load_factor, kma_table** out, char** role_names,
                              uint64_t* role_bytes, uint32_t* n_roles, int* last_kmer_len) {
  if (!path || !out || n_devices < 1 || !device_ids) return fail(KMA_E_INVALID, "null argument");
  *out = nullptr;
  if (role_names) *role_names = nullptr;
  if (int rc = check_k(k)) return rc;
  // the alphabet rule of kma_table_create: A-Z and '*', then up to four other bytes of K-length
  // kmers in byte order
  auto make_lut = [](const bool* seen, uint8_t* lut) {
    standard_lut(lut);
    int extra = 0;
    for (int c = 0; c < 256; ++c)
      if (seen[c] && !lut[c]) {
        if (extra == 4) return KMA_E_ALPHABET;
        lut[c] = (uint8_t)(28 + extra++);
      }
    return KMA_OK;
  };
  kma::KmerTsv tsv;
  std::string err;
  if (int rc = kma::read_kmer_tsv(path, k, (unsigned)std::min<size_t>(16, host_cores()), make_lut,
                                  &tsv, &err))
    return fail(rc, "%s", err.c_str());
  kma_table* t = nullptr;
  if (int rc = create_from_keys(tsv.keys, tsv.fids.data(), tsv.keys.size(), k, device_ids[0],
                                load_factor, tsv.lut, tsv.n_skipped, &t))
    return rc;
  if (n_devices > 1)
    if (int rc = kma_table_replicate(t, n_devices - 1, device_ids + 1)) {
      free_table(t);
      return rc;
    }
  uint64_t bytes = 0;
  for (const std::string& r : tsv.roles) bytes += r.size() + 1;
  if (role_names) {
    char* blob = static_cast<char*>(malloc(std::max<uint64_t>(bytes, 1)));
    if (!blob) {
      free_table(t);
      return fail(KMA_E_NOMEM, "role names: %llu bytes", (unsigned long long)bytes);
    }
    char* p = blob;
    for (const std::string& r : tsv.roles) {
      std::memcpy(p, r.data(), r.size());
      p += r.size();
      *p++ = '\0';
    }
    *role_names = blob;
  }
  if (role_bytes) *role_bytes = bytes;
  if (n_roles) *n_roles = (uint32_t)tsv.roles.size();
  if (last_kmer_len) *last_kmer_len = tsv.last_kmer_len;
  *out = t;
  return KMA_OK;
}

void kma_free(void* p) { free(p); }

int kma_table_create_packed(const uint64_t* keys, const uint32_t* fids, uint64_t n, int k,
                            int device, double load_factor, kma_table** out) {
  if (!out || (n && (!keys || !fids))) return fail(KMA_E_INVALID, "null argument");
  if (int rc = check_k(k)) return rc;
  uint8_t lut[256];
  standard_lut(lut);
  std::vector<uint64_t> kv(keys, keys + n);
  uint64_t skipped = 0;
  const uint64_t lim = 1ull << (5 * k);
  for (uint64_t r = 0; r < n; ++r)
    if (kv[r] == 0 || kv[r] >= lim) kv[r] = 0, ++skipped;
  return create_from_keys(kv, fids, n, k, device, load_factor, lut, skipped, out);
}

int kma_table_replicate(kma_table* t, int n_devices, const int* device_ids) {
  if (!t || n_devices < 0 || (n_devices && !device_ids) || replicas(t).empty())
    return fail(KMA_E_INVALID, "null argument");
  const Replica src = replicas(t)[0];
  const uint64_t bytes = t->n_buckets * bucket_bytes(t->k);
  int n_dev = 0;
  if (hipGetDeviceCount(&n_dev) != hipSuccess) return fail(KMA_E_DEVICE, "hipGetDeviceCount");
  for (int i = 0; i < n_devices; ++i)
    if (device_ids[i] < 0 || device_ids[i] >= n_dev)
      return fail(KMA_E_INVALID, "device %d not present", device_ids[i]);
  // Every destination's slot array and copy stream first; then all copies at once (each on its
  // destination's stream, so each GPU's copy engine pulls replica 0 over its own xGMI link
  // instead of one link at a time); then one wait for all of them.
  struct Dest {
    int dev;
    uint64_t* d = nullptr;
    hipStream_t s = nullptr;
    bool peer = false;  // the destination reads replica 0 directly (peer access enabled)
  };
  std::vector<Dest> dst(n_devices);
  auto cleanup = [&](bool free_slots) {
    for (Dest& x : dst) {
      DeviceScope ds(x.dev);
      if (x.s) (void)hipStreamDestroy(x.s);
      if (free_slots && x.d) (void)hipFree(x.d);
      x.s = nullptr;
    }
  };
  for (int i = 0; i < n_devices; ++i) {
    Dest& x = dst[i];
    x.dev = device_ids[i];
    DeviceScope ds(x.dev);
    hipError_t e = ds.err;
    if (e == hipSuccess) e = hipMalloc(&x.d, bytes);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking);
    if (e == hipSuccess && x.dev != src.device) {
      // Peer access from the destination to replica 0's device, once per pair (an enabled pair
      // stays enabled): its copy engine then pulls the slot array over xGMI. Without it the
      // runtime may stage a peer copy through host memory.
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, x.dev, src.device) == hipSuccess && can) {
        const hipError_t pe = hipDeviceEnablePeerAccess(src.device, 0);
        if (pe == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
        x.peer = pe == hipSuccess || pe == hipErrorPeerAccessAlreadyEnabled;
      }
    }
    if (e != hipSuccess) {
      cleanup(true);
      return fail(e == hipErrorOutOfMemory ? KMA_E_NOMEM : KMA_E_DEVICE,
                  "replica on device %d: %s", x.dev, hipGetErrorString(e));
    }
  }
  const auto t0 = std::chrono::steady_clock::now();
  hipError_t e = hipSuccess;
  for (Dest& x : dst) {
    DeviceScope ds(x.dev);
    e = x.dev == src.device
            ? hipMemcpyAsync(x.d, src.d_slots, bytes, hipMemcpyDeviceToDevice, x.s)
            : hipMemcpyPeerAsync(x.d, x.dev, src.d_slots, src.device, bytes, x.s);
    if (e != hipSuccess) break;
  }
  for (Dest& x : dst) {
    DeviceScope ds(x.dev);
    const hipError_t w = hipStreamSynchronize(x.s);  // every issued copy, even after a failure
    if (e == hipSuccess) e = w;
  }
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (e != hipSuccess) {
    cleanup(true);
    return fail(KMA_E_DEVICE, "replica copies: %s", hipGetErrorString(e));
  }
  cleanup(false);
  for (size_t i = 0; i < dst.size(); ++i)
    if (int rc = add_replica(t, dst[i].dev, dst[i].d, true)) {
      for (size_t j = i; j < dst.size(); ++j) {
        DeviceScope ds(dst[j].dev);
        (void)hipFree(dst[j].d);
      }
      return rc;
    }
  std::lock_guard<std::mutex> g(t->reps_mu);
  t->info.replicate_ms = ms;
  t->info.replicate_bytes = bytes * (uint64_t)n_devices;
  t->info.replicate_peer = 0;
  t->info.replicate_local = 0;
  for (const Dest& x : dst) {
    t->info.replicate_peer += x.peer ? 1 : 0;
    t->info.replicate_local += x.dev == src.device ? 1 : 0;
  }
  return KMA_OK;
}

int kma_table_create_replicated(const char* text, const uint64_t* offsets, const uint32_t* fids,
                                uint64_t n, int k, int n_devices, const int* device_ids,
                                double load_factor, kma_table** out) {
  if (!out || n_devices < 1 || !device_ids) return fail(KMA_E_INVALID, "null argument");
  *out = nullptr;
  kma_table* t = nullptr;
  if (int rc = kma_table_create(text, offsets, fids, n, k, device_ids[0], load_factor, &t))
    return rc;
  if (int rc = kma_table_replicate(t, n_devices - 1, device_ids + 1)) {
    free_table(t);
    return rc;
  }
  *out = t;
  return KMA_OK;
}

int kma_table_replicas(const kma_table* t, int* n, int* device_ids, int cap) {
  if (!t || !n) return fail(KMA_E_INVALID, "null argument");
  const std::vector<Replica> reps = replicas(t);
  *n = (int)reps.size();
  for (int i = 0; i < *n && i < cap && device_ids; ++i) device_ids[i] = reps[i].device;
  return KMA_OK;
}

int kma_table_info_get(const kma_table* table, kma_table_info* out) {
  if (!table || !out) return fail(KMA_E_INVALID, "null argument");
  std::lock_guard<std::mutex> g(table->reps_mu);  // kma_table_replicate writes n_replicas
  *out = table->info;
  return KMA_OK;
}

int kma_table_destroy(kma_table* table) {
  if (!table) return KMA_OK;
  free_table(table);
  return KMA_OK;
}

int kma_table_build_device(void* d_slots, uint64_t n_buckets, int k, int layout,
                           uint32_t* d_winner, const uint64_t* d_keys, const uint32_t* d_fids,
                           uint64_t n, uint32_t* d_status, void* stream) {
  if (int rc = check_k(k)) return rc;
  if (!n_buckets) return fail(KMA_E_INVALID, "null argument");
  int m = 0;
  bool two = false;
  if (int rc = resolve_layout(k, n_buckets, layout, &m, &two)) return rc;
  // d_winner is the chained build's scratch; a two-choice build does not read it.
  if (!d_slots || (!two && !d_winner) || !d_status || (n && (!d_keys || !d_fids)))
    return fail(KMA_E_INVALID, "null argument");
  if (two) {
    return build_two_choice_on_device(static_cast<uint64_t*>(d_slots), n_buckets, k, m, d_keys,
                                      d_fids, n, d_status, static_cast<hipStream_t>(stream));
  }
  return build_on_device(static_cast<uint64_t*>(d_slots), n_buckets, k, m, d_winner, d_keys,
                         d_fids, n, d_status, static_cast<hipStream_t>(stream));
}

int kma_table_wrap_device(void* d_slots, uint64_t n_buckets, int k, int layout, int device,
                          kma_table** out) {
  if (!d_slots || !out || !n_buckets) return fail(KMA_E_INVALID, "null argument");
  if (n_buckets >= kMaxBuckets) return fail(KMA_E_INVALID, "%llu buckets or more",
                                           (unsigned long long)kMaxBuckets);
  if (int rc = check_k(k)) return rc;
  int m = 0;
  bool two = false;
  if (int rc = resolve_layout(k, n_buckets, layout, &m, &two)) return rc;
  if (two && n_buckets < 2)
    return fail(KMA_E_INVALID, "two-choice placement takes K <= 8 and 2 buckets or more");
  uint8_t lut[256];
  standard_lut(lut);
  kma_table* t = new_table(device, k, m, n_buckets, lut, two);
  if (int rc = add_replica(t, device, static_cast<uint64_t*>(d_slots), false)) {
    delete t;
    return rc;
  }
  *out = t;
  return KMA_OK;
}

int kma_table_device_ptr(const kma_table* table, void** d_slots, uint64_t* bytes) {
  if (!table || !d_slots || !bytes || replicas(table).empty())
    return fail(KMA_E_INVALID, "null argument");
  *d_slots = replicas(table)[0].d_slots;
  *bytes = table->n_buckets * bucket_bytes(table->k);
  return KMA_OK;
}

}  // extern "C"

namespace {
void free_protein_scratch(kma_workspace* ws) {
  if (ws->d_gset) (void)hipFree(ws->d_gset);
  if (ws->d_packed) (void)hipFree(ws->d_packed);
  ws->d_gset = nullptr;
  ws->d_packed = nullptr;
  ws->res_cap = 0;
}

void free_contig_scratch(kma_workspace* ws) {
  for (void* p : {(void*)ws->d_cstage, (void*)ws->d_ccounts, (void*)ws->d_cprefix})
    if (p) (void)hipFree(p);
  ws->d_cstage = nullptr;
  ws->d_ccounts = nullptr;
  ws->d_cprefix = nullptr;
  ws->contig_cap = 0;
}

uint64_t contig_blocks(uint64_t n_bases) {
  return std::max<uint64_t>(1, (n_bases + kma::kContigTile - 1) / kma::kContigTile);
}

// Codon table of an NCBI code as 5-bit amino-acid codes (0 = stop or ambiguous).
void codon_codes(const char* code, uint8_t out[64]) {
  for (int i = 0; i < 64; ++i)
    out[i] = (code[i] == '*' || code[i] == 'X') ? 0 : (uint8_t)(code[i] - 'A' + 1);
}

int contig_args(const kma_table* t, const Replica& r, kma_workspace* ws, const uint8_t* d_dna,
                const uint64_t* d_offsets, uint32_t n_contig, uint64_t n_bases, const char* code,
                uint32_t* d_tally, uint32_t n_fid, hipStream_t s, kma::ContigArgs* out) {
  kma::ContigArgs a{};
  a.slots = r.d_slots;
  a.n_buckets = (uint32_t)t->n_buckets;
  a.dna = d_dna;
  a.offsets = d_offsets;
  a.n_contig = n_contig;
  a.total_bases = n_bases;
  a.k = t->k;
  a.mlen = t->mlen;
  a.two_choice = t->two_choice ? 1u : 0u;
  a.staging = ws->d_cstage;
  a.block_counts = ws->d_ccounts;
  // An earlier call failed between its probe and its emit: start clean, ordered on this
  // call's stream (calls on one workspace are ordered on one stream, kmeranno.h).
  if (ws->cpending) KMA_HIP(hipMemsetAsync(ws->d_cprefix, 0, (ws->cgroups + 1) * 8, s));
  ws->cpending = true;
  a.group_sum = ws->d_cprefix;
  a.emit_done = reinterpret_cast<uint32_t*>(ws->d_cprefix + ws->cgroups);
  a.tally = d_tally;
  a.n_fid = d_tally ? n_fid : 0;
  codon_codes(code, a.codon_codes);
  *out = a;
  return KMA_OK;
}

// Canonical-order emission after the probe on s (whose atomics summed the block counts into
// ws's group sums); the emit pass leaves the sums zero for the next call.
int enqueue_contig_emit(kma_workspace* ws, kma::ContigArgs a, kma_hit* d_hits, uint64_t cap,
                        uint64_t* d_n_hits, hipStream_t s) {
  const uint64_t nb = contig_blocks(a.total_bases);
  a.out = d_hits;
  a.cap = d_hits ? cap : 0;
  a.n_hits = d_n_hits;
  KMA_HIP(kma::launch_contigs_emit(a, nb, s));
  ws->cpending = false;
  return KMA_OK;
}

// Records the phase boundaries of one timed device call (nothing when timing is off).
struct PhaseClock {
  hipEvent_t* ev = nullptr;
  int n = 0;
  hipStream_t s = nullptr;
  PhaseClock(kma_workspace* ws, hipStream_t stream, const char* const* names, int n_phases)
      : s(stream) {
    if (!ws->timing) return;
    const uint32_t slot = ws->n_timed++ % kTimingRing;
    ev = &ws->events[kMaxEv * slot];
    ws->names[slot] = names;
    ws->n_phases[slot] = n_phases;
  }
  hipError_t mark() { return ev ? hipEventRecord(ev[n++], s) : hipSuccess; }
};

const char* const kDirectPhases[] = {"annotate_kernel"};
const char* const kPackedPhases[] = {"pack_kernel", "annotate_kernel"};
const char* const kContigPhases[] = {"contigs_probe_kernel", "scan_emit"};

// Proteins per annotate_kernel block (KMA_BLOCK_PROTEINS=1..8 overrides, read per call): 6 for
// batches of more than 4 resident waves of such blocks against a table larger than the Infinity
// Cache, else 4. A block's fixed costs (the
// offsets and first residues round trips, the final chain walks, the vote) are amortized over
// more probe steps with more proteins, while a batch of few waves of blocks ends with a longer
// tail. Measured on MI355X (profiles/r03_ab/r03m, r03n): c5 3.94 / 3.77 / 3.88 ms at 4 / 6 / 8
// (3.87 / 3.72 / 3.84 with queued keys), c2 51 vs 66 us at 4 vs 6. (Round 2, before the walk
// queue and the scratch fix: c5 4.53 / 4.66 / 4.86 ms at 4 / 6 / 8, r02f_block_proteins.log.)
// Round 3 (interleaved A/B, profiles/r03_session2/r03bp_steps.log): c5 (10^8 rows, 1.5 GiB
// table in HBM) 3.59-3.63 / 3.69-3.71 / 3.80-3.81 ms at 6 / 7 / 8; c4 (10^7 rows, a 153 MiB
// table inside the 256 MiB Infinity Cache) 2.752 vs 2.819 ms at 4 vs 6: 6 only for tables
// larger than the Infinity Cache. Round 5, c2 (profiles/r05/c2_opts_r05t/, two runs each):
// 46.6 us at 4 proteins (two-pass grid), 52.4 / 50.0 / 48.0 / 53.9 / 56.6 us at 2 / 3 / 5 / 6 / 8,
// 52.8 without the two-pass grid; and a tapered tail (the batch's last groups of half size, then
// single proteins, so the last blocks to start end sooner; profiles/r05/c2_taper_r05u/) 47.0 /
// 49.3 / 54.0 / 55.1 us for tails of 1/4, 1/2, 1 and 2 resident waves: each group's fixed chain
// (offsets, first residues, final walks, vote) costs more than the shorter tail saves.
uint32_t block_proteins(const kma_workspace* ws, uint32_t n_seq, uint64_t table_bytes) {
  const int64_t f = ws->opt_block_proteins != kOptUnset ? ws->opt_block_proteins
                                                         : opt(KMA_OPT_BLOCK_PROTEINS);
  if (f >= 1 && f <= kma::kBlockProteins) return (uint32_t)f;
  const uint64_t slots = (uint64_t)kma::kProteinOcc * (uint64_t)std::max(ws->n_cu, 1);
  return (uint64_t)n_seq / 6 > 4 * slots && table_bytes > kInfinityCacheBytes ? 6u : 4u;
}

// Deferral of short groups (annotate_kernel's two-pass grid), in probe steps: groups below it
// are annotated after every longer one has started. A fixed-count grid is dispatched in
// block order, so without it a long group dispatched late ends the call alone: at c2 the
// kernel's last ~25 of ~65 us ran with a shrinking set of late long blocks
// (profiles/r02m_block_clock.jsonl; with the groups pre-sorted longest first the kernel took
// 50 us). Automatic for grids of more than one and at most 4 resident waves of blocks (7 per
// CU): measured (profiles/r02m_defer_ab.log) c2 (1.4 waves) 66 -> 54 us, 40k proteins (5.6)
// even, 100k (14) 3% slower, c4 / c5 7% / 3% slower when forced. KMA_DEFER=0 disables it,
// KMA_DEFER=<steps> forces it on any batch (read per call).
uint32_t defer_below(const kma_workspace* ws, uint64_t n_groups) {
  const uint64_t slots = (uint64_t)kma::kProteinOcc * (uint64_t)std::max(ws->n_cu, 1);
  const int64_t f = ws->opt_defer != kOptUnset ? ws->opt_defer : opt(KMA_OPT_DEFER);
  if (f >= 0) return (uint32_t)std::min<int64_t>(64, f);
  return n_groups > slots && n_groups <= 4 * slots ? 3u : 0u;
}

// How the protein kernel gets its residues: ASCII read directly; ASCII packed on the device
// first (pack_kernel into the workspace, then the packed kernel: the device entry point's
// default, KMA_OPT_PACKED_INPUT); a packed stream the caller staged (host entry, packed device
// entry; stream residue `stream_first` = residue offsets[0]).
enum class Input { kAscii, kPackOnDevice, kStream };

// Device calls pack first under KMA_OPT_PACKED_INPUT = 2, or = 1 (the default) for batches of
// at least 2^25 residues: the pack kernel costs a launch (~8 us at c2's 3M residues, where the
// ASCII probe is 3 us faster in total) and pays off only at scale (c4 2.80 vs 2.83 ms, c5 even:
// profiles/r04/ab_r04c.jsonl). Host calls pack under 1 and 2 (the H2D is the bound there).
constexpr uint64_t kPackMinResidues = 1ull << 25;
bool pack_on_device(uint64_t n_residues) {
  const int64_t v = opt(KMA_OPT_PACKED_INPUT);
  return n_residues > 0 && (v == 2 || (v == 1 && n_residues >= kPackMinResidues));
}

// The workspace's packed stream for device calls that pack: allocated by
// kma_workspace_reserve_batch (never here: the device entry points do not allocate).
int ensure_packed(const kma_workspace* ws) {
  if (ws->d_packed) return KMA_OK;
  return fail(KMA_E_CAPACITY, "workspace has no packed stream (kma_workspace_reserve_batch first)");
}

// The protein path on one replica (device buffers, asynchronous on s).
int annotate_proteins_on(const kma_table* t, const Replica& r, kma_workspace* ws,
                         const uint8_t* d_residues, const uint64_t* d_offsets, uint32_t n_seq,
                         uint64_t n_residues, int min_hits, uint32_t flags, int32_t* d_fid,
                         int32_t* d_count, uint8_t* d_status, uint32_t* d_tally, uint32_t n_fid,
                         hipStream_t s, Input input = Input::kAscii, uint64_t stream_first = 0) {
  kma::ProteinArgs a{};
  a.slots = r.d_slots;
  a.n_buckets = (uint32_t)t->n_buckets;
  a.lut = r.d_lut;
  a.residues = input == Input::kPackOnDevice ? ws->d_packed : d_residues;
  a.packed = input != Input::kAscii;
  a.stream_first = input == Input::kStream ? stream_first : 0;
  a.offsets = d_offsets;
  a.n_seq = n_seq;
  a.n_residues = (uint32_t)n_residues;
  a.k = t->k;
  a.mlen = t->mlen;
  a.two_choice = t->two_choice ? 1u : 0u;
  a.min_hits = min_hits;
  a.flags = flags;
  a.out_fid = d_fid;
  a.out_count = d_count;
  a.out_status = d_status;
  a.tally = d_tally;
  a.n_fid = d_tally ? n_fid : 0;
  a.gset = ws->d_gset;
  a.block_proteins = block_proteins(ws, n_seq, t->n_buckets * (uint64_t)kma::kBucketBytes);
  a.n_groups = (n_seq + a.block_proteins - 1) / a.block_proteins;
  a.defer_below = a.n_groups < (1u << 30) ? defer_below(ws, a.n_groups) : 0u;
  const bool pack = input == Input::kPackOnDevice;
  PhaseClock clk(ws, s, pack ? kPackedPhases : kDirectPhases, pack ? 2 : 1);
  KMA_HIP(clk.mark());
  if (pack) {
    KMA_HIP(kma::launch_pack_residues(d_residues, d_offsets, n_residues, r.d_lut, ws->d_packed,
                                      s));
    KMA_HIP(clk.mark());
  }
  KMA_HIP(kma::launch_annotate(a, s));
  KMA_HIP(clk.mark());
  return KMA_OK;
}

int check_protein_call(const kma_table* t, int min_hits, uint32_t flags) {
  if (!t) return fail(KMA_E_INVALID, "null table");
  if (kma::wide_k(t->k))
    return fail(KMA_E_INVALID, "the protein path takes tables of K <= 8 (this table: K = %d)",
                t->k);
  if (min_hits < 1) return fail(KMA_E_INVALID, "Min-hits must be positive.");
  if (flags & ~(KMA_F_END_EXCLUSIVE | KMA_F_MULTISET)) return fail(KMA_E_INVALID, "bad flags");
  return KMA_OK;
}

// One shard [lo, hi) of a host protein call on replica r (host buffers, synchronous).
// Host bytes -> pinned staging -> device, pipelined: the input is cut into pieces of whole
// proteins, one kernel per piece. ASCII input (stage_h2d): the staging pool copies piece i's
// part of the pinned buffer in 2 MiB chunks and ONE copy per piece goes on the copy stream, so
// piece i + 1 is staged while piece i's copy and kernel run (r04g's trace of 153 chunk-sized
// copies kept the DMA engine idle a quarter of the time, profiles/r04/e2e_trace_r04g.json).
// Packed input (the default): streamed segments, below in protein_shard.
hipError_t stage_h2d(uint8_t* d_dst, uint8_t* h_pinned, const uint8_t* src, size_t len,
                     int device, hipStream_t s) {
  constexpr size_t kChunk = 2u << 20;
  const size_t n_chunks = (len + kChunk - 1) / kChunk;
  staging_pool().run(n_chunks, staging_threads(), [&](uint64_t i) {
    const size_t off = i * kChunk;
    std::memcpy(h_pinned + off, src + off, std::min(kChunk, len - off));
  });
  (void)device;
  return len ? hipMemcpyAsync(d_dst, h_pinned, len, hipMemcpyHostToDevice, s) : hipSuccess;
}

// The packed form of stage_h2d (piece-wise copies, kStreamedCopies = 0): stream groups [ga, gb)
// (64 residues, 40 bytes each) packed from src (residue 64 ga onwards; residues past n_res read
// as no code) into the pinned buffer in chunks of 2^15 groups (2M residues) on the staging
// pool, then copied to d_stream in one copy; `tail` extra zero bytes (the kernel's read
// padding) follow the last group.
hipError_t stage_pack_h2d(uint8_t* d_stream, uint8_t* h_stream, const uint8_t* lut,
                          const uint8_t* residues, uint64_t n_res, uint64_t ga, uint64_t gb,
                          uint64_t tail, hipStream_t s) {
  constexpr uint64_t kChunkGroups = 1u << 15;
  const uint64_t n_chunks = std::max<uint64_t>(1, (gb - ga + kChunkGroups - 1) / kChunkGroups);
  staging_pool().run(n_chunks, staging_threads(), [&](uint64_t i) {
    const uint64_t g0 = ga + i * kChunkGroups, g1 = std::min(gb, g0 + kChunkGroups);
    const uint64_t r0 = 64 * g0, r1 = std::min(64 * g1, n_res);
    const uint64_t bytes = 40 * (g1 - g0) + (g1 == gb ? tail : 0);
    kma::pack_residues_host(lut, residues + r0, r1 > r0 ? r1 - r0 : 0, h_stream + 40 * g0, bytes);
  });
  const uint64_t bytes = 40 * (gb - ga) + tail;
  return bytes ? hipMemcpyAsync(d_stream + 40 * ga, h_stream + 40 * ga, bytes,
                                hipMemcpyHostToDevice, s)
               : hipSuccess;
}

// Streamed copies of packed input (protein_shard): the stream is copied in segments as soon as
// they are packed, instead of one copy per piece after the whole piece is packed (KMA_HOST_STREAM
// = 0 builds the piece-wise pipeline for A/B runs).
#ifndef KMA_HOST_STREAM
#define KMA_HOST_STREAM 1
#endif
constexpr bool kStreamedCopies = KMA_HOST_STREAM != 0;

// Host-side phase times of the last host protein shard call (kma_debug_host_profile, for the
// host-call measurements in scripts/e2e_host.py): ms in setup (context, reservations, offsets),
// staging (packing / copying into pinned memory and queueing the copies), launches, the final
// wait for the stream, the output copies, and the whole call; then the staging width and the
// pieces. Also per replica (the first kProfReplicas of a fanned-out call).
constexpr int kProfFields = 8, kProfReplicas = 64;
std::mutex g_prof_mu;
double g_prof[kProfFields] = {};
double g_prof_rep[kProfReplicas][kProfFields] = {};
using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point a) {
  return std::chrono::duration<double, std::milli>(Clock::now() - a).count();
}

int protein_shard(kma_table* t, const Replica& r, int rep, const uint8_t* residues,
                  const uint64_t* offsets, uint32_t lo, uint32_t hi, int min_hits,
                  uint32_t flags, int32_t* out_fid, int32_t* out_count, uint8_t* out_status,
                  uint32_t* tally, uint32_t n_fid) {
  const uint32_t n = hi - lo;
  if (n == 0) return KMA_OK;
  const Clock::time_point t_call = Clock::now();
  double t_stage = 0, t_launch = 0;
  const uint64_t base = offsets[lo], nres = offsets[hi] - base;
  if (nres > kMaxResidues)
    return fail(KMA_E_INVALID, "a protein of %llu residues (limit 2^32 - 128)",
                (unsigned long long)nres);
  HostCtx* c = nullptr;
  if (int rc = acquire_ctx(t, r.device, &c)) return rc;
  CtxGuard guard{t, c};
  DeviceScope ds(r.device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", r.device);
  // KMA_OPT_PACKED_INPUT (default): residues are packed to 5 bits while they are staged (the
  // H2D moves 0.625 bytes per residue) and the packed kernel reads the stream.
  const bool packed = opt(KMA_OPT_PACKED_INPUT) != 0;
  const uint64_t n_groups = (nres + 63) / 64;
  const size_t in_bytes = packed ? (size_t)kma::packed_bytes(nres) : (nres + kResPad + 7) & ~7ull;
  const size_t off_bytes = (n + 1) * 8ull;
  const size_t out_bytes = n * 9ull + (tally ? n_fid * 4ull : 0) + 16;
  KMA_HIP(c->d_in.reserve(in_bytes));
  KMA_HIP(c->d_off.reserve(n + 1));
  KMA_HIP(c->d_out.reserve(out_bytes));
  KMA_HIP(c->h_in.reserve(in_bytes + off_bytes));
  KMA_HIP(c->h_out.reserve(out_bytes));
  if (int rc = kma_workspace_reserve_batch(c->ws, nres, n)) return rc;
  // Stage: rebased offsets, then the residues (and, with the last piece, their zero padding)
  // in pieces of whole proteins, in one pinned buffer. Piece i's copies go on copy stream
  // i % 2 (the offsets with piece 0); the kernel of piece i waits for piece i's event on the
  // compute stream, so the staging and transfer of piece i + 1 run under the kernel of piece i,
  // and two pieces' copies may run at once on two DMA engines (pieces of >= kPieceBytes residues,
  // at most KMA_HOST_PIECES (default 8, <= kMaxPieces; read per call: streamed c5 calls took
  // 5.6-5.7 / 6.0 / 6.1 ms at 8 / 12 / 16 pieces, profiles/r05/e2e_streamed_alt_r05j);
  // a small call is one piece). c5 whole batch: 12.5 ms as one piece, 8.6 ms in 8 (round 2,
  // profiles/r02r_host_pipeline/).
  const int64_t pm = opt(KMA_OPT_HOST_PIECE_MIN);
  const uint64_t kPieceBytes = pm > 0 ? (uint64_t)pm : 16ull << 20;
  const int64_t po = opt(KMA_OPT_HOST_PIECES);
  // packed input: the stream is copied in segments as it is packed (kStreamedCopies)
  const bool streamed = packed && kStreamedCopies;
  const uint64_t max_pieces =
      po > 0 ? std::min<uint64_t>((uint64_t)po, kMaxPieces) : 8;
  uint8_t* hin = c->h_in.p;
  hipStream_t s = c->stream;
  uint64_t* hoff = reinterpret_cast<uint64_t*>(hin + in_bytes);
  rebase_offsets(hoff, offsets + lo, (uint64_t)n + 1, base);
  KMA_HIP(hipMemcpyAsync(c->d_off.p, hoff, off_bytes, hipMemcpyHostToDevice, c->copy[0]));
  uint8_t* dout = c->d_out.p;
  int32_t* d_fid = reinterpret_cast<int32_t*>(dout);
  int32_t* d_cnt = d_fid + n;
  uint32_t* d_tally = tally ? reinterpret_cast<uint32_t*>(d_cnt + n) : nullptr;
  uint8_t* d_st = reinterpret_cast<uint8_t*>(d_cnt + n) + (tally ? n_fid * 4ull : 0);
  if (d_tally) KMA_HIP(hipMemsetAsync(d_tally, 0, n_fid * 4ull, s));
  const int n_pieces = (int)std::max<uint64_t>(1, std::min<uint64_t>(max_pieces, nres / kPieceBytes));
  // Piece sizes. Piece-wise copies: ramp up and down (weights 1, 2, 4, ..., 4, 2, 1): a small
  // first piece starts the link early and a small last piece shortens the tail behind the last
  // copy (round 4's equal eighths left 0.4 ms of kernel and 0.5 ms of output copies after the
  // last H2D, profiles/r04/e2e_trace_r04h.json). Streamed copies: the link no longer waits for
  // a piece, only the kernels do, and those keep up with the link (0.155 vs 0.18 ms per 1/22 of
  // c5), so equal pieces: the tail is one small piece's kernel (a ramp down's halving pieces
  // left kernels queued behind the last copy: 0.78 ms, profiles/r05/e2e_streamed_ramp_r05f).
  // (Also measured on streamed calls: the last four pieces shrinking geometrically, weights 0.6,
  // 0.36, 0.22, 0.13 of the others, cut the kernel after the last copy from ~0.6 to ~0.3 ms but
  // the calls were no faster on two boxes: 5.8-6.7 vs 5.6-7.3 ms and 6.1-6.3 vs 5.6-6.7 ms,
  // profiles/r05/e2e_taper_r05w, r05y.)
  uint64_t wsum = 0, wcum[kMaxPieces + 1] = {0};
  for (int i = 0; i < n_pieces; ++i) {
    const int edge = std::min(i, n_pieces - 1 - i);
    wsum += streamed || n_pieces < 4 ? 1u : (1u << std::min(edge, 2));
    wcum[i + 1] = wsum;
  }
  uint32_t pbeg[kMaxPieces + 1] = {0};  // first protein of each piece (relative to lo)
  const uint8_t* hout = c->h_out.p;
  // piece i's outputs back on the d2h stream once its kernel is done (fid, count, status
  // slices; the tally with the last piece), while later pieces copy and run
  auto outputs_back = [&](int i, uint32_t a, uint32_t b) -> int {
    KMA_HIP(hipEventRecord(c->piece_done[i], s));
    KMA_HIP(hipStreamWaitEvent(c->d2h, c->piece_done[i], 0));
    if (b > a) {
      uint8_t* h = c->h_out.p;
      KMA_HIP(hipMemcpyAsync(h + a * 4ull, d_fid + a, (b - a) * 4ull, hipMemcpyDeviceToHost, c->d2h));
      KMA_HIP(hipMemcpyAsync(h + (n + a) * 4ull, d_cnt + a, (b - a) * 4ull, hipMemcpyDeviceToHost,
                             c->d2h));
      KMA_HIP(hipMemcpyAsync(h + n * 8ull + (tally ? n_fid * 4ull : 0) + a, d_st + a, b - a,
                             hipMemcpyDeviceToHost, c->d2h));
    }
    if (i + 1 == n_pieces && tally)
      KMA_HIP(hipMemcpyAsync(c->h_out.p + n * 8ull, d_tally, n_fid * 4ull, hipMemcpyDeviceToHost,
                             c->d2h));
    KMA_HIP(hipEventRecord(c->out_ready[i], c->d2h));
    return KMA_OK;
  };
  const double t_setup = ms_since(t_call);
  // Piece boundaries: the first protein starting at or after each piece's residue target.
  for (int i = 1; i < n_pieces; ++i) {
    const uint64_t target = nres * wcum[i] / wsum;
    pbeg[i] = (uint32_t)(std::lower_bound(hoff + pbeg[i - 1], hoff + n, target) - hoff);
  }
  pbeg[n_pieces] = n;
  // Piece i's kernel (after its input is on the device: piece_ready[i] on copy stream cs, and
  // with both_copies, piece_ready2[i] on copy[1] as well) and the copy of its outputs.
  auto launch_piece = [&](int i, hipStream_t cs, bool both_copies = false) -> int {
    const uint32_t a = pbeg[i], b = pbeg[i + 1];
    KMA_HIP(hipEventRecord(c->piece_ready[i], cs));
    KMA_HIP(hipStreamWaitEvent(s, c->piece_ready[i], 0));
    if (both_copies) {
      KMA_HIP(hipEventRecord(c->piece_ready2[i], c->copy[1]));
      KMA_HIP(hipStreamWaitEvent(s, c->piece_ready2[i], 0));
    }
    if (b > a)
      if (int rc = annotate_proteins_on(t, r, c->ws, c->d_in.p, c->d_off.p + a, b - a,
                                        hoff[b] - hoff[a], min_hits, flags, d_fid + a,
                                        d_cnt + a, d_st + a, d_tally, n_fid, s,
                                        packed ? Input::kStream : Input::kAscii, hoff[a]))
        return rc;
    return outputs_back(i, a, b);
  };
  if (streamed) {
    // Streamed staging: the whole stream is packed by ONE staging-pool job in chunks of
    // kChunkGroups groups, in stream order, and the calling thread copies it in segments (at most
    // kSegGroups groups, never across a piece boundary) as soon as a segment's chunks are all
    // packed, packing chunks itself while it waits; a piece's kernel follows its last segment.
    // Round 4 packed a whole piece before its one copy: the link idled while each piece was
    // packed (0.24 and 0.30 ms gaps while the pieces ramped up, profiles/r05/e2e_piecewise_r05d/events.jsonl).
    // Segments of >= 2.6 MB keep the copies near the one-copy rate (2 MiB copies: 42 vs 51 GB/s).
    constexpr uint64_t kChunkGroups = 1u << 12, kSegGroups = 1u << 18, kFirstSegGroups = 1u << 16;
    const uint64_t tail = in_bytes - 40 * n_groups;  // the kernel's read padding, zeroed
    struct Seg {
      uint64_t g0, g1;
      int piece;
      bool last;  // the piece's last segment: its kernel follows the copy
      uint32_t chunks;
    };
    std::vector<Seg> segs;
    std::vector<uint32_t> chunk_seg;  // chunk -> segment
    std::vector<uint64_t> chunk_g0;   // chunk -> first group
    uint64_t g = 0;
    for (int i = 0; i < n_pieces; ++i) {  // the group holding a boundary goes with the earlier piece
      const uint64_t g1 = i + 1 < n_pieces
                              ? std::max(g, std::min(n_groups, (hoff[pbeg[i + 1]] + 63) / 64))
                              : n_groups;
      do {
        const uint64_t want = std::min(kSegGroups, kFirstSegGroups << std::min<size_t>(segs.size(), 2));
        const uint64_t e = std::min(g1, g + want);
        uint32_t nch = 0;
        for (uint64_t ch = g; ch < e; ch += kChunkGroups, ++nch) {
          chunk_seg.push_back((uint32_t)segs.size());
          chunk_g0.push_back(ch);
        }
        segs.push_back({g, e, i, e == g1, nch});
        g = e;
      } while (g < g1);
    }
    std::unique_ptr<std::atomic<uint32_t>[]> left(new std::atomic<uint32_t>[segs.size()]);
    for (size_t k = 0; k < segs.size(); ++k) left[k].store(segs[k].chunks, std::memory_order_relaxed);
    int rc_copy = KMA_OK;
    staging_pool().run_with(
        chunk_seg.size(), staging_threads(),
        [&](uint64_t ci) {
          const Seg& sg = segs[chunk_seg[ci]];
          const uint64_t g0 = chunk_g0[ci], g1 = std::min(sg.g1, g0 + kChunkGroups);
          const uint64_t r0 = 64 * g0, r1 = std::min(64 * g1, nres);
          const uint64_t bytes = 40 * (g1 - g0) + (g1 == n_groups ? tail : 0);
          kma::pack_residues_host(t->lut, residues + base + r0, r1 > r0 ? r1 - r0 : 0,
                                  hin + 40 * g0, bytes);
          left[chunk_seg[ci]].fetch_sub(1, std::memory_order_release);
        },
        [&](auto& help) {
          for (size_t k = 0; k < segs.size() && rc_copy == KMA_OK; ++k) {
            const Clock::time_point t_w = Clock::now();
            while (left[k].load(std::memory_order_acquire) != 0)
              if (!help()) std::this_thread::yield();
            const Clock::time_point t_issue = Clock::now();
            t_stage += std::chrono::duration<double, std::milli>(t_issue - t_w).count();
            const Seg& sg = segs[k];
            // (The copies run at ~57 GB/s until the first piece kernel starts, then at ~36 GB/s:
            // the engines' writes into HBM share the fabric with the probe's gathers at their
            // request ceiling. Measured and not kept: the piece kernels reading the packed stream
            // from the pinned buffer over PCIe instead, 5.5 vs 3.4 ms of kernels, calls 7.1-7.7
            // vs 5.3-7.0 ms; the pool packing straight into fine-grained device memory through the
            // BAR, 44 GB/s alone and 7.9 ms beside a DMA that takes 3.4 ms alone, where packing
            // into pinned memory beside it takes 3.4 ms: profiles/r05/host_paths_r05/; and the
            // piece kernels but the last on a CU-masked stream (half the CUs), to leave the copies
            // fabric: no effect in one process alternating both, 5.22-5.47 vs 5.25-5.39 ms,
            // profiles/r05/host_cu_mask/.)
            // Segments alternate over the two copy streams (two DMA engines: 52 vs 44 GB/s on
            // one stream, profiles/r05/e2e_streamed_fifo_r05i), in stream order on each, and a
            // piece's kernel waits for both: a piece's data lands as early as the link allows.
            // (Round 5's first build put whole pieces on alternate streams: consecutive pieces
            // shared the link and every other kernel waited ~0.09 ms for its data,
            // profiles/r05/e2e_streamed_r05h.)
            hipStream_t cs = c->copy[0];
            if (k & 1) cs = c->copy[1];
            const uint64_t bytes = 40 * (sg.g1 - sg.g0) + (sg.g1 == n_groups ? tail : 0);
            if (sg.g1 == n_groups && sg.chunks == 0) std::memset(hin + 40 * n_groups, 0, tail);
            if (bytes) {
              const hipError_t e = hipMemcpyAsync(c->d_in.p + 40 * sg.g0, hin + 40 * sg.g0, bytes,
                                                  hipMemcpyHostToDevice, cs);
              if (e != hipSuccess) rc_copy = fail(KMA_E_DEVICE, "hipMemcpyAsync: %s", hipGetErrorString(e));
            }
            if (rc_copy == KMA_OK && sg.last) rc_copy = launch_piece(sg.piece, c->copy[0], true);
            t_launch += ms_since(t_issue);
          }
          while (help()) {}  // (after an error: the job still completes)
        });
    if (rc_copy) return rc_copy;
  } else {
    uint64_t ga = 0;  // packed: first stream group the piece stages
    for (int i = 0; i < n_pieces; ++i) {
      hipStream_t cs = c->copy[i & 1];
      const Clock::time_point t_piece = Clock::now();
      const uint64_t ra = hoff[pbeg[i]], rb = i + 1 < n_pieces ? hoff[pbeg[i + 1]] : nres;
      if (packed) {  // the group holding the piece boundary goes with the earlier piece
        const uint64_t gb = i + 1 < n_pieces ? std::min(n_groups, (rb + 63) / 64) : n_groups;
        KMA_HIP(stage_pack_h2d(c->d_in.p, hin, t->lut, residues + base, nres, ga, gb,
                               i + 1 == n_pieces ? in_bytes - 40 * n_groups : 0, cs));
        ga = gb;
      } else {
        KMA_HIP(stage_h2d(c->d_in.p + ra, hin + ra, residues + base + ra, rb - ra, r.device, cs));
        if (i + 1 == n_pieces) {
          std::memset(hin + nres, 0, in_bytes - nres);
          KMA_HIP(hipMemcpyAsync(c->d_in.p + nres, hin + nres, in_bytes - nres,
                                 hipMemcpyHostToDevice, cs));
        }
      }
      const Clock::time_point t_staged = Clock::now();
      t_stage += std::chrono::duration<double, std::milli>(t_staged - t_piece).count();
      if (int rc = launch_piece(i, cs)) return rc;
      t_launch += ms_since(t_staged);
    }
  }
  // Pieces' outputs into the caller's arrays as they arrive (the later pieces still copy and
  // run meanwhile).
  double t_wait = 0;
  const Clock::time_point t_o = Clock::now();
  for (int i = 0; i < n_pieces; ++i) {
    const Clock::time_point t_w = Clock::now();
    KMA_HIP(hipEventSynchronize(c->out_ready[i]));
    t_wait += ms_since(t_w);
    const uint32_t a = pbeg[i], b = pbeg[i + 1];
    if (b == a) continue;
    pool_memcpy(out_fid + lo + a, hout + a * 4ull, (b - a) * 4ull);
    pool_memcpy(out_count + lo + a, hout + (n + a) * 4ull, (b - a) * 4ull);
    pool_memcpy(out_status + lo + a, hout + n * 8ull + (tally ? n_fid * 4ull : 0) + a, b - a);
  }
  if (tally) std::memcpy(tally, hout + n * 8ull, n_fid * 4ull);
  {
    const double p[kProfFields] = {t_setup, t_stage, t_launch, t_wait, ms_since(t_o) - t_wait,
                                   ms_since(t_call), (double)staging_threads(), (double)n_pieces};
    std::lock_guard<std::mutex> g(g_prof_mu);
    std::copy(p, p + kProfFields, g_prof);
    if (rep < kProfReplicas) std::copy(p, p + kProfFields, g_prof_rep[rep]);
  }
  return KMA_OK;
}
}  // namespace

extern "C" {

// Not in kmeranno.h: measurement hooks (see g_prof). kma_debug_host_profile: the last shard
// call's phases; kma_debug_host_profile_replica: the last shard call of replica `rep` (its index
// in the table's replica list) of a fanned-out host call.
int kma_debug_host_profile(double* out, int n) {
  if (!out || n < 0) return KMA_E_INVALID;
  std::lock_guard<std::mutex> g(g_prof_mu);
  std::copy(g_prof, g_prof + std::min(n, kProfFields), out);
  return KMA_OK;
}
int kma_debug_host_profile_replica(int rep, double* out, int n) {
  if (!out || n < 0 || rep < 0 || rep >= kProfReplicas) return KMA_E_INVALID;
  std::lock_guard<std::mutex> g(g_prof_mu);
  std::copy(g_prof_rep[rep], g_prof_rep[rep] + std::min(n, kProfFields), out);
  return KMA_OK;
}
// Not in kmeranno.h: the CPUs the library sizes its staging jobs by (host_cores).
int kma_debug_host_cores(void) { return (int)host_cores(); }

int kma_workspace_reserve_contigs(kma_workspace* ws, uint64_t n_bases) {
  if (!ws) return fail(KMA_E_INVALID, "null workspace");
  if (n_bases >= (1ull << 39)) return fail(KMA_E_INVALID, "more than 2^39 bases in one call");
  if (ws->d_cstage && n_bases <= ws->contig_cap) return KMA_OK;
  DeviceScope ds(ws->device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", ws->device);
  free_contig_scratch(ws);
  const uint64_t nb = contig_blocks(n_bases);
  const uint64_t ng = (nb + kma::kScanGroup - 1) / kma::kScanGroup;
  KMA_HIP(hipMalloc(&ws->d_cstage, nb * 2 * kma::kContigTile * sizeof(kma_hit)));
  KMA_HIP(hipMalloc(&ws->d_ccounts, ng * kma::kScanGroup * 4));
  KMA_HIP(hipMalloc(&ws->d_cprefix, (ng + 1) * 8));
  KMA_HIP(hipMemset(ws->d_cprefix, 0, (ng + 1) * 8));
  ws->cgroups = ng;
  ws->cpending = false;
  ws->contig_cap = nb * kma::kContigTile;
  return KMA_OK;
}

int kma_workspace_create(int device, kma_workspace** out) {
  if (!out) return fail(KMA_E_INVALID, "null argument");
  DeviceScope ds(device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", device);
  kma_workspace* w = new kma_workspace();
  w->device = device;
  int n_cu = 0;
  if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
      n_cu > 0)
    w->n_cu = n_cu;
  hipError_t e = hipMalloc(&w->d_gset, 2 * kResPad * 4);  // reserve() grows it
  if (e != hipSuccess) {
    delete w;
    return fail(KMA_E_NOMEM, "workspace: %s", hipGetErrorString(e));
  }
  *out = w;
  return KMA_OK;
}

int kma_workspace_reserve(kma_workspace* ws, uint64_t n_residues) {
  return kma_workspace_reserve_batch(ws, n_residues, n_residues / 16 + 256);
}

int kma_workspace_reserve_batch(kma_workspace* ws, uint64_t n_residues, uint64_t n_seq) {
  if (!ws) return fail(KMA_E_INVALID, "null workspace");
  if (n_residues > kMaxResidues)
    return fail(KMA_E_INVALID, "%llu residues in one call (limit 2^32 - 128)",
                (unsigned long long)n_residues);
  if (n_seq >= (1ull << 31)) return fail(KMA_E_INVALID, "more than 2^31 proteins in one call");
  if (ws->d_gset && n_residues <= ws->res_cap) return KMA_OK;
  DeviceScope ds(ws->device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", ws->device);
  free_protein_scratch(ws);
  KMA_HIP(hipMalloc(&ws->d_gset, 2 * (n_residues + kResPad) * 4));
  ws->res_cap = n_residues;
  // The device calls' packed stream (0.625 B per residue), whatever KMA_OPT_PACKED_INPUT is now:
  // a device call that packs must not allocate (it may be graph-captured). Host
  // contexts' workspaces never pack on the device (their calls stage the stream themselves).
  if (!ws->host_ctx) KMA_HIP(hipMalloc(&ws->d_packed, kma::packed_bytes(n_residues + kResPad)));
  return KMA_OK;
}

int kma_workspace_option_set(kma_workspace* ws, int option, int64_t value) {
  if (!ws) return fail(KMA_E_INVALID, "null workspace");
  if (option != KMA_OPT_BLOCK_PROTEINS && option != KMA_OPT_DEFER)
    return fail(KMA_E_INVALID, "option %d is not a workspace option", option);
  if (value != KMA_OPT_DEFAULT && !option_valid(option, value))
    return fail(KMA_E_INVALID, "option %d: value %lld out of range", option, (long long)value);
  (option == KMA_OPT_BLOCK_PROTEINS ? ws->opt_block_proteins : ws->opt_defer) =
      value == KMA_OPT_DEFAULT ? kOptUnset : value;
  return KMA_OK;
}

int kma_workspace_timing(kma_workspace* ws, int enable) {
  if (!ws) return fail(KMA_E_INVALID, "null workspace");
  DeviceScope ds(ws->device);
  if (enable && ws->events.empty()) {
    ws->events.resize(kMaxEv * kTimingRing);
    for (auto& e : ws->events) KMA_HIP(hipEventCreate(&e));
    ws->names.assign(kTimingRing, nullptr);
    ws->n_phases.assign(kTimingRing, 0);
  }
  ws->timing = enable != 0;
  ws->n_timed = 0;
  return KMA_OK;
}

int kma_workspace_phases_read(kma_workspace* ws, uint32_t* n_calls, int* n_phases,
                              double* phase_ms, const char** phase_names) {
  if (!ws || !n_calls || !n_phases || !phase_ms) return fail(KMA_E_INVALID, "null argument");
  DeviceScope ds(ws->device);
  const uint32_t n = std::min(ws->n_timed, kTimingRing);
  *n_calls = 0;
  *n_phases = 0;
  for (int i = 0; i < KMA_MAX_PHASES; ++i) {
    phase_ms[i] = 0.0;
    if (phase_names) phase_names[i] = nullptr;
  }
  if (n == 0) return KMA_OK;
  const uint32_t last = (ws->n_timed - 1) % kTimingRing;  // calls laid out like the last one
  const char* const* names = ws->names[last];
  const int np = ws->n_phases[last];
  for (uint32_t i = 0; i < n; ++i) {
    if (ws->names[i] != names) continue;
    hipEvent_t* e = &ws->events[kMaxEv * i];
    KMA_HIP(hipEventSynchronize(e[np]));
    for (int ph = 0; ph < np; ++ph) {
      float ms = 0;
      KMA_HIP(hipEventElapsedTime(&ms, e[ph], e[ph + 1]));
      phase_ms[ph] += ms;
    }
    ++*n_calls;
  }
  *n_phases = np;
  if (phase_names)
    for (int ph = 0; ph < np; ++ph) phase_names[ph] = names[ph];
  ws->n_timed = 0;
  return KMA_OK;
}

int kma_workspace_timing_read(kma_workspace* ws, uint32_t* n_calls, double* kernel_ms,
                              double* rest_ms) {
  if (!ws || !n_calls || !kernel_ms || !rest_ms) return fail(KMA_E_INVALID, "null argument");
  double ms[KMA_MAX_PHASES];
  const char* names[KMA_MAX_PHASES];
  int np = 0;
  if (int rc = kma_workspace_phases_read(ws, n_calls, &np, ms, names)) return rc;
  // contigs: (probe, scan + emit); proteins: the whole path (every phase), nothing after it
  const bool contigs = np > 0 && names[0] == kContigPhases[0];
  *kernel_ms = 0;
  *rest_ms = 0;
  for (int ph = 0; ph < np; ++ph) (contigs && ph > 0 ? *rest_ms : *kernel_ms) += ms[ph];
  return KMA_OK;
}

int kma_workspace_destroy(kma_workspace* ws) {
  if (!ws) return KMA_OK;
  DeviceScope ds(ws->device);
  for (auto& e : ws->events) (void)hipEventDestroy(e);
  free_protein_scratch(ws);
  free_contig_scratch(ws);
  delete ws;
  return KMA_OK;
}

int kma_annotate_proteins_device(const kma_table* t, kma_workspace* ws, const uint8_t* d_residues,
                                 const uint64_t* d_offsets, uint32_t n_seq, uint64_t n_residues,
                                 int min_hits, uint32_t flags, int32_t* d_fid, int32_t* d_count,
                                 uint8_t* d_status, uint32_t* d_tally, uint32_t n_fid,
                                 void* stream) {
  if (int rc = check_protein_call(t, min_hits, flags)) return rc;
  if (!ws) return fail(KMA_E_INVALID, "null workspace");
  Replica rep;
  if (!replica_on(t, ws->device, &rep))
    return fail(KMA_E_INVALID, "table has no replica on the workspace's device %d", ws->device);
  const Replica* r = &rep;
  if (n_seq == 0) return KMA_OK;
  if (!d_residues || !d_offsets || !d_fid || !d_count || !d_status)
    return fail(KMA_E_INVALID, "null device buffer");
  if ((uintptr_t)d_residues & 7) return fail(KMA_E_INVALID, "residues must be 8-byte aligned");
  if (n_residues > ws->res_cap)
    return fail(KMA_E_CAPACITY, "workspace reserved for %llu residues, call needs %llu",
                (unsigned long long)ws->res_cap, (unsigned long long)n_residues);
  const bool pack = pack_on_device(n_residues);
  if (pack)
    if (int rc = ensure_packed(ws)) return rc;
  DeviceScope ds(r->device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", r->device);
  return annotate_proteins_on(t, *r, ws, d_residues, d_offsets, n_seq, n_residues, min_hits,
                              flags, d_fid, d_count, d_status, d_tally, n_fid,
                              static_cast<hipStream_t>(stream),
                              pack ? Input::kPackOnDevice : Input::kAscii);
}

uint64_t kma_packed_bytes(uint64_t n_residues) { return kma::packed_bytes(n_residues); }

int kma_pack_residues(const kma_table* t, const uint8_t* residues, uint64_t n, uint8_t* out,
                      uint64_t out_bytes) {
  if ((n && !residues) || !out) return fail(KMA_E_INVALID, "null argument");
  if (out_bytes < kma::packed_bytes(n))
    return fail(KMA_E_CAPACITY, "packed stream of %llu residues needs %llu bytes",
                (unsigned long long)n, (unsigned long long)kma::packed_bytes(n));
  uint8_t std_lut[256];
  if (!t) standard_lut(std_lut);
  const uint8_t* lut = t ? t->lut : std_lut;
  // large streams on the staging pool, in chunks of 2^15 groups (64 residues = 40 bytes each)
  constexpr uint64_t kChunkGroups = 1u << 15;
  const uint64_t n_groups = (n + 63) / 64, n_chunks = (n_groups + kChunkGroups - 1) / kChunkGroups;
  if (n_chunks < 4) {
    kma::pack_residues_host(lut, residues, n, out, out_bytes);
    return KMA_OK;
  }
  staging_pool().run(n_chunks, staging_threads(), [&](uint64_t c) {
    const uint64_t g0 = c * kChunkGroups, g1 = std::min(n_groups, g0 + kChunkGroups);
    const uint64_t r0 = 64 * g0, r1 = std::min(64 * g1, n);
    const uint64_t bytes = g1 == n_groups ? out_bytes - 40 * g0 : 40 * (g1 - g0);
    kma::pack_residues_host(lut, residues + r0, r1 - r0, out + 40 * g0, bytes);
  });
  return KMA_OK;
}

int kma_annotate_packed_device(const kma_table* t, kma_workspace* ws, const uint8_t* d_stream,
                               const uint64_t* d_offsets, uint32_t n_seq, uint64_t n_residues,
                               int min_hits, uint32_t flags, int32_t* d_fid, int32_t* d_count,
                               uint8_t* d_status, uint32_t* d_tally, uint32_t n_fid,
                               void* stream) {
  if (int rc = check_protein_call(t, min_hits, flags)) return rc;
  if (!ws) return fail(KMA_E_INVALID, "null workspace");
  Replica rep;
  if (!replica_on(t, ws->device, &rep))
    return fail(KMA_E_INVALID, "table has no replica on the workspace's device %d", ws->device);
  if (n_seq == 0) return KMA_OK;
  if (!d_stream || !d_offsets || !d_fid || !d_count || !d_status)
    return fail(KMA_E_INVALID, "null device buffer");
  if ((uintptr_t)d_stream & 7) return fail(KMA_E_INVALID, "stream must be 8-byte aligned");
  if (n_residues > ws->res_cap)
    return fail(KMA_E_CAPACITY, "workspace reserved for %llu residues, call needs %llu",
                (unsigned long long)ws->res_cap, (unsigned long long)n_residues);
  DeviceScope ds(rep.device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", rep.device);
  return annotate_proteins_on(t, rep, ws, d_stream, d_offsets, n_seq, n_residues, min_hits, flags,
                              d_fid, d_count, d_status, d_tally, n_fid,
                              static_cast<hipStream_t>(stream), Input::kStream, 0);
}

int kma_annotate_proteins(const kma_table* tc, const uint8_t* residues, const uint64_t* offsets,
                          uint32_t n_seq, int min_hits, uint32_t flags, int32_t* out_fid,
                          int32_t* out_count, uint8_t* out_status, uint32_t* out_tally,
                          uint32_t n_fid) {
  if (int rc = check_protein_call(tc, min_hits, flags)) return rc;
  kma_table* t = const_cast<kma_table*>(tc);  // only the context pool is touched
  if (n_seq == 0) return KMA_OK;
  if (!residues || !offsets || !out_fid || !out_count || !out_status)
    return fail(KMA_E_INVALID, "null argument");
  if (const uint32_t s = offsets_decrease_at(offsets, n_seq); s < n_seq)
    return fail(KMA_E_INVALID, "offsets decrease at %u", s);
  const bool tally = out_tally && n_fid;
  const std::vector<Replica> reps = replicas(t);
  const int nr = (int)std::min<uint64_t>(reps.size(), n_seq);
  const std::vector<uint32_t> b = shard_bounds(offsets, n_seq, nr);
  std::vector<std::vector<uint32_t>> part(tally ? nr : 0, std::vector<uint32_t>(n_fid));
  // A replica's share in slices of at most KMA_OPT_HOST_SLICE residues (default 2^31) of whole
  // proteins, one device call each (the kernels index residues with 32 bits); slice tallies add.
  const int64_t so = opt(KMA_OPT_HOST_SLICE);
  const uint64_t slice = so > 0 ? (uint64_t)so : 1ull << 31;
  const size_t width = staging_width(nr);  // each replica's staging jobs
  const int rc = fan_out(nr, [&](int i) {
    ShardWidth sw(width);
    std::vector<uint32_t> st(tally ? n_fid : 0);
    for (uint32_t lo = b[i]; lo < b[i + 1];) {
      uint32_t hi = (uint32_t)(std::upper_bound(offsets + lo + 1, offsets + b[i + 1] + 1,
                                                offsets[lo] + slice) - offsets) - 1;
      if (hi <= lo) hi = lo + 1;  // one protein longer than a slice: a call of its own
      const bool whole = lo == b[i] && hi == b[i + 1];
      uint32_t* tl = !tally ? nullptr : whole ? part[i].data() : st.data();
      if (int rc = protein_shard(t, reps[i], i, residues, offsets, lo, hi, min_hits, flags,
                                 out_fid, out_count, out_status, tl, n_fid))
        return rc;
      if (tally && !whole)
        for (uint32_t f = 0; f < n_fid; ++f) part[i][f] += st[f];
      lo = hi;
    }
    return (int)KMA_OK;
  });
  if (rc != KMA_OK) return rc;
  for (int i = 0; i < (tally ? nr : 0); ++i)  // the tally reduce of the replicas
    for (uint32_t f = 0; f < n_fid; ++f) out_tally[f] += part[i][f];
  return KMA_OK;
}

uint64_t kma_contig_window_count(const uint64_t* offsets, uint32_t n_contig, int k) {
  uint64_t n = 0;
  for (uint32_t c = 0; c < n_contig; ++c) {
    const int64_t len = (int64_t)(offsets[c + 1] - offsets[c]);
    const int64_t per = len - 3 * k - 2;  // sum over frames of max(0, P_f - K), per strand
    if (per > 0) n += 2 * (uint64_t)per;
  }
  return n;
}

int kma_annotate_contigs_device(const kma_table* t, kma_workspace* ws, const uint8_t* d_dna,
                                const uint64_t* d_offsets, uint32_t n_contig, uint64_t n_bases,
                                int genetic_code, kma_hit* d_hits, uint64_t cap,
                                uint64_t* d_n_hits, uint32_t* d_tally, uint32_t n_fid,
                                void* stream) {
  if (!t || !ws) return fail(KMA_E_INVALID, "null table or workspace");
  Replica rep;
  if (!replica_on(t, ws->device, &rep))
    return fail(KMA_E_INVALID, "table has no replica on the workspace's device %d", ws->device);
  const Replica* r = &rep;
  const char* code = ncbi_code(genetic_code);
  if (!code) return fail(KMA_E_INVALID, "unsupported genetic code %d", genetic_code);
  if (!d_n_hits) return fail(KMA_E_INVALID, "null n_hits");
  hipStream_t s = static_cast<hipStream_t>(stream);
  DeviceScope ds(r->device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", r->device);
  if (n_contig == 0 || n_bases == 0) {
    KMA_HIP(hipMemsetAsync(d_n_hits, 0, 8, s));
    return KMA_OK;
  }
  if (!d_dna || !d_offsets) return fail(KMA_E_INVALID, "null device buffer");
  if (n_bases > ws->contig_cap)
    return fail(KMA_E_CAPACITY, "workspace reserved for %llu bases, call needs %llu",
                (unsigned long long)ws->contig_cap, (unsigned long long)n_bases);
  kma::ContigArgs a;
  if (int rc = contig_args(t, *r, ws, d_dna, d_offsets, n_contig, n_bases, code, d_tally, n_fid,
                           s, &a))
    return rc;
  PhaseClock clk(ws, s, kContigPhases, 2);
  KMA_HIP(clk.mark());
  const uint64_t nb = contig_blocks(n_bases);
  KMA_HIP(kma::launch_contigs_probe(a, nb, s));
  KMA_HIP(clk.mark());
  const int rc = enqueue_contig_emit(ws, a, d_hits, cap, d_n_hits, s);
  if (rc == KMA_OK) KMA_HIP(clk.mark());
  return rc;
}

}  // extern "C"

namespace {
// One shard [lo, hi) of a host 6-frame call on replica r. out_hits == null: count the shard's
// hits into *n_hits and accumulate the tally rows of its contigs (tally = the caller's rows
// lo..hi); else emit the *n_hits hits (contig indices relative to lo) into *out_hits.
// strict: the KmerFactory.Strict two-pass form of the peg join (single replica).
int contig_shard(kma_table* t, const Replica& r, const uint8_t* dna, const uint64_t* offsets,
                 uint32_t lo, uint32_t hi, int genetic_code, bool strict,
                 std::vector<kma_hit>* out_hits, uint64_t* n_hits, uint32_t* tally,
                 uint32_t n_fid) {
  const uint32_t n = hi - lo;
  const uint64_t base = offsets[lo], total = offsets[hi] - base;
  if (!out_hits) *n_hits = 0;
  if (n == 0 || total == 0) return KMA_OK;
  const char* code = ncbi_code(genetic_code);
  HostCtx* c = nullptr;
  if (int rc = acquire_ctx(t, r.device, &c)) return rc;
  CtxGuard guard{t, c};
  DeviceScope ds(r.device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", r.device);
  if (int rc = kma_workspace_reserve_contigs(c->ws, total)) return rc;
  const size_t in_bytes = (total + 64 + 7) & ~7ull, off_bytes = (n + 1) * 8ull;
  const size_t tb = tally ? (size_t)n * n_fid * 4 : 0;
  KMA_HIP(c->d_in.reserve(in_bytes));
  KMA_HIP(c->d_off.reserve(n + 1));
  KMA_HIP(c->h_in.reserve(in_bytes + off_bytes + tb));
  uint8_t* hin = c->h_in.p;
  hipStream_t s = c->stream;
  KMA_HIP(stage_h2d(c->d_in.p, hin, dna + base, total, r.device, s));
  std::memset(hin + total, 0, in_bytes - total);
  KMA_HIP(hipMemcpyAsync(c->d_in.p + total, hin + total, in_bytes - total,
                         hipMemcpyHostToDevice, s));
  uint64_t* hoff = reinterpret_cast<uint64_t*>(hin + in_bytes);
  for (uint32_t i = 0; i <= n; ++i) hoff[i] = offsets[lo + i] - base;
  KMA_HIP(hipMemcpyAsync(c->d_off.p, hoff, off_bytes, hipMemcpyHostToDevice, s));
  // d_out: [n_hits u64, pad | tally]; slot counts (strict) in d_aux; hits in d_hits.
  KMA_HIP(c->d_out.reserve(16 + tb));
  uint64_t* d_n = reinterpret_cast<uint64_t*>(c->d_out.p);
  uint32_t* d_tally = tally ? reinterpret_cast<uint32_t*>(c->d_out.p + 16) : nullptr;
  if (tb) {
    uint8_t* ht = hin + in_bytes + off_bytes;
    std::memcpy(ht, tally, tb);
    KMA_HIP(hipMemcpyAsync(d_tally, ht, tb, hipMemcpyHostToDevice, s));
  }
  kma::ContigArgs a;
  if (int rc = contig_args(t, r, c->ws, c->d_in.p, c->d_off.p, n, total, code, d_tally, n_fid, s,
                           &a))
    return rc;
  const uint64_t nb = contig_blocks(total);
  if (strict) {
    const uint64_t n_slots = t->n_buckets * kma::slots_for_k(t->k);
    KMA_HIP(c->d_aux.reserve(n_slots));
    KMA_HIP(hipMemsetAsync(c->d_aux.p, 0, n_slots * 4, s));
    a.slot_count = c->d_aux.p;
    a.strict_pass = 1;  // count every table key's locations
    uint64_t* const gs = a.group_sum;
    a.group_sum = nullptr;  // no emit follows this pass
    KMA_HIP(kma::launch_contigs_probe(a, nb, s));
    a.group_sum = gs;
    a.strict_pass = 2;  // keep keys with exactly one location
  }
  KMA_HIP(kma::launch_contigs_probe(a, nb, s));
  if (!out_hits) {  // pass 1: count (and tally)
    if (int rc = enqueue_contig_emit(c->ws, a, nullptr, 0, d_n, s)) return rc;
    KMA_HIP(c->h_out.reserve(16 + tb));
    KMA_HIP(hipMemcpyAsync(c->h_out.p, d_n, 8, hipMemcpyDeviceToHost, s));
    if (tb) KMA_HIP(hipMemcpyAsync(c->h_out.p + 16, d_tally, tb, hipMemcpyDeviceToHost, s));
    KMA_HIP(hipStreamSynchronize(s));
    std::memcpy(n_hits, c->h_out.p, 8);
    if (tb) std::memcpy(tally, c->h_out.p + 16, tb);
    return KMA_OK;
  }
  // pass 2: emit into d_hits (sized by pass 1's count, passed in *n_hits)
  const uint64_t cap = *n_hits;
  KMA_HIP(c->d_hits.reserve(std::max<uint64_t>(cap, 1)));
  if (int rc = enqueue_contig_emit(c->ws, a, c->d_hits.p, cap, d_n, s)) return rc;
  KMA_HIP(c->h_out.reserve(16 + cap * sizeof(kma_hit)));
  KMA_HIP(hipMemcpyAsync(c->h_out.p, d_n, 8, hipMemcpyDeviceToHost, s));
  KMA_HIP(hipMemcpyAsync(c->h_out.p + 16, c->d_hits.p, cap * sizeof(kma_hit),
                         hipMemcpyDeviceToHost, s));
  KMA_HIP(hipStreamSynchronize(s));
  uint64_t nh = 0;
  std::memcpy(&nh, c->h_out.p, 8);
  if (nh != cap) return fail(KMA_E_DEVICE, "6-frame pass: %llu hits, then %llu",
                             (unsigned long long)cap, (unsigned long long)nh);
  out_hits->resize(nh);
  std::memcpy(out_hits->data(), c->h_out.p + 16, nh * sizeof(kma_hit));
  return KMA_OK;
}

int annotate_contigs_host(kma_table* t, const uint8_t* dna, const uint64_t* offsets,
                          uint32_t n_contig, int genetic_code, bool strict, kma_hit* out_hits,
                          uint64_t cap, uint64_t* n_hits, uint32_t* out_tally, uint32_t n_fid) {
  if (!t || !n_hits) return fail(KMA_E_INVALID, "null argument");
  if (!ncbi_code(genetic_code))
    return fail(KMA_E_INVALID, "unsupported genetic code %d", genetic_code);
  *n_hits = 0;
  if (n_contig == 0) return KMA_OK;
  if (!dna || !offsets) return fail(KMA_E_INVALID, "null argument");
  for (uint32_t c = 0; c < n_contig; ++c)
    if (offsets[c + 1] < offsets[c]) return fail(KMA_E_INVALID, "offsets decrease at %u", c);
  if (offsets[n_contig] - offsets[0] >= (1ull << 39))
    return fail(KMA_E_INVALID, "more than 2^39 bases in one call");
  const bool tally = out_tally && n_fid;
  const std::vector<Replica> reps = replicas(t);
  const int nr = strict ? 1 : (int)std::min<uint64_t>(reps.size(), n_contig);
  const std::vector<uint32_t> b = shard_bounds(offsets, n_contig, nr);
  // Pass 1 counts (and tallies into copies: nothing is written on KMA_E_CAPACITY); pass 2
  // emits. A shard's hits are produced only if the whole call fits in cap.
  std::vector<uint64_t> nh(nr, 0);
  std::vector<std::vector<uint32_t>> tal(tally ? nr : 0);
  for (int i = 0; i < (tally ? nr : 0); ++i)
    tal[i].assign(out_tally + (uint64_t)b[i] * n_fid, out_tally + (uint64_t)b[i + 1] * n_fid);
  const size_t width = staging_width(nr);
  int rc = fan_out(nr, [&](int i) {
    ShardWidth sw(width);
    return contig_shard(t, reps[i], dna, offsets, b[i], b[i + 1], genetic_code, strict,
                        nullptr, &nh[i], tally ? tal[i].data() : nullptr, n_fid);
  });
  if (rc != KMA_OK) return rc;
  uint64_t total = 0;
  for (uint64_t x : nh) total += x;
  *n_hits = total;
  if (total > cap || (total && !out_hits))
    return fail(KMA_E_CAPACITY, "%llu hits, capacity %llu", (unsigned long long)total,
                (unsigned long long)(out_hits ? cap : 0));
  for (int i = 0; i < (tally ? nr : 0); ++i)
    std::copy(tal[i].begin(), tal[i].end(), out_tally + (uint64_t)b[i] * n_fid);
  if (total == 0) return KMA_OK;
  std::vector<std::vector<kma_hit>> hv(nr);
  rc = fan_out(nr, [&](int i) {
    ShardWidth sw(width);
    if (nh[i] == 0) return KMA_OK;
    return contig_shard(t, reps[i], dna, offsets, b[i], b[i + 1], genetic_code, strict,
                        &hv[i], &nh[i], nullptr, 0);
  });
  if (rc != KMA_OK) return rc;
  uint64_t o = 0;
  for (int i = 0; i < nr; ++i)
    for (const kma_hit& h : hv[i]) {
      out_hits[o] = h;
      out_hits[o++].contig += b[i];
    }
  return KMA_OK;
}
}  // namespace

extern "C" {

int kma_annotate_contigs(const kma_table* t, const uint8_t* dna, const uint64_t* offsets,
                         uint32_t n_contig, int genetic_code, kma_hit* out_hits, uint64_t cap,
                         uint64_t* n_hits, uint32_t* out_tally, uint32_t n_fid) {
  return annotate_contigs_host(const_cast<kma_table*>(t), dna, offsets, n_contig, genetic_code,
                               false, out_hits, cap, n_hits, out_tally, n_fid);
}

int kma_connect_pegs(const kma_table* t, const uint8_t* dna, const uint64_t* offsets,
                     uint32_t n_contig, int genetic_code, int strict, kma_hit* out_hits,
                     uint64_t cap, uint64_t* n_hits) {
  return annotate_contigs_host(const_cast<kma_table*>(t), dna, offsets, n_contig, genetic_code,
                               strict != 0, out_hits, cap, n_hits, nullptr, 0);
}

int kma_peg_table_create(const uint8_t* residues, const uint64_t* offsets, uint32_t n_peg, int k,
                         int device, double load_factor, kma_table** out,
                         uint64_t* n_windows) {
  if (!out) return fail(KMA_E_INVALID, "null argument");
  *out = nullptr;
  if (int rc = check_k(k)) return rc;
  if (load_factor <= 0) load_factor = 0.5;
  if (load_factor > 0.95) return fail(KMA_E_INVALID, "load factor %.3f > 0.95", load_factor);
  if (n_peg > KMA_MAX_FID + 1u) return fail(KMA_E_INVALID, "more than 2^22 pegs");
  if (n_peg && (!residues || !offsets)) return fail(KMA_E_INVALID, "null argument");
  for (uint32_t s = 0; s < n_peg; ++s)
    if (offsets[s + 1] < offsets[s]) return fail(KMA_E_INVALID, "offsets decrease at %u", s);
  const uint64_t base = n_peg ? offsets[0] : 0, total = n_peg ? offsets[n_peg] - base : 0;
  uint8_t lut[256];
  standard_lut(lut);
  DeviceScope ds(device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d): %s", device,
                                        hipGetErrorString(ds.err));
  DevBufs b;
  uint8_t *d_res, *d_lut, *d_flags;
  uint64_t *d_off, *d_keys, *d_keys2, *d_n;
  uint32_t *d_pegs, *d_pegs2;
  const uint64_t nw = std::max<uint64_t>(total, 1);
  KMA_HIP(b.alloc(&d_res, total + 64));
  KMA_HIP(b.alloc(&d_off, (n_peg + 1) * 8ull));
  KMA_HIP(b.alloc(&d_lut, 256));
  KMA_HIP(b.alloc(&d_keys, nw * 8));
  KMA_HIP(b.alloc(&d_keys2, nw * 8));
  KMA_HIP(b.alloc(&d_pegs, nw * 4));
  KMA_HIP(b.alloc(&d_pegs2, nw * 4));
  KMA_HIP(b.alloc(&d_flags, nw));
  KMA_HIP(b.alloc(&d_n, 8));
  KMA_HIP(hipMemset(d_n, 0, 8));
  uint64_t n_sel = 0, windows = 0;
  if (total) {
    std::vector<uint64_t> rel(offsets, offsets + n_peg + 1);
    for (auto& o : rel) o -= base;
    for (uint32_t s = 0; s < n_peg; ++s) {
      const uint64_t L = rel[s + 1] - rel[s];
      if (L > (uint64_t)k) windows += L - k;
    }
    KMA_HIP(hipMemcpy(d_res, residues + base, total, hipMemcpyHostToDevice));
    KMA_HIP(hipMemset(d_res + total, 0, 64));
    KMA_HIP(hipMemcpy(d_off, rel.data(), (n_peg + 1) * 8ull, hipMemcpyHostToDevice));
    KMA_HIP(hipMemcpy(d_lut, lut, 256, hipMemcpyHostToDevice));
    KMA_HIP(kma::launch_peg_windows(d_res, d_off, n_peg, k, d_lut, d_keys, d_pegs, nullptr));
    size_t t1 = 0, t2 = 0;
    KMA_HIP(kma::launch_sort_pairs(nullptr, &t1, d_keys, d_keys2, d_pegs, d_pegs2, total, 5 * k,
                                   nullptr));
    KMA_HIP(kma::launch_select_flagged(nullptr, &t2, d_keys2, d_pegs2, d_flags, d_keys, d_pegs,
                                       d_n, total, nullptr));
    void* d_temp;
    size_t tb = std::max(t1, t2);
    KMA_HIP(b.alloc(&d_temp, tb));
    KMA_HIP(kma::launch_sort_pairs(d_temp, &tb, d_keys, d_keys2, d_pegs, d_pegs2, total, 5 * k,
                                   nullptr));
    KMA_HIP(kma::launch_singleton_flags(d_keys2, total, d_flags, nullptr));
    tb = std::max(t1, t2);
    KMA_HIP(kma::launch_select_flagged(d_temp, &tb, d_keys2, d_pegs2, d_flags, d_keys, d_pegs,
                                       d_n, total, nullptr));
    KMA_HIP(hipMemcpy(&n_sel, d_n, 8, hipMemcpyDeviceToHost));
  }
  if (n_windows) *n_windows = windows;
  const int rc = create_from_device_keys(d_keys, d_pegs, n_sel, k, device, load_factor, lut, out);
  if (rc != KMA_OK) return rc;
  (*out)->info.n_rows = windows;
  return KMA_OK;
}

int kma_build_signatures(const uint8_t* residues, const uint64_t* offsets, const int32_t* roles,
                         uint32_t n_seq, int k, uint32_t flags, int device, uint64_t* out_keys,
                         uint32_t* out_roles, uint64_t cap, uint64_t* n_out) {
  if (!n_out) return fail(KMA_E_INVALID, "null argument");
  *n_out = 0;
  if (int rc = check_k(k)) return rc;
  if (flags & ~KMA_F_END_EXCLUSIVE) return fail(KMA_E_INVALID, "bad flags");
  if (n_seq == 0) return KMA_OK;
  if (!residues || !offsets || !roles) return fail(KMA_E_INVALID, "null argument");
  for (uint32_t s = 0; s < n_seq; ++s) {
    if (offsets[s + 1] < offsets[s]) return fail(KMA_E_INVALID, "offsets decrease at %u", s);
    if (roles[s] >= (int32_t)kma::kBuildNeg)
      return fail(KMA_E_INVALID, "role %d of protein %u >= 2^24 - 1", roles[s], s);
  }
  const uint64_t base = offsets[0], total = offsets[n_seq] - base;
  if (total == 0) return KMA_OK;
  if (total >= (1ull << 31)) return fail(KMA_E_INVALID, "more than 2^31 residues in one call");
  uint8_t lut[256];
  standard_lut(lut);
  std::vector<uint64_t> rel(offsets, offsets + n_seq + 1);
  for (auto& o : rel) o -= base;
  DeviceScope ds(device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d): %s", device,
                                        hipGetErrorString(ds.err));
  DevBufs b;
  uint8_t *d_res, *d_lut, *d_flags;
  uint64_t *d_off, *d_ka, *d_kb, *d_n;
  int32_t* d_roles;
  uint32_t *d_alpha, *d_ta, *d_tb, *d_head, *d_run;
  KMA_HIP(b.alloc(&d_res, total + 64));
  KMA_HIP(b.alloc(&d_off, (n_seq + 1) * 8ull));
  KMA_HIP(b.alloc(&d_roles, n_seq * 4ull));
  KMA_HIP(b.alloc(&d_lut, 256));
  KMA_HIP(b.alloc(&d_ka, total * 8));
  KMA_HIP(b.alloc(&d_kb, total * 8));
  KMA_HIP(b.alloc(&d_ta, total * 4));
  KMA_HIP(b.alloc(&d_tb, total * 4));
  KMA_HIP(b.alloc(&d_head, total * 4));
  KMA_HIP(b.alloc(&d_run, total * 4));
  KMA_HIP(b.alloc(&d_flags, total));
  KMA_HIP(b.alloc(&d_n, 16));
  KMA_HIP(b.alloc(&d_alpha, 4));
  KMA_HIP(hipMemcpy(d_res, residues + base, total, hipMemcpyHostToDevice));
  KMA_HIP(hipMemset(d_res + total, 0, 64));
  KMA_HIP(hipMemcpy(d_off, rel.data(), (n_seq + 1) * 8ull, hipMemcpyHostToDevice));
  KMA_HIP(hipMemcpy(d_roles, roles, n_seq * 4ull, hipMemcpyHostToDevice));
  KMA_HIP(hipMemcpy(d_lut, lut, 256, hipMemcpyHostToDevice));
  KMA_HIP(hipMemset(d_alpha, 0, 4));
  KMA_HIP(kma::launch_build_windows(d_res, d_off, n_seq, d_roles, k,
                                    (flags & KMA_F_END_EXCLUSIVE) ? 1 : 0, d_lut, d_ka, d_ta,
                                    d_alpha, nullptr));
  // (key, role) pairs sorted by key; RoleCounter per key run; select the good runs' heads
  size_t t1 = 0, t2 = 0, t3 = 0;
  KMA_HIP(kma::launch_sort_pairs(nullptr, &t1, d_ka, d_kb, d_ta, d_tb, total, 5 * k, nullptr));
  KMA_HIP(kma::launch_signature_flags(d_kb, d_tb, total, d_flags, d_head, d_run, nullptr, &t2,
                                      nullptr));
  KMA_HIP(kma::launch_select_flagged(nullptr, &t3, d_kb, d_tb, d_flags, d_ka, d_ta, d_n, total,
                                     nullptr));
  const size_t tb = std::max(t1, std::max(t2, t3));
  void* d_temp;
  KMA_HIP(b.alloc(&d_temp, tb ? tb : 1));
  size_t t = tb;
  KMA_HIP(kma::launch_sort_pairs(d_temp, &t, d_ka, d_kb, d_ta, d_tb, total, 5 * k, nullptr));
  t = tb;
  KMA_HIP(kma::launch_signature_flags(d_kb, d_tb, total, d_flags, d_head, d_run, d_temp, &t,
                                      nullptr));
  t = tb;
  KMA_HIP(kma::launch_select_flagged(d_temp, &t, d_kb, d_tb, d_flags, d_ka, d_ta, d_n, total,
                                     nullptr));
  uint64_t n_sel = 0;
  uint32_t alpha = 0;
  KMA_HIP(hipMemcpy(&n_sel, d_n, 8, hipMemcpyDeviceToHost));
  KMA_HIP(hipMemcpy(&alpha, d_alpha, 4, hipMemcpyDeviceToHost));
  if (alpha)
    return fail(KMA_E_ALPHABET, "a protein window holds a byte outside A-Z and '*'");
  *n_out = n_sel;
  if (n_sel > cap || (n_sel && (!out_keys || !out_roles)))
    return fail(KMA_E_CAPACITY, "%llu signature kmers, capacity %llu",
                (unsigned long long)n_sel, (unsigned long long)cap);
  if (n_sel == 0) return KMA_OK;
  KMA_HIP(hipMemcpy(out_keys, d_ka, n_sel * 8, hipMemcpyDeviceToHost));
  KMA_HIP(hipMemcpy(out_roles, d_ta, n_sel * 4, hipMemcpyDeviceToHost));
  return KMA_OK;
}

// ---- ProteinKmers.distance (GeneCopyProcessor.java:129-162) ------------------------------------
int kma_protein_distances(const uint8_t* residues, const uint64_t* offsets, uint32_t n_seq, int k,
                          uint32_t flags, const uint32_t* pair_a, const uint32_t* pair_b,
                          uint64_t n_pairs, int device, uint32_t* out_sim, uint32_t* out_size,
                          double* out_dist) {
  if (k < 2 || k > 12) return fail(KMA_E_INVALID, "kmer size %d outside 2..12", k);
  if (flags & ~KMA_F_END_EXCLUSIVE) return fail(KMA_E_INVALID, "bad flags");
  if (n_pairs && (!pair_a || !pair_b || !out_sim)) return fail(KMA_E_INVALID, "null argument");
  if (n_seq && (!residues || !offsets)) return fail(KMA_E_INVALID, "null argument");
  for (uint64_t i = 0; i < n_pairs; ++i)
    if (pair_a[i] >= n_seq || pair_b[i] >= n_seq)
      return fail(KMA_E_INVALID, "pair %llu indexes a protein >= %u", (unsigned long long)i,
                  n_seq);
  for (uint32_t s = 0; s < n_seq; ++s)
    if (offsets[s + 1] < offsets[s]) return fail(KMA_E_INVALID, "offsets decrease at %u", s);
  const uint64_t base = n_seq ? offsets[0] : 0, total = n_seq ? offsets[n_seq] - base : 0;
  if (total >= (1ull << 31)) return fail(KMA_E_INVALID, "more than 2^31 residues in one call");
  if (n_seq == 0 || (n_pairs == 0 && !out_size)) return KMA_OK;
  DeviceScope ds(device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d): %s", device,
                                        hipGetErrorString(ds.err));
  std::vector<uint64_t> rel(offsets, offsets + n_seq + 1);
  for (auto& o : rel) o -= base;
  DevBufs b;
  uint8_t* d_res;
  uint64_t *d_off, *d_keys, *d_sorted;
  uint32_t *d_size, *d_pa, *d_pb, *d_sim, *d_alpha;
  const uint64_t nw = std::max<uint64_t>(total, 1), np = std::max<uint64_t>(n_pairs, 1);
  KMA_HIP(b.alloc(&d_res, total + 64));
  KMA_HIP(b.alloc(&d_off, (n_seq + 1) * 8ull));
  KMA_HIP(b.alloc(&d_keys, nw * 8));
  KMA_HIP(b.alloc(&d_sorted, nw * 8));
  KMA_HIP(b.alloc(&d_size, n_seq * 4ull));
  KMA_HIP(b.alloc(&d_pa, np * 4));
  KMA_HIP(b.alloc(&d_pb, np * 4));
  KMA_HIP(b.alloc(&d_sim, np * 4));
  KMA_HIP(b.alloc(&d_alpha, 4));
  KMA_HIP(hipMemcpy(d_res, residues + base, total, hipMemcpyHostToDevice));
  KMA_HIP(hipMemset(d_res + total, 0, 64));
  KMA_HIP(hipMemcpy(d_off, rel.data(), (n_seq + 1) * 8ull, hipMemcpyHostToDevice));
  if (n_pairs) {
    KMA_HIP(hipMemcpy(d_pa, pair_a, n_pairs * 4, hipMemcpyHostToDevice));
    KMA_HIP(hipMemcpy(d_pb, pair_b, n_pairs * 4, hipMemcpyHostToDevice));
  }
  KMA_HIP(hipMemset(d_alpha, 0, 4));
  KMA_HIP(kma::launch_window_keys(d_res, d_off, n_seq, k, (flags & KMA_F_END_EXCLUSIVE) ? 1 : 0,
                                  d_keys, d_alpha, nullptr));
  size_t tb = 0;
  KMA_HIP(kma::launch_segmented_sort(nullptr, &tb, d_keys, d_sorted, total, n_seq, d_off,
                                     d_off + 1, 5 * k, nullptr));
  void* d_temp;
  KMA_HIP(b.alloc(&d_temp, tb));
  KMA_HIP(kma::launch_segmented_sort(d_temp, &tb, d_keys, d_sorted, total, n_seq, d_off,
                                     d_off + 1, 5 * k, nullptr));
  KMA_HIP(kma::launch_distinct(d_sorted, d_off, n_seq, d_size, nullptr));
  if (n_pairs)
    KMA_HIP(kma::launch_pairs(d_sorted, d_off, d_size, d_sorted, d_off, d_size, d_pa, d_pb,
                              n_pairs, d_sim, nullptr));
  uint32_t alpha = 0;
  KMA_HIP(hipMemcpy(&alpha, d_alpha, 4, hipMemcpyDeviceToHost));
  if (alpha) return fail(KMA_E_ALPHABET, "a protein window holds a byte outside A-Z and '*'");
  std::vector<uint32_t> size(n_seq);
  KMA_HIP(hipMemcpy(size.data(), d_size, n_seq * 4ull, hipMemcpyDeviceToHost));
  if (out_size) std::memcpy(out_size, size.data(), n_seq * 4ull);
  if (n_pairs) KMA_HIP(hipMemcpy(out_sim, d_sim, n_pairs * 4, hipMemcpyDeviceToHost));
  if (out_dist)
    for (uint64_t i = 0; i < n_pairs; ++i) {
      // SequenceKmers.distance restated: 1 - similarity / union, 1.0 when nothing is shared
      const uint32_t sim = out_sim[i];
      const double uni = (double)size[pair_a[i]] + (double)size[pair_b[i]] - (double)sim;
      out_dist[i] = sim > 0 ? 1.0 - (double)sim / uni : 1.0;
    }
  return KMA_OK;
}

int kma_protein_best_match(const uint8_t* residues, const uint64_t* offsets, uint32_t n_seq, int k,
                           uint32_t flags, const uint32_t* query, const uint64_t* cand_off,
                           const uint32_t* cand, uint32_t n_query, double max_dist, int device,
                           int32_t* out_best, double* out_best_dist) {
  if (n_query && (!query || !cand_off || !out_best)) return fail(KMA_E_INVALID, "null argument");
  const uint64_t n_pairs = n_query ? cand_off[n_query] - cand_off[0] : 0;
  if (n_pairs && !cand) return fail(KMA_E_INVALID, "null argument");
  for (uint32_t q = 0; q < n_query; ++q)
    if (cand_off[q + 1] < cand_off[q]) return fail(KMA_E_INVALID, "cand_off decreases at %u", q);
  std::vector<uint32_t> pa(n_pairs), pb(n_pairs), sim(n_pairs);
  std::vector<double> dist(n_pairs);
  for (uint32_t q = 0; q < n_query; ++q)
    for (uint64_t i = cand_off[q]; i < cand_off[q + 1]; ++i) {
      pa[i - cand_off[0]] = query[q];
      pb[i - cand_off[0]] = cand[i];
    }
  if (int rc = kma_protein_distances(residues, offsets, n_seq, k, flags, pa.data(), pb.data(),
                                     n_pairs, device, sim.data(), nullptr, dist.data()))
    return rc;
  // GeneCopyProcessor.java:135-146: fDist = maxDist; for each candidate in order,
  // if (f2Dist <= fDist) { fDist = f2Dist; found = f2; }
  for (uint32_t q = 0; q < n_query; ++q) {
    double best = max_dist;
    int32_t found = -1;
    for (uint64_t i = cand_off[q]; i < cand_off[q + 1]; ++i) {
      const double d = dist[i - cand_off[0]];
      if (d <= best) {
        best = d;
        found = (int32_t)cand[i];
      }
    }
    out_best[q] = found;
    if (out_best_dist) out_best_dist[q] = best;
  }
  return KMA_OK;
}

}  // extern "C"

extern "C" {

int kma_propose_pegs(const kma_hit* hits, uint64_t n_hits, const uint32_t* peg_len,
                     uint32_t n_peg, int k, double min_strength, double max_fuzz,
                     double min_fuzz, int device, kma_proposal* out, uint64_t cap,
                     uint64_t* n_out, uint64_t* stats) {
  if (!n_out || !stats) return fail(KMA_E_INVALID, "null argument");
  if (int rc = check_k(k)) return rc;
  *n_out = 0;
  stats[0] = stats[1] = stats[2] = stats[3] = 0;
  if (n_hits == 0) return KMA_OK;
  if (!hits || !peg_len || n_peg == 0) return fail(KMA_E_INVALID, "null argument");
  if (cap && !out) return fail(KMA_E_INVALID, "null output");
  if (n_hits >= (1ull << 31)) return fail(KMA_E_INVALID, "more than 2^31 connections");
  if ((uint64_t)n_peg * 6 >= (1ull << 32)) return fail(KMA_E_INVALID, "too many pegs");
  for (uint64_t i = 0; i < n_hits; ++i) {
    const kma_hit& h = hits[i];
    if (h.fid >= n_peg) return fail(KMA_E_INVALID, "connection %llu: peg %u >= %u",
                                    (unsigned long long)i, h.fid, n_peg);
    if (h.strand != '+' && h.strand != '-')
      return fail(KMA_E_INVALID, "connection %llu: strand must be '+' or '-'",
                  (unsigned long long)i);
    if (i && (h.contig < hits[i - 1].contig ||
              (h.contig == hits[i - 1].contig && h.left < hits[i - 1].left)))
      return fail(KMA_E_INVALID, "connections are not in (contig, left) order at %llu",
                  (unsigned long long)i);
  }
  DeviceScope ds(device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d): %s", device,
                                        hipGetErrorString(ds.err));
  const uint64_t n = n_hits;
  DevBufs b;
  kma::PropArgs a{};
  kma_hit* d_hits;
  uint32_t* d_len;
  KMA_HIP(b.alloc(&d_hits, n * sizeof(kma_hit)));
  KMA_HIP(b.alloc(&d_len, n_peg * 4ull));
  for (uint32_t** p : {&a.keys, &a.skeys, &a.idx, &a.sidx, &a.head, &a.list_no, &a.scontig,
                       &a.keep, &a.evidence, &a.out_pos})
    KMA_HIP(b.alloc(p, n * 4));
  KMA_HIP(b.alloc(&a.starts, (n + 1) * 4));
  KMA_HIP(b.alloc(&a.sleft, n * 4));
  KMA_HIP(b.alloc(&a.best, n * 4));
  KMA_HIP(b.alloc(&a.stats, 32));
  KMA_HIP(b.alloc(&a.out, n * sizeof(kma_proposal)));
  a.hits = d_hits;
  a.n = (uint32_t)n;
  a.peg_len = d_len;
  a.n_peg = n_peg;
  a.k = k;
  a.min_strength = min_strength;
  a.max_fuzz = max_fuzz;
  a.min_fuzz = min_fuzz;
  a.cap = n;
  size_t tb = 0;
  KMA_HIP(kma::launch_propose(a, nullptr, &tb, nullptr));
  void* d_temp;
  KMA_HIP(b.alloc(&d_temp, tb ? tb : 1));
  KMA_HIP(hipMemcpy(d_hits, hits, n * sizeof(kma_hit), hipMemcpyHostToDevice));
  KMA_HIP(hipMemcpy(d_len, peg_len, n_peg * 4ull, hipMemcpyHostToDevice));
  KMA_HIP(hipMemset(a.stats, 0, 32));
  KMA_HIP(kma::launch_propose(a, d_temp, &tb, nullptr));
  KMA_HIP(hipMemcpy(stats, a.stats, 32, hipMemcpyDeviceToHost));
  *n_out = stats[3];
  const uint64_t take = std::min<uint64_t>(stats[3], cap);
  if (take) KMA_HIP(hipMemcpy(out, a.out, take * sizeof(kma_proposal), hipMemcpyDeviceToHost));
  if (stats[3] > cap)
    return fail(KMA_E_CAPACITY, "%llu proposals, capacity %llu", (unsigned long long)stats[3],
                (unsigned long long)cap);
  return KMA_OK;
}

}  // extern "C"

namespace {
// Window keys, per-protein sort and distinct sizes of a batch (device buffers in b): the
// ProteinKmers sets of kma_hash_annotate's two sides.
struct KmerSets {
  uint8_t* res = nullptr;
  uint64_t* off = nullptr;
  uint64_t *keys = nullptr, *sorted = nullptr;
  uint32_t *size = nullptr, *owner = nullptr;
  uint8_t* first = nullptr;
  uint64_t total = 0;
};

int kmer_sets(DevBufs& b, const uint8_t* residues, const uint64_t* offsets, uint32_t n, int k,
              uint32_t* d_alpha, KmerSets& ks) {
  const uint64_t base = offsets[0];
  ks.total = offsets[n] - base;
  std::vector<uint64_t> rel(offsets, offsets + n + 1);
  for (auto& o : rel) o -= base;
  const uint64_t nw = std::max<uint64_t>(ks.total, 1);
  KMA_HIP(b.alloc(&ks.res, ks.total + 64));
  KMA_HIP(b.alloc(&ks.off, (n + 1) * 8ull));
  KMA_HIP(b.alloc(&ks.keys, nw * 8));
  KMA_HIP(b.alloc(&ks.sorted, nw * 8));
  KMA_HIP(b.alloc(&ks.size, std::max<uint64_t>(n, 1) * 4));
  KMA_HIP(b.alloc(&ks.owner, nw * 4));
  KMA_HIP(b.alloc(&ks.first, nw));
  KMA_HIP(hipMemcpy(ks.res, residues + base, ks.total, hipMemcpyHostToDevice));
  KMA_HIP(hipMemset(ks.res + ks.total, 0, 64));
  KMA_HIP(hipMemcpy(ks.off, rel.data(), (n + 1) * 8ull, hipMemcpyHostToDevice));
  KMA_HIP(kma::launch_window_keys(ks.res, ks.off, n, k, 0, ks.keys, d_alpha, nullptr));
  size_t tb = 0;
  KMA_HIP(kma::launch_segmented_sort(nullptr, &tb, ks.keys, ks.sorted, ks.total, n, ks.off,
                                     ks.off + 1, 5 * k, nullptr));
  void* d_temp;
  KMA_HIP(b.alloc(&d_temp, tb ? tb : 1));
  KMA_HIP(kma::launch_segmented_sort(d_temp, &tb, ks.keys, ks.sorted, ks.total, n, ks.off,
                                     ks.off + 1, 5 * k, nullptr));
  KMA_HIP(kma::launch_distinct(ks.sorted, ks.off, n, ks.size, nullptr));
  KMA_HIP(kma::launch_owner_first(ks.sorted, ks.off, n, ks.owner, ks.first, nullptr));
  return KMA_OK;
}

int check_batch(const uint8_t* residues, const uint64_t* offsets, uint32_t n, const char* what) {
  if (n && (!residues || !offsets)) return fail(KMA_E_INVALID, "null %s", what);
  for (uint32_t s = 0; s < n; ++s)
    if (offsets[s + 1] < offsets[s]) return fail(KMA_E_INVALID, "%s offsets decrease at %u", what, s);
  if (n && offsets[n] - offsets[0] >= (1ull << 31))
    return fail(KMA_E_INVALID, "more than 2^31 %s residues", what);
  return KMA_OK;
}
}  // namespace

extern "C" {

int kma_hash_annotate(const uint8_t* gres, const uint64_t* goff, uint32_t n_gp,
                      const uint8_t* pres, const uint64_t* poff, uint32_t n_pt, int k,
                      double min_sim, int device, int32_t* out_best, double* out_sim,
                      uint32_t* out_count) {
  if (k < 2 || k > 12) return fail(KMA_E_INVALID, "kmer size %d outside 2..12", k);
  if (!(min_sim >= 0.0 && min_sim < 1.0))
    return fail(KMA_E_INVALID, "Minimum similarity score must be between 0 and 1.");
  if ((n_gp && (!out_best || !out_sim)) || (n_pt && !out_count))
    return fail(KMA_E_INVALID, "null output");
  if (int rc = check_batch(gres, goff, n_gp, "genome protein")) return rc;
  if (int rc = check_batch(pres, poff, n_pt, "prototype")) return rc;
  for (uint32_t i = 0; i < n_gp; ++i) {
    out_best[i] = -1;
    out_sim[i] = 0.0;
  }
  if (n_pt) std::memset(out_count, 0, n_pt * 4ull);
  if (n_gp == 0 || n_pt == 0) return KMA_OK;
  DeviceScope ds(device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d): %s", device,
                                        hipGetErrorString(ds.err));
  DevBufs b;
  uint32_t* d_alpha;
  uint64_t* d_n;  // [0] genome pairs, [1] unique keys, [2] runs
  KMA_HIP(b.alloc(&d_alpha, 4));
  KMA_HIP(b.alloc(&d_n, 32));
  KMA_HIP(hipMemset(d_alpha, 0, 4));
  KMA_HIP(hipMemset(d_n, 0, 32));
  KmerSets g, p;
  if (int rc = kmer_sets(b, gres, goff, n_gp, k, d_alpha, g)) return rc;
  if (int rc = kmer_sets(b, pres, poff, n_pt, k, d_alpha, p)) return rc;
  uint32_t alpha = 0;
  KMA_HIP(hipMemcpy(&alpha, d_alpha, 4, hipMemcpyDeviceToHost));
  if (alpha) return fail(KMA_E_ALPHABET, "a protein window holds a byte outside A-Z and '*'");
  const int kb = 5 * k;
  // genome (key, protein) pairs of distinct keys, sorted by key; unique keys and ranges
  const uint64_t gw = std::max<uint64_t>(g.total, 1);
  uint64_t *gpk, *skey, *ukeys;
  uint32_t *gpp, *sprot, *uidx, *ustart;
  uint8_t* uhead;
  for (uint64_t** q : {&gpk, &skey, &ukeys}) KMA_HIP(b.alloc(q, gw * 8));
  for (uint32_t** q : {&gpp, &sprot, &uidx}) KMA_HIP(b.alloc(q, gw * 4));
  KMA_HIP(b.alloc(&ustart, (gw + 1) * 4));
  KMA_HIP(b.alloc(&uhead, gw));
  size_t need = 0, tb = 0;
  auto grow = [&](size_t t) { need = std::max(need, t); };
  KMA_HIP(kma::prim_select_flagged_u64(nullptr, &tb, g.sorted, g.first, gpk, d_n, g.total, nullptr));
  grow(tb);
  KMA_HIP(kma::prim_select_flagged_u32(nullptr, &tb, g.owner, g.first, gpp, d_n, g.total, nullptr));
  grow(tb);
  KMA_HIP(kma::prim_sort_pairs_u64_u32(nullptr, &tb, gpk, skey, gpp, sprot, g.total, kb, nullptr));
  grow(tb);
  KMA_HIP(kma::prim_excl_sum_u32_u64(nullptr, &tb, nullptr, nullptr, std::max<uint64_t>(p.total, 1), nullptr));
  grow(tb);
  void* temp;
  KMA_HIP(b.alloc(&temp, need ? need : 1));
  tb = need;
  KMA_HIP(kma::prim_select_flagged_u64(temp, &tb, g.sorted, g.first, gpk, d_n, g.total, nullptr));
  tb = need;
  KMA_HIP(kma::prim_select_flagged_u32(temp, &tb, g.owner, g.first, gpp, d_n, g.total, nullptr));
  uint64_t n_pairs = 0;
  KMA_HIP(hipMemcpy(&n_pairs, d_n, 8, hipMemcpyDeviceToHost));
  tb = need;
  KMA_HIP(kma::prim_sort_pairs_u64_u32(temp, &tb, gpk, skey, gpp, sprot, n_pairs, kb, nullptr));
  KMA_HIP(kma::launch_run_heads(skey, n_pairs, uhead, uidx, nullptr));
  tb = need;
  KMA_HIP(kma::prim_select_flagged_u64(temp, &tb, skey, uhead, ukeys, d_n + 1, n_pairs, nullptr));
  tb = need;
  KMA_HIP(kma::prim_select_flagged_u32(temp, &tb, uidx, uhead, ustart, d_n + 1, n_pairs, nullptr));
  KMA_HIP(kma::launch_set_end(ustart, d_n + 1, n_pairs, nullptr));
  // candidates: one (prototype, protein) per shared distinct key
  kma::HashArgs a{};
  a.n_ppos = p.total;
  a.pfirst = p.first;
  a.psorted = p.sorted;
  a.powner = p.owner;
  a.psize = p.size;
  a.ukeys = ukeys;
  a.n_u = d_n + 1;
  a.ustart = ustart;
  a.gprot = sprot;
  a.gsize = g.size;
  a.min_sim = min_sim;
  const uint64_t pw = std::max<uint64_t>(p.total, 1);
  uint64_t* coff;
  KMA_HIP(b.alloc(&a.ccount, pw * 4));
  KMA_HIP(b.alloc(&a.cu, pw * 4));
  KMA_HIP(b.alloc(&coff, pw * 8));
  a.coff = coff;
  KMA_HIP(kma::launch_cand_count(a, nullptr));
  tb = need;
  KMA_HIP(kma::prim_excl_sum_u32_u64(temp, &tb, a.ccount, coff, p.total, nullptr));
  uint64_t last_off = 0;
  uint32_t last_cnt = 0;
  if (p.total) {
    KMA_HIP(hipMemcpy(&last_off, coff + p.total - 1, 8, hipMemcpyDeviceToHost));
    KMA_HIP(hipMemcpy(&last_cnt, a.ccount + p.total - 1, 4, hipMemcpyDeviceToHost));
  }
  const uint64_t n_cand = last_off + last_cnt;
  KMA_HIP(b.alloc(&a.out_count, n_pt * 4ull));
  uint64_t* best_bits;
  uint32_t* best_proto;
  KMA_HIP(b.alloc(&best_bits, n_gp * 8ull));
  KMA_HIP(b.alloc(&best_proto, n_gp * 4ull));
  KMA_HIP(b.alloc(&a.best_bits, n_gp * 8ull));
  KMA_HIP(b.alloc(&a.best_proto, n_gp * 4ull));
  KMA_HIP(hipMemset(a.out_count, 0, n_pt * 4ull));
  for (uint64_t* q : {best_bits, a.best_bits}) KMA_HIP(hipMemset(q, 0, n_gp * 8ull));
  for (uint32_t* q : {best_proto, a.best_proto}) KMA_HIP(hipMemset(q, 0xFF, n_gp * 4ull));
  // Candidates are scored in slices of whole prototypes (file order) whose sort and run-length
  // encoding stay below 2^31 elements (the int counts of the CUB-style APIs this was first written against; rocPRIM's select and sort take size_t, its run-length encode still unsigned); a slice's best per protein
  // replaces the running best only when strictly higher, so earlier prototypes keep ties.
  // KMA_OPT_HASH_SLICE (tests) lowers the slice size.
  uint64_t slice_cap = (1ull << 31) - 1;
  if (const int64_t o = opt(KMA_OPT_HASH_SLICE); o > 0)
    slice_cap = std::min<uint64_t>(slice_cap, (uint64_t)o);
  std::vector<uint64_t> cum(n_pt + 1, 0);
  if (n_cand) {
    uint64_t* d_cum;
    KMA_HIP(b.alloc(&d_cum, (n_pt + 1) * 8ull));
    KMA_HIP(kma::launch_proto_cum(coff, a.ccount, p.off, n_pt, p.total, d_cum, nullptr));
    KMA_HIP(hipMemcpy(cum.data(), d_cum, (n_pt + 1) * 8ull, hipMemcpyDeviceToHost));
  }
  std::vector<uint32_t> cut{0};  // slice boundaries in prototypes
  for (uint32_t q = 0; q < n_pt; ++q) {
    if (cum[q + 1] - cum[q] > (1ull << 31) - 1)
      return fail(KMA_E_CAPACITY, "prototype %u has %llu candidates (limit 2^31 - 1)", q,
                  (unsigned long long)(cum[q + 1] - cum[q]));
    if (q > cut.back() && cum[q + 1] - cum[cut.back()] > slice_cap) cut.push_back(q);
  }
  cut.push_back(n_pt);
  uint64_t max_slice = 0;
  for (size_t i = 0; i + 1 < cut.size(); ++i)
    max_slice = std::max(max_slice, cum[cut[i + 1]] - cum[cut[i]]);
  if (max_slice) {
    uint64_t *cand, *csorted, *runs;
    uint32_t* run_len;
    KMA_HIP(b.alloc(&cand, max_slice * 8));
    KMA_HIP(b.alloc(&csorted, max_slice * 8));
    KMA_HIP(b.alloc(&runs, max_slice * 8));
    KMA_HIP(b.alloc(&run_len, max_slice * 4));
    int pbits = 1;
    while (pbits < 32 && (1ull << pbits) < n_pt) ++pbits;
    size_t t2 = 0, t3 = 0;
    KMA_HIP(kma::prim_sort_keys_u64(nullptr, &t2, cand, csorted, max_slice, 32 + pbits, nullptr));
    KMA_HIP(kma::prim_rle_u64(nullptr, &t3, csorted, runs, run_len, d_n + 2, max_slice, nullptr));
    void* temp2;
    const size_t t23 = std::max(t2, t3);
    KMA_HIP(b.alloc(&temp2, t23 ? t23 : 1));
    std::vector<uint64_t> hoff(n_pt + 1);
    KMA_HIP(hipMemcpy(hoff.data(), p.off, (n_pt + 1) * 8ull, hipMemcpyDeviceToHost));
    a.cand = cand;
    a.runs = runs;
    a.run_len = run_len;
    a.n_runs = d_n + 2;
    for (size_t i = 0; i + 1 < cut.size(); ++i) {
      const uint64_t nc = cum[cut[i + 1]] - cum[cut[i]];
      if (!nc) continue;
      a.pos_lo = hoff[cut[i]] - hoff[0];
      a.pos_hi = hoff[cut[i + 1]] - hoff[0];
      a.cand_base = cum[cut[i]];
      KMA_HIP(kma::launch_cand_emit(a, nullptr));
      t2 = t23;
      KMA_HIP(kma::prim_sort_keys_u64(temp2, &t2, cand, csorted, nc, 32 + pbits, nullptr));
      t3 = t23;
      KMA_HIP(kma::prim_rle_u64(temp2, &t3, csorted, runs, run_len, d_n + 2, nc, nullptr));
      KMA_HIP(kma::launch_score(a, nc, nullptr));
      KMA_HIP(kma::launch_choose(a, nc, nullptr));
      KMA_HIP(kma::launch_merge_best(best_bits, best_proto, a.best_bits, a.best_proto, n_gp,
                                     nullptr));
    }
  }
  std::vector<uint64_t> bits(n_gp);
  std::vector<uint32_t> proto(n_gp);
  KMA_HIP(hipMemcpy(bits.data(), best_bits, n_gp * 8ull, hipMemcpyDeviceToHost));
  KMA_HIP(hipMemcpy(proto.data(), best_proto, n_gp * 4ull, hipMemcpyDeviceToHost));
  KMA_HIP(hipMemcpy(out_count, a.out_count, n_pt * 4ull, hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < n_gp; ++i) {
    if (proto[i] == 0xFFFFFFFFu) continue;
    std::memcpy(&out_sim[i], &bits[i], 8);
    out_best[i] = (int32_t)proto[i];
  }
  return KMA_OK;
}

}  // extern "C"
