// kma_abi.cpp — the C ABI of libkmeranno.so (declared in include/kmeranno.h).
//
// Host-side orchestration only: argument checks, key packing, device allocation and copies,
// and kernel launches (kma_kernels.hip). No compute falls back to the CPU: without a usable
// HIP device every entry point that needs one returns KMA_E_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kmeranno.h"
#include "kma_internal.h"

int kma::minimizer_len(int k, uint64_t n_buckets) {
  static const int forced = [] {
    const char* e = getenv("KMA_MINIMIZER");
    return e ? atoi(e) : 0;
  }();
  const int m6 = k < 6 ? k : 6, m7 = k < 7 ? k : 7;
  if (forced == 6) return m6;
  if (forced == 7) return m7;
  return n_buckets <= (1ull << 22) ? m6 : m7;
}

constexpr uint64_t kHitsPad = 64;
// A protein goes to vote_long_kernel only if its set needs more than K2's LDS gives one
// protein (>= 3/4 kWaveSet - 256, resp. > kVotePool / 2 hits), so it has more than 128 windows.
static_assert(kma::kWaveSet >= 512 && kma::kVotePool >= 256, "pending list bound");
// Two lists of up to n_residues / 128 + 32 records each (a list entry has > 128 windows).
uint64_t pending_cap(uint64_t n_residues) { return 2 * (n_residues / 128 + 32); }

struct kma_table {
  int device = 0;
  int k = 8;
  int mlen = 6;  // minimizer length of the layout (kma::minimizer_len)
  uint64_t n_buckets = 0;
  uint64_t* d_slots = nullptr;
  bool owned = false;
  uint8_t* d_lut = nullptr;
  uint8_t lut[256] = {};
  kma_table_info info = {};
};

struct kma_workspace {
  int device = 0;
  int n_cu = 256;
  uint32_t* d_flag = nullptr;
  uint64_t* d_scratch = nullptr;
  uint32_t* d_hits = nullptr;  // K1 words (fid + 1), then K1 slot ids: u32 per residue each
  kma::PendingRec* d_pending = nullptr;  // K2 -> vote_long list (> 128 windows each)
  uint64_t hits_cap = 0;
  // 6-frame path (kma_workspace_reserve_contigs): staged hits, block counts, scan.
  uint64_t* d_cstage = nullptr;
  uint32_t* d_ccounts = nullptr;
  uint64_t* d_cprefix = nullptr;
  void* d_ctemp = nullptr;
  size_t ctemp_bytes = 0;
  uint64_t contig_cap = 0;  // bases
  // Segmented overlap: K2 of segment i on `side` while K1 of segment i + 1 runs on the call's
  // stream (fork/join through events, graph-capturable).
  hipStream_t side = nullptr;
  std::vector<hipEvent_t> seg_ev;  // fork, per-segment K1 done, join
  // Per-phase timing (kma_workspace_timing): a ring of (start, after K1, end) event triples.
  bool timing = false;
  std::vector<hipEvent_t> events;
  uint32_t n_timed = 0;
};
constexpr uint32_t kTimingRing = 256;
constexpr int kMaxSegments = 8;

// Segments per call (K2 of a segment may run beside K1 of the next); KMA_SEGMENTS overrides.
int segments_for(uint32_t n_seq) {
  static const int forced = [] {
    const char* e = getenv("KMA_SEGMENTS");
    return e ? atoi(e) : 0;
  }();
  // Measured on MI355X (r01): K1 fills every CU, so K2 on the side stream does not overlap it
  // and each extra segment adds a K1 ramp; default 1.
  int s = forced > 0 ? forced : 1;
  return std::max(1, std::min(s, std::min<int>(kMaxSegments, (int)std::max<uint32_t>(1, n_seq))));
}

// Protein path form: the fused probe + vote kernel K12 for batches of at least
// kma::fused_min_proteins proteins, else the two-kernel K1 / K2 pipeline. KMA_FUSED=1 / 0
// forces one form (A/B runs; segmented overlap and the K1/K2 variants need the two-kernel form).
bool fused_form(uint32_t n_seq, int n_cu) {
  const char* e = getenv("KMA_FUSED");  // read per call: tests switch forms in one process
  if (e && (e[0] == '0' || e[0] == '1')) return e[0] == '1';
  return n_seq >= kma::fused_min_proteins(n_cu);
}

namespace {

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

// Device buffers freed on scope exit (host entry points only).
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

void standard_lut(uint8_t lut[256]) {
  std::memset(lut, 0, 256);
  for (int c = 'A'; c <= 'Z'; ++c) lut[c] = (uint8_t)(c - 'A' + 1);
  lut[(uint8_t)'*'] = 27;
}

int check_k(int k) {
  if (k < 1 || k > KMA_MAX_K) return fail(KMA_E_INVALID, "kmer size %d outside 1..%d", k, KMA_MAX_K);
  return KMA_OK;
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
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
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

int make_table_object(int device, int k, uint64_t n_buckets, uint64_t* d_slots, bool owned,
                      const uint8_t lut[256], kma_table** out) {
  kma_table* t = new kma_table();
  t->device = device;
  t->k = k;
  t->mlen = kma::minimizer_len(k, n_buckets);
  t->n_buckets = n_buckets;
  t->d_slots = d_slots;
  t->owned = owned;
  std::memcpy(t->lut, lut, 256);
  hipError_t e = hipMalloc(&t->d_lut, 256);
  if (e == hipSuccess) e = hipMemcpy(t->d_lut, lut, 256, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (t->d_lut) (void)hipFree(t->d_lut);
    delete t;
    return fail(KMA_E_DEVICE, "table LUT upload: %s", hipGetErrorString(e));
  }
  t->info.n_buckets = n_buckets;
  t->info.bytes = n_buckets * 64;
  t->info.k = k;
  t->info.device = device;
  t->info.minimizer_len = t->mlen;
  *out = t;
  return KMA_OK;
}

constexpr uint64_t kMaxBuckets = 1ull << 29;  // slot index and bucket index stay 32-bit

int build_on_device(uint64_t* d_slots, uint64_t n_buckets, int k, uint32_t* d_winner,
                    const uint64_t* d_keys, const uint32_t* d_fids, uint64_t n, uint32_t* d_status,
                    hipStream_t s) {
  if (n_buckets > kMaxBuckets) return fail(KMA_E_INVALID, "more than 2^29 buckets");
  KMA_HIP(hipMemsetAsync(d_slots, 0, n_buckets * 64, s));
  KMA_HIP(hipMemsetAsync(d_winner, 0, n_buckets * kma::kSlotsPerBucket * sizeof(uint32_t), s));
  KMA_HIP(hipMemsetAsync(d_status, 0, 4 * sizeof(uint32_t), s));
  const int m = kma::minimizer_len(k, n_buckets);
  KMA_HIP(kma::launch_build_insert(d_slots, d_winner, (uint32_t)n_buckets, k, m, d_keys, n,
                                   d_status, s));
  KMA_HIP(kma::launch_build_finalize(d_slots, d_winner, d_fids, (uint32_t)n_buckets, k, m,
                                     d_status + 1, s));
  return KMA_OK;
}

// Table from device-resident keys/fids (n rows; fids already checked against KMA_MAX_FID).
int create_from_device_keys(const uint64_t* d_keys, const uint32_t* d_fids, uint64_t n, int k,
                            int device, double lf, const uint8_t lut[256], kma_table** out) {
  const uint64_t nb = kma_table_buckets_for(n, lf);
  if (nb > kMaxBuckets)
    return fail(KMA_E_INVALID, "table too large: %llu buckets", (unsigned long long)nb);
  DevBufs tmp;
  uint32_t *d_winner, *d_status;
  KMA_HIP(tmp.alloc(&d_winner, nb * kma::kSlotsPerBucket * 4));
  KMA_HIP(tmp.alloc(&d_status, 16));
  uint64_t* d_slots = nullptr;
  KMA_HIP(hipMalloc(&d_slots, nb * 64));
  int rc = build_on_device(d_slots, nb, k, d_winner, d_keys, d_fids, n, d_status, nullptr);
  uint32_t st[4] = {};
  if (rc == KMA_OK) {
    hipError_t e = hipMemcpy(st, d_status, 16, hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = fail(KMA_E_DEVICE, "build: %s", hipGetErrorString(e));
    else if (st[0]) rc = fail(KMA_E_TABLE_FULL, "signature table full");
  }
  if (rc == KMA_OK) rc = make_table_object(device, k, nb, d_slots, true, lut, out);
  if (rc != KMA_OK) {
    (void)hipFree(d_slots);
    return rc;
  }
  (*out)->info.n_rows = n;
  (*out)->info.n_entries = st[1];
  (*out)->info.max_probe = st[2];
  int ne = 0;
  for (int c = 0; c < 256; ++c)
    if (lut[c] >= 28) (*out)->info.extra_syms[lut[c] - 28] = (uint8_t)c, ++ne;
  (*out)->info.n_extra_syms = ne;
  return KMA_OK;
}

// Shared by both create forms: keys packed on the host with `lut`.
int create_from_keys(const std::vector<uint64_t>& keys, const uint32_t* fids, uint64_t n, int k,
                     int device, double lf, const uint8_t lut[256], uint64_t n_skipped,
                     kma_table** out) {
  if (lf <= 0) lf = 0.5;
  if (lf > 0.95) return fail(KMA_E_INVALID, "load factor %.3f > 0.95", lf);
  for (uint64_t r = 0; r < n; ++r)
    if (fids[r] > KMA_MAX_FID) return fail(KMA_E_INVALID, "fid %u of row %llu exceeds 2^23-1",
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

}  // namespace

extern "C" {

int kma_abi_version(void) { return KMA_ABI_VERSION; }

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
  if (load_factor <= 0) load_factor = 0.5;
  const double slots = (double)(n_keys ? n_keys : 1) / load_factor;
  uint64_t nb = (uint64_t)((slots + kma::kSlotsPerBucket - 1) / kma::kSlotsPerBucket);
  return nb < 1 ? 1 : nb;
}

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

int kma_table_info_get(const kma_table* table, kma_table_info* out) {
  if (!table || !out) return fail(KMA_E_INVALID, "null argument");
  *out = table->info;
  return KMA_OK;
}

int kma_table_destroy(kma_table* table) {
  if (!table) return KMA_OK;
  DeviceScope ds(table->device);
  if (table->owned && table->d_slots) (void)hipFree(table->d_slots);
  if (table->d_lut) (void)hipFree(table->d_lut);
  delete table;
  return KMA_OK;
}

int kma_table_build_device(void* d_slots, uint64_t n_buckets, int k, uint32_t* d_winner,
                           const uint64_t* d_keys, const uint32_t* d_fids, uint64_t n,
                           uint32_t* d_status, void* stream) {
  if (!d_slots || !d_winner || !d_status || (n && (!d_keys || !d_fids)) || !n_buckets)
    return fail(KMA_E_INVALID, "null argument");
  if (int rc = check_k(k)) return rc;
  return build_on_device(static_cast<uint64_t*>(d_slots), n_buckets, k, d_winner, d_keys, d_fids,
                         n, d_status, static_cast<hipStream_t>(stream));
}

int kma_table_wrap_device(void* d_slots, uint64_t n_buckets, int k, int device, kma_table** out) {
  if (!d_slots || !out || !n_buckets) return fail(KMA_E_INVALID, "null argument");
  if (n_buckets > kMaxBuckets) return fail(KMA_E_INVALID, "more than 2^29 buckets");
  if (int rc = check_k(k)) return rc;
  DeviceScope ds(device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", device);
  uint8_t lut[256];
  standard_lut(lut);
  return make_table_object(device, k, n_buckets, static_cast<uint64_t*>(d_slots), false, lut, out);
}

int kma_table_device_ptr(const kma_table* table, void** d_slots, uint64_t* bytes) {
  if (!table || !d_slots || !bytes) return fail(KMA_E_INVALID, "null argument");
  *d_slots = table->d_slots;
  *bytes = table->n_buckets * 64;
  return KMA_OK;
}

}  // extern "C"

namespace {
void free_contig_scratch(kma_workspace* ws) {
  for (void* p : {(void*)ws->d_cstage, (void*)ws->d_ccounts, (void*)ws->d_cprefix, ws->d_ctemp})
    if (p) (void)hipFree(p);
  ws->d_cstage = nullptr;
  ws->d_ccounts = nullptr;
  ws->d_cprefix = nullptr;
  ws->d_ctemp = nullptr;
  ws->ctemp_bytes = 0;
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

// The 6-frame pass: probe + block compaction and the block-count scan (enqueue_contigs), then
// the canonical-order emit (enqueue_contig_emit; with out = null it only publishes the count).
kma::ContigArgs contig_args(const kma_table* t, kma_workspace* ws, const uint8_t* d_dna,
                            const uint64_t* d_offsets, uint32_t n_contig, uint64_t n_bases,
                            const char* code, uint32_t* d_tally, uint32_t n_fid) {
  kma::ContigArgs a{};
  a.slots = t->d_slots;
  a.n_buckets = (uint32_t)t->n_buckets;
  a.dna = d_dna;
  a.offsets = d_offsets;
  a.n_contig = n_contig;
  a.total_bases = n_bases;
  a.k = t->k;
  a.mlen = t->mlen;
  a.staging = ws->d_cstage;
  a.block_counts = ws->d_ccounts;
  a.prefix = ws->d_cprefix;
  a.tally = d_tally;
  a.n_fid = d_tally ? n_fid : 0;
  codon_codes(code, a.codon_codes);
  return a;
}

int enqueue_contigs(kma_workspace* ws, const kma::ContigArgs& a, hipStream_t s) {
  const uint64_t nb = contig_blocks(a.total_bases);
  KMA_HIP(kma::launch_contigs_probe(a, nb, s));
  size_t tb = ws->ctemp_bytes;
  KMA_HIP(kma::launch_contig_scan(ws->d_ccounts, ws->d_cprefix, nb, ws->d_ctemp, &tb, s));
  return KMA_OK;
}

int enqueue_contig_emit(kma::ContigArgs a, kma_hit* d_hits, uint64_t cap, uint64_t* d_n_hits,
                        hipStream_t s) {
  a.out = d_hits;
  a.cap = d_hits ? cap : 0;
  a.n_hits = d_n_hits;
  KMA_HIP(kma::launch_contigs_emit(a, contig_blocks(a.total_bases), s));
  return KMA_OK;
}
}  // namespace

extern "C" {

int kma_workspace_reserve_contigs(kma_workspace* ws, uint64_t n_bases) {
  if (!ws) return fail(KMA_E_INVALID, "null workspace");
  if (n_bases >= (1ull << 39)) return fail(KMA_E_INVALID, "more than 2^39 bases in one call");
  if (ws->d_cstage && n_bases <= ws->contig_cap) return KMA_OK;
  DeviceScope ds(ws->device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", ws->device);
  free_contig_scratch(ws);
  const uint64_t nb = contig_blocks(n_bases);
  size_t tb = 0;
  KMA_HIP(kma::launch_contig_scan(nullptr, nullptr, nb, nullptr, &tb, nullptr));
  KMA_HIP(hipMalloc(&ws->d_cstage, nb * 2 * kma::kContigTile * 8));
  KMA_HIP(hipMalloc(&ws->d_ccounts, nb * 4));
  KMA_HIP(hipMalloc(&ws->d_cprefix, nb * 8));
  KMA_HIP(hipMalloc(&ws->d_ctemp, tb ? tb : 1));
  ws->ctemp_bytes = tb;
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
  hipError_t e = hipMalloc(&w->d_flag, 16);
  if (e == hipSuccess) e = hipMemset(w->d_flag, 0, 16);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&w->side, hipStreamNonBlocking);
  w->seg_ev.assign(kMaxSegments + 2, nullptr);
  for (auto& ev : w->seg_ev)
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e == hipSuccess)
    e = hipMalloc(&w->d_scratch, (size_t)kma::kFallbackBlocks * kma::kFallbackCap * 8);
  if (e == hipSuccess) e = hipMalloc(&w->d_hits, 2 * kHitsPad * 4);  // reserve() grows it
  if (e == hipSuccess) e = hipMalloc(&w->d_pending, pending_cap(0) * sizeof(kma::PendingRec));
  if (e != hipSuccess) {
    if (w->d_flag) (void)hipFree(w->d_flag);
    delete w;
    return fail(KMA_E_NOMEM, "workspace: %s", hipGetErrorString(e));
  }
  *out = w;
  return KMA_OK;
}

int kma_workspace_reserve(kma_workspace* ws, uint64_t n_residues) {
  if (!ws) return fail(KMA_E_INVALID, "null workspace");
  if (ws->d_hits && n_residues <= ws->hits_cap) return KMA_OK;
  DeviceScope ds(ws->device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", ws->device);
  if (ws->d_hits) (void)hipFree(ws->d_hits);
  ws->d_hits = nullptr;
  ws->hits_cap = 0;
  if (ws->d_pending) (void)hipFree(ws->d_pending);
  ws->d_pending = nullptr;
  // Padded by kHitsPad words (never empty): K2 may read word 0 for a chunk past the end.
  // hits then slot ids, each n_residues + kHitsPad words
  KMA_HIP(hipMalloc(&ws->d_hits, 2 * (n_residues + kHitsPad) * 4));
  KMA_HIP(hipMalloc(&ws->d_pending, pending_cap(n_residues) * sizeof(kma::PendingRec)));
  ws->hits_cap = n_residues;
  return KMA_OK;
}

int kma_workspace_timing(kma_workspace* ws, int enable) {
  if (!ws) return fail(KMA_E_INVALID, "null workspace");
  DeviceScope ds(ws->device);
  if (enable && ws->events.empty()) {
    ws->events.resize(3 * kTimingRing);
    for (auto& e : ws->events) KMA_HIP(hipEventCreate(&e));
  }
  ws->timing = enable != 0;
  ws->n_timed = 0;
  return KMA_OK;
}

int kma_workspace_timing_read(kma_workspace* ws, uint32_t* n_calls, double* probe_ms,
                              double* vote_ms) {
  if (!ws || !n_calls || !probe_ms || !vote_ms) return fail(KMA_E_INVALID, "null argument");
  DeviceScope ds(ws->device);
  const uint32_t n = std::min(ws->n_timed, kTimingRing);
  double p = 0, v = 0;
  for (uint32_t i = 0; i < n; ++i) {
    hipEvent_t* e = &ws->events[3 * i];
    KMA_HIP(hipEventSynchronize(e[2]));
    float a = 0, b = 0;
    KMA_HIP(hipEventElapsedTime(&a, e[0], e[1]));
    KMA_HIP(hipEventElapsedTime(&b, e[1], e[2]));
    p += a;
    v += b;
  }
  *n_calls = n;
  *probe_ms = p;
  *vote_ms = v;
  ws->n_timed = 0;
  return KMA_OK;
}

int kma_protein_form(const kma_workspace* ws, uint32_t n_seq) {
  if (!ws) return fail(KMA_E_INVALID, "null workspace");
  DeviceScope ds(ws->device);
  return fused_form(n_seq, ws->n_cu) ? 1 : 0;
}

int kma_workspace_destroy(kma_workspace* ws) {
  if (!ws) return KMA_OK;
  DeviceScope ds(ws->device);
  for (auto& e : ws->events) (void)hipEventDestroy(e);
  for (auto& e : ws->seg_ev)
    if (e) (void)hipEventDestroy(e);
  if (ws->side) (void)hipStreamDestroy(ws->side);
  (void)hipFree(ws->d_flag);
  (void)hipFree(ws->d_scratch);
  if (ws->d_hits) (void)hipFree(ws->d_hits);
  if (ws->d_pending) (void)hipFree(ws->d_pending);
  free_contig_scratch(ws);
  delete ws;
  return KMA_OK;
}

int kma_annotate_proteins_device(const kma_table* t, kma_workspace* ws, const uint8_t* d_residues,
                                 const uint64_t* d_offsets, uint32_t n_seq, uint64_t n_residues,
                                 int min_hits, uint32_t flags, int32_t* d_fid, int32_t* d_count,
                                 uint8_t* d_status, uint32_t* d_tally, uint32_t n_fid,
                                 void* stream) {
  if (!t || !ws) return fail(KMA_E_INVALID, "null table or workspace");
  if (ws->device != t->device) return fail(KMA_E_INVALID, "workspace on another device");
  if (min_hits < 1) return fail(KMA_E_INVALID, "Min-hits must be positive.");
  if (flags & ~(KMA_F_END_EXCLUSIVE | KMA_F_MULTISET)) return fail(KMA_E_INVALID, "bad flags");
  if (n_seq == 0) return KMA_OK;
  if (!d_residues || !d_offsets || !d_fid || !d_count || !d_status)
    return fail(KMA_E_INVALID, "null device buffer");
  if ((uintptr_t)d_residues & 7) return fail(KMA_E_INVALID, "residues must be 8-byte aligned");
  if (n_residues > ws->hits_cap)
    return fail(KMA_E_CAPACITY, "workspace reserved for %llu residues, call needs %llu",
                (unsigned long long)ws->hits_cap, (unsigned long long)n_residues);
  hipStream_t s = static_cast<hipStream_t>(stream);
  DeviceScope ds(t->device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", t->device);
  kma::ProteinArgs a{};
  a.slots = t->d_slots;
  a.n_buckets = (uint32_t)t->n_buckets;
  a.lut = t->d_lut;
  a.residues = d_residues;
  a.offsets = d_offsets;
  a.n_seq = n_seq;
  a.n_residues = n_residues;
  a.k = t->k;
  a.mlen = t->mlen;
  a.min_hits = min_hits;
  a.flags = flags;
  a.out_fid = d_fid;
  a.out_count = d_count;
  a.out_status = d_status;
  a.tally = d_tally;
  a.n_fid = d_tally ? n_fid : 0;
  a.hits = ws->d_hits;
  a.sids = ws->d_hits + ws->hits_cap + kHitsPad;
  a.overflow_flag = ws->d_flag;
  a.pending = ws->d_pending;
  a.pending_half = (uint32_t)(pending_cap(ws->hits_cap) / 2);
  a.scratch = ws->d_scratch;
  hipEvent_t* ev = nullptr;
  if (ws->timing) {
    ev = &ws->events[3 * (ws->n_timed++ % kTimingRing)];
    KMA_HIP(hipEventRecord(ev[0], s));
  }
  if (fused_form(n_seq, ws->n_cu)) {
    // K12 (probe + vote in one kernel), then vote_long for the pending proteins.
    a.seq_lo = 0;
    a.seq_hi = n_seq;
    a.reset_flag = 0;
    KMA_HIP(hipMemsetAsync(ws->d_flag, 0, 16, s));  // pending-list lengths (K12 appends);
    // the whole 16-B flag block: a byte count 8 over a multiple of 16 costs ~2 us per call
    if (ev) KMA_HIP(hipEventRecord(ev[0], s));     // the probe phase is K12 alone
    KMA_HIP(kma::launch_fused(a, ws->n_cu, s));
    if (ev) KMA_HIP(hipEventRecord(ev[1], s));
    KMA_HIP(kma::launch_long(a, ws->n_cu, s));
    if (ev) KMA_HIP(hipEventRecord(ev[2], s));
    return KMA_OK;
  }
  if (ev) {
    // Timing mode: the phases back to back on the call's stream, so their events bracket them.
    a.seq_lo = 0;
    a.seq_hi = n_seq;
    a.reset_flag = 1;
    KMA_HIP(kma::launch_probe(a, ws->n_cu, s));
    KMA_HIP(hipEventRecord(ev[1], s));
    KMA_HIP(kma::launch_vote(a, ws->n_cu, s));
    KMA_HIP(kma::launch_long(a, ws->n_cu, s));
    KMA_HIP(hipEventRecord(ev[2], s));
    return KMA_OK;
  }
  const int S = segments_for(n_seq);
  if (S > 1) {
    KMA_HIP(hipEventRecord(ws->seg_ev[0], s));  // fork: the side stream sees prior work
    KMA_HIP(hipStreamWaitEvent(ws->side, ws->seg_ev[0], 0));
  }
  for (int i = 0; i < S; ++i) {
    a.seq_lo = (uint32_t)((uint64_t)n_seq * i / S);
    a.seq_hi = (uint32_t)((uint64_t)n_seq * (i + 1) / S);
    a.reset_flag = i == 0;
    KMA_HIP(kma::launch_probe(a, ws->n_cu, s));
    if (S > 1) {
      KMA_HIP(hipEventRecord(ws->seg_ev[1 + i], s));
      KMA_HIP(hipStreamWaitEvent(ws->side, ws->seg_ev[1 + i], 0));
      KMA_HIP(kma::launch_vote(a, ws->n_cu, ws->side));
    } else {
      KMA_HIP(kma::launch_vote(a, ws->n_cu, s));
#ifdef KMA_VOTE_TRACE  // experiment builds only: per-block phase clocks of K2 -> file
      if (const char* f = getenv("KMA_TRACE_FILE")) {
        const uint64_t nb = (n_seq + kma::kVoteProteins - 1) / kma::kVoteProteins;
        std::vector<uint64_t> tr(nb * 8);
        KMA_HIP(hipStreamSynchronize(s));
        KMA_HIP(hipMemcpy(tr.data(), ws->d_scratch, tr.size() * 8, hipMemcpyDeviceToHost));
        if (FILE* o = fopen(f, "wb")) {
          fwrite(tr.data(), 8, tr.size(), o);
          fclose(o);
        }
      }
#endif
    }
  }
  if (S > 1) {
    KMA_HIP(hipEventRecord(ws->seg_ev[kMaxSegments + 1], ws->side));  // join
    KMA_HIP(hipStreamWaitEvent(s, ws->seg_ev[kMaxSegments + 1], 0));
  }
  a.seq_lo = 0;
  a.seq_hi = n_seq;
  KMA_HIP(kma::launch_long(a, ws->n_cu, s));
  return KMA_OK;
}

int kma_annotate_proteins(const kma_table* t, const uint8_t* residues, const uint64_t* offsets,
                          uint32_t n_seq, int min_hits, uint32_t flags, int32_t* out_fid,
                          int32_t* out_count, uint8_t* out_status, uint32_t* out_tally,
                          uint32_t n_fid) {
  if (!t) return fail(KMA_E_INVALID, "null table");
  if (min_hits < 1) return fail(KMA_E_INVALID, "Min-hits must be positive.");
  if (n_seq == 0) return KMA_OK;
  if (!residues || !offsets || !out_fid || !out_count || !out_status)
    return fail(KMA_E_INVALID, "null argument");
  for (uint32_t s = 0; s < n_seq; ++s)
    if (offsets[s + 1] < offsets[s]) return fail(KMA_E_INVALID, "offsets decrease at %u", s);
  DeviceScope ds(t->device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", t->device);
  const uint64_t base = offsets[0], nres = offsets[n_seq] - base;
  std::vector<uint64_t> rel(offsets, offsets + n_seq + 1);
  for (auto& o : rel) o -= base;
  DevBufs b;
  uint8_t *d_res, *d_st;
  uint64_t* d_off;
  int32_t *d_fid, *d_cnt;
  uint32_t* d_tally = nullptr;
  KMA_HIP(b.alloc(&d_res, nres + 32));
  KMA_HIP(b.alloc(&d_off, (n_seq + 1) * 8ull));
  KMA_HIP(b.alloc(&d_fid, n_seq * 4ull));
  KMA_HIP(b.alloc(&d_cnt, n_seq * 4ull));
  KMA_HIP(b.alloc(&d_st, n_seq));
  KMA_HIP(hipMemcpy(d_res, residues + base, nres, hipMemcpyHostToDevice));
  KMA_HIP(hipMemset(d_res + nres, 0, 32));
  KMA_HIP(hipMemcpy(d_off, rel.data(), (n_seq + 1) * 8ull, hipMemcpyHostToDevice));
  if (out_tally && n_fid) {
    KMA_HIP(b.alloc(&d_tally, n_fid * 4ull));
    KMA_HIP(hipMemcpy(d_tally, out_tally, n_fid * 4ull, hipMemcpyHostToDevice));
  }
  kma_workspace* ws = nullptr;
  if (int rc = kma_workspace_create(t->device, &ws)) return rc;
  int rc = kma_workspace_reserve(ws, nres);
  if (rc == KMA_OK)
    rc = kma_annotate_proteins_device(t, ws, d_res, d_off, n_seq, nres, min_hits, flags, d_fid,
                                      d_cnt, d_st, d_tally, d_tally ? n_fid : 0, nullptr);
  hipError_t e = rc == KMA_OK ? hipDeviceSynchronize() : hipSuccess;
  kma_workspace_destroy(ws);
  if (rc != KMA_OK) return rc;
  if (e != hipSuccess) return fail(KMA_E_DEVICE, "annotate: %s", hipGetErrorString(e));
  KMA_HIP(hipMemcpy(out_fid, d_fid, n_seq * 4ull, hipMemcpyDeviceToHost));
  KMA_HIP(hipMemcpy(out_count, d_cnt, n_seq * 4ull, hipMemcpyDeviceToHost));
  KMA_HIP(hipMemcpy(out_status, d_st, n_seq, hipMemcpyDeviceToHost));
  if (d_tally) KMA_HIP(hipMemcpy(out_tally, d_tally, n_fid * 4ull, hipMemcpyDeviceToHost));
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
  if (ws->device != t->device) return fail(KMA_E_INVALID, "workspace on another device");
  const char* code = ncbi_code(genetic_code);
  if (!code) return fail(KMA_E_INVALID, "unsupported genetic code %d", genetic_code);
  if (!d_n_hits) return fail(KMA_E_INVALID, "null n_hits");
  hipStream_t s = static_cast<hipStream_t>(stream);
  DeviceScope ds(t->device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", t->device);
  if (n_contig == 0 || n_bases == 0) {
    KMA_HIP(hipMemsetAsync(d_n_hits, 0, 8, s));
    return KMA_OK;
  }
  if (!d_dna || !d_offsets) return fail(KMA_E_INVALID, "null device buffer");
  if (n_bases > ws->contig_cap)
    return fail(KMA_E_CAPACITY, "workspace reserved for %llu bases, call needs %llu",
                (unsigned long long)ws->contig_cap, (unsigned long long)n_bases);
  const kma::ContigArgs a =
      contig_args(t, ws, d_dna, d_offsets, n_contig, n_bases, code, d_tally, n_fid);
  hipEvent_t* ev = nullptr;  // timing mode: (start, after the probe kernel, end)
  if (ws->timing) {
    ev = &ws->events[3 * (ws->n_timed++ % kTimingRing)];
    KMA_HIP(hipEventRecord(ev[0], s));
  }
  const uint64_t nb = contig_blocks(n_bases);
  KMA_HIP(kma::launch_contigs_probe(a, nb, s));
  if (ev) KMA_HIP(hipEventRecord(ev[1], s));
  size_t tb = ws->ctemp_bytes;
  KMA_HIP(kma::launch_contig_scan(ws->d_ccounts, ws->d_cprefix, nb, ws->d_ctemp, &tb, s));
  const int rc = enqueue_contig_emit(a, d_hits, cap, d_n_hits, s);
  if (rc == KMA_OK && ev) KMA_HIP(hipEventRecord(ev[2], s));
  return rc;
}

int kma_annotate_contigs(const kma_table* t, const uint8_t* dna, const uint64_t* offsets,
                         uint32_t n_contig, int genetic_code, kma_hit* out_hits, uint64_t cap,
                         uint64_t* n_hits, uint32_t* out_tally, uint32_t n_fid) {
  if (!t || !n_hits) return fail(KMA_E_INVALID, "null argument");
  const char* code = ncbi_code(genetic_code);
  if (!code) return fail(KMA_E_INVALID, "unsupported genetic code %d", genetic_code);
  *n_hits = 0;
  if (n_contig == 0) return KMA_OK;
  if (!dna || !offsets) return fail(KMA_E_INVALID, "null argument");
  for (uint32_t c = 0; c < n_contig; ++c)
    if (offsets[c + 1] < offsets[c]) return fail(KMA_E_INVALID, "offsets decrease at %u", c);
  const uint64_t base = offsets[0], total = offsets[n_contig] - base;
  if (total >= (1ull << 39)) return fail(KMA_E_INVALID, "more than 2^39 bases in one call");
  if (total == 0) return KMA_OK;
  std::vector<uint64_t> rel(offsets, offsets + n_contig + 1);
  for (auto& o : rel) o -= base;
  DeviceScope ds(t->device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", t->device);
  kma_workspace* ws = nullptr;
  int rc = kma_workspace_create(t->device, &ws);
  if (rc != KMA_OK) return rc;
  std::unique_ptr<kma_workspace, int (*)(kma_workspace*)> ws_guard(ws, kma_workspace_destroy);
  rc = kma_workspace_reserve_contigs(ws, total);
  if (rc != KMA_OK) return rc;
  DevBufs b;
  uint8_t* d_dna;
  uint64_t *d_off, *d_n;
  uint32_t* d_tally = nullptr;
  kma_hit* d_out = nullptr;
  KMA_HIP(b.alloc(&d_dna, total + 64));
  KMA_HIP(b.alloc(&d_off, (n_contig + 1) * 8ull));
  KMA_HIP(b.alloc(&d_n, 8));
  KMA_HIP(hipMemcpy(d_dna, dna + base, total, hipMemcpyHostToDevice));
  KMA_HIP(hipMemset(d_dna + total, 0, 64));
  KMA_HIP(hipMemcpy(d_off, rel.data(), (n_contig + 1) * 8ull, hipMemcpyHostToDevice));
  const uint64_t tb = out_tally && n_fid ? (uint64_t)n_contig * n_fid * 4 : 0;
  if (tb) {
    KMA_HIP(b.alloc(&d_tally, tb));
    KMA_HIP(hipMemcpy(d_tally, out_tally, tb, hipMemcpyHostToDevice));
  }
  const kma::ContigArgs a =
      contig_args(t, ws, d_dna, d_off, n_contig, total, code, d_tally, n_fid);
  rc = enqueue_contigs(ws, a, nullptr);
  if (rc == KMA_OK) rc = enqueue_contig_emit(a, nullptr, 0, d_n, nullptr);  // count only
  if (rc != KMA_OK) return rc;
  uint64_t nh = 0;
  KMA_HIP(hipMemcpy(&nh, d_n, 8, hipMemcpyDeviceToHost));
  *n_hits = nh;
  // On KMA_E_CAPACITY nothing is written (the tally neither), so the caller can retry.
  if (nh > cap || (nh && !out_hits))
    return fail(KMA_E_CAPACITY, "%llu hits, capacity %llu", (unsigned long long)nh,
                (unsigned long long)(out_hits ? cap : 0));
  if (tb) KMA_HIP(hipMemcpy(out_tally, d_tally, tb, hipMemcpyDeviceToHost));
  if (nh == 0) return KMA_OK;
  KMA_HIP(b.alloc(&d_out, nh * sizeof(kma_hit)));
  rc = enqueue_contig_emit(a, d_out, nh, d_n, nullptr);
  if (rc != KMA_OK) return rc;
  KMA_HIP(hipMemcpy(out_hits, d_out, nh * sizeof(kma_hit), hipMemcpyDeviceToHost));
  return KMA_OK;
}

int kma_peg_table_create(const uint8_t* residues, const uint64_t* offsets, uint32_t n_peg, int k,
                         int device, double load_factor, kma_table** out,
                         uint64_t* n_windows) {
  if (!out) return fail(KMA_E_INVALID, "null argument");
  *out = nullptr;
  if (int rc = check_k(k)) return rc;
  if (load_factor <= 0) load_factor = 0.5;
  if (load_factor > 0.95) return fail(KMA_E_INVALID, "load factor %.3f > 0.95", load_factor);
  if (n_peg > KMA_MAX_FID + 1u) return fail(KMA_E_INVALID, "more than 2^23 pegs");
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

int kma_connect_pegs(const kma_table* t, const uint8_t* dna, const uint64_t* offsets,
                     uint32_t n_contig, int genetic_code, int strict, kma_hit* out_hits,
                     uint64_t cap, uint64_t* n_hits) {
  if (!strict)
    return kma_annotate_contigs(t, dna, offsets, n_contig, genetic_code, out_hits, cap, n_hits,
                                nullptr, 0);
  if (!t || !n_hits) return fail(KMA_E_INVALID, "null argument");
  const char* code = ncbi_code(genetic_code);
  if (!code) return fail(KMA_E_INVALID, "unsupported genetic code %d", genetic_code);
  *n_hits = 0;
  if (n_contig == 0) return KMA_OK;
  if (!dna || !offsets) return fail(KMA_E_INVALID, "null argument");
  for (uint32_t c = 0; c < n_contig; ++c)
    if (offsets[c + 1] < offsets[c]) return fail(KMA_E_INVALID, "offsets decrease at %u", c);
  const uint64_t base = offsets[0], total = offsets[n_contig] - base;
  if (total >= (1ull << 39)) return fail(KMA_E_INVALID, "more than 2^39 bases in one call");
  if (total == 0) return KMA_OK;
  std::vector<uint64_t> rel(offsets, offsets + n_contig + 1);
  for (auto& o : rel) o -= base;
  DeviceScope ds(t->device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d)", t->device);
  kma_workspace* ws = nullptr;
  int rc = kma_workspace_create(t->device, &ws);
  if (rc != KMA_OK) return rc;
  std::unique_ptr<kma_workspace, int (*)(kma_workspace*)> ws_guard(ws, kma_workspace_destroy);
  rc = kma_workspace_reserve_contigs(ws, total);
  if (rc != KMA_OK) return rc;
  DevBufs b;
  uint8_t* d_dna;
  uint64_t *d_off, *d_n;
  uint32_t* d_count;
  kma_hit* d_out = nullptr;
  const uint64_t n_slots = t->n_buckets * kma::kSlotsPerBucket;
  KMA_HIP(b.alloc(&d_dna, total + 64));
  KMA_HIP(b.alloc(&d_off, (n_contig + 1) * 8ull));
  KMA_HIP(b.alloc(&d_n, 8));
  KMA_HIP(b.alloc(&d_count, n_slots * 4));
  KMA_HIP(hipMemcpy(d_dna, dna + base, total, hipMemcpyHostToDevice));
  KMA_HIP(hipMemset(d_dna + total, 0, 64));
  KMA_HIP(hipMemcpy(d_off, rel.data(), (n_contig + 1) * 8ull, hipMemcpyHostToDevice));
  KMA_HIP(hipMemset(d_count, 0, n_slots * 4));
  kma::ContigArgs a = contig_args(t, ws, d_dna, d_off, n_contig, total, code, nullptr, 0);
  a.slot_count = d_count;
  a.strict_pass = 1;  // count every table key's locations
  KMA_HIP(kma::launch_contigs_probe(a, contig_blocks(total), nullptr));
  a.strict_pass = 2;  // keep keys with exactly one location
  rc = enqueue_contigs(ws, a, nullptr);
  if (rc == KMA_OK) rc = enqueue_contig_emit(a, nullptr, 0, d_n, nullptr);
  if (rc != KMA_OK) return rc;
  uint64_t nh = 0;
  KMA_HIP(hipMemcpy(&nh, d_n, 8, hipMemcpyDeviceToHost));
  *n_hits = nh;
  if (nh > cap || (nh && !out_hits))
    return fail(KMA_E_CAPACITY, "%llu hits, capacity %llu", (unsigned long long)nh,
                (unsigned long long)(out_hits ? cap : 0));
  if (nh == 0) return KMA_OK;
  KMA_HIP(b.alloc(&d_out, nh * sizeof(kma_hit)));
  rc = enqueue_contig_emit(a, d_out, nh, d_n, nullptr);
  if (rc != KMA_OK) return rc;
  KMA_HIP(hipMemcpy(out_hits, d_out, nh * sizeof(kma_hit), hipMemcpyDeviceToHost));
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
  uint8_t lut[256];
  standard_lut(lut);
  std::vector<uint64_t> rel(offsets, offsets + n_seq + 1);
  for (auto& o : rel) o -= base;
  DeviceScope ds(device);
  if (ds.err != hipSuccess) return fail(KMA_E_DEVICE, "hipSetDevice(%d): %s", device,
                                        hipGetErrorString(ds.err));
  DevBufs b;
  uint8_t *d_res, *d_lut, *d_flags;
  uint64_t *d_off, *d_a, *d_b, *d_n;
  int32_t* d_roles;
  uint32_t* d_alpha;
  KMA_HIP(b.alloc(&d_res, total + 64));
  KMA_HIP(b.alloc(&d_off, (n_seq + 1) * 8ull));
  KMA_HIP(b.alloc(&d_roles, n_seq * 4ull));
  KMA_HIP(b.alloc(&d_lut, 256));
  KMA_HIP(b.alloc(&d_a, total * 8));
  KMA_HIP(b.alloc(&d_b, total * 8));
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
                                    (flags & KMA_F_END_EXCLUSIVE) ? 1 : 0, d_lut, d_a, d_alpha,
                                    nullptr));
  size_t t1 = 0, t2 = 0, t3 = 0;
  const int bits = 24 + 5 * k;
  KMA_HIP(kma::launch_sort_keys(nullptr, &t1, d_a, d_b, total, bits, nullptr));
  KMA_HIP(kma::launch_unique(nullptr, &t2, d_b, d_a, d_n, total, nullptr));
  KMA_HIP(kma::launch_select_flagged_keys(nullptr, &t3, d_a, d_flags, d_b, d_n + 1, total,
                                          nullptr));
  size_t tb = std::max(t1, std::max(t2, t3));
  void* d_temp;
  KMA_HIP(b.alloc(&d_temp, tb));
  size_t t = tb;
  KMA_HIP(kma::launch_sort_keys(d_temp, &t, d_a, d_b, total, bits, nullptr));  // a -> b
  t = tb;
  KMA_HIP(kma::launch_unique(d_temp, &t, d_b, d_a, d_n, total, nullptr));  // b -> a
  uint64_t n_u = 0;
  uint32_t alpha = 0;
  KMA_HIP(hipMemcpy(&n_u, d_n, 8, hipMemcpyDeviceToHost));
  KMA_HIP(hipMemcpy(&alpha, d_alpha, 4, hipMemcpyDeviceToHost));
  if (alpha)
    return fail(KMA_E_ALPHABET, "a protein window holds a byte outside A-Z and '*'");
  uint64_t n_sel = 0;
  if (n_u) {
    KMA_HIP(kma::launch_signature_flags(d_a, d_n, n_u, d_flags, nullptr));
    t = tb;
    KMA_HIP(kma::launch_select_flagged_keys(d_temp, &t, d_a, d_flags, d_b, d_n + 1, n_u,
                                            nullptr));  // a -> b
    KMA_HIP(hipMemcpy(&n_sel, d_n + 1, 8, hipMemcpyDeviceToHost));
  }
  *n_out = n_sel;
  if (n_sel > cap || (n_sel && (!out_keys || !out_roles)))
    return fail(KMA_E_CAPACITY, "%llu signature kmers, capacity %llu",
                (unsigned long long)n_sel, (unsigned long long)cap);
  if (n_sel == 0) return KMA_OK;
  std::vector<uint64_t> rows(n_sel);
  KMA_HIP(hipMemcpy(rows.data(), d_b, n_sel * 8, hipMemcpyDeviceToHost));
  for (uint64_t i = 0; i < n_sel; ++i) {
    out_keys[i] = rows[i] >> 24;
    out_roles[i] = (uint32_t)(rows[i] & kma::kBuildNeg);
  }
  return KMA_OK;
}

}  // extern "C"
