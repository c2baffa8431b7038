/*
 * kmeranno.h — C ABI of the MI355X-native signature-kmer annotation library (libkmeranno.so).
 *
 * This is the drop-in boundary for the hot path of SEEDtk/kmers.anno (paths relative to the
 * reference's src/main/java/org/theseed/):
 *
 *   - the signature-table load of `apply`
 *       proteins/kmers/anno/ApplyKmerProcessor.java:100-110   -> kma_table_create*
 *                                                                 (kma_table_create_from_tsv
 *                                                                 reads kmerdb.tbl itself)
 *   - the per-protein extraction + lookup + vote loop of `apply`
 *       proteins/kmers/anno/ApplyKmerProcessor.java:122-148   -> kma_annotate_proteins*
 *       (ProteinKmers(...) at :123 is the external org.theseed.sequence extractor)
 *   - the per-genome role tallies of the APPLY report
 *       reports/DefaultApplyKmerReporter.java:43-55           -> `tally` outputs
 *   - the 6-frame contig kmer extractor
 *       proteins/kmers/KmerReference.java:157-203, KmerPosition.java:50-93
 *                                                              -> kma_annotate_contigs*
 *   - ProteinKmers.distance of the gene-copy command
 *       genome/compare/GeneCopyProcessor.java:129-162          -> kma_protein_distances,
 *                                                                 kma_protein_best_match
 *
 * A Java host would bind these through one JNI class; the C++ CLI under
 * kmers.anno_amd/host and the Python ctypes module under kmers.anno_amd/python bind them
 * directly. No HIP or torch types appear here: streams are passed as `void*` (a hipStream_t,
 * NULL = the legacy default stream) and device buffers as plain pointers.
 *
 * Conventions
 *   - Every function returns an int status: KMA_OK (0) or a negative KMA_E_* code. The message
 *     of the last failure on the calling thread is available from kma_last_error().
 *   - "Host" entry points take host buffers owned by the caller and are synchronous.
 *     "_device" entry points take device buffers on the table's device and are asynchronous
 *     on the given stream; they never allocate, free or synchronise (graph-capturable).
 *   - A table is immutable after creation (replicas aside); concurrent annotate calls on one
 *     table are allowed. Host entry points take a per-device context (stream, workspace,
 *     pinned staging) from the table's pool for the call and wait on that stream only;
 *     _device calls must each use their own kma_workspace.
 *   - A table may hold replicas on several devices (kma_table_create_replicated /
 *     kma_table_replicate): host entry points then cut a batch into residue- (base-) balanced
 *     contiguous shards, one host thread per replica, and sum the tallies; _device calls use
 *     the replica on their workspace's device.
 */
#ifndef KMERANNO_H
#define KMERANNO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KMA_ABI_VERSION 7

/* ---- status codes ------------------------------------------------------------------------ */
#define KMA_OK 0
#define KMA_E_INVALID (-1)     /* bad argument (usage error; IllegalArgumentException in Java) */
#define KMA_E_DEVICE (-2)      /* HIP runtime failure / no device                             */
#define KMA_E_NOMEM (-3)       /* device or host allocation failed                            */
#define KMA_E_CAPACITY (-4)    /* an output buffer is too small; *needed count is reported    */
#define KMA_E_ALPHABET (-5)    /* the table needs more than 4 non-[A-Z*] symbols               */
#define KMA_E_TABLE_FULL (-6)  /* probe chain exhausted during build (load factor too high)    */
#define KMA_E_IO (-7)          /* ABI 7: an input file cannot be opened or read (IOException)   */

/* ---- per-protein call status (out_status) -------------------------------------------------
 * Mirrors the three outcomes of ApplyKmerProcessor.java:129-147 plus the reporting threshold:
 *   NONE       no kmer of the protein is in the table            (roleId == null)
 *   CALLED     all hits agree and count >= min_hits               (recordFeature is called)
 *   AMBIGUOUS  two different roles hit                            (badPeg == true)
 *   BELOW_MIN  all hits agree but count < min_hits
 * out_fid is the role's function id for CALLED / BELOW_MIN and -1 otherwise; out_count is the
 * number of distinct table kmers hit for CALLED / BELOW_MIN and 0 otherwise.               */
#define KMA_STATUS_NONE 0
#define KMA_STATUS_CALLED 1
#define KMA_STATUS_AMBIGUOUS 2
#define KMA_STATUS_BELOW_MIN 3
/* (ABI 1 had KMA_STATUS_TOO_LONG = 4 for proteins beyond 2^16 windows; every protein length
 * is voted exactly since ABI 2.)                                                              */

/* ---- extraction flags (kma_annotate_proteins*) ---------------------------------------------
 * Default (0) is the restatement of org.theseed.sequence.ProteinKmers used by `apply`: the SET
 * of distinct length-K substrings at window starts i = 0 .. L-K inclusive.
 *   KMA_F_END_EXCLUSIVE : windows i = 0 .. L-K-1 (the in-repo convention of
 *                         KmerReference.java:134-136, which skips the last kmer)
 *   KMA_F_MULTISET      : count every window hit (no within-protein dedupe)                  */
#define KMA_F_END_EXCLUSIVE 0x1u
#define KMA_F_MULTISET 0x2u

/* ---- key packing ---------------------------------------------------------------------------
 * A kmer of K <= 12 residues packs into 5*K bits, first residue most significant:
 *   key = sum_j code(s[j]) << 5*(K-1-j),  code('A'..'Z') = 1..26, code('*') = 27,
 *   codes 28..31 are assigned (in byte order) to at most four other bytes that occur in the
 *   table's kmers; 0 never occurs, so key 0 is the empty-slot sentinel. Packing is injective,
 *   so key equality is exactly the String.equals of the reference's HashMap lookup.
 * Tables of K <= 8 ("narrow") keep the key's 40 bits, an overflow-filter bit and the fid in one
 * 8-byte slot (kma_bucket_slots() per bucket); tables of K = 9..12 ("wide": the projector's
 * -K, KmerProcessor.java:86-88) use 16-byte slots, four per 64-byte bucket. fid < 2^22 (two
 * bits of each slot's upper word form the bucket's overflow filter; ABI 3 allowed 2^23).
 * The protein path (kma_annotate_proteins*) takes narrow tables: apply's ProteinKmers keeps
 * K = 8 whatever the table holds (ApplyKmerProcessor.java:108 sets KmerReference's K only). */
#define KMA_MAX_K 12
/* Layout codes (kma_table_build_device, kma_table_wrap_device, kma_table_layout_for): the
 * minimizer length m (0 = flat) | KMA_LAYOUT_TWO_CHOICE for two-choice placement (ABI 6)
 * | KMA_LAYOUT_MOD_SAMPLING for the mod-sampling minimizer order (ABI 7; K = 8, m = 6 only: a
 * key's minimizer is its m-mer at the position, modulo K - m + 1, of its smallest residue
 * (rank 31 - code, the first on ties), where the other order takes the m-mer of smallest
 * hash; the creators use it for every K = 8, m = 6 table: it cuts the probe's bucket
 * requests).                                                                                 */
#define KMA_LAYOUT_TWO_CHOICE 0x100
#define KMA_LAYOUT_MOD_SAMPLING 0x40
#define KMA_MAX_FID ((1u << 22) - 1u)


typedef struct kma_table kma_table;         /* opaque: a signature table resident on one GPU */
typedef struct kma_workspace kma_workspace; /* opaque: per-stream scratch for _device calls  */

typedef struct kma_table_info {
  uint64_t n_rows;       /* rows passed to create                                          */
  uint64_t n_skipped;    /* rows whose kmer length != K (can never match; still "loaded")  */
  uint64_t n_entries;    /* distinct keys stored (duplicates resolved last-wins)           */
  uint64_t n_buckets;    /* buckets of kma_bucket_slots() 8-byte slots                     */
  uint64_t bytes;        /* device bytes of the slot array = n_buckets * slots * 8          */
  int32_t k;             /* kmer length                                                    */
  int32_t device;        /* HIP device ordinal                                             */
  uint32_t max_probe;    /* longest bucket chain a stored key needs (1 = home bucket)      */
  uint32_t n_extra_syms; /* bytes mapped to codes 28..31                                   */
  uint8_t extra_syms[4];
  int32_t minimizer_len; /* layout: a key's home bucket is a hash of its minimizer m-mer;
                            0 = flat (hash of the whole key)                               */
  uint64_t n_displaced;  /* keys stored past their home bucket (overflow chains)            */
  int32_t n_replicas;    /* devices holding a copy of the slot array                        */
  int32_t slots_per_bucket; /* kma_bucket_slots_for(k): 8 (16) narrow, 4 wide               */
  double replicate_ms;   /* ABI 6: wall time of the last kma_table_replicate (its copies run
                            concurrently, one stream per destination); 0 before any         */
  uint64_t replicate_bytes; /* ABI 6: bytes that call copied (slot array x destinations)    */
  int32_t two_choice;    /* ABI 6: placement. 1 = two-choice (every key in its home bucket or
                            in one other bucket, a hash of the whole key: a lookup reads at
                            most 2 buckets); 0 = overflow chains                            */
  int32_t minimizer_order; /* ABI 7: how a key's minimizer is chosen among its m-mers (layout
                            code bit KMA_LAYOUT_MOD_SAMPLING): 0 = smallest m-mer hash;
                            1 = mod-sampling (the m-mer at the position, modulo K - m + 1,
                            of the smallest residue: rank 31 - code, the first on ties)      */
  int32_t replicate_peer;  /* ABI 7: copies of the last kma_table_replicate made with peer
                            access enabled (the destination GPU reads replica 0 over xGMI)  */
  int32_t replicate_local; /* ABI 7: copies of that call on replica 0's own device; the rest
                            (replicate_bytes / bytes - peer - local) were left to the runtime
                            without peer access (it may stage them through host memory)     */
} kma_table_info;

/* One 6-frame hit: the kmer at forward 1-based left edge `left` on `strand` ('+' or '-') of
 * contig `contig` is in the table with function `fid`. Emitted in canonical order
 * (contig, left, strand '+' before '-').  Location = [left, left + 3K - 1] on the forward
 * strand, exactly Location.create(contig, dir, left, left + K3) of KmerReference.java:192.  */
typedef struct kma_hit {
  uint32_t contig;
  int32_t left;
  uint32_t fid;
  uint8_t strand; /* '+' or '-'                       */
  uint8_t frame;  /* 1..3 within the strand's sequence */
  uint16_t pad;
} kma_hit;

/* ---- library ------------------------------------------------------------------------------ */
int kma_abi_version(void);
const char* kma_last_error(void);
int kma_device_count(int* out_n);

/* ---- options ---------------------------------------------------------------------------------
 * Library-wide tuning defaults, read by every later call (the library reads no environment
 * variables; tuning builds compiled with -DKMA_TUNING_ENV=1 seed these from KMA_MINIMIZER,
 * KMA_BLOCK_PROTEINS, KMA_DEFER, KMA_HOST_PIECES and KMA_HASH_SLICE). Defaults in brackets.
 *   KMA_OPT_LAYOUT          table creators' layout [-1: size rule + measurement, see
 *                           kma_table_layout_for]; 0 = flat, 6 / 7 = minimizer m = min(K, value)
 *                           in the smallest-hash order; 6 | KMA_LAYOUT_MOD_SAMPLING = m 6 in the
 *                           mod-sampling order (K = 8; the size rule's m = 6 code at K = 8)
 *   KMA_OPT_BLOCK_PROTEINS  proteins per annotate_kernel block [0: by batch and table size];
 *                           1..8
 *   KMA_OPT_DEFER           the protein kernel's two-pass grid [-1: automatic for grids of 1-4
 *                           resident waves]; 0 = off; 1..64 = groups of fewer probe steps start
 *                           after every longer one, on any batch
 *   KMA_OPT_HOST_PIECES     host protein calls: staging / kernel pipeline pieces [0: up to 8];
 *                           1..16
 *   KMA_OPT_HASH_SLICE      kma_hash_annotate: candidates per prototype slice [0: 2^31 - 1]
 *   KMA_OPT_PACKED_INPUT    protein calls [1]: residues are packed to 5 bits before the probe
 *                           and the probe reads the packed stream: host calls while staging
 *                           (the H2D moves 0.625 B per residue) under 1 and 2; device calls
 *                           with a pack kernel into the workspace under 2, and under 1 for
 *                           batches of >= 2^25 residues; 0 = the probe packs ASCII itself
 *   KMA_OPT_HOST_THREADS    host calls: threads staging (copying / packing) the input, the
 *                           whole call's budget split over the replicas it fans out to [0: each
 *                           of n replicas min(16, cores / n), cores = the process's CPUs bounded
 *                           by its cgroup CPU quota]; 1..64
 *   KMA_OPT_HOST_SLICE      host protein calls: residues per device call [0: 2^31]; a replica's
 *                           share of a larger batch is annotated as consecutive slices of
 *                           whole proteins (tallies summed); 1 .. 2^32 - 128 (tests set it low)
 *   KMA_OPT_PLACEMENT       table creators [-1: two-choice placement for K <= 8, chains if that
 *                           build fails, and for K > 8]; 0 = chains only; 1 = as -1
 *   KMA_OPT_HOST_PIECE_MIN  host protein calls: fewest residues per pipeline piece [0: 2^24]; a
 *                           call runs min(KMA_OPT_HOST_PIECES, residues / this) pieces (ABI 7;
 *                           tests set it low to run many pieces on small batches)
 * kma_workspace_option_set overrides KMA_OPT_BLOCK_PROTEINS / KMA_OPT_DEFER for the _device
 * calls made with one workspace (KMA_OPT_DEFAULT: follow the library default again).        */
#define KMA_OPT_LAYOUT 1
#define KMA_OPT_BLOCK_PROTEINS 2
#define KMA_OPT_DEFER 3
#define KMA_OPT_HOST_PIECES 4
#define KMA_OPT_HASH_SLICE 5
#define KMA_OPT_PACKED_INPUT 6
#define KMA_OPT_HOST_THREADS 7
#define KMA_OPT_HOST_SLICE 8
#define KMA_OPT_PLACEMENT 9
#define KMA_OPT_HOST_PIECE_MIN 10
#define KMA_OPT_DEFAULT INT64_MIN
int kma_option_set(int option, int64_t value);
int kma_option_get(int option, int64_t* value);

/* Pack n kmers of length K (rows of `text` delimited by offsets[0..n]) with the standard
 * alphabet + the table's extra symbols. out_keys[r] = 0 for a row that is not of length K or
 * contains a byte the table cannot encode. Host-side helper; no device needed.             */
int kma_pack_kmers(const kma_table* table, const char* text, const uint64_t* offsets, uint64_t n,
                   uint64_t* out_keys);

/* ---- signature table (ApplyKmerProcessor.java:100-110) -------------------------------------
 * Rows are (kmer text, fid) in file order. Duplicate kmers: the LAST row wins (HashMap.put).
 * Rows whose kmer is not of length K are counted in n_skipped and never match (apply's
 * ProteinKmers keeps its own K = 8 whatever KmerReference.setKmerSize(:108) is given).
 * load_factor <= 0 selects the default 0.5.                                                   */
int kma_table_create(const char* text, const uint64_t* offsets, const uint32_t* fids, uint64_t n,
                     int k, int device, double load_factor, kma_table** out);
/* From apply's kmerdb.tbl itself (ABI 7; ApplyKmerProcessor.java:100-108, whose loop reads the
 * file row by row into a HashMap<String,String>): the headerless tab-separated file (kmer in
 * column 0, role id in column 1; TabbedLineReader(file, 2)) is mapped and parsed on the host's
 * cores; a row's role becomes a dense fid in first-seen row order; then as
 * kma_table_create_replicated on device_ids[0 .. n_devices) (last row of a kmer wins, rows not
 * of length K never match). Outputs (each optional): *role_names = the role ids in fid order,
 * each followed by a NUL byte, in one buffer of *role_bytes bytes that the caller releases with
 * kma_free; *n_roles; *last_kmer_len = the last row's kmer length (what :108 passes to
 * KmerReference.setKmerSize). KMA_E_IO if the file cannot be opened or mapped.                */
int kma_table_create_from_tsv(const char* path, int k, int n_devices, const int* device_ids,
                              double load_factor, kma_table** out, char** role_names,
                              uint64_t* role_bytes, uint32_t* n_roles, int* last_kmer_len);
void kma_free(void* p);
/* Same from pre-packed keys (standard alphabet only; key 0 rows are skipped).               */
int kma_table_create_packed(const uint64_t* keys, const uint32_t* fids, uint64_t n, int k,
                            int device, double load_factor, kma_table** out);
int kma_table_info_get(const kma_table* table, kma_table_info* out);
int kma_table_destroy(kma_table* table);
/* u64 slots per bucket of this build's narrow tables: 8 (64-byte buckets, the default) or 16
 * (128-byte). kma_bucket_slots_for(k): slots per bucket of a table of K-mers (narrow: the
 * former; wide, K 9..12: 4 slots of 16 bytes); 0 for an invalid K.                          */
int kma_bucket_slots(void);
int kma_bucket_slots_for(int k);
/* The table's layout choice. Placement (ABI 6): narrow tables (K <= 8) are built with
 * two-choice placement — every key in its home bucket or in one other bucket, a hash of the
 * whole key — so a lookup reads at most two buckets; a two-choice minimizer table with more than
 * 40% of its keys outside their home is also built flat and the flat one kept if it halves them.
 * When that build fails (a key that finds no place after 2,000 evictions: load factors near 1
 * with crowded minimizers) and for wide tables, keys overflow along chains: minimizer layouts
 * (m = min(K,6) up to 2^25 narrow buckets — 2^24 with 16-slot buckets, 2^26 wide ones — else
 * min(K,7)); when more than 15% of the keys land past their home bucket or a chain exceeds 32
 * buckets (keys that pile onto few minimizers), the creators also build the table flat (layout 0)
 * and keep it if it halves the displaced keys or the longest chain. kma_table_layout_for gives
 * the size-derived layout code (m | KMA_LAYOUT_TWO_CHOICE when the creators try that first;
 * KMA_OPT_LAYOUT = 0 / 6 / 7 forces m, KMA_OPT_PLACEMENT = 0 chains).                       */
int kma_table_layout_for(int k, uint64_t n_buckets);

/* ---- replicas (the table replicated on every device of the node) -------------
 * kma_table_create_replicated: kma_table_create on device_ids[0], then kma_table_replicate on
 * the others. kma_table_replicate: copy replica 0's slot array to each listed device (a peer
 * copy over xGMI between MI355X GPUs; a device may be listed twice — two replicas on one GPU,
 * each served by its own host thread and stream). Every destination is allocated first, then
 * all copies are issued at once, each on a stream of its destination (each GPU's copy engine
 * pulls over its own xGMI link), and the call waits for all of them; the time and bytes are in
 * kma_table_info. kma_table_replicas: the replica count and (up to cap) their devices, in
 * shard order.                                                                                */
int kma_table_create_replicated(const char* text, const uint64_t* offsets, const uint32_t* fids,
                                uint64_t n, int k, int n_devices, const int* device_ids,
                                double load_factor, kma_table** out);
int kma_table_replicate(kma_table* table, int n_devices, const int* device_ids);
int kma_table_replicas(const kma_table* table, int* n, int* device_ids, int cap);

/* Device-resident construction for hosts that own device memory (e.g. a torch allocation
 * that is later broadcast over RCCL to the other GPUs of the node).
 *   kma_table_buckets_for : bucket count for n narrow (K <= 8) keys at the load factor;
 *                           kma_table_buckets_for_k for any K
 *   kma_table_build_device: d_slots (info.bytes: n_buckets * 64 bytes, 128 in the 16-slot build)
 *                           and d_winner (n_buckets * S u32, S = kma_bucket_slots_for(k)) are
 *                           caller scratch; keys/fids are device arrays of K-mers; layout -1 =
 *                           kma_table_layout_for's code (in both build and wrap: a table built
 *                           with -1 wraps with -1, unless the caller rebuilt it with an explicit
 *                           code after a failed two-choice build: then it wraps with that code),
 *                           else 0 / min(K,6) / min(K,7) (| KMA_LAYOUT_MOD_SAMPLING), | KMA_LAYOUT_
 *                           TWO_CHOICE for two-choice placement (K <= 8; d_winner unused; the
 *                           build allocates its sort buffers and waits for `stream`); builds on
 *                           `stream`; d_status (4 u32) receives {table full / two-choice build
 *                           failed, entries, longest chain (two-choice: 1 or 2), displaced
 *                           keys} (a caller rebuilds chained when [0] is set, and may rebuild
 *                           with layout 0 when displaced keys are many); fids are masked to 22
 *                           bits; keys that are 0 or not K-mer keys (>= 2^(5K)) are not stored.
 *   kma_table_wrap_device : adopt an already-built slot array of that layout code (not owned;
 *                           the placement and order are not stored in the slots: the code must be
 *                           the one the table was built with).                                   */
uint64_t kma_table_buckets_for(uint64_t n_keys, double load_factor);
uint64_t kma_table_buckets_for_k(uint64_t n_keys, double load_factor, int k);
int kma_table_build_device(void* d_slots, uint64_t n_buckets, int k, int layout,
                           uint32_t* d_winner, const uint64_t* d_keys, const uint32_t* d_fids,
                           uint64_t n, uint32_t* d_status, void* stream);
int kma_table_wrap_device(void* d_slots, uint64_t n_buckets, int k, int layout, int device,
                          kma_table** out);
/* Raw view of the slot array (device pointer) — what an RCCL broadcast moves.               */
int kma_table_device_ptr(const kma_table* table, void** d_slots, uint64_t* bytes);

/* ---- workspaces -----------------------------------------------------------------------------
 * Per-stream scratch of the _device entry points. kma_workspace_reserve_batch sizes it for
 * calls of up to n_residues residues (< 2^32 - 128; n_seq < 2^31 is checked, nothing is kept
 * per protein): 8 bytes per residue of HBM (the distinct-kmer sets of proteins too long for
 * LDS). kma_workspace_reserve(ws, n) = _reserve_batch(ws, n, n / 16 + 256). These are the only
 * calls that allocate.                                                                       */
int kma_workspace_create(int device, kma_workspace** out);
int kma_workspace_reserve(kma_workspace* ws, uint64_t n_residues);
int kma_workspace_reserve_batch(kma_workspace* ws, uint64_t n_residues, uint64_t n_seq);
int kma_workspace_destroy(kma_workspace* ws);
int kma_workspace_option_set(kma_workspace* ws, int option, int64_t value); /* see options */
/* Device timing of the _device calls made with this workspace: with enable = 1 each call
 * records hipEvents on its stream at its phase boundaries. Not for graph capture. Both reads
 * synchronise on the recorded events (the last 256 calls) and clear the accumulators.
 *   _phases_read : the calls laid out like the last one (same entry point): their count, the
 *                  number of phases and each phase's summed milliseconds and name (static
 *                  strings): proteins {annotate_kernel}; contigs {contigs_probe_kernel,
 *                  scan_emit}.
 *   _timing_read : kernel_ms = proteins: every phase / contigs: the probe; rest_ms = contigs:
 *                  the emit pass (offsets from the group sums the probe adds; the phase keeps
 *                  its ABI-3 name scan_emit).                                                */
#define KMA_MAX_PHASES 8
int kma_workspace_timing(kma_workspace* ws, int enable);
int kma_workspace_timing_read(kma_workspace* ws, uint32_t* n_calls, double* kernel_ms,
                              double* rest_ms);
int kma_workspace_phases_read(kma_workspace* ws, uint32_t* n_calls, int* n_phases,
                              double* phase_ms, const char** phase_names);

/* ---- protein annotation (ApplyKmerProcessor.java:118-148) ----------------------------------
 * residues: raw ASCII proteins concatenated; sequence s is residues[offsets[s]..offsets[s+1]).
 * min_hits >= 1 (ApplyKmerProcessor.java:91-92). out_tally (optional, length n_fid) receives
 * += 1 per CALLED protein at its fid (the APPLY report's role counts before column mapping).
 * Host form: synchronous, host buffers. A batch of >= 32 MiB of residues is cut into pieces of
 * whole proteins (up to 8; KMA_OPT_HOST_PIECES overrides, 1..16), one kernel each. Packed input
 * (KMA_OPT_PACKED_INPUT, the default) is packed on KMA_OPT_HOST_THREADS threads in stream order
 * and copied in segments as soon as each is packed, on the context's two copy streams; a
 * piece's kernel follows its last segment (ASCII input: each piece staged, then copied, under
 * the previous piece's kernel). A replica's share of more than 2^31 residues
 * (KMA_OPT_HOST_SLICE) is annotated as consecutive slices of whole proteins, one device call
 * each; only a single protein longer than 2^32 - 128 residues is refused (KMA_E_INVALID).     */
int kma_annotate_proteins(const kma_table* table, const uint8_t* residues,
                          const uint64_t* offsets, uint32_t n_seq, int min_hits, uint32_t flags,
                          int32_t* out_fid, int32_t* out_count, uint8_t* out_status,
                          uint32_t* out_tally, uint32_t n_fid);
/* Device form: every pointer is device memory on the workspace's device (the table has a
 * replica there); `d_residues` is 8-byte aligned and readable for 32 bytes past
 * offsets[n_seq]; n_residues = offsets[n_seq] - offsets[0] (<= the workspace reservation);
 * d_tally (n_fid u32) is accumulated into, not cleared. Asynchronous on `stream`: one kernel
 * launch (annotate_kernel: each window probes the table where it stands, per-protein sets and
 * the vote in LDS), preceded by a pack kernel into the workspace under KMA_OPT_PACKED_INPUT
 * (default: batches of >= 2^25 residues).                                                      */
int kma_annotate_proteins_device(const kma_table* table, kma_workspace* ws,
                                 const uint8_t* d_residues, const uint64_t* d_offsets,
                                 uint32_t n_seq, uint64_t n_residues, int min_hits,
                                 uint32_t flags, int32_t* d_fid, int32_t* d_count,
                                 uint8_t* d_status, uint32_t* d_tally, uint32_t n_fid,
                                 void* stream);

/* ---- packed residue streams ------------------------------------------------------------------
 * The protein kernel's input format: residue j of a call is the 5-bit code (the table's packing,
 * 0 for a byte without a code) at bits [5j, 5j + 5) of a big-endian bit stream — byte b of the
 * stream holds bits [8b, 8b + 8), most significant first; 8 residues fill 5 bytes.
 *   kma_packed_bytes  : stream bytes for n residues, read padding included (40 per 64 + 16)
 *   kma_pack_residues : host packing (AVX2 where the CPU has it) of residues[0, n) into out
 *                       (out_bytes >= kma_packed_bytes(n); the rest is zeroed) with the table's
 *                       codes (table NULL: the standard alphabet); no device needed
 *   kma_annotate_packed_device : kma_annotate_proteins_device on a packed stream already in
 *                       device memory (8-byte aligned): stream residue 0 is residue
 *                       d_offsets[0]; one kernel launch.                                      */
uint64_t kma_packed_bytes(uint64_t n_residues);
int kma_pack_residues(const kma_table* table, const uint8_t* residues, uint64_t n, uint8_t* out,
                      uint64_t out_bytes);
int kma_annotate_packed_device(const kma_table* table, kma_workspace* ws, const uint8_t* d_stream,
                               const uint64_t* d_offsets, uint32_t n_seq, uint64_t n_residues,
                               int min_hits, uint32_t flags, int32_t* d_fid, int32_t* d_count,
                               uint8_t* d_status, uint32_t* d_tally, uint32_t n_fid,
                               void* stream);

/* ---- 6-frame contig annotation (KmerReference.java:157-203 + table probe) -----------------
 * dna: contigs concatenated (any case; bases other than ACGT translate to 'X'); offsets as
 * above. genetic_code: NCBI table id (1, 2, 3, 4, 5, 6, 9, 10, 11, 12, 13, 14, 16, 21, 22, 23,
 * 24, 25). Windows follow processKmers exactly (i < P_f - K end
 * exclusion, '*'/'X' windows skipped). Every remaining window is probed; hits are written in
 * canonical order. If cap is too small, returns KMA_E_CAPACITY with *n_hits = needed.
 * out_tally (optional, n_contig * n_fid u32, row-major by contig) counts hits per function. */
int kma_annotate_contigs(const kma_table* table, const uint8_t* dna, const uint64_t* offsets,
                         uint32_t n_contig, int genetic_code, kma_hit* out_hits, uint64_t cap,
                         uint64_t* n_hits, uint32_t* out_tally, uint32_t n_fid);
/* Device form (same semantics), asynchronous on `stream`: d_dna / d_offsets are device buffers
 * on the table's device (contig s = d_dna[d_offsets[s] .. d_offsets[s+1]); d_offsets[0] may
 * be nonzero); n_bases = offsets[n_contig] - offsets[0] (<= the contig reservation of `ws`);
 * d_dna readable for 64 bytes past the last base. Hits [0, cap) go to d_hits in canonical
 * order and *d_n_hits (device u64) receives the total, which may exceed cap (then the hits
 * past cap are dropped: compare and call again with a larger buffer). d_tally (n_contig x
 * n_fid u32, optional) is accumulated into. Never allocates or synchronises; keeps no host
 * state between calls (the emit pass leaves the workspace's group sums zero), so a call may be
 * captured in a hipGraph and replayed. Calls on one workspace are ordered on one stream.     */
int kma_workspace_reserve_contigs(kma_workspace* ws, uint64_t n_bases);
int kma_annotate_contigs_device(const kma_table* table, kma_workspace* ws, const uint8_t* d_dna,
                                const uint64_t* d_offsets, uint32_t n_contig, uint64_t n_bases,
                                int genetic_code, kma_hit* d_hits, uint64_t cap,
                                uint64_t* d_n_hits, uint32_t* d_tally, uint32_t n_fid,
                                void* stream);
/* ---- peg-kmer join of the projector (KmerProcessor.java:195-207) -----------------------------
 * kma_peg_table_create: the singleton peg kmers of a close genome as a table whose fid is the
 * peg index: every window i < L-K of every peg without 'X' (KmerReference.countPegKmers,
 * KmerReference.java:124-147), counted by kmer over the whole batch; kmers seen exactly once
 * (CountMap.getSingletons via getPegKmers, KmerProcessor.java:320-327) map to their peg.
 * Built on the device (window packing, radix sort, singleton select, table build). Windows with
 * bytes outside A-Z / '*' never equal a translated contig kmer and are left out.
 * *n_windows (optional) receives the number of counted windows; table info n_entries the
 * singletons. n_peg <= 2^22.
 * kma_connect_pegs: every location of a singleton in the new genome's 6-frame contig kmer map
 * connected to its peg (framer.connect(pegId, loc)), i.e. hits with fid = peg index in the
 * canonical order of kma_annotate_contigs. strict != 0 applies KmerFactory.Strict
 * (KmerFactory.java:61-69): kmers with more than one location in the genome are dropped.
 * Capacity handling as kma_annotate_contigs.                                                 */
int kma_peg_table_create(const uint8_t* residues, const uint64_t* offsets, uint32_t n_peg, int k,
                         int device, double load_factor, kma_table** out, uint64_t* n_windows);
int kma_connect_pegs(const kma_table* peg_table, const uint8_t* dna, const uint64_t* offsets,
                     uint32_t n_contig, int genetic_code, int strict, kma_hit* out_hits,
                     uint64_t cap, uint64_t* n_hits);

/* ---- proposal sweep of the projector (KmerProcessor.java:209-264) ----------------------------
 * The connections of one close genome (kma_connect_pegs hits, fid = peg index, in its canonical
 * (contig, left) order) are grouped into framed location lists (FramedLocationLists.connect,
 * FramedLocationLists.java:156-171): one list per frame (strand and the phase of a location's
 * end point) and peg, sorted by (contig, left). For peg p with protein length peg_len[p] (aa),
 * pegLen = 3 peg_len[p], maxLen = (int)(pegLen max_fuzz + 1), minLen = (int)(pegLen min_fuzz),
 * minKmers = (int)(pegLen (min_strength / 3)) (:222-228); a list shorter than minKmers is
 * skipped; every start i <= size - minKmers gets evidence = 1 + #{later locations on i's contig
 * with right < left_i + maxLen} and right = the largest such right edge (or its own), and is a
 * proposal unless right < left_i + minLen (:233-257). Proposals come out in list order (frame
 * '-' phases 0..2, '+' phases 0..2; peg index; start) — Java visits pegs in HashMap order.
 * stats[4]: lists, lists with too few kmers, too-short starts, proposals. The sweep runs on
 * `device`; KMA_E_CAPACITY with *n_out = needed if cap is too small; KMA_E_INVALID if the hits
 * are not in (contig, left) order or a fid >= n_peg. Defaults of the reference: min_strength
 * 0.5, max_fuzz 1.5, min_fuzz 0.8 (KmerProcessor.setDefaults, :141-146).                    */
typedef struct kma_proposal {
  uint32_t peg;
  uint32_t contig;
  int32_t left;
  int32_t right;     /* bestEdge                                      */
  uint32_t evidence; /* kmers of evidence (the first location included) */
  uint8_t strand;    /* '+' or '-'                                    */
  uint8_t frame;     /* list frame: 0..2 '-' phases, 3..5 '+' phases   */
  uint16_t pad;
} kma_proposal;
int kma_propose_pegs(const kma_hit* hits, uint64_t n_hits, const uint32_t* peg_len,
                     uint32_t n_peg, int k, double min_strength, double max_fuzz,
                     double min_fuzz, int device, kma_proposal* out, uint64_t cap,
                     uint64_t* n_out, uint64_t* stats);

/* ---- hash annotator scoring (HashAnnotationProcessor.java:221-328) ---------------------------
 * A genome's distinct protein sequences (the caller keys features by MD5, as GenomeProteinKmers
 * does; proteins holding '*' are left out, :239-241) against the prototypes of the role
 * annotation file in file order (:253-271; the caller drops prototypes shorter than minLen,
 * :148-152). GenomeProteinKmers (external) restated: ProteinKmers sets of distinct K-mers
 * (windows i = 0..L-K), similarity = shared / (|A| + |B| - shared) in double, a prototype
 * becomes a protein's proposal when similarity >= min_sim and above the current one (earlier
 * prototypes win ties). out_best[g] = prototype index or -1 (the default proposal: the old
 * annotation with score 0.0, :285-288), out_sim[g] = its similarity (0.0 if none),
 * out_count[p] = proteins with similarity >= min_sim (processProposal's return). K 2..12,
 * 0 <= min_sim < 1; KMA_E_ALPHABET for bytes outside A-Z / '*'. Runs on `device` (sorts and
 * scans; see kma_hashanno.hip).                                                              */
int kma_hash_annotate(const uint8_t* genome_residues, const uint64_t* genome_offsets,
                      uint32_t n_genome, const uint8_t* proto_residues,
                      const uint64_t* proto_offsets, uint32_t n_proto, int k, double min_sim,
                      int device, int32_t* out_best, double* out_sim, uint32_t* out_count);

/* ---- signature-table construction (BuildKmerProcessor.java:137-223, RoleCounter.java) -------
 * After role resolution by the host (Feature.getUsefulRoles + the interesting-role filter):
 * roles[s] >= 0 is the single good role of an interesting peg, -1 marks a protein buffered for
 * the deletion pass (no good role), any other negative value a peg that is skipped (several
 * good roles). A kmer of ProteinKmers (distinct windows, i = 0..L-K; KMA_F_END_EXCLUSIVE for
 * i < L-K) is kept iff every interesting peg containing it has the same role (RoleCounter
 * isGood) and no buffered protein contains it. Output: (packed key, role) rows sorted by key
 * (the reference prints HashMap order: compare as sets); KMA_E_CAPACITY with *n_out = needed
 * if cap is too small; KMA_E_ALPHABET if a counted window holds a byte outside A-Z / '*'.
 * Roles < 2^24 - 1; K 1..12; < 2^31 residues. Runs on the device: window packing, radix sort
 * of the (key, role) pairs by key, RoleCounter per key run (one role, no buffered protein),
 * select.                                                                                    */
int kma_build_signatures(const uint8_t* residues, const uint64_t* offsets, const int32_t* roles,
                         uint32_t n_seq, int k, uint32_t flags, int device, uint64_t* out_keys,
                         uint32_t* out_roles, uint64_t cap, uint64_t* n_out);

/* ---- ProteinKmers.distance (genome/compare/GeneCopyProcessor.java:129-162) -----------------
 * One batch of proteins (residues, offsets, n_seq); pair i compares proteins pair_a[i] and
 * pair_b[i]. Sets are ProteinKmers of kmer size k (2..12, GeneCopyProcessor -K): the distinct
 * substrings at i = 0 .. L-k (KMA_F_END_EXCLUSIVE: i < L-k). out_sim[i] = |A n B|; out_size
 * (optional, n_seq) = |S| of every protein; out_dist (optional) = 1 - |A n B| / |A u B| in
 * double, 1.0 when the sets share nothing (SequenceKmers.distance, external, restated).
 * KMA_E_ALPHABET if a window holds a byte outside A-Z / '*'. Runs on the device: window keys,
 * segmented radix sort per protein, a binary-search intersection per pair; synchronous.     */
int kma_protein_distances(const uint8_t* residues, const uint64_t* offsets, uint32_t n_seq, int k,
                          uint32_t flags, const uint32_t* pair_a, const uint32_t* pair_b,
                          uint64_t n_pairs, int device, uint32_t* out_sim, uint32_t* out_size,
                          double* out_dist);
/* GeneCopyProcessor's choice (:135-146) for n_query queries: query[q] against the candidates
 * cand[cand_off[q] .. cand_off[q+1]) in order, starting from fDist = max_dist, keeps the LAST
 * candidate with distance <= the running best (`f2Dist <= fDist`). out_best[q] = that
 * candidate's protein index or -1; out_best_dist[q] (optional) = its distance (max_dist if
 * none).                                                                                      */
int kma_protein_best_match(const uint8_t* residues, const uint64_t* offsets, uint32_t n_seq, int k,
                           uint32_t flags, const uint32_t* query, const uint64_t* cand_off,
                           const uint32_t* cand, uint32_t n_query, double max_dist, int device,
                           int32_t* out_best, double* out_best_dist);

/* Window count of the 6-frame extractor before the '*'/'X' filter (for throughput metrics).  */
uint64_t kma_contig_window_count(const uint64_t* offsets, uint32_t n_contig, int k);

#ifdef __cplusplus
}
#endif
#endif /* KMERANNO_H */
