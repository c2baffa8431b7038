/*
 * kma_oracle.c — ORACLE (test infrastructure only; never shipped, never measured as the product).
 *
 * A scalar CPU restatement of the SEEDtk/kmers.anno signature-kmer annotation path, written
 * from the Java sources (paths relative to /root/reference/src/main/java/org/theseed/) with
 * String semantics kept literally: kmers are byte strings compared with memcmp, the signature
 * table is a chained hash map with last-wins put, and a protein's kmers are a set of distinct
 * substrings. It deliberately shares NO code with the product (no 5-bit packing, no bucketed
 * table): it is the checker. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it.
 *
 * Parity status
 *   - 6-frame extraction (orc_contig_kmers), peg kmers (orc_peg_kmers), Location math:
 *     pinned against the reference's own test properties on src/test/small.gto
 *     (test/.../anno/AppTest.java:69-161), re-expressed in tests/test_oracle_golden.py.
 *   - apply vote (orc_apply) and ProteinKmers window semantics: PARITY UNPINNED. The Java
 *     reference cannot run here (no JDK, no org.theseed jars) and no reference test exercises
 *     ApplyKmerProcessor or ProteinKmers. This restatement is cross-checked against an
 *     independent pure-Python restatement (oracle/oracle_py.py) and hand-built edge cases.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_F_END_EXCLUSIVE 0x1u
#define ORC_F_MULTISET 0x2u

/* ------------------------------------------------------------------------------------------ */
/* HashMap<String,String> restated: chained buckets, Java String.hashCode + HashMap.hash spread */
/* ------------------------------------------------------------------------------------------ */
typedef struct orc_node {
  struct orc_node* next;
  uint32_t hash;
  int32_t value;
  int32_t len;
  char key[]; /* len bytes */
} orc_node;

typedef struct orc_table {
  orc_node** buckets;
  uint64_t mask;
  uint64_t size;
} orc_table;

static uint32_t java_string_hash(const char* s, int len) {
  uint32_t h = 0; /* String.hashCode: s[0]*31^(n-1) + ... */
  for (int i = 0; i < len; i++) h = 31u * h + (uint8_t)s[i];
  return h ^ (h >> 16); /* HashMap.hash spread */
}

static void orc_table_grow(orc_table* t) {
  uint64_t nb = (t->mask + 1) * 2;
  orc_node** b = (orc_node**)calloc(nb, sizeof(orc_node*));
  for (uint64_t i = 0; i <= t->mask; i++) {
    orc_node* n = t->buckets[i];
    while (n) {
      orc_node* nx = n->next;
      uint64_t j = n->hash & (nb - 1);
      n->next = b[j];
      b[j] = n;
      n = nx;
    }
  }
  free(t->buckets);
  t->buckets = b;
  t->mask = nb - 1;
}

static void orc_table_put(orc_table* t, const char* key, int len, int32_t value) {
  uint32_t h = java_string_hash(key, len);
  for (orc_node* n = t->buckets[h & t->mask]; n; n = n->next)
    if (n->hash == h && n->len == len && memcmp(n->key, key, (size_t)len) == 0) {
      n->value = value; /* ApplyKmerProcessor.java:106: put -> the last row wins */
      return;
    }
  orc_node* n = (orc_node*)malloc(sizeof(orc_node) + (size_t)len);
  n->hash = h;
  n->value = value;
  n->len = len;
  memcpy(n->key, key, (size_t)len);
  n->next = t->buckets[h & t->mask];
  t->buckets[h & t->mask] = n;
  if (++t->size > (t->mask + 1) / 4 * 3) orc_table_grow(t);
}

/* Returns the value or -1 when absent (HashMap.get -> null). */
int32_t orc_table_get(const orc_table* t, const char* key, int len) {
  uint32_t h = java_string_hash(key, len);
  for (orc_node* n = t->buckets[h & t->mask]; n; n = n->next)
    if (n->hash == h && n->len == len && memcmp(n->key, key, (size_t)len) == 0) return n->value;
  return -1;
}

/* ApplyKmerProcessor.java:101-107: every row of the headerless 2-column file is put, in file
 * order; rows of any length are loaded (they simply never match a K-window). */
orc_table* orc_table_new(const char* text, const uint64_t* offsets, const int32_t* values,
                         uint64_t n) {
  orc_table* t = (orc_table*)calloc(1, sizeof(orc_table));
  uint64_t nb = 16;
  while (nb < n / 2) nb <<= 1;
  t->buckets = (orc_node**)calloc(nb, sizeof(orc_node*));
  t->mask = nb - 1;
  for (uint64_t r = 0; r < n; r++)
    orc_table_put(t, text + offsets[r], (int)(offsets[r + 1] - offsets[r]), values[r]);
  return t;
}

uint64_t orc_table_size(const orc_table* t) { return t->size; }

void orc_table_free(orc_table* t) {
  if (!t) return;
  for (uint64_t i = 0; i <= t->mask; i++) {
    orc_node* n = t->buckets[i];
    while (n) {
      orc_node* nx = n->next;
      free(n);
      n = nx;
    }
  }
  free(t->buckets);
  free(t);
}

/* ------------------------------------------------------------------------------------------ */
/* ProteinKmers(String) restated (external org.theseed.sequence, UNVERIFIED semantics):       */
/* the set of distinct substrings s[i, i+K) for i = 0..L-K (inclusive end by default).        */
/* Set elements are kept as window start indices in first-insertion order.                   */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  int32_t* slots; /* open addressing over window starts, -1 empty */
  uint32_t cap;   /* allocated slots */
  int32_t* order; /* distinct window starts, insertion order */
  uint32_t n;
  uint32_t mask;  /* hash mask of the last build (its capacity - 1) */
} kmer_set;

static void kmer_set_build(kmer_set* s, const char* p, int64_t L, int K, uint32_t flags) {
  int64_t nwin = L - K + ((flags & ORC_F_END_EXCLUSIVE) ? 0 : 1);
  s->n = 0;
  if (nwin <= 0) return;
  uint32_t cap = 16;
  while (cap < (uint64_t)nwin * 2) cap <<= 1;
  if (cap > s->cap) {
    free(s->slots);
    free(s->order);
    s->slots = (int32_t*)malloc(sizeof(int32_t) * cap);
    s->order = (int32_t*)malloc(sizeof(int32_t) * cap);
    s->cap = cap;
  }
  for (uint32_t i = 0; i < cap; i++) s->slots[i] = -1;
  s->mask = cap - 1;
  for (int64_t i = 0; i < nwin; i++) {
    if (flags & ORC_F_MULTISET) { /* every window counts: no set semantics */
      s->order[s->n++] = (int32_t)i;
      continue;
    }
    uint32_t h = java_string_hash(p + i, K) & (cap - 1);
    for (;;) {
      int32_t j = s->slots[h];
      if (j < 0) {
        s->slots[h] = (int32_t)i;
        s->order[s->n++] = (int32_t)i;
        break;
      }
      if (memcmp(p + j, p + i, (size_t)K) == 0) break; /* HashSet.add of an equal String */
      h = (h + 1) & (cap - 1);
    }
  }
}

#define ORC_STATUS_NONE 0
#define ORC_STATUS_CALLED 1
#define ORC_STATUS_AMBIGUOUS 2
#define ORC_STATUS_BELOW_MIN 3

/* ApplyKmerProcessor.runCommand :122-147, literally: iterate the kmer set, probe the table,
 * first hit sets the role, a confirming hit counts, a different role marks the peg bad and
 * stops the loop; the feature is recorded iff role != null && !bad && count >= minHits. */
void orc_apply(const orc_table* t, const uint8_t* residues, const uint64_t* offsets,
               uint32_t n_seq, int K, int min_hits, uint32_t flags, int32_t* out_fid,
               int32_t* out_count, uint8_t* out_status) {
  kmer_set set = {0};
  for (uint32_t s = 0; s < n_seq; s++) {
    const char* p = (const char*)residues + offsets[s];
    int64_t L = (int64_t)(offsets[s + 1] - offsets[s]);
    kmer_set_build(&set, p, L, K, flags);
    int32_t role = -1, count = 0;
    int bad = 0;
    for (uint32_t k = 0; k < set.n && !bad; k++) {
      int32_t possible = orc_table_get(t, p + set.order[k], K);
      if (possible >= 0) {
        if (role < 0) {
          role = possible;
          count = 1;
        } else if (possible == role) {
          count++;
        } else {
          bad = 1;
        }
      }
    }
    if (role < 0) {
      out_fid[s] = -1, out_count[s] = 0, out_status[s] = ORC_STATUS_NONE;
    } else if (bad) {
      out_fid[s] = -1, out_count[s] = 0, out_status[s] = ORC_STATUS_AMBIGUOUS;
    } else {
      out_fid[s] = role, out_count[s] = count;
      out_status[s] = count >= min_hits ? ORC_STATUS_CALLED : ORC_STATUS_BELOW_MIN;
    }
  }
  free(set.slots);
  free(set.order);
}

/* The same loop over all host cores (the CPU baseline's multi-core leg):
 * proteins are independent and the table is read-only after the load, so contiguous ranges
 * of proteins go to n_threads pthreads, each with its own kmer set. */
typedef struct {
  const orc_table* t;
  const uint8_t* residues;
  const uint64_t* offsets;
  uint32_t lo, hi;
  int K, min_hits;
  uint32_t flags;
  int32_t *fid, *count;
  uint8_t* status;
} orc_apply_job;

static void* orc_apply_worker(void* arg) {
  orc_apply_job* j = (orc_apply_job*)arg;
  orc_apply(j->t, j->residues, j->offsets + j->lo, j->hi - j->lo, j->K, j->min_hits, j->flags,
            j->fid + j->lo, j->count + j->lo, j->status + j->lo);
  return 0;
}

void orc_apply_mt(const orc_table* t, const uint8_t* residues, const uint64_t* offsets,
                  uint32_t n_seq, int K, int min_hits, uint32_t flags, int32_t* out_fid,
                  int32_t* out_count, uint8_t* out_status, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  pthread_t th[256];
  orc_apply_job job[256];
  for (int i = 0; i < n_threads; i++) {
    /* interleaved chunks of 64 proteins would balance better; contiguous ranges keep each
     * thread's residues contiguous, and protein lengths are iid in the sample */
    job[i] = (orc_apply_job){t, residues, offsets, (uint32_t)((uint64_t)n_seq * i / n_threads),
                             (uint32_t)((uint64_t)n_seq * (i + 1) / n_threads), K, min_hits,
                             flags, out_fid, out_count, out_status};
    if (pthread_create(&th[i], 0, orc_apply_worker, &job[i]) != 0) { /* run it here */
      orc_apply_worker(&job[i]);
      th[i] = 0;
    }
  }
  for (int i = 0; i < n_threads; i++)
    if (th[i]) pthread_join(th[i], 0);
}

/* ------------------------------------------------------------------------------------------ */
/* DnaTranslator restated (external org.theseed.proteins): codon -> amino acid by NCBI table,  */
/* case-insensitive ACGT, any other base makes the codon 'X'.                                 */
/* ------------------------------------------------------------------------------------------ */
static int base_index(char c) { /* NCBI tables enumerate codons in T, C, A, G order */
  switch (c) {
    case 't': case 'T': case 'u': case 'U': return 0;
    case 'c': case 'C': return 1;
    case 'a': case 'A': return 2;
    case 'g': case 'G': return 3;
    default: return -1;
  }
}

static const char* ncbi_table(int gcode) {
  switch (gcode) {
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
    default: return 0;
  }
}

/* translate(seq, frame, len): codons starting at 1-based `frame`, floor((len-frame+1)/3) aa. */
int64_t orc_translate(const char* dna, int64_t len, int frame, int gcode, char* out) {
  const char* tab = ncbi_table(gcode);
  if (!tab) return -1;
  int64_t n = 0;
  for (int64_t p = frame - 1; p + 3 <= len; p += 3) {
    int a = base_index(dna[p]), b = base_index(dna[p + 1]), c = base_index(dna[p + 2]);
    out[n++] = (a < 0 || b < 0 || c < 0) ? 'X' : tab[a * 16 + b * 4 + c];
  }
  return n;
}

/* Contig.getRSequence restated: reverse complement (case kept, other bytes -> 'n'). The RNA
 * base U pairs like T (U -> A), as DnaTranslator reads U as T on the forward strand: a
 * documented choice (both are external, parity unpinned for U); the kernel does the same. */
void orc_reverse_complement(const char* dna, int64_t len, char* out) {
  for (int64_t i = 0; i < len; i++) {
    char c = dna[len - 1 - i], r;
    switch (c) {
      case 'a': r = 't'; break; case 'c': r = 'g'; break;
      case 'g': r = 'c'; break; case 't': case 'u': r = 'a'; break;
      case 'A': r = 'T'; break; case 'C': r = 'G'; break;
      case 'G': r = 'C'; break; case 'T': case 'U': r = 'A'; break;
      default: r = 'n';
    }
    out[i] = r;
  }
}

/* KmerReference.processKmers :180-203 for one strand, with KmerPosition.calcLeft :60-62 /
 * :78-86. Records are appended while n < cap; the needed count is always returned. */
static uint64_t process_strand(const char* seq, int64_t len, int minus, uint32_t contig,
                               int gcode, int K, char* prot, char* out_kmers,
                               uint32_t* out_contig, int32_t* out_left, uint8_t* out_strand,
                               uint8_t* out_frame, uint64_t n, uint64_t cap) {
  int64_t base = len - 3 * K + 2; /* KmerPosition.Minus: contigLen - kmerLen + 2 */
  for (int frame = 1; frame <= 3; frame++) {
    int64_t P = orc_translate(seq, len, frame, gcode, prot);
    int64_t end = P - K; /* :186-187 the point past the last legal kmer start (exclusive) */
    for (int64_t i = 0; i < end; i++) {
      const char* km = prot + i;
      int ok = 1;
      for (int j = 0; j < K; j++)
        if (km[j] == '*' || km[j] == 'X') { ok = 0; break; } /* :190 containsNone('*','X') */
      if (!ok) continue;
      int64_t left = minus ? base - (i * 3 + frame) : i * 3 + frame;
      if (n < cap) {
        if (out_kmers) memcpy(out_kmers + n * K, km, (size_t)K);
        out_contig[n] = contig;
        out_left[n] = (int32_t)left;
        out_strand[n] = minus ? '-' : '+';
        out_frame[n] = (uint8_t)frame;
      }
      n++;
    }
  }
  return n;
}

/* KmerReference.getContigKmers :157-169 flattened to records (kmer, contig, left, strand,
 * frame) in the reference's own visiting order: contig, + strand then - strand, frame 1..3,
 * window i ascending. */
uint64_t orc_contig_kmers(const uint8_t* dna, const uint64_t* offsets, uint32_t n_contig,
                          int gcode, int K, char* out_kmers, uint32_t* out_contig,
                          int32_t* out_left, uint8_t* out_strand, uint8_t* out_frame,
                          uint64_t cap) {
  uint64_t n = 0;
  if (!ncbi_table(gcode)) return (uint64_t)-1;
  for (uint32_t c = 0; c < n_contig; c++) {
    const char* seq = (const char*)dna + offsets[c];
    int64_t len = (int64_t)(offsets[c + 1] - offsets[c]);
    char* rseq = (char*)malloc((size_t)len + 1);
    char* prot = (char*)malloc((size_t)len / 3 + 2);
    orc_reverse_complement(seq, len, rseq);
    n = process_strand(seq, len, 0, c, gcode, K, prot, out_kmers, out_contig, out_left,
                       out_strand, out_frame, n, cap);
    n = process_strand(rseq, len, 1, c, gcode, K, prot, out_kmers, out_contig, out_left,
                       out_strand, out_frame, n, cap);
    free(rseq);
    free(prot);
  }
  return n;
}

/* Signature-table probe of every 6-frame window (the DNA form of the apply lookup): returns
 * (contig, left, strand, frame, fid) for windows whose kmer is in the table, sorted by
 * (contig, left, strand '+' first). */
typedef struct {
  uint32_t contig;
  int32_t left;
  uint32_t fid;
  uint8_t strand, frame;
} orc_hit;

static int hit_cmp(const void* a, const void* b) {
  const orc_hit *x = (const orc_hit*)a, *y = (const orc_hit*)b;
  if (x->contig != y->contig) return x->contig < y->contig ? -1 : 1;
  if (x->left != y->left) return x->left < y->left ? -1 : 1;
  return (int)x->strand - (int)y->strand; /* '+' (43) < '-' (45) */
}

uint64_t orc_annotate_contigs(const orc_table* t, const uint8_t* dna, const uint64_t* offsets,
                              uint32_t n_contig, int gcode, int K, uint32_t* out_contig,
                              int32_t* out_left, uint8_t* out_strand, uint8_t* out_frame,
                              uint32_t* out_fid, uint64_t cap) {
  uint64_t total = orc_contig_kmers(dna, offsets, n_contig, gcode, K, 0, 0, 0, 0, 0, 0);
  if (total == (uint64_t)-1) return total;
  char* km = (char*)malloc(total * (uint64_t)K + 1);
  uint32_t* ct = (uint32_t*)malloc(sizeof(uint32_t) * (total + 1));
  int32_t* lf = (int32_t*)malloc(sizeof(int32_t) * (total + 1));
  uint8_t* st = (uint8_t*)malloc(total + 1);
  uint8_t* fr = (uint8_t*)malloc(total + 1);
  orc_contig_kmers(dna, offsets, n_contig, gcode, K, km, ct, lf, st, fr, total);
  orc_hit* hits = (orc_hit*)malloc(sizeof(orc_hit) * (total + 1));
  uint64_t nh = 0;
  for (uint64_t r = 0; r < total; r++) {
    int32_t v = orc_table_get(t, km + r * K, K);
    if (v < 0) continue;
    orc_hit h = {ct[r], lf[r], (uint32_t)v, st[r], fr[r]};
    hits[nh++] = h;
  }
  qsort(hits, nh, sizeof(orc_hit), hit_cmp);
  for (uint64_t i = 0; i < nh && i < cap; i++) {
    out_contig[i] = hits[i].contig;
    out_left[i] = hits[i].left;
    out_strand[i] = hits[i].strand;
    out_frame[i] = hits[i].frame;
    out_fid[i] = hits[i].fid;
  }
  free(km), free(ct), free(lf), free(st), free(fr), free(hits);
  return nh;
}

/* KmerReference.countPegKmers :124-147: windows i < L-K (end exclusive), skipping kmers that
 * contain 'X'; location begin = i + 1 on the peg. Records in visiting order. */
uint64_t orc_peg_kmers(const uint8_t* residues, const uint64_t* offsets, uint32_t n_seq, int K,
                       char* out_kmers, uint32_t* out_peg, int32_t* out_left, uint64_t cap) {
  uint64_t n = 0;
  for (uint32_t s = 0; s < n_seq; s++) {
    const char* p = (const char*)residues + offsets[s];
    int64_t end = (int64_t)(offsets[s + 1] - offsets[s]) - K;
    for (int64_t i = 0; i < end; i++) {
      if (memchr(p + i, 'X', (size_t)K)) continue;
      if (n < cap) {
        if (out_kmers) memcpy(out_kmers + n * K, p + i, (size_t)K);
        out_peg[n] = s;
        out_left[n] = (int32_t)(i + 1);
      }
      n++;
    }
  }
  return n;
}

/* The peg-kmer join of the projector, KmerProcessor.java:195-207 with getPegKmers (:320-327),
 * KmerReference.countPegKmers (:124-147) and KmerFactory.findKmers (KmerFactory.java:61-82):
 *   1. count every peg window (i < L-K, no 'X') of the close genome by kmer text; keep the
 *      kmers seen exactly once (CountMap.getSingletons) with the peg they came from;
 *   2. the new genome's contig kmer map (getContigKmers); STRICT (strict != 0) drops kmers with
 *      more than one location;
 *   3. for every singleton peg kmer, every location of it in the map is connected to its peg
 *      (framer.connect(pegId, loc)).
 * The HashSet/HashMap iteration order of the Java loop carries no meaning (the framer sorts),
 * so the connections are returned as (contig, left, strand, frame, peg) sorted canonically,
 * like orc_annotate_contigs. Returns the number of connections. */
uint64_t orc_peg_connect(const uint8_t* residues, const uint64_t* offsets, uint32_t n_peg,
                         const uint8_t* dna, const uint64_t* doffsets, uint32_t n_contig,
                         int gcode, int K, int strict, uint32_t* out_contig, int32_t* out_left,
                         uint8_t* out_strand, uint8_t* out_frame, uint32_t* out_peg,
                         uint64_t cap) {
  const uint64_t np = orc_peg_kmers(residues, offsets, n_peg, K, 0, 0, 0, 0);
  char* pk = (char*)malloc(np * (uint64_t)K + 1);
  uint32_t* pp = (uint32_t*)malloc(sizeof(uint32_t) * (np + 1));
  int32_t* pl = (int32_t*)malloc(sizeof(int32_t) * (np + 1));
  orc_peg_kmers(residues, offsets, n_peg, K, pk, pp, pl, np);
  /* CountMap: value = the peg of the first occurrence, -2 once seen again */
  orc_table* pegs = orc_table_new(0, 0, 0, 0);
  for (uint64_t r = 0; r < np; r++) {
    const int32_t v = orc_table_get(pegs, pk + r * K, K);
    orc_table_put(pegs, pk + r * K, K, v == -1 ? (int32_t)pp[r] : -2);
  }
  const uint64_t nc = orc_contig_kmers(dna, doffsets, n_contig, gcode, K, 0, 0, 0, 0, 0, 0);
  if (nc == (uint64_t)-1) {
    orc_table_free(pegs);
    free(pk), free(pp), free(pl);
    return nc;
  }
  char* ck = (char*)malloc(nc * (uint64_t)K + 1);
  uint32_t* ct = (uint32_t*)malloc(sizeof(uint32_t) * (nc + 1));
  int32_t* lf = (int32_t*)malloc(sizeof(int32_t) * (nc + 1));
  uint8_t* st = (uint8_t*)malloc(nc + 1);
  uint8_t* fr = (uint8_t*)malloc(nc + 1);
  orc_contig_kmers(dna, doffsets, n_contig, gcode, K, ck, ct, lf, st, fr, nc);
  orc_table* locs = orc_table_new(0, 0, 0, 0); /* kmer -> number of locations (STRICT) */
  if (strict)
    for (uint64_t r = 0; r < nc; r++) {
      const int32_t v = orc_table_get(locs, ck + r * K, K);
      orc_table_put(locs, ck + r * K, K, v < 0 ? 1 : v + 1);
    }
  orc_hit* hits = (orc_hit*)malloc(sizeof(orc_hit) * (nc + 1));
  uint64_t nh = 0;
  for (uint64_t r = 0; r < nc; r++) {
    const int32_t v = orc_table_get(pegs, ck + r * K, K);
    if (v < 0) continue; /* not a peg kmer, or not a singleton */
    if (strict && orc_table_get(locs, ck + r * K, K) > 1) continue;
    orc_hit h = {ct[r], lf[r], (uint32_t)v, st[r], fr[r]};
    hits[nh++] = h;
  }
  qsort(hits, nh, sizeof(orc_hit), hit_cmp);
  for (uint64_t i = 0; i < nh && i < cap; i++) {
    out_contig[i] = hits[i].contig;
    out_left[i] = hits[i].left;
    out_strand[i] = hits[i].strand;
    out_frame[i] = hits[i].frame;
    out_peg[i] = hits[i].fid;
  }
  orc_table_free(pegs), orc_table_free(locs);
  free(pk), free(pp), free(pl), free(ck), free(ct), free(lf), free(st), free(fr), free(hits);
  return nh;
}

/* BuildKmerProcessor.runCommand (anno/BuildKmerProcessor.java:137-223) with RoleCounter
 * (kmers/RoleCounter.java:30-55), after role resolution: role[s] >= 0 is the single good role
 * of an interesting peg, -1 marks a buffered protein (no good role), anything else a peg with
 * several good roles (skipped, :163-175). Pass 1: for every distinct kmer of every interesting
 * peg (ProteinKmers set), kmerMap.computeIfAbsent(kmer, RoleCounter(role)).count(role); a kmer
 * counted for a second role is bad and deleted (:178-188). Pass 2: every kmer of a buffered
 * protein is removed (:191-205). Surviving (kmer, role) rows are written in table order (the
 * reference prints HashMap order: compare as sets). Returns the number of rows. */
uint64_t orc_build(const uint8_t* residues, const uint64_t* offsets, const int32_t* role,
                   uint32_t n_seq, int K, uint32_t flags, char* out_kmers, int32_t* out_role,
                   uint64_t cap) {
  orc_table* m = orc_table_new(0, 0, 0, 0);
  kmer_set set = {0};
  for (uint32_t s = 0; s < n_seq; s++) {
    if (role[s] < 0) continue;
    const char* p = (const char*)residues + offsets[s];
    kmer_set_build(&set, p, (int64_t)(offsets[s + 1] - offsets[s]), K, flags & ~ORC_F_MULTISET);
    for (uint32_t j = 0; j < set.n; j++) {
      const char* km = p + set.order[j];
      const int32_t v = orc_table_get(m, km, K);
      if (v == -1) orc_table_put(m, km, K, role[s]);       /* new RoleCounter(role), good hit */
      else if (v >= 0 && v != role[s]) orc_table_put(m, km, K, -3); /* bad: another role */
    }
  }
  for (uint32_t s = 0; s < n_seq; s++) {
    if (role[s] != -1) continue;
    const char* p = (const char*)residues + offsets[s];
    kmer_set_build(&set, p, (int64_t)(offsets[s + 1] - offsets[s]), K, flags & ~ORC_F_MULTISET);
    for (uint32_t j = 0; j < set.n; j++) {
      const char* km = p + set.order[j];
      if (orc_table_get(m, km, K) != -1) orc_table_put(m, km, K, -4); /* kmerMap.remove */
    }
  }
  uint64_t n = 0;
  for (uint64_t b = 0; b <= m->mask; b++)
    for (orc_node* x = m->buckets[b]; x; x = x->next) {
      if (x->value < 0) continue;
      if (n < cap) {
        memcpy(out_kmers + n * K, x->key, (size_t)K);
        out_role[n] = x->value;
      }
      n++;
    }
  free(set.slots), free(set.order);
  orc_table_free(m);
  return n;
}

/* ------------------------------------------------------------------------------------------ */
/* SequenceKmers.distance restated (external org.theseed.sequence, UNVERIFIED semantics), as   */
/* GeneCopyProcessor.runCommand calls it (genome/compare/GeneCopyProcessor.java:137-142):      */
/* similarity = |{distinct kmers of B} n {kmers of A}|, union = |A| + |B| - similarity,        */
/* distance = 1 - similarity / union, or 1.0 when nothing is shared. Kmers are ProteinKmers    */
/* sets of size K (i = 0..L-K; ORC_F_END_EXCLUSIVE: i < L-K).                                  */
/* ------------------------------------------------------------------------------------------ */
static int kmer_set_contains(const kmer_set* s, const char* p, const char* km, int K) {
  if (s->n == 0) return 0;
  uint32_t h = java_string_hash(km, K) & s->mask;
  for (;;) {
    int32_t j = s->slots[h];
    if (j < 0) return 0;
    if (memcmp(p + j, km, (size_t)K) == 0) return 1;
    h = (h + 1) & s->mask;
  }
}

void orc_protein_distances(const uint8_t* residues, const uint64_t* offsets, int K,
                           uint32_t flags, const uint32_t* pair_a, const uint32_t* pair_b,
                           uint64_t n_pairs, uint32_t* out_sim, uint32_t* out_size_a,
                           uint32_t* out_size_b, double* out_dist) {
  kmer_set sa = {0}, sb = {0};
  flags &= ~ORC_F_MULTISET;
  for (uint64_t i = 0; i < n_pairs; i++) {
    const char* pa = (const char*)residues + offsets[pair_a[i]];
    const char* pb = (const char*)residues + offsets[pair_b[i]];
    kmer_set_build(&sa, pa, (int64_t)(offsets[pair_a[i] + 1] - offsets[pair_a[i]]), K, flags);
    kmer_set_build(&sb, pb, (int64_t)(offsets[pair_b[i] + 1] - offsets[pair_b[i]]), K, flags);
    uint32_t sim = 0;
    for (uint32_t j = 0; j < sb.n; j++) sim += (uint32_t)kmer_set_contains(&sa, pa, pb + sb.order[j], K);
    out_sim[i] = sim;
    out_size_a[i] = sa.n;
    out_size_b[i] = sb.n;
    out_dist[i] = sim > 0 ? 1.0 - (double)sim / ((double)sa.n + (double)sb.n - (double)sim) : 1.0;
  }
  free(sa.slots), free(sa.order), free(sb.slots), free(sb.order);
}


/* ---- (f)2: the proposal sweep of the projector ----------------------------------------------
 * KmerProcessor.annotateGenome, KmerProcessor.java:209-264, over the framed location lists of
 * one close genome's connections (FramedLocationLists.connect, FramedLocationLists.java:156-171).
 * Restated external semantics (org.theseed.locations Location / SortedLocationList / Frame are
 * not in the reference; parity unpinned for them):
 *   - a kmer location is (contig, strand, left .. left + 3K - 1); its frame is its strand and the
 *     phase (mod 3) of its end point (right on '+', left on '-'); any definition by absolute
 *     coordinates mod 3 puts the same locations in one list, only the frames' ORDER differs;
 *   - SortedLocationList orders by (contig, left); contigRange(i) = the locations after i on
 *     i's contig;
 *   - lists are visited frame by frame ('-' phases 0, 1, 2, then '+' phases 0, 1, 2) and by peg
 *     index within a frame (Java: HashMap order of the peg ids); starts in list order.
 * Per list: pegLen = 3 * protein length; maxLen = (int)(pegLen * maxFuzz + 1); minLen =
 * (int)(pegLen * minFuzz); minKmers = (int)(pegLen * (minStrength / 3)) (:222-228). A list
 * shorter than minKmers counts as too few; otherwise every start i <= size - minKmers gets
 * evidence = 1 + #{j in contigRange(i) : right_j < left_i + maxLen} and bestEdge = the largest
 * such right (or right_i) (:233-246); bestEdge < left_i + minLen counts as too short, else a
 * proposal (contig, strand, left_i, bestEdge, evidence) for the list's peg (:248-257).
 * Deviation: a start past the list end (minKmers <= 0, which makes the Java loop read past the
 * list) is not visited. stats: [0] lists, [1] too few kmers, [2] too short, [3] proposals. */
typedef struct {
  uint32_t contig, peg;
  int32_t left;
  uint8_t strand, frame;
} orc_loc;

static uint8_t orc_frame_idx(uint8_t strand, int32_t left, int K) {
  const int32_t end = strand == '+' ? left + 3 * K - 1 : left;
  return (uint8_t)((strand == '+' ? 3 : 0) + end % 3);
}

static int loc_cmp(const void* a, const void* b) {
  const orc_loc *x = (const orc_loc*)a, *y = (const orc_loc*)b;
  if (x->frame != y->frame) return x->frame < y->frame ? -1 : 1;
  if (x->peg != y->peg) return x->peg < y->peg ? -1 : 1;
  if (x->contig != y->contig) return x->contig < y->contig ? -1 : 1;
  if (x->left != y->left) return x->left < y->left ? -1 : 1;
  return 0;
}

uint64_t orc_propose(const uint32_t* contig, const int32_t* left, const uint8_t* strand,
                     const uint32_t* peg, uint64_t n, const uint32_t* peg_len, int K,
                     double min_strength, double max_fuzz, double min_fuzz, uint32_t* o_peg,
                     uint32_t* o_contig, uint8_t* o_strand, int32_t* o_left, int32_t* o_right,
                     uint32_t* o_evidence, uint8_t* o_frame, uint64_t cap, uint64_t* stats) {
  orc_loc* L = (orc_loc*)malloc(sizeof(orc_loc) * (n + 1));
  for (uint64_t i = 0; i < n; i++) {
    orc_loc l = {contig[i], peg[i], left[i], strand[i], orc_frame_idx(strand[i], left[i], K)};
    L[i] = l;
  }
  qsort(L, n, sizeof(orc_loc), loc_cmp);
  const int32_t span = 3 * K - 1;  /* right = left + span */
  const double real_strength = min_strength / 3;
  uint64_t n_out = 0;
  stats[0] = stats[1] = stats[2] = stats[3] = 0;
  for (uint64_t s = 0; s < n;) {
    uint64_t e = s + 1;
    while (e < n && L[e].frame == L[s].frame && L[e].peg == L[s].peg) e++;
    const int64_t size = (int64_t)(e - s);
    const int32_t peg_bp = (int32_t)peg_len[L[s].peg] * 3;
    const int32_t max_len = (int32_t)(peg_bp * max_fuzz + 1);
    const int32_t min_len = (int32_t)(peg_bp * min_fuzz);
    const int32_t min_kmers = (int32_t)(peg_bp * real_strength);
    stats[0]++;
    if (min_kmers > size) {
      stats[1]++;
    } else {
      const int64_t last = size - min_kmers;
      for (int64_t i = 0; i <= last && i < size; i++) {
        const orc_loc* f = &L[s + i];
        int32_t evidence = 1;
        const int32_t max_edge = f->left + max_len, min_edge = f->left + min_len;
        int32_t best = f->left + span;
        for (int64_t j = i + 1; j < size && L[s + j].contig == f->contig; j++) {
          const int32_t r = L[s + j].left + span;
          if (r < max_edge) {
            evidence++;
            best = r > best ? r : best;
          }
        }
        if (best < min_edge) {
          stats[2]++;
        } else {
          if (n_out < cap) {
            o_peg[n_out] = f->peg;
            o_contig[n_out] = f->contig;
            o_strand[n_out] = f->strand;
            o_left[n_out] = f->left;
            o_right[n_out] = best;
            o_evidence[n_out] = (uint32_t)evidence;
            o_frame[n_out] = f->frame;
          }
          n_out++;
          stats[3]++;
        }
      }
    }
    s = e;
  }
  free(L);
  return n_out;
}

/* ---- (f)3: the hash annotator's scoring loop ---------------------------------------------------
 * HashAnnotationProcessor.processGenome (HashAnnotationProcessor.java:221-328) with
 * GenomeProteinKmers (external org.theseed.proteins.kmers; restated, parity unpinned):
 * addProtein gives each distinct genome protein a default proposal (score 0.0); processProposal
 * (:259-271) is called for every prototype in file order: for every genome protein sharing at
 * least one distinct K-mer (ProteinKmers windows i = 0..L-K), sim = shared / (|A| + |B| -
 * shared); sim >= minSim counts as a match (the call's return) and, when above the protein's
 * current score, makes the prototype its proposal. Literal restatement: every (prototype,
 * protein) pair by a merge of the two sorted distinct key lists. */
static uint64_t pack_kmer(const uint8_t* p, int K, int* ok) {
  uint64_t v = 0;
  *ok = 1;
  for (int j = 0; j < K; j++) {
    const uint8_t c = p[j];
    uint32_t code = (c >= 'A' && c <= 'Z') ? (uint32_t)(c - 'A' + 1) : (c == '*' ? 27u : 0u);
    if (!code) *ok = 0;
    v = (v << 5) | code;
  }
  return v;
}

static int u64_cmp(const void* a, const void* b) {
  const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? -1 : x > y;
}

/* distinct sorted keys of each sequence: keys[off[s]..off[s]+size[s]) */
static uint64_t* distinct_sets(const uint8_t* res, const uint64_t* off, uint32_t n, int K,
                               uint32_t* size) {
  uint64_t* keys = (uint64_t*)malloc(sizeof(uint64_t) * (off[n] - off[0] + 1));
  for (uint32_t s = 0; s < n; s++) {
    const uint64_t lo = off[s] - off[0];
    const int64_t nw = (int64_t)(off[s + 1] - off[s]) - K + 1;
    uint32_t m = 0;
    for (int64_t i = 0; i < nw; i++) {
      int ok;
      keys[lo + m++] = pack_kmer(res + off[s] + i, K, &ok);
    }
    qsort(keys + lo, m, sizeof(uint64_t), u64_cmp);
    uint32_t d = 0;
    for (uint32_t i = 0; i < m; i++)
      if (i == 0 || keys[lo + i] != keys[lo + i - 1]) keys[lo + d++] = keys[lo + i];
    size[s] = d;
  }
  return keys;
}

void orc_hash_annotate(const uint8_t* gres, const uint64_t* goff, uint32_t n_gp,
                       const uint8_t* pres, const uint64_t* poff, uint32_t n_pt, int K,
                       double min_sim, int32_t* out_best, double* out_sim, uint32_t* out_count) {
  uint32_t* gs = (uint32_t*)malloc(sizeof(uint32_t) * (n_gp + 1));
  uint32_t* ps = (uint32_t*)malloc(sizeof(uint32_t) * (n_pt + 1));
  uint64_t* gk = distinct_sets(gres, goff, n_gp, K, gs);
  uint64_t* pk = distinct_sets(pres, poff, n_pt, K, ps);
  for (uint32_t g = 0; g < n_gp; g++) out_best[g] = -1, out_sim[g] = 0.0;
  for (uint32_t p = 0; p < n_pt; p++) {
    const uint64_t* a = pk + (poff[p] - poff[0]);
    uint32_t matches = 0;
    for (uint32_t g = 0; g < n_gp; g++) {
      const uint64_t* b = gk + (goff[g] - goff[0]);
      uint32_t i = 0, j = 0, shared = 0;
      while (i < ps[p] && j < gs[g]) {
        if (a[i] < b[j]) i++;
        else if (a[i] > b[j]) j++;
        else shared++, i++, j++;
      }
      if (!shared) continue;
      const double sim = (double)shared / ((double)ps[p] + (double)gs[g] - (double)shared);
      if (sim >= min_sim) {
        matches++;
        if (sim > out_sim[g]) out_sim[g] = sim, out_best[g] = (int32_t)p;
      }
    }
    out_count[p] = matches;
  }
  free(gs), free(ps), free(gk), free(pk);
}
