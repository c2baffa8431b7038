"""Seeded synthetic workloads for the BASELINE.json configs (SURVEY.md §8(d) generator).

- protein lengths resampled from the 712 CDS lengths of the reference fixture small.gto
  (data/small_gto_cds_lengths.txt: min 35, median 264, mean 310.5, max 2955);
- residues iid uniform over the 20 standard amino acids;
- F functions, one prototype protein each; the signature table holds prototype 8-mers that are
  unique to one function (BuildKmerProcessor.java:157-208's rule), at most T // F per function,
  padded with random decoy 8-mers up to T rows, rows shuffled;
- queries: 50% prototype copies with 10% per-residue substitution, 40% random proteins,
  10% chimeras (first half of one prototype + second half of another, both mutated);
- role string of fid i is ROLE%07d.
Keys use the standard 5-bit packing of include/kmeranno.h.
"""

from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

AA = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", dtype=np.uint8)
AA_CODES = (AA.astype(np.uint64) - 64)  # 'A' -> 1 ... 'Y' -> 25
_LEN_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data",
                         "small_gto_cds_lengths.txt")


def cds_lengths() -> np.ndarray:
    return np.loadtxt(_LEN_FILE, dtype=np.int64, comments="#")


def window_keys(res: np.ndarray, k: int = 8) -> np.ndarray:
    """Packed keys of every window of one ASCII protein (standard alphabet)."""
    codes = res.astype(np.uint64) - 64
    n = len(res) - k + 1
    if n <= 0:
        return np.zeros(0, np.uint64)
    key = np.zeros(n, np.uint64)
    for j in range(k):
        key = (key << np.uint64(5)) | codes[j:j + n]
    return key


def unpack_key(key: int, k: int = 8) -> str:
    return "".join(chr(64 + ((int(key) >> (5 * (k - 1 - j))) & 31)) for j in range(k))


@dataclass
class Workload:
    keys: np.ndarray       # uint64 [T] packed table kmers (file order)
    fids: np.ndarray       # uint32 [T]
    n_fid: int
    residues: np.ndarray   # uint8 ASCII, padded by 32 zero bytes
    offsets: np.ndarray    # uint64 [n_seq + 1]
    kinds: np.ndarray      # uint8 [n_seq]: 0 copy, 1 random, 2 chimera
    true_fid: np.ndarray   # int32 [n_seq]: source function (-1 random)

    @property
    def n_seq(self) -> int:
        return len(self.offsets) - 1

    @property
    def n_windows(self) -> int:
        L = np.diff(self.offsets).astype(np.int64)
        return int(np.maximum(L - 7, 0).sum())


def _mutate(rng, prot: np.ndarray, rate: float) -> np.ndarray:
    out = prot.copy()
    m = rng.random(len(out)) < rate
    out[m] = AA[rng.integers(0, 20, int(m.sum()))]
    return out


@dataclass
class SignatureSet:
    protos: list           # prototype proteins (uint8 ASCII), one per function
    keys: np.ndarray       # uint64 [T] packed table kmers (file order)
    fids: np.ndarray       # uint32 [T]
    n_fid: int


def make_table(table_size: int, n_fid: int, seed: int, k: int = 8,
               protos_only: bool = False) -> SignatureSet:
    """protos_only: the prototypes alone (what a rank that receives the table by broadcast
    needs to generate its queries); keys and fids are then empty."""
    rng = np.random.default_rng(seed)
    lens = cds_lengths()
    plen = rng.choice(lens, n_fid)
    protos = [AA[rng.integers(0, 20, int(L))] for L in plen]
    if protos_only:
        return SignatureSet(protos, np.zeros(0, np.uint64), np.zeros(0, np.uint32), n_fid)
    pk = [np.unique(window_keys(p, k)) for p in protos]
    all_k = np.concatenate(pk)
    all_f = np.repeat(np.arange(n_fid, dtype=np.uint32), [len(x) for x in pk])
    _, inv, cnt = np.unique(all_k, return_inverse=True, return_counts=True)
    unique_mask = cnt[inv] == 1  # kmer occurs in exactly one function's prototype
    all_k, all_f = all_k[unique_mask], all_f[unique_mask]
    per_fn = max(1, table_size // n_fid)
    # At most per_fn kmers per function (random subset), then decoys up to table_size.
    order = rng.permutation(len(all_k))
    all_k, all_f = all_k[order], all_f[order]
    srt = np.argsort(all_f, kind="stable")
    starts = np.searchsorted(all_f[srt], np.arange(n_fid))
    rank = np.empty(len(all_k), np.int64)
    rank[srt] = np.arange(len(all_k)) - starts[all_f[srt]]
    keep = rank < per_fn
    sig_k, sig_f = all_k[keep][:table_size], all_f[keep][:table_size]
    n_decoy = table_size - len(sig_k)
    dec = np.zeros(n_decoy, np.uint64)
    for _ in range(k):
        dec = (dec << np.uint64(5)) | AA_CODES[rng.integers(0, 20, n_decoy)]
    dec_f = rng.integers(0, n_fid, n_decoy).astype(np.uint32)
    keys = np.concatenate([sig_k, dec])
    fids = np.concatenate([sig_f, dec_f]).astype(np.uint32)
    perm = rng.permutation(len(keys))
    return SignatureSet(protos, keys[perm], fids[perm], n_fid)


def make_queries(sig: SignatureSet, n_seq: int, seed: int, mutation: float = 0.10):
    """(residues padded by 32 bytes, offsets, kinds, true_fid) for one batch."""
    rng = np.random.default_rng(seed)
    lens = cds_lengths()
    protos, n_fid = sig.protos, sig.n_fid
    kinds = rng.choice(np.array([0, 1, 2], np.uint8), n_seq, p=[0.5, 0.4, 0.1])
    true_fid = np.full(n_seq, -1, np.int32)
    seqs = []
    for i in range(n_seq):
        if kinds[i] == 0:
            f = int(rng.integers(0, n_fid))
            true_fid[i] = f
            seqs.append(_mutate(rng, protos[f], mutation))
        elif kinds[i] == 1:
            seqs.append(AA[rng.integers(0, 20, int(rng.choice(lens)))])
        else:
            a, b = rng.integers(0, n_fid, 2)
            pa, pb = protos[int(a)], protos[int(b)]
            true_fid[i] = int(a)
            seqs.append(_mutate(rng, np.concatenate([pa[:len(pa) // 2], pb[len(pb) // 2:]]),
                                mutation))
    offsets = np.zeros(n_seq + 1, np.uint64)
    offsets[1:] = np.cumsum([len(s) for s in seqs])
    residues = np.concatenate(seqs + [np.zeros(32, np.uint8)])
    return residues, offsets, kinds, true_fid


def make_workload(n_seq: int, table_size: int, n_fid: int, seed: int, k: int = 8,
                  mutation: float = 0.10, query_seed: int | None = None) -> Workload:
    sig = make_table(table_size, n_fid, seed, k)
    qs = seed * 1_000_003 + 17 if query_seed is None else query_seed
    residues, offsets, kinds, true_fid = make_queries(sig, n_seq, qs, mutation)
    return Workload(sig.keys, sig.fids, n_fid, residues, offsets, kinds, true_fid)


def role_name(fid: int) -> str:
    return f"ROLE{fid:07d}"


def write_kmer_db(path: str, keys: np.ndarray, fids: np.ndarray, k: int = 8):
    """The headerless kmerdb.tbl of `apply` (kmer<TAB>roleId per row, file order)."""
    codes = np.zeros((len(keys), k + 1), np.uint8)
    for j in range(k):
        codes[:, j] = ((keys >> np.uint64(5 * (k - 1 - j))) & np.uint64(31)).astype(np.uint8) + 64
    codes[:, k] = ord("\t")
    with open(path, "wb") as f:
        step = 1 << 20
        for a in range(0, len(keys), step):
            roles = np.char.add(np.char.mod("ROLE%07d", fids[a:a + step].astype(np.int64)), "\n")
            rows = np.char.add(codes[a:a + step].view(f"S{k + 1}").ravel(),
                               roles.astype("S"))
            f.write(b"".join(rows.tolist()))


def write_roles_in_use(path: str, n_fid: int, every: int = 1):
    """roles.in.use: role id<TAB>description, every `every`-th function."""
    with open(path, "w") as f:
        f.writelines(f"{role_name(i)}\tsynthetic role {i}\n" for i in range(0, n_fid, every))


def write_fasta(path: str, residues: np.ndarray, offsets: np.ndarray, ids, comments=None,
                width: int = 60, chunk: int = 65536) -> int:
    """Protein FASTA (">id comment" headers, sequence lines of `width` residues) of the
    proteins [offsets[i], offsets[i+1]) of `residues`; vectorized over chunks of records (c4's
    1M proteins in a few seconds). Returns the file's size in bytes."""
    n = len(offsets) - 1
    total = 0
    with open(path, "wb") as f:
        for a in range(0, n, chunk):
            b = min(n, a + chunk)
            off = np.asarray(offsets[a:b + 1], np.int64)
            m = b - a
            lens = np.diff(off)
            heads = [f">{ids[i]}" + (f" {comments[i]}" if comments is not None and comments[i]
                                     else "") + "\n" for i in range(a, b)]
            hb = np.frombuffer("".join(heads).encode(), np.uint8)
            hlen = np.fromiter((len(h) for h in heads), np.int64, m)  # ASCII: chars == bytes
            lines = (lens + width - 1) // width
            start = np.zeros(m + 1, np.int64)
            np.cumsum(hlen + lens + lines, out=start[1:])
            out = np.full(int(start[-1]), ord("\n"), np.uint8)  # unwritten slots: line ends
            hstart = np.zeros(m + 1, np.int64)
            np.cumsum(hlen, out=hstart[1:])
            rec = np.repeat(np.arange(m), hlen)
            out[start[rec] + (np.arange(len(hb)) - hstart[rec])] = hb
            rec = np.repeat(np.arange(m), lens)
            p = np.arange(int(off[-1] - off[0]), dtype=np.int64) - (off[rec] - off[0])
            out[start[rec] + hlen[rec] + p + p // width] = residues[int(off[0]):int(off[-1])]
            f.write(out.tobytes())
            total += len(out)
    return total


def write_genome_dir(out_dir: str, sig: SignatureSet, n_genomes: int, pegs_per_genome: int,
                     seed: int, contig_bp: int = 0, first: int = 0) -> list:
    """Synthetic GTO files for `apply` (small.gto-like, in its member order: features of type
    CDS with protein_translation, genetic_code, id, scientific_name, contigs; the function is the peg's true
    role or "hypothetical protein"). Proteins come from make_queries (the SURVEY §8(d) mix);
    each genome gets one random contig of contig_bp bases (skipped by the apply loader, but
    read). Returns [(genome id, residues, offsets)] per genome, in file-name order."""
    os.makedirs(out_dir, exist_ok=True)
    rng = np.random.default_rng(seed)
    out = []
    for g in range(first, first + n_genomes):
        res, off, _, true_fid = make_queries(sig, pegs_per_genome, seed * 7919 + g)
        gid = f"{100000 + g}.{g % 97 + 1}"
        feats = []
        for i in range(pegs_per_genome):
            prot = res[int(off[i]):int(off[i + 1])].tobytes().decode()
            fn = role_name(int(true_fid[i])) if true_fid[i] >= 0 else "hypothetical protein"
            loc = f'[["{gid}.con.0001", {3 * i + 1}, "+", {3 * len(prot) + 3}]]'
            feats.append(f'{{"id": "fig|{gid}.peg.{i + 1}", "type": "CDS", "location": {loc}, '
                         f'"function": "{fn}", "protein_translation": "{prot}", '
                         f'"annotations": [["synthetic", "bench", 0.0]]}}')
        dna = b"acgt"[0:0]
        if contig_bp:
            dna = np.frombuffer(b"acgt", np.uint8)[rng.integers(0, 4, contig_bp)].tobytes()
        # top-level members in small.gto's order (domain, features, genetic_code, id,
        # scientific_name, then contigs: the DNA comes last in SEEDtk GTOs)
        text = (f'{{"domain": "Bacteria", "features": [' + ", ".join(feats) + '], '
                f'"genetic_code": 11, "id": "{gid}", '
                f'"scientific_name": "Synthetica genomica {g}", '
                f'"contigs": [{{"id": "{gid}.con.0001", "dna": "{dna.decode()}"}}]}}')
        with open(os.path.join(out_dir, f"{gid}.gto"), "w") as f:
            f.write(text)
        out.append((gid, res, off))
    order = sorted(range(len(out)), key=lambda i: f"{out[i][0]}.gto")
    return [out[i] for i in order]


# BASELINE.json configs -> (n_seq, table_size, n_fid, seed)
CONFIGS = {
    "c1": (100, 1_000, 100, 1),
    "c2": (10_000, 10_000_000, 10_000, 2),
    "c4": (1_000_000, 10_000_000, 10_000, 4),
    "c5": (1_000_000, 100_000_000, 100_000, 5),
}


def random_contigs(total_bp: int, n_contig: int, seed: int, n_rate: float = 0.0005):
    """Config 3 DNA: contig lengths log-uniform 50 kb..1 Mbp scaled to total_bp, GC 0.5,
    n_rate ambiguous 'n' bases; lower-case like GTO contigs."""
    rng = np.random.default_rng(seed)
    raw = np.exp(rng.uniform(np.log(5e4), np.log(1e6), n_contig))
    lens = np.maximum((raw / raw.sum() * total_bp).astype(np.int64), 100)
    bases = np.frombuffer(b"acgt", np.uint8)
    dna = bases[rng.integers(0, 4, int(lens.sum()))]
    dna[rng.random(len(dna)) < n_rate] = ord("n")
    offsets = np.zeros(n_contig + 1, np.uint64)
    offsets[1:] = np.cumsum(lens)
    return np.concatenate([dna, np.zeros(64, np.uint8)]), offsets


# ---- config 3: 6-frame DNA with planted genes -------------------------------------------------
# NCBI translation table 11 (= 1 for the amino-acid assignment) in TCAG codon order.
_CODE11 = "FFLLSSSSYY**CC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG"
_TCAG = np.frombuffer(b"tcag", np.uint8)


def _codon_choices():
    """aa byte -> array of codons (3 lower-case DNA bytes each) that encode it (code 11)."""
    out = {}
    for i, aa in enumerate(_CODE11):
        codon = _TCAG[[i >> 4, (i >> 2) & 3, i & 3]]
        out.setdefault(ord(aa), []).append(codon)
    return {k: np.array(v, np.uint8) for k, v in out.items()}


def reverse_translate(rng, prot: np.ndarray) -> np.ndarray:
    """A random DNA coding sequence (lower case, code 11, ends with a stop codon) for prot."""
    ch = _codon_choices()
    cod = np.empty((len(prot) + 1, 3), np.uint8)
    for aa in np.unique(prot):
        m = np.flatnonzero(prot == aa)
        opts = ch[int(aa)]
        cod[m] = opts[rng.integers(0, len(opts), len(m))]
    stops = ch[ord("*")]
    cod[-1] = stops[rng.integers(0, len(stops))]
    return cod.reshape(-1)


def reverse_complement(dna: np.ndarray) -> np.ndarray:
    comp = np.arange(256, dtype=np.uint8)
    for a, b in (b"ac", b"ca", b"gt", b"tg", b"AC", b"CA", b"GT", b"TG"):
        comp[a] = b
    for a, b in (b"at", b"ta", b"AT", b"TA"):
        comp[a] = b
    return comp[dna[::-1]]


@dataclass
class ContigWorkload:
    keys: np.ndarray       # uint64 [T] packed table kmers
    fids: np.ndarray       # uint32 [T]
    n_fid: int
    dna: np.ndarray        # uint8 lower-case DNA, padded by 64 zero bytes
    offsets: np.ndarray    # uint64 [n_contig + 1]
    genes: np.ndarray      # int64 [n_gene, 4]: contig, start (0-based), strand (+1/-1), fid

    @property
    def n_contig(self) -> int:
        return len(self.offsets) - 1


def make_contig_workload(total_bp: int = 5_000_000, n_contig: int = 20, seed: int = 3,
                         table_size: int = 10_000_000, n_fid: int = 10_000, k: int = 8,
                         coding: float = 0.5, mutation: float = 0.10) -> ContigWorkload:
    """Config 3: random contigs (log-uniform 50 kb..1 Mbp scaled to total_bp,
    GC 0.5, 0.05% 'n') with genes planted over ~`coding` of the sequence: function prototypes
    mutated at `mutation` per residue, reverse-translated with random synonymous codons
    (code 11) and placed on either strand, non-overlapping."""
    sig = make_table(table_size, n_fid, seed, k)
    dna, offsets = random_contigs(total_bp, n_contig, seed)
    rng = np.random.default_rng(seed * 7919 + 3)
    mean_gene = 3 * 311
    gap_mean = mean_gene * (1 - coding) / coding
    genes = []
    for c in range(n_contig):
        lo, hi = int(offsets[c]), int(offsets[c + 1])
        pos = lo + int(rng.exponential(gap_mean))
        while True:
            f = int(rng.integers(0, n_fid))
            cds = reverse_translate(rng, _mutate(rng, sig.protos[f], mutation))
            if pos + len(cds) > hi:
                break
            strand = 1 if rng.random() < 0.5 else -1
            dna[pos:pos + len(cds)] = cds if strand > 0 else reverse_complement(cds)
            genes.append((c, pos - lo, strand, f))
            pos += len(cds) + int(rng.exponential(gap_mean))
    return ContigWorkload(sig.keys, sig.fids, n_fid, dna, offsets,
                          np.array(genes, np.int64).reshape(-1, 4))


def probed_windows(dna: np.ndarray, offsets: np.ndarray, k: int = 8) -> int:
    """Windows of the 6-frame extractor that are probed (no stop or X residue, within the end
    exclusion of KmerReference.java:186-190), code 11."""
    code = np.frombuffer(_CODE11.encode(), np.uint8)
    lut = np.full(256, 4, np.uint8)
    for i, b in enumerate(b"tcag"):
        lut[b] = i
        lut[b - 32] = i
    total = 0
    for c in range(len(offsets) - 1):
        s = lut[dna[int(offsets[c]):int(offsets[c + 1])]].astype(np.int64)
        n = len(s)
        if n < 3 * k + 3:
            continue
        b0, b1, b2 = s[:-2], s[1:-1], s[2:]
        bad_amb = (b0 | b1 | b2) >= 4
        idx_p = np.where(bad_amb, 0, b0 * 16 + b1 * 4 + b2)
        idx_m = np.where(bad_amb, 0, (b2 ^ 2) * 16 + (b1 ^ 2) * 4 + (b0 ^ 2))
        bad_p = bad_amb | (code[idx_p] == ord("*"))
        bad_m = bad_amb | (code[idx_m] == ord("*"))
        m = len(bad_p)  # codon starts 0 .. n-3
        for bad, lo, hi in ((bad_p, 0, n - 3 * k - 3), (bad_m, 3, n - 3 * k)):
            w = np.zeros(m - 3 * (k - 1), bool)
            for j in range(k):
                w |= bad[3 * j:3 * j + len(w)]
            x = np.arange(len(w))
            total += int((~w & (x >= lo) & (x <= hi)).sum())
    return total
