"""ORACLE twin (test infrastructure only): a pure-Python restatement of the reference path.

Written independently of oracle/kma_oracle.c to cross-check it: Python ``str`` / ``dict`` /
``set`` stand in for Java ``String`` / ``HashMap`` / ``HashSet``, and the genetic code is built
from an amino-acid -> codons listing rather than the NCBI 64-character strings the C oracle
uses. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.
Use it on small inputs only (pure-Python loops).

Citations are relative to /root/reference/src/main/java/org/theseed/.
Parity status: see oracle/kma_oracle.c (6-frame + peg extraction pinned by AppTest
properties on small.gto; the apply vote and ProteinKmers semantics are parity unpinned).
"""

from __future__ import annotations

STATUS_NONE, STATUS_CALLED, STATUS_AMBIGUOUS, STATUS_BELOW_MIN = 0, 1, 2, 3

# Standard code by amino acid (NCBI table 1 / 11).
_STANDARD = {
    "A": "GCT GCC GCA GCG", "R": "CGT CGC CGA CGG AGA AGG", "N": "AAT AAC",
    "D": "GAT GAC", "C": "TGT TGC", "Q": "CAA CAG", "E": "GAA GAG",
    "G": "GGT GGC GGA GGG", "H": "CAT CAC", "I": "ATT ATC ATA", "L": "TTA TTG CTT CTC CTA CTG",
    "K": "AAA AAG", "M": "ATG", "F": "TTT TTC", "P": "CCT CCC CCA CCG",
    "S": "TCT TCC TCA TCG AGT AGC", "T": "ACT ACC ACA ACG", "W": "TGG", "Y": "TAT TAC",
    "V": "GTT GTC GTA GTG", "*": "TAA TAG TGA",
}
_DIFFS = {1: {}, 11: {}, 4: {"TGA": "W"}, 25: {"TGA": "G"}}


def codon_table(gcode: int) -> dict:
    if gcode not in _DIFFS:
        raise ValueError(f"genetic code {gcode} not in the Python twin")
    tab = {c: aa for aa, cs in _STANDARD.items() for c in cs.split()}
    tab.update(_DIFFS[gcode])
    return tab


def translate(dna: str, frame: int, gcode: int) -> str:
    """DnaTranslator.translate(seq, frame, len(seq)) (external; KmerReference.java:184)."""
    tab = codon_table(gcode)
    up = dna.upper().replace("U", "T")
    return "".join(tab.get(up[p:p + 3], "X") for p in range(frame - 1, len(up) - 2, 3))


def reverse_complement(dna: str) -> str:
    """Contig.getRSequence (external; KmerReference.java:166). U pairs like T (U -> A), as
    translate reads U as T: a documented choice, parity unpinned for U."""
    comp = {"a": "t", "c": "g", "g": "c", "t": "a", "A": "T", "C": "G", "G": "C", "T": "A",
            "u": "a", "U": "A"}
    return "".join(comp.get(c, "n") for c in reversed(dna))


def protein_kmers(prot: str, k: int = 8, end_exclusive: bool = False, multiset: bool = False):
    """ProteinKmers(String) (external; ApplyKmerProcessor.java:123), UNVERIFIED semantics:
    distinct substrings prot[i:i+k] for i in 0..len-k (inclusive unless end_exclusive)."""
    n = len(prot) - k + (0 if end_exclusive else 1)
    wins = [prot[i:i + k] for i in range(max(n, 0))]
    return wins if multiset else list(dict.fromkeys(wins))


def load_table(rows):
    """ApplyKmerProcessor.java:101-107: HashMap.put per row, the last row wins."""
    table = {}
    for kmer, role in rows:
        table[kmer] = role
    return table


def apply_protein(table: dict, prot: str, min_hits: int = 5, k: int = 8,
                  end_exclusive: bool = False, multiset: bool = False):
    """ApplyKmerProcessor.java:122-147 -> (status, role or None, count)."""
    role, count, bad = None, 0, False
    for kmer in protein_kmers(prot, k, end_exclusive, multiset):
        possible = table.get(kmer)
        if possible is None:
            continue
        if role is None:
            role, count = possible, 1
        elif possible == role:
            count += 1
        else:
            bad = True
            break
    if role is None:
        return STATUS_NONE, None, 0
    if bad:
        return STATUS_AMBIGUOUS, None, 0
    return (STATUS_CALLED if count >= min_hits else STATUS_BELOW_MIN), role, count


def contig_kmers(contigs, gcode: int = 11, k: int = 8):
    """KmerReference.getContigKmers / processKmers (KmerReference.java:157-203) with
    KmerPosition.calcLeft (KmerPosition.java:60-62, 78-86). Yields
    (kmer, contig_index, left, strand, frame) in the reference's visiting order."""
    for ci, seq in enumerate(contigs):
        n = len(seq)
        for strand, s in (("+", seq), ("-", reverse_complement(seq))):
            base = n - 3 * k + 2
            for frame in (1, 2, 3):
                prot = translate(s, frame, gcode)
                for i in range(len(prot) - k):
                    km = prot[i:i + k]
                    if "*" in km or "X" in km:
                        continue
                    left = i * 3 + frame if strand == "+" else base - (i * 3 + frame)
                    yield km, ci, left, strand, frame


def annotate_contigs(table: dict, contigs, gcode: int = 11, k: int = 8):
    """Every 6-frame window probed in the table; hits sorted (contig, left, '+' first)."""
    hits = [(ci, left, strand, frame, table[km])
            for km, ci, left, strand, frame in contig_kmers(contigs, gcode, k) if km in table]
    hits.sort(key=lambda h: (h[0], h[1], h[2]))
    return hits


def peg_kmers(prots, k: int = 8):
    """KmerReference.countPegKmers (KmerReference.java:124-147): windows i < len-k, no 'X'."""
    for pi, p in enumerate(prots):
        for i in range(len(p) - k):
            km = p[i:i + k]
            if "X" not in km:
                yield km, pi, i + 1


def peg_connect(prots, contigs, gcode: int = 11, k: int = 8, strict: bool = False):
    """KmerProcessor.java:195-207: singleton peg kmers (CountMap.getSingletons of
    countPegKmers) joined with the contig kmer map (KmerFactory STRICT drops kmers with more
    than one location); every location of a singleton is connected to its peg. Returns
    (contig, left, strand, frame, peg) sorted (contig, left, '+' first)."""
    count, first = {}, {}
    for km, pi, _ in peg_kmers(prots, k):
        count[km] = count.get(km, 0) + 1
        first.setdefault(km, pi)
    singles = {km: first[km] for km, c in count.items() if c == 1}
    locs = {}
    for km, ci, left, strand, frame in contig_kmers(contigs, gcode, k):
        locs.setdefault(km, []).append((ci, left, strand, frame))
    if strict:
        locs = {km: v for km, v in locs.items() if len(v) == 1}
    out = [(ci, left, strand, frame, singles[km])
           for km, v in locs.items() if km in singles for ci, left, strand, frame in v]
    out.sort(key=lambda h: (h[0], h[1], h[2]))
    return out


class RoleCounter:
    """kmers/RoleCounter.java:14-78, literally: the role first associated with a kmer, and the
    counts of hits in that role (good) and in any other (bad); good iff no bad hit."""

    def __init__(self, role_id):
        self.role_id = role_id      # RoleCounter(String roleId)  :31-35
        self.good_count = 0
        self.bad_count = 0

    def count(self, role_hit) -> bool:  # :43-50
        ret = self.role_id == role_hit
        if ret:
            self.good_count += 1
        else:
            self.bad_count += 1
        return ret

    def is_good(self) -> bool:  # :55-57
        return self.bad_count == 0


def build_signatures(prots, roles, k: int = 8, end_exclusive: bool = False):
    """BuildKmerProcessor.java:137-223 + RoleCounter: roles[i] >= 0 = the single good role of
    an interesting peg, -1 = a buffered protein, other = skipped. Returns {kmer: role}."""
    counters = {}
    for p, r in zip(prots, roles):
        if r < 0:
            continue
        for km in protein_kmers(p, k, end_exclusive, False):
            # kmerMap.computeIfAbsent(kmer, k -> new RoleCounter(role)).count(role)  :165-175
            counters.setdefault(km, RoleCounter(r)).count(r)
    # kmerMap.values().removeIf(x -> ! x.isGood())  :182-190
    keep = {km: c.role_id for km, c in counters.items() if c.is_good()}
    for p, r in zip(prots, roles):
        if r == -1:
            for km in protein_kmers(p, k, end_exclusive, False):
                keep.pop(km, None)
    return keep


def distance(a: str, b: str, k: int = 8, end_exclusive: bool = False) -> float:
    """ProteinKmers(a).distance(ProteinKmers(b)) (external SequenceKmers.distance, restated;
    GeneCopyProcessor.java:137-142): Jaccard distance of the kmer sets, 1.0 if disjoint."""
    sa = set(protein_kmers(a, k, end_exclusive))
    sb = set(protein_kmers(b, k, end_exclusive))
    sim = len(sa & sb)
    return 1.0 - sim / (len(sa) + len(sb) - sim) if sim else 1.0


def best_match(query: str, cands, max_dist: float, k: int = 8):
    """GeneCopyProcessor.java:135-146: (index of the last candidate with distance <= the
    running best starting at max_dist, or -1; that distance)."""
    best, found = max_dist, -1
    for i, c in enumerate(cands):
        d = distance(query, c, k)
        if d <= best:
            best, found = d, i
    return found, best



def frame_of(strand: str, left: int, k: int = 8) -> int:
    """Location.getFrame restated: strand and phase of the end point ('-' 0..2, '+' 3..5)."""
    end = left + 3 * k - 1 if strand == "+" else left
    return (3 if strand == "+" else 0) + end % 3


def propose(connections, peg_len, k: int = 8, min_strength: float = 0.5, max_fuzz: float = 1.5,
            min_fuzz: float = 0.8):
    """KmerProcessor.java:209-264 over FramedLocationLists (:156-171): connections are
    (contig, left, strand, peg); returns (proposals [(peg, contig, strand, left, right,
    evidence, frame)], [lists, too_few, too_short, proposals])."""
    framer = {}
    for ct, lf, sd, pg in connections:
        framer.setdefault((frame_of(sd, lf, k), pg), []).append((ct, lf))
    span = 3 * k - 1
    real = min_strength / 3
    out, stats = [], [0, 0, 0, 0]
    for (fr, pg) in sorted(framer):
        lst = sorted(framer[(fr, pg)])
        peg_bp = peg_len[pg] * 3
        max_len, min_len = int(peg_bp * max_fuzz + 1), int(peg_bp * min_fuzz)
        min_kmers = int(peg_bp * real)
        stats[0] += 1
        if min_kmers > len(lst):
            stats[1] += 1
            continue
        strand = "+" if fr >= 3 else "-"
        for i in range(min(len(lst) - min_kmers + 1, len(lst))):
            ct, lf = lst[i]
            evidence, best = 1, lf + span
            for ct2, lf2 in lst[i + 1:]:
                if ct2 != ct:
                    break
                if lf2 + span < lf + max_len:
                    evidence += 1
                    best = max(best, lf2 + span)
            if best < lf + min_len:
                stats[2] += 1
            else:
                out.append((pg, ct, strand, lf, best, evidence, fr))
                stats[3] += 1
    return out, stats


def hash_annotate(genome_prots, protos, k: int = 8, min_sim: float = 0.0125):
    """GenomeProteinKmers restated (HashAnnotationProcessor.java:233-306): per genome protein
    the first prototype reaching the best similarity >= min_sim (-1 / 0.0 if none), and the
    matches of every prototype."""
    gsets = [{p[i:i + k] for i in range(len(p) - k + 1)} for p in genome_prots]
    best, sim, counts = [-1] * len(genome_prots), [0.0] * len(genome_prots), []
    for pi, pr in enumerate(protos):
        a = {pr[i:i + k] for i in range(len(pr) - k + 1)}
        m = 0
        for gi, b in enumerate(gsets):
            shared = len(a & b)
            if not shared:
                continue
            s = shared / (len(a) + len(b) - shared)
            if s >= min_sim:
                m += 1
                if s > sim[gi]:
                    sim[gi], best[gi] = s, pi
        counts.append(m)
    return best, sim, counts
