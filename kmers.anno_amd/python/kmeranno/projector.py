"""Host side of the projector's proposal stage (§8(f)2) above kma_propose_pegs.

The GPU computes the proposal sweep of KmerProcessor.annotateGenome
(KmerProcessor.java:209-264, kmeranno.propose_pegs). What consumes it in the reference lives
in org.theseed.locations and the external shared library:
  PegProposalList.propose (locations/PegProposalList.java:67-93): strength / evidence filters and
      one proposal per ORF, the better one kept (PegProposal.betterThan / merge,
      locations/PegProposal.java:63-67,142-156);
  PegProposal.create -> Location.extend(genome) (EXTERNAL: restated below);
  KmerProcessor.makeFeature (:295-312): fig|<genome>.peg.<n> features in list order.
Parity for these is UNPINNED (no reference test exercises them, the external sources are not
available). Restated choices, documented:
  - extend: the ORF in the proposal's frame; the right end moves to the first in-frame stop
    codon at or after the proposal's last codon (included), the left end to the start codon
    (ATG, GTG, TTG) farthest upstream before the previous in-frame stop; no stop before the
    contig end, or no start, gives no proposal (PegProposal.create returns null). '-' strand
    mirrored on the reverse complement. Ambiguous bases never form start or stop codons.
  - PegProposalList keeps one proposal per (contig, strand, end) — the intent of
    PegProposal.equals / hashCode; the Java TreeSet's comparator is inconsistent with equals,
    so its exact tie behaviour depends on tree shape and is not reproduced.
"""
from __future__ import annotations

from dataclasses import dataclass

_STOPS = {11: {"TAA", "TAG", "TGA"}, 1: {"TAA", "TAG", "TGA"}, 4: {"TAA", "TAG"}}
_STARTS = {"ATG", "GTG", "TTG"}
_COMP = str.maketrans("ACGTacgt", "TGCAtgca")


def _revcomp(s: str) -> str:
    return s.translate(_COMP)[::-1]


@dataclass
class Location:
    contig: int
    strand: str
    left: int   # 1-based, inclusive
    right: int

    @property
    def length(self) -> int:
        return self.right - self.left + 1

    @property
    def end(self) -> int:
        return self.right if self.strand == "+" else self.left

    @property
    def begin(self) -> int:
        return self.left if self.strand == "+" else self.right


def extend(dna: str, loc: Location, gcode: int = 11) -> Location | None:
    """Location.extend restated (see module docstring); dna is the contig sequence."""
    stops = _STOPS.get(gcode, _STOPS[11])
    n = len(dna)
    if loc.strand == "+":
        seq, a, b = dna.upper(), loc.left - 1, loc.right - 1  # 0-based codon-aligned span
    else:
        seq, a, b = _revcomp(dna.upper()), n - loc.right, n - loc.left
    if a < 0 or b >= n:
        return None
    last = a + ((b - a + 1) // 3 - 1) * 3  # last whole codon of the span
    p = last
    while p + 3 <= n and seq[p:p + 3] not in stops:
        p += 3
    if p + 3 > n:
        return None  # ran off the contig: no stop
    stop_end = p + 2
    q, start = a, -1
    while q >= 0 and seq[q:q + 3] not in stops:
        if seq[q:q + 3] in _STARTS:
            start = q
        q -= 3
    if start < 0:
        return None
    if loc.strand == "+":
        return Location(loc.contig, "+", start + 1, stop_end + 1)
    return Location(loc.contig, "-", n - stop_end, n - start)


@dataclass
class PegProposal:
    loc: Location
    function: str
    evidence: int

    @property
    def strength(self) -> float:
        return self.evidence / self.loc.length  # PegProposal.getStrength

    def better_than(self, other: "PegProposal") -> bool:  # PegProposal.betterThan :142-147
        return self.evidence > other.evidence or (
            self.evidence == other.evidence and self.loc.length > other.loc.length)

    def merge(self, other: "PegProposal"):  # PegProposal.merge :63-67
        self.function = other.function
        if self.loc.strand == "+":
            self.loc.left = other.loc.begin
        else:
            self.loc.right = other.loc.begin
        self.evidence = other.evidence


class PegProposalList:
    """locations/PegProposalList.java:67-93 (one proposal per ORF end)."""

    def __init__(self, contigs: list[str], min_strength: float, min_evidence: int,
                 gcode: int = 11):
        self.contigs, self.min_strength, self.min_evidence = contigs, min_strength, min_evidence
        self.gcode = gcode
        self.made = self.rejected = self.weak = self.small = self.merged = 0
        self._by_end: dict[tuple, PegProposal] = {}

    def propose(self, loc: Location, function: str, evidence: int) -> PegProposal | None:
        self.made += 1
        real = extend(self.contigs[loc.contig], loc, self.gcode)
        if real is None:
            self.rejected += 1
            return None
        new = PegProposal(real, function, evidence)
        if new.strength < self.min_strength:
            self.weak += 1
            return None
        if evidence < self.min_evidence:
            self.small += 1
            return None
        key = (real.contig, real.strand, real.end)
        old = self._by_end.get(key)
        if old is None:
            self._by_end[key] = new
            return new
        if new.better_than(old):
            old.merge(new)
            self.merged += 1
            return old
        return None

    def __iter__(self):  # contig order: by contig, left edge, then shorter first
        return iter(sorted(self._by_end.values(),
                           key=lambda p: (p.loc.contig, p.loc.left, p.loc.length)))

    def __len__(self):
        return len(self._by_end)


def annotate_proposals(proposals, functions: list[str], contigs: list[str], genome_id: str,
                       min_strength: float = 0.5, min_evidence: int = 10, gcode: int = 11):
    """KmerProcessor.annotateGenome's tail (:250-284): the sweep's proposals (PROPOSAL_DTYPE, in
    list order; peg index -> functions[peg]) through PegProposalList with the DNA strength
    min_strength / 3 (:170), then makeFeature (:295-312): [(fid, function, Location, evidence,
    strength)] in contig order."""
    plist = PegProposalList(contigs, min_strength / 3, min_evidence, gcode)
    for p in proposals:
        loc = Location(int(p["contig"]), chr(p["strand"]), int(p["left"]), int(p["right"]))
        plist.propose(loc, functions[int(p["peg"])], int(p["evidence"]))
    return [(f"fig|{genome_id}.peg.{i}", p.function, p.loc, p.evidence, p.strength)
            for i, p in enumerate(plist, start=1)], plist
