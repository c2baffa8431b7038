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
  - PegProposalList is the reference's literally: a java.util.TreeSet ordered by
    PegProposal.compareTo (PegProposal.java:85-98: contig id, then "equal" when end and strand
    match, else left edge, then shorter first). That comparator is not consistent with equals
    (same left and length on the other strand compare equal; two proposals with one end can
    sit apart when the search path misses one), so which proposals survive depends on the
    tree's shape: _TreeSet restates java.util.TreeMap's red-black put (search, attach,
    fixAfterInsertion with its rotations) so the shape, the equal-key found by add, and the
    in-order iteration are Java's for the same insertion order. merge() moves the kept
    proposal's begin in place (Location.setBegin), as in Java. oracle/proposal_list.py is the
    independent restatement the tests compare with.
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
    contig_id: str = ""  # Location.getContigId (compareTo orders contigs by it)

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
        return Location(loc.contig, "+", start + 1, stop_end + 1, loc.contig_id)
    return Location(loc.contig, "-", n - stop_end, n - start, loc.contig_id)


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

    def compare_to(self, other: "PegProposal") -> int:  # PegProposal.compareTo :85-98
        a, b = self.loc, other.loc
        r = (a.contig_id > b.contig_id) - (a.contig_id < b.contig_id)  # String.compareTo sign
        if r == 0 and (a.end != b.end or a.strand != b.strand):
            r = a.left - b.left
            if r == 0:
                r = a.length - b.length  # shorter locations go first
        return r


class _Node:
    __slots__ = ("key", "left", "right", "parent", "black")

    def __init__(self, key, parent):
        self.key, self.parent = key, parent
        self.left = self.right = None
        self.black = True  # new entries are BLACK until fixAfterInsertion colours them


class _TreeSet:
    """java.util.TreeSet over java.util.TreeMap (red-black, CLR), restated for add() and
    iteration: add returns (True, new) or (False, the entry that compared equal on the search
    path) — the one tailSet(x).first() then returns, since the tree has not changed."""

    def __init__(self, cmp):
        self.cmp, self.root, self.size = cmp, None, 0

    def add(self, key):
        t = self.root
        if t is None:  # addEntryToEmptyMap
            self.root = _Node(key, None)
            self.size = 1
            return True, key
        while True:
            parent = t
            c = self.cmp(key, t.key)
            if c < 0:
                t = t.left
            elif c > 0:
                t = t.right
            else:
                return False, t.key  # the map keeps the old key
            if t is None:
                break
        e = _Node(key, parent)
        if c < 0:
            parent.left = e
        else:
            parent.right = e
        self._fix_after_insertion(e)
        self.size += 1
        return True, key

    @staticmethod
    def _black(x):
        return x is None or x.black

    def _rotate_left(self, p):
        r = p.right
        p.right = r.left
        if r.left is not None:
            r.left.parent = p
        r.parent = p.parent
        if p.parent is None:
            self.root = r
        elif p.parent.left is p:
            p.parent.left = r
        else:
            p.parent.right = r
        r.left, p.parent = p, r

    def _rotate_right(self, p):
        lft = p.left
        p.left = lft.right
        if lft.right is not None:
            lft.right.parent = p
        lft.parent = p.parent
        if p.parent is None:
            self.root = lft
        elif p.parent.right is p:
            p.parent.right = lft
        else:
            p.parent.left = lft
        lft.right, p.parent = p, lft

    def _fix_after_insertion(self, x):
        x.black = False
        while x is not None and x is not self.root and not x.parent.black:
            p = x.parent
            g = p.parent
            if p is (g.left if g else None):
                y = g.right if g else None
                if not self._black(y):
                    p.black, y.black, g.black = True, True, False
                    x = g
                else:
                    if x is p.right:
                        x = p
                        self._rotate_left(x)
                    x.parent.black = True
                    gg = x.parent.parent
                    if gg is not None:
                        gg.black = False
                        self._rotate_right(gg)
            else:
                y = g.left if g else None
                if not self._black(y):
                    p.black, y.black = True, True
                    if g is not None:
                        g.black = False
                    x = g
                else:
                    if x is p.left:
                        x = p
                        self._rotate_right(x)
                    x.parent.black = True
                    gg = x.parent.parent
                    if gg is not None:
                        gg.black = False
                        self._rotate_left(gg)
        self.root.black = True

    def __iter__(self):  # in order (successor walk)
        stack, n = [], self.root
        while stack or n is not None:
            while n is not None:
                stack.append(n)
                n = n.left
            n = stack.pop()
            yield n.key
            n = n.right

    def __len__(self):
        return self.size


class PegProposalList:
    """locations/PegProposalList.java:67-93: the TreeSet of proposals (see module docstring)."""

    def __init__(self, contigs: list[str], min_strength: float, min_evidence: int,
                 gcode: int = 11):
        self.contigs, self.min_strength, self.min_evidence = contigs, min_strength, min_evidence
        self.gcode = gcode
        self.made = self.rejected = self.weak = self.small = self.merged = 0
        self._set = _TreeSet(lambda a, b: a.compare_to(b))

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
        added, old = self._set.add(new)
        if added:
            return new
        if new.better_than(old):  # the duplicate: tailSet(new).first()
            old.merge(new)
            self.merged += 1
            return old
        return None

    def __iter__(self):  # the TreeSet's order
        return iter(self._set)

    def __len__(self):
        return len(self._set)


def annotate_proposals(proposals, functions: list[str], contigs: list[str], genome_id: str,
                       contig_ids: list[str], min_strength: float = 0.5, min_evidence: int = 10,
                       gcode: int = 11):
    """KmerProcessor.annotateGenome's tail (:250-284): the sweep's proposals (PROPOSAL_DTYPE, in
    list order; peg index -> functions[peg]) through PegProposalList with the DNA strength
    min_strength / 3 (:170), then makeFeature (:295-312): [(fid, function, Location, evidence,
    strength)] in the list's order. contig_ids: the genome's contig ids, in contig-index order
    (required: PegProposal.compareTo orders by Location.getContigId, so the TreeSet's order and
    the fig|...peg.N numbering depend on them)."""
    ids = list(contig_ids)
    if len(ids) != len(contigs):
        raise ValueError(f"{len(ids)} contig ids for {len(contigs)} contigs")
    plist = PegProposalList(contigs, min_strength / 3, min_evidence, gcode)
    for p in proposals:
        c = int(p["contig"])
        loc = Location(c, chr(p["strand"]), int(p["left"]), int(p["right"]), ids[c])
        plist.propose(loc, functions[int(p["peg"])], int(p["evidence"]))
    return [(f"fig|{genome_id}.peg.{i}", p.function, p.loc, p.evidence, p.strength)
            for i, p in enumerate(plist, start=1)], plist
