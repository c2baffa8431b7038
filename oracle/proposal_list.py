"""ORACLE (test infrastructure only): a literal restatement of the projector's proposal list.

  locations/PegProposalList.java:67-93   propose(): create, strength / evidence filters, TreeSet
                                          add, on a duplicate tailSet(p).first() and betterThan /
                                          merge
  locations/PegProposal.java:50-58       create(): Location.extend(genome), null -> rejected
  locations/PegProposal.java:63-67       merge(): function, loc.setBegin(other's begin), evidence
  locations/PegProposal.java:85-98       compareTo(): contig id; 0 when end and strand match;
                                          else left edge, then length
  locations/PegProposal.java:142-147     betterThan(): more evidence, then longer
  java.util.TreeMap (JDK)                put / getCeilingEntry / fixAfterInsertion / rotations /
                                          in-order iteration, restated on index arrays

Paths are relative to /root/reference/src/main/java/org/theseed/. Written apart from
kmers.anno_amd/python/kmeranno/projector.py (node objects there, parallel arrays here; the
ceiling search of tailSet(p).first() is walked here as Java walks it, not taken from add) so
that the two cross-check each other. Location and Location.extend are external
(org.theseed:shared); their semantics are restated here (SEEDtk's conventions: begin = left on
'+', right on '-'; end the other; extend = the whole ORF: in-frame stop at or after the last
codon, start codon ATG/GTG/TTG farthest upstream before the previous in-frame stop) and are
parity-unpinned. Only tests/ may import this module.
"""
from __future__ import annotations

RED, BLACK = 0, 1
_STOPS = {11: ("TAA", "TAG", "TGA"), 1: ("TAA", "TAG", "TGA"), 4: ("TAA", "TAG")}
_STARTS = ("ATG", "GTG", "TTG")


class Loc:
    """org.theseed.locations.Location (external), the parts PegProposal uses."""

    def __init__(self, contig_id: str, dir_: str, left: int, right: int):
        self.contig_id, self.dir, self.left, self.right = contig_id, dir_, left, right

    def begin(self):
        return self.left if self.dir == "+" else self.right

    def end(self):
        return self.right if self.dir == "+" else self.left

    def length(self):
        return self.right - self.left + 1

    def set_begin(self, b: int):
        if self.dir == "+":
            self.left = b
        else:
            self.right = b


def extend(seq: str, loc: Loc, gcode: int = 11):
    """Location.extend(genome) restated: a new Loc for the ORF holding loc, or None."""
    stops = _STOPS.get(gcode, _STOPS[11])
    s = seq.upper()
    n = len(s)
    comp = {"A": "T", "C": "G", "G": "C", "T": "A"}

    def codon(i):  # the codon at strand position i (0-based), read on loc's strand
        if loc.dir == "+":
            return s[i:i + 3]
        return "".join(comp.get(c, "N") for c in reversed(s[n - i - 3:n - i]))

    if loc.dir == "+":
        a, b = loc.left - 1, loc.right - 1
    else:
        a, b = n - loc.right, n - loc.left
    if a < 0 or b >= n:
        return None
    i = a + ((b - a + 1) // 3 - 1) * 3
    while i + 3 <= n and codon(i) not in stops:
        i += 3
    if i + 3 > n:
        return None
    stop_last = i + 2
    j, start = a, None
    while j >= 0:
        c = codon(j)
        if c in stops:
            break
        if c in _STARTS:
            start = j
        j -= 3
    if start is None:
        return None
    if loc.dir == "+":
        return Loc(loc.contig_id, "+", start + 1, stop_last + 1)
    return Loc(loc.contig_id, "-", n - stop_last, n - start)


class Proposal:
    def __init__(self, loc: Loc, function: str, evidence: int):
        self.loc, self.function, self.evidence = loc, function, evidence

    def strength(self) -> float:
        return self.evidence / self.loc.length()

    def better_than(self, other) -> bool:
        r = self.evidence > other.evidence
        if not r and self.evidence == other.evidence:
            r = self.loc.length() > other.loc.length()
        return r

    def merge(self, other):
        self.function = other.function
        self.loc.set_begin(other.loc.begin())
        self.evidence = other.evidence

    def compare_to(self, other) -> int:
        a, b = self.loc, other.loc
        if a.contig_id != b.contig_id:
            return -1 if a.contig_id < b.contig_id else 1
        if a.end() != b.end() or a.dir != b.dir:
            r = a.left - b.left
            return r if r != 0 else a.length() - b.length()
        return 0


class JavaTreeSet:
    """java.util.TreeSet<E extends Comparable> over parallel arrays (node i: key, left, right,
    parent, colour; -1 = null)."""

    def __init__(self):
        self.key, self.l, self.r, self.p, self.c = [], [], [], [], []
        self.root = -1

    def _new(self, key, parent):
        self.key.append(key)
        self.l.append(-1)
        self.r.append(-1)
        self.p.append(parent)
        self.c.append(BLACK)
        return len(self.key) - 1

    def _col(self, x):
        return BLACK if x < 0 else self.c[x]

    def _par(self, x):
        return -1 if x < 0 else self.p[x]

    def _lft(self, x):
        return -1 if x < 0 else self.l[x]

    def _rgt(self, x):
        return -1 if x < 0 else self.r[x]

    def _set(self, x, col):
        if x >= 0:
            self.c[x] = col

    def add(self, e) -> bool:  # TreeSet.add = TreeMap.put(e, PRESENT) == null
        t = self.root
        if t < 0:
            self.root = self._new(e, -1)
            return True
        while t >= 0:
            parent = t
            cmp = e.compare_to(self.key[t])
            if cmp < 0:
                t = self.l[t]
            elif cmp > 0:
                t = self.r[t]
            else:
                return False
        x = self._new(e, parent)
        if cmp < 0:
            self.l[parent] = x
        else:
            self.r[parent] = x
        self._fix(x)
        return True

    def ceiling(self, e):  # TreeMap.getCeilingEntry, the entry tailSet(e).first() returns
        p = self.root
        while p >= 0:
            cmp = e.compare_to(self.key[p])
            if cmp < 0:
                if self.l[p] >= 0:
                    p = self.l[p]
                else:
                    return self.key[p]
            elif cmp > 0:
                if self.r[p] >= 0:
                    p = self.r[p]
                else:
                    parent, ch = self.p[p], p
                    while parent >= 0 and ch == self.r[parent]:
                        ch, parent = parent, self.p[parent]
                    return None if parent < 0 else self.key[parent]
            else:
                return self.key[p]
        return None

    def _rot_left(self, p):
        r = self.r[p]
        self.r[p] = self.l[r]
        if self.l[r] >= 0:
            self.p[self.l[r]] = p
        self.p[r] = self.p[p]
        if self.p[p] < 0:
            self.root = r
        elif self.l[self.p[p]] == p:
            self.l[self.p[p]] = r
        else:
            self.r[self.p[p]] = r
        self.l[r] = p
        self.p[p] = r

    def _rot_right(self, p):
        q = self.l[p]
        self.l[p] = self.r[q]
        if self.r[q] >= 0:
            self.p[self.r[q]] = p
        self.p[q] = self.p[p]
        if self.p[p] < 0:
            self.root = q
        elif self.r[self.p[p]] == p:
            self.r[self.p[p]] = q
        else:
            self.l[self.p[p]] = q
        self.r[q] = p
        self.p[p] = q

    def _fix(self, x):  # TreeMap.fixAfterInsertion, with Java's null-tolerant accessors
        self.c[x] = RED
        while x >= 0 and x != self.root and self.c[self.p[x]] == RED:
            if self._par(x) == self._lft(self._par(self._par(x))):
                y = self._rgt(self._par(self._par(x)))
                if self._col(y) == RED:
                    self._set(self._par(x), BLACK)
                    self._set(y, BLACK)
                    self._set(self._par(self._par(x)), RED)
                    x = self._par(self._par(x))
                else:
                    if x == self._rgt(self._par(x)):
                        x = self._par(x)
                        self._rot_left(x)
                    self._set(self._par(x), BLACK)
                    self._set(self._par(self._par(x)), RED)
                    if self._par(self._par(x)) >= 0:
                        self._rot_right(self._par(self._par(x)))
            else:
                y = self._lft(self._par(self._par(x)))
                if self._col(y) == RED:
                    self._set(self._par(x), BLACK)
                    self._set(y, BLACK)
                    self._set(self._par(self._par(x)), RED)
                    x = self._par(self._par(x))
                else:
                    if x == self._lft(self._par(x)):
                        x = self._par(x)
                        self._rot_right(x)
                    self._set(self._par(x), BLACK)
                    self._set(self._par(self._par(x)), RED)
                    if self._par(self._par(x)) >= 0:
                        self._rot_left(self._par(self._par(x)))
        self.c[self.root] = BLACK

    def in_order(self):
        out, stack, n = [], [], self.root
        while stack or n >= 0:
            while n >= 0:
                stack.append(n)
                n = self.l[n]
            n = stack.pop()
            out.append(self.key[n])
            n = self.r[n]
        return out


class ProposalList:
    """PegProposalList(genome, minStrength, minEvidence) with its counters."""

    def __init__(self, contigs: dict, min_strength: float, min_evidence: int, gcode: int = 11):
        self.contigs, self.min_strength, self.min_evidence = contigs, min_strength, min_evidence
        self.gcode = gcode
        self.made = self.rejected = self.weak = self.small = self.merged = 0
        self.set = JavaTreeSet()

    def propose(self, loc: Loc, function: str, evidence: int):
        self.made += 1
        real = extend(self.contigs[loc.contig_id], loc, self.gcode)
        if real is None:
            self.rejected += 1
            return None
        new = Proposal(real, function, evidence)
        if new.strength() < self.min_strength:
            self.weak += 1
        elif evidence < self.min_evidence:
            self.small += 1
        elif self.set.add(new):
            return new
        else:
            old = self.set.ceiling(new)
            if new.better_than(old):
                old.merge(new)
                self.merged += 1
                return old
        return None

    def __iter__(self):
        return iter(self.set.in_order())
