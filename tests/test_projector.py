"""§8(f)2 host stage above the GPU sweep (kmeranno/projector.py: PegProposalList,
Location.extend restated, makeFeature), on the reference's own fixture small.gto projected onto
itself (a 5%-mutated copy of its pegs as the close genome). The proposals come from the C
oracle's join + sweep (the GPU path is bit-exact to it: tests/test_gpu_proposals.py), so this
runs without a GPU. Parity unpinned (external semantics): checked by properties — every feature
is a whole ORF (start codon .. in-frame stop, no internal stop) and the projected features land
on small.gto's own gene ends."""
import numpy as np

from kmeranno import projector

K = 8
_STOP = {"TAA", "TAG", "TGA"}


def _orf_ok(seq):
    cod = [seq[i:i + 3] for i in range(0, len(seq), 3)]
    return (len(seq) % 3 == 0 and cod[0] in ("ATG", "GTG", "TTG") and cod[-1] in _STOP
            and not any(c in _STOP for c in cod[:-1]))


def test_projection_of_small_gto_onto_itself(oracle_c, small_gto):
    rng = np.random.default_rng(9)
    pegs = [f for f in small_gto["features"] if f.get("protein_translation")]
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    close = []
    for f in pegs:
        b = np.frombuffer(f["protein_translation"].encode(), np.uint8).copy()
        m = rng.random(len(b)) < 0.05
        b[m] = aa[rng.integers(0, 20, int(m.sum()))]
        close.append(b.tobytes().decode())
    res, off = oracle_c.pack_strings(close)
    contigs = [c["dna"] for c in small_gto["contigs"]]
    dna, doff = oracle_c.pack_strings(contigs)
    ct, lf, sd, fr, pg = oracle_c.peg_connect(res, off, dna, doff, 11, K, False)
    prop, stats = oracle_c.propose(ct, lf, sd, pg, np.array([len(p) for p in close]), K)
    arr = np.zeros(len(prop["peg"]), [("peg", "<u4"), ("contig", "<u4"), ("left", "<i4"),
                                      ("right", "<i4"), ("evidence", "<u4"), ("strand", "u1"),
                                      ("frame", "u1"), ("pad", "<u2")])
    for key in ("peg", "contig", "left", "right", "evidence", "strand", "frame"):
        arr[key] = prop[key]
    funcs = [f.get("function", "") for f in pegs]
    feats, plist = projector.annotate_proposals(arr, funcs, contigs, small_gto["id"],
                                                [c["id"] for c in small_gto["contigs"]])
    assert plist.made == len(arr) and len(feats) == len(plist) > 0.6 * len(pegs)
    assert plist.rejected + plist.weak + plist.small + len(plist) + plist.merged <= plist.made + len(plist)
    comp = str.maketrans("ACGTacgt", "TGCAtgca")
    for fid, func, loc, ev, strength in feats:
        s = contigs[loc.contig][loc.left - 1:loc.right].upper()
        if loc.strand == "-":
            s = s.translate(comp)[::-1]
        assert _orf_ok(s), (fid, loc)
        assert strength >= 0.5 / 3 and ev >= 10
    # the genome's own genes: (contig, strand, stop end) of every peg
    cid = {c["id"]: i for i, c in enumerate(small_gto["contigs"])}
    ends = set()
    for f in pegs:
        c, beg, strand, ln = f["location"][0]
        beg = int(beg)
        ends.add((cid[c], strand, beg + ln - 1 if strand == "+" else beg - ln + 1))
    hit = sum((loc.contig, loc.strand, loc.end) in ends for _, _, loc, _, _ in feats)
    assert hit >= 0.95 * len(feats), (hit, len(feats))
    assert [f[0] for f in feats[:2]] == [f"fig|{small_gto['id']}.peg.1",
                                         f"fig|{small_gto['id']}.peg.2"]


class _Int:
    """A Comparable for the tree tests (compareTo = integer order, or a coarse key)."""

    def __init__(self, v, coarse=1):
        self.v, self.coarse = v, coarse

    def compare_to(self, o):
        a, b = self.v // self.coarse, o.v // o.coarse
        return (a > b) - (a < b)


def _rb_ok(t):
    """Red-black invariants of the oracle tree: BST order, no red-red, equal black heights."""
    def walk(n):
        if n < 0:
            return 1
        for ch in (t.l[n], t.r[n]):
            if ch >= 0:
                assert t.p[ch] == n
                assert not (t.c[n] == 0 and t.c[ch] == 0), "red-red"
        hl, hr = walk(t.l[n]), walk(t.r[n])
        assert hl == hr
        return hl + (t.c[n] == 1)
    assert t.root < 0 or t.c[t.root] == 1
    walk(t.root)


def test_java_treeset_restatements_agree():
    """projector._TreeSet and oracle/proposal_list.JavaTreeSet (two restatements of
    java.util.TreeMap's put / fixAfterInsertion) build the same trees: same add results,
    same in-order keys, same root; the oracle's is a valid red-black tree."""
    from oracle.proposal_list import JavaTreeSet
    rng = np.random.default_rng(4)
    for trial in range(30):
        n = int(rng.integers(1, 400))
        vals = rng.integers(0, 300, n) if trial % 3 else np.arange(n)  # ascending: rotations
        coarse = 1 if trial % 2 else 3
        a, b = projector._TreeSet(lambda x, y: x.compare_to(y)), JavaTreeSet()
        for v in vals.tolist():
            added_a, _ = a.add(_Int(v, coarse))
            assert added_a == b.add(_Int(v, coarse))
        assert [x.v for x in a] == [x.v for x in b.in_order()]
        assert a.root.key.v == b.key[b.root].v
        _rb_ok(b)
        assert len(a) == len(b.key)


def _oracle_features(props, funcs, contigs, ids, min_strength=0.5, min_evidence=10):
    from oracle.proposal_list import Loc, ProposalList
    plist = ProposalList(dict(zip(ids, contigs)), min_strength / 3, min_evidence)
    for p in props:
        c = int(p["contig"])
        plist.propose(Loc(ids[c], chr(p["strand"]), int(p["left"]), int(p["right"])),
                      funcs[int(p["peg"])], int(p["evidence"]))
    return [(q.function, q.loc.contig_id, q.loc.dir, q.loc.left, q.loc.right, q.evidence)
            for q in plist], plist


def test_proposal_list_is_the_java_treeset():
    """PegProposalList.java:67-93 literally, on proposals built to hit the comparator's
    quirks: two ORFs with the same left edge and length on opposite strands compare equal
    (the second is a duplicate, merged if better); proposals with one end but different
    starts arrive in an order that separates them in the tree. projector.PegProposalList and
    the oracle agree on every kept proposal, its order and the counters."""
    rng = np.random.default_rng(12)
    orf = "ATG" + "".join(rng.choice(["GCT", "AAA", "CTG", "GAT"], 60)) + "TAA"
    contig = ("CCC" + orf + "CC" + "TTA" + "GGG" * 10 + orf[::-1].translate(
        str.maketrans("ACGT", "TGCA")) + "GG") * 3
    ids = ["c1"]
    props = []
    L = len(orf)
    for rep in range(3):
        base = rep * (len(contig) // 3)
        for shift in (0, 30, 60, 9, 90):  # one stop end, several starts inside the ORF
            props.append((0, "+", base + 4 + shift, base + 4 + shift + 23, 50 + (shift * 7) % 11))
        mleft = base + 4 + L + 2 + 3 + 30
        for shift in (0, 30, 60):
            props.append((0, "-", mleft + L - 24 - shift, mleft + L - 1 - shift, 45 + shift % 13))
    arr = np.zeros(len(props), [("peg", "<u4"), ("contig", "<u4"), ("left", "<i4"),
                                ("right", "<i4"), ("evidence", "<u4"), ("strand", "u1"),
                                ("frame", "u1"), ("pad", "<u2")])
    for i, (c, s, lft, rgt, ev) in enumerate(props):
        arr[i] = (i % 4, c, lft, rgt, ev, ord(s), 0, 0)
    funcs = [f"F{i}" for i in range(4)]
    feats, plist = projector.annotate_proposals(arr, funcs, [contig], "g", ids,
                                                min_evidence=10)
    exp, oplist = _oracle_features(arr, funcs, [contig], ids)
    got = [(f[1], ids[f[2].contig], f[2].strand, f[2].left, f[2].right, f[3]) for f in feats]
    assert got == exp and len(got) > 2
    assert (plist.made, plist.rejected, plist.weak, plist.small, plist.merged) == \
        (oplist.made, oplist.rejected, oplist.weak, oplist.small, oplist.merged)
    assert plist.merged > 0


def test_projection_of_small_gto_vs_oracle_list(oracle_c, small_gto):
    """small.gto projected onto itself (the join + sweep of the C oracle, in canonical
    insertion order) through projector.annotate_proposals and through the oracle's literal
    PegProposalList: the same features in the same order (makeFeature numbering), with the
    contigs' own ids ordering the TreeSet."""
    rng = np.random.default_rng(9)
    pegs = [f for f in small_gto["features"] if f.get("protein_translation")]
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    close = []
    for f in pegs:
        b = np.frombuffer(f["protein_translation"].encode(), np.uint8).copy()
        m = rng.random(len(b)) < 0.05
        b[m] = aa[rng.integers(0, 20, int(m.sum()))]
        close.append(b.tobytes().decode())
    res, off = oracle_c.pack_strings(close)
    contigs = [c["dna"] for c in small_gto["contigs"]]
    ids = [c["id"] for c in small_gto["contigs"]]
    dna, doff = oracle_c.pack_strings(contigs)
    ct, lf, sd, fr, pg = oracle_c.peg_connect(res, off, dna, doff, 11, K, False)
    prop, _ = oracle_c.propose(ct, lf, sd, pg, np.array([len(p) for p in close]), K)
    arr = np.zeros(len(prop["peg"]), [("peg", "<u4"), ("contig", "<u4"), ("left", "<i4"),
                                      ("right", "<i4"), ("evidence", "<u4"), ("strand", "u1"),
                                      ("frame", "u1"), ("pad", "<u2")])
    for key in ("peg", "contig", "left", "right", "evidence", "strand", "frame"):
        arr[key] = prop[key]
    funcs = [f.get("function", "") for f in pegs]
    feats, plist = projector.annotate_proposals(arr, funcs, contigs, small_gto["id"],
                                                contig_ids=ids)
    exp, oplist = _oracle_features(arr, funcs, contigs, ids)
    got = [(f[1], ids[f[2].contig], f[2].strand, f[2].left, f[2].right, f[3]) for f in feats]
    assert len(got) > 400 and got == exp
    assert (plist.made, plist.rejected, plist.merged) == (oplist.made, oplist.rejected,
                                                          oplist.merged)


def test_proposal_order_follows_contig_ids_not_indices():
    """PegProposal.compareTo orders by Location.getContigId: the same proposals on two contigs
    whose ids sort against their index order ("zeta" is contig 0, "alpha" contig 1) come out
    with contig 1's first, numbered fig|g.peg.1.., exactly as the oracle's literal TreeSet
    orders them; swapping the ids swaps the order."""
    rng = np.random.default_rng(5)
    orf = "ATG" + "".join(rng.choice(["GCT", "AAA", "CTG", "GAT"], 60)) + "TAA"
    contig = "CCC" + orf + "CCCGGG" + orf + "CC"
    props = []
    for c in (0, 1):
        for start in (4, 4 + len(orf) + 6):  # 1-based ORF starts (in frame)
            for shift in (0, 30, 60):
                props.append((c, "+", start + shift, start + shift + 23, 50 + 3 * c + shift % 7))
    arr = np.zeros(len(props), [("peg", "<u4"), ("contig", "<u4"), ("left", "<i4"),
                                ("right", "<i4"), ("evidence", "<u4"), ("strand", "u1"),
                                ("frame", "u1"), ("pad", "<u2")])
    for i, (c, st, lft, rgt, ev) in enumerate(props):
        arr[i] = (i % 3, c, lft, rgt, ev, ord(st), 0, 0)
    funcs = ["F0", "F1", "F2"]
    orders = []
    for ids in (["zeta", "alpha"], ["alpha", "zeta"]):
        feats, _ = projector.annotate_proposals(arr, funcs, [contig, contig], "g", ids,
                                                min_evidence=10)
        exp, _ = _oracle_features(arr, funcs, [contig, contig], ids)
        got = [(f[1], ids[f[2].contig], f[2].strand, f[2].left, f[2].right, f[3]) for f in feats]
        assert got == exp and len(got) >= 4
        orders.append([ids[f[2].contig] for f in feats])
        assert orders[-1] == sorted(orders[-1])  # contig-id order, whatever the index
    assert orders[0][0] == "alpha" and [f[2].contig for f in feats][0] == 0
