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
    feats, plist = projector.annotate_proposals(arr, funcs, contigs, small_gto["id"])
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
