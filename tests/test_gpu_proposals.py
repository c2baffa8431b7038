"""§8(f)2, the projector's proposal sweep (KmerProcessor.java:209-264 over FramedLocationLists,
FramedLocationLists.java:156-171) on the GPU (kma_propose_pegs) against the C oracle
(orc_propose) and its Python twin, on the peg join of small.gto (the reference's own fixture)
and on synthetic connection sets; bit-exact proposals (peg, contig, strand, left, right,
evidence, frame) in list order, and the sweep's counters. Location / Frame / SortedLocationList
are external to the reference: their restated semantics (oracle/kma_oracle.c) are parity
unpinned."""
import numpy as np
import pytest

from oracle import oracle_py

pytestmark = pytest.mark.gpu
K = 8
FIELDS = ("peg", "contig", "strand", "left", "right", "evidence", "frame")


@pytest.fixture(scope="module")
def kma(native_lib):
    import kmeranno
    assert kmeranno.device_count() >= 1
    return kmeranno


@pytest.fixture(scope="module")
def joined(kma, oracle_c, small_gto):
    """small.gto's pegs mutated 5% as the close genome, projected onto small.gto's contigs:
    (AGGRESSIVE hits, STRICT hits, peg protein lengths)."""
    rng = np.random.default_rng(9)
    prots = [f["protein_translation"] for f in small_gto["features"]
             if f.get("protein_translation")]
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    close = []
    for p in prots:
        b = np.frombuffer(p.encode(), np.uint8).copy()
        m = rng.random(len(b)) < 0.05
        b[m] = aa[rng.integers(0, 20, int(m.sum()))]
        close.append(b.tobytes().decode())
    res, off = oracle_c.pack_strings(close)
    dna, doff = oracle_c.pack_strings([c["dna"] for c in small_gto["contigs"]])
    t, _ = kma.SignatureTable.from_pegs(res, off, K)
    with t:
        agg = kma.connect_pegs(t, dna, doff, 11, False)
        strict = kma.connect_pegs(t, dna, doff, 11, True)
    return agg, strict, np.array([len(p) for p in close], np.uint32)


def _check(kma, oracle_c, hits, peg_len, **kw):
    got, gst = kma.propose_pegs(hits, peg_len, K, **kw)
    exp, est = oracle_c.propose(hits["contig"], hits["left"], hits["strand"], hits["fid"],
                                peg_len, K, **kw)
    assert (gst == est).all(), (gst, est)
    assert len(got) == len(exp["peg"])
    for f in FIELDS:
        assert (got[f] == exp[f]).all(), f
    return got, gst


@pytest.mark.parametrize("params", [dict(), dict(min_strength=0.2),
                                    dict(min_strength=0.05, max_fuzz=2.5, min_fuzz=0.3)],
                         ids=["defaults", "strength0.2", "loose"])
@pytest.mark.parametrize("strict", [False, True])
def test_proposals_small_gto_vs_oracle(kma, oracle_c, joined, params, strict):
    hits = joined[1] if strict else joined[0]
    got, st = _check(kma, oracle_c, hits, joined[2], **params)
    assert st[0] > 500 and st[3] > 100, st  # lists examined, proposals made
    # every proposal's first location is one of its peg's connections on that strand
    keys = set(zip(hits["fid"].tolist(), hits["contig"].tolist(), hits["left"].tolist()))
    assert all((p, c, l) in keys for p, c, l in zip(got["peg"].tolist(), got["contig"].tolist(),
                                                    got["left"].tolist()))
    assert (got["right"] >= got["left"] + 3 * K - 1).all() and (got["evidence"] >= 1).all()


def test_proposals_python_twin(kma, joined):
    """The independent pure-Python restatement agrees on the first 400 pegs' connections."""
    hits = joined[0][joined[0]["fid"] < 400]
    got, st = kma.propose_pegs(hits, joined[2], K, min_strength=0.2)
    conns = [(int(h["contig"]), int(h["left"]), chr(h["strand"]), int(h["fid"])) for h in hits]
    exp, est = oracle_py.propose(conns, joined[2].tolist(), K, 0.2)
    assert list(st) == est
    assert [(int(p["peg"]), int(p["contig"]), chr(p["strand"]), int(p["left"]), int(p["right"]),
             int(p["evidence"]), int(p["frame"])) for p in got] == exp


def test_proposals_synthetic_dense(kma, oracle_c):
    """Dense synthetic connection sets: many contigs, both strands, every phase, long lists
    (lists of thousands of locations: the O(size^2) Java loop vs two binary searches)."""
    rng = np.random.default_rng(5)
    for n, n_peg, n_ctg, span in ((200_000, 300, 7, 60_000), (50_000, 5, 2, 400_000)):
        ct = np.sort(rng.integers(0, n_ctg, n)).astype(np.uint32)
        lf = rng.integers(1, span, n).astype(np.int32)
        sd = np.where(rng.random(n) < 0.5, ord("+"), ord("-")).astype(np.uint8)
        pg = rng.integers(0, n_peg, n).astype(np.uint32)
        h = np.zeros(n, kma.HIT_DTYPE)
        h["contig"], h["left"], h["strand"], h["fid"] = ct, lf, sd, pg
        h = np.unique(h)  # canonical (contig, left, ...) order, no duplicate connection
        h = h[np.lexsort((h["left"], h["contig"]))]
        peg_len = rng.integers(30, 900, n_peg).astype(np.uint32)
        for kw in (dict(), dict(min_strength=0.01, max_fuzz=3.0, min_fuzz=0.1)):
            _check(kma, oracle_c, h, peg_len, **kw)


def test_proposals_edges(kma):
    peg_len = np.array([100, 3], np.uint32)
    got, st = kma.propose_pegs(np.zeros(0, kma.HIT_DTYPE), peg_len, K)
    assert len(got) == 0 and (st == 0).all()
    h = np.zeros(2, kma.HIT_DTYPE)
    h["contig"], h["left"], h["strand"], h["fid"] = [0, 0], [50, 10], ord("+"), [0, 0]
    with pytest.raises(kma.KmerAnnoError):  # not in (contig, left) order
        kma.propose_pegs(h, peg_len, K)
    h["left"] = [10, 50]
    h["fid"] = [0, 2]
    with pytest.raises(kma.KmerAnnoError):  # peg index out of range
        kma.propose_pegs(h, peg_len, K)
    # a 3-aa peg (pegLen 9): minKmers = (int)(9 * 0.1) = 0, so the Java loop would read past
    # the list; every start of the (one-frame) list proposes instead
    h["fid"], h["left"] = [1, 1], [10, 13]
    got, st = kma.propose_pegs(h, peg_len, K, min_strength=0.3)
    assert list(st) == [1, 0, 0, 2] and list(got["evidence"]) == [1, 1]
    assert list(got["right"]) == [33, 36] and list(got["frame"]) == [3, 3]
