"""§8(f)3, the hash annotator's scoring loop (HashAnnotationProcessor.java:221-328 with the
external GenomeProteinKmers restated) on the GPU (kma_hash_annotate) against the C oracle
(orc_hash_annotate, a literal all-pairs restatement) and its Python twin: best prototype,
similarity (bit-exact double) and per-prototype match counts; the per-genome report of
kmeranno.hashanno on the reference's own fixture small.gto. GenomeProteinKmers' semantics are
parity unpinned (external)."""
import numpy as np
import pytest

from oracle import oracle_py

pytestmark = pytest.mark.gpu
AA = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)


@pytest.fixture(scope="module")
def kma(native_lib):
    import kmeranno
    assert kmeranno.device_count() >= 1
    return kmeranno


def _mut(rng, p, rate):
    b = np.frombuffer(p.encode(), np.uint8).copy()
    m = rng.random(len(b)) < rate
    b[m] = AA[rng.integers(0, 20, int(m.sum()))]
    return b.tobytes().decode()


def _both(kma, oracle_c, genome, protos, k, min_sim):
    g, go = oracle_c.pack_strings(genome)
    p, po = oracle_c.pack_strings(protos)
    got = kma.hash_annotate(g, go, p, po, k, min_sim)
    exp = oracle_c.hash_annotate(g, go, p, po, k, min_sim)
    for a, b in zip(got, exp):
        assert (a == b).all()
    return got


@pytest.mark.parametrize("k,min_sim", [(8, 0.0125), (8, 0.3), (5, 0.05), (12, 0.0)])
def test_hash_scores_small_gto_vs_oracle(kma, oracle_c, small_gto, k, min_sim):
    """small.gto's proteins as the genome; prototypes = its proteins mutated 10-40%, shuffled,
    with exact copies and duplicates (ties: the earlier prototype wins)."""
    rng = np.random.default_rng(7)
    prots = [f["protein_translation"] for f in small_gto["features"]
             if f.get("protein_translation")]
    protos = [_mut(rng, p, rng.uniform(0.1, 0.4)) for p in prots]
    rng.shuffle(protos)
    protos += prots[:20] + prots[:5]
    best, sim, cnt = _both(kma, oracle_c, prots, protos, k, min_sim)
    if min_sim <= 0.05:
        assert (best >= 0).mean() > 0.5 and cnt.sum() > len(prots) // 2
    assert (best[:5] >= len(protos) - 25).all() and (sim[:5] == 1.0).all()


def test_hash_scores_python_twin(kma, oracle_c):
    rng = np.random.default_rng(3)
    base = [AA[rng.integers(0, 20, rng.integers(60, 300))].tobytes().decode() for _ in range(80)]
    genome = [_mut(rng, p, 0.05) for p in base[:50]] + ["ACDEFG", ""]
    protos = [_mut(rng, p, 0.25) for p in base] + [base[3], base[3], "MMMMMMMMMMMMMMMMMMMMMMMMMMMM"]
    best, sim, cnt = _both(kma, oracle_c, genome, protos, 8, 0.0125)
    pb, ps, pc = oracle_py.hash_annotate(genome, protos, 8, 0.0125)
    assert best.tolist() == pb and sim.tolist() == ps and cnt.tolist() == pc
    assert best[3] == 80 and best[-1] == -1 and best[-2] == -1


def test_hash_scores_low_complexity_and_scale(kma, oracle_c):
    """1,500 genome proteins x 3,000 prototypes with low-complexity runs shared by many
    proteins (long candidate lists per kmer)."""
    rng = np.random.default_rng(11)
    motif = "GGSGGSGGSGGSGGSGGS"
    base = [AA[rng.integers(0, 20, rng.integers(50, 500))].tobytes().decode()
            + (motif if i % 3 == 0 else "") for i in range(1500)]
    protos = [_mut(rng, base[i % 1500], 0.3) for i in rng.permutation(3000)]
    _both(kma, oracle_c, base, protos, 8, 0.0125)


def test_hash_annotate_report_small_gto(kma, small_gto):
    """kmeranno.hashanno.annotate_genome: the report of processGenome on small.gto with
    prototypes from its own features (mutated, annotations kept or renamed)."""
    from kmeranno import hashanno
    rng = np.random.default_rng(5)
    feats = [(f["id"], f.get("protein_translation", ""), f.get("function", ""))
             for f in small_gto["features"]]
    rows = []
    for i, (fid, p, func) in enumerate(feats):
        if p:
            rows.append((_mut(rng, p, 0.1), func if i % 4 else f"renamed {i}"))
    rows.append(("ACDEFGHIKL" * 3, "too short"))  # dropped: shorter than minLen 50
    protos = hashanno.prototypes_from_rows(rows)
    assert len(protos) == sum(len(p) >= 50 for p, _ in rows) and protos[-1][1] != "too short"
    lines, counts, changes = hashanno.annotate_genome(feats, protos)
    assert len(lines) == len(feats)
    assert counts["new"] == len(changes) > 100 and counts["confirmed"] > 300
    assert counts["default"] < 0.1 * len(feats)
    for line, (fid, p, func) in zip(lines, feats):
        f = line.split("\t")
        assert f[0] == fid and f[3] == func
        if p:
            assert float(f[1]) >= 0.0
        else:
            assert f[1] == "" and f[2] == func


def test_hash_annotate_rejects_bad_input(kma):
    with pytest.raises(kma.KmerAnnoError):
        kma.hash_annotate(np.frombuffer(b"acdefghikl", np.uint8), np.array([0, 10], np.uint64),
                          np.frombuffer(b"ACDEFGHIKL", np.uint8), np.array([0, 10], np.uint64))
    with pytest.raises(kma.KmerAnnoError):
        kma.hash_annotate(np.frombuffer(b"ACDEFGHIKL", np.uint8), np.array([0, 10], np.uint64),
                          np.frombuffer(b"ACDEFGHIKL", np.uint8), np.array([0, 10], np.uint64),
                          min_sim=1.0)


@pytest.mark.parametrize("slice_cand", ["1", "700", "5000"])
def test_hash_scores_in_prototype_slices(kma, oracle_c, small_gto, monkeypatch, slice_cand):
    """Candidates are sorted and run-length encoded in slices of whole prototypes (each below
    hipcub's 2^31 element limit; the KMA_OPT_HASH_SLICE option lowers the slice size here): a slice's best
    similarity replaces the running best only when strictly higher, so ties still go to the
    earlier prototype (exact copies placed in different slices) and the result equals the
    one-slice call and the oracle."""
    rng = np.random.default_rng(21)
    prots = [f["protein_translation"] for f in small_gto["features"]
             if f.get("protein_translation")][:300]
    protos = [_mut(rng, p, rng.uniform(0.1, 0.4)) for p in prots]
    protos = protos[:150] + prots[:10] + protos[150:] + prots[:10]  # ties across slices
    ref = _both(kma, oracle_c, prots, protos, 8, 0.0125)
    kma.set_option(kma.OPT_HASH_SLICE, int(slice_cand))
    got = _both(kma, oracle_c, prots, protos, 8, 0.0125)
    for a, b in zip(got, ref):
        assert (a == b).all()
    assert (got[0][:10] == np.arange(150, 160)).all() and (got[1][:10] == 1.0).all()
