"""GPU parity for ProteinKmers.distance (GeneCopyProcessor.java:129-162):
kma_protein_distances and kma_protein_best_match against the C oracle, bit-exact (integer
set counts, and the distance double formed by the same expression)."""
import numpy as np
import pytest

from oracle import oracle_py

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kma(native_lib):
    import kmeranno
    assert kmeranno.device_count() >= 1
    return kmeranno


def _proteins(seed=0, n=300):
    rng = np.random.default_rng(seed)
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    prots = [aa[rng.integers(0, 20, int(rng.integers(0, 900)))].tobytes().decode()
             for _ in range(n)]
    # relatives: mutated copies, shifted fragments, repeats, tiny and empty proteins
    for i in range(0, 60, 3):
        b = np.frombuffer(prots[i].encode(), np.uint8).copy()
        m = rng.random(len(b)) < 0.08
        b[m] = aa[rng.integers(0, 20, int(m.sum()))]
        prots += [b.tobytes().decode(), prots[i][len(prots[i]) // 3:], prots[i] * 2]
    prots += ["", "ACDEFGH", "ACDEFGHI", "AAAAAAAAAAAAAAAAAAAAAA", "W" * 5000]
    return prots


@pytest.mark.parametrize("k", [2, 5, 8, 12])
@pytest.mark.parametrize("flags", [0, 1])
def test_distances_vs_oracle(kma, oracle_c, k, flags):
    prots = _proteins(1)
    res, off = kma.pack_strings(prots)
    rng = np.random.default_rng(k)
    n = len(prots)
    # random pairs, every protein with itself, and each planted relative with its source
    rel_a = [3 * (j // 3) for j in range(60)]
    rel_b = [300 + j for j in range(60)]
    pa = np.concatenate([rng.integers(0, n, 4000), np.arange(n), rel_a]).astype(np.uint32)
    pb = np.concatenate([rng.integers(0, n, 4000), np.arange(n), rel_b]).astype(np.uint32)
    sim, size, dist = kma.protein_distances(res, off, pa, pb, k, flags)
    esim, esa, esb, edist = oracle_c.protein_distances(res, off, pa, pb, k, flags)
    assert (sim == esim).all() and (size[pa] == esa).all() and (size[pb] == esb).all()
    assert (dist == edist).all()  # same integers, same double expression: bit-exact
    assert (sim[-60:] > 0).sum() > 40 and (dist[4000:4000 + n][size > 0] == 0.0).all()


def test_best_match_gene_copy_rule(kma, oracle_c, small_gto):
    """GeneCopyProcessor.java:135-146 on small.gto's pegs: every peg (query) against all pegs
    of its function (candidates, feature order; the query itself included so that ties at
    distance 0 resolve to the last equal one), maxDist 0.5 and 0.8, K = 8 and 10."""
    feats = [f for f in small_gto["features"] if f.get("protein_translation")]
    prots = [f["protein_translation"] for f in feats]
    funcs = [f.get("function", "") for f in feats]
    by_fn = {}
    for i, fn in enumerate(funcs):
        by_fn.setdefault(fn, []).append(i)
    rng = np.random.default_rng(3)
    # mutated copies as extra candidates so that distances are neither 0 nor 1
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    extra = []
    for i in range(len(prots)):
        b = np.frombuffer(prots[i].encode(), np.uint8).copy()
        m = rng.random(len(b)) < 0.15
        b[m] = aa[rng.integers(0, 20, int(m.sum()))]
        extra.append(b.tobytes().decode())
    allp = prots + extra
    res, off = kma.pack_strings(allp)
    query = np.arange(len(prots), dtype=np.uint32)
    cands = [by_fn[funcs[i]] + [len(prots) + j for j in by_fn[funcs[i]]] for i in range(len(prots))]
    cand_off = np.zeros(len(query) + 1, np.uint64)
    cand_off[1:] = np.cumsum([len(c) for c in cands])
    cand = np.array([x for c in cands for x in c], np.uint32)
    for k, max_dist in ((8, 0.5), (10, 0.8)):
        best, bd = kma.protein_best_match(res, off, query, cand_off, cand, max_dist, k)
        pa = np.repeat(query, np.diff(cand_off).astype(np.int64))
        _, _, _, edist = oracle_c.protein_distances(res, off, pa, cand, k, 0)
        for q in range(len(query)):
            d = edist[cand_off[q]:cand_off[q + 1]]
            fdist, found = max_dist, -1
            for c, x in zip(cand[cand_off[q]:cand_off[q + 1]], d):
                if x <= fdist:
                    fdist, found = x, int(c)
            assert best[q] == found and bd[q] == fdist, q
        assert (best >= 0).sum() > 0.9 * len(query)
    # the pure-Python twin on a few queries
    for q in range(0, len(prots), 97):
        f, d = oracle_py.best_match(allp[q], [allp[c] for c in cands[q]], 0.5)
        b, bdist = kma.protein_best_match(res, off, query[q:q + 1],
                                          np.array([0, len(cands[q])], np.uint64),
                                          np.array(cands[q], np.uint32), 0.5)
        assert (b[0] == (cands[q][f] if f >= 0 else -1)) and bdist[0] == d


def test_distance_rejects_foreign_bytes(kma):
    res, off = kma.pack_strings(["ACDEFGHIKL", "ACDE#GHIKL"])
    with pytest.raises(kma.KmerAnnoError) as e:
        kma.protein_distances(res, off, [0], [1], 8)
    assert e.value.code == kma.E_ALPHABET
