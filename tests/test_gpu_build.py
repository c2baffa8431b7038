"""GPU parity of the signature-table construction: kma_build_signatures
(BuildKmerProcessor.java:137-223 with RoleCounter.java) against the C oracle, bit-exact as sets
of (kmer, role) rows — the reference prints its HashMap in iteration order."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
K = 8


@pytest.fixture(scope="module")
def kma(native_lib):
    import kmeranno
    assert kmeranno.device_count() >= 1
    return kmeranno


def _family_proteins(rng, n_fam=80, n=1500):
    """Proteins drawn from families (mutated 8%), roles from the families with mixing: several
    roles share families (non-discriminating kmers), some proteins are buffered (-1) or
    skipped (-2)."""
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    fams = [aa[rng.integers(0, 20, int(rng.integers(20, 400)))] for _ in range(n_fam)]
    prots, roles = [], []
    for _ in range(n):
        f = int(rng.integers(0, n_fam))
        p = fams[f].copy()
        m = rng.random(len(p)) < 0.08
        p[m] = aa[rng.integers(0, 20, int(m.sum()))]
        prots.append(p.tobytes().decode())
        u = rng.random()
        roles.append(-1 if u < 0.1 else -2 if u < 0.13 else f % 50)
    return prots, roles


@pytest.mark.parametrize("flags", [0, 1])
@pytest.mark.parametrize("k", [8, 10, 12])
def test_build_signatures_vs_oracle(kma, oracle_c, flags, k):
    """The discriminating (kmer, role) rows equal the oracle's, in key order without
    duplicates, at K = 8 and the wide sizes (BuildKmerProcessor -K, :84-87); a window with a
    byte outside A-Z/'*' is refused (KMA_E_ALPHABET)."""
    rng = np.random.default_rng(17 + flags + k)
    prots, roles = _family_proteins(rng)
    prots += ["", "ACDEFGH", "ACDEFGHI", "ACDEFGHIK", "ACDEFGHIKLMN", "ACDEFGHIKLMNP"]
    roles += [3, 3, 4, 5, 6, 7]
    res, off = oracle_c.pack_strings(prots)
    km, rl = oracle_c.build_signatures(res, off, roles, k, flags)
    keys, groles = kma.build_signatures(res, off, roles, k, flags)
    from kmeranno import synth
    got = {synth.unpack_key(x, k): int(r) for x, r in zip(keys.tolist(), groles)}
    exp = {bytes(r).decode(): int(v) for r, v in zip(km, rl)}
    assert len(exp) > 10_000 and got == exp
    assert (np.diff(keys.astype(np.int64)) > 0).all()
    with pytest.raises(kma.KmerAnnoError) as e:
        kma.build_signatures(*oracle_c.pack_strings(["ACDEFGHIKLmNP"]), [0], k)
    assert e.value.code == kma.E_ALPHABET


@pytest.mark.parametrize("k", [8, 10])
def test_build_role_counter_RoleTests(kma, k):
    """test/RoleTests.java:15-36 through kma_build_signatures: a kmer hit twice by roleA (good
    count 2, bad 0) is kept for roleA; hit by roleB afterwards (bad count 1) it is dropped,
    and so when roleB came first; a buffered protein removes it; a skipped peg does not."""
    from kmeranno import synth
    A, B = 0, 1
    shared = "PPMKVLAGHW"[-k:]
    prot = "QQ" + shared + "NN"
    others = {A: "CCCCDEFGHIKLMNPQ", B: "WWWWYYYYVVVVTTTT"}
    for roles, kept in (([A, A], True), ([A, A, B], False), ([B, A], False),
                        ([A, -1], False), ([A, -2], True)):
        prots = [prot] * len(roles) + [others[A], others[B]]
        res, off = kma.pack_strings(prots)
        keys, rl = kma.build_signatures(res, off, roles + [A, B], k)
        got = {synth.unpack_key(x, k): int(r) for x, r in zip(keys.tolist(), rl)}
        assert (shared in got) == kept, roles
        if kept:
            assert got[shared] == A
        assert all(v == A for km, v in got.items() if km in others[A])


def test_build_then_apply_roundtrip(kma, oracle_c):
    """Built rows feed the apply path: a table created from the GPU build calls every
    interesting peg of a family whose kmers survived with its role, as the oracle does."""
    rng = np.random.default_rng(5)
    prots, roles = _family_proteins(rng, n_fam=40, n=600)
    res, off = oracle_c.pack_strings(prots)
    keys, groles = kma.build_signatures(res, off, roles, K)
    from kmeranno import synth
    kmers = [synth.unpack_key(x) for x in keys.tolist()]
    with kma.SignatureTable.from_packed(keys, groles, K) as t:
        fid, cnt, st, _ = kma.annotate_proteins(t, res, off, 5)
    ot = oracle_c.Table(kmers, groles.astype(np.int32))
    efid, ecnt, est = oracle_c.apply(ot, res, off, K, 5, 0)
    assert (st == est).all() and (fid == efid).all() and (cnt == ecnt).all()
    called = (st == kma.STATUS_CALLED) & (np.asarray(roles) >= 0)  # interesting pegs only
    assert called.sum() > 100
    assert (fid[called] == np.asarray(roles)[called]).all()
