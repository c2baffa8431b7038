"""GPU parity at K = 9..12: wide tables (16-byte slots, four per 64-byte bucket).

The projector takes -K up to 12 (KmerProcessor.java:86-88 sets KmerReference's K, used by the
6-frame extractor KmerReference.java:157-203 and the peg kmers :124-147). Keys of 5K bits no
longer fit the narrow 8-byte slot, so these tables use the wide layout (kma_internal.h). Every
6-frame hit and every peg connection must equal the C oracle's, which is written on kmer text
and takes any K; the AppTest property (a hit's kmer is the translation of its location,
AppTest.java:131-138) is re-checked at K = 12.
"""
import numpy as np
import pytest

from oracle import oracle_py

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kma(native_lib):
    import kmeranno
    assert kmeranno.device_count() >= 1
    return kmeranno


@pytest.fixture(params=["auto", "7", "0"], ids=["m-auto", "m7", "flat"])
def layout(request, monkeypatch):
    import kmeranno
    kmeranno.load()
    kmeranno.set_option(kmeranno.OPT_LAYOUT, -1 if request.param == "auto" else int(request.param))
    return request.param


def _contigs(small_gto):
    contigs = [c["dna"] for c in small_gto["contigs"]]
    contigs[2] = contigs[2][:50000] + "nnnNacgtRYk" + contigs[2][50000:]
    contigs += [contigs[0][100:100 + n] for n in range(30, 42)]  # around 3K + 3 bases
    return contigs


@pytest.mark.parametrize("k", [9, 10, 12])
@pytest.mark.parametrize("lf", [0.5, 0.9])
def test_contigs_wide_vs_oracle(kma, oracle_c, small_gto, layout, k, lf):
    """All small.gto contigs (plus ambiguous bases and contigs of 3K-6 .. 3K+5 bases) against a
    table of 200k of their own K-mers (random fids) at load factors 0.5 and 0.9 (overflow
    chains in four-slot buckets): every (contig, left, strand, frame, fid) hit equals the
    oracle's, in canonical order."""
    contigs = _contigs(small_gto)
    dna, off = oracle_c.pack_strings(contigs)
    km, _, _, _, _ = oracle_c.contig_kmers(dna, off, 11, k)
    rng = np.random.default_rng(k)
    pick = rng.choice(len(km), 200_000, replace=False)
    kmers = [bytes(r).decode() for r in km[pick]]
    fids = rng.integers(0, 1000, len(kmers)).astype(np.int32)
    e = oracle_c.annotate_contigs(oracle_c.Table(kmers, fids), dna, off, 11, k)
    with kma.SignatureTable.from_rows(kmers, fids.astype(np.uint32), k, load_factor=lf) as t:
        i = t.info
        assert i.k == k and i.slots_per_bucket == 4 and i.bytes == 64 * i.n_buckets
        assert i.n_entries == len(set(kmers))
        if layout != "auto":
            assert i.minimizer_len == int(layout)
        if lf == 0.9:
            assert i.n_displaced > 0 and i.max_probe >= 2
        hits, tally = kma.annotate_contigs(t, dna, off, 11, n_fid=1000)
    assert len(hits) == len(e[0]) > 100_000
    for a, b in zip((hits["contig"], hits["left"], hits["strand"], hits["frame"], hits["fid"]), e):
        assert (a == b).all()
    expect = np.zeros((len(contigs), 1000), np.uint32)
    np.add.at(expect, (e[0], e[4]), 1)
    assert (tally == expect).all()
    if k == 12:  # AppTest.verifyKmers: translate(getDna(loc)) == kmer
        tab = set(kmers)
        for h in hits[rng.choice(len(hits), 300, replace=False)]:
            seq = contigs[h["contig"]][h["left"] - 1:h["left"] - 1 + 3 * k]
            if h["strand"] == ord("-"):
                seq = oracle_py.reverse_complement(seq)
            assert oracle_py.translate(seq, 1, 11) in tab


@pytest.mark.parametrize("k", [9, 10, 12])
@pytest.mark.parametrize("strict", [False, True])
def test_peg_connect_wide_vs_oracle(kma, oracle_c, small_gto, k, strict):
    """KmerProcessor.java:195-207 at -K 9..12: singleton peg kmers of a mutated copy of
    small.gto's pegs joined with small.gto's 6-frame kmer map, AGGRESSIVE and STRICT."""
    rng = np.random.default_rng(100 + k)
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    prots = [f["protein_translation"] for f in small_gto["features"]
             if f.get("protein_translation")]
    close = []
    for p in prots:
        b = np.frombuffer(p.encode(), np.uint8).copy()
        m = rng.random(len(b)) < 0.04
        b[m] = aa[rng.integers(0, 20, int(m.sum()))]
        close.append(b.tobytes().decode())
    close += prots[:4] + ["", "ACDEFGHIKLMN"[:k], "XXXXXXXXXXXXXXXX"]
    res, off = oracle_c.pack_strings(close)
    dna, doff = oracle_c.pack_strings([c["dna"] for c in small_gto["contigs"]])
    e = oracle_c.peg_connect(res, off, dna, doff, 11, k, strict)
    assert len(e[0]) > 10_000
    t, n_win = kma.SignatureTable.from_pegs(res, off, k)
    assert n_win == sum(max(len(p) - k, 0) for p in close)
    with t:
        assert t.info.slots_per_bucket == 4
        hits = kma.connect_pegs(t, dna, doff, 11, strict)
    assert len(hits) == len(e[0])
    for a, b in zip((hits["contig"], hits["left"], hits["strand"], hits["frame"], hits["fid"]), e):
        assert (a == b).all()


def test_wide_table_api(kma, oracle_c, small_gto):
    """Wide tables through the device-build entry points (kma_table_build_device with K = 11
    keys, wrap, the 6-frame device call); the protein path refuses K > 8 (apply's
    ProteinKmers keeps K = 8); last-wins duplicates and rows of other lengths at K = 10."""
    torch = pytest.importorskip("torch")
    from kmeranno import synth
    k = 11
    contigs = [c["dna"] for c in small_gto["contigs"]][:2]
    dna, off = oracle_c.pack_strings(contigs)
    km, _, _, _, _ = oracle_c.contig_kmers(dna, off, 11, k)
    keys = np.unique(kma.pack_std(km))
    keys = keys[keys != 0][::3]
    fids = (np.arange(len(keys)) % 777).astype(np.uint32)
    assert keys.max() >= 1 << 40  # beyond a narrow slot
    dev = torch.device("cuda", 0)
    nb = kma.buckets_for(len(keys), 0.5, k)
    assert kma.bucket_slots(k) == 4 and nb == -(-2 * len(keys) // 4)
    slots = torch.empty(nb * 8, dtype=torch.int64, device=dev)  # 64 bytes per bucket
    winner = torch.empty(nb * 4, dtype=torch.int32, device=dev)
    status = torch.zeros(4, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    kma.build_device(slots.data_ptr(), nb, winner.data_ptr(),
                     torch.from_numpy(keys.view(np.int64)).to(dev).data_ptr(),
                     torch.from_numpy(fids.view(np.int32)).to(dev).data_ptr(), len(keys),
                     status.data_ptr(), stream, k=k)
    torch.cuda.synchronize()
    st4 = status.cpu().numpy()
    assert st4[0] == 0 and st4[1] == len(keys)
    t = kma.SignatureTable.wrap_device(slots.data_ptr(), nb, k, 0)
    ws = kma.Workspace(0)
    n_bases = int(off[-1])
    ws.reserve_contigs(n_bases)
    d_dna = torch.from_numpy(dna).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    cap = 400_000
    d_hits = torch.zeros(cap * kma.HIT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    d_nh = torch.zeros(1, dtype=torch.int64, device=dev)
    kma.annotate_contigs_device(t, ws, d_dna.data_ptr(), d_off.data_ptr(), len(contigs), n_bases,
                                11, d_hits.data_ptr(), cap, d_nh.data_ptr(), 0, 0, stream)
    torch.cuda.synchronize()
    kmers = [synth.unpack_key(x, k) for x in keys.tolist()]
    e = oracle_c.annotate_contigs(oracle_c.Table(kmers, fids.astype(np.int32)), dna, off, 11, k)
    n = int(d_nh.item())
    assert n == len(e[0]) <= cap
    hits = d_hits.cpu().numpy().view(kma.HIT_DTYPE)[:n]
    for a, b in zip((hits["contig"], hits["left"], hits["strand"], hits["frame"], hits["fid"]), e):
        assert (a == b).all()
    res, poff = kma.pack_strings(["ACDEFGHIKLMNPQ"])
    with pytest.raises(kma.KmerAnnoError) as err:
        kma.annotate_proteins(t, res, poff, 5)
    assert err.value.code == kma.E_INVALID
    ws.close()
    t.close()
    rows = ["ACDEFGHIKL", "ACDEFGHIKL", "ACDEFGHIK", "MNPQRSTVWY"]
    with kma.SignatureTable.from_rows(rows, [1, 2, 3, 4], 10) as t2:
        i = t2.info
        assert (i.n_rows, i.n_skipped, i.n_entries, i.k) == (4, 1, 2, 10)
        d, o = kma.pack_strings(["gcgtgcgatgaatttggccatatcaaactg"])  # ACDEFGHIKL, frame 1 '+'
        hits, _ = kma.annotate_contigs(t2, d, o, 11)
        assert len(hits) == 0  # i < P - K: the only window is the excluded last one
        d, o = kma.pack_strings(["gcgtgcgatgaatttggccatatcaaactgaaa"])
        hits, _ = kma.annotate_contigs(t2, d, o, 11)
        assert [(h["left"], chr(h["strand"]), h["fid"]) for h in hits] == [(1, "+", 2)]
