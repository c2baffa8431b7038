"""GPU parity: libkmeranno.so (HIP, gfx950) against the oracle, bit-exact.

Apply outputs (fid, count, status) per protein and 6-frame hits (contig, left, strand,
frame, fid) must equal the CPU restatement's on the same inputs: the committed golden
vectors, hand-built edge cases, seeded synthetic workloads (BASELINE configs 1-2 shapes)
and size-independent properties at larger sizes.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle_py

pytestmark = pytest.mark.gpu
K = 8


@pytest.fixture(autouse=True, params=["0", "1"], ids=["K1+K2", "K12"])
def protein_form(request, monkeypatch):
    """Every test under both protein-path forms: the two-kernel K1 + K2 pipeline and the fused
    K12 kernel (the library picks by batch size; KMA_FUSED forces one, read per call)."""
    monkeypatch.setenv("KMA_FUSED", request.param)
    return request.param


@pytest.fixture(scope="module")
def kma(native_lib):
    import kmeranno
    assert kmeranno.device_count() >= 1
    return kmeranno


def _roles(rows):
    ids = {}
    for _, r in rows:
        ids.setdefault(r, len(ids))
    return ids


def _gpu_apply(kma, rows, prots, min_hits=5, flags=0, lf=0.5):
    ids = _roles(rows)
    with kma.SignatureTable.from_rows([r[0] for r in rows], [ids[r[1]] for r in rows], K,
                                      load_factor=lf) as t:
        res, off = kma.pack_strings(prots)
        fid, cnt, st, _ = kma.annotate_proteins(t, res, off, min_hits, flags)
    inv = {v: k for k, v in ids.items()}
    return [[int(s), inv.get(int(f)), int(n)] for f, n, s in zip(fid, cnt, st)]


def test_edge_cases_golden(kma):
    for c in json.load(open(os.path.join(GOLDEN, "apply_edge.json"))):
        got = _gpu_apply(kma, [tuple(r) for r in c["rows"]], c["proteins"], c["min_hits"],
                         c["flags"])
        assert got == c["expected"], c["name"]


def test_table_info_and_alphabet(kma):
    rows = [("ACDEFGHI", 0), ("ACDEFGHI", 1), ("ACDEFGH", 2), ("ACDE-GHI", 1)]
    t = kma.SignatureTable.from_rows([r[0] for r in rows], [r[1] for r in rows], K)
    i = t.info
    assert (i.n_rows, i.n_skipped, i.n_entries, i.k) == (4, 1, 2, 8)
    assert i.n_extra_syms == 1 and i.extra_syms[0] == ord("-")
    keys = t.pack(["ACDEFGHI", "ACDE-GHI", "ACDEFGH", "ACDE#GHI"])
    assert keys[0] != 0 and keys[1] != 0 and keys[2] == 0 and keys[3] == 0
    t.close()
    with pytest.raises(kma.KmerAnnoError) as e:
        kma.SignatureTable.from_rows(["A-CDEFGH", "A.CDEFGH", "A,CDEFGH", "A;CDEFGH", "A:CDEFGH"],
                                     [0] * 5, K)
    assert e.value.code == kma.E_ALPHABET


def test_min_hits_must_be_positive(kma):
    t = kma.SignatureTable.from_rows(["ACDEFGHI"], [0], K)
    res, off = kma.pack_strings(["ACDEFGHI"])
    with pytest.raises(kma.KmerAnnoError) as e:
        kma.annotate_proteins(t, res, off, 0)
    assert e.value.code == kma.E_INVALID  # ApplyKmerProcessor.java:91-92


@pytest.mark.parametrize("flags", [0, 1, 2])
def test_config1_golden(kma, flags):
    z = np.load(os.path.join(GOLDEN, "apply_c1.npz"))
    with kma.SignatureTable.from_rows([bytes(r).decode() for r in z["table_kmers"]],
                                      z["table_fids"], K) as t:
        fid, cnt, st, tally = kma.annotate_proteins(t, z["residues"], z["offsets"], 5, flags,
                                                    n_fid=100)
    assert (st == z[f"status_{flags}"]).all()
    assert (fid == z[f"fid_{flags}"]).all()
    assert (cnt == z[f"count_{flags}"]).all()
    called = z[f"fid_{flags}"][z[f"status_{flags}"] == 1]
    assert (tally == np.bincount(called, minlength=100)).all()


@pytest.mark.parametrize("lf", [0.5, 0.9, 0.95])
def test_synthetic_vs_oracle(kma, oracle_c, lf):
    """2,000 proteins vs a 200k-entry table (seeded), packed-key table path, two load factors
    (0.9 forces multi-bucket probe chains)."""
    from kmeranno import synth
    wl = synth.make_workload(2000, 200_000, 2000, seed=11)
    kmers = [synth.unpack_key(x) for x in wl.keys]
    ot = oracle_c.Table(kmers, wl.fids.astype(np.int32))
    efid, ecnt, est = oracle_c.apply(ot, wl.residues, wl.offsets, K, 5, 0)
    with kma.SignatureTable.from_packed(wl.keys, wl.fids, K, load_factor=lf) as t:
        assert t.info.n_entries == ot.size
        if lf == 0.9:
            assert t.info.max_probe >= 2
        fid, cnt, st, _ = kma.annotate_proteins(t, wl.residues, wl.offsets, 5, 0)
    assert (st == est).all() and (fid == efid).all() and (cnt == ecnt).all()
    assert (st == 1).sum() > 500 and (st == 2).sum() > 50


def test_long_proteins_global_dedupe(kma, oracle_c):
    """Proteins with more distinct hits than the per-wave LDS set (1,536) go through the
    global-memory dedupe pass; duplicates inside them still count once."""
    rng = np.random.default_rng(3)
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    prots, rows = [], []
    for L, role in ((3000, "R1"), (6000, "R2"), (1700, "R3"), (2500, "R4")):
        p = aa[rng.integers(0, 20, L)].tobytes().decode()
        p = p + p[:900]  # repeated block: 893 duplicate windows
        prots.append(p)
        rows += [(p[i:i + K], role) for i in range(0, len(p) - K + 1)]
    prots.append(prots[0][:1000] + prots[1][:1000])  # ambiguous long protein
    rows.reverse()
    ids = _roles(rows)
    ot = oracle_c.Table([r[0] for r in rows], [ids[r[1]] for r in rows])
    res, off = oracle_c.pack_strings(prots)
    efid, ecnt, est = oracle_c.apply(ot, res, off, K, 5, 0)
    assert max(ecnt) > 1536
    inv = {v: k for k, v in ids.items()}
    got = _gpu_apply(kma, rows, prots)
    assert got == [[int(s), inv.get(int(f)), int(n)] for f, n, s in zip(efid, ecnt, est)]


def test_empty_and_ragged_batches(kma, oracle_c):
    rows = [("ACDEFGHI", "R1"), ("CDEFGHIK", "R1")]
    prots = ["", "ACDEFGHIK", "", "A" * 7, "ACDEFGHIK" * 40, ""]
    assert _gpu_apply(kma, rows, prots, 1) == [
        list(oracle_py.apply_protein(oracle_py.load_table(rows), p, 1)) for p in prots]
    t = kma.SignatureTable.from_rows(["ACDEFGHI"], [0], K)
    res, off = kma.pack_strings([])
    fid, cnt, st, _ = kma.annotate_proteins(t, res, off, 5)
    assert len(st) == 0


def test_contigs_golden(kma):
    z = np.load(os.path.join(GOLDEN, "contigs_gto.npz"))
    with kma.SignatureTable.from_rows([bytes(r).decode() for r in z["table_kmers"]],
                                      z["table_fids"], K) as t:
        hits, tally = kma.annotate_contigs(t, z["dna"], z["offsets"], 11, n_fid=500)
    assert len(hits) == len(z["hit_left"])
    assert (hits["contig"] == z["hit_contig"]).all()
    assert (hits["left"] == z["hit_left"]).all()
    assert (hits["strand"] == z["hit_strand"]).all()
    assert (hits["frame"] == z["hit_frame"]).all()
    assert (hits["fid"] == z["hit_fid"]).all()
    n_contig = len(z["offsets"]) - 1
    expect = np.zeros((n_contig, 500), np.uint32)
    np.add.at(expect, (z["hit_contig"], z["hit_fid"]), 1)
    assert (tally == expect).all()


@pytest.mark.parametrize("gcode", [11, 4])
def test_contigs_small_gto_vs_oracle(kma, oracle_c, small_gto, gcode):
    """All five small.gto contigs plus boundary-length contigs and ambiguous bases: every
    6-frame window hit equals the oracle's, and (AppTest.java:131-138) each hit's kmer is the
    translation of the DNA at its location."""
    contigs = [c["dna"] for c in small_gto["contigs"]]
    contigs[2] = contigs[2][:50000] + "nnnNacgtRYk" + contigs[2][50000:]
    contigs += [contigs[0][100:100 + n] for n in range(20, 36)]  # 3K-4 .. 3K+11 bases
    dna, off = oracle_c.pack_strings(contigs)
    km, ct, lf, sd, fr = oracle_c.contig_kmers(dna, off, gcode, K)
    rng = np.random.default_rng(5)
    pick = rng.choice(len(km), 200_000, replace=False)
    kmers = [bytes(r).decode() for r in km[pick]]
    fids = rng.integers(0, 1000, len(kmers)).astype(np.int32)
    ot = oracle_c.Table(kmers, fids)
    e = oracle_c.annotate_contigs(ot, dna, off, gcode, K)
    with kma.SignatureTable.from_rows(kmers, fids.astype(np.uint32), K) as t:
        hits, _ = kma.annotate_contigs(t, dna, off, gcode)
        tab = dict(zip(t.pack(kmers).tolist(), kmers))
    for a, b in zip((hits["contig"], hits["left"], hits["strand"], hits["frame"], hits["fid"]), e):
        assert (a == b).all()
    # property: translate(getDna(loc)) == kmer, for a sample of hits
    from kmeranno import synth
    for h in hits[rng.choice(len(hits), 500, replace=False)]:
        seq = contigs[h["contig"]][h["left"] - 1:h["left"] - 1 + 3 * K]
        if h["strand"] == ord("-"):
            seq = oracle_py.reverse_complement(seq)
        assert oracle_py.translate(seq, 1, gcode) in tab.values()
    assert len(hits) > 100_000


def test_device_api_with_torch_buffers(kma):
    """_device entry points on torch-allocated HBM (the bench path), same results as host."""
    torch = pytest.importorskip("torch")
    from kmeranno import synth
    wl = synth.make_workload(3000, 100_000, 1000, seed=21)
    dev = torch.device("cuda", 0)
    nb = kma.buckets_for(len(wl.keys), 0.5)
    slots = torch.empty(nb * 8, dtype=torch.int64, device=dev)
    winner = torch.empty(nb * 8, dtype=torch.int32, device=dev)
    status = torch.zeros(4, dtype=torch.int32, device=dev)
    keys = torch.from_numpy(wl.keys.view(np.int64)).to(dev)
    fids = torch.from_numpy(wl.fids.view(np.int32)).to(dev)
    stream = torch.cuda.current_stream().cuda_stream
    kma.build_device(slots.data_ptr(), nb, winner.data_ptr(), keys.data_ptr(), fids.data_ptr(),
                     len(wl.keys), status.data_ptr(), stream)
    torch.cuda.synchronize()
    assert status[0].item() == 0
    t = kma.SignatureTable.wrap_device(slots.data_ptr(), nb, K, 0)
    n_res = int(wl.offsets[-1])
    ws = kma.Workspace(0, n_res)
    res = torch.from_numpy(wl.residues).to(dev)
    off = torch.from_numpy(wl.offsets.view(np.int64)).to(dev)
    n = wl.n_seq
    fid = torch.empty(n, dtype=torch.int32, device=dev)
    cnt = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    tally = torch.zeros(1000, dtype=torch.int32, device=dev)
    kma.annotate_proteins_device(t, ws, res.data_ptr(), off.data_ptr(), n, n_res, 5, 0,
                                 fid.data_ptr(), cnt.data_ptr(), st.data_ptr(), tally.data_ptr(),
                                 1000, stream)
    torch.cuda.synchronize()
    with kma.SignatureTable.from_packed(wl.keys, wl.fids, K) as th:
        hf, hc, hs, ht = kma.annotate_proteins(th, wl.residues, wl.offsets, 5, 0, n_fid=1000)
    assert (fid.cpu().numpy() == hf).all() and (cnt.cpu().numpy() == hc).all()
    assert (st.cpu().numpy() == hs).all()
    assert (tally.cpu().numpy().astype(np.uint32) == ht).all()
    ws.close()
    t.close()


def test_workspace_phase_timing(kma):
    """kma_workspace_timing: per-phase hipEvent durations of device calls (probe, vote)."""
    torch = pytest.importorskip("torch")
    from kmeranno import synth
    wl = synth.make_workload(500, 20_000, 200, seed=31)
    dev = torch.device("cuda", 0)
    with kma.SignatureTable.from_packed(wl.keys, wl.fids, K) as t:
        n_res = int(wl.offsets[-1])
        ws = kma.Workspace(0, n_res)
        res = torch.from_numpy(wl.residues).to(dev)
        off = torch.from_numpy(wl.offsets.view(np.int64)).to(dev)
        n = wl.n_seq
        outs = [torch.empty(n, dtype=d, device=dev) for d in (torch.int32, torch.int32, torch.uint8)]
        stream = torch.cuda.current_stream().cuda_stream
        ws.timing(True)
        for _ in range(3):
            kma.annotate_proteins_device(t, ws, res.data_ptr(), off.data_ptr(), n, n_res, 5, 0,
                                         *[o.data_ptr() for o in outs], 0, 0, stream)
        calls, probe_ms, vote_ms = ws.timing_read()
        assert calls == 3 and probe_ms > 0 and vote_ms > 0
        assert ws.timing_read()[0] == 0
        with pytest.raises(kma.KmerAnnoError) as e:  # reservation too small
            kma.annotate_proteins_device(t, ws, res.data_ptr(), off.data_ptr(), n, n_res + 1, 5,
                                         0, *[o.data_ptr() for o in outs], 0, 0, stream)
        assert e.value.code == kma.E_CAPACITY
        ws.close()


def test_contigs_device_api_planted_genome(kma, oracle_c):
    """kma_annotate_contigs_device on torch buffers over a synthetic config-3 genome (planted
    genes on both strands, 'n' bases, offsets[0] != 0): hits equal the oracle's in canonical
    order, the total is published even when it exceeds cap (hits past cap dropped), and the
    tally is accumulated into."""
    torch = pytest.importorskip("torch")
    from kmeranno import synth
    wl = synth.make_contig_workload(300_000, 6, 33, table_size=200_000, n_fid=500)
    kmers = [synth.unpack_key(x) for x in wl.keys]
    e = oracle_c.annotate_contigs(oracle_c.Table(kmers, wl.fids.astype(np.int32)), wl.dna,
                                  wl.offsets, 11, K)
    assert len(e[0]) > 1000
    dev = torch.device("cuda", 0)
    # shift the genome by 5 bytes so that d_offsets[0] != 0
    dna = np.concatenate([np.frombuffer(b"ggggg", np.uint8), wl.dna])
    off = wl.offsets + np.uint64(5)
    n_bases = int(off[-1] - off[0])
    with kma.SignatureTable.from_packed(wl.keys, wl.fids, K) as t:
        ws = kma.Workspace(0)
        ws.reserve_contigs(n_bases)
        d_dna = torch.from_numpy(dna).to(dev)
        d_off = torch.from_numpy(off.view(np.int64)).to(dev)
        stream = torch.cuda.current_stream().cuda_stream
        tally = torch.zeros(wl.n_contig * 500, dtype=torch.int32, device=dev)
        d_nh = torch.zeros(1, dtype=torch.int64, device=dev)
        for cap in (len(e[0]) + 7, 100):
            d_hits = torch.zeros(cap * kma.HIT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
            kma.annotate_contigs_device(t, ws, d_dna.data_ptr(), d_off.data_ptr(), wl.n_contig,
                                        n_bases, 11, d_hits.data_ptr(), cap, d_nh.data_ptr(),
                                        tally.data_ptr(), 500, stream)
            torch.cuda.synchronize()
            assert int(d_nh.item()) == len(e[0])
            hits = d_hits.cpu().numpy().view(kma.HIT_DTYPE)[:min(cap, len(e[0]))]
            n = len(hits)
            for a, b in zip((hits["contig"], hits["left"], hits["strand"], hits["frame"],
                             hits["fid"]), e):
                assert (a == b[:n]).all()
        expect = np.zeros((wl.n_contig, 500), np.int64)
        np.add.at(expect, (e[0], e[4]), 2)  # two calls accumulated
        assert (tally.cpu().numpy().reshape(wl.n_contig, 500) == expect).all()
        with pytest.raises(kma.KmerAnnoError) as err:  # reservation too small
            kma.annotate_contigs_device(t, ws, d_dna.data_ptr(), d_off.data_ptr(), wl.n_contig,
                                        n_bases + 10**6, 11, 0, 0, d_nh.data_ptr(),
                                        0, 0, stream)
        assert err.value.code == kma.E_CAPACITY
        ws.close()


@pytest.mark.parametrize("strict", [False, True])
def test_peg_connect_small_gto_vs_oracle(kma, oracle_c, small_gto, strict):
    """A9, KmerProcessor.java:195-207: singleton peg kmers of a close genome (small.gto's pegs,
    mutated 5%, plus exact copies of five pegs so that their kmers are no longer singletons,
    and an 'X' run) joined with the 6-frame kmer map of small.gto's contigs, AGGRESSIVE and
    STRICT: every (contig, left, strand, frame, peg) connection equals the oracle's."""
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
    close[3] = close[3][:40] + "XXX" + close[3][40:]
    close += prots[:5] + ["", "ACDEFGH", "ACDEFGHIK"]
    res, off = oracle_c.pack_strings(close)
    contigs = [c["dna"] for c in small_gto["contigs"]]
    dna, doff = oracle_c.pack_strings(contigs)
    e = oracle_c.peg_connect(res, off, dna, doff, 11, K, strict)
    assert len(e[0]) > 10_000
    t, n_win = kma.SignatureTable.from_pegs(res, off, K)
    assert n_win == sum(max(len(p) - K, 0) for p in close)
    with t:
        hits = kma.connect_pegs(t, dna, doff, 11, strict)
    assert len(hits) == len(e[0])
    for a, b in zip((hits["contig"], hits["left"], hits["strand"], hits["frame"], hits["fid"]), e):
        assert (a == b).all()
