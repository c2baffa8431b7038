"""GPU parity at the sizes bench.py runs (BASELINE.json configs c3, c4, c5).

Every workload is the bench's own (same generator, same seeds, rank 0):
  c3  5 Mbp in 20 contigs (log-uniform 50 kb-1 Mbp, planted genes on both strands) against the
      10^7-row table: every 6-frame hit equals the oracle's (KmerReference.java:157-203), via
      the host entry point and the device entry point the bench times;
  c4  ONE 1M-protein batch against the 10^7-row table, cut into 8 residue-balanced shards the
      way the bench's strong-scaling run cuts it (kmeranno.dist.shard): the shards' outputs
      concatenated equal the whole-batch host call on a 4-replica table, the shard tallies sum
      to the called-fid histogram, and the whole batch is bit-exact vs the oracle
      (ApplyKmerProcessor.java:122-148);
  c5  the 1M-protein batch against the 10^8-row table at load factor 0.5 (the headline): the
      whole batch bit-exact vs the oracle, and whole-batch properties; at 0.9 (the layout the
      creator keeps at that load) equal to the 0.5 answer, plus a 20k sample vs the oracle.
Whole-batch checks load the full table into the oracle; sample checks use the rows the sample
can look up (tests/helpers.py).
"""
import os

import numpy as np
import pytest

from helpers import full_oracle_table, restricted_oracle_table, take_proteins, unpack_keys

pytestmark = pytest.mark.gpu
K = 8


@pytest.fixture(scope="module")
def kma(native_lib):
    import kmeranno
    assert kmeranno.device_count() >= 1
    return kmeranno


@pytest.fixture(scope="module")
def c5data():
    from kmeranno import synth
    n_seq, t_size, n_fid, seed = synth.CONFIGS["c5"]
    sig = synth.make_table(t_size, n_fid, seed, K)
    res, off, kinds, true_fid = synth.make_queries(sig, n_seq, seed * 1_000_003 + 17)
    print(f"c5 workload generated: {len(res)} residues", flush=True)
    return sig, res, off, kinds, true_fid


def _whole_batch_vs_oracle(oracle_c, sig, res, off, fid, cnt, st):
    """Every protein of the batch against the oracle (ApplyKmerProcessor.java:122-148 restated:
    the whole table in its String-keyed chained map), run on 16 host threads."""
    ot = full_oracle_table(oracle_c, sig.keys, sig.fids)
    threads = max(1, min(16, os.cpu_count() or 1))
    efid, ecnt, est = oracle_c.apply_mt(ot, res, off, K, 5, 0, threads)
    assert (st == est).all() and (fid == efid).all() and (cnt == ecnt).all()
    return est


def _sample_vs_oracle(oracle_c, sig, res, off, fid, cnt, st, n=20_000, seed=55):
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(len(off) - 1, n, replace=False))
    sres, soff = take_proteins(res, off, idx)
    ot = restricted_oracle_table(oracle_c, sig.keys, sig.fids, sres)
    efid, ecnt, est = oracle_c.apply(ot, sres, soff, K, 5, 0)
    assert (st[idx] == est).all() and (fid[idx] == efid).all() and (cnt[idx] == ecnt).all()
    return est


@pytest.mark.timeout(600)
def test_config5_size_sample_and_properties(kma, oracle_c, c5data, monkeypatch):
    """BASELINE configs[4]: the 10^8-entry table (1.5 GiB, m = 6 layout) and the 1M-protein
    batch. A random 20k-protein sample of the batch is bit-exact against the oracle; the whole
    batch is checked by properties: the two-pass grid and a second call on uneven shards
    (device entry point on pointer offsets) give identical outputs, the tally equals the
    called-fid histogram, and copies called are called for their own function."""
    torch = pytest.importorskip("torch")
    sig, res, off, kinds, true_fid = c5data
    n_seq, n_fid = len(off) - 1, sig.n_fid
    dev = torch.device("cuda", 0)
    with kma.SignatureTable.from_packed(sig.keys, sig.fids, K) as t:
        assert t.info.minimizer_len == 6 and t.info.n_buckets == 200_000_000 // kma.bucket_slots()
        assert t.info.minimizer_order == 1  # round 6: mod-sampling (K = 8, m = 6)
        assert t.info.n_entries > 0.99 * len(sig.keys)
        fid, cnt, st, tally = kma.annotate_proteins(t, res, off, 5, 0, n_fid=n_fid)
        # property 0: the two-pass grid gives the same outputs on the whole batch
        kma.set_option(kma.OPT_DEFER, 3)
        got = kma.annotate_proteins(t, res, off, 5, 0, n_fid=n_fid)
        for a, b in zip(got, (fid, cnt, st, tally)):
            assert (a == b).all()
        kma.set_option(kma.OPT_DEFER, -1)
        # property 1: the same batch cut into uneven shards through the device entry point
        d_res = torch.from_numpy(res).to(dev)
        d_off = torch.from_numpy(off.view(np.int64)).to(dev)
        d_fid = torch.empty(n_seq, dtype=torch.int32, device=dev)
        d_cnt = torch.empty(n_seq, dtype=torch.int32, device=dev)
        d_st = torch.empty(n_seq, dtype=torch.uint8, device=dev)
        ws = kma.Workspace(0, int(off[-1]))
        stream = torch.cuda.current_stream().cuda_stream
        cuts = [0, 1, 7, 4096, 333_333, 500_001, 999_999, n_seq]
        for lo, hi in zip(cuts[:-1], cuts[1:]):
            kma.annotate_proteins_device(t, ws, d_res.data_ptr(), d_off.data_ptr() + 8 * lo,
                                         hi - lo, int(off[hi] - off[lo]), 5, 0,
                                         d_fid.data_ptr() + 4 * lo, d_cnt.data_ptr() + 4 * lo,
                                         d_st.data_ptr() + lo, 0, 0, stream)
        torch.cuda.synchronize()
        assert (d_fid.cpu().numpy() == fid).all() and (d_cnt.cpu().numpy() == cnt).all()
        assert (d_st.cpu().numpy() == st).all()
        ws.close()
    # property 2: tally = histogram of called fids; copies called carry their own function
    assert (tally == np.bincount(fid[st == 1], minlength=n_fid)).all()
    copies = (kinds == 0) & (st == 1)
    assert copies.sum() > 0.2 * n_seq  # decoy hits make many copies AMBIGUOUS at 10^8
    assert (fid[copies] == true_fid[copies]).mean() > 0.999
    # the whole 1M-protein batch bit-exact against the oracle (round 3: a 20k sample)
    _whole_batch_vs_oracle(oracle_c, sig, res, off, fid, cnt, st)


@pytest.mark.timeout(600)
def test_config5_load_factor_09(kma, oracle_c, c5data, monkeypatch):
    """c5 at load factor 0.9 (10^8 keys in 1.39e7 buckets: long overflow chains): the table
    the creator keeps (its layout rule, kma_abi.cpp create_from_device_keys) answers a 20k
    sample bit-exactly and the whole batch exactly like the LF 0.5 table and like the 0.9
    tables of the other layouts."""
    sig, res, off, _, _ = c5data
    n_fid = sig.n_fid
    kma.set_option(kma.OPT_LAYOUT, -1)
    with kma.SignatureTable.from_packed(sig.keys, sig.fids, K) as t:
        ref = kma.annotate_proteins(t, res, off, 5, 0, n_fid=n_fid)
    with kma.SignatureTable.from_packed(sig.keys, sig.fids, K, load_factor=0.9) as t:
        i = t.info
        kept = i.minimizer_len
        print(f"LF 0.9: layout m={kept} two-choice={i.two_choice}, displaced "
              f"{i.n_displaced / i.n_entries:.2%}, longest probe {i.max_probe}", flush=True)
        assert i.n_buckets == kma.buckets_for(len(sig.keys), 0.9)
        # two-choice placement at the size rule's m = 6: every key in its home or its alt bucket
        assert i.two_choice == 1 and kept == 6 and i.max_probe == 2
        assert i.n_displaced > 0.02 * i.n_entries
        got = kma.annotate_proteins(t, res, off, 5, 0, n_fid=n_fid)
    for a, b in zip(got, ref):
        assert (a == b).all()
    with kma.options(placement=0):  # chains: m = 6 displaces ~24% -> rebuilt m = 7 (~17%)
        with kma.SignatureTable.from_packed(sig.keys, sig.fids, K, load_factor=0.9) as t:
            i = t.info
            assert i.two_choice == 0 and i.minimizer_len == 7 and i.max_probe >= 2
            chained = kma.annotate_proteins(t, res, off, 5, 0, n_fid=n_fid)
    for a, b in zip(chained, ref):
        assert (a == b).all()
    fid, cnt, st, tally = got
    assert (tally == np.bincount(fid[st == 1], minlength=n_fid)).all()
    _sample_vs_oracle(oracle_c, sig, res, off, fid, cnt, st, seed=91)
    for m in {"0", "6", "7"} - {str(kept)}:
        kma.set_option(kma.OPT_LAYOUT, int(m))
        with kma.SignatureTable.from_packed(sig.keys, sig.fids, K, load_factor=0.9) as t:
            assert t.info.minimizer_len == int(m)
            other = kma.annotate_proteins(t, res, off, 5, 0, n_fid=n_fid)
        for a, b in zip(other, ref):
            assert (a == b).all()


@pytest.mark.timeout(600)
def test_config4_shards_vs_whole_batch_and_oracle(kma, oracle_c):
    """BASELINE configs[3] at full size: one 1M-protein batch x the 10^7-row table. The bench's
    strong-scaling cut (kmeranno.dist.shard, 8 residue-balanced shards) through the device
    entry point equals the whole-batch host call on a table with 4 replicas (4 host threads,
    4 streams: the ABI's own residue-balanced fan-out), shard tallies sum to the called-fid
    histogram, and a 20k-protein sample is bit-exact against the oracle."""
    torch = pytest.importorskip("torch")
    from kmeranno import dist as kdist
    from kmeranno import synth
    n_seq, t_size, n_fid, seed = synth.CONFIGS["c4"]
    sig = synth.make_table(t_size, n_fid, seed, K)
    res, off, _, _ = synth.make_queries(sig, n_seq, seed * 1_000_003 + 17)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    with kma.SignatureTable.from_packed(sig.keys, sig.fids, K) as t:
        t.replicate([0, 0, 0])
        assert t.replicas == [0, 0, 0, 0]
        fid, cnt, st, tally = kma.annotate_proteins(t, res, off, 5, 0, n_fid=n_fid)
        bounds = kdist.shard_bounds(off, 8)
        ws = kma.Workspace(0, int(max(off[b1] - off[b0] for b0, b1 in zip(bounds[:-1], bounds[1:]))))
        d_tally = torch.zeros(n_fid, dtype=torch.int32, device=dev)
        parts = []
        for r in range(8):
            sres, soff, lo = kdist.shard(res, off, 8, r)
            n = len(soff) - 1
            assert lo == bounds[r] and n == bounds[r + 1] - bounds[r]
            d_res = torch.from_numpy(sres).to(dev)
            d_off = torch.from_numpy(soff.view(np.int64)).to(dev)
            outs = [torch.empty(n, dtype=d, device=dev) for d in (torch.int32, torch.int32, torch.uint8)]
            kma.annotate_proteins_device(t, ws, d_res.data_ptr(), d_off.data_ptr(), n,
                                         int(soff[-1]), 5, 0, *[o.data_ptr() for o in outs],
                                         d_tally.data_ptr(), n_fid, stream)
            torch.cuda.synchronize()
            parts.append([o.cpu().numpy() for o in outs])
        ws.close()
    for got, whole in zip(zip(*parts), (fid, cnt, st)):
        assert (np.concatenate(got) == whole).all()
    assert (d_tally.cpu().numpy().astype(np.uint32) == tally).all()
    assert (tally == np.bincount(fid[st == 1], minlength=n_fid)).all()
    assert (st == 1).sum() > 0.4 * n_seq
    _whole_batch_vs_oracle(oracle_c, sig, res, off, fid, cnt, st)


@pytest.mark.timeout(600)
def test_config3_bench_size_vs_oracle(kma, oracle_c):
    """BASELINE configs[2] as bench.py runs it: the 5 Mbp, 20-contig genome with planted genes
    against the 10^7-row table. Every 6-frame hit (contig, left, strand, frame, fid) equals the
    oracle's, through the host call and through the device call the bench times (with the
    per-contig tally)."""
    torch = pytest.importorskip("torch")
    from kmeranno import synth
    n_fid = 10_000
    wl = synth.make_contig_workload(5_000_000, 20, 3, 10_000_000, n_fid, K)
    km, _, _, _, _ = oracle_c.contig_kmers(wl.dna, wl.offsets, 11, K)
    keep = np.isin(wl.keys, np.unique(kma.pack_std(km)))
    rows = unpack_keys(wl.keys[keep], K)
    ot = oracle_c.Table.from_buffer(rows.tobytes(), np.arange(len(rows) + 1, dtype=np.uint64) * K,
                                    wl.fids[keep].astype(np.int32))
    e = oracle_c.annotate_contigs(ot, wl.dna, wl.offsets, 11, K)
    assert len(e[0]) > 100_000
    with kma.SignatureTable.from_packed(wl.keys, wl.fids, K) as t:
        hits, tally = kma.annotate_contigs(t, wl.dna, wl.offsets, 11, n_fid=n_fid)
        dev = torch.device("cuda", 0)
        n_bases = int(wl.offsets[-1])
        ws = kma.Workspace(0)
        ws.reserve_contigs(n_bases)
        d_dna = torch.from_numpy(wl.dna).to(dev)
        d_off = torch.from_numpy(wl.offsets.view(np.int64)).to(dev)
        cap = len(e[0]) + 16
        d_hits = torch.zeros(cap * kma.HIT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        d_nh = torch.zeros(1, dtype=torch.int64, device=dev)
        d_tally = torch.zeros(wl.n_contig * n_fid, dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream().cuda_stream
        kma.annotate_contigs_device(t, ws, d_dna.data_ptr(), d_off.data_ptr(), wl.n_contig,
                                    n_bases, 11, d_hits.data_ptr(), cap, d_nh.data_ptr(),
                                    d_tally.data_ptr(), n_fid, stream)
        torch.cuda.synchronize()
        dhits = d_hits.cpu().numpy().view(kma.HIT_DTYPE)[:int(d_nh.item())]
        ws.close()
    for a, d, b in zip((hits["contig"], hits["left"], hits["strand"], hits["frame"], hits["fid"]),
                       (dhits["contig"], dhits["left"], dhits["strand"], dhits["frame"],
                        dhits["fid"]), e):
        assert (a == b).all() and (d == b).all()
    expect = np.zeros((wl.n_contig, n_fid), np.uint32)
    np.add.at(expect, (e[0], e[4]), 1)
    assert (tally == expect).all()
    assert (d_tally.cpu().numpy().reshape(wl.n_contig, n_fid).astype(np.uint32) == expect).all()
