"""GPU parity: libkmeranno.so (HIP, gfx950) against the oracle, bit-exact.

Apply outputs (fid, count, status) per protein and 6-frame hits (contig, left, strand,
frame, fid) must equal the CPU restatement's on the same inputs: the committed golden
vectors, hand-built edge cases, seeded synthetic workloads at the BASELINE config sizes
(c2: 10k proteins vs a 10^7 table; c5: 10^8 table, with a 20k-protein sample checked against
the oracle and the whole 1M batch by properties), under every table layout the library
builds (minimizer m = 6, m = 7, flat), and size-independent properties.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from helpers import restricted_oracle_table, take_proteins
from oracle import oracle_py

pytestmark = pytest.mark.gpu
K = 8


@pytest.fixture(params=["auto", "7", "0", "chained", "6"],
                ids=["m-auto", "m7", "flat", "chained", "m6-random"])
def layout(request, monkeypatch):
    """Table layouts: the size-derived minimizer layout (m = 6 up to 134M keys at load factor
    0.5; at K = 8 in the mod-sampling order, round 6), the m = 7 layout of larger tables, the
    flat fallback, and m = 6 in the smallest-hash order (the size rule's choice for K < 8, and
    before round 6 for every table; forced here) (the KMA_OPT_LAYOUT option, read per table
    creation), each with the default two-choice placement; and the size-derived layout with
    overflow chains (KMA_OPT_PLACEMENT = 0: the placement of wide tables and of a two-choice
    build that fails)."""
    import kmeranno
    kmeranno.load()
    p = request.param
    code = {"auto": -1, "chained": -1}.get(p)
    kmeranno.set_option(kmeranno.OPT_LAYOUT, int(p) if code is None else code)
    kmeranno.set_option(kmeranno.OPT_PLACEMENT, 0 if p == "chained" else -1)
    return p


@pytest.fixture(params=["direct", "defer"])
def path(request, monkeypatch):
    """Grids of the protein kernel: every group in block order (KMA_OPT_DEFER = 0), and the two-pass
    grid deferring groups of fewer than 2 probe steps (forced on every batch; automatic only
    for grids of 1-4 resident waves). The option is read per call."""
    import kmeranno
    kmeranno.load()
    kmeranno.set_option(kmeranno.OPT_DEFER, 0 if request.param == "direct" else 2)
    return request.param


@pytest.fixture(params=["packed", "ascii"])
def input_mode(request):
    """The protein kernel's input: residues packed to 5 bits first (KMA_OPT_PACKED_INPUT = 2:
    on the host while staging, or by the pack kernel for device calls of any size; the default 1
    packs device batches of >= 2^25 residues only), or ASCII packed by the probe itself through
    the LDS LUT (0)."""
    import kmeranno
    kmeranno.load()
    kmeranno.set_option(kmeranno.OPT_PACKED_INPUT, 2 if request.param == "packed" else 0)
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


def _oracle_apply(oracle_c, rows, prots, min_hits=5, flags=0):
    ids = _roles(rows)
    ot = oracle_c.Table([r[0] for r in rows], [ids[r[1]] for r in rows])
    res, off = oracle_c.pack_strings(prots)
    efid, ecnt, est = oracle_c.apply(ot, res, off, K, min_hits, flags)
    inv = {v: k for k, v in ids.items()}
    return [[int(s), inv.get(int(f)), int(n)] for f, n, s in zip(efid, ecnt, est)]


def test_edge_cases_golden(kma, layout, path, input_mode):
    for c in json.load(open(os.path.join(GOLDEN, "apply_edge.json"))):
        got = _gpu_apply(kma, [tuple(r) for r in c["rows"]], c["proteins"], c["min_hits"],
                         c["flags"])
        assert got == c["expected"], c["name"]


def _write_tsv(path, rows, crlf=False, trailing_newline=True):
    eol = "\r\n" if crlf else "\n"
    text = eol.join(k if r is None else f"{k}\t{r}" for k, r in rows)
    path.write_bytes((text + (eol if trailing_newline and rows else "")).encode())


@pytest.mark.parametrize("crlf,trailing", [(False, True), (True, True), (False, False)])
def test_table_from_tsv_edge_golden(kma, tmp_path, crlf, trailing):
    """kma_table_create_from_tsv (the library reads kmerdb.tbl itself, ApplyKmerProcessor.java:
    100-108) against the rows handed to kma_table_create: on every edge case of the golden file
    (duplicate kmers, last row wins; kmers of other lengths; foreign symbols; first-seen role
    order) the same roles in fid order, the same table counts and the same apply outputs
    (equal to the golden expectations); CRLF line ends, a missing final newline and a third
    column are read as TabbedLineReader reads them."""
    for c in json.load(open(os.path.join(GOLDEN, "apply_edge.json"))):
        rows = [tuple(r) for r in c["rows"]]
        f = tmp_path / f"{c['name']}.tbl"
        _write_tsv(f, [(k, f"{r}\tignored third column" if i % 2 else r)
                       for i, (k, r) in enumerate(rows)], crlf, trailing)
        t, roles, last = kma.SignatureTable.from_tsv(str(f), K)
        ids = _roles(rows)
        assert roles == list(ids) and last == len(rows[-1][0]), c["name"]
        with t, kma.SignatureTable.from_rows([r[0] for r in rows], [ids[r[1]] for r in rows],
                                             K) as ref:
            a, b = t.info, ref.info
            assert (a.n_rows, a.n_skipped, a.n_entries, a.n_extra_syms) == \
                (b.n_rows, b.n_skipped, b.n_entries, b.n_extra_syms), c["name"]
            res, off = kma.pack_strings(c["proteins"])
            got = kma.annotate_proteins(t, res, off, c["min_hits"], c["flags"])
            want = kma.annotate_proteins(ref, res, off, c["min_hits"], c["flags"])
            assert all((x == y).all() for x, y in zip(got[:3], want[:3])), c["name"]
        inv = dict(enumerate(roles))
        assert [[int(s), inv.get(int(fi)), int(n)] for fi, n, s in zip(*got[:3])] == \
            c["expected"], c["name"]


def test_table_from_tsv_rows_without_role_and_replicas(kma, tmp_path):
    """A row without a tab has the role "" (TabbedLineReader pads the missing column), empty
    lines are rows with an empty kmer (never matched); the table is replicated over the listed
    devices and answers like the single-device table; 100k rows parse over several chunks."""
    from kmeranno import synth
    wl = synth.make_workload(500, 100_000, 300, seed=43)
    kmers = [synth.unpack_key(x) for x in wl.keys]
    rows = [(k, f"ROLE{int(f):07d}") for k, f in zip(kmers, wl.fids)]
    rows[5] = (rows[5][0], None)
    rows[9] = ("", "ROLE0000001")
    f = tmp_path / "kmerdb.tbl"
    _write_tsv(f, rows)
    ids = {}
    for _, r in rows:
        ids.setdefault(r or "", len(ids))
    t, roles, last = kma.SignatureTable.from_tsv(str(f), K, devices=[0, 0])
    assert roles == list(ids) and last == 8 and t.replicas == [0, 0]
    with t, kma.SignatureTable.from_rows([r[0] for r in rows], [ids[r[1] or ""] for r in rows],
                                         K) as ref:
        assert t.info.n_skipped == 1 and t.info.n_entries == ref.info.n_entries
        got = kma.annotate_proteins(t, wl.residues, wl.offsets, 5, 0, n_fid=len(ids))
        want = kma.annotate_proteins(ref, wl.residues, wl.offsets, 5, 0, n_fid=len(ids))
        assert all((x == y).all() for x, y in zip(got, want))
        assert (got[2] == 1).sum() > 100


def test_table_info_and_alphabet(kma):
    rows = [("ACDEFGHI", 0), ("ACDEFGHI", 1), ("ACDEFGH", 2), ("ACDE-GHI", 1)]
    t = kma.SignatureTable.from_rows([r[0] for r in rows], [r[1] for r in rows], K)
    i = t.info
    assert (i.n_rows, i.n_skipped, i.n_entries, i.k) == (4, 1, 2, 8)
    assert i.n_extra_syms == 1 and i.extra_syms[0] == ord("-")
    assert i.n_replicas == 1 and t.replicas == [0]
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


@pytest.mark.parametrize("at", [0, 65_535, 65_536, 199_998])
def test_host_call_rejects_decreasing_offsets(kma, at):
    """The host entry checks the offsets in chunks on the staging pool: a decrease anywhere (in
    the first chunk, at a chunk's last or first offset, at the end) fails with its index, before
    anything is staged; the untouched offsets still run."""
    t = kma.SignatureTable.from_rows(["ACDEFGHI"], [0], K)
    res, off = kma.pack_strings(["ACDEFGHIK"] * 199_999)
    good = kma.annotate_proteins(t, res, off, 1)
    assert (good[2] == 1).all()
    bad = off.copy()
    bad[at] = bad[at + 1] + 1
    with pytest.raises(kma.KmerAnnoError) as e:
        kma.annotate_proteins(t, res, bad, 1)
    assert e.value.code == kma.E_INVALID and f"offsets decrease at {at}" in str(e.value)
    t.close()


@pytest.mark.parametrize("flags", [0, 1, 2])
def test_config1_golden(kma, layout, flags, path, input_mode):
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


@pytest.mark.parametrize("lf,flags", [(0.5, 0), (0.5, 1), (0.5, 2), (0.9, 0), (0.95, 0)])
def test_synthetic_vs_oracle(kma, oracle_c, layout, path, lf, flags, input_mode):
    """2,000 proteins vs a 200k-entry table (seeded), packed-key table path, load factors up
    to 0.95 (overflow chains and filter bits), both window conventions and multiset counting."""
    from kmeranno import synth
    wl = synth.make_workload(2000, 200_000, 2000, seed=11)
    kmers = [synth.unpack_key(x) for x in wl.keys]
    ot = oracle_c.Table(kmers, wl.fids.astype(np.int32))
    efid, ecnt, est = oracle_c.apply(ot, wl.residues, wl.offsets, K, 5, flags)
    with kma.SignatureTable.from_packed(wl.keys, wl.fids, K, load_factor=lf) as t:
        assert t.info.n_entries == ot.size
        if layout in ("7", "0"):
            assert t.info.minimizer_len == int(layout)
        elif layout == "6" and lf == 0.5:
            assert t.info.minimizer_len == 6 and t.info.minimizer_order == 0
        elif lf == 0.5:  # size rule, few displaced keys: m = 6, mod-sampling at K = 8
            assert t.info.minimizer_len == 6 and t.info.minimizer_order == 1
        if lf <= 0.9:
            assert t.info.two_choice == (0 if layout == "chained" else 1)
        if lf == 0.9:
            assert t.info.max_probe >= 2 and t.info.n_displaced > 0
        fid, cnt, st, _ = kma.annotate_proteins(t, wl.residues, wl.offsets, 5, flags)
    assert (st == est).all() and (fid == efid).all() and (cnt == ecnt).all()
    assert (st == 1).sum() > 500 and (st == 2).sum() > 50


@pytest.mark.parametrize("defer", ["64", "3", "1"])
def test_deferral_thresholds_and_repeated_calls(kma, oracle_c, monkeypatch, defer):
    """The direct kernel's two-pass grid: every group deferred to the second pass (64 steps),
    the automatic threshold (3) and none (1 step); calls in a row at block sizes 4, 1, 5, 7, 8
    and 6: each kernel capacity (K = 8: P = 4 for 1-4, 6 for 5-6, 8 for 7-8) with full and
    partial blocks."""
    from kmeranno import synth
    wl = synth.make_workload(9000, 200_000, 2000, seed=23)
    kmers = [synth.unpack_key(x) for x in wl.keys]
    ot = oracle_c.Table(kmers, wl.fids.astype(np.int32))
    efid, ecnt, est = oracle_c.apply(ot, wl.residues, wl.offsets, K, 5, 0)
    kma.set_option(kma.OPT_DEFER, int(defer))
    with kma.SignatureTable.from_packed(wl.keys, wl.fids, K) as t:
        for bp in ("4", "1", "5", "7", "8", "6"):
            kma.set_option(kma.OPT_BLOCK_PROTEINS, int(bp))
            fid, cnt, st, tally = kma.annotate_proteins(t, wl.residues, wl.offsets, 5, 0,
                                                        n_fid=2000)
            assert (st == est).all() and (fid == efid).all() and (cnt == ecnt).all()
            assert (tally == np.bincount(efid[est == 1], minlength=2000)).all()


def test_long_proteins_lds_and_workspace_sets(kma, oracle_c, layout, path, input_mode):
    """Proteins whose distinct-kmer sets do not fit the block's LDS pool keep them in workspace
    memory: long ones, and short ones behind a long one in the same block; duplicates inside
    them still count once."""
    rng = np.random.default_rng(3)
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    prots, rows = [], []
    for L, role in ((3000, "R1"), (6000, "R2"), (1700, "R3"), (2500, "R4"), (90, "R5"),
                    (2800, "R6"), (40, "R7"), (2900, "R8")):
        p = aa[rng.integers(0, 20, L)].tobytes().decode()
        p = p + p[:min(900, L)]  # repeated block: duplicate windows
        prots.append(p)
        rows += [(p[i:i + K], role) for i in range(0, len(p) - K + 1, 1 + (L % 3))]
    prots.append(prots[0][:1000] + prots[1][:1000])  # ambiguous long protein
    prots += [prots[4], prots[6], prots[2]]           # small ones after a long one
    rows.reverse()
    exp = _oracle_apply(oracle_c, rows, prots)
    assert max(e[2] for e in exp) > 1536
    assert _gpu_apply(kma, rows, prots) == exp


def test_giant_proteins_any_length(kma, oracle_c, path):
    """No length limit (ABI 1 returned TOO_LONG beyond 2^16 windows): proteins of 70k and
    200k residues with repeated blocks, one role and two roles, voted exactly."""
    rng = np.random.default_rng(17)
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    a = aa[rng.integers(0, 20, 50_000)].tobytes().decode()
    b = aa[rng.integers(0, 20, 150_000)].tobytes().decode()
    prots = [a + a[:20_000], b + b[:50_000], a[:30_000] + b[:40_000], "ACDEFGHIKLMN"]
    rows = [(a[i:i + K], "RA") for i in range(0, len(a) - K + 1, 2)]
    rows += [(b[i:i + K], "RB") for i in range(1, len(b) - K + 1, 3)]
    exp = _oracle_apply(oracle_c, rows, prots)
    assert exp[0][0] == 1 and exp[0][2] > 20_000 and exp[2][0] == 2
    assert _gpu_apply(kma, rows, prots) == exp


def test_empty_and_ragged_batches(kma, oracle_c, path):
    rows = [("ACDEFGHI", "R1"), ("CDEFGHIK", "R1")]
    prots = ["", "ACDEFGHIK", "", "A" * 7, "ACDEFGHIK" * 40, ""]
    assert _gpu_apply(kma, rows, prots, 1) == [
        list(oracle_py.apply_protein(oracle_py.load_table(rows), p, 1)) for p in prots]
    t = kma.SignatureTable.from_rows(["ACDEFGHI"], [0], K)
    res, off = kma.pack_strings([])
    fid, cnt, st, _ = kma.annotate_proteins(t, res, off, 5)
    assert len(st) == 0


def test_adversarial_minimizer_keys_fall_back_flat(kma, oracle_c, path):
    """Keys built to share a minimizer (every 8-mer holding one of 40 fixed 6-mers) pile onto
    a few home buckets under the minimizer layout; the creator rebuilds the table flat, and
    the answers stay exact."""
    rng = np.random.default_rng(23)
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)

    # the 40 lowest-hash 6-mers of 200k candidates: the minimizer of any 8-mer holding one
    cand = aa[rng.integers(0, 20, (200_000, 6))]
    packed = np.zeros(len(cand), np.uint64)
    for j in range(6):
        packed = (packed << np.uint64(5)) | (cand[:, j].astype(np.uint64) - np.uint64(64))
    # the minimizer order of kma_internal.h (KMA_HASH_LITE: a multiplicative hash of the 6-mer)
    h = (packed * np.uint64(0x9E3779B1)) & np.uint64(0xFFFFFFFF)
    cores = [cand[i].tobytes().decode() for i in np.argsort(h)[:40]]
    keys = set()
    for c in cores:
        for pos in range(3):
            for x in range(400):
                pre = "".join(chr(aa[(x // 20 ** i) % 20]) for i in range(pos))
                suf = "".join(chr(aa[(x // 20 ** (i + pos)) % 20]) for i in range(2 - pos))
                keys.add(pre + c + suf)
    keys = sorted(keys)
    rows = [(km, f"R{i % 50}") for i, km in enumerate(keys)]
    prots = ["".join(keys[j] for j in rng.integers(0, len(keys), 30)) for _ in range(200)]
    ids = _roles(rows)
    with kma.SignatureTable.from_rows([r[0] for r in rows], [ids[r[1]] for r in rows], K) as t:
        assert t.info.minimizer_len == 0, "crowded minimizer table must be rebuilt flat"
    assert _gpu_apply(kma, rows, prots) == _oracle_apply(oracle_c, rows, prots)


def test_replicated_table_host_fan_out(kma, oracle_c, path):
    """A table with 2 and 8 replicas (all on device 0 here: a host thread and stream per
    replica, the same code path as 8 GPUs) shards a host call by residues; outputs and the
    summed tally equal the single-replica call. Each replica's staging jobs get host_cores() / n
    threads (at most 16); the copies report as same-device ones. On a multi-GPU box, replicas on
    devices 0 and 1 too (peer copies)."""
    from kmeranno import synth
    wl = synth.make_workload(3000, 100_000, 500, seed=29)
    kmers = [synth.unpack_key(x) for x in wl.keys]
    with kma.SignatureTable.from_rows(kmers, wl.fids, K) as t1:
        ref = kma.annotate_proteins(t1, wl.residues, wl.offsets, 5, 0, n_fid=500)
    devsets = [[0, 0], [0] * 8] + ([[0, 1], [1, 0, 1]] if kma.device_count() > 1 else [])
    for devs in devsets:
        with kma.SignatureTable.from_rows_replicated(kmers, wl.fids, devs, K) as t:
            assert t.replicas == devs and t.info.n_replicas == len(devs)
            assert t.info.replicate_local == sum(d == devs[0] for d in devs[1:])
            for _ in range(2):  # second call reuses the pooled host contexts
                got = kma.annotate_proteins(t, wl.residues, wl.offsets, 5, 0, n_fid=500)
                for a, b in zip(got, ref):
                    assert (a == b).all()
            want = max(1, min(16, kma.host_cores() // len(devs)))
            assert all(kma.host_profile(i)["staging_threads"] == want for i in range(len(devs)))
    ot = oracle_c.Table(kmers, wl.fids.astype(np.int32))
    efid, ecnt, est = oracle_c.apply(ot, wl.residues, wl.offsets, K, 5, 0)
    assert (ref[2] == est).all() and (ref[0] == efid).all() and (ref[1] == ecnt).all()


@pytest.mark.parametrize("slice_res,devs", [(50_000, [0]), (137_777, [0, 0]), (1, [0])])
def test_host_call_slices_large_shares(kma, oracle_c, slice_res, devs):
    """A replica's share larger than KMA_OPT_HOST_SLICE residues (2^31 by default: the kernels
    index residues with 32 bits) is annotated as consecutive slices of whole proteins, one
    device call each, instead of being refused; outputs and the tally (summed over slices and
    replicas) equal the oracle's. Slice 1: every protein a call of its own."""
    from kmeranno import synth
    n = 300 if slice_res == 1 else 3000
    wl = synth.make_workload(n, 100_000, 500, seed=37)
    assert slice_res == 1 or wl.offsets[-1] > 4 * slice_res
    kmers = [synth.unpack_key(x) for x in wl.keys]
    with kma.SignatureTable.from_rows_replicated(kmers, wl.fids, devs, K) as t:
        with kma.options(host_slice=slice_res):
            fid, cnt, st, tally = kma.annotate_proteins(t, wl.residues, wl.offsets, 5, 0,
                                                        n_fid=500)
    ot = oracle_c.Table(kmers, wl.fids.astype(np.int32))
    efid, ecnt, est = oracle_c.apply(ot, wl.residues, wl.offsets, K, 5, 0)
    assert (st == est).all() and (fid == efid).all() and (cnt == ecnt).all()
    assert (tally == np.bincount(efid[est == 1], minlength=500)).all()
    assert (st == 1).sum() > 0.2 * n


def test_concurrent_host_callers(kma):
    """Concurrent host calls on one table (each takes its own pooled context and stream)."""
    import threading
    from kmeranno import synth
    wl = synth.make_workload(1500, 50_000, 300, seed=31)
    with kma.SignatureTable.from_packed(wl.keys, wl.fids, K) as t:
        ref = kma.annotate_proteins(t, wl.residues, wl.offsets, 5, 0, n_fid=300)
        errs = []

        def run():
            try:
                for _ in range(3):
                    got = kma.annotate_proteins(t, wl.residues, wl.offsets, 5, 0, n_fid=300)
                    assert all((a == b).all() for a, b in zip(got, ref))
            except Exception as e:  # noqa: BLE001 - collected for the main thread
                errs.append(e)

        th = [threading.Thread(target=run) for _ in range(4)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errs, errs


def _config_table(kma, sig, lf=0.5):
    return kma.SignatureTable.from_packed(sig.keys, sig.fids, K, load_factor=lf)


def test_config2_size_vs_oracle(kma, oracle_c, path, monkeypatch):
    """BASELINE configs[1] at full size: 10k proteins vs the 10^7-entry table, bit-exact
    against the oracle on the rows the batch can look up (tests/helpers.py). The direct case
    also runs the automatic choice (short groups deferred here, as bench.py runs it)."""
    from kmeranno import synth
    n_seq, t_size, n_fid, seed = synth.CONFIGS["c2"]
    sig = synth.make_table(t_size, n_fid, seed, K)
    res, off, kinds, true_fid = synth.make_queries(sig, n_seq, seed * 1_000_003 + 17)
    with _config_table(kma, sig) as t:
        assert t.info.n_buckets == 20_000_000 // kma.bucket_slots()
        assert t.info.minimizer_len == 6
        fid, cnt, st, tally = kma.annotate_proteins(t, res, off, 5, 0, n_fid=n_fid)
        if path == "direct":
            kma.set_option(kma.OPT_DEFER, -1)
            got = kma.annotate_proteins(t, res, off, 5, 0, n_fid=n_fid)
            for a, b in zip(got, (fid, cnt, st, tally)):
                assert (a == b).all()
    ot = restricted_oracle_table(oracle_c, sig.keys, sig.fids, res)
    efid, ecnt, est = oracle_c.apply(ot, res, off, K, 5, 0)
    assert (st == est).all() and (fid == efid).all() and (cnt == ecnt).all()
    assert (tally == np.bincount(efid[est == 1], minlength=n_fid)).all()
    assert (st == 1).sum() > 0.4 * n_seq


@pytest.mark.timeout(300)
@pytest.mark.parametrize("opts,pieces", [
    ({}, 2), ({"host_pieces": 16, "host_threads": 1, "host_piece_min": 1 << 20}, 16),
    ({"host_pieces": 3, "host_threads": 3, "host_piece_min": 1 << 20}, 3),
    ({"packed_input": 0}, 2), ({"packed_input": 0, "host_piece_min": 1 << 20}, 8),
    ({"packed_input": 0, "host_pieces": 5, "host_piece_min": 1 << 20}, 5)],
    ids=["default", "16pieces-1thread", "3pieces-3threads", "ascii", "ascii-8pieces",
         "ascii-5pieces"])
def test_host_call_pipelined_pieces_vs_oracle(kma, oracle_c, opts, pieces):
    """A host call of ~48M residues runs as 2-16 pieces whose H2D overlaps the previous
    piece's kernel (kma_abi.cpp protein_shard): packed input streamed out in segments as the
    staging pool packs it (the calling thread alone with one staging thread), ASCII input piece
    by piece (uneven pieces, weights 1, 2, 4, ..., 4, 2, 1, at 4 pieces and more): every protein,
    including those next to piece and segment boundaries, and the tally (summed over the pieces'
    launches) equal the oracle's. KMA_OPT_HOST_PIECE_MIN lowers the 16 MiB piece floor so that a
    48M-residue call runs the asked pieces; the library's host profile reports the count it ran
    (the piece cases used to run 2 pieces each)."""
    from kmeranno import synth
    sig = synth.make_table(1_000_000, 2000, 41, K)
    res, off, _, _ = synth.make_queries(sig, 160_000, 41 * 1_000_003 + 17)
    assert off[-1] >= 2 * (16 << 20)  # at least two pieces
    with _config_table(kma, sig) as t, kma.options(**opts):
        fid, cnt, st, tally = kma.annotate_proteins(t, res, off, 5, 0, n_fid=2000)
        prof = kma.host_profile()
    assert prof["pieces"] == pieces, prof
    if "host_threads" in opts:
        assert prof["staging_threads"] == opts["host_threads"]
    ot = restricted_oracle_table(oracle_c, sig.keys, sig.fids, res)
    efid, ecnt, est = oracle_c.apply_mt(ot, res, off, K, 5, 0, threads=8)
    assert (st == est).all() and (fid == efid).all() and (cnt == ecnt).all()
    assert (tally == np.bincount(efid[est == 1], minlength=2000)).all()


def test_contigs_golden(kma, layout):
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


@pytest.mark.parametrize("gcode,extra", [(11, 0), (4, 0), (11, 70)])
def test_contigs_small_gto_vs_oracle(kma, oracle_c, small_gto, layout, gcode, extra):
    """All five small.gto contigs plus boundary-length contigs, ambiguous bases and RNA 'u'/'U'
    bases: every 6-frame window hit equals the oracle's, and (AppTest.java:131-138) each hit's
    kmer is the translation of the DNA at its location. extra: that many short contigs more
    (past 64 contigs the kernel searches the offsets instead of caching them all)."""
    contigs = [c["dna"] for c in small_gto["contigs"]]
    contigs[2] = contigs[2][:50000] + "nnnNacgtRYk" + contigs[2][50000:]
    contigs += [contigs[0][100:100 + n] for n in range(20, 36)]  # 3K-4 .. 3K+11 bases
    contigs += [contigs[3][1000 * i:1000 * i + 40 + 37 * i] for i in range(extra)]
    # RNA bases: a stretch of contig 1 as is, with t -> u, and upper case with T -> U
    s = contigs[1][20000:26000]
    contigs += [s, s.replace("t", "u"), s.upper().replace("T", "U")]
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
    # the u/U contigs hit exactly like their t/T source, on both strands
    n = len(contigs)
    src = hits[hits["contig"] == n - 3]
    assert (src["strand"] == ord("-")).any() and (src["strand"] == ord("+")).any()
    for c in (n - 2, n - 1):
        got = hits[hits["contig"] == c]
        assert len(got) == len(src)
        for f in ("left", "strand", "frame", "fid"):
            assert (got[f] == src[f]).all()
    # property: translate(getDna(loc)) == kmer, for a sample of hits
    for h in hits[rng.choice(len(hits), 500, replace=False)]:
        seq = contigs[h["contig"]][h["left"] - 1:h["left"] - 1 + 3 * K]
        if h["strand"] == ord("-"):
            seq = oracle_py.reverse_complement(seq)
        assert oracle_py.translate(seq, 1, gcode) in tab.values()
    assert len(hits) > 100_000


@pytest.mark.parametrize("fill", [1.0, 0.98])
def test_two_choice_build_full_table_reports_or_places_every_key(kma, oracle_c, fill):
    """The two-choice build at (nearly) every slot used, where an insertion can run out of
    evictions: it either reports failure (status[0], the creators' cue to build chained) or
    has placed every row's key (entries = distinct keys, at most one probe beyond home, and
    every protein's vote equals the oracle's); at 98% the chained build of the same rows (the
    fallback) succeeds and votes the same. (At 100% a chained table has no empty slot to stop
    a miss's walk: not a table the creators build.)"""
    torch = pytest.importorskip("torch")
    from kmeranno import synth
    wl = synth.make_workload(1500, 60_000, 500, seed=41)
    dev = torch.device("cuda", 0)
    n_keys = len(np.unique(wl.keys))
    nb = int(np.ceil(n_keys / fill / kma.bucket_slots()))
    keys = torch.from_numpy(wl.keys.view(np.int64)).to(dev)
    fids = torch.from_numpy(wl.fids.view(np.int32)).to(dev)
    stream = torch.cuda.current_stream().cuda_stream
    kmers = [synth.unpack_key(x) for x in wl.keys]
    ot = oracle_c.Table(kmers, wl.fids.astype(np.int32))
    efid, ecnt, est = oracle_c.apply(ot, wl.residues, wl.offsets, K, 5, 0)
    m = kma.layout_for(K, nb) & 0xFF
    results = {}
    builds = [("two", m | kma.LAYOUT_TWO_CHOICE)] + ([("chained", m)] if fill < 1 else [])
    for name, code in builds:
        slots = torch.empty(nb * kma.bucket_slots(), dtype=torch.int64, device=dev)
        winner = torch.empty(nb * kma.bucket_slots(), dtype=torch.int32, device=dev)
        status = torch.zeros(4, dtype=torch.int32, device=dev)
        kma.build_device(slots.data_ptr(), nb, winner.data_ptr(), keys.data_ptr(),
                         fids.data_ptr(), len(wl.keys), status.data_ptr(), stream, layout=code)
        torch.cuda.synchronize()
        st = status.cpu().numpy()
        results[name] = st.tolist()
        if name == "two" and st[0] != 0:
            continue  # reported: a creator would build chained
        assert st[0] == 0 and st[1] == n_keys
        if name == "two":
            assert st[2] in (1, 2)
        with kma.SignatureTable.wrap_device(slots.data_ptr(), nb, K, 0, code) as t:
            fid, cnt, stt, _ = kma.annotate_proteins(t, wl.residues, wl.offsets, 5, 0)
        assert (stt == est).all() and (fid == efid).all() and (cnt == ecnt).all()
    print(f"fill {fill}: {nb} buckets, {n_keys} keys, status {results}")


def test_device_api_with_torch_buffers(kma):
    """_device entry points on torch-allocated HBM (the bench path), same results as host."""
    torch = pytest.importorskip("torch")
    from kmeranno import synth
    wl = synth.make_workload(3000, 100_000, 1000, seed=21)
    dev = torch.device("cuda", 0)
    nb = kma.buckets_for(len(wl.keys), 0.5)
    slots = torch.empty(nb * kma.bucket_slots(), dtype=torch.int64, device=dev)
    winner = torch.empty(nb * kma.bucket_slots(), dtype=torch.int32, device=dev)
    status = torch.zeros(4, dtype=torch.int32, device=dev)
    keys = torch.from_numpy(wl.keys.view(np.int64)).to(dev)
    fids = torch.from_numpy(wl.fids.view(np.int32)).to(dev)
    stream = torch.cuda.current_stream().cuda_stream
    kma.build_device(slots.data_ptr(), nb, winner.data_ptr(), keys.data_ptr(), fids.data_ptr(),
                     len(wl.keys), status.data_ptr(), stream)
    torch.cuda.synchronize()
    st4 = status.cpu().numpy()
    # layout -1 is kma_table_layout_for's code in both the build and the wrap (the
    # wrap used to read -1 as chained): two-choice placement at this size
    code = kma.layout_for(K, nb)
    assert code & kma.LAYOUT_TWO_CHOICE
    assert st4[0] == 0 and st4[1] == len(np.unique(wl.keys)) and st4[2] in (1, 2)
    t = kma.SignatureTable.wrap_device(slots.data_ptr(), nb, K, 0)
    assert t.info.minimizer_len == code & 0x3F and t.info.two_choice == 1
    # the same rows with overflow chains (the code without the two-choice flag) into a second
    # buffer, wrapped with that code
    chained = code & ~kma.LAYOUT_TWO_CHOICE
    slots2 = torch.empty_like(slots)
    status2 = torch.zeros(4, dtype=torch.int32, device=dev)
    kma.build_device(slots2.data_ptr(), nb, winner.data_ptr(), keys.data_ptr(), fids.data_ptr(),
                     len(wl.keys), status2.data_ptr(), stream, layout=chained)
    torch.cuda.synchronize()
    s2 = status2.cpu().numpy()
    assert s2[0] == 0 and s2[1] == st4[1] and s2[2] >= 1
    t2 = kma.SignatureTable.wrap_device(slots2.data_ptr(), nb, K, 0, chained)
    assert t2.info.two_choice == 0 and t2.info.minimizer_len == chained & 0x3F
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
    got2 = kma.annotate_proteins(t2, wl.residues, wl.offsets, 5, 0, n_fid=1000)
    for a, b in zip(got2, (hf, hc, hs, ht)):
        assert (a == b).all()
    t2.close()
    assert (fid.cpu().numpy() == hf).all() and (cnt.cpu().numpy() == hc).all()
    assert (st.cpu().numpy() == hs).all()
    assert (tally.cpu().numpy().astype(np.uint32) == ht).all()
    # a batch whose residues start at an odd offset (blocks' spans are unaligned anyway)
    k0 = 5
    kma.annotate_proteins_device(t, ws, res.data_ptr(), off.data_ptr() + 8 * k0, n - k0,
                                 int(wl.offsets[-1] - wl.offsets[k0]), 5, 0, fid.data_ptr(),
                                 cnt.data_ptr(), st.data_ptr(), 0, 0, stream)
    torch.cuda.synchronize()
    assert (fid.cpu().numpy()[:n - k0] == hf[k0:]).all()
    assert (st.cpu().numpy()[:n - k0] == hs[k0:]).all()
    ws.close()
    t.close()


@pytest.mark.parametrize("reserve", [0, 1000, 1 << 20])
def test_device_call_all_empty_proteins_packed(kma, reserve):
    """A device call whose proteins are all empty (n_residues = 0) under KMA_OPT_PACKED_INPUT = 2,
    on a workspace never reserved, reserved small, or reserved for a call that packs: every
    protein is NONE with count 0, and a packed call on the same workspace afterwards is
    bit-exact (the packed stream is allocated when a call first packs)."""
    torch = pytest.importorskip("torch")
    from kmeranno import synth
    wl = synth.make_workload(200, 20_000, 300, seed=33)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    n = 7
    off0 = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    res0 = torch.zeros(64, dtype=torch.uint8, device=dev)
    fid = torch.full((wl.n_seq,), -7, dtype=torch.int32, device=dev)
    cnt = torch.full((wl.n_seq,), -7, dtype=torch.int32, device=dev)
    st = torch.full((wl.n_seq,), 9, dtype=torch.uint8, device=dev)
    with kma.SignatureTable.from_packed(wl.keys, wl.fids, K) as t, kma.options(packed_input=2):
        ws = kma.Workspace(0, reserve) if reserve else kma.Workspace(0)
        kma.annotate_proteins_device(t, ws, res0.data_ptr(), off0.data_ptr(), n, 0, 5, 0,
                                     fid.data_ptr(), cnt.data_ptr(), st.data_ptr(), 0, 0, stream)
        torch.cuda.synchronize()
        assert (st.cpu().numpy()[:n] == kma.STATUS_NONE).all()
        assert (cnt.cpu().numpy()[:n] == 0).all()
        n_res = int(wl.offsets[-1])
        ws.reserve(n_res, wl.n_seq)
        res = torch.from_numpy(wl.residues).to(dev)
        off = torch.from_numpy(wl.offsets.view(np.int64)).to(dev)
        kma.annotate_proteins_device(t, ws, res.data_ptr(), off.data_ptr(), wl.n_seq, n_res, 5, 0,
                                     fid.data_ptr(), cnt.data_ptr(), st.data_ptr(), 0, 0, stream)
        torch.cuda.synchronize()
        hf, hc, hs, _ = kma.annotate_proteins(t, wl.residues, wl.offsets, 5, 0)
        assert (fid.cpu().numpy() == hf).all() and (cnt.cpu().numpy() == hc).all()
        assert (st.cpu().numpy() == hs).all()
        ws.close()


def test_workspace_timing(kma):
    """kma_workspace_timing: hipEvent durations of device calls (the pack kernel and the
    protein kernel; the protein kernel alone on ASCII input)."""
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
        calls, kernel_ms, rest_ms = ws.timing_read()
        assert calls == 3 and kernel_ms > 0 and rest_ms >= 0
        assert ws.timing_read()[0] == 0
        for _ in range(2):
            kma.annotate_proteins_device(t, ws, res.data_ptr(), off.data_ptr(), n, n_res, 5, 0,
                                         *[o.data_ptr() for o in outs], 0, 0, stream)
        calls, ph = ws.phases_read()  # small batch, default option: the ASCII probe only
        assert calls == 2 and list(ph) == ["annotate_kernel"]
        kma.set_option(kma.OPT_PACKED_INPUT, 2)
        for _ in range(2):
            kma.annotate_proteins_device(t, ws, res.data_ptr(), off.data_ptr(), n, n_res, 5, 0,
                                         *[o.data_ptr() for o in outs], 0, 0, stream)
        calls, ph = ws.phases_read()  # the pack kernel, then the probe (KMA_OPT_PACKED_INPUT 2)
        assert calls == 2 and list(ph) == ["pack_kernel", "annotate_kernel"]
        assert ph["annotate_kernel"] > 0 and ph["pack_kernel"] > 0
        kma.set_option(kma.OPT_PACKED_INPUT, 0)
        kma.annotate_proteins_device(t, ws, res.data_ptr(), off.data_ptr(), n, n_res, 5, 0,
                                     *[o.data_ptr() for o in outs], 0, 0, stream)
        calls, ph = ws.phases_read()
        assert calls == 1 and list(ph) == ["annotate_kernel"] and ph["annotate_kernel"] > 0
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
            # 16 guard records past cap stay untouched
            d_hits = torch.zeros((cap + 16) * kma.HIT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
            kma.annotate_contigs_device(t, ws, d_dna.data_ptr(), d_off.data_ptr(), wl.n_contig,
                                        n_bases, 11, d_hits.data_ptr(), cap, d_nh.data_ptr(),
                                        tally.data_ptr(), 500, stream)
            torch.cuda.synchronize()
            assert int(d_nh.item()) == len(e[0])
            assert not d_hits[cap * kma.HIT_DTYPE.itemsize:].any()
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


def test_contigs_device_graph_capture_replay(kma, oracle_c):
    """kma_annotate_contigs_device keeps no host state between calls (the emit pass's last
    block zeroes the group sums the probe added into), so one call captured in a hipGraph and
    replayed several times gives the oracle's hits and total every time, and the tally grows by
    one call's worth per replay."""
    torch = pytest.importorskip("torch")
    from kmeranno import synth
    wl = synth.make_contig_workload(300_000, 5, 57, table_size=200_000, n_fid=400)
    kmers = [synth.unpack_key(x) for x in wl.keys]
    e = oracle_c.annotate_contigs(oracle_c.Table(kmers, wl.fids.astype(np.int32)), wl.dna,
                                  wl.offsets, 11, K)
    dev = torch.device("cuda", 0)
    n_bases = int(wl.offsets[-1])
    with kma.SignatureTable.from_packed(wl.keys, wl.fids, K) as t:
        ws = kma.Workspace(0)
        ws.reserve_contigs(n_bases)
        d_dna = torch.from_numpy(wl.dna).to(dev)
        d_off = torch.from_numpy(wl.offsets.view(np.int64)).to(dev)
        cap = len(e[0]) + 3
        d_hits = torch.zeros(cap * kma.HIT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        d_nh = torch.zeros(1, dtype=torch.int64, device=dev)
        tally = torch.zeros(wl.n_contig * 400, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            kma.annotate_contigs_device(t, ws, d_dna.data_ptr(), d_off.data_ptr(), wl.n_contig,
                                        n_bases, 11, d_hits.data_ptr(), cap, d_nh.data_ptr(),
                                        tally.data_ptr(), 400,
                                        torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert int(d_nh.item()) == 0  # captured, not run
        for rep in range(1, 4):
            d_hits.zero_()
            d_nh.zero_()
            g.replay()
            torch.cuda.synchronize()
            assert int(d_nh.item()) == len(e[0]), rep
            hits = d_hits.cpu().numpy().view(kma.HIT_DTYPE)[:len(e[0])]
            for a, b in zip((hits["contig"], hits["left"], hits["strand"], hits["frame"],
                             hits["fid"]), e):
                assert (a == b).all(), rep
            expect = np.zeros((wl.n_contig, 400), np.int64)
            np.add.at(expect, (e[0], e[4]), rep)
            assert (tally.cpu().numpy().reshape(wl.n_contig, 400) == expect).all(), rep
        del g
        ws.close()


def test_contigs_device_many_groups_scanned(kma):
    """A device call of more than kDirectGroups x 256 probe blocks (> 268M bases at 1,024
    positions per block: the emit pass scans the group sums first instead of summing them per
    block) equals the same genome cut into calls below that size, hit for hit after re-basing,
    with the same total; then the whole call again on the same workspace."""
    torch = pytest.importorskip("torch")
    from kmeranno import synth
    wl = synth.make_contig_workload(2_000_000, 8, 77, table_size=300_000, n_fid=300)
    # 140 copies of the genome: 280 Mbp in 1,120 contigs (1,069 emit-offset groups of 256
    # probe blocks of 1,024 positions)
    reps = 140
    n0 = int(wl.offsets[-1])
    dna = np.concatenate([np.tile(wl.dna[:n0], reps), np.zeros(64, np.uint8)])
    off = np.concatenate([[0]] + [wl.offsets[1:] + np.uint64(i * n0) for i in range(reps)])
    off = off.astype(np.uint64)
    n_contig, n_bases = len(off) - 1, int(off[-1])
    assert n_bases > 1024 * 256 * 1024
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    with kma.SignatureTable.from_packed(wl.keys, wl.fids, K) as t:
        ws = kma.Workspace(0)
        ws.reserve_contigs(n_bases)
        d_dna = torch.from_numpy(dna).to(dev)
        d_nh = torch.zeros(1, dtype=torch.int64, device=dev)

        def call(lo, hi):
            sub = off[lo:hi + 1]
            d_off = torch.from_numpy(sub.view(np.int64)).to(dev)
            cap = 16_000_000
            d_hits = torch.zeros(cap * kma.HIT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
            kma.annotate_contigs_device(t, ws, d_dna.data_ptr(), d_off.data_ptr(), hi - lo,
                                        int(sub[-1] - sub[0]), 11, d_hits.data_ptr(), cap,
                                        d_nh.data_ptr(), 0, 0, stream)
            torch.cuda.synchronize()
            nh = int(d_nh.item())
            assert nh <= cap
            return d_hits.cpu().numpy().view(kma.HIT_DTYPE)[:nh].copy()

        whole = call(0, n_contig)
        per = len(wl.offsets) - 1
        pieces = []
        for i in range(reps):
            h = call(i * per, (i + 1) * per)
            h["contig"] += i * per
            pieces.append(h)
        again = call(0, n_contig)
        ws.close()
    cut = np.concatenate(pieces)
    assert len(whole) > 100_000 and len(whole) == len(cut)
    for f in ("contig", "left", "strand", "frame", "fid"):
        assert (whole[f] == cut[f]).all() and (again[f] == whole[f]).all()


def test_contigs_device_repeated_calls_of_different_sizes(kma, oracle_c):
    """One workspace, calls alternating between a whole genome and a prefix of its contigs (a
    different number of emit-offset groups): every call must start from clean group sums
    whatever the size of the call before it (the emit pass of each call zeroes them)."""
    torch = pytest.importorskip("torch")
    from kmeranno import synth
    wl = synth.make_contig_workload(400_000, 8, 41, table_size=200_000, n_fid=500)
    kmers = [synth.unpack_key(x) for x in wl.keys]
    ot = oracle_c.Table(kmers, wl.fids.astype(np.int32))
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    cases = []
    for nc in (wl.n_contig, 2, wl.n_contig, 1, 2, wl.n_contig):
        off = wl.offsets[:nc + 1]
        cases.append((nc, off, oracle_c.annotate_contigs(ot, wl.dna[:int(off[-1])], off, 11, K)))
    with kma.SignatureTable.from_packed(wl.keys, wl.fids, K) as t:
        ws = kma.Workspace(0)
        ws.reserve_contigs(int(wl.offsets[-1]))
        d_dna = torch.from_numpy(wl.dna).to(dev)
        d_nh = torch.zeros(1, dtype=torch.int64, device=dev)
        for nc, off, e in cases:
            d_off = torch.from_numpy(off.view(np.int64)).to(dev)
            cap = len(e[0]) + 1
            d_hits = torch.zeros(cap * kma.HIT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
            kma.annotate_contigs_device(t, ws, d_dna.data_ptr(), d_off.data_ptr(), nc,
                                        int(off[-1] - off[0]), 11, d_hits.data_ptr(), cap,
                                        d_nh.data_ptr(), 0, 0, stream)
            torch.cuda.synchronize()
            assert int(d_nh.item()) == len(e[0]), nc
            hits = d_hits.cpu().numpy().view(kma.HIT_DTYPE)[:len(e[0])]
            for a, b in zip((hits["contig"], hits["left"], hits["strand"], hits["frame"],
                             hits["fid"]), e):
                assert (a == b).all(), nc
        ws.close()


def test_contigs_replicated_host_fan_out(kma, oracle_c):
    """6-frame host calls on a two-replica table: contig shards, hits re-based and merged in
    canonical order, tally rows per shard; equal to the single-replica answer."""
    from kmeranno import synth
    wl = synth.make_contig_workload(400_000, 9, 41, table_size=200_000, n_fid=300)
    kmers = [synth.unpack_key(x) for x in wl.keys]
    with kma.SignatureTable.from_rows(kmers, wl.fids, K) as t1:
        h1, t1y = kma.annotate_contigs(t1, wl.dna, wl.offsets, 11, n_fid=300)
    with kma.SignatureTable.from_rows_replicated(kmers, wl.fids, [0, 0], K) as t2:
        h2, t2y = kma.annotate_contigs(t2, wl.dna, wl.offsets, 11, n_fid=300)
    assert (h1 == h2).all() and (t1y == t2y).all() and len(h1) > 1000


@pytest.mark.parametrize("strict", [False, True])
def test_peg_connect_small_gto_vs_oracle(kma, oracle_c, small_gto, layout, strict):
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


def test_packed_stream_device_entry_equals_ascii(kma, oracle_c):
    """kma_annotate_packed_device on a stream packed on the host (kma_pack_residues: the AVX2 /
    scalar packer, the table's codes, extra table symbols included) equals the ASCII kernel and
    the oracle on proteins holding bytes with no code (lower case, digits, 'X', '*', bytes >=
    128: their windows are probed as zero-group keys and miss), called on uneven sub-batches
    whose d_offsets[0] is not 0 (stream residue 0 = residue d_offsets[0])."""
    torch = pytest.importorskip("torch")
    from kmeranno import synth
    rng = np.random.default_rng(77)
    wl = synth.make_workload(3000, 150_000, 700, seed=12)
    res = wl.residues.copy()
    n_res = int(wl.offsets[-1])
    noise = rng.random(n_res) < 0.004
    res[:n_res][noise] = np.frombuffer(b"xq7X*-\xc3", np.uint8)[rng.integers(0, 7, int(noise.sum()))]
    kmers = [synth.unpack_key(x) for x in wl.keys]
    kmers[:40] = [k[:3] + "-" + k[4:] for k in kmers[:40]]  # an extra table symbol ('-')
    ot = oracle_c.Table(kmers, wl.fids.astype(np.int32))
    efid, ecnt, est = oracle_c.apply(ot, res, wl.offsets, K, 5, 0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    with kma.SignatureTable.from_rows(kmers, wl.fids, K) as t:
        assert t.info.n_extra_syms == 1
        ws = kma.Workspace(0, n_res)
        cuts = [0, 1, 2, 999, 1000, 2047, 3000]
        d_off = torch.from_numpy(wl.offsets.view(np.int64)).to(dev)
        outs = [torch.empty(wl.n_seq, dtype=d, device=dev) for d in (torch.int32, torch.int32, torch.uint8)]
        for lo, hi in zip(cuts[:-1], cuts[1:]):
            r0, r1 = int(wl.offsets[lo]), int(wl.offsets[hi])
            stream_h = kma.pack_residues(t, res[r0:r1])
            d_stream = torch.from_numpy(stream_h).to(dev)
            kma.annotate_packed_device(t, ws, d_stream.data_ptr(), d_off.data_ptr() + 8 * lo, hi - lo,
                                       r1 - r0, 5, 0, outs[0].data_ptr() + 4 * lo,
                                       outs[1].data_ptr() + 4 * lo, outs[2].data_ptr() + lo, 0, 0,
                                       stream)
        torch.cuda.synchronize()
        fid, cnt, st = (o.cpu().numpy() for o in outs)
        kma.set_option(kma.OPT_PACKED_INPUT, 0)
        afid, acnt, ast, _ = kma.annotate_proteins(t, res, wl.offsets, 5, 0)
        ws.close()
    assert (st == est).all() and (fid == efid).all() and (cnt == ecnt).all()
    assert (ast == est).all() and (afid == efid).all() and (acnt == ecnt).all()
    assert (st == 1).sum() > 500
