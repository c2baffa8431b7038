"""The C-ABI library loads and exports every symbol include/kmeranno.h declares (CPU only:
no compute calls; only the pure host helpers are exercised)."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def header_functions():
    src = open(os.path.join(ROOT, "include", "kmeranno.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kma_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    import kmeranno
    assert header_functions() == sorted(kmeranno.EXPORTS)


def test_library_exports_every_declared_symbol(native_lib):
    for name in header_functions():
        assert hasattr(native_lib, name), name


def test_abi_version_and_error_string(native_lib):
    assert native_lib.kma_abi_version() == 7
    assert isinstance(native_lib.kma_last_error(), bytes)


def test_options_set_get_validate_restore(native_lib):
    """Tuning options go through the ABI (kma_option_set / _get), not the environment: defaults,
    range checks (KMA_E_INVALID, value unchanged), the context manager restores, and the
    library ignores the old environment variables (a plain build has no KMA_TUNING_ENV)."""
    import kmeranno as k
    for o, v in k.OPT_DEFAULTS.items():
        assert k.get_option(o) == v
    for o, bad in ((k.OPT_LAYOUT, 5), (k.OPT_BLOCK_PROTEINS, 9), (k.OPT_DEFER, 65),
                   (k.OPT_HOST_PIECES, 17), (k.OPT_HASH_SLICE, -1), (k.OPT_PACKED_INPUT, 3),
                   (k.OPT_HOST_THREADS, 65), (k.OPT_HOST_SLICE, -1), (k.OPT_PLACEMENT, 2),
                   (k.OPT_HOST_SLICE, 1 << 32), (k.OPT_HOST_PIECE_MIN, -1), (k.OPT_LAYOUT, 7 | 0x40),
                   (11, 1),
                   (99, 0)):
        with pytest.raises(k.KmerAnnoError) as e:
            k.set_option(o, bad)
        assert e.value.code == k.E_INVALID
    with k.options(layout=6 | k.LAYOUT_MOD_SAMPLING):
        assert k.layout_for(8, 1000) == 6 | k.LAYOUT_MOD_SAMPLING | k.LAYOUT_TWO_CHOICE
        assert k.layout_for(7, 1000) == 6 | k.LAYOUT_TWO_CHOICE  # mod-sampling: K = 8 only
    with k.options(layout=7, block_proteins=1, defer=0, host_pieces=3, hash_slice=1000,
                   packed_input=0, host_threads=4, host_slice=12345, placement=0,
                   host_piece_min=1 << 20):
        assert [k.get_option(o) for o in range(1, 11)] == [7, 1, 0, 3, 1000, 0, 4, 12345, 0,
                                                           1 << 20]
        assert k.layout_for(8, 1000) == 7
    assert [k.get_option(o) for o in range(1, 11)] == [-1, 0, -1, 0, 0, 1, 0, 0, -1, 0]
    assert k.layout_for(8, 1000) == 6 | k.LAYOUT_MOD_SAMPLING | k.LAYOUT_TWO_CHOICE
    assert k.layout_for(7, 1000) == 6 | k.LAYOUT_TWO_CHOICE
    src = open(os.path.join(ROOT, "kmers.anno_amd", "csrc", "kma_abi.cpp")).read()
    assert src.count("getenv(") == 1 and "#if KMA_TUNING_ENV" in src


def test_bucket_sizing_host_helper(native_lib):
    import kmeranno
    s = kmeranno.bucket_slots()
    assert s in (8, 16)
    assert kmeranno.buckets_for(1000, 0.5) == 2000 // s
    assert kmeranno.buckets_for(10**8, 0.75) * s >= 10**8 / 0.75
    assert kmeranno.buckets_for(0, 0.5) == 1
    # wide tables (K 9..12): four 16-byte slots per 64-byte bucket
    assert kmeranno.bucket_slots(8) == s and kmeranno.bucket_slots(12) == 4
    assert kmeranno.bucket_slots(13) == 0 and kmeranno.bucket_slots(0) == 0
    assert kmeranno.buckets_for(1000, 0.5, k=10) == 500


def test_contig_window_count_matches_oracle(native_lib, oracle_c, small_gto):
    """kma_contig_window_count = sum over strands/frames of max(0, P_f - K) (processKmers)."""
    import kmeranno
    contigs = [c["dna"] for c in small_gto["contigs"]]
    _, off = kmeranno.pack_strings(contigs)
    assert kmeranno.contig_window_count(off, 8) == 1_537_176
    for L in range(0, 40):
        o = np.array([0, L], np.uint64)
        expect = sum(2 * max(0, (L - f + 1) // 3 - 8) for f in (1, 2, 3))
        assert kmeranno.contig_window_count(o, 8) == expect, L


def test_table_layout_host_helper(native_lib, monkeypatch):
    """Layout choice: minimizer m = 6 up to 134M keys at load factor 0.5 (2^28 slots), m = 7
    beyond; K = 8, m = 6 tables in the mod-sampling order (round 6: first only beyond the 256
    MiB Infinity Cache, then every size); the KMA_OPT_LAYOUT option forces 0 (flat), 6 / 7 (the
    smallest-hash order) or 6 | mod-sampling, read per call. Narrow tables are tried with
    two-choice placement first (the layout code's flag) unless KMA_OPT_PLACEMENT = 0; wide
    tables never."""
    import kmeranno
    tc, mod = kmeranno.LAYOUT_TWO_CHOICE, kmeranno.LAYOUT_MOD_SAMPLING
    kmeranno.set_option(kmeranno.OPT_LAYOUT, -1)
    nb6 = (1 << 28) // kmeranno.bucket_slots()
    cache = (256 << 20) // (8 * kmeranno.bucket_slots())  # buckets of the Infinity Cache
    assert kmeranno.layout_for(8, nb6) == 6 | mod | tc
    assert kmeranno.layout_for(8, cache + 1) == 6 | mod | tc
    assert kmeranno.layout_for(8, cache) == 6 | mod | tc
    assert kmeranno.layout_for(8, kmeranno.buckets_for(10**7)) == 6 | mod | tc  # c2 / c4
    assert kmeranno.layout_for(8, kmeranno.buckets_for(10**8)) == 6 | mod | tc  # c5
    assert kmeranno.layout_for(8, 1000) == 6 | mod | tc
    assert kmeranno.layout_for(7, nb6) == 6 | tc  # mod-sampling: K = 8 only
    assert kmeranno.layout_for(8, nb6 + 1) == 7 | tc
    assert kmeranno.layout_for(5, 1 << 30) == 5 | tc  # m <= K
    assert kmeranno.layout_for(10, 1000) == 6  # wide: chains
    with kmeranno.options(placement=0):
        assert kmeranno.layout_for(8, nb6) == 6 | mod
    kmeranno.set_option(kmeranno.OPT_LAYOUT, 0)
    assert kmeranno.layout_for(8, 1000) == 0 | tc
    kmeranno.set_option(kmeranno.OPT_LAYOUT, 7)
    assert kmeranno.layout_for(8, 1000) == 7 | tc
    kmeranno.set_option(kmeranno.OPT_LAYOUT, 6)  # the smallest-hash order, forced
    assert kmeranno.layout_for(8, 1000) == 6 | tc
    kmeranno.set_option(kmeranno.OPT_LAYOUT, -1)


def test_choose_layout_rule():
    """kmeranno.choose_layout mirrors the creators' rule (kma_abi.cpp create_from_device_keys).
    Two-choice placement first: kept when it builds (the size rule's m), rebuilt flat when more
    than 40% of the keys are outside their home and flat halves them; a minimizer build that fails
    is retried flat. A failed two-choice build falls back to the chained rule, shown on the round-3 c5 sweep's build statistics {full,
    entries, longest chain, displaced}: m = 6 kept at load factor 0.5, rebuilt m = 7 at 0.75 and
    0.9 (flat halves neither), flat for keys piling onto few minimizers; the kept layout is built
    last."""
    import kmeranno
    tc = kmeranno.LAYOUT_TWO_CHOICE
    n = 99_821_868
    six = 6 | kmeranno.LAYOUT_MOD_SAMPLING  # the size rule's m = 6 code at K = 8 (round 6)
    assert kmeranno.layout_for(8, 25_000_000) == six | tc
    sweep = {  # load factor -> layout -> status
        0.5: {six: [0, n, 10, int(0.0770 * n)], 7: [0, n, 7, int(0.0239 * n)], 0: [0, n, 6, int(0.0086 * n)]},
        0.75: {six: [0, n, 24, int(0.1706 * n)], 7: [0, n, 19, int(0.0936 * n)], 0: [0, n, 17, int(0.0607 * n)]},
        0.9: {six: [0, n, 47, int(0.2449 * n)], 7: [0, n, 39, int(0.1675 * n)], 0: [0, n, 38, int(0.1309 * n)]},
        "adv": {six: [0, 1506982, 290, 1490000], 7: [0, 1506982, 145, 1012000], 0: [0, 1506982, 5, 13000]},
    }
    want = {0.5: six, 0.75: 7, 0.9: 7, "adv": 0}
    for case, st in sweep.items():
        built = []

        def build(m):
            built.append(m)
            return [1, 0, 0, 0] if m & tc else st[m]  # the two-choice build fails
        m, s = kmeranno.choose_layout(8, 25_000_000, build)
        assert built[0] == six | tc
        assert m == want[case] and built[-1] == m and s == st[m], (case, built)
    two = {six | tc: [0, n, 2, int(0.21 * n)], tc: [0, n, 2, int(0.05 * n)]}
    for disp6, expect in ((0.21, six | tc), (0.45, tc), (0.45 - 1, six | tc)):
        built = []
        two[six | tc][3] = int(disp6 * n) if disp6 > 0 else int(0.45 * n)
        if disp6 < 0:  # crowded, but flat does not halve the displaced keys
            two[tc][3] = int(0.30 * n)

        def build2(m):
            built.append(m)
            return two[m]
        m, s = kmeranno.choose_layout(8, 25_000_000, build2)
        assert m == expect and built[-1] == m and s == two[m], (disp6, built)
    # the minimizer two-choice build runs out of evictions (keys piling onto few minimizers):
    # retried flat with two-choice placement, kept when that builds, chains only after both fail
    built = []

    def build3(m):
        built.append(m)
        return [1, 0, 0, 0] if m == six | tc else [0, n, 2, int(0.12 * n)]
    m, s = kmeranno.choose_layout(8, 25_000_000, build3)
    assert m == tc and built == [six | tc, tc] and s[0] == 0


def _pack_reference(res: np.ndarray) -> np.ndarray:
    """The packed stream spelled out bit by bit (include/kmeranno.h): residue j's standard code
    at big-endian stream bits [5j, 5j + 5)."""
    from kmeranno import std_codes
    codes = std_codes(res).astype(np.uint8)
    bits = ((codes[:, None] >> np.arange(4, -1, -1, dtype=np.uint8)) & 1).reshape(-1)
    return np.packbits(bits)  # MSB first, zero-padded to a byte



def test_pack_residues_staging_pool_concurrent(native_lib):
    """Large streams are packed on the library's staging pool (chunks of 2^15 groups): four
    Python threads packing at once (ctypes releases the GIL, so their jobs share the pool) get
    the same streams as one-thread packing (KMA_OPT_HOST_THREADS = 1: the caller alone)."""
    import threading
    import kmeranno
    rng = np.random.default_rng(7)
    alphabet = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY*x", np.uint8)
    arrays = [alphabet[rng.integers(0, len(alphabet), (1 << 23) + 777 * i)] for i in range(4)]
    with kmeranno.options(host_threads=1):
        want = [kmeranno.pack_residues(None, a) for a in arrays]
    got = [None] * 4
    errors = []

    def run(i):
        try:
            for _ in range(3):
                got[i] = kmeranno.pack_residues(None, arrays[i])
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append(e)

    threads = [threading.Thread(target=run, args=(i,)) for i in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors and not any(t.is_alive() for t in threads)
    assert all(np.array_equal(g, w) for g, w in zip(got, want))
    head = _pack_reference(arrays[0][:1 << 16])  # the pool's first chunk against the format
    assert np.array_equal(want[0][:len(head)], head)


@pytest.mark.parametrize("shift", [0, 8, 20, 40])
@pytest.mark.parametrize("n", [511, 512, 4096, 4096 + 520, 100_003])
def test_pack_residues_output_alignment(native_lib, n, shift):
    """kma_pack_residues writes 64-byte aligned outputs in 512-residue blocks by non-temporal
    stores (then the overlapping-store AVX2 steps and the scalar tail) and other outputs by the
    overlapping stores alone: the same stream, no byte written past out_cap."""
    import kmeranno
    rng = np.random.default_rng(n + shift)
    pool = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWYXZ*az-\xff", np.uint8)
    res = pool[rng.integers(0, len(pool), n)]
    need = kmeranno.packed_bytes(n)
    raw = np.full(need + 256, 0xEE, np.uint8)
    base = (-raw.ctypes.data) % 64 + shift  # 64-byte aligned + shift
    out = raw[base:base + need]
    rc = kmeranno.load().kma_pack_residues(None, res, n, out, need)
    assert rc == 0
    want = _pack_reference(res)
    assert (out[:len(want)] == want).all() and not out[len(want):].any()
    assert (raw[:base] == 0xEE).all() and (raw[base + need:] == 0xEE).all()


@pytest.mark.parametrize("n", [0, 1, 7, 8, 9, 63, 64, 65, 200, 4096 + 37, 100_003])
def test_pack_residues_host_matches_bitwise_reference(native_lib, n):
    """kma_pack_residues (AVX2 body + scalar tail, chosen by the CPU) against a bitwise numpy
    spelling of the format, on residues with every byte class: A-Z, '*', lower case, digits,
    bytes >= 128 (no code: a zero group); the padding after the stream is zero."""
    import kmeranno
    rng = np.random.default_rng(n)
    pool = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWYBJOUXZ*az09-\xff\x80", np.uint8)
    res = pool[rng.integers(0, len(pool), n)]
    got = kmeranno.pack_residues(None, res)
    want = _pack_reference(res)
    assert len(got) == kmeranno.packed_bytes(n) == 40 * ((n + 63) // 64) + 16
    assert (got[:len(want)] == want).all() and not got[len(want):].any()


@pytest.mark.parametrize("k,code,ok", [
    (8, 6, True), (8, 7, True), (8, 0, True), (8, 6 | 0x40, True), (8, 6 | 0x40 | 0x100, True),
    (8, -1, True), (7, 6 | 0x40, False), (8, 7 | 0x40, False), (8, 5, False), (8, 0x200, False),
    (10, 6 | 0x100, False), (10, 6, True), (8, 0x80 | 6, False)])
def test_layout_code_validation(native_lib, k, code, ok):
    """kma_table_wrap_device checks its layout code before it touches a device: minimizer
    0 / min(K, 6) / min(K, 7), the mod-sampling order only at K = 8, m = 6, two-choice only for
    K <= 8, no unknown bits (KMA_E_INVALID); a valid code gets as far as the device (KMA_E_DEVICE
    here, no GPU). -1 resolves to kma_table_layout_for's code (build and wrap agree)."""
    import ctypes as C
    import kmeranno
    h = C.c_void_p()
    rc = kmeranno.load().kma_table_wrap_device(C.c_void_p(4096), 1000, k, code, 0, C.byref(h))
    if ok:
        assert rc in (kmeranno.E_DEVICE, kmeranno.OK)
        if rc == kmeranno.OK:
            kmeranno.load().kma_table_destroy(h)
    else:
        assert rc == kmeranno.E_INVALID


def test_host_cores_bounded_by_cgroup_quota(native_lib):
    """The library sizes its staging jobs by the process's CPUs: the affinity mask, bounded by a
    cgroup CPU quota when one is set (a GPU box grants a share of a machine whose every CPU the
    mask lists)."""
    import kmeranno
    n = kmeranno.host_cores()
    assert 1 <= n <= len(os.sched_getaffinity(0))
    quota = None
    if os.path.exists("/sys/fs/cgroup/cpu.max"):
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else -(-int(q) // int(p))
    elif os.path.exists("/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        quota = -(-q // p) if q > 0 else None
    assert n == min(len(os.sched_getaffinity(0)), quota or 1 << 30)


def test_table_from_tsv_host_errors(native_lib, tmp_path):
    """kma_table_create_from_tsv reads the file before any device work: a missing file is
    KMA_E_IO (apply's FileNotFoundException), more than 4 symbols outside [A-Z*] in K-length
    kmers KMA_E_ALPHABET (kma_table_create's rule), a bad K KMA_E_INVALID."""
    import kmeranno
    with pytest.raises(kmeranno.KmerAnnoError) as e:
        kmeranno.SignatureTable.from_tsv(str(tmp_path / "missing.tbl"))
    assert e.value.code == kmeranno.E_IO
    bad = tmp_path / "alpha.tbl"
    bad.write_text("".join(f"AAAAAAA{c}\tR{i}\n" for i, c in enumerate("abcde")))
    with pytest.raises(kmeranno.KmerAnnoError) as e:
        kmeranno.SignatureTable.from_tsv(str(bad))
    assert e.value.code == kmeranno.E_ALPHABET
    with pytest.raises(kmeranno.KmerAnnoError) as e:
        kmeranno.SignatureTable.from_tsv(str(bad), k=13)
    assert e.value.code == kmeranno.E_INVALID
