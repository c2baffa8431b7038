"""The FASTA form of apply (`kma apply-fasta`, SURVEY.md §8(b): protein FASTA read as
FastaInputStream reads it, anno/BuildKmerProcessor.java:196-198).

CPU tests: the C++ reader (host/fasta.cpp, through `kma fasta-dump`) against the Python
restatement of the reader rules (oracle/fasta_reader.py) on hand-built edge cases and seeded
random files, at segment sizes from 1 byte (a segment per record) to the whole file; usage
errors. GPU tests: VERIFY and APPLY reports of synthetic FASTA files against the oracle's calls
(oracle/kma_oracle.c, ApplyKmerProcessor.java:122-147) with the reporters' rules
(rep/VerifyApplyKmerReporter.java:32-45, rep/DefaultApplyKmerReporter.java:43-55). The reader
rules themselves are parity unpinned (FastaInputStream is not in /root/reference)."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG
from oracle import fasta_reader

KMA = os.path.join(PKG, "build", "kma")


@pytest.fixture(scope="module")
def kma_bin():
    if not os.path.exists(KMA):
        subprocess.run(["make", "-s", "-C", PKG, "build/kma"], check=True)
    return KMA


EDGE = [
    b"",
    b"no header at all\nACDEF\n",
    b">only\n",
    b">a\nACDEF",                                      # no final newline
    b"junk line\n>a desc here\nACDE\nFGH\n\n>b\n",        # junk before the first header, blank
    b">a  two spaces\nAC\n>b\tx\ty\nKL\n",                 # comment after ONE separator
    b">a x\r\nACDE\r\nFG\r\n>b\r\nMM\r\n",                 # CRLF
    b">a x\rACDE\rFG\r>b\rMM\r",                           # lone CR (BufferedReader.readLine)
    b">a\nAC>DE\n>b\n",                                   # '>' inside a sequence line
    b"> lead space\nAC\n>\nQQ\n",                          # empty labels
    b">a\nac de*X\n>b\n\n\n>c\nWY",                        # case, spaces, '*', blank records
    b">a\n\r\nAC\n\r>b\n",
]


def _dump(kma_bin, path, batch):
    """The C++ reader's records as `label<TAB>comment<TAB>sequence` lines."""
    r = subprocess.run([kma_bin, "fasta-dump", "--batch", str(batch), str(path)],
                       capture_output=True)
    assert r.returncode == 0, r.stderr
    return r.stdout.split(b"\n")[:-1]


def _expect(data):
    return [b"\t".join(rec) for rec in fasta_reader.read_fasta(data)]


@pytest.mark.parametrize("case", range(len(EDGE)))
def test_fasta_reader_edge_cases(kma_bin, tmp_path, case):
    data = EDGE[case]
    path = tmp_path / "x.faa"
    path.write_bytes(data)
    exp = _expect(data)
    for batch in (1, 2, 5, 16, 1 << 24):
        assert _dump(kma_bin, path, batch) == exp, (batch, exp)


def test_fasta_reader_random_files(kma_bin, tmp_path):
    """Seeded random FASTA-like files (headers, CR / LF / CRLF terminators, blank lines, '>' in
    lines, junk before the first header): the segmented C++ reader equals the restatement at
    segment sizes 1 .. whole file."""
    rng = np.random.default_rng(2024)
    alphabet = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWYacgt*X> ", np.uint8)
    terms = [b"\n", b"\r\n", b"\r"]
    for trial in range(12):
        parts = [b"junk\n"] if trial % 3 == 0 else []
        for r in range(int(rng.integers(1, 40))):
            t = terms[int(rng.integers(0, 3))] if trial % 2 else b"\n"
            parts.append(b">id%d desc %d%s" % (r, int(rng.integers(0, 1000)), t))
            for _ in range(int(rng.integers(0, 5))):
                n = int(rng.integers(0, 70))
                line = alphabet[rng.integers(0, len(alphabet) - 2, n)].tobytes()
                if rng.random() < 0.1:
                    line = line[:n // 2] + b">" + line[n // 2:]
                parts.append(line + t)
        data = b"".join(parts)
        if trial % 4 == 1:
            data = data.rstrip(b"\r\n")
        path = tmp_path / f"r{trial}.faa"
        path.write_bytes(data)
        exp = _expect(data)
        assert len(exp) >= 1
        for batch in (1, 7, 100, 1000, 1 << 24):
            assert _dump(kma_bin, path, batch) == exp, (trial, batch)


def test_fasta_writer_roundtrip(tmp_path):
    """synth.write_fasta (the bench's FASTA writer) reads back as written."""
    from kmeranno import synth
    sig = synth.make_table(50_000, 100, 9, 8)
    res, off, _, _ = synth.make_queries(sig, 500, 11)
    ids = [f"fig|1.1.peg.{i}" for i in range(500)]
    com = [f"role {i}" if i % 3 else "" for i in range(500)]
    path = tmp_path / "w.faa"
    n = synth.write_fasta(str(path), res, off, ids, com, width=60)
    data = path.read_bytes()
    assert n == len(data)
    recs = fasta_reader.read_fasta(data)
    assert [r[0].decode() for r in recs] == ids
    assert [r[1].decode() for r in recs] == com
    assert [r[2] for r in recs] == [res[int(off[i]):int(off[i + 1])].tobytes() for i in range(500)]


def test_apply_fasta_errors(kma_bin, tmp_path):
    (tmp_path / "db.tbl").write_text("ACDEFGHI\tR1\n")
    (tmp_path / "roles").write_text("R1\tx\n")
    r = subprocess.run([kma_bin, "apply-fasta", str(tmp_path / "db.tbl"), str(tmp_path / "roles"),
                        str(tmp_path / "missing.faa")], capture_output=True, text=True)
    assert r.returncode == 1 and "Input FASTA file" in r.stderr and "not found" in r.stderr
    (tmp_path / "p.faa").write_text(">a\nACDEFGHI\n")
    r = subprocess.run([kma_bin, "apply-fasta", "-m", "0", str(tmp_path / "db.tbl"),
                        str(tmp_path / "roles"), str(tmp_path / "p.faa")],
                       capture_output=True, text=True)
    assert r.returncode == 2 and "Min-hits must be positive." in r.stderr
    r = subprocess.run([kma_bin, "apply-fasta", str(tmp_path / "db.tbl"), str(tmp_path / "roles")],
                       capture_output=True, text=True)
    assert r.returncode == 2 and "proteins.faa" in r.stderr
    r = subprocess.run([kma_bin, "apply-fasta", "-h"], capture_output=True, text=True)
    assert r.returncode == 0 and "apply-fasta" in r.stderr


# ---- GPU: reports vs the oracle ----------------------------------------------------------------

def _fasta_inputs(tmp_path, oracle_c, n_files=3, n_seq=3000, n_fid=300):
    from kmeranno import synth
    sig = synth.make_table(300_000, n_fid, 21, 8)
    synth.write_kmer_db(str(tmp_path / "db.tbl"), sig.keys, sig.fids)
    synth.write_roles_in_use(str(tmp_path / "roles"), n_fid, every=2)
    kmers = [synth.unpack_key(x) for x in sig.keys]
    ot = oracle_c.Table(kmers, sig.fids.astype(np.int32))
    col = {synth.role_name(i): j for j, i in enumerate(range(0, n_fid, 2))}
    fdir = tmp_path / "faa"
    fdir.mkdir()
    files = []
    for f in range(n_files):
        res, off, _, true_fid = synth.make_queries(sig, n_seq, 77 + f)
        if f == 1:  # edge records: empty, shorter than K, exactly K
            extra = [b"", b"ACDE", res[int(off[0]):int(off[0]) + 8].tobytes()]
            ext = np.frombuffer(b"".join(extra), np.uint8)
            res = np.concatenate([res[:int(off[-1])], ext])
            off = np.concatenate([off, off[-1] + np.cumsum([len(e) for e in extra]).astype(np.uint64)])
            true_fid = np.concatenate([true_fid, [-1, -1, -1]])
        n = len(off) - 1
        gid = f"{500 + f}.{f + 1}"
        ids = [f"fig|{gid}.peg.{i + 1}" for i in range(n)]
        com = [synth.role_name(int(t)) if t >= 0 else "hypothetical protein" for t in true_fid]
        synth.write_fasta(str(fdir / f"{gid}.faa"), res, off, ids, com, width=60 + 13 * f)
        fid, cnt, st = oracle_c.apply(ot, res, off, 8, 5, 0)
        files.append((gid, ids, com, fid, cnt, st))
    verify = ["genome_id\tpeg_id\trole\thits\tfunction"]
    apply = []
    for gid, ids, com, fid, cnt, st in files:
        counts = [0] * len(col)
        for i in np.flatnonzero(st == 1):
            role = synth.role_name(int(fid[i]))
            verify.append(f"{gid}\t{ids[i]}\t{role}\t{int(cnt[i])}\t{com[i]}")
            if role in col:
                counts[col[role]] += 1
        apply.append(gid + "\t" + "\t".join(map(str, counts)))
    return fdir, files, verify, apply


@pytest.mark.gpu
@pytest.mark.parametrize("threads,batch", [(16, 1 << 24), (4, 20_000), (1, 1 << 40)])
def test_apply_fasta_reports(kma_bin, oracle_c, native_lib, tmp_path, threads, batch):
    """3 FASTA files of 3,000 synthetic proteins (line widths 60 / 73 / 86; edge records: empty,
    shorter than K, exactly K) as a directory: VERIFY rows and APPLY tally rows equal the
    oracle's, in file order, whether a file is one segment or ~50 concurrent calls."""
    fdir, files, verify, apply = _fasta_inputs(tmp_path, oracle_c)
    assert len(verify) > 1000
    base = [kma_bin, "apply-fasta", "--threads", str(threads), "--batch", str(batch),
            str(tmp_path / "db.tbl"), str(tmp_path / "roles")]
    out = subprocess.run(base + [str(fdir)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.splitlines() == verify
    stats = json.loads([ln for ln in out.stderr.splitlines() if "apply-fasta-stats" in ln][0]
                       .split("apply-fasta-stats ", 1)[1])
    assert stats["files"] == 3 and stats["sequences"] == sum(len(f[1]) for f in files)
    assert stats["called"] == len(verify) - 1
    if batch == 20_000:
        assert stats["segments"] > 30
    out = subprocess.run(base[:2] + ["--format", "APPLY"] + base[2:] +
                         [str(fdir / f"{f[0]}.faa") for f in files],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.splitlines() == apply
