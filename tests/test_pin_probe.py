"""The one-command pin of the unpinned external semantics: the committed
expectation tests/golden/pin/expected.txt is exactly what this build's rules predict for the
fixtures scripts/PinProteinKmers.java reads, and the build itself follows those rules on them:
  KMERS  the oracle's ProteinKmers restatement (inclusive windows, a set) and the C oracle agree
         with the expectation, and the probe reads each line of proteins.txt;
  FASTA  the native reader (`kma fasta-dump`) reads edge.faa as the expectation says;
  PEGS   the GTO order rule (features array, pegs only).
The Java side cannot run here (no JDK, no org.theseed jars): parity of these three stays
unpinned until a maintainer runs scripts/pin_external_semantics.sh."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

PIN = os.path.join(ROOT, "tests", "golden", "pin")


def _expected():
    return open(os.path.join(PIN, "expected.txt")).read().splitlines()


def test_expected_matches_assumed_rules():
    sys.path.insert(0, PIN)
    import make_expected
    assert make_expected.expected_lines() == _expected()


def test_kmers_lines_match_c_oracle(oracle_c):
    """The C oracle (the bit-exact checker of the GPU path) counts every KMERS line's distinct
    kmers as the expectation does: a one-role table of those kmers calls the protein with
    count = the set's size."""
    for line in _expected():
        if not line.startswith("KMERS"):
            continue
        _, prot, n, kmers = line.split("\t")
        want = kmers.split(",") if kmers else []
        assert int(n) == len(want) == len(set(want))
        if not want:
            continue
        ot = oracle_c.Table(want, [0] * len(want))
        res, off = oracle_c.pack_strings([prot])
        fid, cnt, st = oracle_c.apply(ot, res, off, 8, 1, 0)
        assert (int(st[0]), int(fid[0]), int(cnt[0])) == (1, 0, int(n)), prot


@pytest.fixture(scope="module")
def kma_bin(native_lib):
    pkg = os.path.join(ROOT, "kmers.anno_amd")
    path = os.path.join(pkg, "build", "kma")
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-C", pkg, "build/kma"], check=True)
    return path


def test_fasta_lines_match_native_reader(kma_bin):
    """`kma fasta-dump` (the native FASTA reader apply-fasta uses; no device needed) reads the
    probe's edge-case file exactly as the expectation's FASTA lines say."""
    got = subprocess.run([kma_bin, "fasta-dump", os.path.join(PIN, "edge.faa")],
                         capture_output=True, timeout=60)
    assert got.returncode == 0, got.stderr
    want = [ln.split("\t", 1)[1] for ln in _expected() if ln.startswith("FASTA")]
    assert got.stdout.decode().splitlines() == want


def test_probe_source_prints_what_the_expectation_holds():
    src = open(os.path.join(ROOT, "scripts", "PinProteinKmers.java")).read()
    for tag in ("\"KMERS\\t\"", "\"FASTA\\t\"", "\"PEGS\\t\""):
        assert tag in src
    kinds = [ln.split("\t")[0] for ln in _expected()]
    assert kinds.count("KMERS") == len(open(os.path.join(PIN, "proteins.txt")).read().split("\n")) - 1
    assert kinds[-1] == "PEGS"
