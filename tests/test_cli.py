"""The C++ host `kma apply` (mirror of ApplyKmerProcessor + its reporters) end to end on the
reference's own genome fixture small.gto. Expected reports are built here from the oracle's
per-protein calls with the reporters' rules (rep/DefaultApplyKmerReporter.java:43-55,
rep/VerifyApplyKmerReporter.java:32-45). Error-path tests need no GPU."""
import gzip
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PKG

KMA = os.path.join(PKG, "build", "kma")


@pytest.fixture(scope="module")
def kma_bin(native_lib):
    if not os.path.exists(KMA):
        subprocess.run(["make", "-s", "-C", PKG, "build/kma"], check=True)
    return KMA


@pytest.fixture(scope="module")
def apply_inputs(tmp_path_factory, small_gto):
    d = tmp_path_factory.mktemp("apply")
    gdir = d / "gtos"
    gdir.mkdir()
    with gzip.open(os.path.join(GOLDEN, "small.gto.gz"), "rb") as f, \
            open(gdir / "97478.30.gto", "wb") as o:
        shutil.copyfileobj(f, o)
    pegs = [f for f in small_gto["features"] if f["type"] == "CDS"]
    rng = np.random.default_rng(17)
    rows = []
    for i, f in enumerate(pegs[:300]):
        p = f["protein_translation"]
        for j in rng.choice(len(p) - 7, 12, replace=False):
            rows.append((p[j:j + 8], f"ROLE{i % 60:03d}"))
    rows.append((pegs[5]["protein_translation"][:8], "ROLE999"))  # makes peg 5 ambiguous
    rows.append(("ACDEFGH", "ROLE001"))  # wrong length: loaded, never matches
    with open(d / "kmerdb.tbl", "w") as f:
        f.writelines(f"{k}\t{r}\n" for k, r in rows)
    roles = [f"ROLE{i:03d}" for i in range(0, 60, 2)] + ["ROLE999"]
    with open(d / "roles.in.use", "w") as f:
        f.writelines(f"{r}\tsome role name {r}\n" for r in roles)
    return d, rows, roles, pegs


def _expected(oracle_c, small_gto, rows, roles, pegs, min_hits):
    ids = {}
    for _, r in rows:
        ids.setdefault(r, len(ids))
    inv = {v: k for k, v in ids.items()}
    t = oracle_c.Table([r[0] for r in rows], [ids[r[1]] for r in rows])
    res, off = oracle_c.pack_strings([f.get("protein_translation", "") for f in pegs])
    fid, cnt, st = oracle_c.apply(t, res, off, 8, min_hits, 0)
    col = {r: i for i, r in enumerate(roles)}
    counts = [0] * len(roles)
    verify = ["genome_id\tpeg_id\trole\thits\tfunction"]
    gid = small_gto["id"]
    for f, fi, c, s in zip(pegs, fid, cnt, st):
        if s == 1:
            role = inv[int(fi)]
            if role in col:
                counts[col[role]] += 1
            verify.append(f"{gid}\t{f['id']}\t{role}\t{int(c)}\t{f.get('function', '')}")
    apply = [gid + "\t" + "\t".join(map(str, counts))]
    return apply, verify


@pytest.mark.gpu
@pytest.mark.parametrize("min_hits", [5, 2])
def test_kma_apply_reports(kma_bin, oracle_c, small_gto, apply_inputs, min_hits):
    d, rows, roles, pegs = apply_inputs
    exp_apply, exp_verify = _expected(oracle_c, small_gto, rows, roles, pegs, min_hits)
    assert sum(int(x) for x in exp_apply[0].split("\t")[1:]) > 20
    args = [kma_bin, "apply", "-m", str(min_hits), str(d / "kmerdb.tbl"),
            str(d / "roles.in.use"), str(d / "gtos")]
    out = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.splitlines() == exp_apply
    out = subprocess.run(args[:2] + ["--format", "VERIFY"] + args[2:], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.splitlines() == exp_verify


@pytest.mark.gpu
@pytest.mark.parametrize("threads,batch", [(6, 0), (1, 1), (4, 500_000), (8, 1 << 40)])
def test_kma_apply_genome_directory_batched(kma_bin, oracle_c, tmp_path, threads, batch):
    """`kma apply` over a directory of 14 synthetic GTOs (600 pegs each, a contig of DNA the
    loader skips): GTOs parsed ahead by a thread pool; batch 0: every parse
    worker makes its own genome's native call (concurrent host calls on one table); batch > 0:
    consecutive genomes batched on the report thread into one native call of >= `batch`
    residues (1: a call per genome, as round 3; 500k: several genomes per call; 2^40: one
    call for the directory). APPLY and VERIFY reports equal the oracle-derived reports line
    for line, genomes in file-name order
    (ApplyKmerProcessor.java:116-151, rep/DefaultApplyKmerReporter.java:43-55)."""
    from kmeranno import synth
    sig = synth.make_table(200_000, 400, 5, 8)
    gdir = tmp_path / "gtos"
    genomes = synth.write_genome_dir(str(gdir), sig, 14, 600, seed=3, contig_bp=20_000)
    synth.write_kmer_db(str(tmp_path / "db.tbl"), sig.keys, sig.fids)
    synth.write_roles_in_use(str(tmp_path / "roles"), 400, every=3)
    kmers = [synth.unpack_key(x) for x in sig.keys]
    ot = oracle_c.Table(kmers, sig.fids.astype(np.int32))
    col = {synth.role_name(i): j for j, i in enumerate(range(0, 400, 3))}
    exp_apply, exp_verify = [], ["genome_id\tpeg_id\trole\thits\tfunction"]
    for gid, res, off in genomes:
        fid, cnt, st = oracle_c.apply(ot, res, off, 8, 5, 0)
        counts = [0] * len(col)
        for i in np.flatnonzero(st == 1):
            role = synth.role_name(int(fid[i]))
            if role in col:
                counts[col[role]] += 1
        exp_apply.append(gid + "\t" + "\t".join(map(str, counts)))
        _, _, _, true_fid = synth.make_queries(sig, 600, 3 * 7919 + int(gid.split(".")[0]) - 100000)
        for i in np.flatnonzero(st == 1):
            fn = synth.role_name(int(true_fid[i])) if true_fid[i] >= 0 else "hypothetical protein"
            exp_verify.append(f"{gid}\tfig|{gid}.peg.{i + 1}\t{synth.role_name(int(fid[i]))}\t"
                              f"{int(cnt[i])}\t{fn}")
    args = [kma_bin, "apply", "--threads", str(threads), "--batch", str(batch),
            str(tmp_path / "db.tbl"), str(tmp_path / "roles"), str(gdir)]
    out = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.splitlines() == exp_apply
    stats = [ln for ln in out.stderr.splitlines() if "apply-stats" in ln]
    assert len(stats) == 1
    st = json.loads(stats[0].split("apply-stats ", 1)[1])
    assert st["genomes"] == 14 and st["proteins"] == 14 * 600
    if batch in (0, 1):
        assert st["calls"] == 14
        assert st["calls_on"] == ("parse workers" if batch == 0 else "caller thread")
    elif batch == 1 << 40:
        assert st["calls"] == 1
    else:
        assert 1 < st["calls"] < 14
    out = subprocess.run(args[:2] + ["--format", "VERIFY"] + args[2:], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.splitlines() == exp_verify


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [0, 1, 1 << 24])
def test_kma_apply_corrupt_gto_mid_directory(kma_bin, oracle_c, tmp_path, batch):
    """A GTO that fails to parse in the middle of the directory: every genome before it is
    reported (as the reference's in-order loop does before its exception,
    ApplyKmerProcessor.java:116-151), then the command fails naming the file; in every call
    mode (a call per parse worker, a call per genome, one batch holding all of them)."""
    from kmeranno import synth
    sig = synth.make_table(100_000, 200, 6, 8)
    gdir = tmp_path / "gtos"
    genomes = synth.write_genome_dir(str(gdir), sig, 8, 300, seed=4)
    synth.write_kmer_db(str(tmp_path / "db.tbl"), sig.keys, sig.fids)
    synth.write_roles_in_use(str(tmp_path / "roles"), 200, every=1)
    bad = gdir / f"{genomes[5][0]}.gto"
    bad.write_text(bad.read_text()[:5000])  # truncated JSON
    ot = oracle_c.Table([synth.unpack_key(x) for x in sig.keys], sig.fids.astype(np.int32))
    exp = []
    for gid, res, off in genomes[:5]:
        fid, _, st = oracle_c.apply(ot, res, off, 8, 5, 0)
        counts = np.bincount(fid[st == 1], minlength=200)
        exp.append(gid + "\t" + "\t".join(map(str, counts.tolist())))
    out = subprocess.run([kma_bin, "apply", "--batch", str(batch), str(tmp_path / "db.tbl"),
                          str(tmp_path / "roles"), str(gdir)],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 1 and bad.name in out.stderr, out.stderr
    assert out.stdout.splitlines() == exp


@pytest.mark.gpu
def test_kma_apply_verify_rows_in_gto_feature_order(kma_bin, oracle_c, small_gto, apply_inputs,
                                                    tmp_path):
    """VERIFY rows follow one documented rule: the order of the GTO's features array (pegs only),
    which is what Genome.getPegs() is taken to return (the Genome class is
    external, its order unpinned). A genome whose pegs are shuffled (ids out of order, RNA
    features in between) reports its called pegs in exactly that file order, not sorted by id."""
    d, rows, roles, pegs = apply_inputs
    rng = np.random.default_rng(5)
    order = rng.permutation(len(pegs))
    feats = []
    for j, i in enumerate(order):
        feats.append(pegs[i])
        if j % 7 == 0:
            feats.append({"id": f"fig|97478.30.rna.{j}", "type": "rna", "function": "tRNA"})
    gto = {"id": "97478.30", "scientific_name": "shuffled", "genetic_code": 11,
           "features": feats}
    gdir = tmp_path / "gtos"
    gdir.mkdir()
    (gdir / "97478.30.gto").write_text(json.dumps(gto))
    _, exp_verify = _expected(oracle_c, small_gto, rows, roles, [pegs[i] for i in order], 5)
    out = subprocess.run([kma_bin, "apply", "--format", "VERIFY", str(d / "kmerdb.tbl"),
                          str(d / "roles.in.use"), str(gdir)], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr
    got = out.stdout.splitlines()
    assert got == exp_verify and len(got) > 20
    ids = [ln.split("\t")[1] for ln in got[1:]]
    assert ids != sorted(ids)  # file order, not id order


def test_kma_apply_errors(kma_bin, apply_inputs, tmp_path):
    d, _, _, _ = apply_inputs
    r = subprocess.run([kma_bin, "apply", str(d / "kmerdb.tbl"), str(d / "roles.in.use"),
                        str(tmp_path / "missing")], capture_output=True, text=True)
    assert r.returncode == 1 and "Input directory" in r.stderr and "not found" in r.stderr
    r = subprocess.run([kma_bin, "apply", "-m", "0", str(d / "kmerdb.tbl"),
                        str(d / "roles.in.use"), str(d / "gtos")], capture_output=True, text=True)
    assert r.returncode == 2 and "Min-hits must be positive." in r.stderr
    r = subprocess.run([kma_bin, "apply", "--format", "TRAIN", "a", "b", "c"],
                       capture_output=True, text=True)
    assert r.returncode == 2
    r = subprocess.run([kma_bin, "frobnicate"], capture_output=True, text=True)
    assert r.returncode == 1 and "Invalid command frobnicate." in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("k", [8, 10])
def test_kma_contigs_report(kma_bin, oracle_c, small_gto, apply_inputs, tmp_path, k):
    """`kma contigs` (6-frame kmers of every genome's contigs probed against a kmer database
    whose last row sets K, as ApplyKmerProcessor.java:108 / KmerProcessor -K do) at K = 8 and
    K = 10 (a wide table): every line equals the oracle's hit (KmerReference.java:157-203)."""
    d, _, _, _ = apply_inputs
    contigs = [c["dna"] for c in small_gto["contigs"]]
    dna, off = oracle_c.pack_strings(contigs)
    km, _, _, _, _ = oracle_c.contig_kmers(dna, off, 11, k)
    rng = np.random.default_rng(k)
    kmers = [bytes(r).decode() for r in km[rng.choice(len(km), 5000, replace=False)]]
    roles = [f"R{i % 37}" for i in range(len(kmers))]
    with open(tmp_path / "db.tbl", "w") as f:
        f.writelines(f"{a}\t{b}\n" for a, b in zip(kmers, roles))
    ids = {}
    for r in roles:
        ids.setdefault(r, len(ids))
    inv = {v: r for r, v in ids.items()}
    ct, lf, sd, fr, fid = oracle_c.annotate_contigs(
        oracle_c.Table(kmers, [ids[r] for r in roles]), dna, off, 11, k)
    gid, cids = small_gto["id"], [c["id"] for c in small_gto["contigs"]]
    exp = ["genome_id\tcontig_id\tstrand\tleft\tright\tframe\trole"] + [
        f"{gid}\t{cids[c]}\t{chr(s)}\t{l}\t{l + 3 * k - 1}\t{f}\t{inv[int(x)]}"
        for c, l, s, f, x in zip(ct, lf, sd, fr, fid)]
    out = subprocess.run([kma_bin, "contigs", str(tmp_path / "db.tbl"), str(d / "gtos")],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.splitlines() == exp and len(exp) > 5000


def _dump_expected(gto):
    lines = [f"{gto.get('id', '')}\t{gto.get('scientific_name', '')}\t"
             f"{int(gto.get('genetic_code', 11))}"]
    for f in gto.get("features", []):
        lines.append("\t".join(str(f.get(k, "")) for k in
                               ("id", "type", "function", "protein_translation")))
    return lines


def test_gto_apply_loader_matches_json(kma_bin, small_gto, tmp_path):
    """apply's GTO loader (host/gto.cpp load_genome_pegs: mapped file, keys as views, skipped
    members never built) reads what a JSON library reads: the reference's small.gto, and a
    GTO holding escapes (quotes, backslashes, \\u, surrogate pairs) in the kept strings,
    brackets and quotes inside skipped strings, nested skipped containers, numbers, booleans
    and null, and a numeric genetic code given as a string."""
    path = tmp_path / "small.gto"
    with gzip.open(os.path.join(GOLDEN, "small.gto.gz"), "rb") as f:
        path.write_bytes(f.read())
    out = subprocess.run([kma_bin, "gto-dump", str(path)], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    assert out.stdout.splitlines() == _dump_expected(small_gto)
    tricky = {
        "id": "123.4", "scientific_name": "Tricky \"quoted\" \\ name é \U0001F600",
        "genetic_code": "4", "domain": "Bacteria", "flag": True, "nothing": None,
        "contigs": [{"id": "c\"1]", "dna": "ac]}gt\\\"" * 50}],
        "subsystems": [{"a": [1, 2.5e3, -7, {"b": "}{][\",\\"}], "c": False}],
        "features": [
            {"id": "fig|123.4.peg.1", "type": "CDS", "location": [["c1", 1, "+", 30]],
             "function": "role \"A\" / \\B\\ ü", "protein_translation": "MKV*LL",
             "annotations": [["x", "y\"}]", 0.5]], "aliases": []},
            {"id": "fig|123.4.rna.1", "type": "rna", "function": "tRNA", "quality": {}},
            {"type": "peg", "id": "fig|123.4.peg.2", "protein_translation": "",
             "family_assignments": [["PGF", "x", "y", "z"]], "function": ""},
        ],
    }
    path = tmp_path / "tricky.gto"
    path.write_text(json.dumps(tricky, indent=1))
    out = subprocess.run([kma_bin, "gto-dump", str(path)], capture_output=True,
                         encoding="utf-8")
    assert out.returncode == 0, out.stderr
    assert out.stdout.splitlines() == _dump_expected(tricky)
    # members in small.gto's order: reading stops after id / scientific_name / genetic_code /
    # features, so bytes after them (here: not even JSON) are never read; the same members
    # with the contigs first are read through
    early = {k: tricky[k] for k in ("features", "genetic_code", "id", "scientific_name")}
    path = tmp_path / "early.gto"
    path.write_text(json.dumps(early)[:-1] + ', "contigs": [{"id": "c1", "dna": "acgt"  <not json')
    out = subprocess.run([kma_bin, "gto-dump", str(path)], capture_output=True, encoding="utf-8")
    assert out.returncode == 0, out.stderr
    assert out.stdout.splitlines() == _dump_expected(tricky)
    late = dict([("contigs", tricky["contigs"])] + list(early.items()))
    path.write_text(json.dumps(late))
    out = subprocess.run([kma_bin, "gto-dump", str(path)], capture_output=True, encoding="utf-8")
    assert out.returncode == 0, out.stderr
    assert out.stdout.splitlines() == _dump_expected(tricky)
