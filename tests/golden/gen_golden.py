"""Generate the committed golden vectors (run from the repo root:
``python tests/golden/gen_golden.py``).

The Java reference cannot run in this environment (no JDK, no org.theseed jars), so the
expected outputs come from the independent pure-Python restatement oracle/oracle_py.py and
are cross-checked here against the C oracle before being written. Inputs:
  apply_edge.json   — tests/edge_cases.py
  apply_c1.npz      — BASELINE config 1 (100 proteins vs 1k-entry 8-mer table, seed 1)
  contigs_gto.npz   — contig 5 of the reference fixture src/test/small.gto (67,417 bp) plus
                      a 2-contig slice of contig 1, against a table of 5,000 of their 6-frame
                      kmers + 5,000 decoys (seed 7)
"""
import gzip
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "kmers.anno_amd", "python")]

from edge_cases import CASES  # noqa: E402
from kmeranno import synth  # noqa: E402
from oracle import c_oracle, oracle_py  # noqa: E402


def role_ids(rows):
    ids = {}
    for _, r in rows:
        ids.setdefault(r, len(ids))
    return ids


def twin_apply(rows, prots, min_hits, flags, k=8):
    table = oracle_py.load_table(rows)
    out = []
    for p in prots:
        st, role, cnt = oracle_py.apply_protein(table, p, min_hits, k, bool(flags & 1),
                                                bool(flags & 2))
        out.append((st, role, cnt))
    return out


def c_apply(rows, prots, min_hits, flags, k=8):
    ids = role_ids(rows)
    t = c_oracle.Table([r[0] for r in rows], [ids[r[1]] for r in rows])
    res, off = c_oracle.pack_strings(prots)
    fid, cnt, st = c_oracle.apply(t, res, off, k, min_hits, flags)
    inv = {v: k_ for k_, v in ids.items()}
    return [(int(s), inv.get(int(f)), int(c)) for f, c, s in zip(fid, cnt, st)]


def gen_edge():
    out = []
    for name, rows, prots, min_hits, flags in CASES:
        exp = twin_apply(rows, prots, min_hits, flags)
        assert exp == c_apply(rows, prots, min_hits, flags), name
        out.append({"name": name, "rows": rows, "proteins": prots, "min_hits": min_hits,
                    "flags": flags, "expected": [list(e) for e in exp]})
    with open(os.path.join(HERE, "apply_edge.json"), "w") as f:
        json.dump(out, f, indent=1)


def gen_c1():
    wl = synth.make_workload(*synth.CONFIGS["c1"])
    kmers = [synth.unpack_key(x) for x in wl.keys]
    rows = list(zip(kmers, [f"ROLE{int(f):07d}" for f in wl.fids]))
    prots = [bytes(wl.residues[int(a):int(b)]).decode()
             for a, b in zip(wl.offsets[:-1], wl.offsets[1:])]
    arrays = {}
    for flags in (0, 1, 2):
        exp = twin_apply(rows, prots, 5, flags)
        assert exp == c_apply(rows, prots, 5, flags)
        arrays[f"status_{flags}"] = np.array([e[0] for e in exp], np.uint8)
        arrays[f"fid_{flags}"] = np.array([-1 if e[1] is None else int(e[1][4:]) for e in exp],
                                          np.int32)
        arrays[f"count_{flags}"] = np.array([e[2] for e in exp], np.int32)
    np.savez_compressed(os.path.join(HERE, "apply_c1.npz"),
                        table_kmers=np.frombuffer("".join(kmers).encode(), np.uint8).reshape(-1, 8),
                        table_fids=wl.fids, residues=wl.residues, offsets=wl.offsets, **arrays)


def gen_contigs():
    with gzip.open(os.path.join(HERE, "small.gto.gz"), "rt") as f:
        g = json.load(f)
    c1 = g["contigs"][0]["dna"]
    contigs = [g["contigs"][4]["dna"], c1[:30000], c1[30000:30023], c1[40000:40031]]
    recs = list(oracle_py.contig_kmers(contigs, 11, 8))
    rng = np.random.default_rng(7)
    uniq = sorted({r[0] for r in recs})
    pick = [uniq[i] for i in rng.choice(len(uniq), 5000, replace=False)]
    aa = "ACDEFGHIKLMNPQRSTVWY"
    decoys = ["".join(aa[j] for j in rng.integers(0, 20, 8)) for _ in range(5000)]
    kmers = pick + decoys
    fids = rng.integers(0, 500, len(kmers)).astype(np.uint32)
    table = dict(zip(kmers, [int(f) for f in fids]))
    hits = oracle_py.annotate_contigs(table, contigs, 11, 8)
    t = c_oracle.Table(kmers, fids.astype(np.int32))
    dna, off = c_oracle.pack_strings(contigs)
    ct, lf, sd, fr, fid = c_oracle.annotate_contigs(t, dna, off, 11, 8)
    assert [(int(a), int(b), chr(c), int(d), int(e)) for a, b, c, d, e in
            zip(ct, lf, sd, fr, fid)] == hits
    np.savez_compressed(os.path.join(HERE, "contigs_gto.npz"), dna=dna, offsets=off,
                        table_kmers=np.frombuffer("".join(kmers).encode(), np.uint8).reshape(-1, 8),
                        table_fids=fids,
                        hit_contig=np.array([h[0] for h in hits], np.uint32),
                        hit_left=np.array([h[1] for h in hits], np.int32),
                        hit_strand=np.array([ord(h[2]) for h in hits], np.uint8),
                        hit_frame=np.array([h[3] for h in hits], np.uint8),
                        hit_fid=np.array([h[4] for h in hits], np.uint32))


if __name__ == "__main__":
    c_oracle.build()
    gen_edge()
    gen_c1()
    gen_contigs()
    print("golden vectors written to", HERE)
