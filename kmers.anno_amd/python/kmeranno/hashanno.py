"""Host side of the hash annotator (§8(f)3) above kma_hash_annotate: the per-genome report of
HashAnnotationProcessor.processGenome (HashAnnotationProcessor.java:221-328).

  - proteins are keyed by sequence (Feature.getMD5 is the MD5 of the translation); blank
    proteins and proteins holding '*' are skipped (:237-241) but still get report lines;
  - the prototypes of the role annotation file are those with a non-blank annotation and a
    protein of at least minLen residues (default 50), in file order (:142-153);
  - a genome protein's proposal is the GPU's best prototype (similarity >= minSim, default
    0.0125), else the default proposal: its own annotation with score 0.0 (GenomeProteinKmers
    restated; parity unpinned). When features share a protein, the first one's annotation is
    the default;
  - report lines "fid\\tscore\\tnew_annotation\\told_annotation" (:281-293; a feature without a
    proposal gets a blank score and its old annotation twice); score 0.0 counts as a default,
    an equal annotation as confirmed, anything else as a change (:295-304).
"""
from __future__ import annotations

import numpy as np

from . import hash_annotate

HEADER = "fid\tscore\tnew_annotation\told_annotation"


def prototypes_from_rows(rows, min_len: int = 50):
    """(protein, annotation) rows of the role annotation file -> the kept prototypes."""
    return [(p, a) for p, a in rows if a and a.strip() and len(p) >= min_len]


def _pack(strs):
    b = [s.encode() for s in strs]
    off = np.zeros(len(b) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in b])
    return np.frombuffer(b"".join(b) or b"\0", np.uint8).copy(), off


def annotate_genome(features, prototypes, k: int = 8, min_sim: float = 0.0125,
                    device: int = 0):
    """features: [(fid, protein or '', function)]; prototypes: [(protein, annotation)].
    Returns (report lines without the header, counts {default, confirmed, new}, change lines)."""
    index, default = {}, []
    for fid, prot, func in features:
        if prot and "*" not in prot and prot not in index:
            index[prot] = len(default)
            default.append(func)
    seqs = list(index)
    gres, goff = _pack(seqs)
    pres, poff = _pack([p for p, _ in prototypes])
    best, sim, _ = hash_annotate(gres, goff, pres, poff, k, min_sim, device)
    lines, changes = [], []
    counts = {"default": 0, "confirmed": 0, "new": 0}
    for fid, prot, func in features:
        g = index.get(prot) if prot else None
        if g is None:
            lines.append(f"{fid}\t\t{func}\t{func}")
            continue
        b = int(best[g])
        score = float(sim[g]) if b >= 0 else 0.0
        new = prototypes[b][1] if b >= 0 else default[g]
        line = f"{fid}\t{score!r}\t{new}\t{func}"
        lines.append(line)
        if score == 0.0:
            counts["default"] += 1
        elif new == func:
            counts["confirmed"] += 1
        else:
            counts["new"] += 1
            changes.append(line)
    return lines, counts, changes
