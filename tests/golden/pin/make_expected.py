"""Writes tests/golden/pin/expected.txt: what scripts/PinProteinKmers.java prints if the three
external semantics this build assumes hold. The assumptions come from the oracle
restatements, not from the reference (no JDK or org.theseed jar exists here):
  KMERS  org.theseed.sequence.ProteinKmers(String) at K = 8: the SET of the substrings at
         i = 0 .. L - 8 inclusive, no filtering (oracle/oracle_py.py protein_kmers);
  FASTA  org.theseed.sequence.FastaInputStream records (oracle/fasta_reader.py);
  PEGS   org.theseed.genome.Genome.getPegs(): the features array's CDS / peg entries in file
         order (host/gto.h Genome::pegs).
A maintainer with the jars runs scripts/pin_external_semantics.sh: an empty diff pins all three.

  python tests/golden/pin/make_expected.py > tests/golden/pin/expected.txt
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(HERE))))
from oracle import fasta_reader, oracle_py  # noqa: E402


def expected_lines():
    out = []
    for prot in open(os.path.join(HERE, "proteins.txt")).read().split("\n")[:-1]:
        kmers = oracle_py.protein_kmers(prot, 8)
        out.append(f"KMERS\t{prot}\t{len(kmers)}\t{','.join(sorted(kmers))}")
    for label, comment, seq in fasta_reader.read_fasta(open(os.path.join(HERE, "edge.faa"), "rb").read()):
        out.append(f"FASTA\t{label.decode()}\t{comment.decode()}\t{seq.decode()}")
    g = json.load(open(os.path.join(HERE, "shuffled.gto")))
    pegs = [f["id"] for f in g["features"] if f.get("type") in ("CDS", "peg")]
    out.append(f"PEGS\t{g['id']}\t{','.join(pegs)}")
    return out


if __name__ == "__main__":
    sys.stdout.write("\n".join(expected_lines()) + "\n")
