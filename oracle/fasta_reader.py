"""Test infrastructure (oracle): a pure-Python restatement of the protein FASTA reader the FASTA
form of apply assumes (host/fasta.h), used only by tests/ and bench.py's parity check.

The reference reads protein FASTA through org.theseed.sequence.FastaInputStream
(anno/BuildKmerProcessor.java:196-198). That class lives in the un-vendored org.theseed:sequence
1.0.0 artifact (pom.xml:48-72), so these rules are a restatement of its assumed behaviour —
parity unpinned by any reference fixture:
  - lines are split as java.io.BufferedReader.readLine splits them ("\\n", "\\r\\n", lone "\\r");
  - a line starting with '>' opens a record: label = text up to the first space or tab,
    comment = everything after that one separator;
  - the other lines up to the next header are concatenated as they are into the sequence;
  - lines before the first header are ignored.
"""
from __future__ import annotations

import re

_LINES = re.compile(rb"\r\n|\r|\n")


def read_lines(data: bytes) -> list[bytes]:
    """BufferedReader.readLine over the whole input (no empty line after a final terminator)."""
    lines = _LINES.split(data)
    if lines and lines[-1] == b"" and data[-1:] in (b"\n", b"\r"):
        lines.pop()
    return lines


def read_fasta(data: bytes) -> list[tuple[bytes, bytes, bytes]]:
    """(label, comment, sequence) of every record, in file order."""
    out = []
    cur = None
    seq: list[bytes] = []
    for line in read_lines(data):
        if line.startswith(b">"):
            if cur is not None:
                out.append((cur[0], cur[1], b"".join(seq)))
            head = line[1:]
            m = re.search(rb"[ \t]", head)
            cur = (head, b"") if m is None else (head[:m.start()], head[m.start() + 1:])
            seq = []
        elif cur is not None:
            seq.append(line)
    if cur is not None:
        out.append((cur[0], cur[1], b"".join(seq)))
    return out
