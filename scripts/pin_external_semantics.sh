#!/bin/bash
# One command that pins (or refutes) the external semantics this build assumes, where a JDK and
# the SEEDtk jars exist (not in this build's image): runs scripts/PinProteinKmers.java on the
# committed fixtures and diffs its output against tests/golden/pin/expected.txt (what the
# assumed rules predict; tests/test_pin_probe.py keeps that file equal to the oracle's rules).
# Usage: SEED_JARS=/path/to/jars bash scripts/pin_external_semantics.sh
cd "$(dirname "$0")/.." || exit 2
: "${SEED_JARS:?set SEED_JARS to the directory holding the org.theseed jars}"
java -cp "$SEED_JARS/*" scripts/PinProteinKmers.java tests/golden/pin > /tmp/pin_actual.txt || exit 2
if diff -u tests/golden/pin/expected.txt /tmp/pin_actual.txt; then
  echo "pinned: ProteinKmers windows, FastaInputStream records and Genome.getPegs order as assumed"
else
  echo "MISMATCH: see the lines above (KMERS -> KMA_F_* flags, FASTA -> host/fasta.cpp, PEGS -> host/gto.cpp)"
  exit 1
fi
