#!/bin/bash
# kma apply over synthetic GTOs with different staging-pool widths (the parse pool, the caller
# and the library's staging threads share the box's CPU quota). Usage: bash scripts/apply_threads_ab.sh <out>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-apply_threads}; mkdir -p $OUT
D=/tmp/kma_apply_ab
python3 - "$D" <<'PY' || exit 1
import os, sys
sys.path[:0] = ["kmers.anno_amd/python"]
from kmeranno import synth
d = sys.argv[1]
sig = synth.make_table(10_000_000, 10_000, 4, 8)
synth.write_kmer_db(os.path.join(d, "kmerdb.tbl"), sig.keys, sig.fids) if os.makedirs(d, exist_ok=True) is None else None
synth.write_roles_in_use(os.path.join(d, "roles.in.use"), 10_000, every=10)
for a in range(0, 300, 50):
    synth.write_genome_dir(os.path.join(d, "gtos"), sig, 50, 4000, seed=8, contig_bp=4_000_000, first=a)
    print("written", a + 50, flush=True)
PY
for rep in 1 2; do
  for st in 16 8 4 2; do
    timeout -k 10 120 kmers.anno_amd/build/kma apply --staging-threads $st $D/kmerdb.tbl $D/roles.in.use $D/gtos > /dev/null 2> $OUT/st${st}_r$rep.log
    echo "st=$st r$rep rc=$? $(grep -o 'apply-stats.*' $OUT/st${st}_r$rep.log)" >> $OUT/steps.log
  done
done
cat $OUT/steps.log
