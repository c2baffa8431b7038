#!/bin/bash
# Round-end pass of the drop-in's regimes: `kma apply` over 500 GTOs, `kma apply-fasta` over
# c4's 1M proteins (both with the native kmerdb.tbl loader since round 6), and the replicated
# table's in-process host fan-out at c5 size (1 / 2 / 4 / 8 replicas on device 0).
# Usage: bash scripts/gpu_end_drop_in.sh <out-subdir>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-drop_in}; mkdir -p $OUT
timeout -k 10 600 python bench.py --workload genomes > $OUT/bench_genomes.json 2> $OUT/bench_genomes.err
r=$?; echo "genomes rc=$r" >> $OUT/steps.log; [ $r = 0 ] || exit $r
timeout -k 10 600 python bench.py --workload fasta > $OUT/bench_fasta.json 2> $OUT/bench_fasta.err
r=$?; echo "fasta rc=$r" >> $OUT/steps.log; [ $r = 0 ] || exit $r
timeout -k 10 600 python scripts/replica_scaling.py > $OUT/replicas.jsonl 2> $OUT/replicas.log
r=$?; echo "replicas rc=$r" >> $OUT/steps.log
cat $OUT/steps.log
exit $r
