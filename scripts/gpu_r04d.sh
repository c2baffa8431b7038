#!/bin/bash
# Round 4: the adversarial layout sweep on the shipped build (once) and the genome-directory
# workload (kma apply over 500 synthetic GTOs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r04d; mkdir -p $OUT
timeout -k 10 300 python3 scripts/layout_sweep.py --adversarial --lfs 0.5,0.9 > $OUT/adversarial.jsonl 2> $OUT/adversarial.log
rc=$?; echo "adversarial rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py --workload genomes > $OUT/genomes.json 2> $OUT/genomes.log
echo "genomes rc=$?" >> $OUT/steps.log
cat $OUT/steps.log
