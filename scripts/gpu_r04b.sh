#!/bin/bash
# Round 4: multi-rank rehearsal tests + kma apply batching tests, then the genome-directory bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r04b; mkdir -p $OUT
df -h /tmp > $OUT/df.txt 2>&1; nproc >> $OUT/df.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py tests/test_cli.py -m gpu -v \
  --timeout 900 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
echo "pytest rc=$?" >> $OUT/steps.log
tail -3 $OUT/pytest.log
timeout -k 10 600 python bench.py --workload genomes > $OUT/genomes.json 2> $OUT/genomes.log
echo "genomes rc=$?" >> $OUT/steps.log
tail -2 $OUT/genomes.log; cat $OUT/steps.log
