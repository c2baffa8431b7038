#!/bin/bash
# End-of-round pass on one box: GPU tests + smoke, then the measurement pass of the shipped build
# (PMC traffic -> profiles/<round>_traffic.json copy under gpurun_out, kernel stats, bench lines,
# SQ counters), the genome-directory line and the FASTA line. The traffic summary is written to $TRAFFIC on the
# box before the bench lines run, so they carry it (copy it back from gpurun_out/<out>/traffic.json).
# Usage: TRAFFIC=profiles/r06_traffic.json [SKIP_TESTS=1] bash scripts/gpu_round_end.sh <out-subdir>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=${1:-round_end}
[ -n "$SKIP_TESTS" ] || bash scripts/gpu_tests.sh $OUT || exit $?
WLS=${WLS:-c5 c2 c3 c4 c5_lf0.75 c5_lf0.9} SECTIONS=${SECTIONS:-traffic stats bench lf sq} TRAFFIC=${TRAFFIC:-profiles/r06_traffic.json} bash scripts/gpu_measure.sh $OUT || exit $?
cp ${TRAFFIC:-profiles/r06_traffic.json} gpurun_out/$OUT/traffic.json
timeout -k 10 600 python bench.py --workload genomes > gpurun_out/$OUT/bench_genomes.log 2> gpurun_out/$OUT/bench_genomes.err
echo "genomes rc=$?" >> gpurun_out/$OUT/steps.log
timeout -k 10 600 python bench.py --workload fasta > gpurun_out/$OUT/bench_fasta.log 2> gpurun_out/$OUT/bench_fasta.err
echo "fasta rc=$?" >> gpurun_out/$OUT/steps.log
cat gpurun_out/$OUT/steps.log
