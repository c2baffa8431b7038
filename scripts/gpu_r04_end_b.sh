#!/bin/bash
# Round 4 end measurement, part B (part A: SECTIONS=traffic of gpu_measure.sh -> profiles/r04_traffic.json):
# kernel stats, the bench lines (c5 with the CPU baseline, c2, c3, c4), SQ counters, the genome-directory line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
SECTIONS="stats bench sq" bash scripts/gpu_measure.sh r04_end_b || exit $?
timeout -k 10 600 python bench.py --workload genomes > gpurun_out/r04_end_b/bench_genomes.log 2> gpurun_out/r04_end_b/bench_genomes.err
echo "genomes rc=$?" >> gpurun_out/r04_end_b/steps.log
cat gpurun_out/r04_end_b/steps.log
