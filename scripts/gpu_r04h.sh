#!/bin/bash
# Round 4: GPU tests on the one-copy-per-piece, two-copy-stream host staging; the c5 host call
# sweep over pieces and its trace; the c5 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r04h; mkdir -p $OUT
bash scripts/gpu_tests.sh r04h || exit $?
timeout -k 10 400 python scripts/e2e_host.py --configs "pieces=8,threads=16;pieces=12,threads=16;pieces=16,threads=16;pieces=16,threads=8;packed=0,pieces=16,threads=16" > $OUT/e2e_sweep.jsonl 2> $OUT/e2e_sweep.log
rc=$?; echo "e2e sweep rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/e2e_trace -o run -- python3 scripts/e2e_host.py --configs "pieces=16,threads=16" --reps 1 --calls 2 > $OUT/e2e_trace.log 2>&1
rc=$?; echo "e2e trace rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.log
rc=$?; echo "bench c5 rc=$rc" >> $OUT/steps.log
python3 scripts/copy_overlap.py $OUT/e2e_trace | tail -n 1 | cut -c1-600
cat $OUT/e2e_sweep.jsonl
cat $OUT/steps.log
