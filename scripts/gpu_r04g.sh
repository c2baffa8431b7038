#!/bin/bash
# Round 4: the c5 host call: a pieces x threads sweep, and one configuration under rocprofv3's
# kernel + memory-copy trace (copy / kernel overlap); the c5 line with the link rates; c3 block
# clocks on the two-pass build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r04g; mkdir -p $OUT
timeout -k 10 400 python scripts/e2e_host.py > $OUT/e2e_sweep.jsonl 2> $OUT/e2e_sweep.log
rc=$?; echo "e2e sweep rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/e2e_trace -o run -- python3 scripts/e2e_host.py --configs "pieces=8,threads=16" --reps 1 --calls 2 > $OUT/e2e_trace.log 2>&1
rc=$?; echo "e2e trace rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.log
rc=$?; echo "bench c5 rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
KMERANNO_LIB=kmers.anno_amd/build/clk/libkmeranno.so timeout -k 10 200 python scripts/block_clock.py c3 > $OUT/clock_c3.json 2> $OUT/clock_c3.log
echo "clock c3 rc=$?" >> $OUT/steps.log
cat $OUT/e2e_sweep.jsonl
cat $OUT/steps.log
