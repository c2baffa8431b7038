#!/bin/bash
# Round 3: c5 A/B on one box: shipped build vs the two-stage pipelined probe loop (pipe) and
# unpaired homes (np2), interleaved; c3 / c2 lines; GPU tests of the 6-frame path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r03h; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
B=kmers.anno_amd/build
step pytest 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py tests/test_gpu_proposals.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "contig or wide or peg or propos"
for v in . pipe np2 . pipe np2; do
  export KMERANNO_LIB=$B/$v/libkmeranno.so
  n=${v/./default}
  step c5_$n 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
  grep -o '"ms_per_step": [0-9.]*' $OUT/c5_$n.log >> $OUT/steps.log
done
unset KMERANNO_LIB
for wl in c3 c2 c3 c2; do
  step $wl 300 python3 bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-extras
  grep -o '"ms_per_step": [0-9.]*\|"phases_ms": {[^}]*}' $OUT/$wl.log >> $OUT/steps.log
done
export KMERANNO_LIB=$B/pipe/libkmeranno.so
step c2_pipe 300 python3 bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline --no-extras
grep -o '"ms_per_step": [0-9.]*' $OUT/c2_pipe.log >> $OUT/steps.log
