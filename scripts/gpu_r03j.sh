#!/bin/bash
# Round 3: scratch-free annotate_kernel. GPU tests, then c5 A/B on one box: shipped build vs
# the previous commit's build (scr: 48 B/lane scratch), queued keys (qkeys) and the no-walk cost
# bound (nowalk), interleaved; c5 FETCH/WRITE_SIZE of the shipped build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r03j; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
B=kmers.anno_amd/build
step pytest 600 python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider
for v in . scr qkeys nowalk . scr qkeys nowalk; do
  export KMERANNO_LIB=$B/$v/libkmeranno.so
  n=${v/./default}
  step c5_$n 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
  grep -o '"ms_per_step": [0-9.]*' $OUT/c5_$n.log >> $OUT/steps.log
done
unset KMERANNO_LIB
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_c5_$c 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_c5_$c -o run -- python3 bench.py --steps 3 --warmup 1 --workload c5 --no-cpu-baseline --no-extras
done
