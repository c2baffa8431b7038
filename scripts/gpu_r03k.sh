#!/bin/bash
# Round 3: scratch-free annotate_kernel. GPU tests, then c5 A/B on one box: shipped build vs
# the the serial chain walks (serial), queued keys (qkeys) and the no-walk cost
# bound (nowalk), interleaved; c5 FETCH/WRITE_SIZE of the shipped build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r03k; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
B=kmers.anno_amd/build
step pytest 600 python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider -x
for v in . serial qkeys nowalk . serial qkeys nowalk; do
  export KMERANNO_LIB=$B/$v/libkmeranno.so
  n=${v/./default}
  step c5_$n 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
  grep -o '"ms_per_step": [0-9.]*' $OUT/c5_$n.log >> $OUT/steps.log
done
unset KMERANNO_LIB
for v in . serial . serial; do
  export KMERANNO_LIB=$B/$v/libkmeranno.so
  n=${v/./default}
  step c5lf9_$n 300 python3 bench.py --steps 10 --warmup 2 --load-factor 0.9 --no-cpu-baseline --no-extras
  grep -o '"ms_per_step": [0-9.]*\|"table_layout_m": [0-9]*' $OUT/c5lf9_$n.log >> $OUT/steps.log
done
