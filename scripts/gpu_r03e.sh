#!/bin/bash
# Round 3: GPU tests + smoke of the current build, c3 bench, c5 / c3 A/B of the tuning variants
# (lane permutation; cost bounds without chain walks / without sets), adversarial layouts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r03e; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
B=kmers.anno_amd/build
step pytest 900 python3 -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
for v in . lanep . nowalk noset; do
  export KMERANNO_LIB=$B/$v/libkmeranno.so
  n=${v/./default}
  step c5_$n 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras
  grep -o '"ms_per_step": [0-9.]*' $OUT/c5_$n.log >> $OUT/steps.log
done
for v in . lanep .; do
  export KMERANNO_LIB=$B/$v/libkmeranno.so
  n=${v/./default}
  step c3_$n 300 python3 bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline --no-extras
  grep -o '"ms_per_step": [0-9.]*' $OUT/c3_$n.log >> $OUT/steps.log
done
unset KMERANNO_LIB
step adv_pair 300 python3 scripts/layout_sweep.py --adversarial --lfs 0.5,0.9
export KMERANNO_LIB=$B/nopair/libkmeranno.so
step adv_nopair 300 python3 scripts/layout_sweep.py --adversarial --lfs 0.5,0.9
