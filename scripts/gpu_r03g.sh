#!/bin/bash
# Round 3: GPU tests of the two-bit filter + lane-permutation build, c5 A/B against one filter
# bit, c3 with the vectorized last-block scan, layout sweep (+ TCC counters) on the new build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r03g; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
B=kmers.anno_amd/build
step pytest 900 python3 -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider
for v in . f1 . f1; do
  export KMERANNO_LIB=$B/$v/libkmeranno.so
  n=${v/./default}
  step c5_$n 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras
  grep -o '"ms_per_step": [0-9.]*' $OUT/c5_$n.log >> $OUT/steps.log
done
unset KMERANNO_LIB
step c3 300 python3 bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline --no-extras
grep -o '"ms_per_step": [0-9.]*' $OUT/c3.log >> $OUT/steps.log
step c2 300 python3 bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline --no-extras
grep -o '"ms_per_step": [0-9.]*' $OUT/c2.log >> $OUT/steps.log
step sweep 300 python3 scripts/layout_sweep.py
step pmc_sweep 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace \
  --output-format csv -d $OUT/pmc_sweep -o run -- python3 scripts/layout_sweep.py --steps 3 --warmup 1
step adv 300 python3 scripts/layout_sweep.py --adversarial --lfs 0.5,0.9
