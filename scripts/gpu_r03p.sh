#!/bin/bash
# Round 3: GPU tests of the build with queued-key chain walks, the scratch-free probe loop and
# adaptive proteins per block; c5 / c2 / c4 lines; c5 layout sweep (m = 6 / 7 / flat x load
# factor) of this build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r03p; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
step pytest 600 python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider -x
grep -E "passed|failed" $OUT/pytest.log | tail -1 >> $OUT/steps.log
for wl in c5 c2 c4 c5; do
  step bench_$wl 300 python3 bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-extras
  echo "$wl $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$wl.log)" >> $OUT/steps.log
done
step sweep 600 python3 scripts/layout_sweep.py --lfs 0.5,0.75,0.9 --steps 10
