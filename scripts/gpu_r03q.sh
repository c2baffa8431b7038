#!/bin/bash
# Round 3 (session 2): GPU tests of the 6-frame path with final records staged by the probe and
# group sums added by the probe's atomics (no group-sum kernel), then c3 lines and kernel stats.
# Usage: scripts/gpu_r03q.sh <out-subdir> [pytest -k expression]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03q}; mkdir -p $OUT
K=${2:-contig or peg or propos or cli or c3 or config3}
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step pytest 600 python3 -u -m pytest tests -m gpu -k "$K" -v --timeout 300 --timeout-method thread -p no:cacheprovider -x
grep -E "passed|failed" $OUT/pytest.log | tail -1 >> $OUT/steps.log
for wl in ${WLS:-c3 c3}; do
  step bench_$wl 300 python3 bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-extras
  echo "$wl $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$wl.log) $(grep -o '"phases_ms": {[^}]*}' $OUT/bench_$wl.log)" >> $OUT/steps.log
done
step stats_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c3 -o run -- python3 bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline --no-extras
