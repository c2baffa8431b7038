#!/bin/bash
# Round-end pass of the default build (paired homes, hashed chains): GPU parity, smoke, bench
# lines (c5 headline with the CPU baseline; c2 / c3 / c4; c5 at load factors 0.75 / 0.9) and
# rocprofv3 kernel stats at c5. Stops at the first step that faults, aborts or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name" | tee -a $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log; tail -1 $OUT/$name.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc; }
step pytest 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c5 600 python bench.py --steps 20 --warmup 3
step bench_c2 300 python bench.py --steps 20 --warmup 3 --workload c2 --no-cpu-baseline
step bench_c3 300 python bench.py --steps 20 --warmup 3 --workload c3 --no-cpu-baseline
step bench_c4 300 python bench.py --steps 10 --warmup 2 --workload c4 --no-cpu-baseline
step bench_c5_lf0.75 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --load-factor 0.75
step bench_c5_lf0.9 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --load-factor 0.9
step prof_c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras
