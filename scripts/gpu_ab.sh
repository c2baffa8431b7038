#!/bin/bash
# A/B of the K1 probe form on one box: pytest (default form), then c2/c5 benches and kernel
# stats under each KMA_PROBE form in $SHAPES (run = default, quad, lane).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
[ -n "$NO_PYTEST" ] || step pytest_gpu 900 python -m pytest tests -x -q -m gpu
for shape in ${SHAPES:-run quad}; do
  export KMA_PROBE=$shape
  step bench_c2_$shape 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
  step prof_c2_$shape 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2_$shape -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
  step prof_c5_$shape 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5_$shape -o run -- python3 bench.py --steps 5 --warmup 1 --workload c5 --no-cpu-baseline
done
