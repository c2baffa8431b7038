#!/bin/bash
# Proteins-per-block A/B (KMA_BLOCK_PROTEINS) on c2 and c5, after the GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for wl in ${WLS:-c2 c5}; do
  for bp in ${BPS:-auto 4 6 8}; do
    if [ $bp = auto ]; then unset KMA_BLOCK_PROTEINS; else export KMA_BLOCK_PROTEINS=$bp; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --workload $wl --no-cpu-baseline --no-extras > $OUT/bp_${wl}_$bp.log 2>&1
    rc=$?; echo "$wl bp=$bp rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/bp_${wl}_$bp.log)"
    [ $rc -eq 0 ] || exit $rc
  done
done
