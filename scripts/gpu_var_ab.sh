#!/bin/bash
# Variant A/B: contig parity under the default build, then bench lines per (variant, workload).
#   RUNS="main:c3 cp1:c3 main:c2 u2:c2 ..." bash scripts/gpu_var_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS ${K_EXPR:+-k "$K_EXPR"} -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $RUNS; do
  v=${r%%:*}; wl=${r##*:}
  lib=kmers.anno_amd/build/libkmeranno.so; [ $v = main ] || lib=kmers.anno_amd/build/$v/libkmeranno.so
  KMERANNO_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --workload $wl --no-cpu-baseline --no-extras ${EXTRA:-} > $OUT/var_${v}_$wl.log 2>&1
  rc=$?; echo "$v $wl rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/var_${v}_$wl.log) $(grep -o '"phases_ms": {[^}]*}' $OUT/var_${v}_$wl.log)"
  [ $rc -eq 0 ] || exit $rc
done
