#!/bin/bash
# Environment A/B: optional GPU tests, then bench lines per (env assignment, workload).
#   RUNS="KMA_RANGE=0:c2 KMA_RANGE=:c2 ..." bash scripts/gpu_env_ab.sh   (NAME= unsets NAME)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS ${K_EXPR:+-k "$K_EXPR"} -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
for r in $RUNS; do
  kv=${r%:*}; wl=${r##*:}; i=$((i + 1))
  name=${kv%%=*}; val=${kv#*=}
  if [ -n "$val" ]; then envcmd=(env "$name=$val"); else envcmd=(env -u "$name"); fi
  "${envcmd[@]}" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --workload $wl --no-cpu-baseline --no-extras ${EXTRA:-} > $OUT/env_${i}_$wl.log 2>&1
  rc=$?; echo "$kv $wl rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/env_${i}_$wl.log) $(grep -o '"phases_ms": {[^}]*}' $OUT/env_${i}_$wl.log)"
  [ $rc -eq 0 ] || exit $rc
done
