#!/bin/bash
# Round 3 (session 2): VALU diet of the probes. GPU tests of the default build (one-multiply
# hashes KMA_HASH_LITE, scalar protein boundaries KMA_SPAN_SCALAR, 16 probe blocks per emit
# block), then c5 A/B against builds without each change, c3/c2/c4 lines, and the c5 layout
# sweep of the default build. Usage: scripts/gpu_r03r.sh <out-subdir>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03r}; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
B=kmers.anno_amd/build
if [ -z "$NOTEST" ]; then
  step pytest 900 python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider -x
  grep -E "passed|failed" $OUT/pytest.log | tail -1 >> $OUT/steps.log
fi
for r in ${RUNS:-main:c5 nolite:c5 nospan:c5 main:c5 main:c3 main:c3 main:c2 main:c4}; do
  v=${r%%:*}; wl=${r##*:}
  lib=$B/libkmeranno.so; [ $v = main ] || lib=$B/$v/libkmeranno.so
  KMERANNO_LIB=$lib step ${v}_$wl 300 python3 bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-extras
  echo "$v $wl $(grep -o '"ms_per_step": [0-9.]*' $OUT/${v}_$wl.log) $(grep -o '"phases_ms": {[^}]*}' $OUT/${v}_$wl.log) $(grep -o 'layout[^"]*' $OUT/${v}_$wl.log | head -1)" >> $OUT/steps.log
done
[ -n "$SWEEP" ] && step sweep 600 python3 scripts/layout_sweep.py --lfs ${SWEEP} --steps 10
exit 0
