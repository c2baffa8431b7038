#!/bin/bash
# Round 3 (session 2): GPU tests + smoke of the final kernels, then a proteins-per-block sweep
# (KMA_BLOCK_PROTEINS, read per call) for c5 / c4 / c2 after this session's VALU changes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03y}; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi; }
if [ -z "$NOTEST" ]; then
  step pytest 600 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider -x
  tail -1 $OUT/pytest.log >> $OUT/steps.log
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
n=0
for r in ${RUNS:-c5:0 c5:4 c5:5 c5:7 c5:8 c5:6 c4:0 c4:4 c4:8 c2:0 c2:2 c2:3 c2:6}; do
  wl=${r%%:*}; bp=${r##*:}
  if [ "$bp" = 0 ]; then unset KMA_BLOCK_PROTEINS; else export KMA_BLOCK_PROTEINS=$bp; fi
  step ${wl}_bp${bp}_$((++n)) 300 python3 bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-extras
  echo "$wl bp=$bp $(grep -o '"ms_per_step": [0-9.]*' $OUT/${wl}_bp${bp}_$n.log)" >> $OUT/steps.log
done
unset KMA_BLOCK_PROTEINS
