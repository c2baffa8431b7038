#!/bin/bash
# Round 3: GPU tests of the big-config and protein paths after the table-size-aware proteins per
# block rule, then c4 / c5 / c2 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03bp2}; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest 600 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider -x
tail -1 $OUT/pytest.log >> $OUT/steps.log
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
for wl in c4 c5 c4 c5 c2; do
  step bench_${wl}_$((++n)) 300 python3 bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-extras
  echo "$wl $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_${wl}_$n.log)" >> $OUT/steps.log
done
