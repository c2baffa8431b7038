#!/bin/bash
# Round 3 end: every GPU test and smoke of the shipped build, then scripts/gpu_r03w.sh's
# measurement pass (PMC traffic -> profiles/r03_traffic.json, kernel stats, bench lines, SQ).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_end}; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest 600 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider -x
tail -1 $OUT/pytest.log >> $OUT/steps.log
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
bash scripts/gpu_r03w.sh ${1:-r03_end}
