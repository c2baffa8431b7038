#!/bin/bash
# Round 3: full GPU test pass + smoke of the build, then the measurement pass
# (scripts/gpu_r03_final.sh: PMC traffic, kernel stats, bench lines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r03i; mkdir -p $OUT
echo "=== pytest $(date +%T)" >> $OUT/steps.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "=== pytest rc=$rc" >> $OUT/steps.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "=== smoke rc=$rc" >> $OUT/steps.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r03_final.sh r03i
