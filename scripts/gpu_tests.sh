#!/bin/bash
# GPU test pass: pytest -m gpu (every test in one process, per-test timeouts) and smoke().
# Usage: bash scripts/gpu_tests.sh <out-subdir> [pytest selection...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tests}; shift; mkdir -p $OUT
SEL=${@:-tests}
echo "=== pytest $(date +%T)" >> $OUT/steps.log
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v --timeout 600 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?
echo "=== pytest rc=$rc" >> $OUT/steps.log
tail -5 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
src=$?
echo "=== smoke rc=$src" >> $OUT/steps.log
cat $OUT/smoke.log | tail -2
exit $(( rc != 0 ? rc : src ))
