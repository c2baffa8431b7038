#!/bin/bash
# One GPU-box session: parity tests, a bench line, and a rocprofv3 kernel-trace summary.
# Stops at the first step that faults, aborts or times out (exit codes other than 0/1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STEPS="${STEPS:-pytest bench prof}"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -5 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    pytest) run pytest_gpu 900 python -m pytest tests -x -q -m gpu ;;
    bench) run bench 900 python bench.py --steps ${BENCH_STEPS:-20} --warmup 3 ${BENCH_ARGS:-} ;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
            -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} ;;
    smoke) run smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
  esac
done
