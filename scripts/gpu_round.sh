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
    pytest) run pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread ;;
    bench) run bench 900 python bench.py --steps ${BENCH_STEPS:-20} --warmup 3 ${BENCH_ARGS:-} ;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
            -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} ;;
    smoke) run smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench3) run bench_c3 900 python bench.py --steps 20 --warmup 3 --workload c3 ;;
    prof3) run prof_c3 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof3 -o run \
            -- python3 bench.py --steps 10 --warmup 2 --workload c3 --no-cpu-baseline ;;
    bench4) run bench_c4 900 python bench.py --steps 10 --warmup 2 --workload c4 --no-cpu-baseline ;;
    bench5) run bench_c5 900 python bench.py --steps 10 --warmup 2 --workload c5 --no-cpu-baseline ;;
    lf) for lf in 0.25 0.35 0.5; do
          run prof_c5_lf$lf 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5_lf$lf -o run \
            -- python3 bench.py --steps 5 --warmup 1 --workload c5 --no-cpu-baseline --load-factor $lf || exit $?; done ;;
    prof5) run prof_c5 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof5 -o run \
            -- python3 bench.py --steps 5 --warmup 1 --workload c5 --no-cpu-baseline ;;
    gather) for cfg in ${GATHER_CFGS:-"16 lane 4" "150 lane 1" "150 lane 2" "150 lane 4" "150 quad 2" "150 quad 4" "150 quad 8" "1536 lane 1" "1536 lane 2" "1536 lane 4" "1536 quad 2" "1536 quad 4" "1536 quad 8" "1536 quad 4 1" "1536 lane 2 1" "6144 quad 4" "6144 lane 2"}; do
              run gather 300 kmers.anno_amd/build/kma_gather_bench $cfg || exit $?
              cat $OUT/gather.log >> $OUT/gather_all.log; done ;;
  esac
done
