#!/bin/bash
# One GPU-box session: parity tests, bench lines, rocprofv3 kernel-trace summaries, A/B runs.
# Stops at the first step that faults, aborts or times out (exit codes other than 0/1).
#   STEPS="pytest bench prof ..." bash scripts/gpu_round.sh
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
  tail -3 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    pytest) run pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps ${BENCH_STEPS:-20} --warmup 3 ${BENCH_ARGS:-} ;;
    bench2) run bench_c2 300 python bench.py --steps 20 --warmup 3 --workload c2 --no-cpu-baseline ;;
    bench3) run bench_c3 300 python bench.py --steps 20 --warmup 3 --workload c3 --no-cpu-baseline ;;
    bench4) run bench_c4 300 python bench.py --steps 10 --warmup 2 --workload c4 --no-cpu-baseline ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
            -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras ${BENCH_ARGS:-} ;;
    prof2) run prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof2 -o run \
            -- python3 bench.py --steps 10 --warmup 2 --workload c2 --no-cpu-baseline --no-extras ;;
    prof3) run prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof3 -o run \
            -- python3 bench.py --steps 10 --warmup 2 --workload c3 --no-cpu-baseline --no-extras ;;
    variants) for v in ${VARIANTS:-s16}; do  # VAR_ENV="KMA_MINIMIZER=6 ..." per run
          for wl in ${VAR_WLS:-c2 c5}; do
            env KMERANNO_LIB=kmers.anno_amd/build/$v/libkmeranno.so ${VAR_ENV:-} true || exit 2
            KMERANNO_LIB=kmers.anno_amd/build/$v/libkmeranno.so run var_${v}_${wl}${VAR_TAG:-} 300 \
              env ${VAR_ENV:-KMA_NOTHING=1} python bench.py --steps 10 --warmup 2 --workload $wl \
              --no-cpu-baseline --no-extras || exit $?
          done; done ;;
    lf) for lf in ${LFS:-0.5 0.75 0.9}; do
          run bench_c5_lf$lf 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras \
            --load-factor $lf || exit $?; done ;;
    gather) for cfg in ${GATHER_CFGS:-"1536 quad 4" "1536 quad 8" "1536 oct 4" "1536 oct 8" "150 quad 4" "150 oct 4"}; do
              run gather 120 kmers.anno_amd/build/kma_gather_bench $cfg || exit $?
              cat $OUT/gather.log >> $OUT/gather_all.log; done ;;
  esac
done
