#!/bin/bash
# Paired-home A/B (KMA_PAIR_HOME): GPU parity under the main build (and optionally the pair
# build), then c5 / c2 / c3 bench lines per (library, forced layout).
#   PAIR_TESTS=pair2 RUNS="main:c5:7 pair:c5:7 pair2:c5:6:0.9" bash scripts/gpu_pair_ab.sh
# (RUNS entries: library:workload[:forced layout[:load factor]])
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
T="timeout -k 10"
if [ -n "$MAIN_TESTS" ]; then
  $T 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_main.log 2>&1
  rc=$?; tail -2 $OUT/pytest_main.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PAIR_TESTS" ]; then
  KMERANNO_LIB=kmers.anno_amd/build/$PAIR_TESTS/libkmeranno.so $T 600 python -u -m pytest tests -x -q -m gpu \
    --timeout 300 --timeout-method thread > $OUT/pytest_pair.log 2>&1
  rc=$?; tail -2 $OUT/pytest_pair.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $RUNS; do
  IFS=: read -r v wl m lf <<< "$r"
  lib=kmers.anno_amd/build/libkmeranno.so; [ $v = main ] || lib=kmers.anno_amd/build/$v/libkmeranno.so
  envm=KMA_NOTHING=1; [ -n "$m" ] && envm=KMA_MINIMIZER=$m
  KMERANNO_LIB=$lib $T 300 env $envm python bench.py --steps 20 --warmup 3 --workload $wl \
    --no-cpu-baseline --no-extras ${lf:+--load-factor $lf} ${EXTRA:-} > $OUT/pair_${v}_${wl}_m$m$lf.log 2>&1
  rc=$?
  echo "$v $wl m=$m lf=$lf rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/pair_${v}_${wl}_m$m$lf.log) $(grep -o 'layout m=[^,]*, longest chain [0-9]*, displaced [0-9.%]*' $OUT/pair_${v}_${wl}_m$m$lf.log)"
  [ $rc -eq 0 ] || exit $rc
done
