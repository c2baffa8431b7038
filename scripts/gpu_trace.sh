#!/bin/bash
# K2 per-phase traces (KMA_VOTE_TRACE builds from `make variant`) for each variant in $VARIANTS:
# c2 and c5 bench lines (phases_ms) plus the trace of the last untimed call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
[ -n "$NO_PYTEST" ] || step pytest_gpu 900 python -m pytest tests -x -q -m gpu
for v in $VARIANTS; do
  export KMERANNO_LIB=$PWD/kmers.anno_amd/build/$v/libkmeranno.so
  KMA_TRACE_FILE=$OUT/tr_c2_$v.bin step bench_c2_$v 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
  KMA_TRACE_FILE=$OUT/tr_c5_$v.bin step bench_c5_$v 600 python bench.py --steps 3 --warmup 1 --workload c5 --no-cpu-baseline
done
