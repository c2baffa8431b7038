#!/bin/bash
# Round-end pass of the paired-home build: GPU parity, smoke, bench lines (c5 headline with the
# CPU baseline; c2 / c3 / c4), rocprofv3 kernel stats at c5, and one L2 / fabric-request PMC pass
# per layout at c5 (paired m = 7 and m = 6, unpaired m = 7: does line sharing cut requests?).
# Stops at the first step that faults, aborts or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name" | tee -a $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log; tail -2 $OUT/$name.log
  [ $rc -eq 0 ] || exit $rc; }
step pytest 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c5 600 python bench.py --steps 20 --warmup 3
step bench_c2 300 python bench.py --steps 20 --warmup 3 --workload c2 --no-cpu-baseline
step bench_c3 300 python bench.py --steps 20 --warmup 3 --workload c3 --no-cpu-baseline
step bench_c4 300 python bench.py --steps 10 --warmup 2 --workload c4 --no-cpu-baseline
step prof_c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras
C="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
(export KMA_MINIMIZER=7; step pmc_pair_m7 600 rocprofv3 --pmc $C --kernel-trace --output-format csv \
  -d $OUT/pmc_pair_m7 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras) || exit $?
(export KMA_MINIMIZER=6; step pmc_pair_m6 600 rocprofv3 --pmc $C --kernel-trace --output-format csv \
  -d $OUT/pmc_pair_m6 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras) || exit $?
(export KMERANNO_LIB=kmers.anno_amd/build/nopair/libkmeranno.so KMA_MINIMIZER=7
 step pmc_nopair_m7 600 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_nopair_m7 \
  -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras) || exit $?
