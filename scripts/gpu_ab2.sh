#!/bin/bash
# A/B of table layouts and K1 forms on one box. Each case in $CASES is
# name=ENV1=v1,ENV2=v2 (env for the bench; KMERANNO_LIB=<v> picks the A/B build
# kmers.anno_amd/build/<v>/libkmeranno.so of `make variant VNAME=<v>`):
# a c2 bench line plus c2/c5 kernel stats per case. Parity runs first (default + other K1 forms).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
if [ -z "$NO_PYTEST" ]; then
  step pytest_gpu 900 python -m pytest tests -x -q -m gpu
  for shape in ${PARITY_SHAPES:-run lane}; do
    KMA_PROBE=$shape step pytest_$shape 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu
  done
fi
for c in ${CASES:-"min=KMA_PROBE=run"}; do
  name=${c%%=*}; envs=${c#*=}
  ( for kv in ${envs//,/ }; do
      case $kv in KMERANNO_LIB=*) kv=KMERANNO_LIB=$PWD/kmers.anno_amd/build/${kv#*=}/libkmeranno.so ;; esac
      export "$kv"; done
    step bench_c2_$name 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
    step prof_c2_$name 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2_$name -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
    [ -n "$NO_C5" ] || step prof_c5_$name 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5_$name -o run -- python3 bench.py --steps 5 --warmup 1 --workload c5 --no-cpu-baseline
  ) || exit $?
done
