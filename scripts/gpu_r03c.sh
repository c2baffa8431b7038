#!/bin/bash
# Round 3: c5 layout x load-factor sweep (shipped paired-home build and the unpaired variant),
# adversarial keys, TCC counter passes per case, and cost bounds of the chain walks / sets.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r03c; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi; }
B=kmers.anno_amd/build
export KMERANNO_LIB=$B/libkmeranno.so
step sweep_pair 300 python3 scripts/layout_sweep.py
step adv_pair 300 python3 scripts/layout_sweep.py --adversarial --lfs 0.5,0.9
step pmc_pair 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace \
  --output-format csv -d $OUT/pmc_pair -o run -- python3 scripts/layout_sweep.py --steps 3 --warmup 1
for v in lanep nowalk noset .; do
  export KMERANNO_LIB=$B/$v/libkmeranno.so
  step bench_${v/./default} 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras
done
export KMERANNO_LIB=$B/nopair/libkmeranno.so
step sweep_nopair 300 python3 scripts/layout_sweep.py
step adv_nopair 300 python3 scripts/layout_sweep.py --adversarial --lfs 0.5,0.9
step pmc_nopair 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace \
  --output-format csv -d $OUT/pmc_nopair -o run -- python3 scripts/layout_sweep.py --steps 3 --warmup 1
unset KMERANNO_LIB
step pytest_contigs 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_wide.py tests/test_cli.py tests/test_gpu_configs.py -m gpu \
  -k "contigs or config3 or peg or wide"
step bench_c3 300 python3 bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline --no-extras
