#!/bin/bash
# Round 3: c5 layout x load-factor sweep, shipped (paired homes) and unpaired builds, with TCC
# counter passes per case; adversarial keys.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r03d; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi; }
B=kmers.anno_amd/build
step sweep_pair 300 python3 scripts/layout_sweep.py
step pmc_pair 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace \
  --output-format csv -d $OUT/pmc_pair -o run -- python3 scripts/layout_sweep.py --steps 3 --warmup 1
export KMERANNO_LIB=$B/nopair/libkmeranno.so
step sweep_nopair 300 python3 scripts/layout_sweep.py
step pmc_nopair 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace \
  --output-format csv -d $OUT/pmc_nopair -o run -- python3 scripts/layout_sweep.py --steps 3 --warmup 1
step adv_nopair 300 python3 scripts/layout_sweep.py --adversarial --lfs 0.5,0.9
unset KMERANNO_LIB
step adv_pair 300 python3 scripts/layout_sweep.py --adversarial --lfs 0.5,0.9
