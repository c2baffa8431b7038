#!/bin/bash
# Round 3, first GPU pass: c5 layout x load-factor sweep on the shipped build (paired homes) and
# the unpaired variant (build/nopair), the adversarial key set, and one TCC counter pass per build
# (fabric read requests per case; kernel-trace only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r03a; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi; }
NP=kmers.anno_amd/build/nopair/libkmeranno.so
export KMERANNO_LIB=kmers.anno_amd/build/sweep/libkmeranno.so  # snapshot of the shipped build
step sweep_pair 300 python3 scripts/layout_sweep.py
step sweep_nopair 300 env KMERANNO_LIB=$NP python3 scripts/layout_sweep.py
step adv_pair 300 python3 scripts/layout_sweep.py --adversarial --lfs 0.5,0.9
step adv_nopair 300 env KMERANNO_LIB=$NP python3 scripts/layout_sweep.py --adversarial --lfs 0.5,0.9
step pmc_pair 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace \
  --output-format csv -d $OUT/pmc_pair -o run -- python3 scripts/layout_sweep.py --steps 3 --warmup 1
export KMERANNO_LIB=$NP  # read by the binding (no env hop under the profiler)
step pmc_nopair 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace \
  --output-format csv -d $OUT/pmc_nopair -o run -- python3 scripts/layout_sweep.py --steps 3 --warmup 1
