#!/bin/bash
# HBM traffic of K1 per MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE in
# separate --pmc passes (kernel-trace only), calibrated on kma_gather_bench's random 64-B line
# reads of a known count (the guide calls non-streaming widths uncalibrated), plus L2 hit data.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
GB=kmers.anno_amd/build/kma_gather_bench
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  tag=$(echo $c | cut -d' ' -f1)
  step pmc_gather_$tag 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_gather_$tag -o run -- $GB ${GATHER_MIB:-1536} quad 4
  for wl in ${WLS:-c2 c3 c5}; do
    step pmc_${wl}_$tag 900 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_${wl}_$tag -o run -- python3 bench.py --steps 3 --warmup 1 --workload $wl --no-cpu-baseline
  done
done
