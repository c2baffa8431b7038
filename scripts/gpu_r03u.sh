#!/bin/bash
# Round 3 (session 2) final build, call 1: every GPU test, smoke, then the PMC traffic passes of
# the dominant kernels (FETCH_SIZE / WRITE_SIZE / TCC requests, one rocprofv3 run per pass,
# calibrated on kma_gather_bench) -> profiles/r03_traffic.json (the bench's roofline source).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03u}; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest 600 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider -x
tail -1 $OUT/pytest.log >> $OUT/steps.log
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
GB=kmers.anno_amd/build/kma_gather_bench
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  tag=$(echo $c | cut -d' ' -f1)
  step pmc_gather_$tag 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_gather_$tag -o run -- $GB 1536 quad 4
  for wl in ${WLS:-c5 c2 c3 c4}; do
    step pmc_${wl}_$tag 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_${wl}_$tag -o run -- python3 bench.py --steps 3 --warmup 1 --workload $wl --no-cpu-baseline --no-extras
  done
done
step traffic 60 python3 scripts/traffic_summary.py $OUT 8388608
cp $OUT/traffic.log profiles/r03_traffic.json
