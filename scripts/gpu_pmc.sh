#!/bin/bash
# Counter passes (rocprofv3 --pmc, kernel-trace only) over a short bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
WL=${WL:-c2}
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1
echo "list rc=$?"
timeout -k 10 900 rocprofv3 -i scripts/pmc/pass1.txt --kernel-trace --output-format csv -d $OUT/pmc_$WL -o pmc \
  -- python3 bench.py --steps 3 --warmup 1 --workload $WL --no-cpu-baseline > $OUT/pmc_$WL.log 2>&1
echo "pmc rc=$?"
