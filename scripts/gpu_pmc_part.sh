#!/bin/bash
# PMC passes (one counter set per pass, kernel-trace only) over the partitioned protein path.
#   WL=c4 bash scripts/gpu_pmc_part.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
WL=${WL:-c4}
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  echo "=== pass $i: $line" >> $OUT/steps.log
  timeout -k 10 300 rocprofv3 --pmc $line --kernel-trace --output-format csv -d $OUT/pmc_${WL}_$i -o run \
    -- python3 bench.py --steps 2 --warmup 1 --workload $WL --no-cpu-baseline --no-extras > $OUT/pmc_${WL}_$i.log 2>&1
  rc=$?
  echo "=== pass $i rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then tail -5 $OUT/pmc_${WL}_$i.log; exit $rc; fi
done < ${PASSES:-scripts/pmc/part.txt}
