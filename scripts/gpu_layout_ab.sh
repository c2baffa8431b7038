#!/bin/bash
# A/B of table layouts at c5: 64-B buckets m=7 (default) / m=6, 128-B buckets (s16, s16w2) m=6 / m=7.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
WL=${WL:-c5}
run() {  # name lib minimizer
  echo "=== $1" >> $OUT/steps.log
  KMERANNO_LIB=$2 KMA_MINIMIZER=$3 timeout -k 10 300 python bench.py --steps 10 --warmup 2 \
    --workload $WL --no-cpu-baseline --no-extras > $OUT/ab_$1.log 2>&1
  local rc=$?
  echo "=== $1 rc=$rc" >> $OUT/steps.log
  grep -o '"ms_per_step": [0-9.]*' $OUT/ab_$1.log
  grep -o 'layout m=[0-9], longest chain [0-9]*, displaced [0-9.]*%' $OUT/ab_$1.log
  [ $rc -eq 0 ] || exit $rc
}
L=kmers.anno_amd/build
for cfg in ${CFGS:-"s8m7 $L/libkmeranno.so 7" "s8m6 $L/libkmeranno.so 6" "s16w2m6 $L/s16w2/libkmeranno.so 6" "s16w2m7 $L/s16w2/libkmeranno.so 7" "s16m6 $L/s16/libkmeranno.so 6"}; do
  run $cfg
done
