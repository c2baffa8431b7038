#!/bin/bash
# Round 3: chain queue of packed keys at 192 (7 blocks per CU) / 96 entries per wave (LDS for
# 8 blocks per CU) x proteins per block (KMA_BLOCK_PROTEINS), c5 and c2, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r03n; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
B=kmers.anno_amd/build
for rep in 1 2; do
  for cfg in sqkeys:6 q192:6 q96:4 q96:6 q96:8 q96p6:5 q96p6:6; do
    v=${cfg%:*}; bp=${cfg#*:}
    export KMERANNO_LIB=$B/$v/libkmeranno.so KMA_BLOCK_PROTEINS=$bp
    step c5_${v}_bp${bp}_$rep 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
    echo "c5 $v bp$bp $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5_${v}_bp${bp}_$rep.log)" >> $OUT/steps.log
  done
done
for rep in 1 2; do
  for cfg in sqkeys:4 sqkeys:6 q96:4 q96:6 q96p6:6; do
    v=${cfg%:*}; bp=${cfg#*:}
    export KMERANNO_LIB=$B/$v/libkmeranno.so KMA_BLOCK_PROTEINS=$bp
    step c2_${v}_bp${bp}_$rep 300 python3 bench.py --workload c2 --steps 50 --warmup 5 --no-cpu-baseline --no-extras
    echo "c2 $v bp$bp $(grep -o '"ms_per_step": [0-9.]*' $OUT/c2_${v}_bp${bp}_$rep.log)" >> $OUT/steps.log
  done
done
