#!/bin/bash
# Round 3: proteins per block (KMA_BLOCK_PROTEINS 4 / 6 / 8) x chain-walk variants at c5:
# serial walks (serial), serial walks with queued keys (sqkeys), no walks (nowalk: cost bound).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r03m; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
B=kmers.anno_amd/build
for rep in 1 2; do
  for bp in 4 6 8; do
    for v in serial sqkeys nowalk; do
      export KMERANNO_LIB=$B/$v/libkmeranno.so KMA_BLOCK_PROTEINS=$bp
      step c5_${v}_bp${bp}_$rep 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
      grep -o '"ms_per_step": [0-9.]*' $OUT/c5_${v}_bp${bp}_$rep.log >> $OUT/steps.log
    done
  done
done
