#!/bin/bash
# c5 load-factor sweep of the shipped kernel (LF 0.5 / 0.75 / 0.9): one bench line
# per LF (roofline, layout, per-phase kernel time), the chain-walk counts of each LF from the
# counting variant (make variant VNAME=count VFLAGS=-DKMA_TUNE_COUNT), and a rocprofv3 --stats
# of the LF 0.9 command. Usage: bash scripts/gpu_lf_sweep.sh <out-subdir> [lfs...]
# Stops at the first step that does not exit 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-lf_sweep}; mkdir -p $OUT
shift
LFS=${*:-0.5 0.75 0.9}
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi; }
for lf in $LFS; do
  step bench_c5_lf$lf 300 python3 -u bench.py --workload c5 --load-factor $lf --no-cpu-baseline --no-extras
  if [ -f kmers.anno_amd/build/count/libkmeranno.so ]; then
    KMERANNO_LIB=kmers.anno_amd/build/count/libkmeranno.so step walk_c5_lf$lf 300 python3 -u scripts/walk_stats.py c5 $lf
  fi
done
if [ -n "$STATS_LF" ]; then
  step stats_c5_lf$STATS_LF 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c5_lf$STATS_LF -o run -- python3 bench.py --workload c5 --load-factor $STATS_LF --steps 20 --warmup 3 --no-cpu-baseline --no-extras
fi
