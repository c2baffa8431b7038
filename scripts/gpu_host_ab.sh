#!/bin/bash
# ABAB of the c5 host call (scripts/e2e_host.py) across library builds: the shipped library and
# build/<variant>/libkmeranno.so, two rounds, one process per run, then a kernel + memory-copy
# trace of each build's call (scripts/host_call_timeline.py summarizes them).
#   [CFG=pieces=0,threads=16] bash scripts/gpu_host_ab.sh <out-subdir> <variant> [<variant> ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift; VS="$@"; CFG=${CFG:-pieces=0,threads=16}; mkdir -p $OUT
for rep in 1 2; do
  for lib in default $VS; do
    if [ $lib = default ]; then unset KMERANNO_LIB; else export KMERANNO_LIB=kmers.anno_amd/build/$lib/libkmeranno.so; fi
    timeout -k 10 300 python3 -u scripts/e2e_host.py --configs "$CFG" --reps 2 > $OUT/e2e_${lib}_r$rep.jsonl 2> $OUT/e2e_${lib}_r$rep.log
    rc=$?; echo "e2e $lib r$rep rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
  done
done
for lib in default $VS; do
  if [ $lib = default ]; then unset KMERANNO_LIB; else export KMERANNO_LIB=kmers.anno_amd/build/$lib/libkmeranno.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_$lib -o run -- python3 scripts/e2e_host.py --configs "$CFG" --reps 1 > $OUT/trace_$lib.log 2>&1
  rc=$?; echo "trace $lib rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
  python3 scripts/host_call_timeline.py $OUT/trace_$lib > $OUT/timeline_$lib.jsonl
done
for f in $OUT/e2e_*.jsonl; do python3 -c "
import json,sys
for l in open('$f'):
    j=json.loads(l); print('$f'.split('/')[-1], j['config'], round(j['ms'],3), j['host_profile_ms']['total'])"; done
