#!/bin/bash
# Generic GPU step runner: each argument line "name|timeout|command" runs under its own
# timeout, output to gpurun_out/<out>/<name>.log; stops at the first step that does not exit 0.
# Usage: bash scripts/gpu_steps.sh <out-subdir> "name|secs|cmd" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-steps}; mkdir -p $OUT
shift
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; t=${rest%%|*}; cmd=${rest#*|}
  echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t bash -c "$cmd" > $OUT/$name.log 2>&1; rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then tail -30 $OUT/$name.log; exit $rc; fi
done
