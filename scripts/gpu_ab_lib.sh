#!/bin/bash
# ABAB of one bench workload across library builds: the shipped library ("default") and the
# variants build/<name>/libkmeranno.so, two rounds, one process per run.
#   [EXTRA="--load-factor 0.9"] [TAG=lf09] bash scripts/gpu_ab_lib.sh <out-subdir> <workload> <variant> [<variant> ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/$1; WL=$2; shift 2; mkdir -p $OUT; T=${TAG:+_$TAG}
for rep in 1 2; do
  for lib in default "$@"; do
    if [ $lib = default ]; then unset KMERANNO_LIB; else export KMERANNO_LIB=kmers.anno_amd/build/$lib/libkmeranno.so; fi
    timeout -k 10 300 python bench.py --workload $WL --no-cpu-baseline --no-extras $EXTRA > $OUT/${WL}${T}_${lib}_r$rep.json 2> $OUT/${WL}${T}_${lib}_r$rep.log
    rc=$?; echo "$WL$T $lib r$rep rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
  done
done
python3 - "$OUT" "$WL$T" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(f"{sys.argv[1]}/{sys.argv[2]}_*.json")):  # (argv[2]: workload + tag)
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in d["phases_ms"].items()})
PY
