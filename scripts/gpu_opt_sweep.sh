#!/bin/bash
# One bench workload under several ABI option sets (bench.py --option), one process per run,
# two rounds: bash scripts/gpu_opt_sweep.sh <out-subdir> <workload> "<opts>" ["<opts>" ...]
# where <opts> is a space-separated list of name=value ("-" = library defaults).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/$1; WL=$2; shift 2; mkdir -p $OUT
for rep in 1 2; do
  i=0
  for set in "$@"; do
    i=$((i + 1)); args=()
    [ "$set" = "-" ] || for o in $set; do args+=(--option "$o"); done
    timeout -k 10 300 python bench.py --workload $WL --no-cpu-baseline --no-extras "${args[@]}" \
      > $OUT/${WL}_s${i}_r$rep.json 2> $OUT/${WL}_s${i}_r$rep.log
    rc=$?; echo "$WL s$i [$set] r$rep rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
  done
done
python3 - "$OUT" "$WL" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(f"{sys.argv[1]}/{sys.argv[2]}_s*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["config"].get("options"), round(d["ms_per_step"], 4),
          {k: round(v, 4) for k, v in d["phases_ms"].items()})
PY
