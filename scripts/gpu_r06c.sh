#!/bin/bash
# Round 6: the mod-sampling order on the 10^7 table (Infinity-Cache resident; the size rule keeps
# it in the random order): c4 / c2 / c3 ABAB, default vs KMA_OPT_LAYOUT = 6 | MOD_SAMPLING (70).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06c}; mkdir -p $OUT
for rep in 1 2; do
  for wl in c4 c2 c3; do
    for arm in random mod; do
      X=""; [ $arm = mod ] && X="--option layout=70"
      timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-extras $X > $OUT/${wl}_${arm}_r$rep.json 2> $OUT/${wl}_${arm}_r$rep.log
      r=$?; echo "$wl $arm r$rep rc=$r" >> $OUT/steps.log; [ $r = 0 ] || exit $r
    done
  done
done
python3 - "$OUT" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(f"{sys.argv[1]}/c*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in d["phases_ms"].items()})
PY
