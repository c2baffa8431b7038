#!/bin/bash
# Round 6 experiment: the single-residue mod-sampling order on the 10^7 table (c4 / c2 / c3,
# which the size rule leaves in the random order), forced through KMA_OPT_LAYOUT = 6 | MOD
# (70), ABAB against the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06j}; mkdir -p $OUT
for rep in 1 2; do
  for wl in c4 c2 c3; do
    for arm in rnd mod; do
      opt=""; [ $arm = mod ] && opt="--option layout=70"
      timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-extras $opt > $OUT/${wl}_${arm}_r$rep.json 2> $OUT/${wl}_${arm}_r$rep.log
      r=$?; echo "$wl $arm r$rep rc=$r" >> $OUT/steps.log; [ $r = 0 ] || exit $r
    done
  done
done
python3 - "$OUT" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(f"{sys.argv[1]}/c*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in d["phases_ms"].items()}, d["config"].get("table_minimizer_order"))
PY
