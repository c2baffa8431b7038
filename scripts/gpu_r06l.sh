#!/bin/bash
# Round 6 experiment: block sizes <= 4 in the P = 8 kernel (build/cap8, built from the shipped
# sources with that one dispatch changed) against the shipped P = 4 dispatch, c4 / c2 ABAB,
# with the 10^7 table in the mod-sampling order.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06l}; mkdir -p $OUT
for rep in 1 2; do
  for wl in c4 c2; do
    for arm in p4 p8; do
      if [ $arm = p8 ]; then export KMERANNO_LIB=kmers.anno_amd/build/cap8/libkmeranno.so; else unset KMERANNO_LIB; fi
      timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-extras > $OUT/${wl}_${arm}_r$rep.json 2> $OUT/${wl}_${arm}_r$rep.log
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
