#!/bin/bash
# Round 6 experiment: which half of r06g's change (bitop3 match: build/mo keeps only it; gather
# without the kNone select: build/go keeps only it) moves c4 / c5 / c2, against build/base
# (before both) and the new default build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06h}; mkdir -p $OUT
for rep in 1 2; do
  for wl in c4 c5 c2; do
    for arm in base new mo go; do
      if [ $arm = new ]; then unset KMERANNO_LIB; else export KMERANNO_LIB=kmers.anno_amd/build/$arm/libkmeranno.so; fi
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
