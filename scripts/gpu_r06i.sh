#!/bin/bash
# Round 6 experiment: protein kernels instantiated at the capacity a call needs (P = 4 / 6 / 8
# proteins per block for K = 8) against build/base (every call in the P = 8 kernel): the GPU
# suite with the new build, then c5 / c4 / c2 ABAB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=${1:-r06i}
bash scripts/gpu_tests.sh $OUT; rc=$?
[ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/$OUT
for rep in 1 2; do
  for wl in c5 c4 c2; do
    for arm in base new; do
      if [ $arm = new ]; then unset KMERANNO_LIB; else export KMERANNO_LIB=kmers.anno_amd/build/base/libkmeranno.so; fi
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
