#!/bin/bash
# Round 4: GPU tests with the 6-frame tile loads issued before the contig search and the ASCII
# protein kernel's LUT store deferred; ABAB c2 / c3 against the previous commit (build/pre);
# the c5 host call with its host-side phase profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r04i; mkdir -p $OUT
bash scripts/gpu_tests.sh r04i || exit $?
for rep in 1 2; do
  for lib in default pre; do
    if [ $lib = default ]; then unset KMERANNO_LIB; else export KMERANNO_LIB=kmers.anno_amd/build/$lib/libkmeranno.so; fi
    for wl in c2 c3; do
      timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-extras > $OUT/${wl}_${lib}_r$rep.json 2> $OUT/${wl}_${lib}_r$rep.log
      rc=$?; echo "$wl $lib r$rep rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
    done
  done
done
unset KMERANNO_LIB
timeout -k 10 400 python scripts/e2e_host.py --configs "pieces=8,threads=16;pieces=16,threads=16;packed=0,pieces=16,threads=16" > $OUT/e2e_sweep.jsonl 2> $OUT/e2e_sweep.log
rc=$?; echo "e2e sweep rc=$rc" >> $OUT/steps.log
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r04i/c*_r*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in d["phases_ms"].items()})
PY
cat $OUT/e2e_sweep.jsonl
cat $OUT/steps.log
