#!/bin/bash
# Round 6 experiment: c5 proteins per block under the capacity-matched kernels (6: P = 6; 7 and
# 8: P = 8; 5: P = 6), KMA_OPT_BLOCK_PROTEINS through bench's --option, ABAB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06k}; mkdir -p $OUT
for rep in 1 2; do
  for bp in 6 7 5 8; do
    timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --no-extras --option block_proteins=$bp > $OUT/c5_bp${bp}_r$rep.json 2> $OUT/c5_bp${bp}_r$rep.log
    r=$?; echo "c5 bp$bp r$rep rc=$r" >> $OUT/steps.log; [ $r = 0 ] || exit $r
  done
done
python3 - "$OUT" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(f"{sys.argv[1]}/c*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in d["phases_ms"].items()})
PY
