#!/bin/bash
# c3 ABAB: sequential 256-position slices per 6-frame probe block, 2 (default) vs 3 / 4
# (build/seq3, build/seq4: -DKMA_CONTIG_SEQ=3 / 4).  bash scripts/gpu_ab_contig_seq.sh <out-subdir>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab_seq}; mkdir -p $OUT
for rep in 1 2; do
  for lib in default seq3 seq4; do
    if [ $lib = default ]; then unset KMERANNO_LIB; else export KMERANNO_LIB=kmers.anno_amd/build/$lib/libkmeranno.so; fi
    timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline --no-extras > $OUT/c3_${lib}_r$rep.json 2> $OUT/c3_${lib}_r$rep.log
    rc=$?; echo "c3 $lib r$rep rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
  done
done
python3 - "$OUT" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/c3_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in d["phases_ms"].items()})
PY
