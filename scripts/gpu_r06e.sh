#!/bin/bash
# Round 6 experiment: adjacent windows per lane (build/adj, -DKMA_ADJ_WIN=1): parity subset with
# the variant library, then c5 / c4 / c2 ABAB against the shipped build. The variant measured
# slower at c5 and was removed from the sources; this script is the record of
# how profiles/r06/adjacent_windows_r06e/ was taken.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06e}; mkdir -p $OUT
KMERANNO_LIB=kmers.anno_amd/build/adj/libkmeranno.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -v --timeout 600 --timeout-method thread \
  -p no:cacheprovider -k "synthetic_vs_oracle or edge_cases or long_proteins or giant or config1 or config5_size or config2" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/steps.log; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for wl in c5 c4 c2; do
    for arm in default adj; do
      if [ $arm = adj ]; then export KMERANNO_LIB=kmers.anno_amd/build/adj/libkmeranno.so; else unset KMERANNO_LIB; fi
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
