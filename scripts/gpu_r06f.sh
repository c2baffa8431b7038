#!/bin/bash
# Round 6 experiment: the mod-sampling order over single residues (t = 1, ranks 31 - code, the
# position's shift from a nibble table; build/t1, -DKMA_MOD_T1=1) against t = 3 (shipped):
# parity of the mod-order cases with the variant library, then c5 (LF 0.5, 0.9) ABAB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06f}; mkdir -p $OUT
KMERANNO_LIB=kmers.anno_amd/build/t1/libkmeranno.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -v --timeout 600 --timeout-method thread \
  -p no:cacheprovider -k "mod or config5 or synthetic_vs_oracle" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/steps.log; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for wl in c5 c5_lf0.9; do
    wa="--workload ${wl%%_lf*}"; [ "$wl" != "${wl#*_lf}" ] && wa="$wa --load-factor ${wl#*_lf}"
    [ $rep = 2 ] && [ $wl = c5_lf0.9 ] && continue
    for arm in t3 t1; do
      if [ $arm = t1 ]; then export KMERANNO_LIB=kmers.anno_amd/build/t1/libkmeranno.so; else unset KMERANNO_LIB; fi
      timeout -k 10 300 python bench.py $wa --no-cpu-baseline --no-extras > $OUT/${wl}_${arm}_r$rep.json 2> $OUT/${wl}_${arm}_r$rep.log
      r=$?; echo "$wl $arm r$rep rc=$r" >> $OUT/steps.log; [ $r = 0 ] || exit $r
    done
  done
done
for arm in t3 t1; do
  if [ $arm = t1 ]; then export KMERANNO_LIB=kmers.anno_amd/build/t1/libkmeranno.so; else unset KMERANNO_LIB; fi
  timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --no-extras > $OUT/c5_${arm}_r3.json 2> $OUT/c5_${arm}_r3.log
  r=$?; echo "c5 $arm r3 rc=$r" >> $OUT/steps.log; [ $r = 0 ] || exit $r
done
python3 - "$OUT" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(f"{sys.argv[1]}/c*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in d["phases_ms"].items()})
PY
