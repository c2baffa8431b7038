#!/bin/bash
# Round 6, second GPU pass: the changed GPU tests (device build/wrap under the new -1 rule, the
# native TSV loader, the mod-sampling layout); c5 ABAB of the minimizer orders: mod-sampling
# (the shipped size rule), its open-closed variant (build/modopen, -DKMA_MOD_OPEN=1) and the
# random order (KMA_OPT_LAYOUT = 6).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06b}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 600 --timeout-method thread \
  -p no:cacheprovider -k "torch_buffers or from_tsv or synthetic_vs_oracle or edge_cases or replicated or pipelined" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/steps.log; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2; do
  for arm in mod modopen random; do
    X=""; unset KMERANNO_LIB
    [ $arm = random ] && X="--option layout=6"
    [ $arm = modopen ] && export KMERANNO_LIB=kmers.anno_amd/build/modopen/libkmeranno.so
    timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --no-extras $X > $OUT/c5_${arm}_r$rep.json 2> $OUT/c5_${arm}_r$rep.log
    r=$?; echo "c5 $arm r$rep rc=$r" >> $OUT/steps.log; [ $r = 0 ] || exit $r
  done
done
python3 - "$OUT" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(f"{sys.argv[1]}/c5_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in d["phases_ms"].items()}, d["config"].get("table_minimizer_order"))
PY
exit $rc
