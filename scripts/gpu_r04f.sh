#!/bin/bash
# Round 4: GPU tests on the one-pass 6-frame build (look-back emission); c3 as ABAB runs against
# the two-pass library (build/emit2) and four sequential slices per block (build/seq4); c3
# block clocks; the c5 line with the PCIe link rates; SQ counters of c5 with and without the
# vote record (build/vote) to explain the LDS bank conflicts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r04f; mkdir -p $OUT
bash scripts/gpu_tests.sh r04f || exit $?
for rep in 1 2; do
  for lib in default emit2 seq4; do
    if [ $lib = default ]; then unset KMERANNO_LIB; else export KMERANNO_LIB=kmers.anno_amd/build/$lib/libkmeranno.so; fi
    timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline --no-extras > $OUT/c3_${lib}_r$rep.json 2> $OUT/c3_${lib}_r$rep.log
    rc=$?; echo "c3 $lib r$rep rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
  done
done
unset KMERANNO_LIB
KMERANNO_LIB=kmers.anno_amd/build/clk/libkmeranno.so timeout -k 10 200 python scripts/block_clock.py c3 > $OUT/clock_c3.json 2> $OUT/clock_c3.log
rc=$?; echo "clock c3 rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.log
rc=$?; echo "bench c5 rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
SECTIONS=sq SQ_WLS=c5 bash scripts/gpu_measure.sh r04f/sq_cur || exit $?
KMERANNO_LIB=kmers.anno_amd/build/vote/libkmeranno.so SECTIONS=sq SQ_WLS=c5 bash scripts/gpu_measure.sh r04f/sq_vote || exit $?
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r04f/c3_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 4), d["phases_ms"], d["config"]["hits_per_gpu"])
d = json.loads(open("gpurun_out/r04f/c5.json").read().strip().splitlines()[-1])
print("c5", d["ms_per_step"], d["phases_ms"], json.dumps(d.get("e2e_host_call")))
PY
cat $OUT/steps.log
