#!/bin/bash
# Round 4: full GPU tests; interleaved A/B of the protein step (packed input on / off) on this
# build and on the previous commit's library (build/prev: before the vote-record change); the
# c5 bench line; the 6-frame probe with two sequential slices per block vs one (build/seq1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r04c; mkdir -p $OUT
bash scripts/gpu_tests.sh r04c tests/test_gpu_multirank.py || exit $?
timeout -k 10 400 python scripts/ab_protein.py > $OUT/ab_cur.jsonl 2> $OUT/ab_cur.log
rc=$?; echo "ab cur rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
KMERANNO_LIB=kmers.anno_amd/build/prev/libkmeranno.so timeout -k 10 400 python scripts/ab_protein.py \
  --workloads c5 --configs "packed=1" > $OUT/ab_prev.jsonl 2> $OUT/ab_prev.log
rc=$?; echo "ab prev rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
KMERANNO_LIB=kmers.anno_amd/build/fb3/libkmeranno.so timeout -k 10 400 python scripts/ab_protein.py \
  --workloads c5,c2 --configs "packed=1" > $OUT/ab_fb3.jsonl 2> $OUT/ab_fb3.log
rc=$?; echo "ab fb3 rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.log
echo "bench c5 rc=$?" >> $OUT/steps.log
for rep in 1; do
  for lib in default seq1; do
    if [ $lib = default ]; then unset KMERANNO_LIB; else export KMERANNO_LIB=kmers.anno_amd/build/$lib/libkmeranno.so; fi
    timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline --no-extras > $OUT/c3_${lib}_r$rep.json 2> $OUT/c3_${lib}_r$rep.log
    rc=$?; echo "c3 $lib r$rep rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
  done
done
unset KMERANNO_LIB
# tuning builds: chain-walk event counts at c5, block timelines at c2 and c3
KMERANNO_LIB=kmers.anno_amd/build/count/libkmeranno.so timeout -k 10 300 python scripts/walk_stats.py c5 > $OUT/walk_c5.json 2> $OUT/walk_c5.log
echo "walk c5 rc=$?" >> $OUT/steps.log
KMERANNO_LIB=kmers.anno_amd/build/countfb3/libkmeranno.so timeout -k 10 300 python scripts/walk_stats.py c5 > $OUT/walk_c5_fb3.json 2> $OUT/walk_c5_fb3.log
echo "walk c5 fb3 rc=$?" >> $OUT/steps.log
KMERANNO_LIB=kmers.anno_amd/build/clk/libkmeranno.so timeout -k 10 200 python scripts/block_clock.py c2 > $OUT/clock_c2.json 2> $OUT/clock_c2.log
echo "clock c2 rc=$?" >> $OUT/steps.log
KMERANNO_LIB=kmers.anno_amd/build/clk/libkmeranno.so timeout -k 10 200 python scripts/block_clock.py c3 > $OUT/clock_c3.json 2> $OUT/clock_c3.log
echo "clock c3 rc=$?" >> $OUT/steps.log
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r04c/c3_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 4), d["phases_ms"])
for f in ("ab_cur", "ab_prev", "ab_fb3"):
    for line in open(f"gpurun_out/r04c/{f}.jsonl"):
        d = json.loads(line)
        print(f, d["workload"], d["config"], d["rep"], round(d["ms"], 4), {k: round(v, 4) for k, v in d["phases_ms"].items()}, d["outputs_equal_first_arm"])
PY
