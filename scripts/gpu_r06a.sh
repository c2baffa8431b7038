#!/bin/bash
# Round 6, first GPU pass: the GPU tests + smoke; c5 ABAB of the mod-sampling minimizer order
# (the size rule's choice for the 10^8 table) against the random order (KMA_OPT_LAYOUT = 6);
# c2 ABAB of the one-wave-block grid (KMA_OPT_BLOCK_WAVES = 1, 1 or 2 proteins per block);
# the in-process replica fan-out at c5 size with 1 / 2 / 4 / 8 replicas on device 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06a}; mkdir -p $OUT
bash scripts/gpu_tests.sh ${1:-r06a}; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2; do
  for arm in mod random; do
    X=""; [ $arm = random ] && X="--option layout=6"
    timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --no-extras $X > $OUT/c5_${arm}_r$rep.json 2> $OUT/c5_${arm}_r$rep.log
    r=$?; echo "c5 $arm r$rep rc=$r" >> $OUT/steps.log; [ $r = 0 ] || exit $r
  done
done
for rep in 1 2; do
  for arm in block4 wave1 wave2; do
    X=""; [ $arm = wave1 ] && X="--option block_waves=1"; [ $arm = wave2 ] && X="--option block_waves=1 --option block_proteins=2"
    timeout -k 10 300 python bench.py --workload c2 --no-cpu-baseline --no-extras $X > $OUT/c2_${arm}_r$rep.json 2> $OUT/c2_${arm}_r$rep.log
    r=$?; echo "c2 $arm r$rep rc=$r" >> $OUT/steps.log; [ $r = 0 ] || exit $r
  done
done
timeout -k 10 600 python scripts/replica_scaling.py > $OUT/replicas.jsonl 2> $OUT/replicas.log
r=$?; echo "replicas rc=$r" >> $OUT/steps.log
python3 - "$OUT" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(f"{sys.argv[1]}/c[25]_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in d["phases_ms"].items()})
for l in open(f"{sys.argv[1]}/replicas.jsonl"):
    d = json.loads(l)
    print(d["replicas"], round(d["call_ms"], 2), round(d["stage_ms_max"], 2), d["staging_threads"], d["outputs_equal_one_replica"])
PY
exit $r
