#!/bin/bash
# Round 4: full GPU tests; interleaved A/B of the protein step (packed input on / off) on this
# build and on the previous commit's library (build/prev: before the vote-record change); the
# adversarial layout sweep; the genome-directory workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r04c; mkdir -p $OUT
bash scripts/gpu_tests.sh r04c || exit $?
timeout -k 10 400 python scripts/ab_protein.py > $OUT/ab_cur.jsonl 2> $OUT/ab_cur.log
rc=$?; echo "ab cur rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
KMERANNO_LIB=kmers.anno_amd/build/prev/libkmeranno.so timeout -k 10 400 python scripts/ab_protein.py \
  --configs "packed=1" > $OUT/ab_prev.jsonl 2> $OUT/ab_prev.log
rc=$?; echo "ab prev rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.log
echo "bench c5 rc=$?" >> $OUT/steps.log
timeout -k 10 300 python3 scripts/layout_sweep.py --adversarial --lfs 0.5,0.9 > $OUT/adversarial.jsonl 2> $OUT/adversarial.log
echo "adversarial rc=$?" >> $OUT/steps.log
timeout -k 10 600 python bench.py --workload genomes > $OUT/genomes.json 2> $OUT/genomes.log
echo "genomes rc=$?" >> $OUT/steps.log
python3 - <<'PY'
import json
for f in ("ab_cur", "ab_prev"):
    for line in open(f"gpurun_out/r04c/{f}.jsonl"):
        d = json.loads(line)
        print(f, d["workload"], d["config"], d["rep"], round(d["ms"], 4), {k: round(v, 4) for k, v in d["phases_ms"].items()}, d["outputs_equal_first_arm"])
PY
