#!/bin/bash
# Round 4: GPU tests on the staging-pool build; c5 bench line (host call e2e); the vote-record
# A/B as ABAB runs (this build vs build/prev, one process each); a c2 sweep of proteins per block
# and deferral on the ASCII probe; the genome-directory workload; the adversarial layout sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r04e; mkdir -p $OUT
bash scripts/gpu_tests.sh r04e || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.log
rc=$?; echo "bench c5 rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python scripts/ab_protein.py --workloads c5 --configs "packed=2" --reps 1 >> $OUT/ab_vote.jsonl 2>> $OUT/ab_vote.log
  rc=$?; echo "ab cur $rep rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
  KMERANNO_LIB=kmers.anno_amd/build/prev/libkmeranno.so timeout -k 10 300 python scripts/ab_protein.py \
    --workloads c5 --configs "packed=1" --reps 1 >> $OUT/ab_vote.jsonl 2>> $OUT/ab_vote.log
  rc=$?; echo "ab prev $rep rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
done
timeout -k 10 300 python scripts/ab_protein.py --workloads c2 --reps 3 --configs \
  "packed=0,block_proteins=4;packed=0,block_proteins=3;packed=0,block_proteins=2;packed=0,block_proteins=4,defer=0;packed=0,block_proteins=2,defer=0;packed=2,block_proteins=4" \
  > $OUT/ab_c2.jsonl 2> $OUT/ab_c2.log
rc=$?; echo "ab c2 rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py --workload genomes > $OUT/genomes.json 2> $OUT/genomes.log
rc=$?; echo "genomes rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 scripts/layout_sweep.py --adversarial --lfs 0.5,0.9 > $OUT/adversarial.jsonl 2> $OUT/adversarial.log
echo "adversarial rc=$?" >> $OUT/steps.log
python3 - <<'PY'
import json
for f in ("ab_vote", "ab_c2"):
    for line in open(f"gpurun_out/r04e/{f}.jsonl"):
        d = json.loads(line)
        print(f, d["workload"], d["config"], d["rep"], d["library"][-30:], round(d["ms"], 4),
              {k: round(v, 4) for k, v in d["phases_ms"].items()}, d["outputs_equal_first_arm"])
PY
cat gpurun_out/r04e/steps.log
