#!/bin/bash
# Round 4: packed residue input. Full GPU tests, then an interleaved A/B of the protein step
# with the pack kernel + packed probe (1) against the ASCII probe (0) at c5 / c4 / c2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r04c; mkdir -p $OUT
bash scripts/gpu_tests.sh r04c || exit $?
for rep in 1 2; do
  for wl in c5 c4 c2; do
    for pk in 1 0; do
      timeout -k 10 300 python bench.py --workload $wl --packed-input $pk --no-cpu-baseline \
        $( [ $rep = 2 ] && echo --no-extras ) > $OUT/${wl}_p${pk}_r${rep}.json 2> $OUT/${wl}_p${pk}_r${rep}.log
      rc=$?; echo "$wl p$pk r$rep rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
    done
  done
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r04c/c*_p*_r*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    e=d.get('e2e_host_call',{})
    print(f.split('/')[-1], round(d['ms_per_step'],4), d['phases_ms'], 'e2e', round(e.get('ms',0),3))
PY
# the adversarial layout sweep (2,000 shared minimizers) on the shipped build, once
timeout -k 10 300 python3 scripts/layout_sweep.py --adversarial --lfs 0.5,0.9 > $OUT/adversarial.jsonl 2> $OUT/adversarial.log
echo "adversarial rc=$?" >> $OUT/steps.log
timeout -k 10 700 python bench.py --workload genomes > $OUT/genomes.json 2> $OUT/genomes.log
echo "genomes rc=$?" >> $OUT/steps.log
