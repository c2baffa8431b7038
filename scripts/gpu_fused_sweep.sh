#!/bin/bash
# Fused K12 vs two-kernel K1/K2 across batch sizes (10M-entry table): where K12 starts to win.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out
mkdir -p $OUT
for n in 10000 20000 40000 100000 300000; do
  for f in 1 0; do
    KMA_FUSED=$f timeout -k 10 300 python bench.py --workload c4 --n-seq $n --steps 20 --warmup 3 --no-cpu-baseline > $OUT/sweep_${n}_$f.log 2>&1 || { tail -20 $OUT/sweep_${n}_$f.log; exit 1; }
    grep '^{' $OUT/sweep_${n}_$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('n=$n fused=$f', '%.3e' % d['value'], 'ms/step %.4f' % d['ms_per_step'])"
  done
done
