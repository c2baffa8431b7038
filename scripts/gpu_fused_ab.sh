#!/bin/bash
# Fused K12 vs two-kernel K1/K2: GPU parity under both, then c2 and c5 bench lines for each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
T="timeout -k 10"
$T 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_fused.log 2>&1 || { tail -30 $OUT/pytest_fused.log; exit 1; }
tail -2 $OUT/pytest_fused.log
KMA_FUSED=0 $T 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_2k.log 2>&1 || { tail -30 $OUT/pytest_2k.log; exit 1; }
tail -2 $OUT/pytest_2k.log
for wl in c2 c5; do
  for f in "KMA_FUSED=1 KMA_FUSED_P=4" "KMA_FUSED=1 KMA_FUSED_P=8" "KMA_FUSED=0"; do
    tag=$(echo $f | tr ' =' '__')
    env $f $T 400 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_${wl}_$tag.log 2>&1 || { tail -20 $OUT/bench_${wl}_$tag.log; exit 1; }
    grep '^{' $OUT/bench_${wl}_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl $f', '%.3e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['phases_ms'])"
  done
done
