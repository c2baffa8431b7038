#!/bin/bash
# Residency A/B: default build vs KMA_SGPR_CAP build (K1/K12 SGPRs capped so the hardware admits
# the blocks per CU the occupancy API reports). Parity under the capped build first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out; mkdir -p $OUT
T="timeout -k 10"
SG=kmers.anno_amd/build/sg/libkmeranno.so
KMERANNO_LIB=$SG $T 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_sg.log 2>&1 || { tail -30 $OUT/pytest_sg.log; exit 1; }
tail -1 $OUT/pytest_sg.log
for wl in c2 c5; do
  for lib in default sg; do
    if [ $lib = sg ]; then export KMERANNO_LIB=$SG; else unset KMERANNO_LIB; fi
    $T 400 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline > $OUT/ab_${wl}_$lib.log 2>&1 || { tail -20 $OUT/ab_${wl}_$lib.log; exit 1; }
    grep '^{' $OUT/ab_${wl}_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl $lib', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['phases_ms'])"
  done
done
