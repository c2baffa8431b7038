#!/bin/bash
# Round-end evidence: GPU parity, the bench lines (c2 headline, c3, c5) and kernel-trace stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
T="timeout -k 10"
$T 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
$T 400 python bench.py --steps 20 --warmup 3 > $OUT/bench_c2.log 2>&1 || { tail -20 $OUT/bench_c2.log; exit 1; }
$T 400 python bench.py --steps 20 --warmup 3 --workload c3 > $OUT/bench_c3.log 2>&1 || { tail -20 $OUT/bench_c3.log; exit 1; }
$T 600 python bench.py --steps 10 --warmup 2 --workload c5 --no-cpu-baseline > $OUT/bench_c5.log 2>&1 || { tail -20 $OUT/bench_c5.log; exit 1; }
$T 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof3 -o run -- python3 bench.py --steps 10 --warmup 2 --workload c3 --no-cpu-baseline > $OUT/prof3.log 2>&1 || exit 1
for f in c2 c3 c5; do grep '^{' $OUT/bench_$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', '%.3e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['phases_ms'], 'frac %.3f' % d['roofline']['frac'])"; done
