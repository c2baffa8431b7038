#!/bin/bash
# Round-5 pass: GPU tests, then the c5 load-factor sweep with two-choice placement (the default)
# and the chained tables beside it on the same box (A/B), rocprofv3 --stats at LF 0.9.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=${1:-r05c}
bash scripts/gpu_steps.sh $OUT "gputests|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" || exit $?
STATS_LF=0.9 bash scripts/gpu_lf_sweep.sh $OUT 0.5 0.75 0.9 || exit $?
bash scripts/gpu_steps.sh $OUT \
  "bench_c5_lf0.5_chainedB|300|python3 -u bench.py --workload c5 --load-factor 0.5 --placement chained --no-cpu-baseline --no-extras" \
  "bench_c5_lf0.9_chainedB|300|python3 -u bench.py --workload c5 --load-factor 0.9 --placement chained --no-cpu-baseline --no-extras" \
  "bench_c5_lf0.5_twoB|300|python3 -u bench.py --workload c5 --load-factor 0.5 --no-cpu-baseline --no-extras"
