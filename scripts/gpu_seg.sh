#!/bin/bash
# Segmented K1/K2 overlap: parity under forced segments, then c2/c5 benches per segment count.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step pytest_gpu 900 python -m pytest tests -x -q -m gpu
KMA_SEGMENTS=3 step pytest_gpu_seg3 900 python -m pytest tests -x -q -m gpu
for sg in 1 2 3 4; do KMA_SEGMENTS=$sg step bench_c2_s$sg 600 python bench.py --steps 30 --warmup 3 --no-cpu-baseline; done
for sg in 1 4 8; do KMA_SEGMENTS=$sg step bench_c5_s$sg 900 python bench.py --steps 8 --warmup 2 --workload c5 --no-cpu-baseline; done
