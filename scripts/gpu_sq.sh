#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run per pass, kernel-trace only) over short bench runs:
# wave cycles split into busy-issue / parked / issue-stall, instruction mix, for the dominant
# kernels of the workloads in $WLS. Usage: scripts/gpu_sq.sh <out-subdir>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-sq}; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi; }
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
for wl in ${WLS:-c3 c5}; do
  i=0
  for c in "$P1" "$P2"; do
    i=$((i + 1))
    step sq_${wl}_p$i 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/sq_${wl}_p$i -o run -- python3 bench.py --steps 3 --warmup 1 --workload $wl --no-cpu-baseline --no-extras
  done
done
step summary 60 python3 scripts/sq_summary.py $OUT
